// Shared helpers for the gfx950 kernels behind include/kdstep.h.
// Wave = 64 lanes everywhere (CDNA4); never use warp-32 idioms here.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>
#include <cmath>
#include <cstdlib>

#include "../../include/kdstep.h"

namespace kd {

// ------------------------------------------------------------------ errors ----
void set_error(const std::string& msg);
int fail(int code, const std::string& msg);

#define KD_CHECK_ARG(cond, msg)                                   \
    do {                                                          \
        if (!(cond)) return ::kd::fail(KD_ERR_ARG, (msg));        \
    } while (0)
#define KD_CHECK_SHAPE(cond, msg)                                 \
    do {                                                          \
        if (!(cond)) return ::kd::fail(KD_ERR_SHAPE, (msg));      \
    } while (0)
#define KD_CHECK_ALIGN(ptr, bytes, msg)                                          \
    do {                                                                         \
        if (((uintptr_t)(ptr)) % (bytes) != 0) return ::kd::fail(KD_ERR_ALIGN, (msg)); \
    } while (0)
#define KD_LAUNCH_CHECK(what)                                                    \
    do {                                                                         \
        hipError_t e__ = hipGetLastError();                                      \
        if (e__ != hipSuccess)                                                   \
            return ::kd::fail(KD_ERR_LAUNCH, std::string(what) + ": " + hipGetErrorString(e__)); \
    } while (0)

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// ------------------------------------------------------------------- types ----
typedef __bf16 bf16;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) uint32_t u32x4;
typedef __attribute__((ext_vector_type(2))) uint32_t u32x2;

// SiLU / sigmoid with v_exp_f32 + v_rcp_f32 instead of an IEEE fp32 division (~10 instructions
// each). Every SiLU of the build (GEMM epilogues, k_swiglu_fwd / bwd, the decode GEMV) uses these
// forms, so the fused and unfused paths stay bit-identical.
// exp(-x) as v_exp_f32 (2^y) of y = x * -log2(e), written out: the packed SwiGLU epilogue
// (gemm.hip silu_mul_pair) repeats exactly these operations two elements at a time
#define KD_SILU_LOG2E 1.4426950408889634f
__device__ __forceinline__ float sigmoid_fast(float x) { return __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(x * -KD_SILU_LOG2E)); }
__device__ __forceinline__ float silu_fast(float x) { return x * sigmoid_fast(x); }
// transpose of the RoPE rotation of a (first-half, second-half) element pair (HF5 qwen2
// apply_rotary_pos_emb, backward): k_qkv_merge and the attention backward's fused-gradient
// epilogues share it, so both produce the same bits -- the fused multiply-adds written out: left to
// -ffp-contract the two call sites contracted differently (1 ulp apart on 5 of 358 k elements)
__device__ __forceinline__ void rope_t(float g1, float g2, float c, float sn, float& y1, float& y2) {
    y1 = __builtin_fmaf(g1, c, g2 * sn);
    y2 = __builtin_fmaf(g2, c, -(g1 * sn));
}
// SwiGLU backward of one element: d = dL/dh, h = silu(g) * u -> (dL/dg, dL/du); shared by
// k_swiglu_bwd and the fused dgrad epilogue (KD_ACT_DSWIGLU), so both agree bit for bit
__device__ __forceinline__ void swiglu_grad(float d, float g, float u, float& dg, float& du) {
    const float sg = sigmoid_fast(g);
    du = d * (g * sg);
    dg = d * u * sg * (1.f + g * (1.f - sg));
}
// gelu_pytorch_tanh'(x): gelu = x * s, s = sigmoid(2u) = (1 + tanh u) / 2, u = k0 (x + k1 x^3):
// gelu' = s + 2 x s (1 - s) u', u' = k0 (1 + 3 k1 x^2); s by one v_exp_f32 + v_rcp_f32
__device__ __forceinline__ float gelu_tanh_grad(float x) {
    constexpr float k0 = 0.7978845608028654f, k1 = 0.044715f;
    constexpr float c0 = -2.f * 0.7978845608028654f * 1.4426950408889634f, c1 = c0 * 0.044715f;
    const float x2 = x * x;
    const float sg = __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(x * fmaf(c1, x2, c0)));
    return sg + 2.f * x * sg * (1.f - sg) * k0 * fmaf(3.f * k1, x2, 1.f);
}

__device__ __forceinline__ float bf2f(bf16 x) { return (float)x; }
__device__ __forceinline__ bf16 f2bf(float x) { return (bf16)x; }

// ------------------------------------------------------------- reductions ----
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// top-2 with deterministic tie-break: larger value first, lower index on ties (the KD loss's
// teacher klogits, DT:170-171; used by k_row_stats and the lm_head GEMM's row statistics).
// Branch-free (selects only): the if/else-if form made hipcc keep (v1, i1, v2, i2) in a
// scratch array indexed per lane (36 B of private memory, a scratch round trip per push).
__device__ __forceinline__ bool top2_better(float a, int ia, float b, int ib) {
    return a > b || (a == b && ia < ib);
}
__device__ __forceinline__ void top2_push(float v, int i, float& v1, int& i1, float& v2, int& i2) {
    const bool b1 = top2_better(v, i, v1, i1);
    const bool b2 = top2_better(v, i, v2, i2);
    const float nv2 = b1 ? v1 : (b2 ? v : v2);
    const int ni2 = b1 ? i1 : (b2 ? i : i2);
    v1 = b1 ? v : v1;
    i1 = b1 ? i : i1;
    v2 = nv2;
    i2 = ni2;
}

// Block-wide sum over NW waves using a caller-provided LDS scratch of >= NW floats.
template <int NW>
__device__ __forceinline__ float block_sum(float v, float* scratch) {
    v = wave_sum(v);
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    __syncthreads();
    if (l == 0) scratch[w] = v;
    __syncthreads();
    float r = 0.f;
#pragma unroll
    for (int i = 0; i < NW; ++i) r += scratch[i];
    return r;
}
template <int NW>
__device__ __forceinline__ float block_max(float v, float* scratch) {
    v = wave_max(v);
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    __syncthreads();
    if (l == 0) scratch[w] = v;
    __syncthreads();
    float r = -INFINITY;
#pragma unroll
    for (int i = 0; i < NW; ++i) r = fmaxf(r, scratch[i]);
    return r;
}

inline int ceil_div(int64_t a, int64_t b) { return (int)((a + b - 1) / b); }

// RoPE rotate_half pair (HF5 qwen2 apply_rotary_pos_emb), the one arithmetic shared by
// k_qkv_split and the q|k|v scatter GEMM epilogue: first half x1 -> x1 cos - x2 sin, second
// half x2 -> x2 cos + x1 sin (explicit fma: both kernels round identically)
__device__ __forceinline__ float rope_first(float x1, float x2, float cs, float sn) { return fmaf(x1, cs, -(x2 * sn)); }
__device__ __forceinline__ float rope_second(float x2, float x1, float cs, float sn) { return fmaf(x2, cs, x1 * sn); }

// A/B and diagnostic switches: read from the environment only in the tools' A/B library
// (KD_AB_BUILD, `python csrc/build.py --ab`); the product library always takes the default, so
// no environment variable changes which kernel or plan it runs.
inline int ab_knob(const char* name, int dflt) {
#ifdef KD_AB_BUILD
    const char* e = std::getenv(name);
    return e ? std::atoi(e) : dflt;
#else
    (void)name;
    return dflt;
#endif
}

}  // namespace kd
