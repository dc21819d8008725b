// Memory-bound layer kernels of the KD step (vectorised 16-B bf16 access, fp32 math).
//
// Each replaces a PyTorch / transformers op reached from the reference's forward
// (DT:206-271) or its autograd backward:
//   layernorm_fwd/bwd   nn.LayerNorm eps 1e-6 (SigLIP layer_norm1/2, post_layernorm;
//                       HF5 siglip :325-357, :567) + the post-LN hook's token mean (DT:243)
//   rmsnorm_fwd/bwd     Qwen2RMSNorm eps 1e-6 (HF5 qwen2 :35-55)
//   qkv_split / merge   q/k/v view+transpose + RoPE theta=1e6 rotate_half (HF5 qwen2 :60-140)
//   swiglu_fwd/bwd      down(silu(gate) * up) (HF5 qwen2 Qwen2MLP)
//   act_bwd             gelu_pytorch_tanh (SigLIP MLP) / gelu erf (projector) derivatives
//   patchify            Conv2d(3,1152,14,stride 14) as im2col (HF5 siglip :116-186)
//   embed_assemble/bwd  embed_tokens + masked_scatter of packed image features
//                       (HF5 llava_onevision :280-343, :510-513)
//   colsum              bias gradients
//   row_group_mean      hook_out.mean(dim=1) (DT:243-244)
//   ntxent_fwd_bwd      normalize + contrastive_loss (DT:246-248, :393-416)
//   adamw               torch.optim.AdamW (DT:198-201) on flat fp32 master weights
//   sumsq               gradient norm
#include "common.h"

#include <cstdlib>

namespace kd {
namespace {

constexpr int NT = 256;

__device__ __forceinline__ void load8(const bf16* p, float* f) {
    bf16x8 v = *(const bf16x8*)p;
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] = (float)v[j];
}
__device__ __forceinline__ void load8(const float* p, float* f) {
    const f32x4 a = *(const f32x4*)p, b = *(const f32x4*)(p + 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) { f[j] = a[j]; f[4 + j] = b[j]; }
}
__device__ __forceinline__ void store8(bf16* p, const float* f) {
    bf16x8 v;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (bf16)f[j];
    *(bf16x8*)p = v;
}

// -------------------------------------------------------------- LayerNorm ----
// one wave per row, D % 8 == 0, D <= 64 * 8 * 8; x bf16 or fp32 (XT: the fp32 residual stream)
template <bool RMS, typename XT>
__global__ void __launch_bounds__(NT) k_norm_fwd(const XT* __restrict__ x, int64_t ldx, const bf16* __restrict__ w,
                                                 const bf16* __restrict__ bias, bf16* __restrict__ y, int64_t ldy,
                                                 float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                 int R, int D, float eps) {
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (row >= R) return;
    const XT* xr = x + (int64_t)row * ldx;
    float f[8][8];
    const int nch = D / 8;
    float s = 0.f, ss = 0.f;
#pragma unroll
    for (int it = 0; it < 8; ++it) {
        const int c = lane + it * 64;
        if (c < nch) {
            load8(xr + c * 8, f[it]);
#pragma unroll
            for (int j = 0; j < 8; ++j) { s += f[it][j]; ss += f[it][j] * f[it][j]; }
        }
    }
    s = wave_sum(s);
    float mean = RMS ? 0.f : s / D;
    float var;
    if (RMS) {
        var = wave_sum(ss) / D;
    } else {
        // two-pass variance for accuracy
        float v2 = 0.f;
#pragma unroll
        for (int it = 0; it < 8; ++it) {
            const int c = lane + it * 64;
            if (c < nch)
#pragma unroll
                for (int j = 0; j < 8; ++j) { const float dd = f[it][j] - mean; v2 += dd * dd; }
        }
        var = wave_sum(v2) / D;
    }
    const float rstd = rsqrtf(var + eps);
    bf16* yr = y + (int64_t)row * ldy;
#pragma unroll
    for (int it = 0; it < 8; ++it) {
        const int c = lane + it * 64;
        if (c < nch) {
            float wv[8], o[8];
            load8(w + c * 8, wv);
            if (!RMS) {
                float bv[8];
                load8(bias + c * 8, bv);
#pragma unroll
                for (int j = 0; j < 8; ++j) o[j] = (f[it][j] - mean) * rstd * wv[j] + bv[j];
            } else {
#pragma unroll
                for (int j = 0; j < 8; ++j) o[j] = f[it][j] * rstd * wv[j];
            }
            store8(yr + c * 8, o);
        }
    }
    if (lane == 0) {
        if (mean_out) mean_out[row] = mean;
        if (rstd_out) rstd_out[row] = rstd;
    }
}

// dx = rstd * (w*dy - mean(w*dy) - xhat * mean(w*dy*xhat))   (LayerNorm)
// dx = rstd * (w*dy - xhat * mean(w*dy*xhat))                (RMSNorm, xhat = x*rstd)
// dw/db partial sums over the rows a workgroup handles -> fp32 [gridDim.x, D].
// One wave per row; IT = ceil(D / 512) 16-B chunks per lane. The rows of a wave go through
// a two-deep register pipeline: x, dy, the previous dx (accumulate) and the row's stats of
// row i+1 are in flight while row i is reduced and written (one row at a time, with the
// dx re-load after the reduction, the kernel ran at ~1.5 TB/s).
constexpr int NW_NORM = NT / 64;   // waves per k_norm_bwd workgroup
// x chunk of 8 elements as loaded: bf16x8, or two f32x4 for the fp32 residual stream
template <typename XT> struct XChunk {
    bf16x8 v;
    __device__ __forceinline__ void load(const bf16* p) { v = *(const bf16x8*)p; }
    __device__ __forceinline__ float get(int j) const { return (float)v[j]; }
};
template <> struct XChunk<float> {
    f32x4 a, b;
    __device__ __forceinline__ void load(const float* p) { a = *(const f32x4*)p; b = *(const f32x4*)(p + 4); }
    __device__ __forceinline__ float get(int j) const { return j < 4 ? a[j] : b[j - 4]; }
};

// k_norm_fwd with every load of the row issued first: IT = ceil(D / 512) chunks per lane, the chunk index
// clamped into the row so no load sits under a lane-dependent branch (k_norm_fwd's conditional loads were
// each followed by their own vmcnt(0): seven serial memory round trips per 3584-wide row), the weight /
// bias chunks loaded beside x. The arithmetic and its order are k_norm_fwd's (bit-identical).
template <bool RMS, int IT, typename XT>
__global__ void __launch_bounds__(NT) k_norm_fwd2(const XT* __restrict__ x, int64_t ldx, const bf16* __restrict__ w,
                                                  const bf16* __restrict__ bias, bf16* __restrict__ y, int64_t ldy,
                                                  float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                  int R, int D, float eps) {
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (row >= R) return;
    const XT* xr = x + (int64_t)row * ldx;
    const int nch = D / 8;
    XChunk<XT> xc[IT];
    bf16x8 wc[IT], bc[IT];
#pragma unroll
    for (int it = 0; it < IT; ++it) {
        const int c = min(lane + it * 64, nch - 1);
        xc[it].load(xr + c * 8);
        wc[it] = *(const bf16x8*)(w + c * 8);
        if (!RMS) bc[it] = *(const bf16x8*)(bias + c * 8);
    }
    float s = 0.f, ss = 0.f;
#pragma unroll
    for (int it = 0; it < IT; ++it) {
        if (lane + it * 64 < nch) {
#pragma unroll
            for (int j = 0; j < 8; ++j) { const float f = xc[it].get(j); s += f; ss += f * f; }
        }
    }
    s = wave_sum(s);
    const float mean = RMS ? 0.f : s / D;
    float var;
    if (RMS) {
        var = wave_sum(ss) / D;
    } else {
        float v2 = 0.f;
#pragma unroll
        for (int it = 0; it < IT; ++it) {
            if (lane + it * 64 < nch)
#pragma unroll
                for (int j = 0; j < 8; ++j) { const float dd = xc[it].get(j) - mean; v2 += dd * dd; }
        }
        var = wave_sum(v2) / D;
    }
    const float rstd = rsqrtf(var + eps);
    bf16* yr = y + (int64_t)row * ldy;
#pragma unroll
    for (int it = 0; it < IT; ++it) {
        const int c = lane + it * 64;
        if (c < nch) {
            float o[8];
            if (!RMS) {
#pragma unroll
                for (int j = 0; j < 8; ++j) o[j] = (xc[it].get(j) - mean) * rstd * (float)wc[it][j] + (float)bc[it][j];
            } else {
#pragma unroll
                for (int j = 0; j < 8; ++j) o[j] = xc[it].get(j) * rstd * (float)wc[it][j];
            }
            store8(yr + c * 8, o);
        }
    }
    if (lane == 0) {
        if (mean_out) mean_out[row] = mean;
        if (rstd_out) rstd_out[row] = rstd;
    }
}

// dy chunk of 8 elements: bf16 per row, or (GDY) fp32 per row GROUP -- the post_layernorm hook's
// gradient, d(pooled tile feature) spread as d / np over the tile's np rows (DT:243-244) without
// rounding it to bf16: a bf16 value repeated over 729 rows is a coherent error, and the two tiles'
// post_layernorm.bias contributions cancel to ~1e-3 of each (tools/ntx_bias_study.py)
template <bool GDY> struct DyChunk {
    bf16x8 v;
    __device__ __forceinline__ void load(const void* p) { v = *(const bf16x8*)p; }
    __device__ __forceinline__ float get(int j) const { return (float)v[j]; }
};
template <> struct DyChunk<true> {
    f32x4 a, b;
    __device__ __forceinline__ void load(const void* p) { a = *(const f32x4*)p; b = *((const f32x4*)p + 1); }
    __device__ __forceinline__ float get(int j) const { return j < 4 ? a[j] : b[j - 4]; }
};

template <bool RMS, int IT, typename XT, bool GDY = false>
__global__ void __launch_bounds__(NT) k_norm_bwd(const XT* __restrict__ x, int64_t ldx, const bf16* __restrict__ w,
                                                 const void* __restrict__ dy, int64_t lddy,
                                                 const float* __restrict__ mean_in, const float* __restrict__ rstd_in,
                                                 bf16* __restrict__ dx, int64_t lddx, int dx_accum,
                                                 float* __restrict__ dw_part, float* __restrict__ db_part,
                                                 int R, int D, int rows_per_block, int gP = 1, float gscale = 1.f) {
    extern __shared__ __attribute__((aligned(16))) float sacc[];  // [4 waves][2][D] per workgroup
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int nch = D / 8;
    float pw[IT][8], pb[IT][8], wr[IT][8];
    // the weight chunks: unconditional loads (chunk index clamped; a chunk past the row is never
    // used), all in flight at once -- a load under the lane-dependent test waited for itself
#pragma unroll
    for (int it = 0; it < IT; ++it) {
#pragma unroll
        for (int j = 0; j < 8; ++j) { pw[it][j] = 0.f; pb[it][j] = 0.f; }
        load8(w + min(lane + it * 64, nch - 1) * 8, wr[it]);
    }
    const int r_begin = blockIdx.x * rows_per_block;
    const int r_end = min(R, r_begin + rows_per_block);
    struct Row { XChunk<XT> x[IT]; DyChunk<GDY> g[IT]; bf16x8 p[IT]; float mean, rstd; };
    // every load is unconditional (row and chunk clamped into range, dx read even when not
    // accumulated): with a data-dependent number of loads in flight hipcc can only wait
    // vmcnt(0), which drains the next row's loads and undoes the pipeline
    auto load = [&](Row& t, int row_) {
        const int row = min(row_, R - 1);
        const XT* xr = x + (int64_t)row * ldx;
        const char* gr = (const char*)dy + (GDY ? (int64_t)(row / gP) * lddy * 4 : (int64_t)row * lddy * 2);
        const bf16* pr = dx + (int64_t)row * lddx;
#pragma unroll
        for (int it = 0; it < IT; ++it) {
            const int c = min(lane + it * 64, nch - 1);
            t.x[it].load(xr + c * 8);
            t.g[it].load(gr + c * 8 * (GDY ? 4 : 2));
            t.p[it] = *(const bf16x8*)(pr + c * 8);
        }
        t.mean = RMS ? 0.f : mean_in[row];
        t.rstd = rstd_in[row];
    };
    auto process = [&](const Row& t, int row) {
        const float mean = t.mean, rstd = t.rstd;
        float a1 = 0.f, a2 = 0.f;
#pragma unroll
        for (int it = 0; it < IT; ++it) {
            if (lane + it * 64 >= nch) continue;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const float xv = t.x[it].get(j), dv = GDY ? t.g[it].get(j) * gscale : t.g[it].get(j);
                const float xh = (xv - mean) * rstd;
                const float g = dv * wr[it][j];
                a1 += g;
                a2 += g * xh;
                pw[it][j] += dv * xh;
                pb[it][j] += dv;
            }
        }
        a1 = wave_sum(a1) / D;
        a2 = wave_sum(a2) / D;
        bf16* dxr = dx + (int64_t)row * lddx;
#pragma unroll
        for (int it = 0; it < IT; ++it) {
            const int c = lane + it * 64;
            if (c < nch) {
                float o[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const float xh = (t.x[it].get(j) - mean) * rstd;
                    const float dv = GDY ? t.g[it].get(j) * gscale : t.g[it].get(j);
                    o[j] = rstd * (dv * wr[it][j] - (RMS ? 0.f : a1) - xh * a2);
                    if (dx_accum) o[j] += (float)t.p[it][j];
                }
                store8(dxr + c * 8, o);
            }
        }
    };
    Row r0, r1;
    int row = r_begin + wv;
    load(r0, row);
    for (; row < r_end; row += 8) {   // two rows per trip: the buffers stay compile-time named
        load(r1, row + 4);
        process(r0, row);
        if (row + 4 >= r_end) break;
        load(r0, row + 8);
        process(r1, row + 4);
    }
    // block sum of the 4 waves' dw/db partials: each wave stores its own [2][D] slice (16-B
    // stores, no LDS atomics: ds_add_f32 at a 32-B lane stride was 16-way bank-conflicted),
    // then every thread adds the 4 slices of its columns in a fixed order
    float* mine = sacc + (size_t)wv * 2 * D;
#pragma unroll
    for (int it = 0; it < IT; ++it) {
        const int c = lane + it * 64;
        if (c < nch) {
            *(f32x4*)(mine + c * 8) = (f32x4){pw[it][0], pw[it][1], pw[it][2], pw[it][3]};
            *(f32x4*)(mine + c * 8 + 4) = (f32x4){pw[it][4], pw[it][5], pw[it][6], pw[it][7]};
            *(f32x4*)(mine + D + c * 8) = (f32x4){pb[it][0], pb[it][1], pb[it][2], pb[it][3]};
            *(f32x4*)(mine + D + c * 8 + 4) = (f32x4){pb[it][4], pb[it][5], pb[it][6], pb[it][7]};
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < D; i += NT) {
        if (dw_part) dw_part[(int64_t)blockIdx.x * D + i] = ((sacc[i] + sacc[2 * D + i]) + sacc[4 * D + i]) + sacc[6 * D + i];
        if (db_part)
            db_part[(int64_t)blockIdx.x * D + i] = ((sacc[D + i] + sacc[3 * D + i]) + sacc[5 * D + i]) + sacc[7 * D + i];
    }
}

// out[d] (+)= sum_p part[p][d]: 16 columns x 64 row lanes per 1024-thread block, each lane
// with RP_U independent loads in flight (the planes are L2/MALL-hot; with D = 896 a
// 64-column block gave 14 workgroups whose lanes each waited out P/16 dependent loads),
// then a fixed-order LDS tree (deterministic)
constexpr int RP_C = 16, RP_R = 64, RP_U = 8;
__global__ void __launch_bounds__(1024) k_reduce_parts(const float* __restrict__ part, int P, int D,
                                                       float* __restrict__ out, int accum) {
    __shared__ float red[RP_R][RP_C + 1];
    const int cx = threadIdx.x % RP_C, ry = threadIdx.x / RP_C;
    const int d = blockIdx.x * RP_C + cx;
    float s = 0.f;
    if (d < D) {
        int p = ry;
        for (; p + (RP_U - 1) * RP_R < P; p += RP_U * RP_R) {
            float v[RP_U];
#pragma unroll
            for (int u = 0; u < RP_U; ++u) v[u] = part[(int64_t)(p + u * RP_R) * D + d];
#pragma unroll
            for (int u = 0; u < RP_U; ++u) s += v[u];
        }
        for (; p < P; p += RP_R) s += part[(int64_t)p * D + d];
    }
    red[ry][cx] = s;
    __syncthreads();
    for (int h = RP_R / 2; h > 0; h >>= 1) {
        if (ry < h) red[ry][cx] += red[ry + h][cx];
        __syncthreads();
    }
    if (ry == 0 && d < D) out[d] = accum ? out[d] + red[0][cx] : red[0][cx];
}

// ------------------------------------------------------------------ q/k/v ----
// qkv [M = B*S, (nq + 2 nkv) * hd] -> q [B,nq,S,HDP], k/v [B,nkv,S,HDP] (zero pad),
// with RoPE (rotate_half convention) on q and k when cos/sin tables are given.
// One thread per (token, head, VEC-wide chunk of the first half): the chunk and its
// rotate_half partner (i + hd/2) are read, rotated and written as VEC-wide vectors;
// chunks past hd/2 zero the padding [hd, hdp).
template <int VEC>
__global__ void k_qkv_split(const bf16* __restrict__ qkv, int64_t ld, bf16* __restrict__ q, bf16* __restrict__ k,
                            bf16* __restrict__ v, const float* __restrict__ cos_t, const float* __restrict__ sin_t,
                            int B, int S, int nq, int nkv, int hd, int hdp) {
    typedef bf16 vec_t __attribute__((ext_vector_type(VEC)));
    const int heads = nq + 2 * nkv;
    const int hh = hd / 2;
    const int nch = hh / VEC, npad = (hdp - hd) / VEC, per = nch + npad;
    const int64_t total = (int64_t)B * S * heads * per;
    for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total; idx += (int64_t)gridDim.x * blockDim.x) {
        const int ci = (int)(idx % per);
        const int64_t th = idx / per;
        const int head = (int)(th % heads);
        const int64_t tok = th / heads;
        const int s = (int)(tok % S), b = (int)(tok / S);
        bf16* dst;
        int hidx, nh;
        if (head < nq) { dst = q; hidx = head; nh = nq; }
        else if (head < nq + nkv) { dst = k; hidx = head - nq; nh = nkv; }
        else { dst = v; hidx = head - nq - nkv; nh = nkv; }
        bf16* drow = dst + (((int64_t)b * nh + hidx) * S + s) * hdp;
        if (ci < nch) {
            const int i = ci * VEC;
            const bf16* srow = qkv + tok * ld + (int64_t)head * hd;
            vec_t a = *(const vec_t*)(srow + i), c2 = *(const vec_t*)(srow + i + hh);
            if (cos_t && head < nq + nkv) {
                const float* cr = cos_t + (int64_t)s * hh + i;
                const float* sr = sin_t + (int64_t)s * hh + i;
#pragma unroll
                for (int e = 0; e < VEC; ++e) {
                    const float x1 = (float)a[e], x2 = (float)c2[e], cs = cr[e], sn = sr[e];
                    a[e] = (bf16)rope_first(x1, x2, cs, sn);
                    c2[e] = (bf16)rope_second(x2, x1, cs, sn);
                }
            }
            *(vec_t*)(drow + i) = a;
            *(vec_t*)(drow + i + hh) = c2;
        } else {
            *(vec_t*)(drow + hd + (ci - nch) * VEC) = (vec_t){};
        }
    }
}

// inverse: dq (fp32, [B,nq,S,HDP]), dk/dv (bf16 [B,nkv,S,HDP]) -> dqkv [M, (nq+2nkv)*hd],
// VEC-wide chunks of the first half and their partners, transposed rotation
template <int VEC>
__global__ void k_qkv_merge(const float* __restrict__ dq, const bf16* __restrict__ dk, const bf16* __restrict__ dv,
                            bf16* __restrict__ dqkv, int64_t ld, const float* __restrict__ cos_t,
                            const float* __restrict__ sin_t, int B, int S, int nq, int nkv, int hd, int hdp) {
    typedef bf16 vec_t __attribute__((ext_vector_type(VEC)));
    const int heads = nq + 2 * nkv, hh = hd / 2, nch = hh / VEC;
    const int64_t total = (int64_t)B * S * heads * nch;
    for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total; idx += (int64_t)gridDim.x * blockDim.x) {
        const int i = (int)(idx % nch) * VEC;
        const int64_t th = idx / nch;
        const int head = (int)(th % heads);
        const int64_t tok = th / heads;
        const int s = (int)(tok % S), b = (int)(tok / S);
        float g1[VEC], g2[VEC];
        if (head < nq) {
            const float* r = dq + (((int64_t)b * nq + head) * S + s) * hdp;
#pragma unroll
            for (int e = 0; e < VEC; ++e) { g1[e] = r[i + e]; g2[e] = r[i + hh + e]; }
        } else {
            const bool isk = head < nq + nkv;
            const int hidx = isk ? head - nq : head - nq - nkv;
            const bf16* r = (isk ? dk : dv) + (((int64_t)b * nkv + hidx) * S + s) * hdp;
            const vec_t a = *(const vec_t*)(r + i), c2 = *(const vec_t*)(r + i + hh);
#pragma unroll
            for (int e = 0; e < VEC; ++e) { g1[e] = (float)a[e]; g2[e] = (float)c2[e]; }
        }
        if (cos_t && head < nq + nkv) {  // transpose of the rotation
            const float* cr = cos_t + (int64_t)s * hh + i;
            const float* sr = sin_t + (int64_t)s * hh + i;
#pragma unroll
            for (int e = 0; e < VEC; ++e) {
                const float c = cr[e], sn = sr[e];
                float y1, y2;
                rope_t(g1[e], g2[e], c, sn, y1, y2);
                g1[e] = y1; g2[e] = y2;
            }
        }
        vec_t o1, o2;
#pragma unroll
        for (int e = 0; e < VEC; ++e) { o1[e] = (bf16)g1[e]; o2[e] = (bf16)g2[e]; }
        bf16* d = dqkv + tok * ld + (int64_t)head * hd;
        *(vec_t*)(d + i) = o1;
        *(vec_t*)(d + i + hh) = o2;
    }
}

// ------------------------------------------------------------------ SwiGLU ----
// gu [M, 2I] = [gate | up] -> h [M, I] = silu(gate) * up
__global__ void k_swiglu_fwd(const bf16* __restrict__ gu, int64_t ldg, bf16* __restrict__ h, int64_t ldh, int M, int I) {
    const int n8 = I / 8;
    const int64_t total = (int64_t)M * n8;
    for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total; idx += (int64_t)gridDim.x * blockDim.x) {
        const int64_t m = idx / n8;
        const int c = (int)(idx % n8) * 8;
        float g[8], u[8], o[8];
        load8(gu + m * ldg + c, g);
        load8(gu + m * ldg + I + c, u);
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = silu_fast(g[j]) * u[j];
        store8(h + m * ldh + c, o);
    }
}

__global__ void k_swiglu_bwd(const bf16* __restrict__ gu, int64_t ldg, const bf16* __restrict__ dh, int64_t ldh,
                             bf16* __restrict__ dgu, int64_t ldd, int M, int I) {
    const int n8 = I / 8;
    const int64_t total = (int64_t)M * n8;
    for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total; idx += (int64_t)gridDim.x * blockDim.x) {
        const int64_t m = idx / n8;
        const int c = (int)(idx % n8) * 8;
        float g[8], u[8], d[8], og[8], ou[8];
        load8(gu + m * ldg + c, g);
        load8(gu + m * ldg + I + c, u);
        load8(dh + m * ldh + c, d);
#pragma unroll
        for (int j = 0; j < 8; ++j) swiglu_grad(d[j], g[j], u[j], og[j], ou[j]);
        store8(dgu + m * ldd + c, og);
        store8(dgu + m * ldd + I + c, ou);
    }
}

// dx = dy * act'(pre)
__global__ void k_act_bwd(const bf16* __restrict__ pre, const bf16* __restrict__ dy, bf16* __restrict__ dx,
                          int64_t n, int act) {
    const int64_t n8 = n / 8;
    for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < n8; idx += (int64_t)gridDim.x * blockDim.x) {
        float x[8], d[8], o[8];
        load8(pre + idx * 8, x);
        load8(dy + idx * 8, d);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            float dv;
            if (act == KD_ACT_GELU_TANH) {
                dv = gelu_tanh_grad(x[j]);
            } else if (act == KD_ACT_GELU_ERF) {
                const float cdf = 0.5f * (1.f + erff(x[j] * 0.7071067811865476f));
                const float pdf = 0.3989422804014327f * __expf(-0.5f * x[j] * x[j]);
                dv = cdf + x[j] * pdf;
            } else {  // silu
                const float sg = sigmoid_fast(x[j]);
                dv = sg * (1.f + x[j] * (1.f - sg));
            }
            o[j] = d[j] * dv;
        }
        store8(dx + idx * 8, o);
    }
}

// -------------------------------------------------------------- patchify ----
// pixels [NI, 3, IMG, IMG] (fp32 or bf16) -> rows [NI * P*P, Kp] bf16, k = c*ps*ps + kh*ps + kw
template <typename T>
__global__ void k_patchify(const T* __restrict__ px, bf16* __restrict__ out, int NI, int img, int ps, int Kp) {
    const int P = img / ps, K = 3 * ps * ps;
    const int64_t rows = (int64_t)NI * P * P;
    const int64_t total = rows * Kp;
    for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total; idx += (int64_t)gridDim.x * blockDim.x) {
        const int k = (int)(idx % Kp);
        const int64_t r = idx / Kp;
        float v = 0.f;
        if (k < K) {
            const int c = k / (ps * ps), kh = (k / ps) % ps, kw = k % ps;
            const int pidx = (int)(r % (P * P));
            const int64_t n = r / (P * P);
            const int py = pidx / P, pxx = pidx % P;
            v = (float)px[((n * 3 + c) * img + (int64_t)py * ps + kh) * img + (int64_t)pxx * ps + kw];
        }
        out[idx] = (bf16)v;
    }
}

// --------------------------------------------------------- embed assemble ----
// src[t] >= 0 : image feature row src[t]; -1 : image newline; -2 : token embedding of ids[t]
template <typename OT>   // bf16, or fp32 (the first value of an fp32 residual stream: exact)
__global__ void k_embed_assemble(const int64_t* __restrict__ ids, const int* __restrict__ src, const bf16* __restrict__ table,
                                 const bf16* __restrict__ feats, const bf16* __restrict__ newline, OT* __restrict__ out,
                                 int M, int H, int vocab, int* __restrict__ err) {
    const int t = blockIdx.x;
    if (t >= M) return;
    const int s = src[t];
    const bf16* from;
    if (s >= 0) from = feats + (int64_t)s * H;
    else if (s == -1) from = newline;
    else {
        const int64_t id = ids[t];
        if (id < 0 || id >= vocab) { if (threadIdx.x == 0) atomicOr(err, 1); return; }
        from = table + id * H;
    }
    for (int c = threadIdx.x * 8; c < H; c += blockDim.x * 8) {
        const bf16x8 v = *(const bf16x8*)(from + c);
        if constexpr (sizeof(OT) == 4) {
            *(f32x4*)(out + (int64_t)t * H + c) = (f32x4){(float)v[0], (float)v[1], (float)v[2], (float)v[3]};
            *(f32x4*)(out + (int64_t)t * H + c + 4) = (f32x4){(float)v[4], (float)v[5], (float)v[6], (float)v[7]};
        } else {
            *(bf16x8*)(out + (int64_t)t * H + c) = v;
        }
    }
}

__global__ void k_embed_bwd(const int64_t* __restrict__ ids, const int* __restrict__ src, const bf16* __restrict__ dout,
                            float* __restrict__ dtable, bf16* __restrict__ dfeats, float* __restrict__ dnewline, int M, int H) {
    const int t = blockIdx.x;
    if (t >= M) return;
    const int s = src[t];
    const bf16* g = dout + (int64_t)t * H;
    if (s >= 0) {
        if (dfeats)
            for (int c = threadIdx.x * 8; c < H; c += blockDim.x * 8)
                *(bf16x8*)(dfeats + (int64_t)s * H + c) = *(const bf16x8*)(g + c);
    } else if (s == -1) {
        if (dnewline)
            for (int c = threadIdx.x; c < H; c += blockDim.x) atomicAdd(dnewline + c, (float)g[c]);
    } else if (dtable) {
        float* row = dtable + ids[t] * H;
        for (int c = threadIdx.x; c < H; c += blockDim.x) atomicAdd(row + c, (float)g[c]);
    }
}

// ---------------------------------------------------------------- colsum ----
// out[n] (+)= sum_m dy[m][n] ; grid.x over 256-column groups of 8 (2048 cols), grid.y row chunks
__global__ void __launch_bounds__(256) k_colsum(const bf16* __restrict__ dy, int64_t ld, int M, int N,
                                                float* __restrict__ out, int rows_per) {
    // 32 eight-column chunks x 8 row lanes; a wave reads 2 rows x 512 contiguous bytes
    __shared__ float red[8][32 * 8 + 4];
    const int cx = threadIdx.x & 31, ry = threadIdx.x >> 5;
    const int c = (blockIdx.x * 32 + cx) * 8;
    const int r0 = blockIdx.y * rows_per, r1 = min(M, r0 + rows_per);
    float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (c < N) {
#pragma unroll 4
        for (int r = r0 + ry; r < r1; r += 8) {
            float f[8];
            load8(dy + (int64_t)r * ld + c, f);
#pragma unroll
            for (int j = 0; j < 8; ++j) s[j] += f[j];
        }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) red[ry][cx * 8 + j] = s[j];
    __syncthreads();
    const int col = threadIdx.x;   // 256 columns of the block
    float t = 0.f;
#pragma unroll
    for (int y = 0; y < 8; ++y) t += red[y][col];
    const int gc = blockIdx.x * 256 + col;
    if (gc < N) atomicAdd(out + gc, t);
}

// ------------------------------------------------------- row-group mean ----
// out[g][d] = mean_{p < P} x[g*P + p][d] (fp32)
__global__ void k_row_group_mean(const bf16* __restrict__ x, int64_t ld, int G, int P, int D, float* __restrict__ out) {
    const int gi = blockIdx.y;
    const int d = blockIdx.x * blockDim.x + threadIdx.x;
    if (d >= D || gi >= G) return;
    float s = 0.f;
    for (int p = 0; p < P; ++p) s += (float)x[((int64_t)gi * P + p) * ld + d];
    out[(int64_t)gi * D + d] = s / P;
}

// dx[g*P+p][d] = dpool[g][d] / P (broadcast)
__global__ void k_row_group_mean_bwd(const float* __restrict__ dpool, int G, int P, int D, bf16* __restrict__ dx, int64_t ld,
                                     const float* __restrict__ scale_dev) {
    const float sc = scale_dev ? *scale_dev : 1.f;
    const int64_t total = (int64_t)G * P * D;
    for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total; idx += (int64_t)gridDim.x * blockDim.x) {
        const int d = (int)(idx % D);
        const int64_t r = idx / D;
        const int g = (int)(r / P);
        dx[r * ld + d] = (bf16)(dpool[(int64_t)g * D + d] * sc / P);
    }
}

// ---------------------------------------------------------------- NT-Xent ----
// one workgroup; n <= 64 features of dim D.  fs/ft pooled (pre-normalisation) student /
// teacher features.  DT:246-248 normalises once, contrastive_loss normalises again
// (idempotent up to rounding; both applied).  loss = CE(S T^T / tau, arange).
// FEATS_LDS: the normalised features are staged in LDS (2 n D floats, n <= 16 at D = 1152);
// otherwise every read recomputes x / n1 / n2 from the (L2-resident) inputs — the same
// arithmetic, so both builds give identical results.
template <bool FEATS_LDS>
__global__ void __launch_bounds__(NT) k_ntxent(const float* __restrict__ fs, const float* __restrict__ ft, int n, int D,
                                               float tau, float weight, float* __restrict__ loss_out,
                                               float* __restrict__ dfs, float grad_scale) {
    extern __shared__ __attribute__((aligned(16))) float sm[];  // logits[n][n], norms[4n](, s_hat[n][D], t_hat[n][D])
    float* lg = sm;
    float* nrm = lg + n * n;  // [4n]: |fs|, |s1|, |ft|, |t1|
    float* sh = nrm + 4 * n;
    float* th = sh + n * D;
    auto SH = [&](int i, int d) -> float {
        return FEATS_LDS ? sh[i * D + d] : fs[(int64_t)i * D + d] / nrm[i] / nrm[n + i];
    };
    auto TH = [&](int j, int d) -> float {
        return FEATS_LDS ? th[j * D + d] : ft[(int64_t)j * D + d] / nrm[2 * n + j] / nrm[3 * n + j];
    };
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    // norms (two normalisations, each x / max(|x|, 1e-12))
    for (int r = w; r < 2 * n; r += 4) {
        const float* src = r < n ? fs + (int64_t)r * D : ft + (int64_t)(r - n) * D;
        float s2 = 0.f;
        for (int d = lane; d < D; d += 64) s2 += src[d] * src[d];
        s2 = wave_sum(s2);
        const float n1 = fmaxf(sqrtf(s2), 1e-12f);
        float s3 = 0.f;
        for (int d = lane; d < D; d += 64) { const float y = src[d] / n1; s3 += y * y; }
        s3 = wave_sum(s3);
        const float n2 = fmaxf(sqrtf(s3), 1e-12f);
        if (FEATS_LDS) {
            float* dst = r < n ? sh + r * D : th + (r - n) * D;
            for (int d = lane; d < D; d += 64) dst[d] = src[d] / n1 / n2;
        }
        if (lane == 0) {
            if (r < n) { nrm[r] = n1; nrm[n + r] = n2; }
            else { nrm[2 * n + r - n] = n1; nrm[3 * n + r - n] = n2; }
        }
    }
    __syncthreads();
    for (int e = w; e < n * n; e += 4) {
        const int i = e / n, j = e % n;
        float s = 0.f;
        for (int d = lane; d < D; d += 64) s += SH(i, d) * TH(j, d);
        s = wave_sum(s);
        if (lane == 0) lg[e] = s / tau;
    }
    __syncthreads();
    // softmax rows, loss, dlogits (in place: lg <- (softmax - onehot) / n * weight)
    __shared__ float lrow[64];
    if (tid < n) {
        float m = -INFINITY;
        for (int j = 0; j < n; ++j) m = fmaxf(m, lg[tid * n + j]);
        float z = 0.f;
        for (int j = 0; j < n; ++j) z += __expf(lg[tid * n + j] - m);
        lrow[tid] = logf(z) + m - lg[tid * n + tid];
        for (int j = 0; j < n; ++j) {
            const float pj = __expf(lg[tid * n + j] - m) / z;
            lg[tid * n + j] = (pj - (j == tid ? 1.f : 0.f)) / n * weight * grad_scale;
        }
    }
    __syncthreads();
    if (tid == 0) {
        float L = 0.f;
        for (int i = 0; i < n; ++i) L += lrow[i];
        loss_out[0] = L / n * weight;
        loss_out[1] = L / n;
    }
    if (!dfs) return;
    // d s_hat_i = sum_j dlg_ij t_hat_j / tau ; then back through the two normalisations
    for (int i = w; i < n; i += 4) {
        // y = s_hat = u / n2, u = x / n1.  dL/du = (g - y (y.g)) / n2 ; dL/dx = (dL/du - u (u.dL/du)) / n1
        float yg = 0.f;
        for (int d = lane; d < D; d += 64) {
            float g = 0.f;
            for (int j = 0; j < n; ++j) g += lg[i * n + j] * TH(j, d);
            g /= tau;
            dfs[(int64_t)i * D + d] = g;  // scratch
            yg += g * SH(i, d);
        }
        yg = wave_sum(yg);
        const float n1 = nrm[i], n2 = nrm[n + i];
        float uq = 0.f;
        for (int d = lane; d < D; d += 64) {
            const float y = SH(i, d);
            const float gu = (dfs[(int64_t)i * D + d] - y * yg) / n2;
            dfs[(int64_t)i * D + d] = gu;
            uq += gu * (y * n2);  // u = y * n2
        }
        uq = wave_sum(uq);
        for (int d = lane; d < D; d += 64) {
            const float u = SH(i, d) * n2;
            dfs[(int64_t)i * D + d] = (dfs[(int64_t)i * D + d] - u * uq) / n1;
        }
    }
}

// ---------------------------------------------------------------- AdamW ----
// torch.optim.AdamW semantics: p -= lr*wd*p; m = b1 m + (1-b1) g; v = b2 v + (1-b2) g^2;
// p -= (lr / (1-b1^t)) * m / (sqrt(v) / sqrt(1-b2^t) + eps).  Master fp32, working copy bf16.
template <int U, bool NTL, bool CW = false>
__global__ void k_adamw(float* __restrict__ p, bf16* __restrict__ pb, const float* __restrict__ g, float* __restrict__ m,
                        float* __restrict__ v, int64_t n, float lr, float b1, float b2, float eps, float wd,
                        float bc1, float inv_bc2s, const float* __restrict__ gscale, const int32_t* __restrict__ skip,
                        int n_skip) {
    // a step whose batch raised a device error (the sticky error words of the step, see
    // kd_adamw) leaves every weight and moment untouched
    int bad = 0;
    for (int j = 0; j < n_skip; ++j) bad |= skip[j];
    if (bad) return;
    const float gs = gscale ? *gscale : 1.f;
    // torch.optim.AdamW's order (step_size = lr / bc1, denom = sqrt(v) / sqrt(bc2) + eps, p -=
    // step_size * m / denom) with the two per-element IEEE divisions and the correctly rounded sqrt
    // replaced by v_sqrt_f32, v_rcp_f32 and the host's reciprocal of sqrt(bc2): 55 -> ~14 VALU per
    // parameter, which held the kernel below the HBM rate.  m and v are computed as before (same
    // bits); the update term moves by a few ulp of itself, ~1e-3 of an ulp of p at lr 1e-3
    // (tests/test_layers_gpu.py::test_adamw_matches_torch: p to 1e-6, the bf16 copy exactly)
    const float step_size = lr / bc1;   // inv_bc2s = 1 / sqrt(1 - b2^t), from the host
    auto step = [&](float& pi, float& mi, float& vi, float graw) {
        const float gi = graw * gs;
        pi = pi * (1.f - lr * wd);
        mi = b1 * mi + (1.f - b1) * gi;
        vi = b2 * vi + (1.f - b2) * gi * gi;
        const float denom = fmaf(__builtin_amdgcn_sqrtf(vi), inv_bc2s, eps);
        pi = fmaf(-step_size, mi * __builtin_amdgcn_rcpf(denom), pi);
    };
    // 4 parameters per thread and iteration: 16-B loads / stores of p, g, m, v, 8-B bf16 stores
    // (same per-element arithmetic as the scalar tail)
    const bool vec = (((uintptr_t)p | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v) & 15) == 0 && ((uintptr_t)pb & 7) == 0;
    const int64_t n4 = vec ? n >> 2 : 0;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    // U chunks per thread and iteration, every load issued before the first store (a small grid
    // -- KD_ADAMW_GRID -- then still keeps 16 x 16 B in flight per lane)
    auto ld = [](const float* a, int64_t i) {
        if constexpr (NTL) return __builtin_nontemporal_load((const f32x4*)a + i);
        else return *((const f32x4*)a + i);
    };
    // CW: each wave owns contiguous runs of U x 64 16-B chunks (U KiB of every tensor) instead of
    // lane-strided chunks a grid apart
    const int64_t wgl = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6, nw = stride >> 6;
    const int lane = threadIdx.x & 63;
    if (CW) i0 = wgl * 64 * U + lane;
    const int64_t ustep = CW ? 64 : stride, istep = CW ? nw * 64 * U : U * stride;
    for (; i0 + (U - 1) * ustep < n4; i0 += istep) {
        f32x4 pv[U], mv[U], vv[U], gv[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t i = i0 + u * ustep;
            pv[u] = ld(p, i);
            mv[u] = ld(m, i);
            vv[u] = ld(v, i);
            gv[u] = ld(g, i);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t i = i0 + u * ustep;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                float pe = pv[u][e], me = mv[u][e], ve = vv[u][e];
                step(pe, me, ve, gv[u][e]);
                pv[u][e] = pe;
                mv[u][e] = me;
                vv[u][e] = ve;
            }
            const bf16x4 pbv = bf16x4{(bf16)pv[u][0], (bf16)pv[u][1], (bf16)pv[u][2], (bf16)pv[u][3]};
            __builtin_nontemporal_store(mv[u], (f32x4*)m + i);
            __builtin_nontemporal_store(vv[u], (f32x4*)v + i);
            __builtin_nontemporal_store(pv[u], (f32x4*)p + i);
            __builtin_nontemporal_store(pbv, (bf16x4*)pb + i);
        }
    }
    for (int64_t i = i0; i < n4; i += ustep) {
        // every byte is touched once: non-temporal loads / stores (4.79 -> 4.65 ms for 894 M
        // parameters, tools/bench_adamw.py)
        f32x4 pv = __builtin_nontemporal_load((const f32x4*)p + i), mv = __builtin_nontemporal_load((const f32x4*)m + i);
        f32x4 vv = __builtin_nontemporal_load((const f32x4*)v + i);
        const f32x4 gv = __builtin_nontemporal_load((const f32x4*)g + i);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            float pe = pv[e], me = mv[e], ve = vv[e];
            step(pe, me, ve, gv[e]);
            pv[e] = pe;
            mv[e] = me;
            vv[e] = ve;
        }
        const bf16x4 pbv = bf16x4{(bf16)pv[0], (bf16)pv[1], (bf16)pv[2], (bf16)pv[3]};
        __builtin_nontemporal_store(mv, (f32x4*)m + i);
        __builtin_nontemporal_store(vv, (f32x4*)v + i);
        __builtin_nontemporal_store(pv, (f32x4*)p + i);
        __builtin_nontemporal_store(pbv, (bf16x4*)pb + i);
    }
    for (int64_t i = (n4 << 2) + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        float pi = p[i], mi = m[i], vi = v[i];
        step(pi, mi, vi, g[i]);
        m[i] = mi;
        v[i] = vi;
        p[i] = pi;
        pb[i] = (bf16)pi;
    }
}

__global__ void k_sumsq(const float* __restrict__ x, int64_t n, float* __restrict__ out) {
    __shared__ float red[4];
    float s = 0.f;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) s += x[i] * x[i];
    s = block_sum<4>(s, red);
    if (threadIdx.x == 0) atomicAdd(out, s);
}

// y = x * (*s) (s may be NULL: a copy); y may alias x
__global__ void k_scale_f32(const float* x, const float* __restrict__ s, float* y, int64_t n) {
    const float sc = s ? *s : 1.f;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) y[i] = x[i] * sc;
}

__global__ void k_scalar_mul(const float* __restrict__ a, const float* __restrict__ b, float* __restrict__ out, int n) {
    const int i = threadIdx.x;
    if (i < n) out[i] = a[i] * b[i];
}

__global__ void k_cast_f32_bf16(const float* __restrict__ x, bf16* __restrict__ y, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) y[i] = (bf16)x[i];
}

__global__ void k_cast_bf16_f32(const bf16* __restrict__ x, float* __restrict__ y, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) y[i] = (float)x[i];
}

// src[b*L + l] for inputs_embeds assembly: the j-th image token of sample b takes
// map[b*map_ld + j] (a packed feature row, or -1 for image_newline); text tokens -2.
// Counts that differ from map_len[b] flag err (HF raises "Image features and image tokens
// do not match", HF5 llava_onevision :460-470).  One workgroup per sample.
__global__ void __launch_bounds__(256) k_image_src_map(const int64_t* __restrict__ ids, int L, int64_t image_token,
                                                       const int* __restrict__ map, int map_ld,
                                                       const int* __restrict__ map_len, int* __restrict__ src,
                                                       int* __restrict__ err) {
    __shared__ int counts[256];
    const int b = blockIdx.x, t = threadIdx.x;
    const int per = (L + 255) / 256;
    const int l0 = t * per, l1 = min(L, l0 + per);
    int c = 0;
    for (int l = l0; l < l1; ++l) c += (ids[(int64_t)b * L + l] == image_token);
    counts[t] = c;
    __syncthreads();
    // inclusive scan (Hillis-Steele)
    for (int o = 1; o < 256; o <<= 1) {
        const int v = t >= o ? counts[t - o] : 0;
        __syncthreads();
        counts[t] += v;
        __syncthreads();
    }
    int j = counts[t] - c;  // exclusive prefix
    const int n = map_len[b];
    for (int l = l0; l < l1; ++l) {
        const int64_t id = ids[(int64_t)b * L + l];
        int sv = -2;
        if (id == image_token) {
            sv = j < n ? map[(int64_t)b * map_ld + j] : -2;
            ++j;
        }
        src[(int64_t)b * L + l] = sv;
    }
    if (t == 255 && counts[255] != n) atomicOr(err, 2);
}

inline int grid_for(int64_t work, int per_block = 256, int cap = 8192) {
    int64_t g = (work + per_block - 1) / per_block;
    return (int)(g < 1 ? 1 : (g > cap ? cap : g));
}

}  // namespace

// ------------------------------------------------------------------ launchers ----
int launch_norm_fwd(int rms, const void* x, int64_t ldx, const void* w, const void* b, void* y, int64_t ldy,
                    float* mean, float* rstd, int R, int D, float eps, void* stream, int x_f32) {
    KD_CHECK_ARG(x && w && y && (rms || b), "norm_fwd: null pointer");
    KD_CHECK_SHAPE(D % 8 == 0 && D <= 4096 && ldx % 8 == 0 && ldy % 8 == 0, "norm_fwd: D must be a multiple of 8, <= 4096");
    const dim3 grid((R + 3) / 4);
    hipStream_t st = as_stream(stream);
    // KD_NORM_FWD_V=1 (read per call): the previous kernel, for A/B
    if (ab_knob("KD_NORM_FWD_V", 2) != 1) {
        const int it = (D / 8 + 63) / 64;
#define KD_NF2(ITV)                                                                                                   \
    do {                                                                                                               \
        if (x_f32) {                                                                                                   \
            if (rms) hipLaunchKernelGGL((k_norm_fwd2<true, ITV, float>), grid, dim3(NT), 0, st, (const float*)x, ldx,   \
                                        (const bf16*)w, nullptr, (bf16*)y, ldy, mean, rstd, R, D, eps);                \
            else hipLaunchKernelGGL((k_norm_fwd2<false, ITV, float>), grid, dim3(NT), 0, st, (const float*)x, ldx,      \
                                    (const bf16*)w, (const bf16*)b, (bf16*)y, ldy, mean, rstd, R, D, eps);             \
        } else {                                                                                                       \
            if (rms) hipLaunchKernelGGL((k_norm_fwd2<true, ITV, bf16>), grid, dim3(NT), 0, st, (const bf16*)x, ldx,     \
                                        (const bf16*)w, nullptr, (bf16*)y, ldy, mean, rstd, R, D, eps);                \
            else hipLaunchKernelGGL((k_norm_fwd2<false, ITV, bf16>), grid, dim3(NT), 0, st, (const bf16*)x, ldx,        \
                                    (const bf16*)w, (const bf16*)b, (bf16*)y, ldy, mean, rstd, R, D, eps);             \
        }                                                                                                              \
    } while (0)
        switch (it) {
            case 1: KD_NF2(1); break;
            case 2: KD_NF2(2); break;
            case 3: KD_NF2(3); break;
            case 4: KD_NF2(4); break;
            case 5: KD_NF2(5); break;
            case 6: KD_NF2(6); break;
            case 7: KD_NF2(7); break;
            default: KD_NF2(8); break;
        }
#undef KD_NF2
        KD_LAUNCH_CHECK("k_norm_fwd2");
        return KD_OK;
    }
    if (x_f32) {
        if (rms) hipLaunchKernelGGL((k_norm_fwd<true, float>), grid, dim3(NT), 0, st, (const float*)x, ldx, (const bf16*)w,
                                    nullptr, (bf16*)y, ldy, mean, rstd, R, D, eps);
        else hipLaunchKernelGGL((k_norm_fwd<false, float>), grid, dim3(NT), 0, st, (const float*)x, ldx, (const bf16*)w,
                                (const bf16*)b, (bf16*)y, ldy, mean, rstd, R, D, eps);
    } else {
        if (rms) hipLaunchKernelGGL((k_norm_fwd<true, bf16>), grid, dim3(NT), 0, st, (const bf16*)x, ldx, (const bf16*)w,
                                    nullptr, (bf16*)y, ldy, mean, rstd, R, D, eps);
        else hipLaunchKernelGGL((k_norm_fwd<false, bf16>), grid, dim3(NT), 0, st, (const bf16*)x, ldx, (const bf16*)w,
                                (const bf16*)b, (bf16*)y, ldy, mean, rstd, R, D, eps);
    }
    KD_LAUNCH_CHECK("k_norm_fwd");
    return KD_OK;
}

// workgroups of k_norm_bwd: ~8 rows each (2 per wave), at most 512 (2 per CU)
static int norm_bwd_blocks(int R) {
    static const int cap = ab_knob("KD_NORM_BWD_BLOCKS", 512);
    return std::max(1, std::min(cap, (R + 7) / 8));
}

size_t norm_bwd_ws(int R, int D) {
    return (size_t)norm_bwd_blocks(R) * D * 4 * 2;
}

int launch_norm_bwd(int rms, const void* x, int64_t ldx, const void* w, const void* dy, int64_t lddy, const float* mean,
                    const float* rstd, void* dx, int64_t lddx, int dx_accum, float* dw, float* db, int accum_w,
                    void* ws, size_t ws_bytes, int R, int D, void* stream, int x_f32, int dy_group) {
    KD_CHECK_ARG(x && w && dy && rstd && dx && (rms || mean), "norm_bwd: null pointer");
    KD_CHECK_ARG(dy_group == 0 || (!rms && dy_group > 0 && R % dy_group == 0 && (uintptr_t)dy % 16 == 0 && lddy % 4 == 0),
                 "norm_bwd: a grouped fp32 dy is for LayerNorm, rows a multiple of the group, 16-B rows");
    KD_CHECK_SHAPE(D % 8 == 0 && D <= 2048, "norm_bwd: D must be a multiple of 8, <= 2048");
    const int nb = norm_bwd_blocks(R);
    const int rows_per = (R + nb - 1) / nb;
    if (ws_bytes < (size_t)nb * D * 8) return fail(KD_ERR_WORKSPACE, "norm_bwd: workspace");
    float* dwp = (float*)ws;
    float* dbp = dwp + (size_t)nb * D;
    hipStream_t st = as_stream(stream);
    const size_t smem = (size_t)NW_NORM * 2 * D * 4;
#define KD_NB(RMSV, ITV)                                                                                          \
    do {                                                                                                           \
        if (dy_group && !RMSV) {                                                                                   \
            if (x_f32)                                                                                             \
                hipLaunchKernelGGL((k_norm_bwd<false, ITV, float, true>), dim3(nb), dim3(NT), smem, st,              \
                                   (const float*)x, ldx, (const bf16*)w, dy, lddy, mean, rstd, (bf16*)dx, lddx,       \
                                   dx_accum, dw ? dwp : nullptr, db ? dbp : nullptr, R, D, rows_per, dy_group,        \
                                   1.f / dy_group);                                                                 \
            else                                                                                                   \
                hipLaunchKernelGGL((k_norm_bwd<false, ITV, bf16, true>), dim3(nb), dim3(NT), smem, st,               \
                                   (const bf16*)x, ldx, (const bf16*)w, dy, lddy, mean, rstd, (bf16*)dx, lddx,        \
                                   dx_accum, dw ? dwp : nullptr, db ? dbp : nullptr, R, D, rows_per, dy_group,        \
                                   1.f / dy_group);                                                                 \
        } else if (x_f32)                                                                                          \
            hipLaunchKernelGGL((k_norm_bwd<RMSV, ITV, float>), dim3(nb), dim3(NT), smem, st, (const float*)x, ldx,   \
                               (const bf16*)w, dy, lddy, mean, rstd, (bf16*)dx, lddx, dx_accum,                      \
                               dw ? dwp : nullptr, (RMSV || !db) ? nullptr : dbp, R, D, rows_per);                 \
        else                                                                                                       \
            hipLaunchKernelGGL((k_norm_bwd<RMSV, ITV, bf16>), dim3(nb), dim3(NT), smem, st, (const bf16*)x, ldx,     \
                               (const bf16*)w, dy, lddy, mean, rstd, (bf16*)dx, lddx, dx_accum,                      \
                               dw ? dwp : nullptr, (RMSV || !db) ? nullptr : dbp, R, D, rows_per);                 \
    } while (0)
    const int it = (D + 511) / 512;
    if (rms) {
        if (it == 1) KD_NB(true, 1); else if (it == 2) KD_NB(true, 2); else if (it == 3) KD_NB(true, 3); else KD_NB(true, 4);
    } else {
        if (it == 1) KD_NB(false, 1); else if (it == 2) KD_NB(false, 2); else if (it == 3) KD_NB(false, 3); else KD_NB(false, 4);
    }
#undef KD_NB
    KD_LAUNCH_CHECK("k_norm_bwd");
    if (dw) hipLaunchKernelGGL(k_reduce_parts, dim3((D + RP_C - 1) / RP_C), dim3(1024), 0, st, dwp, nb, D, dw, accum_w);
    if (db) hipLaunchKernelGGL(k_reduce_parts, dim3((D + RP_C - 1) / RP_C), dim3(1024), 0, st, dbp, nb, D, db, accum_w);
    KD_LAUNCH_CHECK("k_reduce_parts");
    return KD_OK;
}

int launch_qkv_split(const void* qkv, int64_t ld, void* q, void* k, void* v, const float* cos_t, const float* sin_t,
                     int B, int S, int nq, int nkv, int hd, int hdp, void* stream) {
    KD_CHECK_ARG(qkv && q && k && v, "qkv_split: null pointer");
    KD_CHECK_SHAPE(hd % 2 == 0 && hdp >= hd && hdp % 2 == 0, "qkv_split: head dims");
    const int hh = hd / 2;
    auto ok = [&](int vec) {
        const uintptr_t al = (uintptr_t)vec * 2 - 1;
        return hh % vec == 0 && (hdp - hd) % vec == 0 && ld % vec == 0 && hdp % vec == 0 &&
               !((uintptr_t)qkv & al) && !((uintptr_t)q & al) && !((uintptr_t)k & al) && !((uintptr_t)v & al);
    };
    const int vec = ok(8) ? 8 : ok(4) ? 4 : ok(2) ? 2 : 1;
    const int64_t work = (int64_t)B * S * (nq + 2 * nkv) * (hh / vec + (hdp - hd) / vec);
#define LQS(VEC)                                                                                                 \
    hipLaunchKernelGGL(k_qkv_split<VEC>, dim3(grid_for(work)), dim3(256), 0, as_stream(stream), (const bf16*)qkv, ld, \
                       (bf16*)q, (bf16*)k, (bf16*)v, cos_t, sin_t, B, S, nq, nkv, hd, hdp)
    if (vec == 8) LQS(8); else if (vec == 4) LQS(4); else if (vec == 2) LQS(2); else LQS(1);
#undef LQS
    KD_LAUNCH_CHECK("k_qkv_split");
    return KD_OK;
}

int launch_qkv_merge(const float* dq, const void* dk, const void* dv, void* dqkv, int64_t ld, const float* cos_t,
                     const float* sin_t, int B, int S, int nq, int nkv, int hd, int hdp, void* stream) {
    KD_CHECK_ARG(dq && dk && dv && dqkv, "qkv_merge: null pointer");
    KD_CHECK_SHAPE(hd % 2 == 0 && hdp >= hd, "qkv_merge: head dims");
    const int hh = hd / 2;
    auto ok = [&](int vec) {
        const uintptr_t al = (uintptr_t)vec * 2 - 1;
        return hh % vec == 0 && ld % vec == 0 && hdp % vec == 0 && !((uintptr_t)dqkv & al) && !((uintptr_t)dk & al) &&
               !((uintptr_t)dv & al);
    };
    const int vec = ok(8) ? 8 : ok(4) ? 4 : ok(2) ? 2 : 1;
    const int64_t work = (int64_t)B * S * (nq + 2 * nkv) * (hh / vec);
#define LQM(VEC)                                                                                                   \
    hipLaunchKernelGGL(k_qkv_merge<VEC>, dim3(grid_for(work)), dim3(256), 0, as_stream(stream), dq, (const bf16*)dk, \
                       (const bf16*)dv, (bf16*)dqkv, ld, cos_t, sin_t, B, S, nq, nkv, hd, hdp)
    if (vec == 8) LQM(8); else if (vec == 4) LQM(4); else if (vec == 2) LQM(2); else LQM(1);
#undef LQM
    KD_LAUNCH_CHECK("k_qkv_merge");
    return KD_OK;
}

int launch_swiglu_fwd(const void* gu, int64_t ldg, void* h, int64_t ldh, int M, int I, void* stream) {
    KD_CHECK_ARG(gu && h, "swiglu_fwd: null pointer");
    KD_CHECK_SHAPE(I % 8 == 0 && ldg % 8 == 0 && ldh % 8 == 0, "swiglu_fwd: I % 8");
    hipLaunchKernelGGL(k_swiglu_fwd, dim3(grid_for((int64_t)M * I / 8)), dim3(256), 0, as_stream(stream), (const bf16*)gu,
                       ldg, (bf16*)h, ldh, M, I);
    KD_LAUNCH_CHECK("k_swiglu_fwd");
    return KD_OK;
}

int launch_swiglu_bwd(const void* gu, int64_t ldg, const void* dh, int64_t ldh, void* dgu, int64_t ldd, int M, int I,
                      void* stream) {
    KD_CHECK_ARG(gu && dh && dgu, "swiglu_bwd: null pointer");
    KD_CHECK_SHAPE(I % 8 == 0, "swiglu_bwd: I % 8");
    hipLaunchKernelGGL(k_swiglu_bwd, dim3(grid_for((int64_t)M * I / 8)), dim3(256), 0, as_stream(stream), (const bf16*)gu,
                       ldg, (const bf16*)dh, ldh, (bf16*)dgu, ldd, M, I);
    KD_LAUNCH_CHECK("k_swiglu_bwd");
    return KD_OK;
}

int launch_act_bwd(const void* pre, const void* dy, void* dx, int64_t n, int act, void* stream) {
    KD_CHECK_ARG(pre && dy && dx, "act_bwd: null pointer");
    KD_CHECK_SHAPE(n % 8 == 0, "act_bwd: n % 8");
    KD_CHECK_ARG(act >= KD_ACT_GELU_TANH && act <= KD_ACT_SILU, "act_bwd: act");
    hipLaunchKernelGGL(k_act_bwd, dim3(grid_for(n / 8)), dim3(256), 0, as_stream(stream), (const bf16*)pre,
                       (const bf16*)dy, (bf16*)dx, n, act);
    KD_LAUNCH_CHECK("k_act_bwd");
    return KD_OK;
}

int launch_patchify(const void* px, int px_dtype, void* out, int NI, int img, int ps, int Kp, void* stream) {
    KD_CHECK_ARG(px && out, "patchify: null pointer");
    KD_CHECK_SHAPE(img >= ps && Kp >= 3 * ps * ps, "patchify: shape");  // conv floors: 384/14 -> 27
    const int64_t work = (int64_t)NI * (img / ps) * (img / ps) * Kp;
    if (px_dtype == KD_DTYPE_F32)
        hipLaunchKernelGGL(k_patchify<float>, dim3(grid_for(work)), dim3(256), 0, as_stream(stream), (const float*)px,
                           (bf16*)out, NI, img, ps, Kp);
    else
        hipLaunchKernelGGL(k_patchify<bf16>, dim3(grid_for(work)), dim3(256), 0, as_stream(stream), (const bf16*)px,
                           (bf16*)out, NI, img, ps, Kp);
    KD_LAUNCH_CHECK("k_patchify");
    return KD_OK;
}

int launch_embed_assemble(const int64_t* ids, const int* src, const void* table, const void* feats, const void* newline,
                          void* out, int M, int H, int vocab, int* err, void* stream, int out_f32) {
    KD_CHECK_ARG(ids && src && table && out && err, "embed_assemble: null pointer");
    KD_CHECK_SHAPE(H % 8 == 0, "embed_assemble: H % 8");
    if (out_f32)
        hipLaunchKernelGGL(k_embed_assemble<float>, dim3(M), dim3(128), 0, as_stream(stream), ids, src, (const bf16*)table,
                           (const bf16*)feats, (const bf16*)newline, (float*)out, M, H, vocab, err);
    else
        hipLaunchKernelGGL(k_embed_assemble<bf16>, dim3(M), dim3(128), 0, as_stream(stream), ids, src, (const bf16*)table,
                           (const bf16*)feats, (const bf16*)newline, (bf16*)out, M, H, vocab, err);
    KD_LAUNCH_CHECK("k_embed_assemble");
    return KD_OK;
}

int launch_embed_bwd(const int64_t* ids, const int* src, const void* dout, float* dtable, void* dfeats, float* dnewline,
                     int M, int H, void* stream) {
    KD_CHECK_ARG(ids && src && dout, "embed_bwd: null pointer");
    hipLaunchKernelGGL(k_embed_bwd, dim3(M), dim3(128), 0, as_stream(stream), ids, src, (const bf16*)dout, dtable,
                       (bf16*)dfeats, dnewline, M, H);
    KD_LAUNCH_CHECK("k_embed_bwd");
    return KD_OK;
}

int launch_colsum(const void* dy, int64_t ld, int M, int N, float* out, int accumulate, void* stream) {
    KD_CHECK_ARG(dy && out, "colsum: null pointer");
    KD_CHECK_SHAPE(N % 8 == 0 && ld % 8 == 0, "colsum: N % 8");
    hipStream_t st = as_stream(stream);
    if (!accumulate && hipMemsetAsync(out, 0, (size_t)N * 4, st) != hipSuccess) return fail(KD_ERR_LAUNCH, "colsum memset");
    const int rows_per = 64;
    dim3 grid((N + 255) / 256, (M + rows_per - 1) / rows_per);
    hipLaunchKernelGGL(k_colsum, grid, dim3(256), 0, st, (const bf16*)dy, ld, M, N, out, rows_per);
    KD_LAUNCH_CHECK("k_colsum");
    return KD_OK;
}

int launch_row_group_mean(const void* x, int64_t ld, int G, int P, int D, float* out, void* stream) {
    KD_CHECK_ARG(x && out, "row_group_mean: null pointer");
    hipLaunchKernelGGL(k_row_group_mean, dim3((D + 255) / 256, G), dim3(256), 0, as_stream(stream), (const bf16*)x, ld, G, P,
                       D, out);
    KD_LAUNCH_CHECK("k_row_group_mean");
    return KD_OK;
}

int launch_row_group_mean_bwd(const float* dpool, int G, int P, int D, void* dx, int64_t ld, const float* scale_dev,
                              void* stream) {
    KD_CHECK_ARG(dpool && dx, "row_group_mean_bwd: null pointer");
    hipLaunchKernelGGL(k_row_group_mean_bwd, dim3(grid_for((int64_t)G * P * D)), dim3(256), 0, as_stream(stream), dpool, G,
                       P, D, (bf16*)dx, ld, scale_dev);
    KD_LAUNCH_CHECK("k_row_group_mean_bwd");
    return KD_OK;
}

int launch_ntxent(const float* fs, const float* ft, int n, int D, float tau, float weight, float* loss_out, float* dfs,
                  float grad_scale, void* stream) {
    KD_CHECK_ARG(fs && ft && loss_out, "ntxent: null pointer");
    KD_CHECK_SHAPE(n >= 1 && n <= 64, "ntxent: 1 <= n <= 64");
    KD_CHECK_SHAPE(D >= 1, "ntxent: D >= 1");
    const size_t small = ((size_t)n * n + 4 * n) * 4, full = small + (size_t)2 * n * D * 4;
    if (full <= 160 * 1024)
        hipLaunchKernelGGL(k_ntxent<true>, dim3(1), dim3(NT), full, as_stream(stream), fs, ft, n, D, tau, weight,
                           loss_out, dfs, grad_scale);
    else
        hipLaunchKernelGGL(k_ntxent<false>, dim3(1), dim3(NT), small, as_stream(stream), fs, ft, n, D, tau, weight,
                           loss_out, dfs, grad_scale);
    KD_LAUNCH_CHECK("k_ntxent");
    return KD_OK;
}

int launch_adamw(float* p, void* pb, const float* g, float* m, float* v, int64_t n, float lr, float b1, float b2,
                 float eps, float wd, int step, const float* gscale, const int32_t* skip, int n_skip, void* stream) {
    KD_CHECK_ARG(p && pb && g && m && v && step >= 1, "adamw: bad argument");
    KD_CHECK_ARG(n_skip >= 0 && n_skip <= 64 && (n_skip == 0 || skip), "adamw: bad skip words");
    const float bc1 = 1.f - powf(b1, (float)step);
    const float inv_bc2s = (float)(1.0 / std::sqrt((double)(1.f - powf(b2, (float)step))));   // 1 / sqrt(bias correction 2)
    // The workgroup count: two 256-thread workgroups per CU (512 on MI355X), grid-striding over the
    // parameters.  Round 5: against the former 16384 (one per 4 K parameters) AdamW alone runs 4.97
    // instead of 5.24 ms (5.4 vs 5.1 TB/s), and beside the next teacher forward the c1 step gains
    // 0.4-0.8 % on three boxes (`profiles/r05/adamw_grid.txt`); 128 / 256 / 768 / 1024 measured
    // slower.  KD_ADAMW_GRID (A/B library, read per call) overrides it.
    static int cus = 0;
    if (cus == 0) {
        int dev = 0, c = 0;
        if (hipGetDevice(&dev) == hipSuccess &&
            hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && c > 0)
            cus = c;
        else
            cus = 256;
    }
    int grid = grid_for(n, 256, 2 * cus);
    if (const int cap = ab_knob("KD_ADAMW_GRID", 0); cap > 0) grid = std::min(grid_for(n, 256, 16384), cap);
    // eight 16-B chunks of each tensor in flight per lane (tools/bench_adamw.py, one box: 5.13-5.15 ms
    // vs 5.22-5.28 with four; the CW build -- each wave on contiguous 8 KiB runs -- 5.08-5.16, not kept)
#define KD_ADAMW_LAUNCH(U, NTL, CW)                                                                                   \
    hipLaunchKernelGGL((k_adamw<U, NTL, CW>), dim3(grid), dim3(256), 0, as_stream(stream), p, (bf16*)pb, g, m, v, n, \
                       lr, b1, b2, eps, wd, bc1, inv_bc2s, gscale, skip, n_skip)
#ifdef KD_AB_BUILD
    // KD_ADAMW_V: 1 = four chunks, temporal loads; 2 = two chunks; 3 = four; 4 = eight, contiguous per wave
    const int av = ab_knob("KD_ADAMW_V", 0);
    if (av == 1) KD_ADAMW_LAUNCH(4, false, false);
    else if (av == 2) KD_ADAMW_LAUNCH(2, true, false);
    else if (av == 3) KD_ADAMW_LAUNCH(4, true, false);
    else if (av == 4) KD_ADAMW_LAUNCH(8, true, true);
    else
#endif
    KD_ADAMW_LAUNCH(8, true, false);
#undef KD_ADAMW_LAUNCH
    KD_LAUNCH_CHECK("k_adamw");
    return KD_OK;
}

int launch_image_src_map(const int64_t* ids, int B, int L, int64_t image_token, const int* map, int map_ld,
                         const int* map_len, int* src, int* err, void* stream) {
    KD_CHECK_ARG(ids && map && map_len && src && err, "image_src_map: null pointer");
    hipLaunchKernelGGL(k_image_src_map, dim3(B), dim3(256), 0, as_stream(stream), ids, L, image_token, map, map_ld,
                       map_len, src, err);
    KD_LAUNCH_CHECK("k_image_src_map");
    return KD_OK;
}

int launch_sumsq(const float* x, int64_t n, float* out, void* stream) {
    KD_CHECK_ARG(x && out, "sumsq: null pointer");
    hipLaunchKernelGGL(k_sumsq, dim3(grid_for(n, 256, 2048)), dim3(256), 0, as_stream(stream), x, n, out);
    KD_LAUNCH_CHECK("k_sumsq");
    return KD_OK;
}

int launch_scale_f32(const float* x, const float* s_dev, float* y, int64_t n, void* stream) {
    KD_CHECK_ARG(x && y, "scale_f32: null pointer");
    KD_CHECK_SHAPE(n >= 0, "scale_f32: n < 0");
    if (n == 0) return KD_OK;
    hipLaunchKernelGGL(k_scale_f32, dim3((unsigned)std::min<int64_t>((n + 255) / 256, 4096)), dim3(256), 0, as_stream(stream),
                       x, s_dev, y, n);
    KD_LAUNCH_CHECK("k_scale_f32");
    return KD_OK;
}

int launch_scalar_mul(const float* a, const float* b, float* out, int n, void* stream) {
    KD_CHECK_ARG(a && b && out, "scalar_mul: null pointer");
    KD_CHECK_SHAPE(n >= 0 && n <= 1024, "scalar_mul: n must be in [0, 1024]");
    if (n == 0) return KD_OK;
    hipLaunchKernelGGL(k_scalar_mul, dim3(1), dim3(n), 0, as_stream(stream), a, b, out, n);
    KD_LAUNCH_CHECK("k_scalar_mul");
    return KD_OK;
}

int launch_cast_bf16_f32(const void* x, float* y, int64_t n, void* stream) {
    KD_CHECK_ARG(x && y, "cast: null pointer");
    hipLaunchKernelGGL(k_cast_bf16_f32, dim3(grid_for(n, 256, 16384)), dim3(256), 0, as_stream(stream), (const bf16*)x, y, n);
    KD_LAUNCH_CHECK("k_cast_bf16_f32");
    return KD_OK;
}

// Read `bytes` once (16-B loads, grid-strided) so they sit in the Infinity Cache / L2 for the next
// kernel (kd_prefetch): the step reads each weight a whole step after its last use, and a GEMM that
// meets cold weights stalls on them tile by tile; a streaming read moves them at full HBM rate.
__global__ void k_prefetch(const u32x4* __restrict__ p, int64_t n16) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (int64_t)gridDim.x * blockDim.x) {
        const u32x4 v = p[i];
        asm volatile("" ::"v"(v));   // keep the load
    }
}

int launch_prefetch(const void* ptr, uint64_t bytes, int grid, void* stream) {
    KD_CHECK_ARG(ptr != nullptr, "prefetch: null pointer");
    KD_CHECK_ALIGN(ptr, 16, "prefetch: 16-B aligned");
    const int64_t n16 = (int64_t)(bytes / 16);
    if (n16 == 0) return KD_OK;
    const int g = grid > 0 ? grid : (int)std::min<int64_t>((n16 + 255) / 256, 1024);
    hipLaunchKernelGGL(k_prefetch, dim3(g), dim3(256), 0, as_stream(stream), (const u32x4*)ptr, n16);
    KD_LAUNCH_CHECK("k_prefetch");
    return KD_OK;
}

int launch_cast_f32_bf16(const float* x, void* y, int64_t n, void* stream) {
    KD_CHECK_ARG(x && y, "cast: null pointer");
    hipLaunchKernelGGL(k_cast_f32_bf16, dim3(grid_for(n, 256, 16384)), dim3(256), 0, as_stream(stream), x, (bf16*)y, n);
    KD_LAUNCH_CHECK("k_cast_f32_bf16");
    return KD_OK;
}

}  // namespace kd
