// bf16 MFMA GEMM for gfx950:  C[M,N] = epilogue( alpha * sum_k A[m,k] * B[n,k] )
//
// Every nn.Linear of the step runs here (SigLIP q/k/v/out/fc1/fc2, projector, Qwen2
// q/k/v/o/gate/up/down, lm_head; forward, dgrad and wgrad) — the reference reaches
// them through torch.nn.functional.linear inside transformers.
//
// Operand layouts (no transpose kernels anywhere):
//   K-major  : operand row r at ptr + r*ld, its K elements contiguous   (forward X, W)
//   MN-major : operand stored [K][rows], rows contiguous                (backward dY, X, W)
// Forward  Y  = X W^T      : A=X  K-major,  B=W  K-major
// Dgrad    dX = dY W       : A=dY K-major,  B=W  MN-major (W[n][k] is [K'=n][rows'=k])
// Wgrad    dW = dY^T X     : A=dY MN-major, B=X  MN-major
//
// Tile 128x128x64, 256 threads = 4 waves (2x2), each wave 64x64 = 4x4 MFMA 16x16x32
// tiles.  Global->LDS by LDS-DMA (buffer_load ... lds, 16 B per lane) into two LDS
// buffers; the next K-tile's DMA is in flight while the current one is consumed.
// Buffer descriptors give zeros out of range, which handles every M/N/K tail.
// LDS images are XOR-swizzled on the SOURCE address (the DMA destination is
// lane-linear): K-major tiles [128 rows][64 k] read by ds_read_b128; MN-major tiles
// [64 k][128 rows] read transposed by ds_read_b64_tr_b16.  Both conflict-free for the
// 16x16x32 operand access pattern (derivation in DESIGN.md §GEMM).
#include "common.h"

namespace kd {
namespace {

constexpr int BM = 128, BN = 128, BK = 64, NTH = 256;
constexpr int TILE_BYTES = 128 * 64 * 2;  // 16 KiB per operand tile
constexpr uint32_t OOB = 0x80000000u;     // voffset beyond every num_records -> zeros

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4_t;

struct GemmP {
    const bf16* A; const bf16* B; void* C;
    const void* bias; const bf16* resid; bf16* aux; const float* alpha_dev;
    int64_t lda, ldb, ldc, ldr, ld_aux;
    int M, N, K;
    float alpha;
    int c_f32, accumulate, bias_f32, act, res_mod;
};

__device__ __forceinline__ uint32_t sw_k(int row) { return (uint32_t)((row >> 1) & 7); }
__device__ __forceinline__ uint32_t sw_mn(int k) { return (uint32_t)(((k & 3) | (((k >> 3) & 1) << 2)) << 1); }

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}

__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t rs, char* lds_dst, uint32_t voff) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void_t*)lds_dst, 16, voff, 0, 0, 0);
}

// Stage one 128-row x 64-k operand tile into LDS (each wave issues 4 x 1 KiB).
template <bool MN>
__device__ __forceinline__ void stage(char* tile, const bf16* ptr, int64_t ld, int r0, int rows_total,
                                      int k0, int K, int wid, int lane) {
    if (!MN) {
        // base at row r0; num_records bounds the valid rows
        const int rows_valid = min(128, rows_total - r0);
        const uint64_t bytes = (uint64_t)rows_valid * (uint64_t)ld * 2u;
        auto rs = make_rsrc(ptr + (int64_t)r0 * ld, bytes > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)bytes);
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const int i = wid * 4 + s;
            const int row = 8 * i + (lane >> 3);
            const int gc = (lane & 7) ^ (int)sw_k(row);
            const int k = k0 + gc * 8;
            const uint32_t voff = (k < K) ? (uint32_t)(((int64_t)row * ld + k) * 2) : OOB;
            dma16(rs, tile + i * 1024, voff);
        }
    } else {
        // operand stored [K][rows]; base at k-row k0, column r0
        const int kvalid = min(64, K - k0);
        const uint64_t bytes = (uint64_t)kvalid * (uint64_t)ld * 2u;
        auto rs = make_rsrc(ptr + (int64_t)k0 * ld + r0, bytes > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)bytes);
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const int i = wid * 4 + s;
            const int kr = 4 * i + (lane >> 4);
            const int gc = (lane & 15) ^ (int)sw_mn(kr);
            const int row = r0 + gc * 8;
            const uint32_t voff = (kr < kvalid && row < rows_total) ? (uint32_t)(((int64_t)kr * ld + gc * 8) * 2) : OOB;
            dma16(rs, tile + i * 1024, voff);
        }
    }
}

// Read the 16x32 operand fragment for tile rows [rb, rb+16), k-substep ks.
template <bool MN>
__device__ __forceinline__ bf16x8 frag(const char* tile, int rb, int ks, int lane) {
    if (!MN) {
        const int r = rb + (lane & 15);
        const int kc = ks * 4 + (lane >> 4);
        return *(const bf16x8*)(tile + r * 128 + ((kc ^ (int)sw_k(r)) << 4));
    } else {
        const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
        const int cc = (rb >> 3) + (p >> 1);
        const int kr0 = ks * 32 + 8 * g + q;
        const int kr1 = kr0 + 4;
        const char* a0 = tile + kr0 * 256 + ((cc ^ (int)sw_mn(kr0)) << 4) + ((p & 1) << 3);
        const char* a1 = tile + kr1 * 256 + ((cc ^ (int)sw_mn(kr1)) << 4) + ((p & 1) << 3);
        bf16x4 h0 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4_t*)a0);
        bf16x4 h1 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4_t*)a1);
        bf16x8 r;
        r[0] = h0[0]; r[1] = h0[1]; r[2] = h0[2]; r[3] = h0[3];
        r[4] = h1[0]; r[5] = h1[1]; r[6] = h1[2]; r[7] = h1[3];
        return r;
    }
}

__device__ __forceinline__ float gelu_tanh(float x) {
    const float k0 = 0.7978845608028654f, k1 = 0.044715f;
    return 0.5f * x * (1.f + tanhf(k0 * (x + k1 * x * x * x)));
}
__device__ __forceinline__ float gelu_erf(float x) { return 0.5f * x * (1.f + erff(x * 0.7071067811865476f)); }

__device__ __forceinline__ float apply_act(float x, int act) {
    switch (act) {
        case KD_ACT_GELU_TANH: return gelu_tanh(x);
        case KD_ACT_GELU_ERF: return gelu_erf(x);
        case KD_ACT_SILU: return x / (1.f + __expf(-x));
        default: return x;
    }
}

template <bool A_MN, bool B_MN>
__global__ void __launch_bounds__(NTH, 2) k_gemm(GemmP p) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wm = wid >> 1, wn = wid & 1;
    const int tiles_m = (p.M + BM - 1) / BM;
    // XCD-aware bijective remap: blocks b, b+8, ... share an XCD -> give them consecutive tiles
    const int nwg = gridDim.x, b = blockIdx.x;
    const int q8 = nwg / 8, r8 = nwg % 8, x = b % 8;
    const int wg = (x < r8 ? x * (q8 + 1) : r8 * (q8 + 1) + (x - r8) * q8) + b / 8;
    const int tm = wg % tiles_m, tn = wg / tiles_m;
    const int m0 = tm * BM, n0 = tn * BN;

    f32x4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

    const int nkt = (p.K + BK - 1) / BK;
    // LDS: buffer c at smem + c*32 KiB: [A tile 16 KiB | B tile 16 KiB]
    stage<A_MN>(smem, p.A, p.lda, m0, p.M, 0, p.K, wid, lane);
    stage<B_MN>(smem + TILE_BYTES, p.B, p.ldb, n0, p.N, 0, p.K, wid, lane);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();

    for (int kt = 0; kt < nkt; ++kt) {
        const int cur = kt & 1;
        if (kt + 1 < nkt) {
            char* nb = smem + (cur ^ 1) * 2 * TILE_BYTES;
            stage<A_MN>(nb, p.A, p.lda, m0, p.M, (kt + 1) * BK, p.K, wid, lane);
            stage<B_MN>(nb + TILE_BYTES, p.B, p.ldb, n0, p.N, (kt + 1) * BK, p.K, wid, lane);
        }
        const char* ta = smem + cur * 2 * TILE_BYTES;
        const char* tb = ta + TILE_BYTES;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            bf16x8 af[4], bfr[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) af[i] = frag<A_MN>(ta, wm * 64 + i * 16, ks, lane);
#pragma unroll
            for (int j = 0; j < 4; ++j) bfr[j] = frag<B_MN>(tb, wn * 64 + j * 16, ks, lane);
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }

    // ---------------------------------------------------------------- epilogue
    float alpha = p.alpha;
    if (p.alpha_dev) alpha *= *p.alpha_dev;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int col = n0 + wn * 64 + j * 16 + (lane & 15);
            if (col >= p.N) continue;
            float bcol = 0.f;
            if (p.bias) bcol = p.bias_f32 ? ((const float*)p.bias)[col] : (float)((const bf16*)p.bias)[col];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = m0 + wm * 64 + i * 16 + (lane >> 4) * 4 + r;
                if (row >= p.M) continue;
                float v = acc[i][j][r] * alpha + bcol;
                if (p.aux) p.aux[(int64_t)row * p.ld_aux + col] = (bf16)v;
                v = apply_act(v, p.act);
                if (p.resid) v += (float)p.resid[(int64_t)(p.res_mod > 0 ? row % p.res_mod : row) * p.ldr + col];
                const int64_t o = (int64_t)row * p.ldc + col;
                if (p.c_f32) {
                    float* c = (float*)p.C;
                    c[o] = p.accumulate ? c[o] + v : v;
                } else {
                    bf16* c = (bf16*)p.C;
                    c[o] = p.accumulate ? (bf16)((float)c[o] + v) : (bf16)v;
                }
            }
        }
    }
}

}  // namespace

int launch_gemm(const kd_gemm_desc* d, void* stream_) {
    KD_CHECK_ARG(d != nullptr, "gemm: null descriptor");
    KD_CHECK_ARG(d->A && d->B && d->C, "gemm: null operand");
    KD_CHECK_SHAPE(d->M > 0 && d->N > 0 && d->K > 0, "gemm: empty shape");
    KD_CHECK_ARG(d->a_layout == KD_LAYOUT_K_MAJOR || d->a_layout == KD_LAYOUT_MN_MAJOR, "gemm: a_layout");
    KD_CHECK_ARG(d->b_layout == KD_LAYOUT_K_MAJOR || d->b_layout == KD_LAYOUT_MN_MAJOR, "gemm: b_layout");
    KD_CHECK_ARG(d->c_dtype == KD_DTYPE_BF16 || d->c_dtype == KD_DTYPE_F32, "gemm: c_dtype");
    KD_CHECK_ARG(d->act >= KD_ACT_NONE && d->act <= KD_ACT_SILU, "gemm: act");
    KD_CHECK_ALIGN(d->A, 16, "gemm: A must be 16-B aligned");
    KD_CHECK_ALIGN(d->B, 16, "gemm: B must be 16-B aligned");
    KD_CHECK_SHAPE(d->lda % 8 == 0 && d->ldb % 8 == 0, "gemm: lda/ldb must be multiples of 8");
    if (d->a_layout == KD_LAYOUT_K_MAJOR) {
        KD_CHECK_SHAPE(d->K % 8 == 0 && d->lda >= d->K, "gemm: K-major A needs K % 8 == 0, lda >= K");
    } else {
        KD_CHECK_SHAPE(d->M % 8 == 0 && d->lda >= d->M, "gemm: MN-major A needs M % 8 == 0, lda >= M");
        KD_CHECK_SHAPE((uint64_t)64 * d->lda * 2 < 0xFFFFFFFFull, "gemm: lda too large");
    }
    if (d->b_layout == KD_LAYOUT_K_MAJOR) {
        KD_CHECK_SHAPE(d->K % 8 == 0 && d->ldb >= d->K, "gemm: K-major B needs K % 8 == 0, ldb >= K");
    } else {
        KD_CHECK_SHAPE(d->N % 8 == 0 && d->ldb >= d->N, "gemm: MN-major B needs N % 8 == 0, ldb >= N");
    }
    KD_CHECK_SHAPE(d->ldc >= d->N, "gemm: ldc < N");
    KD_CHECK_SHAPE(!d->residual || d->ldr >= d->N, "gemm: ldr < N");
    KD_CHECK_SHAPE(!d->aux || d->ld_aux >= d->N, "gemm: ld_aux < N");
    KD_CHECK_SHAPE((uint64_t)128 * (d->a_layout == KD_LAYOUT_K_MAJOR ? d->lda : 0) * 2 < 0xFFFFFFFFull,
                   "gemm: lda too large");
    GemmP p;
    p.A = (const bf16*)d->A; p.B = (const bf16*)d->B; p.C = d->C;
    p.bias = d->bias; p.resid = (const bf16*)d->residual; p.aux = (bf16*)d->aux; p.alpha_dev = d->alpha_dev;
    p.lda = d->lda; p.ldb = d->ldb; p.ldc = d->ldc; p.ldr = d->ldr; p.ld_aux = d->ld_aux;
    p.M = d->M; p.N = d->N; p.K = d->K; p.alpha = d->alpha;
    p.c_f32 = d->c_dtype == KD_DTYPE_F32; p.accumulate = d->accumulate; p.bias_f32 = d->bias_dtype == KD_DTYPE_F32;
    p.act = d->act;
    p.res_mod = d->residual_row_mod;
    const int tiles = ceil_div(d->M, BM) * ceil_div(d->N, BN);
    const size_t smem = 4 * TILE_BYTES;
    hipStream_t st = as_stream(stream_);
    const bool amn = d->a_layout == KD_LAYOUT_MN_MAJOR, bmn = d->b_layout == KD_LAYOUT_MN_MAJOR;
    if (!amn && !bmn) hipLaunchKernelGGL((k_gemm<false, false>), dim3(tiles), dim3(NTH), smem, st, p);
    else if (!amn && bmn) hipLaunchKernelGGL((k_gemm<false, true>), dim3(tiles), dim3(NTH), smem, st, p);
    else if (amn && bmn) hipLaunchKernelGGL((k_gemm<true, true>), dim3(tiles), dim3(NTH), smem, st, p);
    else hipLaunchKernelGGL((k_gemm<true, false>), dim3(tiles), dim3(NTH), smem, st, p);
    KD_LAUNCH_CHECK("k_gemm");
    return KD_OK;
}

}  // namespace kd
