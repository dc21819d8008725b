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
    int64_t kchunk;        // split-K: K elements per split (gridDim.y splits)
    int64_t split_stride;  // split-K: fp32 elements between consecutive partial planes
};

__device__ __forceinline__ uint32_t sw_k(int row) { return (uint32_t)((row >> 1) & 7); }
__device__ __forceinline__ uint32_t sw_mn(int k) { return (uint32_t)(((k & 3) | (((k >> 3) & 1) << 2)) << 1); }

// num_records is always kept below 2^31 (launch checks guarantee the real extents are), so
// the out-of-range voffset OOB = 2^31 can never address memory.
__device__ __forceinline__ uint32_t rec_bytes(int64_t rows, int64_t ld) {
    const int64_t b = rows * ld * 2;
    return b <= 0 ? 0u : (b >= 0x7FFFFFFFll ? 0x7FFFFFFFu : (uint32_t)b);
}

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
        auto rs = make_rsrc(ptr + (int64_t)r0 * ld, rec_bytes(rows_valid, ld));
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
        const int kvalid = max(0, min(64, K - k0));
        auto rs = make_rsrc(ptr + (int64_t)min(k0, K) * ld + r0, rec_bytes(kvalid, ld));
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

// Block -> tile map: (1) XCD-aware bijective remap, so the blocks dispatched to one XCD
// (b, b+8, ...) get consecutive ids; (2) grouped order, GM tile-rows at a time, so the
// ~32 co-resident blocks of an XCD share GM A-panels and 32/GM B-panels in its L2.
__device__ __forceinline__ void tile_of(int tiles_m, int tiles_n, int& tm, int& tn) {
    const int nwg = gridDim.x, b = blockIdx.x;
    const int q8 = nwg / 8, r8 = nwg % 8, x = b % 8;
    const int wg = (x < r8 ? x * (q8 + 1) : r8 * (q8 + 1) + (x - r8) * q8) + b / 8;
    constexpr int GM = 8;
    const int group = wg / (GM * tiles_n);
    const int first_m = group * GM;
    const int gm = min(tiles_m - first_m, GM);
    const int idx = wg - group * GM * tiles_n;
    tm = first_m + idx % gm;
    tn = idx / gm;
}

template <bool A_MN, bool B_MN>
__global__ void __launch_bounds__(NTH, 2) k_gemm(GemmP p) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wm = wid >> 1, wn = wid & 1;
    int tm, tn;
    tile_of((p.M + BM - 1) / BM, (p.N + BN - 1) / BN, tm, tn);
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
            __builtin_amdgcn_sched_barrier(0);  // every LDS read in flight before the first MFMA
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


// =============================================================================
// v2: 256x256 (or 256x128 / 128x256) tile, 512 threads = 8 waves, BK = 32, a 4-stage
// LDS-DMA ring with 3 stages in flight (counted vmcnt, raw s_barrier: the DMA of the
// next stages stays in flight across barriers), 1 workgroup per CU, and an epilogue
// staged through LDS so every global store / residual load is a 16-B row chunk.
// 256x256 halves the L2->CU bytes per FLOP of the 128x128 v1 tile (128 FLOP/B).
//   K-major stage image [rows][32 k] (64-B rows), chunk ^ F4[(row>>2)&3]   (b128 reads)
//   MN-major stage image [32 k][rows] (2*rows-B rows), chunk ^ sw_mn(k)   (tr_b16 reads)
// Both swizzles are conflict-free for the 16x16x32 fragment reads (checked by
// enumeration).
// =============================================================================
constexpr int BK2 = 32, NST = 4, NTH2 = 512;

__device__ __forceinline__ int f4(int row) { return (0x1320 >> (((row >> 2) & 3) * 4)) & 3; }  // [0,2,3,1]

template <int R, bool MN>
__device__ __forceinline__ void stage2(char* tile, const bf16* ptr, int64_t ld, int r0, int rows_total, int k0, int K,
                                       int wid, int lane, __amdgpu_buffer_rsrc_t rs_k) {
    constexpr int NI = R / 16;           // 1-KiB wave-instructions per operand stage
    constexpr int PER = NI / 8;          // per wave (8 waves)
    if (!MN) {
#pragma unroll
        for (int s = 0; s < PER; ++s) {
            const int i = wid * PER + s;
            const int row = 16 * i + (lane >> 2);
            const int gc = (lane & 3) ^ f4(row);
            const int k = k0 + gc * 8;
            const uint32_t voff = (k < K) ? (uint32_t)(((int64_t)row * ld + k) * 2) : OOB;
            dma16(rs_k, tile + i * 1024, voff);
        }
    } else {
        constexpr int CPR = R / 8;       // 16-B chunks per k-row
        constexpr int KPI = 64 / CPR;    // k-rows per wave-instruction
        const int kvalid = max(0, min(BK2, K - k0));   // past-the-end stages: no records at all
        auto rs = make_rsrc(ptr + (int64_t)min(k0, K) * ld + r0, rec_bytes(kvalid, ld));
#pragma unroll
        for (int s = 0; s < PER; ++s) {
            const int i = wid * PER + s;
            const int kr = i * KPI + lane / CPR;
            const int gc = (lane % CPR) ^ (int)sw_mn(kr);
            const int row = r0 + gc * 8;
            const uint32_t voff = (kr < kvalid && row < rows_total) ? (uint32_t)(((int64_t)kr * ld + gc * 8) * 2) : OOB;
            dma16(rs, tile + i * 1024, voff);
        }
    }
}

template <int R, bool MN>
__device__ __forceinline__ bf16x8 frag2(const char* tile, int rb, int lane) {
    if (!MN) {
        const int r = rb + (lane & 15);
        const int c = lane >> 4;
        return *(const bf16x8*)(tile + r * 64 + ((c ^ f4(r)) << 4));
    } else {
        constexpr int RB = R * 2;
        const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
        const int cc = (rb >> 3) + (p >> 1);
        const int kr0 = 8 * g + q, kr1 = kr0 + 4;
        const char* a0 = tile + kr0 * RB + ((cc ^ (int)sw_mn(kr0)) << 4) + ((p & 1) << 3);
        const char* a1 = tile + kr1 * RB + ((cc ^ (int)sw_mn(kr1)) << 4) + ((p & 1) << 3);
        bf16x4 h0 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4_t*)a0);
        bf16x4 h1 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4_t*)a1);
        bf16x8 r;
        r[0] = h0[0]; r[1] = h0[1]; r[2] = h0[2]; r[3] = h0[3];
        r[4] = h1[0]; r[5] = h1[1]; r[6] = h1[2]; r[7] = h1[3];
        return r;
    }
}

template <int N> __device__ __forceinline__ void wait_vm() {
    if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else if constexpr (N == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    else if constexpr (N == 3) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
    else if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else if constexpr (N == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if constexpr (N == 9) asm volatile("s_waitcnt vmcnt(9)" ::: "memory");
    else if constexpr (N == 12) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
    else if constexpr (N == 15) asm volatile("s_waitcnt vmcnt(15)" ::: "memory");
    else if constexpr (N == 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    else if constexpr (N == 24) asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
    else static_assert(N == 0, "unsupported vmcnt");
}

template <int BM, int BN, int NS = NST>
constexpr size_t gemm2_lds() {
    // pipeline ring vs the epilogue staging (bf16 tile with 16-B padded rows, or half an fp32 tile)
    constexpr size_t ring = (size_t)NS * (BM + BN) * BK2 * 2;
    constexpr size_t ep16 = (size_t)BM * (BN * 2 + 16);
    constexpr size_t ep32 = (size_t)(BM / 2) * (BN * 4 + 16);
    return ring > ep16 ? (ring > ep32 ? ring : ep32) : (ep16 > ep32 ? ep16 : ep32);
}


template <int BM, int BN, int WM, int WN, int TM, int TN, int MT, int NT, int NTHR = NTH2>
__device__ __forceinline__ void epilogue2(const GemmP& p, f32x4 (&acc)[MT][NT], char* smem, int m0, int n0, int wm, int wn,
                                          int lane, int tid) {
    // ---------------------------------------------------------------- epilogue
    float alpha = p.alpha;
    if (p.alpha_dev) alpha *= *p.alpha_dev;
    // alpha, bias, aux (pre-activation), activation in registers
#pragma unroll
    for (int j = 0; j < NT; ++j) {
        const int col = n0 + wn * TN + j * 16 + (lane & 15);
        float bcol = 0.f;
        if (p.bias && col < p.N) bcol = p.bias_f32 ? ((const float*)p.bias)[col] : (float)((const bf16*)p.bias)[col];
#pragma unroll
        for (int i = 0; i < MT; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                float v = acc[i][j][r] * alpha + bcol;
                if (p.aux) {
                    const int row = m0 + wm * TM + i * 16 + (lane >> 4) * 4 + r;
                    if (row < p.M && col < p.N) p.aux[(int64_t)row * p.ld_aux + col] = (bf16)v;
                }
                acc[i][j][r] = apply_act(v, p.act);
            }
    }
    if (!p.c_f32) {
        constexpr int RS = BN * 2 + 16;   // padded LDS row (bytes)
#pragma unroll
        for (int i = 0; i < MT; ++i)
#pragma unroll
            for (int j = 0; j < NT; ++j)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int lr = wm * TM + i * 16 + (lane >> 4) * 4 + r;
                    const int lc = wn * TN + j * 16 + (lane & 15);
                    *(bf16*)(smem + lr * RS + lc * 2) = (bf16)acc[i][j][r];
                }
        __syncthreads();
        constexpr int CPR = BN / 8;
        for (int idx = tid; idx < BM * CPR; idx += NTHR) {
            const int lr = idx / CPR, c = idx % CPR;
            const int row = m0 + lr, col = n0 + c * 8;
            if (row >= p.M || col >= p.N) continue;
            bf16x8 v = *(const bf16x8*)(smem + lr * RS + c * 16);
            bf16* dst = (bf16*)p.C + (int64_t)row * p.ldc + col;
            if (p.resid || p.accumulate) {
                float f[8];
#pragma unroll
                for (int e = 0; e < 8; ++e) f[e] = (float)v[e];
                if (p.resid) {
                    const int rr = p.res_mod > 0 ? row % p.res_mod : row;
                    bf16x8 rv = *(const bf16x8*)(p.resid + (int64_t)rr * p.ldr + col);
#pragma unroll
                    for (int e = 0; e < 8; ++e) f[e] += (float)rv[e];
                }
                if (p.accumulate) {
                    bf16x8 cv = *(const bf16x8*)dst;
#pragma unroll
                    for (int e = 0; e < 8; ++e) f[e] += (float)cv[e];
                }
#pragma unroll
                for (int e = 0; e < 8; ++e) v[e] = (bf16)f[e];
            }
            *(bf16x8*)dst = v;
        }
    } else {
        constexpr int RS = BN * 4 + 16;
        constexpr int HR = BM / 2;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
#pragma unroll
            for (int i = 0; i < MT; ++i) {
                const int lr0 = wm * TM + i * 16;
                if (lr0 < h * HR || lr0 >= (h + 1) * HR) continue;
#pragma unroll
                for (int j = 0; j < NT; ++j)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int lr = lr0 + (lane >> 4) * 4 + r - h * HR;
                        const int lc = wn * TN + j * 16 + (lane & 15);
                        *(float*)(smem + lr * RS + lc * 4) = acc[i][j][r];
                    }
            }
            __syncthreads();
            constexpr int CPR = BN / 4;
            for (int idx = tid; idx < HR * CPR; idx += NTHR) {
                const int lr = idx / CPR, c = idx % CPR;
                const int row = m0 + h * HR + lr, col = n0 + c * 4;
                if (row >= p.M || col >= p.N) continue;
                f32x4 v = *(const f32x4*)(smem + lr * RS + c * 16);
                float* dst = (float*)p.C + (int64_t)row * p.ldc + col;
                if (p.resid) {
                    const int rr = p.res_mod > 0 ? row % p.res_mod : row;
#pragma unroll
                    for (int e = 0; e < 4; ++e) v[e] += (float)p.resid[(int64_t)rr * p.ldr + col + e];
                }
                if (p.accumulate) v += *(const f32x4*)dst;
                *(f32x4*)dst = v;
            }
            __syncthreads();
        }
    }
}

template <int BM, int BN, bool A_MN, bool B_MN>
__global__ void __launch_bounds__(NTH2, 1) k_gemm2(GemmP p) {
    constexpr int WM = (BM == 256 && BN == 256) ? 2 : (BM == 256 ? 4 : 2);
    constexpr int WN = 8 / WM;
    constexpr int TM = BM / WM, TN = BN / WN, MT = TM / 16, NT = TN / 16;
    constexpr int SA = BM * BK2 * 2, SB = BN * BK2 * 2, SS = SA + SB;
    constexpr int G = (BM / 16) / 8 + (BN / 16) / 8;   // DMA wave-instructions per stage per wave
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wm = wid / WN, wn = wid % WN;
    int tm, tn;
    tile_of((p.M + BM - 1) / BM, (p.N + BN - 1) / BN, tm, tn);
    const int m0 = tm * BM, n0 = tn * BN;

    // K-major descriptors are fixed per block (base at the block's first row)
    __amdgpu_buffer_rsrc_t rsA = make_rsrc(p.A, 0), rsB = make_rsrc(p.B, 0);
    if (!A_MN) rsA = make_rsrc(p.A + (int64_t)m0 * p.lda, rec_bytes(min(BM, p.M - m0), p.lda));
    if (!B_MN) rsB = make_rsrc(p.B + (int64_t)n0 * p.ldb, rec_bytes(min(BN, p.N - n0), p.ldb));

    f32x4 acc[MT][NT];
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

    const int nk = (p.K + BK2 - 1) / BK2;
#pragma unroll
    for (int st = 0; st < NST - 1; ++st) {
        if (st < nk) {
            char* base = smem + st * SS;
            stage2<BM, A_MN>(base, p.A, p.lda, m0, p.M, st * BK2, p.K, wid, lane, rsA);
            stage2<BN, B_MN>(base + SA, p.B, p.ldb, n0, p.N, st * BK2, p.K, wid, lane, rsB);
        }
    }
    for (int t = 0; t < nk; ++t) {
        // stage t must have landed: the stages issued after it (<= 2) may stay in flight
        const int after = min(NST - 2, nk - 1 - t);
        if (after >= 2) wait_vm<2 * G>();
        else if (after == 1) wait_vm<G>();
        else wait_vm<0>();
        __builtin_amdgcn_s_barrier();
        if (t + NST - 1 < nk) {
            char* base = smem + ((t + NST - 1) % NST) * SS;
            stage2<BM, A_MN>(base, p.A, p.lda, m0, p.M, (t + NST - 1) * BK2, p.K, wid, lane, rsA);
            stage2<BN, B_MN>(base + SA, p.B, p.ldb, n0, p.N, (t + NST - 1) * BK2, p.K, wid, lane, rsB);
        }
        const char* ta = smem + (t % NST) * SS;
        const char* tb = ta + SA;
        bf16x8 af[MT], bfr[NT];
#pragma unroll
        for (int j = 0; j < NT; ++j) bfr[j] = frag2<BN, B_MN>(tb, wn * TN + j * 16, lane);
#pragma unroll
        for (int i = 0; i < MT; ++i) af[i] = frag2<BM, A_MN>(ta, wm * TM + i * 16, lane);
        __builtin_amdgcn_sched_barrier(0);  // every LDS read in flight before the first MFMA
#pragma unroll
        for (int i = 0; i < MT; ++i)
#pragma unroll
            for (int j = 0; j < NT; ++j)
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();

    epilogue2<BM, BN, WM, WN, TM, TN, MT, NT>(p, acc, smem, m0, n0, wm, wn, lane, tid);
}


// =============================================================================
// v3: v2's tiles and 4-stage LDS ring, software-pipelined one stage deeper: the
// fragments of stage t+1 are read into a second register set WHILE the MFMAs of stage t
// run, and the DMA of stage t+4 is interleaved with them too (sched_group_barrier), so
// after a barrier the MFMA pipe never waits for LDS or for DMA issue.
// Iteration t: lgkmcnt(0) [frags of t in registers, my reads of buffer t done] ->
//   vmcnt(stage t+1 landed) -> s_barrier [everyone done with buffer t; stage t+1 visible]
//   -> {DMA stage t+4 -> buffer t%4, LDS reads of stage t+1 -> set nxt} || MFMAs(t, set cur)
// =============================================================================
template <int BM, int BN, bool A_MN, bool B_MN, int NS = NST, int ABL = 0>
__global__ void __launch_bounds__(NTH2, 1) k_gemm3(GemmP p_) {
    GemmP p = p_;
    if (gridDim.y > 1) {   // split-K: this grid row owns K range [k0, k0 + kchunk) -> fp32 partial plane
        const int64_t k0 = (int64_t)blockIdx.y * p.kchunk;
        p.K = (int)min((int64_t)p.K - k0, p.kchunk);
        p.A += A_MN ? k0 * p.lda : k0;
        p.B += B_MN ? k0 * p.ldb : k0;
        p.C = (float*)p.C + (int64_t)blockIdx.y * p.split_stride;
    }
    constexpr int WM = (BM == 256 && BN == 256) ? 2 : (BM == 256 ? 4 : 2);
    constexpr int WN = 8 / WM;
    constexpr int TM = BM / WM, TN = BN / WN, MT = TM / 16, NT = TN / 16;
    constexpr int SA = BM * BK2 * 2, SB = BN * BK2 * 2, SS = SA + SB;
    constexpr int G = (BM / 16) / 8 + (BN / 16) / 8;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wm = wid / WN, wn = wid % WN;
    int tm, tn;
    tile_of((p.M + BM - 1) / BM, (p.N + BN - 1) / BN, tm, tn);
    const int m0 = tm * BM, n0 = tn * BN;
    __amdgpu_buffer_rsrc_t rsA = make_rsrc(p.A, 0), rsB = make_rsrc(p.B, 0);
    if (!A_MN) rsA = make_rsrc(p.A + (int64_t)m0 * p.lda, rec_bytes(min(BM, p.M - m0), p.lda));
    if (!B_MN) rsB = make_rsrc(p.B + (int64_t)n0 * p.ldb, rec_bytes(min(BN, p.N - n0), p.ldb));
    f32x4 acc[MT][NT];
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
    const int nk = (p.K + BK2 - 1) / BK2;
    auto dma = [&](int st) {
        char* base = smem + (st % NS) * SS;
        stage2<BM, A_MN>(base, p.A, p.lda, m0, p.M, st * BK2, p.K, wid, lane, rsA);
        stage2<BN, B_MN>(base + SA, p.B, p.ldb, n0, p.N, st * BK2, p.K, wid, lane, rsB);
    };
#pragma unroll
    for (int st = 0; st < NS; ++st) dma(st);
    wait_vm<(NS - 1) * G>();   // stage 0 landed: stages 1..NS-1 may stay in flight
    __builtin_amdgcn_s_barrier();
    bf16x8 aA[MT], bA[NT], aB[MT], bB[NT];
#pragma unroll
    for (int j = 0; j < NT; ++j) bA[j] = frag2<BN, B_MN>(smem + SA, wn * TN + j * 16, lane);
#pragma unroll
    for (int i = 0; i < MT; ++i) aA[i] = frag2<BM, A_MN>(smem, wm * TM + i * 16, lane);

#define KD_G3_STEP(CUR_A, CUR_B, NXT_A, NXT_B)                                                           \
    {                                                                                                     \
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                                                \
        if (ABL != 1) wait_vm<(NS - 2) * G>();   \
        if (ABL != 2) __builtin_amdgcn_s_barrier();   \
        __builtin_amdgcn_sched_barrier(0);                                                                \
        if (ABL != 1) dma(t + NS);   \
        if (ABL != 3) {   \
            const char* na = smem + ((t + 1) % NS) * SS;                                                  \
            _Pragma("unroll") for (int j = 0; j < NT; ++j) NXT_B[j] = frag2<BN, B_MN>(na + SA, wn * TN + j * 16, lane); \
            _Pragma("unroll") for (int i = 0; i < MT; ++i) NXT_A[i] = frag2<BM, A_MN>(na, wm * TM + i * 16, lane);      \
        } else {   \
            _Pragma("unroll") for (int j = 0; j < NT; ++j) NXT_B[j] = CUR_B[j];   \
            _Pragma("unroll") for (int i = 0; i < MT; ++i) NXT_A[i] = CUR_A[i];   \
        }   \
        _Pragma("unroll") for (int i = 0; i < MT; ++i)                                                    \
            _Pragma("unroll") for (int j = 0; j < NT; ++j)                                                \
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(CUR_A[i], CUR_B[j], acc[i][j], 0, 0, 0); \
        _Pragma("unroll") for (int k = 0; k < G; ++k) {                                                   \
            __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);                                            \
            __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);                                            \
        }                                                                                                 \
        _Pragma("unroll") for (int k = 0; k < MT + NT; ++k) {                                             \
            __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);                                            \
            __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);                                            \
        }                                                                                                 \
        __builtin_amdgcn_sched_group_barrier(0x008, MT * NT - 2 * (G + MT + NT), 0);                      \
        __builtin_amdgcn_sched_barrier(0);                                                                \
    }
    // every iteration issues exactly one DMA stage (past the end: all out of range -> no memory
    // traffic, zero-filled buffers nobody reads) and one stage of fragment reads, so the
    // waits are uniform: stage t+1 landed <=> at most 2 younger stages in flight.
    int t = 0;
    for (; t + 1 < nk; t += 2) {
        KD_G3_STEP(aA, bA, aB, bB);
        ++t;
        KD_G3_STEP(aB, bB, aA, bA);
        --t;
    }
    if (t < nk) KD_G3_STEP(aA, bA, aB, bB);
#undef KD_G3_STEP
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    epilogue2<BM, BN, WM, WN, TM, TN, MT, NT>(p, acc, smem, m0, n0, wm, wn, lane, tid);
}

// =============================================================================
// v4: 256x256 tile, BK = 64, two K-tile buffers (A | B, 64 KiB each), 8 waves as 2 (M)
// x 4 (N) groups, each wave 128x64 of C. A K-tile runs as 4 phases, one C quadrant
// (64x32, 16 MFMAs over K = 64) per phase:
//   load section: ds_read this phase's fragments (+ DMA of half of K-tile k+1 in phases
//                 0 and 1; counted vmcnt(0) for K-tile k+1 in phase 3)
//   s_barrier -> lgkmcnt(0) -> setprio(1) MFMA x16 setprio(0) -> s_barrier
// The wm = 1 group runs one barrier behind the wm = 0 group, so on every SIMD (one wave
// of each group) one wave's MFMA cluster overlaps the other's load section.
// Hazards (barrier counts): K-tile k+1's DMA lands (vmcnt 0) in phase 3 before the
// barrier that both groups pass before reading it; buffer k&1 is last read in phase 2
// of K-tile k and rewritten from phase 0 of K-tile k+2, >= 4 barriers later.
// K-major LDS image: 128-B rows, 16-B chunk c of row r stored at slot c ^ ((r >> 1) & 7)
// (conflict-free for the ds_read_b128 lane groups); MN-major: two stacked 32-deep
// images of v2/v3's layout.
// =============================================================================
constexpr int BK4 = 64;

template <bool MN>
__device__ __forceinline__ void stage4(char* tile, const bf16* ptr, int64_t ld, int r0, int rows_total, int k0, int K,
                                       int wid, int lane, int h, __amdgpu_buffer_rsrc_t rs_k) {
    if (!MN) {
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            const int i = 16 * h + wid * 2 + s;
            const int row = i * 8 + (lane >> 3);
            const int gc = (lane & 7) ^ ((row >> 1) & 7);
            const int k = k0 + gc * 8;
            const uint32_t voff = (k < K) ? (uint32_t)(((int64_t)row * ld + k) * 2) : OOB;
            dma16(rs_k, tile + i * 1024, voff);
        }
    } else {
        const int kvalid = max(0, min(BK4, K - k0));
        auto rs = make_rsrc(ptr + (int64_t)min(k0, K) * ld + r0, rec_bytes(kvalid, ld));
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            const int i = 16 * h + wid * 2 + s;
            const int kr = i * 2 + (lane >> 5);
            const int gc = (lane & 31) ^ (int)sw_mn(kr);
            const int row = r0 + gc * 8;
            const uint32_t voff = (kr < kvalid && row < rows_total) ? (uint32_t)(((int64_t)kr * ld + gc * 8) * 2) : OOB;
            dma16(rs, tile + i * 1024, voff);
        }
    }
}

template <bool MN>
__device__ __forceinline__ bf16x8 frag4(const char* tile, int rb, int kk, int lane) {
    if (!MN) {
        const int r = rb + (lane & 15);
        const int c = kk * 4 + (lane >> 4);
        return *(const bf16x8*)(tile + r * 128 + ((c ^ ((r >> 1) & 7)) << 4));
    } else {
        return frag2<256, true>(tile + kk * 32 * 512, rb, lane);
    }
}

template <bool A_MN, bool B_MN>
__global__ void __launch_bounds__(NTH2, 1) k_gemm4(GemmP p_) {
    GemmP p = p_;
    if (gridDim.y > 1) {   // split-K (as v3)
        const int64_t k0 = (int64_t)blockIdx.y * p.kchunk;
        p.K = (int)min((int64_t)p.K - k0, p.kchunk);
        p.A += A_MN ? k0 * p.lda : k0;
        p.B += B_MN ? k0 * p.ldb : k0;
        p.C = (float*)p.C + (int64_t)blockIdx.y * p.split_stride;
    }
    constexpr int OPB = 256 * BK4 * 2;   // one operand of one K-tile
    constexpr int KTB = 2 * OPB;         // one K-tile buffer
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wm = wid >> 2, wn = wid & 3;
    int tm, tn;
    tile_of((p.M + 255) / 256, (p.N + 255) / 256, tm, tn);
    const int m0 = tm * 256, n0 = tn * 256;
    __amdgpu_buffer_rsrc_t rsA = make_rsrc(p.A, 0), rsB = make_rsrc(p.B, 0);
    if (!A_MN) rsA = make_rsrc(p.A + (int64_t)m0 * p.lda, rec_bytes(min(256, p.M - m0), p.lda));
    if (!B_MN) rsB = make_rsrc(p.B + (int64_t)n0 * p.ldb, rec_bytes(min(256, p.N - n0), p.ldb));
    f32x4 acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
    const int nk = (p.K + BK4 - 1) / BK4;
    auto dma_half = [&](int kt, int h) {
        char* base = smem + (kt & 1) * KTB;
        stage4<A_MN>(base, p.A, p.lda, m0, p.M, kt * BK4, p.K, wid, lane, h, rsA);
        stage4<B_MN>(base + OPB, p.B, p.ldb, n0, p.N, kt * BK4, p.K, wid, lane, h, rsB);
    };
    dma_half(0, 0);
    dma_half(0, 1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (wm == 1) __builtin_amdgcn_s_barrier();   // stagger the two wave groups by one barrier
    __builtin_amdgcn_sched_barrier(0);

    bf16x8 af[4][2], b0[2][2], b1[2][2];
    const int ra0 = wm * 128, cb0 = wn * 64;
#define KD_G4_MMA(QM, QN, BF)                                                                              \
    {                                                                                                      \
        __builtin_amdgcn_s_barrier();                                                                      \
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                                                 \
        __builtin_amdgcn_sched_barrier(0);                                                                 \
        __builtin_amdgcn_s_setprio(1);                                                                     \
        _Pragma("unroll") for (int kk = 0; kk < 2; ++kk)                                                   \
            _Pragma("unroll") for (int i = 0; i < 4; ++i)                                                  \
                _Pragma("unroll") for (int j = 0; j < 2; ++j)                                              \
                    acc[(QM) * 4 + i][(QN) * 2 + j] =                                                      \
                        __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][kk], BF[j][kk], acc[(QM) * 4 + i][(QN) * 2 + j], 0, 0, 0); \
        __builtin_amdgcn_s_setprio(0);                                                                     \
        __builtin_amdgcn_sched_barrier(0);                                                                 \
        __builtin_amdgcn_s_barrier();                                                                      \
        __builtin_amdgcn_sched_barrier(0);                                                                 \
    }
    for (int kt = 0; kt < nk; ++kt) {
        const char* ta = smem + (kt & 1) * KTB;
        const char* tb = ta + OPB;
        const bool pf = kt + 1 < nk;
        // phase 0: B(qn 0), A(qm 0); DMA half 0 of K-tile kt+1
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
#pragma unroll
            for (int j = 0; j < 2; ++j) b0[j][kk] = frag4<B_MN>(tb, cb0 + j * 16, kk, lane);
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
#pragma unroll
            for (int i = 0; i < 4; ++i) af[i][kk] = frag4<A_MN>(ta, ra0 + i * 16, kk, lane);
        if (pf) dma_half(kt + 1, 0);
        KD_G4_MMA(0, 0, b0)
        // phase 1: B(qn 1); DMA half 1
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
#pragma unroll
            for (int j = 0; j < 2; ++j) b1[j][kk] = frag4<B_MN>(tb, cb0 + 32 + j * 16, kk, lane);
        if (pf) dma_half(kt + 1, 1);
        KD_G4_MMA(0, 1, b1)
        // phase 2: A(qm 1)
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
#pragma unroll
            for (int i = 0; i < 4; ++i) af[i][kk] = frag4<A_MN>(ta, ra0 + 64 + i * 16, kk, lane);
        KD_G4_MMA(1, 0, b0)
        // phase 3: K-tile kt+1 landed (my DMAs); the barrier publishes everyone's
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        KD_G4_MMA(1, 1, b1)
    }
#undef KD_G4_MMA
    if (wm == 0) __builtin_amdgcn_s_barrier();   // rebalance the barrier count
    __syncthreads();
    epilogue2<256, 256, 2, 4, 128, 64, 8, 4>(p, acc, smem, m0, n0, wm, wn, lane, tid);
}

// =============================================================================
// v6: v3's tile (256x256, 8 waves 2x4, wave 128x64) and 4-slot BK=32 LDS ring, run as
// two phases per stage with the wave groups ping-ponging: the wm = 1 group trails the
// wm = 0 group by one barrier, so on every SIMD one wave's 16-MFMA cluster overlaps the
// other wave's load section.
//   phase a (stage t): ds_read B(t) + A(t) rows 0..63 ; s_barrier ; lgkmcnt(0) ;
//                      setprio(1) 16 MFMA setprio(0) ; s_barrier
//   phase b (stage t): ds_read A(t) rows 64..127 ; DMA stage t+3 -> slot (t+3)%4 ;
//                      vmcnt(2G) [stage t+1 landed] ; s_barrier ; lgkmcnt(0) ; MFMA ; s_barrier
// WAR: slot (t+3)%4 held stage t-1, whose last reads (phase b of t-1) every wave retired
// (lgkmcnt 0) before the barrier that precedes either group's phase b of stage t.
// RAW: stage t+1 is read in phase a of t+1, after the barrier that follows both groups'
// vmcnt waits. DMA past the last stage is issued anyway (out-of-range, zero-fill) so the
// counts stay uniform.
// =============================================================================
template <bool A_MN, bool B_MN>
__global__ void __launch_bounds__(NTH2, 1) k_gemm6(GemmP p_) {
    GemmP p = p_;
    if (gridDim.y > 1) {
        const int64_t k0 = (int64_t)blockIdx.y * p.kchunk;
        p.K = (int)min((int64_t)p.K - k0, p.kchunk);
        p.A += A_MN ? k0 * p.lda : k0;
        p.B += B_MN ? k0 * p.ldb : k0;
        p.C = (float*)p.C + (int64_t)blockIdx.y * p.split_stride;
    }
    constexpr int BM = 256, BN = 256, NS = 4;
    constexpr int SA = BM * BK2 * 2, SS = SA + BN * BK2 * 2;
    constexpr int G = 4;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wm = wid >> 2, wn = wid & 3;
    int tm, tn;
    tile_of((p.M + BM - 1) / BM, (p.N + BN - 1) / BN, tm, tn);
    const int m0 = tm * BM, n0 = tn * BN;
    __amdgpu_buffer_rsrc_t rsA = make_rsrc(p.A, 0), rsB = make_rsrc(p.B, 0);
    if (!A_MN) rsA = make_rsrc(p.A + (int64_t)m0 * p.lda, rec_bytes(min(BM, p.M - m0), p.lda));
    if (!B_MN) rsB = make_rsrc(p.B + (int64_t)n0 * p.ldb, rec_bytes(min(BN, p.N - n0), p.ldb));
    f32x4 acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
    const int nk = (p.K + BK2 - 1) / BK2;
    auto dma = [&](int st) {
        char* base = smem + (st % NS) * SS;
        stage2<BM, A_MN>(base, p.A, p.lda, m0, p.M, st * BK2, p.K, wid, lane, rsA);
        stage2<BN, B_MN>(base + SA, p.B, p.ldb, n0, p.N, st * BK2, p.K, wid, lane, rsB);
    };
    dma(0); dma(1); dma(2);
    wait_vm<2 * G>();
    __builtin_amdgcn_s_barrier();
    if (wm == 1) __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    bf16x8 af[4], bfr[4];
    const int ra = wm * 128, cb = wn * 64;
#define KD_G6_MMA(I0)                                                                                       \
    {                                                                                                       \
        __builtin_amdgcn_s_barrier();                                                                       \
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                                                  \
        __builtin_amdgcn_sched_barrier(0);                                                                  \
        __builtin_amdgcn_s_setprio(1);                                                                      \
        _Pragma("unroll") for (int i = 0; i < 4; ++i)                                                       \
            _Pragma("unroll") for (int j = 0; j < 4; ++j)                                                   \
                acc[(I0) + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[(I0) + i][j], 0, 0, 0); \
        __builtin_amdgcn_s_setprio(0);                                                                      \
        __builtin_amdgcn_sched_barrier(0);                                                                  \
        __builtin_amdgcn_s_barrier();                                                                       \
        __builtin_amdgcn_sched_barrier(0);                                                                  \
    }
    for (int t = 0; t < nk; ++t) {
        const char* ta = smem + (t % NS) * SS;
        // phase a
#pragma unroll
        for (int j = 0; j < 4; ++j) bfr[j] = frag2<BN, B_MN>(ta + SA, cb + j * 16, lane);
#pragma unroll
        for (int i = 0; i < 4; ++i) af[i] = frag2<BM, A_MN>(ta, ra + i * 16, lane);
        KD_G6_MMA(0)
        // phase b
#pragma unroll
        for (int i = 0; i < 4; ++i) af[i] = frag2<BM, A_MN>(ta, ra + 64 + i * 16, lane);
        dma(t + 3);
        wait_vm<2 * G>();
        KD_G6_MMA(4)
    }
#undef KD_G6_MMA
    if (wm == 0) __builtin_amdgcn_s_barrier();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    epilogue2<256, 256, 2, 4, 128, 64, 8, 4>(p, acc, smem, m0, n0, wm, wn, lane, tid);
}

// =============================================================================
// v5: 256x256 tile, BK = 64, FOUR waves (one per SIMD) of 128x128 each, two 64 KiB LDS
// stages (v4's image layouts). One wave per SIMD, so each wave pipelines its own work:
//   step t (F0 = kk 0 fragments of stage t, already read):
//     lgkmcnt(0) ; 64 MFMA(F0), the first 32 interleaved with the 16 DMA instructions
//     of stage t+1 (-> the other buffer) and the 16 reads of F1 (kk 1 of stage t)
//     lgkmcnt(0) ; 32 MFMA(F1, rows 0..63)
//     vmcnt(0) ; s_barrier      [stage t+1 landed for everyone; stage t-1's buffer free]
//     32 MFMA(F1, rows 64..127) interleaved with the 16 reads of F0 of stage t+1
// WAR: the buffer refilled in step t held stage t-1, whose last reads (F1 of t-1) every
// wave retired before the barrier of step t-1. RAW: stage t+1 is read only after the
// barrier of step t, behind every wave's vmcnt(0).
// =============================================================================
constexpr int NTH5 = 256;

// one 1-KiB wave-instruction (index i of 32) of a BK=64 operand stage (v4 layout)
template <bool MN>
__device__ __forceinline__ void dma5(char* tile, __amdgpu_buffer_rsrc_t rs, int64_t ld, int rows_total, int r0,
                                     int k0, int K, int kvalid, int i, int lane) {
    if (!MN) {
        const int row = i * 8 + (lane >> 3);
        const int gc = (lane & 7) ^ ((row >> 1) & 7);
        const int k = k0 + gc * 8;
        const uint32_t voff = (k < K) ? (uint32_t)(((int64_t)row * ld + k) * 2) : OOB;
        dma16(rs, tile + i * 1024, voff);
    } else {
        const int kr = i * 2 + (lane >> 5);
        const int gc = (lane & 31) ^ (int)sw_mn(kr);
        const int row = r0 + gc * 8;
        const uint32_t voff = (kr < kvalid && row < rows_total) ? (uint32_t)(((int64_t)kr * ld + gc * 8) * 2) : OOB;
        dma16(rs, tile + i * 1024, voff);
    }
}

template <bool A_MN, bool B_MN>
__global__ void __launch_bounds__(NTH5, 1) k_gemm5(GemmP p_) {
    GemmP p = p_;
    if (gridDim.y > 1) {
        const int64_t k0 = (int64_t)blockIdx.y * p.kchunk;
        p.K = (int)min((int64_t)p.K - k0, p.kchunk);
        p.A += A_MN ? k0 * p.lda : k0;
        p.B += B_MN ? k0 * p.ldb : k0;
        p.C = (float*)p.C + (int64_t)blockIdx.y * p.split_stride;
    }
    constexpr int OPB = 256 * BK4 * 2, KTB = 2 * OPB;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wm = wid >> 1, wn = wid & 1;
    int tm, tn;
    tile_of((p.M + 255) / 256, (p.N + 255) / 256, tm, tn);
    const int m0 = tm * 256, n0 = tn * 256;
    __amdgpu_buffer_rsrc_t rsAk = make_rsrc(p.A, 0), rsBk = make_rsrc(p.B, 0);
    if (!A_MN) rsAk = make_rsrc(p.A + (int64_t)m0 * p.lda, rec_bytes(min(256, p.M - m0), p.lda));
    if (!B_MN) rsBk = make_rsrc(p.B + (int64_t)n0 * p.ldb, rec_bytes(min(256, p.N - n0), p.ldb));
    const int nk = (p.K + BK4 - 1) / BK4;
    // descriptors of stage st: K-major fixed; MN-major per stage (k rows of the stage)
    auto rs_of = [&](bool mn, const bf16* ptr, int64_t ld, int r0, __amdgpu_buffer_rsrc_t rk, int st, int& kvalid) {
        if (!mn) { kvalid = BK4; return rk; }
        const int k0 = st * BK4;
        kvalid = max(0, min(BK4, p.K - k0));
        return make_rsrc(ptr + (int64_t)min(k0, p.K) * ld + r0, rec_bytes(kvalid, ld));
    };
    f32x4 acc[8][8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
    bf16x8 f0a[8], f0b[8], f1a[8], f1b[8];
    const int ra = wm * 128, cb = wn * 128;
    {   // prologue: stage 0 -> buffer 0, F0(0)
        int kva, kvb;
        const auto ra_ = rs_of(A_MN, p.A, p.lda, m0, rsAk, 0, kva);
        const auto rb_ = rs_of(B_MN, p.B, p.ldb, n0, rsBk, 0, kvb);
#pragma unroll
        for (int s8 = 0; s8 < 8; ++s8) {
            dma5<A_MN>(smem, ra_, p.lda, p.M, m0, 0, p.K, kva, wid * 8 + s8, lane);
            dma5<B_MN>(smem + OPB, rb_, p.ldb, p.N, n0, 0, p.K, kvb, wid * 8 + s8, lane);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
#pragma unroll
        for (int i = 0; i < 8; ++i) f0a[i] = frag4<A_MN>(smem, ra + i * 16, 0, lane);
#pragma unroll
        for (int j = 0; j < 8; ++j) f0b[j] = frag4<B_MN>(smem + OPB, cb + j * 16, 0, lane);
    }
    for (int t = 0; t < nk; ++t) {
        const char* ta = smem + (t & 1) * KTB;
        const char* tb = ta + OPB;
        char* na = smem + ((t + 1) & 1) * KTB;
        int kva, kvb;
        const auto ra_ = rs_of(A_MN, p.A, p.lda, m0, rsAk, t + 1, kva);
        const auto rb_ = rs_of(B_MN, p.B, p.ldb, n0, rsBk, t + 1, kvb);
        const int k1 = (t + 1) * BK4;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        // 64 MFMA(F0); the first 32 in pairs, each pair behind one DMA of stage t+1 and one
        // F1 fragment read (order pinned with sched_barrier: the scheduler would bunch the DMA)
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            if (q < 8) dma5<A_MN>(na, ra_, p.lda, p.M, m0, k1, p.K, kva, wid * 8 + q, lane);
            else dma5<B_MN>(na + OPB, rb_, p.ldb, p.N, n0, k1, p.K, kvb, wid * 8 + q - 8, lane);
            if (q < 8) f1a[q] = frag4<A_MN>(ta, ra + q * 16, 1, lane);
            else f1b[q - 8] = frag4<B_MN>(tb, cb + (q - 8) * 16, 1, lane);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                const int m = 2 * q + e, i = m >> 3, j = m & 7;
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f0a[i], f0b[j], acc[i][j], 0, 0, 0);
            }
            __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int m = 32; m < 64; ++m)
            acc[m >> 3][m & 7] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f0a[m >> 3], f0b[m & 7], acc[m >> 3][m & 7], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 8; ++j)
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f1a[i], f1b[j], acc[i][j], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        // 32 MFMA(F1, rows 64..127) in pairs, each behind one read of F0 of stage t+1
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            if (q < 8) f0a[q] = frag4<A_MN>(na, ra + q * 16, 0, lane);
            else f0b[q - 8] = frag4<B_MN>(na + OPB, cb + (q - 8) * 16, 0, lane);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                const int m = 2 * q + e, i = 4 + (m >> 3), j = m & 7;
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f1a[i], f1b[j], acc[i][j], 0, 0, 0);
            }
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __syncthreads();
    epilogue2<256, 256, 2, 2, 128, 128, 8, 8, NTH5>(p, acc, smem, m0, n0, wm, wn, lane, tid);
}

// =============================================================================
// v7: v3's 4-slot BK=32 LDS ring (three stages in flight) with v5's four waves of
// 128x128 (half the fragment reads per MFMA of the 8-wave 128x64 layout).
//   iteration t: lgkmcnt(0) [fragments of t in registers] ; vmcnt(2 stages x 8) [stage
//   t+1 landed] ; s_barrier ; 64 MFMA(t) in 8 units of {1 DMA of stage t+4 -> slot t%4,
//   2 fragment reads of stage t+1, 8 MFMA}, order pinned by sched_barrier.
// WAR: slot t%4 was last read (fragments of t, during iteration t-1) before every wave's
// lgkmcnt(0) + barrier of iteration t. RAW: stage t+1 is read after the barrier that
// follows every wave's vmcnt for it. DMA past the last stage is issued anyway
// (out-of-range, zero-fill) so the counts stay uniform.
// =============================================================================
template <bool MN>
__device__ __forceinline__ void dma7(char* tile, __amdgpu_buffer_rsrc_t rs, int64_t ld, int rows_total, int r0, int k0,
                                     int K, int kvalid, int i, int lane) {
    if (!MN) {   // 256 rows x 64 B, 16 rows per 1-KiB instruction
        const int row = 16 * i + (lane >> 2);
        const int gc = (lane & 3) ^ f4(row);
        const int k = k0 + gc * 8;
        const uint32_t voff = (k < K) ? (uint32_t)(((int64_t)row * ld + k) * 2) : OOB;
        dma16(rs, tile + i * 1024, voff);
    } else {     // 32 k-rows x 512 B, 2 k-rows per instruction
        const int kr = i * 2 + (lane >> 5);
        const int gc = (lane & 31) ^ (int)sw_mn(kr);
        const int row = r0 + gc * 8;
        const uint32_t voff = (kr < kvalid && row < rows_total) ? (uint32_t)(((int64_t)kr * ld + gc * 8) * 2) : OOB;
        dma16(rs, tile + i * 1024, voff);
    }
}

template <bool A_MN, bool B_MN>
__global__ void __launch_bounds__(NTH5, 1) k_gemm7(GemmP p_) {
    GemmP p = p_;
    if (gridDim.y > 1) {
        const int64_t k0 = (int64_t)blockIdx.y * p.kchunk;
        p.K = (int)min((int64_t)p.K - k0, p.kchunk);
        p.A += A_MN ? k0 * p.lda : k0;
        p.B += B_MN ? k0 * p.ldb : k0;
        p.C = (float*)p.C + (int64_t)blockIdx.y * p.split_stride;
    }
    constexpr int NS = 4, SA = 256 * BK2 * 2, SS = 2 * SA;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wm = wid >> 1, wn = wid & 1;
    int tm, tn;
    tile_of((p.M + 255) / 256, (p.N + 255) / 256, tm, tn);
    const int m0 = tm * 256, n0 = tn * 256;
    __amdgpu_buffer_rsrc_t rsAk = make_rsrc(p.A, 0), rsBk = make_rsrc(p.B, 0);
    if (!A_MN) rsAk = make_rsrc(p.A + (int64_t)m0 * p.lda, rec_bytes(min(256, p.M - m0), p.lda));
    if (!B_MN) rsBk = make_rsrc(p.B + (int64_t)n0 * p.ldb, rec_bytes(min(256, p.N - n0), p.ldb));
    const int nk = (p.K + BK2 - 1) / BK2;
    auto rs_of = [&](bool mn, const bf16* ptr, int64_t ld, int r0, __amdgpu_buffer_rsrc_t rk, int st, int& kvalid) {
        if (!mn) { kvalid = BK2; return rk; }
        const int k0 = st * BK2;
        kvalid = max(0, min(BK2, p.K - k0));
        return make_rsrc(ptr + (int64_t)min(k0, p.K) * ld + r0, rec_bytes(kvalid, ld));
    };
    // DMA instruction u (0..7) of this wave for stage st: A instructions wid*4 + u (u < 4),
    // B instructions wid*4 + u - 4
    auto dma_u = [&](int st, int u, __amdgpu_buffer_rsrc_t ra_, __amdgpu_buffer_rsrc_t rb_, int kva, int kvb) {
        char* base = smem + (st % NS) * SS;
        if (u < 4) dma7<A_MN>(base, ra_, p.lda, p.M, m0, st * BK2, p.K, kva, wid * 4 + u, lane);
        else dma7<B_MN>(base + SA, rb_, p.ldb, p.N, n0, st * BK2, p.K, kvb, wid * 4 + u - 4, lane);
    };
    f32x4 acc[8][8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
    const int ra = wm * 128, cb = wn * 128;
#pragma unroll
    for (int st = 0; st < NS; ++st) {
        int kva, kvb;
        const auto ra_ = rs_of(A_MN, p.A, p.lda, m0, rsAk, st, kva);
        const auto rb_ = rs_of(B_MN, p.B, p.ldb, n0, rsBk, st, kvb);
#pragma unroll
        for (int u = 0; u < 8; ++u) dma_u(st, u, ra_, rb_, kva, kvb);
    }
    wait_vm<24>();   // stage 0 landed
    __builtin_amdgcn_s_barrier();
    bf16x8 xa[8], xb[8], ya[8], yb[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) xa[i] = frag2<256, A_MN>(smem, ra + i * 16, lane);
#pragma unroll
    for (int j = 0; j < 8; ++j) xb[j] = frag2<256, B_MN>(smem + SA, cb + j * 16, lane);

#define KD_G7_STEP(CA, CB, NA, NB)                                                                           \
    {                                                                                                         \
        int kva, kvb;                                                                                         \
        const auto ra_ = rs_of(A_MN, p.A, p.lda, m0, rsAk, t + NS, kva);                                      \
        const auto rb_ = rs_of(B_MN, p.B, p.ldb, n0, rsBk, t + NS, kvb);                                      \
        const char* na = smem + ((t + 1) % NS) * SS;                                                          \
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                                                    \
        wait_vm<16>();                                                                                        \
        __builtin_amdgcn_s_barrier();                                                                         \
        __builtin_amdgcn_sched_barrier(0);                                                                    \
        _Pragma("unroll") for (int u = 0; u < 8; ++u) {                                                       \
            dma_u(t + NS, u, ra_, rb_, kva, kvb);                                                             \
            NA[u] = frag2<256, A_MN>(na, ra + u * 16, lane);                                                  \
            NB[u] = frag2<256, B_MN>(na + SA, cb + u * 16, lane);                                             \
            __builtin_amdgcn_sched_barrier(0);                                                                \
            _Pragma("unroll") for (int j = 0; j < 8; ++j)                                                     \
                acc[u][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(CA[u], CB[j], acc[u][j], 0, 0, 0);        \
            __builtin_amdgcn_sched_barrier(0);                                                                \
        }                                                                                                     \
    }
    int t = 0;
    for (; t + 1 < nk; t += 2) {
        KD_G7_STEP(xa, xb, ya, yb);
        ++t;
        KD_G7_STEP(ya, yb, xa, xb);
        --t;
    }
    if (t < nk) KD_G7_STEP(xa, xb, ya, yb);
#undef KD_G7_STEP
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __syncthreads();
    epilogue2<256, 256, 2, 2, 128, 128, 8, 8, NTH5>(p, acc, smem, m0, n0, wm, wn, lane, tid);
}

// split-K fold: C = epilogue(sum_s partial[s]) with the full epilogue of the descriptor
// (alpha, alpha_dev, bias, aux, act, residual, accumulate), 4 columns per thread
__global__ void k_splitk_reduce(const float* __restrict__ ws, int S, GemmP p) {
    const int c4 = p.N / 4;
    const int64_t total = (int64_t)p.M * c4;
    float alpha = p.alpha;
    if (p.alpha_dev) alpha *= *p.alpha_dev;
    for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total; idx += (int64_t)gridDim.x * blockDim.x) {
        const int64_t row = idx / c4;
        const int col = (int)(idx % c4) * 4;
        const float* src = ws + row * p.N + col;
        f32x4 v = *(const f32x4*)src;
        for (int s = 1; s < S; ++s) v += *(const f32x4*)(src + (int64_t)s * p.split_stride);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            float x = v[e] * alpha;
            if (p.bias) x += p.bias_f32 ? ((const float*)p.bias)[col + e] : (float)((const bf16*)p.bias)[col + e];
            if (p.aux) p.aux[row * p.ld_aux + col + e] = (bf16)x;
            v[e] = apply_act(x, p.act);
        }
        if (p.resid) {
            const bf16x4 r = *(const bf16x4*)(p.resid + (p.res_mod > 0 ? row % p.res_mod : row) * p.ldr + col);
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] += (float)r[e];
        }
        if (p.c_f32) {
            float* dst = (float*)p.C + row * p.ldc + col;
            if (p.accumulate) v += *(const f32x4*)dst;
            *(f32x4*)dst = v;
        } else {
            bf16* dst = (bf16*)p.C + row * p.ldc + col;
            bf16x4 o;
            if (p.accumulate) {
                const bf16x4 c = *(const bf16x4*)dst;
#pragma unroll
                for (int e = 0; e < 4; ++e) v[e] += (float)c[e];
            }
#pragma unroll
            for (int e = 0; e < 4; ++e) o[e] = (bf16)v[e];
            *(bf16x4*)dst = o;
        }
    }
}

// Tile / split-K plan for the 8-wave kernels. Cost model in units of one 32-deep k-step
// of a 256x256 tile on one CU (~0.9 us): waves x (k-steps x tile cost + fixed per-tile
// prologue/epilogue), plus the partial-plane traffic at ~5 TB/s. Constants fitted to a
// tile x split sweep over every GEMM shape of the KD step (tools/tune_gemm.py): the
// model's picks are within 0.1% of the measured best over those 34 shapes.
struct GemmPlan { int var; int split; int64_t kchunk; };

GemmPlan plan_gemm(const kd_gemm_desc* d, uint64_t ws_cap) {
    const int64_t M = d->M, N = d->N;
    const int64_t tiles[3] = {(int64_t)ceil_div(d->M, 256) * ceil_div(d->N, 256),
                              (int64_t)ceil_div(d->M, 256) * ceil_div(d->N, 128),
                              (int64_t)ceil_div(d->M, 128) * ceil_div(d->N, 256)};
    const double step[3] = {1.0, 0.70, 0.65};   // 256x256, 256x128, 128x256
    const double fixed[3] = {24.0, 12.0, 6.0};
    const int64_t nk = ceil_div(d->K, BK2);
    const int fv = (d->variant >= 8 && d->variant <= 15) ? 0 : (d->variant >= 5 ? d->variant - 5 : (d->variant >= 2 ? d->variant - 2 : -1));
    const bool split_ok = d->variant == 0 || d->variant >= 5;
    const double out_b = (double)M * N * ((d->c_dtype == KD_DTYPE_F32 ? 4 : 2) * (d->accumulate ? 2 : 1) +
                                          (d->residual ? 2 : 0) + (d->aux ? 2 : 0));
    GemmPlan best{fv >= 0 ? fv + 2 : 2, 1, d->K};
    double bt = 1e300;
    for (int v = 0; v < 3; ++v) {
        if (fv >= 0 && v != fv) continue;
        for (int S = 1; S <= 32; ++S) {
            if (d->split_k == 1 && S != 1) continue;
            if (d->split_k > 1 && S != d->split_k && S != 1) continue;
            if (S > 1 && !split_ok) continue;
            const int64_t kcs = (nk + S - 1) / S;
            if (S > 1 && ((nk + kcs - 1) / kcs != S)) continue;          // empty trailing split
            if (S > 1 && d->split_k <= 1 && kcs < 8) continue;           // too little work per split
            if (S > 1 && (uint64_t)S * M * N * 4 > ws_cap) continue;
            const int64_t waves = (tiles[v] * S + 255) / 256;
            double t = (double)waves * ((double)kcs * step[v] + fixed[v]);
            if (S > 1) t += ((double)S * M * N * 8 + out_b) / 4.5e6;
            if (d->split_k > 1 && S == d->split_k) t = -1;              // forced
            if (t < bt) { bt = t; best = GemmPlan{v + 2, S, kcs * BK2}; }
        }
    }
    return best;
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
        KD_CHECK_SHAPE((uint64_t)64 * d->lda * 2 < 0x7FFFFFFFull, "gemm: lda too large");
    }
    if (d->b_layout == KD_LAYOUT_K_MAJOR) {
        KD_CHECK_SHAPE(d->K % 8 == 0 && d->ldb >= d->K, "gemm: K-major B needs K % 8 == 0, ldb >= K");
    } else {
        KD_CHECK_SHAPE(d->N % 8 == 0 && d->ldb >= d->N, "gemm: MN-major B needs N % 8 == 0, ldb >= N");
    }
    KD_CHECK_SHAPE(d->ldc >= d->N, "gemm: ldc < N");
    KD_CHECK_SHAPE(!d->residual || d->ldr >= d->N, "gemm: ldr < N");
    KD_CHECK_SHAPE(!d->aux || d->ld_aux >= d->N, "gemm: ld_aux < N");
    KD_CHECK_SHAPE((uint64_t)256 * d->lda * 2 < 0x7FFFFFFFull && (uint64_t)256 * d->ldb * 2 < 0x7FFFFFFFull,
                   "gemm: leading dimension too large for 31-bit buffer records");
    GemmP p;
    p.A = (const bf16*)d->A; p.B = (const bf16*)d->B; p.C = d->C;
    p.bias = d->bias; p.resid = (const bf16*)d->residual; p.aux = (bf16*)d->aux; p.alpha_dev = d->alpha_dev;
    p.lda = d->lda; p.ldb = d->ldb; p.ldc = d->ldc; p.ldr = d->ldr; p.ld_aux = d->ld_aux;
    p.M = d->M; p.N = d->N; p.K = d->K; p.alpha = d->alpha;
    p.c_f32 = d->c_dtype == KD_DTYPE_F32; p.accumulate = d->accumulate; p.bias_f32 = d->bias_dtype == KD_DTYPE_F32;
    p.act = d->act;
    p.res_mod = d->residual_row_mod;
    p.kchunk = d->K; p.split_stride = 0;
    hipStream_t st = as_stream(stream_);
    const bool amn = d->a_layout == KD_LAYOUT_MN_MAJOR, bmn = d->b_layout == KD_LAYOUT_MN_MAJOR;
    const bool c_ok16 = (d->ldc % 8 == 0) && ((uintptr_t)d->C % 16 == 0) && (!d->residual || ((d->ldr % 8 == 0) &&
                        ((uintptr_t)d->residual % 16 == 0)));
    const bool v2_ok = d->N % 8 == 0 && c_ok16 && d->M >= 128 && d->N >= 128 &&
                       ((uint64_t)d->M * d->N >= (1ull << 20) || (d->workspace && d->K >= 2048 && d->split_k != 1)) &&
                       (!amn || d->M % 8 == 0) && (!bmn || d->N % 8 == 0) &&
                       (uint64_t)BK2 * (amn ? d->lda : 0) * 2 < 0x7FFFFFFFull;
    const int force = d->variant;   // 0 auto, 1 v1, 2/3/4 v2 256x256/256x128/128x256, 5/6/7 v3 same tiles,
                                    // 8 v4 256x256, 9 v3 256x256 with a 5-stage ring, 10 v6 256x256 ping-pong,
                                    // 11/12/13 timing ablations of v3 (no DMA / no barrier / no fragment
                                    // reads in the loop: WRONG results, tools/ablate_gemm.py only),
                                    // 14 v5 256x256 four waves of 128x128, 15 v7 (v3 ring, 4 waves)
    if ((force == 0 && v2_ok) || (force >= 2 && v2_ok)) {
        const bool v3 = force == 0 || force >= 5;
        const GemmPlan pl = plan_gemm(d, d->workspace ? d->workspace_bytes : 0);
        const int var = pl.var;
        GemmP pk = p;   // the tile kernels' parameters (split-K: plain fp32 partial planes)
        if (pl.split > 1) {
            KD_CHECK_ARG(d->workspace && d->workspace_bytes >= (uint64_t)pl.split * d->M * d->N * 4,
                         "gemm: split-K workspace too small");
            pk.C = d->workspace; pk.ldc = d->N; pk.c_f32 = 1; pk.accumulate = 0; pk.alpha = 1.f;
            pk.alpha_dev = nullptr; pk.bias = nullptr; pk.aux = nullptr; pk.resid = nullptr; pk.act = KD_ACT_NONE;
            pk.kchunk = pl.kchunk; pk.split_stride = (int64_t)d->M * d->N;
        }
        const dim3 gy(1, pl.split, 1);
        const bool v4 = force == 8, v5 = force == 9, v6 = force == 10, v7 = force == 14, v8 = force == 15;
#define L2(BMv, BNv, AM, BMN)                                                                                     \
    if (v4 && BMv == 256 && BNv == 256)                                                                           \
        hipLaunchKernelGGL((k_gemm4<AM, BMN>), dim3(ceil_div(d->M, 256) * ceil_div(d->N, 256), gy.y), dim3(NTH2),   \
                           (gemm2_lds<256, 256>()), st, pk);                                                      \
    else if (v8 && BMv == 256 && BNv == 256)                                                                      \
        hipLaunchKernelGGL((k_gemm7<AM, BMN>), dim3(ceil_div(d->M, 256) * ceil_div(d->N, 256), gy.y), dim3(NTH5),   \
                           (gemm2_lds<256, 256>()), st, pk);                                                      \
    else if (v7 && BMv == 256 && BNv == 256)                                                                      \
        hipLaunchKernelGGL((k_gemm5<AM, BMN>), dim3(ceil_div(d->M, 256) * ceil_div(d->N, 256), gy.y), dim3(NTH5),   \
                           (gemm2_lds<256, 256>()), st, pk);                                                      \
    else if (force >= 11 && force <= 13 && BMv == 256 && BNv == 256) {                                              \
        if (force == 11) hipLaunchKernelGGL((k_gemm3<256, 256, AM, BMN, 4, 1>), dim3(ceil_div(d->M, 256) * ceil_div(d->N, 256), gy.y), \
                                            dim3(NTH2), (gemm2_lds<256, 256>()), st, pk);                         \
        else if (force == 12) hipLaunchKernelGGL((k_gemm3<256, 256, AM, BMN, 4, 2>), dim3(ceil_div(d->M, 256) * ceil_div(d->N, 256), gy.y), \
                                                 dim3(NTH2), (gemm2_lds<256, 256>()), st, pk);                    \
        else hipLaunchKernelGGL((k_gemm3<256, 256, AM, BMN, 4, 3>), dim3(ceil_div(d->M, 256) * ceil_div(d->N, 256), gy.y), \
                                dim3(NTH2), (gemm2_lds<256, 256>()), st, pk);                                     \
    } else if (v6 && BMv == 256 && BNv == 256)                                                                      \
        hipLaunchKernelGGL((k_gemm6<AM, BMN>), dim3(ceil_div(d->M, 256) * ceil_div(d->N, 256), gy.y), dim3(NTH2),   \
                           (gemm2_lds<256, 256>()), st, pk);                                                      \
    else if (v5 && BMv == 256 && BNv == 256)                                                                      \
        hipLaunchKernelGGL((k_gemm3<256, 256, AM, BMN, 5>), dim3(ceil_div(d->M, 256) * ceil_div(d->N, 256), gy.y),  \
                           dim3(NTH2), (gemm2_lds<256, 256, 5>()), st, pk);                                       \
    else if (v3) hipLaunchKernelGGL((k_gemm3<BMv, BNv, AM, BMN>), dim3(ceil_div(d->M, BMv) * ceil_div(d->N, BNv), gy.y), \
                               dim3(NTH2), (gemm2_lds<BMv, BNv>()), st, pk);                                        \
    else hipLaunchKernelGGL((k_gemm2<BMv, BNv, AM, BMN>), dim3(ceil_div(d->M, BMv) * ceil_div(d->N, BNv)),         \
                            dim3(NTH2), (gemm2_lds<BMv, BNv>()), st, pk)
#define L2SEL(BMv, BNv)                                     \
    if (!amn && !bmn) L2(BMv, BNv, false, false);           \
    else if (!amn && bmn) L2(BMv, BNv, false, true);        \
    else if (amn && bmn) L2(BMv, BNv, true, true);          \
    else L2(BMv, BNv, true, false);
        if (var == 2) { L2SEL(256, 256) }
        else if (var == 3) { L2SEL(256, 128) }
        else { L2SEL(128, 256) }
#undef L2SEL
#undef L2
        KD_LAUNCH_CHECK("k_gemm2");
        if (pl.split > 1) {
            p.split_stride = (int64_t)d->M * d->N;
            const int64_t work = (int64_t)d->M * d->N / 4;
            hipLaunchKernelGGL(k_splitk_reduce, dim3((unsigned)std::min<int64_t>((work + 255) / 256, 16384)), dim3(256), 0,
                               st, (const float*)d->workspace, pl.split, p);
            KD_LAUNCH_CHECK("k_splitk_reduce");
        }
        return KD_OK;
    }
    const int tiles = ceil_div(d->M, BM) * ceil_div(d->N, BN);
    const size_t smem = 4 * TILE_BYTES;
    if (!amn && !bmn) hipLaunchKernelGGL((k_gemm<false, false>), dim3(tiles), dim3(NTH), smem, st, p);
    else if (!amn && bmn) hipLaunchKernelGGL((k_gemm<false, true>), dim3(tiles), dim3(NTH), smem, st, p);
    else if (amn && bmn) hipLaunchKernelGGL((k_gemm<true, true>), dim3(tiles), dim3(NTH), smem, st, p);
    else hipLaunchKernelGGL((k_gemm<true, false>), dim3(tiles), dim3(NTH), smem, st, p);
    KD_LAUNCH_CHECK("k_gemm");
    return KD_OK;
}

size_t gemm_workspace_size(const kd_gemm_desc* d) {
    if (!d || d->M <= 0 || d->N <= 0 || d->K <= 0 || d->variant == 1) return 0;
    const GemmPlan pl = plan_gemm(d, ~0ull);
    return pl.split > 1 ? (size_t)pl.split * d->M * d->N * 4 : 0;
}

}  // namespace kd
