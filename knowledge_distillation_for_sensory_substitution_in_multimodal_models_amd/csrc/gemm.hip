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

#include <cstring>
#include <type_traits>
#ifdef KD_AB_BUILD
#include <hipblaslt/hipblaslt.h>   // tools/ab/gemm_blas.inc (KD_GEMM_BLAS): the A/B library only
#endif

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
    int res_f32;           // residual is fp32 (the fp32 residual stream; C is then fp32 too)
    // q|k|v scatter epilogue (kd_gemm_desc.qkv; forward K-major GEMMs on the tiled kernels): the
    // tile (bias added, rounded to bf16 as the unfused GEMM output) goes straight to head-major
    // q / k / v [B, heads, S, hdp] with RoPE on q and k (cos / sin [S, hd/2]) and the [hd, hdp)
    // padding zeroed — k_qkv_split's arithmetic, without the [M, N] round trip through HBM
    bf16 *sq, *sk, *sv;
    const float *rcos, *rsin;
    int sS, snq, snkv, shd, shdp;
    int64_t kchunk;        // split-K: K elements per split (gridDim.y splits)
    int64_t split_stride;  // split-K: fp32 elements between consecutive partial planes
    int glu;               // SwiGLU epilogue (v8, K-major): I = N/2; B rows [0,I) gate, [I,2I) up; 0 = off
    int tile0;             // first linear tile (grouped order) of this launch: the split tail of a hybrid plan
    const float* sa;       // fp8 path: per-row scale of A [M] (dequantised A = sa[m] * qa[m, k])
    const float* sb;       // fp8 path: per-row scale of B [N] (per output channel)
    // the launch grid, passed explicitly: a kernel that reads gridDim gets the 256-B block of
    // hidden kernel arguments, and the HIP runtime's per-stream kernel-argument pool (~1 MB)
    // then holds ~2000 queued GEMM launches instead of ~5000 before hipLaunchKernel blocks
    int gx, gy;
    // per-row softmax statistics of the bf16 tile (kd_gemm_desc.row_stats; v8, K-major forward)
    float* rst;
    int rst_nt, rst_vs, rst_top2;
    float rst_inv_t;
    // stream-K (v8, variant 21, round 6): the first sk_dp linear tiles (whole waves) run as plain
    // data-parallel tiles, then the launch's sk_grid workgroups split the remaining tiles'
    // sk_steps-deep K loops evenly (one workgroup's run may cover the end of one tile and the start
    // of the next).  A tile covered by several runs is folded INSIDE the launch: every piece stores
    // its fp32 accumulators (fragment-native layout) to its run's slot in sk_ws, then takes a ticket
    // from sk_cnt[tile]; the last arriver sums the pieces in piece order and runs the full epilogue
    // (no fold launch, no partial-plane round trip for the last piece).  0 = off.
    int sk_steps, sk_grid;
    float* sk_ws;
    int sk_dp;
    int* sk_cnt;
    int gm;                // tile rows per group of the grouped tile order (0: GM_GROUP)
    // k-loop start stagger (v8, K % 32 == 0, K >= 2048): the tiles of row group j of ngrp start
    // their K loop at stage j * nk / ngrp and wrap, so the XCDs (each a chunk of one group) stream
    // different K stages at once while each XCD still shares its L2 (cold: teacher lm_head, q|k|v,
    // o_proj, down_proj -4 %, gate|up -1 %; c1 step +0.7 %, profiles/r05/gemm_stagger.txt); 0 = off
    int stagger;
    int stag_g;            // group height the stagger's row groups use (0: gm); v8n takes v8's, so both sum alike
};

// stream-K: the workgroup whose run [floor(tot w / G), floor(tot (w+1) / G)) holds step s
__host__ __device__ inline int sk_wg_of(int64_t s, int64_t tot, int G) { return (int)(((s + 1) * G - 1) / tot); }

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

// gelu_pytorch_tanh: 0.5 x (1 + tanh(u)), u = k0 (x + k1 x^3), evaluated as x * sigmoid(2u) =
// x / (1 + 2^(-2 u log2 e)): one v_exp_f32 + one v_rcp_f32 (~8 instructions) instead of the
// library tanhf (~40 with its range branches), which made the SigLIP fc1 epilogue cost as much
// as its K = 1152 main loop. Limits: x -> -inf gives -0 (2^+inf), x -> +inf gives x.
__device__ __forceinline__ float gelu_tanh(float x) {
    constexpr float c0 = -2.f * 0.7978845608028654f * 1.4426950408889634f;   // -2 k0 log2(e)
    constexpr float c1 = c0 * 0.044715f;
    const float e = __builtin_amdgcn_exp2f(x * fmaf(c1, x * x, c0));
    return x * __builtin_amdgcn_rcpf(1.f + e);
}
__device__ __forceinline__ float gelu_erf(float x) { return 0.5f * x * (1.f + erff(x * 0.7071067811865476f)); }

__device__ __forceinline__ float apply_act(float x, int act) {
    switch (act) {
        case KD_ACT_GELU_TANH: return gelu_tanh(x);
        case KD_ACT_GELU_ERF: return gelu_erf(x);
        case KD_ACT_SILU: return silu_fast(x);
        default: return x;
    }
}

// Linear tile id -> (tm, tn) in grouped order, GM tile-rows at a time, so the ~32
// co-resident blocks of an XCD share GM A-panels and 32/GM B-panels in its L2.
constexpr int GM_GROUP = 8;
__host__ __device__ inline void tile_grouped(int wg, int tiles_m, int tiles_n, int& tm, int& tn, int gm_ = 0) {
    const int GM = gm_ > 0 ? gm_ : GM_GROUP;
    const int group = wg / (GM * tiles_n);
    const int first_m = group * GM;
    const int gm = min(tiles_m - first_m, GM);
    const int idx = wg - group * GM * tiles_n;
    tm = first_m + idx % gm;
    tn = idx / gm;
}

// Tile rows per group for a GEMM of tiles_m x tiles_n tiles (one value per GEMM call: every
// launch of a hybrid / split plan must walk the same order). Each XCD runs a contiguous chunk
// of nwg/8 linear tiles, ~32 at a time: prefer a group height g that divides tiles_m and the
// chunk (every XCD's chunk is whole columns of one group: no XCD straddles two groups), with
// the fewest distinct A + B k-slices among 32 co-resident tiles, g + 32/g (g = 6, 5, 7, 4, 8).
// Measured on the 6144 x 37888 x 3584 gate|up GEMM (24 x 148 tiles, chunks of 444): g = 6
// 1260-1276 us, g = 3 1279-1285, g = 4 1315-1338, g = 8 1341-1358, g = 12 1331, g = 24 1362-1388
// (profiles/r02/gemm_group_height.txt).
inline int pick_gm(int tiles_m, int tiles_n) {
    static const int env = ab_knob("KD_GEMM_GM", 0);
    if (env > 0) return env;
    const int64_t nwg = (int64_t)tiles_m * tiles_n;
    if (nwg % 8 == 0) {
        const int64_t chunk = nwg / 8;
        for (int g : {6, 5, 7, 4, 8})
            if (tiles_m % g == 0 && chunk % g == 0) return g;
    }
    return 4;   // no clean split: 4 measured ahead of 8 (SigLIP fc2 81 vs 87 us, lm_head wgrad 1668 vs 1715 us)
}

// Block -> tile map: XCD-aware bijective remap (the blocks dispatched to one XCD, b, b+8,
// ..., get consecutive ids), offset by the launch's first tile, then the grouped order.
__device__ __forceinline__ void tile_of(int nwg, int tiles_m, int tiles_n, int& tm, int& tn, int tile0 = 0, int gm = 0) {
    const int b = blockIdx.x;
    const int q8 = nwg / 8, r8 = nwg % 8, x = b % 8;
    const int wg = (x < r8 ? x * (q8 + 1) : r8 * (q8 + 1) + (x - r8) * q8) + b / 8 + tile0;
    tile_grouped(wg, tiles_m, tiles_n, tm, tn, gm);
}

template <bool A_MN, bool B_MN>
__global__ void __launch_bounds__(NTH, 2) k_gemm(GemmP p) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wm = wid >> 1, wn = wid & 1;
    int tm, tn;
    tile_of(p.gx, (p.M + BM - 1) / BM, (p.N + BN - 1) / BN, tm, tn);
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
                if (p.resid) {
                    const int64_t ro = (int64_t)(p.res_mod > 0 ? row % p.res_mod : row) * p.ldr + col;
                    v += p.res_f32 ? ((const float*)p.resid)[ro] : (float)p.resid[ro];
                }
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
// Stage layouts of the 256-row kernels (v3, v8). v3: 256x256 (or 256x128 / 128x256) tile,
// 512 threads = 8 waves, BK = 32, a 4-stage LDS-DMA ring with 3 stages in flight (counted vmcnt, raw s_barrier: the DMA of the
// next stages stays in flight across barriers), 1 workgroup per CU, and an epilogue
// staged through LDS so every global store / residual load is a 16-B row chunk.
// 256x256 halves the L2->CU bytes per FLOP of the 128x128 v1 tile (128 FLOP/B).
//   K-major stage image [rows][32 k] (64-B rows), chunk ^ F4[(row>>2)&3]   (b128 reads)
//   MN-major stage image [32 k][rows] (2*rows-B rows), chunk ^ sw_mn(k)   (tr_b16 reads)
// Both swizzles are conflict-free for the 16x16x32 fragment reads (checked by
// enumeration).
// =============================================================================
// read-modify-write epilogues: chunks per load group (epi_flush_g; 8 measured best, no spills
// in the k-loops) and the q|k|v scatter's (its cos / sin loads; 4 spilled in v3)
constexpr int EPI_G = 8, QKV_G = 2;
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

// Transposed LDS read through inline asm. With the builtin, hipcc cannot tell the read
// from the in-flight LDS-DMA writes of later stages and emits s_waitcnt vmcnt(0) before
// the first one of every k-step, draining the whole prefetch ring (MN-major GEMMs ran
// 30-65 % slower than K-major ones, SQ_WAIT_ANY 0.30 -> 0.50 of wave cycles). The asm
// result is NOT tracked by the compiler's lgkmcnt waits: every caller retires these reads
// with its own s_waitcnt lgkmcnt(0) before the fragments are used (v3: start of the next
// step; v8: the step-end sync).
template <int OFF>
__device__ __forceinline__ bf16x4 ds_read_tr_asm(const char* lds) {
    u32x2 r;
    asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(r) : "v"((uint32_t)(uintptr_t)lds), "i"(OFF));
    return __builtin_bit_cast(bf16x4, r);
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
        const int kr0 = 8 * g + q;   // kr1 = kr0 + 4 has the same swizzle (sw_mn ignores bit 2)
        const char* a0 = tile + kr0 * RB + ((cc ^ (int)sw_mn(kr0)) << 4) + ((p & 1) << 3);
        const bf16x4 h0 = ds_read_tr_asm<0>(a0);
        const bf16x4 h1 = ds_read_tr_asm<4 * RB>(a0);
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


// Accumulator layout of the 256-row kernels (v3, v8, v9): the MFMA is issued with the B
// fragment as its A operand and the A fragment as its B operand, i.e. it computes the 16x16
// tile of C^T, so lane l holds C[row = l & 15][cols 4 (l >> 4) .. +3] — four CONSECUTIVE
// columns of one row.  The epilogue's LDS staging is then one 8-B (bf16) / 16-B (fp32) store
// per lane and 16x16 tile instead of four 2-B / 4-B stores (4x fewer LDS write instructions
// in a store-issue-bound epilogue), and a lane's bias is 4 consecutive columns.
__device__ __forceinline__ int acc_row(int lane) { return lane & 15; }
__device__ __forceinline__ int acc_col(int lane) { return (lane >> 4) * 4; }

// Epilogue of the 256-row kernels. Every condition is wave-uniform and hoisted out of the
// per-element loops (a per-element switch on the activation compiled to ~2,800 branches
// and dominated the v8 tile time); the accumulators are only read (so v8's stay in the
// AGPR file), one 16x16 tile at a time, into an LDS image that is then written out in
// 16-B row chunks: pre = alpha*acc + bias -> [aux <- pre] -> C <- act(pre) (+ resid, + C).
// L32: the accumulators of v11's 32x32x16 MFMAs (C^T blocks, MFMA operands swapped) viewed as
// f32x4 [MT = 4 row blocks of 32][NT = 16]: j = 4 bj + g holds C[32 i + (l & 31)][32 bj + 8 g +
// 4 (l >> 5) + 0..3] -- again four consecutive columns of one row per lane and group.
template <bool L32>
__device__ __forceinline__ int acc_col_of(int j, int lane) {
    return L32 ? (j >> 2) * 32 + 8 * (j & 3) + 4 * (lane >> 5) : j * 16 + acc_col(lane);
}

template <int ACT, int TM, int TN, int MT, int NT, bool F32, bool L32 = false>
__device__ __forceinline__ void epi_to_lds(const f32x4 (&acc)[MT][NT], char* smem, int rs, float alpha,
                                           const f32x4 (&bcol)[NT], int wm, int wn, int lane, int r_lo, int r_hi) {
#pragma unroll
    for (int i = 0; i < MT; ++i) {
        const int lr0 = wm * TM + i * (L32 ? 32 : 16);
        if (lr0 < r_lo || lr0 >= r_hi) continue;
        const int lr = lr0 - r_lo + (L32 ? (lane & 31) : acc_row(lane));
#pragma unroll
        for (int j = 0; j < NT; ++j) {
            const f32x4 a = acc[i][j];
            const int lc = wn * TN + acc_col_of<L32>(j, lane);
            float v[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = apply_act(a[r] * alpha + bcol[j][r], ACT);
            if (F32) *(f32x4*)(smem + lr * rs + lc * 4) = (f32x4){v[0], v[1], v[2], v[3]};
            else *(bf16x4*)(smem + lr * rs + lc * 2) = (bf16x4){(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
        }
    }
}

template <int TM, int TN, int MT, int NT, bool F32, bool L32 = false>
__device__ __forceinline__ void epi_to_lds_act(int act, const f32x4 (&acc)[MT][NT], char* smem, int rs, float alpha,
                                               const f32x4 (&bcol)[NT], int wm, int wn, int lane, int r_lo, int r_hi) {
    switch (act) {
        case KD_ACT_GELU_TANH: epi_to_lds<KD_ACT_GELU_TANH, TM, TN, MT, NT, F32, L32>(acc, smem, rs, alpha, bcol, wm, wn, lane, r_lo, r_hi); break;
        case KD_ACT_GELU_ERF: epi_to_lds<KD_ACT_GELU_ERF, TM, TN, MT, NT, F32, L32>(acc, smem, rs, alpha, bcol, wm, wn, lane, r_lo, r_hi); break;
        case KD_ACT_SILU: epi_to_lds<KD_ACT_SILU, TM, TN, MT, NT, F32, L32>(acc, smem, rs, alpha, bcol, wm, wn, lane, r_lo, r_hi); break;
        default: epi_to_lds<KD_ACT_NONE, TM, TN, MT, NT, F32, L32>(acc, smem, rs, alpha, bcol, wm, wn, lane, r_lo, r_hi); break;
    }
}

// LDS image rows [0, ROWS) -> global rows m0 + lr, 16-B chunks (+ resid, + dst).
// A thread's chunks share one column (NTHR % CPR == 0) and step RSTEP rows; they go G at a
// time, the G residual / old-C loads all issued before the group's first store.  Loads placed
// after the previous chunk's store cannot be hoisted by the compiler (the store may alias
// them), so the one-chunk-at-a-time loop kept ONE 16-B load per lane in flight and the
// read-modify-write epilogues moved their extra bytes at ~1.7 TB/s (tools/epi_cost.py).
template <int ROWS, int BN, int NTHR, bool F32, bool RES, bool RF, bool ACC>
__device__ __forceinline__ void epi_flush_g(const GemmP& p, const char* smem, int rs, void* dst_, int64_t ld, int m0,
                                            int n0, int tid, bool full) {
    constexpr int EPC = F32 ? 4 : 8;   // elements per 16-B chunk
    constexpr int CPR = BN / EPC;
    static_assert(NTHR % CPR == 0 && (ROWS * CPR) % NTHR == 0, "epi_flush: chunk map");
    constexpr int RSTEP = NTHR / CPR, PER = ROWS * CPR / NTHR, G = PER < EPI_G ? PER : EPI_G;
    static_assert(PER % G == 0, "epi_flush: group");
    using RT = std::conditional_t<RF, f32x4, std::conditional_t<F32, bf16x4, bf16x8>>;   // residual chunk
    using VT = std::conditional_t<F32, f32x4, bf16x8>;                                    // C chunk
    const int c = tid % CPR, lr0 = tid / CPR;
    const int col = n0 + c * EPC;
    if (!full && col >= p.N) return;
#pragma unroll 1
    for (int g0 = 0; g0 < PER; g0 += G) {
        RT rv[G];
        VT cv[G];
        if constexpr (RES || ACC) {
#pragma unroll
            for (int u = 0; u < G; ++u) {   // unconditional (rows clamped): a load inside a branch got its own vmcnt(0)
                const int row = full ? m0 + lr0 + (g0 + u) * RSTEP : min(m0 + lr0 + (g0 + u) * RSTEP, p.M - 1);
                if constexpr (RES) {
                    const int64_t rr = p.res_mod > 0 ? row % p.res_mod : row;
                    if constexpr (RF) rv[u] = *(const f32x4*)((const float*)p.resid + rr * p.ldr + col);
                    else rv[u] = *(const RT*)(p.resid + rr * p.ldr + col);
                }
                if constexpr (ACC) {
                    if constexpr (F32) cv[u] = *(const f32x4*)((const float*)dst_ + (int64_t)row * ld + col);
                    else cv[u] = *(const bf16x8*)((const bf16*)dst_ + (int64_t)row * ld + col);
                }
            }
        }
#pragma unroll
        for (int u = 0; u < G; ++u) {
            const int lr = lr0 + (g0 + u) * RSTEP, row = m0 + lr;
            if (!full && row >= p.M) continue;
            if constexpr (F32) {
                f32x4 v = *(const f32x4*)(smem + lr * rs + c * 16);
                if constexpr (RES) {
                    if constexpr (RF) v += rv[u];
                    else {
#pragma unroll
                        for (int e = 0; e < 4; ++e) v[e] += (float)rv[u][e];
                    }
                }
                if constexpr (ACC) v += cv[u];
                *(f32x4*)((float*)dst_ + (int64_t)row * ld + col) = v;
            } else {
                bf16x8 v = *(const bf16x8*)(smem + lr * rs + c * 16);
                if constexpr (RES || ACC) {
                    float f[8];
#pragma unroll
                    for (int e = 0; e < 8; ++e) f[e] = (float)v[e];
                    if constexpr (RES) {
#pragma unroll
                        for (int e = 0; e < 8; ++e) f[e] += (float)rv[u][e];
                    }
                    if constexpr (ACC) {
#pragma unroll
                        for (int e = 0; e < 8; ++e) f[e] += (float)cv[u][e];
                    }
#pragma unroll
                    for (int e = 0; e < 8; ++e) v[e] = (bf16)f[e];
                }
                *(bf16x8*)((bf16*)dst_ + (int64_t)row * ld + col) = v;
            }
        }
    }
}

template <int ROWS, int BN, int NTHR, bool F32, bool RES, bool ACC>
__device__ __forceinline__ void epi_flush(const GemmP& p, const char* smem, int rs, void* dst_, int64_t ld, int m0, int n0,
                                          int tid, bool full) {
    // an fp32 C reads an fp32 or a bf16 residual (p.res_f32); a bf16 C a bf16 one
    if (F32 && RES && p.res_f32) epi_flush_g<ROWS, BN, NTHR, F32, RES, F32 && RES, ACC>(p, smem, rs, dst_, ld, m0, n0, tid, full);
    else epi_flush_g<ROWS, BN, NTHR, F32, RES, false, ACC>(p, smem, rs, dst_, ld, m0, n0, tid, full);
}

template <int ROWS, int BN, int NTHR, bool F32>
__device__ __forceinline__ void epi_flush_sel(const GemmP& p, const char* smem, int rs, void* dst, int64_t ld, int m0, int n0,
                                              int tid, bool full, bool res, bool accum) {
    if (!res && !accum) epi_flush<ROWS, BN, NTHR, F32, false, false>(p, smem, rs, dst, ld, m0, n0, tid, full);
    else if (res && !accum) epi_flush<ROWS, BN, NTHR, F32, true, false>(p, smem, rs, dst, ld, m0, n0, tid, full);
    else if (!res && accum) epi_flush<ROWS, BN, NTHR, F32, false, true>(p, smem, rs, dst, ld, m0, n0, tid, full);
    else epi_flush<ROWS, BN, NTHR, F32, true, true>(p, smem, rs, dst, ld, m0, n0, tid, full);
}

// Backward-activation flush (KD_ACT_DGELU_TANH / KD_ACT_DSWIGLU): the staged bf16 tile is the
// activation's output gradient v (exactly the unfused GEMM output); multiply by act'(aux)
// with the same per-element functions as k_act_bwd / k_swiglu_bwd.  Chunks G at a time with
// their aux loads issued first (epi_flush_g).
template <int ROWS, int BN, int NTHR, bool GLU>
__device__ __forceinline__ void epi_flush_dact_g(const GemmP& p, const char* smem, int rs, int m0, int n0, int tid, bool full) {
    constexpr int CPR = BN / 8;
    static_assert(NTHR % CPR == 0 && (ROWS * CPR) % NTHR == 0, "epi_flush_dact: chunk map");
    constexpr int RSTEP = NTHR / CPR, PER = ROWS * CPR / NTHR, G = PER < EPI_G ? PER : EPI_G;
    static_assert(PER % G == 0, "epi_flush_dact: group");
    const int c = tid % CPR, lr0 = tid / CPR;
    const int col = n0 + c * 8;
    if (!full && col >= p.N) return;
#pragma unroll 1
    for (int g0 = 0; g0 < PER; g0 += G) {
        bf16x8 x0[G], x1[G];
#pragma unroll
        for (int u = 0; u < G; ++u) {   // unconditional (rows clamped), as in epi_flush_g
            const int row = full ? m0 + lr0 + (g0 + u) * RSTEP : min(m0 + lr0 + (g0 + u) * RSTEP, p.M - 1);
            const bf16* ar = p.aux + (int64_t)row * p.ld_aux + col;
            x0[u] = *(const bf16x8*)ar;
            if constexpr (GLU) x1[u] = *(const bf16x8*)(ar + p.N);
        }
#pragma unroll
        for (int u = 0; u < G; ++u) {
            const int lr = lr0 + (g0 + u) * RSTEP, row = m0 + lr;
            if (!full && row >= p.M) continue;
            const bf16x8 v = *(const bf16x8*)(smem + lr * rs + c * 16);
            bf16* cr = (bf16*)p.C + (int64_t)row * p.ldc + col;
            if constexpr (GLU) {
                bf16x8 og, ou;
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    float dg, du;
                    swiglu_grad((float)v[e], (float)x0[u][e], (float)x1[u][e], dg, du);
                    og[e] = (bf16)dg;
                    ou[e] = (bf16)du;
                }
                *(bf16x8*)cr = og;
                *(bf16x8*)(cr + p.N) = ou;
            } else {
                bf16x8 o;
#pragma unroll
                for (int e = 0; e < 8; ++e) o[e] = (bf16)((float)v[e] * gelu_tanh_grad((float)x0[u][e]));
                *(bf16x8*)cr = o;
            }
        }
    }
}

template <int ROWS, int BN, int NTHR>
__device__ __forceinline__ void epi_flush_dact(const GemmP& p, const char* smem, int rs, int m0, int n0, int tid, bool full) {
    if (p.act == KD_ACT_DSWIGLU) epi_flush_dact_g<ROWS, BN, NTHR, true>(p, smem, rs, m0, n0, tid, full);
    else epi_flush_dact_g<ROWS, BN, NTHR, false>(p, smem, rs, m0, n0, tid, full);
}

// bias of NT groups of 4 consecutive columns (the transposed accumulator layout), the dtype
// branch outside the loads so all NT vector loads are in flight together (cols[j] % 4 == 0;
// N % 8 == 0 on the tiled kernels: the clamp keeps the 4 columns inside [0, N))
template <int NT>
__device__ __forceinline__ void load_bias4(const GemmP& p, const int (&cols)[NT], f32x4 (&b)[NT]) {
    if (p.bias_f32) {
        const float* bp = (const float*)p.bias;
        f32x4 t[NT];
#pragma unroll
        for (int j = 0; j < NT; ++j) t[j] = *(const f32x4*)(bp + cols[j]);
#pragma unroll
        for (int j = 0; j < NT; ++j) b[j] = t[j];
    } else {
        const bf16* bp = (const bf16*)p.bias;
        bf16x4 t[NT];
#pragma unroll
        for (int j = 0; j < NT; ++j) t[j] = *(const bf16x4*)(bp + cols[j]);
#pragma unroll
        for (int j = 0; j < NT; ++j) b[j] = (f32x4){(float)t[j][0], (float)t[j][1], (float)t[j][2], (float)t[j][3]};
    }
}

// bias of NT columns with the dtype branch outside the loads, so all NT loads are in flight
// together: a per-element `bias_f32 ? f32 : bf16` select made hipcc wait for each load in turn
// (NT dependent memory round trips per tile: +22-24 us on the 7B q|k|v GEMM, 28 calls a step)
template <int NT>
__device__ __forceinline__ void load_bias(const GemmP& p, const int (&cols)[NT], float (&b)[NT]) {
    if (p.bias_f32) {
        const float* bp = (const float*)p.bias;
        float t[NT];
#pragma unroll
        for (int j = 0; j < NT; ++j) t[j] = bp[cols[j]];
#pragma unroll
        for (int j = 0; j < NT; ++j) b[j] = t[j];
    } else {
        const bf16* bp = (const bf16*)p.bias;
        bf16 t[NT];
#pragma unroll
        for (int j = 0; j < NT; ++j) t[j] = bp[cols[j]];
#pragma unroll
        for (int j = 0; j < NT; ++j) b[j] = (float)t[j];
    }
}

// q|k|v scatter flush: LDS bf16 image rows [0, ROWS) x BN -> head-major q / k / v (+RoPE), every
// head of the tile whole in it (256 % hd == 0 or no RoPE), 8-column chunks (hd % 8 == 0).  A
// thread's chunks share one column, so the head / destination tensor / rotate_half partner are
// computed once; the rows go G at a time with their cos / sin loads issued first (epi_flush_g).
template <int ROWS, int BN, int NTHR>
__device__ __forceinline__ void epi_flush_qkv(const GemmP& p, const char* smem, int rs, int m0, int n0, int tid) {
    constexpr int CPR = BN / 8;
    static_assert(NTHR % CPR == 0 && (ROWS * CPR) % NTHR == 0, "epi_flush_qkv: chunk map");
    constexpr int RSTEP = NTHR / CPR, PER = ROWS * CPR / NTHR, G = PER < QKV_G ? PER : QKV_G;
    static_assert(PER % G == 0, "epi_flush_qkv: group");
    const int hd = p.shd, hh = hd >> 1, hdp = p.shdp, S = p.sS, nq = p.snq, nkv = p.snkv;
    const int c = tid % CPR, lr0 = tid / CPR;
    const int col = n0 + c * 8;
    if (col >= p.N) return;
    const int head = col / hd, d0 = col - head * hd;
    bf16* base;
    int hidx, nh;
    if (head < nq) { base = p.sq; hidx = head; nh = nq; }
    else if (head < nq + nkv) { base = p.sk; hidx = head - nq; nh = nkv; }
    else { base = p.sv; hidx = head - nq - nkv; nh = nkv; }
    const bool rope = p.rcos && head < nq + nkv;
    const bool first = d0 < hh;
    const int pc = first ? c * 8 + hh : c * 8 - hh;   // the rotate_half partner, same head, same tile
    const int ri = first ? d0 : d0 - hh;
    const bool last = d0 + 8 == hd;
#pragma unroll 1
    for (int g0 = 0; g0 < PER; g0 += G) {
        f32x4 c0[G], c1[G], s0[G], s1[G];
        int bq[G], sq[G];   // (batch, position) of the row (clamped to M - 1)
#pragma unroll
        for (int u = 0; u < G; ++u) {   // unconditional loads (rows clamped), as in epi_flush_g
            const int row = min(m0 + lr0 + (g0 + u) * RSTEP, p.M - 1);
            const int b = row / S, sr = row - b * S;
            bq[u] = b;
            sq[u] = sr;
            if (p.rcos) {
                const float* cp = p.rcos + (int64_t)sr * hh + ri;
                const float* sp = p.rsin + (int64_t)sr * hh + ri;
                c0[u] = *(const f32x4*)cp; c1[u] = *(const f32x4*)(cp + 4);
                s0[u] = *(const f32x4*)sp; s1[u] = *(const f32x4*)(sp + 4);
            }
        }
#pragma unroll
        for (int u = 0; u < G; ++u) {
            const int lr = lr0 + (g0 + u) * RSTEP;
            if (m0 + lr >= p.M) continue;
            bf16* drow = base + (((int64_t)bq[u] * nh + hidx) * S + sq[u]) * hdp;
            bf16x8 v = *(const bf16x8*)(smem + lr * rs + c * 16);
            if (rope) {
                const bf16x8 pv = *(const bf16x8*)(smem + lr * rs + pc * 2);
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    const float cs = e < 4 ? c0[u][e] : c1[u][e - 4], sn = e < 4 ? s0[u][e] : s1[u][e - 4];
                    const float x = (float)v[e], y = (float)pv[e];
                    v[e] = (bf16)(first ? rope_first(x, y, cs, sn) : rope_second(x, y, cs, sn));
                }
            }
            *(bf16x8*)(drow + d0) = v;
            if (last)
                for (int d = hd; d < hdp; d += 8) *(bf16x8*)(drow + d) = (bf16x8){};
        }
    }
}

// Row statistics of the staged bf16 tile (kd_gemm_desc.row_stats): one thread per tile row
// (256 rows, 256 threads), one online pass over its 256 LDS values, the arithmetic of
// k_row_stats (__expf, chunk-filtered top-2) on the bf16-rounded values the loss reads.
// Measured cost (tools/rst_cost.py): +1170 us on the 7B lm_head (+22%), +374 us on the 0.5B one
// -- 1-2 exps per element run with one wave per SIMD and nothing to overlap them with, which is
// more than the separate HBM-bound k_row_stats pass it removes (0.93 ms a step), so the step
// keeps that pass by default.  LDS rows are RS-byte strided (RS / 4 = 4 mod 64 banks).
__device__ __forceinline__ void epi_row_stats(const GemmP& p, const char* smem, int rs, int m0, int n0, int tid) {
    const int row = m0 + tid;
    if (row >= p.M) return;
    const int ncols = min(256, p.N - n0);
    const int nvs = max(0, min(ncols, (p.rst_vs > 0 ? p.rst_vs : p.N) - n0));
    const bf16x8* rp = (const bf16x8*)(smem + tid * rs);
    // one online pass (k_row_stats' arithmetic): the max moves chunk by chunk and rescales the
    // sums; at T = 1 one exp per element feeds both sums (the sum below vs is kept relative to
    // the running max of all columns and rebased on the max below vs at the end)
    float m_all = -INFINITY, m_vs = -INFINITY, v1 = -INFINITY, v2 = -INFINITY;
    float z1 = 0.f, zt = 0.f;
    int i1 = 0x7fffffff, i2 = 0x7fffffff;
    const bool top2 = p.rst_top2 != 0;
    const float invT = p.rst_inv_t;
    const bool t1 = invT == 1.f;
    const int nch = ncols / 8, nvch = nvs / 8;
    for (int c0 = 0; c0 < nch; c0 += 4) {
        bf16x8 x[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) x[u] = c0 + u < nch ? rp[c0 + u] : (bf16x8){};
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int c = c0 + u;
            if (c >= nch) break;
            float f[8], cm = -INFINITY;
#pragma unroll
            for (int j = 0; j < 8; ++j) { f[j] = (float)x[u][j]; cm = fmaxf(cm, f[j]); }
            if (cm > m_all) {
                if (m_all != -INFINITY) {
                    const float sc = __expf(m_all - cm);
                    z1 *= sc;
                    if (t1) zt *= sc;
                }
                m_all = cm;
            }
            const bool in_vs = c < nvch;
            float e1 = 0.f, et = 0.f;
            if (t1) {
#pragma unroll
                for (int j = 0; j < 8; ++j) e1 += __expf(f[j] - m_all);
                et = e1;
            } else {
#pragma unroll
                for (int j = 0; j < 8; ++j) e1 += __expf(f[j] - m_all);
                if (in_vs) {
                    if (cm > m_vs) { if (m_vs != -INFINITY) zt *= __expf((m_vs - cm) * invT); m_vs = cm; }
#pragma unroll
                    for (int j = 0; j < 8; ++j) et += __expf((f[j] - m_vs) * invT);
                }
            }
            z1 += e1;
            if (in_vs) {
                zt += et;
                if (t1) m_vs = fmaxf(m_vs, cm);
                const int col = n0 + 8 * c;
                if (top2 && (cm > v2 || (cm == v2 && col < i2))) {
#pragma unroll
                    for (int j = 0; j < 8; ++j) top2_push(f[j], col + j, v1, i1, v2, i2);
                }
            }
        }
    }
    if (t1 && m_vs != -INFINITY) zt *= __expf(m_all - m_vs);   // sum exp(c - m_vs) below vs
    float* o = p.rst + ((int64_t)row * p.rst_nt + n0 / 256) * 8;
    *(f32x4*)o = (f32x4){m_all, z1, m_vs, nvs > 0 ? zt : 0.f};
    *(f32x4*)(o + 4) = (f32x4){v1, __int_as_float(i1), v2, __int_as_float(i2)};
}

// HAS_ACT: the activation epilogue is instantiated for the forward (K-major x K-major) kernels
// only; the launcher rejects an activation with MN-major operands or an fp32 output.
// ST (diagnostic stamp builds): mk[0] = s_memtime after the bf16 LDS staging and its barrier,
// mk[1] = after the flush's stores are issued (plain bf16 output only)
template <int BM, int BN, int WM, int WN, int TM, int TN, int MT, int NT, int NTHR = NTH2, bool HAS_ACT = true,
          bool RST = false, bool L32 = false, bool ST = false>
__device__ __forceinline__ void epilogue2(const GemmP& p, const f32x4 (&acc)[MT][NT], char* smem, int m0, int n0, int wm,
                                          int wn, int lane, int tid, uint64_t* mk = nullptr) {
    const bool full = m0 + BM <= p.M && n0 + BN <= p.N;
    float alpha = p.alpha;
    if (p.alpha_dev) alpha *= *p.alpha_dev;
    f32x4 bcol[NT];
#pragma unroll
    for (int j = 0; j < NT; ++j) bcol[j] = (f32x4){0.f, 0.f, 0.f, 0.f};
    if (p.bias) {
        int cols[NT];
#pragma unroll
        for (int j = 0; j < NT; ++j) cols[j] = min(n0 + wn * TN + acc_col_of<L32>(j, lane), p.N - 4);
        load_bias4<NT>(p, cols, bcol);
    }
    constexpr int RS16 = BN * 2 + 16, RS32 = BN * 4 + 16;
    if (HAS_ACT && p.sq) {   // q|k|v scatter (+RoPE) straight from the bf16 tile
        epi_to_lds<KD_ACT_NONE, TM, TN, MT, NT, false, L32>(acc, smem, RS16, alpha, bcol, wm, wn, lane, 0, BM);
        __syncthreads();
        epi_flush_qkv<BM, BN, NTHR>(p, smem, RS16, m0, n0, tid);
        return;
    }
    if (p.act == KD_ACT_DGELU_TANH || p.act == KD_ACT_DSWIGLU) {   // aux is READ (the forward pre-activation)
        epi_to_lds<KD_ACT_NONE, TM, TN, MT, NT, false, L32>(acc, smem, RS16, alpha, bcol, wm, wn, lane, 0, BM);
        __syncthreads();
        epi_flush_dact<BM, BN, NTHR>(p, smem, RS16, m0, n0, tid, full);
        return;
    }
    if (p.aux) {   // pre-activation (bf16) for the backward
        epi_to_lds<KD_ACT_NONE, TM, TN, MT, NT, false, L32>(acc, smem, RS16, alpha, bcol, wm, wn, lane, 0, BM);
        __syncthreads();
        epi_flush<BM, BN, NTHR, false, false, false>(p, smem, RS16, p.aux, p.ld_aux, m0, n0, tid, full);
        __syncthreads();
    }
    const bool res = p.resid != nullptr, accum = p.accumulate != 0;
    if (!p.c_f32) {
        if (HAS_ACT) epi_to_lds_act<TM, TN, MT, NT, false, L32>(p.act, acc, smem, RS16, alpha, bcol, wm, wn, lane, 0, BM);
        else epi_to_lds<KD_ACT_NONE, TM, TN, MT, NT, false, L32>(acc, smem, RS16, alpha, bcol, wm, wn, lane, 0, BM);
        __syncthreads();
        if constexpr (ST) mk[0] = __builtin_amdgcn_s_memtime();
        epi_flush_sel<BM, BN, NTHR, false>(p, smem, RS16, p.C, p.ldc, m0, n0, tid, full, res, accum);
        if constexpr (ST) mk[1] = __builtin_amdgcn_s_memtime();
        if constexpr (RST) epi_row_stats(p, smem, RS16, m0, n0, tid);
    } else {
#pragma unroll
        for (int h = 0; h < 2; ++h) {   // fp32: two half tiles of BM/2 rows
            epi_to_lds<KD_ACT_NONE, TM, TN, MT, NT, true, L32>(acc, smem, RS32, alpha, bcol, wm, wn, lane, h * BM / 2, (h + 1) * BM / 2);
            __syncthreads();
            epi_flush_sel<BM / 2, BN, NTHR, true>(p, smem, RS32, p.C, p.ldc, m0 + h * BM / 2, n0, tid, full, res, accum);
            __syncthreads();
        }
    }
}

// the accumulators as bf16 into the LDS image, unscaled (alpha == 1, no bias: a * 1 + 0 == a for
// every accumulator -- they start at +0, so none is -0 -- and the FMA of epi_to_lds is skipped)
template <int TM, int TN, int MT, int NT, bool L32>
__device__ __forceinline__ void epi_to_lds_raw(const f32x4 (&acc)[MT][NT], char* smem, int rs, int wm, int wn, int lane) {
#pragma unroll
    for (int i = 0; i < MT; ++i) {
        const int lr = wm * TM + i * (L32 ? 32 : 16) + (L32 ? (lane & 31) : acc_row(lane));
#pragma unroll
        for (int j = 0; j < NT; ++j) {
            const f32x4 a = acc[i][j];
            const int lc = wn * TN + acc_col_of<L32>(j, lane);
            *(bf16x4*)(smem + lr * rs + lc * 2) = (bf16x4){(bf16)a[0], (bf16)a[1], (bf16)a[2], (bf16)a[3]};
        }
    }
}

// this lane's index in its wave, recomputed (v_mbcnt) instead of read from a register the k-loop
// spilled: an epilogue that reloads it from scratch waits a memory round trip first
__device__ __forceinline__ int lane_now() {
    int l;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
    return l;
}

// silu(g) * u of two bf16 pairs (words: element 2k in the low half), in the arithmetic of
// silu_fast / k_swiglu_fwd (common.h) as packed fp32 operations: the same IEEE operations in the
// same order, two elements per v_pk_mul / v_pk_add, so the result is bit-identical
__device__ __forceinline__ uint32_t silu_mul_pair(uint32_t gw, uint32_t uw) {
    typedef __attribute__((ext_vector_type(2))) float f2;
    const f2 g = {__uint_as_float(gw << 16), __uint_as_float(gw & 0xffff0000u)};
    const f2 u = {__uint_as_float(uw << 16), __uint_as_float(uw & 0xffff0000u)};
    const f2 t = g * (f2){-KD_SILU_LOG2E, -KD_SILU_LOG2E};
    f2 e = {__builtin_amdgcn_exp2f(t.x), __builtin_amdgcn_exp2f(t.y)};
    e = e + (f2){1.f, 1.f};
    const f2 r = {__builtin_amdgcn_rcpf(e.x), __builtin_amdgcn_rcpf(e.y)};
    const f2 o = (g * r) * u;
    const bf16 lo = (bf16)o.x, hi = (bf16)o.y;
    return (uint32_t)__builtin_bit_cast(uint16_t, lo) | ((uint32_t)__builtin_bit_cast(uint16_t, hi) << 16);
}

// SwiGLU epilogue (KD_ACT_SWIGLU, v8 only): the 256-column tile holds gate features
// [nb, nb+128) in columns 0-127 and the matching up features in columns 128-255 (the B
// rows are gathered that way by the DMA), so C[:, nb + c] = silu(gate) * up needs no
// second pass over HBM: pre-activations are staged once as bf16 in LDS (the rounding the
// unfused GEMM output had), then one pass per 8-column chunk reads its gate and up chunks,
// writes them to aux ([M, 2I] gate | up, for the backward) when asked, and combines them in
// fp32 exactly as k_swiglu_fwd does. Stores are buffer stores on one descriptor per output
// (rows past M fall outside its range and are dropped: no per-row test), a lane's column offset
// in a VGPR and the row step in the scalar offset.
// ST (diagnostic, forced variant 28): mk[0] = s_memtime after the LDS staging (incl. its barrier),
// mk[1] = after the combined pass behind a vmcnt(0) drain.
template <int TM, int TN, int MT, int NT, int NTHR, bool L32 = false, bool ST = false>
__device__ __forceinline__ void epilogue_glu(const GemmP& p, const f32x4 (&acc)[MT][NT], char* smem, int m0, int nb, int wm,
                                             int wn, int lane, int tid, uint64_t* mk = nullptr) {
    float alpha = p.alpha;
    if (p.alpha_dev) alpha *= *p.alpha_dev;
    constexpr int RS = 256 * 2 + 16;
    const int ln = lane_now();
    if (alpha == 1.f) {
        epi_to_lds_raw<TM, TN, MT, NT, L32>(acc, smem, RS, wm, wn, ln);
    } else {
        f32x4 bcol[NT];
#pragma unroll
        for (int j = 0; j < NT; ++j) bcol[j] = (f32x4){0.f, 0.f, 0.f, 0.f};
        epi_to_lds<KD_ACT_NONE, TM, TN, MT, NT, false, L32>(acc, smem, RS, alpha, bcol, wm, wn, ln, 0, 256);
    }
    __syncthreads();
    if (ST) mk[0] = __builtin_amdgcn_s_memtime();
    constexpr int RSTEP = NTHR / 16, PER = 256 / RSTEP;
    const int t = (wm * (256 / TN) + wn) * 64 + ln;   // == tid, from wave-uniform values and v_mbcnt
    const int c = t & 15, lr0 = t >> 4;
    const int rows = min(256, p.M - m0);
    const int I = p.glu;
    const __amdgpu_buffer_rsrc_t rc = make_rsrc((const bf16*)p.C + (int64_t)m0 * p.ldc + nb, rec_bytes(rows, p.ldc));
    const uint32_t vc = (uint32_t)((lr0 * p.ldc + c * 8) * 2);
    const int sc = RSTEP * (int)p.ldc * 2;
    const char* src = smem + lr0 * RS + c * 16;
    if (p.aux) {
        const __amdgpu_buffer_rsrc_t ra = make_rsrc(p.aux + (int64_t)m0 * p.ld_aux, rec_bytes(rows, p.ld_aux));
        const uint32_t vg = (uint32_t)((lr0 * p.ld_aux + nb + c * 8) * 2), vu = vg + (uint32_t)(I * 2);
        const int sa = RSTEP * (int)p.ld_aux * 2;
#pragma unroll 4
        for (int it = 0; it < PER; ++it) {
            const u32x4 g = *(const u32x4*)(src + it * RSTEP * RS);
            const u32x4 u = *(const u32x4*)(src + it * RSTEP * RS + 256);
            __builtin_amdgcn_raw_buffer_store_b128(g, ra, vg, it * sa, 0);
            __builtin_amdgcn_raw_buffer_store_b128(u, ra, vu, it * sa, 0);
            const u32x4 o = {silu_mul_pair(g[0], u[0]), silu_mul_pair(g[1], u[1]), silu_mul_pair(g[2], u[2]),
                             silu_mul_pair(g[3], u[3])};
            __builtin_amdgcn_raw_buffer_store_b128(o, rc, vc, it * sc, 0);
        }
    } else {
#pragma unroll 4
        for (int it = 0; it < PER; ++it) {
            const u32x4 g = *(const u32x4*)(src + it * RSTEP * RS);
            const u32x4 u = *(const u32x4*)(src + it * RSTEP * RS + 256);
            const u32x4 o = {silu_mul_pair(g[0], u[0]), silu_mul_pair(g[1], u[1]), silu_mul_pair(g[2], u[2]),
                             silu_mul_pair(g[3], u[3])};
            __builtin_amdgcn_raw_buffer_store_b128(o, rc, vc, it * sc, 0);
        }
    }
    (void)lane; (void)tid;
    if (ST) { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); mk[1] = __builtin_amdgcn_s_memtime(); }
}
#ifdef KD_AB_BUILD
#include "gemm_glu_epi_v0.inc"   // tools/ab/gemm_glu_epi_v0.inc: the round-4 SwiGLU epilogue (KD_GLU_EPI_V0)
#endif  // KD_AB_BUILD

// =============================================================================
// v3: the tiles above and their 4-stage LDS ring, software-pipelined one stage deeper: the
// fragments of stage t+1 are read into a second register set WHILE the MFMAs of stage t
// run, and the DMA of stage t+4 is interleaved with them too (sched_group_barrier), so
// after a barrier the MFMA pipe never waits for LDS or for DMA issue.
// Iteration t: lgkmcnt(0) [frags of t in registers, my reads of buffer t done] ->
//   vmcnt(stage t+1 landed) -> s_barrier [everyone done with buffer t; stage t+1 visible]
//   -> {DMA stage t+4 -> buffer t%4, LDS reads of stage t+1 -> set nxt} || MFMAs(t, set cur)
// =============================================================================
template <int BM, int BN, bool A_MN, bool B_MN, int NS = NST>
__global__ void __launch_bounds__(NTH2, 1) k_gemm3(GemmP p_) {
    GemmP p = p_;
    if (p.gy > 1) {   // split-K: this grid row owns K range [k0, k0 + kchunk) -> fp32 partial plane
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
    tile_of(p.gx, (p.M + BM - 1) / BM, (p.N + BN - 1) / BN, tm, tn, p.tile0, p.gm);
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
        wait_vm<(NS - 2) * G>();                                                                          \
        __builtin_amdgcn_s_barrier();                                                                     \
        __builtin_amdgcn_sched_barrier(0);                                                                \
        dma(t + NS);                                                                                      \
        {                                                                                                 \
            const char* na = smem + ((t + 1) % NS) * SS;                                                  \
            _Pragma("unroll") for (int j = 0; j < NT; ++j) NXT_B[j] = frag2<BN, B_MN>(na + SA, wn * TN + j * 16, lane); \
            _Pragma("unroll") for (int i = 0; i < MT; ++i) NXT_A[i] = frag2<BM, A_MN>(na, wm * TM + i * 16, lane);      \
        }                                                                                                 \
        _Pragma("unroll") for (int i = 0; i < MT; ++i)                                                    \
            _Pragma("unroll") for (int j = 0; j < NT; ++j)                                                \
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(CUR_B[j], CUR_A[i], acc[i][j], 0, 0, 0); \
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
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");   // incl. the asm tr reads
    __builtin_amdgcn_sched_barrier(0);
    __syncthreads();
    epilogue2<BM, BN, WM, WN, TM, TN, MT, NT, NTH2, !A_MN && !B_MN>(p, acc, smem, m0, n0, wm, wn, lane, tid);
}

// =============================================================================
// v8: 256x256 tile, FOUR waves (one per SIMD), each 128x128 of C = 8x8 MFMA 16x16x32
// tiles, v3's 4-slot BK=32 LDS-DMA ring (three stages in flight). The 256 accumulator
// registers live in the AGPR file for the whole kernel (MFMA through asm with an "a"
// operand): with the builtin, hipcc splits them over both files and moves ~330
// registers per iteration between them. VGPRs hold two fragment sets (stage t in use,
// stage t+1 being read) and the loop-invariant per-lane DMA offsets.
// One wave per SIMD issues everything itself, so every non-MFMA instruction goes into its
// own MFMA gap (a DMA issue costs ~60 cycles of MFMA pipe if it shares a 16-cycle gap with
// other work; MI355X_MICROARCH.md constants table):
//   step t (slot t%4, unrolled x4 so every slot index is a constant), unit u = 0..7:
//     8 MFMA acc[u][*] += CA[u] * CB[*]; between them: 1 DMA of stage t+4 -> slot t%4,
//     and in units 0-3 four fragment reads of stage t+1 -> NXT
//     before the last MFMA of the step: lgkmcnt(0) [NXT complete] ; vmcnt(16) [stage t+2
//     landed] ; s_barrier
// WAR: slot (t+1)%4 (refilled in step t+1) held stage t+1, whose reads every wave retired
// (lgkmcnt 0) before the barrier at the end of step t. RAW: stage t+2 is read in step t+1,
// after the barrier that follows every wave's vmcnt for it. DMA past the last stage is
// issued anyway (all lanes out of range: no memory traffic, the slot is never read) so
// the counts stay uniform.
// K-major operands: one descriptor per block, per-lane voffset fixed, the stage's k
// offset in soffset. MN-major: one descriptor per stage (its k rows), voffset fixed.
// =============================================================================
constexpr int NTH8 = 256, NS8 = 4;

__device__ __forceinline__ void mfma_agpr(f32x4& acc, const bf16x8& a, const bf16x8& b) {
    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}

// The last MFMA of every k-step, with the wait states its result needs before ANY read of the
// accumulators in the SAME asm statement, taken when `last` (the tile's final k-step) is set.
// asm MFMAs are invisible to the compiler's hazard recognizer: a register-allocator copy of an
// accumulator placed at the k-loop exit (a merge of the remainder branches) read AGPRs before
// the MFMA writing them had finished (81,336 wrong elements in the persistent-v8 experiment,
// DESIGN §5).  With the drain inside this statement nothing can be scheduled between the final
// MFMA and its wait states; earlier MFMAs retire in order before it.  32 wait states >= the
// 16-pass XDL result latency (MI355X ISA: VALU read of an XDL result).  The branch is inside
// the asm (scalar, uniform): no new basic block for the allocator to put copies in.
__device__ __forceinline__ void mfma_agpr_last(f32x4& acc, const bf16x8& a, const bf16x8& b, int last) {
    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0\n\t"
                 "s_cmp_eq_u32 %3, 0\n\t"
                 "s_cbranch_scc1 .Lkd_mfma_nodrain%=\n\t"
                 "s_nop 15\n\t"
                 "s_nop 15\n"
                 ".Lkd_mfma_nodrain%=:"
                 : "+a"(acc) : "v"(a), "v"(b), "s"(__builtin_amdgcn_readfirstlane(last)) : "scc");
}

// per-lane byte offset of this wave's DMA instruction i (0..15 of an operand stage)
template <bool MN>
__device__ __forceinline__ uint32_t voff8(int i, int lane, int64_t ld, int r0, int rows_total) {
    if (!MN) {   // [256 rows][32 k]: 16 rows x 64 B per instruction
        const int row = 16 * i + (lane >> 2);
        const int gc = (lane & 3) ^ f4(row);
        return (uint32_t)((int64_t)row * ld * 2 + gc * 16);
    } else {     // [32 k][256 rows]: 2 k-rows x 512 B per instruction
        const int kr = 2 * i + (lane >> 5);
        const int gc = (lane & 31) ^ (int)sw_mn(kr);
        return (r0 + gc * 8 < rows_total) ? (uint32_t)((int64_t)kr * ld * 2 + gc * 16) : OOB;
    }
}

// EXP: bit 2 = the fused SwiGLU build (KD_ACT_SWIGLU: gathered gate|up B rows, GLU epilogue;
// its own kernel, so its launches are exactly the gate|up GEMMs in a kernel trace; the
// production non-GLU build carries no GLU code). Diagnostic variants 17-19 only: bit 0 writes per-wave s_memtime
// cycle totals (step-end sync, MFMA units, prologue, epilogue) as uint32 to p.aux (which
// then carries no pre-activation output); bit 1 drops the in-loop DMA (timing ablation:
// WRONG results); bit 6 re-reads stage 0 for every stage (same addresses, L2-hot:
// separates issue cost from memory-system cost; WRONG results).
// Bit 3 (K-major x K-major only): REGISTER staging instead of LDS-DMA. A k-step's 64
// MFMAs (16x16x32, each holding the SIMD's vector issue for 8 of its 16 cycles) leave 512
// issue cycles for everything else, and its 8 LDS-DMA pieces cost ~60 each (more beside
// 16 fragment reads: MI355X_MICROARCH constants table) — the measured step is 1243 cycles,
// not 1024, and the kernel keeps the matrix pipe 65-66% busy where hipBLASLt keeps it 77-81%
// (profiles/r03/pmc_vs_blas.txt). Here unit u of step t writes piece u of stage t+4 (loaded
// during step t-1) into slot t%4 with one ds_write_b128 at the same lane-linear position the
// DMA wrote, then loads piece u of stage t+5 into the same 4 VGPRs (buffer load, the same
// pre-swizzled source offset): same LDS image, same ring, same barriers. Measured (forced
// variant 22, tools/ab_gemm_rs.py): bit-exact, and 2-11% SLOWER than the LDS-DMA build on every
// forward shape of the step (gate|up+SwiGLU 1291 -> 1379 us, lm_head 5320 -> 5808 us): the DMA
// issue is not what holds v8 below hipBLASLt's MFMA-busy fraction. Kept as a forced variant only.
// one 256x256 output tile over p's K range (the whole K, a split-K plane or a stream-K piece)
// the in-launch fold of a stream-K tile shared by several runs (GemmP.sk_*): piece `piece` of `np`
// of SK tile `t` (first k-step tb of the SK range's tot steps over G runs; run wf holds piece 0)
// (split-K with the in-launch fold, variant 32: tot = 0, the tile's S splits are pieces wf = 0 .. np - 1
// with slots split_base + piece)
struct SkFold {
    float* part; int* cnt;
    int64_t tot, tb;
    int G, wf, piece, np, t;
    int64_t split_base;
};
constexpr int SK_TILE_F32 = 256 * 256;   // one partial tile: 4 waves x 64 accumulator quads x 64 lanes x 4
// a run's partial slots: 0 = its first piece (its range starts inside that tile), 1 = its last; in
// split mode the tile's S consecutive slots
__device__ __forceinline__ float* sk_slot(const SkFold& f, int w) {
    if (f.tot == 0) return f.part + (f.split_base + w) * SK_TILE_F32;
    const int64_t s0 = f.tot * w / f.G;
    return f.part + ((int64_t)w * 2 + (s0 >= f.tb ? 0 : 1)) * SK_TILE_F32;
}
// after a piece's main loop: publish its accumulators, take the tile's ticket; the last arriver
// folds every piece in piece order (x0 + x1 + ...: the same sum whichever piece arrives last) into
// acc and returns true (it then runs the epilogue), the others return false.  Guideline 16 counter
// form: plain 16-B stores, every wave drains, barrier, one lane's agent-scope release + ticket;
// the last arriver's agent-scope acquire before any wave reads another piece.
__device__ __forceinline__ bool sk_fold_tile(const SkFold& f, f32x4 (&acc)[8][8], int tid, int lane, int wid,
                                          char* smem) {
    const int64_t lo = ((int64_t)wid * 64 * 64 + lane) * 4;   // + a * 256: quad a of this lane
    float* mine = sk_slot(f, f.wf + f.piece) + lo;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) *(f32x4*)(mine + (i * 8 + j) * 256) = acc[i][j];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int* flag = (int*)smem;   // the staging array (the one __shared__ object): free after the loop
    if (tid == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const int old = __hip_atomic_fetch_add(f.cnt + f.t, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int last = old == f.np - 1;
        if (last) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        flag[0] = last;
    }
    __syncthreads();
    const int last = flag[0];
    __syncthreads();   // the epilogue restages through the same LDS
    if (!last) return false;
#pragma unroll
    for (int h = 0; h < 4; ++h) {   // 16 quads at a time: 64 VGPRs of loads in flight
        f32x4 v[16];
        if (f.piece == 0) {
#pragma unroll
            for (int a = 0; a < 16; ++a) v[a] = acc[(h * 16 + a) / 8][(h * 16 + a) % 8];
        } else {
            const float* src = sk_slot(f, f.wf) + lo;
#pragma unroll
            for (int a = 0; a < 16; ++a) v[a] = *(const f32x4*)(src + (h * 16 + a) * 256);
        }
        for (int pc = 1; pc < f.np; ++pc) {
            if (pc == f.piece) {
#pragma unroll
                for (int a = 0; a < 16; ++a) v[a] += acc[(h * 16 + a) / 8][(h * 16 + a) % 8];
            } else {
                const float* src = sk_slot(f, f.wf + pc) + lo;
                f32x4 x[16];
#pragma unroll
                for (int a = 0; a < 16; ++a) x[a] = *(const f32x4*)(src + (h * 16 + a) * 256);
#pragma unroll
                for (int a = 0; a < 16; ++a) v[a] += x[a];
            }
        }
#pragma unroll
        for (int a = 0; a < 16; ++a) acc[(h * 16 + a) / 8][(h * 16 + a) % 8] = v[a];
    }
    return true;
}

template <bool A_MN, bool B_MN, int EXP>
__device__ __forceinline__ void g8_tile(GemmP p, int tm, int tn, char* smem, const SkFold* fold = nullptr) {
    constexpr bool STAMP = EXP & 1, NODMA = EXP & 2, HOT = EXP & 64;
    constexpr bool RS = (EXP & 8) && !A_MN && !B_MN;
    // bit 5: the epilogue also writes the tile's row statistics (kd_gemm_desc.row_stats, the
    // lm_head GEMMs of the KD step): a build of its own, so the plain forward kernel carries none
    // of that code and the lm_head launches are their own line in a kernel trace
    constexpr bool RSTATS = (EXP & 32) && !A_MN && !B_MN;
    // bit 8: B PRE-TILED (kd_gemm_desc.b_pretiled, kd_gemm_pretile): the K-major B operand is stored
    // as each 256-row tile's stages, [tile][stage][256 rows][64 B] with the LDS chunk swizzle (and, for
    // the SwiGLU build, the gate|up row gather) already applied, zero-padded past N and K, so every
    // DMA instruction reads ONE contiguous KiB (8 whole cache lines) instead of 16 half-lines, and
    // lands the same LDS image (bit-identical results)
    constexpr bool TB = (EXP & 256) && !B_MN && !RS;
    const int nkt = (p.K + BK2 - 1) / BK2;   // stages per pre-tiled tile

    uint32_t* stamps = nullptr;
    // the SwiGLU stamp build (variant 28) keeps its aux output: stamps go to the workspace (p.sk_ws)
    if (STAMP) {
        if ((EXP & 4) && !B_MN) stamps = (uint32_t*)p.sk_ws;
        else { stamps = (uint32_t*)p.aux; p.aux = nullptr; }
    }
    uint64_t mk[2] = {0, 0};
    uint64_t s_pro = 0, s_bar = 0, s_units = 0, s_epi = 0, ts0 = 0;
    uint64_t rt0 = 0;
    if (STAMP) { ts0 = __builtin_amdgcn_s_memtime(); rt0 = __builtin_amdgcn_s_memrealtime(); }
    constexpr int SA = 256 * BK2 * 2, SS = 2 * SA;   // 16 KiB per operand, 32 KiB per slot
    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);   // provably uniform: LDS-DMA bases in SGPRs
    const int wm = wid >> 1, wn = wid & 1;
    const int m0 = tm * 256, n0 = tn * 256;
    const int K = p.K;
    const int nk = (K + BK2 - 1) / BK2, nk_full = K / BK2;
    // staggered k start (GemmP.stagger): stage st of the loop reads K stage (st + rot) mod nk; the
    // stages past the end (st >= nk) stay the zero-filled out-of-range DMAs they are unrotated. rot
    // is a function of the tile ROW group alone (grp of ngrp, the grouped order's g rows each; a
    // group is whole XCD chunks), so every launch over the same rows -- the SwiGLU build, pre-tiled
    // B, the row-statistics build, the plain GEMM -- sums each output in the same order. Short K
    // loops (nk < 64: the student's K = 896 lm_head measured 1-2 % slower rotated) start at 0.
    int rot = 0;
    if (p.stagger && nk_full == nk && nk >= 64) {
        const int g = p.stag_g > 0 ? p.stag_g : (p.gm > 0 ? p.gm : GM_GROUP), ngrp = ((p.M + 255) / 256 + g - 1) / g;
        rot = (int)(((int64_t)(tm / g) * nk) / ngrp);
    }
    auto kst = [&](int st) { return (rot == 0 || st >= nk) ? st : (st + rot >= nk ? st + rot - nk : st + rot); };
    const __amdgpu_buffer_rsrc_t rsAk = make_rsrc(p.A + (A_MN ? 0 : (int64_t)m0 * p.lda), A_MN ? 0u : rec_bytes(min(256, p.M - m0), p.lda));
    constexpr bool glu = !B_MN && (EXP & 4);   // gate rows [nb, nb+128) and up rows [I+nb, I+nb+128)
    const int nb = tn * 128;
    const __amdgpu_buffer_rsrc_t rsBk =
        TB ? make_rsrc(p.B + (int64_t)tn * nkt * (256 * BK2), (uint32_t)nkt * (256 * BK2 * 2))
           : glu ? make_rsrc(p.B, rec_bytes(p.N, p.ldb))
                 : make_rsrc(p.B + (B_MN ? 0 : (int64_t)n0 * p.ldb), B_MN ? 0u : rec_bytes(min(256, p.N - n0), p.ldb));
    uint32_t va[4], vb[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        va[u] = voff8<A_MN>(wid * 4 + u, lane, p.lda, m0, p.M);
        vb[u] = voff8<B_MN>(wid * 4 + u, lane, p.ldb, n0, p.N);
        if (glu && !TB) {   // tile row r -> weight row (r < 128 ? nb + r : I + nb + r - 128); same LDS swizzle
            const int row = 16 * (wid * 4 + u) + (lane >> 2);
            const int gc = (lane & 3) ^ f4(row);
            const int wrow = row < 128 ? nb + row : p.glu + nb + row - 128;
            vb[u] = (uint32_t)((int64_t)wrow * p.ldb * 2 + gc * 16);
        }
        if (TB) vb[u] = (uint32_t)((wid * 4 + u) * 1024 + lane * 16);   // lane-linear KiB of the stage image
    }
    // one DMA instruction (u: 0..3 operand A, 4..7 operand B) of stage st into slot sl;
    // FULL: the stage lies wholly inside K (no per-lane tail masking)
    auto dma = [&](int st, int sl, int u, auto full_tag) {
        constexpr bool FULL = decltype(full_tag)::value;
        if (NODMA) return;
        const bool isA = u < 4;
        const bool mn = isA ? A_MN : B_MN;
        const int i = wid * 4 + (u & 3);
        char* dst = smem + sl * SS + (isA ? 0 : SA) + i * 1024;
        uint32_t v = isA ? va[u & 3] : vb[u & 3];
        if (TB && !isA) {   // one contiguous KiB of stage st (zero-padded past K); past the last stage: zeros
            int soff = kst(st) * (256 * BK2 * 2);
            if (!FULL && st >= nkt) { v = OOB; soff = 0; }
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rsBk, (lds_void_t*)dst, 16, v, soff, 0, 0);
            return;
        }
        if (!mn) {
            int soff = HOT ? 0 : kst(st) * BK2 * 2;
            if (!FULL) {
                const int kleft = K - st * BK2;   // valid k of this stage (<= 0: past the end)
                if (kleft < BK2) {                // zero the chunks at k >= K
                    const int row = 16 * i + (lane >> 2);
                    const int gc = (lane & 3) ^ f4(row);
                    if (gc * 8 >= kleft) v = OOB;
                    if (kleft <= 0) soff = 0;
                }
            }
            __builtin_amdgcn_raw_ptr_buffer_load_lds(isA ? rsAk : rsBk, (lds_void_t*)dst, 16, v, soff, 0, 0);
        } else {
            const bf16* base = isA ? p.A + m0 : p.B + n0;
            const int64_t ld = isA ? p.lda : p.ldb;
            const int kv = FULL ? BK2 : max(0, min(BK2, K - st * BK2));
            const int ks = kst(st);
            const __amdgpu_buffer_rsrc_t rs = make_rsrc(base + (int64_t)(FULL ? ks * BK2 : min(ks * BK2, K)) * ld, rec_bytes(kv, ld));
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void_t*)dst, 16, v, 0, 0, 0);
        }
    };
    using FullT = std::integral_constant<bool, true>;
    using PartT = std::integral_constant<bool, false>;
    // register staging (RS): piece u of stage st -> rsb[u] (the DMA's source offsets), and
    // rsb[u] -> its lane-linear 16 B of slot sl
    u32x4 rsb[8];
    auto rs_load = [&](int st, int u, auto full_tag) {
        constexpr bool FULL = decltype(full_tag)::value;
        const bool isA = u < 4;
        const int i = wid * 4 + (u & 3);
        uint32_t v = isA ? va[u & 3] : vb[u & 3];
        int soff = kst(st) * BK2 * 2;
        if (!FULL) {
            const int kleft = K - st * BK2;
            if (kleft < BK2) {
                const int row = 16 * i + (lane >> 2);
                const int gc = (lane & 3) ^ f4(row);
                if (gc * 8 >= kleft) v = OOB;
                if (kleft <= 0) soff = 0;
            }
        }
        rsb[u] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(isA ? rsAk : rsBk, v, soff, 0));
    };
    auto rs_write = [&](int sl, int u) {
        const int i = wid * 4 + (u & 3);
        *(u32x4*)(smem + sl * SS + (u < 4 ? 0 : SA) + i * 1024 + lane * 16) = rsb[u];
    };
    f32x4 acc[8][8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
    const int ra = wm * 128, cb = wn * 128;
    if (RS) {   // stages 0..3 into slots 0..3 (two register sets in flight), then stage 4 -> rsb
        u32x4 alt[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) rs_load(0, u, PartT{});
#pragma unroll
        for (int st = 0; st < NS8; ++st) {
#pragma unroll
            for (int u = 0; u < 8; ++u) alt[u] = rsb[u];
#pragma unroll
            for (int u = 0; u < 8; ++u) rs_load(st + 1, u, PartT{});
#pragma unroll
            for (int u = 0; u < 8; ++u) *(u32x4*)(smem + st * SS + (u < 4 ? 0 : SA) + (wid * 4 + (u & 3)) * 1024 + lane * 16) = alt[u];
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    } else {
#pragma unroll
        for (int st = 0; st < NS8; ++st)
#pragma unroll
            for (int u = 0; u < 8; ++u) dma(st, st, u, PartT{});
        if (NODMA) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        else wait_vm<24>();   // stage 0 landed (stages 1..3 may stay in flight)
    }
    __builtin_amdgcn_s_barrier();
    uint64_t tprev = 0;
    if (STAMP) { tprev = __builtin_amdgcn_s_memtime(); s_pro = tprev - ts0; }
    bf16x8 xa[8], xb[8], ya[8], yb[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
        xa[u] = frag2<256, A_MN>(smem, ra + u * 16, lane);
        xb[u] = frag2<256, B_MN>(smem + SA, cb + u * 16, lane);
    }
    // step-end sync (also closes the prologue): my reads of the current slot are done,
    // the stage the next step reads has landed for every wave
#define KD_G8_SYNC()                                                                                         \
    {                                                                                                         \
        uint64_t ta_ = 0, tb_ = 0;                                                                            \
        if (STAMP) ta_ = __builtin_amdgcn_s_memtime();                                                        \
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                                                    \
        if (!NODMA && !RS) wait_vm<16>();                                                                     \
        __builtin_amdgcn_s_barrier();                                                                         \
        if (STAMP) {                                                                                          \
            tb_ = __builtin_amdgcn_s_memtime();                                                               \
            s_units += ta_ - tprev; s_bar += tb_ - ta_; tprev = tb_;                                          \
        }                                                                                                     \
    }
    KD_G8_SYNC()
    __builtin_amdgcn_sched_barrier(0);
#define KD_SB __builtin_amdgcn_sched_barrier(0);
#define KD_G8_STEP(SL, CA, CB, NA, NB, FT)                                                                   \
    {                                                                                                         \
        const int t_ = t + (SL);                                                                              \
        const char* na_ = smem + (((SL) + 1) % NS8) * SS;                                                     \
        _Pragma("unroll") for (int u = 0; u < 8; ++u) {                                                       \
            mfma_agpr(acc[u][0], CB[0], CA[u]); KD_SB                                                         \
            if (RS) { rs_write((SL), u); rs_load(t_ + NS8 + 1, u, FT{}); }                                    \
            else dma(t_ + NS8, (SL), u, FT{});                                                                \
            KD_SB                                                                                             \
            mfma_agpr(acc[u][1], CB[1], CA[u]); KD_SB                                                         \
            if (u < 4) NA[2 * u] = frag2<256, A_MN>(na_, ra + 2 * u * 16, lane);                              \
            KD_SB                                                                                             \
            mfma_agpr(acc[u][2], CB[2], CA[u]); mfma_agpr(acc[u][3], CB[3], CA[u]); KD_SB                     \
            if (u < 4) NB[2 * u] = frag2<256, B_MN>(na_ + SA, cb + 2 * u * 16, lane);                         \
            KD_SB                                                                                             \
            mfma_agpr(acc[u][4], CB[4], CA[u]); mfma_agpr(acc[u][5], CB[5], CA[u]); KD_SB                     \
            if (u < 4) NA[2 * u + 1] = frag2<256, A_MN>(na_, ra + (2 * u + 1) * 16, lane);                    \
            KD_SB                                                                                             \
            mfma_agpr(acc[u][6], CB[6], CA[u]); KD_SB                                                         \
            if (u < 4) NB[2 * u + 1] = frag2<256, B_MN>(na_ + SA, cb + (2 * u + 1) * 16, lane);               \
            if (u == 7) KD_G8_SYNC()                                                                          \
            KD_SB                                                                                             \
            if (u == 7) mfma_agpr_last(acc[u][7], CB[7], CA[u], t_ + 1 == nk);                                \
            else mfma_agpr(acc[u][7], CB[7], CA[u]);                                                          \
            KD_SB                                                                                             \
        }                                                                                                     \
    }
    int t = 0;
    for (; t + 2 * NS8 + (RS ? 1 : 0) <= nk_full; t += NS8) {   // every DMA / staged load of these steps lies inside K
        KD_G8_STEP(0, xa, xb, ya, yb, FullT)
        KD_G8_STEP(1, ya, yb, xa, xb, FullT)
        KD_G8_STEP(2, xa, xb, ya, yb, FullT)
        KD_G8_STEP(3, ya, yb, xa, xb, FullT)
    }
    for (; t + NS8 <= nk; t += NS8) {
        KD_G8_STEP(0, xa, xb, ya, yb, PartT)
        KD_G8_STEP(1, ya, yb, xa, xb, PartT)
        KD_G8_STEP(2, xa, xb, ya, yb, PartT)
        KD_G8_STEP(3, ya, yb, xa, xb, PartT)
    }
    const int rem = nk - t;
    if (rem > 0) KD_G8_STEP(0, xa, xb, ya, yb, PartT)
    if (rem > 1) KD_G8_STEP(1, ya, yb, xa, xb, PartT)
    if (rem > 2) KD_G8_STEP(2, xa, xb, ya, yb, PartT)
#undef KD_G8_STEP
#undef KD_G8_SYNC
#undef KD_SB
    // drain the ring (out-of-range DMAs still write LDS) and the MFMA pipe before the
    // accumulators are read back (asm MFMAs are invisible to the hazard recognizer)
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_nop 15\n\ts_nop 15" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    uint64_t te0 = 0;
    if (STAMP) { te0 = __builtin_amdgcn_s_memtime(); s_units += te0 - tprev; }
    __syncthreads();
    if constexpr ((EXP & (1024 | 2048)) != 0) {   // stream-K / split-K fold builds: a published piece ends here
        if (fold != nullptr && !sk_fold_tile(*fold, acc, tid, lane, wid, smem)) return;
    }
#ifdef KD_AB_BUILD
    if constexpr (!A_MN && !B_MN && (EXP & 512)) epilogue_glu_v0<128, 128, 8, 8, NTH8>(p, acc, smem, m0, nb, wm, wn, lane, tid);
    else
#endif
    if (!A_MN && !B_MN && glu) epilogue_glu<128, 128, 8, 8, NTH8, false, STAMP>(p, acc, smem, m0, nb, wm, wn, lane, tid, mk);
    else epilogue2<256, 256, 2, 2, 128, 128, 8, 8, NTH8, !A_MN && !B_MN, RSTATS, false, STAMP>(p, acc, smem, m0, n0, wm, wn, lane, tid, mk);
    if (STAMP) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const uint64_t te1 = __builtin_amdgcn_s_memtime();
        s_epi = te1 - te0;
        if (lane == 0) {
            uint32_t* o = stamps + ((int64_t)(blockIdx.y * p.gx + blockIdx.x) * 4 + wid) * 8;
            // glu: o[1] = LDS staging (incl. the barrier), o[2] = the aux + silu * up pass;
            // plain bf16 output: o[1] = LDS staging (incl. the barrier), o[2] = the flush's store
            // issue, and the epilogue total o[5] includes the store drain (vmcnt(0)) after it
            o[0] = (uint32_t)s_pro; o[1] = mk[0] ? (uint32_t)(mk[0] - te0) : 0; o[2] = mk[1] ? (uint32_t)(mk[1] - mk[0]) : 0;
            o[3] = (uint32_t)s_bar;
            o[4] = (uint32_t)s_units; o[5] = (uint32_t)s_epi; o[6] = (uint32_t)(te1 - ts0); o[7] = (uint32_t)nk;
            if (glu && wid == 0) {   // placement record per workgroup, past the per-wave block:
                // real-time start / end (100 MHz), HW_ID (CU / SE of this workgroup), XCC_ID
                uint32_t* w = stamps + (int64_t)p.gx * 4 * 8 + (int64_t)blockIdx.x * 4;
                w[0] = (uint32_t)rt0; w[1] = (uint32_t)__builtin_amdgcn_s_memrealtime();
                w[2] = (uint32_t)__builtin_amdgcn_s_getreg((31 << 11) | 4);
                w[3] = (uint32_t)__builtin_amdgcn_s_getreg((31 << 11) | 20);
            }
        }
    }
}

#ifdef KD_AB_BUILD   // v8n: no faster than the plan in the step; A/B library only
#include "gemm_v8n.inc"   // tools/ab/gemm_v8n.inc: v8n (256x128 tiles, two workgroups per CU, forced variant 30)
#endif  // KD_AB_BUILD

#ifdef KD_AB_BUILD   // v11 / v12: measured slower than v8 in the step; tools' A/B library only
#include "gemm_v11_v12.inc"   // tools/ab/gemm_v11_v12.inc: v11 (32x32x16 MFMAs) and v12 (whole-line staging)
#endif  // KD_AB_BUILD

template <bool A_MN, bool B_MN, int EXP = 0>
__global__ void __launch_bounds__(NTH8, 1) k_gemm8(GemmP p_) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tiles_m = (p_.M + 255) / 256, tiles_n = (p_.N + 255) / 256;
    if constexpr ((EXP & 1024) != 0) {   // the stream-K build (variant 21): data-parallel whole waves, then runs
        const int nkt = p_.sk_steps, G = p_.sk_grid;
        const bool dp = (int)blockIdx.x < p_.sk_dp;
        // run w of workgroup i (sk_dp % 8 == 0, so workgroup i sits on XCD i % 8): the runs of one XCD
        // are consecutive, i.e. a contiguous stretch of the grouped tile order (L2-shared panels)
        const int i = (int)blockIdx.x - p_.sk_dp;
        const int q8 = G / 8, r8 = G % 8, x = i % 8;
        const int w = (x < r8 ? x * (q8 + 1) : r8 * (q8 + 1) + (x - r8) * q8) + i / 8;
        const int64_t tot = (int64_t)(tiles_m * tiles_n - p_.sk_dp) * nkt;
        int64_t s0 = dp ? 0 : tot * w / G;
        const int64_t s1 = dp ? 1 : tot * (w + 1) / G;
        while (s0 < s1) {   // ONE g8_tile call site (one inlined copy of the tile body)
            GemmP q = p_;
            int tm, tn;
            int64_t e = s1;
            SkFold f;
            const SkFold* fp = nullptr;
            if (dp) {
                tile_of(p_.sk_dp, tiles_m, tiles_n, tm, tn, 0, p_.gm);
            } else {
                const int t = (int)(s0 / nkt);
                const int64_t tb = (int64_t)t * nkt;
                e = min(s1, tb + nkt);
                const int wf = sk_wg_of(tb, tot, G), wl = sk_wg_of(tb + nkt - 1, tot, G);
                const int64_t k0 = (s0 - tb) * BK2;
                q.K = (int)min((int64_t)p_.K - k0, (e - s0) * BK2);
                q.A += A_MN ? k0 * q.lda : k0;
                q.B += B_MN ? k0 * q.ldb : k0;
                tile_grouped(p_.sk_dp + t, tiles_m, tiles_n, tm, tn, p_.gm);
                if (wl > wf) {   // a piece of a shared tile: folded in this launch by its last arriver
                    q.stagger = 0;
                    f = SkFold{p_.sk_ws, p_.sk_cnt, tot, tb, G, wf, w - wf, wl - wf + 1, t, 0};
                    fp = &f;
                }
            }
            g8_tile<A_MN, B_MN, EXP>(q, tm, tn, smem, fp);
            s0 = e;
            __syncthreads();   // the next piece's DMA refills the LDS the epilogue staged through
        }
        return;
    }
    if constexpr ((EXP & 2048) != 0) {   // split-K with the in-launch fold (variant 32): no partial planes,
        // no reduce launch -- split blockIdx.y publishes its accumulators, the tile's last arriver sums the
        // S pieces in split order and runs the full epilogue
        GemmP q = p_;
        const int64_t k0 = (int64_t)blockIdx.y * q.kchunk;
        q.K = (int)min((int64_t)q.K - k0, q.kchunk);
        q.A += A_MN ? k0 * q.lda : k0;
        q.B += B_MN ? k0 * q.ldb : k0;
        q.stagger = 0;
        int tm, tn;
        tile_of(q.gx, tiles_m, tiles_n, tm, tn, q.tile0, q.gm);
        // this launch's tile index (tile_of's remap without the first-tile offset): tickets and slots
        const int b = blockIdx.x, q8 = q.gx / 8, r8 = q.gx % 8, x = b % 8;
        const int lt = (x < r8 ? x * (q8 + 1) : r8 * (q8 + 1) + (x - r8) * q8) + b / 8;
        const SkFold f{q.sk_ws, q.sk_cnt, 0, 0, 1, 0, (int)blockIdx.y, q.gy, lt, (int64_t)lt * q.gy};
        g8_tile<A_MN, B_MN, EXP>(q, tm, tn, smem, &f);
        return;
    }
    GemmP p = p_;
    if (p.gy > 1) {   // split-K: this grid row owns K range [k0, k0 + kchunk) -> fp32 partial plane
        const int64_t k0 = (int64_t)blockIdx.y * p.kchunk;
        p.K = (int)min((int64_t)p.K - k0, p.kchunk);
        p.A += A_MN ? k0 * p.lda : k0;
        p.B += B_MN ? k0 * p.ldb : k0;
        p.C = (float*)p.C + (int64_t)blockIdx.y * p.split_stride;
    }
    int tm, tn;
    tile_of(p.gx, tiles_m, tiles_n, tm, tn, p.tile0, p.gm);
    g8_tile<A_MN, B_MN, EXP>(p, tm, tn, smem);
}

#ifdef KD_AB_BUILD   // v9: equal speed to v8 on the step's shapes, not in the plan; A/B library only
#include "gemm_v9.inc"   // tools/ab/gemm_v9.inc: v9 (eight-wave ping-pong)
#include "gemm_blas.inc"   // tools/ab/gemm_blas.inc: plain GEMMs through hipBLASLt (KD_GEMM_BLAS)
#endif  // KD_AB_BUILD


// =============================================================================
// f8: v8's structure on fp8 (OCP e4m3) operands, for the fp8 teacher (BASELINE config c4):
//   C = epilogue(alpha * sa[m] * sb[n] * sum_k qa[m,k] qb[n,k])
// qa / qb e4m3 with a per-row (token) and a per-output-channel fp32 scale, fp32
// accumulation in the AGPR file. v_mfma_scale_f32_32x32x64_f8f6f4 with unit block scales
// (e8m0 127 = 2^0) takes a 64-deep K step per instruction at twice the bf16 MFMA rate
// (MI355X_MICROARCH.md § Matrix cores: the block-scaled e4m3 form, 2x bf16 per clock).
// A stage is 64 K bytes of 256 rows per operand: the same [256 rows][64 B] image and
// swizzle as v8's bf16 BK=32 stage, so the DMA offsets, the 4-slot ring (three stages in
// flight, counted vmcnt, raw barriers) and the WAR/RAW argument of v8 carry over; per step
// each wave issues 16 MFMAs (4x4 tiles of 32x32 over its 128x128 quadrant), 8 DMAs of
// stage t+4 and 16 ds_read_b128 of stage t+1's fragments.
// Fragment (32x32x64, e4m3): lane l holds row (l & 31), k = 32 (l >> 5) + [0, 32) = two
// 16-B chunks of that row's 64-B stage row; C/D: col = l & 31, row = (reg & 3) +
// 8 (reg >> 2) + 4 (l >> 5).  Checked against a torch fp32 product of the dequantised
// operands (tests/test_fp8_gpu.py).
// =============================================================================
typedef __attribute__((ext_vector_type(8))) int i32x8;
typedef __attribute__((ext_vector_type(16))) float f32x16;

__device__ __forceinline__ uint32_t rec_bytes1(int64_t rows, int64_t ld) {
    const int64_t b = rows * ld;
    return b <= 0 ? 0u : (b >= 0x7FFFFFFFll ? 0x7FFFFFFFu : (uint32_t)b);
}

__device__ __forceinline__ void mfma_f8(f32x16& acc, const i32x8& a, const i32x8& b, int unit_scale) {
    asm volatile("v_mfma_scale_f32_32x32x64_f8f6f4 %0, %1, %2, %0, %3, %3 op_sel_hi:[0,0,0]"
                 : "+a"(acc) : "v"(a), "v"(b), "v"(unit_scale));
}

// the k-step's last fp8 MFMA with the result wait states in the same asm statement when
// `last` (see mfma_agpr_last)
__device__ __forceinline__ void mfma_f8_last(f32x16& acc, const i32x8& a, const i32x8& b, int unit_scale, int last) {
    asm volatile("v_mfma_scale_f32_32x32x64_f8f6f4 %0, %1, %2, %0, %3, %3 op_sel_hi:[0,0,0]\n\t"
                 "s_cmp_eq_u32 %4, 0\n\t"
                 "s_cbranch_scc1 .Lkd_mfma8_nodrain%=\n\t"
                 "s_nop 15\n\t"
                 "s_nop 15\n"
                 ".Lkd_mfma8_nodrain%=:"
                 : "+a"(acc) : "v"(a), "v"(b), "v"(unit_scale), "s"(__builtin_amdgcn_readfirstlane(last)) : "scc");
}

__device__ __forceinline__ i32x8 frag_f8(const char* tile, int r, int h) {
    const char* rowp = tile + r * 64;
    const int sw = f4(r);
    const u32x4 lo = *(const u32x4*)(rowp + (((2 * h) ^ sw) << 4));
    const u32x4 hi = *(const u32x4*)(rowp + (((2 * h + 1) ^ sw) << 4));
    i32x8 v;
    v[0] = (int)lo[0]; v[1] = (int)lo[1]; v[2] = (int)lo[2]; v[3] = (int)lo[3];
    v[4] = (int)hi[0]; v[5] = (int)hi[1]; v[6] = (int)hi[2]; v[7] = (int)hi[3];
    return v;
}

constexpr int F8_RS = 256 * 2 + 16;               // bf16 epilogue image row stride (bytes)
constexpr int F8_EPI = 256 * F8_RS;               // epilogue image bytes; the tile's row scales follow
constexpr size_t F8_LDS = (size_t)F8_EPI + 1024;  // > the 128 KiB ring

// pre-activation (and activation ACT) of the 4x4 32x32 accumulator tiles -> bf16 LDS image
template <int ACT>
__device__ __forceinline__ void f8_to_lds(const f32x16 (&acc)[4][4], char* smem, const float* sa_l, const float (&sbv)[4],
                                          const float (&bcol)[4], float alpha, int ra, int cb, int lane) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int lc = cb + 32 * j + (lane & 31);
            const float cs = alpha * sbv[j];
#pragma unroll
            for (int reg = 0; reg < 16; ++reg) {
                const int lr = ra + 32 * i + (reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5);
                const float v = apply_act(acc[i][j][reg] * cs * sa_l[lr] + bcol[j], ACT);
                *(bf16*)(smem + lr * F8_RS + lc * 2) = (bf16)v;
            }
        }
}

// ACT is a template parameter (one epilogue copy per build): with the activation switch and
// an aux pass in one kernel the epilogue's register demand made hipcc spill accumulators right
// after the last (asm, hazard-invisible) MFMA, before its results had landed.
template <int EXP, int ACT>
__global__ void __launch_bounds__(NTH8, 1) k_gemm8f8(GemmP p) {
    constexpr bool glu = EXP & 4;
    constexpr int SA = 256 * 64, SS = 2 * SA;   // 16 KiB per operand stage, 32 KiB per slot
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wid >> 1, wn = wid & 1;
    int tm, tn;
    tile_of(p.gx, (p.M + 255) / 256, glu ? (p.N / 256) : (p.N + 255) / 256, tm, tn, p.tile0, p.gm);
    const int m0 = tm * 256, n0 = tn * 256, nb = tn * 128;
    const int K = p.K;
    const int nk = (K + 63) / 64, nk_full = K / 64;
    const char* A8 = (const char*)p.A;
    const char* B8 = (const char*)p.B;
    const __amdgpu_buffer_rsrc_t rsA = make_rsrc(A8 + (int64_t)m0 * p.lda, rec_bytes1(min(256, p.M - m0), p.lda));
    const __amdgpu_buffer_rsrc_t rsB = glu ? make_rsrc(B8, rec_bytes1(p.N, p.ldb))
                                           : make_rsrc(B8 + (int64_t)n0 * p.ldb, rec_bytes1(min(256, p.N - n0), p.ldb));
    uint32_t va[4], vb[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {   // [256 rows][64 B]: 16 rows x 64 B per wave-instruction
        const int row = 16 * (wid * 4 + u) + (lane >> 2);
        const int gc = (lane & 3) ^ f4(row);
        va[u] = (uint32_t)((int64_t)row * p.lda + gc * 16);
        const int wrow = glu ? (row < 128 ? nb + row : p.glu + nb + row - 128) : row;
        vb[u] = (uint32_t)((int64_t)wrow * p.ldb + gc * 16);
    }
    auto dma = [&](int st, int sl, int u, auto full_tag) {
        constexpr bool FULL = decltype(full_tag)::value;
        const bool isA = u < 4;
        const int i = wid * 4 + (u & 3);
        char* dst = smem + sl * SS + (isA ? 0 : SA) + i * 1024;
        uint32_t v = isA ? va[u & 3] : vb[u & 3];
        int soff = st * 64;
        if (!FULL) {
            const int kleft = K - st * 64;   // valid k bytes of this stage (<= 0: past the end)
            if (kleft < 64) {
                const int row = 16 * i + (lane >> 2);
                const int gc = (lane & 3) ^ f4(row);
                if (gc * 16 >= kleft) v = OOB;
                if (kleft <= 0) soff = 0;
            }
        }
        __builtin_amdgcn_raw_ptr_buffer_load_lds(isA ? rsA : rsB, (lds_void_t*)dst, 16, v, soff, 0, 0);
    };
    using FullT = std::integral_constant<bool, true>;
    using PartT = std::integral_constant<bool, false>;
    f32x16 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    const int unit = 0x7F7F7F7F;   // e8m0 block scale 2^0 in every byte
    const int ra = wm * 128, cb = wn * 128, lr32 = lane & 31, h = lane >> 5;
#pragma unroll
    for (int st = 0; st < NS8; ++st)
#pragma unroll
        for (int u = 0; u < 8; ++u) dma(st, st, u, PartT{});
    wait_vm<24>();   // stage 0 landed (stages 1..3 may stay in flight)
    __builtin_amdgcn_s_barrier();
    i32x8 xa[4], xb[4], ya[4], yb[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        xa[u] = frag_f8(smem, ra + 32 * u + lr32, h);
        xb[u] = frag_f8(smem + SA, cb + 32 * u + lr32, h);
    }
#define KD_F8_SYNC()                                      \
    {                                                     \
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); \
        wait_vm<16>();                                    \
        __builtin_amdgcn_s_barrier();                     \
    }
    KD_F8_SYNC()
    __builtin_amdgcn_sched_barrier(0);
#define KD_SB __builtin_amdgcn_sched_barrier(0);
#define KD_F8_STEP(SL, CA, CB, NA, NB, FT)                                                         \
    {                                                                                               \
        const int t_ = t + (SL);                                                                    \
        const char* na_ = smem + (((SL) + 1) % NS8) * SS;                                           \
        _Pragma("unroll") for (int u = 0; u < 16; ++u) {                                            \
            if (u == 15) KD_F8_SYNC()                                                               \
            KD_SB                                                                                   \
            if (u == 15) mfma_f8_last(acc[3][3], CA[3], CB[3], unit, t_ + 1 == nk);                 \
            else mfma_f8(acc[u >> 2][u & 3], CA[u >> 2], CB[u & 3], unit);                          \
            KD_SB                                                                                   \
            if (u < 8) {                                                                            \
                dma(t_ + NS8, (SL), u, FT{}); KD_SB                                                 \
                if (u < 4) NA[u] = frag_f8(na_, ra + 32 * u + lr32, h);                             \
                else NB[u - 4] = frag_f8(na_ + SA, cb + 32 * (u - 4) + lr32, h);                    \
                KD_SB                                                                               \
            }                                                                                       \
        }                                                                                           \
    }
    int t = 0;
    for (; t + 2 * NS8 <= nk_full; t += NS8) {   // every DMA of these steps lies inside K
        KD_F8_STEP(0, xa, xb, ya, yb, FullT)
        KD_F8_STEP(1, ya, yb, xa, xb, FullT)
        KD_F8_STEP(2, xa, xb, ya, yb, FullT)
        KD_F8_STEP(3, ya, yb, xa, xb, FullT)
    }
    for (; t + NS8 <= nk; t += NS8) {
        KD_F8_STEP(0, xa, xb, ya, yb, PartT)
        KD_F8_STEP(1, ya, yb, xa, xb, PartT)
        KD_F8_STEP(2, xa, xb, ya, yb, PartT)
        KD_F8_STEP(3, ya, yb, xa, xb, PartT)
    }
    const int rem = nk - t;
    if (rem > 0) KD_F8_STEP(0, xa, xb, ya, yb, PartT)
    if (rem > 1) KD_F8_STEP(1, ya, yb, xa, xb, PartT)
    if (rem > 2) KD_F8_STEP(2, xa, xb, ya, yb, PartT)
#undef KD_F8_STEP
#undef KD_F8_SYNC
#undef KD_SB
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_nop 15\n\ts_nop 15" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __syncthreads();
    // ---- epilogue: per-row scales of the tile into LDS past the image, per-lane column scales
    float alpha = p.alpha;
    if (p.alpha_dev) alpha *= *p.alpha_dev;
    float* sa_l = (float*)(smem + F8_EPI);
    if (tid < 256) sa_l[tid] = (m0 + tid < p.M) ? p.sa[m0 + tid] : 0.f;
    float sbv[4], bcol[4] = {0.f, 0.f, 0.f, 0.f};
    int gcols[4];
    bool ins[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int lc = cb + 32 * j + lr32;
        const int gcol = glu ? (lc < 128 ? nb + lc : p.glu + nb + lc - 128) : n0 + lc;
        ins[j] = gcol < p.N;
        gcols[j] = min(gcol, p.N - 1);
        sbv[j] = p.sb[gcols[j]];
    }
    if (p.bias) load_bias<4>(p, gcols, bcol);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        sbv[j] = ins[j] ? sbv[j] : 0.f;
        bcol[j] = ins[j] ? bcol[j] : 0.f;
    }
    __syncthreads();
    if (glu) {
        f8_to_lds<KD_ACT_NONE>(acc, smem, sa_l, sbv, bcol, alpha, ra, cb, lane);
        __syncthreads();
        const int I = p.glu;
        const bool full = m0 + 256 <= p.M;
        if (p.aux) {
#pragma unroll 4
            for (int idx = tid; idx < 256 * 32; idx += NTH8) {
                const int lr = idx >> 5, c = idx & 31, row = m0 + lr;
                if (!full && row >= p.M) continue;
                const int col = c < 16 ? nb + c * 8 : I + nb + (c - 16) * 8;
                *(bf16x8*)(p.aux + (int64_t)row * p.ld_aux + col) = *(const bf16x8*)(smem + lr * F8_RS + c * 16);
            }
        }
#pragma unroll 4
        for (int idx = tid; idx < 256 * 16; idx += NTH8) {
            const int lr = idx >> 4, c = idx & 15, row = m0 + lr;
            if (!full && row >= p.M) continue;
            const bf16x8 g = *(const bf16x8*)(smem + lr * F8_RS + c * 16);
            const bf16x8 u = *(const bf16x8*)(smem + lr * F8_RS + 256 + c * 16);
            bf16x8 o;
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const float gf = (float)g[e];
                o[e] = (bf16)(silu_fast(gf) * (float)u[e]);
            }
            *(bf16x8*)((bf16*)p.C + (int64_t)row * p.ldc + nb + c * 8) = o;
        }
        return;
    }
    const bool full = m0 + 256 <= p.M && n0 + 256 <= p.N;
    f8_to_lds<ACT>(acc, smem, sa_l, sbv, bcol, alpha, ra, cb, lane);
    __syncthreads();
    epi_flush_sel<256, 256, NTH8, false>(p, smem, F8_RS, p.C, p.ldc, m0, n0, tid, full, p.resid != nullptr,
                                        p.accumulate != 0);
}

// Row quantisation to e4m3 with one fp32 scale per row: scale = amax / 448 (1 for an
// all-zero row), q = RNE_e4m3(clamp(x * (448 / amax), +-448)) — per-token activations and
// per-output-channel weights of the fp8 GEMM. One workgroup per row, two passes over the
// (L1/L2-resident) row.
__global__ void __launch_bounds__(256) k_quant_rows_f8(const bf16* __restrict__ x, int64_t ldx, int K,
                                                       uint8_t* __restrict__ q, int64_t ldq, float* __restrict__ scale) {
    __shared__ float red[4];
    const int64_t row = blockIdx.x;
    const bf16* xr = x + row * ldx;
    float amax = 0.f;
    for (int k = threadIdx.x * 8; k < K; k += 256 * 8) {
        const bf16x8 v = *(const bf16x8*)(xr + k);
#pragma unroll
        for (int e = 0; e < 8; ++e) amax = fmaxf(amax, fabsf((float)v[e]));
    }
    amax = wave_max(amax);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = amax;
    __syncthreads();
    amax = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    const float inv = amax > 0.f ? 448.f / amax : 1.f;
    if (threadIdx.x == 0) scale[row] = amax > 0.f ? amax / 448.f : 1.f;
    uint8_t* qr = q + row * ldq;
    for (int k = threadIdx.x * 8; k < K; k += 256 * 8) {
        const bf16x8 v = *(const bf16x8*)(xr + k);
        float f[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) f[e] = fminf(fmaxf((float)v[e] * inv, -448.f), 448.f);
        uint32_t w0 = __builtin_amdgcn_cvt_pk_fp8_f32(f[0], f[1], 0u, false);
        w0 = __builtin_amdgcn_cvt_pk_fp8_f32(f[2], f[3], w0, true);
        uint32_t w1 = __builtin_amdgcn_cvt_pk_fp8_f32(f[4], f[5], 0u, false);
        w1 = __builtin_amdgcn_cvt_pk_fp8_f32(f[6], f[7], w1, true);
        *(u32x2*)(qr + k) = (u32x2){w0, w1};
    }
}

// split-K fold: C = epilogue(sum_s partial[s]) with the full epilogue of the descriptor
// (alpha, alpha_dev, bias, aux, act, residual, accumulate), over the split tiles only
// (linear tiles [tile0, tile0 + gridDim.x) of a BM x BN tiling, grouped order as in the
// GEMM launch); blockIdx.y takes a BM / gridDim.y row slab of its tile (one 4-column chunk
// per thread: many blocks, every load of a block in flight at once), the S partial loads
// of a chunk issued together.
__global__ void __launch_bounds__(256) k_splitk_reduce(const float* __restrict__ ws, int S0, GemmP p, int BMr, int BNr) {
    // items (tile, row slab) = (p.gx tiles) x (p.gy slabs), strided over a 1-D grid of at most that many
    // workgroups (the launch may cap it: KD_SK_REDUCE_GRID, A/B)
    const int nitems = p.gx * p.gy;
    for (int it = (int)blockIdx.x; it < nitems; it += (int)gridDim.x) {
        const int bxi = it / p.gy, byi = it - bxi * p.gy;
        const int S = S0;
        int tm, tn;
        const int tiles_m = (p.M + BMr - 1) / BMr, tiles_n = (p.N + BNr - 1) / BNr;
        tile_grouped(p.tile0 + bxi, tiles_m, tiles_n, tm, tn, p.gm);
        const int rows_per = BMr / p.gy;
        const int r0 = tm * BMr + byi * rows_per;
        const int r1 = min(r0 + rows_per, p.M);
        const int c0 = tn * BNr, cw = min(BNr, p.N - c0);
        const int c4 = cw / 4;   // N % 8 == 0 on this path
        float alpha = p.alpha;
        if (p.alpha_dev) alpha *= *p.alpha_dev;
        for (int idx = threadIdx.x; idx < (r1 - r0) * c4; idx += 256) {
            const int64_t row = r0 + idx / c4;
            const int col = c0 + (idx % c4) * 4;
            const float* src = ws + row * p.N + col;
            f32x4 v = *(const f32x4*)src;
            int s = 1;
            for (; s + 3 < S; s += 4) {
                const f32x4 a = *(const f32x4*)(src + (int64_t)s * p.split_stride);
                const f32x4 b = *(const f32x4*)(src + (int64_t)(s + 1) * p.split_stride);
                const f32x4 c = *(const f32x4*)(src + (int64_t)(s + 2) * p.split_stride);
                const f32x4 d = *(const f32x4*)(src + (int64_t)(s + 3) * p.split_stride);
                v += a; v += b; v += c; v += d;
            }
            if (s + 1 < S) {   // same summation order, both loads in flight
                const f32x4 a = *(const f32x4*)(src + (int64_t)s * p.split_stride);
                const f32x4 b = *(const f32x4*)(src + (int64_t)(s + 1) * p.split_stride);
                v += a; v += b;
                s += 2;
            }
            if (s < S) v += *(const f32x4*)(src + (int64_t)s * p.split_stride);
            float bv[4] = {0.f, 0.f, 0.f, 0.f};
            if (p.bias) {
                const int bc[4] = {col, col + 1, col + 2, col + 3};
                load_bias<4>(p, bc, bv);
            }
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                float x = v[e] * alpha;
                if (p.bias) x += bv[e];
                if (p.aux) p.aux[row * p.ld_aux + col + e] = (bf16)x;
                v[e] = apply_act(x, p.act);
            }
            if (p.resid) {
                const int64_t ro = (p.res_mod > 0 ? row % p.res_mod : row) * p.ldr + col;
                if (p.res_f32) {
                    v += *(const f32x4*)((const float*)p.resid + ro);
                } else {
                    const bf16x4 r = *(const bf16x4*)(p.resid + ro);
#pragma unroll
                    for (int e = 0; e < 4; ++e) v[e] += (float)r[e];
                }
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
}

// Kernel / tile / split-K plan. Cost model in microseconds: waves x (32-deep k-steps per
// split x per-step tile cost + fixed per-tile prologue/epilogue), plus the fp32
// partial-plane traffic of a split. Candidates: v3 256x256 / 256x128 / 128x256 (8 waves)
// and v8 256x256 (4 waves), each with its own constants for K-major x K-major operands
// and for the layouts with an MN-major operand (tr_b16 fragment reads). Constants fitted
// (least squares on log time, tools/fit_plan.py) to a kernel x tile x split sweep over all
// 42 GEMM shapes of the c1 KD step (tools/tune_gemm.py, profiles/r01/gemm_tune.jsonl): the
// model's picks are within 0.4% of the measured best per step. A split can be confined to
// the tiles past the last whole wave (hybrid: whole waves unsplit, then the tail tiles
// x S splits), priced by the same constants.
// var: 2/3/4 v3 tiles, 16 v8, 20 v9; split > 1 with dp_tiles > 0: the first dp_tiles tiles (whole
// waves of 256) run unsplit with the full epilogue, only the tail tiles are split-K
// var 21: stream-K on v8 (split = the partial planes its workspace needs)
struct GemmPlan { int var; int split; int64_t kchunk; int dp_tiles; };
constexpr int SK_GRID = 256;   // stream-K workgroups: one per CU

// stream-K workspace: one int ticket per run tile (a 256-B block, zeroed per launch), then two
// 256 KB partial-tile slots per run (its first and its last piece)
inline size_t sk_cnt_bytes(int64_t sk_tiles) { return (size_t)((sk_tiles * 4 + 255) / 256) * 256; }
inline size_t sk_workspace_bytes(int64_t sk_tiles) {
    return sk_cnt_bytes(sk_tiles) + (size_t)SK_GRID * 2 * 256 * 256 * 4;
}
// data-parallel tiles ahead of the runs: whole waves, all but the last (so every run holds more than
// one tile's worth of k-steps when there are several waves: "DP + two-tile stream-K")
inline int64_t sk_dp_tiles(int64_t tiles, int64_t nk) {
    (void)nk;
    return tiles >= 2 * SK_GRID ? (tiles / SK_GRID - 1) * SK_GRID : 0;
}

#ifdef KD_AB_BUILD
// KD_GLU_EPI_V0=1: the SwiGLU GEMM with the previous (unpacked) epilogue, for A/B (read per call)
bool glu_epi_v0() {
    const char* e = std::getenv("KD_GLU_EPI_V0");
    return e && std::atoi(e) != 0;
}
#endif

GemmPlan plan_gemm(const kd_gemm_desc* d, uint64_t ws_cap) {
    const int64_t M = d->M, N = d->N;
    const int64_t t256 = (int64_t)ceil_div(d->M, 256) * ceil_div(d->N, 256);
    const int64_t tiles[5] = {t256, (int64_t)ceil_div(d->M, 256) * ceil_div(d->N, 128),
                              (int64_t)ceil_div(d->M, 128) * ceil_div(d->N, 256), t256, t256};
    const bool kk = d->a_layout == KD_LAYOUT_K_MAJOR && d->b_layout == KD_LAYOUT_K_MAJOR;
    // per variant (v3 256x256, 256x128, 128x256; v8; v9): {K-major x K-major, MN-major operand}
    // refitted in round 4 to the step's CACHE STATE (profiles/r04/gemm_tune_cold.jsonl,
    // tools/tune_gemm_cold.py: every candidate timed with operand B cold -- the step reads each
    // weight / saved activation a whole step after its last use -- and operand A just written);
    // the round-3 constants came from warm back-to-back calls, which favour shallow prefetch and
    // unsplit tails ({{0.7524, 0.5218, 0.5092, 0.6844, 0.7183}, {0.7375, 0.5501, 0.5469, 0.6022,
    // 0.6876}}, {{5.253, 3.402, 3.414, 8.478, 5.888}, {5.885, 3.479, 3.398, 8.695, 8.442}}, 7.711e6,
    // 5.623).  v9 keeps its round-3 constants (not in the automatic choice).
    // KD_PLAN_SET=3 selects the round-3 constants (A/B); KD_GEMM_HYBRID=0 drops the hybrid plans.
    static const double step_c4[2][5] = {{0.8167, 0.5676, 0.5775, 0.7550, 0.7183}, {0.8016, 0.6139, 0.6026, 0.6942, 0.6876}};
    static const double fixed_c4[2][5] = {{8.830, 5.440, 5.343, 11.954, 5.888}, {9.291, 5.201, 5.162, 12.159, 8.442}};
    static const double step_c3[2][5] = {{0.7524, 0.5218, 0.5092, 0.6844, 0.7183}, {0.7375, 0.5501, 0.5469, 0.6022, 0.6876}};
    static const double fixed_c3[2][5] = {{5.253, 3.402, 3.414, 8.478, 5.888}, {5.885, 3.479, 3.398, 8.695, 8.442}};
    static const bool set3 = ab_knob("KD_PLAN_SET", 4) == 3;
    static const bool hybrid_on = ab_knob("KD_GEMM_HYBRID", 1) != 0;
    // A/B: the cost model's split count capped (KD_SPLIT_CAP) and its partial-plane cost scaled
    // (KD_SPLIT_PENALTY, percent) -- the model is fitted on isolated calls, the step runs two streams
    static const int split_cap = ab_knob("KD_SPLIT_CAP", 32);
    static const double split_pen = ab_knob("KD_SPLIT_PENALTY", 100) / 100.0;
    const double (&step_c)[2][5] = set3 ? step_c3 : step_c4;
    const double (&fixed_c)[2][5] = set3 ? fixed_c3 : fixed_c4;
    const double kBW = set3 ? 7.711e6 : 9.109e6;          // partial-plane bytes per microsecond
    const double kSplitLaunch = set3 ? 5.623 : 6.499;     // the reduce kernel (us); a hybrid plan launches two more kernels
    constexpr bool kV9Auto = false;   // v9 enters the model's choice once its constants are fitted
    const double* step = step_c[kk ? 0 : 1];
    const double* fixed = fixed_c[kk ? 0 : 1];
    const int vcode[5] = {2, 3, 4, 16, 20};
    const int64_t nk = ceil_div(d->K, BK2);
    // forced: variants 2/5 v3 256x256, 3/6 256x128, 4/7 128x256, 16+ v8; 0 = model's choice
    const int fv = d->variant == 20 ? 4 : (d->variant >= 16 ? 3 : (d->variant >= 5 ? d->variant - 5 : (d->variant >= 2 ? d->variant - 2 : -1)));
    const double out_e = (double)((d->c_dtype == KD_DTYPE_F32 ? 4 : 2) * (d->accumulate ? 2 : 1) +
                                  (d->residual ? (d->residual_dtype == KD_DTYPE_F32 ? 4 : 2) : 0) +
                                  (d->aux ? 2 : 0));   // epilogue bytes per element
    const double out_b = (double)M * N * out_e;
    const int tbm[5] = {256, 256, 128, 256, 256}, tbn[5] = {256, 128, 256, 256, 256};
    GemmPlan best{fv >= 0 ? vcode[fv] : 2, 1, d->K, 0};
    double bt = 1e300;
    for (int v = 0; v < 5; ++v) {
        if (fv >= 0 && v != fv) continue;
        if (v == 4 && !kV9Auto && fv != 4) continue;
        for (int S = 1; S <= 32; ++S) {
            if (d->split_k == 1 && S != 1) continue;
            if (d->split_k > 1 && S != d->split_k && S != 1) continue;
            const int64_t kcs = (nk + S - 1) / S;
            if (S > 1 && ((nk + kcs - 1) / kcs != S)) continue;          // empty trailing split
            if (S > 1 && d->split_k <= 1 && kcs < 8) continue;           // too little work per split
            if (S > 1 && (uint64_t)S * M * N * 4 > ws_cap) continue;
            if (S > split_cap && d->split_k <= 0) continue;
            const int64_t waves = (tiles[v] * S + 255) / 256;
            double t = (double)waves * ((double)kcs * step[v] + fixed[v]);
            if (S > 1) t += ((double)S * M * N * 8 * split_pen + out_b) / kBW + kSplitLaunch;
            if (d->split_k > 1 && S == d->split_k) t = -1;              // forced
            if (t < bt) { bt = t; best = GemmPlan{vcode[v], S, kcs * BK2, 0}; }
            // hybrid: whole waves unsplit, the tail tiles split S ways (model's choice only)
            const int64_t dp = (tiles[v] / 256) * 256, tail = tiles[v] - dp;
            if (hybrid_on && S > 1 && d->split_k <= 0 && dp > 0 && tail > 0) {
                const double tb = (double)tbm[v] * tbn[v];
                double th = (double)(dp / 256) * ((double)nk * step[v] + fixed[v]) +
                            (double)((tail * S + 255) / 256) * ((double)kcs * step[v] + fixed[v]) +
                            ((double)S * tail * tb * 8 * split_pen + tail * tb * out_e) / kBW + 2 * kSplitLaunch;
                if (th < bt) { bt = th; best = GemmPlan{vcode[v], S, kcs * BK2, (int)dp}; }
            }
        }
    }
    // stream-K on v8 (variant 21): all but the last whole wave of tiles data-parallel, then SK_GRID
    // workgroups take equal runs of the remaining tiles' k-steps (runs cross tile boundaries); a
    // tile shared by several runs is folded inside the launch by its last-arriving piece (round 6).
    // The round-2 build (every tile in runs, fp32 partial planes folded by a second launch) measured
    // slower than the split-K / hybrid plans on every backward shape of the step (1152x1152x5832
    // wgrad 71 vs 39 us, 6144x896x9728 dgrad 155 vs 149 us, down_proj 1020 vs 710 us).
    if (d->variant == 21 && d->split_k <= 1) {   // (split_k 1: the fused dact / q|k|v epilogues; not a K split)
        const int64_t dp = sk_dp_tiles(t256, nk);
        if ((t256 - dp) * nk >= 2 * SK_GRID && sk_workspace_bytes(t256 - dp) <= ws_cap) {
            bt = 0;
            best = GemmPlan{21, 1, d->K, (int)dp};
        }
    }
    return best;
}

}  // namespace


int launch_gemm_f8(const kd_gemm_desc* d, void* stream_) {
    KD_CHECK_ARG(d->a_layout == KD_LAYOUT_K_MAJOR && d->b_layout == KD_LAYOUT_K_MAJOR, "gemm fp8: K-major operands only");
    KD_CHECK_ARG(d->a_scale && d->b_scale, "gemm fp8: null a_scale / b_scale");
    KD_CHECK_ARG(d->c_dtype == KD_DTYPE_BF16, "gemm fp8: bf16 output");
    KD_CHECK_ARG(d->split_k <= 1, "gemm fp8: no split-K");
    KD_CHECK_ARG(!d->residual || d->residual_dtype == KD_DTYPE_BF16, "gemm fp8: bf16 residual only");
    KD_CHECK_ALIGN(d->A, 16, "gemm fp8: A must be 16-B aligned");
    KD_CHECK_ALIGN(d->B, 16, "gemm fp8: B must be 16-B aligned");
    KD_CHECK_SHAPE(d->K % 16 == 0 && d->lda % 16 == 0 && d->ldb % 16 == 0 && d->lda >= d->K && d->ldb >= d->K,
                   "gemm fp8: K, lda, ldb must be multiples of 16 (lda, ldb >= K)");
    KD_CHECK_SHAPE((uint64_t)256 * d->lda < 0x7FFFFFFFull && (uint64_t)256 * d->ldb < 0x7FFFFFFFull,
                   "gemm fp8: leading dimension too large for 31-bit buffer records");
    const bool c_ok16 = (d->ldc % 8 == 0) && ((uintptr_t)d->C % 16 == 0) &&
                        (!d->residual || ((d->ldr % 8 == 0) && ((uintptr_t)d->residual % 16 == 0))) &&
                        (!d->aux || ((d->ld_aux % 8 == 0) && ((uintptr_t)d->aux % 16 == 0)));
    KD_CHECK_SHAPE(d->N % 8 == 0 && c_ok16, "gemm fp8: N % 8 == 0 and 16-B aligned C / residual / aux rows");
    KD_CHECK_SHAPE(d->ldc >= (d->act == KD_ACT_SWIGLU ? d->N / 2 : d->N), "gemm fp8: ldc < N (N/2 for swiglu)");
    KD_CHECK_SHAPE(!d->residual || d->ldr >= d->N, "gemm fp8: ldr < N");
    KD_CHECK_SHAPE(!d->aux || d->ld_aux >= d->N, "gemm fp8: ld_aux < N");
    GemmP p;
    std::memset(&p, 0, sizeof(p));
    p.A = (const bf16*)d->A; p.B = (const bf16*)d->B; p.C = d->C;
    p.bias = d->bias; p.resid = (const bf16*)d->residual; p.aux = (bf16*)d->aux; p.alpha_dev = d->alpha_dev;
    p.lda = d->lda; p.ldb = d->ldb; p.ldc = d->ldc; p.ldr = d->ldr; p.ld_aux = d->ld_aux;
    p.M = d->M; p.N = d->N; p.K = d->K; p.alpha = d->alpha;
    p.c_f32 = 0; p.accumulate = d->accumulate; p.bias_f32 = d->bias_dtype == KD_DTYPE_F32;
    p.act = d->act; p.res_mod = d->residual_row_mod;
    p.kchunk = d->K; p.sa = d->a_scale; p.sb = d->b_scale;
    hipStream_t st = as_stream(stream_);
    if (d->act == KD_ACT_SWIGLU) {
        KD_CHECK_SHAPE(d->N % 256 == 0, "gemm fp8 swiglu: N = 2I needs I % 128 == 0");
        KD_CHECK_ARG(!d->bias && !d->residual && !d->accumulate, "gemm fp8 swiglu: no bias / residual / accumulate");
        p.glu = d->N / 2; p.act = KD_ACT_NONE;
        p.gx = ceil_div(d->M, 256) * (d->N / 256); p.gy = 1;
        p.gm = pick_gm(ceil_div(d->M, 256), d->N / 256);
        hipLaunchKernelGGL((k_gemm8f8<4, KD_ACT_NONE>), dim3(p.gx), dim3(NTH8), F8_LDS, st, p);
        KD_LAUNCH_CHECK("k_gemm8f8<swiglu>");
        return KD_OK;
    }
    KD_CHECK_ARG(!d->aux, "gemm fp8: aux (pre-activation) output only with KD_ACT_SWIGLU");
    const dim3 grid(ceil_div(d->M, 256) * ceil_div(d->N, 256));
    p.gx = (int)grid.x; p.gy = 1;
    p.gm = pick_gm(ceil_div(d->M, 256), ceil_div(d->N, 256));
    switch (d->act) {
        case KD_ACT_GELU_TANH: hipLaunchKernelGGL((k_gemm8f8<0, KD_ACT_GELU_TANH>), grid, dim3(NTH8), F8_LDS, st, p); break;
        case KD_ACT_GELU_ERF: hipLaunchKernelGGL((k_gemm8f8<0, KD_ACT_GELU_ERF>), grid, dim3(NTH8), F8_LDS, st, p); break;
        case KD_ACT_SILU: hipLaunchKernelGGL((k_gemm8f8<0, KD_ACT_SILU>), grid, dim3(NTH8), F8_LDS, st, p); break;
        default: hipLaunchKernelGGL((k_gemm8f8<0, KD_ACT_NONE>), grid, dim3(NTH8), F8_LDS, st, p); break;
    }
    KD_LAUNCH_CHECK("k_gemm8f8");
    return KD_OK;
}

int launch_quant_rows_f8(const void* x, int64_t ldx, int R, int K, void* q, int64_t ldq, float* scale, void* stream) {
    KD_CHECK_ARG(x && q && scale, "quant_rows_fp8: null pointer");
    KD_CHECK_SHAPE(R >= 0 && K > 0 && K % 16 == 0 && ldx >= K && ldq >= K && ldx % 8 == 0 && ldq % 8 == 0,
                   "quant_rows_fp8: K % 16 == 0, ldx / ldq >= K and multiples of 8");
    KD_CHECK_ALIGN(x, 16, "quant_rows_fp8: x must be 16-B aligned");
    KD_CHECK_ALIGN(q, 8, "quant_rows_fp8: q must be 8-B aligned");
    if (R == 0) return KD_OK;
    hipLaunchKernelGGL(k_quant_rows_f8, dim3(R), dim3(256), 0, as_stream(stream), (const bf16*)x, ldx, K, (uint8_t*)q, ldq,
                       scale);
    KD_LAUNCH_CHECK("k_quant_rows_f8");
    return KD_OK;
}


// kd_gemm_pretile: W [N][K] (row stride ldw) -> the v8 K-major stage images of B, tile by tile:
// [ceil(N / 256) tiles][ceil(K / 32) stages][256 rows][4 chunks of 8], position (row r, chunk pc)
// holding logical chunk pc ^ f4(r) (the ring's swizzle), zeros past N and K; glu_I > 0 (the SwiGLU
// build, N = 2 glu_I): tile t's rows [0, 128) are gate rows 128 t + r, rows [128, 256) up rows
// glu_I + 128 t + r - 128.  One thread per 16-B chunk.
__global__ void k_pretile_b(const bf16* __restrict__ W, int64_t ldw, int N, int K, int glu_I, int nkt, int64_t total,
                            bf16* __restrict__ out) {
    for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total; idx += (int64_t)gridDim.x * blockDim.x) {
        const int pc = (int)(idx & 3), r = (int)((idx >> 2) & 255);
        const int64_t ts = idx >> 10;
        const int st = (int)(ts % nkt), t = (int)(ts / nkt);
        const int wrow = glu_I > 0 ? (r < 128 ? 128 * t + r : glu_I + 128 * t + r - 128) : 256 * t + r;
        const int k = st * BK2 + 8 * (pc ^ f4(r));
        bf16x8 v = (bf16x8){};
        if (wrow < N && k < K) v = *(const bf16x8*)(W + (int64_t)wrow * ldw + k);
        *(bf16x8*)(out + idx * 8) = v;
    }
}

size_t gemm_pretile_size(int N, int K, int glu) {
    if (N <= 0 || K <= 0) return 0;
    const int64_t tiles = glu ? (N / 256) : ceil_div(N, 256);
    return (size_t)tiles * ceil_div(K, BK2) * 256 * BK2 * 2;
}

int launch_gemm_pretile(const void* W, int64_t ldw, int N, int K, int glu, void* out, void* stream) {
    KD_CHECK_ARG(W && out, "gemm_pretile: null pointer");
    KD_CHECK_SHAPE(N > 0 && K > 0 && K % 8 == 0 && ldw >= K && ldw % 8 == 0, "gemm_pretile: K % 8 == 0, ldw >= K");
    KD_CHECK_SHAPE(!glu || N % 256 == 0, "gemm_pretile: the SwiGLU layout needs N = 2I with I % 128 == 0");
    KD_CHECK_ALIGN(W, 16, "gemm_pretile: W must be 16-B aligned");
    KD_CHECK_ALIGN(out, 16, "gemm_pretile: out must be 16-B aligned");
    const int nkt = ceil_div(K, BK2);
    const int64_t total = (int64_t)(gemm_pretile_size(N, K, glu) / 16);
    const int grid = (int)std::min<int64_t>((total + 255) / 256, 65536);
    hipLaunchKernelGGL(k_pretile_b, dim3(grid), dim3(256), 0, as_stream(stream), (const bf16*)W, ldw, N, K,
                       glu ? N / 2 : 0, nkt, total, (bf16*)out);
    KD_LAUNCH_CHECK("k_pretile_b");
    return KD_OK;
}

#ifdef KD_AB_BUILD
// v11 (32x32x16 MFMAs) in place of v8 for K-major x K-major tiles: forced variant 23, or
// KD_GEMM_V11=1 wherever v8 would run (opt-in; 24 forces v8 for A/B)
static bool use_v11(int variant) {
    if (variant == 23) return true;
    if (variant != 0 && variant != 16) return false;
    static const int env = [] { const char* e = std::getenv("KD_GEMM_V11"); return e ? std::atoi(e) : -1; }();
    return env == 1;
}

// v12 (whole-line staging of K-major operands, bit-identical to v8): forced variant 26, or
// KD_GEMM_V12=1 wherever v8 would run (opt-in; 24 forces v8).  Measured faster than v8 only with
// the weights warm in the Infinity Cache (back-to-back calls, profiles/r04/ab_v12_vs_v8.txt); in
// the step's cache state -- every weight read cold, a whole step after its last use -- slower than
// v8 on every shape (profiles/r04/ab_cold.txt): its stage pairs halve the prefetch depth.
static bool use_v12(int variant) {
    if (variant == 26) return true;
    if (variant != 0 && variant != 16) return false;
    static const int env = [] { const char* e = std::getenv("KD_GEMM_V12"); return e ? std::atoi(e) : -1; }();
    return env == 1;
}
#endif

// the variants kd_gemm accepts: 0 auto, 1 v1, 2-7 v3 tiles, 16 v8, 21 stream-K, 24 (= 16); the
// tools' A/B library (KD_AB_BUILD: python csrc/build.py --ab) also the negative-result and
// diagnostic builds 17-20, 22, 23, 26-28
// workgroups of a split-K / stream-K fold launch over `items` (tile, row slab) items: one each, or
// at most KD_SK_REDUCE_GRID (A/B: the fold runs beside the other stream's GEMMs)
static unsigned reduce_grid(int items) {
    const int cap = ab_knob("KD_SK_REDUCE_GRID", 0);
    return (unsigned)(cap > 0 && cap < items ? cap : items);
}

static bool variant_known(int v) {
    if ((v >= 0 && v <= 7) || v == 16 || v == 21 || v == 24 || v == 32) return true;
#ifdef KD_AB_BUILD
    if ((v >= 17 && v <= 20) || v == 22 || v == 23 || (v >= 26 && v <= 28) || v == 30) return true;
#endif
    return false;
}

// stream-K launch setup over `tiles` 256 x 256 tiles: the data-parallel prefix, the run grid, the
// tickets (zeroed by a memset node ahead of every launch: Guideline 16) and the partial-tile slots
static bool sk_fits(int64_t tiles, int64_t nk, const kd_gemm_desc* d) {
    const int64_t dp = sk_dp_tiles(tiles, nk);
    return (tiles - dp) * nk >= 2 * SK_GRID && d->workspace && d->workspace_bytes >= sk_workspace_bytes(tiles - dp);
}
static int sk_setup(GemmP& q, int64_t tiles, const kd_gemm_desc* d, hipStream_t st) {
    const int64_t dp = sk_dp_tiles(tiles, ceil_div(d->K, BK2));
    KD_CHECK_ARG(d->workspace && d->workspace_bytes >= sk_workspace_bytes(tiles - dp), "gemm: stream-K workspace too small");
    q.sk_steps = ceil_div(d->K, BK2); q.sk_grid = SK_GRID; q.sk_dp = (int)dp;
    q.sk_cnt = (int*)d->workspace;
    q.sk_ws = (float*)((char*)d->workspace + sk_cnt_bytes(tiles - dp));
    q.gx = (int)dp + SK_GRID; q.gy = 1; q.tile0 = 0;
    if (hipMemsetAsync(q.sk_cnt, 0, sk_cnt_bytes(tiles - dp), st) != hipSuccess)
        return fail(KD_ERR_LAUNCH, "gemm: stream-K ticket memset");
    return KD_OK;
}

int launch_gemm(const kd_gemm_desc* d, void* stream_) {
    KD_CHECK_ARG(d != nullptr, "gemm: null descriptor");
    KD_CHECK_ARG(d->A && d->B && (d->C || d->qkv), "gemm: null operand");
    KD_CHECK_SHAPE(d->M > 0 && d->N > 0 && d->K > 0, "gemm: empty shape");
    KD_CHECK_ARG(d->a_layout == KD_LAYOUT_K_MAJOR || d->a_layout == KD_LAYOUT_MN_MAJOR, "gemm: a_layout");
    KD_CHECK_ARG(d->b_layout == KD_LAYOUT_K_MAJOR || d->b_layout == KD_LAYOUT_MN_MAJOR, "gemm: b_layout");
    KD_CHECK_ARG(d->c_dtype == KD_DTYPE_BF16 || d->c_dtype == KD_DTYPE_F32, "gemm: c_dtype");
    KD_CHECK_ARG(d->ab_dtype == KD_DTYPE_BF16 || d->ab_dtype == KD_DTYPE_FP8_E4M3, "gemm: ab_dtype");
    KD_CHECK_ARG(!d->qkv || d->ab_dtype == KD_DTYPE_BF16, "gemm qkv: bf16 operands only");
    KD_CHECK_ARG(!d->b_pretiled || (d->ab_dtype == KD_DTYPE_BF16 && d->a_layout == KD_LAYOUT_K_MAJOR &&
                                    d->b_layout == KD_LAYOUT_K_MAJOR && !d->row_stats && d->split_k <= 1 &&
                                    (d->variant == 0 || d->variant == 16 || d->variant == 24)),
                 "gemm b_pretiled: K-major bf16 operands on the 256x256 v8 kernel, no split-K / row_stats");
    if (d->ab_dtype == KD_DTYPE_FP8_E4M3) return launch_gemm_f8(d, stream_);
    KD_CHECK_ARG(d->act >= KD_ACT_NONE && d->act <= KD_ACT_DSWIGLU, "gemm: act");
    const bool dact = d->act == KD_ACT_DGELU_TANH || d->act == KD_ACT_DSWIGLU;
    KD_CHECK_ARG(d->act == KD_ACT_NONE || dact || (d->a_layout == KD_LAYOUT_K_MAJOR && d->b_layout == KD_LAYOUT_K_MAJOR &&
                                                   d->c_dtype == KD_DTYPE_BF16),
                 "gemm: an activation epilogue needs K-major operands and a bf16 output");
    if (dact) {
        const int64_t w = d->act == KD_ACT_DSWIGLU ? 2 * (int64_t)d->N : d->N;
        KD_CHECK_ARG(d->aux && d->c_dtype == KD_DTYPE_BF16 && !d->bias && !d->residual && !d->accumulate && d->split_k <= 1 &&
                     d->variant != 1,
                     "gemm backward activation: aux (forward pre-activation), bf16 C, no bias / residual / accumulate / split-K");
        KD_CHECK_SHAPE(d->N % 8 == 0 && d->ldc >= w && d->ld_aux >= w && d->ldc % 8 == 0 && d->ld_aux % 8 == 0 &&
                       (uintptr_t)d->aux % 16 == 0, "gemm backward activation: ldc / ld_aux >= N (2N for dswiglu), 16-B rows");
    }
    KD_CHECK_ARG(variant_known(d->variant),
                 "gemm: unknown variant (the diagnostic / A-B builds 17-20, 22, 23, 26-28 are in the tools' A/B library only)");
    KD_CHECK_ALIGN(d->A, 16, "gemm: A must be 16-B aligned");
    KD_CHECK_ALIGN(d->B, 16, "gemm: B must be 16-B aligned");
    // the tiled epilogues load a lane's 4 bias columns as one f32x4 / bf16x4 vector (load_bias4)
    KD_CHECK_ALIGN(d->bias, d->bias_dtype == KD_DTYPE_F32 ? 16 : 8, "gemm: bias must be 16-B (fp32) / 8-B (bf16) aligned");
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
    KD_CHECK_SHAPE(d->qkv || d->ldc >= (d->act == KD_ACT_SWIGLU ? d->N / 2 : d->N), "gemm: ldc < N (N/2 for swiglu)");
    KD_CHECK_SHAPE(!d->residual || d->ldr >= d->N, "gemm: ldr < N");
    KD_CHECK_ARG(!d->residual || d->residual_dtype == KD_DTYPE_BF16 ||
                 (d->residual_dtype == KD_DTYPE_F32 && d->c_dtype == KD_DTYPE_F32 && d->act == KD_ACT_NONE),
                 "gemm: an fp32 residual needs an fp32 C and no activation epilogue");
    KD_CHECK_SHAPE(!d->aux || d->ld_aux >= d->N, "gemm: ld_aux < N");
    KD_CHECK_SHAPE((uint64_t)256 * d->lda * 2 < 0x7FFFFFFFull && (uint64_t)256 * d->ldb * 2 < 0x7FFFFFFFull,
                   "gemm: leading dimension too large for 31-bit buffer records");
#ifdef KD_AB_BUILD
    {
        const int bl = ab_knob("KD_GEMM_BLAS", 0);
        if (bl && blas_eligible(d) && (bl == 1 || blas_wins(d))) return blas_gemm(d, as_stream(stream_));
    }
#endif
    GemmP p;
    p.A = (const bf16*)d->A; p.B = (const bf16*)d->B; p.C = d->C;
    p.bias = d->bias; p.resid = (const bf16*)d->residual; p.aux = (bf16*)d->aux; p.alpha_dev = d->alpha_dev;
    p.lda = d->lda; p.ldb = d->ldb; p.ldc = d->ldc; p.ldr = d->ldr; p.ld_aux = d->ld_aux;
    p.M = d->M; p.N = d->N; p.K = d->K; p.alpha = d->alpha;
    p.c_f32 = d->c_dtype == KD_DTYPE_F32; p.accumulate = d->accumulate; p.bias_f32 = d->bias_dtype == KD_DTYPE_F32;
    p.act = d->act;
    p.res_mod = d->residual_row_mod;
    p.res_f32 = d->residual && d->residual_dtype == KD_DTYPE_F32;
    p.sq = p.sk = p.sv = nullptr; p.rcos = p.rsin = nullptr;
    p.sS = p.snq = p.snkv = p.shd = p.shdp = 0;
    if (d->qkv) {
        const kd_qkv_scatter& q = *d->qkv;
        const bool rope = q.cos_t != nullptr;
        KD_CHECK_ARG(q.q && q.k && q.v && (rope == (q.sin_t != nullptr)), "gemm qkv: null q / k / v or cos without sin");
        KD_CHECK_ARG(d->act == KD_ACT_NONE && !d->residual && !d->aux && !d->accumulate && d->c_dtype == KD_DTYPE_BF16 &&
                     d->a_layout == KD_LAYOUT_K_MAJOR && d->b_layout == KD_LAYOUT_K_MAJOR && d->split_k <= 1,
                     "gemm qkv: K-major operands, no activation / residual / aux / accumulate / split-K");
        KD_CHECK_SHAPE(q.S > 0 && d->M % q.S == 0 && q.nq > 0 && q.nkv > 0 && d->N == (q.nq + 2 * q.nkv) * q.hd &&
                       q.hd % 8 == 0 && q.hdp % 8 == 0 && q.hdp >= q.hd && (!rope || (q.hd % 16 == 0 && 128 % q.hd == 0)),
                       "gemm qkv: N = (nq + 2 nkv) hd, M % S == 0, hd / hdp % 8 == 0, RoPE heads dividing 128");
        KD_CHECK_ALIGN(q.q, 16, "gemm qkv: q must be 16-B aligned");
        KD_CHECK_ALIGN(q.k, 16, "gemm qkv: k must be 16-B aligned");
        KD_CHECK_ALIGN(q.v, 16, "gemm qkv: v must be 16-B aligned");
        p.sq = (bf16*)q.q; p.sk = (bf16*)q.k; p.sv = (bf16*)q.v; p.rcos = q.cos_t; p.rsin = q.sin_t;
        p.sS = q.S; p.snq = q.nq; p.snkv = q.nkv; p.shd = q.hd; p.shdp = q.hdp;
    }
    p.kchunk = d->K; p.split_stride = 0; p.glu = 0; p.tile0 = 0;
    p.sa = p.sb = nullptr; p.gx = 0; p.gy = 1;
    p.sk_steps = 0; p.sk_grid = 0; p.sk_ws = nullptr; p.sk_dp = 0; p.sk_cnt = nullptr;
    p.gm = 0;
    p.rst = nullptr; p.rst_nt = p.rst_vs = p.rst_top2 = 0; p.rst_inv_t = 1.f;
    p.stagger = ab_knob("KD_GEMM_STAGGER", 1);
    p.stag_g = 0;
    hipStream_t st = as_stream(stream_);
    const bool amn = d->a_layout == KD_LAYOUT_MN_MAJOR, bmn = d->b_layout == KD_LAYOUT_MN_MAJOR;
    const bool c_ok16 = (d->qkv || ((d->ldc % 8 == 0) && ((uintptr_t)d->C % 16 == 0))) &&
                        (!d->residual || ((d->ldr % 8 == 0) && ((uintptr_t)d->residual % 16 == 0)));
    const bool big_ok = d->N % 8 == 0 && c_ok16 && d->M >= 128 && d->N >= 128 &&
                        ((uint64_t)d->M * d->N >= (1ull << 20) || (d->workspace && d->K >= 2048 && d->split_k != 1)) &&
                        (!amn || d->M % 8 == 0) && (!bmn || d->N % 8 == 0) &&
                        (uint64_t)BK2 * (amn ? d->lda : 0) * 2 < 0x7FFFFFFFull;
    KD_CHECK_ARG(!dact || big_ok, "gemm backward activation: needs the tiled kernels (M, N >= 128, M*N >= 2^20)");
    KD_CHECK_ARG(!d->qkv || (big_ok && d->variant != 1),
                 "gemm qkv: needs the tiled kernels (M, N >= 128, M*N >= 2^20)");
    kd_gemm_desc d1;
    if ((dact || d->qkv) && d->split_k != 1) {   // the fused backward activation / q|k|v scatter are never split-K
        d1 = *d;
        d1.split_k = 1;
        d = &d1;
    }
    if (d->row_stats) {   // the lm_head GEMM with the KD loss's row statistics, on v8 (no split)
        KD_CHECK_ARG(!amn && !bmn && d->c_dtype == KD_DTYPE_BF16 && !d->bias && d->act == KD_ACT_NONE && !d->residual &&
                         !d->aux && !d->accumulate && !d->qkv && d->ab_dtype == KD_DTYPE_BF16,
                     "gemm row_stats: K-major bf16 operands, bf16 C, no bias / act / residual / aux / accumulate");
        KD_CHECK_SHAPE(d->N % 8 == 0 && (d->row_stats_vs <= 0 || d->row_stats_vs % 8 == 0) && big_ok,
                       "gemm row_stats: N and row_stats_vs multiples of 8, the tiled kernels' shapes");
        KD_CHECK_ARG(d->row_stats_inv_t > 0.f, "gemm row_stats: row_stats_inv_t must be > 0");
        KD_CHECK_ALIGN(d->row_stats, 16, "gemm row_stats: 16-B aligned");
        GemmP pk = p;
        pk.rst = d->row_stats; pk.rst_nt = ceil_div(d->N, 256); pk.rst_vs = d->row_stats_vs;
        pk.rst_inv_t = d->row_stats_inv_t; pk.rst_top2 = d->row_stats_top2 ? 1 : 0;
        pk.gm = pick_gm(ceil_div(d->M, 256), ceil_div(d->N, 256));
        const dim3 grid(ceil_div(d->M, 256) * ceil_div(d->N, 256), 1);
        pk.gx = (int)grid.x; pk.gy = 1; pk.tile0 = 0;
        hipLaunchKernelGGL((k_gemm8<false, false, 32>), grid, dim3(NTH8), (gemm2_lds<256, 256>()), st, pk);
        KD_LAUNCH_CHECK("k_gemm8 (row stats)");
        return KD_OK;
    }
    if (d->act == KD_ACT_SWIGLU) {   // fused gate|up GEMM + silu(gate) * up, on v8
        KD_CHECK_SHAPE(d->N % 256 == 0 && d->M >= 1, "gemm swiglu: N = 2I needs I % 128 == 0");
        KD_CHECK_ARG(!d->bias && !d->residual && !d->accumulate && d->split_k <= 1,
                     "gemm swiglu: no bias / residual / accumulate / split-K");
        KD_CHECK_ARG(!amn && !bmn && d->c_dtype == KD_DTYPE_BF16 && c_ok16 && d->ldc >= d->N / 2,
                     "gemm swiglu: K-major operands, 16-B aligned bf16 output [M, N/2]");
        KD_CHECK_ARG(!d->aux || (d->ld_aux % 8 == 0 && (uintptr_t)d->aux % 16 == 0), "gemm swiglu: aux alignment");
        GemmP pk = p;
        pk.glu = d->N / 2; pk.act = KD_ACT_NONE;
        pk.gm = pick_gm(ceil_div(d->M, 256), d->N / 256);
        const dim3 grid(ceil_div(d->M, 256) * (d->N / 256), 1);
        pk.gx = (int)grid.x; pk.gy = 1;
#ifdef KD_AB_BUILD
        if (d->variant == 20) hipLaunchKernelGGL((k_gemm9<false, false>), grid, dim3(NTH9), (gemm2_lds<256, 256>()), st, pk);
        else if (!d->b_pretiled && use_v11(d->variant)) hipLaunchKernelGGL((k_gemm11<4>), grid, dim3(NTH8), (gemm2_lds<256, 256>()), st, pk);
        else if (d->variant == 27) hipLaunchKernelGGL((k_gemm12<4 | 256>), grid, dim3(NTH8), (gemm2_lds<256, 256>()), st, pk);
        else if (!d->b_pretiled && use_v12(d->variant)) hipLaunchKernelGGL((k_gemm12<4>), grid, dim3(NTH8), (gemm2_lds<256, 256>()), st, pk);
        else if (d->variant == 22)
            hipLaunchKernelGGL((k_gemm8<false, false, 12>), grid, dim3(NTH8), (gemm2_lds<256, 256>()), st, pk);
        else if (d->variant == 28) {   // stamp build: per-wave cycle totals to the workspace (tools/stamp_glu.py)
            KD_CHECK_ARG(d->workspace && d->workspace_bytes >= (uint64_t)grid.x * (4 * 8 + 4) * 4, "gemm swiglu stamps: workspace");
            pk.sk_ws = (float*)d->workspace;
            hipLaunchKernelGGL((k_gemm8<false, false, 5>), grid, dim3(NTH8), (gemm2_lds<256, 256>()), st, pk);
        }
        else if (glu_epi_v0()) hipLaunchKernelGGL((k_gemm8<false, false, 4 | 512>), grid, dim3(NTH8), (gemm2_lds<256, 256>()), st, pk);
        else
#endif
        if (d->b_pretiled) hipLaunchKernelGGL((k_gemm8<false, false, 4 | 256>), grid, dim3(NTH8), (gemm2_lds<256, 256>()), st, pk);
        else if (d->variant == 21 && sk_fits(grid.x, ceil_div(d->K, BK2), d)) {   // stream-K (v8 SwiGLU build)
            if (const int rc = sk_setup(pk, grid.x, d, st); rc != KD_OK) return rc;
            hipLaunchKernelGGL((k_gemm8<false, false, 4 | 1024>), dim3(pk.gx), dim3(NTH8), (gemm2_lds<256, 256>()), st, pk);
        }
        else hipLaunchKernelGGL((k_gemm8<false, false, 4>), grid, dim3(NTH8), (gemm2_lds<256, 256>()), st, pk);
        KD_LAUNCH_CHECK("k_gemm<swiglu>");
        return KD_OK;
    }
    if (d->b_pretiled) {   // the v8 kernel over every tile, unsplit (the pre-tiled layout is per 256-row tile)
        KD_CHECK_ARG(d->N % 8 == 0 && c_ok16, "gemm b_pretiled: N % 8 == 0 and 16-B aligned C / residual rows");
        GemmP q = p;
        q.gm = pick_gm(ceil_div(d->M, 256), ceil_div(d->N, 256));
        const dim3 grid(ceil_div(d->M, 256) * ceil_div(d->N, 256), 1);
        q.gx = (int)grid.x; q.gy = 1; q.tile0 = 0;
        hipLaunchKernelGGL((k_gemm8<false, false, 256>), grid, dim3(NTH8), (gemm2_lds<256, 256>()), st, q);
        KD_LAUNCH_CHECK("k_gemm8 (b_pretiled)");
        return KD_OK;
    }
#ifdef KD_AB_BUILD
    // v8n (256x128, two workgroups per CU), forced (variant 30); K-major operands, unsplit.  As the
    // auto choice for SigLIP's q|k|v scatter (62.5 vs 71.2 us alone, profiles/r05/v8n_qkv_ab.txt) the
    // c1 step measured no faster (29.05-29.09 vs 29.08-29.13 samples/s), so the plan does not use it
    if (d->variant == 30) {
        // the q|k|v scatter takes 128-column tiles when a RoPE pair never straddles them (no RoPE, or
        // 128 % head_dim == 0: a tile is whole heads)
        KD_CHECK_ARG(!amn && !bmn && (!d->qkv || !d->qkv->cos_t || 128 % d->qkv->hd == 0) && !d->row_stats &&
                     !d->b_pretiled && !dact && d->act != KD_ACT_SWIGLU && d->split_k <= 1 && d->N % 8 == 0 && c_ok16,
                     "gemm variant 30 (v8n): K-major A and B, no SwiGLU / backward activation / row statistics / split, "
                     "N % 8 == 0; a RoPE q|k|v scatter needs 128 % head_dim == 0");
        GemmP q = p;
        q.gm = pick_gm(ceil_div(d->M, 256), ceil_div(d->N, 128));
        q.stag_g = pick_gm(ceil_div(d->M, 256), ceil_div(d->N, 256));   // v8's row groups: v8's bits
        const dim3 grid(ceil_div(d->M, 256) * ceil_div(d->N, 128), 1);
        q.gx = (int)grid.x; q.gy = 1; q.tile0 = 0;
        hipLaunchKernelGGL((k_gemm8n<0>), grid, dim3(NTH8), (gemm2_lds<256, 128, NS8N>()), st, q);
        KD_LAUNCH_CHECK("k_gemm8n");
        return KD_OK;
    }
#endif
    const int force = d->variant;   // 0 auto, 1 v1 128x128, 2/5 v3 256x256, 3/6 v3 256x128, 4/7 v3 128x256,
                                    // 16 v8 256x256 (4 waves, AGPR accumulators), 17-19 v8 diagnostics, 22 v8 register-staged (negative result, kept for A/B)
    if (force != 1 && big_ok) {
        const GemmPlan pl = plan_gemm(d, d->workspace ? d->workspace_bytes : 0);
        const int tbm = pl.var == 4 ? 128 : 256, tbn = pl.var == 3 ? 128 : 256;
        const int tiles = ceil_div(d->M, tbm) * ceil_div(d->N, tbn);
        p.gm = pick_gm(ceil_div(d->M, tbm), ceil_div(d->N, tbn));
        if (pl.var == 21) {   // stream-K (v8): whole waves data-parallel, the rest in runs, folded in-launch
            GemmP q = p;
            if (const int rc = sk_setup(q, tiles, d, st); rc != KD_OK) return rc;
            const size_t lds = gemm2_lds<256, 256>();
            const dim3 grid(q.gx);
            if (!amn && !bmn) hipLaunchKernelGGL((k_gemm8<false, false, 1024>), grid, dim3(NTH8), lds, st, q);
            else if (!amn && bmn) hipLaunchKernelGGL((k_gemm8<false, true, 1024>), grid, dim3(NTH8), lds, st, q);
            else if (amn && bmn) hipLaunchKernelGGL((k_gemm8<true, true, 1024>), grid, dim3(NTH8), lds, st, q);
            else hipLaunchKernelGGL((k_gemm8<true, false, 1024>), grid, dim3(NTH8), lds, st, q);
            KD_LAUNCH_CHECK("k_gemm8 (stream-K)");
            return KD_OK;
        }
        // one launch of the planned kernel over linear tiles [q.tile0, q.tile0 + nt), gy K splits
        auto launch_tiles = [&](const GemmP& q0, int nt, unsigned gy) {
            const dim3 grid((unsigned)nt, gy);
            GemmP q = q0;
            q.gx = nt; q.gy = (int)gy;
#ifdef KD_AB_BUILD
            if (pl.var == 20) {   // v9
                const size_t lds = gemm2_lds<256, 256>();
                if (!amn && !bmn) hipLaunchKernelGGL((k_gemm9<false, false>), grid, dim3(NTH9), lds, st, q);
                else if (!amn && bmn) hipLaunchKernelGGL((k_gemm9<false, true>), grid, dim3(NTH9), lds, st, q);
                else if (amn && bmn) hipLaunchKernelGGL((k_gemm9<true, true>), grid, dim3(NTH9), lds, st, q);
                else hipLaunchKernelGGL((k_gemm9<true, false>), grid, dim3(NTH9), lds, st, q);
            } else
#endif
            if (pl.var == 16) {   // v8; forced variants 17-19 are its diagnostic builds (EXP bits above)
                const size_t lds = gemm2_lds<256, 256>();
#define L8(E)                                                                                                   \
    {                                                                                                           \
        if (!amn && !bmn) hipLaunchKernelGGL((k_gemm8<false, false, E>), grid, dim3(NTH8), lds, st, q);         \
        else if (!amn && bmn) hipLaunchKernelGGL((k_gemm8<false, true, E>), grid, dim3(NTH8), lds, st, q);      \
        else if (amn && bmn) hipLaunchKernelGGL((k_gemm8<true, true, E>), grid, dim3(NTH8), lds, st, q);        \
        else hipLaunchKernelGGL((k_gemm8<true, false, E>), grid, dim3(NTH8), lds, st, q);                       \
    }
#define L8K(E)                                                                                                  \
    {                                                                                                           \
        if (!amn && !bmn) hipLaunchKernelGGL((k_gemm8<false, false, E>), grid, dim3(NTH8), lds, st, q);         \
        else L8(0)                                                                                              \
    }
#ifdef KD_AB_BUILD
                if (!amn && !bmn && use_v11(force)) {   // v11: the same tiles on 32x32x16 MFMAs
                    hipLaunchKernelGGL((k_gemm11<0>), grid, dim3(NTH8), lds, st, q);
                    return;
                }
                if (!amn && !bmn && force == 27) {   // v12 without the odd-step barriers (A/B)
                    hipLaunchKernelGGL((k_gemm12<256>), grid, dim3(NTH8), lds, st, q);
                    return;
                }
                if (!amn && !bmn && use_v12(force)) {   // v12: the same tiles, whole-line K-major staging
                    hipLaunchKernelGGL((k_gemm12<0>), grid, dim3(NTH8), lds, st, q);
                    return;
                }
                switch (force) {   // the diagnostic builds exist for the forward (K-major x K-major) layout only
                    case 17: L8(1) break;   // stamps: every layout
                    case 18: L8K(2) break;
                    case 19: L8K(64) break;
                    case 22: L8K(8) break;
                    default: L8(0) break;
                }
#else
                L8(0)
                (void)force;
#endif
#undef L8K
#undef L8
            } else {
#define L3(BMv, BNv, AM, BMN) hipLaunchKernelGGL((k_gemm3<BMv, BNv, AM, BMN>), grid, dim3(NTH2), (gemm2_lds<BMv, BNv>()), st, q)
#define L3SEL(BMv, BNv)                                     \
    if (!amn && !bmn) L3(BMv, BNv, false, false);           \
    else if (!amn && bmn) L3(BMv, BNv, false, true);        \
    else if (amn && bmn) L3(BMv, BNv, true, true);          \
    else L3(BMv, BNv, true, false);
                if (pl.var == 2) { L3SEL(256, 256) }
                else if (pl.var == 3) { L3SEL(256, 128) }
                else { L3SEL(128, 256) }
#undef L3SEL
#undef L3
            }
        };
        if (pl.split <= 1) {
            p.tile0 = 0;
            launch_tiles(p, tiles, 1);
            KD_LAUNCH_CHECK("k_gemm (tiles)");
            return KD_OK;
        }
        KD_CHECK_ARG(d->workspace && d->workspace_bytes >= (uint64_t)pl.split * d->M * d->N * 4,
                     "gemm: split-K workspace too small");
        if (pl.dp_tiles > 0) {   // hybrid: whole waves unsplit with the full epilogue
            p.tile0 = 0;
            launch_tiles(p, pl.dp_tiles, 1);
            KD_LAUNCH_CHECK("k_gemm (whole waves)");
        }
        if (force == 32 && pl.var == 16) {   // v8 split tiles folded in-launch (no planes, no reduce launch)
            const int nt = tiles - pl.dp_tiles;
            const size_t cnt_b = sk_cnt_bytes(nt);
            KD_CHECK_ARG(d->workspace_bytes >= cnt_b + (size_t)nt * pl.split * SK_TILE_F32 * 4,
                         "gemm: split-K fold workspace too small");
            GemmP q = p;
            q.kchunk = pl.kchunk; q.tile0 = pl.dp_tiles; q.gx = nt; q.gy = pl.split;
            q.sk_cnt = (int*)d->workspace; q.sk_ws = (float*)((char*)d->workspace + cnt_b);
            if (hipMemsetAsync(q.sk_cnt, 0, cnt_b, st) != hipSuccess) return fail(KD_ERR_LAUNCH, "gemm: split-K ticket memset");
            const dim3 grid((unsigned)nt, (unsigned)pl.split);
            const size_t lds = gemm2_lds<256, 256>();
            if (!amn && !bmn) hipLaunchKernelGGL((k_gemm8<false, false, 2048>), grid, dim3(NTH8), lds, st, q);
            else if (!amn && bmn) hipLaunchKernelGGL((k_gemm8<false, true, 2048>), grid, dim3(NTH8), lds, st, q);
            else if (amn && bmn) hipLaunchKernelGGL((k_gemm8<true, true, 2048>), grid, dim3(NTH8), lds, st, q);
            else hipLaunchKernelGGL((k_gemm8<true, false, 2048>), grid, dim3(NTH8), lds, st, q);
            KD_LAUNCH_CHECK("k_gemm8 (split-K fold)");
            return KD_OK;
        }
        GemmP pk = p;   // the split tiles write plain fp32 partial planes
        pk.C = d->workspace; pk.ldc = d->N; pk.c_f32 = 1; pk.accumulate = 0; pk.alpha = 1.f;
        pk.alpha_dev = nullptr; pk.bias = nullptr; pk.aux = nullptr; pk.resid = nullptr; pk.act = KD_ACT_NONE;
        pk.kchunk = pl.kchunk; pk.split_stride = (int64_t)d->M * d->N; pk.tile0 = pl.dp_tiles;
        launch_tiles(pk, tiles - pl.dp_tiles, (unsigned)pl.split);
        KD_LAUNCH_CHECK("k_gemm (split tiles)");
        p.split_stride = (int64_t)d->M * d->N;
        p.tile0 = pl.dp_tiles;
        p.gx = tiles - pl.dp_tiles; p.gy = tbm * tbn / 1024;
        // one float4 column chunk per thread: BM / (1024 / BN) row slabs of 1024 / BN rows per tile
        hipLaunchKernelGGL(k_splitk_reduce, dim3(reduce_grid(p.gx * p.gy)), dim3(256), 0, st,
                           (const float*)d->workspace, pl.split, p, tbm, tbn);
        KD_LAUNCH_CHECK("k_splitk_reduce");
        return KD_OK;
    }
    const int tiles = ceil_div(d->M, BM) * ceil_div(d->N, BN);
    const size_t smem = 4 * TILE_BYTES;
    p.gx = tiles; p.gy = 1;
    if (!amn && !bmn) hipLaunchKernelGGL((k_gemm<false, false>), dim3(tiles), dim3(NTH), smem, st, p);
    else if (!amn && bmn) hipLaunchKernelGGL((k_gemm<false, true>), dim3(tiles), dim3(NTH), smem, st, p);
    else if (amn && bmn) hipLaunchKernelGGL((k_gemm<true, true>), dim3(tiles), dim3(NTH), smem, st, p);
    else hipLaunchKernelGGL((k_gemm<true, false>), dim3(tiles), dim3(NTH), smem, st, p);
    KD_LAUNCH_CHECK("k_gemm");
    return KD_OK;
}

int gemm_plan_query(const kd_gemm_desc* d, int32_t* var, int32_t* split, int32_t* dp) {
    KD_CHECK_ARG(d && var && split && dp, "gemm_plan: null pointer");
    KD_CHECK_SHAPE(d->M > 0 && d->N > 0 && d->K > 0, "gemm_plan: empty shape");
    const bool amn = d->a_layout == KD_LAYOUT_MN_MAJOR, bmn = d->b_layout == KD_LAYOUT_MN_MAJOR;
    const bool big_ok = d->N % 8 == 0 && d->M >= 128 && d->N >= 128 &&
                        ((uint64_t)d->M * d->N >= (1ull << 20) || (d->workspace && d->K >= 2048 && d->split_k != 1)) &&
                        (!amn || d->M % 8 == 0) && (!bmn || d->N % 8 == 0);
    if (d->act == KD_ACT_SWIGLU) { *var = 16; *split = 1; *dp = 0; return KD_OK; }
#ifdef KD_AB_BUILD
    if (d->variant == 30) { *var = 30; *split = 1; *dp = 0; return KD_OK; }   // v8n (launch_gemm)
#endif
    if (d->variant == 1 || !big_ok) { *var = 1; *split = 1; *dp = 0; return KD_OK; }
    const GemmPlan pl = plan_gemm(d, d->workspace ? d->workspace_bytes : 0);
    *var = pl.var; *split = pl.split; *dp = pl.dp_tiles;
    return KD_OK;
}

size_t gemm_workspace_size(const kd_gemm_desc* d) {
    if (!d || d->M <= 0 || d->N <= 0 || d->K <= 0 || d->variant == 1 || d->act == KD_ACT_SWIGLU) return 0;
    const GemmPlan pl = plan_gemm(d, ~0ull);
    if (pl.var == 21) return sk_workspace_bytes((int64_t)ceil_div(d->M, 256) * ceil_div(d->N, 256) - pl.dp_tiles);
    return pl.split > 1 ? (size_t)pl.split * d->M * d->N * 4 : 0;
}

}  // namespace kd
