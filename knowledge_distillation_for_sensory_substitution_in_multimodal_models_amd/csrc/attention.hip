// Flash attention forward / backward for gfx950 (MFMA 16x16x32 bf16, fp32 softmax).
//
// Replaces the attention the reference reaches through transformers:
//   Qwen2 causal GQA (HF5 qwen2 :80-140; 7B: 28q/4kv hd128, 0.5B: 14q/2kv hd64)
//   SigLIP non-causal MHA (HF5 siglip :250-307; 16 heads x hd72, seq 729)
// scores = q k^T * hd^-0.5, softmax in fp32, P rounded to bf16 for the PV product.
//
// Layouts: q/k/v [B, heads, S, HDP] bf16 (head dim zero-padded to HDP in {64,96,128});
//          o / do [B, S, H, hd] bf16 (token-major: what o_proj consumes / produces);
//          lse [B, H, S] fp32 (natural log of sum exp(score)).
//
// Forward (per workgroup: 64 query rows of one head, 4 waves x 16 rows):
//   S^T = K Q^T (MFMA A = K rows from LDS, B = Q in registers) so each lane owns ONE
//   query's scores (4 keys x 4 tiles): the softmax max/sum are lane-local plus two
//   cross-lane xors, the O^T = V^T P^T accumulator is lane-local per query (rescale with
//   no shuffles), and P^T's registers ARE the B operand of the PV MFMA (key order
//   permuted consistently with the V^T fragment read by ds_read_b64_tr_b16).
// Backward (per workgroup: 64 keys of one kv head, 4 waves x 16 keys; loops over the
//   group's query heads and 32-row query tiles): S = Q K^T and dP = dO V^T with the key
//   on the lane, so P / dS registers feed dV^T += dO^T P and dK^T += Q^T dS directly;
//   dS goes through LDS once for dQ += dS K, accumulated with fp32 atomics.
#include "common.h"

#include <cstdlib>
#include <type_traits>

namespace kd {
namespace {

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4_t;
typedef __attribute__((ext_vector_type(2))) float f32x2;
constexpr uint32_t OOB = 0x80000000u;

struct AttnP {
    const bf16* q; const bf16* k; const bf16* v;
    bf16* o; float* lse;
    int B, H, HKV, S, hd;
    float scale_log2;  // hd^-0.5 * log2(e)
};

template <int HDP> struct Geo {
    static constexpr int RB = (HDP == 64) ? 128 : 256;  // LDS row bytes
    static constexpr int KSTEPS = HDP / 32;
    static constexpr int DT = (HDP == 64) ? 4 : (HDP == 96 ? 5 : 8);  // 16-wide d tiles covering hd
};

// chunk-level XOR swizzles (16-B chunks) for the K image (ds_read_b128) and the
// V image (ds_read_b64_tr_b16); see the derivations in DESIGN.md §Attention
template <int RB> __device__ __forceinline__ int swK(int r) { return RB == 256 ? (r & 15) : ((r >> 1) & 7); }
template <int RB> __device__ __forceinline__ int swV(int r) { return RB == 256 ? ((r & 7) << 1) : (((r >> 1) & 3) << 1); }

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}

// 64 rows x HDP of a [S][HDP] head slab -> LDS image [64][RB] with chunk swizzle SW
template <int HDP, bool VIMG>
__device__ __forceinline__ void stage_kv(char* lds, const bf16* slab, int row0, int S, int wid, int lane) {
    constexpr int RB = Geo<HDP>::RB;
    constexpr int ROWS_PER = 1024 / RB;       // rows per wave-instruction
    constexpr int CH = RB / 16;               // chunks per LDS row
    constexpr int NINSTR = 64 / ROWS_PER;     // wave-instructions per tile
    const int rows_valid = min(64, S - row0);
    auto rs = rsrc(slab + (int64_t)row0 * HDP, (uint32_t)(rows_valid * HDP * 2));
#pragma unroll
    for (int s = 0; s < NINSTR / 4; ++s) {
        const int i = wid * (NINSTR / 4) + s;
        const int r = i * ROWS_PER + lane / CH;
        const int c = lane % CH;
        const int gc = c ^ (VIMG ? swV<RB>(r) : swK<RB>(r));
        const uint32_t voff = (gc * 8 < HDP) ? (uint32_t)((r * HDP + gc * 8) * 2) : OOB;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void_t*)(lds + i * 1024), 16, voff, 0, 0, 0);
    }
}

template <int RB>
__device__ __forceinline__ bf16x8 k_frag(const char* lds, int row, int chunk) {
    return *(const bf16x8*)(lds + row * RB + ((chunk ^ swK<RB>(row)) << 4));
}

// transposed 4-row read: rows r0+q (q = lane-in-group >> 2), cols d0 + 4p .. +3
template <int RB>
__device__ __forceinline__ bf16x4 tr_read(const char* lds, int r, int d) {
    const int c = d >> 3;
    const char* a = lds + r * RB + ((c ^ swV<RB>(r)) << 4) + ((d & 4) << 1);
    return __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4_t*)a);
}

// The same transposed read through inline asm: with the builtin, hipcc cannot tell it from
// the in-flight LDS-DMA of the next K/V tile and waits vmcnt(0) before the first one,
// so the prefetch only overlapped QK^T + softmax, not PV. The caller retires these reads
// with its own lgkmcnt(0) (+ sched_barrier) before the MFMAs that consume them.
template <int RB>
__device__ __forceinline__ bf16x4 tr_read_asm(const char* lds, int r, int d) {
    const int c = d >> 3;
    const char* a = lds + r * RB + ((c ^ swV<RB>(r)) << 4) + ((d & 4) << 1);
    u32x2 v;
    asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(v) : "v"((uint32_t)(uintptr_t)a));
    return __builtin_bit_cast(bf16x4, v);
}

// The same read from a precomputed per-lane LDS byte address plus an immediate offset (the
// buffer / row part of the address is a compile-time constant in the unrolled tile loop).
template <int OFF>
__device__ __forceinline__ bf16x4 tr_read_off(uint32_t addr) {
    u32x2 v;
    asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "i"(OFF));
    return __builtin_bit_cast(bf16x4, v);
}

// NQ query sub-tiles of 16 rows per wave (workgroup = 4 waves x 16·NQ rows): every K
// fragment (b128) and V^T fragment (tr_b16) read from LDS feeds NQ MFMAs, so LDS bytes
// per FLOP drop by NQ (at NQ = 1 the kernel was bound by its LDS reads: one 64-key tile =
// 32 KiB of fragment reads per wave for a 16 x 64 block of scores).
template <int HDP, bool CAUSAL, int NQ>
__global__ void __launch_bounds__(256, 2) k_attn_fwd(AttnP p) {
    constexpr int RB = Geo<HDP>::RB, KS = Geo<HDP>::KSTEPS, DT = Geo<HDP>::DT;
    constexpr int TILE = 64 * RB;
    // HDP 96 holds hd <= 80 (SigLIP: 72): the QK^T products take two 32-deep MFMA steps and
    // one 16-deep step (v_mfma_f32_16x16x16_bf16) over dims [64, 80) instead of a third
    // 32-deep step over zero padding
    constexpr bool HALF = HDP == 96;
    constexpr int KSF = HALF ? KS - 1 : KS;
    constexpr int QBLK = 64 * NQ;   // query rows per workgroup
    extern __shared__ __attribute__((aligned(16))) char smem[];  // [2][K TILE | V TILE]
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int g = lane >> 4, li = lane & 15;
    const int nqb = (p.S + QBLK - 1) / QBLK;
    // grid (H, B, query blocks): every head's longest causal block is dispatched first, the
    // shortest fill the tail
    const int qb = CAUSAL ? (nqb - 1 - (int)blockIdx.z) : (int)blockIdx.z;
    const int h = blockIdx.x, b = blockIdx.y, kvh = h / (p.H / p.HKV);
    const bf16* Q = p.q + ((int64_t)(b * p.H + h) * p.S) * HDP;
    const bf16* K = p.k + ((int64_t)(b * p.HKV + kvh) * p.S) * HDP;
    const bf16* V = p.v + ((int64_t)(b * p.HKV + kvh) * p.S) * HDP;
    int myq[NQ];
#pragma unroll
    for (int j = 0; j < NQ; ++j) myq[j] = qb * QBLK + wid * 16 * NQ + j * 16 + li;

    bf16x8 qf[NQ][KS];
    bf16x4 qh[NQ];
#pragma unroll
    for (int j = 0; j < NQ; ++j) {
#pragma unroll
        for (int kk = 0; kk < KSF; ++kk) {
            if (myq[j] < p.S) qf[j][kk] = *(const bf16x8*)(Q + (int64_t)myq[j] * HDP + kk * 32 + 8 * g);
            else qf[j][kk] = (bf16x8){};
        }
        if (HALF) qh[j] = myq[j] < p.S ? *(const bf16x4*)(Q + (int64_t)myq[j] * HDP + KSF * 32 + 4 * g) : (bf16x4){};
    }
    f32x4 o[NQ][DT];
#pragma unroll
    for (int j = 0; j < NQ; ++j)
#pragma unroll
        for (int d = 0; d < DT; ++d) o[j][d] = (f32x4){0.f, 0.f, 0.f, 0.f};
    float m[NQ], l[NQ];
#pragma unroll
    for (int j = 0; j < NQ; ++j) { m[j] = -INFINITY; l[j] = 0.f; }

    const int nkv_all = (p.S + 63) / 64;
    const int nkv = CAUSAL ? min((qb + 1) * QBLK / 64, nkv_all) : nkv_all;
    stage_kv<HDP, false>(smem, K, 0, p.S, wid, lane);
    stage_kv<HDP, true>(smem + TILE, V, 0, p.S, wid, lane);
    // per-lane LDS byte offsets of the fragment reads: the swizzles depend on the lane only,
    // so the buffer, the key tile kt and the 32-key step ks are immediate offsets of the
    // ds_read instructions in the tile loop (unrolled by two: even tiles read buffer 0)
    int koff[KS];
#pragma unroll
    for (int kk = 0; kk < KS; ++kk) koff[kk] = li * RB + (((kk * 4 + g) ^ swK<RB>(li)) << 4);
    // the 16-deep step's A fragment: row li, dims 32 KSF + 4g + [0, 4) = 8 B of chunk 4 KSF + g/2
    const int khoff = li * RB + (((KSF * 4 + (g >> 1)) ^ swK<RB>(li)) << 4) + (g & 1) * 8;
    uint32_t vaddr[DT];
    {
        const uint32_t sbase = (uint32_t)(uintptr_t)smem;
        const int r = 4 * g + (li >> 2);
#pragma unroll
        for (int d = 0; d < DT; ++d) {
            const int dc = d * 16 + 4 * (li & 3);
            vaddr[d] = sbase + TILE + r * RB + ((((dc >> 3) ^ swV<RB>(r))) << 4) + ((dc & 4) << 1);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();

    auto tile = [&](const int t, auto buf_c) {
        constexpr int BUF = decltype(buf_c)::value;
        if (t + 1 < nkv) {
            char* nb = smem + (BUF ^ 1) * 2 * TILE;
            stage_kv<HDP, false>(nb, K, (t + 1) * 64, p.S, wid, lane);
            stage_kv<HDP, true>(nb + TILE, V, (t + 1) * 64, p.S, wid, lane);
        }
        const char* kt_l = smem + BUF * 2 * TILE;
        // ---- S^T tiles: rows = keys 16kt + 4g + r, col = the lane's query of sub-tile j
        f32x4 sc[NQ][4];
#pragma unroll
        for (int kt = 0; kt < 4; ++kt) {
#pragma unroll
            for (int j = 0; j < NQ; ++j) sc[j][kt] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int kk = 0; kk < KSF; ++kk) {
                const bf16x8 kf = *(const bf16x8*)(kt_l + koff[kk] + kt * 16 * RB);
#pragma unroll
                for (int j = 0; j < NQ; ++j)
                    sc[j][kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[j][kk], sc[j][kt], 0, 0, 0);
            }
            if (HALF) {
                const bf16x4 kh = *(const bf16x4*)(kt_l + khoff + kt * 16 * RB);
#pragma unroll
                for (int j = 0; j < NQ; ++j)
                    sc[j][kt] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(kh, qh[j], sc[j][kt], 0, 0, 0);
            }
        }
        // ---- online softmax in the log2 domain. The mask is applied only on tiles that
        // cross the causal diagonal or the sequence end (wave-uniform test); the scale is
        // folded into the exponent's fma; v_exp_f32 directly (exp2f adds range handling).
        // Lazy rescale: the exponent reference m only moves when the tile's max exceeds it
        // by more than 8 (P <= 2^8 otherwise, exact in fp32 accumulation and bf16 range), so
        // the O rescale (8·DT multiplies per sub-tile) runs on a few tiles per row only.
        const int key0 = t * 64 + 4 * g;
        bf16x8 pf[NQ][2];
#pragma unroll
        for (int j = 0; j < NQ; ++j) {
            const int qlo = qb * QBLK + wid * 16 * NQ + j * 16;   // first query of this sub-tile
            if (t * 64 + 63 >= p.S || (CAUSAL && t * 64 + 63 > qlo)) {
#pragma unroll
                for (int kt = 0; kt < 4; ++kt)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int key = key0 + 16 * kt + r;
                        if (key >= p.S || (CAUSAL && key > myq[j])) sc[j][kt][r] = -INFINITY;
                    }
            }
            float mt = -INFINITY;
#pragma unroll
            for (int kt = 0; kt < 4; ++kt)
#pragma unroll
                for (int r = 0; r < 4; ++r) mt = fmaxf(mt, sc[j][kt][r]);
            mt = fmaxf(mt, __shfl_xor(mt, 16, 64));
            mt = fmaxf(mt, __shfl_xor(mt, 32, 64));
            const float mts = mt * p.scale_log2;   // scale > 0: max commutes
            const bool move = mts > m[j] + 8.f;   // also the first tile with a finite score (m = -inf)
            if (__ballot(move)) {
                const float mn = move ? mts : m[j];
                const float alpha = __builtin_amdgcn_exp2f(m[j] - mn);   // m = -inf: 0 (O, l are 0)
                l[j] *= alpha;
#pragma unroll
                for (int d = 0; d < DT; ++d) o[j][d] *= alpha;
                m[j] = mn;
            }
            const float mref = (m[j] == -INFINITY) ? 0.f : m[j];
            float ls = 0.f;
#pragma unroll
            for (int kt = 0; kt < 4; ++kt)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float e = __builtin_amdgcn_exp2f(fmaf(sc[j][kt][r], p.scale_log2, -mref));
                    sc[j][kt][r] = e;
                    ls += e;
                }
            l[j] += ls;
#pragma unroll
            for (int ks = 0; ks < 2; ++ks)
#pragma unroll
                for (int r = 0; r < 4; ++r) { pf[j][ks][r] = (bf16)sc[j][2 * ks][r]; pf[j][ks][4 + r] = (bf16)sc[j][2 * ks + 1][r]; }
        }
        // ---- O^T += V^T P^T, two 32-key steps; each V^T fragment feeds the NQ sub-tiles
        auto pv = [&](auto ks_c) {
            constexpr int KS_ = decltype(ks_c)::value;
            constexpr int OFF0 = BUF * 2 * TILE + (32 * KS_) * RB, OFF1 = OFF0 + 16 * RB;
            bf16x4 v0[DT], v1[DT];
#pragma unroll
            for (int d = 0; d < DT; ++d) {
                v0[d] = tr_read_off<OFF0>(vaddr[d]);
                v1[d] = tr_read_off<OFF1>(vaddr[d]);
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int d = 0; d < DT; ++d) {
                bf16x8 vf;
                vf[0] = v0[d][0]; vf[1] = v0[d][1]; vf[2] = v0[d][2]; vf[3] = v0[d][3];
                vf[4] = v1[d][0]; vf[5] = v1[d][1]; vf[6] = v1[d][2]; vf[7] = v1[d][3];
#pragma unroll
                for (int j = 0; j < NQ; ++j) o[j][d] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pf[j][KS_], o[j][d], 0, 0, 0);
            }
        };
        pv(std::integral_constant<int, 0>{});
        pv(std::integral_constant<int, 1>{});
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    };
    int t = 0;
    for (; t + 1 < nkv; t += 2) {
        tile(t, std::integral_constant<int, 0>{});
        tile(t + 1, std::integral_constant<int, 1>{});
    }
    if (t < nkv) tile(t, std::integral_constant<int, 0>{});
#pragma unroll
    for (int j = 0; j < NQ; ++j) {
        float lj = l[j];
        lj += __shfl_xor(lj, 16, 64);
        lj += __shfl_xor(lj, 32, 64);
        if (myq[j] < p.S) {
            const float inv = 1.f / lj;
            bf16* orow = p.o + (((int64_t)b * p.S + myq[j]) * p.H + h) * p.hd;
#pragma unroll
            for (int d = 0; d < DT; ++d) {
                const int dd = d * 16 + 4 * g;
                if (dd < p.hd) {
                    bf16x4 w;
#pragma unroll
                    for (int r = 0; r < 4; ++r) w[r] = (bf16)(o[j][d][r] * inv);
                    *(bf16x4*)(orow + dd) = w;
                }
            }
            if (g == 0 && p.lse) p.lse[((int64_t)b * p.H + h) * p.S + myq[j]] = (m[j] + log2f(lj)) * 0.6931471805599453f;
        }
    }
}

// ------------------------------------------------------------------ backward ----
struct AttnBwdP {
    const bf16* q; const bf16* k; const bf16* v;   // [B, heads, S, HDP]
    const bf16* dO;                                  // [B, S, H, hd]
    const float* lse; const float* delta;           // [B, H, S]
    float* dq;                                      // [B, H, S, HDP] fp32 (scaled)
    bf16* dk; bf16* dv;                             // [B, HKV, S, HDP]
    float* dkp; float* dvp;                         // GQA partials [B, H, S, HDP] fp32 (grp > 1)
    int B, H, HKV, S, hd;
    float scale, scale_log2;
};

// 64 rows x ncols of a row-strided matrix (token-major dO) -> swK LDS image [64][RB];
// columns >= ncols and rows >= S land as zeros (out-of-range buffer offsets)
template <int HDP>
__device__ __forceinline__ void stage_rows_dma(char* lds, const bf16* base, int64_t row_stride, int ncols, int row0,
                                               int S, int wid, int lane) {
    constexpr int RB = Geo<HDP>::RB;
    constexpr int ROWS_PER = 1024 / RB, CH = RB / 16, NINSTR = 64 / ROWS_PER;
    const int rows_valid = min(64, S - row0);
    const uint32_t bytes = rows_valid <= 0 ? 0u : (uint32_t)(((int64_t)(rows_valid - 1) * row_stride + ncols) * 2);
    auto rs = rsrc(base + (int64_t)row0 * row_stride, bytes);
#pragma unroll
    for (int s = 0; s < NINSTR / 4; ++s) {
        const int i = wid * (NINSTR / 4) + s;
        const int r = i * ROWS_PER + lane / CH;
        const int c = lane % CH;
        const int gc = c ^ swK<RB>(r);
        const uint32_t voff = (gc * 8 < ncols && r < rows_valid) ? (uint32_t)((r * row_stride + gc * 8) * 2) : OOB;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void_t*)(lds + i * 1024), 16, voff, 0, 0, 0);
    }
}

// 64 consecutive fp32 of a [S] row (lse / delta) -> LDS, one dword per lane (wave 0 only)
__device__ __forceinline__ void stage_vec64(float* lds, const float* base, int row0, int S, int lane) {
    const int rows_valid = min(64, S - row0);
    auto rs = rsrc(base + row0, rows_valid <= 0 ? 0u : (uint32_t)(rows_valid * 4));
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void_t*)lds, 4, lane < rows_valid ? (uint32_t)(lane * 4) : OOB,
                                             0, 0, 0);
}

// transposed read from a swK-swizzled image (rows r, 4 consecutive cols starting at d)
template <int RB>
__device__ __forceinline__ bf16x4 tr_read_k(const char* lds, int r, int d) {
    const int c = d >> 3;
    const char* a = lds + r * RB + ((c ^ swK<RB>(r)) << 4) + ((d & 4) << 1);
    return __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4_t*)a);
}

// asm form of tr_read_k (see tr_read_asm): retired by the caller's lgkmcnt(0)
template <int RB>
__device__ __forceinline__ bf16x4 tr_read_k_asm(const char* lds, int r, int d) {
    const int c = d >> 3;
    const char* a = lds + r * RB + ((c ^ swK<RB>(r)) << 4) + ((d & 4) << 1);
    u32x2 v;
    asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(v) : "v"((uint32_t)(uintptr_t)a));
    return __builtin_bit_cast(bf16x4, v);
}

__device__ __forceinline__ bf16x8 cat4(bf16x4 a, bf16x4 b) {
    bf16x8 r;
    r[0] = a[0]; r[1] = a[1]; r[2] = a[2]; r[3] = a[3];
    r[4] = b[0]; r[5] = b[1]; r[6] = b[2]; r[7] = b[3];
    return r;
}

// dK / dV for 64 keys of ONE query head (4 waves x 16 keys, key on the lane), looping
// over 64-row query tiles double-buffered through LDS-DMA (Q, dO images + lse, delta):
//   S = Q K^T, dP = dO V^T  (A = Q / dO rows from LDS, B = K / V fragments in registers)
//   dV^T += dO^T P, dK^T += Q^T dS  (A = transposed LDS reads, B = P / dS registers)
// MHA writes bf16 dK (scaled) / dV; GQA writes fp32 per-query-head partials that
// k_attn_group_sum folds over the group (deterministic, no atomics).
template <int HDP, bool CAUSAL>
__global__ void __launch_bounds__(256, 2) k_attn_bwd_dkdv(AttnBwdP p) {
    constexpr int RB = Geo<HDP>::RB, KS = Geo<HDP>::KSTEPS, DT = Geo<HDP>::DT;
    constexpr int TILE = 64 * RB, BUF = 2 * TILE + 512;
    constexpr bool HALF = HDP == 96;   // hd <= 80: a 16-deep last step (see k_attn_fwd)
    constexpr int KSF = HALF ? KS - 1 : KS;
    extern __shared__ __attribute__((aligned(16))) char smem[];   // [2][Q TILE | dO TILE | lse2 64 | delta 64]
    // the wave index is wave-uniform (readfirstlane): the edge test below is a scalar branch
    const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int g = lane >> 4, li = lane & 15;
    // grid (H, B, key blocks): key block 0 (the most causal query tiles) of every head first
    const int kb0 = blockIdx.z * 64;
    const int h = blockIdx.x, b = blockIdx.y;
    const int grp = p.H / p.HKV, kvh = h / grp;
    const bf16* K = p.k + ((int64_t)(b * p.HKV + kvh) * p.S) * HDP;
    const bf16* V = p.v + ((int64_t)(b * p.HKV + kvh) * p.S) * HDP;
    const bf16* Q = p.q + ((int64_t)(b * p.H + h) * p.S) * HDP;
    const bf16* dO = p.dO + ((int64_t)b * p.S * p.H + h) * p.hd;   // row q at + q*H*hd
    const float* LSE = p.lse + ((int64_t)b * p.H + h) * p.S;
    const float* DEL = p.delta + ((int64_t)b * p.H + h) * p.S;
    const int64_t ldo = (int64_t)p.H * p.hd;
    const int mykey = kb0 + wid * 16 + li;

    bf16x8 kf[KS], vf[KS];
    bf16x4 kh = {}, vh = {};
#pragma unroll
    for (int kk = 0; kk < KSF; ++kk) {
        if (mykey < p.S) {
            kf[kk] = *(const bf16x8*)(K + (int64_t)mykey * HDP + kk * 32 + 8 * g);
            vf[kk] = *(const bf16x8*)(V + (int64_t)mykey * HDP + kk * 32 + 8 * g);
        } else {
            kf[kk] = (bf16x8){}; vf[kk] = (bf16x8){};
        }
    }
    if (HALF && mykey < p.S) {
        kh = *(const bf16x4*)(K + (int64_t)mykey * HDP + KSF * 32 + 4 * g);
        vh = *(const bf16x4*)(V + (int64_t)mykey * HDP + KSF * 32 + 4 * g);
    }
    f32x4 dk[DT], dv[DT];
#pragma unroll
    for (int d = 0; d < DT; ++d) { dk[d] = (f32x4){0.f, 0.f, 0.f, 0.f}; dv[d] = dk[d]; }

    // per-lane LDS byte offsets inside one buffer (the swizzles depend on the lane only):
    // row fragments (rows 16qs + li, + 16 qs RB immediate), the 16-deep step's fragment, and
    // the transposed reads (rows 32ks + 4g + li/4 (+16): + (32ks + 16) RB immediate)
    int qoff[KS];
#pragma unroll
    for (int kk = 0; kk < KS; ++kk) qoff[kk] = li * RB + (((kk * 4 + g) ^ swK<RB>(li)) << 4);
    const int qhoff = li * RB + (((KSF * 4 + (g >> 1)) ^ swK<RB>(li)) << 4) + (g & 1) * 8;
    int troff[DT];
    {
        const int r = 4 * g + (li >> 2);
#pragma unroll
        for (int d = 0; d < DT; ++d)
            troff[d] = r * RB + (((2 * d + ((li & 3) >> 1)) ^ swK<RB>(r)) << 4) + (li & 1) * 8;
    }

    const int nqt = (p.S + 63) / 64;
    const int qt0 = CAUSAL ? (int)blockIdx.z : 0;
    // lse reaches LDS pre-scaled to log2 units (wave 0: a register load issued with the
    // tile's DMA, written after the tile's compute), delta by LDS-DMA
    float lse_nx = 0.f;
    auto stage = [&](char* buf, int qt) {
        stage_kv<HDP, false>(buf, Q, qt * 64, p.S, wid, lane);
        stage_rows_dma<HDP>(buf + TILE, dO, ldo, p.hd, qt * 64, p.S, wid, lane);
        if (wid == 0) {
            lse_nx = qt * 64 + lane < p.S ? LSE[qt * 64 + lane] : 0.f;
            stage_vec64((float*)(buf + 2 * TILE + 256), DEL, qt * 64, p.S, lane);
        }
    };
    auto put_lse = [&](char* buf) {
        if (wid == 0) ((float*)(buf + 2 * TILE))[lane] = lse_nx * 1.4426950408889634f;
    };
    stage(smem, qt0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    put_lse(smem);
    __syncthreads();
    for (int qt = qt0; qt < nqt; ++qt) {
        const int cur = (qt - qt0) & 1;
        if (qt + 1 < nqt) stage(smem + (cur ^ 1) * BUF, qt + 1);
        const char* lQ = smem + cur * BUF;
        const char* lO = lQ + TILE;
        const float* lL = (const float*)(lQ + 2 * TILE);
        const float* lD = lL + 64;
        const int q0 = qt * 64;
        // S, dP: rows q = q0 + 16qs + 4g + r, col = my key
        f32x4 s[4], dp[4];
#pragma unroll
        for (int qs = 0; qs < 4; ++qs) {
            s[qs] = (f32x4){0.f, 0.f, 0.f, 0.f};
            dp[qs] = s[qs];
#pragma unroll
            for (int kk = 0; kk < KSF; ++kk) {
                s[qs] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(*(const bf16x8*)(lQ + qoff[kk] + qs * 16 * RB), kf[kk],
                                                               s[qs], 0, 0, 0);
                dp[qs] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(*(const bf16x8*)(lO + qoff[kk] + qs * 16 * RB), vf[kk],
                                                                dp[qs], 0, 0, 0);
            }
            if (HALF) {
                s[qs] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(*(const bf16x4*)(lQ + qhoff + qs * 16 * RB), kh, s[qs],
                                                                 0, 0, 0);
                dp[qs] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(*(const bf16x4*)(lO + qhoff + qs * 16 * RB), vh, dp[qs],
                                                                  0, 0, 0);
            }
        }
        // mask only where the tile crosses the diagonal or an edge (wave-uniform branch):
        // masked scores become -inf, so P = 0 there (the empty volatile asm keeps the branch:
        // hipcc would otherwise speculate the compares into every tile)
        if (q0 + 63 >= p.S || kb0 + wid * 16 + 15 >= p.S || (CAUSAL && kb0 + wid * 16 + 15 > q0)) {
            asm volatile("" ::: "memory");
#pragma unroll
            for (int qs = 0; qs < 4; ++qs)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int q = q0 + 16 * qs + 4 * g + r;
                    if (q >= p.S || mykey >= p.S || (CAUSAL && mykey > q)) s[qs][r] = -INFINITY;
                }
        }
        // P = 2^(s·scale_log2 - lse2), dS = P (dP - delta): packed fp32 pairs (v_pk_fma / add / mul)
        const f32x2 sl2 = {p.scale_log2, p.scale_log2};
#pragma unroll
        for (int qs = 0; qs < 4; ++qs) {
            const f32x4 l2 = *(const f32x4*)(lL + 16 * qs + 4 * g), dl = *(const f32x4*)(lD + 16 * qs + 4 * g);
#pragma unroll
            for (int r = 0; r < 4; r += 2) {
                const f32x2 x = f32x2{s[qs][r], s[qs][r + 1]} * sl2 - f32x2{l2[r], l2[r + 1]};
                const f32x2 pv = {__builtin_amdgcn_exp2f(x[0]), __builtin_amdgcn_exp2f(x[1])};
                const f32x2 ds = pv * (f32x2{dp[qs][r], dp[qs][r + 1]} - f32x2{dl[r], dl[r + 1]});
                s[qs][r] = pv[0]; s[qs][r + 1] = pv[1];
                dp[qs][r] = ds[0]; dp[qs][r + 1] = ds[1];
            }
        }
        // dV^T += dO^T P ; dK^T += Q^T dS over two 32-query steps
        const uint32_t bq = (uint32_t)(uintptr_t)lQ;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            bf16x8 pfr, dsf;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                pfr[r] = (bf16)s[2 * ks][r]; pfr[4 + r] = (bf16)s[2 * ks + 1][r];
                dsf[r] = (bf16)dp[2 * ks][r]; dsf[4 + r] = (bf16)dp[2 * ks + 1][r];
            }
            bf16x4 o0[DT], o1[DT], x0[DT], x1[DT];
#pragma unroll
            for (int d = 0; d < DT; ++d) {
                const uint32_t a = bq + troff[d];
                if (ks == 0) {
                    o0[d] = tr_read_off<TILE>(a);
                    o1[d] = tr_read_off<TILE + 16 * RB>(a);
                    x0[d] = tr_read_off<0>(a);
                    x1[d] = tr_read_off<16 * RB>(a);
                } else {
                    o0[d] = tr_read_off<TILE + 32 * RB>(a);
                    o1[d] = tr_read_off<TILE + 48 * RB>(a);
                    x0[d] = tr_read_off<32 * RB>(a);
                    x1[d] = tr_read_off<48 * RB>(a);
                }
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int d = 0; d < DT; ++d) {
                dv[d] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cat4(o0[d], o1[d]), pfr, dv[d], 0, 0, 0);
                dk[d] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cat4(x0[d], x1[d]), dsf, dk[d], 0, 0, 0);
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (qt + 1 < nqt) put_lse(smem + (cur ^ 1) * BUF);
        __syncthreads();
    }
    // lane owns key = mykey, d = 16d + 4g + r
    if (mykey < p.S) {
        if (grp == 1) {
            bf16* dKr = p.dk + ((int64_t)(b * p.HKV + kvh) * p.S + mykey) * HDP;
            bf16* dVr = p.dv + ((int64_t)(b * p.HKV + kvh) * p.S + mykey) * HDP;
#pragma unroll
            for (int d = 0; d < DT; ++d) {
                const int dd = d * 16 + 4 * g;
                bf16x4 wk, wv;
#pragma unroll
                for (int r = 0; r < 4; ++r) { wk[r] = (bf16)(dk[d][r] * p.scale); wv[r] = (bf16)dv[d][r]; }
                *(bf16x4*)(dKr + dd) = wk;
                *(bf16x4*)(dVr + dd) = wv;
            }
        } else {
            float* dKr = p.dkp + ((int64_t)(b * p.H + h) * p.S + mykey) * HDP;
            float* dVr = p.dvp + ((int64_t)(b * p.H + h) * p.S + mykey) * HDP;
#pragma unroll
            for (int d = 0; d < DT; ++d) {
                const int dd = d * 16 + 4 * g;
                *(f32x4*)(dKr + dd) = dk[d];
                *(f32x4*)(dVr + dd) = dv[d];
            }
        }
    }
}

// dK[b,kvh] = scale * sum_{h in group} dKp[b,h], dV likewise (d < 16*DT columns)
__global__ void k_attn_group_sum(const float* __restrict__ dkp, const float* __restrict__ dvp, bf16* __restrict__ dk,
                                 bf16* __restrict__ dv, int B, int H, int HKV, int S, int hdp, int dcols, float scale) {
    const int grp = H / HKV, c4 = dcols / 4;
    const int64_t total = (int64_t)B * HKV * S * c4;
    for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total; idx += (int64_t)gridDim.x * blockDim.x) {
        const int c = (int)(idx % c4) * 4;
        const int64_t rs = idx / c4;               // (b, kvh, s)
        const int s = (int)(rs % S);
        const int64_t bk = rs / S;
        const int kvh = (int)(bk % HKV), b = (int)(bk / HKV);
        f32x4 ak = (f32x4){0.f, 0.f, 0.f, 0.f}, av = ak;
        for (int j = 0; j < grp; ++j) {
            const int64_t off = (((int64_t)b * H + kvh * grp + j) * S + s) * hdp + c;
            ak += *(const f32x4*)(dkp + off);
            av += *(const f32x4*)(dvp + off);
        }
        bf16x4 wk, wv;
#pragma unroll
        for (int r = 0; r < 4; ++r) { wk[r] = (bf16)(ak[r] * scale); wv[r] = (bf16)av[r]; }
        *(bf16x4*)(dk + rs * hdp + c) = wk;
        *(bf16x4*)(dv + rs * hdp + c) = wv;
    }
}

// dQ for 64·NQ query rows of one head (4 waves x NQ sub-tiles of 16 rows, query on the
// lane), the forward's structure: K / V tiles double-buffered through LDS-DMA, S^T = K Q^T
// and dP^T = V dO^T recomputed, dS^T in registers feeds dQ^T += K^T dS^T (A = transposed K
// reads). Every K / V / K^T fragment read from LDS feeds the NQ sub-tiles.
// No atomics: each workgroup owns its rows of dQ.
template <int HDP, bool CAUSAL, int NQ>
__global__ void __launch_bounds__(256, 2) k_attn_bwd_dq(AttnBwdP p) {
    constexpr int RB = Geo<HDP>::RB, KS = Geo<HDP>::KSTEPS, DT = Geo<HDP>::DT;
    constexpr int TILE = 64 * RB;
    constexpr bool HALF = HDP == 96;   // hd <= 80: a 16-deep last step (see k_attn_fwd)
    constexpr int KSF = HALF ? KS - 1 : KS;
    constexpr int QBLK = 64 * NQ;
    extern __shared__ __attribute__((aligned(16))) char smem[];   // [2][K TILE | V TILE]
    // wave-uniform wave index (readfirstlane): the per-sub-tile edge test is a scalar branch
    const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int g = lane >> 4, li = lane & 15;
    const int nqb = (p.S + QBLK - 1) / QBLK;
    // grid (H, B, query blocks): every head's longest causal block is dispatched first, the
    // shortest fill the tail
    const int qb = CAUSAL ? (nqb - 1 - (int)blockIdx.z) : (int)blockIdx.z;
    const int h = blockIdx.x, b = blockIdx.y, kvh = h / (p.H / p.HKV);
    const bf16* Q = p.q + ((int64_t)(b * p.H + h) * p.S) * HDP;
    const bf16* K = p.k + ((int64_t)(b * p.HKV + kvh) * p.S) * HDP;
    const bf16* V = p.v + ((int64_t)(b * p.HKV + kvh) * p.S) * HDP;
    int myq[NQ];
    bool qok[NQ];
    bf16x8 qf[NQ][KS], df[NQ][KS];
    bf16x4 qh[NQ], dh[NQ];
    float lse2[NQ], dl[NQ];
#pragma unroll
    for (int j = 0; j < NQ; ++j) {
        myq[j] = qb * QBLK + wid * 16 * NQ + j * 16 + li;
        qok[j] = myq[j] < p.S;
        const bf16* dOr = p.dO + (((int64_t)b * p.S + myq[j]) * p.H + h) * p.hd;
#pragma unroll
        for (int kk = 0; kk < KSF; ++kk) {
            const int d0 = kk * 32 + 8 * g;
            qf[j][kk] = qok[j] ? *(const bf16x8*)(Q + (int64_t)myq[j] * HDP + d0) : (bf16x8){};
            df[j][kk] = (qok[j] && d0 < p.hd) ? *(const bf16x8*)(dOr + d0) : (bf16x8){};
        }
        if (HALF) {   // dims 32 KSF + 4g + [0, 4); dO rows hold hd (a multiple of 4) columns
            const int d0 = KSF * 32 + 4 * g;
            qh[j] = qok[j] ? *(const bf16x4*)(Q + (int64_t)myq[j] * HDP + d0) : (bf16x4){};
            dh[j] = (qok[j] && d0 < p.hd) ? *(const bf16x4*)(dOr + d0) : (bf16x4){};
        }
        lse2[j] = qok[j] ? p.lse[((int64_t)b * p.H + h) * p.S + myq[j]] * 1.4426950408889634f : 0.f;
        dl[j] = qok[j] ? p.delta[((int64_t)b * p.H + h) * p.S + myq[j]] : 0.f;
    }
    f32x4 acc[NQ][DT];
#pragma unroll
    for (int j = 0; j < NQ; ++j)
#pragma unroll
        for (int d = 0; d < DT; ++d) acc[j][d] = (f32x4){0.f, 0.f, 0.f, 0.f};

    // per-lane LDS byte offsets inside one buffer (see k_attn_bwd_dkdv)
    int koff[KS];
#pragma unroll
    for (int kk = 0; kk < KS; ++kk) koff[kk] = li * RB + (((kk * 4 + g) ^ swK<RB>(li)) << 4);
    const int khoff = li * RB + (((KSF * 4 + (g >> 1)) ^ swK<RB>(li)) << 4) + (g & 1) * 8;
    int troff[DT];
    {
        const int r = 4 * g + (li >> 2);
#pragma unroll
        for (int d = 0; d < DT; ++d)
            troff[d] = r * RB + (((2 * d + ((li & 3) >> 1)) ^ swK<RB>(r)) << 4) + (li & 1) * 8;
    }
    const int nkv_all = (p.S + 63) / 64;
    const int nkv = CAUSAL ? min((qb + 1) * QBLK / 64, nkv_all) : nkv_all;
    stage_kv<HDP, false>(smem, K, 0, p.S, wid, lane);
    stage_kv<HDP, false>(smem + TILE, V, 0, p.S, wid, lane);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int t = 0; t < nkv; ++t) {
        const int cur = t & 1;
        if (t + 1 < nkv) {
            char* nb = smem + (cur ^ 1) * 2 * TILE;
            stage_kv<HDP, false>(nb, K, (t + 1) * 64, p.S, wid, lane);
            stage_kv<HDP, false>(nb + TILE, V, (t + 1) * 64, p.S, wid, lane);
        }
        const char* lK = smem + cur * 2 * TILE;
        const char* lV = lK + TILE;
        // S^T, dP^T tiles: rows = keys 16kt + 4g + r, col = the lane's query of sub-tile j
        f32x4 sc[NQ][4], dp[NQ][4];
#pragma unroll
        for (int kt = 0; kt < 4; ++kt) {
#pragma unroll
            for (int j = 0; j < NQ; ++j) { sc[j][kt] = (f32x4){0.f, 0.f, 0.f, 0.f}; dp[j][kt] = sc[j][kt]; }
#pragma unroll
            for (int kk = 0; kk < KSF; ++kk) {
                const bf16x8 kf = *(const bf16x8*)(lK + koff[kk] + kt * 16 * RB);
                const bf16x8 vf = *(const bf16x8*)(lV + koff[kk] + kt * 16 * RB);
#pragma unroll
                for (int j = 0; j < NQ; ++j) {
                    sc[j][kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[j][kk], sc[j][kt], 0, 0, 0);
                    dp[j][kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, df[j][kk], dp[j][kt], 0, 0, 0);
                }
            }
            if (HALF) {
                const bf16x4 kh = *(const bf16x4*)(lK + khoff + kt * 16 * RB);
                const bf16x4 vh = *(const bf16x4*)(lV + khoff + kt * 16 * RB);
#pragma unroll
                for (int j = 0; j < NQ; ++j) {
                    sc[j][kt] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(kh, qh[j], sc[j][kt], 0, 0, 0);
                    dp[j][kt] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(vh, dh[j], dp[j][kt], 0, 0, 0);
                }
            }
        }
        bf16x8 dsf[NQ][2];
#pragma unroll
        for (int j = 0; j < NQ; ++j) {
            const int qlo = qb * QBLK + wid * 16 * NQ + j * 16;   // first query of this sub-tile
            // masked scores -> -inf (P = 0) only on tiles crossing the diagonal or an edge
            if (qlo + 15 >= p.S || t * 64 + 63 >= p.S || (CAUSAL && t * 64 + 63 > qlo)) {
                asm volatile("" ::: "memory");   // keep the branch (no speculated compares)
#pragma unroll
                for (int kt = 0; kt < 4; ++kt)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int key = t * 64 + 16 * kt + 4 * g + r;
                        if (!qok[j] || key >= p.S || (CAUSAL && key > myq[j])) sc[j][kt][r] = -INFINITY;
                    }
            }
            const f32x2 sl2 = {p.scale_log2, p.scale_log2}, ls2 = {lse2[j], lse2[j]}, dl2 = {dl[j], dl[j]};
#pragma unroll
            for (int kt = 0; kt < 4; ++kt)
#pragma unroll
                for (int r = 0; r < 4; r += 2) {
                    const f32x2 x = f32x2{sc[j][kt][r], sc[j][kt][r + 1]} * sl2 - ls2;
                    const f32x2 pv = {__builtin_amdgcn_exp2f(x[0]), __builtin_amdgcn_exp2f(x[1])};
                    const f32x2 ds = pv * (f32x2{dp[j][kt][r], dp[j][kt][r + 1]} - dl2);
                    dp[j][kt][r] = ds[0]; dp[j][kt][r + 1] = ds[1];
                }
#pragma unroll
            for (int ks = 0; ks < 2; ++ks)
#pragma unroll
                for (int r = 0; r < 4; ++r) { dsf[j][ks][r] = (bf16)dp[j][2 * ks][r]; dsf[j][ks][4 + r] = (bf16)dp[j][2 * ks + 1][r]; }
        }
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            bf16x4 k0[DT], k1[DT];
#pragma unroll
            for (int d = 0; d < DT; ++d) {
                const uint32_t a = (uint32_t)(uintptr_t)lK + troff[d];
                if (ks == 0) { k0[d] = tr_read_off<0>(a); k1[d] = tr_read_off<16 * RB>(a); }
                else { k0[d] = tr_read_off<32 * RB>(a); k1[d] = tr_read_off<48 * RB>(a); }
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int d = 0; d < DT; ++d) {
                const bf16x8 kt8 = cat4(k0[d], k1[d]);
#pragma unroll
                for (int j = 0; j < NQ; ++j) acc[j][d] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kt8, dsf[j][ks], acc[j][d], 0, 0, 0);
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }
#pragma unroll
    for (int j = 0; j < NQ; ++j)
        if (qok[j]) {
            float* dQr = p.dq + ((int64_t)(b * p.H + h) * p.S + myq[j]) * HDP;
#pragma unroll
            for (int d = 0; d < DT; ++d) *(f32x4*)(dQr + d * 16 + 4 * g) = acc[j][d] * p.scale;
        }
}

// delta[b,h,q] = sum_d dO[b,q,h,d] * O[b,q,h,d]: one thread per (b, q, h) row, 16-B loads
// (hd % 8 == 0; every row load of both tensors in flight at once). One wave per row with
// a 2-B load per lane spent 38 us per call on 11 MB.
__global__ void k_attn_delta(const bf16* __restrict__ O, const bf16* __restrict__ dO, float* __restrict__ delta,
                             int B, int H, int S, int hd) {
    const int row = blockIdx.x * blockDim.x + threadIdx.x;
    if (row >= B * S * H) return;
    const int h = row % H, bq = row / H, q = bq % S, b = bq / S;
    const bf16* o = O + (int64_t)row * hd;
    const bf16* d = dO + (int64_t)row * hd;
    float acc = 0.f;
    for (int c = 0; c < hd; c += 8) {
        const bf16x8 a = *(const bf16x8*)(o + c), g = *(const bf16x8*)(d + c);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc += (float)a[e] * (float)g[e];
    }
    delta[((int64_t)b * H + h) * S + q] = acc;
}

}  // namespace

int launch_attn_fwd(const kd_attn_desc* d, void* stream_) {
    KD_CHECK_ARG(d && d->q && d->k && d->v && d->o, "attn_fwd: null pointer");
    KD_CHECK_SHAPE(d->B > 0 && d->S > 0 && d->H > 0 && d->HKV > 0 && d->H % d->HKV == 0, "attn_fwd: heads");
    KD_CHECK_SHAPE(d->hd > 0 && d->hd <= d->hdp && d->hd % 4 == 0, "attn_fwd: hd");
    KD_CHECK_SHAPE(d->hdp == 64 || d->hdp == 96 || d->hdp == 128, "attn_fwd: padded head dim must be 64/96/128");
    KD_CHECK_SHAPE(!(d->hdp == 96 && d->hd > 80) && !(d->hdp == 64 && d->hd > 64), "attn_fwd: hd exceeds tile cover");
    AttnP p{(const bf16*)d->q, (const bf16*)d->k, (const bf16*)d->v, (bf16*)d->o, d->lse,
            d->B, d->H, d->HKV, d->S, d->hd, (float)(1.4426950408889634 / std::sqrt((double)d->hd))};
    // NQ query sub-tiles per wave (KD_ATTN_FWD_NQ=1 restores one, for A/B)
    static const int nq = [] { const char* e = std::getenv("KD_ATTN_FWD_NQ"); return (e && e[0] == '1') ? 1 : 2; }();
    dim3 grid(d->H, d->B, (d->S + 64 * nq - 1) / (64 * nq));
    hipStream_t st = as_stream(stream_);
    const int rb = d->hdp == 64 ? 128 : 256;
    const size_t smem = 2 * 2 * 64 * rb;
#define LAUNCH(HD, C)                                                                                \
    do {                                                                                             \
        if (nq == 2) hipLaunchKernelGGL((k_attn_fwd<HD, C, 2>), grid, dim3(256), smem, st, p);       \
        else hipLaunchKernelGGL((k_attn_fwd<HD, C, 1>), grid, dim3(256), smem, st, p);               \
    } while (0)
    if (d->hdp == 64) { if (d->causal) LAUNCH(64, true); else LAUNCH(64, false); }
    else if (d->hdp == 96) { if (d->causal) LAUNCH(96, true); else LAUNCH(96, false); }
    else { if (d->causal) LAUNCH(128, true); else LAUNCH(128, false); }
#undef LAUNCH
    KD_LAUNCH_CHECK("k_attn_fwd");
    return KD_OK;
}

size_t attn_bwd_workspace_size(const kd_attn_bwd_desc* d) {
    if (!d || d->HKV <= 0 || d->H == d->HKV) return 0;
    return (size_t)2 * d->B * d->H * d->S * d->hdp * 4;
}

int launch_attn_bwd(const kd_attn_bwd_desc* d, void* stream_) {
    KD_CHECK_ARG(d && d->q && d->k && d->v && d->o && d->dO && d->lse && d->delta && d->dq && d->dk && d->dv,
                 "attn_bwd: null pointer");
    KD_CHECK_SHAPE(d->B > 0 && d->S > 0 && d->HKV > 0 && d->H % d->HKV == 0 && d->hd % 4 == 0 && d->hd <= d->hdp,
                   "attn_bwd: shape");
    KD_CHECK_SHAPE(d->hdp == 64 || d->hdp == 96 || d->hdp == 128, "attn_bwd: padded head dim must be 64/96/128");
    KD_CHECK_SHAPE(!(d->hdp == 96 && d->hd > 80) && !(d->hdp == 64 && d->hd > 64), "attn_bwd: hd exceeds tile cover");
    KD_CHECK_SHAPE(d->hd % 8 == 0, "attn_bwd: hd must be a multiple of 8 (16-B dO rows)");
    const size_t need = attn_bwd_workspace_size(d);
    if (need && (!d->workspace || d->workspace_bytes < need))
        return fail(KD_ERR_WORKSPACE, "attn_bwd: GQA needs kd_attn_bwd_workspace_size() bytes of workspace");
    hipStream_t st = as_stream(stream_);
    {
        const int rows = d->B * d->S * d->H;
        hipLaunchKernelGGL(k_attn_delta, dim3((rows + 255) / 256), dim3(256), 0, st, (const bf16*)d->o,
                           (const bf16*)d->dO, d->delta, d->B, d->H, d->S, d->hd);
        KD_LAUNCH_CHECK("k_attn_delta");
    }
    const double sc = 1.0 / std::sqrt((double)d->hd);
    float* dkp = need ? (float*)d->workspace : nullptr;
    float* dvp = need ? dkp + (size_t)d->B * d->H * d->S * d->hdp : nullptr;
    AttnBwdP p{(const bf16*)d->q, (const bf16*)d->k, (const bf16*)d->v, (const bf16*)d->dO, d->lse, d->delta,
               d->dq, (bf16*)d->dk, (bf16*)d->dv, dkp, dvp, d->B, d->H, d->HKV, d->S, d->hd, (float)sc,
               (float)(sc * 1.4426950408889634)};
    dim3 grid(d->H, d->B, (d->S + 63) / 64);
    static const int nq_dq = [] { const char* e = std::getenv("KD_ATTN_DQ_NQ"); return (e && e[0] == '1') ? 1 : 2; }();
    dim3 grid_q(d->H, d->B, (d->S + 64 * nq_dq - 1) / (64 * nq_dq));
    const int rb = d->hdp == 64 ? 128 : 256;
    const size_t smem_kv = 2 * (2 * 64 * rb + 512);
    const size_t smem_q = 2 * 2 * 64 * rb;
#define LAUNCH(HD, C)                                                                         \
    do {                                                                                      \
        hipLaunchKernelGGL((k_attn_bwd_dkdv<HD, C>), grid, dim3(256), smem_kv, st, p);       \
        KD_LAUNCH_CHECK("k_attn_bwd_dkdv");                                                   \
        if (nq_dq == 2) hipLaunchKernelGGL((k_attn_bwd_dq<HD, C, 2>), grid_q, dim3(256), smem_q, st, p); \
        else hipLaunchKernelGGL((k_attn_bwd_dq<HD, C, 1>), grid_q, dim3(256), smem_q, st, p);            \
        KD_LAUNCH_CHECK("k_attn_bwd_dq");                                                     \
    } while (0)
    if (d->hdp == 64) { if (d->causal) LAUNCH(64, true); else LAUNCH(64, false); }
    else if (d->hdp == 96) { if (d->causal) LAUNCH(96, true); else LAUNCH(96, false); }
    else { if (d->causal) LAUNCH(128, true); else LAUNCH(128, false); }
#undef LAUNCH
    if (need) {
        const int dcols = 16 * (d->hdp == 64 ? 4 : (d->hdp == 96 ? 5 : 8));
        const int64_t work = (int64_t)d->B * d->HKV * d->S * dcols / 4;
        hipLaunchKernelGGL(k_attn_group_sum, dim3((unsigned)std::min<int64_t>((work + 255) / 256, 8192)), dim3(256), 0, st,
                           dkp, dvp, (bf16*)d->dk, (bf16*)d->dv, d->B, d->H, d->HKV, d->S, d->hdp, dcols, (float)sc);
        KD_LAUNCH_CHECK("k_attn_group_sum");
    }
    return KD_OK;
}

}  // namespace kd
