// Flash attention forward / backward for gfx950 (bf16 MFMAs, fp32 softmax).
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
// Forward, default k_attn_fwd32 (per workgroup: 128 query rows of one head, 4 waves x 32
//   rows, 32x32x16 MFMAs): S^T = K Q^T so each lane pair (l, l ^ 32) owns ONE query's
//   scores; max / sum are lane-local plus one v_permlane32_swap, the O^T = V^T P^T
//   accumulator is lane-local per query, and the S accumulator registers ARE the B operand
//   of the PV MFMA (key order permuted consistently with the V^T fragment read by
//   ds_read_b64_tr_b16).  k_attn_fwd (16x16x32, 64 rows per workgroup) stays for A/B
//   (KD_ATTN_FWD_V=16).
// Backward: dK / dV per 128 keys of one kv head (k_attn_bwd_dkdv2: 4 waves x two 16-key
//   sub-tiles; head dim 128: k_attn_bwd_dkdv, 64 keys), looping over the group's query heads
//   and 32-row query tiles: S = Q K^T and dP = dO V^T with the key on the lane, so P / dS
//   registers feed dV^T += dO^T P and dK^T += Q^T dS directly.  dQ by its own kernel
//   (k_attn_bwd_dq: S and dP recomputed per query tile, no atomics).
#include "common.h"

#include <algorithm>
#include <cstdlib>
#include <utility>
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

// (h, b, z) of this workgroup in a grid (H, B, NZ) whose z is a query block.  The dispatcher deals
// workgroup L = x + H (y + B z) to XCD L % 8 (MI355X_MICROARCH: workgroup dispatch), so with the plain
// mapping the G = H / HKV query heads of one GQA group -- which read the SAME K / V tiles -- land on G
// different XCDs and every XCD's L2 fetches the group's K / V (rocprofv3 FETCH 4.9x q + k + v on the
// 7B teacher's causal forward, round 4).  Here the G heads of one (z, b, kv head) group run on one XCD
// at consecutive dispatch slots there (group grp -> XCD grp % 8), and the groups keep their z order
// per XCD (z = 0 first: the heaviest causal blocks).  Bijective whenever HKV B NZ % 8 == 0; else, and
// for MHA (G = 1), the plain mapping.
__device__ __forceinline__ void gqa_xcd_map(int H, int HKV, int B, int& h, int& b, int& z) {
    const int G = H / HKV, ngroups = HKV * B * (int)gridDim.z;
    if (G > 1 && (ngroups & 7) == 0) {
        const int L = (int)(blockIdx.x + H * (blockIdx.y + B * blockIdx.z));
        const int xcd = L & 7, slot = L >> 3;
        const int grp = (slot / G) * 8 + xcd;
        h = (grp % HKV) * G + slot % G;
        b = (grp / HKV) % B;
        z = grp / (HKV * B);
    } else {
        h = blockIdx.x; b = blockIdx.y; z = blockIdx.z;
    }
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

#ifdef KD_AB_BUILD   // the round-2 16x16x32 forward (forced variant 16): the tools' A/B library only
#include "attention_fwd16.inc"   // tools/ab/attention_fwd16.inc: the round-2 16x16x32 attention forward (forced variant 16)
#endif  // KD_AB_BUILD

// ------------------------------------------------------- forward, 32x32x16 MFMAs ----
// The 16x16x32 kernel above is bound by VECTOR ISSUE, not by the matrix pipe: a 16x16x32
// MFMA holds its SIMD's vector issue for 8 of its 16 cycles, so with ~170 softmax VALU per
// 64 MFMAs (32 exps at 8 cycles) a SIMD's two waves need ~2,700 issue cycles per 2,048 MFMA
// cycles (MFMA pipe ~35% busy, measured 25%). A 32x32x16 MFMA holds issue for 8 of its 32
// cycles: the same FLOPs leave 3x the issue slots for the softmax.
//   S^T (32 keys x 32 queries) = K Q^T: lane l owns query l & 31, keys 8(i>>2) + 4(l>>5) + (i&3)
//   in register i; two such tiles per 64-key tile = 32 scores per lane, the other 32 in lane
//   l ^ 32 (row max: one v_permlane32_swap). The accumulator IS the B operand of the PV
//   product (registers 8s'..8s'+7 -> k-step s' in the permuted key order), and the V^T A
//   operand is read in that same order by two ds_read_b64_tr_b16 per MFMA (keys 16s + 4h + q
//   and 16s + 8 + 4h + q). O^T (32 dims x 32 queries) keeps the query on the lane: the online
//   rescale stays lane-local.
// Per wave: 32 queries (4 waves = 128 rows per workgroup, as k_attn_fwd<.., NQ = 2>); per
// 64-key tile 16 QK^T + 16 PV MFMAs of 32 cycles (hd 128). Causal: a wave skips the MFMAs of
// tiles wholly above its diagonal (the workgroup still stages them for its other waves).

// V image swizzle for the 32x32x16 transposed reads: a 32-lane half reads 4 consecutive rows
// x 64 B; the XOR moves the 4 rows into 4 different 64-B bank blocks (256-B rows: chunk ^ 4(r&3);
// 128-B rows: rows r and r+2 share banks, chunk ^ 4((r>>1)&1))
template <int RB> __device__ __forceinline__ int swV32(int r) { return RB == 256 ? ((r & 3) << 2) : (((r >> 1) & 1) << 2); }

template <int HDP, bool VIMG>
__device__ __forceinline__ void stage_kv32(char* lds, const bf16* slab, int row0, int S, int wid, int lane) {
    constexpr int RB = Geo<HDP>::RB;
    constexpr int ROWS_PER = 1024 / RB, CH = RB / 16, NINSTR = 64 / ROWS_PER;
    const int rows_valid = min(64, S - row0);
    auto rs = rsrc(slab + (int64_t)row0 * HDP, rows_valid <= 0 ? 0u : (uint32_t)(rows_valid * HDP * 2));
#pragma unroll
    for (int s = 0; s < NINSTR / 4; ++s) {
        const int i = wid * (NINSTR / 4) + s;
        const int r = i * ROWS_PER + lane / CH;
        const int c = lane % CH;
        const int gc = c ^ (VIMG ? swV32<RB>(r) : swK<RB>(r));
        const uint32_t voff = (gc * 8 < HDP) ? (uint32_t)((r * HDP + gc * 8) * 2) : OOB;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void_t*)(lds + i * 1024), 16, voff, 0, 0, 0);
    }
}

typedef __attribute__((ext_vector_type(16))) float f32x16;

__device__ __forceinline__ bf16x8 cat4(bf16x4 a, bf16x4 b) {
    bf16x8 r;
    r[0] = a[0]; r[1] = a[1]; r[2] = a[2]; r[3] = a[3];
    r[4] = b[0]; r[5] = b[1]; r[6] = b[2]; r[7] = b[3];
    return r;
}


// v of lanes l & 31 and (l & 31) + 32 in every lane (one v_permlane32_swap): max / sum over the
// two halves, in the same operand order in both (bit-identical results)
__device__ __forceinline__ float half_max(float v) {
    auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
// s_waitcnt lgkmcnt(N) that names the 8 asm-read registers it retires ("+v": the compiler can
// neither read them before the wait nor place a copy of them above it)
template <int N> __device__ __forceinline__ void wait_lgkm_def8(u32x2 (&r)[8]) {
    asm volatile("s_waitcnt lgkmcnt(%8)" : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]),
                 "+v"(r[6]), "+v"(r[7]) : "i"(N) : "memory");
}
__device__ __forceinline__ float half_sum(float v) {
    auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// Register staging of one 64-row K or V tile (RS build of k_attn_fwd32): the attention guide
// measures LDS-DMA pieces at 100-185 issue cycles each inside a phase that also reads LDS, and
// a wave-tile here issues 8 of them (as many cycles as its 32 MFMAs); a buffer load to VGPRs
// plus a ds_write_b128 costs a fraction of that. Piece pi (1 KiB) = rows [pi R, pi R + R),
// R = 1024 / RB; lane -> row pi R + lane / CH, logical 16-B chunk lane % CH, written to the
// swizzled LDS position. Rows >= S and chunks past HDP load as zeros (buffer range check).
template <int HDP> struct Stage {
    static constexpr int RB = Geo<HDP>::RB, R = 1024 / RB, CH = RB / 16, NL = 64 / R / 4;   // pieces per wave
    uint32_t goff;         // per-lane global byte offset inside a piece (OOB past HDP)
    uint32_t kw[NL], vw;   // per-lane LDS byte offsets of the K pieces (swK depends on the piece) and V
    __device__ __forceinline__ void init(int wid, int lane) {
        const int c = lane % CH, rr = lane / CH;
        goff = (c * 8 < HDP) ? (uint32_t)((rr * HDP + c * 8) * 2) : OOB;
#pragma unroll
        for (int i = 0; i < NL; ++i) {
            const int r = (wid * NL + i) * R + rr;
            kw[i] = (uint32_t)(r * RB + ((c ^ swK<RB>(r)) << 4));
        }
        const int r0 = wid * NL * R + rr;   // swV32 is the same for every piece of the wave
        vw = (uint32_t)(r0 * RB + ((c ^ swV32<RB>(r0)) << 4));
    }
    __device__ __forceinline__ void load(u32x4 (&st)[NL], const bf16* slab, int row0, int S, int wid) const {
        const int rows_valid = min(64, S - row0);
        const auto rs = rsrc(slab + (int64_t)row0 * HDP, rows_valid <= 0 ? 0u : (uint32_t)(rows_valid * HDP * 2));
#pragma unroll
        for (int i = 0; i < NL; ++i)
            st[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, goff, (wid * NL + i) * R * HDP * 2, 0));
    }
    __device__ __forceinline__ void write_k(char* lds, const u32x4 (&st)[NL]) const {
#pragma unroll
        for (int i = 0; i < NL; ++i) *(u32x4*)(lds + kw[i]) = st[i];
    }
    __device__ __forceinline__ void write_v(char* lds, const u32x4 (&st)[NL]) const {
#pragma unroll
        for (int i = 0; i < NL; ++i) *(u32x4*)(lds + vw + i * 1024) = st[i];
    }
};

// ST (diagnostic build, KD_ATTN_FWD_V=34, tools/stamp_attn.py): per-wave s_memtime totals
// (prologue, tile compute, end-of-tile wait + barrier, epilogue, whole wave, tiles computed)
// written as uint32 over the wave's own first Q row after its Q fragments are loaded (the
// tool passes a scratch Q; nothing else reads that row: Q rows belong to one workgroup)
// NW waves per workgroup (query block of 32 NW rows; NW = 6 forced variant 36 / the host's choice
// where it balances the grid better: SigLIP's 729 queries are 4 blocks of 192 (512 workgroups, one
// round on 256 CUs x 2) instead of 6 blocks of 128 (768: a second, half-empty round).  Waves 4 and 5
// stage nothing (the K/V DMA stays on waves 0-3); three waves per SIMD: <= 168 VGPRs.
template <int HDP, bool CAUSAL, bool RS, bool ST = false, int NW = 4>
__global__ void __launch_bounds__(64 * NW, NW == 4 ? 2 : 3) k_attn_fwd32(AttnP p) {
    static_assert(NW == 4 || (NW == 6 && !RS && !ST), "k_attn_fwd32: 6 waves only for the LDS-DMA build");
    constexpr int QB = 32 * NW;   // query rows per workgroup
    uint64_t st_t0 = 0, st_pro = 0, st_cmp = 0, st_bar = 0, st_prev = 0;
    int st_n = 0;
    uint64_t st_r0 = 0;
    if (ST) { st_t0 = __builtin_amdgcn_s_memtime(); st_r0 = __builtin_amdgcn_s_memrealtime(); }
    constexpr int RB = Geo<HDP>::RB;
    constexpr int TILE = 64 * RB;
    constexpr int KS = HDP == 96 ? 5 : HDP / 16;               // 16-deep QK^T steps (hd <= 16 KS)
    constexpr int ND = HDP == 64 ? 2 : (HDP == 96 ? 3 : 4);    // 32-dim O^T tiles
    extern __shared__ __attribute__((aligned(16))) char smem[];  // [2][K TILE | V TILE]
    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int r32 = lane & 31, hf = lane >> 5;
    const int nqb = (p.S + QB - 1) / QB;
    int h, b, zb;
    gqa_xcd_map(p.H, p.HKV, p.B, h, b, zb);
    const int qb = CAUSAL ? (nqb - 1 - zb) : zb;
    const int kvh = h / (p.H / p.HKV);
    const bf16* Q = p.q + ((int64_t)(b * p.H + h) * p.S) * HDP;
    const bf16* K = p.k + ((int64_t)(b * p.HKV + kvh) * p.S) * HDP;
    const bf16* V = p.v + ((int64_t)(b * p.HKV + kvh) * p.S) * HDP;
    const int q0 = qb * QB + wid * 32;   // the wave's first query (uniform)
    const bool stager = NW == 4 || wid < 4;   // the waves that issue the K/V LDS-DMA
    const int myq = q0 + r32;

    bf16x8 qf[KS];
#pragma unroll
    for (int kk = 0; kk < KS; ++kk)
        qf[kk] = myq < p.S ? *(const bf16x8*)(Q + (int64_t)myq * HDP + kk * 16 + 8 * hf) : (bf16x8){};
    f32x16 o[ND];
#pragma unroll
    for (int d = 0; d < ND; ++d)
#pragma unroll
        for (int i = 0; i < 16; ++i) o[d][i] = 0.f;
    float m = -INFINITY, l = 0.f;

    const int nkv_all = (p.S + 63) / 64;
    const int nkv = CAUSAL ? min(((qb + 1) * QB + 63) / 64, nkv_all) : nkv_all;
    const int nkv_w = CAUSAL ? min(nkv, (q0 + 31) / 64 + 1) : nkv;   // tiles with a key <= the wave's last query
    Stage<HDP> stg;
    u32x4 stk[Stage<HDP>::NL], stv[Stage<HDP>::NL];
    if (RS) {
        stg.init(wid, lane);
        stg.load(stk, K, 0, p.S, wid);
        stg.load(stv, V, 0, p.S, wid);
        stg.write_k(smem, stk);
        stg.write_v(smem + TILE, stv);
    } else if (stager) {
        stage_kv32<HDP, false>(smem, K, 0, p.S, wid, lane);
        stage_kv32<HDP, true>(smem + TILE, V, 0, p.S, wid, lane);
    }
    // per-lane LDS byte offsets; buffer, 32-key sub-tile and 16-key step are immediates
    uint32_t koff[KS];
#pragma unroll
    for (int kk = 0; kk < KS; ++kk)
        koff[kk] = (uint32_t)(uintptr_t)smem + r32 * RB + (((2 * kk + hf) ^ swK<RB>(r32)) << 4);
    uint32_t vaddr[ND];
    {
        const uint32_t sbase = (uint32_t)(uintptr_t)smem;
        const int row = 4 * hf + ((lane >> 2) & 3);
#pragma unroll
        for (int d = 0; d < ND; ++d) {
            const int col = 32 * d + 16 * ((lane >> 4) & 1) + 4 * (lane & 3);
            vaddr[d] = sbase + TILE + row * RB + ((((col >> 3) ^ swV32<RB>(row))) << 4) + ((col & 4) << 1);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (ST) { st_prev = __builtin_amdgcn_s_memtime(); st_pro = st_prev - st_t0; }

    auto tile = [&](const int t, auto buf_c) {
        constexpr int BUF = decltype(buf_c)::value;
        if (t + 1 < nkv) {
            if (RS) {   // loads now, LDS writes after this tile's reads (buffer BUF ^ 1 is free:
                        // every wave passed the barrier that ended tile t - 1, its last reader)
                stg.load(stk, K, (t + 1) * 64, p.S, wid);
                stg.load(stv, V, (t + 1) * 64, p.S, wid);
            } else if (stager) {
                char* nb = smem + (BUF ^ 1) * 2 * TILE;
                stage_kv32<HDP, false>(nb, K, (t + 1) * 64, p.S, wid, lane);
                stage_kv32<HDP, true>(nb + TILE, V, (t + 1) * 64, p.S, wid, lane);
            }
        }
        if (t < nkv_w) {
            // S^T = K Q^T: the K fragments by asm ds_read_b128 with counted waits (the builtin
            // loads were each waited for right before their MFMA: the compiler reused one
            // register set). Sub-tile 0's reads go out first; each of sub-tile 1's reads is
            // issued after the MFMA that frees its registers' counterpart.
            f32x16 sc[2];
#pragma unroll
            for (int kt = 0; kt < 2; ++kt)
#pragma unroll
                for (int i = 0; i < 16; ++i) sc[kt][i] = 0.f;
            u32x4 ka[KS], kb[KS];
#pragma unroll
            for (int kk = 0; kk < KS; ++kk)
                asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(ka[kk]) : "v"(koff[kk]), "i"(BUF * 2 * TILE));
#pragma unroll
            for (int kk = 0; kk < KS; ++kk) {
                // the counted wait names the register it retires (ka[kk], the oldest read in
                // flight), so no compiler copy of it can be placed before the wait
                asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(ka[kk]) : "i"(KS - 1) : "memory");
                __builtin_amdgcn_sched_barrier(0);
                sc[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, ka[kk]), qf[kk], sc[0], 0, 0, 0);
                __builtin_amdgcn_sched_barrier(0);
                asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(kb[kk]) : "v"(koff[kk]), "i"(BUF * 2 * TILE + 32 * RB));
            }
#pragma unroll
            for (int kk = 0; kk < KS; ++kk) {
                asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(kb[kk]) : "i"(KS - 1 - kk) : "memory");
                __builtin_amdgcn_sched_barrier(0);
                sc[1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, kb[kk]), qf[kk], sc[1], 0, 0, 0);
            }
            __builtin_amdgcn_sched_barrier(0);
            // mask only on tiles that cross the diagonal or the sequence end (uniform test)
            if (t * 64 + 63 >= p.S || (CAUSAL && t * 64 + 63 > q0)) {
#pragma unroll
                for (int kt = 0; kt < 2; ++kt)
#pragma unroll
                    for (int i = 0; i < 16; ++i) {
                        const int key = t * 64 + 32 * kt + 8 * (i >> 2) + 4 * hf + (i & 3);
                        if (key >= p.S || (CAUSAL && key > myq)) sc[kt][i] = -INFINITY;
                    }
            }
            float mt = -INFINITY;
#pragma unroll
            for (int kt = 0; kt < 2; ++kt)
#pragma unroll
                for (int i = 0; i < 16; ++i) mt = fmaxf(mt, sc[kt][i]);
            mt = half_max(mt);
            // online softmax in the log2 domain with the lazy rescale of k_attn_fwd (the
            // reference max moves only when the tile's max exceeds it by more than 8)
            const float mts = mt * p.scale_log2;
            const bool move = mts > m + 8.f;
            if (__ballot(move)) {
                const float mn = move ? mts : m;
                const float alpha = __builtin_amdgcn_exp2f(m - mn);
                l *= alpha;
#pragma unroll
                for (int d = 0; d < ND; ++d) o[d] *= alpha;
                m = mn;
            }
            const float mref = (m == -INFINITY) ? 0.f : m;
            float ls[4] = {0.f, 0.f, 0.f, 0.f};   // four independent add chains
#pragma unroll
            for (int kt = 0; kt < 2; ++kt)
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    const float e = __builtin_amdgcn_exp2f(fmaf(sc[kt][i], p.scale_log2, -mref));
                    sc[kt][i] = e;
                    ls[i & 3] += e;
                }
            l += (ls[0] + ls[1]) + (ls[2] + ls[3]);
            bf16x8 pf[4];
#pragma unroll
            for (int s = 0; s < 4; ++s)
#pragma unroll
                for (int j = 0; j < 8; ++j) pf[s][j] = (bf16)sc[s >> 1][8 * (s & 1) + j];
            // O^T += V^T P^T: per 32-dim tile 8 transposed reads (4 key steps x 2 halves), the
            // next tile's reads in flight while this one's MFMAs run
            u32x2 vr[2][8];
#define KD_F32_RD(D, SET)                                                                                        \
    _Pragma("unroll") for (int s = 0; s < 4; ++s) {                                                              \
        asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(vr[SET][2 * s]) : "v"(vaddr[D]), "i"(BUF * 2 * TILE + (16 * s) * RB));     \
        asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(vr[SET][2 * s + 1]) : "v"(vaddr[D]), "i"(BUF * 2 * TILE + (16 * s + 8) * RB)); \
    }
#define KD_F32_MM(D, SET)                                                                                        \
    _Pragma("unroll") for (int s = 0; s < 4; ++s) {                                                              \
        const bf16x8 vf = cat4(__builtin_bit_cast(bf16x4, vr[SET][2 * s]), __builtin_bit_cast(bf16x4, vr[SET][2 * s + 1])); \
        o[D] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pf[s], o[D], 0, 0, 0);                                 \
    }
// the counted wait retires the 8 reads of vr[SET] (the older set in flight) and names them
#define KD_F32_WAIT(N, SET) wait_lgkm_def8<N>(vr[SET]); __builtin_amdgcn_sched_barrier(0);
            KD_F32_RD(0, 0)
            KD_F32_RD(1, 1)
            KD_F32_WAIT(8, 0)
            KD_F32_MM(0, 0)
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (ND > 2) { KD_F32_RD(2, 0) KD_F32_WAIT(8, 1) }
            else { KD_F32_WAIT(0, 1) }
            KD_F32_MM(1, 1)
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (ND > 2) {
                if constexpr (ND > 3) { KD_F32_RD(3, 1) KD_F32_WAIT(8, 0) }
                else { KD_F32_WAIT(0, 0) }
                KD_F32_MM(2, 0)
                __builtin_amdgcn_sched_barrier(0);
                if constexpr (ND > 3) {
                    KD_F32_WAIT(0, 1)
                    KD_F32_MM(3, 1)
                }
            }
#undef KD_F32_RD
#undef KD_F32_MM
#undef KD_F32_WAIT
        }
        if (RS && t + 1 < nkv) {
            char* nb = smem + (BUF ^ 1) * 2 * TILE;
            stg.write_k(nb, stk);
            stg.write_v(nb + TILE, stv);
        }
        uint64_t ta = 0;
        if (ST) { ta = __builtin_amdgcn_s_memtime(); st_cmp += ta - st_prev; st_n += t < nkv_w; }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (ST) { st_prev = __builtin_amdgcn_s_memtime(); st_bar += st_prev - ta; }
    };
    int t = 0;
    for (; t + 1 < nkv; t += 2) {
        tile(t, std::integral_constant<int, 0>{});
        tile(t + 1, std::integral_constant<int, 1>{});
    }
    if (t < nkv) tile(t, std::integral_constant<int, 0>{});
    l = half_sum(l);
    if (ST) {
        const uint64_t te = __builtin_amdgcn_s_memtime();
        if (lane == 0) {
            uint32_t* w = (uint32_t*)(const_cast<bf16*>(Q) + (int64_t)q0 * HDP);
            w[0] = (uint32_t)st_pro; w[1] = (uint32_t)st_cmp; w[2] = (uint32_t)st_bar;
            w[3] = (uint32_t)(te - st_prev); w[4] = (uint32_t)(te - st_t0); w[5] = (uint32_t)st_n; w[6] = (uint32_t)nkv;
            w[7] = (uint32_t)(__builtin_amdgcn_s_memrealtime() - st_r0);   // 100 MHz ticks
        }
    }
    if (myq < p.S) {
        const float inv = 1.f / l;
        bf16* orow = p.o + (((int64_t)b * p.S + myq) * p.H + h) * p.hd;
#pragma unroll
        for (int d = 0; d < ND; ++d)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int dd = 32 * d + 8 * g + 4 * hf;
                if (dd < p.hd) {
                    bf16x4 w;
#pragma unroll
                    for (int r = 0; r < 4; ++r) w[r] = (bf16)(o[d][4 * g + r] * inv);
                    *(bf16x4*)(orow + dd) = w;
                }
            }
        if (hf == 0 && p.lse) p.lse[((int64_t)b * p.H + h) * p.S + myq] = (m + log2f(l)) * 0.6931471805599453f;
    }
}

#ifdef KD_AB_BUILD   // k_attn_fwd64 / k_attn_fwd32p: measured slower; A/B library only
#include "attention_fwd64_fwd32p.inc"   // tools/ab/attention_fwd64_fwd32p.inc: k_attn_fwd64 / k_attn_fwd32p and the other forward / backward A/B variants
#endif  // KD_AB_BUILD

// ------------------------------------------------------------------ backward ----
struct AttnBwdP {
    const bf16* q; const bf16* k; const bf16* v;   // [B, heads, S, HDP]
    const bf16* dO;                                  // [B, S, H, hd]
    const bf16* o;                                   // [B, S, H, hd] (k_attn_bwd_dq computes delta from it)
    const float* lse; float* delta;                 // [B, H, S] (delta: written by k_attn_bwd_dq)
    float* dq;                                      // [B, H, S, HDP] fp32 (scaled)
    bf16* dk; bf16* dv;                             // [B, HKV, S, HDP]
    float* dkp; float* dvp;                         // GQA partials [B, H, S, HDP] fp32 (grp > 1)
    int B, H, HKV, S, hd;
    float scale, scale_log2;
    // optional token-major [B*S, (H + 2 HKV) hd] bf16 output (kd_qkv_merge's layout, no RoPE; MHA):
    // dq | dk | dv written there directly instead of dq / dk / dv
    bf16* dqkv; int64_t ld_qkv;
    const float *rcos, *rsin;   // with dqkv: RoPE tables [S, hd/2] -> dq and dk rotated back (k_qkv_merge's transpose)
};

// this lane's 4 consecutive columns [dd, dd + 4) of head `head` at token (b, s) in the merged
// dqkv row (columns past hd are head-dim padding: not written)
__device__ __forceinline__ void put_qkv4(const AttnBwdP& p, int b, int s, int head, int dd, const bf16x4& w) {
    if (dd < p.hd) *(bf16x4*)(p.dqkv + ((int64_t)b * p.S + s) * p.ld_qkv + (int64_t)head * p.hd + dd) = w;
}

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
                if (p.dqkv) {
                    put_qkv4(p, b, mykey, p.H + kvh, dd, wk);
                    put_qkv4(p, b, mykey, p.H + p.HKV + kvh, dd, wv);
                } else {
                    *(bf16x4*)(dKr + dd) = wk;
                    *(bf16x4*)(dVr + dd) = wv;
                }
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

// k_attn_bwd_dkdv with TWO 16-key sub-tiles per wave (4 waves x 32 keys = 128 keys per
// workgroup): every Q / dO row fragment and every transposed dO^T / Q^T read from LDS feeds
// both sub-tiles' MFMAs. With one 16-key sub-tile a wave moves ~1 KiB of LDS per MFMA
// (SigLIP: 44 KiB of fragment reads per 44 MFMAs per query tile, the CU's 256 B/clk at the
// full MFMA rate): the kernel was LDS-bound at ~0.15 of peak. The 64-row query tile is taken
// in two 32-row halves so the S / dP registers do not double. Same arithmetic per element as
// k_attn_bwd_dkdv (bit-identical outputs).
template <int HDP, bool CAUSAL>
__global__ void __launch_bounds__(256, 2) k_attn_bwd_dkdv2(AttnBwdP p) {
    constexpr int RB = Geo<HDP>::RB, KS = Geo<HDP>::KSTEPS, DT = Geo<HDP>::DT;
    constexpr int TILE = 64 * RB, BUF = 2 * TILE + 512;
    constexpr bool HALF = HDP == 96;
    constexpr int KSF = HALF ? KS - 1 : KS;
    extern __shared__ __attribute__((aligned(16))) char smem[];   // [2][Q TILE | dO TILE | lse2 64 | delta 64]
    const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int g = lane >> 4, li = lane & 15;
    const int kb0 = blockIdx.z * 128;
    const int h = blockIdx.x, b = blockIdx.y;
    const int grp = p.H / p.HKV, kvh = h / grp;
    const bf16* K = p.k + ((int64_t)(b * p.HKV + kvh) * p.S) * HDP;
    const bf16* V = p.v + ((int64_t)(b * p.HKV + kvh) * p.S) * HDP;
    const bf16* Q = p.q + ((int64_t)(b * p.H + h) * p.S) * HDP;
    const bf16* dO = p.dO + ((int64_t)b * p.S * p.H + h) * p.hd;
    const float* LSE = p.lse + ((int64_t)b * p.H + h) * p.S;
    const float* DEL = p.delta + ((int64_t)b * p.H + h) * p.S;
    const int64_t ldo = (int64_t)p.H * p.hd;
    const int kw0 = kb0 + wid * 32;   // the wave's first key (uniform)
    int mykey[2];
    bf16x8 kf[2][KS], vf[2][KS];
    bf16x4 kh[2], vh[2];
#pragma unroll
    for (int c = 0; c < 2; ++c) {
        mykey[c] = kw0 + 16 * c + li;
        kh[c] = (bf16x4){}; vh[c] = (bf16x4){};
#pragma unroll
        for (int kk = 0; kk < KSF; ++kk) {
            if (mykey[c] < p.S) {
                kf[c][kk] = *(const bf16x8*)(K + (int64_t)mykey[c] * HDP + kk * 32 + 8 * g);
                vf[c][kk] = *(const bf16x8*)(V + (int64_t)mykey[c] * HDP + kk * 32 + 8 * g);
            } else {
                kf[c][kk] = (bf16x8){}; vf[c][kk] = (bf16x8){};
            }
        }
        if (HALF && mykey[c] < p.S) {
            kh[c] = *(const bf16x4*)(K + (int64_t)mykey[c] * HDP + KSF * 32 + 4 * g);
            vh[c] = *(const bf16x4*)(V + (int64_t)mykey[c] * HDP + KSF * 32 + 4 * g);
        }
    }
    f32x4 dk[2][DT], dv[2][DT];
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int d = 0; d < DT; ++d) { dk[c][d] = (f32x4){0.f, 0.f, 0.f, 0.f}; dv[c][d] = dk[c][d]; }

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
    const int qt0 = CAUSAL ? kb0 / 64 : 0;
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
        const uint32_t bq = (uint32_t)(uintptr_t)lQ;
        // a 32-row half with no query at or past any of this wave's keys contributes nothing
        // (causal: every P is 0); skip its MFMAs (uniform)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            const int qh0 = q0 + 32 * ks;
            // no key of this wave (past the sequence end) or no query at or past one (causal): P = 0
            if (kw0 >= p.S || (CAUSAL && qh0 + 31 < kw0)) continue;
            // S, dP for query rows qh0 + 16qs' + 4g + r (qs' = 0, 1) and both key sub-tiles
            f32x4 s[2][2], dp[2][2];
#pragma unroll
            for (int qq = 0; qq < 2; ++qq) {
                const int qs = 2 * ks + qq;
#pragma unroll
                for (int c = 0; c < 2; ++c) { s[c][qq] = (f32x4){0.f, 0.f, 0.f, 0.f}; dp[c][qq] = s[c][qq]; }
#pragma unroll
                for (int kk = 0; kk < KSF; ++kk) {
                    const bf16x8 qa = *(const bf16x8*)(lQ + qoff[kk] + qs * 16 * RB);
                    const bf16x8 oa = *(const bf16x8*)(lO + qoff[kk] + qs * 16 * RB);
#pragma unroll
                    for (int c = 0; c < 2; ++c) {
                        s[c][qq] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qa, kf[c][kk], s[c][qq], 0, 0, 0);
                        dp[c][qq] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(oa, vf[c][kk], dp[c][qq], 0, 0, 0);
                    }
                }
                if (HALF) {
                    const bf16x4 qa = *(const bf16x4*)(lQ + qhoff + qs * 16 * RB);
                    const bf16x4 oa = *(const bf16x4*)(lO + qhoff + qs * 16 * RB);
#pragma unroll
                    for (int c = 0; c < 2; ++c) {
                        s[c][qq] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(qa, kh[c], s[c][qq], 0, 0, 0);
                        dp[c][qq] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(oa, vh[c], dp[c][qq], 0, 0, 0);
                    }
                }
            }
            if (qh0 + 31 >= p.S || kw0 + 31 >= p.S || (CAUSAL && kw0 + 31 > qh0)) {
                asm volatile("" ::: "memory");
#pragma unroll
                for (int c = 0; c < 2; ++c)
#pragma unroll
                    for (int qq = 0; qq < 2; ++qq)
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            const int q = qh0 + 16 * qq + 4 * g + r;
                            if (q >= p.S || mykey[c] >= p.S || (CAUSAL && mykey[c] > q)) s[c][qq][r] = -INFINITY;
                        }
            }
            const f32x2 sl2 = {p.scale_log2, p.scale_log2};
            bf16x8 pfr[2], dsf[2];
#pragma unroll
            for (int qq = 0; qq < 2; ++qq) {
                const int qs = 2 * ks + qq;
                const f32x4 l2 = *(const f32x4*)(lL + 16 * qs + 4 * g), dl = *(const f32x4*)(lD + 16 * qs + 4 * g);
#pragma unroll
                for (int c = 0; c < 2; ++c)
#pragma unroll
                    for (int r = 0; r < 4; r += 2) {
                        const f32x2 x = f32x2{s[c][qq][r], s[c][qq][r + 1]} * sl2 - f32x2{l2[r], l2[r + 1]};
                        const f32x2 pv = {__builtin_amdgcn_exp2f(x[0]), __builtin_amdgcn_exp2f(x[1])};
                        const f32x2 ds = pv * (f32x2{dp[c][qq][r], dp[c][qq][r + 1]} - f32x2{dl[r], dl[r + 1]});
                        pfr[c][4 * qq + r] = (bf16)pv[0]; pfr[c][4 * qq + r + 1] = (bf16)pv[1];
                        dsf[c][4 * qq + r] = (bf16)ds[0]; dsf[c][4 * qq + r + 1] = (bf16)ds[1];
                    }
            }
            // dV^T += dO^T P ; dK^T += Q^T dS: each transposed read feeds both key sub-tiles
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
                const bf16x8 ov = cat4(o0[d], o1[d]), xv = cat4(x0[d], x1[d]);
#pragma unroll
                for (int c = 0; c < 2; ++c) {
                    dv[c][d] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ov, pfr[c], dv[c][d], 0, 0, 0);
                    dk[c][d] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xv, dsf[c], dk[c][d], 0, 0, 0);
                }
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (qt + 1 < nqt) put_lse(smem + (cur ^ 1) * BUF);
        __syncthreads();
    }
#pragma unroll
    for (int c = 0; c < 2; ++c) {
        if (mykey[c] >= p.S) continue;
        if (grp == 1) {
            bf16* dKr = p.dk + ((int64_t)(b * p.HKV + kvh) * p.S + mykey[c]) * HDP;
            bf16* dVr = p.dv + ((int64_t)(b * p.HKV + kvh) * p.S + mykey[c]) * HDP;
#pragma unroll
            for (int d = 0; d < DT; ++d) {
                const int dd = d * 16 + 4 * g;
                bf16x4 wk, wv;
#pragma unroll
                for (int r = 0; r < 4; ++r) { wk[r] = (bf16)(dk[c][d][r] * p.scale); wv[r] = (bf16)dv[c][d][r]; }
                if (p.dqkv) {
                    put_qkv4(p, b, mykey[c], p.H + kvh, dd, wk);
                    put_qkv4(p, b, mykey[c], p.H + p.HKV + kvh, dd, wv);
                } else {
                    *(bf16x4*)(dKr + dd) = wk;
                    *(bf16x4*)(dVr + dd) = wv;
                }
            }
        } else {
            float* dKr = p.dkp + ((int64_t)(b * p.H + h) * p.S + mykey[c]) * HDP;
            float* dVr = p.dvp + ((int64_t)(b * p.H + h) * p.S + mykey[c]) * HDP;
#pragma unroll
            for (int d = 0; d < DT; ++d) {
                const int dd = d * 16 + 4 * g;
                *(f32x4*)(dKr + dd) = dk[c][d];
                *(f32x4*)(dVr + dd) = dv[c][d];
            }
        }
    }
}

// The GQA group sum written straight into the fused q|k|v gradient row (kd_attn_bwd_desc.dqkv): one
// thread per 4-column chunk pair (c, c + hd/2) of a (b, kvh, s) row, dk and dv rounded to bf16 exactly
// as k_attn_group_sum does, then dk rotated back (RoPE tables; k_qkv_merge's arithmetic on those bf16
// values) -- bit-identical to k_attn_group_sum + k_qkv_merge.
__global__ void k_attn_group_sum_qkv(const float* __restrict__ dkp, const float* __restrict__ dvp, bf16* __restrict__ dqkv,
                                     int64_t ld, const float* __restrict__ rcos, const float* __restrict__ rsin, int B,
                                     int H, int HKV, int S, int hd, int hdp, float scale) {
    const int grp = H / HKV, hh = hd / 2, c4 = hh / 4;
    const int64_t total = (int64_t)B * HKV * S * c4;
    for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total; idx += (int64_t)gridDim.x * blockDim.x) {
        const int c = (int)(idx % c4) * 4;
        const int64_t rs = idx / c4;               // (b, kvh, s)
        const int s = (int)(rs % S);
        const int64_t bk = rs / S;
        const int kvh = (int)(bk % HKV), b = (int)(bk / HKV);
        f32x4 ak1 = (f32x4){0.f, 0.f, 0.f, 0.f}, av1 = ak1, ak2 = ak1, av2 = ak1;
        for (int j = 0; j < grp; ++j) {
            const int64_t off = (((int64_t)b * H + kvh * grp + j) * S + s) * hdp + c;
            ak1 += *(const f32x4*)(dkp + off);
            av1 += *(const f32x4*)(dvp + off);
            ak2 += *(const f32x4*)(dkp + off + hh);
            av2 += *(const f32x4*)(dvp + off + hh);
        }
        bf16x4 k1, k2, v1, v2;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            k1[r] = (bf16)(ak1[r] * scale); k2[r] = (bf16)(ak2[r] * scale);
            v1[r] = (bf16)av1[r]; v2[r] = (bf16)av2[r];
        }
        if (rcos) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                float y1, y2;
                rope_t((float)k1[r], (float)k2[r], rcos[(int64_t)s * hh + c + r], rsin[(int64_t)s * hh + c + r], y1, y2);
                k1[r] = (bf16)y1; k2[r] = (bf16)y2;
            }
        }
        bf16* row = dqkv + ((int64_t)b * S + s) * ld;
        bf16* kr = row + (int64_t)(H + kvh) * hd;
        bf16* vr = row + (int64_t)(H + HKV + kvh) * hd;
        *(bf16x4*)(kr + c) = k1;
        *(bf16x4*)(kr + c + hh) = k2;
        *(bf16x4*)(vr + c) = v1;
        *(bf16x4*)(vr + c + hh) = v2;
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
    int h, b, zb;
    gqa_xcd_map(p.H, p.HKV, p.B, h, b, zb);
    const int qb = CAUSAL ? (nqb - 1 - zb) : zb;
    const int kvh = h / (p.H / p.HKV);
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
        const int64_t orow = (((int64_t)b * p.S + myq[j]) * p.H + h) * p.hd;
        const bf16* dOr = p.dO + orow;
        const bf16* Or = p.o + orow;
        // delta = rowsum(dO * O) (the softmax backward's row constant), fused here: the lane's dO
        // chunks (the dP operand) times the same chunks of O, summed over the 4 lanes of the row
        float dsum = 0.f;
#pragma unroll
        for (int kk = 0; kk < KSF; ++kk) {
            const int d0 = kk * 32 + 8 * g;
            qf[j][kk] = qok[j] ? *(const bf16x8*)(Q + (int64_t)myq[j] * HDP + d0) : (bf16x8){};
            df[j][kk] = (qok[j] && d0 < p.hd) ? *(const bf16x8*)(dOr + d0) : (bf16x8){};
            const bf16x8 of = (qok[j] && d0 < p.hd) ? *(const bf16x8*)(Or + d0) : (bf16x8){};
#pragma unroll
            for (int e = 0; e < 8; ++e) dsum = __builtin_fmaf((float)df[j][kk][e], (float)of[e], dsum);
        }
        if (HALF) {   // dims 32 KSF + 4g + [0, 4); dO rows hold hd (a multiple of 4) columns
            const int d0 = KSF * 32 + 4 * g;
            qh[j] = qok[j] ? *(const bf16x4*)(Q + (int64_t)myq[j] * HDP + d0) : (bf16x4){};
            dh[j] = (qok[j] && d0 < p.hd) ? *(const bf16x4*)(dOr + d0) : (bf16x4){};
            const bf16x4 oh = (qok[j] && d0 < p.hd) ? *(const bf16x4*)(Or + d0) : (bf16x4){};
#pragma unroll
            for (int e = 0; e < 4; ++e) dsum = __builtin_fmaf((float)dh[j][e], (float)oh[e], dsum);
        }
        dsum += __shfl_xor(dsum, 16, 64);
        dsum += __shfl_xor(dsum, 32, 64);
        dl[j] = qok[j] ? dsum : 0.f;
        // the dK / dV kernel, launched after this one, reads delta
        if (qok[j] && g == 0) p.delta[((int64_t)b * p.H + h) * p.S + myq[j]] = dsum;
        lse2[j] = qok[j] ? p.lse[((int64_t)b * p.H + h) * p.S + myq[j]] * 1.4426950408889634f : 0.f;
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
            if (p.dqkv) {   // the merged row: (bf16) of the scaled fp32 value, as kd_qkv_merge rounds it
                f32x4 v[DT];
#pragma unroll
                for (int d = 0; d < DT; ++d) v[d] = acc[j][d] * p.scale;
                if (p.rcos) {   // RoPE transpose: columns c and c + hd/2 (d-tiles d and d + hd/32) sit in this lane
                    const int hh = p.hd / 2, dh = hh / 16;
                    const float* cr = p.rcos + (int64_t)myq[j] * hh;
                    const float* sr = p.rsin + (int64_t)myq[j] * hh;
#pragma unroll
                    for (int d = 0; d < DT; ++d) {
                        if (d >= dh || d + dh >= DT) continue;
                        const int i = d * 16 + 4 * g;
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            float y1, y2;
                            rope_t(v[d][r], v[d + dh][r], cr[i + r], sr[i + r], y1, y2);
                            v[d][r] = y1; v[d + dh][r] = y2;
                        }
                    }
                }
#pragma unroll
                for (int d = 0; d < DT; ++d)
                    put_qkv4(p, b, myq[j], h, d * 16 + 4 * g, (bf16x4){(bf16)v[d][0], (bf16)v[d][1], (bf16)v[d][2], (bf16)v[d][3]});
            } else {
                float* dQr = p.dq + ((int64_t)(b * p.H + h) * p.S + myq[j]) * HDP;
#pragma unroll
                for (int d = 0; d < DT; ++d) *(f32x4*)(dQr + d * 16 + 4 * g) = acc[j][d] * p.scale;
            }
        }
}


// ------------------------------------------------------ backward, 32x32x16 MFMAs ----
// The 16x16x32 backward above runs at ~0.17 of the MFMA peak (an MFMA of 16 cycles holds the
// SIMD's issue for 8 of them, and every 16x16 tile carries its own LDS fragment reads). The same
// products on 32x32x16 MFMAs (issue held 8 of 32 cycles, half the LDS bytes per FLOP), with the
// forward's layout tricks:
//   k_attn_bwd_dq32 (product, head dims 64 / 96): per wave 32 queries (query on the lane).
//     S^T = K Q^T and dP^T = V dO^T (A = K / V rows from LDS, B = the wave's Q / dO rows in
//     registers), dS^T in the same registers, then dQ^T += K^T dS^T with the dS^T accumulator as
//     the B operand (keys in the forward's permuted order, K^T by ds_read_b64_tr_b16 in that order).
//   k_attn_bwd_dkdv32 (A/B library only, tools/ab/attention_bwd_dkdv32.inc: slower than
//     k_attn_bwd_dkdv2 at hd 96): per wave 32 keys (key on the lane), dV^T += dO^T P and
//     dK^T += Q^T dS with P / dS as the B operand (queries permuted the same way).
// Measured bound of dq32 (DESIGN.md §3 Attention, timing builds): the grid (1.44 rounds of
// two-per-SIMD waves at SigLIP's 729 queries) and the per-wave chain, not memory or VALU issue.
// One LDS image per tile serves both read directions (swQ below); all LDS reads in the loops
// are asm with counted lgkmcnt waits (a compiler-visible LDS read beside the in-flight LDS-DMA
// of the next tile is preceded by vmcnt(0)).

// swQ: chunk swizzle of an image read by rows (ds_read_b128: a 16-lane group reads one chunk
// of 16 rows whose indices cover every residue mod 16) AND by the 32x32 transposed reads (a
// 32-lane half reads 4 consecutive rows x 64 B). A bijection of the row's low 4 bits (RB 256)
// or bits 1-3 (RB 128, two rows per 256-B bank line) onto the chunk index -- row reads
// conflict-free -- whose top bits (RB 256: chunk bits 2-3 from row bits 0-1; RB 128: chunk bit 2
// from row bit 1, beside the row parity) put 4 consecutive rows in 4 different 64-B bank blocks.
template <int RB> __device__ __forceinline__ int swQ(int r) {
    return RB == 256 ? (((r & 3) << 2) | ((r >> 2) & 3)) : ((((r >> 1) & 1) << 2) | ((r >> 2) & 3));
}

// 64 rows x ncols of a row-strided bf16 matrix (ld elements per row) -> swQ image [64][RB];
// rows >= S and columns >= ncols land as zeros (out-of-range buffer offsets)
template <int HDP>
__device__ __forceinline__ void stage_q32(char* lds, const bf16* base, int64_t ld, int ncols, int row0, int S, int wid,
                                          int lane) {
    constexpr int RB = Geo<HDP>::RB, ROWS_PER = 1024 / RB, CH = RB / 16, NINSTR = 64 / ROWS_PER;
    const int rows_valid = min(64, S - row0);
    const uint32_t bytes = rows_valid <= 0 ? 0u : (uint32_t)(((int64_t)(rows_valid - 1) * ld + ncols) * 2);
    auto rs = rsrc(base + (int64_t)(rows_valid <= 0 ? 0 : row0) * ld, bytes);
#pragma unroll
    for (int s = 0; s < NINSTR / 4; ++s) {
        const int i = wid * (NINSTR / 4) + s;
        const int r = i * ROWS_PER + lane / CH;
        const int gc = (lane % CH) ^ swQ<RB>(r);
        const uint32_t voff = (gc * 8 < ncols && r < rows_valid) ? (uint32_t)((r * ld + gc * 8) * 2) : OOB;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void_t*)(lds + i * 1024), 16, voff, 0, 0, 0);
    }
}

// LDS reads at a per-lane address + an immediate offset (`off` must fold to a constant once the
// caller is inlined and unrolled)
__device__ __forceinline__ u32x4 ds_b128(uint32_t addr, const int off) {
    u32x4 v;
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "i"(off));
    return v;
}
__device__ __forceinline__ u32x2 ds_tr(uint32_t addr, const int off) {
    u32x2 v;
    asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "i"(off));
    return v;
}
// s_waitcnt lgkmcnt(N) naming the register it retires (no compiler copy above the wait)
template <int N, typename T> __device__ __forceinline__ void wait_lgkm(T& r) {
    asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(r) : "i"(N) : "memory");
}

// compile-time loop: f(std::integral_constant<int, I>) for I = 0 .. N-1
template <typename F, int... I>
__device__ __forceinline__ void sfor_impl(F&& f, std::integer_sequence<int, I...>) { (f(std::integral_constant<int, I>{}), ...); }
template <int N, typename F> __device__ __forceinline__ void sfor(F&& f) { sfor_impl(f, std::make_integer_sequence<int, N>{}); }

// two KS-step MFMA chains, A rows read from LDS, B in registers:
//   c0 += A(rows at a + OFF0) . b0,  c1 += A(rows at a + OFF1) . b1   (16-deep steps kk = 0 .. KS-1)
// every read issued one MFMA ahead of its use; `a[kk]` is the lane's byte address of step kk.
// INIT: c0 / c1 start from i0 / i1 (4 x 4 dwords each, LDS reads the caller issued before this
// call), retired by the first fragment wait, which names them (LDS returns in order)
// FILL(std::integral_constant<int, m>) runs after the m-th MFMA (m = 0 .. 2 KS - 1) is issued: VALU
// work of an earlier tile placed in the MFMA gaps (sched_barrier-fenced, so it stays there).
struct NoFill {
    template <typename T> __device__ __forceinline__ void operator()(T) const {}
};
template <int KS, int OFF0, int OFF1, bool INIT = false, typename FILL = NoFill>
__device__ __forceinline__ void chain2(f32x16& c0, f32x16& c1, const uint32_t (&a)[KS], const bf16x8 (&b0)[KS],
                                       const bf16x8 (&b1)[KS], u32x4 (&i0)[4], u32x4 (&i1)[4], FILL fill = FILL{}) {
    u32x4 x0[KS], x1[KS];
#pragma unroll
    for (int kk = 0; kk < KS; ++kk) x0[kk] = ds_b128(a[kk], OFF0);
    sfor<KS>([&](auto kc) {
        constexpr int kk = decltype(kc)::value;
        // in flight after x0[kk]: x0[kk + 1 ..] and x1[.. kk - 1]
        if constexpr (INIT && kk == 0) {
            asm volatile("s_waitcnt lgkmcnt(%9)"
                         : "+v"(x0[0]), "+v"(i0[0]), "+v"(i0[1]), "+v"(i0[2]), "+v"(i0[3]), "+v"(i1[0]), "+v"(i1[1]),
                           "+v"(i1[2]), "+v"(i1[3])
                         : "i"(KS - 1)
                         : "memory");
#pragma unroll
            for (int g = 0; g < 4; ++g)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    c0[4 * g + r] = __uint_as_float(i0[g][r]);
                    c1[4 * g + r] = __uint_as_float(i1[g][r]);
                }
        } else {
            wait_lgkm<KS - 1>(x0[kk]);
        }
        __builtin_amdgcn_sched_barrier(0);
        c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, x0[kk]), b0[kk], c0, 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
        x1[kk] = ds_b128(a[kk], OFF1);
        fill(std::integral_constant<int, kk>{});
        __builtin_amdgcn_sched_barrier(0);
    });
    sfor<KS>([&](auto kc) {
        constexpr int kk = decltype(kc)::value;
        wait_lgkm<KS - 1 - kk>(x1[kk]);
        __builtin_amdgcn_sched_barrier(0);
        c1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, x1[kk]), b1[kk], c1, 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
        fill(std::integral_constant<int, KS + kk>{});
        __builtin_amdgcn_sched_barrier(0);
    });
    __builtin_amdgcn_sched_barrier(0);
}

// s_waitcnt lgkmcnt(M), then every register of `r` named (no use of them above the wait): the M
// LDS reads issued after r's last are left in flight
template <int M, int N> __device__ __forceinline__ void wait_lgkm_n(u32x2 (&r)[N]) {
    asm volatile("s_waitcnt lgkmcnt(%0)" ::"i"(M) : "memory");
#pragma unroll
    for (int i = 0; i < N; ++i) asm volatile("" : "+v"(r[i]));
}
// plain f32 subtract / multiply as single instructions (the compiler's SLP pass would pair them
// into v_pk_* ops, which cost more than two single ops beside MFMAs)
__device__ __forceinline__ float f32_sub(float a, float b) {
    float r;
    asm("v_sub_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ float f32_mul(float a, float b) {
    float r;
    asm("v_mul_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
// s_waitcnt lgkmcnt(0), then every register of `r` named (no use of them above the wait)
template <int N> __device__ __forceinline__ void wait_lgkm0_all(u32x2 (&r)[N]) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int i = 0; i < N; ++i) asm volatile("" : "+v"(r[i]));
}

// per-lane byte addresses of the 32x32 transposed reads (the forward's V^T pattern): lane reads
// rows 4 hf + ((lane >> 2) & 3) (x = 0) and + 8 (x = 1), 4 columns at 32 D + 16 ((lane >> 4) & 1)
// + 4 (lane & 3); further rows (16 s, 32 ks) are immediates (swQ reads only row bits 0-3)
template <int HDP, int ND>
__device__ __forceinline__ void tr_addrs32(uint32_t (&ta)[ND][2], uint32_t base, int lane) {
    constexpr int RB = Geo<HDP>::RB;
    const int row = 4 * (lane >> 5) + ((lane >> 2) & 3);
#pragma unroll
    for (int d = 0; d < ND; ++d)
#pragma unroll
        for (int x = 0; x < 2; ++x) {
            const int r = row + 8 * x;
            const int col = 32 * d + 16 * ((lane >> 4) & 1) + 4 * (lane & 3);
            ta[d][x] = base + r * RB + ((((col >> 3) ^ swQ<RB>(r))) << 4) + ((col & 4) << 1);
        }
}

// dQ for 128 query rows of one head (4 waves x 32 queries), K / V tiles of 64 keys double-
// buffered by LDS-DMA; also writes delta = rowsum(dO * O) for the dK / dV kernel (launched after)
// DIAG (A/B library timing diagnostics only; wrong results): 1 = no K/V staging after the first tile
// (compute + barriers alone), 2 = staging without the end-of-tile vmcnt / barrier wait, 3 = neither
// staging nor waits (compute alone), 4 = as 3 with every tile taking the edge path
// PIPE: interior tiles software-pipelined (softmax in the MFMA gaps; 182 / 236 VGPRs at hd 64 / 96).
// The product runs it at two workgroups per CU; the unpipelined build (163 VGPRs at hd 64: three per CU)
// measured equal at hd 96 and 4 % slower at hd 64 (A/B: KD_ATTN_BWD_V=3).
template <int HDP, bool CAUSAL, int OCC = 2, int DIAG = 0, bool PIPE = true>
__global__ void __launch_bounds__(256, OCC) k_attn_bwd_dq32(AttnBwdP p) {
    // hd 128 would need lgkmcnt(16) below (the counter holds 15) and more VGPRs than two waves allow
    static_assert(HDP == 64 || HDP == 96, "k_attn_bwd_dq32: head dims 64 / 96");
    constexpr int RB = Geo<HDP>::RB, TILE = 64 * RB;
    constexpr int KS = HDP == 96 ? 5 : HDP / 16;              // 16-deep steps (hd <= 16 KS)
    constexpr int ND = HDP == 64 ? 2 : (HDP == 96 ? 3 : 4);   // 32-dim dQ^T tiles
    extern __shared__ __attribute__((aligned(16))) char smem[];   // [2][K TILE | V TILE], swQ images
    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int r32 = lane & 31, hf = lane >> 5;
    const int nqb = (p.S + 127) / 128;
    int h, b, zb;
    gqa_xcd_map(p.H, p.HKV, p.B, h, b, zb);
    const int qb = CAUSAL ? (nqb - 1 - zb) : zb;
    const int kvh = h / (p.H / p.HKV);
    const bf16* Q = p.q + ((int64_t)(b * p.H + h) * p.S) * HDP;
    const bf16* K = p.k + ((int64_t)(b * p.HKV + kvh) * p.S) * HDP;
    const bf16* V = p.v + ((int64_t)(b * p.HKV + kvh) * p.S) * HDP;
    const int q0 = qb * 128 + wid * 32;   // the wave's first query (uniform)
    const int myq = q0 + r32;
    const bool qok = myq < p.S;

    // the lane's Q and dO chunks (the B operands), delta = rowsum(dO * O) over both lane halves
    bf16x8 qf[KS], df[KS];
    float dsum = 0.f;
    {
        const int64_t orow = (((int64_t)b * p.S + (qok ? myq : 0)) * p.H + h) * p.hd;
#pragma unroll
        for (int kk = 0; kk < KS; ++kk) {
            const int d0 = 16 * kk + 8 * hf;
            qf[kk] = qok ? *(const bf16x8*)(Q + (int64_t)myq * HDP + d0) : (bf16x8){};
            const bool in = qok && d0 < p.hd;
            df[kk] = in ? *(const bf16x8*)(p.dO + orow + d0) : (bf16x8){};
            const bf16x8 of = in ? *(const bf16x8*)(p.o + orow + d0) : (bf16x8){};
#pragma unroll
            for (int e = 0; e < 8; ++e) dsum = __builtin_fmaf((float)df[kk][e], (float)of[e], dsum);
        }
    }
    dsum = half_sum(dsum);
    const float dl = qok ? dsum : 0.f;
    if (qok && hf == 0) p.delta[((int64_t)b * p.H + h) * p.S + myq] = dsum;
    const float lse2 = qok ? p.lse[((int64_t)b * p.H + h) * p.S + myq] * 1.4426950408889634f : 0.f;

    f32x16 acc[ND];
#pragma unroll
    for (int d = 0; d < ND; ++d)
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[d][i] = 0.f;

    const int nkv_all = (p.S + 63) / 64;
    const int nkv = CAUSAL ? min((qb * 128 + 127) / 64 + 1, nkv_all) : nkv_all;
    // tiles with a key <= the wave's last query (none for a wave past the sequence end)
    const int nkv_w = q0 >= p.S ? 0 : (CAUSAL ? min(nkv, (q0 + 31) / 64 + 1) : nkv);
    stage_q32<HDP>(smem, K, HDP, HDP, 0, p.S, wid, lane);
    stage_q32<HDP>(smem + TILE, V, HDP, HDP, 0, p.S, wid, lane);
    const uint32_t sbase = (uint32_t)(uintptr_t)smem;
    uint32_t ra[KS];   // row reads: row r32 (+ 32 kt), chunk 2 kk + hf
#pragma unroll
    for (int kk = 0; kk < KS; ++kk) ra[kk] = sbase + r32 * RB + (((2 * kk + hf) ^ swQ<RB>(r32)) << 4);
    uint32_t ta[ND][2];
    tr_addrs32<HDP, ND>(ta, sbase, lane);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();

    auto tile = [&](const int t, auto buf_c) {
        constexpr int BUF = decltype(buf_c)::value;
        constexpr int KO = BUF * 2 * TILE, VO = KO + TILE;
        if (DIAG != 1 && DIAG != 3 && DIAG != 4 && t + 1 < nkv) {
            char* nb = smem + (BUF ^ 1) * 2 * TILE;
            stage_q32<HDP>(nb, K, HDP, HDP, (t + 1) * 64, p.S, wid, lane);
            stage_q32<HDP>(nb + TILE, V, HDP, HDP, (t + 1) * 64, p.S, wid, lane);
        }
        const bool edge = DIAG == 4 || t * 64 + 63 >= p.S || (CAUSAL && t * 64 + 63 > q0);   // a key past S or a query
        if (PIPE && t < nkv_w && !edge) {
            // interior tile, software-pipelined: the softmax of keys 0-31 runs in the MFMA gaps of
            // keys 32-63's S^T / dP^T chains, that of keys 32-63 in the gaps of dQ's first two key steps
            f32x16 sc[2], dp[2];
#pragma unroll
            for (int kt = 0; kt < 2; ++kt)
#pragma unroll
                for (int i = 0; i < 16; ++i) { sc[kt][i] = 0.f; dp[kt][i] = 0.f; }
            u32x4 nz[4];
            bf16x8 dsf[4];
            // dS^T elements [I0, I0 + N) of sub-tile KT, staged so no result is used by the next
            // instruction (fma .. exp .. sub .. mul), single-lane f32 ops (no packed pairs beside MFMAs)
            auto sm = [&](auto kt_c, auto i0_c, auto n_c) {
                constexpr int KT = decltype(kt_c)::value, I0 = decltype(i0_c)::value, N = decltype(n_c)::value;
                if constexpr (N > 0) {
                    float x[N], y[N];
                    sfor<N>([&](auto j) { x[j] = fmaf(sc[KT][I0 + j], p.scale_log2, -lse2); });
                    sfor<N>([&](auto j) { x[j] = __builtin_amdgcn_exp2f(x[j]); });
                    sfor<N>([&](auto j) { y[j] = f32_sub(dp[KT][I0 + j], dl); });
                    sfor<N>([&](auto j) {
                        constexpr int i = I0 + decltype(j)::value;
                        dsf[2 * KT + (i >> 3)][i & 7] = (bf16)f32_mul(x[j], y[j]);
                    });
                }
            };
            // slot m of n slots gets elements [lo(m), lo(m + 1)) of `cnt` starting at `base`
            auto part = [&](auto kt_c, auto base_c, auto cnt_c, auto n_c, auto m_c) {
                constexpr int base = decltype(base_c)::value, cnt = decltype(cnt_c)::value;
                constexpr int n = decltype(n_c)::value, m = decltype(m_c)::value;
                constexpr int lo = base + cnt * m / n, hi = base + cnt * (m + 1) / n;
                sm(kt_c, std::integral_constant<int, lo>{}, std::integral_constant<int, hi - lo>{});
            };
            using I0c = std::integral_constant<int, 0>;
            using I1c = std::integral_constant<int, 1>;
            chain2<KS, KO, VO>(sc[0], dp[0], ra, qf, df, nz, nz);   // keys 0-31: S^T = K Q^T, dP^T = V dO^T
            // keys 32-63, sub-tile 0's softmax in MFMA gaps 2 .. 2 KS - 1 (dP^T of keys 0-31 lands first)
            chain2<KS, KO + 32 * RB, VO + 32 * RB, false>(sc[1], dp[1], ra, qf, df, nz, nz, [&](auto m_c) {
                constexpr int m = decltype(m_c)::value;
                if constexpr (m >= 2)
                    part(I0c{}, I0c{}, std::integral_constant<int, 16>{}, std::integral_constant<int, 2 * KS - 2>{},
                         std::integral_constant<int, m - 2>{});
            });
            // dQ^T += K^T dS^T: key steps 0-1 (keys 0-31) beside sub-tile 1's first 8 elements, key step 2
            // beside its last 8, then key step 3; every K^T read issued before the first of these MFMAs
            u32x2 kc[ND * 4], kd[ND * 4];
#pragma unroll
            for (int d = 0; d < ND; ++d)
#pragma unroll
                for (int s = 0; s < 2; ++s) {
                    kc[4 * d + 2 * s] = ds_tr(ta[d][0], KO + 16 * s * RB);
                    kc[4 * d + 2 * s + 1] = ds_tr(ta[d][1], KO + 16 * s * RB);
                }
#pragma unroll
            for (int d = 0; d < ND; ++d)
#pragma unroll
                for (int s = 0; s < 2; ++s) {
                    kd[4 * d + 2 * s] = ds_tr(ta[d][0], KO + 16 * (s + 2) * RB);
                    kd[4 * d + 2 * s + 1] = ds_tr(ta[d][1], KO + 16 * (s + 2) * RB);
                }
            __builtin_amdgcn_sched_barrier(0);
            wait_lgkm_n<ND * 4>(kc);   // the kd reads (issued after) may still be in flight
            __builtin_amdgcn_sched_barrier(0);
            sfor<2 * ND>([&](auto m_c) {
                constexpr int m = decltype(m_c)::value, d = m >> 1, s = m & 1;
                acc[d] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
                    cat4(__builtin_bit_cast(bf16x4, kc[4 * d + 2 * s]), __builtin_bit_cast(bf16x4, kc[4 * d + 2 * s + 1])),
                    dsf[s], acc[d], 0, 0, 0);
                __builtin_amdgcn_sched_barrier(0);
                part(I1c{}, I0c{}, std::integral_constant<int, 8>{}, std::integral_constant<int, 2 * ND>{}, m_c);
                __builtin_amdgcn_sched_barrier(0);
            });
            wait_lgkm0_all(kd);
            __builtin_amdgcn_sched_barrier(0);
            sfor<ND>([&](auto d_c) {
                constexpr int d = decltype(d_c)::value;
                acc[d] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
                    cat4(__builtin_bit_cast(bf16x4, kd[4 * d]), __builtin_bit_cast(bf16x4, kd[4 * d + 1])), dsf[2], acc[d], 0, 0, 0);
                __builtin_amdgcn_sched_barrier(0);
                part(I1c{}, std::integral_constant<int, 8>{}, std::integral_constant<int, 8>{}, std::integral_constant<int, ND>{}, d_c);
                __builtin_amdgcn_sched_barrier(0);
            });
#pragma unroll
            for (int d = 0; d < ND; ++d)
                acc[d] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
                    cat4(__builtin_bit_cast(bf16x4, kd[4 * d + 2]), __builtin_bit_cast(bf16x4, kd[4 * d + 3])), dsf[3], acc[d], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
        } else if (t < nkv_w) {
            f32x16 sc[2], dp[2];
#pragma unroll
            for (int kt = 0; kt < 2; ++kt)
#pragma unroll
                for (int i = 0; i < 16; ++i) { sc[kt][i] = 0.f; dp[kt][i] = 0.f; }
            u32x4 nz[4];
            chain2<KS, KO, KO + 32 * RB>(sc[0], sc[1], ra, qf, qf, nz, nz);   // S^T = K Q^T (two 32-key sub-tiles)
            chain2<KS, VO, VO + 32 * RB>(dp[0], dp[1], ra, df, df, nz, nz);   // dP^T = V dO^T
            if (edge) {
#pragma unroll
                for (int kt = 0; kt < 2; ++kt)
#pragma unroll
                    for (int i = 0; i < 16; ++i) {
                        const int key = t * 64 + 32 * kt + 8 * (i >> 2) + 4 * hf + (i & 3);
                        if (key >= p.S || (CAUSAL && key > myq)) sc[kt][i] = -INFINITY;
                    }
            }
            // dS^T = P (dP - delta), P = 2^(s scale_log2 - lse2); packed to bf16 in the forward's
            // permuted key order (k-step s: registers 8 (s & 1) .. + 7 of sub-tile s >> 1)
            bf16x8 dsf[4];
#pragma unroll
            for (int s = 0; s < 4; ++s)
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const int kt = s >> 1, i = 8 * (s & 1) + j;
                    const float pe = __builtin_amdgcn_exp2f(fmaf(sc[kt][i], p.scale_log2, -lse2));
                    dsf[s][j] = (bf16)(pe * (dp[kt][i] - dl));
                }
            // dQ^T += K^T dS^T: per 32-dim tile 8 transposed K reads (4 key steps x rows +0 / +8)
            u32x2 kr[2][8];
#define KD_DQ_RD(D, SET)                                                              \
    _Pragma("unroll") for (int s = 0; s < 4; ++s) {                                   \
        kr[SET][2 * s] = ds_tr(ta[D][0], KO + 16 * s * RB);                           \
        kr[SET][2 * s + 1] = ds_tr(ta[D][1], KO + 16 * s * RB);                       \
    }
#define KD_DQ_MM(D, SET)                                                                                           \
    _Pragma("unroll") for (int s = 0; s < 4; ++s) {                                                                \
        const bf16x8 kv = cat4(__builtin_bit_cast(bf16x4, kr[SET][2 * s]), __builtin_bit_cast(bf16x4, kr[SET][2 * s + 1])); \
        acc[D] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kv, dsf[s], acc[D], 0, 0, 0);                           \
    }
#define KD_DQ_WAIT(N, SET) wait_lgkm_def8<N>(kr[SET]); __builtin_amdgcn_sched_barrier(0);
            KD_DQ_RD(0, 0)
            KD_DQ_RD(1, 1)
            KD_DQ_WAIT(8, 0)
            KD_DQ_MM(0, 0)
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (ND > 2) { KD_DQ_RD(2, 0) KD_DQ_WAIT(8, 1) }
            else { KD_DQ_WAIT(0, 1) }
            KD_DQ_MM(1, 1)
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (ND > 2) {
                if constexpr (ND > 3) { KD_DQ_RD(3, 1) KD_DQ_WAIT(8, 0) }
                else { KD_DQ_WAIT(0, 0) }
                KD_DQ_MM(2, 0)
                __builtin_amdgcn_sched_barrier(0);
                if constexpr (ND > 3) {
                    KD_DQ_WAIT(0, 1)
                    KD_DQ_MM(3, 1)
                }
            }
#undef KD_DQ_RD
#undef KD_DQ_MM
#undef KD_DQ_WAIT
        }
        if (DIAG < 2) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
        }
    };
    int t = 0;
    for (; t + 1 < nkv; t += 2) {
        tile(t, std::integral_constant<int, 0>{});
        tile(t + 1, std::integral_constant<int, 1>{});
    }
    if (t < nkv) tile(t, std::integral_constant<int, 0>{});

    // lane = query myq, register 4 g + r of tile D = dim 32 D + 8 g + 4 hf + r
    if (qok) {
        if (p.dqkv) {   // the merged row: (bf16) of the scaled fp32 value, as kd_qkv_merge rounds it
            f32x16 v[ND];
#pragma unroll
            for (int d = 0; d < ND; ++d) v[d] = acc[d] * p.scale;
            if (p.rcos) {   // RoPE transpose (hd == HDP, hd % 32 == 0): columns c, c + hd/2 are tiles D, D + ND/2
                const int hh = p.hd / 2;
                const float* cr = p.rcos + (int64_t)myq * hh;
                const float* sr = p.rsin + (int64_t)myq * hh;
#pragma unroll
                for (int d = 0; d < ND / 2; ++d)
#pragma unroll
                    for (int i = 0; i < 16; ++i) {
                        const int c = 32 * d + 8 * (i >> 2) + 4 * hf + (i & 3);
                        float y1, y2;
                        rope_t(v[d][i], v[d + ND / 2][i], cr[c], sr[c], y1, y2);
                        v[d][i] = y1; v[d + ND / 2][i] = y2;
                    }
            }
#pragma unroll
            for (int d = 0; d < ND; ++d)
#pragma unroll
                for (int g = 0; g < 4; ++g)
                    put_qkv4(p, b, myq, h, 32 * d + 8 * g + 4 * hf,
                             (bf16x4){(bf16)v[d][4 * g], (bf16)v[d][4 * g + 1], (bf16)v[d][4 * g + 2], (bf16)v[d][4 * g + 3]});
        } else {
            float* dQr = p.dq + ((int64_t)(b * p.H + h) * p.S + myq) * HDP;
#pragma unroll
            for (int d = 0; d < ND; ++d)
#pragma unroll
                for (int g = 0; g < 4; ++g)
                    *(f32x4*)(dQr + 32 * d + 8 * g + 4 * hf) =
                        (f32x4){acc[d][4 * g], acc[d][4 * g + 1], acc[d][4 * g + 2], acc[d][4 * g + 3]} * p.scale;
        }
    }
}

#ifdef KD_AB_BUILD
#include "attention_bwd_dkdv32.inc"   // tools/ab/attention_bwd_dkdv32.inc: the 32x32x16 dK / dV kernel (KD_ATTN_BWD_V=32)
#endif  // KD_AB_BUILD

}  // namespace

#ifdef KD_AB_BUILD
// the six-wave forward by default: not yet (A/B with forced variant 36 first); head dim 128
// needs more than the 168 VGPRs of three waves per SIMD (it spilled), so it keeps four waves
static bool fwd_nw6(const kd_attn_desc* d) {
    (void)d;
    return false;
}
template <int HD, bool C>
void launch_fwd_nw6(dim3 grid, size_t smem, hipStream_t st, const AttnP& p) {
    if constexpr (HD == 128) {
        grid.z = (p.S + 127) / 128;
        hipLaunchKernelGGL((k_attn_fwd32<HD, C, false>), grid, dim3(256), smem, st, p);
    } else {
        hipLaunchKernelGGL((k_attn_fwd32<HD, C, false, false, 6>), grid, dim3(384), smem, st, p);
    }
}

#endif  // KD_AB_BUILD

int launch_attn_fwd(const kd_attn_desc* d, void* stream_) {
    KD_CHECK_ARG(d && d->q && d->k && d->v && d->o, "attn_fwd: null pointer");
    KD_CHECK_SHAPE(d->B > 0 && d->S > 0 && d->H > 0 && d->HKV > 0 && d->H % d->HKV == 0, "attn_fwd: heads");
    KD_CHECK_SHAPE(d->hd > 0 && d->hd <= d->hdp && d->hd % 4 == 0, "attn_fwd: hd");
    KD_CHECK_SHAPE(d->hdp == 64 || d->hdp == 96 || d->hdp == 128, "attn_fwd: padded head dim must be 64/96/128");
    KD_CHECK_SHAPE(!(d->hdp == 96 && d->hd > 80) && !(d->hdp == 64 && d->hd > 64), "attn_fwd: hd exceeds tile cover");
    AttnP p{(const bf16*)d->q, (const bf16*)d->k, (const bf16*)d->v, (bf16*)d->o, d->lse,
            d->B, d->H, d->HKV, d->S, d->hd, (float)(1.4426950408889634 / std::sqrt((double)d->hd))};
    hipStream_t st = as_stream(stream_);
    const int rb = d->hdp == 64 ? 128 : 256;
    const size_t smem = 2 * 2 * 64 * rb;
#ifdef KD_AB_BUILD
    // KD_ATTN_FWD_V (A/B and diagnostics; read per call, so a test can switch variants inside one
    // process): unset / 32 = k_attn_fwd32 (LDS-DMA staging, the product kernel), 64 = k_attn_fwd64
    // (two query blocks per wave), 35 = its register-staged build, 33 = the sub-tile-pipelined
    // k_attn_fwd32p, 34 = the stamp build, 36 = six-wave workgroups, 16 = the 16x16x32 k_attn_fwd
    // (KD_ATTN_FWD_NQ=1: one query sub-tile per wave)
    static const int nq = [] { const char* e = std::getenv("KD_ATTN_FWD_NQ"); return (e && e[0] == '1') ? 1 : 2; }();
    const char* fve = std::getenv("KD_ATTN_FWD_V");
    const int fv = fve ? std::atoi(fve) : 0;
    const bool v16 = fv == 16, nw6 = fv == 36, w64 = fv == 64;
    dim3 grid(d->H, d->B, v16 ? (d->S + 64 * nq - 1) / (64 * nq)
                              : (w64 ? (d->S + 255) / 256 : (d->S + (nw6 ? 191 : 127)) / (nw6 ? 192 : 128)));
#define LAUNCH(HD, C)                                                                                \
    do {                                                                                             \
        if (nw6) launch_fwd_nw6<HD, C>(grid, smem, st, p);                                           \
        else if (w64) hipLaunchKernelGGL((k_attn_fwd64<HD, C>), grid, dim3(256), smem, st, p);       \
        else if (fv == 0 || fv == 32) hipLaunchKernelGGL((k_attn_fwd32<HD, C, false>), grid, dim3(256), smem, st, p); \
        else if (fv == 35) hipLaunchKernelGGL((k_attn_fwd32<HD, C, true>), grid, dim3(256), smem, st, p); \
        else if (fv == 33) hipLaunchKernelGGL((k_attn_fwd32p<HD, C>), grid, dim3(256), smem, st, p); \
        else if (fv == 34) hipLaunchKernelGGL((k_attn_fwd32<HD, C, false, true>), grid, dim3(256), smem, st, p); \
        else if (nq == 2) hipLaunchKernelGGL((k_attn_fwd<HD, C, 2>), grid, dim3(256), smem, st, p);  \
        else hipLaunchKernelGGL((k_attn_fwd<HD, C, 1>), grid, dim3(256), smem, st, p);               \
    } while (0)
#else
    const dim3 grid(d->H, d->B, (d->S + 127) / 128);
#define LAUNCH(HD, C) hipLaunchKernelGGL((k_attn_fwd32<HD, C, false>), grid, dim3(256), smem, st, p)
#endif
    if (d->hdp == 64) { if (d->causal) LAUNCH(64, true); else LAUNCH(64, false); }
    else if (d->hdp == 96) { if (d->causal) LAUNCH(96, true); else LAUNCH(96, false); }
    else { if (d->causal) LAUNCH(128, true); else LAUNCH(128, false); }
#undef LAUNCH
    KD_LAUNCH_CHECK("k_attn_fwd");
    return KD_OK;
}

// dK / dV launch: the two-sub-tile kernel for head dims 64 / 96 (at 128 its 2 x 2 x DT
// accumulator tiles do not fit beside the fragments: the one-sub-tile kernel there; the 7B
// teacher never runs a backward)
template <int HD, bool C>
void launch_dq1(dim3 grid, size_t smem, hipStream_t st, const AttnBwdP& p) {
#ifdef KD_AB_BUILD
    hipLaunchKernelGGL((k_attn_bwd_dq<HD, C, 1>), grid, dim3(256), smem, st, p);
#else
    (void)grid; (void)smem; (void)st; (void)p;
#endif
}

template <int HD, bool C>
void launch_dkdv(bool kv16, dim3 grid, size_t smem, hipStream_t st, const AttnBwdP& p) {
    if constexpr (HD == 128) {
        grid.z = (p.S + 63) / 64;
        hipLaunchKernelGGL((k_attn_bwd_dkdv<HD, C>), grid, dim3(256), smem, st, p);
    } else {
#ifdef KD_AB_BUILD
        if (kv16) hipLaunchKernelGGL((k_attn_bwd_dkdv<HD, C>), grid, dim3(256), smem, st, p);
        else
#endif
        hipLaunchKernelGGL((k_attn_bwd_dkdv2<HD, C>), grid, dim3(256), smem, st, p);
        (void)kv16;
    }
}

// dQ (+ delta) by the 32x32x16 k_attn_bwd_dq32 (head dims 64 / 96). A/B library: `diag` 1 = the
// unpipelined build (hd 64: three workgroups per CU), 2-5 = its DIAG builds 1-4
template <int HD, bool C>
int launch_dq32(int diag, dim3 grid_q, size_t smem_q, hipStream_t st, const AttnBwdP& p) {
    if constexpr (HD == 128) {
        (void)diag; (void)grid_q; (void)smem_q; (void)st; (void)p;
        return fail(KD_ERR_SHAPE, "attn_bwd: no 32x32 dQ kernel for head dim 128");
    } else {
#ifdef KD_AB_BUILD
        if (diag == 1) hipLaunchKernelGGL((k_attn_bwd_dq32<HD, C, HD == 64 ? 3 : 2, 0, false>), grid_q, dim3(256), smem_q, st, p);
        else if (diag == 2) hipLaunchKernelGGL((k_attn_bwd_dq32<HD, C, 2, 1>), grid_q, dim3(256), smem_q, st, p);
        else if (diag == 3) hipLaunchKernelGGL((k_attn_bwd_dq32<HD, C, 2, 2>), grid_q, dim3(256), smem_q, st, p);
        else if (diag == 4) hipLaunchKernelGGL((k_attn_bwd_dq32<HD, C, 2, 3>), grid_q, dim3(256), smem_q, st, p);
        else if (diag == 5) hipLaunchKernelGGL((k_attn_bwd_dq32<HD, C, 2, 4>), grid_q, dim3(256), smem_q, st, p);
        else
#endif
        hipLaunchKernelGGL((k_attn_bwd_dq32<HD, C>), grid_q, dim3(256), smem_q, st, p);
        (void)diag;
        KD_LAUNCH_CHECK("k_attn_bwd_dq32");
        return KD_OK;
    }
}

// dQ by the 16x16x32 k_attn_bwd_dq: head dim 128 in the product (no 32x32 build there; the teacher
// runs no backward in the step), every head dim in the A/B library (the round-6 pair, KD_ATTN_BWD_V=2)
template <int HD, bool C>
int launch_dq16(int nq, dim3 grid_q, size_t smem_q, hipStream_t st, const AttnBwdP& p) {
#ifdef KD_AB_BUILD
    constexpr bool avail = true;
#else
    constexpr bool avail = HD == 128;
#endif
    if constexpr (!avail) {
        (void)nq; (void)grid_q; (void)smem_q; (void)st; (void)p;
        return fail(KD_ERR_SHAPE, "attn_bwd: the 16x16 dQ kernel runs head dim 128 only (k_attn_bwd_dq32 below)");
    } else {
        if (nq == 2) hipLaunchKernelGGL((k_attn_bwd_dq<HD, C, 2>), grid_q, dim3(256), smem_q, st, p);
        else launch_dq1<HD, C>(grid_q, smem_q, st, p);
        KD_LAUNCH_CHECK("k_attn_bwd_dq");
        return KD_OK;
    }
}

#ifdef KD_AB_BUILD
template <int HD, bool C>
int launch_dkdv32(dim3 grid, size_t smem_kv, hipStream_t st, const AttnBwdP& p) {
    if constexpr (HD == 128) {
        (void)grid; (void)smem_kv; (void)st; (void)p;
        return fail(KD_ERR_SHAPE, "attn_bwd: no 32x32 dK / dV kernel for head dim 128");
    } else {
        hipLaunchKernelGGL((k_attn_bwd_dkdv32<HD, C>), grid, dim3(256), smem_kv, st, p);
        KD_LAUNCH_CHECK("k_attn_bwd_dkdv32");
        return KD_OK;
    }
}
#endif  // KD_AB_BUILD

size_t attn_bwd_workspace_size(const kd_attn_bwd_desc* d) {
    if (!d || d->HKV <= 0 || d->H == d->HKV) return 0;
    return (size_t)2 * d->B * d->H * d->S * d->hdp * 4;
}

int launch_attn_bwd(const kd_attn_bwd_desc* d, void* stream_) {
    KD_CHECK_ARG(d && d->q && d->k && d->v && d->o && d->dO && d->lse && d->delta && (d->dqkv || (d->dq && d->dk && d->dv)),
                 "attn_bwd: null pointer");
    KD_CHECK_ARG(!d->dqkv || (d->ld_qkv >= (int64_t)(d->H + 2 * d->HKV) * d->hd && d->ld_qkv % 4 == 0 &&
                              (uintptr_t)d->dqkv % 8 == 0),
                 "attn_bwd: dqkv needs ld_qkv >= (H + 2 HKV) hd (a multiple of 4) and an 8-B aligned base");
    KD_CHECK_ARG(!d->cos_t == !d->sin_t && (!d->cos_t || (d->dqkv && d->H != d->HKV && d->hd == d->hdp && d->hd % 32 == 0)),
                 "attn_bwd: RoPE tables only with dqkv, GQA (H > HKV) and hd == hdp, hd % 32 == 0");
    KD_CHECK_ARG(!d->dqkv || d->H == d->HKV || (d->hd % 8 == 0),
                 "attn_bwd: dqkv with GQA needs hd % 8 == 0");
    KD_CHECK_SHAPE(d->B > 0 && d->S > 0 && d->HKV > 0 && d->H % d->HKV == 0 && d->hd % 4 == 0 && d->hd <= d->hdp,
                   "attn_bwd: shape");
    KD_CHECK_SHAPE(d->hdp == 64 || d->hdp == 96 || d->hdp == 128, "attn_bwd: padded head dim must be 64/96/128");
    KD_CHECK_SHAPE(!(d->hdp == 96 && d->hd > 80) && !(d->hdp == 64 && d->hd > 64), "attn_bwd: hd exceeds tile cover");
    KD_CHECK_SHAPE(d->hd % 8 == 0, "attn_bwd: hd must be a multiple of 8 (16-B dO rows)");
    const size_t need = attn_bwd_workspace_size(d);
    if (need && (!d->workspace || d->workspace_bytes < need))
        return fail(KD_ERR_WORKSPACE, "attn_bwd: GQA needs kd_attn_bwd_workspace_size() bytes of workspace");
    hipStream_t st = as_stream(stream_);
    // delta = rowsum(dO * O) is computed by the dQ kernel (its lanes hold the dO rows already) and
    // written for the dK / dV kernel, which therefore runs second
    const double sc = 1.0 / std::sqrt((double)d->hd);
    float* dkp = need ? (float*)d->workspace : nullptr;
    float* dvp = need ? dkp + (size_t)d->B * d->H * d->S * d->hdp : nullptr;
    AttnBwdP p{(const bf16*)d->q, (const bf16*)d->k, (const bf16*)d->v, (const bf16*)d->dO, (const bf16*)d->o, d->lse, d->delta,
               d->dq, (bf16*)d->dk, (bf16*)d->dv, dkp, dvp, d->B, d->H, d->HKV, d->S, d->hd, (float)sc,
               (float)(sc * 1.4426950408889634), (bf16*)d->dqkv, d->ld_qkv, d->cos_t, d->sin_t};
#ifdef KD_AB_BUILD
    // head dims 64 / 96 (A/B; read per call): unset / 0 = the product pair (k_attn_bwd_dq32 +
    // k_attn_bwd_dkdv2); 2 = the round-6 16x16x32 pair (k_attn_bwd_dq + k_attn_bwd_dkdv2); 16 = the
    // one-sub-tile dK / dV kernel; 32 = k_attn_bwd_dq32 + k_attn_bwd_dkdv32; 3 / 5-8 = dq32 unpipelined
    // (hd 64: three workgroups per CU) / its DIAG builds 1-4 (timing only). KD_ATTN_DQ_NQ=1: one query sub-tile per
    // 16x16 dQ wave
    const char* bve = std::getenv("KD_ATTN_BWD_V");
    const int bv = bve ? std::atoi(bve) : 0;
    const bool kv16 = bv == 16, dq32 = bv != 2 && bv != 16, kv32 = bv == 32;
    const int diag = bv == 3 ? 1 : (bv >= 5 && bv <= 8 ? bv - 3 : 0);
    static const int nq_dq = [] { const char* e = std::getenv("KD_ATTN_DQ_NQ"); return (e && e[0] == '1') ? 1 : 2; }();
#else
    constexpr bool kv16 = false, dq32 = true;
    constexpr int diag = 0, nq_dq = 2;
#endif
    dim3 grid(d->H, d->B, kv16 ? (d->S + 63) / 64 : (d->S + 127) / 128);
    const int qrows = dq32 ? 128 : 64 * nq_dq;   // query rows per dQ workgroup
    dim3 grid_q(d->H, d->B, (d->S + qrows - 1) / qrows);
    const int rb = d->hdp == 64 ? 128 : 256;
    const size_t smem_kv = 2 * (2 * 64 * rb + 512);
    const size_t smem_q = 2 * 2 * 64 * rb;
#ifdef KD_AB_BUILD
#define KD_AB_KV32(HD, C)                                                                     \
    if (HD != 128 && kv32) {                                                                  \
        const int rc = launch_dkdv32<HD, C>(grid, smem_kv, st, p);                            \
        if (rc != KD_OK) return rc;                                                           \
        break;                                                                                \
    }
#else
#define KD_AB_KV32(HD, C)
#endif
#define LAUNCH(HD, C)                                                                         \
    do {                                                                                      \
        if (HD != 128 && dq32) {                                                              \
            const int rc = launch_dq32<HD, C>(diag, grid_q, smem_q, st, p);                   \
            if (rc != KD_OK) return rc;                                                       \
        } else {                                                                              \
            const int rc = launch_dq16<HD, C>(nq_dq, grid_q, smem_q, st, p);                  \
            if (rc != KD_OK) return rc;                                                       \
        }                                                                                     \
        KD_AB_KV32(HD, C)                                                                     \
        launch_dkdv<HD, C>(kv16, grid, smem_kv, st, p);                                       \
        KD_LAUNCH_CHECK("k_attn_bwd_dkdv");                                                   \
    } while (0)
    if (d->hdp == 64) { if (d->causal) LAUNCH(64, true); else LAUNCH(64, false); }
    else if (d->hdp == 96) { if (d->causal) LAUNCH(96, true); else LAUNCH(96, false); }
    else { if (d->causal) LAUNCH(128, true); else LAUNCH(128, false); }
#undef LAUNCH
#undef KD_AB_KV32
    if (need) {
        const int dcols = 16 * (d->hdp == 64 ? 4 : (d->hdp == 96 ? 5 : 8));
        const int64_t work = (int64_t)d->B * d->HKV * d->S * dcols / 4;
        if (d->dqkv) {
            const int64_t work2 = (int64_t)d->B * d->HKV * d->S * (d->hd / 8);
            hipLaunchKernelGGL(k_attn_group_sum_qkv, dim3((unsigned)std::min<int64_t>((work2 + 255) / 256, 8192)), dim3(256), 0,
                               st, dkp, dvp, (bf16*)d->dqkv, d->ld_qkv, d->cos_t, d->sin_t, d->B, d->H, d->HKV, d->S, d->hd,
                               d->hdp, (float)sc);
        } else {
            hipLaunchKernelGGL(k_attn_group_sum, dim3((unsigned)std::min<int64_t>((work + 255) / 256, 8192)), dim3(256), 0, st,
                               dkp, dvp, (bf16*)d->dk, (bf16*)d->dv, d->B, d->H, d->HKV, d->S, d->hdp, dcols, (float)sc);
        }
        KD_LAUNCH_CHECK("k_attn_group_sum");
    }
    return KD_OK;
}

}  // namespace kd
