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

namespace kd {
namespace {

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4_t;
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

template <int HDP, bool CAUSAL>
__global__ void __launch_bounds__(256, 2) k_attn_fwd(AttnP p) {
    constexpr int RB = Geo<HDP>::RB, KS = Geo<HDP>::KSTEPS, DT = Geo<HDP>::DT;
    constexpr int TILE = 64 * RB;
    extern __shared__ __attribute__((aligned(16))) char smem[];  // [2][K TILE | V TILE]
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int g = lane >> 4, li = lane & 15;
    const int nqb = (p.S + 63) / 64;
    const int qb = CAUSAL ? (nqb - 1 - (int)blockIdx.x) : (int)blockIdx.x;
    const int h = blockIdx.y, b = blockIdx.z, kvh = h / (p.H / p.HKV);
    const bf16* Q = p.q + ((int64_t)(b * p.H + h) * p.S) * HDP;
    const bf16* K = p.k + ((int64_t)(b * p.HKV + kvh) * p.S) * HDP;
    const bf16* V = p.v + ((int64_t)(b * p.HKV + kvh) * p.S) * HDP;
    const int q0 = qb * 64 + wid * 16;
    const int myq = q0 + li;

    bf16x8 qf[KS];
#pragma unroll
    for (int kk = 0; kk < KS; ++kk) {
        if (myq < p.S) qf[kk] = *(const bf16x8*)(Q + (int64_t)myq * HDP + kk * 32 + 8 * g);
        else qf[kk] = (bf16x8){};
    }
    f32x4 o[DT];
#pragma unroll
    for (int d = 0; d < DT; ++d) o[d] = (f32x4){0.f, 0.f, 0.f, 0.f};
    float m = -INFINITY, l = 0.f;

    const int nkv = CAUSAL ? min(qb + 1, (p.S + 63) / 64) : (p.S + 63) / 64;
    stage_kv<HDP, false>(smem, K, 0, p.S, wid, lane);
    stage_kv<HDP, true>(smem + TILE, V, 0, p.S, wid, lane);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();

    for (int t = 0; t < nkv; ++t) {
        const int cur = t & 1;
        if (t + 1 < nkv) {
            char* nb = smem + (cur ^ 1) * 2 * TILE;
            stage_kv<HDP, false>(nb, K, (t + 1) * 64, p.S, wid, lane);
            stage_kv<HDP, true>(nb + TILE, V, (t + 1) * 64, p.S, wid, lane);
        }
        const char* kt_l = smem + cur * 2 * TILE;
        const char* vt_l = kt_l + TILE;
        // ---- S^T tiles: rows = keys 16kt + 4g + r, col = my query
        f32x4 s[4];
#pragma unroll
        for (int kt = 0; kt < 4; ++kt) {
            s[kt] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int kk = 0; kk < KS; ++kk)
                s[kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(k_frag<RB>(kt_l, 16 * kt + li, kk * 4 + g), qf[kk], s[kt], 0, 0, 0);
        }
        float mt = -INFINITY;
#pragma unroll
        for (int kt = 0; kt < 4; ++kt)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int key = t * 64 + 16 * kt + 4 * g + r;
                float v = s[kt][r] * p.scale_log2;
                if (key >= p.S || (CAUSAL && key > myq)) v = -INFINITY;
                s[kt][r] = v;
                mt = fmaxf(mt, v);
            }
        mt = fmaxf(mt, __shfl_xor(mt, 16, 64));
        mt = fmaxf(mt, __shfl_xor(mt, 32, 64));
        const float mn = fmaxf(m, mt);
        const float alpha = (mn == -INFINITY) ? 1.f : exp2f(m - mn);
        float ls = 0.f;
#pragma unroll
        for (int kt = 0; kt < 4; ++kt)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float e = (mn == -INFINITY) ? 0.f : exp2f(s[kt][r] - mn);
                s[kt][r] = e;
                ls += e;
            }
        l = l * alpha + ls;
        m = mn;
#pragma unroll
        for (int d = 0; d < DT; ++d) o[d] *= alpha;
        // ---- O^T += V^T P^T, two 32-key steps
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            bf16x8 pf;
#pragma unroll
            for (int r = 0; r < 4; ++r) { pf[r] = (bf16)s[2 * ks][r]; pf[4 + r] = (bf16)s[2 * ks + 1][r]; }
            const int kr = 32 * ks + 4 * g + (li >> 2);
#pragma unroll
            for (int d = 0; d < DT; ++d) {
                const int dc = d * 16 + 4 * (li & 3);
                bf16x4 v0 = tr_read<RB>(vt_l, kr, dc);
                bf16x4 v1 = tr_read<RB>(vt_l, kr + 16, dc);
                bf16x8 vf;
                vf[0] = v0[0]; vf[1] = v0[1]; vf[2] = v0[2]; vf[3] = v0[3];
                vf[4] = v1[0]; vf[5] = v1[1]; vf[6] = v1[2]; vf[7] = v1[3];
                o[d] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pf, o[d], 0, 0, 0);
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }
    l += __shfl_xor(l, 16, 64);
    l += __shfl_xor(l, 32, 64);
    if (myq < p.S) {
        const float inv = 1.f / l;
        bf16* orow = p.o + (((int64_t)b * p.S + myq) * p.H + h) * p.hd;
#pragma unroll
        for (int d = 0; d < DT; ++d) {
            const int dd = d * 16 + 4 * g;
            if (dd < p.hd) {
                bf16x4 w;
#pragma unroll
                for (int r = 0; r < 4; ++r) w[r] = (bf16)(o[d][r] * inv);
                *(bf16x4*)(orow + dd) = w;
            }
        }
        if (g == 0 && p.lse) p.lse[((int64_t)b * p.H + h) * p.S + myq] = (m + log2f(l)) * 0.6931471805599453f;
    }
}

// ------------------------------------------------------------------ backward ----
struct AttnBwdP {
    const bf16* q; const bf16* k; const bf16* v;   // [B, heads, S, HDP]
    const bf16* dO;                                  // [B, S, H, hd]
    const float* lse; const float* delta;           // [B, H, S]
    float* dq;                                      // [B, H, S, HDP] fp32, pre-zeroed
    bf16* dk; bf16* dv;                             // [B, HKV, S, HDP]
    int B, H, HKV, S, hd;
    float scale, scale_log2;
};

// stage 32 rows x HDP of a [S][row_stride] matrix (hd real columns) into an LDS image
// [32][RB] swizzled with swK (register staging: 16-B loads, ds_write_b128)
template <int HDP>
__device__ __forceinline__ void stage_rows32(char* lds, const bf16* base, int64_t row_stride, int row0, int S,
                                             int ncols, int tid) {
    constexpr int RB = Geo<HDP>::RB, CH = RB / 16;
    for (int i = tid; i < 32 * CH; i += 256) {
        const int r = i / CH, c = i % CH;
        bf16x8 val = (bf16x8){};
        if (c * 8 < ncols && row0 + r < S) val = *(const bf16x8*)(base + (int64_t)(row0 + r) * row_stride + c * 8);
        *(bf16x8*)(lds + r * RB + ((c ^ swK<RB>(r)) << 4)) = val;
    }
}

// transposed read from a swK-swizzled image (rows r, 4 consecutive cols starting at d)
template <int RB>
__device__ __forceinline__ bf16x4 tr_read_k(const char* lds, int r, int d) {
    const int c = d >> 3;
    const char* a = lds + r * RB + ((c ^ swK<RB>(r)) << 4) + ((d & 4) << 1);
    return __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4_t*)a);
}

template <int HDP, bool CAUSAL>
__global__ void __launch_bounds__(256, 1) k_attn_bwd(AttnBwdP p) {
    constexpr int RB = Geo<HDP>::RB, KS = Geo<HDP>::KSTEPS, DT = Geo<HDP>::DT;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    char* lK = smem;                    // [64 keys][RB]  (swK image)
    char* lQ = lK + 64 * RB;            // [32 q][RB]
    char* lO = lQ + 32 * RB;            // [32 q][RB]    dO
    char* lS = lO + 32 * RB;            // [32 q][64 keys] bf16 dS, 128-B rows (swizzled)
    float* lL = (float*)(lS + 32 * 128);  // lse*log2e [32], delta [32]
    float* lD = lL + 32;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int g = lane >> 4, li = lane & 15;
    const int kb0 = blockIdx.x * 64;
    const int kvh = blockIdx.y, b = blockIdx.z;
    const int grp = p.H / p.HKV;
    const bf16* K = p.k + ((int64_t)(b * p.HKV + kvh) * p.S) * HDP;
    const bf16* V = p.v + ((int64_t)(b * p.HKV + kvh) * p.S) * HDP;
    const int mykey = kb0 + wid * 16 + li;

    // K image for the dQ product; K / V fragments (B operands) in registers
    stage_rows32<HDP>(lK, K, HDP, kb0, p.S, HDP, tid);
    stage_rows32<HDP>(lK + 32 * RB, K, HDP, kb0 + 32, p.S, HDP, tid);
    bf16x8 kf[KS], vf[KS];
#pragma unroll
    for (int kk = 0; kk < KS; ++kk) {
        if (mykey < p.S) {
            kf[kk] = *(const bf16x8*)(K + (int64_t)mykey * HDP + kk * 32 + 8 * g);
            vf[kk] = *(const bf16x8*)(V + (int64_t)mykey * HDP + kk * 32 + 8 * g);
        } else {
            kf[kk] = (bf16x8){}; vf[kk] = (bf16x8){};
        }
    }
    f32x4 dk[DT], dv[DT];
#pragma unroll
    for (int d = 0; d < DT; ++d) { dk[d] = (f32x4){0.f, 0.f, 0.f, 0.f}; dv[d] = dk[d]; }

    const int qt_first = CAUSAL ? (kb0 / 32) : 0;
    const int nqt = (p.S + 31) / 32;
    for (int hh = 0; hh < grp; ++hh) {
        const int h = kvh * grp + hh;
        const bf16* Q = p.q + ((int64_t)(b * p.H + h) * p.S) * HDP;
        const bf16* dO = p.dO + ((int64_t)b * p.S * p.H + h) * p.hd;  // row q at + q*H*hd
        const float* LSE = p.lse + ((int64_t)b * p.H + h) * p.S;
        const float* DEL = p.delta + ((int64_t)b * p.H + h) * p.S;
        float* dQ = p.dq + ((int64_t)(b * p.H + h) * p.S) * HDP;
        for (int qt = qt_first; qt < nqt; ++qt) {
            const int q0 = qt * 32;
            __syncthreads();  // previous iteration done with lQ/lO/lS
            stage_rows32<HDP>(lQ, Q, HDP, q0, p.S, HDP, tid);
            stage_rows32<HDP>(lO, dO, (int64_t)p.H * p.hd, q0, p.S, p.hd, tid);
            if (tid < 32) {
                const int q = q0 + tid;
                lL[tid] = q < p.S ? LSE[q] * 1.4426950408889634f : 0.f;
                lD[tid] = q < p.S ? DEL[q] : 0.f;
            }
            __syncthreads();
            // S = Q K^T, dP = dO V^T : rows q = 16qs + 4g + r, col = my key
            f32x4 s[2], dp[2];
#pragma unroll
            for (int qs = 0; qs < 2; ++qs) {
                s[qs] = (f32x4){0.f, 0.f, 0.f, 0.f};
                dp[qs] = s[qs];
#pragma unroll
                for (int kk = 0; kk < KS; ++kk) {
                    s[qs] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(k_frag<RB>(lQ, 16 * qs + li, kk * 4 + g), kf[kk], s[qs], 0, 0, 0);
                    dp[qs] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(k_frag<RB>(lO, 16 * qs + li, kk * 4 + g), vf[kk], dp[qs], 0, 0, 0);
                }
            }
            bf16x8 pfr, dsf;
#pragma unroll
            for (int qs = 0; qs < 2; ++qs)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int ql = 16 * qs + 4 * g + r, q = q0 + ql;
                    float pv = exp2f(s[qs][r] * p.scale_log2 - lL[ql]);
                    if (q >= p.S || mykey >= p.S || (CAUSAL && mykey > q)) pv = 0.f;
                    const float ds = pv * (dp[qs][r] - lD[ql]);
                    pfr[qs * 4 + r] = (bf16)pv;
                    dsf[qs * 4 + r] = (bf16)ds;
                    // dS -> LDS [q][key] (128-B rows, chunk swizzle on q)
                    const int key = wid * 16 + li;
                    const int ch = key >> 3;
                    *(bf16*)(lS + ql * 128 + (((ch ^ ((ql >> 1) & 7))) << 4) + (key & 7) * 2) = (bf16)ds;
                }
            // dV^T += dO^T P ; dK^T += Q^T dS   (A: transposed reads of the dO / Q images)
#pragma unroll
            for (int d = 0; d < DT; ++d) {
                const int dc = d * 16 + 4 * (li & 3);
                const int qr = 4 * g + (li >> 2);
                bf16x4 a0 = tr_read_k<RB>(lO, qr, dc), a1 = tr_read_k<RB>(lO, qr + 16, dc);
                bf16x8 af;
                af[0] = a0[0]; af[1] = a0[1]; af[2] = a0[2]; af[3] = a0[3];
                af[4] = a1[0]; af[5] = a1[1]; af[6] = a1[2]; af[7] = a1[3];
                dv[d] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, pfr, dv[d], 0, 0, 0);
                bf16x4 c0 = tr_read_k<RB>(lQ, qr, dc), c1 = tr_read_k<RB>(lQ, qr + 16, dc);
                bf16x8 cf;
                cf[0] = c0[0]; cf[1] = c0[1]; cf[2] = c0[2]; cf[3] = c0[3];
                cf[4] = c1[0]; cf[5] = c1[1]; cf[6] = c1[2]; cf[7] = c1[3];
                dk[d] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cf, dsf, dk[d], 0, 0, 0);
            }
            __syncthreads();
            // dQ[32 q][hd] += dS[32][64] K[64][hd]: 2 x DT output tiles over 4 waves
            for (int tix = wid; tix < 2 * DT; tix += 4) {
                const int qs = tix / DT, d = tix % DT;
                f32x4 acc = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int ks = 0; ks < 2; ++ks) {
                    const int qrow = 16 * qs + li;
                    const int ch = ks * 4 + g;
                    const bf16x8 af = *(const bf16x8*)(lS + qrow * 128 + ((ch ^ ((qrow >> 1) & 7)) << 4));
                    const int kr = 32 * ks + 8 * g + (li >> 2);   // B[k = key][col = d]
                    const int dc = d * 16 + 4 * (li & 3);
                    bf16x4 b0 = tr_read_k<RB>(lK, kr, dc), b1 = tr_read_k<RB>(lK, kr + 4, dc);
                    bf16x8 bf;
                    bf[0] = b0[0]; bf[1] = b0[1]; bf[2] = b0[2]; bf[3] = b0[3];
                    bf[4] = b1[0]; bf[5] = b1[1]; bf[6] = b1[2]; bf[7] = b1[3];
                    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bf, acc, 0, 0, 0);
                }
                const int dcol = d * 16 + li;
                if (dcol < p.hd) {
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int q = q0 + 16 * qs + 4 * g + r;
                        if (q < p.S) atomicAdd(dQ + (int64_t)q * HDP + dcol, acc[r] * p.scale);
                    }
                }
            }
        }
    }
    // write dK (scaled), dV: lane owns key = mykey, d = 16d + 4g + r
    if (mykey < p.S) {
        bf16* dKr = p.dk + ((int64_t)(b * p.HKV + kvh) * p.S + mykey) * HDP;
        bf16* dVr = p.dv + ((int64_t)(b * p.HKV + kvh) * p.S + mykey) * HDP;
#pragma unroll
        for (int d = 0; d < DT; ++d) {
            const int dd = d * 16 + 4 * g;
            bf16x4 wk, wv;
#pragma unroll
            for (int r = 0; r < 4; ++r) { wk[r] = (bf16)(dk[d][r] * p.scale); wv[r] = (bf16)dv[d][r]; }
            if (dd < HDP) { *(bf16x4*)(dKr + dd) = wk; *(bf16x4*)(dVr + dd) = wv; }
        }
    }
}

// delta[b,h,q] = sum_d dO[b,q,h,d] * O[b,q,h,d]
__global__ void k_attn_delta(const bf16* __restrict__ O, const bf16* __restrict__ dO, float* __restrict__ delta,
                             int B, int H, int S, int hd) {
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);   // one wave per (b, q, h)
    const int lane = threadIdx.x & 63;
    if (row >= B * S * H) return;
    const int h = row % H, bq = row / H, q = bq % S, b = bq / S;
    const bf16* o = O + (int64_t)row * hd;
    const bf16* d = dO + (int64_t)row * hd;
    float acc = 0.f;
    for (int i = lane; i < hd; i += 64) acc += (float)o[i] * (float)d[i];
    acc = wave_sum(acc);
    if (lane == 0) delta[((int64_t)b * H + h) * S + q] = acc;
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
    dim3 grid((d->S + 63) / 64, d->H, d->B);
    hipStream_t st = as_stream(stream_);
    const int rb = d->hdp == 64 ? 128 : 256;
    const size_t smem = 2 * 2 * 64 * rb;
#define LAUNCH(HD, C) hipLaunchKernelGGL((k_attn_fwd<HD, C>), grid, dim3(256), smem, st, p)
    if (d->hdp == 64) { if (d->causal) LAUNCH(64, true); else LAUNCH(64, false); }
    else if (d->hdp == 96) { if (d->causal) LAUNCH(96, true); else LAUNCH(96, false); }
    else { if (d->causal) LAUNCH(128, true); else LAUNCH(128, false); }
#undef LAUNCH
    KD_LAUNCH_CHECK("k_attn_fwd");
    return KD_OK;
}

int launch_attn_bwd(const kd_attn_bwd_desc* d, void* stream_) {
    KD_CHECK_ARG(d && d->q && d->k && d->v && d->o && d->dO && d->lse && d->delta && d->dq && d->dk && d->dv,
                 "attn_bwd: null pointer");
    KD_CHECK_SHAPE(d->H % d->HKV == 0 && d->hd % 4 == 0 && d->hd <= d->hdp, "attn_bwd: shape");
    KD_CHECK_SHAPE(d->hdp == 64 || d->hdp == 96 || d->hdp == 128, "attn_bwd: padded head dim must be 64/96/128");
    KD_CHECK_SHAPE(d->hd % 8 == 0, "attn_bwd: hd must be a multiple of 8 (16-B dO rows)");
    hipStream_t st = as_stream(stream_);
    {
        const int rows = d->B * d->S * d->H;
        hipLaunchKernelGGL(k_attn_delta, dim3((rows + 3) / 4), dim3(256), 0, st, (const bf16*)d->o,
                           (const bf16*)d->dO, d->delta, d->B, d->H, d->S, d->hd);
        KD_LAUNCH_CHECK("k_attn_delta");
    }
    if (hipMemsetAsync(d->dq, 0, (size_t)d->B * d->H * d->S * d->hdp * 4, st) != hipSuccess)
        return fail(KD_ERR_LAUNCH, "attn_bwd: memset dq");
    const double sc = 1.0 / std::sqrt((double)d->hd);
    AttnBwdP p{(const bf16*)d->q, (const bf16*)d->k, (const bf16*)d->v, (const bf16*)d->dO, d->lse, d->delta,
               d->dq, (bf16*)d->dk, (bf16*)d->dv, d->B, d->H, d->HKV, d->S, d->hd, (float)sc,
               (float)(sc * 1.4426950408889634)};
    dim3 grid((d->S + 63) / 64, d->HKV, d->B);
    const int rb = d->hdp == 64 ? 128 : 256;
    const size_t smem = 64 * rb + 32 * rb * 2 + 32 * 128 + 64 * 4;
#define LAUNCH(HD, C) hipLaunchKernelGGL((k_attn_bwd<HD, C>), grid, dim3(256), smem, st, p)
    if (d->hdp == 64) { if (d->causal) LAUNCH(64, true); else LAUNCH(64, false); }
    else if (d->hdp == 96) { if (d->causal) LAUNCH(96, true); else LAUNCH(96, false); }
    else { if (d->causal) LAUNCH(128, true); else LAUNCH(128, false); }
#undef LAUNCH
    KD_LAUNCH_CHECK("k_attn_bwd");
    return KD_OK;
}

}  // namespace kd
