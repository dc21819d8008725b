// Fused KD-loss forward+backward over [B*L, V] bf16 logits (HBM-bound).
//
// Replaces, in one launch sequence, the reference's per-step logit losses:
//   compute_loca_loss      DT:141-194 / LB:208-261   (KD_LOSS_LOCA)
//   compute_vision_loss KL DT:330-343                 (KD_LOSS_KL)
//   compute_loss KL(log_target=True) FB:205-219       (KD_LOSS_KL_LOGTARGET)
//   the in-model student CE (HF ForCausalLMLoss: shift by one, ignore -100, mean)
// and the autograd backward of all of them w.r.t. the student logits.
//
// Kernels (one row = one (b, l) position, grid-strided over rows; every lane keeps 4 / 2
// 16-B chunks of a row in flight so one workgroup's loads cover the HBM latency):
//   k_row_stats : one pass over teacher+student rows (256 threads per row) -> max /
//                 sum-exp at T and 1 (one exp per element when T = 1),
//                 teacher top-2 (LoCa "klogits", DT:170-171), gathers at the label;
//                 LoCa: records the LAST row-major position per label id and per
//                 klogit id (atomicMax) — the global last-write-wins semantics of
//                 `loca[:, :, labels] = X` (DT:184-185; SURVEY §4 KAT 1).
//   k_ovr_mask  : bitmask of overridden vocab columns and their override values q
//                 (LoCa only; one [V] table, so the per-row passes gather nothing).
//   k_loss_grad : pass A sums the KD term and the row scalar S, pass B writes
//                 dlogits; one 1024-thread workgroup per CU (256 rows in flight), so
//                 pass B's re-read of the row is served by the Infinity Cache.
//   k_finalize  : deterministic fp64 reduction of the per-row partials.
#include "common.h"

namespace kd {
namespace {

constexpr int NT = 256;  // threads per workgroup (row statistics, finalize)
constexpr int NW = NT / 64;
constexpr int RS_U = 4;  // 16-B chunks in flight per lane in k_row_stats
#ifndef KD_LG_NT        // tuning overrides (tools/gpu_loss_cfg.sh builds variants with -D)
#define KD_LG_NT 1024
#endif
#ifndef KD_LG_U
#define KD_LG_U 2
#endif
#ifndef KD_LG_ROWS
#define KD_LG_ROWS 256
#endif
constexpr int LG_NT = KD_LG_NT, LG_NW = LG_NT / 64;   // k_loss_grad: one 16-wave workgroup per CU
constexpr int LG_U = KD_LG_U;      // chunk pairs in flight per lane in k_loss_grad
constexpr int LG_ROWS = KD_LG_ROWS;   // rows in flight (workgroups) in k_loss_grad

struct RowStats {
    float mt, zt;     // teacher max over [0,V_s) and sum exp((t-mt)/T)
    float mtf, ztf;   // teacher max over [0,V_t) and sum exp(t-mtf)  (teacher CE)
    float ms, zs;     // student max and sum exp((s-ms)/T)
    float zs1;        // student sum exp(s-ms)
    float ce;         // student CE of this row (0 if no valid shifted label)
    float tce;        // teacher CE of this row
    float ovx, ovy;   // LoCa override values X = 1 - s(1-p_gt), Y = s p_k
    int i1, i2;       // teacher top-1 / top-2 index over [0,V_s)
    int lab;          // label at this position (LoCa gather index)
    int lab_next;     // shifted CE label (-100 => ignored)
    int valid;        // 1 if lab_next is a CE target
};
static_assert(sizeof(RowStats) == 64, "RowStats layout");

struct Layout {
    size_t stats, lab_last, klo_last, mask, ovr, part_kl, gran, err, total;
};

// k_loss_grad_loca_rr: RC 16-B chunks per lane and tensor (5: two 512-thread workgroups per CU, the
// default; 3: three, KD_LOSS_RR_C=3), so a slice is <= 512 RC chunks; granules sized for RC = 3
inline int rr_nsl(int V, int rc = 5) { const int nch = V / 8, sc = 512 * rc; return (nch + sc - 1) / sc; }

__host__ __device__ inline size_t align16(size_t x) { return (x + 15) & ~size_t(15); }

inline Layout make_layout(int B, int L, int V) {
    Layout lo{};
    const size_t rows = (size_t)B * L;
    size_t off = 0;
    lo.err = off;      off = align16(off + 16);   // error word first: kd_loss_check reads ws[0]
    lo.stats = off;    off = align16(off + rows * sizeof(RowStats));
    lo.lab_last = off; off = align16(off + (size_t)V * 4);
    lo.klo_last = off; off = align16(off + (size_t)V * 4);
    lo.mask = off;     off = align16(off + (size_t)((V + 63) / 64) * 8);
    lo.ovr = off;      off = align16(off + (size_t)V * 8);   // q [V], then log2 q [V]
    lo.part_kl = off;  off = align16(off + rows * 4);
    lo.gran = off;     off = align16(off + rows * (size_t)rr_nsl(V, 3) * 16);   // k_loss_grad_loca_rr hand-off granules
    lo.total = off;
    return lo;
}

// top2_push / top2_better: common.h

// merge an online (max, sum-exp-at-invT) pair
__device__ __forceinline__ void lse_merge(float& m, float& z, float m2, float z2, float invT) {
    if (m2 == -INFINITY) return;
    if (m == -INFINITY) { m = m2; z = z2; return; }
    if (m2 > m) { z = z * __expf((m - m2) * invT) + z2; m = m2; }
    else        { z = z + z2 * __expf((m2 - m) * invT); }
}

// error word of the workspace (kd_loss_check) and, when given, the caller's err_out
// (read asynchronously by the host): bits, first offending label and its row
__device__ __forceinline__ void report_label(int* err, int* err_ext, int bit, int64_t lab, int row) {
    atomicOr(err, 1);
    if (err_ext != nullptr) {
        atomicOr(err_ext, bit);
        if (atomicCAS(err_ext + 3, 0, 1) == 0) {
            err_ext[1] = (int)lab;
            err_ext[2] = row;
        }
    }
}

// Modes (RS_FULL: one pass over both logit tensors):
//  RS_PART  the per-row max / sum-exp / top-2 come from the lm_head GEMMs' epilogue partials
//           (kd_gemm_desc.row_stats: [rows, ceil(V / 256), 8] per model, merged with the same lse_merge /
//           top2_push as the wave reductions below) instead of a pass over both logit tensors; the label
//           gathers, the CE and the LoCa override values are unchanged (a few single-element reads).
//  RS_SONLY the student's {max, sum exp at 1/T, sum exp at 1} only, into s_aux [rows][4]
//           (kd_loss_student_stats: run on the student's stream right after its lm_head, beside the
//           teacher's last layers); T_ must be null.
//  RS_SPRE  the student's values read from s_aux (an RS_SONLY pass over the same rows): only the
//           teacher's logits are read here.  RS_SONLY runs the student loop and the reductions of
//           RS_FULL unchanged (the teacher's partials stay -inf / 0, which lse_merge skips), so the
//           statistics -- and the loss -- are the same bits as one RS_FULL pass.
enum { RS_FULL = 0, RS_PART = 1, RS_SONLY = 2, RS_SPRE = 3 };
template <int MODE>
__global__ void __launch_bounds__(NT)
k_row_stats(const bf16* __restrict__ T_, int64_t ld_t, int V_t,
            const bf16* __restrict__ S_, int64_t ld_s, int V_s,
            const int64_t* __restrict__ labels, int L, int rows,
            int variant, float invT, float alpha, int want_tce,
            RowStats* __restrict__ stats, int* __restrict__ lab_last,
            int* __restrict__ klo_last, int* __restrict__ err, int* __restrict__ err_ext, int row_base,
            const float* __restrict__ s_part, const float* __restrict__ t_part, float* __restrict__ s_aux) {
    constexpr bool PART = MODE == RS_PART;
    __shared__ float sm[NW * 8];
    __shared__ int si[NW * 2];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const bool has_t = MODE != RS_SONLY && (T_ != nullptr);
    for (int r = blockIdx.x; r < rows; r += gridDim.x) {
        const bf16* srow = S_ + (int64_t)r * ld_s;
        const bf16* trow = has_t ? T_ + (int64_t)r * ld_t : nullptr;
        float ms = -INFINITY, zs = 0.f, zs1 = 0.f;
        float mt = -INFINITY, zt = 0.f, mtf = -INFINITY, ztf = 0.f;
        float v1 = -INFINITY, v2 = -INFINITY;
        int i1 = 0x7fffffff, i2 = 0x7fffffff;
        if constexpr (PART) {
            // student tiles {max, sum at 1, max below V_s (= the same), sum at 1/T}; teacher tiles
            // {max over V_t, sum at 1, max over V_s, sum at 1/T, top-2}
            const int nts = (V_s + 255) / 256, ntt = (V_t + 255) / 256;
            for (int j = tid; j < nts; j += NT) {
                const f32x4 a = *(const f32x4*)(s_part + ((int64_t)r * nts + j) * 8);
                float mm = ms;
                lse_merge(ms, zs, a[2], a[3], invT);
                lse_merge(mm, zs1, a[0], a[1], 1.f);
            }
            if (has_t) {
                for (int j = tid; j < ntt; j += NT) {
                    const f32x4 a = *(const f32x4*)(t_part + ((int64_t)r * ntt + j) * 8);
                    const f32x4 c = *(const f32x4*)(t_part + ((int64_t)r * ntt + j) * 8 + 4);
                    lse_merge(mtf, ztf, a[0], a[1], 1.f);
                    lse_merge(mt, zt, a[2], a[3], invT);
                    top2_push(c[0], __float_as_int(c[1]), v1, i1, v2, i2);
                    top2_push(c[2], __float_as_int(c[3]), v1, i1, v2, i2);
                }
            }
        } else {
        // ---- student: max / sum-exp at T and at 1 (same max); RS_U chunks in flight per lane
        const bool t1 = invT == 1.f;   // T = 1 (LB): the two sums coincide, one exp per element
        if (MODE != RS_SPRE)
        for (int v0 = tid * 8; v0 < V_s; v0 += NT * 8 * RS_U) {
            bf16x8 xs[RS_U];
#pragma unroll
            for (int u = 0; u < RS_U; ++u) {
                const int v = v0 + u * NT * 8;
                if (v < V_s) xs[u] = *(const bf16x8*)(srow + v);
            }
#pragma unroll
            for (int u = 0; u < RS_U; ++u) {
                if (v0 + u * NT * 8 >= V_s) break;
                float f[8], cm = -INFINITY;
#pragma unroll
                for (int j = 0; j < 8; ++j) { f[j] = (float)xs[u][j]; cm = fmaxf(cm, f[j]); }
                if (cm > ms) {
                    if (ms != -INFINITY) { zs *= __expf((ms - cm) * invT); if (!t1) zs1 *= __expf(ms - cm); }
                    ms = cm;
                }
                if (t1) {
#pragma unroll
                    for (int j = 0; j < 8; ++j) zs += __expf(f[j] - ms);
                } else {
#pragma unroll
                    for (int j = 0; j < 8; ++j) { zs += __expf((f[j] - ms) * invT); zs1 += __expf(f[j] - ms); }
                }
            }
        }
        if (t1) zs1 = zs;
        // ---- teacher: max/sum over V_s at T, top-2 over V_s; max/sum over V_t at 1
        if (has_t) {
            // thr: the largest lane second-best of this wave so far, a lower bound of the row's
            // second-largest value (every lane's v2 is <= the row's top value's runner-up or ties
            // it), refreshed per outer step.  A chunk whose max is below it cannot hold a top-2
            // element, so once thr has risen (after a few hundred elements of random logits) the
            // whole wave skips the per-element insertion instead of running it whenever any one of
            // its 64 lanes has a candidate.  Elements equal to thr still go in (index tie-break).
            float thr = -INFINITY;
            for (int v0 = tid * 8; v0 < V_t; v0 += NT * 8 * RS_U) {
                bf16x8 xt[RS_U];
#pragma unroll
                for (int u = 0; u < RS_U; ++u) {
                    const int v = v0 + u * NT * 8;
                    if (v < V_t) xt[u] = *(const bf16x8*)(trow + v);
                }
#pragma unroll
                for (int u = 0; u < RS_U; ++u) {
                    const int v = v0 + u * NT * 8;
                    if (v >= V_t) break;
                    float f[8], cm = -INFINITY, cmf = -INFINITY;
                    const bool in_s = v < V_s;  // V_s % 8 == 0: chunks never straddle
#pragma unroll
                    for (int j = 0; j < 8; ++j) { f[j] = (float)xt[u][j]; cmf = fmaxf(cmf, f[j]); }
                    if (in_s) cm = cmf;
                    if (want_tce && t1) {
                        // T = 1: one exp per element feeds both sums, all relative to the V_t max;
                        // zt is rebased on the V_s max after the loop
                        if (cmf > mtf) {
                            if (mtf != -INFINITY) { const float sc = __expf(mtf - cmf); ztf *= sc; zt *= sc; }
                            mtf = cmf;
                        }
                        float e8 = 0.f;
#pragma unroll
                        for (int j = 0; j < 8; ++j) e8 += __expf(f[j] - mtf);
                        ztf += e8;
                        if (in_s) { zt += e8; mt = fmaxf(mt, cm); }
                    } else {
                        if (want_tce) {
                            if (cmf > mtf) { if (mtf != -INFINITY) ztf *= __expf(mtf - cmf); mtf = cmf; }
#pragma unroll
                            for (int j = 0; j < 8; ++j) ztf += __expf(f[j] - mtf);
                        }
                        if (in_s) {
                            if (cm > mt) { if (mt != -INFINITY) zt *= __expf((mt - cm) * invT); mt = cm; }
#pragma unroll
                            for (int j = 0; j < 8; ++j) zt += __expf((f[j] - mt) * invT);
                        }
                    }
                    if (in_s && cm >= thr) {
                        if (cm > v2 || (cm == v2 && v < i2)) {   // a chunk that can change the top-2
#pragma unroll
                            for (int j = 0; j < 8; ++j) top2_push(f[j], v + j, v1, i1, v2, i2);
                        }
                    }
                }
                float t2 = v2;
#pragma unroll
                for (int o = 32; o > 0; o >>= 1) t2 = fmaxf(t2, __shfl_xor(t2, o, 64));
                thr = t2;
            }
        }
        if (has_t && want_tce && t1 && mt != -INFINITY) zt *= __expf(mtf - mt);   // sum exp(t - mt) over V_s
        }

        // ---- wave reductions
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            float oms = __shfl_xor(ms, o, 64), ozs = __shfl_xor(zs, o, 64), ozs1 = __shfl_xor(zs1, o, 64);
            float m1 = ms, zz1 = zs1;
            lse_merge(ms, zs, oms, ozs, invT);
            lse_merge(m1, zz1, oms, ozs1, 1.f);
            zs1 = zz1;
            float omt = __shfl_xor(mt, o, 64), ozt = __shfl_xor(zt, o, 64);
            lse_merge(mt, zt, omt, ozt, invT);
            float omtf = __shfl_xor(mtf, o, 64), oztf = __shfl_xor(ztf, o, 64);
            lse_merge(mtf, ztf, omtf, oztf, 1.f);
            float ov1 = __shfl_xor(v1, o, 64), ov2 = __shfl_xor(v2, o, 64);
            int oi1 = __shfl_xor(i1, o, 64), oi2 = __shfl_xor(i2, o, 64);
            top2_push(ov1, oi1, v1, i1, v2, i2);
            top2_push(ov2, oi2, v1, i1, v2, i2);
        }
        __syncthreads();
        if (lane == 0) {
            sm[w * 8 + 0] = ms; sm[w * 8 + 1] = zs; sm[w * 8 + 2] = zs1;
            sm[w * 8 + 3] = mt; sm[w * 8 + 4] = zt; sm[w * 8 + 5] = mtf; sm[w * 8 + 6] = ztf;
            sm[w * 8 + 7] = v1; si[w * 2 + 0] = i1; si[w * 2 + 1] = i2;
        }
        // v2 of each wave kept in a second LDS slot set
        __shared__ float sv2[NW];
        if (lane == 0) sv2[w] = v2;
        __syncthreads();
        if (MODE == RS_SONLY) {
            if (tid == 0) {
                float Ms = sm[0], Zs = sm[1], Zs1 = sm[2];
                for (int k = 1; k < NW; ++k) {
                    float m1 = Ms, z1 = Zs1;
                    lse_merge(Ms, Zs, sm[k * 8 + 0], sm[k * 8 + 1], invT);
                    lse_merge(m1, z1, sm[k * 8 + 0], sm[k * 8 + 2], 1.f);
                    Zs1 = z1;
                }
                *(f32x4*)(s_aux + (int64_t)r * 4) = f32x4{Ms, Zs, Zs1, 0.f};
            }
            __syncthreads();
            continue;
        }
        if (tid == 0) {
            float Ms = sm[0], Zs = sm[1], Zs1 = sm[2], Mt = sm[3], Zt = sm[4], Mtf = sm[5], Ztf = sm[6];
            float V1 = sm[7], V2 = sv2[0];
            int I1 = si[0], I2 = si[1];
            for (int k = 1; k < NW; ++k) {
                float m1 = Ms, z1 = Zs1;
                lse_merge(Ms, Zs, sm[k * 8 + 0], sm[k * 8 + 1], invT);
                lse_merge(m1, z1, sm[k * 8 + 0], sm[k * 8 + 2], 1.f);
                Zs1 = z1;
                lse_merge(Mt, Zt, sm[k * 8 + 3], sm[k * 8 + 4], invT);
                lse_merge(Mtf, Ztf, sm[k * 8 + 5], sm[k * 8 + 6], 1.f);
                top2_push(sm[k * 8 + 7], si[k * 2 + 0], V1, I1, V2, I2);
                top2_push(sv2[k], si[k * 2 + 1], V1, I1, V2, I2);
            }
            if (MODE == RS_SPRE) {   // the student's statistics from kd_loss_student_stats
                const f32x4 a = *(const f32x4*)(s_aux + (int64_t)r * 4);
                Ms = a[0]; Zs = a[1]; Zs1 = a[2];
            }
            RowStats st;
            st.ms = Ms; st.zs = Zs; st.zs1 = Zs1;
            st.mt = Mt; st.zt = Zt; st.mtf = Mtf; st.ztf = Ztf;
            st.i1 = I1; st.i2 = I2;
            const int b = r / L, l = r - b * L;
            const int64_t lab = labels[r];
            const int64_t labn = (l + 1 < L) ? labels[r + 1] : -100;
            st.lab = (int)lab;
            st.lab_next = (int)labn;
            // student / teacher CE on the shifted label
            const bool labn_ok = (labn == -100) || (labn >= 0 && labn < V_s);
            if (!labn_ok) report_label(err, err_ext, 2, labn, r + 1 + row_base);
            st.valid = (labn >= 0 && labn < V_s) ? 1 : 0;
            st.ce = 0.f; st.tce = 0.f;
            if (st.valid) {
                const float sl = (float)srow[labn];
                st.ce = logf(Zs1) + Ms - sl;
                if (has_t && want_tce) st.tce = logf(Ztf) + Mtf - (float)trow[labn];
            }
            st.ovx = 0.f; st.ovy = 0.f;
            if (variant == KD_LOSS_LOCA) {
                if (lab < 0 || lab >= V_s) {
                    report_label(err, err_ext, 1, lab, r + row_base);  // reference: gather out of bounds (DT:166)
                } else {
                    // p_gt, p_k (DT:166, :174), sigma, s (DT:177-180)
                    const float p_gt = __expf(((float)trow[lab] - Mt) * invT) / Zt;
                    const float p_k = __expf((V2 - Mt) * invT) / Zt;
                    const float sigma = 1.f / (1.f - p_gt + p_k);
                    const float sc = alpha * sigma;
                    // X = 1 - s*(sum(p_T) - p_gt) with sum(p_T) = 1 (DT:184)
                    st.ovx = 1.f - sc * (1.f - p_gt);
                    st.ovy = sc * p_k;  // DT:185
                    atomicMax(&lab_last[lab], r);
                    atomicMax(&klo_last[I2], r);
                }
            }
            stats[r] = st;
        }
        __syncthreads();
    }
}

__global__ void k_ovr_mask(const int* __restrict__ lab_last, const int* __restrict__ klo_last,
                           const RowStats* __restrict__ stats, int V, unsigned long long* __restrict__ mask,
                           float* __restrict__ ovr) {
    const int v = blockIdx.x * blockDim.x + threadIdx.x;
    const int kl = v < V ? klo_last[v] : -1, ll = v < V ? lab_last[v] : -1;
    const bool on = kl >= 0 || ll >= 0;
    const unsigned long long bits = __ballot(on);
    // word k exists iff 64k < V (a "v < V + 63" bound wrote one word past the table when
    // 64 | V, into ovr[0..1], racing with the block that owns them)
    if ((threadIdx.x & 63) == 0 && v < V) mask[v >> 6] = bits;
    // klogits are written second (DT:185) and win over the label columns (DT:184)
    // {q, log2 q} with log2 q := 0 for q <= 0 (the KL term's 0 * log 0 = 0; a negative
    // override contributes -q log c only, as in the generic path)
    if (v < V) {
        const float q = kl >= 0 ? stats[kl].ovy : (ll >= 0 ? stats[ll].ovx : 0.f);
        // NaN marks a column without an override (the LoCa fast path's select)
        ovr[v] = on ? q : __builtin_nanf("");
        ovr[V + v] = q > 0.f ? __log2f(q) : 0.f;
    }
}

template <int VARIANT>
__device__ __forceinline__ void
loss_grad_body(const bf16* __restrict__ T_, int64_t ld_t,
            const bf16* __restrict__ S_, int64_t ld_s, int V,
            int rows, float invT, float clamp_min,
            const RowStats* __restrict__ stats,
            const float* __restrict__ ovr,
            const unsigned long long* __restrict__ mask_g,
            float kd_coef,   // kd_weight * T / N * grad_scale
            float ce_coef,   // ce_weight / n_valid * grad_scale   (host-computed count)
            bf16* __restrict__ D_, int64_t ld_d, float* __restrict__ part_kl,
            unsigned long long* smask, float* red) {
    const int tid = threadIdx.x;
    const int nwords = (V + 63) / 64;
    if (VARIANT == KD_LOSS_LOCA) {
        for (int i = tid; i < nwords; i += LG_NT) smask[i] = mask_g[i];
        __syncthreads();
    }
    const float log_clamp = logf(clamp_min);
    for (int r = blockIdx.x; r < rows; r += gridDim.x) {
        const RowStats st = stats[r];
        const bf16* srow = S_ + (int64_t)r * ld_s;
        const bf16* trow = (VARIANT != KD_LOSS_NONE) ? T_ + (int64_t)r * ld_t : nullptr;
        const float log_zs = logf(st.zs);
        const float inv_zt = (VARIANT != KD_LOSS_NONE) ? 1.f / st.zt : 0.f;
        const float log_zt = (VARIANT != KD_LOSS_NONE) ? logf(st.zt) : 0.f;
        float Ssum = 0.f;
        if (VARIANT != KD_LOSS_NONE) {
            // ---- pass A: KD term and S
            float term = 0.f, sacc = 0.f;
            for (int v0 = tid * 8; v0 < V; v0 += LG_NT * 8 * LG_U) {
              bf16x8 xtu[LG_U], xsu[LG_U];
#pragma unroll
              for (int u = 0; u < LG_U; ++u) {
                  const int v = v0 + u * LG_NT * 8;
                  if (v < V) { xtu[u] = *(const bf16x8*)(trow + v); xsu[u] = *(const bf16x8*)(srow + v); }
              }
#pragma unroll
              for (int u = 0; u < LG_U; ++u) {
                const int v = v0 + u * LG_NT * 8;
                if (v >= V) break;
                const bf16x8 xt = xtu[u], xs = xsu[u];
                unsigned int mbits = 0;
                if (VARIANT == KD_LOSS_LOCA) mbits = (unsigned)(smask[v >> 6] >> (v & 63)) & 0xffu;
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const float lt = ((float)xt[j] - st.mt) * invT;  // log-space teacher (unnormalised)
                    const float pT = __expf(lt) * inv_zt;
                    const float lps = ((float)xs[j] - st.ms) * invT - log_zs;
                    if (VARIANT == KD_LOSS_LOCA) {
                        float q = pT, logq = lt - log_zt;
                        if (mbits & (1u << j)) {
                            q = ovr[v + j];
                            logq = logf(q);
                        }
                        const float ps = __expf(lps);
                        const bool unc = ps >= clamp_min;
                        const float logc = unc ? lps : log_clamp;
                        term += (q > 0.f ? q * logq : 0.f) - q * logc;
                        sacc += unc ? q : 0.f;
                    } else if (VARIANT == KD_LOSS_KL) {
                        term += (pT > 0.f ? pT * (lt - log_zt) : 0.f) - pT * lps;
                        sacc += pT;
                    } else {  // KL_LOGTARGET quirk: exp(p_T) * (p_T - log p_S)
                        const float e = __expf(pT);
                        term += e * (pT - lps);
                        sacc += e;
                    }
                }
              }
            }
            term = block_sum<LG_NW>(term, red);
            Ssum = block_sum<LG_NW>(sacc, red);
            if (tid == 0) part_kl[r] = term;
        } else {
            if (tid == 0) part_kl[r] = 0.f;
        }
        if (D_ != nullptr) {
            // ---- pass B: dlogits
            const float log_zs1 = logf(st.zs1);
            const bool t1 = invT == 1.f && st.zs1 == st.zs;   // the CE softmax == the KD softmax at T = 1
            const float cec = st.valid ? ce_coef : 0.f;
            bf16* drow = D_ + (int64_t)r * ld_d;
            for (int v0 = tid * 8; v0 < V; v0 += LG_NT * 8 * LG_U) {
              bf16x8 xsu[LG_U], xtu[LG_U];
#pragma unroll
              for (int u = 0; u < LG_U; ++u) {
                  const int v = v0 + u * LG_NT * 8;
                  if (v < V) {
                      xsu[u] = *(const bf16x8*)(srow + v);
                      if (VARIANT != KD_LOSS_NONE) xtu[u] = *(const bf16x8*)(trow + v);
                  }
              }
#pragma unroll
              for (int u = 0; u < LG_U; ++u) {
                const int v = v0 + u * LG_NT * 8;
                if (v >= V) break;
                const bf16x8 xs = xsu[u];
                bf16x8 xt;
                if (VARIANT != KD_LOSS_NONE) xt = xtu[u];
                unsigned int mbits = 0;
                if (VARIANT == KD_LOSS_LOCA) mbits = (unsigned)(smask[v >> 6] >> (v & 63)) & 0xffu;
                bf16x8 out;
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const float sv = (float)xs[j];
                    float g = 0.f, ps_keep = 0.f;
                    if (VARIANT != KD_LOSS_NONE) {
                        const float lt = ((float)xt[j] - st.mt) * invT;
                        const float pT = __expf(lt) * inv_zt;
                        const float ps = __expf((sv - st.ms) * invT - log_zs);
                        ps_keep = ps;
                        float gq;
                        if (VARIANT == KD_LOSS_LOCA) {
                            float q = pT;
                            if (mbits & (1u << j)) q = ovr[v + j];
                            gq = (ps >= clamp_min) ? q : 0.f;
                        } else if (VARIANT == KD_LOSS_KL) {
                            gq = pT;
                        } else {
                            gq = __expf(pT);
                        }
                        g = kd_coef * (ps * Ssum - gq);
                    }
                    if (cec != 0.f) {
                        const float p1 = (VARIANT != KD_LOSS_NONE && t1) ? ps_keep : __expf(sv - st.ms - log_zs1);
                        g += cec * (p1 - ((v + j) == st.lab_next ? 1.f : 0.f));
                    }
                    out[j] = (bf16)g;
                }
                *(bf16x8*)(drow + v) = out;
              }
            }
        }
    }
}

// LoCa fast path: the per-element arithmetic in base-2 log space with per-row constants
// (the generic body above spends ~35 VALU + 3 exps per element in pass A and ~28 + 3 in
// pass B, which made the kernel VALU-bound, not HBM-bound):
//   lq = t*a - cq = log2 p_T,   lps = s*a - cs = log2 p_S,   a = log2(e) / T
//   log2 c = max(lps, log2 clamp)   (c = clamp(p_S, min=1e-8), DT:162);  unc = lps >= log2 clamp
//   pass A: term2 += q (log2 q - log2 c),  S += unc ? q : 0      (term = ln 2 * term2)
//   pass B: g = kd_coef (p_S S - unc q) + cec (p1 - onehot),  p1 = p_S when T = 1
// Overridden columns (LoCa's `loca[:, :, labels] = X` / klogits, DT:184-185) take q and
// log2 q from the table (NaN = not overridden); a chunk loads it only when its mask byte
// is set.  The CE's one-hot (one element per row) is rewritten after pass B by the lane
// that owns it, with the same arithmetic.
constexpr float KD_LOG2E = 1.4426950408889634f;
constexpr float KD_LN2 = 0.6931471805599453f;

__device__ __forceinline__ float ex2(float x) { return __builtin_amdgcn_exp2f(x); }

__device__ __forceinline__ void bf16x8_to_f32(const bf16x8& x, float* f) {
    const u32x4 u = __builtin_bit_cast(u32x4, x);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        f[2 * k] = __uint_as_float(u[k] << 16);
        f[2 * k + 1] = __uint_as_float(u[k] & 0xffff0000u);
    }
}

struct LocaRow {
    float a, cq, cs, cqk, c1, K, cec, lcl, kd_coef;
};

// pass B's gradient of one element from kd_coef * q (also the one-hot fix-up: identical
// arithmetic)
template <bool T1>
__device__ __forceinline__ float loca_grad(const LocaRow& R, float qk, float s) {
    const float lps = fmaf(s, R.a, -R.cs);
    float g = fmaf(ex2(lps), R.K, lps >= R.lcl ? -qk : 0.f);
    if (!T1) g = fmaf(ex2(fmaf(s, KD_LOG2E, -R.c1)), R.cec, g);
    return g;
}

template <bool T1>
__global__ void __launch_bounds__(LG_NT)
k_loss_grad_loca(const bf16* __restrict__ T_, int64_t ld_t, const bf16* __restrict__ S_, int64_t ld_s,
                 int V, int rows, float invT, float clamp_min, const RowStats* __restrict__ stats,
                 const float* __restrict__ ovr, const unsigned long long* __restrict__ mask_g,
                 const float* __restrict__ coefs, bf16* __restrict__ D_, int64_t ld_d,
                 float* __restrict__ part_kl) {
    extern __shared__ __attribute__((aligned(16))) unsigned long long smask[];
    __shared__ float red[LG_NW];
    const float ce_coef = coefs[1], kd_coef = coefs[2];   // both / the stored dlogits scale
    const int tid = threadIdx.x;
    const int nwords = (V + 63) / 64;
    for (int i = tid; i < nwords; i += LG_NT) smask[i] = mask_g[i];
    __syncthreads();
    LocaRow R;
    R.a = invT * KD_LOG2E;
    R.lcl = log2f(clamp_min);
    R.kd_coef = kd_coef;
    const float lk = kd_coef > 0.f ? log2f(kd_coef) : -INFINITY;   // q * kd_coef = 2^(lq + lk)
    for (int r = blockIdx.x; r < rows; r += gridDim.x) {
        const RowStats st = stats[r];
        const bf16* srow = S_ + (int64_t)r * ld_s;
        const bf16* trow = T_ + (int64_t)r * ld_t;
        R.cq = (st.mt * invT + logf(st.zt)) * KD_LOG2E;
        R.cs = (st.ms * invT + logf(st.zs)) * KD_LOG2E;
        // ---- pass A: KD term and S (element pairs in packed fp32: v_pk_fma / v_pk_add)
        typedef __attribute__((ext_vector_type(2))) float f32x2;
        const f32x2 a2 = {R.a, R.a}, cq2 = {R.cq, R.cq}, cs2 = {R.cs, R.cs};
        f32x2 term2 = {0.f, 0.f}, sacc2 = {0.f, 0.f};
        for (int v0 = tid * 8; v0 < V; v0 += LG_NT * 8 * LG_U) {
            bf16x8 xtu[LG_U], xsu[LG_U];
#pragma unroll
            for (int u = 0; u < LG_U; ++u) {
                const int v = v0 + u * LG_NT * 8;
                if (v < V) { xtu[u] = *(const bf16x8*)(trow + v); xsu[u] = *(const bf16x8*)(srow + v); }
            }
#pragma unroll
            for (int u = 0; u < LG_U; ++u) {
                const int v = v0 + u * LG_NT * 8;
                if (v >= V) break;
                float t[8], sv[8], lq[8], q[8], lps[8];
                bf16x8_to_f32(xtu[u], t);
                bf16x8_to_f32(xsu[u], sv);
#pragma unroll
                for (int j = 0; j < 8; j += 2) {
                    const f32x2 lq2 = f32x2{t[j], t[j + 1]} * a2 - cq2;
                    const f32x2 lp2 = f32x2{sv[j], sv[j + 1]} * a2 - cs2;
                    lq[j] = lq2.x; lq[j + 1] = lq2.y;
                    lps[j] = lp2.x; lps[j + 1] = lp2.y;
                    q[j] = ex2(lq[j]);
                    q[j + 1] = ex2(lq[j + 1]);
                }
                if ((smask[v >> 6] >> (v & 63)) & 0xffu) {   // V % 8 == 0: aligned 16-B table loads
                    const f32x4 o0 = *(const f32x4*)(ovr + v), o1 = *(const f32x4*)(ovr + v + 4);
                    const f32x4 l0 = *(const f32x4*)(ovr + V + v), l1 = *(const f32x4*)(ovr + V + v + 4);
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        const float o = j < 4 ? o0[j] : o1[j - 4];
                        const bool on = o == o;
                        q[j] = on ? o : q[j];
                        lq[j] = on ? (j < 4 ? l0[j] : l1[j - 4]) : lq[j];
                    }
                }
#pragma unroll
                for (int j = 0; j < 8; j += 2) {
                    const f32x2 q2 = {q[j], q[j + 1]};
                    const f32x2 lc2 = {fmaxf(lps[j], R.lcl), fmaxf(lps[j + 1], R.lcl)};
                    term2 = q2 * (f32x2{lq[j], lq[j + 1]} - lc2) + term2;
                    sacc2 += f32x2{lps[j] >= R.lcl ? q[j] : 0.f, lps[j + 1] >= R.lcl ? q[j + 1] : 0.f};
                }
            }
        }
        const float term = block_sum<LG_NW>(term2.x + term2.y, red);
        const float Ssum = block_sum<LG_NW>(sacc2.x + sacc2.y, red);
        if (tid == 0) part_kl[r] = term * KD_LN2;
        if (D_ == nullptr) continue;
        // ---- pass B: dlogits
        R.cec = st.valid ? ce_coef : 0.f;
        R.K = kd_coef * Ssum + (T1 ? R.cec : 0.f);
        R.cqk = R.cq - lk;
        R.c1 = (st.ms + logf(st.zs1)) * KD_LOG2E;
        bf16* drow = D_ + (int64_t)r * ld_d;
        for (int v0 = tid * 8; v0 < V; v0 += LG_NT * 8 * LG_U) {
            bf16x8 xtu[LG_U], xsu[LG_U];
#pragma unroll
            for (int u = 0; u < LG_U; ++u) {
                const int v = v0 + u * LG_NT * 8;
                if (v < V) { xsu[u] = *(const bf16x8*)(srow + v); xtu[u] = *(const bf16x8*)(trow + v); }
            }
#pragma unroll
            for (int u = 0; u < LG_U; ++u) {
                const int v = v0 + u * LG_NT * 8;
                if (v >= V) break;
                float t[8], sv[8], qk[8];
                bf16x8_to_f32(xtu[u], t);
                bf16x8_to_f32(xsu[u], sv);
#pragma unroll
                for (int j = 0; j < 8; ++j) qk[j] = ex2(fmaf(t[j], R.a, -R.cqk));
                if ((smask[v >> 6] >> (v & 63)) & 0xffu) {
                    const f32x4 o0 = *(const f32x4*)(ovr + v), o1 = *(const f32x4*)(ovr + v + 4);
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        const float o = j < 4 ? o0[j] : o1[j - 4];
                        qk[j] = o == o ? o * kd_coef : qk[j];
                    }
                }
                bf16x8 out;
#pragma unroll
                for (int j = 0; j < 8; ++j) out[j] = (bf16)loca_grad<T1>(R, qk[j], sv[j]);
                *(bf16x8*)(drow + v) = out;
            }
        }
        // the CE one-hot: the lane that wrote labn's chunk rewrites that element (program
        // order makes its second store land after the first)
        const int labn = st.lab_next;
        if (st.valid && ((labn >> 3) & (LG_NT - 1)) == tid) {
            float qk = ex2(fmaf((float)trow[labn], R.a, -R.cqk));
            if ((smask[labn >> 6] >> (labn & 63)) & 1ull) qk = ovr[labn] * kd_coef;
            const float g = loca_grad<T1>(R, qk, (float)srow[labn]);
            drow[labn] = (bf16)(g - R.cec);
        }
    }
}

// Register-resident LoCa (round 4): k_loss_grad_loca reads every row twice (pass A for S,
// pass B for dlogits) and the second read missed the caches (rocprofv3 FETCH_SIZE 2.08x the two
// logit tensors: a row is 608 KB, far above a CU's share of its XCD's 4 MB L2).  Here a row is
// cut into nsl column slices of <= RR_NT * RR_C 16-B chunks per tensor, one per workgroup, and
// each lane keeps its RR_C chunks of the teacher and of the student row in REGISTERS between
// the passes, so HBM sees one read of each logit tensor and one write of dlogits (two 512-thread
// workgroups per CU, 160 KB of loads in flight; holding the next row in a second register set
// instead leaves one workgroup per CU and measured 2.0x slower: too few waves for the VALU).  The slices
// of a row exchange their pass-A partials (KD term, S) through 8-B granules {tag, value} stored
// write-through at agent scope (cdna_hip_programming.md §6 G16 R2: no fence, no flag); every
// slice sums the nsl partials in slice order, so all of a row's workgroups use the same S.
// The grid is nsl x (resident workgroups / nsl) persistent workgroups (row groups stride the rows),
// so on an idle GPU all of a row's slices run together.  Correctness does not depend on it: a slice
// polls its partners' granules for a bounded time (rr_poll_ticks) and then computes any absent
// partial itself -- the same body (pass_a) over the same chunks with the same lane mapping and
// reduction order, so the same bits the absent slice stores -- and reloads its own chunks.  When
// other work holds CUs (a concurrent stream, a CU mask) the kernel slows down; it never waits on a
// workgroup that is not running and never fails.
// Same per-element arithmetic as k_loss_grad_loca; the row sums differ in fp32 order only.
// Round 5: the LoCa override values of a slice's masked chunks (q and log2 q: one table for the whole
// launch, a lane's chunks fixed) are copied once into an LDS image (<= ov_cap 64-B slots; a slice with
// more reads the global table as before), so the per-row passes issue no override-table loads on the
// in-order vector-memory counter (c1 loss 2361-2382 -> 2115-2156 us, the same bits); with them gone,
// pass B loads chunk j of the row group's next row as soon as chunk j is computed (-1 %), the CE
// one-hot then applied inside its chunk (the same arithmetic as the separate rewrite, the same bits).
constexpr int RR_NT = 512, RR_NW = RR_NT / 64;
constexpr int RR_C = 5;                                   // 16-B chunks of each tensor per lane per row (max)
constexpr int RR_SLICE = RR_NT * RR_C;                    // max chunks per slice
constexpr int RR_MAX_SL = 16;                             // slices per row (V <= 327,680)
constexpr int RR_MASK_W = RR_SLICE * 8 / 64 + 2;          // mask words a slice spans
typedef __attribute__((address_space(1))) unsigned long long gu64;

__device__ __forceinline__ void gran_store(unsigned long long* p, float v) {
    __hip_atomic_store((gu64*)p, (1ull << 32) | __float_as_uint(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long gran_load(const unsigned long long* p) {
    return __hip_atomic_load((const gu64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t slice_rsrc(const void* base, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}

#ifdef KD_AB_BUILD
// KD_RR_STAMPS=1 (A/B build): wave 0 of every workgroup adds its s_memtime cycles per phase of a row
// (loads + pass A, block sums, hand-off, pass B + stores, rows) to rr_stamps[block][8]
__device__ unsigned long long rr_stamps[4096 * 8];
#define KD_RR_STAMP(k, v) do { if (stamp && wid == 0 && lane == 0) atomicAdd(&rr_stamps[blockIdx.x * 8 + (k)], (v)); } while (0)
#else
#define KD_RR_STAMP(k, v) do { } while (0)
#endif
template <bool T1, int RC>
__global__ void __launch_bounds__(RR_NT, RC >= 5 ? 4 : 6)
k_loss_grad_loca_rr(const bf16* __restrict__ T_, int64_t ld_t, const bf16* __restrict__ S_, int64_t ld_s,
                    int V, int rows, float invT, float clamp_min, const RowStats* __restrict__ stats,
                    const float* __restrict__ ovr, const unsigned long long* __restrict__ mask_g,
                    const float* __restrict__ coefs, bf16* __restrict__ D_, int64_t ld_d,
                    float* __restrict__ part_kl, int nsl, int cps, int n_rg,
                    unsigned long long* __restrict__ gran, uint32_t poll_ticks, int stamp, int ov_cap, int pf,
                    int* __restrict__ standin_count) {
#ifndef KD_AB_BUILD
    stamp = 0;   // the product build carries no stamps (every stamp branch folds away)
#endif
    // the slice's override values (q and log2 q of every overridden column of the lane's chunks), in
    // LDS: ov_cap 64-B slots, one per chunk with a set mask byte, in (chunk j, wave, lane) order
    extern __shared__ __attribute__((aligned(16))) f32x4 ov_img[];
    __shared__ int wcnt[RC * RR_NW];
    __shared__ unsigned long long smask[RR_MASK_W];
    __shared__ float red[2 * RR_NW];
    __shared__ float row_sums[2];
    __shared__ float gv[2 * RR_MAX_SL];   // the row's slice partials, slice order
    __shared__ int miss_s;                // slices whose partials did not arrive within poll_ticks
    const float ce_coef = coefs[1], kd_coef = coefs[2];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    // the plain mapping: a row group's nsl slices are consecutive workgroups (so, dealt round-robin, on
    // nsl different XCDs).  Placing them on one XCD (round 5) measured SLOWER: k_loss_grad_loca_rr
    // 1812 us vs 1508-1536 us at c1 (profiles/r05), with 4 more VGPRs spilled.  A per-slice compacted
    // LDS copy of the override values costs 25-30 VGPRs in each pass body and spilled 51-65 VGPRs at the
    // 128-VGPR bound of two 512-thread workgroups per CU; neither is kept.
    const int sl = (int)(blockIdx.x % (unsigned)nsl), rg = (int)(blockIdx.x / (unsigned)nsl);
    const int c_lo = sl * cps, c_hi = min(V >> 3, c_lo + cps);   // this workgroup's chunks [c_lo, c_hi)
    const int w_lo = (c_lo * 8) >> 6;
    const uint32_t vo = (uint32_t)tid * 16;
    for (int i = tid; i < RR_MASK_W; i += RR_NT) {
        const int w = w_lo + i;
        smask[i] = w < ((V + 63) >> 6) ? mask_g[w] : 0ull;
    }
    __syncthreads();
    // the override mask is one table for the whole launch and the slice is fixed per
    // workgroup: a lane's RC mask bytes, once
    // per chunk j a 12-bit field of mb: bit 0 = its mask byte is set, bits 1-11 = its override-image slot
    uint64_t mb = 0;
#pragma unroll
    for (int j = 0; j < RC; ++j) {
        const int c = c_lo + tid + j * RR_NT;
        if (c < c_hi && ((smask[((c * 8) >> 6) - w_lo] >> ((c * 8) & 63)) & 0xffull)) mb |= 1ull << (12 * j);
    }
    // the override image: the masked chunks' slots (base of this wave's run for chunk j + the lane's
    // rank among the wave's masked lanes), filled once -- the table is one for the whole launch and a
    // lane's chunks are fixed, so every row reads the same values.  With it the per-row passes issue
    // no override-table loads on the vector-memory counter, which retires in order: the next row's
    // chunks can be loaded during pass B without every table wait also waiting for them.  A slice
    // with more masked chunks than ov_cap reads the table from global memory, as before.
    {
        uint64_t bal[RC];
#pragma unroll
        for (int j = 0; j < RC; ++j) {
            bal[j] = __ballot((mb >> (12 * j)) & 1u);
            if (lane == 0) wcnt[j * RR_NW + wid] = __popcll(bal[j]);
        }
        __syncthreads();
        int nmask = 0;
#pragma unroll
        for (int j = 0; j < RC; ++j)
            for (int w = 0; w < RR_NW; ++w) {
                if (w == wid && ((mb >> (12 * j)) & 1u)) {
                    const int slot = nmask + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(bal[j] >> 32),
                                                                           __builtin_amdgcn_mbcnt_lo((uint32_t)bal[j], 0u));
                    mb |= (uint64_t)(slot & 2047) << (12 * j + 1);
                }
                nmask += wcnt[j * RR_NW + w];
            }
        if (nmask > ov_cap) ov_cap = -1;   // uniform: every thread summed the same counts
    }
    const bool use_lds = ov_cap >= 0;
    auto oslot = [&](int j) { return (int)((mb >> (12 * j + 1)) & 2047u); };
    if (use_lds) {
#pragma unroll
        for (int j = 0; j < RC; ++j)
            if ((mb >> (12 * j)) & 1u) {
                const int v = (c_lo + tid + j * RR_NT) * 8;
                f32x4* o = ov_img + 4 * oslot(j);
                o[0] = *(const f32x4*)(ovr + v);
                o[1] = *(const f32x4*)(ovr + v + 4);
                o[2] = *(const f32x4*)(ovr + V + v);
                o[3] = *(const f32x4*)(ovr + V + v + 4);
            }
        __syncthreads();
    }
    using LdsT = std::integral_constant<bool, true>;
    using GlbT = std::integral_constant<bool, false>;
    LocaRow R;
    R.a = invT * KD_LOG2E;
    R.lcl = log2f(clamp_min);
    R.kd_coef = kd_coef;
    const float lk = kd_coef > 0.f ? log2f(kd_coef) : -INFINITY;
    typedef __attribute__((ext_vector_type(2))) float f32x2;
    typedef bf16x8 Set[RC];
    // chunks [lo, hi) of row r (this lane's: lo + tid + j RR_NT) through buffer descriptors (SGPRs)
    // and ONE lane offset: out-of-slice chunks read zeros (never used); 64-bit per-chunk addresses
    // hoisted out of the row loop spilled
    auto load = [&](Set& xt, Set& xs, int r, int lo, int hi) {
        const uint32_t nb = (uint32_t)(hi - lo) * 16;
        const __amdgpu_buffer_rsrc_t rT = slice_rsrc(T_ + (int64_t)r * ld_t + lo * 8, nb);
        const __amdgpu_buffer_rsrc_t rS = slice_rsrc(S_ + (int64_t)r * ld_s + lo * 8, nb);
#pragma unroll
        for (int j = 0; j < RC; ++j) {
            xt[j] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rT, vo, j * RR_NT * 16, 0));
            xs[j] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rS, vo, j * RR_NT * 16, 0));
        }
    };
    // pass A (k_loss_grad_loca's arithmetic) over the chunks [lo, hi) held in (xt, xs), mask bytes mbx:
    // the lane's KD-term and S partials.  The ONE body both a slice's own partial and a stand-in's
    // recomputation of it run, so both give the same bits.
    auto pass_a = [&](const Set& xt, const Set& xs, int lo, int hi, uint64_t mbx, auto lds_tag, f32x2& term2, f32x2& sacc2) {
        constexpr bool lds = decltype(lds_tag)::value;
        const f32x2 a2 = {R.a, R.a}, cq2 = {R.cq, R.cq}, cs2 = {R.cs, R.cs};
        term2 = f32x2{0.f, 0.f};
        sacc2 = f32x2{0.f, 0.f};
#pragma unroll
        for (int j = 0; j < RC; ++j) {
            const int c = lo + tid + j * RR_NT;
            if (c >= hi) break;
            const int v = c * 8;
            float t[8], sv[8], lq[8], q[8], lps[8];
            bf16x8_to_f32(xt[j], t);
            bf16x8_to_f32(xs[j], sv);
#pragma unroll
            for (int k = 0; k < 8; k += 2) {
                const f32x2 lq2 = f32x2{t[k], t[k + 1]} * a2 - cq2;
                const f32x2 lp2 = f32x2{sv[k], sv[k + 1]} * a2 - cs2;
                lq[k] = lq2.x; lq[k + 1] = lq2.y;
                lps[k] = lp2.x; lps[k + 1] = lp2.y;
                q[k] = ex2(lq[k]);
                q[k + 1] = ex2(lq[k + 1]);
            }
            if ((mbx >> (12 * j)) & 1u) {
                f32x4 o0, o1, l0, l1;
                if constexpr (lds) {
                    const f32x4* o = ov_img + 4 * oslot(j);
                    o0 = o[0]; o1 = o[1]; l0 = o[2]; l1 = o[3];
                } else {
                    o0 = *(const f32x4*)(ovr + v); o1 = *(const f32x4*)(ovr + v + 4);
                    l0 = *(const f32x4*)(ovr + V + v); l1 = *(const f32x4*)(ovr + V + v + 4);
                }
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    const float o = k < 4 ? o0[k] : o1[k - 4];
                    const bool on = o == o;
                    q[k] = on ? o : q[k];
                    lq[k] = on ? (k < 4 ? l0[k] : l1[k - 4]) : lq[k];
                }
            }
#pragma unroll
            for (int k = 0; k < 8; k += 2) {
                const f32x2 qq = {q[k], q[k + 1]};
                const f32x2 lc2 = {fmaxf(lps[k], R.lcl), fmaxf(lps[k + 1], R.lcl)};
                term2 = qq * (f32x2{lq[k], lq[k + 1]} - lc2) + term2;
                sacc2 += f32x2{lps[k] >= R.lcl ? q[k] : 0.f, lps[k + 1] >= R.lcl ? q[k + 1] : 0.f};
            }
        }
    };
    // the block's two sums of the lanes' partials, in one LDS round; valid in wave 0
    auto block_sums = [&](f32x2 term2, f32x2 sacc2, float& tp, float& sp) {
        const float tw = wave_sum(term2.x + term2.y), sw = wave_sum(sacc2.x + sacc2.y);
        if (lane == 0) { red[wid] = tw; red[RR_NW + wid] = sw; }
        __syncthreads();
        tp = 0.f; sp = 0.f;
        if (wid == 0) {
#pragma unroll
            for (int i = 0; i < RR_NW; ++i) { tp += red[i]; sp += red[RR_NW + i]; }
        }
    };
    // row r from registers (xt, xs)
    // row r from registers (xt, xs); returns true when pass B has already loaded row rn's chunks into them
    // LDS (the override image is in use, a compile-time tag: one code path each, so neither carries
    // the other's registers): the override values come from the image and pass B may prefetch
    auto row = [&](Set& xt, Set& xs, int r, int rn, uint64_t ts0, auto lds_tag) -> bool {
        constexpr bool LDS = decltype(lds_tag)::value;
        const RowStats st = stats[r];
        R.cq = (st.mt * invT + logf(st.zt)) * KD_LOG2E;
        R.cs = (st.ms * invT + logf(st.zs)) * KD_LOG2E;
        f32x2 term2, sacc2;
        pass_a(xt, xs, c_lo, c_hi, mb, lds_tag, term2, sacc2);
        uint64_t ts1 = 0;
        if (stamp) { ts1 = __builtin_amdgcn_s_memtime(); KD_RR_STAMP(0, ts1 - ts0); }
        float tp, sp;
        block_sums(term2, sacc2, tp, sp);
        uint64_t ts2 = 0;
        if (stamp) { ts2 = __builtin_amdgcn_s_memtime(); KD_RR_STAMP(1, ts2 - ts1); }
        if (wid == 0) {
            int miss = 0;
            if (nsl > 1) {
                // hand the slice partials over through the row's 2 nsl granules; poll them for at most
                // poll_ticks of the 100 MHz real-time clock (the slices of a row run together when
                // they are co-resident: microseconds apart)
                unsigned long long* g = gran + (int64_t)r * nsl * 2;
                if (lane == 0) { gran_store(g + 2 * sl, tp); gran_store(g + 2 * sl + 1, sp); }
                const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
                unsigned long long x = 1ull << 32;
                for (;;) {
                    x = lane < 2 * nsl ? gran_load(g + lane) : (1ull << 32);
                    if (__all((unsigned)(x >> 32) == 1u)) break;
                    if (__builtin_amdgcn_s_memrealtime() - t0 > poll_ticks) break;
                    __builtin_amdgcn_s_sleep(2);
                }
                const bool have = (unsigned)(x >> 32) == 1u;
                if (lane < 2 * nsl) gv[lane] = lane == 2 * sl ? tp : (lane == 2 * sl + 1 ? sp : __uint_as_float((unsigned)x));
                const uint64_t absent = __ballot(!have) & ((2 * nsl < 64 ? (1ull << (2 * nsl)) : 0ull) - 1ull);
                for (int s2 = 0; s2 < nsl; ++s2) miss |= ((absent >> (2 * s2)) & 3ull) ? (1 << s2) : 0;
            } else if (lane == 0) {
                gv[0] = tp; gv[1] = sp;
            }
            if (lane == 0) miss_s = miss;
        }
        __syncthreads();
        const int miss = miss_s;
        uint64_t ts3 = 0;
        if (stamp) { ts3 = __builtin_amdgcn_s_memtime(); KD_RR_STAMP(2, ts3 - ts2); }
        if (miss) {
            // a slice of this row is not running now (its workgroup is not resident beside this one:
            // other work holds CUs): compute its partials here with the same body and lane mapping, so
            // they are the bits it stores itself, then restore this slice's chunks.  Progress never
            // depends on co-residency; kd_loss_params.standin_count shows when this path runs.
            if (standin_count != nullptr && tid == 0) atomicAdd(standin_count, __popc((unsigned)miss));
            for (int s2 = 0; s2 < nsl; ++s2) {
                if (!((miss >> s2) & 1)) continue;
                const int lo2 = s2 * cps, hi2 = min(V >> 3, lo2 + cps);
                uint64_t mb2 = 0;
#pragma unroll
                for (int j = 0; j < RC; ++j) {
                    const int c = lo2 + tid + j * RR_NT;
                    if (c < hi2 && ((mask_g[(c * 8) >> 6] >> ((c * 8) & 63)) & 0xffull)) mb2 |= 1ull << (12 * j);
                }
                load(xt, xs, r, lo2, hi2);
                pass_a(xt, xs, lo2, hi2, mb2, GlbT{}, term2, sacc2);
                float t2, s3;
                block_sums(term2, sacc2, t2, s3);
                if (tid == 0) { gv[2 * s2] = t2; gv[2 * s2 + 1] = s3; }
                __syncthreads();   // red is reused by the next slice
            }
            load(xt, xs, r, c_lo, c_hi);
        }
        if (tid == 0) {
            float a = 0.f, b = 0.f;
            for (int s2 = 0; s2 < nsl; ++s2) { a += gv[2 * s2]; b += gv[2 * s2 + 1]; }   // slice order
            row_sums[0] = a; row_sums[1] = b;
            if (sl == 0) part_kl[r] = a * KD_LN2;
        }
        __syncthreads();
        const float Ssum = row_sums[1];
        if (D_ == nullptr) return false;
        // ---- pass B from the registers
        R.cec = st.valid ? ce_coef : 0.f;
        R.K = kd_coef * Ssum + (T1 ? R.cec : 0.f);
        R.cqk = R.cq - lk;
        R.c1 = (st.ms + logf(st.zs1)) * KD_LOG2E;
        bf16* drow = D_ + (int64_t)r * ld_d;
        const __amdgpu_buffer_rsrc_t rD = slice_rsrc(drow + c_lo * 8, (uint32_t)(c_hi - c_lo) * 16);
        // pf: chunk j of row rn goes into (xt[j], xs[j]) as soon as chunk j of row r is computed; the
        // CE one-hot is then applied inside its chunk (the same arithmetic as the rewrite below, so the
        // same bits) instead of by a second store that would re-read the row's logits
        const bool pre = LDS && pf && rn < rows;
        const uint32_t nb = (uint32_t)(c_hi - c_lo) * 16;
        const __amdgpu_buffer_rsrc_t rTn = slice_rsrc(T_ + (int64_t)(pre ? rn : r) * ld_t + c_lo * 8, nb);
        const __amdgpu_buffer_rsrc_t rSn = slice_rsrc(S_ + (int64_t)(pre ? rn : r) * ld_s + c_lo * 8, nb);
        const int labn = st.lab_next;
        const int oh_c = (pre && st.valid) ? (labn >> 3) : -1, oh_k = labn & 7;
#pragma unroll
        for (int j = 0; j < RC; ++j) {
            const int c = c_lo + tid + j * RR_NT;
            if (c >= c_hi) break;
            const int v = c * 8;
            float t[8], sv[8], qk[8];
            bf16x8_to_f32(xt[j], t);
            bf16x8_to_f32(xs[j], sv);
#pragma unroll
            for (int k = 0; k < 8; ++k) qk[k] = ex2(fmaf(t[k], R.a, -R.cqk));
            if ((mb >> (12 * j)) & 1u) {
                f32x4 o0, o1;
                if constexpr (LDS) {
                    const f32x4* o = ov_img + 4 * oslot(j);
                    o0 = o[0]; o1 = o[1];
                } else {
                    o0 = *(const f32x4*)(ovr + v); o1 = *(const f32x4*)(ovr + v + 4);
                }
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    const float o = k < 4 ? o0[k] : o1[k - 4];
                    qk[k] = o == o ? o * kd_coef : qk[k];
                }
            }
            if (pre) {
                xt[j] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rTn, vo, j * RR_NT * 16, 0));
                xs[j] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rSn, vo, j * RR_NT * 16, 0));
            }
            bf16x8 out;
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                float g = loca_grad<T1>(R, qk[k], sv[k]);
                if (c == oh_c && k == oh_k) g -= R.cec;
                out[k] = (bf16)g;
            }
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, out), rD, vo, j * RR_NT * 16, 0);
        }
        // the CE one-hot: the lane that wrote labn's chunk rewrites that element (program order)
        if (st.valid && !pre) {
            const int c = labn >> 3;
            if (c >= c_lo && c < c_hi && (c - c_lo) % RR_NT == tid) {
                const bf16* trow = T_ + (int64_t)r * ld_t;
                const bf16* srow = S_ + (int64_t)r * ld_s;
                float qk = ex2(fmaf((float)trow[labn], R.a, -R.cqk));
                if ((smask[(labn >> 6) - w_lo] >> (labn & 63)) & 1ull) qk = ovr[labn] * kd_coef;
                const float g = loca_grad<T1>(R, qk, (float)srow[labn]);
                drow[labn] = (bf16)(g - R.cec);
            }
        }
        if (stamp) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            const uint64_t ts4 = __builtin_amdgcn_s_memtime();
            KD_RR_STAMP(3, ts4 - ts3);
            KD_RR_STAMP(4, 1ull);
        }
        return pre;
    };
    auto run = [&](auto lds_tag) {
        Set xt, xs;
        bool have = false;
        for (int r = rg; r < rows; r += n_rg) {
            const uint64_t ts0 = stamp ? __builtin_amdgcn_s_memtime() : 0;
            if (!have) load(xt, xs, r, c_lo, c_hi);
            have = row(xt, xs, r, r + n_rg, ts0, lds_tag);
        }
    };
    if (use_lds) run(LdsT{});
    else run(GlbT{});
}

__global__ void k_finalize(const RowStats* __restrict__ stats, const float* __restrict__ part_kl,
                           int rows, double kl_scale, float kd_weight, float ce_weight,
                           float out_scale, int out_acc, float* __restrict__ out) {
    __shared__ double red[4][NW];
    double kl = 0, ce = 0, tce = 0, nv = 0;
    for (int r = threadIdx.x; r < rows; r += NT) {
        kl += part_kl[r];
        const RowStats& st = stats[r];
        ce += st.ce; tce += st.tce; nv += st.valid;
    }
    kl = wave_sum_d(kl); ce = wave_sum_d(ce); tce = wave_sum_d(tce); nv = wave_sum_d(nv);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) { red[0][w] = kl; red[1][w] = ce; red[2][w] = tce; red[3][w] = nv; }
    __syncthreads();
    if (threadIdx.x == 0) {
        double a = 0, b = 0, c = 0, n = 0;
        for (int i = 0; i < NW; ++i) { a += red[0][i]; b += red[1][i]; c += red[2][i]; n += red[3][i]; }
        const double kd = a * kl_scale;
        // HF CE: mean over valid targets (NaN when there are none, as torch's mean of empty)
        const double ce_m = b / n, tce_m = c / n;
        const double v[4] = {kd, ce_m, tce_m, kd_weight * kd + ce_weight * ce_m};
        for (int i = 0; i < 4; ++i) out[i] = (out_acc ? out[i] : 0.f) + (float)(out_scale * v[i]);
    }
}

// count of valid shifted labels (the CE mean's denominator lives on the device: no host
// sync) and the gradient coefficients coefs = {n_valid, ce_coef / c, kd_coef / c}, where c
// is the scale the dlogits are stored relative to (dlogits = dz / c):
//   dscale == NULL       c = 1
//   dscale, !given       c = ce_coef (= ce_weight * grad_scale / n_valid) if > 0, else kd_coef
//                        if > 0, else 1; written to *dscale
//   dscale, given        c = *dscale (an earlier call's: loss groups share one scale)
// Why: every row's one-hot element of the CE gradient is ce_coef * (p - 1) ~ -ce_coef, the
// SAME value in every row; rounded to bf16 it carries the same relative error (up to 2^-9)
// in every row, a systematic bias of the whole student gradient (+0.13 % of its norm on the
// tiny fixtures).  Stored relative to c it is ~ -1, exact in bf16; the consumer multiplies
// c back in fp32 (the dgrad / wgrad GEMMs' alpha_dev).
__global__ void k_count_valid(const int64_t* __restrict__ labels, int B, int L, int V, float ce_num,
                              float kd_coef, float* __restrict__ dscale, int given, float* __restrict__ coefs) {
    float* out = coefs;
    __shared__ float red[NW];
    float c = 0.f;
    for (int r = threadIdx.x; r < B * L; r += NT) {
        const int l = r % L;
        if (l + 1 < L) {
            const int64_t x = labels[r + 1];
            c += (x >= 0 && x < V) ? 1.f : 0.f;
        }
    }
    c = block_sum<NW>(c, red);
    if (threadIdx.x == 0) {
        *out = c;
        const float cec = c > 0.f ? ce_num / c : 0.f;
        float sc = 1.f;
        if (dscale != nullptr) {
            if (given) sc = *dscale;
            else {
                sc = cec > 0.f ? cec : (kd_coef > 0.f ? kd_coef : 1.f);
                *dscale = sc;
            }
        }
        coefs[1] = cec / sc;
        coefs[2] = kd_coef / sc;
    }
}

template <int VARIANT>
__global__ void __launch_bounds__(LG_NT)
k_loss_grad(const bf16* __restrict__ T_, int64_t ld_t, const bf16* __restrict__ S_, int64_t ld_s,
            int V, int rows, float invT, float clamp_min, const RowStats* __restrict__ stats,
            const float* __restrict__ ovr,
            const unsigned long long* __restrict__ mask_g, const float* __restrict__ coefs,
            bf16* __restrict__ D_, int64_t ld_d, float* __restrict__ part_kl) {
    extern __shared__ __attribute__((aligned(16))) unsigned long long smask[];
    __shared__ float red[LG_NW];
    const float ce_coef = coefs[1], kd_coef = coefs[2];
    loss_grad_body<VARIANT>(T_, ld_t, S_, ld_s, V, rows, invT, clamp_min, stats, ovr,
                            mask_g, kd_coef, ce_coef, D_, ld_d, part_kl, smask, red);
}

// LDS override-image slots of k_loss_grad_loca_rr<., rc> (64 B each): what leaves two (rc = 5) or three
// (rc = 3) workgroups per CU their share of the 160 KB beside the kernel's static arrays
inline int rr_ov_cap(int rc) { return rc >= 5 ? 1152 : 704; }
inline size_t rr_smem(int rc) { return (size_t)rr_ov_cap(rc) * 64; }

// resident k_loss_grad_loca_rr<., rc> workgroups on the current device (cached per device and rc):
// CUs x min(occupancy answer, the workgroups per CU its __launch_bounds__ reserves registers for:
// 2 at rc = 5, 3 at rc = 3) -- the occupancy API can answer one block high (MI355X_MICROARCH)
int rr_resident(int rc) {
    static int cache[64][2] = {};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 0;
    const int k = rc >= 5 ? 0 : 1, cap = rc >= 5 ? 2 : 3;
    if (cache[dev][k] == 0) {
        int cus = 0, nb = 0;
        const void* fn = rc >= 5 ? (const void*)k_loss_grad_loca_rr<true, 5> : (const void*)k_loss_grad_loca_rr<true, 3>;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
            hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, fn, RR_NT, rr_smem(rc)) != hipSuccess)
            cus = nb = 0;
        cache[dev][k] = cus * std::min(nb, cap) > 0 ? cus * std::min(nb, cap) : -1;
    }
    return cache[dev][k] > 0 ? cache[dev][k] : 0;
}

// chunks per lane of the register-resident kernel: 5 (default) or KD_LOSS_RR_C=3 (read per call)
int rr_chunks() {
    return ab_knob("KD_LOSS_RR_C", 5) == 3 ? 3 : 5;
}

// poll budget of a slice waiting for its row's other slices, in ticks of the 100 MHz real-time
// clock: 200 us by default (co-resident slices of a row arrive microseconds apart); after it the
// slice computes the absent partials itself.  kd_loss_params.rr_poll_us_p1 (tests: 1 = no wait, every
// slice recomputes every other slice's partials, which must give the same bits)
uint32_t rr_poll_ticks(int32_t us_p1) {
    const long us = us_p1 > 0 ? (long)us_p1 - 1 : 200;
    return (uint32_t)std::min<long>(us * 100, 100000000L);
}

}  // namespace

int launch_kd_loss(const void* teacher, int64_t ld_t, int V_t, const void* student, int64_t ld_s,
                   int V_s, const int64_t* labels, int B, int L, kd_loss_params p, float* loss_out,
                   void* dlogits, int64_t ld_d, void* ws, size_t ws_bytes, void* stream_) {
    hipStream_t stream = as_stream(stream_);
    const int variant = p.variant;
    KD_CHECK_ARG(variant >= KD_LOSS_NONE && variant <= KD_LOSS_KL_LOGTARGET, "kd_loss: bad variant");
    KD_CHECK_ARG(student && labels && loss_out && ws, "kd_loss: null pointer");
    KD_CHECK_ARG(variant == KD_LOSS_NONE || teacher, "kd_loss: teacher logits required");
    KD_CHECK_SHAPE(B > 0 && L > 0 && V_s > 0, "kd_loss: empty shape");
    KD_CHECK_SHAPE(V_s % 8 == 0 && ld_s % 8 == 0 && ld_s >= V_s, "kd_loss: V_s/ld_s must be multiples of 8");
    KD_CHECK_ALIGN(student, 16, "kd_loss: student logits must be 16-B aligned");
    if (teacher) {
        KD_CHECK_SHAPE(V_t >= V_s && V_t % 8 == 0 && ld_t % 8 == 0 && ld_t >= V_t,
                       "kd_loss: teacher V_t/ld_t must be multiples of 8 and V_t >= V_s");
        KD_CHECK_ALIGN(teacher, 16, "kd_loss: teacher logits must be 16-B aligned");
    }
    if (dlogits) {
        KD_CHECK_SHAPE(ld_d % 8 == 0 && ld_d >= V_s, "kd_loss: ld_d must be a multiple of 8");
        KD_CHECK_ALIGN(dlogits, 16, "kd_loss: dlogits must be 16-B aligned");
    }
    KD_CHECK_ARG(p.temperature > 0.f, "kd_loss: temperature must be > 0");
    const Layout lo = make_layout(B, L, V_s);
    if (ws_bytes < lo.total) return fail(KD_ERR_WORKSPACE, "kd_loss: workspace too small");
    char* w = (char*)ws;
    RowStats* stats = (RowStats*)(w + lo.stats);
    int* lab_last = (int*)(w + lo.lab_last);
    int* klo_last = (int*)(w + lo.klo_last);
    unsigned long long* mask = (unsigned long long*)(w + lo.mask);
    float* ovr = (float*)(w + lo.ovr);
    float* part_kl = (float*)(w + lo.part_kl);
    int* err = (int*)(w + lo.err);
    float* coefs = (float*)(w + lo.err + 4);   // {n_valid, ce coef, kd coef} (k_count_valid)
    const int rows = B * L;
    const float invT = 1.f / p.temperature;
    const bf16* T_ = (const bf16*)(variant == KD_LOSS_NONE ? nullptr : teacher);
    const bf16* S_ = (const bf16*)student;

    if (hipMemsetAsync(err, 0, 16, stream) != hipSuccess) return fail(KD_ERR_LAUNCH, "kd_loss: memset");
    if (variant == KD_LOSS_LOCA) {
        if (hipMemsetAsync(lab_last, 0xff, (size_t)V_s * 4, stream) != hipSuccess ||
            hipMemsetAsync(klo_last, 0xff, (size_t)V_s * 4, stream) != hipSuccess)
            return fail(KD_ERR_LAUNCH, "kd_loss: memset tables");
    }
    // k_row_stats: one workgroup per row (the dispatcher balances them); a grid of 2048 row-strided
    // workgroups left 512 of them (3 rows each) on a third of the CUs after the first 1536 (six
    // per CU) finished.  KD_RS_GRID=n: a grid of n row-strided workgroups (A/B).
    const int rs_cap = std::max(1, ab_knob("KD_RS_GRID", 1 << 30));
    const int grid = std::min(rows, rs_cap);
    const bool part = p.s_row_stats != nullptr;
    KD_CHECK_ARG(!(part && p.s_stats), "kd_loss: s_row_stats and s_stats are exclusive");
    if (part) {
        KD_CHECK_ARG(!T_ || p.t_row_stats, "kd_loss: s_row_stats without t_row_stats");
        KD_CHECK_ALIGN(p.s_row_stats, 16, "kd_loss: s_row_stats must be 16-B aligned");
        KD_CHECK_ALIGN(p.t_row_stats, 16, "kd_loss: t_row_stats must be 16-B aligned");
        hipLaunchKernelGGL(k_row_stats<RS_PART>, dim3(grid), dim3(NT), 0, stream, T_, ld_t, T_ ? V_t : 0, S_, ld_s,
                           V_s, labels, L, rows, variant, invT, p.alpha, (T_ && p.teacher_ce) ? 1 : 0, stats,
                           lab_last, klo_last, err, p.err_out, p.row_base, p.s_row_stats, p.t_row_stats, nullptr);
    } else if (p.s_stats) {
        KD_CHECK_ALIGN(p.s_stats, 16, "kd_loss: s_stats must be 16-B aligned");
        hipLaunchKernelGGL(k_row_stats<RS_SPRE>, dim3(grid), dim3(NT), 0, stream, T_, ld_t, T_ ? V_t : 0, S_, ld_s,
                           V_s, labels, L, rows, variant, invT, p.alpha, (T_ && p.teacher_ce) ? 1 : 0, stats,
                           lab_last, klo_last, err, p.err_out, p.row_base, nullptr, nullptr,
                           const_cast<float*>(p.s_stats));
    } else {
        hipLaunchKernelGGL(k_row_stats<RS_FULL>, dim3(grid), dim3(NT), 0, stream, T_, ld_t, T_ ? V_t : 0, S_, ld_s,
                           V_s, labels, L, rows, variant, invT, p.alpha, (T_ && p.teacher_ce) ? 1 : 0, stats,
                           lab_last, klo_last, err, p.err_out, p.row_base, nullptr, nullptr, nullptr);
    }
    KD_LAUNCH_CHECK("k_row_stats");
    if (variant == KD_LOSS_LOCA) {
        const int nb = (V_s + 255) / 256;
        hipLaunchKernelGGL(k_ovr_mask, dim3(nb), dim3(256), 0, stream, lab_last, klo_last, stats, V_s, mask, ovr);
        KD_LAUNCH_CHECK("k_ovr_mask");
    }
    const double N = (double)rows * (double)V_s;
    const float T = p.temperature;
    const float kd_coef = (float)((double)p.kd_weight * T / N * p.grad_scale);
    const float ce_num = p.ce_weight * p.grad_scale;
    hipLaunchKernelGGL(k_count_valid, dim3(1), dim3(NT), 0, stream, labels, B, L, V_s, ce_num,
                       variant == KD_LOSS_NONE ? 0.f : kd_coef, p.dscale, p.dscale_given ? 1 : 0, coefs);
    KD_LAUNCH_CHECK("k_count_valid");
    const size_t smem = variant == KD_LOSS_LOCA ? (size_t)((V_s + 63) / 64) * 8 : 0;
    if (smem > 150 * 1024) return fail(KD_ERR_SHAPE, "kd_loss: vocab too large for LDS mask");
    bf16* D_ = (bf16*)dlogits;
    // one 16-wave workgroup per CU: ~256 rows in flight, so pass B's re-read of a row (both
    // logits, 2 x 304 KB at V = 152K) is served by the 256 MB Infinity Cache, not HBM
    const int lg_grid = rows < LG_ROWS ? rows : LG_ROWS;
#define KD_LAUNCH_LG(VAR)                                                                          \
    hipLaunchKernelGGL(k_loss_grad<VAR>, dim3(lg_grid), dim3(LG_NT), smem, stream, T_, ld_t, S_, ld_s, \
                       V_s, rows, invT, p.clamp_min, stats, ovr, mask, coefs, D_, ld_d, part_kl)
    const bool loca_fast = variant == KD_LOSS_LOCA && kd_coef >= 0.f && T_ != nullptr;
    const int rc = rr_chunks();
    const int nsl = rr_nsl(V_s, rc);
    const int resident = rr_resident(rc);
    if (loca_fast && p.loca_path == 0 && nsl <= RR_MAX_SL && resident >= 2 * nsl) {
        // register-resident slices (k_loss_grad_loca_rr): resident / nsl row groups of nsl workgroups,
        // sized so that all of them fit at once on an idle GPU; a slice whose partner is not running
        // (other work holds CUs) stands in for it after the poll budget, so nothing depends on that
        const int cps = (V_s / 8 + nsl - 1) / nsl;
        const int n_rg = std::min(resident / nsl, rows);
        unsigned long long* gran = (unsigned long long*)(w + lo.gran);
        if (nsl > 1 && hipMemsetAsync(gran, 0, (size_t)rows * nsl * 16, stream) != hipSuccess)
            return fail(KD_ERR_LAUNCH, "kd_loss: memset granules");
#define KD_LAUNCH_RR(T1v, RCv)                                                                                   \
    hipLaunchKernelGGL((k_loss_grad_loca_rr<T1v, RCv>), dim3(n_rg * nsl), dim3(RR_NT), rr_smem(RCv), stream, T_, ld_t,   \
                       S_, ld_s, V_s, rows, invT, p.clamp_min, stats, ovr, mask, coefs, D_, ld_d, part_kl, nsl, cps, n_rg, \
                       gran, rr_poll_ticks(p.rr_poll_us_p1), ab_knob("KD_RR_STAMPS", 0),                          \
                       ab_knob("KD_RR_OV", 1) ? rr_ov_cap(RCv) : -1, ab_knob("KD_RR_PF", 1), p.standin_count)
        if (rc == 5) { if (invT == 1.f) KD_LAUNCH_RR(true, 5); else KD_LAUNCH_RR(false, 5); }
        else { if (invT == 1.f) KD_LAUNCH_RR(true, 3); else KD_LAUNCH_RR(false, 3); }
#undef KD_LAUNCH_RR
    } else if (loca_fast && invT == 1.f) {
        hipLaunchKernelGGL(k_loss_grad_loca<true>, dim3(lg_grid), dim3(LG_NT), smem, stream, T_, ld_t, S_, ld_s, V_s,
                           rows, invT, p.clamp_min, stats, ovr, mask, coefs, D_, ld_d, part_kl);
    } else if (loca_fast) {
        hipLaunchKernelGGL(k_loss_grad_loca<false>, dim3(lg_grid), dim3(LG_NT), smem, stream, T_, ld_t, S_, ld_s, V_s,
                           rows, invT, p.clamp_min, stats, ovr, mask, coefs, D_, ld_d, part_kl);
    } else switch (variant) {
        case KD_LOSS_NONE: KD_LAUNCH_LG(KD_LOSS_NONE); break;
        case KD_LOSS_LOCA: KD_LAUNCH_LG(KD_LOSS_LOCA); break;
        case KD_LOSS_KL: KD_LAUNCH_LG(KD_LOSS_KL); break;
        default: KD_LAUNCH_LG(KD_LOSS_KL_LOGTARGET); break;
    }
#undef KD_LAUNCH_LG
    KD_LAUNCH_CHECK("k_loss_grad");
    const double kl_scale = (variant == KD_LOSS_NONE) ? 0.0 : (double)T * T / N;
    hipLaunchKernelGGL(k_finalize, dim3(1), dim3(NT), 0, stream, stats, part_kl, rows, kl_scale,
                       p.kd_weight, p.ce_weight, p.out_scale, p.out_accumulate ? 1 : 0, loss_out);
    KD_LAUNCH_CHECK("k_finalize");
    return KD_OK;
}

int launch_kd_student_stats(const void* student, int64_t ld_s, int V_s, int rows, float temperature, float* out,
                            void* stream_) {
    KD_CHECK_ARG(student && out, "kd_loss_student_stats: null pointer");
    KD_CHECK_SHAPE(rows > 0 && V_s > 0, "kd_loss_student_stats: empty shape");
    KD_CHECK_SHAPE(V_s % 8 == 0 && ld_s % 8 == 0 && ld_s >= V_s, "kd_loss_student_stats: V_s/ld_s must be multiples of 8");
    KD_CHECK_ALIGN(student, 16, "kd_loss_student_stats: student logits must be 16-B aligned");
    KD_CHECK_ALIGN(out, 16, "kd_loss_student_stats: out must be 16-B aligned");
    KD_CHECK_ARG(temperature > 0.f, "kd_loss_student_stats: temperature must be > 0");
    // KD_SS_GRID (A/B): a cap on this launch's row-strided workgroups (it runs beside the teacher forward)
    const int rs_cap = std::max(1, ab_knob("KD_SS_GRID", ab_knob("KD_RS_GRID", 1 << 30)));
    // the RS_FULL arguments the student loop reads; the label / LoCa tail is not run
    hipLaunchKernelGGL(k_row_stats<RS_SONLY>, dim3(std::min(rows, rs_cap)), dim3(NT), 0, as_stream(stream_), nullptr,
                       (int64_t)0, 0, (const bf16*)student, ld_s, V_s, nullptr, 1, rows, 0, 1.f / temperature, 0.f, 0,
                       nullptr, nullptr, nullptr, nullptr, nullptr, 0, nullptr, nullptr, out);
    KD_LAUNCH_CHECK("k_row_stats<student>");
    return KD_OK;
}

size_t kd_loss_ws(int B, int L, int V) { return make_layout(B, L, V).total; }

int kd_loss_check_impl(const void* ws_, void* stream_) {
    int h = 0;  // error word is at workspace offset 0
    KD_CHECK_ARG(ws_ != nullptr, "kd_loss_check: null workspace");
    if (hipStreamSynchronize(as_stream(stream_)) != hipSuccess) return fail(KD_ERR_LAUNCH, "kd_loss_check: sync");
    if (hipMemcpy(&h, ws_, 4, hipMemcpyDeviceToHost) != hipSuccess) return fail(KD_ERR_LAUNCH, "kd_loss_check: copy");
    if (h) return fail(KD_ERR_LABEL_RANGE, "kd_loss: label outside [0, V) (LoCa gathers at every label; "
                                            "CE targets must be -100 or in range)");
    return KD_OK;
}

}  // namespace kd

#ifdef KD_AB_BUILD
// A/B build: read (and clear) k_loss_grad_loca_rr's per-workgroup phase stamps (KD_RR_STAMPS=1)
extern "C" int kd_ab_rr_stamps(unsigned long long* host, int n, int clear) {
    if (n > 4096 * 8) n = 4096 * 8;
    if (hipDeviceSynchronize() != hipSuccess) return 6;
    if (host && hipMemcpyFromSymbol(host, HIP_SYMBOL(kd::rr_stamps), (size_t)n * 8) != hipSuccess) return 6;
    if (clear) {
        static unsigned long long zeros[4096 * 8];
        if (hipMemcpyToSymbol(HIP_SYMBOL(kd::rr_stamps), zeros, sizeof(zeros)) != hipSuccess) return 6;
    }
    return 0;
}
#endif
