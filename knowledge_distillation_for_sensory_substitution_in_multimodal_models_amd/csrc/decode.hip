// Student generate(): single-token decode attention over a KV cache, and the greedy token
// choice with the logits processors the reference's evaluation sets (gfx950).
//
// Replaces, in LlavaOnevisionForConditionalGeneration.generate as called by
// evaluation/onevisionv3/evaluate_onevision.py:185-195 (max_new_tokens=32,
// repetition_penalty=1.2, no_repeat_ngram_size=2, greedy: do_sample is unset, so temperature
// is inert):
//   k_attn_decode   the SDPA of one new query row against the cached keys/values of every
//                   layer (Qwen2 GQA, scale hd^-0.5, fp32 softmax)
//   k_gen_select    RepetitionPenaltyLogitsProcessor (score < 0 ? score * p : score / p on every
//                   token id present in the sequence, float32), NoRepeatNGramLogitsProcessor
//                   (bans every token that would repeat an n-gram of the sequence), then the
//                   greedy argmax (lowest index on ties, as torch.argmax), appended to the
//                   device-resident sequence (no host sync per token).
#include "common.h"

namespace kd {

namespace {

constexpr int NT = 256;

// Split-KV decode attention (flash-decoding): workgroup (h, c) handles keys [c*CH, c*CH + CH)
// of query head h and writes its partial (max, sum, unnormalised output) to the workspace;
// k_attn_decode_combine merges the partials of a head.  Chunks at or past n exit after writing
// an empty partial, so the grid depends only on smax (fixed under graph capture).
// The step's own key/value row (k_new/v_new [HKV, hdp]) stands in for cache position n - 1 and
// is stored there by chunk 0 of the first query head of each KV group (read by later steps only).
// n = *cur_dev when cur_dev is given: the position lives on the device.
constexpr int CH = 64;   // keys per workgroup: 4 lanes per key for the scores, 4 key groups for P.V

template <int HD>
__global__ void __launch_bounds__(NT) k_attn_decode_part(const bf16* __restrict__ q, const bf16* __restrict__ k_new,
                                                         const bf16* __restrict__ v_new, bf16* __restrict__ kc,
                                                         bf16* __restrict__ vc, float* __restrict__ part, int H,
                                                         int HKV, int hdp, int smax, int n,
                                                         const int* __restrict__ cur_dev, float scale) {
    __shared__ float p_s[CH];
    __shared__ float red[8];
    __shared__ float acc_s[NT];
    if (cur_dev) n = *cur_dev;
    const int h = blockIdx.x, c = blockIdx.y, nch = gridDim.y, kvh = h / (H / HKV);
    float* pp = part + ((size_t)h * nch + c) * (HD + 2);
    const int j0 = c * CH;
    bf16* K = kc + (size_t)kvh * smax * hdp;
    bf16* V = vc + (size_t)kvh * smax * hdp;
    const bf16* kn = k_new + (size_t)kvh * hdp;
    const bf16* vn = v_new + (size_t)kvh * hdp;
    if (c == 0 && h % (H / HKV) == 0)
        for (int d = threadIdx.x; d < hdp; d += NT) {
            K[(size_t)(n - 1) * hdp + d] = kn[d];
            V[(size_t)(n - 1) * hdp + d] = vn[d];
        }
    if (j0 >= n) {   // empty chunk
        if (threadIdx.x == 0) { pp[0] = -INFINITY; pp[1] = 0.f; }
        if (threadIdx.x < HD) pp[2 + threadIdx.x] = 0.f;
        return;
    }
    // scores: key j0 + threadIdx/4, lane quarter (threadIdx & 3) covers HD/4 dims
    constexpr int DQ = HD / 4;
    const int kj = j0 + (threadIdx.x >> 2), qd = (threadIdx.x & 3) * DQ;
    float s = -INFINITY;
    if (kj < n) {
        const bf16* kr = (kj == n - 1 ? kn : K + (size_t)kj * hdp) + qd;
        const bf16* qh = q + (size_t)h * hdp + qd;
        float a = 0.f;
#pragma unroll
        for (int d = 0; d < DQ; d += 8) {
            const bf16x8 k8 = *(const bf16x8*)(kr + d);
            const bf16x8 q8 = *(const bf16x8*)(qh + d);
#pragma unroll
            for (int e = 0; e < 8; ++e) a += (float)q8[e] * (float)k8[e];
        }
        a += __shfl_xor(a, 1, 64);
        a += __shfl_xor(a, 2, 64);
        s = a * scale;
    }
    const float m = block_max<NT / 64>(s, red);
    const float pv = kj < n ? __expf(s - m) : 0.f;
    if ((threadIdx.x & 3) == 0) p_s[threadIdx.x >> 2] = pv;
    const float l = block_sum<NT / 64>((threadIdx.x & 3) == 0 ? pv : 0.f, red);   // barriers publish p_s
    constexpr int G = NT / HD;
    const int d = threadIdx.x % HD, g = threadIdx.x / HD;
    float acc = 0.f;
    const int jend = min(CH, n - j0);
    for (int jj = g; jj < jend; jj += G) {
        const int j = j0 + jj;
        acc += p_s[jj] * (float)(j == n - 1 ? vn[d] : V[(size_t)j * hdp + d]);
    }
    acc_s[threadIdx.x] = acc;
    __syncthreads();
    if (g == 0) {
        float tsum = 0.f;
#pragma unroll
        for (int i = 0; i < G; ++i) tsum += acc_s[i * HD + d];
        pp[2 + d] = tsum;
        if (d == 0) { pp[0] = m; pp[1] = l; }
    }
}

constexpr int MAX_CH = 512;   // chunks per head (smax <= 32768)

// Merge the nch partials of head h: chunk maxima and weights staged in LDS (one load round
// trip), then 256 threads = HD dims x (256 / HD) chunk groups accumulate in parallel.
template <int HD>
__global__ void __launch_bounds__(NT) k_attn_decode_combine(const float* __restrict__ part, int nch,
                                                            bf16* __restrict__ o) {
    __shared__ float ms[MAX_CH], red[8], acc_s[NT];
    const int h = blockIdx.x;
    const float* pp = part + (size_t)h * nch * (HD + 2);
    float m = -INFINITY;
    for (int c = threadIdx.x; c < nch; c += NT) {
        ms[c] = pp[(size_t)c * (HD + 2)];
        m = fmaxf(m, ms[c]);
    }
    m = block_max<NT / 64>(m, red);
    float l = 0.f;
    for (int c = threadIdx.x; c < nch; c += NT) {
        const float w = ms[c] == -INFINITY ? 0.f : __expf(ms[c] - m);
        ms[c] = w;
        l += w * pp[(size_t)c * (HD + 2) + 1];
    }
    l = block_sum<NT / 64>(l, red);   // barriers publish the weights in ms[]
    constexpr int G = NT / HD;
    const int d = threadIdx.x % HD, g = threadIdx.x / HD;
    float acc = 0.f;
    for (int c = g; c < nch; c += G) acc += ms[c] * pp[(size_t)c * (HD + 2) + 2 + d];
    acc_s[threadIdx.x] = acc;
    __syncthreads();
    if (g == 0) {
        float tsum = 0.f;
#pragma unroll
        for (int i = 0; i < G; ++i) tsum += acc_s[i * HD + d];
        o[(size_t)h * HD + d] = (bf16)(tsum / l);
    }
}

// Stage the token row x[K] into LDS as fp32; with norm_w, as kd_norm_fwd's RMSNorm output
// (bf16(x * rsqrt(mean(x^2) + eps) * w), rounded to bf16 as the unfused kernel stores it), so the
// norm costs no launch of its own.
__device__ __forceinline__ void stage_x(const bf16* __restrict__ x, const bf16* __restrict__ norm_w, float eps, int K,
                                        float* xs, float* red) {
    float ss = 0.f;
    for (int k = threadIdx.x; k < K; k += NT) {
        const float v = (float)x[k];
        xs[k] = v;
        ss += v * v;
    }
    if (norm_w) {
        const float rstd = rsqrtf(block_sum<NT / 64>(ss, red) / K + eps);
        for (int k = threadIdx.x; k < K; k += NT) xs[k] = (float)(bf16)(xs[k] * rstd * (float)norm_w[k]);
    }
    __syncthreads();
}

// Decode GEMV: y[n] = epilogue(sum_k x[k] * W[n][k]) for one token row, one wave per output
// (two weight rows, n and I + n, for the SwiGLU form).  Weight rows are read once, 16 B per lane,
// so the decode step streams its weights at HBM rate instead of running 256-row GEMM tiles at
// M = 1.  EPI: 0 none, 1 + bias[n], 2 + residual[n], 3 silu(row n) * (row I + n).
template <int EPI>
__global__ void __launch_bounds__(NT) k_gemv(const bf16* __restrict__ x, const bf16* __restrict__ W, int64_t ldw,
                                             const bf16* __restrict__ extra, bf16* __restrict__ y, int N, int K,
                                             int I, const bf16* __restrict__ norm_w, float eps) {
    extern __shared__ float xs[];
    __shared__ float red[8];
    stage_x(x, norm_w, eps, K, xs, red);
    const int n = blockIdx.x * (NT / 64) + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (n >= N) return;
    const bf16* r0 = W + (size_t)n * ldw;
    const bf16* r1 = W + (size_t)(I + n) * ldw;
    float a0 = 0.f, a1 = 0.f;
    for (int k = lane * 8; k < K; k += 512) {
        const bf16x8 w0 = *(const bf16x8*)(r0 + k);
#pragma unroll
        for (int e = 0; e < 8; ++e) a0 += xs[k + e] * (float)w0[e];
        if constexpr (EPI == 3) {
            const bf16x8 w1 = *(const bf16x8*)(r1 + k);
#pragma unroll
            for (int e = 0; e < 8; ++e) a1 += xs[k + e] * (float)w1[e];
        }
    }
    a0 = wave_sum(a0);
    if constexpr (EPI == 3) a1 = wave_sum(a1);
    if (lane == 0) {
        float v = a0;
        if constexpr (EPI == 1 || EPI == 2) v += (float)extra[n];
        if constexpr (EPI == 3) v = silu_fast(a0) * a1;
        y[n] = (bf16)v;
    }
}

// Row-per-workgroup form of k_gemv for few output rows with long K (o_proj / down_proj of the
// 0.5B student: N = 896, K up to 4864): 256 threads split K, block reduction, so N workgroups
// instead of N / 4 keep every CU streaming.
template <int EPI>
__global__ void __launch_bounds__(NT) k_gemv_rows(const bf16* __restrict__ x, const bf16* __restrict__ W, int64_t ldw,
                                                  const bf16* __restrict__ extra, bf16* __restrict__ y, int K, int I,
                                                  const bf16* __restrict__ norm_w, float eps) {
    extern __shared__ float xs[];
    __shared__ float red[8];
    stage_x(x, norm_w, eps, K, xs, red);
    const int n = blockIdx.x;
    const bf16* r0 = W + (size_t)n * ldw;
    const bf16* r1 = W + (size_t)(I + n) * ldw;
    float a0 = 0.f, a1 = 0.f;
    for (int k = threadIdx.x * 8; k < K; k += NT * 8) {
        const bf16x8 w0 = *(const bf16x8*)(r0 + k);
#pragma unroll
        for (int e = 0; e < 8; ++e) a0 += xs[k + e] * (float)w0[e];
        if constexpr (EPI == 3) {
            const bf16x8 w1 = *(const bf16x8*)(r1 + k);
#pragma unroll
            for (int e = 0; e < 8; ++e) a1 += xs[k + e] * (float)w1[e];
        }
    }
    a0 = block_sum<NT / 64>(a0, red);
    if constexpr (EPI == 3) a1 = block_sum<NT / 64>(a1, red);
    if (threadIdx.x == 0) {
        float v = a0;
        if constexpr (EPI == 1 || EPI == 2) v += (float)extra[n];
        if constexpr (EPI == 3) v = silu_fast(a0) * a1;
        y[n] = (bf16)v;
    }
}

// One workgroup of 1024 threads: flags in the workspace (bit 0 = seen, bit 1 = banned), then
// the processed-score argmax.  seq [len + 1] int64 (the new token is written at seq[len]).
__global__ void __launch_bounds__(1024) k_gen_select(const bf16* __restrict__ logits, int V, int64_t* __restrict__ seq,
                                                     int len, int* __restrict__ cur_dev, float penalty, int ngram,
                                                     uint8_t* __restrict__ flags, int64_t* __restrict__ out) {
    __shared__ float sv[16];
    __shared__ int si[16];
    if (cur_dev) len = *cur_dev;
    {   // clear the flags, 16 B per store (flags is 256-B aligned workspace)
        const int v16 = V >> 4;
        for (int i = threadIdx.x; i < v16; i += blockDim.x) ((u32x4*)flags)[i] = u32x4{0u, 0u, 0u, 0u};
        for (int i = (v16 << 4) + threadIdx.x; i < V; i += blockDim.x) flags[i] = 0;
    }
    __syncthreads();
    // RepetitionPenaltyLogitsProcessor: every id of the sequence (prompt + generated)
    if (penalty != 1.0f)
        for (int i = threadIdx.x; i < len; i += blockDim.x) {
            const int64_t t = seq[i];
            if (t >= 0 && t < V) flags[t] |= 1;
        }
    __syncthreads();   // the two processors OR different bits into the same bytes
    // NoRepeatNGramLogitsProcessor: the last (ngram - 1) tokens as a prefix; ban the token that
    // followed every earlier occurrence of that prefix (only once cur_len + 1 >= ngram)
    if (ngram > 0 && len + 1 >= ngram)
        for (int i = threadIdx.x; i + ngram <= len; i += blockDim.x) {
            bool match = true;
            for (int k = 0; k < ngram - 1; ++k) match &= seq[i + k] == seq[len - ngram + 1 + k];
            if (match) {
                const int64_t t = seq[i + ngram - 1];
                if (t >= 0 && t < V) flags[t] |= 2;
            }
        }
    __syncthreads();
    float best = -INFINITY;
    int bi = 0x7fffffff;
    auto consider = [&](int i, float s, uint32_t f) {
        if (f & 1) s = s < 0.f ? __fmul_rn(s, penalty) : __fdiv_rn(s, penalty);
        if (f & 2) s = -INFINITY;
        if (s > best || (s == best && i < bi)) { best = s; bi = i; }   // NaN never wins
    };
    const int v8 = ((uintptr_t)logits & 15) == 0 ? V >> 3 : 0;   // 8 logits (16 B) + 8 flags per step
    for (int c = threadIdx.x; c < v8; c += blockDim.x) {
        const bf16x8 lv = ((const bf16x8*)logits)[c];
        const u32x2 fv = ((const u32x2*)flags)[c];
#pragma unroll
        for (int e = 0; e < 8; ++e) consider(c * 8 + e, (float)lv[e], ((e < 4 ? fv.x : fv.y) >> (8 * (e & 3))) & 255u);
    }
    for (int i = (v8 << 3) + threadIdx.x; i < V; i += blockDim.x) consider(i, (float)logits[i], flags[i]);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const float ov = __shfl_xor(best, off, 64);
        const int oi = __shfl_xor(bi, off, 64);
        if (ov > best || (ov == best && oi < bi)) { best = ov; bi = oi; }
    }
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) { sv[w] = best; si[w] = bi; }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int k = 1; k < (int)(blockDim.x >> 6); ++k)
            if (sv[k] > best || (sv[k] == best && si[k] < bi)) { best = sv[k]; bi = si[k]; }
        if (bi == 0x7fffffff) bi = 0;   // every score -inf: torch.argmax returns 0
        seq[len] = bi;
        if (out) *out = bi;
        if (cur_dev) *cur_dev = len + 1;
    }
}

// cos/sin row of position *cur_dev - 1 into fixed one-row buffers (what kd_qkv_split reads).
__global__ void k_rope_row(const float* __restrict__ cos_t, const float* __restrict__ sin_t, int hh,
                           const int* __restrict__ cur_dev, float* __restrict__ cos_row, float* __restrict__ sin_row) {
    const int pos = *cur_dev - 1;
    for (int i = threadIdx.x; i < hh; i += blockDim.x) {
        cos_row[i] = cos_t[(size_t)pos * hh + i];
        sin_row[i] = sin_t[(size_t)pos * hh + i];
    }
}

}  // namespace

int launch_rope_row(const float* cos_t, const float* sin_t, int hh, const int* cur_dev, float* cos_row, float* sin_row,
                    void* stream) {
    KD_CHECK_ARG(cos_t && sin_t && cur_dev && cos_row && sin_row, "rope_row: null pointer");
    KD_CHECK_SHAPE(hh > 0, "rope_row: hh must be positive");
    hipLaunchKernelGGL(k_rope_row, dim3(1), dim3(256), 0, as_stream(stream), cos_t, sin_t, hh, cur_dev, cos_row,
                       sin_row);
    KD_LAUNCH_CHECK("k_rope_row");
    return KD_OK;
}

size_t attn_decode_ws(int H, int hd, int smax) {
    return (size_t)H * ((smax + CH - 1) / CH) * (hd + 2) * sizeof(float);
}

int launch_attn_decode(const void* q, const void* k_new, const void* v_new, void* kc, void* vc, void* o, int H,
                       int HKV, int hd, int hdp, int smax, int n, const int* cur_dev, void* ws, size_t ws_bytes,
                       void* stream) {
    KD_CHECK_ARG(q && k_new && v_new && kc && vc && o && ws, "attn_decode: null pointer");
    KD_CHECK_SHAPE(hd == 64 || hd == 128, "attn_decode: head dim must be 64 or 128");
    KD_CHECK_SHAPE(hdp >= hd && hdp % 8 == 0, "attn_decode: hdp must be >= hd and a multiple of 8");
    KD_CHECK_SHAPE(H > 0 && HKV > 0 && H % HKV == 0, "attn_decode: heads must be a multiple of kv heads");
    KD_CHECK_SHAPE(smax > 0 && smax <= MAX_CH * CH && (cur_dev || (n > 0 && n <= smax)),
                   "attn_decode: need 0 < n <= smax <= 32768");
    KD_CHECK_ALIGN(q, 16, "attn_decode: q misaligned");
    KD_CHECK_ALIGN(kc, 16, "attn_decode: k cache misaligned");
    KD_CHECK_ALIGN(k_new, 16, "attn_decode: k_new misaligned");
    if (ws_bytes < attn_decode_ws(H, hd, smax)) return fail(KD_ERR_WORKSPACE, "attn_decode: workspace too small");
    const int nch = (smax + CH - 1) / CH;
    const float scale = 1.0f / sqrtf((float)hd);
    hipStream_t s = as_stream(stream);
    float* part = (float*)ws;
    if (hd == 64) {
        hipLaunchKernelGGL(k_attn_decode_part<64>, dim3(H, nch), dim3(NT), 0, s, (const bf16*)q, (const bf16*)k_new,
                           (const bf16*)v_new, (bf16*)kc, (bf16*)vc, part, H, HKV, hdp, smax, n, cur_dev, scale);
        hipLaunchKernelGGL(k_attn_decode_combine<64>, dim3(H), dim3(NT), 0, s, part, nch, (bf16*)o);
    } else {
        hipLaunchKernelGGL(k_attn_decode_part<128>, dim3(H, nch), dim3(NT), 0, s, (const bf16*)q, (const bf16*)k_new,
                           (const bf16*)v_new, (bf16*)kc, (bf16*)vc, part, H, HKV, hdp, smax, n, cur_dev, scale);
        hipLaunchKernelGGL(k_attn_decode_combine<128>, dim3(H), dim3(NT), 0, s, part, nch, (bf16*)o);
    }
    KD_LAUNCH_CHECK("k_attn_decode");
    return KD_OK;
}

int launch_gemv(const void* x, const void* W, int64_t ldw, const void* extra, void* y, int N, int K, int epi, int I,
                const void* norm_w, float eps, void* stream) {
    KD_CHECK_ARG(x && W && y, "gemv: null pointer");
    KD_CHECK_ARG(epi >= 0 && epi <= 3 && (epi == 0 || epi == 3 || extra), "gemv: epilogue 0..3 (1, 2 need extra)");
    KD_CHECK_SHAPE(N > 0 && K > 0 && K % 8 == 0 && K <= 16384 && ldw >= K && ldw % 8 == 0,
                   "gemv: K must be a multiple of 8 (<= 16384), ldw >= K and a multiple of 8");
    KD_CHECK_ALIGN(W, 16, "gemv: W misaligned");
    const dim3 grid((N + NT / 64 - 1) / (NT / 64));
    const size_t lds = (size_t)K * sizeof(float);
    hipStream_t s = as_stream(stream);
    const bf16 *xb = (const bf16*)x, *Wb = (const bf16*)W, *eb = (const bf16*)extra, *nw = (const bf16*)norm_w;
    if (N < 4096 && K >= 512) {   // few rows: one workgroup per row, K split over 256 threads
        switch (epi) {
            case 0: hipLaunchKernelGGL(k_gemv_rows<0>, dim3(N), dim3(NT), lds, s, xb, Wb, ldw, eb, (bf16*)y, K, I, nw, eps); break;
            case 1: hipLaunchKernelGGL(k_gemv_rows<1>, dim3(N), dim3(NT), lds, s, xb, Wb, ldw, eb, (bf16*)y, K, I, nw, eps); break;
            case 2: hipLaunchKernelGGL(k_gemv_rows<2>, dim3(N), dim3(NT), lds, s, xb, Wb, ldw, eb, (bf16*)y, K, I, nw, eps); break;
            default: hipLaunchKernelGGL(k_gemv_rows<3>, dim3(N), dim3(NT), lds, s, xb, Wb, ldw, eb, (bf16*)y, K, I, nw, eps);
        }
        KD_LAUNCH_CHECK("k_gemv_rows");
        return KD_OK;
    }
    switch (epi) {
        case 0: hipLaunchKernelGGL(k_gemv<0>, grid, dim3(NT), lds, s, xb, Wb, ldw, eb, (bf16*)y, N, K, I, nw, eps); break;
        case 1: hipLaunchKernelGGL(k_gemv<1>, grid, dim3(NT), lds, s, xb, Wb, ldw, eb, (bf16*)y, N, K, I, nw, eps); break;
        case 2: hipLaunchKernelGGL(k_gemv<2>, grid, dim3(NT), lds, s, xb, Wb, ldw, eb, (bf16*)y, N, K, I, nw, eps); break;
        default: hipLaunchKernelGGL(k_gemv<3>, grid, dim3(NT), lds, s, xb, Wb, ldw, eb, (bf16*)y, N, K, I, nw, eps);
    }
    KD_LAUNCH_CHECK("k_gemv");
    return KD_OK;
}

int launch_gen_select(const void* logits, int V, int64_t* seq, int len, int* cur_dev, float penalty, int ngram,
                      void* flags_ws, size_t ws_bytes, int64_t* out, void* stream) {
    KD_CHECK_ARG(logits && seq && flags_ws, "gen_select: null pointer");
    KD_CHECK_SHAPE(V > 0 && (cur_dev || len > 0), "gen_select: V and len must be positive");
    KD_CHECK_ARG(penalty > 0.f && ngram >= 0, "gen_select: penalty must be > 0 and ngram >= 0");
    if (ws_bytes < (size_t)V) return fail(KD_ERR_WORKSPACE, "gen_select: workspace must hold V bytes");
    hipLaunchKernelGGL(k_gen_select, dim3(1), dim3(1024), 0, as_stream(stream), (const bf16*)logits, V, seq, len,
                       cur_dev, penalty, ngram, (uint8_t*)flags_ws, out);
    KD_LAUNCH_CHECK("k_gen_select");
    return KD_OK;
}

}  // namespace kd
