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

// One workgroup per query head.  q [H, hdp] bf16 (head-major, one token), caches
// [HKV, smax, hdp] bf16, o [H, hd] bf16.  Scores for all n keys live in LDS (n <= smax).
template <int HD>
__global__ void __launch_bounds__(NT) k_attn_decode(const bf16* __restrict__ q, const bf16* __restrict__ kc,
                                                    const bf16* __restrict__ vc, bf16* __restrict__ o, int H,
                                                    int HKV, int hdp, int smax, int n, float scale) {
    extern __shared__ float sh[];   // [n] scores, then [NT / HD][HD] partial outputs
    __shared__ float red[8];
    const int h = blockIdx.x, kvh = h / (H / HKV);
    const bf16* qh = q + (size_t)h * hdp;
    const bf16* K = kc + (size_t)kvh * smax * hdp;
    const bf16* V = vc + (size_t)kvh * smax * hdp;
    float qv[HD];
#pragma unroll
    for (int d = 0; d < HD; ++d) qv[d] = (float)qh[d];
    float mx = -INFINITY;
    for (int j = threadIdx.x; j < n; j += NT) {
        const bf16* kr = K + (size_t)j * hdp;
        float s = 0.f;
#pragma unroll
        for (int d = 0; d < HD; d += 8) {
            const bf16x8 kv8 = *(const bf16x8*)(kr + d);
#pragma unroll
            for (int e = 0; e < 8; ++e) s += qv[d + e] * (float)kv8[e];
        }
        s *= scale;
        sh[j] = s;
        mx = fmaxf(mx, s);
    }
    mx = block_max<NT / 64>(mx, red);
    float sum = 0.f;
    for (int j = threadIdx.x; j < n; j += NT) {
        const float p = __expf(sh[j] - mx);
        sh[j] = p;
        sum += p;
    }
    sum = block_sum<NT / 64>(sum, red);   // its barriers also publish sh[]
    constexpr int G = NT / HD;            // key groups
    const int d = threadIdx.x % HD, g = threadIdx.x / HD;
    float acc = 0.f;
    for (int j = g; j < n; j += G) acc += sh[j] * (float)V[(size_t)j * hdp + d];
    float* part = sh + ((n + 3) & ~3);
    part[g * HD + d] = acc;
    __syncthreads();
    if (g == 0) {
        float t = 0.f;
#pragma unroll
        for (int i = 0; i < G; ++i) t += part[i * HD + d];
        o[(size_t)h * HD + d] = (bf16)(t / sum);
    }
}

// One workgroup of 1024 threads: flags in the workspace (bit 0 = seen, bit 1 = banned), then
// the processed-score argmax.  seq [len + 1] int64 (the new token is written at seq[len]).
__global__ void __launch_bounds__(1024) k_gen_select(const bf16* __restrict__ logits, int V, int64_t* __restrict__ seq,
                                                     int len, float penalty, int ngram, uint8_t* __restrict__ flags,
                                                     int64_t* __restrict__ out) {
    __shared__ float sv[16];
    __shared__ int si[16];
    for (int i = threadIdx.x; i < V; i += blockDim.x) flags[i] = 0;
    __syncthreads();
    // RepetitionPenaltyLogitsProcessor: every id of the sequence (prompt + generated)
    if (penalty != 1.0f)
        for (int i = threadIdx.x; i < len; i += blockDim.x) {
            const int64_t t = seq[i];
            if (t >= 0 && t < V) flags[t] |= 1;
        }
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
    for (int i = threadIdx.x; i < V; i += blockDim.x) {
        float s = (float)logits[i];
        const uint8_t f = flags[i];
        if (f & 1) s = s < 0.f ? __fmul_rn(s, penalty) : __fdiv_rn(s, penalty);
        if (f & 2) s = -INFINITY;
        if (s > best || (s == best && i < bi)) { best = s; bi = i; }   // NaN never wins
    }
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
    }
}

}  // namespace

int launch_attn_decode(const void* q, const void* kc, const void* vc, void* o, int H, int HKV, int hd, int hdp,
                       int smax, int n, void* stream) {
    KD_CHECK_ARG(q && kc && vc && o, "attn_decode: null pointer");
    KD_CHECK_SHAPE(hd == 64 || hd == 128, "attn_decode: head dim must be 64 or 128");
    KD_CHECK_SHAPE(hdp >= hd && hdp % 8 == 0, "attn_decode: hdp must be >= hd and a multiple of 8");
    KD_CHECK_SHAPE(H > 0 && HKV > 0 && H % HKV == 0, "attn_decode: heads must be a multiple of kv heads");
    KD_CHECK_SHAPE(n > 0 && n <= smax && n <= 30000, "attn_decode: 0 < n <= smax <= 30000");
    KD_CHECK_ALIGN(q, 16, "attn_decode: q misaligned");
    KD_CHECK_ALIGN(kc, 16, "attn_decode: k cache misaligned");
    const size_t lds = (size_t)(((n + 3) & ~3) + NT) * sizeof(float);
    const float scale = 1.0f / sqrtf((float)hd);
    hipStream_t s = as_stream(stream);
    if (hd == 64)
        hipLaunchKernelGGL(k_attn_decode<64>, dim3(H), dim3(NT), lds, s, (const bf16*)q, (const bf16*)kc,
                           (const bf16*)vc, (bf16*)o, H, HKV, hdp, smax, n, scale);
    else
        hipLaunchKernelGGL(k_attn_decode<128>, dim3(H), dim3(NT), lds, s, (const bf16*)q, (const bf16*)kc,
                           (const bf16*)vc, (bf16*)o, H, HKV, hdp, smax, n, scale);
    KD_LAUNCH_CHECK("k_attn_decode");
    return KD_OK;
}

int launch_gen_select(const void* logits, int V, int64_t* seq, int len, float penalty, int ngram, void* flags_ws,
                      size_t ws_bytes, int64_t* out, void* stream) {
    KD_CHECK_ARG(logits && seq && flags_ws, "gen_select: null pointer");
    KD_CHECK_SHAPE(V > 0 && len > 0, "gen_select: V and len must be positive");
    KD_CHECK_ARG(penalty > 0.f && ngram >= 0, "gen_select: penalty must be > 0 and ngram >= 0");
    if (ws_bytes < (size_t)V) return fail(KD_ERR_WORKSPACE, "gen_select: workspace must hold V bytes");
    hipLaunchKernelGGL(k_gen_select, dim3(1), dim3(1024), 0, as_stream(stream), (const bf16*)logits, V, seq, len,
                       penalty, ngram, (uint8_t*)flags_ws, out);
    KD_LAUNCH_CHECK("k_gen_select");
    return KD_OK;
}

}  // namespace kd
