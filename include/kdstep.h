/*
 * kdstep.h — C-ABI of the MI355X-native online-KD training step (gfx950).
 *
 * Drop-in boundary for the reference's per-step hot path
 *   OnlineKnowledgeDistillationLLavaOneVision.training_step / forward
 *   (distillation/knowledge_distillation7b_double_trouble/phase1/
 *    OnlineKnowledgeDistillationLLavaOneVision.py:123-131, :206-271)
 * and the third-party HF arithmetic it calls into (SigLIP, Qwen2, LLaVA-OV pack,
 * causal-LM CE).  The reference has no FFI of its own (it is pure Python); every
 * entry point below replaces a PyTorch/transformers call site that is cited next
 * to it.  Conventions:
 *
 *  - Every function returns an int status (kd_status).  0 = OK.  On failure a
 *    thread-local message is available from kd_last_error().
 *  - All pointers are DEVICE pointers unless the parameter name ends in _host.
 *    The caller (PyTorch) owns every buffer; the library never allocates or frees
 *    caller memory.  Workspaces are sized with the matching *_workspace_size().
 *  - `stream` is a hipStream_t passed as void*.  All calls are asynchronous and
 *    stream-ordered: no hidden device synchronisation.
 *  - bf16 tensors are raw 16-bit storage (uint16_t / __bf16); fp32 is float.
 *  - Leading dimensions (ld*) are in ELEMENTS.
 *  - Descriptor structs (kd_gemm_desc, kd_attn_desc, kd_attn_bwd_desc, kd_loss_params, ...) grow
 *    by appending fields; every release that appends one bumps KD_ABI_VERSION.  Callers MUST
 *    zero-initialise a descriptor (`kd_gemm_desc d = {0};` / memset) before filling it, so a
 *    field they do not know is 0 = "off", and should check kd_abi_version() == KD_ABI_VERSION
 *    at load time (the Python binding refuses a mismatched library).
 *    ABI 6 -> 7: kd_gemm diagnostic variants (17-20, 22, 23, 25-28) are no longer accepted by
 *    the product library (A/B builds only); kd_loss err bit 4 is no longer set.
 *    ABI 6 -> 7 also changed kd_model_backward's dpost from a bf16 per-row gradient
 *    [n_tiles*np, v_hidden] to an fp32 per-tile gradient [n_tiles, v_hidden] (same void*).
 *    ABI 7 -> 8: kd_loss_params.s_stats appended; kd_loss_student_stats added.
 *    ABI 8 -> 9: kd_loss_params.loca_path / rr_poll_us_p1 / standin_count appended (the library
 *    reads no environment variable for the loss kernel any more); kd_model_backward's on_layer_done also fires for the embeddings / projector
 *    (KD_CB_EMBED_PROJECTOR) and after each SigLIP layer (KD_CB_VISION_LAYER(i), negative codes);
 *    a callback written for ABI 8 must ignore layer < 0.
 */
#ifndef KDSTEP_H
#define KDSTEP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum {
    KD_OK = 0,
    KD_ERR_SHAPE = 1,        /* inconsistent / unsupported shape                       */
    KD_ERR_DTYPE = 2,        /* unsupported dtype enum                                 */
    KD_ERR_ALIGN = 3,        /* pointer / leading dimension misaligned (16 B needed)   */
    KD_ERR_ARCH = 4,         /* device is not gfx950                                   */
    KD_ERR_LABEL_RANGE = 5,  /* a label is outside [0, V) where the reference gathers  */
    KD_ERR_LAUNCH = 6,       /* HIP launch / runtime error                             */
    KD_ERR_ARG = 7,          /* null pointer or invalid enum / parameter               */
    KD_ERR_WORKSPACE = 8     /* workspace too small                                    */
} kd_status;

/* ---------------------------------------------------------------- library ---- */
int kd_abi_version(void);                 /* returns KD_ABI_VERSION                  */
const char* kd_last_error(void);          /* thread-local, never NULL                */
int kd_device_is_gfx950(int device);      /* 1 if device `device` is gfx950, else 0  */

#define KD_ABI_VERSION 9

/* ------------------------------------------------------------- KD losses ---- */
/* Variants of the logit loss.  Each replaces one reference function:
 *  KD_LOSS_LOCA         compute_loca_loss, DT:141-194 (T=0.8) and LB:208-261 (T=1):
 *                       KL(calibrated teacher || clamp(p_S,1e-8)), mean over B*L*V,
 *                       x T^2, with the global last-write-wins column overrides.
 *  KD_LOSS_KL           compute_vision_loss's KL term, DT:330-343:
 *                       kl_div(log_softmax(s/T), softmax(t/T), 'mean') * T^2.
 *  KD_LOSS_KL_LOGTARGET FB compute_loss, FB:205-219 (and LB compute_loss LB:177-190):
 *                       kl_div(log_softmax(s/T), softmax(t/T), 'mean', log_target=True)*T^2
 *                       = mean(exp(p_T) * (p_T - log p_S)) * T^2.
 *  KD_LOSS_NONE         no teacher term (student CE only; BD SFT step, BD:90-109).
 * The student CE is the in-model causal-LM loss (shift by one, ignore -100, mean over
 * valid labels), HF ForCausalLMLoss; the teacher CE (computed and discarded by the
 * reference at DT:228) is reported as a side output when teacher logits are given. */
typedef enum {
    KD_LOSS_NONE = 0,
    KD_LOSS_LOCA = 1,
    KD_LOSS_KL = 2,
    KD_LOSS_KL_LOGTARGET = 3
} kd_loss_variant;

typedef struct {
    int32_t variant;        /* kd_loss_variant                                         */
    float temperature;      /* T (self.T: DT 0.8, LB 1.0, FB 0.8)                       */
    float alpha;            /* LoCa alpha (compute_loca_loss default 0.8)               */
    float kd_weight;        /* weight of the (T^2-scaled) KD term in the total          */
    float ce_weight;        /* weight of the student CE in the total                    */
    float grad_scale;       /* dlogits multiplier (upstream dL/dtotal, e.g. 1/accum)    */
    float clamp_min;        /* LoCa clamp of p_S before log (1e-8, DT:161-162)           */
    int32_t teacher_ce;     /* 1: also compute the teacher's (unused) CE side output    */
    float out_scale;        /* loss_out receives out_scale * value (set 1 for plain use) */
    int32_t out_accumulate; /* 1: loss_out += out_scale * value (loss groups, §8e)      */
    int32_t* err_out;       /* optional device int32[4], caller-zeroed, never reset here:
                               [0] |= 1 LoCa gather label outside [0, V_s) (DT:166),
                                      2 CE target outside {-100} u [0, V_s),
                                      (4: reserved; unused since ABI 7);
                               [1] first offending label, [2] its row + row_base,
                               [3] claim flag                                          */
    int32_t row_base;       /* added to the row reported in err_out[2]                   */
    float* dscale;          /* optional device float: dlogits are stored relative to a scale
                               c (dlogits = d(total)/d(logits) * grad_scale / c) and the
                               consumer multiplies c back in fp32 (e.g. kd_gemm alpha_dev).
                               c = the CE coefficient ce_weight * grad_scale / n_valid (else
                               the KD coefficient) is written here, so the CE one-hot
                               element, the same value in every row, is ~ -1 (exact in
                               bf16) instead of a bf16-rounded -1/n_valid (a systematic
                               bias of the whole gradient).  NULL: c = 1.               */
    int32_t dscale_given;   /* 1: read c from *dscale (an earlier call's; loss groups)    */
    /* optional: the lm_head GEMMs' row statistics (kd_gemm_desc.row_stats) of THESE rows — the
       student's with row_stats_vs = V_s and inv_t = 1/T, the teacher's with row_stats_vs = V_s,
       inv_t = 1/T and top-2 — instead of the loss's own pass over both logit tensors
       (k_row_stats). Same values up to fp32 summation order. Both or neither (KD_LOSS_NONE:
       the student's alone). */
    const float* s_row_stats;
    const float* t_row_stats;
    /* optional (ABI 8): the student's statistics of THESE rows from kd_loss_student_stats (run
       earlier, e.g. on the student's stream right after its lm_head, while the teacher finishes);
       the loss then reads only the teacher's logits for its statistics. Bit-identical results.
       Exclusive with s_row_stats. */
    const float* s_stats;
    /* optional (ABI 9): the LoCa kernel (0 = the product default).  loca_path 0: register-resident
       row slices (k_loss_grad_loca_rr) where they fit, 1: the two-read k_loss_grad_loca (same terms up
       to the fp32 order of the row sums).  rr_poll_us_p1: the register-resident kernel's poll budget
       for a partner slice's partials, in microseconds + 1 (0 = the default 200 us; 1 = no wait: every
       partner partial recomputed by the waiting slice itself, which must give the same bits). */
    int32_t loca_path;
    int32_t rr_poll_us_p1;
    /* optional (ABI 9): device int32, += the number of partner partials the register-resident kernel
       recomputed because the partner slice was not running within the poll budget (0 on an idle or
       evenly shared GPU; the fallback only slows the step down, this shows when it fires) */
    int32_t* standin_count;
} kd_loss_params;

/* loss_out (device float[4]): [0] KD term (mean, incl. T^2, unweighted)
 *                             [1] student CE   [2] teacher CE   [3] total
 * dlogits: d(total)/d(student_logits) * grad_scale (/ *dscale), bf16 [B*L, ld_d] (may be NULL).
 * labels: int64 [B, L] (row-major).  LoCa requires every label in [0, V_s): a label
 * outside raises KD_ERR_LABEL_RANGE from kd_loss_check() (the reference raises
 * RuntimeError from gather, DT:166) and is recorded in params.err_out (read
 * asynchronously by the caller, no device sync).  teacher may be NULL for KD_LOSS_NONE.
 * V_t >= V_s: the teacher is sliced to its first V_s columns (DT:155). */
size_t kd_loss_workspace_size(int B, int L, int V_s);
int kd_loss_fwd_bwd(const void* teacher_logits, int64_t ld_t, int V_t,
                    const void* student_logits, int64_t ld_s, int V_s,
                    const int64_t* labels, int B, int L,
                    kd_loss_params params,
                    float* loss_out, void* dlogits, int64_t ld_d,
                    void* workspace, size_t workspace_bytes, void* stream);
/* Synchronises `stream` and reports a device-side error recorded in `workspace` by the
 * last kd_loss_fwd_bwd (KD_ERR_LABEL_RANGE), else KD_OK. */
int kd_loss_check(const void* workspace, void* stream);
/* The student half of kd_loss_fwd_bwd's per-row statistics (the log_softmax normalisers of
 * DT:158-162 / LB:225-229 and of the HF causal-LM CE): stats_out fp32 [rows][4] =
 * {max, sum exp((s - max)/T), sum exp(s - max), 0} over the first V_s columns of each row,
 * 16-B aligned.  Hand it to kd_loss_fwd_bwd as params.s_stats with the same rows and T. */
int kd_loss_student_stats(const void* student_logits, int64_t ld_s, int V_s, int rows, float temperature,
                          float* stats_out, void* stream);

/* ------------------------------------------------------------------ GEMM ---- */
/* C[M,N] = epilogue(alpha * sum_k A[m,k] B[n,k]), bf16 operands, fp32 accumulation
 * (MFMA 16x16x32).  Replaces every torch.nn.functional.linear of the step (SigLIP,
 * projector, Qwen2, lm_head: HF5 siglip :250-322, llava_onevision :131-150,
 * qwen2 :35-140, llava_onevision :762) and their autograd dgrad / wgrad.
 *  a_layout K_MAJOR : A[m][k] at A + m*lda + k        MN_MAJOR : A stored [k][m]
 *  b_layout K_MAJOR : B[n][k] at B + n*ldb + k        MN_MAJOR : B stored [k][n]
 * epilogue, in order: v = alpha*(*alpha_dev if set)*acc + bias[n]; aux[m][n] = v (bf16);
 *   v = act(v); v += residual[m][n]; C = v or C += v (accumulate).
 * Requirements: 16-B aligned A/B; ld % 8 == 0; K % 8 == 0 for K-major operands,
 * rows % 8 == 0 for MN-major ones.  Any M/N/K otherwise (tails read as zeros). */
typedef enum { KD_LAYOUT_K_MAJOR = 0, KD_LAYOUT_MN_MAJOR = 1 } kd_layout;
typedef enum { KD_DTYPE_BF16 = 0, KD_DTYPE_F32 = 1, KD_DTYPE_FP8_E4M3 = 2 } kd_dtype;
/* KD_ACT_SWIGLU: Qwen2MLP's act_fn(gate_proj(x)) * up_proj(x) (HF5 qwen2 :35-50) fused into
 * the gate|up GEMM: B = [gate; up] is [N = 2I][K] (I % 128 == 0), C is [M][I] =
 * silu(v[:, :I]) * v[:, I:] with v = alpha * acc rounded to bf16 first (as the unfused
 * GEMM output), aux (optional) receives v [M][2I] for the backward.  K-major operands,
 * bf16 C, no bias / residual / accumulate / split-K. */
/* Backward activations, fused into the DGRAD GEMM that produces the activation's output
 * gradient (any operand layouts; bf16 C; no bias / residual / accumulate; never split-K; aux =
 * the forward pre-activation, READ):
 * KD_ACT_DGELU_TANH: C[m][n] = v * gelu_tanh'(aux[m][n])      (SigLIP MLP: fc2 dgrad -> dfc1-out)
 * KD_ACT_DSWIGLU   : aux = [gate | up] [M][2N] (ld_aux >= 2N), C is [M][2N] (ldc >= 2N):
 *   C[m][n] = v * up * silu'(gate), C[m][N + n] = v * silu(gate)  (Qwen2 MLP: down dgrad -> dgate|dup)
 * with v = alpha * acc rounded to bf16 first, so C equals the unfused GEMM followed by the
 * activation-backward kernel bit for bit. */
typedef enum { KD_ACT_NONE = 0, KD_ACT_GELU_TANH = 1, KD_ACT_GELU_ERF = 2, KD_ACT_SILU = 3,
               KD_ACT_SWIGLU = 4, KD_ACT_DGELU_TANH = 5, KD_ACT_DSWIGLU = 6 } kd_act;

typedef struct {
    int32_t M, N, K;
    int32_t a_layout, b_layout;
    const void* A; int64_t lda;
    const void* B; int64_t ldb;
    void* C; int64_t ldc;
    int32_t c_dtype;          /* kd_dtype                                   */
    int32_t accumulate;       /* 1: C += result                             */
    float alpha;
    const float* alpha_dev;   /* optional device scalar multiplied into alpha */
    const void* bias;         /* optional [N]                               */
    int32_t bias_dtype;       /* kd_dtype of bias                           */
    int32_t act;              /* kd_act                                     */
    const void* residual;     /* optional bf16 [M][N] added after act       */
    int64_t ldr;
    void* aux;                /* optional bf16 [M][N] pre-activation output */
    int64_t ld_aux;
    int32_t residual_row_mod; /* >0: residual row index = m % residual_row_mod (SigLIP pos-emb) */
    int32_t variant;          /* 0 auto (cost model); forced (tests/tools): 1 128x128 4-wave; 2|5 / 3|6 / 4|7
                                 256x256 / 256x128 / 128x256 8-wave; 16 256x256 4-wave (v8, AGPR
                                 accumulators); 24 = 16; 21 stream-K on 16 (256 workgroups take equal runs
                                 of the tiles' k-steps, shared tiles folded from fp32 partial planes; needs
                                 workspace).  The A/B library (csrc/build.py --ab) also accepts the
                                 diagnostic / negative-result builds 17-20, 22, 23, 26-28 and 30 (v8n: 256x128
                                 4-wave at two workgroups per CU, bit-identical to 16; tools/README.md);
                                 this library rejects them. */
    int32_t split_k;          /* 0 auto (cost model, bounded by workspace); 1 off; >1 forced K splits */
    void* workspace;          /* optional fp32 split-K partials; NULL disables splitting */
    uint64_t workspace_bytes;
    int32_t ab_dtype;         /* operand dtype: KD_DTYPE_BF16 (0) or KD_DTYPE_FP8_E4M3 (fp8 path) */
    const float* a_scale;     /* fp8 path: per-row scale of A [M] (A = a_scale[m] * qa[m][k])     */
    const float* b_scale;     /* fp8 path: per-row scale of B [N] (per output channel)           */
    int32_t residual_dtype;   /* kd_dtype of residual: KD_DTYPE_BF16 (0) or KD_DTYPE_F32 (an fp32
                                 residual stream; then C must be fp32 and act NONE; bf16 path only) */
    const struct kd_qkv_scatter* qkv;   /* optional: q|k|v scatter epilogue (below); C unused */
    /* optional: per-row softmax statistics of C, emitted by the epilogue (the lm_head GEMM feeding
       kd_loss_fwd_bwd: the loss then skips its own pass over the logits, DT:155-192). For every
       row m and 256-column tile j, 8 floats at row_stats + (m * ceil(N / 256) + j) * 8, over the
       tile's bf16-rounded C (what the loss reads):
         [0] max over the tile's columns < N        [1] sum exp(c - [0])
         [2] max over its columns < row_stats_vs    [3] sum exp((c - [2]) * row_stats_inv_t)
         [4..7] top-2 over columns < row_stats_vs: value, index (int32 bits), value, index
                (larger value first, lower index on ties; only when row_stats_top2)
       Requires bf16 C, K-major bf16 operands, no bias / activation / residual / aux /
       accumulate; runs the 256x256 kernel without split-K. */
    float* row_stats;
    int32_t row_stats_vs;      /* column bound of [2..7] (the student vocab V_s); <= 0: N */
    float row_stats_inv_t;     /* 1 / T of [3] */
    int32_t row_stats_top2;
    /* optional: B is PRE-TILED (kd_gemm_pretile below) instead of a [N][K] matrix: every DMA of the
       256x256 kernel then reads one contiguous KiB (whole cache lines). K-major bf16 operands, the
       256x256 v8 kernel (variant 0 / 16 / 24), no split-K or row_stats; bit-identical results. For
       frozen weights (the teacher): tile once, multiply many times. ldb is ignored. */
    int32_t b_pretiled;
} kd_gemm_desc;

/* Pre-tiled B for kd_gemm_desc.b_pretiled: W [N][K] (row stride ldw, K % 8 == 0) rewritten as
 * [ceil(N / 256) tiles][ceil(K / 32) stages][256 rows][32 k] -- each stage the exact LDS image the
 * 256x256 kernel stages (16-B chunks swizzled per row), zero past N and K.  glu = 1: the layout of
 * the fused SwiGLU GEMM (act KD_ACT_SWIGLU, N = 2I, I % 128 == 0): tile t holds gate rows
 * [128 t, 128 t + 128) then up rows [I + 128 t, I + 128 t + 128).  Enqueued on `stream`. */
size_t kd_gemm_pretile_size(int N, int K, int glu);
int kd_gemm_pretile(const void* W, int64_t ldw, int N, int K, int glu, void* out, void* stream);
/* q|k|v scatter epilogue of a fused projection GEMM (the attention input of SigLIP / Qwen2:
 * HF5 siglip :250-270, qwen2 :80-110 view / transpose / apply_rotary_pos_emb): the output tile,
 * bias added and rounded to bf16 as the plain GEMM's C, is written straight to head-major
 * q [B, nq, S, hdp], k / v [B, nkv, S, hdp] (rows m = b * S + s; columns [q heads | k heads |
 * v heads] of hd), RoPE rotate_half applied to q and k when cos_t / sin_t ([S, hd/2] fp32) are
 * given, the [hd, hdp) padding zeroed — kd_qkv_split's result bit for bit, without C's round
 * trip through HBM.  K-major bf16 operands, no activation / residual / aux / accumulate /
 * split-K, the tiled kernels' shapes (M, N >= 128, M * N >= 2^20); hd % 8 == 0; with RoPE
 * hd % 16 == 0 and 128 % hd == 0. */
typedef struct kd_qkv_scatter {
    void* q; void* k; void* v;
    const float* cos_t; const float* sin_t;
    int32_t S, nq, nkv, hd, hdp;
} kd_qkv_scatter;
/* fp8 path (ab_dtype = KD_DTYPE_FP8_E4M3; the fp8 teacher of BASELINE config c4): A and B are
 * OCP e4m3 bytes, both K-major, K % 16 == 0, lda / ldb % 16 == 0 (bytes = elements), 16-B
 * aligned; C = epilogue(alpha * a_scale[m] * b_scale[n] * sum_k qa[m][k] qb[n][k]) with the
 * epilogue above (bias / act / residual / SWIGLU; aux only with SWIGLU), bf16 C, no split-K.  MFMA
 * v_mfma_scale_f32_32x32x64_f8f6f4 (unit block scales), fp32 accumulation. */

/* Bytes of workspace the auto (or forced) split-K plan for `desc` wants; 0 = no split.
 * With split-K the K range is cut into S chunks, each an independent tile grid writing
 * fp32 partials, and one reduce pass applies the epilogue above (deterministic). */
size_t kd_gemm_workspace_size(const kd_gemm_desc* desc);

/* The plan kd_gemm would run for `desc` (inspection only; no device work): kernel variant
 * (1 v1, 2/3/4 v3 256x256 / 256x128 / 128x256, 16 v8, 21 stream-K v8), K splits (stream-K:
 * the partial planes its workspace holds), and how many leading tiles (whole waves of 256)
 * run unsplit before the split tail (0 = every tile split). */
int kd_gemm_plan(const kd_gemm_desc* desc, int32_t* variant, int32_t* split_k, int32_t* dp_tiles);

int kd_gemm(const kd_gemm_desc* desc, void* stream);

/* ------------------------------------------------------------- attention ---- */
/* Fused flash attention (scores = q k^T * hd^-0.5, fp32 softmax), replacing the SDPA /
 * eager attention transformers dispatches for Qwen2 (causal GQA, HF5 qwen2 :80-140) and
 * SigLIP (non-causal MHA, HF5 siglip :250-307).
 * q [B,H,S,hdp], k/v [B,HKV,S,hdp] bf16 with head dim zero-padded to hdp in {64,96,128};
 * o [B,S,H,hd] bf16 (token-major), lse [B,H,S] fp32 (may be NULL in forward-only use). */
typedef struct {
    const void* q; const void* k; const void* v;
    void* o; float* lse;
    int32_t B, H, HKV, S, hd, hdp, causal;
} kd_attn_desc;
int kd_attn_fwd(const kd_attn_desc* desc, void* stream);

/* Backward: dO [B,S,H,hd]; delta workspace [B,H,S] fp32 (rowsum(dO * O), computed by the dQ
 * kernel and read by the dK/dV kernel); dq fp32 [B,H,S,hdp] (scaled, overwritten); dk/dv bf16
 * [B,HKV,S,hdp]. Two kernels (dQ per query block, then dK/dV per key block and query head), no
 * atomics. GQA (H > HKV) needs `workspace` of
 * kd_attn_bwd_workspace_size() bytes for the per-query-head dK/dV partials. */
typedef struct {
    const void* q; const void* k; const void* v; const void* o; const void* dO;
    const float* lse; float* delta; float* dq; void* dk; void* dv;
    int32_t B, H, HKV, S, hd, hdp, causal;
    void* workspace; uint64_t workspace_bytes;
    /* optional: the token-major bf16 [B*S, ld_qkv] gradient of a fused q|k|v projection, columns
     * [0, H hd) dq | [H hd, (H + HKV) hd) dk | [(H + HKV) hd, (H + 2 HKV) hd) dv -- kd_qkv_merge's layout,
     * bit-identical to kd_attn_bwd + kd_qkv_merge -- written directly; dq / dk / dv are then not
     * written (may be NULL). NULL: the head-major dq / dk / dv above. */
    void* dqkv; int64_t ld_qkv;
    /* with dqkv and GQA: RoPE tables [S, hd/2] fp32 (kd_qkv_split's); dq and dk are rotated back as
     * kd_qkv_merge does (hd == hdp, hd % 32 == 0). NULL: no rotation. */
    const float* cos_t; const float* sin_t;
} kd_attn_bwd_desc;
size_t kd_attn_bwd_workspace_size(const kd_attn_bwd_desc* desc);
int kd_attn_bwd(const kd_attn_bwd_desc* desc, void* stream);

/* ------------------------------------------------------------ layer ops ---- */
/* LayerNorm (rms = 0; nn.LayerNorm, SigLIP, HF5 siglip :325-357, :567) or RMSNorm
 * (rms = 1; Qwen2RMSNorm, HF5 qwen2 :35-55) over rows of D (D % 8 == 0, D <= 4096).
 * x: kd_dtype x_dtype (bf16, or fp32 for an fp32 residual stream); y bf16.
 * mean/rstd fp32 [R] saved for backward (mean unused for RMS, may be NULL). */
int kd_norm_fwd(int rms, const void* x, int64_t ldx, const void* weight, const void* bias, void* y, int64_t ldy,
                float* mean, float* rstd, int R, int D, float eps, int x_dtype, void* stream);
/* dx (bf16, or += when dx_accum) and fp32 dweight/dbias (+= when accum_w); D <= 2048. */
size_t kd_norm_bwd_workspace_size(int R, int D);
int kd_norm_bwd(int rms, const void* x, int64_t ldx, const void* weight, const void* dy, int64_t lddy,
                const float* mean, const float* rstd, void* dx, int64_t lddx, int dx_accum,
                float* dweight, float* dbias, int accum_w, void* workspace, size_t workspace_bytes,
                int R, int D, int x_dtype, void* stream);
/* q/k/v split of a fused projection output qkv [B*S, (nq+2nkv)*hd] into padded head-major
 * q/k/v (+ RoPE rotate_half with fp32 cos/sin tables [S, hd/2] when non-NULL; HF5 qwen2
 * apply_rotary_pos_emb) and its transpose for the backward (dq fp32). */
int kd_qkv_split(const void* qkv, int64_t ld, void* q, void* k, void* v, const float* cos_t, const float* sin_t,
                 int B, int S, int nq, int nkv, int hd, int hdp, void* stream);
int kd_qkv_merge(const float* dq, const void* dk, const void* dv, void* dqkv, int64_t ld, const float* cos_t,
                 const float* sin_t, int B, int S, int nq, int nkv, int hd, int hdp, void* stream);
/* SwiGLU of Qwen2MLP: h = silu(gate) * up with gu = [gate | up] (width 2I). */
int kd_swiglu_fwd(const void* gu, int64_t ldg, void* h, int64_t ldh, int M, int I, void* stream);
int kd_swiglu_bwd(const void* gu, int64_t ldg, const void* dh, int64_t ldh, void* dgu, int64_t ldd, int M, int I,
                  void* stream);
/* dx = dy * act'(pre) for kd_act (gelu_pytorch_tanh: SigLIP MLP; gelu: projector). */
int kd_act_bwd(const void* pre, const void* dy, void* dx, int64_t n, int act, void* stream);
/* SigLIP patch embedding as im2col: pixels [NI,3,img,img] (kd_dtype) -> [NI*(img/ps)^2, Kp]
 * bf16 with k = c*ps*ps + kh*ps + kw, zero padded to Kp (HF5 siglip :116-186). */
int kd_patchify(const void* pixels, int pixel_dtype, void* out, int NI, int img, int ps, int Kp, void* stream);
/* inputs_embeds assembly = embed_tokens(ids) + masked_scatter of the packed image features
 * (HF5 llava_onevision :280-343, :510-513).  src[t] >= 0: feature row; -1: image_newline;
 * -2: token embedding.  err (device int) is OR-ed with 1 on an id outside [0, vocab). */
int kd_embed_assemble(const int64_t* ids, const int32_t* src, const void* table, const void* feats,
                      const void* newline, void* out, int M, int H, int vocab, int32_t* err, void* stream);
/* Device-side index map for kd_embed_assemble: the j-th image token (id == image_token)
 * of sample b reads map[b*map_ld + j] (feature row or -1 = newline), text tokens -2.
 * err |= 2 when a sample's image-token count differs from map_len[b]. */
int kd_image_src_map(const int64_t* ids, int B, int L, int64_t image_token, const int32_t* map, int map_ld,
                     const int32_t* map_len, int32_t* src, int32_t* err, void* stream);
int kd_embed_bwd(const int64_t* ids, const int32_t* src, const void* dout, float* dtable, void* dfeats,
                 float* dnewline, int M, int H, void* stream);
/* bias gradient: out[n] (+)= sum_m dy[m][n] (fp32). */
int kd_colsum(const void* dy, int64_t ld, int M, int N, float* out, int accumulate, void* stream);
/* hook feature pooling (DT:243-244): out[g][d] = mean_p x[g*P+p][d] (fp32), and its backward. */
int kd_row_group_mean(const void* x, int64_t ld, int G, int P, int D, float* out, void* stream);
int kd_row_group_mean_bwd(const float* dpool, int G, int P, int D, void* dx, int64_t ld, const float* scale_dev,
                          void* stream);
/* NT-Xent (DT:246-248 + contrastive_loss DT:393-416): loss_out[0] = weight * loss,
 * loss_out[1] = loss; dfs = d(weight*loss)/d(fs) * grad_scale (may be NULL). n <= 64. */
int kd_ntxent(const float* fs, const float* ft, int n, int D, float tau, float weight, float* loss_out,
              float* dfs, float grad_scale, void* stream);
/* torch.optim.AdamW step (DT:198-201) on flat fp32 master params with a bf16 working copy;
 * gscale (device, optional) multiplies the gradient first.  skip_words (device, n_skip <= 64
 * int32, optional): if any is nonzero the step changes nothing — pass the step's error words
 * (kd_loss_params.err_out, kd_model_forward's err) so that a batch the reference would have
 * rejected (DT:166) never updates the weights, without a host wait before the update. */
int kd_adamw(float* param, void* param_bf16, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t n,
             float lr, float beta1, float beta2, float eps, float weight_decay, int step, const float* gscale,
             const int32_t* skip_words, int n_skip, void* stream);
/* out[i] = a[i] * b[i], i < n (device scalars: e.g. the upstream gradient times the
 * dlogits scale of kd_loss_params.dscale, for kd_gemm's alpha_dev). */
int kd_scalar_mul(const float* a, const float* b, float* out, int n, void* stream);
/* y[i] = x[i] * (*s_dev), i < n (s_dev NULL: a copy; y may alias x): e.g. the NT-Xent feature gradient
 * times the upstream gradient, the hook gradient kd_model_backward takes. */
int kd_scale_f32(const float* x, const float* s_dev, float* y, int64_t n, void* stream);
/* out[0] += sum x^2 (gradient norm). */
int kd_sumsq(const float* x, int64_t n, float* out, void* stream);
/* bytes zero bytes at ptr, stream-ordered (optimizer.zero_grad() on the flat gradient:
 * torch.optim.Optimizer.zero_grad(set_to_none=False) that Lightning calls after each step). */
int kd_zero(void* ptr, uint64_t bytes, void* stream);
int kd_cast_f32_bf16(const float* x, void* y, int64_t n, void* stream);
/* Read `bytes` at `ptr` once (16-B loads; grid workgroups of 256 threads, <= 0: automatic) so that
 * the next kernel finds them in the Infinity Cache / L2 (weights read cold a step after their last use). */
int kd_prefetch(const void* ptr, uint64_t bytes, int grid, void* stream);
/* y (fp32) = x (bf16), n elements (the bf16 gradient all-reduce buckets, dp.GradSync). */
int kd_cast_bf16_f32(const void* x, float* y, int64_t n, void* stream);
/* fp8 row quantisation (the fp8 GEMM's operands): per row r of x (bf16 [R][K], K % 16 == 0)
 * scale[r] = amax_r / 448 (1 for an all-zero row) and q[r][k] = e4m3(clamp(x[r][k] * 448 /
 * amax_r, +-448)), round to nearest even (OCP e4m3fn bytes). */
int kd_quant_rows_fp8(const void* x, int64_t ldx, int R, int K, void* q, int64_t ldq, float* scale, void* stream);

/* ------------------------------------------------------ depth transform ---- */
/* Depth image -> 3-channel uint8 image (normalised depth, Prewitt gradient magnitude,
 * Prewitt gradient angle), replacing CustomSUNRGBDDatasetOneVision.
 * convert_depth_image_into_3D (dataset/dataloader/OneVision/CustomSUNRGBDDatasetOneVision.py:64-112:
 * per-image min/max normalisation to uint8, scipy.ndimage.convolve with the Prewitt kernels in
 * mode='reflect', sqrt / arctan2, safe_normalize to uint8, np.dstack).
 * depth: [B, H, W] of dtype 0 = uint16 (the PNG's 16-bit samples), 1 = int32 (PIL mode "I"),
 * 2 = float32; out: [B, H, W, 3] uint8.  Each image is normalised by its own range. */
size_t kd_depth_to_3ch_workspace_size(int B, int H, int W);
int kd_depth_to_3ch(const void* depth, int dtype, int B, int H, int W, uint8_t* out, void* workspace,
                    size_t workspace_bytes, void* stream);

/* ------------------------------------------------ image preprocessing ---- */
/* The image half of the reference's collate_fn (DM:124-146, the LLaVA-OneVision processor on the
 * RGB / 3-channel depth uint8 images = transformers LlavaOnevisionImageProcessor._preprocess,
 * PIL backend).
 * kd_image_resize_u8: PIL Image.resize((out_w, out_h), BICUBIC) of an [H, W, 3] uint8 image
 *   (Pillow libImaging/Resample.c: int32 taps with 22 fraction bits, horizontal then vertical
 *   8-bit pass), bit-exact.  Same size = copy.  Downscale factor <= 15.
 * kd_anyres_tiles: pixel_values [n_out, 3, patch, patch] (float32 or bf16) of one image:
 *   tile 0 from `base` (the image resized to patch x patch), tiles 1..(bh/patch)*(bw/patch) cut
 *   from the (bh, bw) canvas holding `resized` ([nh, nw, 3], the aspect-preserving resize)
 *   centred on zeros (get_image_patches / _pad_for_patching / divide_to_patches), rescaled by
 *   1/255 and normalised with mean_std_host = {mean[3], std[3]}; tiles past the image's own
 *   count are zero (_pad_for_batching).  out_dtype: 0 = float32, 1 = bf16. */
size_t kd_image_resize_workspace_size(int H, int W, int out_h, int out_w);
int kd_image_resize_u8(const uint8_t* in, int H, int W, uint8_t* out, int out_h, int out_w, void* workspace,
                       size_t workspace_bytes, void* stream);
int kd_anyres_tiles(const uint8_t* base, const uint8_t* resized, int nh, int nw, int bh, int bw, int patch,
                    int n_out, const float* mean_std_host, void* out, int out_dtype, void* stream);

/* ------------------------------------------------------------ generate() ---- */
/* Student generate() (evaluation/onevisionv3/evaluate_onevision.py:185-195: greedy,
 * max_new_tokens=32, repetition_penalty=1.2, no_repeat_ngram_size=2).
 * The sequence length may live on the device (cur_dev, int32: tokens in the sequence, the one
 * being decoded included) so that a decode step has fixed arguments and replays from one HIP
 * graph; with cur_dev NULL the host value (n / len) is used.
 * kd_attn_decode: SDPA of one new token per head against the KV cache of a layer:
 *   q [H, hdp] bf16 (head-major, RoPE applied), k_new/v_new [HKV, hdp] the token's own key/value
 *   (stored into the caches at position n - 1), caches [HKV, smax, hdp] bf16, o [H, hd] bf16;
 *   scale hd^-0.5, fp32 softmax over positions [0, n).
 * kd_gen_select: RepetitionPenaltyLogitsProcessor + NoRepeatNGramLogitsProcessor + greedy argmax
 *   (lowest index on ties) over one row of bf16 logits [V]; seq (int64, device) holds the len ids
 *   so far (prompt + generated) and receives the new token at seq[len]; out (optional) also
 *   receives it; *cur_dev (if given) supplies len and is incremented.  workspace >= V bytes.
 * kd_rope_row: cos/sin row of position *cur_dev - 1 ([.., hh] tables) into one-row buffers. */
size_t kd_attn_decode_workspace_size(int H, int hd, int smax);
int kd_attn_decode(const void* q, const void* k_new, const void* v_new, void* k_cache, void* v_cache, void* o,
                   int H, int HKV, int hd, int hdp, int smax, int n, const int32_t* cur_dev, void* workspace,
                   size_t workspace_bytes, void* stream);
/* Decode GEMV (one token row through an nn.Linear): y[N] bf16 = epilogue(W[N, K] x'[K]), fp32
 * accumulation; epilogue 0 none, 1 + bias[N], 2 + residual[N] (both in `extra`), 3 SwiGLU over the
 * adjacent gate|up weight: y[n] = silu(W[n] x') * (W[inter + n] x'), N = inter.  x' = x, or with
 * norm_w the Qwen2RMSNorm of x (weight norm_w, eps) as kd_norm_fwd computes it (fused prologue). */
int kd_gemv(const void* x, const void* W, int64_t ldw, const void* extra, void* y, int N, int K, int epilogue,
            int inter, const void* norm_w, float eps, void* stream);
int kd_gen_select(const void* logits, int V, int64_t* seq, int len, int32_t* cur_dev, float repetition_penalty,
                  int no_repeat_ngram, void* workspace, size_t workspace_bytes, int64_t* out, void* stream);
int kd_rope_row(const float* cos_table, const float* sin_table, int hh, const int32_t* cur_dev, float* cos_row,
                float* sin_row, void* stream);

/* --------------------------------------------------------- model runtime ---- */
/* One LLaVA-OneVision instance (SigLIP -> projector -> anyres pack -> Qwen2 -> lm_head)
 * whose forward and backward layer loops run in the library (SURVEY §8b "teacher forward"
 * / "student forward and backward with saved-activation workspace handles").  Replaces
 * the reference's model calls
 *   self.teacher_model(input_ids=, pixel_values=, image_sizes=, labels=)   DT:228 (no_grad)
 *   self.student_model(input_ids=, pixel_values=, image_sizes=, labels=)   DT:238
 * and the autograd backward Lightning runs through the student for `loss` (DT:123-131).
 * The arithmetic is transformers' (HF5 siglip :116-357, llava_onevision :131-150,
 * :280-343, :510-513, qwen2 :35-300).
 *
 * Weights: one flat bf16 buffer in the transformers-4.45 state_dict order whose layout
 * kd_model_param_info() defines (every tensor 16-B aligned; fused q|k|v and gate|up are
 * adjacent); gradients (trainable models): a flat fp32 buffer of the same layout,
 * accumulated into (+=).  The caller owns both; the handle only keeps the pointers. */
typedef struct {
    int32_t v_hidden, v_inter, v_layers, v_heads, v_patch, v_image;   /* SigLIP          */
    float v_eps;
    int32_t t_hidden, t_inter, t_layers, t_heads, t_kv_heads, t_head_dim, t_vocab, t_tie; /* Qwen2 */
    float t_rope_theta, t_eps;
    int64_t image_token_id;                                            /* 151646           */
    int32_t projector_act;                                             /* kd_act (GELU_ERF)*/
} kd_model_config;

/* Parameter layout: count, then per index the 4.45 name, flat offset and element count
 * (storage shape rows x cols; cols = 0 for 1-D).  The SigLIP conv weight is stored
 * im2col-flattened [hidden, 3*patch*patch padded to a multiple of 8]. */
int kd_model_param_count(const kd_model_config* cfg);
int64_t kd_model_param_numel(const kd_model_config* cfg);          /* flat length (padded) */
int kd_model_param_info(const kd_model_config* cfg, int index, char* name, int name_cap, int64_t* offset,
                        int64_t* numel, int64_t* rows, int64_t* cols);

/* anyres pack plan on the host (transformers' select_best_resolution / unpad_image /
 * pack_image_features for the 384-px tile grid of the -ov checkpoints, anyres_max_9): for
 * sample b with image_sizes_host[b] = (H, W), map_host[b][j] = the flattened vision-feature
 * row of its j-th image token, or -1 (image_newline); len_host[b] = its image-token count;
 * the rest of the row is -2.  The input of kd_image_src_map.  Tile layout of the feature
 * rows: tiles > 0 = `tiles` tiles per sample (sample b from tile b * tiles); tiles == 0 =
 * compact: each sample's REAL tiles only (1 + the grid: 2 for 336x336, 5 for 480x640),
 * sample b from the sum of the earlier samples' counts — what the reference's model runs
 * through the vision tower (HF5 llava_onevision: pixel_values unpadded per image_sizes). */
int kd_anyres_batch_map(const int64_t* image_sizes_host, int B, int tiles, int32_t* map_host, int map_ld,
                        int32_t* len_host);

typedef struct kd_model kd_model;
int kd_model_create(const kd_model_config* cfg, const void* weights, float* grad, kd_model** out);
void kd_model_destroy(kd_model* m);
/* freeze masks (DT:468-523): which regions receive weight gradients */
int kd_model_set_trainable(kd_model* m, int vision, int projector, int language);

/* fp32 residual streams: vision / language != 0 keeps that tower's hidden state x (the
 * stream every layer adds into: SigLIP encoder, Qwen2 decoder) in fp32 — the residual adds
 * in the o_proj / fc2 / down_proj GEMM epilogues in fp32, the norms read fp32 — instead of
 * rounding it to bf16 after every add (the reference's own precision: fp32 in LB / FB, the
 * residual adds of fp16 autocast in DT, which run in fp32).  Default off.  The fp8 GEMM adds
 * a bf16 residual only: a tower whose residual linears (SigLIP out_proj / fc2, Qwen2 o_proj /
 * down_proj) run in fp8 (kd_model_set_fp8_families) keeps a bf16 stream.  Changes the
 * forward / backward workspace sizes. */
int kd_model_set_residual_f32(kd_model* m, int vision, int language);

/* fp8 teacher (BASELINE config c4): e4m3 copies of every linear weight the forward's GEMMs
 * read (all 2-D weights but the patch-embedding conv, the position embedding and
 * embed_tokens) in a uint8 buffer with the bf16 buffer's element offsets, plus one fp32
 * scale per weight row (kd_model_fp8_scale_count floats, spec order).  quantize fills both
 * from the bound bf16 weights (kd_quant_rows_fp8 per weight); set_fp8 binds them (NULL
 * unbinds) for a model without a grad buffer: its forward then quantises each linear's
 * input rows per token and runs the fp8 GEMM (kd_gemm fp8 path). */
int64_t kd_model_fp8_scale_count(const kd_model* m);
int kd_model_quantize_fp8(const kd_model* m, void* q, float* scales, void* stream);
int kd_model_set_fp8(kd_model* m, const void* q, const float* scales);
/* Which linear families run on the fp8 path once fp8 weights are bound (default all); the
 * others keep the bf16 GEMM on the same weights.  e4m3 costs ~3.7 % rel-L2 per GEMM output
 * whatever the scaling (3 mantissa bits), and on the random-init teacher these
 * errors add in quadrature along the ~220 GEMMs of the forward, so a policy trades accuracy
 * for fp8 MFMA throughput family by family (tools/fp8_depth_study.py --families). */
typedef enum {
    KD_FP8_VISION = 1,      /* SigLIP q|k|v, out_proj, fc1, fc2                           */
    KD_FP8_PROJECTOR = 2,   /* multi_modal_projector linear_1 / linear_2                  */
    KD_FP8_LM_ATTN = 4,     /* Qwen2 q|k|v, o_proj                                        */
    KD_FP8_LM_MLP = 8,      /* Qwen2 gate|up, down_proj                                   */
    KD_FP8_LM_HEAD = 16,    /* lm_head                                                    */
    KD_FP8_ALL = 31
} kd_fp8_family;
int kd_model_set_fp8_families(kd_model* m, int families);

/* Row statistics of the lm_head logits (kd_gemm_desc.row_stats, same layout), written by the
 * lm_head GEMM's epilogue of every later kd_model_forward that produces logits: partials fp32
 * [B*L, ceil(vocab / 256), 8]; vs / inv_t / top2 as kd_gemm_desc.row_stats_*.  The lm_head then
 * runs bf16 (an fp8 lm_head family is ignored while this is set).  partials = NULL turns it off. */
int kd_model_set_row_stats(kd_model* m, float* partials, int vs, float inv_t, int top2);

/* Forward.  ids int64 [B, L]; pixels [n_tiles, 3, image, image] (kd_dtype: the batch's
 * vision tiles, e.g. the compact real tiles of kd_anyres_batch_map(tiles = 0)); src int32 [B*L]
 * from kd_image_src_map; rope_cos/rope_sin fp32 [L, head_dim/2] (Qwen2RotaryEmbedding:
 * inv_freq = 1 / theta^(2i/hd) in fp32, angle = pos * inv_freq).  save = 1 keeps every
 * activation the backward reads in `workspace` (the saved-activation handle: pass the
 * same pointer to kd_model_backward and leave it untouched until then).
 * Outputs: hn bf16 [B*L, t_hidden] (final-norm hidden state); post_ln (optional) bf16
 * [n_tiles*np, v_hidden] (the vision post_layernorm output the reference hooks, DT:100-121);
 * logits (optional) bf16 [B*L, vocab] (lm_head); kv_k / kv_v (optional, host arrays of
 * t_layers device pointers) receive each layer's roped keys / values [B, kv_heads, L,
 * head_dim] (generate()'s prefill).  err: kd_embed_assemble's error word. */
size_t kd_model_forward_workspace_size(const kd_model* m, int B, int L, int n_tiles, int save);
int kd_model_forward(kd_model* m, const int64_t* ids, const void* pixels, int pixel_dtype, const int32_t* src,
                     const float* rope_cos, const float* rope_sin, int B, int L, int n_tiles, int save,
                     void* workspace, size_t workspace_bytes, void* hn, void* post_ln, void* logits,
                     void* const* kv_k, void* const* kv_v, int32_t* err, void* stream);

/* Backward of a save = 1 forward (fwd_workspace) from dhn (bf16 [B*L, t_hidden], grad of
 * hn) and dpost (optional, fp32 [n_tiles, v_hidden]: the gradient w.r.t. each tile's MEAN post_ln
 * feature, the hook's pooling DT:243-244; spread as dpost / np over the tile's np rows in fp32,
 * never rounded to bf16 -- since ABI 7, was a bf16 [n_tiles*np, v_hidden] row gradient) into the
 * grad buffer (+=).  Weight
 * gradients run on wgrad_stream beside the dgrad chain on `stream`; `stream` waits for
 * all of it before returning.  Work already queued on wgrad_stream (e.g. the caller's
 * lm_head wgrad into a tied embedding) is ordered before the embedding backward.
 * on_layer_done (optional) marks a part of the gradient final as soon as its backward is
 * enqueued on `stream` / wgrad_stream (bucketed data-parallel all-reduce; a
 * callback that launches a collective first makes its stream wait for wgrad_stream):
 *   layer in [0, t_layers)      Qwen2 layer `layer`, top-down (after the final norm / lm_head);
 *   KD_CB_EMBED_PROJECTOR (-1)  embed_tokens, image_newline and the projector (ABI 9; fired when
 *                               the language model or the projector is trainable);
 *   KD_CB_VISION_LAYER(i)       SigLIP layer i, top-down, with post_layernorm (ABI 9; trainable
 *                               vision tower only).  The patch / position embeddings come last:
 *                               they are final when kd_model_backward returns. */
typedef void (*kd_layer_cb)(void* user, int layer);
#define KD_CB_EMBED_PROJECTOR (-1)
#define KD_CB_VISION_LAYER(i) (-2 - (i))
size_t kd_model_backward_workspace_size(const kd_model* m, int B, int L, int n_tiles);
int kd_model_backward(kd_model* m, const void* fwd_workspace, const int64_t* ids, const int32_t* src,
                      const float* rope_cos, const float* rope_sin, int B, int L, int n_tiles,
                      const void* dhn, const void* dpost, void* workspace, size_t workspace_bytes,
                      void* stream, void* wgrad_stream, kd_layer_cb on_layer_done, void* user);

/* GEMM timer (measurement): while enabled, every kd_gemm launch (the ABI entry and the
 * model runtime's) is bracketed by HIP events on its stream.  kd_timer_read synchronises
 * record i's end event and returns its key "<kind>:<M>x<N>x<K>:<f32|bf16>[:acc]", kind =
 * gemm_{k|n}{k|n} (A / B layout), gemm_kk_swiglu, gemm_f8 / gemm_f8_swiglu (fp8 path), its FLOPs
 * and milliseconds. */
void kd_timer_enable(int on);
int kd_timer_count(void);
int kd_timer_read(int i, char* key, int key_cap, double* flops, float* ms);
void kd_timer_reset(void);

#ifdef __cplusplus
}
#endif
#endif /* KDSTEP_H */
