// Model runtime: the LLaVA-OneVision forward and backward layer loops in C++ (include/kdstep.h
// "model runtime").  The reference calls transformers' LlavaOnevisionForConditionalGeneration
// for the teacher under no_grad (DT:228) and for the student (DT:238), and Lightning's
// autograd runs the student backward; here both loops issue the library's kernels straight
// from C++ onto the caller's HIP streams (one host call per model per step instead of
// ~700-1000 Python launches).
//
// Memory: the caller hands in one workspace per call, sized by the *_workspace_size
// queries; a bump allocator carves it in a fixed order, so the backward re-derives every
// saved activation's address from the forward's workspace pointer alone.  save = 1 keeps
// one buffer per layer for each activation the backward reads; save = 0 reuses one set of
// buffers across layers (stream order makes the reuse safe).
//
// Weight gradients (dW = dY^T X and bias column sums) run on a second stream beside the
// dgrad chain (dX = dY W), which is what the next layer waits for: the student's small-N
// backward GEMMs (hidden 896, SigLIP 1152) leave CUs idle that the other stream fills.
// The dgrad chain waits on the lane only before it updates dx in place (the lane reads
// dx); every other buffer the lane reads is rewritten only after such a wait (see
// lm_backward), so single buffers suffice.
#include "common.h"
#include "launchers.h"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

namespace kd {

// ================================================================ GEMM timer ====
namespace {
struct TimerRec {
    std::string key;
    double flops;
    hipEvent_t e0, e1;
};
std::mutex g_timer_mu;
std::vector<TimerRec> g_timer;
bool g_timer_on = false;
}  // namespace

int gemm_timed(const kd_gemm_desc* d, void* stream) {
    if (!g_timer_on) return launch_gemm(d, stream);
    TimerRec r;
    const bool swiglu = d->act == KD_ACT_SWIGLU, f8 = d->ab_dtype == KD_DTYPE_FP8_E4M3;
    // kinds: gemm_<A layout><B layout> (k = K-major, n = MN-major); the fused epilogues with extra
    // elementwise work of their own are kinds of their own (_swiglu forward; _dact: the dgrad
    // with the activation backward, KD_ACT_DGELU_TANH / KD_ACT_DSWIGLU)
    const bool dact = d->act == KD_ACT_DGELU_TANH || d->act == KD_ACT_DSWIGLU;
    r.key = swiglu ? std::string(f8 ? "gemm_f8_swiglu" : "gemm_kk_swiglu")
                   : (f8 ? std::string("gemm_f8") : std::string("gemm_") + (d->a_layout ? 'n' : 'k') + (d->b_layout ? 'n' : 'k') +
                                                        (dact ? "_dact" : ""));
    r.key += ":" + std::to_string(d->M) + "x" + std::to_string(d->N) + "x" + std::to_string(d->K) + ":" +
             (d->c_dtype == KD_DTYPE_F32 ? "f32" : "bf16") + (d->accumulate ? ":acc" : "");
    r.flops = 2.0 * d->M * d->N * d->K;
    (void)hipEventCreate(&r.e0);
    (void)hipEventCreate(&r.e1);
    (void)hipEventRecord(r.e0, as_stream(stream));
    const int st = launch_gemm(d, stream);
    (void)hipEventRecord(r.e1, as_stream(stream));
    std::lock_guard<std::mutex> g(g_timer_mu);
    g_timer.push_back(r);
    return st;
}

// ============================================================ parameter layout ====
namespace {

struct Spec {
    std::string name;
    int64_t rows, cols;   // storage shape (cols = 0: 1-D)
    int64_t offset, numel;
};

struct Cfg {
    kd_model_config c;
    int v_hd() const { return c.v_hidden / c.v_heads; }
    int v_hdp() const { return v_hd() <= 64 ? 64 : (v_hd() <= 80 ? 96 : 128); }   // attention head-dim padding
    int grid() const { return c.v_image / c.v_patch; }
    int np() const { return grid() * grid(); }
    int kpatch() const { return (3 * c.v_patch * c.v_patch + 7) / 8 * 8; }
    int qd() const { return c.t_heads * c.t_head_dim; }
    int kvd() const { return c.t_kv_heads * c.t_head_dim; }
};

// The order of modeling.param_specs (transformers-4.45 state_dict order), offsets aligned to
// 8 elements (16 B).
std::vector<Spec> make_specs(const Cfg& C, int64_t* total) {
    const kd_model_config& c = C.c;
    std::vector<Spec> S;
    int64_t off = 0;
    auto add = [&](const std::string& n, int64_t r, int64_t cl) {
        off = (off + 7) / 8 * 8;
        const int64_t ne = cl ? r * cl : r;
        S.push_back({n, r, cl, off, ne});
        off += ne;
    };
    const std::string vp = "vision_tower.vision_model.";
    const int64_t D = c.v_hidden, I = c.v_inter;
    add(vp + "embeddings.patch_embedding.weight", D, C.kpatch());
    add(vp + "embeddings.patch_embedding.bias", D, 0);
    add(vp + "embeddings.position_embedding.weight", C.np(), D);
    for (int i = 0; i < c.v_layers; ++i) {
        const std::string p = vp + "encoder.layers." + std::to_string(i) + ".";
        for (const char* n : {"q", "k", "v"}) add(p + "self_attn." + n + "_proj.weight", D, D);
        for (const char* n : {"q", "k", "v"}) add(p + "self_attn." + n + "_proj.bias", D, 0);
        add(p + "self_attn.out_proj.weight", D, D);
        add(p + "self_attn.out_proj.bias", D, 0);
        add(p + "layer_norm1.weight", D, 0);
        add(p + "layer_norm1.bias", D, 0);
        add(p + "mlp.fc1.weight", I, D);
        add(p + "mlp.fc1.bias", I, 0);
        add(p + "mlp.fc2.weight", D, I);
        add(p + "mlp.fc2.bias", D, 0);
        add(p + "layer_norm2.weight", D, 0);
        add(p + "layer_norm2.bias", D, 0);
    }
    add(vp + "post_layernorm.weight", D, 0);
    add(vp + "post_layernorm.bias", D, 0);
    const int64_t H = c.t_hidden, TI = c.t_inter, qd = C.qd(), kd = C.kvd();
    add("multi_modal_projector.linear_1.weight", H, D);
    add("multi_modal_projector.linear_1.bias", H, 0);
    add("multi_modal_projector.linear_2.weight", H, H);
    add("multi_modal_projector.linear_2.bias", H, 0);
    add("image_newline", H, 0);
    const std::string lp = "language_model.model.";
    add(lp + "embed_tokens.weight", c.t_vocab, H);
    for (int i = 0; i < c.t_layers; ++i) {
        const std::string p = lp + "layers." + std::to_string(i) + ".";
        add(p + "self_attn.q_proj.weight", qd, H);
        add(p + "self_attn.k_proj.weight", kd, H);
        add(p + "self_attn.v_proj.weight", kd, H);
        add(p + "self_attn.q_proj.bias", qd, 0);
        add(p + "self_attn.k_proj.bias", kd, 0);
        add(p + "self_attn.v_proj.bias", kd, 0);
        add(p + "self_attn.o_proj.weight", H, qd);
        add(p + "mlp.gate_proj.weight", TI, H);
        add(p + "mlp.up_proj.weight", TI, H);
        add(p + "mlp.down_proj.weight", H, TI);
        add(p + "input_layernorm.weight", H, 0);
        add(p + "post_attention_layernorm.weight", H, 0);
    }
    add(lp + "norm.weight", H, 0);
    if (!c.t_tie) add("language_model.lm_head.weight", c.t_vocab, H);
    *total = (off + 7) / 8 * 8;
    return S;
}

// The fp8 linears: every 2-D weight a GEMM reads as its B operand, i.e. all but the
// patch-embedding conv (K = 3*14*14, bf16), the position embedding (a residual) and
// embed_tokens (a gather; the tied student head is never fp8).  Scales follow in spec order.
std::vector<int64_t> fp8_scale_offsets(const Cfg& C, const std::vector<Spec>& S, int64_t* total) {
    std::vector<int64_t> off(S.size(), -1);
    int64_t n = 0;
    for (size_t i = 0; i < S.size(); ++i) {
        const std::string& nm = S[i].name;
        if (S[i].cols == 0 || nm.find("patch_embedding") != std::string::npos ||
            nm.find("position_embedding") != std::string::npos || nm.find("embed_tokens") != std::string::npos)
            continue;
        off[i] = n;
        n += S[i].rows;
    }
    (void)C;
    *total = n;
    return off;
}

bool cfg_ok(const kd_model_config* c) {
    return c && c->v_hidden > 0 && c->v_heads > 0 && c->v_hidden % c->v_heads == 0 && c->v_layers >= 0 &&
           c->v_patch > 0 && c->v_image >= c->v_patch && c->t_hidden > 0 && c->t_heads > 0 &&
           c->t_kv_heads > 0 && c->t_heads % c->t_kv_heads == 0 && c->t_layers >= 0 && c->t_vocab > 0 &&
           (c->t_head_dim == 64 || c->t_head_dim == 128) && c->v_hidden / c->v_heads <= 128;
}

// per-layer parameter indices into the spec list
enum VisField { VQW, VKW, VVW, VQB, VKB, VVB, VOW, VOB, VLN1W, VLN1B, VFC1W, VFC1B, VFC2W, VFC2B, VLN2W, VLN2B, VNF };
enum LmField { LQW, LKW, LVW, LQB, LKB, LVB, LOW, LGW, LUW, LDW, LINW, LPOSTW, LNF };

}  // namespace

}  // namespace kd

struct kd_model {
    kd::Cfg C;
    std::vector<kd::Spec> specs;
    int64_t numel = 0;
    const kd::bf16* w = nullptr;
    float* g = nullptr;
    int train_vision = 0, train_projector = 0, train_language = 0;
    int lane_split_k = 0;     // split-K of the lane's GEMMs (KD_WGRAD_SPLIT_K; 0 = cost model)
    // fp32 residual streams (kd_model_set_residual_f32): the SigLIP / Qwen2 hidden state x that
    // every layer adds into is kept in fp32 (GEMM epilogues add the residual in fp32 and write
    // fp32; the norms read fp32) instead of being rounded to bf16 after every add
    int rf32_v = 0, rf32_t = 0;
    std::vector<hipEvent_t> ev_pool;
    size_t ev_next = 0;
    // fp8 teacher (BASELINE config c4): e4m3 copies of the linear weights (same element
    // offsets as `w`) and one fp32 scale per weight row at soff[param]; nullptr = bf16 path
    const uint8_t* f8q = nullptr;
    const float* f8s = nullptr;
    std::vector<int64_t> soff;   // per spec: first scale index (-1: not an fp8 linear)
    std::vector<int> fam;        // per spec: its kd_fp8_family bit (0: not an fp8 linear)
    int f8_families = KD_FP8_ALL;   // which families run on the fp8 path (kd_model_set_fp8_families)
    // lm_head row statistics for the KD loss (kd_model_set_row_stats); nullptr = off
    float* rst = nullptr;
    int rst_vs = 0, rst_top2 = 0;
    float rst_inv_t = 1.f;
    int64_t n_scales = 0;
    // spec indices
    int i_patch_w = 0, i_patch_b = 1, i_pos = 2, i_vis0 = 3, i_post_w, i_post_b, i_p1w, i_p1b, i_p2w, i_p2b, i_newline,
        i_embed, i_lm0, i_norm, i_head;

    int64_t off(int idx) const { return specs[idx].offset; }
    const kd::bf16* W(int idx) const { return w + off(idx); }
    float* G(int idx) const { return g + off(idx); }
    int vis(int layer, int f) const { return i_vis0 + layer * kd::VNF + f; }
    int lm(int layer, int f) const { return i_lm0 + layer * kd::LNF + f; }
    hipEvent_t event() {   // reused round-robin: a wait is enqueued long before its event comes round again
        if (ev_pool.empty()) {
            ev_pool.resize(1024);
            for (auto& e : ev_pool) (void)hipEventCreateWithFlags(&e, hipEventDisableTiming);
        }
        return ev_pool[ev_next++ % ev_pool.size()];
    }
};

namespace kd {
namespace {

constexpr size_t SPLITK_WS = (size_t)384 << 20;   // fp32 split-K partial planes per stream (ops.py GEMM_SPLITK_WS)

// bump allocator over a caller workspace; base == nullptr: sizing pass
struct Arena {
    char* base;
    size_t off = 0;
    explicit Arena(void* b) : base((char*)b) {}
    template <class T>
    T* take(size_t n) {
        off = (off + 255) & ~(size_t)255;
        T* p = base ? (T*)(base + off) : nullptr;
        off += n * sizeof(T);
        return p;
    }
};

// ------------------------------------------------------------- GEMM helpers ----
struct Op {   // one GEMM operand: pointer, leading dim, layout
    const void* p;
    int64_t ld;
    int layout;
};
inline Op km(const void* p, int64_t ld) { return {p, ld, KD_LAYOUT_K_MAJOR}; }   // [rows][k]
inline Op mn(const void* p, int64_t ld) { return {p, ld, KD_LAYOUT_MN_MAJOR}; }  // stored [k][rows]

struct GemmArgs {
    const void* bias = nullptr;
    int act = KD_ACT_NONE;
    const void* residual = nullptr;
    int64_t ldr = 0;
    void* aux = nullptr;
    int64_t ld_aux = 0;
    int residual_row_mod = 0;
    int accumulate = 0;
    int c_f32 = 0;
    int bias_f32 = 0;
    int split_k = 0;
    int res_f32 = 0;   // fp32 residual (then c_f32 too)
    const kd_qkv_scatter* qkv = nullptr;   // q|k|v scatter epilogue (C unused)
    float* row_stats = nullptr;            // lm_head row statistics (kd_gemm_desc.row_stats)
    int rs_vs = 0, rs_top2 = 0;
    float rs_inv_t = 1.f;
};

// split-K default of the runtime's GEMMs (KD_GEMM_SPLIT_K: 0 = the cost model, 1 = never split)
static const int g_split_default = ab_knob("KD_GEMM_SPLIT_K", 0);

int gemm(hipStream_t s, void* ws, int M, int N, int K, Op a, Op b, void* C, int64_t ldc, const GemmArgs& g) {
    kd_gemm_desc d;
    std::memset(&d, 0, sizeof(d));
    d.M = M; d.N = N; d.K = K;
    d.a_layout = a.layout; d.b_layout = b.layout;
    d.A = a.p; d.lda = a.ld; d.B = b.p; d.ldb = b.ld;
    d.C = C; d.ldc = ldc;
    d.c_dtype = g.c_f32 ? KD_DTYPE_F32 : KD_DTYPE_BF16;
    d.accumulate = g.accumulate;
    d.alpha = 1.f;
    d.bias = g.bias; d.bias_dtype = g.bias_f32 ? KD_DTYPE_F32 : KD_DTYPE_BF16;
    d.act = g.act;
    d.residual = g.residual; d.ldr = g.ldr;
    d.residual_dtype = g.res_f32 ? KD_DTYPE_F32 : KD_DTYPE_BF16;
    d.qkv = g.qkv;
    d.aux = g.aux; d.ld_aux = g.ld_aux;
    d.residual_row_mod = g.residual_row_mod;
    d.split_k = g.split_k ? g.split_k : g_split_default;
    if (d.split_k != 1 && ws) { d.workspace = ws; d.workspace_bytes = SPLITK_WS; }
    d.row_stats = g.row_stats; d.row_stats_vs = g.rs_vs; d.row_stats_inv_t = g.rs_inv_t; d.row_stats_top2 = g.rs_top2;
    return gemm_timed(&d, s);
}

// the dgrad GEMMs feeding an activation backward run it in their epilogue (KD_ACT_DGELU_TANH /
// KD_ACT_DSWIGLU) where the tiled GEMM kernels take the shape; KD_FUSE_DACT=0 turns it off (A/B)
static const bool g_fuse_dact = ab_knob("KD_FUSE_DACT", 1) != 0;
static bool fused_dact_ok(int64_t M, int64_t N) {
    return g_fuse_dact && M >= 128 && N >= 128 && N % 8 == 0 && M * N >= (int64_t)1 << 20;
}

#define KD_TRY(x)                    \
    do {                             \
        const int st__ = (x);        \
        if (st__ != KD_OK) return st__; \
    } while (0)

// the weight-gradient lane: a second stream ordered after the dgrad chain at each hand-off
struct Lane {
    kd_model* m;
    hipStream_t main, lane;
    void* ws;
    void begin() {   // lane waits for everything queued on the main stream so far
        hipEvent_t e = m->event();
        (void)hipEventRecord(e, main);
        (void)hipStreamWaitEvent(lane, e, 0);
    }
    hipEvent_t end() {
        hipEvent_t e = m->event();
        (void)hipEventRecord(e, lane);
        return e;
    }
    // dW[N_out, K_in] (fp32 +=) = dy[M, N_out]^T x[M, K_in]
    int wgrad(int M, int Nout, int Kin, const void* dy, int64_t lddy, const void* x, int64_t ldx, float* dW) {
        GemmArgs g;
        g.accumulate = 1;
        g.c_f32 = 1;
        g.split_k = m->lane_split_k;
        return gemm(lane, ws, Nout, Kin, M, mn(dy, lddy), mn(x, ldx), dW, Kin, g);
    }
    int colsum(const void* dy, int64_t ld, int M, int N, float* out) {
        return launch_colsum(dy, ld, M, N, out, 1, lane);
    }
};
inline void wait(hipStream_t s, hipEvent_t e) {
    if (e) (void)hipStreamWaitEvent(s, e, 0);
}

// ------------------------------------------------------ forward buffer plan ----
// the residual-stream tensors (x, x_mid, x_*_last) are bf16 or fp32 (kd_model::rf32_v / rf32_t)
struct VisLayerBufs {
    void *x, *x_mid;
    bf16 *h, *q, *k, *v, *o, *h2, *pre, *u;
    float *m1, *r1, *lse, *m2, *r2;
};
struct LmLayerBufs {
    void *x, *x_mid;
    bf16 *h, *q, *k, *v, *o, *h2, *gu, *a;
    float *r1, *lse, *r2;
};
struct FwdPlan {
    bf16* rows;
    std::vector<VisLayerBufs> vl;
    void* x_vis_last;             // vl.back() output (saved) / ping-pong
    bf16* x_vis_bf;               // x_vis_last as bf16 (the projector's GEMM operand; == x_vis_last if bf16)
    bf16* qkv_v;
    void* x_vis[2];               // save = 0 ping-pong
    float *pm, *pr;
    bf16 *ppre, *z, *feats;
    std::vector<LmLayerBufs> ll;
    void* x_lm_last;
    bf16* qkv_t;
    void* x_lm[2];
    float* rf;
    uint8_t* qa;    // fp8 path: the current linear's activation rows, e4m3 [M][K] ...
    float* sa;      // ... and their scales [M]
    void* splitk;
    size_t bytes;
};

// n_tiles: the vision tiles of the whole batch (the pixel rows; samples may have different counts)
FwdPlan plan_forward(const kd_model* m, int B, int L, int n_tiles, int save, void* base) {
    const Cfg& C = m->C;
    const kd_model_config& c = C.c;
    Arena A(base);
    FwdPlan P;
    const int NI = n_tiles, np = C.np();
    const int64_t NT = (int64_t)NI * np, D = c.v_hidden, Iv = c.v_inter, hdp = C.v_hdp();
    const int64_t M = (int64_t)B * L, H = c.t_hidden, TI = c.t_inter, qd = C.qd(), kvd = C.kvd(), hd = c.t_head_dim;
    P.rows = A.take<bf16>(NT * C.kpatch());
    const int64_t ev = m->rf32_v ? 4 : 2, et = m->rf32_t ? 4 : 2;   // residual-stream element bytes
    // vision
    P.vl.resize(c.v_layers);
    P.qkv_v = A.take<bf16>(NT * 3 * D);
    if (save) {
        for (int i = 0; i < c.v_layers; ++i) {
            VisLayerBufs& b = P.vl[i];
            b.x = A.take<char>(NT * D * ev);
            b.h = A.take<bf16>(NT * D);
            b.q = A.take<bf16>((int64_t)NI * c.v_heads * np * hdp);
            b.k = A.take<bf16>((int64_t)NI * c.v_heads * np * hdp);
            b.v = A.take<bf16>((int64_t)NI * c.v_heads * np * hdp);
            b.o = A.take<bf16>(NT * D);
            b.x_mid = A.take<char>(NT * D * ev);
            b.h2 = A.take<bf16>(NT * D);
            b.pre = A.take<bf16>(NT * Iv);
            b.u = A.take<bf16>(NT * Iv);
            b.m1 = A.take<float>(NT);
            b.r1 = A.take<float>(NT);
            b.lse = A.take<float>((int64_t)NI * c.v_heads * np);
            b.m2 = A.take<float>(NT);
            b.r2 = A.take<float>(NT);
        }
        P.x_vis_last = A.take<char>(NT * D * ev);
        P.x_vis[0] = P.x_vis[1] = nullptr;
    } else {
        VisLayerBufs b{};
        P.x_vis[0] = A.take<char>(NT * D * ev);
        P.x_vis[1] = A.take<char>(NT * D * ev);
        b.h = A.take<bf16>(NT * D);
        b.q = A.take<bf16>((int64_t)NI * c.v_heads * np * hdp);
        b.k = A.take<bf16>((int64_t)NI * c.v_heads * np * hdp);
        b.v = A.take<bf16>((int64_t)NI * c.v_heads * np * hdp);
        b.o = A.take<bf16>(NT * D);
        b.x_mid = A.take<char>(NT * D * ev);
        b.h2 = A.take<bf16>(NT * D);
        b.u = A.take<bf16>(NT * Iv);
        for (int i = 0; i < c.v_layers; ++i) {
            P.vl[i] = b;
            P.vl[i].x = P.x_vis[i & 1];
        }
        P.x_vis_last = P.x_vis[c.v_layers & 1];
    }
    P.x_vis_bf = m->rf32_v ? A.take<bf16>(NT * D) : (bf16*)P.x_vis_last;
    P.pm = A.take<float>(NT);
    P.pr = A.take<float>(NT);
    // projector
    P.ppre = save ? A.take<bf16>(NT * H) : nullptr;
    P.z = A.take<bf16>(NT * H);
    P.feats = A.take<bf16>(NT * H);
    // language model
    P.ll.resize(c.t_layers);
    P.qkv_t = A.take<bf16>(M * (qd + 2 * kvd));
    const bool fused_swiglu = TI % 128 == 0;
    if (save) {
        for (int i = 0; i < c.t_layers; ++i) {
            LmLayerBufs& b = P.ll[i];
            b.x = A.take<char>(M * H * et);
            b.h = A.take<bf16>(M * H);
            b.q = A.take<bf16>(M * qd);
            b.k = A.take<bf16>(M * kvd);
            b.v = A.take<bf16>(M * kvd);
            b.o = A.take<bf16>(M * qd);
            b.x_mid = A.take<char>(M * H * et);
            b.h2 = A.take<bf16>(M * H);
            b.gu = A.take<bf16>(M * 2 * TI);
            b.a = A.take<bf16>(M * TI);
            b.r1 = A.take<float>(M);
            b.lse = A.take<float>((int64_t)B * c.t_heads * L);
            b.r2 = A.take<float>(M);
        }
        P.x_lm_last = A.take<char>(M * H * et);
        P.x_lm[0] = P.x_lm[1] = nullptr;
    } else {
        LmLayerBufs b{};
        P.x_lm[0] = A.take<char>(M * H * et);
        P.x_lm[1] = A.take<char>(M * H * et);
        b.h = A.take<bf16>(M * H);
        b.q = A.take<bf16>(M * qd);
        b.k = A.take<bf16>(M * kvd);
        b.v = A.take<bf16>(M * kvd);
        b.o = A.take<bf16>(M * qd);
        b.x_mid = A.take<char>(M * H * et);
        b.h2 = A.take<bf16>(M * H);
        b.gu = fused_swiglu ? nullptr : A.take<bf16>(M * 2 * TI);
        b.a = A.take<bf16>(M * TI);
        for (int i = 0; i < c.t_layers; ++i) {
            P.ll[i] = b;
            P.ll[i].x = P.x_lm[i & 1];
        }
        P.x_lm_last = P.x_lm[c.t_layers & 1];
    }
    P.rf = A.take<float>(M);
    (void)hd;
    if (m->f8q) {   // the widest linear input of either tower
        const int64_t R = M > NT ? M : NT;
        int64_t Kx = D > Iv ? D : Iv;
        for (int64_t k : {H, qd, TI}) Kx = Kx > k ? Kx : k;
        P.qa = A.take<uint8_t>(R * Kx);
        P.sa = A.take<float>(R);
    } else {
        P.qa = nullptr;
        P.sa = nullptr;
    }
    P.splitk = A.take<char>(SPLITK_WS);
    P.bytes = A.off + 256;
    return P;
}

// ------------------------------------------------------------------ forward ----
// One nn.Linear of the forward: the bf16 MFMA GEMM, or on the fp8 path (weights bound by
// kd_model_set_fp8) the activation rows quantised to e4m3 with a per-row scale and the fp8
// GEMM against the e4m3 weight rows and their per-channel scales (kdstep.h, fp8 path).
// KD_PREFETCH_W=1 (A/B): a streaming read of a forward linear's weights (kd_prefetch) right before
// its GEMM -- every weight is read a whole step after its last use, and a GEMM that meets cold
// weights stalls on them tile by tile (tools/ab_cold.py --prefetch)
static const int g_prefetch_w = ab_knob("KD_PREFETCH_W", 0);

int lin(kd_model* m, const FwdPlan& P, hipStream_t s, int M, int N, int K, const bf16* x, int64_t ldx, int widx,
        void* out, int64_t ldo, const GemmArgs& g) {
    const bool f8 = m->f8q && m->soff[widx] >= 0 && (m->fam[widx] & m->f8_families) && !g.row_stats;
    if (g_prefetch_w)
        KD_TRY(launch_prefetch(f8 ? (const void*)(m->f8q + m->off(widx)) : (const void*)m->W(widx),
                               (uint64_t)N * K * (f8 ? 1 : 2), 0, s));
    if (!f8)
        return gemm(s, P.splitk, M, N, K, km(x, ldx), km(m->W(widx), K), out, ldo, g);
    KD_TRY(launch_quant_rows_f8(x, ldx, M, K, P.qa, K, P.sa, s));
    kd_gemm_desc d;
    std::memset(&d, 0, sizeof(d));
    d.M = M; d.N = N; d.K = K;
    d.a_layout = KD_LAYOUT_K_MAJOR; d.b_layout = KD_LAYOUT_K_MAJOR;
    d.A = P.qa; d.lda = K; d.B = m->f8q + m->off(widx); d.ldb = K;
    d.C = out; d.ldc = ldo; d.c_dtype = KD_DTYPE_BF16;
    d.accumulate = g.accumulate; d.alpha = 1.f;
    d.bias = g.bias; d.bias_dtype = g.bias_f32 ? KD_DTYPE_F32 : KD_DTYPE_BF16;
    d.act = g.act; d.residual = g.residual; d.ldr = g.ldr; d.aux = g.aux; d.ld_aux = g.ld_aux;
    d.residual_row_mod = g.residual_row_mod;
    d.split_k = 1;
    d.ab_dtype = KD_DTYPE_FP8_E4M3; d.a_scale = P.sa; d.b_scale = m->f8s + m->soff[widx];
    return gemm_timed(&d, s);
}

// the fused q|k|v projection + view / transpose (+ RoPE) of the attention input: one GEMM whose
// epilogue writes head-major q / k / v (kd_qkv_scatter) where the tiled kernels take the shape
// and the weight is on the bf16 path; else the GEMM into `qkv` and k_qkv_split (same bits).
// KD_FUSE_QKV=0 turns the fusion off (A/B).
static const bool g_fuse_qkv = ab_knob("KD_FUSE_QKV", 1) != 0;

int qkv_proj(kd_model* m, const FwdPlan& P, hipStream_t s, int M, int K, const bf16* x, int widx, const void* bias,
             bf16* qkv, void* q, void* k, void* v, const float* cs, const float* sn, int B, int S, int nq, int nkv,
             int hd, int hdp) {
    const int N = (nq + 2 * nkv) * hd;
    GemmArgs g;
    g.bias = bias;
    const bool fp8 = m->f8q && m->soff[widx] >= 0 && (m->fam[widx] & m->f8_families);
    if (g_fuse_qkv && !fp8 && M >= 128 && N >= 128 && N % 8 == 0 && (int64_t)M * N >= ((int64_t)1 << 20) &&
        hd % 8 == 0 && hdp % 8 == 0 && (!cs || (hd % 16 == 0 && 128 % hd == 0))) {
        kd_qkv_scatter sc{q, k, v, cs, sn, S, nq, nkv, hd, hdp};
        g.qkv = &sc;
        g.split_k = 1;
        if (g_prefetch_w) KD_TRY(launch_prefetch(m->W(widx), (uint64_t)N * K * 2, 0, s));
        return gemm(s, P.splitk, M, N, K, km(x, K), km(m->W(widx), K), nullptr, 0, g);
    }
    KD_TRY(lin(m, P, s, M, N, K, x, K, widx, qkv, N, g));
    return launch_qkv_split(qkv, N, q, k, v, cs, sn, B, S, nq, nkv, hd, hdp, s);
}

int vision_forward(kd_model* m, const FwdPlan& P, const void* pixels, int px_dtype, int NI, int save, void* post,
                   hipStream_t s) {
    const Cfg& C = m->C;
    const kd_model_config& c = C.c;
    const int np = C.np(), D = c.v_hidden, Iv = c.v_inter, hdp = C.v_hdp(), hd = C.v_hd();
    const int NT = NI * np;
    KD_TRY(launch_patchify(pixels, px_dtype, P.rows, NI, c.v_image, c.v_patch, C.kpatch(), s));
    void* x0 = c.v_layers ? P.vl[0].x : P.x_vis_last;
    const int f32 = m->rf32_v;
    {
        GemmArgs g;
        g.bias = m->W(m->i_patch_b);
        g.residual = m->W(m->i_pos);
        g.ldr = D;
        g.residual_row_mod = np;
        g.c_f32 = f32;
        KD_TRY(gemm(s, P.splitk, NT, D, C.kpatch(), km(P.rows, C.kpatch()), km(m->W(m->i_patch_w), C.kpatch()), x0, D, g));
    }
    for (int i = 0; i < c.v_layers; ++i) {
        const VisLayerBufs& b = P.vl[i];
        void* x_out = (i + 1 < c.v_layers) ? P.vl[i + 1].x : P.x_vis_last;
        KD_TRY(launch_norm_fwd(0, b.x, D, m->W(m->vis(i, VLN1W)), m->W(m->vis(i, VLN1B)), b.h, D, save ? b.m1 : nullptr,
                               save ? b.r1 : nullptr, NT, D, c.v_eps, s, f32));
        KD_TRY(qkv_proj(m, P, s, NT, D, b.h, m->vis(i, VQW), m->W(m->vis(i, VQB)), P.qkv_v, b.q, b.k, b.v, nullptr,
                        nullptr, NI, np, c.v_heads, c.v_heads, hd, hdp));
        {
            kd_attn_desc a{b.q, b.k, b.v, b.o, save ? b.lse : nullptr, NI, c.v_heads, c.v_heads, np, hd, hdp, 0};
            KD_TRY(launch_attn_fwd(&a, s));
        }
        {
            GemmArgs g;
            g.bias = m->W(m->vis(i, VOB));
            g.residual = b.x;
            g.ldr = D;
            g.res_f32 = g.c_f32 = f32;
            KD_TRY(lin(m, P, s, NT, D, D, b.o, D, m->vis(i, VOW), b.x_mid, D, g));
        }
        KD_TRY(launch_norm_fwd(0, b.x_mid, D, m->W(m->vis(i, VLN2W)), m->W(m->vis(i, VLN2B)), b.h2, D,
                               save ? b.m2 : nullptr, save ? b.r2 : nullptr, NT, D, c.v_eps, s, f32));
        {
            GemmArgs g;
            g.bias = m->W(m->vis(i, VFC1B));
            g.act = KD_ACT_GELU_TANH;
            g.aux = save ? b.pre : nullptr;
            g.ld_aux = Iv;
            KD_TRY(lin(m, P, s, NT, Iv, D, b.h2, D, m->vis(i, VFC1W), b.u, Iv, g));
        }
        {
            GemmArgs g;
            g.bias = m->W(m->vis(i, VFC2B));
            g.residual = b.x_mid;
            g.ldr = D;
            g.res_f32 = g.c_f32 = f32;
            KD_TRY(lin(m, P, s, NT, D, Iv, b.u, Iv, m->vis(i, VFC2W), x_out, D, g));
        }
    }
    if (post)
        KD_TRY(launch_norm_fwd(0, P.x_vis_last, D, m->W(m->i_post_w), m->W(m->i_post_b), post, D, save ? P.pm : nullptr,
                               save ? P.pr : nullptr, NT, D, c.v_eps, s, f32));
    if (f32)   // the projector's GEMM operand (hidden_states[-1], HF5 llava_onevision :131-150)
        KD_TRY(launch_cast_f32_bf16((const float*)P.x_vis_last, P.x_vis_bf, NT * (int64_t)D, s));
    return KD_OK;
}

int lm_forward(kd_model* m, const FwdPlan& P, const float* cs, const float* sn, int B, int L, int save, void* hn,
               void* const* kv_k, void* const* kv_v, hipStream_t s) {
    const kd_model_config& c = m->C.c;
    const int M = B * L, H = c.t_hidden, TI = c.t_inter, qd = m->C.qd(), kvd = m->C.kvd(), hd = c.t_head_dim;
    const bool fused = TI % 128 == 0;
    const int f32 = m->rf32_t;
    for (int i = 0; i < c.t_layers; ++i) {
        const LmLayerBufs& b = P.ll[i];
        void* x_out = (i + 1 < c.t_layers) ? P.ll[i + 1].x : P.x_lm_last;
        KD_TRY(launch_norm_fwd(1, b.x, H, m->W(m->lm(i, LINW)), nullptr, b.h, H, nullptr, save ? b.r1 : nullptr, M, H,
                               c.t_eps, s, f32));
        void* k = kv_k ? kv_k[i] : b.k;
        void* v = kv_v ? kv_v[i] : b.v;
        KD_TRY(qkv_proj(m, P, s, M, H, b.h, m->lm(i, LQW), m->W(m->lm(i, LQB)), P.qkv_t, b.q, k, v, cs, sn, B, L,
                        c.t_heads, c.t_kv_heads, hd, hd));
        {
            kd_attn_desc a{b.q, k, v, b.o, save ? b.lse : nullptr, B, c.t_heads, c.t_kv_heads, L, hd, hd, 1};
            KD_TRY(launch_attn_fwd(&a, s));
        }
        {
            GemmArgs g;
            g.residual = b.x;
            g.ldr = H;
            g.res_f32 = g.c_f32 = f32;
            KD_TRY(lin(m, P, s, M, H, qd, b.o, qd, m->lm(i, LOW), b.x_mid, H, g));
        }
        KD_TRY(launch_norm_fwd(1, b.x_mid, H, m->W(m->lm(i, LPOSTW)), nullptr, b.h2, H, nullptr, save ? b.r2 : nullptr, M,
                               H, c.t_eps, s, f32));
        if (fused) {   // SwiGLU in the gate|up GEMM's epilogue; gate|up kept only for the backward
            GemmArgs g;
            g.act = KD_ACT_SWIGLU;
            g.aux = save ? b.gu : nullptr;
            g.ld_aux = 2 * TI;
            KD_TRY(lin(m, P, s, M, 2 * TI, H, b.h2, H, m->lm(i, LGW), b.a, TI, g));
        } else {
            GemmArgs g;
            KD_TRY(lin(m, P, s, M, 2 * TI, H, b.h2, H, m->lm(i, LGW), b.gu, 2 * TI, g));
            KD_TRY(launch_swiglu_fwd(b.gu, 2 * TI, b.a, TI, M, TI, s));
        }
        {
            GemmArgs g;
            g.residual = b.x_mid;
            g.ldr = H;
            g.res_f32 = g.c_f32 = f32;
            KD_TRY(lin(m, P, s, M, H, TI, b.a, TI, m->lm(i, LDW), x_out, H, g));
        }
    }
    return launch_norm_fwd(1, P.x_lm_last, H, m->W(m->i_norm), nullptr, hn, H, nullptr, save ? P.rf : nullptr, M, H,
                           c.t_eps, s, f32);
}

// ---------------------------------------------------------- backward plan ----
struct BwdPlan {
    bf16 *dx, *da, *dgu, *dh2, *do_, *dk, *dv, *dqkv, *dh, *demb;   // language model
    float *dq, *delta;
    bf16 *dfeats, *dz, *dxv, *du, *dh2v, *dov, *dqkvv, *dhv;   // projector / vision (attention writes dqkvv directly)
    float *deltav;
    float* dqv = nullptr; bf16 *dkv = nullptr, *dvv = nullptr;   // KD_ATTN_DQKV=0 (A/B): head-major + kd_qkv_merge
    void *attn_ws, *attn_ws_v, *norm_ws;
    size_t attn_ws_bytes, attn_ws_v_bytes, norm_ws_bytes;
    void *splitk_main, *splitk_lane;
    size_t bytes;
};

kd_attn_bwd_desc lm_attn_desc(const kd_model* m, int B, int L) {
    const kd_model_config& c = m->C.c;
    kd_attn_bwd_desc d;
    std::memset(&d, 0, sizeof(d));
    d.B = B; d.H = c.t_heads; d.HKV = c.t_kv_heads; d.S = L; d.hd = c.t_head_dim; d.hdp = c.t_head_dim; d.causal = 1;
    return d;
}
kd_attn_bwd_desc vis_attn_desc(const kd_model* m, int NI) {
    const kd_model_config& c = m->C.c;
    kd_attn_bwd_desc d;
    std::memset(&d, 0, sizeof(d));
    d.B = NI; d.H = c.v_heads; d.HKV = c.v_heads; d.S = m->C.np(); d.hd = m->C.v_hd(); d.hdp = m->C.v_hdp(); d.causal = 0;
    return d;
}

BwdPlan plan_backward(const kd_model* m, int B, int L, int n_tiles, void* base) {
    const Cfg& C = m->C;
    const kd_model_config& c = C.c;
    Arena A(base);
    BwdPlan P;
    const int NI = n_tiles, np = C.np();
    const int64_t NT = (int64_t)NI * np, D = c.v_hidden, Iv = c.v_inter, hdp = C.v_hdp();
    const int64_t M = (int64_t)B * L, H = c.t_hidden, TI = c.t_inter, qd = C.qd(), kvd = C.kvd();
    P.dx = A.take<bf16>(M * H);
    P.da = A.take<bf16>(M * TI);
    P.dgu = A.take<bf16>(M * 2 * TI);
    P.dh2 = A.take<bf16>(M * H);
    P.do_ = A.take<bf16>(M * qd);
    // the attention backward writes the fused q|k|v gradient directly (kd_attn_bwd_desc.dqkv, RoPE
    // rotated back in-kernel: grouped-query attention); plain multi-head attention with RoPE
    // (t_kv_heads == t_heads) and KD_ATTN_DQKV=0 (A/B) take the head-major dq / dk / dv +
    // kd_qkv_merge path (the MHA dK kernel writes its result unrotated)
    const bool merge_ab = ab_knob("KD_ATTN_DQKV", 1) == 0 || c.t_kv_heads == c.t_heads;
    P.dq = merge_ab ? A.take<float>(M * qd) : nullptr;
    P.dk = merge_ab ? A.take<bf16>(M * kvd) : nullptr;
    P.dv = merge_ab ? A.take<bf16>(M * kvd) : nullptr;
    P.delta = A.take<float>((int64_t)B * c.t_heads * L);
    P.dqkv = A.take<bf16>(M * (qd + 2 * kvd));
    P.dh = A.take<bf16>(M * H);
    P.demb = P.dx;   // the LM backward's dx is d(inputs_embeds)
    kd_attn_bwd_desc ad = lm_attn_desc(m, B, L);
    P.attn_ws_bytes = attn_bwd_workspace_size(&ad);
    P.attn_ws = P.attn_ws_bytes ? A.take<char>(P.attn_ws_bytes) : nullptr;
    P.dfeats = A.take<bf16>(NT * H);
    P.dz = A.take<bf16>(NT * H);
    P.dxv = A.take<bf16>(NT * D);
    P.du = A.take<bf16>(NT * Iv);
    P.dh2v = A.take<bf16>(NT * D);
    P.dov = A.take<bf16>(NT * D);
    P.deltav = A.take<float>((int64_t)NI * c.v_heads * np);
    if (ab_knob("KD_ATTN_DQKV", 1) == 0) {
        P.dqv = A.take<float>((int64_t)NI * c.v_heads * np * hdp);
        P.dkv = A.take<bf16>((int64_t)NI * c.v_heads * np * hdp);
        P.dvv = A.take<bf16>((int64_t)NI * c.v_heads * np * hdp);
    }
    P.dqkvv = A.take<bf16>(NT * 3 * D);
    P.dhv = A.take<bf16>(NT * D);
    kd_attn_bwd_desc vd = vis_attn_desc(m, NI);
    P.attn_ws_v_bytes = attn_bwd_workspace_size(&vd);
    P.attn_ws_v = P.attn_ws_v_bytes ? A.take<char>(P.attn_ws_v_bytes) : nullptr;
    const int64_t Rmax = M > NT ? M : NT;
    const int Dmax = (int)(H > D ? H : D);
    P.norm_ws_bytes = norm_bwd_ws((int)Rmax, Dmax);
    P.norm_ws = A.take<char>(P.norm_ws_bytes);
    P.splitk_main = A.take<char>(SPLITK_WS);
    P.splitk_lane = A.take<char>(SPLITK_WS);
    P.bytes = A.off + 256;
    return P;
}

// ----------------------------------------------------------------- backward ----
int lm_backward(kd_model* m, const FwdPlan& F, const BwdPlan& P, const float* cs, const float* sn, int B, int L,
                const void* dhn, Lane& lane, hipStream_t s, kd_layer_cb cb, void* user) {
    const kd_model_config& c = m->C.c;
    const int M = B * L, H = c.t_hidden, TI = c.t_inter, qd = m->C.qd(), kvd = m->C.kvd(), hd = c.t_head_dim;
    const bool gw = m->train_language != 0;
    const int f32 = m->rf32_t;
    KD_TRY(launch_norm_bwd(1, F.x_lm_last, H, m->W(m->i_norm), dhn, H, nullptr, F.rf, P.dx, H, 0,
                           gw ? m->G(m->i_norm) : nullptr, nullptr, 1, P.norm_ws, P.norm_ws_bytes, M, H, s, f32));
    for (int i = c.t_layers - 1; i >= 0; --i) {
        const LmLayerBufs& b = F.ll[i];
        GemmArgs g0;
        // MLP: dgu = swiglu'(gu) (dx Wdown) -- one GEMM with the KD_ACT_DSWIGLU epilogue where the
        // tiled kernels run it, else the GEMM + k_swiglu_bwd (same bits) ; dh2 = dgu [Wgate; Wup]
        if (fused_dact_ok(M, TI)) {
            GemmArgs gs;
            gs.act = KD_ACT_DSWIGLU; gs.aux = b.gu; gs.ld_aux = 2 * TI; gs.split_k = 1;
            KD_TRY(gemm(s, P.splitk_main, M, TI, H, km(P.dx, H), mn(m->W(m->lm(i, LDW)), TI), P.dgu, 2 * TI, gs));
        } else {
            KD_TRY(gemm(s, P.splitk_main, M, TI, H, km(P.dx, H), mn(m->W(m->lm(i, LDW)), TI), P.da, TI, g0));
        }
        hipEvent_t ev = nullptr;
        if (gw) {
            lane.begin();
            KD_TRY(lane.wgrad(M, H, TI, P.dx, H, b.a, TI, m->G(m->lm(i, LDW))));
            ev = lane.end();
        }
        if (!fused_dact_ok(M, TI)) KD_TRY(launch_swiglu_bwd(b.gu, 2 * TI, P.da, TI, P.dgu, 2 * TI, M, TI, s));
        KD_TRY(gemm(s, P.splitk_main, M, H, 2 * TI, km(P.dgu, 2 * TI), mn(m->W(m->lm(i, LGW)), H), P.dh2, H, g0));
        if (gw) {
            lane.begin();
            KD_TRY(lane.wgrad(M, 2 * TI, H, P.dgu, 2 * TI, b.h2, H, m->G(m->lm(i, LGW))));
            lane.end();
        }
        wait(s, ev);   // dx is updated in place next (the lane read it)
        KD_TRY(launch_norm_bwd(1, b.x_mid, H, m->W(m->lm(i, LPOSTW)), P.dh2, H, nullptr, b.r2, P.dx, H, 1,
                               gw ? m->G(m->lm(i, LPOSTW)) : nullptr, nullptr, 1, P.norm_ws, P.norm_ws_bytes, M, H, s,
                               f32));
        // attention: do = dx Wo ; flash backward ; dqkv (RoPE undone) ; dh = dqkv Wqkv
        KD_TRY(gemm(s, P.splitk_main, M, qd, H, km(P.dx, H), mn(m->W(m->lm(i, LOW)), qd), P.do_, qd, g0));
        ev = nullptr;
        if (gw) {
            lane.begin();
            KD_TRY(lane.wgrad(M, H, qd, P.dx, H, b.o, qd, m->G(m->lm(i, LOW))));
            ev = lane.end();
        }
        {
            kd_attn_bwd_desc d = lm_attn_desc(m, B, L);
            d.q = b.q; d.k = b.k; d.v = b.v; d.o = b.o; d.dO = P.do_; d.lse = b.lse; d.delta = P.delta;
            d.workspace = P.attn_ws; d.workspace_bytes = P.attn_ws_bytes;
            if (P.dq) { d.dq = P.dq; d.dk = P.dk; d.dv = P.dv; }
            else { d.dqkv = P.dqkv; d.ld_qkv = qd + 2 * kvd; d.cos_t = cs; d.sin_t = sn; }   // RoPE rotated back in-kernel
            KD_TRY(launch_attn_bwd(&d, s));
        }
        if (P.dq)
            KD_TRY(launch_qkv_merge(P.dq, P.dk, P.dv, P.dqkv, qd + 2 * kvd, cs, sn, B, L, c.t_heads, c.t_kv_heads, hd, hd, s));
        KD_TRY(gemm(s, P.splitk_main, M, H, qd + 2 * kvd, km(P.dqkv, qd + 2 * kvd), mn(m->W(m->lm(i, LQW)), H), P.dh, H,
                    g0));
        if (gw) {
            lane.begin();
            KD_TRY(lane.wgrad(M, qd + 2 * kvd, H, P.dqkv, qd + 2 * kvd, b.h, H, m->G(m->lm(i, LQW))));
            KD_TRY(lane.colsum(P.dqkv, qd + 2 * kvd, M, qd + 2 * kvd, m->G(m->lm(i, LQB))));
            lane.end();
        }
        wait(s, ev);
        KD_TRY(launch_norm_bwd(1, b.x, H, m->W(m->lm(i, LINW)), P.dh, H, nullptr, b.r1, P.dx, H, 1,
                               gw ? m->G(m->lm(i, LINW)) : nullptr, nullptr, 1, P.norm_ws, P.norm_ws_bytes, M, H, s,
                               f32));
        if (cb) cb(user, i);
    }
    return KD_OK;
}

int vision_backward(kd_model* m, const FwdPlan& F, const BwdPlan& P, int NI, const void* dpost, Lane& lane,
                    hipStream_t s, kd_layer_cb cb, void* user) {
    const Cfg& C = m->C;
    const kd_model_config& c = C.c;
    const int np = C.np(), D = c.v_hidden, Iv = c.v_inter, hdp = C.v_hdp(), hd = C.v_hd();
    const int NT = NI * np;
    const bool gw = m->train_vision != 0;
    bf16* dx = P.dxv;
    const int f32 = m->rf32_v;
    if (dpost)
        KD_TRY(launch_norm_bwd(0, F.x_vis_last, D, m->W(m->i_post_w), dpost, D, F.pm, F.pr, dx, D, 1,
                               gw ? m->G(m->i_post_w) : nullptr, gw ? m->G(m->i_post_b) : nullptr, 1, P.norm_ws,
                               P.norm_ws_bytes, NT, D, s, f32, np));   // dpost: fp32 per tile, / np per row
    GemmArgs g0;
    for (int i = c.v_layers - 1; i >= 0; --i) {
        const VisLayerBufs& b = F.vl[i];
        const bool fuse_gelu = fused_dact_ok(NT, Iv);
        if (fuse_gelu) {   // du = gelu'(pre) (dx Wfc2) in one GEMM (KD_ACT_DGELU_TANH epilogue)
            GemmArgs gd;
            gd.act = KD_ACT_DGELU_TANH; gd.aux = b.pre; gd.ld_aux = Iv; gd.split_k = 1;
            KD_TRY(gemm(s, P.splitk_main, NT, Iv, D, km(dx, D), mn(m->W(m->vis(i, VFC2W)), Iv), P.du, Iv, gd));
        } else {
            KD_TRY(gemm(s, P.splitk_main, NT, Iv, D, km(dx, D), mn(m->W(m->vis(i, VFC2W)), Iv), P.du, Iv, g0));
        }
        hipEvent_t ev = nullptr;
        if (gw) {
            lane.begin();
            KD_TRY(lane.wgrad(NT, D, Iv, dx, D, b.u, Iv, m->G(m->vis(i, VFC2W))));
            KD_TRY(lane.colsum(dx, D, NT, D, m->G(m->vis(i, VFC2B))));
            ev = lane.end();
        }
        if (!fuse_gelu) KD_TRY(launch_act_bwd(b.pre, P.du, P.du, (int64_t)NT * Iv, KD_ACT_GELU_TANH, s));   // dpre in place
        KD_TRY(gemm(s, P.splitk_main, NT, D, Iv, km(P.du, Iv), mn(m->W(m->vis(i, VFC1W)), D), P.dh2v, D, g0));
        if (gw) {
            lane.begin();
            KD_TRY(lane.wgrad(NT, Iv, D, P.du, Iv, b.h2, D, m->G(m->vis(i, VFC1W))));
            KD_TRY(lane.colsum(P.du, Iv, NT, Iv, m->G(m->vis(i, VFC1B))));
            lane.end();
        }
        wait(s, ev);
        KD_TRY(launch_norm_bwd(0, b.x_mid, D, m->W(m->vis(i, VLN2W)), P.dh2v, D, b.m2, b.r2, dx, D, 1,
                               gw ? m->G(m->vis(i, VLN2W)) : nullptr, gw ? m->G(m->vis(i, VLN2B)) : nullptr, 1, P.norm_ws,
                               P.norm_ws_bytes, NT, D, s, f32));
        KD_TRY(gemm(s, P.splitk_main, NT, D, D, km(dx, D), mn(m->W(m->vis(i, VOW)), D), P.dov, D, g0));
        ev = nullptr;
        if (gw) {
            lane.begin();
            KD_TRY(lane.wgrad(NT, D, D, dx, D, b.o, D, m->G(m->vis(i, VOW))));
            KD_TRY(lane.colsum(dx, D, NT, D, m->G(m->vis(i, VOB))));
            ev = lane.end();
        }
        {
            kd_attn_bwd_desc d = vis_attn_desc(m, NI);
            d.q = b.q; d.k = b.k; d.v = b.v; d.o = b.o; d.dO = P.dov; d.lse = b.lse; d.delta = P.deltav;
            d.workspace = P.attn_ws_v; d.workspace_bytes = P.attn_ws_v_bytes;
            // MHA, no RoPE: dq | dk | dv straight into the fused q|k|v gradient (no kd_qkv_merge pass)
            if (P.dqv) { d.dq = P.dqv; d.dk = P.dkv; d.dv = P.dvv; }
            else { d.dqkv = P.dqkvv; d.ld_qkv = 3 * D; }
            KD_TRY(launch_attn_bwd(&d, s));
        }
        if (P.dqv)
            KD_TRY(launch_qkv_merge(P.dqv, P.dkv, P.dvv, P.dqkvv, 3 * D, nullptr, nullptr, NI, np, c.v_heads, c.v_heads,
                                    hd, hdp, s));
        KD_TRY(gemm(s, P.splitk_main, NT, D, 3 * D, km(P.dqkvv, 3 * D), mn(m->W(m->vis(i, VQW)), D), P.dhv, D, g0));
        if (gw) {
            lane.begin();
            KD_TRY(lane.wgrad(NT, 3 * D, D, P.dqkvv, 3 * D, b.h, D, m->G(m->vis(i, VQW))));
            KD_TRY(lane.colsum(P.dqkvv, 3 * D, NT, 3 * D, m->G(m->vis(i, VQB))));
            lane.end();
        }
        wait(s, ev);
        KD_TRY(launch_norm_bwd(0, b.x, D, m->W(m->vis(i, VLN1W)), P.dhv, D, b.m1, b.r1, dx, D, 1,
                               gw ? m->G(m->vis(i, VLN1W)) : nullptr, gw ? m->G(m->vis(i, VLN1B)) : nullptr, 1, P.norm_ws,
                               P.norm_ws_bytes, NT, D, s, f32));
        // layer i's gradients (and post_layernorm's) are enqueued: the caller may all-reduce them
        // while the layers below run (ABI 9; the weight gradients are on the lane, which the
        // callback joins before it launches a collective)
        if (cb && gw) cb(user, KD_CB_VISION_LAYER(i));
    }
    if (gw) {   // patch embedding (im2col GEMM), its bias and the position embedding
        lane.begin();
        KD_TRY(lane.wgrad(NT, D, C.kpatch(), dx, D, F.rows, C.kpatch(), m->G(m->i_patch_w)));
        KD_TRY(lane.colsum(dx, D, NT, D, m->G(m->i_patch_b)));
        KD_TRY(lane.colsum(dx, (int64_t)np * D, NI, np * D, m->G(m->i_pos)));
        lane.end();
    }
    return KD_OK;
}

}  // namespace
}  // namespace kd


// ================================================================ anyres plan ====
// Host-side pack plan of LLaVA-OneVision's anyres image features (the C restatement of
// anyres.py, itself transformers' select_best_resolution / get_anyres_image_grid_shape /
// unpad_image / pack_image_features, HF5 llava_onevision :152-343): for each image token of
// each sample, the flattened vision feature row it takes ([B*tiles*729] rows; tile 0 = the
// base image, then the grid tiles) or -1 for image_newline. Pinpoints: 384 x {1..6} squared
// grid (the checkpoints' image_grid_pinpoints); max 9 patches (anyres_max_9).
namespace {
constexpr int AR_PATCH = 384, AR_GRID = 27, AR_TILE = AR_GRID * AR_GRID;

void best_resolution(int oh, int ow, int& bh, int& bw) {
    double best_eff = 0, best_waste = 1e300;
    bh = bw = 0;
    for (int h = 384; h <= 2304; h += 384)
        for (int w = 384; w <= 2304; w += 384) {
            const double scale = std::min((double)w / ow, (double)h / oh);
            const long long dw = (long long)(ow * scale), dh = (long long)(oh * scale);
            const double eff = (double)std::min(dw * dh, (long long)ow * oh);
            const double waste = (double)w * h - eff;
            if (eff > best_eff || (eff == best_eff && waste < best_waste)) {
                best_eff = eff; best_waste = waste; bh = h; bw = w;
            }
        }
}

// Python's int(round(x, 7)) for the x of unpad_image (x > 0)
long long round7_int(double x) { return (long long)(std::nearbyint(x * 1e7) / 1e7); }

int pack_map(int oh, int ow, int base, int32_t* out, int cap) {
    int bh, bw;
    best_resolution(oh, ow, bh, bw);
    const int nph = bh / AR_PATCH, npw = bw / AR_PATCH;
    int n = 0;
    auto put = [&](int v) { if (n < cap) out[n] = v; ++n; };
    for (int p = 0; p < AR_TILE; ++p) put(base + p);
    const int H = nph * AR_GRID, W = npw * AR_GRID;
    int r0 = 0, r1 = H, c0 = 0, c1 = W;
    if ((double)ow / oh > (double)W / H) {
        const long long new_h = round7_int(oh * ((double)W / ow));
        const int pad = (int)((H - new_h) / 2);
        r0 = pad; r1 = H - pad;
    } else {
        const long long new_w = round7_int(ow * ((double)H / oh));
        const int pad = (int)((W - new_w) / 2);
        c0 = pad; c1 = W - pad;
    }
    const int ch = r1 - r0, cw = c1 - c0;
    if (std::sqrt((double)ch * cw / (9.0 * AR_TILE)) > 1.1) return -1;   // anyres_max_9 downsampling: unsupported
    for (int R = r0; R < r1; ++R) {
        const int ph = R / AR_GRID, y = R % AR_GRID;
        for (int Cc = c0; Cc < c1; ++Cc) {
            const int pw = Cc / AR_GRID, x = Cc % AR_GRID;
            put(base + (1 + ph * npw + pw) * AR_TILE + y * AR_GRID + x);
        }
        put(-1);
    }
    return n;
}
}  // namespace
// ================================================================== C ABI ====
extern "C" {

int kd_anyres_batch_map(const int64_t* image_sizes_host, int B, int tiles, int32_t* map_host, int map_ld,
                        int32_t* len_host) {
    KD_CHECK_ARG(image_sizes_host && map_host && len_host, "kd_anyres_batch_map: null pointer");
    KD_CHECK_SHAPE(B > 0 && tiles >= 0 && map_ld > 0, "kd_anyres_batch_map: B, map_ld must be positive, tiles >= 0");
    int base_tile = 0;   // compact layout (tiles == 0): sample b's tiles follow sample b-1's real ones
    for (int b = 0; b < B; ++b) {
        const int oh = (int)image_sizes_host[2 * b], ow = (int)image_sizes_host[2 * b + 1];
        KD_CHECK_SHAPE(oh > 0 && ow > 0, "kd_anyres_batch_map: image sizes must be positive");
        int bh, bw;
        best_resolution(oh, ow, bh, bw);
        const int own = (bh / 384) * (bw / 384) + 1;   // the image's real tiles (base + grid)
        KD_CHECK_SHAPE(tiles == 0 || own <= tiles, "kd_anyres_batch_map: the batch has too few tiles per sample");
        int32_t* row = map_host + (int64_t)b * map_ld;
        const int n = pack_map(oh, ow, (tiles ? b * tiles : base_tile) * AR_TILE, row, map_ld);
        base_tile += own;
        KD_CHECK_SHAPE(n >= 0, "kd_anyres_batch_map: anyres_max_9 downsampling of very large grids is not supported");
        KD_CHECK_SHAPE(n <= map_ld, "kd_anyres_batch_map: map_ld too small");
        for (int j = n; j < map_ld; ++j) row[j] = -2;
        len_host[b] = n;
    }
    return KD_OK;
}

int kd_model_param_count(const kd_model_config* cfg) {
    if (!kd::cfg_ok(cfg)) {
        kd::fail(KD_ERR_ARG, "kd_model_param_count: invalid config");
        return -1;
    }
    int64_t tot;
    return (int)kd::make_specs(kd::Cfg{*cfg}, &tot).size();
}

int64_t kd_model_param_numel(const kd_model_config* cfg) {
    if (!kd::cfg_ok(cfg)) {
        kd::fail(KD_ERR_ARG, "kd_model_param_numel: invalid config");
        return -1;
    }
    int64_t tot;
    kd::make_specs(kd::Cfg{*cfg}, &tot);
    return tot;
}

int kd_model_param_info(const kd_model_config* cfg, int index, char* name, int name_cap, int64_t* offset,
                        int64_t* numel, int64_t* rows, int64_t* cols) {
    KD_CHECK_ARG(kd::cfg_ok(cfg), "kd_model_param_info: invalid config");
    int64_t tot;
    const auto S = kd::make_specs(kd::Cfg{*cfg}, &tot);
    KD_CHECK_ARG(index >= 0 && index < (int)S.size(), "kd_model_param_info: index out of range");
    const auto& s = S[index];
    if (name && name_cap > 0) {
        std::strncpy(name, s.name.c_str(), name_cap - 1);
        name[name_cap - 1] = 0;
    }
    if (offset) *offset = s.offset;
    if (numel) *numel = s.numel;
    if (rows) *rows = s.rows;
    if (cols) *cols = s.cols;
    return KD_OK;
}

int kd_model_create(const kd_model_config* cfg, const void* weights, float* grad, kd_model** out) {
    KD_CHECK_ARG(out, "kd_model_create: null out");
    KD_CHECK_ARG(kd::cfg_ok(cfg), "kd_model_create: invalid config (head dims: text 64|128, vision <= 128)");
    KD_CHECK_ARG(weights, "kd_model_create: null weights");
    KD_CHECK_ALIGN(weights, 16, "kd_model_create: weights must be 16-B aligned");
    kd_model* m = new kd_model();
    m->C = kd::Cfg{*cfg};
    m->specs = kd::make_specs(m->C, &m->numel);
    m->w = (const kd::bf16*)weights;
    m->g = grad;
    const int on = grad ? 1 : 0;
    m->train_vision = m->train_projector = m->train_language = on;
    m->lane_split_k = kd::ab_knob("KD_WGRAD_SPLIT_K", 0);
    m->i_post_w = m->i_vis0 + cfg->v_layers * kd::VNF;
    m->i_post_b = m->i_post_w + 1;
    m->i_p1w = m->i_post_b + 1;
    m->i_p1b = m->i_p1w + 1;
    m->i_p2w = m->i_p1b + 1;
    m->i_p2b = m->i_p2w + 1;
    m->i_newline = m->i_p2b + 1;
    m->i_embed = m->i_newline + 1;
    m->i_lm0 = m->i_embed + 1;
    m->i_norm = m->i_lm0 + cfg->t_layers * kd::LNF;
    m->i_head = cfg->t_tie ? m->i_embed : m->i_norm + 1;
    m->soff = kd::fp8_scale_offsets(m->C, m->specs, &m->n_scales);
    m->fam.assign(m->specs.size(), 0);
    for (size_t i = 0; i < m->specs.size(); ++i) {
        if (m->soff[i] < 0) continue;
        const std::string& nm = m->specs[i].name;
        m->fam[i] = nm.rfind("vision_tower", 0) == 0 ? KD_FP8_VISION
                  : nm.rfind("multi_modal_projector", 0) == 0 ? KD_FP8_PROJECTOR
                  : nm.find("self_attn") != std::string::npos ? KD_FP8_LM_ATTN
                  : nm.find(".mlp.") != std::string::npos ? KD_FP8_LM_MLP
                  : KD_FP8_LM_HEAD;
    }
    *out = m;
    return KD_OK;
}

void kd_model_destroy(kd_model* m) {
    if (!m) return;
    for (auto& e : m->ev_pool) (void)hipEventDestroy(e);
    delete m;
}

int kd_model_set_trainable(kd_model* m, int vision, int projector, int language) {
    KD_CHECK_ARG(m, "kd_model_set_trainable: null model");
    KD_CHECK_ARG(m->g || !(vision || projector || language), "kd_model_set_trainable: model has no grad buffer");
    m->train_vision = vision != 0;
    m->train_projector = projector != 0;
    m->train_language = language != 0;
    return KD_OK;
}

// the fp8 GEMM epilogue adds a bf16 residual only: a tower whose residual-adding linears (SigLIP
// out_proj / fc2, Qwen2 o_proj / down_proj) run in fp8 keeps a bf16 residual stream
static bool fp8_stream_ok(bool f8, int fam, int rf32_v, int rf32_t) {
    return !f8 || ((!rf32_v || !(fam & KD_FP8_VISION)) && (!rf32_t || !(fam & (KD_FP8_LM_ATTN | KD_FP8_LM_MLP))));
}

int kd_model_set_residual_f32(kd_model* m, int vision, int language) {
    KD_CHECK_ARG(m, "kd_model_set_residual_f32: null model");
    KD_CHECK_ARG(fp8_stream_ok(m->f8q, m->f8_families, vision, language),
                 "kd_model_set_residual_f32: the tower's residual linears run in fp8 (bf16 residual only)");
    m->rf32_v = vision != 0;
    m->rf32_t = language != 0;
    return KD_OK;
}

int64_t kd_model_fp8_scale_count(const kd_model* m) { return m ? m->n_scales : -1; }

int kd_model_quantize_fp8(const kd_model* m, void* q, float* scales, void* stream) {
    KD_CHECK_ARG(m && q && scales, "kd_model_quantize_fp8: null pointer");
    KD_CHECK_ALIGN(q, 16, "kd_model_quantize_fp8: q must be 16-B aligned");
    for (size_t i = 0; i < m->specs.size(); ++i) {
        if (m->soff[i] < 0) continue;
        const kd::Spec& sp = m->specs[i];
        KD_CHECK_SHAPE(sp.offset % 16 == 0 && sp.cols % 16 == 0, "kd_model_quantize_fp8: " + sp.name +
                                                                     " is not 16-B aligned / K % 16 != 0");
        KD_TRY(kd::launch_quant_rows_f8(m->W((int)i), sp.cols, (int)sp.rows, (int)sp.cols, (uint8_t*)q + sp.offset,
                                        sp.cols, scales + m->soff[i], stream));
    }
    return KD_OK;
}

int kd_model_set_row_stats(kd_model* m, float* partials, int vs, float inv_t, int top2) {
    KD_CHECK_ARG(m, "kd_model_set_row_stats: null model");
    KD_CHECK_ARG(!partials || inv_t > 0.f, "kd_model_set_row_stats: inv_t must be > 0");
    KD_CHECK_ALIGN(partials, 16, "kd_model_set_row_stats: partials must be 16-B aligned");
    m->rst = partials; m->rst_vs = vs; m->rst_inv_t = inv_t; m->rst_top2 = top2 ? 1 : 0;
    return KD_OK;
}

int kd_model_set_fp8_families(kd_model* m, int families) {
    KD_CHECK_ARG(m, "kd_model_set_fp8_families: null model");
    KD_CHECK_ARG((families & ~KD_FP8_ALL) == 0, "kd_model_set_fp8_families: unknown family bits");
    KD_CHECK_ARG(fp8_stream_ok(m->f8q, families, m->rf32_v, m->rf32_t),
                 "kd_model_set_fp8_families: an fp32 residual stream's residual linears cannot run in fp8");
    m->f8_families = families;
    return KD_OK;
}

int kd_model_set_fp8(kd_model* m, const void* q, const float* scales) {
    KD_CHECK_ARG(m, "kd_model_set_fp8: null model");
    KD_CHECK_ARG((q == nullptr) == (scales == nullptr), "kd_model_set_fp8: q and scales go together");
    KD_CHECK_ARG(!q || !m->g, "kd_model_set_fp8: fp8 weights are for a frozen (no-grad) model, e.g. the teacher");
    KD_CHECK_ALIGN(q, 16, "kd_model_set_fp8: q must be 16-B aligned");
    KD_CHECK_ARG(fp8_stream_ok(q != nullptr, m->f8_families, m->rf32_v, m->rf32_t),
                 "kd_model_set_fp8: an fp32 residual stream's residual linears cannot run in fp8");
    m->f8q = (const uint8_t*)q;
    m->f8s = scales;
    return KD_OK;
}

size_t kd_model_forward_workspace_size(const kd_model* m, int B, int L, int n_tiles, int save) {
    if (!m || B <= 0 || L <= 0 || n_tiles <= 0) return 0;
    return kd::plan_forward(m, B, L, n_tiles, save, nullptr).bytes;
}

size_t kd_model_backward_workspace_size(const kd_model* m, int B, int L, int n_tiles) {
    if (!m || B <= 0 || L <= 0 || n_tiles <= 0) return 0;
    return kd::plan_backward(m, B, L, n_tiles, nullptr).bytes;
}

int kd_model_forward(kd_model* m, const int64_t* ids, const void* pixels, int pixel_dtype, const int32_t* src,
                     const float* rope_cos, const float* rope_sin, int B, int L, int n_tiles, int save,
                     void* workspace, size_t workspace_bytes, void* hn, void* post_ln, void* logits,
                     void* const* kv_k, void* const* kv_v, int32_t* err, void* stream) {
    using namespace kd;
    KD_CHECK_ARG(m && ids && pixels && src && rope_cos && rope_sin && workspace && hn && err,
                 "kd_model_forward: null pointer");
    KD_CHECK_SHAPE(B > 0 && L > 0 && n_tiles > 0, "kd_model_forward: B, L, n_tiles must be positive");
    KD_CHECK_ARG(pixel_dtype == KD_DTYPE_BF16 || pixel_dtype == KD_DTYPE_F32, "kd_model_forward: pixel dtype");
    const FwdPlan P = plan_forward(m, B, L, n_tiles, save, workspace);
    KD_CHECK_ARG(workspace_bytes >= P.bytes, "kd_model_forward: workspace too small");
    const kd_model_config& c = m->C.c;
    hipStream_t s = as_stream(stream);
    const int NI = n_tiles, M = B * L, H = c.t_hidden;
    KD_TRY(vision_forward(m, P, pixels, pixel_dtype, NI, save, post_ln, s));
    {   // projector: linear_1 -> gelu -> linear_2 (HF5 llava_onevision :131-150)
        const int NT = NI * m->C.np(), D = c.v_hidden;
        GemmArgs g;
        g.bias = m->W(m->i_p1b);
        g.act = c.projector_act;
        g.aux = save ? P.ppre : nullptr;
        g.ld_aux = H;
        KD_TRY(lin(m, P, s, NT, H, D, P.x_vis_bf, D, m->i_p1w, P.z, H, g));
        GemmArgs g2;
        g2.bias = m->W(m->i_p2b);
        KD_TRY(lin(m, P, s, NT, H, H, P.z, H, m->i_p2w, P.feats, H, g2));
    }
    // inputs_embeds: token embeddings + the packed image features (masked_scatter)
    void* emb = c.t_layers ? P.ll[0].x : P.x_lm_last;
    KD_TRY(launch_embed_assemble(ids, src, m->W(m->i_embed), P.feats, m->W(m->i_newline), emb, M, H, c.t_vocab, err, s,
                                 m->rf32_t));
    KD_TRY(lm_forward(m, P, rope_cos, rope_sin, B, L, save, hn, kv_k, kv_v, s));
    if (logits) {
        GemmArgs g;
        if (m->rst) { g.row_stats = m->rst; g.rs_vs = m->rst_vs; g.rs_inv_t = m->rst_inv_t; g.rs_top2 = m->rst_top2; }
        KD_TRY(lin(m, P, s, M, c.t_vocab, H, (const bf16*)hn, H, m->i_head, logits, c.t_vocab, g));
    }
    return KD_OK;
}

int kd_model_backward(kd_model* m, const void* fwd_workspace, const int64_t* ids, const int32_t* src,
                      const float* rope_cos, const float* rope_sin, int B, int L, int n_tiles, const void* dhn,
                      const void* dpost, void* workspace, size_t workspace_bytes, void* stream, void* wgrad_stream,
                      kd_layer_cb on_layer_done, void* user) {
    using namespace kd;
    KD_CHECK_ARG(m && fwd_workspace && ids && src && rope_cos && rope_sin && dhn && workspace && wgrad_stream,
                 "kd_model_backward: null pointer");
    KD_CHECK_ARG(m->g, "kd_model_backward: the model has no grad buffer");
    KD_CHECK_SHAPE(B > 0 && L > 0 && n_tiles > 0, "kd_model_backward: B, L, n_tiles must be positive");
    const FwdPlan F = plan_forward(m, B, L, n_tiles, 1, const_cast<void*>(fwd_workspace));
    const BwdPlan P = plan_backward(m, B, L, n_tiles, workspace);
    KD_CHECK_ARG(workspace_bytes >= P.bytes, "kd_model_backward: workspace too small");
    const kd_model_config& c = m->C.c;
    hipStream_t s = as_stream(stream);
    Lane lane{m, s, as_stream(wgrad_stream), P.splitk_lane};
    // work the caller queued on the lane before this call (the lm_head wgrad into a tied
    // embedding) precedes the embedding backward below
    hipEvent_t entry = m->event();
    (void)hipEventRecord(entry, lane.lane);
    const int NI = n_tiles, NT = NI * m->C.np(), M = B * L, H = c.t_hidden, D = c.v_hidden;
    KD_TRY(lm_backward(m, F, P, rope_cos, rope_sin, B, L, dhn, lane, s, on_layer_done, user));
    wait(s, entry);
    const bool need_vision = m->train_vision != 0;
    KD_TRY(launch_embed_bwd(ids, src, P.demb, m->train_language ? m->G(m->i_embed) : nullptr, P.dfeats,
                            m->train_projector ? m->G(m->i_newline) : nullptr, M, H, s));
    {   // projector backward
        GemmArgs g0;
        KD_TRY(gemm(s, P.splitk_main, NT, H, H, km(P.dfeats, H), mn(m->W(m->i_p2w), H), P.dz, H, g0));
        if (m->train_projector) {
            lane.begin();
            KD_TRY(lane.wgrad(NT, H, H, P.dfeats, H, F.z, H, m->G(m->i_p2w)));
            KD_TRY(lane.colsum(P.dfeats, H, NT, H, m->G(m->i_p2b)));
            lane.end();
        }
        KD_TRY(launch_act_bwd(F.ppre, P.dz, P.dz, (int64_t)NT * H, c.projector_act, s));   // dpre in place
        if (m->train_projector) {
            lane.begin();
            KD_TRY(lane.wgrad(NT, H, D, P.dz, H, F.x_vis_bf, D, m->G(m->i_p1w)));
            KD_TRY(lane.colsum(P.dz, H, NT, H, m->G(m->i_p1b)));
            lane.end();
        }
        if (need_vision) KD_TRY(gemm(s, P.splitk_main, NT, D, H, km(P.dz, H), mn(m->W(m->i_p1w), D), P.dxv, D, g0));
    }
    // embed_tokens, image_newline and the projector are final (ABI 9)
    if (on_layer_done && (m->train_language || m->train_projector)) on_layer_done(user, KD_CB_EMBED_PROJECTOR);
    if (need_vision) KD_TRY(vision_backward(m, F, P, NI, dpost, lane, s, on_layer_done, user));
    // the caller reads the grads (and reuses these buffers) after this: join the lane
    hipEvent_t done = m->event();
    (void)hipEventRecord(done, lane.lane);
    (void)hipStreamWaitEvent(s, done, 0);
    KD_LAUNCH_CHECK("kd_model_backward");
    return KD_OK;
}

void kd_timer_enable(int on) { kd::g_timer_on = on != 0; }

int kd_timer_count(void) {
    std::lock_guard<std::mutex> g(kd::g_timer_mu);
    return (int)kd::g_timer.size();
}

int kd_timer_read(int i, char* key, int key_cap, double* flops, float* ms) {
    std::lock_guard<std::mutex> g(kd::g_timer_mu);
    KD_CHECK_ARG(i >= 0 && i < (int)kd::g_timer.size(), "kd_timer_read: index out of range");
    auto& r = kd::g_timer[i];
    if (hipEventSynchronize(r.e1) != hipSuccess) return kd::fail(KD_ERR_LAUNCH, "kd_timer_read: event sync failed");
    float t = 0.f;
    (void)hipEventElapsedTime(&t, r.e0, r.e1);
    if (key && key_cap > 0) {
        std::strncpy(key, r.key.c_str(), key_cap - 1);
        key[key_cap - 1] = 0;
    }
    if (flops) *flops = r.flops;
    if (ms) *ms = t;
    return KD_OK;
}

void kd_timer_reset(void) {
    std::lock_guard<std::mutex> g(kd::g_timer_mu);
    for (auto& r : kd::g_timer) {
        (void)hipEventDestroy(r.e0);
        (void)hipEventDestroy(r.e1);
    }
    kd::g_timer.clear();
}

}  // extern "C"
