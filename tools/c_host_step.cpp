// A non-Python host driving one full KD training step through the C ABI alone
// (include/kdstep.h): the logit-based module's step (LB:125-169 forward, LoCa at T = 1,
// LB:208-261) = teacher forward -> student forward -> fused loss fwd+bwd -> lm_head
// dgrad / tied-embedding wgrad -> student backward -> gradient norm -> AdamW.
//
//   c_host_step <bundle dir>      (reads the files below, writes <dir>/out.txt)
//
// Bundle (little-endian raw arrays, written by tests/test_c_host_gpu.py):
//   meta.txt        B L tiles; the two kd_model_config's as 17 numbers each
//   teacher.bin     bf16 flat teacher weights (kd_model_param_info layout)
//   student.bin     bf16 flat student weights
//   rgb_ids.bin, depth_ids.bin, labels.bin   int64 [B, L]
//   rgb_px.bin, depth_px.bin                 bf16 [B*tiles, 3, 384, 384]
//   image_sizes.bin                          int64 [B, 2]
// out.txt: the four loss terms (KD, student CE, teacher CE, total), the gradient's sum of
// squares, and the sum of the updated bf16 weights after one AdamW step.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "kdstep.h"

#define HIP(x)                                                                         \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(2);                                                              \
        }                                                                              \
    } while (0)
#define KD(x)                                                                          \
    do {                                                                               \
        int s_ = (x);                                                                  \
        if (s_ != KD_OK) {                                                             \
            std::fprintf(stderr, "%s:%d %s -> %d: %s\n", __FILE__, __LINE__, #x, s_, kd_last_error()); \
            std::exit(3);                                                              \
        }                                                                              \
    } while (0)

static std::vector<char> slurp(const std::string& path) {
    FILE* f = std::fopen(path.c_str(), "rb");
    if (!f) { std::fprintf(stderr, "cannot open %s\n", path.c_str()); std::exit(1); }
    std::fseek(f, 0, SEEK_END);
    const long n = std::ftell(f);
    std::fseek(f, 0, SEEK_SET);
    std::vector<char> b(n);
    if (n && std::fread(b.data(), 1, n, f) != (size_t)n) std::exit(1);
    std::fclose(f);
    return b;
}

template <class T>
static T* upload(const std::vector<char>& h) {
    void* d = nullptr;
    HIP(hipMalloc(&d, h.size() ? h.size() : 16));
    HIP(hipMemcpy(d, h.data(), h.size(), hipMemcpyHostToDevice));
    return (T*)d;
}

static void* dalloc(size_t n) {
    void* d = nullptr;
    HIP(hipMalloc(&d, n ? n : 16));
    return d;
}

static void read_cfg(FILE* f, kd_model_config& c) {
    double v[17];
    for (double& x : v)
        if (std::fscanf(f, "%lf", &x) != 1) std::exit(1);
    c.v_hidden = (int)v[0]; c.v_inter = (int)v[1]; c.v_layers = (int)v[2]; c.v_heads = (int)v[3];
    c.v_patch = (int)v[4]; c.v_image = (int)v[5]; c.v_eps = (float)v[6];
    c.t_hidden = (int)v[7]; c.t_inter = (int)v[8]; c.t_layers = (int)v[9]; c.t_heads = (int)v[10];
    c.t_kv_heads = (int)v[11]; c.t_head_dim = (int)v[12]; c.t_vocab = (int)v[13]; c.t_tie = (int)v[14];
    c.t_rope_theta = (float)v[15]; c.t_eps = (float)v[16];
    c.image_token_id = 151646;
    c.projector_act = KD_ACT_GELU_ERF;
}

// Qwen2RotaryEmbedding tables [L, hd/2] in fp32: inv_freq = 1 / theta^(2i/hd), angle = pos * inv_freq
static void rope(int L, int hd, float theta, std::vector<float>& c, std::vector<float>& s) {
    const int hh = hd / 2;
    c.resize((size_t)L * hh);
    s.resize((size_t)L * hh);
    for (int i = 0; i < hh; ++i) {
        const float inv = 1.0f / std::pow(theta, (float)(2 * i) / (float)hd);
        for (int p = 0; p < L; ++p) {
            const float a = (float)p * inv;
            c[(size_t)p * hh + i] = std::cos(a);
            s[(size_t)p * hh + i] = std::sin(a);
        }
    }
}

int main(int argc, char** argv) {
    if (argc < 2) { std::fprintf(stderr, "usage: %s <bundle dir>\n", argv[0]); return 1; }
    const std::string dir = argv[1];
    HIP(hipSetDevice(0));
    if (!kd_device_is_gfx950(0)) { std::fprintf(stderr, "not a gfx950 device\n"); return 4; }
    int B, L, tiles;
    kd_model_config tc{}, sc{};
    {
        FILE* f = std::fopen((dir + "/meta.txt").c_str(), "r");
        if (!f || std::fscanf(f, "%d %d %d", &B, &L, &tiles) != 3) return 1;
        read_cfg(f, tc);
        read_cfg(f, sc);
        std::fclose(f);
    }
    hipStream_t main_s, lane_s;
    HIP(hipStreamCreate(&main_s));
    HIP(hipStreamCreate(&lane_s));

    // ---- weights, grads, optimizer state
    const int64_t nt = kd_model_param_numel(&tc), ns = kd_model_param_numel(&sc);
    const std::vector<char> tw_h = slurp(dir + "/teacher.bin"), sw_h = slurp(dir + "/student.bin");
    if ((int64_t)tw_h.size() != 2 * nt || (int64_t)sw_h.size() != 2 * ns) { std::fprintf(stderr, "weight size\n"); return 1; }
    void* tw = upload<char>(tw_h);
    void* sw = upload<char>(sw_h);
    float* grad = (float*)dalloc(ns * 4);
    float* master = (float*)dalloc(ns * 4);
    float* m1 = (float*)dalloc(ns * 4);
    float* m2 = (float*)dalloc(ns * 4);
    HIP(hipMemsetAsync(grad, 0, ns * 4, main_s));
    HIP(hipMemsetAsync(m1, 0, ns * 4, main_s));
    HIP(hipMemsetAsync(m2, 0, ns * 4, main_s));
    {   // fp32 master copy of the bf16 weights (exact: bf16 -> fp32 is a shift)
        std::vector<float> mh(ns);
        const uint16_t* b = (const uint16_t*)sw_h.data();
        for (int64_t i = 0; i < ns; ++i) { uint32_t u = (uint32_t)b[i] << 16; std::memcpy(&mh[i], &u, 4); }
        HIP(hipMemcpy(master, mh.data(), ns * 4, hipMemcpyHostToDevice));
    }
    kd_model *teacher = nullptr, *student = nullptr;
    KD(kd_model_create(&tc, tw, nullptr, &teacher));
    KD(kd_model_set_residual_f32(teacher, 1, 0));   // the drop-in module's teacher: fp32 SigLIP stream
    KD(kd_model_create(&sc, sw, grad, &student));
    KD(kd_model_set_residual_f32(student, 1, 1));   // fp32 residual streams, as the drop-in module's student

    // ---- batch
    const int64_t* rgb_ids = upload<int64_t>(slurp(dir + "/rgb_ids.bin"));
    const int64_t* depth_ids = upload<int64_t>(slurp(dir + "/depth_ids.bin"));
    const int64_t* labels = upload<int64_t>(slurp(dir + "/labels.bin"));
    const void* rgb_px = upload<char>(slurp(dir + "/rgb_px.bin"));
    const void* depth_px = upload<char>(slurp(dir + "/depth_px.bin"));
    const std::vector<char> isz = slurp(dir + "/image_sizes.bin");

    // ---- anyres pack plan -> per-token source rows (host plan, device expansion)
    const int ld = 8192;
    std::vector<int32_t> map_h((size_t)B * ld), len_h(B);
    KD(kd_anyres_batch_map((const int64_t*)isz.data(), B, tiles, map_h.data(), ld, len_h.data()));
    int32_t* map_d = (int32_t*)dalloc(map_h.size() * 4);
    int32_t* len_d = (int32_t*)dalloc(B * 4);
    HIP(hipMemcpy(map_d, map_h.data(), map_h.size() * 4, hipMemcpyHostToDevice));
    HIP(hipMemcpy(len_d, len_h.data(), B * 4, hipMemcpyHostToDevice));
    int32_t* src_t = (int32_t*)dalloc((size_t)B * L * 4);
    int32_t* src_s = (int32_t*)dalloc((size_t)B * L * 4);
    int32_t* err = (int32_t*)dalloc(16);
    HIP(hipMemsetAsync(err, 0, 16, main_s));
    KD(kd_image_src_map(rgb_ids, B, L, tc.image_token_id, map_d, ld, len_d, src_t, err, main_s));
    KD(kd_image_src_map(depth_ids, B, L, sc.image_token_id, map_d, ld, len_d, src_s, err + 1, main_s));
    std::vector<float> ct, st, cs, ss;
    rope(L, tc.t_head_dim, tc.t_rope_theta, ct, st);
    rope(L, sc.t_head_dim, sc.t_rope_theta, cs, ss);
    float* cos_t = (float*)dalloc(ct.size() * 4);
    float* sin_t = (float*)dalloc(st.size() * 4);
    float* cos_s = (float*)dalloc(cs.size() * 4);
    float* sin_s = (float*)dalloc(ss.size() * 4);
    HIP(hipMemcpy(cos_t, ct.data(), ct.size() * 4, hipMemcpyHostToDevice));
    HIP(hipMemcpy(sin_t, st.data(), st.size() * 4, hipMemcpyHostToDevice));
    HIP(hipMemcpy(cos_s, cs.data(), cs.size() * 4, hipMemcpyHostToDevice));
    HIP(hipMemcpy(sin_s, ss.data(), ss.size() * 4, hipMemcpyHostToDevice));

    // ---- teacher forward (no_grad, DT:228) and student forward with saved activations (DT:238)
    const int M = B * L, Vt = tc.t_vocab, Vs = sc.t_vocab, H = sc.t_hidden;
    const size_t twsb = kd_model_forward_workspace_size(teacher, B, L, B * tiles, 0);
    const size_t swsb = kd_model_forward_workspace_size(student, B, L, B * tiles, 1);
    void* tws = dalloc(twsb);
    void* sws = dalloc(swsb);
    void* hn_t = dalloc((size_t)M * tc.t_hidden * 2);
    void* hn_s = dalloc((size_t)M * H * 2);
    void* t_logits = dalloc((size_t)M * Vt * 2);
    void* s_logits = dalloc((size_t)M * Vs * 2);
    KD(kd_model_forward(teacher, rgb_ids, rgb_px, KD_DTYPE_BF16, src_t, cos_t, sin_t, B, L, B * tiles, 0, tws, twsb, hn_t,
                        nullptr, t_logits, nullptr, nullptr, err, main_s));
    KD(kd_model_forward(student, depth_ids, depth_px, KD_DTYPE_BF16, src_s, cos_s, sin_s, B, L, B * tiles, 1, sws, swsb,
                        hn_s, nullptr, s_logits, nullptr, nullptr, err + 1, main_s));

    // ---- fused LoCa (T = 1, LB:164-165) + student CE, forward and d/dlogits
    float* loss4 = (float*)dalloc(16);
    void* dlogits = dalloc((size_t)M * Vs * 2);
    const size_t lwsb = kd_loss_workspace_size(B, L, Vs);
    void* lws = dalloc(lwsb);
    kd_loss_params lp{};
    lp.variant = KD_LOSS_LOCA; lp.temperature = 1.f; lp.alpha = 0.8f; lp.kd_weight = 1.f; lp.ce_weight = 1.f;
    lp.grad_scale = 1.f; lp.clamp_min = 1e-8f; lp.teacher_ce = 1; lp.out_scale = 1.f; lp.out_accumulate = 0;
    lp.err_out = err + 2; lp.row_base = 0;
    // dlogits relative to the CE coefficient (kd_loss_params.dscale), multiplied back by the GEMMs
    float* dscale = (float*)dalloc(4);
    lp.dscale = dscale; lp.dscale_given = 0;
    KD(kd_loss_fwd_bwd(t_logits, Vt, Vt, s_logits, Vs, Vs, labels, B, L, lp, loss4, dlogits, Vs, lws, lwsb, main_s));

    // ---- lm_head (tied to embed_tokens in the 0.5B): dgrad dhn = dlogits W, wgrad on the lane
    int64_t emb_off = -1, emb_n = 0;
    {
        char name[256];
        for (int i = 0, n = kd_model_param_count(&sc); i < n; ++i) {
            int64_t off, numel, r, c;
            KD(kd_model_param_info(&sc, i, name, sizeof name, &off, &numel, &r, &c));
            if (std::strcmp(name, "language_model.model.embed_tokens.weight") == 0) { emb_off = off; emb_n = numel; }
        }
        if (emb_off < 0 || !sc.t_tie) { std::fprintf(stderr, "expected a tied student head\n"); return 1; }
    }
    void* dhn = dalloc((size_t)M * H * 2);
    const size_t splitk = (size_t)384 << 20;
    void* wsm = dalloc(splitk);
    void* wsl = dalloc(splitk);
    kd_gemm_desc g{};
    g.M = M; g.N = H; g.K = Vs; g.a_layout = KD_LAYOUT_K_MAJOR; g.b_layout = KD_LAYOUT_MN_MAJOR;
    g.A = dlogits; g.lda = Vs; g.B = (char*)sw + emb_off * 2; g.ldb = H; g.C = dhn; g.ldc = H;
    g.c_dtype = KD_DTYPE_BF16; g.alpha = 1.f; g.alpha_dev = dscale; g.workspace = wsm; g.workspace_bytes = splitk;
    KD(kd_gemm(&g, main_s));
    hipEvent_t ev;
    HIP(hipEventCreate(&ev));
    HIP(hipEventRecord(ev, main_s));
    HIP(hipStreamWaitEvent(lane_s, ev, 0));
    kd_gemm_desc w{};
    w.M = Vs; w.N = H; w.K = M; w.a_layout = KD_LAYOUT_MN_MAJOR; w.b_layout = KD_LAYOUT_MN_MAJOR;
    w.A = dlogits; w.lda = Vs; w.B = hn_s; w.ldb = H; w.C = grad + emb_off; w.ldc = H;
    w.c_dtype = KD_DTYPE_F32; w.accumulate = 1; w.alpha = 1.f; w.alpha_dev = dscale; w.workspace = wsl;
    w.workspace_bytes = splitk;
    KD(kd_gemm(&w, lane_s));

    // ---- student backward (every trainable grad, +=), weight gradients on the lane
    const size_t bwsb = kd_model_backward_workspace_size(student, B, L, B * tiles);
    void* bws = dalloc(bwsb);
    KD(kd_model_backward(student, sws, depth_ids, src_s, cos_s, sin_s, B, L, B * tiles, dhn, nullptr, bws, bwsb, main_s,
                         lane_s, nullptr, nullptr));

    // ---- gradient norm, AdamW (torch.optim.AdamW defaults of configure_optimizers, DT:198-201)
    float* ss2 = (float*)dalloc(4);
    HIP(hipMemsetAsync(ss2, 0, 4, main_s));
    KD(kd_sumsq(grad, ns, ss2, main_s));
    KD(kd_adamw(master, sw, grad, m1, m2, ns, 1e-5f, 0.9f, 0.999f, 1e-8f, 1e-2f, 1, nullptr, nullptr, 0, main_s));
    HIP(hipStreamSynchronize(main_s));

    float l4[4], g2;
    int32_t e[4];
    HIP(hipMemcpy(l4, loss4, 16, hipMemcpyDeviceToHost));
    HIP(hipMemcpy(&g2, ss2, 4, hipMemcpyDeviceToHost));
    HIP(hipMemcpy(e, err, 16, hipMemcpyDeviceToHost));
    std::vector<uint16_t> wn(ns);
    HIP(hipMemcpy(wn.data(), sw, ns * 2, hipMemcpyDeviceToHost));
    double wsum = 0;
    for (int64_t i = 0; i < ns; ++i) { uint32_t u = (uint32_t)wn[i] << 16; float x; std::memcpy(&x, &u, 4); wsum += x; }
    FILE* o = std::fopen((dir + "/out.txt").c_str(), "w");
    std::fprintf(o, "%.9g %.9g %.9g %.9g\n%.9g\n%.12g\n%d %d %d\n", l4[0], l4[1], l4[2], l4[3], g2, wsum, e[0], e[1], e[2]);
    std::fclose(o);
    std::printf("loss terms %.6g %.6g %.6g %.6g grad sumsq %.6g\n", l4[0], l4[1], l4[2], l4[3], g2);
    kd_model_destroy(teacher);
    kd_model_destroy(student);
    (void)emb_n;
    return 0;
}
