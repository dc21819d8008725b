// extern "C" entry points of include/kdstep.h.  Thin: argument plumbing only;
// every kernel lives in its own translation unit.
#include "common.h"
#include "launchers.h"
#include <cstring>

namespace kd {

static thread_local std::string g_last_error = "";

void set_error(const std::string& msg) { g_last_error = msg; }
int fail(int code, const std::string& msg) {
    g_last_error = msg;
    return code;
}

}  // namespace kd

extern "C" {

int kd_abi_version(void) { return KD_ABI_VERSION; }

const char* kd_last_error(void) { return kd::g_last_error.c_str(); }

int kd_device_is_gfx950(int device) {
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) return 0;
    return std::strncmp(prop.gcnArchName, "gfx950", 6) == 0 ? 1 : 0;
}

size_t kd_loss_workspace_size(int B, int L, int V_s) { return kd::kd_loss_ws(B, L, V_s); }

int kd_loss_fwd_bwd(const void* teacher_logits, int64_t ld_t, int V_t, const void* student_logits,
                    int64_t ld_s, int V_s, const int64_t* labels, int B, int L, kd_loss_params params,
                    float* loss_out, void* dlogits, int64_t ld_d, void* workspace,
                    size_t workspace_bytes, void* stream) {
    return kd::launch_kd_loss(teacher_logits, ld_t, V_t, student_logits, ld_s, V_s, labels, B, L,
                              params, loss_out, dlogits, ld_d, workspace, workspace_bytes, stream);
}

int kd_loss_check(const void* workspace, void* stream) { return kd::kd_loss_check_impl(workspace, stream); }

int kd_loss_student_stats(const void* student_logits, int64_t ld_s, int V_s, int rows, float temperature,
                          float* stats_out, void* stream) {
    return kd::launch_kd_student_stats(student_logits, ld_s, V_s, rows, temperature, stats_out, stream);
}

int kd_gemm(const kd_gemm_desc* desc, void* stream) { return kd::gemm_timed(desc, stream); }
size_t kd_gemm_pretile_size(int N, int K, int glu) { return kd::gemm_pretile_size(N, K, glu); }
int kd_gemm_pretile(const void* W, int64_t ldw, int N, int K, int glu, void* out, void* stream) {
    return kd::launch_gemm_pretile(W, ldw, N, K, glu, out, stream);
}
size_t kd_gemm_workspace_size(const kd_gemm_desc* desc) { return kd::gemm_workspace_size(desc); }
int kd_gemm_plan(const kd_gemm_desc* desc, int32_t* variant, int32_t* split_k, int32_t* dp_tiles) {
    return kd::gemm_plan_query(desc, variant, split_k, dp_tiles);
}
int kd_attn_fwd(const kd_attn_desc* d, void* s) { return kd::launch_attn_fwd(d, s); }
int kd_attn_bwd(const kd_attn_bwd_desc* d, void* s) { return kd::launch_attn_bwd(d, s); }
size_t kd_attn_bwd_workspace_size(const kd_attn_bwd_desc* d) { return kd::attn_bwd_workspace_size(d); }
int kd_norm_fwd(int rms, const void* x, int64_t ldx, const void* w, const void* b, void* y, int64_t ldy, float* mean,
                float* rstd, int R, int D, float eps, int x_dtype, void* s) {
    KD_CHECK_ARG(x_dtype == KD_DTYPE_BF16 || x_dtype == KD_DTYPE_F32, "kd_norm_fwd: x_dtype");
    return kd::launch_norm_fwd(rms, x, ldx, w, b, y, ldy, mean, rstd, R, D, eps, s, x_dtype == KD_DTYPE_F32);
}
size_t kd_norm_bwd_workspace_size(int R, int D) { return kd::norm_bwd_ws(R, D); }
int kd_norm_bwd(int rms, const void* x, int64_t ldx, const void* w, const void* dy, int64_t lddy, const float* mean,
                const float* rstd, void* dx, int64_t lddx, int dx_accum, float* dw, float* db, int accum_w, void* ws,
                size_t wsb, int R, int D, int x_dtype, void* s) {
    KD_CHECK_ARG(x_dtype == KD_DTYPE_BF16 || x_dtype == KD_DTYPE_F32, "kd_norm_bwd: x_dtype");
    return kd::launch_norm_bwd(rms, x, ldx, w, dy, lddy, mean, rstd, dx, lddx, dx_accum, dw, db, accum_w, ws, wsb, R, D, s,
                               x_dtype == KD_DTYPE_F32);
}
int kd_qkv_split(const void* qkv, int64_t ld, void* q, void* k, void* v, const float* c, const float* sn, int B, int S,
                 int nq, int nkv, int hd, int hdp, void* s) {
    return kd::launch_qkv_split(qkv, ld, q, k, v, c, sn, B, S, nq, nkv, hd, hdp, s);
}
int kd_qkv_merge(const float* dq, const void* dk, const void* dv, void* dqkv, int64_t ld, const float* c, const float* sn,
                 int B, int S, int nq, int nkv, int hd, int hdp, void* s) {
    return kd::launch_qkv_merge(dq, dk, dv, dqkv, ld, c, sn, B, S, nq, nkv, hd, hdp, s);
}
int kd_swiglu_fwd(const void* gu, int64_t ldg, void* h, int64_t ldh, int M, int I, void* s) {
    return kd::launch_swiglu_fwd(gu, ldg, h, ldh, M, I, s);
}
int kd_swiglu_bwd(const void* gu, int64_t ldg, const void* dh, int64_t ldh, void* dgu, int64_t ldd, int M, int I, void* s) {
    return kd::launch_swiglu_bwd(gu, ldg, dh, ldh, dgu, ldd, M, I, s);
}
int kd_act_bwd(const void* pre, const void* dy, void* dx, int64_t n, int act, void* s) {
    return kd::launch_act_bwd(pre, dy, dx, n, act, s);
}
int kd_patchify(const void* px, int dt, void* out, int NI, int img, int ps, int Kp, void* s) {
    return kd::launch_patchify(px, dt, out, NI, img, ps, Kp, s);
}
int kd_embed_assemble(const int64_t* ids, const int32_t* src, const void* table, const void* feats, const void* nl,
                      void* out, int M, int H, int vocab, int32_t* err, void* s) {
    return kd::launch_embed_assemble(ids, src, table, feats, nl, out, M, H, vocab, err, s);
}
int kd_embed_bwd(const int64_t* ids, const int32_t* src, const void* dout, float* dtable, void* dfeats, float* dnl, int M,
                 int H, void* s) {
    return kd::launch_embed_bwd(ids, src, dout, dtable, dfeats, dnl, M, H, s);
}
int kd_colsum(const void* dy, int64_t ld, int M, int N, float* out, int acc, void* s) {
    return kd::launch_colsum(dy, ld, M, N, out, acc, s);
}
int kd_row_group_mean(const void* x, int64_t ld, int G, int P, int D, float* out, void* s) {
    return kd::launch_row_group_mean(x, ld, G, P, D, out, s);
}
int kd_row_group_mean_bwd(const float* dp, int G, int P, int D, void* dx, int64_t ld, const float* sc, void* s) {
    return kd::launch_row_group_mean_bwd(dp, G, P, D, dx, ld, sc, s);
}
int kd_ntxent(const float* fs, const float* ft, int n, int D, float tau, float w, float* lo, float* dfs, float gs, void* s) {
    return kd::launch_ntxent(fs, ft, n, D, tau, w, lo, dfs, gs, s);
}
int kd_adamw(float* p, void* pb, const float* g, float* m, float* v, int64_t n, float lr, float b1, float b2, float eps,
             float wd, int step, const float* gscale, const int32_t* skip, int n_skip, void* s) {
    return kd::launch_adamw(p, pb, g, m, v, n, lr, b1, b2, eps, wd, step, gscale, skip, n_skip, s);
}
int kd_sumsq(const float* x, int64_t n, float* out, void* s) { return kd::launch_sumsq(x, n, out, s); }
int kd_scale_f32(const float* x, const float* s_dev, float* y, int64_t n, void* s) {
    return kd::launch_scale_f32(x, s_dev, y, n, s);
}
int kd_scalar_mul(const float* a, const float* b, float* out, int n, void* s) {
    return kd::launch_scalar_mul(a, b, out, n, s);
}
int kd_zero(void* ptr, uint64_t bytes, void* s) {
    KD_CHECK_ARG(ptr || bytes == 0, "zero: null pointer");
    if (bytes == 0) return KD_OK;
    const hipError_t e = hipMemsetAsync(ptr, 0, bytes, kd::as_stream(s));
    if (e != hipSuccess) return kd::fail(KD_ERR_LAUNCH, std::string("kd_zero: ") + hipGetErrorString(e));
    return KD_OK;
}
int kd_image_src_map(const int64_t* ids, int B, int L, int64_t tok, const int32_t* map, int ld, const int32_t* len,
                     int32_t* src, int32_t* err, void* s) {
    return kd::launch_image_src_map(ids, B, L, tok, map, ld, len, src, err, s);
}
int kd_cast_f32_bf16(const float* x, void* y, int64_t n, void* s) { return kd::launch_cast_f32_bf16(x, y, n, s); }
int kd_prefetch(const void* ptr, uint64_t bytes, int grid, void* s) { return kd::launch_prefetch(ptr, bytes, grid, s); }
int kd_cast_bf16_f32(const void* x, float* y, int64_t n, void* s) { return kd::launch_cast_bf16_f32(x, y, n, s); }
int kd_quant_rows_fp8(const void* x, int64_t ldx, int R, int K, void* q, int64_t ldq, float* scale, void* s) {
    return kd::launch_quant_rows_f8(x, ldx, R, K, q, ldq, scale, s);
}
size_t kd_depth_to_3ch_workspace_size(int B, int H, int W) { return kd::depth3_ws(B, H, W); }
int kd_depth_to_3ch(const void* depth, int dtype, int B, int H, int W, uint8_t* out, void* ws, size_t ws_bytes,
                    void* s) {
    return kd::launch_depth3(depth, dtype, B, H, W, out, ws, ws_bytes, s);
}
size_t kd_attn_decode_workspace_size(int H, int hd, int smax) { return kd::attn_decode_ws(H, hd, smax); }
int kd_attn_decode(const void* q, const void* kn, const void* vn, void* kc, void* vc, void* o, int H, int HKV, int hd,
                   int hdp, int smax, int n, const int32_t* cur, void* ws, size_t wsb, void* s) {
    return kd::launch_attn_decode(q, kn, vn, kc, vc, o, H, HKV, hd, hdp, smax, n, cur, ws, wsb, s);
}
int kd_gemv(const void* x, const void* W, int64_t ldw, const void* extra, void* y, int N, int K, int epi, int I,
            const void* norm_w, float eps, void* s) {
    return kd::launch_gemv(x, W, ldw, extra, y, N, K, epi, I, norm_w, eps, s);
}
int kd_gen_select(const void* logits, int V, int64_t* seq, int len, int32_t* cur, float penalty, int ngram, void* ws,
                  size_t wsb, int64_t* out, void* s) {
    return kd::launch_gen_select(logits, V, seq, len, cur, penalty, ngram, ws, wsb, out, s);
}
int kd_rope_row(const float* c, const float* sn, int hh, const int32_t* cur, float* cr, float* sr, void* s) {
    return kd::launch_rope_row(c, sn, hh, cur, cr, sr, s);
}
size_t kd_image_resize_workspace_size(int H, int W, int oh, int ow) { return kd::image_resize_ws(H, W, oh, ow); }
int kd_image_resize_u8(const uint8_t* in, int H, int W, uint8_t* out, int oh, int ow, void* ws, size_t ws_bytes,
                       void* s) {
    return kd::launch_image_resize(in, H, W, out, oh, ow, ws, ws_bytes, s);
}
int kd_anyres_tiles(const uint8_t* base, const uint8_t* resized, int nh, int nw, int bh, int bw, int patch, int n_out,
                    const float* mean_std_host, void* out, int out_dtype, void* s) {
    return kd::launch_anyres_tiles(base, resized, nh, nw, bh, bw, patch, n_out, mean_std_host, out, out_dtype, s);
}

}  // extern "C"
