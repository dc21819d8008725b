// Internal launchers of the kernel translation units (called by abi.hip's extern "C"
// entry points and by the model runtime, model.hip).
#pragma once
#include "common.h"

namespace kd {

int launch_kd_loss(const void* teacher, int64_t ld_t, int V_t, const void* student, int64_t ld_s,
                   int V_s, const int64_t* labels, int B, int L, kd_loss_params p, float* loss_out,
                   void* dlogits, int64_t ld_d, void* ws, size_t ws_bytes, void* stream);
size_t kd_loss_ws(int B, int L, int V);
int launch_kd_student_stats(const void* student, int64_t ld_s, int V_s, int rows, float temperature, float* out,
                            void* stream);
int kd_loss_check_impl(const void* ws, void* stream);
int launch_gemm(const kd_gemm_desc* d, void* stream);
size_t gemm_workspace_size(const kd_gemm_desc* d);
size_t gemm_pretile_size(int N, int K, int glu);
int launch_gemm_pretile(const void* W, int64_t ldw, int N, int K, int glu, void* out, void* stream);
int gemm_plan_query(const kd_gemm_desc* d, int32_t* var, int32_t* split, int32_t* dp);
int launch_attn_fwd(const kd_attn_desc* d, void* stream);
int launch_attn_bwd(const kd_attn_bwd_desc* d, void* stream);
size_t attn_bwd_workspace_size(const kd_attn_bwd_desc* d);
int launch_norm_fwd(int rms, const void* x, int64_t ldx, const void* w, const void* b, void* y, int64_t ldy,
                    float* mean, float* rstd, int R, int D, float eps, void* stream, int x_f32 = 0);
size_t norm_bwd_ws(int R, int D);
int launch_norm_bwd(int rms, const void* x, int64_t ldx, const void* w, const void* dy, int64_t lddy, const float* mean,
                    const float* rstd, void* dx, int64_t lddx, int dx_accum, float* dw, float* db, int accum_w,
                    void* ws, size_t ws_bytes, int R, int D, void* stream, int x_f32 = 0, int dy_group = 0);
int launch_qkv_split(const void* qkv, int64_t ld, void* q, void* k, void* v, const float* cos_t, const float* sin_t,
                     int B, int S, int nq, int nkv, int hd, int hdp, void* stream);
int launch_qkv_merge(const float* dq, const void* dk, const void* dv, void* dqkv, int64_t ld, const float* cos_t,
                     const float* sin_t, int B, int S, int nq, int nkv, int hd, int hdp, void* stream);
int launch_swiglu_fwd(const void* gu, int64_t ldg, void* h, int64_t ldh, int M, int I, void* stream);
int launch_swiglu_bwd(const void* gu, int64_t ldg, const void* dh, int64_t ldh, void* dgu, int64_t ldd, int M, int I,
                      void* stream);
int launch_act_bwd(const void* pre, const void* dy, void* dx, int64_t n, int act, void* stream);
int launch_patchify(const void* px, int px_dtype, void* out, int NI, int img, int ps, int Kp, void* stream);
int launch_embed_assemble(const int64_t* ids, const int* src, const void* table, const void* feats, const void* newline,
                          void* out, int M, int H, int vocab, int* err, void* stream, int out_f32 = 0);
int launch_embed_bwd(const int64_t* ids, const int* src, const void* dout, float* dtable, void* dfeats, float* dnewline,
                     int M, int H, void* stream);
int launch_colsum(const void* dy, int64_t ld, int M, int N, float* out, int accumulate, void* stream);
int launch_row_group_mean(const void* x, int64_t ld, int G, int P, int D, float* out, void* stream);
int launch_row_group_mean_bwd(const float* dpool, int G, int P, int D, void* dx, int64_t ld, const float* sc, void* stream);
int launch_ntxent(const float* fs, const float* ft, int n, int D, float tau, float weight, float* loss_out, float* dfs,
                  float grad_scale, void* stream);
int launch_adamw(float* p, void* pb, const float* g, float* m, float* v, int64_t n, float lr, float b1, float b2,
                 float eps, float wd, int step, const float* gscale, const int32_t* skip, int n_skip, void* stream);
int launch_sumsq(const float* x, int64_t n, float* out, void* stream);
int launch_scalar_mul(const float* a, const float* b, float* out, int n, void* stream);
int launch_scale_f32(const float* x, const float* s_dev, float* y, int64_t n, void* stream);
int launch_image_src_map(const int64_t* ids, int B, int L, int64_t image_token, const int* map, int map_ld,
                         const int* map_len, int* src, int* err, void* stream);
int launch_quant_rows_f8(const void* x, int64_t ldx, int R, int K, void* q, int64_t ldq, float* scale, void* stream);
int launch_cast_f32_bf16(const float* x, void* y, int64_t n, void* stream);
int launch_prefetch(const void* ptr, uint64_t bytes, int grid, void* stream);
int launch_cast_bf16_f32(const void* x, float* y, int64_t n, void* stream);
size_t depth3_ws(int B, int H, int W);
size_t image_resize_ws(int H, int W, int oh, int ow);
size_t attn_decode_ws(int H, int hd, int smax);
int launch_attn_decode(const void* q, const void* k_new, const void* v_new, void* kc, void* vc, void* o, int H,
                       int HKV, int hd, int hdp, int smax, int n, const int* cur_dev, void* ws, size_t ws_bytes,
                       void* stream);
int launch_gemv(const void* x, const void* W, int64_t ldw, const void* extra, void* y, int N, int K, int epi, int I,
                const void* norm_w, float eps, void* stream);
int launch_gen_select(const void* logits, int V, int64_t* seq, int len, int* cur_dev, float penalty, int ngram,
                      void* flags_ws, size_t ws_bytes, int64_t* out, void* stream);
int launch_rope_row(const float* cos_t, const float* sin_t, int hh, const int* cur_dev, float* cos_row, float* sin_row,
                    void* stream);
int launch_image_resize(const uint8_t* in, int H, int W, uint8_t* out, int oh, int ow, void* ws, size_t ws_bytes,
                        void* stream);
int launch_anyres_tiles(const uint8_t* base, const uint8_t* resized, int nh, int nw, int bh, int bw, int patch,
                        int n_out, const float* mean_std_host, void* out, int out_dtype, void* stream);
int launch_depth3(const void* depth, int dtype, int B, int H, int W, void* out, void* ws, size_t ws_bytes,
                  void* stream);

// GEMM launch through the optional event timer (model.hip): every kd_gemm of the library
int gemm_timed(const kd_gemm_desc* d, void* stream);

}  // namespace kd
