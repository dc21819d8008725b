// extern "C" entry points of include/kdstep.h.  Thin: argument plumbing only;
// every kernel lives in its own translation unit.
#include "common.h"
#include <cstring>

namespace kd {

static thread_local std::string g_last_error = "";

void set_error(const std::string& msg) { g_last_error = msg; }
int fail(int code, const std::string& msg) {
    g_last_error = msg;
    return code;
}

// launchers (defined in the kernel translation units)
int launch_kd_loss(const void* teacher, int64_t ld_t, int V_t, const void* student, int64_t ld_s,
                   int V_s, const int64_t* labels, int B, int L, kd_loss_params p, float* loss_out,
                   void* dlogits, int64_t ld_d, void* ws, size_t ws_bytes, void* stream);
size_t kd_loss_ws(int B, int L, int V);
int kd_loss_check_impl(const void* ws, void* stream);
int launch_gemm(const kd_gemm_desc* d, void* stream);

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

int kd_gemm(const kd_gemm_desc* desc, void* stream) { return kd::launch_gemm(desc, stream); }

}  // extern "C"
