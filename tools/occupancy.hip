// Resident workgroups per CU of the attention forward kernels, from the HIP occupancy API
// (build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -I include tools/occupancy.hip -o /tmp/occ)
#include "../knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd/csrc/attention.hip"
#include <cstdio>

namespace kd { int fail(int code, const std::string&) { return code; } }

template <typename K> static void show(const char* name, K k, size_t smem) {
    int n = -1;
    hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k, 256, smem);
    hipFuncAttributes a{};
    (void)hipFuncGetAttributes(&a, (const void*)k);
    printf("%-40s smem %6zu  blocks/CU %d (%s)  regs %d  static lds %zu\n", name, smem, n, hipGetErrorString(e), a.numRegs,
           a.sharedSizeBytes);
}

int main() {
    using namespace kd;
    show("k_attn_fwd<128,true,2>", k_attn_fwd<128, true, 2>, 65536);
    show("k_attn_fwd32<128,true,false>", k_attn_fwd32<128, true, false>, 65536);
    show("k_attn_fwd32<128,false,false>", k_attn_fwd32<128, false, false>, 65536);
    show("k_attn_fwd32<128,true,true>", k_attn_fwd32<128, true, true>, 65536);
    show("k_attn_fwd32<64,true,false>", k_attn_fwd32<64, true, false>, 32768);
    show("k_attn_fwd32<96,false,false>", k_attn_fwd32<96, false, false>, 65536);
    show("k_attn_fwd32<128,true,false> 48K", k_attn_fwd32<128, true, false>, 49152);
    int dev = 0; hipDeviceProp_t pr{};
    (void)hipGetDeviceProperties(&pr, dev);
    printf("sharedMemPerMultiprocessor %zu maxSharedMemoryPerMultiProcessor %zu sharedMemPerBlock %zu\n",
           pr.sharedMemPerBlock, pr.maxSharedMemoryPerMultiProcessor, pr.sharedMemPerBlock);
    return 0;
}
