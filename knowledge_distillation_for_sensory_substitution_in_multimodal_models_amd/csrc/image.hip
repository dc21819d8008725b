// LLaVA-OneVision image preprocessing on the GPU (gfx950): PIL-exact bicubic resize and the
// anyres pad / tile / rescale / normalize that produce `pixel_values`.
//
// Replaces the image half of the reference's collate_fn (DM:124-146: the HF processor run on the
// RGB and the 3-channel depth uint8 images), i.e. LlavaOnevisionImageProcessor._preprocess:
//   resize        PIL Image.resize(BICUBIC) of a uint8 RGB image.  Pillow's libImaging/Resample.c
//                 algorithm, restated: per output coordinate, bicubic (a = -0.5) taps over a
//                 support of 2 * max(scale, 1), normalised in double and quantised to int32 with
//                 22 fraction bits (precompute_coeffs + normalize_coeffs_8bpc); a horizontal pass
//                 into a uint8 temporary, then a vertical pass, each accumulating in int32 from
//                 1 << 21 and clipping to uint8 (clip8).  Integer arithmetic: bit-exact.
//   anyres tiles  the whole image resized to 384x384 first, then the aspect-preserving resize
//                 centred on a zero canvas of the best pinpoint resolution and cut into 384x384
//                 tiles (get_image_patches, _pad_for_patching, divide_to_patches)
//   rescale/norm  float32(float64(u8) * (1/255)), then (x - mean) / std in float32, HWC -> CHW;
//                 tiles past the image's own count are zero (_pad_for_batching)
//
// Kernels: k_resize_coeffs (one thread per output coordinate, per axis), k_resize_h / k_resize_v
// (one thread per output pixel, 3 channels, taps read through L1/L2: the images are a few MB),
// k_anyres_tiles (4 consecutive output elements per thread, one 16-B fp32 / 8-B bf16 store).
#include "common.h"

namespace kd {

namespace {

constexpr int PRECISION_BITS = 22;
constexpr int MAX_KSIZE = 64;   // downscale factor <= 15

__device__ __forceinline__ double bicubic_filter(double x) {
#pragma clang fp contract(off)
    const double a = -0.5;
    if (x < 0.0) x = -x;
    if (x < 1.0) return ((a + 2.0) * x - (a + 3.0)) * x * x + 1;
    if (x < 2.0) return (((x - 5) * x + 8) * x - 4) * a;
    return 0.0;
}

int host_ksize(int in_size, int out_size) {
#pragma clang fp contract(off)
    double filterscale = (double)(float)in_size / out_size;
    if (filterscale < 1.0) filterscale = 1.0;
    return (int)ceil(2.0 * filterscale) * 2 + 1;
}

__global__ void __launch_bounds__(256) k_resize_coeffs(int in_size, int out_size, int ksize, int* __restrict__ bounds,
                                                       int* __restrict__ kk) {
#pragma clang fp contract(off)
    const int xx = blockIdx.x * blockDim.x + threadIdx.x;
    if (xx >= out_size) return;
    const double scale = (double)(float)in_size / out_size;
    const double filterscale = scale < 1.0 ? 1.0 : scale;
    const double support = 2.0 * filterscale;
    const double center = 0.0 + (xx + 0.5) * scale;
    const double ss = 1.0 / filterscale;
    int xmin = (int)(center - support + 0.5);
    if (xmin < 0) xmin = 0;
    int xmax = (int)(center + support + 0.5);
    if (xmax > in_size) xmax = in_size;
    xmax -= xmin;
    double ww = 0.0;
    for (int x = 0; x < xmax; ++x) ww += bicubic_filter((x + xmin - center + 0.5) * ss);
    for (int x = 0; x < ksize; ++x) {
        int q = 0;
        if (x < xmax) {
            double w = bicubic_filter((x + xmin - center + 0.5) * ss);
            if (ww != 0.0) w /= ww;
            q = w < 0 ? (int)(-0.5 + w * (1 << PRECISION_BITS)) : (int)(0.5 + w * (1 << PRECISION_BITS));
        }
        kk[(size_t)xx * ksize + x] = q;
    }
    bounds[2 * xx] = xmin;
    bounds[2 * xx + 1] = xmax;
}

__device__ __forceinline__ uint32_t clip8(int v) {
    if (v >= (1 << PRECISION_BITS << 8)) return 255u;
    if (v <= 0) return 0u;
    return (uint32_t)(v >> PRECISION_BITS);
}

// out[y][xx][c] = clip8(sum_x in[y][xmin + x][c] * k[xx][x])   (ResampleHorizontal_8bpc)
__global__ void __launch_bounds__(256) k_resize_h(const uint8_t* __restrict__ in, int H, int W, uint8_t* __restrict__ out,
                                                  int ow, int ksize, const int* __restrict__ bounds,
                                                  const int* __restrict__ kk) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)H * ow) return;
    const int y = (int)(i / ow), xx = (int)(i - (int64_t)y * ow);
    const int xmin = bounds[2 * xx], n = bounds[2 * xx + 1];
    const int* k = kk + (size_t)xx * ksize;
    const uint8_t* row = in + ((size_t)y * W + xmin) * 3;
    int s0 = 1 << (PRECISION_BITS - 1), s1 = s0, s2 = s0;
    for (int x = 0; x < n; ++x) {
        const int w = k[x];
        s0 += (int)row[3 * x] * w;
        s1 += (int)row[3 * x + 1] * w;
        s2 += (int)row[3 * x + 2] * w;
    }
    uint8_t* o = out + (size_t)i * 3;
    o[0] = (uint8_t)clip8(s0);
    o[1] = (uint8_t)clip8(s1);
    o[2] = (uint8_t)clip8(s2);
}

// out[yy][x][c] = clip8(sum_y in[ymin + y][x][c] * k[yy][y])   (ResampleVertical_8bpc)
__global__ void __launch_bounds__(256) k_resize_v(const uint8_t* __restrict__ in, int W, uint8_t* __restrict__ out,
                                                  int oh, int ksize, const int* __restrict__ bounds,
                                                  const int* __restrict__ kk) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)oh * W) return;
    const int yy = (int)(i / W), x = (int)(i - (int64_t)yy * W);
    const int ymin = bounds[2 * yy], n = bounds[2 * yy + 1];
    const int* k = kk + (size_t)yy * ksize;
    const uint8_t* col = in + ((size_t)ymin * W + x) * 3;
    int s0 = 1 << (PRECISION_BITS - 1), s1 = s0, s2 = s0;
    for (int y = 0; y < n; ++y) {
        const int w = k[y];
        const uint8_t* p = col + (size_t)y * W * 3;
        s0 += (int)p[0] * w;
        s1 += (int)p[1] * w;
        s2 += (int)p[2] * w;
    }
    uint8_t* o = out + (size_t)i * 3;
    o[0] = (uint8_t)clip8(s0);
    o[1] = (uint8_t)clip8(s1);
    o[2] = (uint8_t)clip8(s2);
}

struct NormArgs {
    float mean[3], std[3];
};

__device__ __forceinline__ float rescale_normalize(uint32_t v, float mean, float std) {
#pragma clang fp contract(off)
    const float x = (float)((double)v * (1.0 / 255.0));   // rescale: float64 multiply, cast to float32
    return __fdiv_rn(__fsub_rn(x, mean), std);             // normalize: float32
}

// pixel_values[t][c][y][x] for t < n_out.  Tile 0 = base (the whole image at patch x patch);
// tile t >= 1 = canvas tile (t - 1) of the (bh x bw) zero canvas holding `resized` (nh x nw) at
// its centre; tiles t > n_real are zero.  Each thread: 4 consecutive x of one (t, c, y).
template <typename OutT>
__global__ void __launch_bounds__(256) k_anyres_tiles(const uint8_t* __restrict__ base, const uint8_t* __restrict__ resized,
                                                      int nh, int nw, int py, int px, int bw, int patch, int n_real,
                                                      int n_out, NormArgs na, OutT* __restrict__ out) {
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int qpr = patch >> 2;  // quads per row
    const int64_t total = (int64_t)n_out * 3 * patch * qpr;
    if (q >= total) return;
    const int xq = (int)(q % qpr);
    int64_t r = q / qpr;
    const int y = (int)(r % patch);
    r /= patch;
    const int c = (int)(r % 3);
    const int t = (int)(r / 3);
    const int x0 = xq * 4;
    float v[4];
    if (t >= n_real) {
        v[0] = v[1] = v[2] = v[3] = 0.f;
    } else if (t == 0) {
        const uint8_t* p = base + ((size_t)y * patch + x0) * 3 + c;
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = rescale_normalize(p[3 * k], na.mean[c], na.std[c]);
    } else {
        const int tpr = bw / patch, ti = (t - 1) / tpr, tj = (t - 1) - ti * tpr;
        const int ry = ti * patch + y - py, cx = tj * patch + x0 - px;   // (py, px): centred paste offset
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int rx = cx + k;
            uint32_t u = 0;   // _pad_for_patching pads the uint8 image with 0 before rescale/normalize
            if (ry >= 0 && ry < nh && rx >= 0 && rx < nw) u = resized[((size_t)ry * nw + rx) * 3 + c];
            v[k] = rescale_normalize(u, na.mean[c], na.std[c]);
        }
    }
    OutT* o = out + (size_t)q * 4;
    if constexpr (sizeof(OutT) == 4) {
        *(f32x4*)o = f32x4{v[0], v[1], v[2], v[3]};
    } else {
        *(bf16x4*)o = bf16x4{(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
    }
}

size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

}  // namespace

size_t image_resize_ws(int H, int W, int oh, int ow) {
    if (H <= 0 || W <= 0 || oh <= 0 || ow <= 0) return 0;
    const int kh = host_ksize(W, ow), kv = host_ksize(H, oh);
    return align256(sizeof(int) * 2 * (size_t)ow) + align256(sizeof(int) * (size_t)ow * kh) +
           align256(sizeof(int) * 2 * (size_t)oh) + align256(sizeof(int) * (size_t)oh * kv) +
           align256((size_t)H * ow * 3);
}

int launch_image_resize(const uint8_t* in, int H, int W, uint8_t* out, int oh, int ow, void* ws, size_t ws_bytes,
                        void* stream) {
    KD_CHECK_ARG(in && out, "image_resize: null pointer");
    KD_CHECK_SHAPE(H > 0 && W > 0 && oh > 0 && ow > 0, "image_resize: sizes must be positive");
    KD_CHECK_SHAPE((int64_t)H * W * 3 < ((int64_t)1 << 31) && (int64_t)oh * ow * 3 < ((int64_t)1 << 31) &&
                       (int64_t)H * ow * 3 < ((int64_t)1 << 31),
                   "image_resize: image too large");
    const int kh = host_ksize(W, ow), kv = host_ksize(H, oh);
    KD_CHECK_SHAPE(kh <= MAX_KSIZE && kv <= MAX_KSIZE, "image_resize: downscale factor above 15 not supported");
    hipStream_t s = as_stream(stream);
    if (oh == H && ow == W) {  // PIL: same size -> copy
        if (hipMemcpyAsync(out, in, (size_t)H * W * 3, hipMemcpyDeviceToDevice, s) != hipSuccess)
            return fail(KD_ERR_LAUNCH, "image_resize: copy failed");
        return KD_OK;
    }
    KD_CHECK_ARG(ws != nullptr, "image_resize: null workspace");
    if (ws_bytes < image_resize_ws(H, W, oh, ow)) return fail(KD_ERR_WORKSPACE, "image_resize: workspace too small");
    char* p = (char*)ws;
    int* bh = (int*)p;
    p += align256(sizeof(int) * 2 * (size_t)ow);
    int* kh_ = (int*)p;
    p += align256(sizeof(int) * (size_t)ow * kh);
    int* bv = (int*)p;
    p += align256(sizeof(int) * 2 * (size_t)oh);
    int* kv_ = (int*)p;
    p += align256(sizeof(int) * (size_t)oh * kv);
    uint8_t* tmp = (uint8_t*)p;
    const bool need_h = ow != W, need_v = oh != H;
    if (need_h) {
        hipLaunchKernelGGL(k_resize_coeffs, dim3(ceil_div(ow, 256)), dim3(256), 0, s, W, ow, kh, bh, kh_);
        uint8_t* dst = need_v ? tmp : out;
        hipLaunchKernelGGL(k_resize_h, dim3(ceil_div((int64_t)H * ow, 256)), dim3(256), 0, s, in, H, W, dst, ow, kh, bh,
                           kh_);
    }
    if (need_v) {
        hipLaunchKernelGGL(k_resize_coeffs, dim3(ceil_div(oh, 256)), dim3(256), 0, s, H, oh, kv, bv, kv_);
        const uint8_t* src = need_h ? tmp : in;
        hipLaunchKernelGGL(k_resize_v, dim3(ceil_div((int64_t)oh * ow, 256)), dim3(256), 0, s, src, ow, out, oh, kv,
                           bv, kv_);
    }
    KD_LAUNCH_CHECK("k_resize_*");
    return KD_OK;
}

int launch_anyres_tiles(const uint8_t* base, const uint8_t* resized, int nh, int nw, int bh, int bw, int patch,
                        int n_out, const float* mean_std_host, void* out, int out_dtype, void* stream) {
    KD_CHECK_ARG(base && out && mean_std_host, "anyres_tiles: null pointer");
    KD_CHECK_ARG(out_dtype == 0 || out_dtype == 1, "anyres_tiles: out_dtype must be 0 (float32) or 1 (bf16)");
    KD_CHECK_SHAPE(patch > 0 && patch % 4 == 0 && patch < 4096, "anyres_tiles: patch must be a positive multiple of 4");
    KD_CHECK_SHAPE(bh > 0 && bw > 0 && bh % patch == 0 && bw % patch == 0 && bh < 32768 && bw < 32768,
                   "anyres_tiles: best resolution must be a multiple of the patch size");
    KD_CHECK_SHAPE(nh > 0 && nw > 0 && nh <= bh && nw <= bw, "anyres_tiles: resized image larger than the canvas");
    KD_CHECK_ARG(resized != nullptr, "anyres_tiles: null resized image");
    const int n_real = 1 + (bh / patch) * (bw / patch);
    KD_CHECK_SHAPE(n_out >= 1, "anyres_tiles: n_out must be >= 1");
    KD_CHECK_ALIGN(out, out_dtype == 0 ? 16 : 8, "anyres_tiles: out misaligned");
    NormArgs na;
    for (int c = 0; c < 3; ++c) {
        na.mean[c] = mean_std_host[c];
        na.std[c] = mean_std_host[3 + c];
    }
    const int py = (bh - nh) / 2, px = (bw - nw) / 2;   // _get_padding_size: divmod(target - size, 2)
    const int64_t quads = (int64_t)n_out * 3 * patch * (patch / 4);
    const dim3 grid(ceil_div(quads, 256));
    hipStream_t s = as_stream(stream);
    const int nr = n_real < n_out ? n_real : n_out;
    if (out_dtype == 0)
        hipLaunchKernelGGL(k_anyres_tiles<float>, grid, dim3(256), 0, s, base, resized, nh, nw, py, px, bw, patch, nr,
                           n_out, na, (float*)out);
    else
        hipLaunchKernelGGL(k_anyres_tiles<bf16>, grid, dim3(256), 0, s, base, resized, nh, nw, py, px, bw, patch, nr,
                           n_out, na, (bf16*)out);
    KD_LAUNCH_CHECK("k_anyres_tiles");
    return KD_OK;
}

}  // namespace kd
