// Depth image -> 3-channel uint8 image on the GPU (gfx950).
//
// Replaces CustomSUNRGBDDatasetOneVision.convert_depth_image_into_3D
// (dataset/dataloader/OneVision/CustomSUNRGBDDatasetOneVision.py:64-112), the step that
// turns each SUNRGBD depth PNG into the 3-channel image the student's processor consumes:
//   ch0 = uint8(255 * (d - min d) / (max d - min d))                     (DS:89-94)
//   Gx, Gy = scipy.ndimage.convolve(ch0, Prewitt Kx / Ky, mode='reflect') (DS:71-76, 97-98)
//   ch1 = safe_normalize(sqrt(Gx^2 + Gy^2)),  ch2 = safe_normalize(arctan2(Gy, Gx))  (DS:79-83, 101-106)
// Output layout is the reference's np.dstack: [B, H, W, 3] uint8, channel-interleaved.
//
// Passes (the two global min/max reductions of the reference force three sweeps):
//   k_depth_minmax      per-block min/max of the depth                         (reads 2-4 B/px)
//   k_depth_range<1>    per-image (min, max - min) from those partials (one block per image)
//   k_depth_grad        16x64-pixel tiles: the (18x66) halo window is quantised to ch0 ONCE
//                       into LDS, Prewitt Gx/Gy from LDS, per-block min/max of Gm and theta
//                       through exact integer / order keys (sqrt, atan2 once per block);
//                       writes one packed uint32 per pixel (ch0 | Gx | Gy, 30 bits) (4 B/px)
//   k_depth_range<2>    per-image ranges of Gm and theta
//   k_depth_pack        4 pixels per thread: one 16-B load of packed words, Gm/theta recomputed
//                       (same functions -> same floats), 12 contiguous output bytes as 3 dwords
// No atomics: a pass writes at most 256 per-block partials per image, reduced by the next
// range kernel, so the workspace needs no zeroing.
//
// Arithmetic follows numpy float32 step by step (mul, then correctly rounded div, truncating
// cast), so ch0 and ch1 are bit-exact.  Gx, Gy are small integers (|G| <= 765), exact in any
// precision; sqrt via f64 then rounded is identical to numpy's float32 sqrt for every
// reachable Gx^2+Gy^2 (checked exhaustively, tests/test_depth.py).  arctan2 is computed in
// f64 and rounded once (correctly rounded float32); numpy's float32 arctan2 is SIMD-library
// dependent at the last ulp, so ch2 can differ by one only where the reference's value sits
// within float32 rounding of an integer boundary (the tests bound exactly that).
#include "common.h"

namespace kd {

namespace {

constexpr int DT_U16 = 0, DT_I32 = 1, DT_F32 = 2;
constexpr int NT = 256;       // threads per block, 4 waves
constexpr int MAX_NB = 256;   // blocks per image (= partials per image, one per thread)

template <int DT>
__device__ __forceinline__ float load_depth(const void* p, int64_t i) {
    if constexpr (DT == DT_U16) return (float)((const uint16_t*)p)[i];
    else if constexpr (DT == DT_I32) return (float)((const int32_t*)p)[i];
    else return ((const float*)p)[i];
}

__device__ __forceinline__ float wave_min(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fminf(v, __shfl_xor(v, o, 64));
    return v;
}

// Block-wide (min, max) of NT threads' values; every thread gets the result.
__device__ __forceinline__ void block_minmax(float& lo, float& hi, float* sc) {
    lo = wave_min(lo);
    hi = wave_max(hi);
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    __syncthreads();
    if (l == 0) { sc[w] = lo; sc[4 + w] = hi; }
    __syncthreads();
    lo = fminf(fminf(sc[0], sc[1]), fminf(sc[2], sc[3]));
    hi = fmaxf(fmaxf(sc[4], sc[5]), fmaxf(sc[6], sc[7]));
}

// Reduce the nb partials (stride `stride` floats, pairs at offset `off`) of one image.
__device__ __forceinline__ void reduce_partials(const float* part, int nb, int stride, int off, float& lo,
                                                float& hi, float* sc) {
    lo = INFINITY;
    hi = -INFINITY;
    if ((int)threadIdx.x < nb) {
        lo = part[threadIdx.x * stride + off];
        hi = part[threadIdx.x * stride + off + 1];
    }
    block_minmax(lo, hi, sc);
}

// numpy: (255.0 * (x - lo) / den).astype(np.uint8) in float32.  den already holds the
// reference's (max - min) with its `max = min + 1e-6` fix-up for a flat range.  The x86 cast
// numpy uses maps NaN (0/0 when the fix-up rounds away) to 0 and wraps modulo 256.
__device__ __forceinline__ uint32_t quant255(float x, float lo, float den) {
#pragma clang fp contract(off)
    const float r = __fdiv_rn(__fmul_rn(255.0f, __fsub_rn(x, lo)), den);
    if (!(r >= 0.f)) return 0u;
    return (uint32_t)(int)r & 255u;
}

__device__ __forceinline__ float range_den(float lo, float hi) {
#pragma clang fp contract(off)
    if (hi == lo) hi = __fadd_rn(lo, 1e-6f);  // DS:81-82 / DS:92-93, float32 (NEP 50)
    return __fsub_rn(hi, lo);
}

template <int DT>
__global__ void __launch_bounds__(NT) k_depth_minmax(const void* __restrict__ depth, int HW, int nb,
                                                     float* __restrict__ part) {
    __shared__ float sc[8];
    const int b = blockIdx.y;
    const void* img = (const char*)depth + (size_t)b * HW * (DT == DT_U16 ? 2 : 4);
    float lo = INFINITY, hi = -INFINITY;
    for (int p = blockIdx.x * NT + threadIdx.x; p < HW; p += nb * NT) {
        const float v = load_depth<DT>(img, p);
        lo = fminf(lo, v);
        hi = fmaxf(hi, v);
    }
    block_minmax(lo, hi, sc);
    if (threadIdx.x == 0) {
        part[((size_t)b * nb + blockIdx.x) * 2 + 0] = lo;
        part[((size_t)b * nb + blockIdx.x) * 2 + 1] = hi;
    }
}

// One block per image: NP (min, max) partial pairs -> NP (min, max - min with the fix-up).
template <int NP>
__global__ void __launch_bounds__(NT) k_depth_range(const float* __restrict__ part, int nb,
                                                    float* __restrict__ rng) {
    __shared__ float sc[8];
    const int b = blockIdx.x;
#pragma unroll
    for (int j = 0; j < NP; ++j) {
        float lo, hi;
        reduce_partials(part + (size_t)b * nb * 2 * NP, nb, 2 * NP, 2 * j, lo, hi, sc);
        if (threadIdx.x == 0) {
            rng[b * 2 * NP + 2 * j] = lo;
            rng[b * 2 * NP + 2 * j + 1] = range_den(lo, hi);
        }
    }
}

constexpr int TR = 16, TC = 64;               // output tile; 256 threads = 64 columns x 4 row groups
constexpr int LR = TR + 2, LC = TC + 2;       // halo window

__device__ __forceinline__ int reflect_idx(int i, int n) {
    i = i < 0 ? -i - 1 : (i >= n ? 2 * n - i - 1 : i);  // scipy 'reflect' (d c b a | a b c d | d c b a)
    return min(max(i, 0), n - 1);                      // window rows past a tail tile: never used
}

__device__ __forceinline__ float grad_mag(int gx, int gy) { return (float)sqrt((double)(gx * gx + gy * gy)); }
__device__ __forceinline__ float grad_ang(int gx, int gy) { return (float)atan2((double)gy, (double)gx); }

// Exact order key of atan2(gy, gx) over (-pi, pi] for integer |gx|, |gy| <= 765: the "diamond
// angle" (quadrant + |y|/(|x|+|y|)), shifted so that gy < 0 maps below 0.  Distinct directions
// differ by >= 1/1530^2 in it, far above f64 rounding, and proportional (gx, gy) give the same
// correctly rounded quotient, so key order == angle order with ties exactly on equal angles:
// the block min/max of theta needs one f64 division per pixel instead of an atan2.
__device__ __forceinline__ double angle_key(int x, int y) {
    if (y >= 0) {
        if (x > 0 || (x == 0 && y == 0)) return y == 0 ? 0.0 : (double)y / (double)(x + y);
        return 1.0 + (double)(-x) / (double)(y - x);          // x <= 0: (pi/2, pi]
    }
    if (x < 0) return -2.0 + (double)(-y) / (double)(-x - y);  // (-pi, -pi/2)
    return -1.0 + (double)x / (double)(x - y);                 // [-pi/2, 0)
}

// Block-wide arg-min / arg-max of (key, packed direction); returns the winners' directions.
__device__ __forceinline__ void block_argminmax(double kmin, uint32_t pmin, double kmax, uint32_t pmax,
                                                double* skey, uint32_t* spair, uint32_t& omin, uint32_t& omax) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const double k1 = __shfl_xor(kmin, o, 64), k2 = __shfl_xor(kmax, o, 64);
        const uint32_t p1 = __shfl_xor(pmin, o, 64), p2 = __shfl_xor(pmax, o, 64);
        if (k1 < kmin) { kmin = k1; pmin = p1; }
        if (k2 > kmax) { kmax = k2; pmax = p2; }
    }
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    __syncthreads();
    if (l == 0) { skey[w] = kmin; skey[4 + w] = kmax; spair[w] = pmin; spair[4 + w] = pmax; }
    __syncthreads();
    omin = spair[0];
    omax = spair[4];
    double a = skey[0], z = skey[4];
#pragma unroll
    for (int i = 1; i < 4; ++i) {
        if (skey[i] < a) { a = skey[i]; omin = spair[i]; }
        if (skey[4 + i] > z) { z = skey[4 + i]; omax = spair[4 + i]; }
    }
}

__device__ __forceinline__ uint32_t pack_dir(int gx, int gy) {
    return (uint32_t)(gx + 1024) | ((uint32_t)(gy + 1024) << 11);
}
__device__ __forceinline__ float dir_ang(uint32_t p) {
    return grad_ang((int)(p & 2047u) - 1024, (int)((p >> 11) & 2047u) - 1024);
}

template <int DT>
__global__ void __launch_bounds__(NT) k_depth_grad(const void* __restrict__ depth, int H, int W, int tiles_x,
                                                   int ntiles, int nb, const float* __restrict__ rng_d,
                                                   uint32_t* __restrict__ packed, float* __restrict__ part_g) {
    __shared__ int win[LR][LC + 1];
    __shared__ float sc[8];
    __shared__ double skey[8];
    __shared__ uint32_t spair[8];
    const int b = blockIdx.y;
    const int HW = H * W;
    const void* img = (const char*)depth + (size_t)b * HW * (DT == DT_U16 ? 2 : 4);
    const float lo = rng_d[2 * b], den = rng_d[2 * b + 1];
    const int c = threadIdx.x & (TC - 1), rg = threadIdx.x >> 6;

    // min/max of Gm^2 (exact ints, as float) and arg-min/max of the angle key; sqrt / atan2 run
    // once per block on the winners (k_depth_pack recomputes them per pixel, same functions)
    float nl = INFINITY, nh = -INFINITY;
    double kl = INFINITY, kh = -INFINITY;
    uint32_t pl = pack_dir(0, 0), ph = pack_dir(0, 0);
    for (int t = blockIdx.x; t < ntiles; t += nb) {
        const int ty = t / tiles_x, tx = t - ty * tiles_x;
        const int r0 = ty * TR, c0 = tx * TC;
        __syncthreads();  // the previous tile's window is consumed
        for (int e = threadIdx.x; e < LR * LC; e += NT) {
            const int lr = e / LC, lc = e - lr * LC;
            const int gr = reflect_idx(r0 + lr - 1, H), gc = reflect_idx(c0 + lc - 1, W);
            win[lr][lc] = (int)quant255(load_depth<DT>(img, gr * W + gc), lo, den);
        }
        __syncthreads();
        if (c0 + c < W) {
#pragma unroll
            for (int k = 0; k < TR / 4; ++k) {
                const int r = rg * (TR / 4) + k;
                if (r0 + r >= H) break;
                // convolve() flips the kernel: Gx = sum_r d[i+r][j-1] - d[i+r][j+1],
                //                              Gy = sum_c d[i-1][j+c] - d[i+1][j+c]
                const int gx = (win[r][c] + win[r + 1][c] + win[r + 2][c]) -
                               (win[r][c + 2] + win[r + 1][c + 2] + win[r + 2][c + 2]);
                const int gy = (win[r][c] + win[r][c + 1] + win[r][c + 2]) -
                               (win[r + 2][c] + win[r + 2][c + 1] + win[r + 2][c + 2]);
                packed[(size_t)b * HW + (r0 + r) * W + c0 + c] =
                    (uint32_t)win[r + 1][c + 1] | ((uint32_t)(gx + 1024) << 8) | ((uint32_t)(gy + 1024) << 19);
                const float n2 = (float)(gx * gx + gy * gy);
                nl = fminf(nl, n2);
                nh = fmaxf(nh, n2);
                const double key = angle_key(gx, gy);
                if (key < kl) { kl = key; pl = pack_dir(gx, gy); }
                if (key > kh) { kh = key; ph = pack_dir(gx, gy); }
            }
        }
    }
    block_minmax(nl, nh, sc);
    uint32_t dl, dh;
    block_argminmax(kl, pl, kh, ph, skey, spair, dl, dh);
    if (threadIdx.x == 0) {
        float* o = part_g + ((size_t)b * nb + blockIdx.x) * 4;
        o[0] = (float)sqrt((double)nl);   // == grad_mag of the arg-min pixel (n2 is an exact int)
        o[1] = (float)sqrt((double)nh);
        o[2] = dir_ang(dl);
        o[3] = dir_ang(dh);
    }
}

__device__ __forceinline__ uint32_t pixel3(uint32_t w, const float* __restrict__ rg) {
    const int gx = (int)((w >> 8) & 2047u) - 1024, gy = (int)((w >> 19) & 2047u) - 1024;
    const uint32_t m = quant255(grad_mag(gx, gy), rg[0], rg[1]);
    const uint32_t a = quant255(grad_ang(gx, gy), rg[2], rg[3]);
    return (w & 255u) | (m << 8) | (a << 16);
}

__global__ void __launch_bounds__(NT) k_depth_pack(const uint32_t* __restrict__ packed, int64_t total, int HW,
                                                   const float* __restrict__ rng_g, uint8_t* __restrict__ out) {
    const int64_t quads = total >> 2;
    for (int64_t q = (int64_t)blockIdx.x * NT + threadIdx.x; q < quads; q += (int64_t)gridDim.x * NT) {
        const u32x4 w = ((const u32x4*)packed)[q];
        const int64_t base = q * 4;
        const int b0 = (int)(base / HW);
        const int64_t next = (int64_t)(b0 + 1) * HW;  // first pixel of the next image
        uint32_t px[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) px[k] = pixel3(w[k], rng_g + 4 * (b0 + (base + k >= next)));
        uint32_t* o = (uint32_t*)(out + base * 3);                 // 4-B aligned: 12*q
        o[0] = px[0] | (px[1] << 24);
        o[1] = (px[1] >> 8) | (px[2] << 16);
        o[2] = (px[2] >> 16) | (px[3] << 8);
    }
    if (blockIdx.x == 0 && threadIdx.x < (total & 3)) {           // tail pixels
        const int64_t p = (quads << 2) + threadIdx.x;
        const uint32_t v = pixel3(packed[p], rng_g + 4 * (int)(p / HW));
        out[p * 3] = (uint8_t)v;
        out[p * 3 + 1] = (uint8_t)(v >> 8);
        out[p * 3 + 2] = (uint8_t)(v >> 16);
    }
}

int blocks_per_image(int64_t HW) {
    const int64_t nb = (HW + 4 * NT - 1) / (4 * NT);
    return (int)(nb < MAX_NB ? (nb > 0 ? nb : 1) : MAX_NB);
}

size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

struct DepthWs {
    float *part_d, *rng_d, *part_g, *rng_g;
    uint32_t* packed;
    size_t bytes;
    int nbm, tiles_x, ntiles, nbg;
};

DepthWs depth_ws_layout(int B, int H, int W, void* base) {
    DepthWs w{};
    const int64_t HW = (int64_t)H * W;
    w.nbm = blocks_per_image(HW);
    w.tiles_x = (W + TC - 1) / TC;
    w.ntiles = w.tiles_x * ((H + TR - 1) / TR);
    w.nbg = w.ntiles < MAX_NB ? w.ntiles : MAX_NB;
    size_t off = 0;
    auto take = [&](size_t n) { char* p = (char*)base + off; off += align256(n); return p; };
    w.part_d = (float*)take((size_t)B * w.nbm * 2 * sizeof(float));
    w.rng_d = (float*)take((size_t)B * 2 * sizeof(float));
    w.part_g = (float*)take((size_t)B * w.nbg * 4 * sizeof(float));
    w.rng_g = (float*)take((size_t)B * 4 * sizeof(float));
    w.packed = (uint32_t*)take((size_t)B * HW * sizeof(uint32_t));
    w.bytes = off;
    return w;
}

}  // namespace

size_t depth3_ws(int B, int H, int W) {
    if (B <= 0 || H <= 0 || W <= 0) return 0;
    return depth_ws_layout(B, H, W, nullptr).bytes;
}

int launch_depth3(const void* depth, int dtype, int B, int H, int W, void* out, void* ws, size_t ws_bytes,
                  void* stream) {
    KD_CHECK_ARG(depth && out && ws, "depth_to_3ch: null pointer");
    KD_CHECK_ARG(dtype == DT_U16 || dtype == DT_I32 || dtype == DT_F32,
                 "depth_to_3ch: dtype must be 0 (uint16), 1 (int32) or 2 (float32)");
    KD_CHECK_SHAPE(B > 0 && H > 0 && W > 0, "depth_to_3ch: B, H, W must be positive");
    KD_CHECK_SHAPE((int64_t)H * W < ((int64_t)1 << 31) / 4, "depth_to_3ch: image too large");
    KD_CHECK_ALIGN(depth, dtype == DT_U16 ? 2 : 4, "depth_to_3ch: depth pointer misaligned");
    KD_CHECK_ALIGN(out, 4, "depth_to_3ch: out must be 4-B aligned");
    KD_CHECK_ALIGN(ws, 256, "depth_to_3ch: workspace must be 256-B aligned");
    if (ws_bytes < depth3_ws(B, H, W)) return fail(KD_ERR_WORKSPACE, "depth_to_3ch: workspace too small");
    const int HW = H * W;
    const DepthWs w = depth_ws_layout(B, H, W, ws);
    hipStream_t s = as_stream(stream);
    const dim3 gm(w.nbm, B), gg(w.nbg, B);
    switch (dtype) {
        case DT_U16:
            hipLaunchKernelGGL(k_depth_minmax<DT_U16>, gm, dim3(NT), 0, s, depth, HW, w.nbm, w.part_d);
            hipLaunchKernelGGL(k_depth_range<1>, dim3(B), dim3(NT), 0, s, w.part_d, w.nbm, w.rng_d);
            hipLaunchKernelGGL(k_depth_grad<DT_U16>, gg, dim3(NT), 0, s, depth, H, W, w.tiles_x, w.ntiles, w.nbg,
                               w.rng_d, w.packed, w.part_g);
            break;
        case DT_I32:
            hipLaunchKernelGGL(k_depth_minmax<DT_I32>, gm, dim3(NT), 0, s, depth, HW, w.nbm, w.part_d);
            hipLaunchKernelGGL(k_depth_range<1>, dim3(B), dim3(NT), 0, s, w.part_d, w.nbm, w.rng_d);
            hipLaunchKernelGGL(k_depth_grad<DT_I32>, gg, dim3(NT), 0, s, depth, H, W, w.tiles_x, w.ntiles, w.nbg,
                               w.rng_d, w.packed, w.part_g);
            break;
        default:
            hipLaunchKernelGGL(k_depth_minmax<DT_F32>, gm, dim3(NT), 0, s, depth, HW, w.nbm, w.part_d);
            hipLaunchKernelGGL(k_depth_range<1>, dim3(B), dim3(NT), 0, s, w.part_d, w.nbm, w.rng_d);
            hipLaunchKernelGGL(k_depth_grad<DT_F32>, gg, dim3(NT), 0, s, depth, H, W, w.tiles_x, w.ntiles, w.nbg,
                               w.rng_d, w.packed, w.part_g);
    }
    hipLaunchKernelGGL(k_depth_range<2>, dim3(B), dim3(NT), 0, s, w.part_g, w.nbg, w.rng_g);
    const int64_t total = (int64_t)B * HW;
    const int64_t quads = total >> 2;
    const int grid = (int)std::max<int64_t>(1, std::min<int64_t>((quads + NT - 1) / NT, 4096));
    hipLaunchKernelGGL(k_depth_pack, dim3(grid), dim3(NT), 0, s, w.packed, total, HW, w.rng_g, (uint8_t*)out);
    KD_LAUNCH_CHECK("k_depth_*");
    return KD_OK;
}

}  // namespace kd
