// Device-side image preprocessing for real-data training: caffe/tf normalisation, affine warp and
// bilinear resize into the zero-padded NHWC batch.
//
// Spec: keras-retinanet Generator.preprocess_group_entry = preprocess_image (caffe BGR mean
// subtraction) -> random affine (cv2.warpAffine, TransformParameters fill_mode/interpolation/cval)
// -> resize_image (cv2.resize INTER_LINEAR) -> compute_inputs (zero pad, top-left) (SURVEY §2.2
// E-KR-image/E-KR-transform, K22; reached from /root/reference/train.py:179-193).  The sampling
// arithmetic matches csrc/cpu/runtime_cpu.cpp (mxr_cpu_warp_affine / mxr_cpu_resize_bilinear) so the
// host and device paths agree to float rounding; tests/test_kernels_gpu.py pins that.
//
// Layout: images are HWC with 3 channels (BGR); one thread per output pixel writes its 3 channels.
// Coordinates are computed in double exactly as the host path does (the warp's inverse matrix is
// formed on the host in double and passed by value).
#include "common.h"

namespace {
constexpr int kBlock = 256;

__device__ __forceinline__ int border_index(int i, int n, int mode, bool& outside) {
  outside = false;
  if (i >= 0 && i < n) return i;
  switch (mode) {
    case 1: return i < 0 ? 0 : n - 1;
    case 2: {
      if (n == 1) return 0;
      const int p = 2 * (n - 1);
      i = ((i % p) + p) % p;
      return i < n ? i : p - i;
    }
    case 3: return ((i % n) + n) % n;
    default: outside = true; return 0;
  }
}

struct Norm { float scale, m0, m1, m2; };

__device__ __forceinline__ float norm_px(const uint8_t* p, int c, const Norm& nm) {
  const float m = c == 0 ? nm.m0 : (c == 1 ? nm.m1 : nm.m2);
  return (float)p[c] * nm.scale - m;
}

// dst[y, x, c] = normalise(src)[Minv * (x, y)] (bilinear or nearest), or plain normalise when warp == 0
__global__ __launch_bounds__(kBlock) void warp_norm_kernel(const uint8_t* __restrict__ src, int H, int W,
                                                           float* __restrict__ dst, int OH, int OW, double ia, double ib,
                                                           double ic, double id, double ie, double iff, int warp,
                                                           int interp, int border, float cval, Norm nm) {
  const long long total = (long long)OH * OW;
  for (long long i = blockIdx.x * (long long)kBlock + threadIdx.x; i < total; i += (long long)gridDim.x * kBlock) {
    const int x = (int)(i % OW), y = (int)(i / OW);
    float* o = dst + i * 3;
    if (!warp) {
      const uint8_t* p = src + i * 3;
#pragma unroll
      for (int c = 0; c < 3; ++c) o[c] = norm_px(p, c, nm);
      continue;
    }
    const double sxf = ia * x + ib * y + ic;
    const double syf = id * x + ie * y + iff;
    if (interp == 0) {
      bool o1, o2;
      const int xi = border_index((int)llround(sxf), W, border, o1);
      const int yi = border_index((int)llround(syf), H, border, o2);
      const uint8_t* p = src + ((long long)yi * W + xi) * 3;
#pragma unroll
      for (int c = 0; c < 3; ++c) o[c] = (o1 || o2) ? cval : norm_px(p, c, nm);
      continue;
    }
    const int x0 = (int)floor(sxf), y0 = (int)floor(syf);
    const float tx = (float)(sxf - x0), ty = (float)(syf - y0);
    bool ox0, ox1, oy0, oy1;
    const int xa = border_index(x0, W, border, ox0), xb = border_index(x0 + 1, W, border, ox1);
    const int ya = border_index(y0, H, border, oy0), yb = border_index(y0 + 1, H, border, oy1);
    const uint8_t* p00 = src + ((long long)ya * W + xa) * 3;
    const uint8_t* p01 = src + ((long long)ya * W + xb) * 3;
    const uint8_t* p10 = src + ((long long)yb * W + xa) * 3;
    const uint8_t* p11 = src + ((long long)yb * W + xb) * 3;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const float v00 = (ox0 || oy0) ? cval : norm_px(p00, c, nm);
      const float v01 = (ox1 || oy0) ? cval : norm_px(p01, c, nm);
      const float v10 = (ox0 || oy1) ? cval : norm_px(p10, c, nm);
      const float v11 = (ox1 || oy1) ? cval : norm_px(p11, c, nm);
      const float top = v00 + (v01 - v00) * tx, bot = v10 + (v11 - v10) * tx;
      o[c] = top + (bot - top) * ty;
    }
  }
}

// cv2.resize INTER_LINEAR (half-pixel centres, edge clamp) of an HWC float image into a batch slot
// with row pitch ld (elements); the padding of the slot is left untouched (pre-zeroed).
template <typename T>
__global__ __launch_bounds__(kBlock) void resize_kernel(const float* __restrict__ src, int H, int W,
                                                        T* __restrict__ dst, int OH, int OW, long long ld) {
  const double sy = (double)H / OH, sx = (double)W / OW;
  const long long total = (long long)OH * OW;
  for (long long i = blockIdx.x * (long long)kBlock + threadIdx.x; i < total; i += (long long)gridDim.x * kBlock) {
    const int x = (int)(i % OW), y = (int)(i / OW);
    double f = (x + 0.5) * sx - 0.5;
    int xi = (int)floor(f);
    double t = f - xi;
    if (xi < 0) { xi = 0; t = 0; }
    if (xi >= W - 1) { xi = W - 1; t = 0; }
    const int xj = min(xi + 1, W - 1);
    const float tx = (float)t;
    f = (y + 0.5) * sy - 0.5;
    int yi = (int)floor(f);
    t = f - yi;
    if (yi < 0) { yi = 0; t = 0; }
    if (yi >= H - 1) { yi = H - 1; t = 0; }
    const int yj = min(yi + 1, H - 1);
    const float ty = (float)t;
    const float* a = src + ((long long)yi * W + xi) * 3;
    const float* b = src + ((long long)yi * W + xj) * 3;
    const float* c = src + ((long long)yj * W + xi) * 3;
    const float* e = src + ((long long)yj * W + xj) * 3;
    T* o = dst + (long long)y * ld + (long long)x * 3;
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) {
      const float top = a[ch] + (b[ch] - a[ch]) * tx;
      const float bot = c[ch] + (e[ch] - c[ch]) * tx;
      o[ch] = Cvt<T>::from_f(top + (bot - top) * ty);
    }
  }
}
}  // namespace

// M is the 2x3 src->dst affine (the warp samples src at M^-1 * dst, like cv2.warpAffine without
// WARP_INVERSE_MAP).  warp == 0 skips the warp (normalise only; M ignored, OH/OW must equal H/W).
MXR_API int mxr_image_warp_normalize(const uint8_t* src, int H, int W, float* dst, int OH, int OW, const double* M,
                                     int warp, int interp, int border, float cval, float scale, float m0, float m1,
                                     float m2, hipStream_t stream) {
  if (H <= 0 || W <= 0 || OH <= 0 || OW <= 0) return -1;
  if (!warp && (OH != H || OW != W)) return -2;
  double ia = 0, ib = 0, ic = 0, id = 0, ie = 0, iff = 0;
  if (warp) {
    const double a = M[0], b = M[1], c = M[2], d = M[3], e = M[4], f = M[5];
    double det = a * e - b * d;
    det = det != 0 ? 1.0 / det : 0.0;
    ia = e * det; ib = -b * det; id = -d * det; ie = a * det;
    ic = -(ia * c + ib * f); iff = -(id * c + ie * f);
  }
  Norm nm{scale, m0, m1, m2};
  const long long n = (long long)OH * OW;
  hipLaunchKernelGGL(warp_norm_kernel, dim3(mxr_grid(n, kBlock, 16384)), dim3(kBlock), 0, stream, src, H, W, dst, OH,
                     OW, ia, ib, ic, id, ie, iff, warp, interp, border, cval, nm);
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

// dtype: 0 fp32 slot, 1 bf16 slot
MXR_API int mxr_image_resize_into(const float* src, int H, int W, void* dst, int OH, int OW, long long ld, int dtype,
                                  hipStream_t stream) {
  if (H <= 0 || W <= 0 || OH <= 0 || OW <= 0 || ld < 3LL * OW) return -1;
  const long long n = (long long)OH * OW;
  if (dtype == 0)
    hipLaunchKernelGGL(resize_kernel<float>, dim3(mxr_grid(n, kBlock, 16384)), dim3(kBlock), 0, stream, src, H, W,
                       (float*)dst, OH, OW, ld);
  else
    hipLaunchKernelGGL(resize_kernel<bf16_t>, dim3(mxr_grid(n, kBlock, 16384)), dim3(kBlock), 0, stream, src, H, W,
                       (bf16_t*)dst, OH, OW, ld);
  return hipGetLastError() == hipSuccess ? 0 : -3;
}
