// NHWC max-pool (TF 'same', -inf padding) and FPN nearest-upsample + lateral add, fwd and bwd.
//
// Spec: keras-resnet pool1 = MaxPooling2D(3, strides=2, padding='same') and
// keras-retinanet UpsampleLike = tf.image.resize_images(NEAREST, align_corners=False) followed by
// Add (P4_merged / P3_merged).  TF1 nearest: src = min(floor(dst*in/out), in-1),
// which is NOT a plain x2 for 84 -> 167.  The backward of the upsample is a deterministic gather
// over the (monotone) inverse index ranges -- no atomics.
// All kernels move 8 channels (16 B of bf16) per thread.
#include <cstdlib>

#include "common.h"

namespace {
constexpr int kBlock = 256;

template <typename T> struct V8;
template <> struct V8<bf16_t> { typedef uint4 type; };
template <> struct V8<float> { struct type { float4 a, b; }; };

// out[n, oy, ox, c] = max over the 3x3 window; arg[n, oy, ox, c] = window index (ky*k+kx) of the first max.
// relu_in: x is a ReLU output, so a window whose max is 0 passes no gradient (relu'(0) = 0): its arg is
// set to 255, which the backward never matches -- the ReLU backward of the producer is fused away.
// 32-bit index math (N*H*W*C/8 < 2^31 is checked on the host): 64-bit division is emulated on CDNA.
template <typename T>
__global__ __launch_bounds__(kBlock) void maxpool_fwd(const T* __restrict__ x, T* __restrict__ y, uint8_t* __restrict__ arg,
                                                      int N, int H, int W, int C, int Ho, int Wo, int k, int s, int pt,
                                                      int pl, int relu_in) {
  const int CV = C >> 3;
  const int total = N * Ho * Wo * CV;
  for (int i = blockIdx.x * kBlock + threadIdx.x; i < total; i += gridDim.x * kBlock) {
    const int cv = i % CV;
    int r = i / CV;
    const int ox = r % Wo;
    r /= Wo;
    const int oy = r % Ho;
    const int n = r / Ho;
    float best[8];
    uint8_t bi[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { best[j] = -INFINITY; bi[j] = 0; }
    for (int ky = 0; ky < k; ++ky) {
      const int iy = oy * s - pt + ky;
      if (iy < 0 || iy >= H) continue;
      for (int kx = 0; kx < k; ++kx) {
        const int ix = ox * s - pl + kx;
        if (ix < 0 || ix >= W) continue;
        const T* src = x + ((size_t)(n * H + iy) * W + ix) * C + cv * 8;
        T v[8];
        *reinterpret_cast<typename V8<T>::type*>(v) = *reinterpret_cast<const typename V8<T>::type*>(src);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float f = Cvt<T>::to_f(v[j]);
          if (f > best[j]) { best[j] = f; bi[j] = (uint8_t)(ky * k + kx); }
        }
      }
    }
    T o[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      o[j] = Cvt<T>::from_f(best[j]);
      if (relu_in && !(best[j] > 0.f)) bi[j] = 255;
    }
    const size_t oo = (size_t)i * 8;   // (((n*Ho + oy)*Wo + ox)*C + cv*8
    *reinterpret_cast<typename V8<T>::type*>(y + oo) = *reinterpret_cast<typename V8<T>::type*>(o);
    *reinterpret_cast<uint2*>(arg + oo) = *reinterpret_cast<uint2*>(bi);
  }
}

// 3x3 / stride-2 bf16 specialisation of maxpool_fwd (the stem's pool1): the nine window loads are issued
// together (an out-of-range tap reads a clamped in-range pixel and is masked to -inf afterwards) instead
// of one per branch of the generic loop; the compare order -- and so the first-max tie rule -- is unchanged.
__global__ __launch_bounds__(kBlock) void maxpool_fwd_k3s2(const bf16_t* __restrict__ x, bf16_t* __restrict__ y,
                                                           uint8_t* __restrict__ arg, int N, int H, int W, int C, int Ho, int Wo, int pt, int pl,
                                                           int relu_in) {
  const int CV = C >> 3;
  const int total = N * Ho * Wo * CV;
  for (int i = blockIdx.x * kBlock + threadIdx.x; i < total; i += gridDim.x * kBlock) {
    const int cv = i % CV;
    int r = i / CV;
    const int ox = r % Wo;
    r /= Wo;
    const int oy = r % Ho;
    const int n = r / Ho;
    uint4 v[9];
    bool ok[9];
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int iy = oy * 2 - pt + t / 3, ix = ox * 2 - pl + t % 3;
      ok[t] = iy >= 0 && iy < H && ix >= 0 && ix < W;
      const int cy = min(max(iy, 0), H - 1), cx = min(max(ix, 0), W - 1);
      const bf16_t* src = x + ((size_t)(n * H + cy) * W + cx) * C + cv * 8;
      v[t] = *reinterpret_cast<const uint4*>(src);
    }
    float best[8];
    uint8_t bi[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { best[j] = -INFINITY; bi[j] = 0; }
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const uint32_t w[4] = {v[t].x, v[t].y, v[t].z, v[t].w};
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float f = ok[t] ? bf2f((bf16_t)(j & 1 ? w[j >> 1] >> 16 : w[j >> 1] & 0xffff)) : -INFINITY;
        if (f > best[j]) { best[j] = f; bi[j] = (uint8_t)t; }
      }
    }
    bf16_t o[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      o[j] = f2bf(best[j]);
      if (relu_in && !(best[j] > 0.f)) bi[j] = 255;
    }
    const size_t oo = (size_t)i * 8;
    *reinterpret_cast<uint4*>(y + oo) = *reinterpret_cast<uint4*>(o);
    *reinterpret_cast<uint2*>(arg + oo) = *reinterpret_cast<uint2*>(bi);
  }
}

// dx[n, iy, ix, c] = sum of dy over the (<= ceil(k/s)^2) windows whose argmax is (iy, ix)
template <typename T>
__global__ __launch_bounds__(kBlock) void maxpool_bwd(const T* __restrict__ dy, const uint8_t* __restrict__ arg,
                                                      T* __restrict__ dx, int N, int H, int W, int C, int Ho, int Wo,
                                                      int k, int s, int pt, int pl) {
  const int CV = C >> 3;
  const int total = N * H * W * CV;
  for (int i = blockIdx.x * kBlock + threadIdx.x; i < total; i += gridDim.x * kBlock) {
    const int cv = i % CV;
    int r = i / CV;
    const int ix = r % W;
    r /= W;
    const int iy = r % H;
    const int n = r / H;
    float acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = 0.f;
    // windows oy with oy*s - pt <= iy <= oy*s - pt + k - 1
    const int oy0 = max(0, (iy + pt - k + s) / s), oy1 = min(Ho - 1, (iy + pt) / s);
    const int ox0 = max(0, (ix + pl - k + s) / s), ox1 = min(Wo - 1, (ix + pl) / s);
    for (int oy = oy0; oy <= oy1; ++oy) {
      const int ky = iy - (oy * s - pt);
      if (ky < 0 || ky >= k) continue;
      for (int ox = ox0; ox <= ox1; ++ox) {
        const int kx = ix - (ox * s - pl);
        if (kx < 0 || kx >= k) continue;
        const size_t oo = ((size_t)(n * Ho + oy) * Wo + ox) * C + cv * 8;
        uint8_t a[8];
        *reinterpret_cast<uint2*>(a) = *reinterpret_cast<const uint2*>(arg + oo);
        const uint8_t me = (uint8_t)(ky * k + kx);
        bool any = false;
#pragma unroll
        for (int j = 0; j < 8; ++j) any |= a[j] == me;
        if (!any) continue;
        T g[8];
        *reinterpret_cast<typename V8<T>::type*>(g) = *reinterpret_cast<const typename V8<T>::type*>(dy + oo);
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (a[j] == me) acc[j] += Cvt<T>::to_f(g[j]);
      }
    }
    T o[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = Cvt<T>::from_f(acc[j]);
    *reinterpret_cast<typename V8<T>::type*>(dx + (size_t)i * 8) = *reinterpret_cast<typename V8<T>::type*>(o);
  }
}

// 3x3 / stride-2 specialisation: thread (n, j, i, cv) owns the 2x2 input pixels u = iy + pt in {2j, 2j+1},
// v = ix + pl in {2i, 2i+1}; they are covered only by windows oy in {j-1, j}, ox in {i-1, i}, so the
// thread loads those 4 (arg, dy) pairs once (neighbours share them through the cache) instead of
// re-deriving the window set per pixel.  Window-local index me = ky*3 + kx with ky = u - 2*oy.
__global__ __launch_bounds__(kBlock) void maxpool_bwd_k3s2(const bf16_t* __restrict__ dy, const uint8_t* __restrict__ arg,
                                                         bf16_t* __restrict__ dx, int N, int H, int W, int C, int Ho,
                                                         int Wo, int pt, int pl, int Hb, int Wb) {
  const int CV = C >> 3;
  const int total = N * Hb * Wb * CV;
  for (int t = blockIdx.x * kBlock + threadIdx.x; t < total; t += gridDim.x * kBlock) {
    const int cv = t % CV;
    int r = t / CV;
    const int i = r % Wb;
    r /= Wb;
    const int j = r % Hb;
    const int n = r / Hb;
    uint8_t a[2][2][8];
    float g[2][2][8];
#pragma unroll
    for (int wy = 0; wy < 2; ++wy)
#pragma unroll
      for (int wx = 0; wx < 2; ++wx) {
        const int oy = j - 1 + wy, ox = i - 1 + wx;
        if (oy >= 0 && oy < Ho && ox >= 0 && ox < Wo) {
          const size_t oo = ((size_t)(n * Ho + oy) * Wo + ox) * C + cv * 8;
          *reinterpret_cast<uint2*>(a[wy][wx]) = *reinterpret_cast<const uint2*>(arg + oo);
          bf16_t h[8];
          *reinterpret_cast<uint4*>(h) = *reinterpret_cast<const uint4*>(dy + oo);
#pragma unroll
          for (int c = 0; c < 8; ++c) g[wy][wx][c] = bf2f(h[c]);
        } else {
#pragma unroll
          for (int c = 0; c < 8; ++c) { a[wy][wx][c] = 255; g[wy][wx][c] = 0.f; }
        }
      }
#pragma unroll
    for (int d = 0; d < 2; ++d) {
      const int iy = 2 * j + d - pt;
      if (iy < 0 || iy >= H) continue;
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int ix = 2 * i + e - pl;
        if (ix < 0 || ix >= W) continue;
        float acc[8];
#pragma unroll
        for (int c = 0; c < 8; ++c) acc[c] = 0.f;
        // windows (wy, wx) covering (d, e): wy = 1 always (ky = d); wy = 0 only for d = 0 (ky = 2)
#pragma unroll
        for (int wy = 0; wy < 2; ++wy) {
          if (wy == 0 && d == 1) continue;
          const int ky = wy == 1 ? d : 2;
#pragma unroll
          for (int wx = 0; wx < 2; ++wx) {
            if (wx == 0 && e == 1) continue;
            const int kx = wx == 1 ? e : 2;
            const uint8_t me = (uint8_t)(ky * 3 + kx);
#pragma unroll
            for (int c = 0; c < 8; ++c)
              if (a[wy][wx][c] == me) acc[c] += g[wy][wx][c];
          }
        }
        bf16_t o[8];
#pragma unroll
        for (int c = 0; c < 8; ++c) o[c] = f2bf(acc[c]);
        *reinterpret_cast<uint4*>(dx + ((size_t)(n * H + iy) * W + ix) * C + cv * 8) = *reinterpret_cast<uint4*>(o);
      }
    }
  }
}

// y[n, Y, X, c] = lat[n, Y, X, c] + x[n, iy(Y), ix(X), c]
template <typename T>
__global__ __launch_bounds__(kBlock) void upsample_add_fwd(const T* __restrict__ x, const T* __restrict__ lat,
                                                           T* __restrict__ y, const int* __restrict__ iy_of,
                                                           const int* __restrict__ ix_of, int N, int h, int w, int H,
                                                           int W, int C) {
  const int CV = C / 8;
  const long long total = (long long)N * H * W * CV;
  for (long long i = blockIdx.x * (long long)kBlock + threadIdx.x; i < total; i += (long long)gridDim.x * kBlock) {
    const int cv = (int)(i % CV);
    long long r = i / CV;
    const int X = (int)(r % W); r /= W;
    const int Y = (int)(r % H);
    const int n = (int)(r / H);
    const long long o = i * 8;
    const long long si = (((long long)n * h + iy_of[Y]) * w + ix_of[X]) * C + cv * 8;
    T a[8], b[8], c[8];
    *reinterpret_cast<typename V8<T>::type*>(a) = *reinterpret_cast<const typename V8<T>::type*>(lat + o);
    *reinterpret_cast<typename V8<T>::type*>(b) = *reinterpret_cast<const typename V8<T>::type*>(x + si);
#pragma unroll
    for (int j = 0; j < 8; ++j) c[j] = Cvt<T>::from_f(Cvt<T>::to_f(a[j]) + Cvt<T>::to_f(b[j]));
    *reinterpret_cast<typename V8<T>::type*>(y + o) = *reinterpret_cast<typename V8<T>::type*>(c);
  }
}

// dx[n, sy, sx, c] = sum_{Y in rows(sy), X in cols(sx)} dy[n, Y, X, c]
template <typename T>
__global__ __launch_bounds__(kBlock) void upsample_bwd(const T* __restrict__ dy, T* __restrict__ dx,
                                                       const int* __restrict__ ystart, const int* __restrict__ xstart,
                                                       int N, int h, int w, int H, int W, int C) {
  const int CV = C / 8;
  const long long total = (long long)N * h * w * CV;
  for (long long i = blockIdx.x * (long long)kBlock + threadIdx.x; i < total; i += (long long)gridDim.x * kBlock) {
    const int cv = (int)(i % CV);
    long long r = i / CV;
    const int sx = (int)(r % w); r /= w;
    const int sy = (int)(r % h);
    const int n = (int)(r / h);
    float acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = 0.f;
    for (int Y = ystart[sy]; Y < ystart[sy + 1]; ++Y)
      for (int X = xstart[sx]; X < xstart[sx + 1]; ++X) {
        T g[8];
        *reinterpret_cast<typename V8<T>::type*>(g) =
            *reinterpret_cast<const typename V8<T>::type*>(dy + (((long long)n * H + Y) * W + X) * C + cv * 8);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += Cvt<T>::to_f(g[j]);
      }
    T o[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = Cvt<T>::from_f(acc[j]);
    *reinterpret_cast<typename V8<T>::type*>(dx + i * 8) = *reinterpret_cast<typename V8<T>::type*>(o);
  }
}
}  // namespace

#define DISPATCH(dtype, K, ...) \
  do { if (dtype == 1) K<bf16_t><<<grid, kBlock, 0, stream>>>(__VA_ARGS__); else K<float><<<grid, kBlock, 0, stream>>>(__VA_ARGS__); } while (0)

// impl: 0 = the generic kernel, 1 = the 3x3 / stride-2 bf16 specialisation where it applies (identical
// outputs and argmax bytes: tests/test_kernels_gpu.py; ops.native.maxpool_fwd_raw picks by measurement)
MXR_API int mxr_maxpool_fwd(const void* x, void* y, uint8_t* arg, int N, int H, int W, int C, int Ho, int Wo, int k,
                            int s, int pt, int pl, int relu_in, int dtype, int impl, hipStream_t stream) {
  if (C % 8 || (long long)N * H * W * C >= 0x7fffffffLL) return -1;
  const int grid = mxr_grid((long long)N * Ho * Wo * (C / 8), kBlock, 16384);
  if (dtype == 1 && k == 3 && s == 2 && impl == 1)
    maxpool_fwd_k3s2<<<grid, kBlock, 0, stream>>>((const bf16_t*)x, (bf16_t*)y, arg, N, H, W, C, Ho, Wo, pt, pl,
                                                  relu_in);
  else if (dtype == 1)
    maxpool_fwd<bf16_t><<<grid, kBlock, 0, stream>>>((const bf16_t*)x, (bf16_t*)y, arg, N, H, W, C, Ho, Wo, k, s, pt, pl,
                                                     relu_in);
  else
    maxpool_fwd<float><<<grid, kBlock, 0, stream>>>((const float*)x, (float*)y, arg, N, H, W, C, Ho, Wo, k, s, pt, pl,
                                                    relu_in);
  return (int)hipGetLastError();
}

MXR_API int mxr_maxpool_bwd(const void* dy, const uint8_t* arg, void* dx, int N, int H, int W, int C, int Ho, int Wo,
                            int k, int s, int pt, int pl, int dtype, hipStream_t stream) {
  if (C % 8 || (long long)N * H * W * C >= 0x7fffffffLL) return -1;
  if (dtype == 1 && k == 3 && s == 2 && pt >= 0 && pt <= 1 && pl >= 0 && pl <= 1) {
    const int Hb = (H + pt + 1) / 2, Wb = (W + pl + 1) / 2;
    const int g2 = mxr_grid((long long)N * Hb * Wb * (C / 8), kBlock, 16384);
    maxpool_bwd_k3s2<<<g2, kBlock, 0, stream>>>((const bf16_t*)dy, arg, (bf16_t*)dx, N, H, W, C, Ho, Wo, pt, pl, Hb, Wb);
    return (int)hipGetLastError();
  }
  const int grid = mxr_grid((long long)N * H * W * (C / 8), kBlock, 16384);
  if (dtype == 1)
    maxpool_bwd<bf16_t><<<grid, kBlock, 0, stream>>>((const bf16_t*)dy, arg, (bf16_t*)dx, N, H, W, C, Ho, Wo, k, s, pt, pl);
  else
    maxpool_bwd<float><<<grid, kBlock, 0, stream>>>((const float*)dy, arg, (float*)dx, N, H, W, C, Ho, Wo, k, s, pt, pl);
  return (int)hipGetLastError();
}

MXR_API int mxr_upsample_add_fwd(const void* x, const void* lat, void* y, const int* iy_of, const int* ix_of, int N,
                                 int h, int w, int H, int W, int C, int dtype, hipStream_t stream) {
  if (C % 8) return -1;
  const int grid = mxr_grid((long long)N * H * W * (C / 8), kBlock, 16384);
  if (dtype == 1)
    upsample_add_fwd<bf16_t><<<grid, kBlock, 0, stream>>>((const bf16_t*)x, (const bf16_t*)lat, (bf16_t*)y, iy_of, ix_of,
                                                          N, h, w, H, W, C);
  else
    upsample_add_fwd<float><<<grid, kBlock, 0, stream>>>((const float*)x, (const float*)lat, (float*)y, iy_of, ix_of, N,
                                                         h, w, H, W, C);
  return (int)hipGetLastError();
}

MXR_API int mxr_upsample_bwd(const void* dy, void* dx, const int* ystart, const int* xstart, int N, int h, int w, int H,
                             int W, int C, int dtype, hipStream_t stream) {
  if (C % 8) return -1;
  const int grid = mxr_grid((long long)N * h * w * (C / 8), kBlock, 16384);
  if (dtype == 1)
    upsample_bwd<bf16_t><<<grid, kBlock, 0, stream>>>((const bf16_t*)dy, (bf16_t*)dx, ystart, xstart, N, h, w, H, W, C);
  else
    upsample_bwd<float><<<grid, kBlock, 0, stream>>>((const float*)dy, (float*)dx, ystart, xstart, N, h, w, H, W, C);
  return (int)hipGetLastError();
}
