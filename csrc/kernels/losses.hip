// Fused sigmoid-focal and smooth-L1 losses: loss partial sums AND input gradients in one pass.
//
// Spec: keras-retinanet losses.focal(alpha=0.25, gamma=2) / smooth_l1(sigma=3) compiled at
// /root/reference/train.py:99-102.  Keras evaluates the focal weight on the
// sigmoid probability and the BCE on the probability clipped to [1e-7, 1-1e-7]; in logit space
// that is BCE(clamp(x, LOGIT_LO, LOGIT_HI)) with zero gradient outside the clamp.  Anchors with
// state -1 are dropped; both losses are divided by max(1, #positives of the local batch), read
// from device memory (written by the anchor-target kernel), so nothing syncs with the host.
//
// The classification tensor is B x 200,700 x 80 (16M logits/image) -> memory-bound: every thread
// moves 16 B per load/store (8 bf16 or 4 f32), one read of the logits and one write of dlogits.
#include "common.h"
#include "focal_common.h"

namespace {

constexpr int kBlock = 256;

template <typename T, int V>
struct Vec;
template <> struct Vec<bf16_t, 8> { typedef uint4 type; };
template <> struct Vec<float, 4> { typedef float4 type; };

// logits/dlogits: [rows, C] row-major; state/label: [rows].
template <typename T, int V>
__global__ __launch_bounds__(kBlock) void focal_kernel(const T* __restrict__ logits, const int8_t* __restrict__ state,
                                                       const int32_t* __restrict__ label, const int* __restrict__ npos,
                                                       T* __restrict__ dlogits, float* __restrict__ partials,
                                                       long long nvec, int C, float alpha, float gamma, float lo,
                                                       float hi, int grp, int ld) {
  __shared__ float red[16];
  const float inv = 1.0f / fmaxf(1.0f, (float)(*npos));
  const bool g2 = gamma == 2.0f;
  float acc = 0.f;
  typedef typename Vec<T, V>::type VT;
  const VT* in = reinterpret_cast<const VT*>(logits);
  VT* out = reinterpret_cast<VT*>(dlogits);
  for (long long i = blockIdx.x * (long long)kBlock + threadIdx.x; i < nvec; i += (long long)gridDim.x * kBlock) {
    const long long e0 = i * V;
    long long row;
    int c0;
    if (e0 < 0x7fffffffLL) {   // 32-bit division (64-bit integer division is emulated on CDNA)
      const int e = (int)e0, r = e / C;
      row = r;
      c0 = e - r * C;
    } else {
      row = e0 / C;
      c0 = (int)(e0 - row * C);
    }
    const int s = state[row];
    VT v = in[i];
    T xs[V];
    *reinterpret_cast<VT*>(xs) = v;
    T gs[V];
    if (s == -1) {
#pragma unroll
      for (int j = 0; j < V; ++j) gs[j] = Cvt<T>::from_f(0.f);
    } else {
      const int lab = (s == 1) ? label[row] : -1;
#pragma unroll
      for (int j = 0; j < V; ++j) {
        float l, g;
        focal_elem(Cvt<T>::to_f(xs[j]), (c0 + j) == lab, alpha, gamma, g2, lo, hi, l, g);
        acc += l;
        gs[j] = Cvt<T>::from_f(g * inv);
      }
    }
    if (ld > 0)   // padded gradient layout: rows grouped by grp (anchors per pixel), group stride ld
      *reinterpret_cast<VT*>(dlogits + (row / grp) * (long long)ld + (row % grp) * (long long)C + c0) =
          *reinterpret_cast<VT*>(gs);
    else
      out[i] = *reinterpret_cast<VT*>(gs);
  }
  const float bs = block_sum(acc, red);
  if (threadIdx.x == 0) partials[blockIdx.x] = bs;
}

// bf16 fast path (32-bit indexing, < 2^31 elements): U independent 16-B vectors in flight per thread
// per iteration -- the one-vector loop above leaves the kernel latency-bound at ~2.4 TB/s.
// CC / GG > 0: the class count C and the anchor group size compile-time constants (80 / 9 for COCO): the
// per-vector row / column and padded-row divisions become multiply-shifts instead of ~40-instruction
// integer divisions.
// G2: gamma == 2 -- focal_neg_g2_inr per logit (the clip bounds are asymmetric in fp32: -16.118 / 15.942).  (With a runtime gamma
// the compiler if-converts the __powf branch of focal_neg and evaluates it -- log, exp, frexp, ldexp, range
// reduction -- for every element: 4x the instructions.)
template <int U, int CC = 0, int GG = 0, bool G2 = false>
__global__ __launch_bounds__(kBlock) void focal_bf16_kernel(const bf16_t* __restrict__ logits,
                                                            const int8_t* __restrict__ state,
                                                            const int32_t* __restrict__ label,
                                                            const int* __restrict__ npos, bf16_t* __restrict__ dlogits,
                                                            float* __restrict__ partials, int nvec, int C_, float alpha,
                                                            float gamma, float lo, float hi, int grp_, int ld) {
  __shared__ float red[16];
  const int C = CC > 0 ? CC : C_;
  const int grp = GG > 0 ? GG : grp_;
  const float inv = 1.0f / fmaxf(1.0f, (float)(*npos));
  const bool g2 = G2 || gamma == 2.0f;
  const float e_lo = __expf(-fabsf(lo)), e_hi = __expf(-fabsf(hi));
  float acc = 0.f;
  const uint4* in = reinterpret_cast<const uint4*>(logits);
  const int stride = gridDim.x * kBlock;
  for (int base = blockIdx.x * kBlock + threadIdx.x; base < nvec; base += stride * U) {
    uint4 v[U];
    int row[U], c0[U], st[U], lab[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = base + u * stride;
      st[u] = -2;
      if (i < nvec) {
        const int e = i * 8;
        row[u] = e / C;
        c0[u] = e - row[u] * C;
        st[u] = state[row[u]];
        lab[u] = label[row[u]];
        v[u] = in[i];
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (st[u] == -2) continue;
      const bf16_t* xs = reinterpret_cast<const bf16_t*>(&v[u]);
      bf16_t gs[8];
      if (st[u] == -1) {
#pragma unroll
        for (int j = 0; j < 8; ++j) gs[j] = 0;
      } else {
        const int lb = st[u] == 1 ? lab[u] - c0[u] : -1;   // the positive class inside this vector, if any
        float gv[8];
        if constexpr (G2) {
          // every logit as a background class inside the clip range; a logit outside it (a confident
          // negative late in training) sends the vector down the exact path (focal_common.h)
          float x8[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) x8[j] = bf2f(xs[j]);
          acc += focal8_g2(x8, lb, alpha, gamma, lo, hi, e_lo, e_hi, inv, gv);
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            float l;
            focal_neg(bf2f(xs[j]), alpha, gamma, g2, lo, hi, e_lo, e_hi, l, gv[j]);
            acc += j == lb ? 0.f : l;
          }
          if (lb >= 0 && lb < 8) {                        // rare: one element takes the y = 1 branch
            float l, g;
            focal_elem(bf2f(xs[lb]), true, alpha, gamma, g2, lo, hi, l, g);
            acc += l;
#pragma unroll
            for (int j = 0; j < 8; ++j) gv[j] = j == lb ? g : gv[j];
          }
#pragma unroll
          for (int j = 0; j < 8; ++j) gv[j] *= inv;
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) gs[j] = f2bf(gv[j]);
      }
      const int o = ld > 0 ? (row[u] / grp) * ld + (row[u] % grp) * C + c0[u] : (base + u * stride) * 8;
      *reinterpret_cast<uint4*>(dlogits + o) = *reinterpret_cast<const uint4*>(gs);
    }
  }
  const float bs = block_sum(acc, red);
  if (threadIdx.x == 0) partials[blockIdx.x] = bs;
}

// Scalar fallback for C not divisible by the vector width.
template <typename T>
__global__ __launch_bounds__(kBlock) void focal_kernel_scalar(const T* __restrict__ logits, const int8_t* __restrict__ state,
                                                              const int32_t* __restrict__ label, const int* __restrict__ npos,
                                                              T* __restrict__ dlogits, float* __restrict__ partials,
                                                              long long n, int C, float alpha, float gamma, float lo, float hi) {
  __shared__ float red[16];
  const float inv = 1.0f / fmaxf(1.0f, (float)(*npos));
  const bool g2 = gamma == 2.0f;
  float acc = 0.f;
  for (long long i = blockIdx.x * (long long)kBlock + threadIdx.x; i < n; i += (long long)gridDim.x * kBlock) {
    const long long row = i / C;
    const int c = (int)(i - row * C);
    const int s = state[row];
    float g = 0.f;
    if (s != -1) {
      float l;
      focal_elem(Cvt<T>::to_f(logits[i]), s == 1 && label[row] == c, alpha, gamma, g2, lo, hi, l, g);
      acc += l;
    }
    dlogits[i] = Cvt<T>::from_f(g * inv);
  }
  const float bs = block_sum(acc, red);
  if (threadIdx.x == 0) partials[blockIdx.x] = bs;
}

// Deterministic final reduction: out[0] = sum(partials) / max(1, npos).
__global__ __launch_bounds__(256) void finalize_kernel(const float* __restrict__ partials, int n, const int* __restrict__ npos,
                                                       float* __restrict__ out) {
  __shared__ float red[16];
  float acc = 0.f;
  for (int i = threadIdx.x; i < n; i += blockDim.x) acc += partials[i];
  const float s = block_sum(acc, red);
  if (threadIdx.x == 0) out[0] = s / fmaxf(1.0f, (float)(*npos));
}

// Smooth-L1 over positive anchors. pred/dpred: [rows, 4] (T), target: [rows, 4] f32.
template <typename T>
__global__ __launch_bounds__(kBlock) void smooth_l1_kernel(const T* __restrict__ pred, const float* __restrict__ target,
                                                           const int8_t* __restrict__ state, const int* __restrict__ npos,
                                                           T* __restrict__ dpred, float* __restrict__ partials,
                                                           long long rows, float sigma2, int grp, int ld) {
  __shared__ float red[16];
  const float inv = 1.0f / fmaxf(1.0f, (float)(*npos));
  const float thr = 1.0f / sigma2;
  float acc = 0.f;
  for (long long r = blockIdx.x * (long long)kBlock + threadIdx.x; r < rows; r += (long long)gridDim.x * kBlock) {
    T g[4];
    if (state[r] == 1) {
      const float4 t = reinterpret_cast<const float4*>(target)[r];
      const float tt[4] = {t.x, t.y, t.z, t.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float d = Cvt<T>::to_f(pred[r * 4 + j]) - tt[j];
        const float ad = fabsf(d);
        float l, gr;
        if (ad < thr) {
          l = 0.5f * sigma2 * ad * ad;
          gr = sigma2 * d;
        } else {
          l = ad - 0.5f / sigma2;
          gr = d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f);
        }
        acc += l;
        g[j] = Cvt<T>::from_f(gr * inv);
      }
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) g[j] = Cvt<T>::from_f(0.f);
    }
    // grp / ld: the packed regression head's zero-padded [rows / grp][ld] gradient rows
    T* d = dpred + (ld > 0 ? (r / grp) * ld + (r % grp) * 4 : r * 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) d[j] = g[j];
  }
  const float bs = block_sum(acc, red);
  if (threadIdx.x == 0) partials[blockIdx.x] = bs;
}

constexpr int kLossGrid = 2048;

}  // namespace

// dtype: 0 = f32, 1 = bf16.  partials must hold kLossGrid floats; out one float.
MXR_API int mxr_focal_fwd_bwd(const void* logits, const int8_t* state, const int32_t* label, const int* npos,
                              void* dlogits, float* partials, float* out, long long rows, int C, float alpha,
                              float gamma, float lo, float hi, int dtype, int grp, int ld, hipStream_t stream) {
  const long long n = rows * (long long)C;
  // grp / ld: write dlogits into a padded [rows / grp][ld] layout (the packed head's 768-wide pixel rows)
  if (ld > 0 && (dtype != 1 || C % 8 || grp <= 0 || (long long)grp * C > ld || rows % grp)) return -1;
  const long long nout = ld > 0 ? rows / (grp > 0 ? grp : 1) * ld : n;
  if (dtype == 1 && C % 8 == 0 && n < 0x7fffffffLL && nout < 0x7fffffffLL) {
    if (C == 80 && (ld <= 0 || grp == 9) && gamma == 2.0f)
      focal_bf16_kernel<4, 80, 9, true><<<kLossGrid, kBlock, 0, stream>>>((const bf16_t*)logits, state, label, npos,
                                                                          (bf16_t*)dlogits, partials, (int)(n / 8), C,
                                                                          alpha, gamma, lo, hi, grp, ld);
    else if (C == 80 && (ld <= 0 || grp == 9))
      focal_bf16_kernel<4, 80, 9><<<kLossGrid, kBlock, 0, stream>>>((const bf16_t*)logits, state, label, npos,
                                                                    (bf16_t*)dlogits, partials, (int)(n / 8), C, alpha,
                                                                    gamma, lo, hi, grp, ld);
    else
      focal_bf16_kernel<4><<<kLossGrid, kBlock, 0, stream>>>((const bf16_t*)logits, state, label, npos,
                                                             (bf16_t*)dlogits, partials, (int)(n / 8), C, alpha, gamma,
                                                             lo, hi, grp, ld);
  } else if (dtype == 1 && C % 8 == 0) {
    const long long nvec = n / 8;
    focal_kernel<bf16_t, 8><<<kLossGrid, kBlock, 0, stream>>>((const bf16_t*)logits, state, label, npos,
                                                              (bf16_t*)dlogits, partials, nvec, C, alpha, gamma, lo, hi,
                                                              grp, ld);
  } else if (dtype == 0 && C % 4 == 0) {
    const long long nvec = n / 4;
    focal_kernel<float, 4><<<kLossGrid, kBlock, 0, stream>>>((const float*)logits, state, label, npos,
                                                             (float*)dlogits, partials, nvec, C, alpha, gamma, lo, hi,
                                                             0, 0);
  } else if (dtype == 1) {
    focal_kernel_scalar<bf16_t><<<kLossGrid, kBlock, 0, stream>>>((const bf16_t*)logits, state, label, npos,
                                                                  (bf16_t*)dlogits, partials, n, C, alpha, gamma, lo, hi);
  } else {
    focal_kernel_scalar<float><<<kLossGrid, kBlock, 0, stream>>>((const float*)logits, state, label, npos,
                                                                 (float*)dlogits, partials, n, C, alpha, gamma, lo, hi);
  }
  finalize_kernel<<<1, 256, 0, stream>>>(partials, kLossGrid, npos, out);
  return (int)hipGetLastError();
}

MXR_API int mxr_smooth_l1_fwd_bwd(const void* pred, const float* target, const int8_t* state, const int* npos,
                                  void* dpred, float* partials, float* out, long long rows, float sigma, int dtype,
                                  int grp, int ld, hipStream_t stream) {
  const float s2 = sigma * sigma;
  if (ld > 0 && (grp <= 0 || 4LL * grp > ld || rows % grp)) return -1;
  if (dtype == 1)
    smooth_l1_kernel<bf16_t><<<kLossGrid, kBlock, 0, stream>>>((const bf16_t*)pred, target, state, npos,
                                                               (bf16_t*)dpred, partials, rows, s2, grp, ld);
  else
    smooth_l1_kernel<float><<<kLossGrid, kBlock, 0, stream>>>((const float*)pred, target, state, npos,
                                                              (float*)dpred, partials, rows, s2, grp, ld);
  finalize_kernel<<<1, 256, 0, stream>>>(partials, kLossGrid, npos, out);
  return (int)hipGetLastError();
}

MXR_API int mxr_loss_grid() { return kLossGrid; }

// the fixed-order final reduction of n loss partials (the focal epilogue of conv_hx32.hip / conv_hx32_f8.hip)
void mxr_loss_finalize_launch(const float* partials, int n, const int* npos, float* out, hipStream_t stream) {
  finalize_kernel<<<1, 256, 0, stream>>>(partials, n, npos, out);
}
