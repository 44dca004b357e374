// Keras-Adam + clipnorm over the flat fp32 parameter/gradient buffers (multi-tensor, fused).
//
// Spec: keras.optimizers.adam(lr=1e-5, clipnorm=0.001) at /root/reference/train.py:104
// (SURVEY §2.8.7): global-norm clip, lr_t = lr*sqrt(1-b2^t)/(1-b1^t), eps OUTSIDE the bias
// correction.  Hyper-parameters and the step counter live in device memory, so the whole
// optimizer is graph-capturable and never syncs with the host:
//   hyper[0] = lr_t (written by the prologue), hyper[1] = lr, iteration counter int64.
// The same pass refreshes the bf16 "compute" weights (W * frozen-BN scale) the forward reads.
#include "common.h"

namespace {

struct Chunk {
  long long start;   // flat element offset
  int len;           // elements in this chunk (multiple of 4 except possibly the last of a segment)
  int seg;           // segment index
};
struct Seg {
  long long offset;     // flat offset of the segment
  long long scale_off;  // offset into the scale vector (per output channel) or -1
  int row_len;          // elements per output channel
  int has_copy;         // write the bf16 compute copy
};

constexpr int kBlock = 256;

__global__ void adam_prologue(float* hyper, long long* iter, float b1, float b2) {
  const long long t = *iter + 1;
  const float lr = hyper[1];
  hyper[0] = lr * sqrtf(1.f - powf(b2, (float)t)) / (1.f - powf(b1, (float)t));
  *iter = t;
}

__global__ __launch_bounds__(kBlock) void adam_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                      float* __restrict__ m, float* __restrict__ v,
                                                      bf16_t* __restrict__ wcopy, const float* __restrict__ scales,
                                                      const Chunk* __restrict__ chunks, const Seg* __restrict__ segs,
                                                      const float* __restrict__ grad_scale,
                                                      const float* __restrict__ hyper, float b1, float b2, float eps) {
  const Chunk c = chunks[blockIdx.x];
  const Seg s = segs[c.seg];
  const float gs = *grad_scale;
  const float lr_t = hyper[0];
  const long long base = c.start;
  // chunk starts are 4-aligned (segments are 64-aligned, chunk length multiple of 4)
  const int nv = c.len >> 2;
  for (int i = threadIdx.x; i < nv; i += kBlock) {
    const long long e = base + 4LL * i;
    float4 pp = *reinterpret_cast<const float4*>(p + e);
    const float4 gg = *reinterpret_cast<const float4*>(g + e);
    float4 mm = *reinterpret_cast<const float4*>(m + e);
    float4 vv = *reinterpret_cast<const float4*>(v + e);
    float* pa = &pp.x; const float* ga = &gg.x; float* ma = &mm.x; float* va = &vv.x;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float gj = ga[j] * gs;
      ma[j] = b1 * ma[j] + (1.f - b1) * gj;
      va[j] = b2 * va[j] + (1.f - b2) * gj * gj;
      pa[j] -= lr_t * ma[j] / (sqrtf(va[j]) + eps);
    }
    *reinterpret_cast<float4*>(p + e) = pp;
    *reinterpret_cast<float4*>(m + e) = mm;
    *reinterpret_cast<float4*>(v + e) = vv;
    if (s.has_copy) {
      const long long le = e - s.offset;
      ushort4 w;
      unsigned short* wa = &w.x;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float sc = 1.f;
        if (s.scale_off >= 0) sc = scales[s.scale_off + (le + j) / s.row_len];
        wa[j] = f2bf(pa[j] * sc);
      }
      *reinterpret_cast<ushort4*>(wcopy + e) = w;
    }
  }
  // scalar tail (segment lengths that are not multiples of 4)
  for (int i = (nv << 2) + threadIdx.x; i < c.len; i += kBlock) {
    const long long e = base + i;
    const float gj = g[e] * gs;
    const float mj = b1 * m[e] + (1.f - b1) * gj;
    const float vj = b2 * v[e] + (1.f - b2) * gj * gj;
    const float pj = p[e] - lr_t * mj / (sqrtf(vj) + eps);
    m[e] = mj; v[e] = vj; p[e] = pj;
    if (s.has_copy) {
      float sc = 1.f;
      if (s.scale_off >= 0) sc = scales[s.scale_off + (e - s.offset) / s.row_len];
      wcopy[e] = f2bf(pj * sc);
    }
  }
}

// Refresh only the bf16 compute copy (after loading weights / broadcast).
__global__ __launch_bounds__(kBlock) void copy_kernel(const float* __restrict__ p, bf16_t* __restrict__ wcopy,
                                                      const float* __restrict__ scales, const Chunk* __restrict__ chunks,
                                                      const Seg* __restrict__ segs) {
  const Chunk c = chunks[blockIdx.x];
  const Seg s = segs[c.seg];
  if (!s.has_copy) return;
  for (int i = threadIdx.x; i < c.len; i += kBlock) {
    const long long e = c.start + i;
    float sc = 1.f;
    if (s.scale_off >= 0) sc = scales[s.scale_off + (e - s.offset) / s.row_len];
    wcopy[e] = f2bf(p[e] * sc);
  }
}

constexpr int kNormGrid = 1024;

__global__ __launch_bounds__(kBlock) void sumsq_kernel(const float* __restrict__ g, long long n, float* __restrict__ partials) {
  __shared__ float red[16];
  float acc = 0.f;
  const long long nv = n >> 2;
  const float4* g4 = reinterpret_cast<const float4*>(g);
  for (long long i = blockIdx.x * (long long)kBlock + threadIdx.x; i < nv; i += (long long)gridDim.x * kBlock) {
    const float4 x = g4[i];
    acc += x.x * x.x + x.y * x.y + x.z * x.z + x.w * x.w;
  }
  for (long long i = (nv << 2) + blockIdx.x * (long long)kBlock + threadIdx.x; i < n; i += (long long)gridDim.x * kBlock)
    acc += g[i] * g[i];
  const float s = block_sum(acc, red);
  if (threadIdx.x == 0) partials[blockIdx.x] = s;
}

// out[0] = norm = sqrt(sum) * norm_mul ; out[1] = clip factor * scale_mul (the Adam grad scale)
__global__ __launch_bounds__(256) void norm_finalize(const float* __restrict__ partials, int n, float norm_mul,
                                                     float clipnorm, float scale_mul, float* __restrict__ out) {
  __shared__ float red[16];
  float acc = 0.f;
  for (int i = threadIdx.x; i < n; i += blockDim.x) acc += partials[i];
  const float s = block_sum(acc, red);
  if (threadIdx.x == 0) {
    const float norm = sqrtf(s) * norm_mul;
    float f = 1.f;
    if (clipnorm > 0.f && norm >= clipnorm) f = clipnorm / norm;
    out[0] = norm;
    out[1] = f * scale_mul;
  }
}

__global__ __launch_bounds__(kBlock) void scale_kernel(float* __restrict__ g, long long n, const float* __restrict__ s) {
  const float f = *s;
  const long long nv = n >> 2;
  float4* g4 = reinterpret_cast<float4*>(g);
  for (long long i = blockIdx.x * (long long)kBlock + threadIdx.x; i < nv; i += (long long)gridDim.x * kBlock) {
    float4 x = g4[i];
    x.x *= f; x.y *= f; x.z *= f; x.w *= f;
    g4[i] = x;
  }
  for (long long i = (nv << 2) + blockIdx.x * (long long)kBlock + threadIdx.x; i < n; i += (long long)gridDim.x * kBlock)
    g[i] *= f;
}

}  // namespace

MXR_API int mxr_chunk_struct_sizes(int* out) {
  out[0] = sizeof(Chunk);
  out[1] = sizeof(Seg);
  return 0;
}

MXR_API int mxr_adam_step(float* p, const float* g, float* m, float* v, void* wcopy, const float* scales,
                          const void* chunks, int nchunks, const void* segs, const float* grad_scale, float* hyper,
                          long long* iter, float b1, float b2, float eps, hipStream_t stream) {
  adam_prologue<<<1, 1, 0, stream>>>(hyper, iter, b1, b2);
  adam_kernel<<<nchunks, kBlock, 0, stream>>>(p, g, m, v, (bf16_t*)wcopy, scales, (const Chunk*)chunks,
                                              (const Seg*)segs, grad_scale, hyper, b1, b2, eps);
  return (int)hipGetLastError();
}

MXR_API int mxr_refresh_copy(const float* p, void* wcopy, const float* scales, const void* chunks, int nchunks,
                             const void* segs, hipStream_t stream) {
  copy_kernel<<<nchunks, kBlock, 0, stream>>>(p, (bf16_t*)wcopy, scales, (const Chunk*)chunks, (const Seg*)segs);
  return (int)hipGetLastError();
}

// out: 2 floats (norm, grad scale). partials: kNormGrid floats.
MXR_API int mxr_grad_norm_clip(const float* g, long long n, float* partials, float norm_mul, float clipnorm,
                               float scale_mul, float* out, hipStream_t stream) {
  sumsq_kernel<<<kNormGrid, kBlock, 0, stream>>>(g, n, partials);
  norm_finalize<<<1, 256, 0, stream>>>(partials, kNormGrid, norm_mul, clipnorm, scale_mul, out);
  return (int)hipGetLastError();
}

MXR_API int mxr_scale_inplace(float* g, long long n, const float* s, hipStream_t stream) {
  scale_kernel<<<mxr_grid(n / 4 + 1, kBlock, 4096), kBlock, 0, stream>>>(g, n, s);
  return (int)hipGetLastError();
}

MXR_API int mxr_norm_grid() { return kNormGrid; }
