// Prediction-graph kernels: RegressBoxes + ClipBoxes (fused), bitmask NMS.
//
// Spec: keras-retinanet layers RegressBoxes / ClipBoxes / FilterDetections used by retinanet_bbox
// (/root/reference/train.py:95,408).  Decode is the inverse corner-offset encoding
// (std 0.2); clip bounds x to [0, W], y to [0, H].  NMS follows tf.image.non_max_suppression:
// boxes pre-sorted by score, suppress when IoU > threshold, IoU WITHOUT the +1 convention, at most
// max_output boxes kept.  Mask kernel: one 64-bit word per (box, column-block of 64); the
// sequential keep scan runs in a single workgroup on the device.
#include "common.h"

namespace {
constexpr int kBlock = 256;

__global__ __launch_bounds__(kBlock) void decode_clip_kernel(const float* __restrict__ anchors, const void* __restrict__ deltas,
                                                             int dtype, float* __restrict__ boxes, long long total, int A,
                                                             float std_, float H, float W) {
  for (long long i = blockIdx.x * (long long)kBlock + threadIdx.x; i < total; i += (long long)gridDim.x * kBlock) {
    const int a = (int)(i % A);
    const float4 an = reinterpret_cast<const float4*>(anchors)[a];
    float d[4];
    if (dtype == 1) {
      const bf16_t* dp = (const bf16_t*)deltas + i * 4;
#pragma unroll
      for (int j = 0; j < 4; ++j) d[j] = bf2f(dp[j]);
    } else {
      const float4 dd = reinterpret_cast<const float4*>(deltas)[i];
      d[0] = dd.x; d[1] = dd.y; d[2] = dd.z; d[3] = dd.w;
    }
    const float aw = an.z - an.x, ah = an.w - an.y;
    float4 b;
    b.x = fminf(fmaxf(an.x + d[0] * std_ * aw, 0.f), W);
    b.y = fminf(fmaxf(an.y + d[1] * std_ * ah, 0.f), H);
    b.z = fminf(fmaxf(an.z + d[2] * std_ * aw, 0.f), W);
    b.w = fminf(fmaxf(an.w + d[3] * std_ * ah, 0.f), H);
    reinterpret_cast<float4*>(boxes)[i] = b;
  }
}

__device__ __forceinline__ float iou_plain(const float4 a, const float4 b) {
  const float aa = fmaxf(a.z - a.x, 0.f) * fmaxf(a.w - a.y, 0.f);
  const float ab = fmaxf(b.z - b.x, 0.f) * fmaxf(b.w - b.y, 0.f);
  const float iw = fmaxf(fminf(a.z, b.z) - fmaxf(a.x, b.x), 0.f);
  const float ih = fmaxf(fminf(a.w, b.w) - fmaxf(a.y, b.y), 0.f);
  const float inter = iw * ih;
  const float u = aa + ab - inter;
  return u > 0.f ? inter / u : 0.f;
}

// grid (colblocks, rowblocks), block 64: thread t handles row r = rb*64+t against column block cb.
__global__ __launch_bounds__(64) void nms_mask_kernel(const float* __restrict__ boxes, int n, float thr,
                                                      unsigned long long* __restrict__ mask, int words) {
  __shared__ float4 cb[64];
  const int rb = blockIdx.y, cbk = blockIdx.x;
  const int c = cbk * 64 + threadIdx.x;
  if (c < n) cb[threadIdx.x] = reinterpret_cast<const float4*>(boxes)[c];
  __syncthreads();
  const int r = rb * 64 + threadIdx.x;
  if (r >= n) return;
  const float4 me = reinterpret_cast<const float4*>(boxes)[r];
  unsigned long long bits = 0ull;
  const int ncol = min(64, n - cbk * 64);
  for (int j = 0; j < ncol; ++j) {
    const int cj = cbk * 64 + j;
    if (cj > r && iou_plain(me, cb[j]) > thr) bits |= (1ull << j);
  }
  mask[(long long)r * words + cbk] = bits;
}

// One workgroup: sequential greedy scan, removed bits in LDS. keep[i] = index, count in *nkeep.
__global__ __launch_bounds__(256) void nms_reduce_kernel(const unsigned long long* __restrict__ mask, int n, int words,
                                                         int max_out, int* __restrict__ keep, int* __restrict__ nkeep) {
  extern __shared__ unsigned long long removed[];
  for (int w = threadIdx.x; w < words; w += blockDim.x) removed[w] = 0ull;
  __syncthreads();
  int k = 0;
  for (int i = 0; i < n && k < max_out; ++i) {
    const bool sup = (removed[i >> 6] >> (i & 63)) & 1ull;
    __syncthreads();
    if (!sup) {
      if (threadIdx.x == 0) keep[k] = i;
      ++k;
      const unsigned long long* row = mask + (long long)i * words;
      for (int w = threadIdx.x; w < words; w += blockDim.x) removed[w] |= row[w];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) *nkeep = k;
}
__global__ void zero_count_kernel(int* c) {
  if (threadIdx.x == 0) c[0] = 0;
}
}  // namespace

MXR_API int mxr_decode_clip(const float* anchors, const void* deltas, int dtype, float* boxes, int B, int A, float std_,
                            float H, float W, hipStream_t stream) {
  const long long total = (long long)B * A;
  decode_clip_kernel<<<mxr_grid(total, kBlock, 8192), kBlock, 0, stream>>>(anchors, deltas, dtype, boxes, total, A, std_,
                                                                           H, W);
  return (int)hipGetLastError();
}

// boxes sorted by descending score. mask: n * ceil(n/64) u64 workspace.
MXR_API int mxr_nms(const float* boxes, int n, float thr, int max_out, unsigned long long* mask, int* keep, int* nkeep,
                    hipStream_t stream) {
  if (n <= 0) {
    zero_count_kernel<<<1, 64, 0, stream>>>(nkeep);
    return (int)hipGetLastError();
  }
  const int words = (n + 63) / 64;
  dim3 grid(words, words);
  nms_mask_kernel<<<grid, 64, 0, stream>>>(boxes, n, thr, mask, words);
  const size_t lds = (size_t)words * sizeof(unsigned long long);
  if (lds > 64 * 1024) return -2;
  nms_reduce_kernel<<<1, 256, lds, stream>>>(mask, n, words, max_out, keep, nkeep);
  return (int)hipGetLastError();
}
