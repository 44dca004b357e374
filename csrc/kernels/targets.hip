// Anchor-target assignment on the device (replaces the reference's CPU numpy + Cython path).
//
// Spec: keras-retinanet utils.anchors.anchor_targets_bbox + compute_overlap.pyx (entered at
// /root/reference/train.py:51,429):
//   IoU with the "+1 pixel" convention; argmax over gt (first max wins); positive if
//   IoU >= 0.5, ignore if 0.4 <= IoU < 0.5, negative below; anchors whose centre lies outside
//   the unpadded image (cx >= W or cy >= H) are ignored; regression = corner offsets / anchor
//   w,h / 0.2.  Images without boxes: every anchor negative (except outside ones).
// Output is compact: state int8 (-1/0/1), label int32, regression f32x4, plus the number of
// positives of the whole local batch (the focal / smooth-L1 normaliser) via one integer
// atomic per wave.  One block = 256 anchors of one image; gt boxes are staged through LDS.
#include "common.h"

namespace {
constexpr int kBlock = 256;
constexpr int kTile = 256;  // gt boxes per LDS tile

__global__ __launch_bounds__(kBlock) void anchor_targets_kernel(
    const float* __restrict__ anchors, const float* __restrict__ centers, int A, const float* __restrict__ gt, int G, const int* __restrict__ gt_count,
    const int* __restrict__ image_hw, int8_t* __restrict__ state, int32_t* __restrict__ label,
    float* __restrict__ reg, int* __restrict__ npos, float neg_thr, float pos_thr, float inv_std) {
  __shared__ float sg[kTile * 5];
  const int b = blockIdx.y;
  const int a = blockIdx.x * kBlock + threadIdx.x;
  const int cnt = min(gt_count[b], G);
  float ax1 = 0.f, ay1 = 0.f, ax2 = 0.f, ay2 = 0.f;
  if (a < A) {
    const float4 an = reinterpret_cast<const float4*>(anchors)[a];
    ax1 = an.x; ay1 = an.y; ax2 = an.z; ay2 = an.w;
  }
  const float area_a = (ax2 - ax1 + 1.f) * (ay2 - ay1 + 1.f);
  float best = -1.f;
  int arg = 0;
  const float* gb = gt + (long long)b * G * 5;
  for (int t0 = 0; t0 < cnt; t0 += kTile) {
    const int nt = min(kTile, cnt - t0);
    __syncthreads();
    for (int i = threadIdx.x; i < nt * 5; i += kBlock) sg[i] = gb[t0 * 5 + i];
    __syncthreads();
    for (int j = 0; j < nt; ++j) {
      const float gx1 = sg[j * 5 + 0], gy1 = sg[j * 5 + 1], gx2 = sg[j * 5 + 2], gy2 = sg[j * 5 + 3];
      const float iw = fminf(ax2, gx2) - fmaxf(ax1, gx1) + 1.f;
      const float ih = fminf(ay2, gy2) - fmaxf(ay1, gy1) + 1.f;
      float iou = 0.f;
      if (iw > 0.f && ih > 0.f) {
        const float inter = iw * ih;
        const float ua = area_a + (gx2 - gx1 + 1.f) * (gy2 - gy1 + 1.f) - inter;
        iou = inter / ua;
      }
      if (iou > best) { best = iou; arg = t0 + j; }
    }
  }
  int is_pos = 0;
  if (a < A) {
    const long long o = (long long)b * A + a;
    int st;
    float mx1, my1, mx2, my2;
    int lab = 0;
    if (cnt > 0) {
      st = best < neg_thr ? 0 : (best >= pos_thr ? 1 : -1);
      const float* g = gb + arg * 5;
      mx1 = g[0]; my1 = g[1]; mx2 = g[2]; my2 = g[3];
      lab = (int)g[4];
    } else {
      st = 0;
      mx1 = ax1; my1 = ay1; mx2 = ax2; my2 = ay2;
    }
    // centres pre-rounded DOWN from float64 on the host: same outside test as the fp64 reference
    const float cx = centers[2 * a], cy = centers[2 * a + 1];
    if (cx >= (float)image_hw[2 * b + 1] || cy >= (float)image_hw[2 * b]) st = -1;
    const float aw = ax2 - ax1, ah = ay2 - ay1;
    float4 r;
    r.x = (mx1 - ax1) / aw * inv_std;
    r.y = (my1 - ay1) / ah * inv_std;
    r.z = (mx2 - ax2) / aw * inv_std;
    r.w = (my2 - ay2) / ah * inv_std;
    reinterpret_cast<float4*>(reg)[o] = r;
    state[o] = (int8_t)st;
    label[o] = lab;
    is_pos = st == 1;
  }
  const int w = wave_sum_i(is_pos);
  if ((threadIdx.x & 63) == 0 && w) atomicAdd(npos, w);
}
__global__ void zero_count_kernel(int* c) {
  if (threadIdx.x == 0) c[0] = 0;
}
}  // namespace

// npos is zeroed here (a one-thread kernel on the same stream: a hipMemsetAsync is a runtime blit that
// measured 170-490 us of idle GPU in front of it at each step start) before the kernel accumulates into it.
MXR_API int mxr_anchor_targets(const float* anchors, const float* centers, int A, const float* gt, int B, int G, const int* gt_count,
                               const int* image_hw, int8_t* state, int32_t* label, float* reg, int* npos,
                               float neg_thr, float pos_thr, float box_std, hipStream_t stream) {
  zero_count_kernel<<<1, 64, 0, stream>>>(npos);
  dim3 grid((A + kBlock - 1) / kBlock, B);
  anchor_targets_kernel<<<grid, kBlock, 0, stream>>>(anchors, centers, A, gt, G, gt_count, image_hw, state, label, reg, npos,
                                                     neg_thr, pos_thr, 1.0f / box_std);
  return (int)hipGetLastError();
}
