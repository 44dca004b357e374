// Batched FilterDetections on the device: score threshold + per-class greedy NMS for a whole batch in
// two launches, with no per-class host round trip.
//
// Spec: keras-retinanet FilterDetections (class_specific_filter, nms) inside retinanet_bbox
// (/root/reference/train.py:95,408 and the evaluation callbacks at :133-142):
// per image and class, keep the anchors whose sigmoid score exceeds score_threshold, run
// tf.image.non_max_suppression (boxes in descending score order, suppress IoU > threshold, IoU without
// the +1 convention, at most max_detections kept), then keep the top max_detections over all classes.
//
// * select: one pass over the (B, A, C) logits, 8 classes per 16-B load; a passing (image, class) element
//   appends its sort key (score bits << 32 | ~anchor: descending score, ascending anchor on ties, the
//   stable order of the torch oracle) to that segment's candidate list (capacity cap; the count keeps
//   counting past it so the host can see an overflow);
// * nms: one 256-thread workgroup per (image, class) segment: bitonic sort of the keys in LDS, then a
//   greedy scan in chunks of 64 candidates -- boxes decoded + clipped on the fly from the anchors and the
//   regression deltas (only candidates are ever decoded); each chunk is tested against the boxes kept
//   so far by all four waves, the intra-chunk suppression is a 64 x 64 bit matrix, and one lane walks the
//   64 bits in score order.  A segment whose count exceeded the capacity is re-run by the host exactly
//   (its full candidate list sorted on the device and fed through the same kernel, sorted-input mode).
#include "common.h"

// decode, IoU and sigmoid follow the oracle's operation order with IEEE rounding and no FMA contraction,
// so that NMS decisions on near-ties match the torch oracle (ops/boxes.py)
#pragma clang fp contract(off)

namespace {

constexpr int FD_BLOCK = 256;
constexpr int FD_CAP_MAX = 8192;     // keys per segment held in LDS (64 KiB)
constexpr int FD_MAXDET = 512;

__device__ __forceinline__ float fd_iou(const float4 a, const float4 b) {
  const float aa = fmaxf(a.z - a.x, 0.f) * fmaxf(a.w - a.y, 0.f);
  const float ab = fmaxf(b.z - b.x, 0.f) * fmaxf(b.w - b.y, 0.f);
  const float iw = fmaxf(fminf(a.z, b.z) - fmaxf(a.x, b.x), 0.f);
  const float ih = fmaxf(fminf(a.w, b.w) - fmaxf(a.y, b.y), 0.f);
  const float inter = iw * ih;
  const float u = aa + ab - inter;
  return u > 0.f ? __fdiv_rn(inter, u) : 0.f;
}

__device__ __forceinline__ float fd_sigmoid(float x) { return __fdiv_rn(1.f, 1.f + expf(-x)); }

// scores in (0, 1): the float bits order like the values
__device__ __forceinline__ unsigned long long fd_key(float p, int a) {
  return ((unsigned long long)__float_as_uint(p) << 32) | (unsigned long long)(0xffffffffu - (unsigned)a);
}

template <typename T>
__global__ __launch_bounds__(FD_BLOCK) void filter_select_kernel(const T* __restrict__ cls, long long nvec,
                                                                  int C, int A, float thr, int* __restrict__ cnt,
                                                                  unsigned long long* __restrict__ cand, int cap) {
  const int vpr = C >> 3;   // 8-class groups per anchor row
  for (long long v = blockIdx.x * (long long)FD_BLOCK + threadIdx.x; v < nvec; v += (long long)gridDim.x * FD_BLOCK) {
    float xs[8];
    if constexpr (sizeof(T) == 2) {
      const uint4 raw = reinterpret_cast<const uint4*>(cls)[v];
      const uint32_t w[4] = {raw.x, raw.y, raw.z, raw.w};
#pragma unroll
      for (int q = 0; q < 8; ++q) xs[q] = bf2f((bf16_t)((w[q >> 1] >> (16 * (q & 1))) & 0xffff));
    } else {
      const float4 r0 = reinterpret_cast<const float4*>(cls)[2 * v], r1 = reinterpret_cast<const float4*>(cls)[2 * v + 1];
      xs[0] = r0.x; xs[1] = r0.y; xs[2] = r0.z; xs[3] = r0.w; xs[4] = r1.x; xs[5] = r1.y; xs[6] = r1.z; xs[7] = r1.w;
    }
    const long long row = v / vpr;               // = b * A + a
    const int c0 = (int)(v - row * vpr) * 8;
    const int b = (int)(row / A), a = (int)(row - (long long)b * A);
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const float x = xs[q];
      const float p = fd_sigmoid(x);
      if (p > thr) {
        const int seg = b * C + c0 + q;
        const int slot = atomicAdd(cnt + seg, 1);
        if (slot < cap) cand[(long long)seg * cap + slot] = fd_key(p, a);
      }
    }
  }
}

// sorted == 0: keys = cand + seg * cap (count cnt[seg], sorted here); sorted == 1: keys already sorted
// descending, n = cnt[0], result written to segment seg_out.
__global__ __launch_bounds__(FD_BLOCK) void filter_nms_kernel(
    const unsigned long long* __restrict__ cand, const int* __restrict__ cnt, int cap, int sorted, int seg_out,
    const float* __restrict__ anchors, const void* __restrict__ deltas, int ddtype, int A, int C, float H, float W,
    float box_std, float nms_thr, int max_det, float* __restrict__ out_score, float* __restrict__ out_box,
    int* __restrict__ out_cnt, int* __restrict__ overflow) {
  __shared__ unsigned long long keys[FD_CAP_MAX];
  __shared__ float4 kept[FD_MAXDET];
  __shared__ float4 cbox[64];
  __shared__ float cscore[64];
  __shared__ unsigned long long rowbits[64];
  __shared__ unsigned long long supbits[4];
  __shared__ int s_kept;
  const int seg = sorted ? seg_out : blockIdx.x;
  const int b = seg / C;
  const int tid = threadIdx.x;
  int n;
  const unsigned long long* src;
  if (sorted) {
    n = cnt[0];
    src = cand;
  } else {
    const int c = cnt[seg];
    if (c > cap) {           // exact re-run by the host
      if (tid == 0) {
        overflow[seg] = 1;
        out_cnt[seg] = 0;
      }
      return;
    }
    n = c;
    src = cand + (long long)seg * cap;
    // bitonic sort (descending) of the n keys, padded with 0 to a power of two
    int np = 1;
    while (np < n) np <<= 1;
    for (int i = tid; i < np; i += FD_BLOCK) keys[i] = i < n ? src[i] : 0ull;
    __syncthreads();
    for (int k = 2; k <= np; k <<= 1) {
      for (int j = k >> 1; j > 0; j >>= 1) {
        for (int i = tid; i < np; i += FD_BLOCK) {
          const int l = i ^ j;
          if (l > i) {
            const unsigned long long x = keys[i], y = keys[l];
            const bool desc = (i & k) == 0;
            if (desc ? (x < y) : (x > y)) {
              keys[i] = y;
              keys[l] = x;
            }
          }
        }
        __syncthreads();
      }
    }
  }
  if (tid == 0) s_kept = 0;
  __syncthreads();
  const int lane = tid & 63, part = tid >> 6;
  for (int s = 0; s < n; s += 64) {
    if (s_kept >= max_det) break;
    // decode + clip the chunk's boxes (RegressBoxes + ClipBoxes)
    if (tid < 64) {
      float4 bx = make_float4(0.f, 0.f, 0.f, 0.f);
      float sc = -1.f;
      if (s + tid < n) {
        const unsigned long long key = sorted ? src[s + tid] : keys[s + tid];
        const int a = (int)(0xffffffffu - (unsigned)(key & 0xffffffffull));
        sc = __uint_as_float((unsigned)(key >> 32));
        const float4 an = reinterpret_cast<const float4*>(anchors)[a];
        const long long di = ((long long)b * A + a) * 4;
        float d[4];
        if (ddtype == 1) {
#pragma unroll
          for (int j = 0; j < 4; ++j) d[j] = bf2f(((const bf16_t*)deltas)[di + j]);
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) d[j] = ((const float*)deltas)[di + j];
        }
        const float aw = an.z - an.x, ah = an.w - an.y;
        bx.x = fminf(fmaxf(an.x + d[0] * box_std * aw, 0.f), W);
        bx.y = fminf(fmaxf(an.y + d[1] * box_std * ah, 0.f), H);
        bx.z = fminf(fmaxf(an.z + d[2] * box_std * aw, 0.f), W);
        bx.w = fminf(fmaxf(an.w + d[3] * box_std * ah, 0.f), H);
      }
      cbox[tid] = bx;
      cscore[tid] = sc;
    }
    if (tid < 4) supbits[tid] = 0ull;
    __syncthreads();
    const int nk = s_kept;
    const int nc = min(64, n - s);
    // suppression by the boxes kept so far: wave `part` tests kept boxes part, part + 4, ...
    {
      bool sup = false;
      if (lane < nc)
        for (int j = part; j < nk && !sup; j += 4) sup = fd_iou(cbox[lane], kept[j]) > nms_thr;
      const unsigned long long m = __ballot(sup);
      if (lane == 0) supbits[part] = m;
      // intra-chunk pairs: wave `part` builds rows lane for columns in its 16-wide slice, merged below
      unsigned long long bits = 0ull;
      if (lane < nc)
        for (int j = part * 16; j < part * 16 + 16; ++j)
          if (j > lane && j < nc && fd_iou(cbox[lane], cbox[j]) > nms_thr) bits |= 1ull << j;
      if (part == 0) rowbits[lane] = 0ull;
      __syncthreads();
      if (bits) atomicOr(&rowbits[lane], bits);
    }
    __syncthreads();
    if (tid == 0) {
      unsigned long long alive = ~(supbits[0] | supbits[1] | supbits[2] | supbits[3]);
      if (nc < 64) alive &= (1ull << nc) - 1ull;
      int k = nk;
      while (alive && k < max_det) {
        const int l = __ffsll((long long)alive) - 1;
        kept[k] = cbox[l];
        out_score[(long long)seg * max_det + k] = cscore[l];
        reinterpret_cast<float4*>(out_box)[(long long)seg * max_det + k] = cbox[l];
        ++k;
        alive &= ~rowbits[l];
        alive &= ~(1ull << l);
      }
      s_kept = k;
    }
    __syncthreads();
  }
  if (tid == 0) out_cnt[seg] = s_kept;
}

}  // namespace

// cls: (B, A, C) logits, dtype 1 = bf16, 0 = fp32 (C % 8 == 0); cnt: B * C ints (zeroed by the caller);
// cand: B * C * cap keys.
MXR_API int mxr_filter_select(const void* cls, int dtype, int B, int A, int C, float score_thr, int* cnt, void* cand,
                              int cap, hipStream_t stream) {
  if (C % 8 != 0 || cap <= 0 || cap > FD_CAP_MAX) return -1;
  const long long nvec = (long long)B * A * (C / 8);
  const int grid = mxr_grid(nvec, FD_BLOCK, 16384);
  if (dtype == 1)
    filter_select_kernel<bf16_t><<<grid, FD_BLOCK, 0, stream>>>((const bf16_t*)cls, nvec, C, A, score_thr, cnt,
                                                                (unsigned long long*)cand, cap);
  else
    filter_select_kernel<float><<<grid, FD_BLOCK, 0, stream>>>((const float*)cls, nvec, C, A, score_thr, cnt,
                                                               (unsigned long long*)cand, cap);
  return (int)hipGetLastError();
}

// sorted == 0: one workgroup per segment of `cand`; sorted == 1: one workgroup for the pre-sorted keys in
// `cand` (count in cnt[0]) writing segment seg_out.  Outputs: out_score (B * C * max_det), out_box
// (B * C * max_det * 4), out_cnt (B * C), overflow (B * C; set where a segment exceeded cap).
MXR_API int mxr_filter_nms(const void* cand, const int* cnt, int cap, int sorted, int seg_out, int nseg,
                           const float* anchors, const void* deltas, int ddtype, int A, int C, float H, float W,
                           float box_std, float nms_thr, int max_det, float* out_score, float* out_box, int* out_cnt,
                           int* overflow, hipStream_t stream) {
  if (max_det <= 0 || max_det > FD_MAXDET || cap > FD_CAP_MAX) return -1;
  filter_nms_kernel<<<sorted ? 1 : nseg, FD_BLOCK, 0, stream>>>(
      (const unsigned long long*)cand, cnt, cap, sorted, seg_out, anchors, deltas, ddtype, A, C, H, W, box_std,
      nms_thr, max_det, out_score, out_box, out_cnt, overflow);
  return (int)hipGetLastError();
}
