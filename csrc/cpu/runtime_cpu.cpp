// Host-side native runtime for batchai_retinanet_horovod_coco_amd (C ABI, loaded with ctypes).
//
// Replaces the native code the reference reaches through its dependencies:
//   N10 keras-retinanet compute_overlap.pyx (Cython)  -> mxr_cpu_compute_overlap (+1 IoU)
//   N11 OpenCV cv2.resize / cv2.warpAffine            -> mxr_cpu_resize_bilinear / mxr_cpu_warp_affine
//   N9  TF CPU non_max_suppression                     -> mxr_cpu_nms
//   N12 pycocotools maskApi bbox IoU (with iscrowd)    -> mxr_cpu_coco_iou
//       COCOeval greedy detection / gt matching        -> mxr_cpu_coco_match
//   N14 TensorBoard event-file CRC32C                  -> mxr_crc32c
// All loops are OpenMP-parallel over the outer dimension.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <numeric>
#include <vector>

#define API extern "C" __attribute__((visibility("default")))

// ------------------------------------------------------------------------------- IoU (+1)
API void mxr_cpu_compute_overlap(const double* boxes, long long n, const double* q, long long k, double* out) {
#pragma omp parallel for schedule(static)
  for (long long i = 0; i < n; ++i) {
    const double* b = boxes + 4 * i;
    for (long long j = 0; j < k; ++j) {
      const double* g = q + 4 * j;
      const double area_q = (g[2] - g[0] + 1) * (g[3] - g[1] + 1);
      double iw = std::min(b[2], g[2]) - std::max(b[0], g[0]) + 1;
      double r = 0.0;
      if (iw > 0) {
        double ih = std::min(b[3], g[3]) - std::max(b[1], g[1]) + 1;
        if (ih > 0) {
          const double ua = (b[2] - b[0] + 1) * (b[3] - b[1] + 1) + area_q - iw * ih;
          r = iw * ih / ua;
        }
      }
      out[i * k + j] = r;
    }
  }
}

// ------------------------------------------------------------------------------- resize
// cv2.resize(INTER_LINEAR) on float32 HWC images: half-pixel centres, edge clamping.
API void mxr_cpu_resize_bilinear(const float* src, int H, int W, int C, float* dst, int OH, int OW) {
  const double sy = (double)H / OH, sx = (double)W / OW;
  std::vector<int> x0(OW), x1(OW);
  std::vector<float> fx(OW);
  for (int x = 0; x < OW; ++x) {
    double f = (x + 0.5) * sx - 0.5;
    int i = (int)std::floor(f);
    double t = f - i;
    if (i < 0) { i = 0; t = 0; }
    if (i >= W - 1) { i = W - 1; t = 0; }
    x0[x] = i; x1[x] = std::min(i + 1, W - 1); fx[x] = (float)t;
  }
#pragma omp parallel for schedule(static)
  for (int y = 0; y < OH; ++y) {
    double f = (y + 0.5) * sy - 0.5;
    int i = (int)std::floor(f);
    double t = f - i;
    if (i < 0) { i = 0; t = 0; }
    if (i >= H - 1) { i = H - 1; t = 0; }
    const int i1 = std::min(i + 1, H - 1);
    const float ty = (float)t;
    const float* r0 = src + (long long)i * W * C;
    const float* r1 = src + (long long)i1 * W * C;
    float* d = dst + (long long)y * OW * C;
    for (int x = 0; x < OW; ++x) {
      const float tx = fx[x];
      const float* a = r0 + x0[x] * C; const float* b = r0 + x1[x] * C;
      const float* c = r1 + x0[x] * C; const float* e = r1 + x1[x] * C;
      for (int ch = 0; ch < C; ++ch) {
        const float top = a[ch] + (b[ch] - a[ch]) * tx;
        const float bot = c[ch] + (e[ch] - c[ch]) * tx;
        d[x * C + ch] = top + (bot - top) * ty;
      }
    }
  }
}

// ------------------------------------------------------------------------------- warpAffine
// dst(x, y) = src(M^-1 [x, y, 1]) with bilinear (interp=1) or nearest (interp=0) sampling.
// border: 0 constant(cval), 1 replicate ('nearest'), 2 reflect_101 ('reflect'), 3 wrap.
static inline int border_index(int i, int n, int mode, bool& outside) {
  outside = false;
  if (i >= 0 && i < n) return i;
  switch (mode) {
    case 1: return i < 0 ? 0 : n - 1;
    case 2: {
      if (n == 1) return 0;
      int p = 2 * (n - 1);
      i = ((i % p) + p) % p;
      return i < n ? i : p - i;
    }
    case 3: return ((i % n) + n) % n;
    default: outside = true; return 0;
  }
}

API void mxr_cpu_warp_affine(const float* src, int H, int W, int C, const double* M /* 2x3 src->dst */, float* dst,
                             int OH, int OW, int interp, int border, float cval) {
  // invert the 2x3 affine
  const double a = M[0], b = M[1], c = M[2], d = M[3], e = M[4], f = M[5];
  double det = a * e - b * d;
  det = det != 0 ? 1.0 / det : 0.0;
  const double ia = e * det, ib = -b * det, id = -d * det, ie = a * det;
  const double ic = -(ia * c + ib * f), iff = -(id * c + ie * f);
#pragma omp parallel for schedule(static)
  for (int y = 0; y < OH; ++y) {
    for (int x = 0; x < OW; ++x) {
      const double sxf = ia * x + ib * y + ic;
      const double syf = id * x + ie * y + iff;
      float* o = dst + ((long long)y * OW + x) * C;
      if (interp == 0) {
        bool out1, out2;
        const int xi = border_index((int)std::lround(sxf), W, border, out1);
        const int yi = border_index((int)std::lround(syf), H, border, out2);
        for (int ch = 0; ch < C; ++ch) o[ch] = (out1 || out2) ? cval : src[((long long)yi * W + xi) * C + ch];
        continue;
      }
      const int x0 = (int)std::floor(sxf), y0 = (int)std::floor(syf);
      const float tx = (float)(sxf - x0), ty = (float)(syf - y0);
      bool ox0, ox1, oy0, oy1;
      const int xa = border_index(x0, W, border, ox0), xb = border_index(x0 + 1, W, border, ox1);
      const int ya = border_index(y0, H, border, oy0), yb = border_index(y0 + 1, H, border, oy1);
      for (int ch = 0; ch < C; ++ch) {
        const float v00 = (ox0 || oy0) ? cval : src[((long long)ya * W + xa) * C + ch];
        const float v01 = (ox1 || oy0) ? cval : src[((long long)ya * W + xb) * C + ch];
        const float v10 = (ox0 || oy1) ? cval : src[((long long)yb * W + xa) * C + ch];
        const float v11 = (ox1 || oy1) ? cval : src[((long long)yb * W + xb) * C + ch];
        const float top = v00 + (v01 - v00) * tx, bot = v10 + (v11 - v10) * tx;
        o[ch] = top + (bot - top) * ty;
      }
    }
  }
}

// ------------------------------------------------------------------------------- NMS
// Greedy NMS, no +1 (tf.image.non_max_suppression). Returns number kept; keep[] = indices.
API int mxr_cpu_nms(const float* boxes, const float* scores, int n, float thr, int max_out, int* keep) {
  std::vector<int> order(n);
  std::iota(order.begin(), order.end(), 0);
  std::stable_sort(order.begin(), order.end(), [&](int i, int j) { return scores[i] > scores[j]; });
  std::vector<char> sup(n, 0);
  int k = 0;
  for (int oi = 0; oi < n && k < max_out; ++oi) {
    const int i = order[oi];
    if (sup[i]) continue;
    keep[k++] = i;
    const float* a = boxes + 4 * i;
    const float aa = std::max(a[2] - a[0], 0.f) * std::max(a[3] - a[1], 0.f);
    for (int oj = oi + 1; oj < n; ++oj) {
      const int j = order[oj];
      if (sup[j]) continue;
      const float* b = boxes + 4 * j;
      const float ab = std::max(b[2] - b[0], 0.f) * std::max(b[3] - b[1], 0.f);
      const float iw = std::max(std::min(a[2], b[2]) - std::max(a[0], b[0]), 0.f);
      const float ih = std::max(std::min(a[3], b[3]) - std::max(a[1], b[1]), 0.f);
      const float inter = iw * ih, u = aa + ab - inter;
      if (u > 0 && inter / u > thr) sup[j] = 1;
    }
  }
  return k;
}

// ------------------------------------------------------------------------------- COCO IoU
// pycocotools bbox IoU: boxes as [x, y, w, h]; for crowd gt the denominator is the det area.
API void mxr_cpu_coco_iou(const double* dt, int nd, const double* gt, int ng, const unsigned char* iscrowd,
                          double* out) {
#pragma omp parallel for schedule(static) if (nd * (long long)ng > 4096)
  for (int i = 0; i < nd; ++i) {
    const double* d = dt + 4 * i;
    const double da = d[2] * d[3];
    for (int j = 0; j < ng; ++j) {
      const double* g = gt + 4 * j;
      const double iw = std::min(d[0] + d[2], g[0] + g[2]) - std::max(d[0], g[0]);
      const double ih = std::min(d[1] + d[3], g[1] + g[3]) - std::max(d[1], g[1]);
      double r = 0.0;
      if (iw > 0 && ih > 0) {
        const double inter = iw * ih;
        const double u = iscrowd[j] ? da : da + g[2] * g[3] - inter;
        r = u > 0 ? inter / u : 0.0;
      }
      out[(long long)i * ng + j] = r;
    }
  }
}

// ------------------------------------------------------------------------------- COCO greedy matching
// One (image, category, area range) of the bbox evaluation, every IoU threshold at once.  Detections arrive in score
// order (the caller's stable sort, cut at maxDet); ``order`` lists the gt columns of ``iou`` (nd x ng, original gt
// order) with the area-range / ignore-flagged gts last.  A detection takes the best-IoU gt still free (crowd gts
// stay free) at or above the threshold; once it holds a regular gt it never moves to an ignored one.  ``match``
// (nt x nd) receives the position in ``order`` of the matched gt, or -1.
API void mxr_cpu_coco_match(const double* iou, int nd, int ng, const int* order, const unsigned char* gt_ig,
                            const unsigned char* crowd, const double* thr, int nt, int* match) {
  std::vector<unsigned char> taken((size_t)std::max(ng, 1));
  for (int t = 0; t < nt; ++t) {
    std::fill(taken.begin(), taken.end(), 0);
    const double lim = std::min(thr[t], 1.0 - 1e-10);
    int* mt = match + (long long)t * nd;
    for (int d = 0; d < nd; ++d) {
      const double* row = iou + (long long)d * ng;
      double best = lim;
      int m = -1;
      for (int g = 0; g < ng; ++g) {
        const int c = order[g];
        if (taken[g] && !crowd[c]) continue;
        if (m >= 0 && !gt_ig[m] && gt_ig[g]) break;     // regular gts come first: an ignored one never wins
        const double v = row[c];
        if (v < best) continue;
        best = v;
        m = g;
      }
      mt[d] = m;
      if (m >= 0) taken[m] = 1;
    }
  }
}

// ------------------------------------------------------------------------------- CRC32C
static uint32_t crc_table[256];
static bool crc_init = false;
static void init_crc() {
  for (uint32_t i = 0; i < 256; ++i) {
    uint32_t c = i;
    for (int k = 0; k < 8; ++k) c = (c & 1) ? (0x82F63B78u ^ (c >> 1)) : (c >> 1);
    crc_table[i] = c;
  }
  crc_init = true;
}

API uint32_t mxr_crc32c(const unsigned char* data, long long n, uint32_t crc) {
  if (!crc_init) init_crc();
  crc = ~crc;
  for (long long i = 0; i < n; ++i) crc = crc_table[(crc ^ data[i]) & 0xff] ^ (crc >> 8);
  return ~crc;
}
