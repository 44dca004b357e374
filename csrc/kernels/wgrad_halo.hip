// Halo-staged weight gradient of 3x3 / stride-1 / pad-1 convolutions (single level or the packed
// pyramid of the heads):  dW[co][ky][kx][ci] = sum_p dy[p][co] * x[p + (ky-1, kx-1)][ci].
//
// The implicit-GEMM wgrad (conv_wgrad_pipe.hip) stages an im2col tile per 32 pixels, i.e. every input
// pixel is fetched once per tap: ~64 MAC per staged byte, which leaves it L2-bound near 700 TF/s.
// Here a block owns a (128 co) x (9 taps x 64 ci) slice of dW and walks 2 x 64 output-pixel tiles:
// * per tile it stages dy [128 px][128 co] (256-B rows) and the input halo [4 x 66 px][64 ci] (128-B
//   rows) once -- all 9 taps read the same halo rows, shifted -- ~150 MAC per staged byte;
// * both MFMA operands come out of LDS with ds_read_b64_tr_b16 (A[co][p] from dy rows, B[p][ci] from
//   halo rows); 32-B chunks are XOR-swizzled by row bits so the 8 rows a 32-lane half reads fall on
//   distinct banks;
// * 8 waves = 2 co halves x 4 ci tiles, 4 x 9 = 36 accumulator tiles each; the next tile's dy / halo
//   chunks are fetched into registers while this tile runs on the MFMA;
// * blocks of one pixel split but different (co, ci) slices are consecutive after the XCD remap, so
//   they share one L2; each block writes an fp32 partial, reduced in fixed order (mxr_wgrad_reduce_launch).
// Tiles come from a host table {image, level, oy0, ox0}; each level has its own R x C box shape
// (R * C <= 128, picked on the host to waste the fewest slots: 167 columns -> 3 x 42, 84 -> 3 x 42, ...).
#include "conv_common.h"

typedef __attribute__((ext_vector_type(4))) short s16x4;

void mxr_wgrad_reduce_launch(const float* part, int splits, long long n, int K, const float* scale, float* out,
                             int accumulate, hipStream_t stream);

namespace {
constexpr int kTR = 2, kTC = 64, kHR = kTR + 2, kHC = kTC + 2;
constexpr int kNT = 512;
constexpr int kCoT = 128, kCiT = 64;
constexpr int kDyChunks = kTR * kTC * (kCoT / 8);   // 16-B chunks of the dy tile (16 per pixel)
constexpr int kXChunks = kHR * kHC * (kCiT / 8);    // 16-B chunks of the halo (8 per pixel)
constexpr int kDyPT = (kDyChunks + kNT - 1) / kNT;
constexpr int kXPT = (kXChunks + kNT - 1) / kNT;

struct HWLevels {
  int H[MXR_MAXLEV], W[MXR_MAXLEV], off[MXR_MAXLEV];
  int R[MXR_MAXLEV], C[MXR_MAXLEV];   // tile shape per level: R rows x C cols, R * C <= 128 slots
  int img;   // pixels per image (all levels)
};
constexpr int kHRows = kHR * kHC;       // halo rows staged per tile (max over tile shapes)

__device__ __forceinline__ int lv(const int* a, int l) {
  int v = a[0];
  v = l == 1 ? a[1] : v;
  v = l == 2 ? a[2] : v;
  v = l == 3 ? a[3] : v;
  v = l == 4 ? a[4] : v;
  return v;
}

__device__ __forceinline__ s16x4 tr_read(const char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(p));
}
// 128-B rows (4 chunks of 32 B): 2-bit swizzle; 256-B rows (8 chunks): 3-bit swizzle
__device__ __forceinline__ int swz2(int r) { return ((r >> 1) & 1) | (((r >> 3) & 1) << 1); }
__device__ __forceinline__ int swz3(int r) { return (r & 3) | (((r >> 3) & 1) << 2); }

struct HWRegs {
  uint4 d[kDyPT];
  uint4 h[kXPT];
};

// FC == kTC: every tile of the launch is a fixed 2 x 64 box (compile-time shifts); FC == 0: per-level boxes
template <int FC>
__device__ __forceinline__ void hw_load(HWRegs& r, const bf16_t* __restrict__ x, const bf16_t* __restrict__ dy, int ldy,
                                        int cin, int cout, int co0, int ci0, const int4 tl, const HWLevels& L) {
  const int b = tl.x, l = tl.y, oy0 = tl.z, ox0 = tl.w;
  const int H = lv(L.H, l), W = lv(L.W, l);
  const int R = FC ? kTR : lv(L.R, l), C = FC ? FC : lv(L.C, l);
  const size_t base = (size_t)b * L.img + lv(L.off, l);
#pragma unroll
  for (int j = 0; j < kDyPT; ++j) {
    const int i = threadIdx.x + kNT * j;
    const int p = i >> 4, c8 = i & 15;
    const int rr = p / C, cc = p - rr * C;
    const int oy = oy0 + rr, ox = ox0 + cc;
    uint4 v = make_uint4(0u, 0u, 0u, 0u);
    if (i < kDyChunks && rr < R && oy < H && ox < W && co0 + c8 * 8 < cout)
      v = *reinterpret_cast<const uint4*>(dy + (base + (size_t)oy * W + ox) * ldy + co0 + c8 * 8);
    r.d[j] = v;
  }
  const int HC = C + 2, nh = FC ? kHRows : (R + 2) * HC;
#pragma unroll
  for (int j = 0; j < kXPT; ++j) {
    const int i = threadIdx.x + kNT * j;
    const int hp = i >> 3, c8 = i & 7;
    const int hr = hp / HC, hc = hp - hr * HC;
    const int iy = oy0 - 1 + hr, ix = ox0 - 1 + hc;
    uint4 v = make_uint4(0u, 0u, 0u, 0u);
    if (i < kXChunks && hp < nh && iy >= 0 && iy < H && ix >= 0 && ix < W)
      v = *reinterpret_cast<const uint4*>(x + (base + (size_t)iy * W + ix) * cin + ci0 + c8 * 8);
    r.h[j] = v;
  }
}

template <int FC>
__global__ __launch_bounds__(kNT, 1) void wgrad_halo_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ dy,
                                                           int ldy, const int4* __restrict__ tiles, int ntiles,
                                                           int splits, int split_base, int n_co, int n_ci, int cin,
                                                           int cout, HWLevels L, float* __restrict__ part) {
  __shared__ __attribute__((aligned(16))) char xs[kHR * kHC * 128];
  __shared__ __attribute__((aligned(16))) char dys[kTR * kTC * 256];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int g = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
  const int cit = wv & 3, coh = wv >> 2;
  const int wid = xcd_remap(blockIdx.x, gridDim.x);
  const int ci_s = wid % n_ci;
  const int rest = wid / n_ci;
  const int co_s = rest % n_co;
  const int split = rest / n_co;
  const int co0 = co_s * kCoT, ci0 = ci_s * kCiT;
  const int t0 = (int)((long long)ntiles * split / splits), t1 = (int)((long long)ntiles * (split + 1) / splits);

  f32x4 acc[4][9];
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
#pragma unroll
    for (int j = 0; j < 9; ++j) acc[mt][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  HWRegs r;
  int cur_c = 1;
  if (t0 < t1) {
    const int4 tl = tiles[t0];
    hw_load<FC>(r, x, dy, ldy, cin, cout, co0, ci0, tl, L);
    cur_c = FC ? FC : lv(L.C, tl.y);
  }
  for (int t = t0; t < t1; ++t) {
    const int C = FC ? FC : cur_c, HC = C + 2;
    __syncthreads();   // the previous tile's LDS reads are done
#pragma unroll
    for (int j = 0; j < kDyPT; ++j) {
      const int i = tid + kNT * j;
      if (i < kDyChunks) {
        const int p = i >> 4, c8 = i & 15;
        *reinterpret_cast<uint4*>(dys + p * 256 + 32 * ((c8 >> 1) ^ swz3(p)) + 16 * (c8 & 1)) = r.d[j];
      }
    }
#pragma unroll
    for (int j = 0; j < kXPT; ++j) {
      const int i = tid + kNT * j;
      if (i < kXChunks) {
        const int hp = i >> 3, c8 = i & 7;
        *reinterpret_cast<uint4*>(xs + hp * 128 + 32 * ((c8 >> 1) ^ swz2(hp)) + 16 * (c8 & 1)) = r.h[j];
      }
    }
    __syncthreads();
    if (t + 1 < t1) {
      const int4 tl = tiles[t + 1];
      hw_load<FC>(r, x, dy, ldy, cin, cout, co0, ci0, tl, L);
      cur_c = FC ? FC : lv(L.C, tl.y);
    }
#pragma unroll 1
    for (int st = 0; st < kTR * kTC / 32; ++st) {
      const int p0 = 32 * st + 8 * g + q, p1 = p0 + 4;
      bf16x8 a[4];
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        const int m = 4 * coh + mt;
        const s16x4 lo = tr_read(dys + p0 * 256 + 32 * (m ^ swz3(p0)) + 8 * pp);
        const s16x4 hi = tr_read(dys + p1 * 256 + 32 * (m ^ swz3(p1)) + 8 * pp);
        a[mt] = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
      // slot -> (row, col) of this tile's R x C box; dead slots (zero dy rows) read any in-range halo row
      const int q0 = p0 / C, q1 = p1 / C;
      const int r0 = q0 * HC + (p0 - q0 * C), r1 = q1 * HC + (p1 - q1 * C);
#pragma unroll
      for (int j = 0; j < 9; ++j) {
        const int d = (j / 3) * HC + (j % 3);
        int h0 = r0 + d, h1 = r1 + d;
        if (!FC) {
          h0 = h0 < kHRows ? h0 : 0;
          h1 = h1 < kHRows ? h1 : 0;
        }
        const s16x4 lo = tr_read(xs + h0 * 128 + 32 * (cit ^ swz2(h0)) + 8 * pp);
        const s16x4 hi = tr_read(xs + h1 * 128 + 32 * (cit ^ swz2(h1)) + 8 * pp);
        const bf16x8 bb = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
#pragma unroll
        for (int mt = 0; mt < 4; ++mt)
          acc[mt][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[mt], bb, acc[mt][j], 0, 0, 0);
      }
    }
  }
  // partial [split][cout][9][cin]: C[row = co][col = ci]
  float* dst = part + (size_t)(split_base + split) * cout * 9 * cin;
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
#pragma unroll
    for (int j = 0; j < 9; ++j)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int co = co0 + 16 * (4 * coh + mt) + 4 * g + rr;
        if (co < cout) dst[((size_t)co * 9 + j) * cin + ci0 + 16 * cit + (lane & 15)] = acc[mt][j][rr];
      }
}
}  // namespace

// dw (cout, 3, 3, cin) fp32 (+)= scale * dW over the tiles (table of int4 {image, level, oy0, ox0});
// the first nwide tiles use the fixed 2 x 64 box (their levels must have C == 64), the rest their level's
// box.  ws >= splits * cout * 9 * cin floats.  cin % 64 == 0, ldy % 8 == 0, cout <= ldy.
MXR_API int mxr_wgrad_halo(const void* x, const void* dy, int ldy, const void* tiles, int ntiles, int nwide,
                           int splits, int nlev, const int* H, const int* W, const int* off, const int* R, const int* C,
                           int img, int cin, int cout, float* ws, const float* scale, float* dw, int accumulate,
                           hipStream_t stream) {
  if (cin % kCiT || ldy % 8 || cout > ldy || nlev < 1 || nlev > MXR_MAXLEV || ntiles <= 0 || splits <= 0 ||
      nwide < 0 || nwide > ntiles)
    return -1;
  HWLevels L;
  for (int l = 0; l < MXR_MAXLEV; ++l) {
    L.H[l] = l < nlev ? H[l] : 0;
    L.W[l] = l < nlev ? W[l] : 0;
    L.off[l] = l < nlev ? off[l] : 0;
    L.R[l] = l < nlev ? R[l] : 1;
    L.C[l] = l < nlev ? C[l] : 1;
    // every box and its halo must fit the staged tile: R * C <= 128 slots, (R + 2) * (C + 2) <= halo rows
    if (l < nlev && (W[l] <= 0 || R[l] < 1 || C[l] < 1 || C[l] > kTC || R[l] * C[l] > kTR * kTC ||
                     (R[l] + 2) * (C[l] + 2) > kHRows))
      return -1;
  }
  L.img = img;
  const int nnar = ntiles - nwide;
  // splits shared in proportion to the tiles; each class gets at least one if it has tiles
  int sw = nwide ? (int)(((long long)splits * nwide + ntiles / 2) / ntiles) : 0;
  if (nwide && sw < 1) sw = 1;
  if (nnar && sw > splits - 1) sw = splits - 1;
  const int sn = splits - sw;
  if ((nwide && sw < 1) || (nnar && sn < 1)) return -1;
  const int n_co = (cout + kCoT - 1) / kCoT, n_ci = cin / kCiT;
  if ((long long)splits * n_co * n_ci > 0x7fffffffLL) return -1;
  const int4* tb = (const int4*)tiles;
  if (nwide)
    wgrad_halo_kernel<kTC><<<sw * n_co * n_ci, kNT, 0, stream>>>((const bf16_t*)x, (const bf16_t*)dy, ldy, tb, nwide,
                                                                 sw, 0, n_co, n_ci, cin, cout, L, ws);
  if (nnar)
    wgrad_halo_kernel<0><<<sn * n_co * n_ci, kNT, 0, stream>>>((const bf16_t*)x, (const bf16_t*)dy, ldy, tb + nwide,
                                                               nnar, sn, sw, n_co, n_ci, cin, cout, L, ws);
  mxr_wgrad_reduce_launch(ws, splits, (long long)cout * 9 * cin, 9 * cin, scale, dw, accumulate, stream);
  return (int)hipGetLastError();
}
