// Weight gradient of the 64-channel 3x3 / stride-1 / pad-1 convs (res2 branch2b):
// dW[co][ky][kx][ci] = sum_p dy[p][co] * x[p + (ky-1, kx-1)][ci] over M = B*200*334 pixels.
//
// The generic wgrad kernels treat this as a K = 576 implicit GEMM whose pixel operand is gathered
// once per tap; at 64 channels that makes them load-bound (~250 TF/s).  Here the 9 taps share ONE
// staged input tile:
// * a block walks 2 x 64 output-pixel tiles persistently; per tile it stages the dy tile [128 px][64 co]
//   and the input halo [4 x 66 px][64 ci] in LDS (128-B rows, 32-B chunks XOR-swizzled by row bits
//   1 and 3 so the 8 rows a 32-lane half reads fall on distinct banks);
// * both MFMA operands come out of LDS with ds_read_b64_tr_b16: A[co][p] from dy rows, B[p][ci] for tap
//   (ky, kx) from the halo rows of pixels p shifted by (ky, kx) -- a tap is only a row offset;
// * the reduction runs over 32-pixel steps; 8 waves split the 64 x 576 gradient (ci tile x co half,
//   all 9 taps: 18 accumulator tiles each) so it lives in registers until the block writes its fp32
//   partial, which mxr_wgrad_reduce_launch sums (fixed order, BN scale folded);
// * the next tile's global chunks are loaded into registers while this tile runs on the MFMA.
#include "conv_common.h"

typedef __attribute__((ext_vector_type(4))) short s16x4;

void mxr_wgrad_reduce_launch(const float* part, int splits, long long n, int K, const float* scale, float* out,
                             int accumulate, hipStream_t stream);

namespace {
constexpr int kTR = 2, kTC = 64, kHR = kTR + 2, kHC = kTC + 2;
constexpr int kKW = 9 * 64;

__device__ __forceinline__ s16x4 tr_read(const char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(p));
}
__device__ __forceinline__ int swz(int r) { return ((r >> 1) & 1) | (((r >> 3) & 1) << 1); }

// 8 waves: wave w owns ci tile (w & 3) and co half (w >> 2) -> 2 co tiles x 9 taps = 18 accumulators,
// which leaves room to hold the NEXT tile's dy / halo chunks in registers while this tile is on the MFMA
// (the one-tile-at-a-time version waited on its global loads ~60 % of the time).
constexpr int kNT = 512;
constexpr int kDyChunks = kTR * kTC * 8;          // 16-B chunks of the dy tile
constexpr int kXChunks = kHR * kHC * 8;           // 16-B chunks of the input halo
constexpr int kDyPT = (kDyChunks + kNT - 1) / kNT;
constexpr int kXPT = (kXChunks + kNT - 1) / kNT;

struct W64Regs {
  uint4 d[kDyPT];
  uint4 h[kXPT];
};

__device__ __forceinline__ void w64_load(W64Regs& r, const bf16_t* __restrict__ x, const bf16_t* __restrict__ dy, int t,
                                         int H, int W, int tiles_x, int tiles_y) {
  int b = t;
  const int tx = b % tiles_x;
  b /= tiles_x;
  const int ty = b % tiles_y;
  const int n = b / tiles_y;
  const int oy0 = ty * kTR, ox0 = tx * kTC;
#pragma unroll
  for (int j = 0; j < kDyPT; ++j) {
    const int i = threadIdx.x + kNT * j;
    const int p = i >> 3, c8 = i & 7;
    const int oy = oy0 + (p >> 6), ox = ox0 + (p & 63);
    uint4 v = make_uint4(0u, 0u, 0u, 0u);
    if (i < kDyChunks && oy < H && ox < W)
      v = *reinterpret_cast<const uint4*>(dy + (((size_t)n * H + oy) * W + ox) * 64 + c8 * 8);
    r.d[j] = v;
  }
#pragma unroll
  for (int j = 0; j < kXPT; ++j) {
    const int i = threadIdx.x + kNT * j;
    const int hp = i >> 3, c8 = i & 7;
    const int hr = hp / kHC, hc = hp - hr * kHC;
    const int iy = oy0 - 1 + hr, ix = ox0 - 1 + hc;
    uint4 v = make_uint4(0u, 0u, 0u, 0u);
    if (i < kXChunks && iy >= 0 && iy < H && ix >= 0 && ix < W)
      v = *reinterpret_cast<const uint4*>(x + (((size_t)n * H + iy) * W + ix) * 64 + c8 * 8);
    r.h[j] = v;
  }
}

__global__ __launch_bounds__(kNT, 1) void wgrad3x3_c64_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ dy,
                                                             float* __restrict__ part, int H, int W, int tiles_x,
                                                             int tiles_y, int ntiles) {
  __shared__ __attribute__((aligned(16))) char xs[kHR * kHC * 128];
  __shared__ __attribute__((aligned(16))) char dys[kTR * kTC * 128];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int g = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
  const int cit = wv & 3, coh = wv >> 2;
  f32x4 acc[2][9];
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int j = 0; j < 9; ++j) acc[mt][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  W64Regs r;
  int t = blockIdx.x;
  if (t < ntiles) w64_load(r, x, dy, t, H, W, tiles_x, tiles_y);
  for (; t < ntiles; t += gridDim.x) {
    __syncthreads();   // the previous tile's LDS reads are done
#pragma unroll
    for (int j = 0; j < kDyPT; ++j) {
      const int i = tid + kNT * j;
      if (i < kDyChunks) {
        const int p = i >> 3, c8 = i & 7;
        *reinterpret_cast<uint4*>(dys + p * 128 + 32 * ((c8 >> 1) ^ swz(p)) + 16 * (c8 & 1)) = r.d[j];
      }
    }
#pragma unroll
    for (int j = 0; j < kXPT; ++j) {
      const int i = tid + kNT * j;
      if (i < kXChunks) {
        const int hp = i >> 3, c8 = i & 7;
        *reinterpret_cast<uint4*>(xs + hp * 128 + 32 * ((c8 >> 1) ^ swz(hp)) + 16 * (c8 & 1)) = r.h[j];
      }
    }
    __syncthreads();
    if (t + (int)gridDim.x < ntiles) w64_load(r, x, dy, t + gridDim.x, H, W, tiles_x, tiles_y);
#pragma unroll 2
    for (int st = 0; st < kTR * kTC / 32; ++st) {
      const int p0 = 32 * st + 8 * g + q, p1 = p0 + 4;
      bf16x8 a[2];
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) {
        const int m = 2 * coh + mt;
        const s16x4 lo = tr_read(dys + p0 * 128 + 32 * (m ^ swz(p0)) + 8 * pp);
        const s16x4 hi = tr_read(dys + p1 * 128 + 32 * (m ^ swz(p1)) + 8 * pp);
        a[mt] = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
      const int r0 = (p0 >> 6) * kHC + (p0 & 63), r1 = (p1 >> 6) * kHC + (p1 & 63);
#pragma unroll
      for (int j = 0; j < 9; ++j) {           // tap j = ky*3 + kx
        const int d = (j / 3) * kHC + (j % 3);
        const int h0 = r0 + d, h1 = r1 + d;
        const s16x4 lo = tr_read(xs + h0 * 128 + 32 * (cit ^ swz(h0)) + 8 * pp);
        const s16x4 hi = tr_read(xs + h1 * 128 + 32 * (cit ^ swz(h1)) + 8 * pp);
        const bf16x8 bb = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
#pragma unroll
        for (int mt = 0; mt < 2; ++mt)
          acc[mt][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[mt], bb, acc[mt][j], 0, 0, 0);
      }
    }
  }
  // C[row = co][col = ci]: col = lane & 15 of ci tile cit, rows 4g + r of co tile 2*coh + mt
  float* dst = part + (size_t)blockIdx.x * 64 * kKW;
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int j = 0; j < 9; ++j)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr)
        dst[(16 * (2 * coh + mt) + 4 * g + rr) * kKW + j * 64 + 16 * cit + (lane & 15)] = acc[mt][j][rr];
}
}  // namespace

static int wgrad3x3_c64_blocks(long long ntiles) { return (int)(ntiles < 256 ? ntiles : 256); }   // 1 per CU

// floats of workspace mxr_wgrad3x3_c64 needs (ops/native_conv.py mirrors the block count)
MXR_API long long mxr_wgrad3x3_c64_ws(int N, int H, int W) {
  const long long nt = (long long)N * ((H + kTR - 1) / kTR) * ((W + kTC - 1) / kTC);
  return (long long)wgrad3x3_c64_blocks(nt) * 64 * kKW;
}

// dw (64, 3, 3, 64) fp32 (+)= scale[co] * weight gradient; x, dy (N, H, W, 64) bf16 (stride 1, pad 1)
MXR_API int mxr_wgrad3x3_c64(const void* x, const void* dy, float* ws, const float* scale, float* dw, int N, int H,
                             int W, int accumulate, hipStream_t stream) {
  if (N <= 0 || H <= 0 || W <= 0) return -1;
  const int tiles_x = (W + kTC - 1) / kTC, tiles_y = (H + kTR - 1) / kTR;
  const long long ntiles = (long long)N * tiles_x * tiles_y;
  if (ntiles > 0x7fffffffLL || (long long)N * H * W * 64 >= 0x7fffffffLL * 4LL) return -1;
  const int nb = wgrad3x3_c64_blocks(ntiles);
  wgrad3x3_c64_kernel<<<nb, kNT, 0, stream>>>((const bf16_t*)x, (const bf16_t*)dy, ws, H, W, tiles_x, tiles_y,
                                              (int)ntiles);
  mxr_wgrad_reduce_launch(ws, nb, 64LL * kKW, kKW, scale, dw, accumulate, stream);
  return (int)hipGetLastError();
}
