// ResNet stem conv1: 7x7 / stride 2 / Cin 3 / Cout 64 on MFMA, with the frozen-BN shift and ReLU fused.
//
// Spec: keras-resnet `ZeroPadding2D(3)` -> `conv1` 7x7 s2 valid, no bias -> `bn_conv1` -> ReLU
// (K1 "conv1 M=266,800/img N=64 K=147").  Cin = 3 is too narrow for the implicit-GEMM
// kernels (K per tap must be a multiple of 64), and the library path costs ~1 ms/step at batch 16
// (conv + NCHW copy + bias + clamp passes).  This kernel is a direct conv:
//
// * block = 4 waves = a 4-row x 64-column output tile; the input patch it needs (13 x 134 pixels) is
//   staged once in LDS with the 3 channels padded to 4 (8 B per pixel);
// * GEMM view per wave: C[cout][pixel] = A[cout][k] * B[k][pixel], K = 7 ky-steps of 32 with
//   k = kx*4 + ci (kx < 8, ci < 4; kx = 7 and ci = 3 carry zero weights).  For one ky the 8 k's a lane
//   owns are pixel (2*ox + 2g .. 2*ox + 2g + 1) x 4 channels = 16 contiguous, aligned LDS bytes:
//   one ds_read_b128 per B fragment;
// * the weights (64 x 224 bf16, packed on the host side once per step) live in registers for the whole
//   block: 4 cout tiles x 7 k-steps of A fragments;
// * epilogue: + shift, ReLU, bf16; each lane owns 4 consecutive output channels of one pixel.
#include "common.h"

namespace {
typedef __attribute__((ext_vector_type(8))) short bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

constexpr int kTR = 4, kTC = 64;                   // output tile
constexpr int kPR = 2 * kTR + 5, kPC = 2 * kTC + 6; // input patch (rows, cols)
constexpr int kKS = 7;                             // k-steps (one per ky)
constexpr int kKP = kKS * 32;                      // packed K per output channel

constexpr int kWRow = kKP + 8;                     // LDS weight row (bf16): 464 B, conflict-free b128 reads
constexpr int kORow = 72;                          // epilogue tile row (bf16): 64 couts + 16 B
constexpr int kPPT = (kPR * kPC + 255) / 256;      // patch pixels per thread

// The patch as whole row segments: row r of tile t covers bytes [rowbase + ix0 * 6, + kPC * 6) of the 3-channel
// image, fetched as 4-B words (dword kRD * r + d = the word at a0(r) + d) -- 4.5x fewer global load
// instructions and ~3.5x fewer cache-line accesses than three 2-B loads per pixel (the per-pixel form cost ~0.1 ms
// of the 0.3 ms forward and of the weight gradient: profiles/r6_stem_patch_rows.txt).  Words outside the image
// row are not loaded (zero); stem_patch_from_rows unpacks them into the padded [r][c] x 4-channel patch.
constexpr int kRD = (kPC * 6 + 2 + 3) / 4;            // words per patch row (+ the 2-B misalignment)
// PR patch rows staged by NT threads: words / pixels per thread, staging bytes
template <int PR, int NT>
struct PRows {
  static constexpr int RW = (PR * kRD + NT - 1) / NT, PPT = (PR * kPC + NT - 1) / NT, RawB = PR * kRD * 4;
};
constexpr int kRW = PRows<kPR, 256>::RW;
constexpr int kRawB = PRows<kPR, 256>::RawB;

struct StemTile {
  int n, iy0, ix0;
};
__device__ __forceinline__ StemTile stem_tile(int t, int pt, int pl, int tiles_x, int tiles_y) {
  int b = t;
  const int tx = b % tiles_x;
  b /= tiles_x;
  const int ty = b % tiles_y;
  return {b / tiles_y, ty * kTR * 2 - pt, tx * kTC * 2 - pl};
}

// the PR x kPC patch with its top-left input pixel (iy0, ix0) of image n, as row words into rv
template <int PR, int NT, int RW>
__device__ __forceinline__ void stem_fetch_rows(uint32_t (&rv)[RW], const bf16_t* __restrict__ x, const StemTile T,
                                                int H, int W) {
  static_assert(RW == PRows<PR, NT>::RW, "words per thread");
  const uint32_t* xw = reinterpret_cast<const uint32_t*>(x);
#pragma unroll
  for (int j = 0; j < RW; ++j) {
    const int i = threadIdx.x + NT * j;
    const int r = i / kRD, d = i - r * kRD;
    const int iy = T.iy0 + r;
    uint32_t v = 0u;
    if (r < PR && iy >= 0 && iy < H) {
      const long long rowb = ((long long)T.n * H + iy) * W * 6;       // the image row's first byte
      const long long a0 = (rowb + (long long)T.ix0 * 6) >> 2;          // floor: the segment's first word
      const long long w = a0 + d;
      const long long lo = rowb + (long long)max(T.ix0, 0) * 6, hi = rowb + (long long)min(T.ix0 + kPC, W) * 6;
      // (a word straddling the row's first / last byte reads up to 2 B of the neighbouring row -- or, past the
      // tensor's last row, of the allocation's padding: torch's caching allocator rounds blocks to 512 B and the
      // tensor is 4-B aligned, so the word is inside the allocation; those bytes are never unpacked)
      if (w * 4 + 4 > lo && w * 4 < hi) v = xw[w];
    }
    rv[j] = v;
  }
}

// rv (this thread's words) -> raw (LDS) -> barrier -> the padded patch (4 x bf16 per pixel, zeros outside the image)
template <int PR, int NT, int RW>
__device__ __forceinline__ void stem_patch_from_rows(uint2* __restrict__ patch, uint32_t* __restrict__ raw,
                                                     const uint32_t (&rv)[RW], const StemTile T, int H, int W) {
  static_assert(RW == PRows<PR, NT>::RW, "words per thread");
#pragma unroll
  for (int j = 0; j < RW; ++j) {
    const int i = threadIdx.x + NT * j;
    if (i < PR * kRD) raw[i] = rv[j];
  }
  __syncthreads();
  const unsigned short* rb = reinterpret_cast<const unsigned short*>(raw);
#pragma unroll
  for (int j = 0; j < PRows<PR, NT>::PPT; ++j) {
    const int i = threadIdx.x + NT * j;
    if (i >= PR * kPC) break;
    const int r = i / kPC, c = i - r * kPC;
    const int iy = T.iy0 + r, ix = T.ix0 + c;
    uint2 v = make_uint2(0u, 0u);
    if (iy >= 0 && iy < H && ix >= 0 && ix < W) {
      // the row segment's misalignment: its first byte 6 ((n H + iy) W + ix0) is 2 mod 4 exactly when that pixel
      // index is odd (the parity survives 32-bit wrap-around)
      const int sh = ((((unsigned)T.n * H + iy) * W + T.ix0) & 1u) << 1;
      const int e = (r * kRD * 4 + sh + c * 6) >> 1;   // the pixel's first 2-B element in raw
      v.x = (uint32_t)rb[e] | ((uint32_t)rb[e + 1] << 16);
      v.y = (uint32_t)rb[e + 2];
    }
    patch[i] = v;
  }
}

// Persistent: block b walks tiles b, b + grid, ...; the next tile's patch is fetched into registers
// while the current one is on the MFMA; the weights sit in LDS for the block's lifetime.
__global__ __launch_bounds__(256, 2) void stem_fwd_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ wpk,
                                                         const float* __restrict__ shift, bf16_t* __restrict__ y,
                                                         int H, int W, int Ho, int Wo, int pt, int pl, int tiles_x,
                                                         int tiles_y, int ntiles, int relu) {
  // the patch and the epilogue tile share LDS (a block barrier separates the last patch read from the
  // first epilogue write), so two blocks fit on a CU
  constexpr int kPatchB = kPPT * 256 * 8, kOtB = 4 * 64 * kORow * 2;
  static_assert(kPatchB + kRawB <= kOtB, "the row words fit behind the patch inside the epilogue tile");
  __shared__ __attribute__((aligned(16))) char sbuf[kPatchB > kOtB ? kPatchB : kOtB];
  __shared__ __attribute__((aligned(16))) bf16_t wl[64 * kWRow];
  uint2* patch = reinterpret_cast<uint2*>(sbuf);
  bf16_t* ot = reinterpret_cast<bf16_t*>(sbuf);
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int g = lane >> 4, r16 = lane & 15;
  for (int i = tid; i < 64 * (kKP / 8); i += 256) {
    const int co = i / (kKP / 8), c8 = i - co * (kKP / 8);
    *reinterpret_cast<uint4*>(wl + co * kWRow + c8 * 8) = *reinterpret_cast<const uint4*>(wpk + co * kKP + c8 * 8);
  }
  float sh[4][4];
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
#pragma unroll
    for (int r = 0; r < 4; ++r) sh[mt][r] = shift ? shift[16 * mt + 4 * g + r] : 0.f;

  uint32_t* raw = reinterpret_cast<uint32_t*>(sbuf + kPatchB);   // behind the patch, inside the epilogue tile
  uint32_t rv[kRW];
  int t = blockIdx.x;
  if (t < ntiles) stem_fetch_rows<kPR, 256>(rv, x, stem_tile(t, pt, pl, tiles_x, tiles_y), H, W);
  for (; t < ntiles; t += gridDim.x) {
    __syncthreads();   // previous tile's epilogue reads of the shared area are done
    stem_patch_from_rows<kPR, 256>(patch, raw, rv, stem_tile(t, pt, pl, tiles_x, tiles_y), H, W);
    __syncthreads();
    if (t + (int)gridDim.x < ntiles)
      stem_fetch_rows<kPR, 256>(rv, x, stem_tile(t + gridDim.x, pt, pl, tiles_x, tiles_y), H, W);

    f32x4 acc[4][4];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) acc[mt][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
    const uint2* prow = patch + (2 * wv) * kPC + 2 * g;
#pragma unroll
    for (int s = 0; s < kKS; ++s) {
      bf16x8 wa[4];
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
        wa[mt] = *reinterpret_cast<const bf16x8*>(wl + (16 * mt + r16) * kWRow + 32 * s + 8 * g);
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        const bf16x8 bb = *reinterpret_cast<const bf16x8*>(prow + s * kPC + 2 * (nt * 16 + r16));
#pragma unroll
        for (int mt = 0; mt < 4; ++mt)
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[mt], bb, acc[mt][nt], 0, 0, 0);
      }
    }

    int b = t;
    const int tx = b % tiles_x;
    b /= tiles_x;
    const int ty = b % tiles_y;
    const int n = b / tiles_y;
    // epilogue through a per-wave LDS tile [64 px][64 co] bf16 (stem has no residual: rounding once
    // before staging is the same rounding): each output pixel row is then written as 128 contiguous
    // bytes by 8 lanes of 16 B instead of 16 scattered 8-B pieces
    const int oy = ty * kTR + wv;
    bf16_t* T = ot + wv * 64 * kORow;
    __syncthreads();   // every wave is done reading the patch this tile overwrites
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          v[r] = acc[mt][nt][r] + sh[mt][r];
          if (relu) v[r] = fmaxf(v[r], 0.f);
        }
        uint2 o;
        o.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
        o.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
        *reinterpret_cast<uint2*>(T + (nt * 16 + r16) * kORow + 16 * mt + 4 * g) = o;
      }
    __builtin_amdgcn_wave_barrier();
    if (oy < Ho) {
      bf16_t* yrow = y + ((size_t)n * Ho + oy) * Wo * 64;
#pragma unroll
      for (int pass = 0; pass < 8; ++pass) {
        const int p = pass * 8 + (lane >> 3), c = lane & 7;
        const int ox = tx * kTC + p;
        if (ox < Wo)
          *reinterpret_cast<uint4*>(yrow + (size_t)ox * 64 + 8 * c) =
              *reinterpret_cast<const uint4*>(T + p * kORow + 8 * c);
      }
    }
  }
}

// conv1 + BN + ReLU + pool1 (3x3 / s2, the relu-aware argmax of maxpool_fwd_k3s2) as ONE kernel: the 0.5 GB
// conv-output tensor is never written nor read back.  Tile = 2 pool rows x 31 pool columns, which need 5 conv rows
// (the last one is the next tile's first: recomputed) x 63 conv columns (+ 1 unused: the waves' 4 x 16-pixel
// n-tiles).  Each wave computes ALL 5 conv rows of its 16-column slab (the A fragments of a k-step are shared by
// the rows), the 5 x 64 x 64 conv tile goes through LDS with the forward's rounding (shift, ReLU, bf16), and the
// pool windows read it there: max and first-max index in maxpool_fwd_k3s2's tap order, 255 for a zero window.
constexpr int kPPR = 2, kPPC = 31;            // pool rows / columns per tile
constexpr int kSR = 2 * kPPR + 1;             // conv rows per tile
constexpr int kPRP = 2 * kSR + 5;             // input patch rows

__global__ __launch_bounds__(256, 2) void stem_pool_fwd_kernel(
    const bf16_t* __restrict__ x, const bf16_t* __restrict__ wpk, const float* __restrict__ shift,
    bf16_t* __restrict__ yp, uint8_t* __restrict__ arg, int H, int W, int Ho, int Wo, int pt, int pl, int Hp, int Wp,
    int qt, int ql, int tiles_x, int tiles_y, int ntiles) {
  constexpr int kPatchB = PRows<kPRP, 256>::PPT * 256 * 8, kOtB = kSR * 64 * kORow * 2;
  constexpr int RW = PRows<kPRP, 256>::RW;
  static_assert(kPatchB + PRows<kPRP, 256>::RawB <= kOtB, "patch + row words inside the conv tile area");
  static_assert(2 * (kPPC - 1) + 2 < 64 && 2 * (kPPR - 1) + 2 < kSR, "pool windows inside the conv tile");
  __shared__ __attribute__((aligned(16))) char sbuf[kOtB];
  __shared__ __attribute__((aligned(16))) bf16_t wl[64 * kWRow];
  uint2* patch = reinterpret_cast<uint2*>(sbuf);
  uint32_t* raw = reinterpret_cast<uint32_t*>(sbuf + kPatchB);
  bf16_t* ot = reinterpret_cast<bf16_t*>(sbuf);
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int g = lane >> 4, r16 = lane & 15;
  for (int i = tid; i < 64 * (kKP / 8); i += 256) {
    const int co = i / (kKP / 8), c8 = i - co * (kKP / 8);
    *reinterpret_cast<uint4*>(wl + co * kWRow + c8 * 8) = *reinterpret_cast<const uint4*>(wpk + co * kKP + c8 * 8);
  }
  __shared__ __attribute__((aligned(16))) float shs[64];   // the BN shift (read by the epilogue: no 16 live VGPRs)
  if (tid < 64) shs[tid] = shift ? shift[tid] : 0.f;

  // tile t -> image n, pool origin (kPPR T, kPPC U), conv origin (r0, c0), input patch origin
  auto tile_of = [&](int t, int& T, int& U, int& r0, int& c0) {
    int b = t;
    U = b % tiles_x;
    b /= tiles_x;
    T = b % tiles_y;
    const int n = b / tiles_y;
    r0 = 2 * kPPR * T - qt;
    c0 = 2 * kPPC * U - ql;
    return StemTile{n, 2 * r0 - pt, 2 * c0 - pl};
  };
  uint32_t rv[RW];
  int t = blockIdx.x;
  if (t < ntiles) {
    int T, U, r0, c0;
    stem_fetch_rows<kPRP, 256>(rv, x, tile_of(t, T, U, r0, c0), H, W);
  }
  for (; t < ntiles; t += gridDim.x) {
    int T, U, r0, c0;
    const StemTile st = tile_of(t, T, U, r0, c0);
    __syncthreads();   // the previous tile's pool reads of the shared area are done
    stem_patch_from_rows<kPRP, 256>(patch, raw, rv, st, H, W);
    __syncthreads();
    if (t + (int)gridDim.x < ntiles) {
      int T2, U2, r2, c2;
      stem_fetch_rows<kPRP, 256>(rv, x, tile_of(t + gridDim.x, T2, U2, r2, c2), H, W);
    }

    f32x4 acc[kSR][4];
#pragma unroll
    for (int row = 0; row < kSR; ++row)
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) acc[row][mt] = f32x4{0.f, 0.f, 0.f, 0.f};
    const uint2* pcol = patch + 2 * g + 2 * (16 * wv + r16);
#pragma unroll
    for (int s = 0; s < kKS; ++s) {
      bf16x8 wa[4];
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
        wa[mt] = *reinterpret_cast<const bf16x8*>(wl + (16 * mt + r16) * kWRow + 32 * s + 8 * g);
#pragma unroll
      for (int row = 0; row < kSR; ++row) {
        const bf16x8 bb = *reinterpret_cast<const bf16x8*>(pcol + (2 * row + s) * kPC);
#pragma unroll
        for (int mt = 0; mt < 4; ++mt)
          acc[row][mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[mt], bb, acc[row][mt], 0, 0, 0);
      }
    }
    __syncthreads();   // every wave is done reading the patch the conv tile overwrites
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      const float4 sv = *reinterpret_cast<const float4*>(shs + 16 * mt + 4 * g);
      const float sh[4] = {sv.x, sv.y, sv.z, sv.w};
#pragma unroll
      for (int row = 0; row < kSR; ++row) {
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = fmaxf(acc[row][mt][r] + sh[r], 0.f);
        uint2 o;
        o.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
        o.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
        *reinterpret_cast<uint2*>(ot + (row * 64 + 16 * wv + r16) * kORow + 16 * mt + 4 * g) = o;
      }
    }
    __syncthreads();
    const int n = st.n;
    for (int item = tid; item < kPPR * kPPC * 8; item += 256) {
      const int cv = item & 7, q = item >> 3;
      const int pc = q % kPPC, pr = q / kPPC;
      const int py = kPPR * T + pr, px = kPPC * U + pc;
      if (py >= Hp || px >= Wp) continue;
      float best[8];
      uint8_t bi[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) { best[j] = -INFINITY; bi[j] = 0; }
#pragma unroll
      for (int tp = 0; tp < 9; ++tp) {
        const int lr = 2 * pr + tp / 3, lc = 2 * pc + tp % 3;
        const int sr = r0 + lr, sc = c0 + lc;
        if (sr < 0 || sr >= Ho || sc < 0 || sc >= Wo) continue;
        const uint4 v = *reinterpret_cast<const uint4*>(ot + (lr * 64 + lc) * kORow + cv * 8);
        const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float f = bf2f((bf16_t)(j & 1 ? w4[j >> 1] >> 16 : w4[j >> 1] & 0xffff));
          if (f > best[j]) { best[j] = f; bi[j] = (uint8_t)tp; }
        }
      }
      uint32_t ow[4], aw[2] = {0u, 0u};
#pragma unroll
      for (int j = 0; j < 8; j += 2) ow[j >> 1] = (uint32_t)f2bf(best[j]) | ((uint32_t)f2bf(best[j + 1]) << 16);
#pragma unroll
      for (int j = 0; j < 8; ++j) aw[j >> 2] |= (uint32_t)(best[j] > 0.f ? bi[j] : 255) << (8 * (j & 3));
      const size_t oo = (((size_t)n * Hp + py) * Wp + px) * 64 + cv * 8;
      *reinterpret_cast<uint4*>(yp + oo) = make_uint4(ow[0], ow[1], ow[2], ow[3]);
      *reinterpret_cast<uint2*>(arg + oo) = make_uint2(aw[0], aw[1]);
    }
  }
}

// w (64, 7, 7, 3) fp32 master weights * per-channel scale -> packed bf16 (64, 7, 8, 4): k = ky*32 + kx*4 + ci
__global__ void stem_pack_kernel(const float* __restrict__ w, const float* __restrict__ scale, bf16_t* __restrict__ wpk) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= 64 * kKP) return;
  const int co = i / kKP, k = i - co * kKP;
  const int ky = k >> 5, kx = (k >> 2) & 7, ci = k & 3;
  float v = 0.f;
  if (kx < 7 && ci < 3) v = w[((co * 7 + ky) * 7 + kx) * 3 + ci] * (scale ? scale[co] : 1.f);
  wpk[i] = f2bf(v);
}

// ---------------------------------------------------------------------------------------------- wgrad
// dW[co][k] = sum_p dy[p][co] * patch_p[k] over every output pixel p, in the packed k = ky*32 + kx*4 + ci
// of the forward (224 columns; kx = 7 / ci = 3 columns are discarded by the reduction).
// Persistent blocks walk the same 4x64 output tiles; per tile the reduction runs over its 256 pixels in
// 8 MFMA steps of 32.  Both operands come out of LDS with ds_read_b64_tr_b16 (a 16-lane group reads 4
// rows x 16 columns and each lane gets one column down the 4 rows):
// * A[co][p] from the dy tile in its natural [p][co] layout (128-B rows, 32-B chunks XOR-swizzled by
//   pixel bits 1 and 3 so the 8 rows a 32-lane half reads hit distinct banks);
// * B[p][k] straight from the forward's padded patch: for one ky the 32 k's of pixel p are the 64
//   contiguous bytes at patch[2*oy + ky][2*ox ..] -- consecutive pixels' rows overlap, which the
//   transposed read does not mind.  No im2col, no shifted copies.
// Wave w owns the 4 co tiles and k tiles {w, w+4, w+8, w+12} (< 14); each block writes its 64 x 224
// fp32 partial and stem_wgrad_reduce sums them, applies the BN scale and drops the padding columns.
typedef __attribute__((ext_vector_type(4))) short s16x4;
constexpr int kKW = kKP;   // partial columns

__device__ __forceinline__ s16x4 tr_read(const char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(p));
}
__device__ __forceinline__ int dy_swz(int p) { return ((p >> 1) & 1) | (((p >> 3) & 1) << 1); }

// Pool-fused mode (parg != nullptr): dy is the POOLED gradient [N, Hp, Wp, 64] and parg the relu-aware
// argmax of pool1 (3x3 / s2, pads qt / ql): each dy1 chunk of the conv-output tile is gathered from the
// <= 4 windows covering that pixel (the maxpool_bwd_k3s2 rule), so the 0.5 GB conv-output gradient is
// never written or read back (stem_wgrad_kernel's POOL form).
struct PoolArgs {
  const uint8_t* arg;
  int Hp, Wp, qt, ql;
};


// POOL: dy is pool1's OUTPUT gradient; per tile the pooled gradient rows / columns covering its conv pixels (<= 3 x
// 33 pooled pixels) and their argmax are staged in LDS (prefetched into registers during the previous tile) and
// each conv-output gradient chunk is gathered from there (the <= 4 windows of maxpool_bwd_k3s2's rule) straight
// into the dy tile: neither the 0.5 GB conv-output gradient nor a global gather per chunk.
constexpr int kQR = 3, kQC = 34;                         // staged pooled rows / columns
constexpr int kQPix = kQR * kQC;
constexpr int kQU4 = kQPix * 12;                          // 16-B units: 8 of gradient + 4 of argmax per pixel
constexpr int kQPT = (kQU4 + 255) / 256;

template <int POOL>
__global__ __launch_bounds__(256, 2) void stem_wgrad_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ dy,
                                                           float* __restrict__ part, int N, int H, int W, int Ho, int Wo,
                                                           int pt, int pl, int tiles_x, int tiles_y, PoolArgs pa) {
  __shared__ __attribute__((aligned(16))) uint2 patch[kPR * kPC];
  __shared__ __attribute__((aligned(16))) char dys[256 * 128];
  __shared__ __attribute__((aligned(16))) uint32_t raw[kPR * kRD];
  __shared__ __attribute__((aligned(16))) uint4 qst[POOL ? kQU4 : 1];   // [pixel][8 x 16 B gradient | 4 x 16 B argmax]
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int g = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
  const int ntiles = N * tiles_x * tiles_y;
  f32x4 acc[4][4];
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[mt][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // the next tile's dy chunks and patch pixels are fetched into registers while this tile is on the
  // MFMA (staging was exposed: one tile at a time waits on its global loads)
  uint4 dv[POOL ? kQPT : 8];
  uint32_t rv[kRW];
  // POOL: the staged window of tile (oy0, ox0): pooled rows wy0 .., columns wx0 ..
  auto qorigin = [&](int oy0, int ox0, int& wy0, int& wx0) {
    wy0 = (oy0 + pa.qt - 1) >> 1;    // ceil((oy0 + qt - 2) / 2): the first window reaching row oy0
    wx0 = (ox0 + pa.ql - 1) >> 1;
  };
  auto fetch = [&](int tt) {
    int b = tt;
    const int tx = b % tiles_x;
    b /= tiles_x;
    const int ty = b % tiles_y;
    const int n = b / tiles_y;
    const int oy0 = ty * kTR, ox0 = tx * kTC;
    if constexpr (POOL) {
      int wy0, wx0;
      qorigin(oy0, ox0, wy0, wx0);
#pragma unroll
      for (int j = 0; j < kQPT; ++j) {
        const int i = tid + 256 * j;
        const int px = i / 12, u = i - px * 12;
        const int wy = wy0 + px / kQC, wx = wx0 + px % kQC;
        // outside the pooled map: zero gradient, argmax 255 (never a tap)
        uint4 v = u < 8 ? make_uint4(0u, 0u, 0u, 0u) : make_uint4(~0u, ~0u, ~0u, ~0u);
        if (i < kQU4 && wy >= 0 && wy < pa.Hp && wx >= 0 && wx < pa.Wp) {
          const size_t o = ((size_t)(n * pa.Hp + wy) * pa.Wp + wx) * 64;
          v = u < 8 ? *reinterpret_cast<const uint4*>(dy + o + u * 8)
                    : *reinterpret_cast<const uint4*>(pa.arg + o + (u - 8) * 16);
        }
        dv[j] = v;
      }
      stem_fetch_rows<kPR, 256>(rv, x, stem_tile(tt, pt, pl, tiles_x, tiles_y), H, W);
      return;
    }
#pragma unroll
    for (int j = 0; j < (POOL ? 0 : 8); ++j) {
      const int i = tid + 256 * j;
      const int p = i >> 3, c8 = i & 7;
      const int oy = oy0 + (p >> 6), ox = ox0 + (p & 63);
      uint4 v = make_uint4(0u, 0u, 0u, 0u);
      if (oy < Ho && ox < Wo) v = *reinterpret_cast<const uint4*>(dy + (((size_t)n * Ho + oy) * Wo + ox) * 64 + c8 * 8);
      dv[j] = v;
    }
    stem_fetch_rows<kPR, 256>(rv, x, stem_tile(tt, pt, pl, tiles_x, tiles_y), H, W);
  };
  if ((int)blockIdx.x < ntiles) fetch(blockIdx.x);
  for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
    __syncthreads();   // previous tile's reads are done
    if constexpr (POOL) {
#pragma unroll
      for (int j = 0; j < kQPT; ++j) {
        const int i = tid + 256 * j;
        if (i < kQU4) qst[i] = dv[j];
      }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int i = tid + 256 * j;
        const int p = i >> 3, c8 = i & 7;
        *reinterpret_cast<uint4*>(dys + p * 128 + 32 * ((c8 >> 1) ^ dy_swz(p)) + 16 * (c8 & 1)) = dv[j];
      }
    }
    stem_patch_from_rows<kPR, 256>(patch, raw, rv, stem_tile(t, pt, pl, tiles_x, tiles_y), H, W);   // (its barrier
    // also publishes the staged pooled window)
    if constexpr (POOL) {
      int b = t;
      const int tx = b % tiles_x;
      b /= tiles_x;
      const int ty = b % tiles_y;
      const int oy0 = ty * kTR, ox0 = tx * kTC;
      int wy0, wx0;
      qorigin(oy0, ox0, wy0, wx0);
      const uint8_t* qa = reinterpret_cast<const uint8_t*>(qst);
      const bf16_t* qg = reinterpret_cast<const bf16_t*>(qst);
#pragma nounroll
      for (int j = 0; j < 8; ++j) {   // (not unrolled: the block's accumulators and both prefetches hold ~220 VGPRs)
        const int i = tid + 256 * j;
        const int p = i >> 3, c8 = i & 7;
        const int oy = oy0 + (p >> 6), ox = ox0 + (p & 63);
        float acc8[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        if (oy < Ho && ox < Wo) {
          const int u = oy + pa.qt, v = ox + pa.ql;   // window wy covers rows 2 wy - qt .. + 2
#pragma unroll
          for (int a = 0; a < 2; ++a) {
            const int wy = (u >> 1) - a, ky = u - 2 * wy;
            if (ky > 2 || wy < wy0) continue;
#pragma unroll
            for (int bb = 0; bb < 2; ++bb) {
              const int wx = (v >> 1) - bb, kx = v - 2 * wx;
              if (kx > 2 || wx < wx0) continue;
              const int qp = (wy - wy0) * kQC + (wx - wx0);
              const uint2 am = *reinterpret_cast<const uint2*>(qa + (size_t)qp * 192 + 128 + c8 * 8);
              const uint32_t me = (uint32_t)(ky * 3 + kx);
              const uint32_t a4[2] = {am.x, am.y};
              bool any = false;
#pragma unroll
              for (int e = 0; e < 8; ++e) any |= ((a4[e >> 2] >> (8 * (e & 3))) & 0xffu) == me;
              if (!any) continue;
              const uint4 gq = *reinterpret_cast<const uint4*>(qg + (size_t)qp * 96 + c8 * 8);
              const uint32_t g4[4] = {gq.x, gq.y, gq.z, gq.w};
#pragma unroll
              for (int e = 0; e < 8; ++e)
                if (((a4[e >> 2] >> (8 * (e & 3))) & 0xffu) == me)
                  acc8[e] += __uint_as_float((e & 1 ? g4[e >> 1] >> 16 : g4[e >> 1] & 0xffffu) << 16);
            }
          }
        }
        uint32_t w4[4];
#pragma unroll
        for (int e = 0; e < 8; e += 2) w4[e >> 1] = (uint32_t)f2bf(acc8[e]) | ((uint32_t)f2bf(acc8[e + 1]) << 16);
        *reinterpret_cast<uint4*>(dys + p * 128 + 32 * ((c8 >> 1) ^ dy_swz(p)) + 16 * (c8 & 1)) =
            make_uint4(w4[0], w4[1], w4[2], w4[3]);
      }
    }
    __syncthreads();
    if (t + (int)gridDim.x < ntiles) fetch(t + gridDim.x);
#pragma unroll 2
    for (int st = 0; st < 8; ++st) {
      bf16x8 a[4];
      const int p0 = 32 * st + 8 * g + q, p1 = p0 + 4;
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        const s16x4 lo = tr_read(dys + p0 * 128 + 32 * (mt ^ dy_swz(p0)) + 8 * pp);
        const s16x4 hi = tr_read(dys + p1 * 128 + 32 * (mt ^ dy_swz(p1)) + 8 * pp);
        a[mt] = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
      const char* b0 = reinterpret_cast<const char*>(patch + 2 * (p0 >> 6) * kPC + 2 * (p0 & 63)) + 8 * pp;
      const char* b1 = reinterpret_cast<const char*>(patch + 2 * (p1 >> 6) * kPC + 2 * (p1 & 63)) + 8 * pp;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int kt = wv + 4 * j;
        if (kt >= 14) continue;          // wave-uniform
        const int off = (kt >> 1) * kPC * 8 + 32 * (kt & 1);
        const s16x4 lo = tr_read(b0 + off), hi = tr_read(b1 + off);
        const bf16x8 bb = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
#pragma unroll
        for (int mt = 0; mt < 4; ++mt)
          acc[mt][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[mt], bb, acc[mt][j], 0, 0, 0);
      }
    }
  }
  // C[row = co][col = k]: col = lane&15 + 16*kt, rows 4g + r of co tile mt
  float* dst = part + (size_t)blockIdx.x * 64 * kKW;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int kt = wv + 4 * j;
    if (kt >= 14) continue;
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) dst[(16 * mt + 4 * g + r) * kKW + 16 * kt + (lane & 15)] = acc[mt][j][r];
  }
}

// dw (64, 7, 7, 3) (+)= scale[co] * sum over blocks of part[b][co][ky*32 + kx*4 + ci]
// block = 16 columns x 16 block-strided partial sums, finished through LDS
__global__ __launch_bounds__(256) void stem_wgrad_reduce_kernel(const float* __restrict__ part, int nb,
                                                                const float* __restrict__ scale,
                                                                float* __restrict__ dw, int accumulate) {
  __shared__ float red[16][17];
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  const int col = blockIdx.x * 16 + tx;            // < 64 * 224
  float s = 0.f;
  for (int b = ty; b < nb; b += 16) s += part[(size_t)b * 64 * kKW + col];
  red[ty][tx] = s;
  __syncthreads();
  if (ty) return;
  for (int i = 1; i < 16; ++i) s += red[i][tx];
  const int co = col / kKW, k = col - co * kKW;
  const int ky = k >> 5, kx = (k >> 2) & 7, ci = k & 3;
  if (kx >= 7 || ci >= 3) return;
  if (scale) s *= scale[co];
  const int o = ((co * 7 + ky) * 7 + kx) * 3 + ci;
  dw[o] = accumulate ? dw[o] + s : s;
}
}  // namespace

// y (N, Ho, Wo, 64) = relu?(conv7x7s2(x (N, H, W, 3), wpk) + shift); wpk from mxr_stem_pack.
MXR_API int mxr_stem_fwd(const void* x, const void* wpk, const float* shift, void* y, int N, int H, int W, int Ho,
                         int Wo, int pt, int pl, int relu, hipStream_t stream) {
  // patch pixels outside the image are zero-filled (bounds-checked loads), so any geometry is in range
  if (N <= 0 || H <= 0 || W <= 0 || Ho <= 0 || Wo <= 0) return -1;
  const int tiles_x = (Wo + kTC - 1) / kTC, tiles_y = (Ho + kTR - 1) / kTR;
  const long long ntiles = (long long)N * tiles_x * tiles_y;
  if (ntiles > 0x7fffffffLL) return -1;
  const int grid = (int)(ntiles < 512 ? ntiles : 512);   // 2 resident blocks per CU
  stem_fwd_kernel<<<grid, 256, 0, stream>>>((const bf16_t*)x, (const bf16_t*)wpk, shift, (bf16_t*)y, H, W, Ho, Wo, pt,
                                            pl, tiles_x, tiles_y, (int)ntiles, relu);
  return (int)hipGetLastError();
}

// conv1 + BN shift + ReLU + pool1 (3x3 / s2, pads qt / ql, relu-aware argmax) in one kernel: yp / arg are the
// pool's [N, Hp, Wp, 64] output and argmax (mxr_maxpool_fwd's contract with relu_in); the conv output (Ho x Wo)
// is never stored.
MXR_API int mxr_stem_pool_fwd(const void* x, const void* wpk, const float* shift, void* yp, void* arg, int N, int H,
                              int W, int Ho, int Wo, int pt, int pl, int Hp, int Wp, int qt, int ql,
                              hipStream_t stream) {
  if (N <= 0 || H <= 0 || W <= 0 || Ho <= 0 || Wo <= 0 || Hp <= 0 || Wp <= 0) return -1;
  if ((long long)N * Hp * Wp * 64 >= (1LL << 31)) return -2;
  const int tiles_x = (Wp + kPPC - 1) / kPPC, tiles_y = (Hp + kPPR - 1) / kPPR;
  const long long ntiles = (long long)N * tiles_x * tiles_y;
  if (ntiles > 0x7fffffffLL) return -1;
  const int grid = (int)(ntiles < 512 ? ntiles : 512);   // 2 resident blocks per CU
  stem_pool_fwd_kernel<<<grid, 256, 0, stream>>>((const bf16_t*)x, (const bf16_t*)wpk, shift, (bf16_t*)yp,
                                                 (uint8_t*)arg, H, W, Ho, Wo, pt, pl, Hp, Wp, qt, ql, tiles_x, tiles_y,
                                                 (int)ntiles);
  return (int)hipGetLastError();
}

MXR_API int mxr_stem_pack(const float* w, const float* scale, void* wpk, hipStream_t stream) {
  stem_pack_kernel<<<(64 * kKP + 255) / 256, 256, 0, stream>>>(w, scale, (bf16_t*)wpk);
  return (int)hipGetLastError();
}

// persistent wgrad grid; ws must hold stem_wgrad_blocks(ntiles) * 64 * 224 floats (ops/stem.py mirrors this)
static int stem_wgrad_blocks(long long ntiles) { return (int)(ntiles < 512 ? ntiles : 512); }

// dw (64, 7, 7, 3) fp32 (+)= scale * conv1 weight gradient from x (N, H, W, 3) and dy (N, Ho, Wo, 64) bf16
// parg != nullptr: dy is pool1's output gradient [N, Hp, Wp, 64] and parg its relu-aware argmax (pads qt, ql)
MXR_API int mxr_stem_wgrad(const void* x, const void* dy, float* ws, const float* scale, float* dw, int N, int H, int W,
                           int Ho, int Wo, int pt, int pl, int accumulate, const uint8_t* parg, int Hp, int Wp, int qt,
                           int ql, hipStream_t stream) {
  if (N <= 0 || H <= 0 || W <= 0 || Ho <= 0 || Wo <= 0) return -1;
  if (parg && (Hp <= 0 || Wp <= 0 || qt < 0 || qt > 1 || ql < 0 || ql > 1)) return -1;   // 3x3 / s2 pool only
  PoolArgs pa{parg, Hp, Wp, qt, ql};
  const int tiles_x = (Wo + kTC - 1) / kTC, tiles_y = (Ho + kTR - 1) / kTR;
  const long long ntiles = (long long)N * tiles_x * tiles_y;
  if (ntiles > 0x7fffffffLL) return -1;
  const int nb = stem_wgrad_blocks(ntiles);
  if (parg)
    stem_wgrad_kernel<1><<<nb, 256, 0, stream>>>((const bf16_t*)x, (const bf16_t*)dy, ws, N, H, W, Ho, Wo, pt, pl,
                                                 tiles_x, tiles_y, pa);
  else
    stem_wgrad_kernel<0><<<nb, 256, 0, stream>>>((const bf16_t*)x, (const bf16_t*)dy, ws, N, H, W, Ho, Wo, pt, pl,
                                                 tiles_x, tiles_y, pa);
  stem_wgrad_reduce_kernel<<<64 * kKW / 16, 256, 0, stream>>>(ws, nb, scale, dw, accumulate);
  return (int)hipGetLastError();
}
