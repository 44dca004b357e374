// Streaming 1x1 convolution for narrow reductions (K = Cin in {64, 128, 256}), NHWC bf16 on MFMA.
//
// The backbone's bottleneck 1x1 layers (64->256, 128->512, 256->1024, the 256->64 /
// 512->128 reductions and their data gradients) have K <= 256: far too short for the deep K pipeline
// of conv_pipe.hip (its ring never fills) and memory-bound on paper -- at 1.07M pixels a 64->256
// layer with a residual moves 1.2 GB and needs only ~2 MFMA per pixel.  So this kernel streams:
//
// * the weight slice [BN couts][K] is staged in LDS ONCE per block (rows padded by 32 B: the 16 lanes of each
//   ds_read_b128 lane group land on 16 distinct 4-bank groups) and the block then walks pixel tiles
//   persistently (grid.x blocks per cout slice);
// * per pixel tile each wave owns 16 pixels x BN couts: the B operand (x^T, 8 consecutive channels
//   of one pixel) comes straight from global memory as one 16-B load per lane per 32-deep k-step --
//   no LDS round trip -- and the NEXT tile's loads are issued before this tile's MFMAs;
// * C[co][pixel] (A = W) goes through a per-wave fp32 LDS tile, 64 couts at a time, and comes back as
//   8 consecutive couts per lane: the epilogue (bias / frozen-BN shift, residual, accumulate, ReLU,
//   relu-gradient mask -- the conv_pipe.hip semantics, in that order) reads and writes whole 128-B row
//   segments with 16-B lanes.
//
// Stride-2 forward (Caffe-style branch2a / branch1) reads input pixel (2*oy, 2*ox).
#include "conv_common.h"

namespace {

constexpr int kTRow = 68;   // epilogue tile row (fp32): 64 couts + 4 (the float4 writes of a 16-lane group spread)

__device__ __forceinline__ void add8(float (&v)[8], const uint4 rr) {
  const uint32_t w4[4] = {rr.x, rr.y, rr.z, rr.w};
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    v[2 * r] += bf2f((bf16_t)(w4[r] & 0xffff));
    v[2 * r + 1] += bf2f((bf16_t)(w4[r] >> 16));
  }
}

// PF: the epilogue operands (residual, previous output, relu-gradient mask) of the NEXT tile are loaded into
// registers together with its X rows, one tile ahead (BN = 64 only: 2 passes x 3 x 16 B per lane), so the
// epilogue never waits a memory latency of its own -- memory-bound layers (the 256 -> 64 data gradient with
// accumulate + mask moves 0.96 GB at 200 x 334 x 16) ran at ~3 TB/s with the loads issued in the epilogue
template <int K, int BN, int PF = 0>
__global__ __launch_bounds__(256, 2) void c1x1_kernel(const bf16_t* __restrict__ X, const bf16_t* __restrict__ Wt,
                                                     const float* __restrict__ bias, const bf16_t* __restrict__ R,
                                                     const bf16_t* __restrict__ Mk, bf16_t* __restrict__ Y, int M,
                                                     int N, int H, int W, int Ho, int Wo, int stride, int relu,
                                                     int accumulate, int mtiles) {
  constexpr int KS = K / 32;          // k-steps
  constexpr int NT = BN / 16;         // cout tiles per wave
  // LDS row (bf16), +32 B: ds_read_b128 serves a wave as four 16-lane groups {0-3, 12-15, 20-27}, {4-11, 16-19,
  // 28-31} (+32): with a 16-B pad lanes (g, i16) and (g + 1, i16 - 4..) of one group shared bank slots (2-way,
  // measured 37-42 % LDS conflict cycles); a 32-B pad gives each group's 16 rows distinct slots for every K
  constexpr int ROW = K + 16;
  __shared__ __attribute__((aligned(16))) bf16_t wl[BN * ROW];
  __shared__ __attribute__((aligned(16))) float tl[4 * 16 * kTRow];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int g = lane >> 4, i16 = lane & 15;
  const int co0 = blockIdx.y * BN;

  for (int i = tid; i < BN * (K / 8); i += 256) {
    const int r = i / (K / 8), c8 = i - r * (K / 8);
    uint4 v = make_uint4(0u, 0u, 0u, 0u);
    if (co0 + r < N) v = *reinterpret_cast<const uint4*>(Wt + (size_t)(co0 + r) * K + c8 * 8);
    *reinterpret_cast<uint4*>(wl + r * ROW + c8 * 8) = v;
  }
  const int HoWo = Ho * Wo;

  auto load_x = [&](int t, bf16x8 (&bx)[KS]) {
    const int m = t * 64 + wv * 16 + i16;
    if (m < M) {
      size_t in;
      if (stride == 1) {
        in = (size_t)m;
      } else {
        const int n = m / HoWo, rem = m - n * HoWo;
        const int oy = rem / Wo, ox = rem - oy * Wo;
        in = ((size_t)n * H + oy * stride) * W + ox * stride;
      }
      const bf16_t* src = X + in * K + 8 * g;
#pragma unroll
      for (int s = 0; s < KS; ++s) bx[s] = *reinterpret_cast<const bf16x8*>(src + 32 * s);
    } else {
#pragma unroll
      for (int s = 0; s < KS; ++s) bx[s] = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
    }
  };

  static_assert(!PF || BN == 64, "epilogue prefetch: one 64-cout chunk");
  const bf16_t* Yacc = accumulate ? Y : nullptr;
  // epilogue operands of tile t (pass = 0, 1): lane's pixel / cout chunk as in the epilogue below
  auto load_e = [&](int t, Epi8 (&e)[2]) {
#pragma unroll
    for (int pass = 0; pass < 2; ++pass) {
      const int p = pass * 8 + (lane >> 3), cc = 8 * (lane & 7);
      const int m = t * 64 + wv * 16 + p, co = co0 + cc;
      if (m < M && co < N) {
        const size_t off = (size_t)m * N + co;
        epi_load8(e[pass], (const bf16_t*)R, off, Yacc, (const bf16_t*)Mk, off);
      } else {
        e[pass].r = e[pass].y = e[pass].m = make_uint4(0u, 0u, 0u, 0u);
      }
    }
  };

  bf16x8 bx[KS];
  Epi8 ex[PF ? 2 : 1];
  int t = blockIdx.x;
  if (t < mtiles) {
    load_x(t, bx);
    if constexpr (PF) load_e(t, ex);
  }
  __syncthreads();
  for (; t < mtiles; t += gridDim.x) {
    bf16x8 cur[KS];
#pragma unroll
    for (int s = 0; s < KS; ++s) cur[s] = bx[s];
    Epi8 ecur[PF ? 2 : 1];
    if constexpr (PF) {
      ecur[0] = ex[0];
      ecur[1] = ex[1];
    }
    if (t + (int)gridDim.x < mtiles) {
      load_x(t + gridDim.x, bx);
      if constexpr (PF) load_e(t + gridDim.x, ex);
    }

    // keep the weight fragments in LDS: without this the compiler hoists every (loop-invariant) LDS
    // read out of the tile loop and spills
    asm volatile("" ::: "memory");
    f32x4 acc[NT];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) acc[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < KS; ++s)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        const bf16x8 a = *reinterpret_cast<const bf16x8*>(wl + (16 * nt + i16) * ROW + 32 * s + 8 * g);
        acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, cur[s], acc[nt], 0, 0, 0);
      }

    // epilogue through a per-wave LDS tile, 64 couts at a time: C is written as [pixel][co] fp32 and read
    // back 8 consecutive couts per lane, so every global access (residual, accumulate, mask, store) is a
    // 16-B lane of a contiguous 128-B row segment.
    float* T = tl + wv * 16 * kTRow;
#pragma unroll
    for (int c = 0; c < NT / 4; ++c) {
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int q = 0; q < 4; ++q) *reinterpret_cast<f32x4*>(T + i16 * kTRow + 16 * q + 4 * g) = acc[4 * c + q];
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int pass = 0; pass < 2; ++pass) {
        const int p = pass * 8 + (lane >> 3), cc = 8 * (lane & 7);
        const int m = t * 64 + wv * 16 + p, co = co0 + 64 * c + cc;
        if (m >= M || co >= N) continue;
        float v[8];
        const f32x4 lo = *reinterpret_cast<const f32x4*>(T + p * kTRow + cc);
        const f32x4 hi = *reinterpret_cast<const f32x4*>(T + p * kTRow + cc + 4);
        v[0] = lo[0]; v[1] = lo[1]; v[2] = lo[2]; v[3] = lo[3];
        v[4] = hi[0]; v[5] = hi[1]; v[6] = hi[2]; v[7] = hi[3];
        const size_t off = (size_t)m * N + co;
        if (bias) {
          const float4 b0 = *reinterpret_cast<const float4*>(bias + co);
          const float4 b1 = *reinterpret_cast<const float4*>(bias + co + 4);
          v[0] += b0.x; v[1] += b0.y; v[2] += b0.z; v[3] += b0.w;
          v[4] += b1.x; v[5] += b1.y; v[6] += b1.z; v[7] += b1.w;
        }
        if constexpr (PF) epi_apply8(v, ecur[pass], (const bf16_t*)R, Yacc, (const bf16_t*)Mk, relu);
        else epi_sweep8(v, (const bf16_t*)R, off, Yacc, (const bf16_t*)Mk, off, relu);
        uint4 o;
        o.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
        o.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
        o.z = (uint32_t)f2bf(v[4]) | ((uint32_t)f2bf(v[5]) << 16);
        o.w = (uint32_t)f2bf(v[6]) | ((uint32_t)f2bf(v[7]) << 16);
        *reinterpret_cast<uint4*>(Y + off) = o;
      }
    }
  }
}

template <int K, int BN, int PF = 0>
int launch_c1x1(const void* X, const void* Wt, const float* bias, const void* R, const void* Mk, void* Y, int M, int N,
                int H, int W, int Ho, int Wo, int stride, int relu, int accumulate, int blocks_per_slice,
                hipStream_t stream) {
  const int mtiles = (M + 63) / 64;
  const int nslices = (N + BN - 1) / BN;
  int gx = blocks_per_slice > 0 ? blocks_per_slice : (1024 + nslices - 1) / nslices;
  if (gx > mtiles) gx = mtiles;
  if (gx < 1) gx = 1;
  c1x1_kernel<K, BN, PF><<<dim3(gx, nslices), 256, 0, stream>>>(
      (const bf16_t*)X, (const bf16_t*)Wt, bias, (const bf16_t*)R, (const bf16_t*)Mk, (bf16_t*)Y, M, N, H, W, Ho, Wo,
      stride, relu, accumulate, mtiles);
  return (int)hipGetLastError();
}
}  // namespace

// Y (M, N) = epilogue(X (pixels, K) * Wt (N, K)^T); variant = cout slice BN (64 / 128 / 256, BN*K <= 32768);
// bn = 65: BN 64 with the epilogue operands prefetched a tile ahead (PF).
// Output pixel m of an (Ho, Wo) grid reads input pixel (oy*stride, ox*stride) of an (H, W) grid.
MXR_API int mxr_conv1x1_stream(const void* X, const void* Wt, const float* bias, const void* R, const void* Mk, void* Y,
                               int M, int N, int K, int H, int W, int Ho, int Wo, int stride, int relu, int accumulate,
                               int bn, int blocks_per_slice, hipStream_t stream) {
  if (M <= 0 || N <= 0 || N % 8 || (stride != 1 && stride != 2)) return -1;
  if (stride == 1 && (H * W != Ho * Wo)) return -1;
#define C1(KK, BB)                                                                                               \
  if (K == KK && bn == BB)                                                                                       \
    return launch_c1x1<KK, BB>(X, Wt, bias, R, Mk, Y, M, N, H, W, Ho, Wo, stride, relu, accumulate, blocks_per_slice, \
                               stream);
  C1(64, 64) C1(64, 128) C1(64, 256)
  C1(128, 64) C1(128, 128) C1(128, 256)
  C1(256, 64) C1(256, 128)
#undef C1
  if (bn == 65) {
    if (K == 64) return launch_c1x1<64, 64, 1>(X, Wt, bias, R, Mk, Y, M, N, H, W, Ho, Wo, stride, relu, accumulate, blocks_per_slice, stream);
    if (K == 128) return launch_c1x1<128, 64, 1>(X, Wt, bias, R, Mk, Y, M, N, H, W, Ho, Wo, stride, relu, accumulate, blocks_per_slice, stream);
    if (K == 256) return launch_c1x1<256, 64, 1>(X, Wt, bias, R, Mk, Y, M, N, H, W, Ho, Wo, stride, relu, accumulate, blocks_per_slice, stream);
  }
  return -2;
}
