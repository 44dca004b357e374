// Halo-staged 3x3 / stride-1 / pad-1 NHWC convolution with fp8 operands on the block-scaled
// v_mfma_scale_f32_32x32x64_f8f6f4 (twice the bf16 MFMA rate per clock), for gfx950: the fp8 form of
// conv_hx32.hip (BASELINE config 5; the packed head layers built at /root/reference/train.py:91).
//
// The LDS geometry is conv_hx32.hip's BYTE for byte: a 64-channel fp8 chunk is 64 B per pixel row, held as
// two 32-B planes (channels 0-31 / 32-63) with the 16-B half u of row h at h * 32 + 16 (u ^ (h >> 3 & 1)).
// What changes:
//
// * one chunk = 64 channels = ONE K-step per tap (K = 64 per MFMA): a kernel row is 3 steps of TI x TJ
//   MFMAs of 64 cycles, the same cycles per row as the bf16 kernel's 6 steps of 32-cycle MFMAs, but over
//   twice the channels -- half the chunks, half the DMA, half the barriers per output tile;
// * a fragment is 32 B per lane (row lane % 32, plane lane / 32 = bytes 32 (lane / 32) .. + 31 of the
//   64-B K row): two ds_read_b128 of the two 16-B halves of the lane's plane row.  A (weights) and B
//   (pixels) use the same lane -> k assignment, so the contraction pairs identical k in any internal order;
//   the 16-lane read groups stay conflict-free (same rows and halves as the bf16 kernel);
// * unit MX block scales (127): the real scales are per tensor (activations, inv_x) and per output channel
//   (weights, inv_w[co]), applied in the epilogue with the bias: y = acc * inv_x * inv_w[co] + b[co];
// * BF = 1 is the data-gradient form: the pixel operand (dY) is e5m2, the weights e4m3, and the fused fp8
//   copy of the output (dX for the next data gradient) is e5m2;
// * the epilogue optionally writes the fp8 copy of y for the next fp8 layer with the delayed scale of
//   F8Out (fp8_common.h) and max-reduces amax(|y|) (one atomic per block).
//
// tile = BCO output channels x 256 pixel slots (ops/halo.py boxes); 8 waves as 2 (co) x 4 (pixels), each
// (BCO / 2) x 64 = TI x 2 accumulators of 32 x 32.
#include <type_traits>

#include "common.h"
#include "conv_common.h"
#include "focal_common.h"
#include "fp8_common.h"
#include "halo_tile.h"

typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(8))) int i32x8;
typedef __attribute__((ext_vector_type(4))) int i32x4;

namespace {

constexpr int Q2_PLANE = HX_HMAX * 32;      // one 32-B plane of the halo image
constexpr int Q2_HBYTES = 2 * Q2_PLANE;     // one halo buffer (one 64-channel chunk)
constexpr int Q2_HPC = 2 * HX_HMAX / 32;    // 1-KiB halo pieces per chunk (28)
constexpr float Q2_QMAX_E4M3 = 448.f, Q2_QMAX_E5M2 = 57344.f;

template <int N>
__device__ __forceinline__ void q2_vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ void q2_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

template <int I, int N, typename F>
__device__ __forceinline__ void q2_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    q2_for<I + 1, N>(f);
  }
}

__device__ __forceinline__ uint32_t q2_relu2(uint32_t x) {
  typedef __attribute__((ext_vector_type(2))) short s16x2;
  const s16x2 r = __builtin_elementwise_max(__builtin_bit_cast(s16x2, x), s16x2{0, 0});
  return __builtin_bit_cast(uint32_t, r);
}

// relu-gradient mask on two packed bf16 outputs: keep o's half where the mask half is > 0 as a bf16 (positive
// bf16 bit patterns are the positive int16s; -0.0 = 0x8000 is not), with three packed 16-bit integer ops
__device__ __forceinline__ uint32_t q2_mask2(uint32_t o, uint32_t m) {
  typedef __attribute__((ext_vector_type(2))) short s16x2;
  typedef __attribute__((ext_vector_type(2))) unsigned short u16x2;
  const s16x2 mp = __builtin_elementwise_max(__builtin_bit_cast(s16x2, m), s16x2{0, 0});
  const u16x2 keep = __builtin_elementwise_min(__builtin_bit_cast(u16x2, mp), u16x2{1, 1});
  return __builtin_bit_cast(uint32_t, __builtin_bit_cast(u16x2, o) * keep);
}

// compile-time epilogue forms (conv3x3_hx32_f8_kernel's EPI; 0 = read the form from the arguments).  BITS: the
// relu-gradient mask as one bit per element (conv_common.h's bitmask): written by a relu form, read by a MASK form;
// NOY: no bf16 output at all (a tower layer whose only readers take its fp8 copy and its bitmask)
constexpr int HX8_FAST = 1, HX8_RELU = 2, HX8_MASK = 4, HX8_ACC = 8, HX8_AMAX = 16, HX8_EMIT = 32, HX8_BITS = 64,
              HX8_NOY = 128, HX8_FOCAL = 256;   // FOCAL: the classification final's fused focal loss (conv_hx32.hip FOC)

// the bitmask byte of 8 packed bf16 outputs (4 dwords): bit j set where output j is a positive bf16 (after the
// relu every other value is +0)
__device__ __forceinline__ uint32_t q2_bits8(const uint4 o) {
  const uint32_t w[4] = {o.x, o.y, o.z, o.w};
  uint32_t b = 0;
#pragma unroll
  for (int e = 0; e < 4; ++e) b |= ((uint32_t)((w[e] & 0xffffu) != 0u) << (2 * e)) | ((uint32_t)((w[e] >> 16) != 0u) << (2 * e + 1));
  return b;
}

// keep-mask of packed bf16 dword e (channels 2 e, 2 e + 1) from a bitmask byte
__device__ __forceinline__ uint32_t q2_keep2(uint32_t byte, int e) {
  return ((0u - ((byte >> (2 * e)) & 1u)) & 0xffffu) | ((0u - ((byte >> (2 * e + 1)) & 1u)) & 0xffff0000u);
}

// an opaque copy of x (the compiler cannot hoist what is computed from it); a __device__ function of its own:
// the VGPR constraint written directly in the kernel template made the host pass drop the kernel stubs
__device__ __forceinline__ int q2_opaque(int x) {
  asm volatile("" : "+v"(x));
  return x;
}

// the 32-B operand of a lane: the two 16-B halves (logical order) of its plane row, swizzle bit sw
__device__ __forceinline__ i32x8 q2_frag(const char* row, int sw) {
  const i32x4 lo = *reinterpret_cast<const i32x4*>(row + (sw << 4));
  const i32x4 hi = *reinterpret_cast<const i32x4*>(row + ((sw ^ 1) << 4));
  return i32x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

template <int BCO, int BF, int EPI>
__global__ __launch_bounds__(512, 2) void conv3x3_hx32_f8_kernel(
    const uint8_t* __restrict__ X, const uint8_t* __restrict__ Wt, const float* __restrict__ inv_x,
    const float* __restrict__ inv_w, const float* __restrict__ bias, const bf16_t* __restrict__ Rs,
    const bf16_t* __restrict__ Mk, bf16_t* __restrict__ Y, const uint8_t* __restrict__ zpage,
    const HaloTile* __restrict__ tiles, ConvGeom g, int relu, int accumulate, int tiles_co, F8Out fo,
    FocalArgs fa) {
  constexpr int NW = 8, WCO = 2, WPX = NW / WCO;
  constexpr int HQ = (Q2_HPC + NW - 1) / NW;   // halo pieces per wave per chunk (a piece past 28 repeats one)
  constexpr int WT_CO = BCO / WCO, WT_PIX = HX_PB / WPX;
  constexpr int TI = WT_CO / 32, TJ = WT_PIX / 32;
  constexpr int WPL = BCO * 32;     // one weight plane: BCO rows x 32 B
  constexpr int TAPB = 2 * WPL;     // one tap
  constexpr int STAGE = 3 * TAPB;   // one kernel row
  constexpr int HOFF = 2 * STAGE;   // halo buffers after the 2-slot weight ring
  constexpr int BOFF = HOFF + 2 * Q2_HBYTES;   // bias [BCO] then dequant scale [BCO] (floats)
  constexpr int NG = BCO / 32;
  constexpr int NWP = 6 * NG / NW;  // weight pieces per wave per kernel row
  constexpr int NVO = NW >= NG ? 1 : NG / NW;
  static_assert(NWP * NW == 6 * NG && (NW % NG == 0 || NG % NW == 0), "weight pieces split evenly");
  static_assert(TI >= 1 && TJ == 2, "wave tile");

  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int cin = g.cin, cout = g.cout;
  const int nch = cin >> 6;
  const int hsub = (lane & 1) ^ ((lane >> 4) & 1);
  const int wg = wave % NG;
  const int wco = wave / WPX, wpx = wave % WPX;
  const int fh = lane >> 5;    // the plane this lane's fragments read (k = 32 fh .. 32 fh + 31)
  const int arow = wco * WT_CO + (lane & 31);
  const int aoff = fh * WPL + arow * 32, asw = (arow >> 3) & 1;
  const auto wrsrc = __builtin_amdgcn_make_buffer_rsrc((void*)Wt, (short)0, cout * 9 * cin, 0x00020000);

  const int item = xcd_remap(blockIdx.x, gridDim.x);
  const int co0 = (item % tiles_co) * BCO;
  const HaloTile& T = tiles[item / tiles_co];

  // weight DMA: packed [tap][chunk][plane][cout][32 B]; voffset = the lane's row (clamped) + half
  int wvoff[NVO];
#pragma unroll
  for (int v = 0; v < NVO; ++v) wvoff[v] = min(co0 + (wg + NW * v) * 32 + (lane >> 1), cout - 1) * 32 + hsub * 16;
  // halo DMA sources: piece k = 32 halo rows (k / 2) x plane (k % 2); byte offset of the lane's 16 B in
  // chunk 0, -1 = outside the level
  int hsrc[HQ];
#pragma unroll
  for (int q = 0; q < HQ; ++q) {
    int k = wave + NW * q;
    if (k >= Q2_HPC) k -= NW;
    const int h = (k >> 1) * 32 + (lane >> 1);
    HX_SELECT(hoff, h)
    int hoff = T.b[0].hoff, ib = T.b[0].in_base, H = T.b[0].H, W = T.b[0].W, y0 = T.b[0].y0, x0 = T.b[0].x0,
        C = T.b[0].C;
#pragma unroll
    for (int t = 1; t < HX_BOX; ++t)
      if (sel == t) {
        hoff = T.b[t].hoff; ib = T.b[t].in_base; H = T.b[t].H; W = T.b[t].W;
        y0 = T.b[t].y0; x0 = T.b[t].x0; C = T.b[t].C;
      }
    int off = -1;
    if (h < T.nhalo) {
      const int pw = C + 2;
      const int loc = h - hoff;
      const int hr = fdiv(loc, pw), hc = loc - hr * pw;
      const int y = y0 - 1 + hr, x = x0 - 1 + hc;
      if ((unsigned)y < (unsigned)H && (unsigned)x < (unsigned)W) off = (ib + y * W + x) * cin + (k & 1) * 32 + hsub * 16;
    }
    hsrc[q] = off;
  }
  // pixel slots of the lane's B fragments: halo row of tap (0, 0), halo pitch, output element offset
  int hb[TJ], hp[TJ], mo[TJ];
#pragma unroll
  for (int j = 0; j < TJ; ++j) {
    const int p = wpx * WT_PIX + j * 32 + (lane & 31);
    HX_SELECT(sbeg, p)
    int sb = T.b[0].sbeg, ho = T.b[0].hoff, C = T.b[0].C, ob = T.b[0].out_base, W = T.b[0].W, y0 = T.b[0].y0,
        x0 = T.b[0].x0;
#pragma unroll
    for (int t = 1; t < HX_BOX; ++t)
      if (sel == t) {
        sb = T.b[t].sbeg; ho = T.b[t].hoff; C = T.b[t].C; ob = T.b[t].out_base; W = T.b[t].W; y0 = T.b[t].y0;
        x0 = T.b[t].x0;
      }
    if (p < T.nslot) {
      const int loc = p - sb;
      const int r = fdiv(loc, C), c = loc - r * C;
      hb[j] = ho + r * (C + 2) + c;
      hp[j] = C + 2;
      mo[j] = (ob + (y0 + r) * W + x0 + c) * cout;
    } else {
      hb[j] = 0;
      hp[j] = 0;
      mo[j] = -1;
    }
  }

  // (the per-lane arrays go in as pointer parameters: capturing an array whose bound is a local constexpr made
  // the host pass drop the kernel stubs, as in conv_hx32.hip)
  auto issue_w = [&](const int* vo, int ky, int c, int slot, int m0, int m1) {
#pragma unroll
    for (int m = m0; m < m1; ++m) {
      const int k = wave + NW * m;
      const int kx = k / (2 * NG), p = (k / NG) & 1;
      const int v = NVO == 1 ? 0 : m % NVO;
      const int soff = (((ky * 3 + kx) * nch + c) * 2 + p) * cout * 32;
      char* dst = smem + slot * STAGE + kx * TAPB + p * WPL + (wg + NW * v) * 1024;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(wrsrc, (__attribute__((address_space(3))) void*)dst, 16, vo[v], soff,
                                                0, 0);
    }
  };
  auto issue_halo = [&](const int* hs, int c, int buf, int q0, int q1) {
#pragma unroll
    for (int q = q0; q < q1; ++q) {
      int k = wave + NW * q;
      if (k >= Q2_HPC) k -= NW;
      char* dst = smem + HOFF + buf * Q2_HBYTES + (k & 1) * Q2_PLANE + (k >> 1) * 1024;
      const uintptr_t a = hs[q] >= 0 ? (uintptr_t)(X + (long long)hs[q] + c * 64) : (uintptr_t)zpage;
      glds16((const void*)a, dst);
    }
  };

  f32x16 acc[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  // one kernel row ky of a chunk: 3 taps = 3 steps x TI groups; group (n, i) = the TJ MFMAs of weight
  // fragment i of tap n.  Reads run one group ahead (A, double-buffered) and one step ahead (B, at the
  // step's first group): 48 fragment VGPRs, as the bf16 kernel (a double-buffered A / B set per step
  // spilled at 32 B per fragment).  dma(n) goes out in step n's first group.
  auto stage = [&](auto kyc, auto slotc, auto bufc, auto&& dma) {
    constexpr int ky = decltype(kyc)::value, slot = decltype(slotc)::value, buf = decltype(bufc)::value;
    // the B addresses are computed here, per row, from an opaque copy of the slot's halo row: left to
    // itself the compiler hoists all 2 x 3 x 3 x TJ x 2 of them out of the chunk loop and spills
    int bo[TJ][3], bs[TJ][3];
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
      const int h0 = q2_opaque(hb[j] + ky * hp[j]);
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        const int h = h0 + kx;
        bo[j][kx] = HOFF + buf * Q2_HBYTES + fh * Q2_PLANE + h * 32;
        bs[j][kx] = (h >> 3) & 1;
      }
    }
    const char* ws = smem + slot * STAGE + aoff;
    i32x8 fa[2], fb[2][TJ];
    fa[0] = q2_frag(ws, asw);
#pragma unroll
    for (int j = 0; j < TJ; ++j) fb[0][j] = q2_frag(smem + bo[j][0], bs[j][0]);
    __builtin_amdgcn_sched_group_barrier(0x0100, 2 + 2 * TJ, 0);
    q2_for<0, 3 * TI>([&](auto gc) {
      constexpr int gi = decltype(gc)::value, n = gi / TI, i = gi % TI;
      constexpr int nd = i == 0 ? decltype(dma(std::integral_constant<int, n>{}))::value : 0;
      if constexpr (i == 0) dma(std::integral_constant<int, n>{});
      constexpr int g1 = gi + 1;
      constexpr int nra = g1 < 3 * TI ? 2 : 0;
      if constexpr (g1 < 3 * TI) fa[g1 & 1] = q2_frag(ws + (g1 / TI) * TAPB + (g1 % TI) * 1024, asw);
      constexpr int nrb = (i == 0 && n + 1 < 3) ? 2 * TJ : 0;
      if constexpr (nrb > 0) {
#pragma unroll
        for (int j = 0; j < TJ; ++j) fb[(n + 1) & 1][j] = q2_frag(smem + bo[j][n + 1], bs[j][n + 1]);
      }
#pragma unroll
      for (int j = 0; j < TJ; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(fa[gi & 1], fb[n & 1][j], acc[i][j], 0, BF, 0, 127,
                                                                    0, 127);
      // MFMA j followed by its share of the group's reads, then of its DMA pieces
      constexpr int NRD = nra + nrb;
      q2_for<0, TJ>([&](auto jc) {
        constexpr int j = decltype(jc)::value;
        constexpr int r = NRD * (j + 1) / TJ - NRD * j / TJ;
        constexpr int d = nd * (j + 1) / TJ - nd * j / TJ;
        __builtin_amdgcn_sched_group_barrier(0x0008, 1, 0);
        if constexpr (r > 0) __builtin_amdgcn_sched_group_barrier(0x0100, r, 0);
        if constexpr (d > 0) __builtin_amdgcn_sched_group_barrier(0x0010, d, 0);
      });
      __builtin_amdgcn_sched_barrier(0);
    });
  };

  // ---- prologue: chunk 0's halo and weight row 0, the tile's bias and dequantisation scales
  issue_halo(hsrc, 0, 0, 0, HQ);
  issue_w(wvoff, 0, 0, 0, 0, NWP);
  {
    float4 bv4 = make_float4(0.f, 0.f, 0.f, 0.f), sv4 = bv4;
    if (threadIdx.x < BCO / 4 && co0 + 4 * (int)threadIdx.x < cout) {
      const float sx = *inv_x;
      const float4 w4 = *reinterpret_cast<const float4*>(inv_w + co0 + 4 * threadIdx.x);
      sv4 = make_float4(sx * w4.x, sx * w4.y, sx * w4.z, sx * w4.w);
      if (bias != nullptr) bv4 = *reinterpret_cast<const float4*>(bias + co0 + 4 * threadIdx.x);
    }
    q2_vm_wait<0>();
    if (threadIdx.x < BCO / 4) {
      *reinterpret_cast<float4*>(smem + BOFF + 16 * threadIdx.x) = bv4;
      *reinterpret_cast<float4*>(smem + BOFF + BCO * 4 + 16 * threadIdx.x) = sv4;
    }
  }
  q2_sync();

  auto chunk = [&](int c, auto bufc) {
    constexpr int buf = decltype(bufc)::value;
    const bool more = c + 1 < nch;
    const int cn = more ? c + 1 : c;   // past the last chunk the DMA keeps its shape (reloads, unread)
    q2_for<0, 3>([&](auto kyc) {
      constexpr int ky = decltype(kyc)::value;
      constexpr int slot = (buf + ky) & 1;   // stage s = 3 c + ky uses weight slot s % 2 (3 c + ky = c + ky mod 2)
      const int wky = ky < 2 ? ky + 1 : 0, wc = ky < 2 ? c : cn;
      auto dma = [&](auto nc) {
        constexpr int n = decltype(nc)::value;
        // weights of the next row: steps 0-1; the next chunk's halo (row 0 only): steps 1-2
        constexpr int WS = (NWP + 1) / 2;
        constexpr int m0 = n == 0 ? 0 : (n == 1 ? WS : NWP), m1 = n == 0 ? WS : NWP;
        if constexpr (m1 > m0) issue_w(wvoff, wky, wc, slot ^ 1, m0, m1);
        constexpr bool hs = ky == 0 && n >= 1;
        constexpr int HS = (HQ + 1) / 2;
        constexpr int q0 = hs ? (n - 1) * HS : 0, q1 = hs ? (n == 1 ? HS : HQ) : 0;
        if constexpr (q1 > q0) issue_halo(hsrc, cn, buf ^ 1, q0, q1);
        return std::integral_constant<int, (m1 > m0 ? m1 - m0 : 0) + (q1 - q0)>{};
      };
      stage(kyc, std::integral_constant<int, slot>{}, bufc, dma);
      // (also after the last row of the last chunk: a branch here made the register allocator spill the
      // accumulators around it)
      if constexpr (ky == 0) q2_vm_wait<HQ>();   // the next row's weights; the halo by the end of row 1
      else q2_vm_wait<0>();
      q2_sync();
    });
  };
  // the weight slot of stage s = 3 c + ky is s % 2 = (c + ky) % 2; the chunk loop runs by two so the
  // slot / buffer parities are compile-time
  for (int c = 0; c < nch; c += 2) {   // nch is even (cin % 128 == 0)
    chunk(c, std::integral_constant<int, 0>{});
    chunk(c + 1, std::integral_constant<int, 1>{});
  }
  q2_vm_wait<0>();

  // ---- epilogue straight from the accumulators (conv_hx32.hip's): lane l of a 32 x 32 tile holds pixel
  // l % 32, channels 8 q + 4 (l / 32) + 0..3; dequantise + bias, two v_permlane32_swap per pair of channel
  // quads give each lane 8 consecutive channels -> one 16-B bf16 store (and an 8-B fp8 store) per lane.
  // EPI != 0 is a compile-time form (HX8_*): its operands and steps are constants, so the unrolled epilogue has
  // no per-chunk pointer tests or branches, and its relu-gradient mask goes on the packed bf16 words
  // (q2_mask2); EPI == 0 reads the form from the arguments (residual, bitmasks, anything uncommon).
  constexpr bool GEN = EPI == 0;
  constexpr bool K_MASK = (EPI & HX8_MASK) != 0;
  constexpr bool K_BITS = (EPI & HX8_BITS) != 0, K_NOY = (EPI & HX8_NOY) != 0, K_FOC = (EPI & HX8_FOCAL) != 0;
  float foc_acc = 0.f, foc_inv = 0.f, foc_elo = 0.f, foc_ehi = 0.f;   // K_FOC: the block's loss, 1 / #positives
  if constexpr (K_FOC) {
    foc_inv = 1.0f / fmaxf(1.0f, (float)(*fa.npos));
    foc_elo = __expf(-fabsf(fa.lo));
    foc_ehi = __expf(-fabsf(fa.hi));
  }
  uint8_t* const mkb = (uint8_t*)((uintptr_t)Mk & ~(uintptr_t)1);   // the bitmask (K_BITS forms)
  const bool do_relu = GEN ? relu != 0 : (EPI & HX8_RELU) != 0;
  const bool do_amax = GEN ? fo.amax3 != nullptr : (EPI & HX8_AMAX) != 0;
  const bool do_emit = GEN ? fo.Yq != nullptr : (EPI & HX8_EMIT) != 0;
  const bf16_t* Rs_ = GEN ? Rs : nullptr;
  const bf16_t* Mk_ = GEN ? Mk : nullptr;      // (the compile-time masked form reads Mk itself)
  const bf16_t* Yacc = (GEN ? accumulate != 0 : (EPI & HX8_ACC) != 0) ? Y : nullptr;
  constexpr float QMAX = (BF || K_FOC) ? Q2_QMAX_E5M2 : Q2_QMAX_E4M3;   // (FOCAL emits the e5m2 gradient rows)
  float qs = 0.f, tmax = 0.f;
  if (do_amax) {
    const float prev = fo.amax3[(fo.phase + 2) % 3];
    qs = prev > 0.f ? QMAX / (fo.margin * prev) : 0.f;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      fo.amax3[(fo.phase + 1) % 3] = 0.f;
      if (fo.inv_out) *fo.inv_out = fo.margin * prev / QMAX;
    }
  }
  const bool plain = Rs_ == nullptr && Yacc == nullptr && Mk_ == nullptr;   // uniform
#pragma unroll
  for (int i = 0; i < TI; ++i) {
    float4 bv[4], sv[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int cl = wco * WT_CO + i * 32 + 8 * q + 4 * fh;
      bv[q] = *reinterpret_cast<const float4*>(smem + BOFF + 4 * cl);
      sv[q] = *reinterpret_cast<const float4*>(smem + BOFF + BCO * 4 + 4 * cl);
    }
    // this i's residual / accumulate / mask operands, all issued before any is used
    Epi8 ep[TJ][2];
    uint4 mw[TJ][2];
    uint32_t mbyte[TJ][2];
    if (!plain) {
#pragma unroll
      for (int j = 0; j < TJ; ++j)
#pragma unroll
        for (int qp = 0; qp < 2; ++qp) {
          const int cg = co0 + wco * WT_CO + i * 32 + 16 * qp + 8 * fh;
          if (mo[j] >= 0 && cg < cout) epi_load8(ep[j][qp], Rs_, mo[j] + cg, Yacc, Mk_, mo[j] + cg);
        }
    }
    if constexpr (K_MASK) {
#pragma unroll
      for (int j = 0; j < TJ; ++j)
#pragma unroll
        for (int qp = 0; qp < 2; ++qp) {
          const int cg = co0 + wco * WT_CO + i * 32 + 16 * qp + 8 * fh;
          if constexpr (K_BITS) {
            mbyte[j][qp] = 0u;
            if (mo[j] >= 0 && cg < cout) mbyte[j][qp] = mkb[(mo[j] + cg) >> 3];
          } else {
            mw[j][qp] = make_uint4(0u, 0u, 0u, 0u);
            if (mo[j] >= 0 && cg < cout) mw[j][qp] = *reinterpret_cast<const uint4*>(Mk + mo[j] + cg);
          }
        }
    }
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
      float f[4][4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        f[q][0] = acc[i][j][4 * q] * sv[q].x + bv[q].x;
        f[q][1] = acc[i][j][4 * q + 1] * sv[q].y + bv[q].y;
        f[q][2] = acc[i][j][4 * q + 2] * sv[q].z + bv[q].z;
        f[q][3] = acc[i][j][4 * q + 3] * sv[q].w + bv[q].w;
      }
      uint32_t pk[4][2];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        pk[q][0] = (uint32_t)f2bf(f[q][0]) | ((uint32_t)f2bf(f[q][1]) << 16);
        pk[q][1] = (uint32_t)f2bf(f[q][2]) | ((uint32_t)f2bf(f[q][3]) << 16);
      }
#pragma unroll
      for (int qp = 0; qp < 2; ++qp)
#pragma unroll
        for (int d = 0; d < 2; ++d) {
          const auto r = __builtin_amdgcn_permlane32_swap(pk[2 * qp][d], pk[2 * qp + 1][d], false, false);
          pk[2 * qp][d] = r[0];
          pk[2 * qp + 1][d] = r[1];
        }
#pragma unroll
      for (int qp = 0; qp < 2; ++qp) {
        const int cg = co0 + wco * WT_CO + i * 32 + 16 * qp + 8 * fh;
        if (mo[j] < 0 || cg >= cout) continue;
        const int off = mo[j] + cg;
        uint4 o = make_uint4(pk[2 * qp][0], pk[2 * qp][1], pk[2 * qp + 1][0], pk[2 * qp + 1][1]);
        float v[8];
        if (plain) {
          if constexpr (K_MASK && K_BITS) {
            const uint32_t mb = mbyte[j][qp];
            o.x &= q2_keep2(mb, 0); o.y &= q2_keep2(mb, 1); o.z &= q2_keep2(mb, 2); o.w &= q2_keep2(mb, 3);
          } else if constexpr (K_MASK) {
            const uint4 m = mw[j][qp];
            o.x = q2_mask2(o.x, m.x); o.y = q2_mask2(o.y, m.y); o.z = q2_mask2(o.z, m.z); o.w = q2_mask2(o.w, m.w);
          }
          if (do_relu) {
            o.x = q2_relu2(o.x); o.y = q2_relu2(o.y); o.z = q2_relu2(o.z); o.w = q2_relu2(o.w);
          }
          if constexpr (K_BITS && !K_MASK) mkb[off >> 3] = (uint8_t)q2_bits8(o);   // the relu form writes the bits
          const uint32_t w4[4] = {o.x, o.y, o.z, o.w};
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            v[2 * e] = bf2f((bf16_t)(w4[e] & 0xffff));
            v[2 * e + 1] = bf2f((bf16_t)(w4[e] >> 16));
          }
        } else {
          const uint32_t w4[4] = {o.x, o.y, o.z, o.w};
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            v[2 * e] = bf2f((bf16_t)(w4[e] & 0xffff));
            v[2 * e + 1] = bf2f((bf16_t)(w4[e] >> 16));
          }
          epi_apply8(v, ep[j][qp], Rs_, Yacc, Mk_, do_relu);
          o.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
          o.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
          o.z = (uint32_t)f2bf(v[4]) | ((uint32_t)f2bf(v[5]) << 16);
          o.w = (uint32_t)f2bf(v[6]) | ((uint32_t)f2bf(v[7]) << 16);
        }
        if constexpr (K_FOC) {
          // (conv_hx32.hip's FOC epilogue: 80 classes, a chunk inside one anchor; focal_common.h)
          const int pix = mo[j] / cout;
          const int a = cg / 80, c0 = cg - a * 80;
          const long long row = (long long)pix * fa.A + a;
          const int st = fa.state[row];
          float gv[8];
          if (st == -1) {
#pragma unroll
            for (int e = 0; e < 8; ++e) gv[e] = 0.f;
          } else {
            foc_acc += focal8_g2(v, st == 1 ? fa.label[row] - c0 : -1, fa.alpha, fa.gamma, fa.lo, fa.hi, foc_elo,
                                 foc_ehi, foc_inv, gv);
          }
          if constexpr (K_NOY) {
            // the gradient rows as their e5m2 copy only (delayed scale of fo; the fp8 backward reads nothing else)
#pragma unroll
            for (int e = 0; e < 8; ++e) tmax = fmaxf(tmax, fabsf(gv[e]));
            uint2 q2;
            q2.x = pack4_e5m2(gv[0] * qs, gv[1] * qs, gv[2] * qs, gv[3] * qs);
            q2.y = pack4_e5m2(gv[4] * qs, gv[5] * qs, gv[6] * qs, gv[7] * qs);
            *reinterpret_cast<uint2*>(fo.Yq + (long long)pix * fa.ld + cg) = q2;
          } else {
            uint4 go;
            go.x = (uint32_t)f2bf(gv[0]) | ((uint32_t)f2bf(gv[1]) << 16);
            go.y = (uint32_t)f2bf(gv[2]) | ((uint32_t)f2bf(gv[3]) << 16);
            go.z = (uint32_t)f2bf(gv[4]) | ((uint32_t)f2bf(gv[5]) << 16);
            go.w = (uint32_t)f2bf(gv[6]) | ((uint32_t)f2bf(gv[7]) << 16);
            *reinterpret_cast<uint4*>(fa.dpad + (long long)pix * fa.ld + cg) = go;
          }
        } else if constexpr (!K_NOY) {
          *reinterpret_cast<uint4*>(Y + off) = o;
        }
        if (do_amax && !K_FOC) {
#pragma unroll
          for (int e = 0; e < 8; ++e) tmax = fmaxf(tmax, fabsf(v[e]));
          if (do_emit) {
            uint2 q2;
            if constexpr (BF) {
              q2.x = pack4_e5m2(v[0] * qs, v[1] * qs, v[2] * qs, v[3] * qs);
              q2.y = pack4_e5m2(v[4] * qs, v[5] * qs, v[6] * qs, v[7] * qs);
            } else {
              q2.x = pack4_e4m3(v[0] * qs, v[1] * qs, v[2] * qs, v[3] * qs);
              q2.y = pack4_e4m3(v[4] * qs, v[5] * qs, v[6] * qs, v[7] * qs);
            }
            *reinterpret_cast<uint2*>(fo.Yq + off) = q2;
          }
        }
      }
    }
  }
  if constexpr (K_FOC) {   // the block's loss partial (fixed order: deterministic)
    __shared__ float fred[16];
    const float bs = block_sum(foc_acc, fred);
    if (threadIdx.x == 0) fa.partials[blockIdx.x] = bs;
  }
  if (do_amax) {    // block max -> ONE atomic per block (values >= 0: int order == float order); one atomic per
                    // wave on the single amax word serialised at L2 and doubled the data-gradient kernel's time
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) tmax = fmaxf(tmax, __shfl_xor(tmax, o));
    float* red = reinterpret_cast<float*>(smem + BOFF + 2 * BCO * 4);
    if (lane == 0) red[wave] = tmax;
    __syncthreads();
    if (threadIdx.x == 0) {
      float mx = red[0];
#pragma unroll
      for (int w = 1; w < NW; ++w) mx = fmaxf(mx, red[w]);
      atomicMax(reinterpret_cast<int*>(fo.amax3 + fo.phase), __float_as_int(mx));
    }
  }
}

template <int BCO, int BF, int EPI>
int launch_hx8(const uint8_t* X, const uint8_t* Wt, const float* ix, const float* iw, const float* bias,
               const bf16_t* R, const bf16_t* Mk, bf16_t* Y, const uint8_t* zpage, const HaloTile* tiles, int ntiles,
               const ConvGeom& g, int relu, int accumulate, const F8Out& fo, hipStream_t stream,
               const FocalArgs& fa = FocalArgs{}) {
  const int tiles_co = (g.cout + BCO - 1) / BCO;
  const long long nwork = (long long)tiles_co * ntiles;
  if (nwork > 0x7fffffffLL || nwork < 1) return -3;
  const size_t lds = (size_t)6 * BCO * 64 + 2 * (size_t)Q2_HBYTES + 2 * BCO * 4 + 8 * 4;
  auto kern = conv3x3_hx32_f8_kernel<BCO, BF, EPI>;
  static bool attr_set = false;
  if (!attr_set) {
    hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr_set = true;
  }
  kern<<<(unsigned)nwork, 512, lds, stream>>>(X, Wt, ix, iw, bias, R, Mk, Y, zpage, tiles, g, relu, accumulate,
                                             tiles_co, fo, fa);
  return (int)hipGetLastError();
}

// the compile-time epilogue forms of the 256-channel tiles (the head layers' tuned winners): forward relu with /
// without its fp8 copy, the final's plain form; data gradient with the relu-gradient mask with / without the e5m2
// copy of dX, the towers' accumulating join, plain.  Everything else runs the generic form.
template <int BCO, int BF>
int launch_form(const uint8_t* X, const uint8_t* Wt, const float* ix, const float* iw, const float* bias,
                const bf16_t* R, const bf16_t* Mk, bf16_t* Y, const uint8_t* zpage, const HaloTile* tiles, int ntiles,
                const ConvGeom& g, int relu, int accumulate, const F8Out& fo, hipStream_t stream) {
#define HX8_L(E) return launch_hx8<BCO, BF, E>(X, Wt, ix, iw, bias, R, Mk, Y, zpage, tiles, ntiles, g, relu, accumulate, \
                                              fo, stream)
  if constexpr (BCO == 256) {
    const bool bits = Mk != nullptr && ((uintptr_t)Mk & 1);
    if (R == nullptr) {
      const int f = HX8_FAST | (relu ? HX8_RELU : 0) | (Mk && !relu ? HX8_MASK : 0) | (accumulate ? HX8_ACC : 0) |
                    (fo.amax3 ? HX8_AMAX : 0) | (fo.Yq ? HX8_EMIT : 0) | (bits ? HX8_BITS : 0) | (Y ? 0 : HX8_NOY);
      if constexpr (BF == 0) {
        switch (f) {
          case HX8_FAST: HX8_L(HX8_FAST);
          case HX8_FAST | HX8_RELU: HX8_L(HX8_FAST | HX8_RELU);
          case HX8_FAST | HX8_RELU | HX8_AMAX: HX8_L(HX8_FAST | HX8_RELU | HX8_AMAX);
          case HX8_FAST | HX8_RELU | HX8_AMAX | HX8_EMIT: HX8_L(HX8_FAST | HX8_RELU | HX8_AMAX | HX8_EMIT);
          case HX8_FAST | HX8_RELU | HX8_AMAX | HX8_EMIT | HX8_BITS | HX8_NOY:
            HX8_L(HX8_FAST | HX8_RELU | HX8_AMAX | HX8_EMIT | HX8_BITS | HX8_NOY);
          default: break;
        }
      } else {
        switch (f) {
          case HX8_FAST: HX8_L(HX8_FAST);
          case HX8_FAST | HX8_ACC: HX8_L(HX8_FAST | HX8_ACC);
          case HX8_FAST | HX8_MASK: HX8_L(HX8_FAST | HX8_MASK);
          case HX8_FAST | HX8_MASK | HX8_AMAX: HX8_L(HX8_FAST | HX8_MASK | HX8_AMAX);
          case HX8_FAST | HX8_MASK | HX8_AMAX | HX8_EMIT: HX8_L(HX8_FAST | HX8_MASK | HX8_AMAX | HX8_EMIT);
          case HX8_FAST | HX8_MASK | HX8_BITS | HX8_AMAX: HX8_L(HX8_FAST | HX8_MASK | HX8_BITS | HX8_AMAX);
          case HX8_FAST | HX8_MASK | HX8_BITS | HX8_AMAX | HX8_EMIT:
            HX8_L(HX8_FAST | HX8_MASK | HX8_BITS | HX8_AMAX | HX8_EMIT);
          case HX8_FAST | HX8_MASK | HX8_BITS | HX8_AMAX | HX8_EMIT | HX8_NOY:
            HX8_L(HX8_FAST | HX8_MASK | HX8_BITS | HX8_AMAX | HX8_EMIT | HX8_NOY);
          default: break;
        }
      }
    }
  }
  if (Y == nullptr) return -7;   // no bf16 output: compile-time forms only
  HX8_L(0);
#undef HX8_L
}

// OHWI fp8 [cout][9][cin] -> [tap][cin / 64][2][cout][32 B]: one thread per 16 B of output
__global__ void hx8_pack_kernel(const uint4* __restrict__ W, uint4* __restrict__ Wp, int cout, int cin, long long n) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int h = (int)(i & 1);
  long long r = i >> 1;
  const int co = (int)(r % cout);
  r /= cout;
  const int p = (int)(r & 1);
  r >>= 1;
  const int nch = cin >> 6;
  const int c = (int)(r % nch);
  const int tap = (int)(r / nch);
  Wp[i] = W[((long long)co * 9 + tap) * (cin >> 4) + c * 4 + p * 2 + h];
}

}  // namespace

MXR_API int mxr_hx8_pack_weights(const void* W, void* Wp, int cout, int cin, hipStream_t stream) {
  if (cin % 64 != 0 || cout < 1) return -1;
  const long long n = (long long)cout * 9 * cin / 16;
  hx8_pack_kernel<<<(unsigned)((n + 255) / 256), 256, 0, stream>>>((const uint4*)W, (uint4*)Wp, cout, cin, n);
  return (int)hipGetLastError();
}

// X: fp8 NHWC (scale *inv_x; e5m2 when variant & 2 -- the data-gradient form), Wt: fp8 e4m3 weights PACKED by
// mxr_hx8_pack_weights (row scale inv_w[co]), Y: bf16 (R residual, Mk relu-gradient mask, accumulate);
// Yq / amax3 / inv_out / phase / margin: fused fp8 copy of y for the next layer (all null = off).  Mk with bit 0
// set is a bitmask (conv_common.h): written by a relu form, read as the relu-gradient mask otherwise.  Y may be
// null for a relu layer that writes its fp8 copy and bitmask (the readers of a tower layer under fp8), and for a
// masked data gradient that writes its e5m2 copy (the dX of an fp8 tower layer: its producer's backward reads only
// the copy -- data and weight gradients, and the bias sums of conv_wgrad_p8_f8's BIAS form).
// variant: bit 0 = 128-channel tiles (else 256), bit 1 = data-gradient form (e5m2 pixels / fp8 output).
// Requires a 3x3 / stride-1 / pad-1 geometry with equal input / output levels, cin % 128 == 0, cout % 8 == 0,
// the tile table of ops/halo.py, (pixels + 1) * max(cin, cout) < 2^31, cout * 9 * cin < 2^31.
MXR_API int mxr_conv3x3_hx32_f8(const void* X, const void* Wt, const float* inv_x, const float* inv_w,
                                const float* bias, const void* R, const void* Mk, void* Y, const void* zpage,
                                const ConvGeom* g, const void* tiles, int ntiles, int relu, int accumulate, void* Yq,
                                float* amax3, float* inv_out, int phase, float margin, int variant,
                                hipStream_t stream) {
  if (g->cin % 128 != 0 || g->cout % 8 != 0) return -1;
  if (g->kh != 3 || g->kw != 3 || g->stride != 1 || g->pt != 1 || g->pl != 1 || g->ostride != 1) return -2;
  if (g->in_img != g->out_img || (g->M + 1) * (long long)std::max(g->cin, g->cout) >= (1LL << 31)) return -4;
  if ((long long)g->cout * 9 * g->cin >= (1LL << 31)) return -4;
  if (Yq && !amax3) return -5;
  // no bf16 output (Y null): only a relu layer that writes its fp8 copy and its bitmask has readers left, or a data
  // gradient (variant bit 1) that writes its e5m2 copy, masked by a bitmask (the readers of a tower layer's dX under fp8)
  if (Y == nullptr && !(Yq && Mk && ((uintptr_t)Mk & 1) && !accumulate && !R && (relu || ((variant & 2) && !bias))))
    return -7;
  const uint8_t *x = (const uint8_t*)X, *w = (const uint8_t*)Wt, *z = (const uint8_t*)zpage;
  const bf16_t *r = (const bf16_t*)R, *mk = (const bf16_t*)Mk;
  bf16_t* y = (bf16_t*)Y;
  const HaloTile* t = (const HaloTile*)tiles;
  const F8Out fo{(uint8_t*)Yq, amax3, inv_out, phase % 3, margin};
  switch (variant) {
    case 0: return launch_form<256, 0>(x, w, inv_x, inv_w, bias, r, mk, y, z, t, ntiles, *g, relu, accumulate, fo, stream);
    case 1: return launch_form<128, 0>(x, w, inv_x, inv_w, bias, r, mk, y, z, t, ntiles, *g, relu, accumulate, fo, stream);
    case 2: return launch_form<256, 1>(x, w, inv_x, inv_w, bias, r, mk, y, z, t, ntiles, *g, relu, accumulate, fo, stream);
    case 3: return launch_form<128, 1>(x, w, inv_x, inv_w, bias, r, mk, y, z, t, ntiles, *g, relu, accumulate, fo, stream);
    default: return -6;
  }
}

void mxr_loss_finalize_launch(const float* partials, int n, const int* npos, float* out, hipStream_t stream);

// The fp8 classification final (256-channel tiles, e4m3 operands, per-tensor / per-channel scales) with the
// sigmoid-focal loss fused into its epilogue: mxr_conv3x3_hx32_focal's contract (no logits; dpad rows and *out,
// partials for ceil(cout / 256) * ntiles blocks; 80 classes, gamma 2).  Wt packed by mxr_hx8_quant_pack.
// dq != nullptr: the gradient rows leave as their e5m2 copy ONLY (dq [M, ld] bytes, columns >= cout untouched;
// delayed scale: amax3 / phase / margin as the F8Out forms, inv_out = the copy's scale) and dpad is not written.
MXR_API int mxr_conv3x3_hx32_f8_focal_q(const void* X, const void* Wt, const float* inv_x, const float* inv_w,
                                        const float* bias, const void* zpage, const ConvGeom* g, const void* tiles,
                                        int ntiles, const int8_t* state, const int32_t* label, const int* npos,
                                        void* dpad, int ld, int A, int C, float alpha, float gamma, float lo, float hi,
                                        float* partials, int nparts, float* out, void* dq, float* amax3,
                                        float* inv_out, int phase, float margin, hipStream_t stream) {
  if (g->cin % 128 != 0 || g->cout % 8 != 0) return -1;
  if (g->kh != 3 || g->kw != 3 || g->stride != 1 || g->pt != 1 || g->pl != 1 || g->ostride != 1) return -2;
  if (g->in_img != g->out_img || (g->M + 1) * (long long)std::max(g->cin, g->cout) >= (1LL << 31)) return -4;
  if ((long long)g->cout * 9 * g->cin >= (1LL << 31)) return -4;
  if (C != 80 || gamma != 2.0f || A * C != g->cout || ld < g->cout || ld % 8 != 0) return -8;
  const long long nwork = (long long)((g->cout + 255) / 256) * ntiles;
  if (nparts < nwork || (long long)g->M * ld >= (1LL << 31)) return -9;
  if (dq ? (!amax3 || phase < 0 || !(margin > 0.f)) : dpad == nullptr) return -5;
  const FocalArgs fa{state, label, npos, (bf16_t*)dpad, partials, ld, A, alpha, gamma, lo, hi};
  int rc;
  if (dq) {
    const F8Out fo{(uint8_t*)dq, amax3, inv_out, phase % 3, margin};
    rc = launch_hx8<256, 0, HX8_FAST | HX8_FOCAL | HX8_AMAX | HX8_EMIT | HX8_NOY>(
        (const uint8_t*)X, (const uint8_t*)Wt, inv_x, inv_w, bias, nullptr, nullptr, nullptr, (const uint8_t*)zpage,
        (const HaloTile*)tiles, ntiles, *g, 0, 0, fo, stream, fa);
  } else {
    const F8Out fo{nullptr, nullptr, nullptr, 0, 1.f};
    rc = launch_hx8<256, 0, HX8_FAST | HX8_FOCAL>((const uint8_t*)X, (const uint8_t*)Wt, inv_x, inv_w, bias, nullptr,
                                                  nullptr, nullptr, (const uint8_t*)zpage, (const HaloTile*)tiles,
                                                  ntiles, *g, 0, 0, fo, stream, fa);
  }
  if (rc) return rc;
  mxr_loss_finalize_launch(partials, (int)nwork, npos, out, stream);
  return (int)hipGetLastError();
}

MXR_API int mxr_conv3x3_hx32_f8_focal(const void* X, const void* Wt, const float* inv_x, const float* inv_w,
                                      const float* bias, const void* zpage, const ConvGeom* g, const void* tiles,
                                      int ntiles, const int8_t* state, const int32_t* label, const int* npos,
                                      void* dpad, int ld, int A, int C, float alpha, float gamma, float lo, float hi,
                                      float* partials, int nparts, float* out, hipStream_t stream) {
  return mxr_conv3x3_hx32_f8_focal_q(X, Wt, inv_x, inv_w, bias, zpage, g, tiles, ntiles, state, label, npos, dpad, ld, A,
                                     C, alpha, gamma, lo, hi, partials, nparts, out, nullptr, nullptr, nullptr, 0, 1.f,
                                     stream);
}
