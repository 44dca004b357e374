// Halo-staged 3x3 / stride-1 / pad-1 NHWC bf16 convolution (forward and stride-1 data gradient) on the
// 32x32x16 bf16 MFMA, for gfx950.
//
// Same job and tile table as conv_halo.hip (the head towers / finals over the packed pyramid, the FPN
// smoothing convs, the backbone 3x3 convs: SURVEY §2.6 K1/K2, the layers built at
// /root/reference/train.py:91), redesigned around what its counters and timing-only builds showed
// (profiles/r2_pmc_head_kernels.txt, profiles/r3_hx32_diag.txt):
//
// * LDS images are split into two 32-B "planes" per row (channels 0-15 / 16-31 of a 32-channel chunk),
//   16-B half u of row h at h * 32 + 16 * (u ^ (h >> 3 & 1)).  The 32x32x16 operand read (lane l: row
//   l % 32, half l / 32) of ANY 32 consecutive rows then hits 16 distinct bank slots in every 16-lane
//   group of ds_read_b128 -- including the halo reads of the kx = 1, 2 taps, which start at an arbitrary
//   row (conv_halo.hip's 16x16x32 layout cannot be swizzled conflict-free for every shift: 24 % of its
//   LDS cycles were bank conflicts);
// * the weights are PACKED once per call (mxr_hx32_pack_weights: [tap][chunk][plane][cout][16]) so a
//   1-KiB DMA piece is 1 KiB contiguous, and come in through buffer_load ... lds with ONE per-lane voffset
//   and the tap / chunk / plane in the scalar soffset;
// * a barrier per kernel ROW (3 taps = 48 MFMAs of 32 cycles per wave) instead of per tap: the weight
//   ring has two 3-tap slots, the halo two buffers; the DMA pieces are spread between the MFMAs of the
//   row's first steps; the next chunk's halo is fetched during the current chunk;
// * the epilogue goes straight from the accumulators to memory (bias + ReLU on packed bf16, two
//   v_permlane32_swap per 16-B store): no LDS image, no barrier, no per-chunk pixel decode (the staged
//   sweep of conv_halo.hip costs ~2.6k VALU per lane per tile);
// * PERS: a persistent grid (one block per CU) walks the tiles; the NEXT tile's halo and first weight
//   row are fetched during the current tile's last chunk, so neither the prologue DMA nor the block
//   turnaround is exposed between tiles.
//
// tile = BCO output channels x 256 pixel slots (ops/halo.py boxes); 8 waves as 2 (co) x 4 (pixels), each
// (BCO / 2) x 64 = TI x 2 accumulators of 32 x 32.
#include <type_traits>

#include "common.h"
#include "conv_common.h"
#include "focal_common.h"
#include "halo_tile.h"

typedef __attribute__((ext_vector_type(16))) float f32x16;

namespace {

constexpr int H2_PLANE = HX_HMAX * 32;                // one 32-B plane of the halo image
constexpr int H2_HBYTES = 2 * H2_PLANE;               // one halo buffer
constexpr int H2_HPC = 2 * HX_HMAX / 32;              // 1-KiB halo pieces per chunk (28)

template <int N>
__device__ __forceinline__ void h2_vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ void h2_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

template <int I, int N, typename F>
__device__ __forceinline__ void h2_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    h2_for<I + 1, N>(f);
  }
}

// ReLU of two packed bf16 values (v_pk_max_i16 against 0: every negative value and -0 become +0)
__device__ __forceinline__ uint32_t h2_relu2(uint32_t x) {
  typedef __attribute__((ext_vector_type(2))) short s16x2;
  const s16x2 r = __builtin_elementwise_max(__builtin_bit_cast(s16x2, x), s16x2{0, 0});
  return __builtin_bit_cast(uint32_t, r);
}

// relu-gradient mask on two packed bf16 outputs: keep o's half where the mask half is > 0 as a bf16 (positive
// bf16 bit patterns are the positive int16s; -0.0 = 0x8000 is not), three packed 16-bit integer ops
__device__ __forceinline__ uint32_t h2_mask2(uint32_t o, uint32_t m) {
  typedef __attribute__((ext_vector_type(2))) short s16x2;
  typedef __attribute__((ext_vector_type(2))) unsigned short u16x2;
  const s16x2 mp = __builtin_elementwise_max(__builtin_bit_cast(s16x2, m), s16x2{0, 0});
  const u16x2 keep = __builtin_elementwise_min(__builtin_bit_cast(u16x2, mp), u16x2{1, 1});
  return __builtin_bit_cast(uint32_t, __builtin_bit_cast(u16x2, o) * keep);
}

// the bitmask byte of 8 packed bf16 outputs (bit j: output j is a positive bf16 -- after the relu every other value
// is +0), and the keep-mask of packed dword e from such a byte
__device__ __forceinline__ uint32_t h2_bits8(const uint4 o) {
  const uint32_t w[4] = {o.x, o.y, o.z, o.w};
  uint32_t b = 0;
#pragma unroll
  for (int e = 0; e < 4; ++e) b |= ((uint32_t)((w[e] & 0xffffu) != 0u) << (2 * e)) | ((uint32_t)((w[e] >> 16) != 0u) << (2 * e + 1));
  return b;
}
__device__ __forceinline__ uint32_t h2_keep2(uint32_t byte, int e) {
  return ((0u - ((byte >> (2 * e)) & 1u)) & 0xffffu) | ((0u - ((byte >> (2 * e + 1)) & 1u)) & 0xffff0000u);
}

// byte offset of 16-B half u of row h inside a plane image (32 B per row)
__device__ __forceinline__ int h2_off(int h, int u) { return (h << 5) + ((u ^ ((h >> 3) & 1)) << 4); }

// PERS: persistent grid (needs an even chunk count).
// HL: halo image layout. 0 = two 32-B planes per pixel (a DMA piece = 32 pixels x 32 B: 32 cache lines
// of which 32 B each are used); 1 = 64-B pixel rows, 16-B chunk c of row h at 16 (c ^ (h >> 2 & 3)) --
// equally conflict-free for the 32x32x16 reads of any 32 consecutive rows, and a piece = 16 pixels x
// 64 B contiguous each (16 lines, half of each used).
// DIAG (timing-only builds, wrong results; never raced by the tuner): bit 0 = the weight descriptor has
// zero records (every weight DMA dropped by the range check), bit 1 = no halo DMA, bit 3 = no epilogue,
// bit 4 = every halo piece from the zero page (same instructions and waits: the cost of the gather pattern),
// bit 5 = every halo piece 1 KiB contiguous (random data, the weight-DMA pattern)
// NWV: waves per block -- 8 (2 co x 4 px, (BCO / 2) x 64 per wave, two waves per SIMD) or 4 (2 x 2,
// (BCO / 2) x 128 per wave, one wave per SIMD: a third fewer LDS fragment bytes per MFMA)
// HB1: ONE halo buffer (the next chunk's halo is loaded after the current chunk, not during it) so that a
// 128-channel block fits 77 KiB of LDS and 128 VGPRs and TWO blocks share a CU: each block's halo loads and
// epilogue then overlap the other block's MFMAs instead of idling the CU (non-persistent grids only)
// WR3: a THREE-slot weight ring (stage s in slot s % 3 = ky) with the weights fetched TWO stages ahead: twice the
// weight bytes in flight per CU (non-persistent, two halo buffers; 128 KiB of LDS at BCO 128)
// MK: the compile-time masked data-gradient epilogue (bf16 relu-gradient mask, no bias / relu / residual /
// accumulate): one tile row's mask words issued together, the mask applied to the packed bf16 words (h2_mask2)
// (MK = 2: the same with the relu mask as a bitmask -- conv_common.h's layout, one byte per 8 channels)
// FOC (> 0: the class count): the classification final's fused focal loss -- the logits never reach memory; each
// 8-logit chunk becomes its focal gradient in the padded dY rows (FocalArgs) and a loss term (one partial per block)
// BW: the plain relu forward also writes its output's bitmask (Mk, pointer bit 0 set): one byte store per chunk
template <int BCO, int PERS, int DIAG = 0, int HL = 0, int NWV = 8, int HB1 = 0, int WR3 = 0, int MK = 0, int FOC = 0,
          int BW = 0, int M16 = 0>
__global__ __launch_bounds__(NWV * 64, (HB1 ? (NWV == 4 ? 3 : 4) : (NWV == 8 ? 2 : 1))) void conv3x3_hx32_kernel(
    const bf16_t* __restrict__ X, const bf16_t* __restrict__ Wt, const float* __restrict__ bias,
    const bf16_t* __restrict__ Rs, const bf16_t* __restrict__ Mk, bf16_t* __restrict__ Y,
    const bf16_t* __restrict__ zpage, const HaloTile* __restrict__ tiles, ConvGeom g, int relu, int accumulate,
    int tiles_co, int nwork, FocalArgs fa) {
  uint8_t* const mkb = (uint8_t*)((uintptr_t)Mk & ~(uintptr_t)1);   // MK = 2 / BW: the bitmask
  constexpr int NW = NWV, WCO = 2, WPX = NW / WCO;
  constexpr int H2_HQ = (H2_HPC + NW - 1) / NW;   // halo pieces per wave per chunk (a piece past 28 repeats one)
  constexpr int WT_CO = BCO / WCO, WT_PIX = HX_PB / WPX;
  constexpr int MS = M16 ? 16 : 32;   // MFMA tile edge: 16x16x32 (M16) or 32x32x16
  constexpr int TI = WT_CO / MS, TJ = WT_PIX / MS;
  using AccT = std::conditional_t<M16 != 0, f32x4, f32x16>;
  constexpr int AE = M16 ? 4 : 16;
  constexpr int WPL = BCO * 32;     // one weight plane: BCO rows x 32 B
  constexpr int TAPB = 2 * WPL;     // one tap
  constexpr int STAGE = 3 * TAPB;   // one kernel row (3 taps)
  constexpr int NSLOT = WR3 ? 3 : 2;
  constexpr int HOFF = NSLOT * STAGE;   // the halo buffers follow the weight ring
  constexpr int BOFF = HOFF + (HB1 ? 1 : 2) * H2_HBYTES;   // then two BCO-float bias buffers (tile parity)
  static_assert(!(HB1 && PERS), "one halo buffer: non-persistent grids only");
  static_assert(!(WR3 && (PERS || HB1)), "three-slot ring: non-persistent, two halo buffers");
  constexpr int NG = BCO / 32;      // 32-row weight groups
  constexpr int NWP = 6 * NG / NW;  // weight pieces per wave per stage
  constexpr int WPS = (NWP + 2) / 3;     // weight pieces per step (steps 0-2)
  constexpr int HPS = (H2_HQ + 1) / 2;   // halo pieces per step (steps 3-4 of row 0)
  constexpr int NVO = NW >= NG ? 1 : NG / NW;   // row groups (voffsets) per wave
  static_assert(NWP * NW == 6 * NG && (NW % NG == 0 || NG % NW == 0), "weight pieces split evenly");
  static_assert(TI >= 1 && TJ >= 2, "wave tile");
  static_assert(!M16 || (HL == 0 && TI % 2 == 0 && TJ % 2 == 0 && (DIAG & 64) == 0), "M16: plane layout, even tiles");

  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int cin = g.cin, cout = g.cout;
  const int nch = cin >> 5;
  // a DMA lane loads 16-B half hsub of its row into LDS half (lane & 1): the plane swizzle, applied at
  // the source (LDS-DMA writes lane l at base + 16 l; the rows of a piece start at a multiple of 32)
  const int hsub = M16 ? (lane & 1) : ((lane & 1) ^ ((lane >> 4) & 1));   // M16: unswizzled rows
  const int wg = wave % NG;   // this wave's (first) 32-row weight group
  const int wco = wave / WPX, wpx = wave % WPX;
  const int fh = lane >> 5;   // the 16-B half of a row a fragment lane reads (k = 8 fh .. 8 fh + 7)
  // A (weights): row wco * WT_CO + lane % 32 (+ 32 i: same swizzle bit), half fh
  // M16: row wco * WT_CO + lane % 16 (+ 16 i), plane lane / 32, half lane / 16 % 2 (k = 8 (lane / 16) .. + 7 of the
  // 32-channel chunk) of the UNswizzled plane images: any 16 consecutive rows read conflict-free
  const int aoff = M16 ? (lane >> 5) * WPL + (wco * WT_CO + (lane & 15)) * 32 + ((lane >> 4) & 1) * 16
                       : h2_off(wco * WT_CO + (lane & 31), fh);
  const auto wrsrc = __builtin_amdgcn_make_buffer_rsrc((void*)Wt, (short)0, (DIAG & 1) ? 0 : cout * 9 * cin * 2,
                                                       0x00020000);

  // ---- per-tile state.  Weight DMA: packed [tap][chunk][plane][cout][16], so the lane's row offset is
  // the voffset and (tap, chunk, plane) the soffset; rows past cout are clamped (they feed only outputs
  // that are never stored).  Halo: piece k = 32 halo rows (k / 2) x plane (k % 2), wave w issues
  // k = w + 8 q; hsrc = element offset of the lane's 16 B in chunk 0, -1 = outside the level.
  auto tile_co0 = [&](int item) { return (item % tiles_co) * BCO; };
  auto w_voff = [&](int co0, int* vo) {   // (pointer params: an array-reference parameter typed by a local constexpr made hipcc drop the kernel host stubs)
#pragma unroll
    for (int v = 0; v < NVO; ++v) vo[v] = min(co0 + (wg + NW * v) * 32 + (lane >> 1), cout - 1) * 32 + hsub * 16;
  };
  auto decode_halo = [&](int item, int* hs) {
    const HaloTile& T = tiles[item / tiles_co];
#pragma unroll
    for (int q = 0; q < H2_HQ; ++q) {
      int k = wave + NW * q;
      if (k >= H2_HPC) k -= NW;
      const int h = HL ? k * 16 + (lane >> 2) : (k >> 1) * 32 + (lane >> 1);
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
        if ((unsigned)y < (unsigned)H && (unsigned)x < (unsigned)W)
          off = (ib + y * W + x) * cin + (HL ? ((lane & 3) ^ ((lane >> 4) & 3)) * 8 : (k & 1) * 16 + hsub * 8);
      }
      hs[q] = off;
    }
  };
  // B (pixels): lane's slot p = wpx * 64 + j * 32 + lane % 32 -> halo row of tap (0, 0), the box's halo
  // pitch and the slot's output element offset (channel 0; -1 = empty slot: it reads halo row 0, its
  // results are discarded)
  int hb[TJ], hp[TJ], mo[TJ];
  auto decode_frag = [&](int item) {
    const HaloTile& T = tiles[item / tiles_co];
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
      const int p = wpx * WT_PIX + j * MS + (lane & (MS - 1));
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
  };

  // weight pieces [m0, m1) of this wave for kernel row ky of chunk c, into ring slot `slot`
  auto issue_w = [&](const int* voff, int ky, int c, int slot, int m0, int m1) {
#pragma unroll
    for (int m = m0; m < m1; ++m) {
      const int k = wave + NW * m;
      const int kx = k / (2 * NG), p = (k / NG) & 1;
      const int v = NVO == 1 ? 0 : m % NVO;     // piece m's row group: wg + NW v
      const int soff = (((ky * 3 + kx) * nch + c) * 2 + p) * cout * 32;
      char* dst = smem + slot * STAGE + kx * TAPB + p * WPL + (wg + NW * v) * 1024;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(wrsrc, (__attribute__((address_space(3))) void*)dst, 16, voff[v], soff,
                                                0, 0);
    }
  };
  // halo pieces [q0, q1) of chunk c into buffer buf, from hs (or hn: the next tile's, when `next`)
  auto issue_halo = [&](const int* hs, const int* hn, bool next, int c, int buf, int q0, int q1) {
    if constexpr (DIAG & 2) return;
#pragma unroll
    for (int q = q0; q < q1; ++q) {
      int k = wave + NW * q;
      if (k >= H2_HPC) k -= NW;
      char* dst = smem + HOFF + buf * H2_HBYTES + (HL ? k * 1024 : (k & 1) * H2_PLANE + (k >> 1) * 1024);
      const int o = next ? hn[q] : hs[q];
      uintptr_t a = (o >= 0 && !(DIAG & 16)) ? (uintptr_t)(X + (long long)o + c * 32) : (uintptr_t)zpage;
      if constexpr ((DIAG & 32) != 0) a = (uintptr_t)(X + c * 16384 + k * 512 + lane * 8);
      glds16((const void*)a, dst);
    }
  };
  // the tile's bias, into bias buffer bb (loaded by the first BCO / 4 threads; visible after a barrier)
  auto load_bias = [&](int co0) {
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (bias != nullptr && threadIdx.x < BCO / 4 && co0 + 4 * (int)threadIdx.x < cout)
      v = *reinterpret_cast<const float4*>(bias + co0 + 4 * threadIdx.x);
    return v;
  };
  auto store_bias = [&](int bb, float4 v) {
    if (threadIdx.x < BCO / 4) *reinterpret_cast<float4*>(smem + BOFF + bb * BCO * 4 + 16 * threadIdx.x) = v;
  };

  AccT acc[TI][TJ];

  // one kernel row ky of one chunk: 3 taps x 2 K-halves = 6 steps of TI x TJ MFMAs; the next step's
  // fragment reads interleaved one per MFMA (double-buffered), then dma(n)'s pieces one per MFMA
  auto stage = [&](auto kyc, auto slotc, auto bufc, auto&& dma) {
    constexpr int ky = decltype(kyc)::value, slot = decltype(slotc)::value, buf = decltype(bufc)::value;
    if constexpr (M16) {
      // 16x16x32: ONE K = 32 step per tap (both planes).  The tap's MFMAs run i-major in groups of TJ (co sub-tile
      // i against the TJ pixel sub-tiles), A fragment i + 2 read during group i, the next tap's B fragments during
      // its last two groups: ~3 A and at most 2 TJ B fragments live (the 32x32x16 form's register budget).  Six
      // half-steps n = 2 kx + h of TI / 2 groups (the DMA pieces are placed per half-step, as in that form)
      constexpr int TIH = TI / 2;
      static_assert(TJ % 2 == 0 && TI >= 2 && TI % 2 == 0, "M16 read schedule");
      int bq[TJ];
#pragma unroll
      for (int j = 0; j < TJ; ++j)
        bq[j] = HOFF + (HB1 ? 0 : buf) * H2_HBYTES + (lane >> 5) * H2_PLANE + (hb[j] + ky * hp[j]) * 32 +
                ((lane >> 4) & 1) * 16;
      const char* ws = smem + slot * STAGE + aoff;
      bf16x8 fa[3][TI], fb[3][TJ];
      auto rA = [&](auto kxc, auto ic) {
        constexpr int kx = decltype(kxc)::value, i = decltype(ic)::value;
        fa[kx][i] = *reinterpret_cast<const bf16x8*>(ws + kx * TAPB + i * 512);
      };
      auto rB = [&](auto kxc, auto jc) {
        constexpr int kx = decltype(kxc)::value, j = decltype(jc)::value;
        fb[kx][j] = *reinterpret_cast<const bf16x8*>(smem + bq[j] + kx * 32);
      };
      rA(std::integral_constant<int, 0>{}, std::integral_constant<int, 0>{});
      rA(std::integral_constant<int, 0>{}, std::integral_constant<int, 1>{});
      h2_for<0, TJ>([&](auto jc) { rB(std::integral_constant<int, 0>{}, jc); });
      __builtin_amdgcn_sched_group_barrier(0x0100, 2 + TJ, 0);
      h2_for<0, 6>([&](auto nc) {
        constexpr int n = decltype(nc)::value, kx = n >> 1, h = n & 1;
        constexpr int nd = decltype(dma(nc))::value;   // DMA instructions issued at this half-step
        dma(nc);
        h2_for<0, TIH>([&](auto gc) {
          constexpr int g = decltype(gc)::value, i = h * TIH + g;
          // reads of this group: A fragment i + 2 (or the next tap's first two), the next tap's B in the last two
          constexpr bool ra = i + 2 < TI || kx + 1 < 3;
          constexpr int nb = (i >= TI - 2 && kx + 1 < 3) ? TJ / 2 : 0;
          if constexpr (i + 2 < TI) rA(std::integral_constant<int, kx>{}, std::integral_constant<int, i + 2>{});
          else if constexpr (kx + 1 < 3)
            rA(std::integral_constant<int, kx + 1>{}, std::integral_constant<int, i + 2 - TI>{});
          if constexpr (nb > 0)
            h2_for<0, nb>([&](auto bc) {
              rB(std::integral_constant<int, kx + 1>{},
                 std::integral_constant<int, (i - (TI - 2)) * (TJ / 2) + decltype(bc)::value>{});
            });
#pragma unroll
          for (int j = 0; j < TJ; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[kx][i], fb[kx][j], acc[i][j], 0, 0, 0);
          // schedule: (MFMA, read) pairs, then this group's share of the half-step's DMA pieces between MFMAs
          constexpr int NRD = (ra ? 1 : 0) + nb;
          constexpr int NR = NRD < TJ ? NRD : TJ;
          h2_for<0, NR>([&](auto) {
            __builtin_amdgcn_sched_group_barrier(0x0008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x0100, 1, 0);
          });
          if constexpr (NRD > NR) __builtin_amdgcn_sched_group_barrier(0x0100, NRD - NR, 0);
          constexpr int d0 = g * nd / TIH, d1 = (g + 1) * nd / TIH;
          constexpr int NM = TJ - NR;
          constexpr int NDG = d1 - d0 < NM ? d1 - d0 : NM;
          h2_for<0, NDG>([&](auto) {
            __builtin_amdgcn_sched_group_barrier(0x0008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x0010, 1, 0);
          });
          if constexpr (d1 - d0 > NDG) __builtin_amdgcn_sched_group_barrier(0x0010, d1 - d0 - NDG, 0);
          if constexpr (NM > NDG) __builtin_amdgcn_sched_group_barrier(0x0008, NM - NDG, 0);
          __builtin_amdgcn_sched_barrier(0);   // nothing crosses a group: the reads stay two groups ahead of their use
        });
      });
      return;
    } else {
    int ba[TJ][3][2];
#pragma unroll
    for (int j = 0; j < TJ; ++j)
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        const int h = hb[j] + ky * hp[j] + kx;
        if constexpr (HL) {
#pragma unroll
          for (int kh = 0; kh < 2; ++kh) ba[j][kx][kh] = HOFF + (HB1 ? 0 : buf) * H2_HBYTES + h * 64 + (((2 * kh + fh) ^ ((h >> 2) & 3)) << 4);
        } else {
          ba[j][kx][0] = HOFF + (HB1 ? 0 : buf) * H2_HBYTES + h2_off(h, fh);
          ba[j][kx][1] = ba[j][kx][0] + H2_PLANE;
        }
      }
    const char* ws = smem + slot * STAGE + aoff;
    auto rd = [&](auto nc, bf16x8* a, bf16x8* b) {
      constexpr int n = decltype(nc)::value, kx = n >> 1, kh = n & 1;
#pragma unroll
      for (int i = 0; i < TI; ++i) a[i] = *reinterpret_cast<const bf16x8*>(ws + kx * TAPB + kh * WPL + i * 1024);
#pragma unroll
      for (int j = 0; j < TJ; ++j) b[j] = *reinterpret_cast<const bf16x8*>(smem + ba[j][kx][kh]);
    };
    bf16x8 fa[2][TI], fb[2][TJ];
    rd(std::integral_constant<int, 0>{}, fa[0], fb[0]);
    __builtin_amdgcn_sched_group_barrier(0x0100, TI + TJ, 0);
    h2_for<0, 6>([&](auto nc) {
      constexpr int n = decltype(nc)::value;
      constexpr int nd = decltype(dma(nc))::value;   // DMA instructions issued at this step
      dma(nc);
      if constexpr (n + 1 < 6) rd(std::integral_constant<int, n + 1>{}, fa[(n + 1) & 1], fb[(n + 1) & 1]);
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j) {
          if constexpr ((DIAG & 64) != 0) {
            // timing only: the same FLOPs as two 16x16x32 MFMAs on the same operands (the MFMA shape's clock)
            constexpr int o = (n & 1) * 8;
            f32x4 lo = {acc[i][j][o], acc[i][j][o + 1], acc[i][j][o + 2], acc[i][j][o + 3]};
            f32x4 hi = {acc[i][j][o + 4], acc[i][j][o + 5], acc[i][j][o + 6], acc[i][j][o + 7]};
            lo = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[n & 1][i], fb[n & 1][j], lo, 0, 0, 0);
            hi = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[n & 1][i], fb[n & 1][j], hi, 0, 0, 0);
#pragma unroll
            for (int e = 0; e < 4; ++e) { acc[i][j][o + e] = lo[e]; acc[i][j][o + 4 + e] = hi[e]; }
          } else {
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[n & 1][i], fb[n & 1][j], acc[i][j], 0, 0, 0);
          }
        }
      constexpr int MF = (DIAG & 64) ? 2 : 1;   // MFMA instructions per (i, j)
      constexpr int NRD = n + 1 < 6 ? TI + TJ : 0;
      constexpr int NR = NRD < TI * TJ ? NRD : TI * TJ;
      h2_for<0, NR>([&](auto) {
        __builtin_amdgcn_sched_group_barrier(0x0008, MF, 0);
        __builtin_amdgcn_sched_group_barrier(0x0100, 1, 0);
      });
      if constexpr (NRD > NR) __builtin_amdgcn_sched_group_barrier(0x0100, NRD - NR, 0);
      constexpr int NM = TI * TJ - NR;
      constexpr int ND = nd < NM ? nd : NM;
      h2_for<0, ND>([&](auto) {
        __builtin_amdgcn_sched_group_barrier(0x0008, MF, 0);
        __builtin_amdgcn_sched_group_barrier(0x0010, 1, 0);
      });
      if constexpr (nd > ND) __builtin_amdgcn_sched_group_barrier(0x0010, nd - ND, 0);
      if constexpr (NM > ND) __builtin_amdgcn_sched_group_barrier(0x0008, MF * (NM - ND), 0);
    });
    }
  };

  // ---- first tile: its halo (chunk 0) and weight row (chunk 0, ky 0), its bias
  int item = PERS ? (int)blockIdx.x : xcd_remap(blockIdx.x, gridDim.x);
  float foc_acc = 0.f, foc_inv = 0.f, foc_elo = 0.f, foc_ehi = 0.f;   // FOC: the block's loss, 1 / #positives
  if constexpr (FOC > 0) {
    foc_inv = 1.0f / fmaxf(1.0f, (float)(*fa.npos));
    foc_elo = __expf(-fabsf(fa.lo));
    foc_ehi = __expf(-fabsf(fa.hi));
  }
  int co0 = tile_co0(item);
  int wvoff[NVO];
  w_voff(co0, wvoff);
  int hsrc[H2_HQ];
  decode_halo(item, hsrc);
  issue_halo(hsrc, hsrc, false, 0, 0, 0, H2_HQ);
  issue_w(wvoff, 0, 0, 0, 0, NWP);
  if constexpr (WR3) issue_w(wvoff, 1, 0, 1, 0, NWP);   // two stages ahead: stage 1 too
  {
    const float4 bv4 = load_bias(co0);
    decode_frag(item);
    h2_vm_wait<0>();
    store_bias(0, bv4);
  }
  h2_sync();

  for (int bb = 0;; bb ^= 1) {
    // the next tile of this block (PERS), its DMA sources decoded now: its halo and first weight row go
    // out during this tile's last chunk (into the buffer / slot that chunk leaves free)
    const int nitem = item + (int)gridDim.x;
    const bool has_next = PERS && nitem < nwork;
    int nco0 = co0, nwvoff[NVO], nhsrc[H2_HQ];
#pragma unroll
    for (int v = 0; v < NVO; ++v) nwvoff[v] = wvoff[v];
#pragma unroll
    for (int q = 0; q < H2_HQ; ++q) nhsrc[q] = hsrc[q];
    if (has_next) {
      nco0 = tile_co0(nitem);
      w_voff(nco0, nwvoff);
      decode_halo(nitem, nhsrc);
    }
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int j = 0; j < TJ; ++j)
#pragma unroll
        for (int e = 0; e < AE; ++e) acc[i][j][e] = 0.f;

    // stage s = 3 c + ky uses weight slot s % 2 = (c + ky) % 2 and halo buffer c % 2; the chunk loop is
    // unrolled by two so both are compile-time
    auto chunk = [&](int c, auto bufc) {
      constexpr int buf = decltype(bufc)::value;
      const bool more = c + 1 < nch;
      const bool chain = !more && has_next;   // last chunk, and a next tile to prefetch for
      // past the last chunk without a next tile the DMA keeps its shape and reloads chunk c into the free
      // slot / buffer (nobody reads them; the wait before the epilogue covers them): no branch in a stage
      const int cn = more ? c + 1 : (chain ? 0 : c);
      h2_for<0, 3>([&](auto kyc) {
        constexpr int ky = decltype(kyc)::value;
        constexpr int slot = WR3 ? ky : ((buf + ky) & 1);
        // the next stage's weights go into the other slot, whose last reader (the previous stage) every
        // wave has passed; the next chunk's halo into the other buffer (last read by the previous chunk).
        // WR3: the stage TWO ahead, into the slot of the previous stage ((ky + 2) % 3)
        constexpr int wslot = WR3 ? (ky + 2) % 3 : (slot ^ 1);
        const int wky = WR3 ? (ky + 2) % 3 : (ky < 2 ? ky + 1 : 0);
        const int wc = WR3 ? (ky == 0 ? c : cn) : (ky < 2 ? c : cn);
        int wv[NVO];
#pragma unroll
        for (int v = 0; v < NVO; ++v) wv[v] = (ky == 2 && chain) ? nwvoff[v] : wvoff[v];
        auto dma = [&](auto nc) {
          constexpr int n = decltype(nc)::value;
          constexpr int m0 = n * WPS < NWP ? n * WPS : NWP, m1 = (n + 1) * WPS < NWP ? (n + 1) * WPS : NWP;
          if constexpr (m1 > m0) issue_w(wv, wky, wc, wslot, m0, m1);
          constexpr bool hs = ky == 0 && n >= 3 && n < 5 && !(DIAG & 2) && !HB1;
          constexpr int q0 = hs ? (n - 3) * HPS : 0, q1 = hs ? ((n - 2) * HPS < H2_HQ ? (n - 2) * HPS : H2_HQ) : 0;
          if constexpr (q1 > q0) issue_halo(hsrc, nhsrc, chain, cn, buf ^ 1, q0, q1);
          return std::integral_constant<int, (m1 - m0) + (q1 - q0)>{};
        };
        stage(kyc, std::integral_constant<int, slot>{}, bufc, dma);
        if (ky < 2 || more) {
          // the next stage's weights must have landed; the next chunk's halo (issued after them in row 0)
          // only by the end of row 1.  WR3: the stage-(ky + 2) weights of this stage stay in flight, and the
          // next chunk's halo (row 0, after them) until the end of row 2
          if constexpr (WR3) {
            if constexpr (ky < 2) h2_vm_wait<NWP + H2_HQ>();
            else h2_vm_wait<NWP>();
          } else if constexpr (ky == 0 && !HB1) h2_vm_wait<(DIAG & 2) ? 0 : H2_HQ>();
          else h2_vm_wait<0>();
          h2_sync();
          if constexpr (HB1 && ky == 2) {
            // every wave is past its last read of this chunk's halo: load the next chunk's into the one buffer
            issue_halo(hsrc, nhsrc, false, cn, 0, 0, H2_HQ);
            h2_vm_wait<0>();
            h2_sync();
          }
        }
      });
    };
    for (int c = 0; c < nch; c += 2) {
      chunk(c, std::integral_constant<int, 0>{});
      if (c + 1 < nch) chunk(c + 1, std::integral_constant<int, 1>{});
    }

    // ---- epilogue straight from the accumulators: lane l of a 32 x 32 tile holds pixel l % 32, channels
    // 8 q + 4 (l / 32) + 0..3 (q = 0..3); bias, bf16 packing, then per channel pair (q, q + 1) two
    // v_permlane32_swap give each lane 8 CONSECUTIVE channels -> one 16-B store per lane (residual /
    // accumulate / mask read at the same 16 B), 2 x TI x TJ stores per lane.  Its stores overlap the
    // next tile's DMA, already in flight.
    if constexpr (DIAG & 8) {
      float sacc = 0.f;
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j) sacc += acc[i][j][0] + acc[i][j][AE - 1];
      if (sacc == 1234.5f) Y[threadIdx.x] = 0;   // keeps the accumulators alive
    } else {
      const bf16_t* Yacc = (MK || FOC || BW) ? nullptr : (accumulate ? Y : nullptr);
      const bf16_t* Rs_ = (MK || FOC || BW) ? nullptr : Rs;
      const bf16_t* Mk_ = (MK || FOC || BW) ? nullptr : Mk;
      const bool plain = Rs_ == nullptr && Yacc == nullptr && Mk_ == nullptr;   // uniform
      // one lane's 8 consecutive channels cg.. of output element offset off (pixel offset mo_): mask / relu / bitmask
      // or the general sweep, then the store (or the focal gradient)
      auto put8 = [&](uint4 o, int off, int cg, int mo_, uint32_t mb, uint4 m) {
        if (plain) {
          if constexpr (MK == 2) {
            o.x &= h2_keep2(mb, 0); o.y &= h2_keep2(mb, 1); o.z &= h2_keep2(mb, 2); o.w &= h2_keep2(mb, 3);
          } else if constexpr (MK != 0) {
            o.x = h2_mask2(o.x, m.x); o.y = h2_mask2(o.y, m.y); o.z = h2_mask2(o.z, m.z); o.w = h2_mask2(o.w, m.w);
          }
          // bias (+ ReLU) only: ReLU on the packed bf16 (it commutes with the rounding)
          if (!MK && relu) {
            o.x = h2_relu2(o.x); o.y = h2_relu2(o.y); o.z = h2_relu2(o.z); o.w = h2_relu2(o.w);
          }
          if constexpr (BW != 0) mkb[off >> 3] = (uint8_t)h2_bits8(o);   // the relu output's bitmask
        } else {
          const uint32_t w4[4] = {o.x, o.y, o.z, o.w};
          float v[8];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            v[2 * e] = bf2f((bf16_t)(w4[e] & 0xffff));
            v[2 * e + 1] = bf2f((bf16_t)(w4[e] >> 16));
          }
          epi_sweep8(v, Rs_, off, Yacc, Mk_, off, relu);
          o.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
          o.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
          o.z = (uint32_t)f2bf(v[4]) | ((uint32_t)f2bf(v[5]) << 16);
          o.w = (uint32_t)f2bf(v[6]) | ((uint32_t)f2bf(v[7]) << 16);
        }
        if constexpr (FOC > 0) {
          // anchor row of this chunk (80 % 8 == 0: a chunk never straddles two anchors), its focal gradient
          // into the padded dY row, its loss into the block's partial (focal_common.h: the loss kernel's math)
          const int pix = mo_ / cout;
          const int a = cg / FOC, c0 = cg - a * FOC;
          const long long row = (long long)pix * fa.A + a;
          const int st = fa.state[row];
          float gv[8];
          if (st == -1) {
#pragma unroll
            for (int e = 0; e < 8; ++e) gv[e] = 0.f;
          } else {
            const int lb = st == 1 ? fa.label[row] - c0 : -1;
            const uint32_t w4[4] = {o.x, o.y, o.z, o.w};
            float v[8];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              v[2 * e] = bf2f((bf16_t)(w4[e] & 0xffff));
              v[2 * e + 1] = bf2f((bf16_t)(w4[e] >> 16));
            }
            foc_acc += focal8_g2(v, lb, fa.alpha, fa.gamma, fa.lo, fa.hi, foc_elo, foc_ehi, foc_inv, gv);
          }
          uint4 go;
          go.x = (uint32_t)f2bf(gv[0]) | ((uint32_t)f2bf(gv[1]) << 16);
          go.y = (uint32_t)f2bf(gv[2]) | ((uint32_t)f2bf(gv[3]) << 16);
          go.z = (uint32_t)f2bf(gv[4]) | ((uint32_t)f2bf(gv[5]) << 16);
          go.w = (uint32_t)f2bf(gv[6]) | ((uint32_t)f2bf(gv[7]) << 16);
          *reinterpret_cast<uint4*>(fa.dpad + (long long)pix * fa.ld + cg) = go;
        } else {
          *reinterpret_cast<uint4*>(Y + off) = o;
        }
      };
      if constexpr (M16) {
        // lane l of a 16 x 16 tile holds pixel l % 16, channels 4 (l / 16) + 0..3.  Per co sub-tile i and pixel
        // sub-tile pair (j, j + 1): bias, bf16 packing, then one v_permlane32_swap and one v_permlane16_swap per
        // packed dword give each lane 8 CONSECUTIVE channels of one pixel (lane rows 0 / 1: tile j, channels 0-7 /
        // 8-15; rows 2 / 3: tile j + 1) -> one 16-B store per lane per pair
        const int lrow = lane >> 4;
        const int hsel = -(lrow >> 1);   // lane rows 2 / 3: the second tile of the pair
#pragma unroll
        for (int i = 0; i < TI; ++i) {
          const float4 bv = *reinterpret_cast<const float4*>(smem + BOFF + bb * BCO * 4 +
                                                             4 * (wco * WT_CO + i * 16 + 4 * lrow));
          const int cg = co0 + wco * WT_CO + i * 16 + 8 * (lrow & 1);   // the lane's first of 8 channels (swapped)
          uint32_t mbyte[TJ / 2];
          uint4 mw[MK == 1 ? TJ / 2 : 1];
#pragma unroll
          for (int jp = 0; jp < TJ / 2; ++jp) {
            const int mo_ = mo[2 * jp] + ((mo[2 * jp + 1] - mo[2 * jp]) & hsel);   // (arithmetic: no indexed mo)
            mbyte[jp] = 0u;
            if constexpr (MK == 2) {
              if (mo_ >= 0 && cg < cout) mbyte[jp] = mkb[(mo_ + cg) >> 3];
            } else if constexpr (MK == 1) {
              mw[jp] = make_uint4(0u, 0u, 0u, 0u);
              if (mo_ >= 0 && cg < cout) mw[jp] = *reinterpret_cast<const uint4*>(Mk + mo_ + cg);
            }
          }
#pragma unroll
          for (int jp = 0; jp < TJ / 2; ++jp) {
            const AccT& A = acc[i][2 * jp];
            const AccT& B = acc[i][2 * jp + 1];
            uint32_t pa[2], pb[2];
            pa[0] = (uint32_t)f2bf(A[0] + bv.x) | ((uint32_t)f2bf(A[1] + bv.y) << 16);
            pa[1] = (uint32_t)f2bf(A[2] + bv.z) | ((uint32_t)f2bf(A[3] + bv.w) << 16);
            pb[0] = (uint32_t)f2bf(B[0] + bv.x) | ((uint32_t)f2bf(B[1] + bv.y) << 16);
            pb[1] = (uint32_t)f2bf(B[2] + bv.z) | ((uint32_t)f2bf(B[3] + bv.w) << 16);
#pragma unroll
            for (int d = 0; d < 2; ++d) {
              // lanes 32-63 of A <-> lanes 0-31 of B, then odd lane rows of A <-> even lane rows of B
              const auto r = __builtin_amdgcn_permlane32_swap(pa[d], pb[d], false, false);
              const auto t = __builtin_amdgcn_permlane16_swap(r[0], r[1], false, false);
              pa[d] = t[0];
              pb[d] = t[1];
            }
            const int mo_ = mo[2 * jp] + ((mo[2 * jp + 1] - mo[2 * jp]) & hsel);   // (arithmetic: no indexed mo)
            if (mo_ < 0 || cg >= cout) continue;
            uint4 m = make_uint4(0u, 0u, 0u, 0u);
            if constexpr (MK == 1) m = mw[jp];
            put8(make_uint4(pa[0], pa[1], pb[0], pb[1]), mo_ + cg, cg, mo_, mbyte[jp], m);
          }
        }
      } else {
#pragma unroll
      for (int i = 0; i < TI; ++i) {
        uint4 mw[TJ][2];
        uint32_t mbyte[TJ][2];
        if constexpr (MK != 0) {
#pragma unroll
          for (int j = 0; j < TJ; ++j)
#pragma unroll
            for (int qp = 0; qp < 2; ++qp) {
              const int cg = co0 + wco * WT_CO + i * 32 + 16 * qp + 8 * fh;
              if constexpr (MK == 2) {
                mbyte[j][qp] = 0u;
                if (mo[j] >= 0 && cg < cout) mbyte[j][qp] = mkb[(mo[j] + cg) >> 3];
              } else {
                mw[j][qp] = make_uint4(0u, 0u, 0u, 0u);
                if (mo[j] >= 0 && cg < cout) mw[j][qp] = *reinterpret_cast<const uint4*>(Mk + mo[j] + cg);
              }
            }
        }
        float4 bv[4];
#pragma unroll
        for (int q = 0; q < 4; ++q)
          bv[q] = *reinterpret_cast<const float4*>(smem + BOFF + bb * BCO * 4 +
                                                   4 * (wco * WT_CO + i * 32 + 8 * q + 4 * fh));
#pragma unroll
        for (int j = 0; j < TJ; ++j) {
          uint32_t pk[4][2];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            pk[q][0] = (uint32_t)f2bf(acc[i][j][4 * q] + bv[q].x) | ((uint32_t)f2bf(acc[i][j][4 * q + 1] + bv[q].y) << 16);
            pk[q][1] = (uint32_t)f2bf(acc[i][j][4 * q + 2] + bv[q].z) | ((uint32_t)f2bf(acc[i][j][4 * q + 3] + bv[q].w) << 16);
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
            const int cg = co0 + wco * WT_CO + i * 32 + 16 * qp + 8 * fh;   // this lane's first of 8 channels
            if (mo[j] < 0 || cg >= cout) continue;
            put8(make_uint4(pk[2 * qp][0], pk[2 * qp][1], pk[2 * qp + 1][0], pk[2 * qp + 1][1]), mo[j] + cg, cg, mo[j],
                 MK == 2 ? mbyte[j][qp] : 0u, MK == 1 ? mw[j][qp] : make_uint4(0u, 0u, 0u, 0u));
          }
        }
      }
      }
    }
    if (!has_next) break;
    // ---- switch to the next tile: its bias into the other buffer, its fragment addressing; its first
    // halo / weight row were issued during the last chunk
    item = nitem;
    co0 = nco0;
#pragma unroll
    for (int v = 0; v < NVO; ++v) wvoff[v] = nwvoff[v];
#pragma unroll
    for (int q = 0; q < H2_HQ; ++q) hsrc[q] = nhsrc[q];
    const float4 bv4 = load_bias(co0);
    decode_frag(item);
    h2_vm_wait<0>();
    store_bias(bb ^ 1, bv4);
    h2_sync();
  }
  h2_vm_wait<0>();   // the last chunk's (unused) DMA lands before the workgroup's LDS is released
  if constexpr (FOC > 0) {   // the block's loss partial (fixed order: deterministic)
    __shared__ float fred[16];
    const float bs = block_sum(foc_acc, fred);
    if (threadIdx.x == 0) fa.partials[blockIdx.x] = bs;
  }
}

template <int BCO, int PERS, int DIAG = 0, int HL = 0, int NWV = 8, int HB1 = 0, int WR3 = 0, int MK = 0, int FOC = 0,
          int BW = 0, int M16 = 0>
int launch_hx32(const bf16_t* X, const bf16_t* Wt, const float* bias, const bf16_t* R, const bf16_t* Mk, bf16_t* Y,
                const bf16_t* zpage, const HaloTile* tiles, int ntiles, const ConvGeom& g, int relu, int accumulate,
                hipStream_t stream, const FocalArgs& fa = FocalArgs{}) {
  const int tiles_co = (g.cout + BCO - 1) / BCO;
  const long long nwork = (long long)tiles_co * ntiles;
  if (nwork > 0x7fffffffLL || nwork < 1) return -3;
  if (PERS && (g.cin / 32) % 2 != 0) return -5;   // the chaining assumes an even chunk count
  const size_t lds = (size_t)(WR3 ? 9 : 6) * BCO * 64 + (HB1 ? 1 : 2) * (size_t)H2_HBYTES + 2 * BCO * 4;
  auto kern = conv3x3_hx32_kernel<BCO, PERS, DIAG, HL, NWV, HB1, WR3, MK, FOC, BW, M16>;
  static bool attr_set = false;
  static int ncu = 0;
  if (!attr_set) {
    hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    int dev = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    if (ncu < 1) ncu = 256;
    attr_set = true;
  }
  // PERS: one block per CU (the LDS allows no second one), each walking tiles b, b + grid, ...
  const long long grid = PERS ? std::min<long long>(nwork, ncu) : nwork;
  kern<<<(unsigned)grid, NWV * 64, lds, stream>>>(X, Wt, bias, R, Mk, Y, zpage, tiles, g, relu, accumulate, tiles_co,
                                                    (int)nwork, fa);
  return (int)hipGetLastError();
}

// OHWI [cout][9][cin] -> [tap][cin / 32][2][cout][16]: one thread per 16 B of output
__global__ void hx32_pack_kernel(const uint4* __restrict__ W, uint4* __restrict__ Wp, int cout, int cin, long long n) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int h = (int)(i & 1);            // 16-B half of the 32-B row
  long long r = i >> 1;
  const int co = (int)(r % cout);
  r /= cout;
  const int p = (int)(r & 1);
  r >>= 1;
  const int nch = cin >> 5;
  const int c = (int)(r % nch);
  const int tap = (int)(r / nch);
  Wp[i] = W[((long long)co * 9 + tap) * (cin >> 3) + c * 4 + p * 2 + h];
}

// Batched form: every hx32-eligible weight of the model (forward copies and flipped data-gradient copies)
// packed by ONE launch per optimizer step.  Segment s packs src[s] (OHWI, cout x 9 x cin) into
// dst + doff[s]; ustart[s] = its first 16-B unit in the launch (prefix sums, ustart[nseg] = total).
struct PackSeg {
  long long src;    // byte address of the OHWI weights
  long long doff;   // element offset in the packed buffer
  long long ustart; // first 16-B unit of this segment
  int cout, cin;
};

__global__ void hx32_pack_batch_kernel(const PackSeg* __restrict__ segs, int nseg, uint4* __restrict__ dst,
                                       long long total) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  int lo = 0, hi = nseg - 1;   // last segment whose ustart <= i
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (segs[mid].ustart <= i) lo = mid; else hi = mid - 1;
  }
  const PackSeg s = segs[lo];
  const long long u = i - s.ustart;
  const int h = (int)(u & 1);
  long long r = u >> 1;
  const int co = (int)(r % s.cout);
  r /= s.cout;
  const int p = (int)(r & 1);
  r >>= 1;
  const int nch = s.cin >> 5;
  const int c = (int)(r % nch);
  const int tap = (int)(r / nch);
  const uint4* W = reinterpret_cast<const uint4*>(s.src);
  dst[s.doff / 8 + u] = W[((long long)co * 9 + tap) * (s.cin >> 3) + c * 4 + p * 2 + h];
}

}  // namespace

MXR_API int mxr_hx32_pack_batch(const void* segs, int nseg, void* dst, long long total_units, hipStream_t stream) {
  if (nseg < 1 || total_units < 1) return -1;
  const long long nb = (total_units + 255) / 256;
  if (nb > 0x7fffffffLL) return -2;
  hx32_pack_batch_kernel<<<(unsigned)nb, 256, 0, stream>>>((const PackSeg*)segs, nseg, (uint4*)dst, total_units);
  return (int)hipGetLastError();
}

MXR_API int mxr_hx32_pack_weights(const void* W, void* Wp, int cout, int cin, hipStream_t stream) {
  if (cin % 32 != 0 || cout < 1) return -1;
  const long long n = (long long)cout * 9 * cin / 8;
  hx32_pack_kernel<<<(unsigned)((n + 255) / 256), 256, 0, stream>>>((const uint4*)W, (uint4*)Wp, cout, cin, n);
  return (int)hipGetLastError();
}

// variant: 0 = 256 co x 256 px (154 KiB LDS), 1 = 128 co x 256 px (105 KiB), 2 / 3 = the same on a
// persistent grid (even chunk count only), 4 / 5 = 0 / 1 with 64-B halo rows (HL 1), 6 = 1 with one halo
// buffer (77 KiB, two blocks per CU), 7 = 1 with a three-slot weight ring fetched two stages ahead (129 KiB).
// (A plane-sequenced one-halo-buffer form with role-split DMA -- three half-stages of halo lead in one buffer --
// ran level with variant 6 in isolation and 0.5 % slower in the step: profiles/r4_hx32_plane_sequenced.txt,
// profiles/r4_ab_hx32_8.txt; removed.)
// 100 + DIAG = timing-only
// builds of variant 2, compiled only into the diagnostic library (MXR_DIAG_KERNELS; MXR_KERNEL_LIB=<that .so>).  (The 4-wave form, NWV 4, measured 5-15 % slower than 8 waves on every head shape:
// profiles/r3_hx32_variants.txt.)
// Wt: the weights PACKED by mxr_hx32_pack_weights.  Requires a 3x3 / stride-1 / pad-1 geometry with
// equal input / output levels, cin % 32 == 0, cout % 8 == 0, the tile table of ops/halo.py,
// (pixels + 1) * max(cin, cout) < 2^31 and cout * 9 * cin * 2 < 2^31 (the weight buffer descriptor).
MXR_API int mxr_conv3x3_hx32(const void* X, const void* Wt, const float* bias, const void* R, const void* Mk,
                             void* Y, const void* zpage, const ConvGeom* g, const void* tiles, int ntiles, int relu,
                             int accumulate, int variant, hipStream_t stream) {
  if (g->cin % 32 != 0 || g->cout % 8 != 0) return -1;
  if (g->kh != 3 || g->kw != 3 || g->stride != 1 || g->pt != 1 || g->pl != 1 || g->ostride != 1) return -2;
  if (g->in_img != g->out_img || (g->M + 1) * (long long)std::max(g->cin, g->cout) >= (1LL << 31)) return -4;
  if ((long long)g->cout * 9 * g->cin * 2 >= (1LL << 31)) return -4;
  const bf16_t *x = (const bf16_t*)X, *w = (const bf16_t*)Wt, *r = (const bf16_t*)R, *mk = (const bf16_t*)Mk;
  const bf16_t* z = (const bf16_t*)zpage;
  const HaloTile* t = (const HaloTile*)tiles;
  bf16_t* y = (bf16_t*)Y;
  // the masked data gradient of the winning variants (0, 6) runs the compile-time masked epilogue (bf16 mask or
  // bitmask), the plain relu forward writing a bitmask its compile-time form (BW)
  const bool bits = mk != nullptr && ((uintptr_t)mk & 1);
  const bool mk_fast = mk != nullptr && r == nullptr && !accumulate && !relu;
  if (mk_fast && variant == 0 && !bits)
    return launch_hx32<256, 0, 0, 0, 8, 0, 0, 1>(x, w, bias, r, mk, y, z, t, ntiles, *g, relu, accumulate, stream);
  if (mk_fast && variant == 6 && !bits)
    return launch_hx32<128, 0, 0, 0, 8, 1, 0, 1>(x, w, bias, r, mk, y, z, t, ntiles, *g, relu, accumulate, stream);
  if (mk_fast && variant == 0 && bits)
    return launch_hx32<256, 0, 0, 0, 8, 0, 0, 2>(x, w, bias, r, mk, y, z, t, ntiles, *g, relu, accumulate, stream);
  if (mk_fast && variant == 6 && bits)
    return launch_hx32<128, 0, 0, 0, 8, 1, 0, 2>(x, w, bias, r, mk, y, z, t, ntiles, *g, relu, accumulate, stream);
  if (mk_fast && variant == 10 && !bits)
    return launch_hx32<256, 0, 0, 0, 8, 0, 0, 1, 0, 0, 1>(x, w, bias, r, mk, y, z, t, ntiles, *g, relu, accumulate, stream);
  if (mk_fast && variant == 10 && bits)
    return launch_hx32<256, 0, 0, 0, 8, 0, 0, 2, 0, 0, 1>(x, w, bias, r, mk, y, z, t, ntiles, *g, relu, accumulate, stream);
  if (mk_fast && variant == 11 && !bits)
    return launch_hx32<128, 0, 0, 0, 8, 1, 0, 1, 0, 0, 1>(x, w, bias, r, mk, y, z, t, ntiles, *g, relu, accumulate, stream);
  if (mk_fast && variant == 11 && bits)
    return launch_hx32<128, 0, 0, 0, 8, 1, 0, 2, 0, 0, 1>(x, w, bias, r, mk, y, z, t, ntiles, *g, relu, accumulate, stream);
  const bool bw_fast = bits && relu && r == nullptr && !accumulate;
  if (bw_fast && variant == 0)
    return launch_hx32<256, 0, 0, 0, 8, 0, 0, 0, 0, 1>(x, w, bias, r, mk, y, z, t, ntiles, *g, relu, accumulate, stream);
  if (bw_fast && variant == 6)
    return launch_hx32<128, 0, 0, 0, 8, 1, 0, 0, 0, 1>(x, w, bias, r, mk, y, z, t, ntiles, *g, relu, accumulate, stream);
  if (bw_fast && variant == 10)
    return launch_hx32<256, 0, 0, 0, 8, 0, 0, 0, 0, 1, 1>(x, w, bias, r, mk, y, z, t, ntiles, *g, relu, accumulate, stream);
  if (bw_fast && variant == 11)
    return launch_hx32<128, 0, 0, 0, 8, 1, 0, 0, 0, 1, 1>(x, w, bias, r, mk, y, z, t, ntiles, *g, relu, accumulate, stream);
  switch (variant) {
    case 0: return launch_hx32<256, 0>(x, w, bias, r, mk, y, z, t, ntiles, *g, relu, accumulate, stream);
    case 1: return launch_hx32<128, 0>(x, w, bias, r, mk, y, z, t, ntiles, *g, relu, accumulate, stream);
    case 2: return launch_hx32<256, 1>(x, w, bias, r, mk, y, z, t, ntiles, *g, relu, accumulate, stream);
    case 3: return launch_hx32<128, 1>(x, w, bias, r, mk, y, z, t, ntiles, *g, relu, accumulate, stream);
    case 4: return launch_hx32<256, 0, 0, 1>(x, w, bias, r, mk, y, z, t, ntiles, *g, relu, accumulate, stream);
    case 5: return launch_hx32<128, 0, 0, 1>(x, w, bias, r, mk, y, z, t, ntiles, *g, relu, accumulate, stream);
    case 6: return launch_hx32<128, 0, 0, 0, 8, 1>(x, w, bias, r, mk, y, z, t, ntiles, *g, relu, accumulate, stream);
    case 7: return launch_hx32<128, 0, 0, 0, 8, 0, 1>(x, w, bias, r, mk, y, z, t, ntiles, *g, relu, accumulate, stream);
    // 64-channel tiles for the narrow layers (the 64-padded regression final, the stage-2 64 -> 64 convs): 4 waves
    // (2 co x 2 px, 32 x 128 per wave); 9 with one halo buffer (53 KiB: three blocks share a CU)
    case 8: return launch_hx32<64, 0, 0, 0, 4>(x, w, bias, r, mk, y, z, t, ntiles, *g, relu, accumulate, stream);
    case 9: return launch_hx32<64, 0, 0, 0, 4, 1>(x, w, bias, r, mk, y, z, t, ntiles, *g, relu, accumulate, stream);
    // 10 / 11 / 12: variants 0 / 6 / 1 on the 16x16x32 MFMA (M16: unswizzled plane images, one K = 32 step per tap)
    case 10: return launch_hx32<256, 0, 0, 0, 8, 0, 0, 0, 0, 0, 1>(x, w, bias, r, mk, y, z, t, ntiles, *g, relu, accumulate, stream);
    case 11: return launch_hx32<128, 0, 0, 0, 8, 1, 0, 0, 0, 0, 1>(x, w, bias, r, mk, y, z, t, ntiles, *g, relu, accumulate, stream);
    case 12: return launch_hx32<128, 0, 0, 0, 8, 0, 0, 0, 0, 0, 1>(x, w, bias, r, mk, y, z, t, ntiles, *g, relu, accumulate, stream);
    // 13 / 14 / 15: the persistent grids 2 / 3 and the three-slot weight ring 7 on the 16x16x32 MFMA
    case 13: return launch_hx32<256, 1, 0, 0, 8, 0, 0, 0, 0, 0, 1>(x, w, bias, r, mk, y, z, t, ntiles, *g, relu, accumulate, stream);
    case 14: return launch_hx32<128, 1, 0, 0, 8, 0, 0, 0, 0, 0, 1>(x, w, bias, r, mk, y, z, t, ntiles, *g, relu, accumulate, stream);
    case 15: return launch_hx32<128, 0, 0, 0, 8, 0, 1, 0, 0, 0, 1>(x, w, bias, r, mk, y, z, t, ntiles, *g, relu, accumulate, stream);
    // (the 64-channel tiles on the 16x16x32 MFMA measured 6 % faster than variant 8 but 10 % slower than 9 -- its
    // one-halo-buffer form spills at 168 VGPRs: profiles/r6_hx32_m16_ab.txt; not built)
#ifdef MXR_DIAG_KERNELS   // timing-only builds: _lib/diag/libmxr_kernels.so (build.py --diag), never the production library
    case 101: return launch_hx32<256, 1, 1>(x, w, bias, r, mk, y, z, t, ntiles, *g, relu, accumulate, stream);
    case 102: return launch_hx32<256, 1, 2>(x, w, bias, r, mk, y, z, t, ntiles, *g, relu, accumulate, stream);
    case 103: return launch_hx32<256, 1, 3>(x, w, bias, r, mk, y, z, t, ntiles, *g, relu, accumulate, stream);
    case 108: return launch_hx32<256, 1, 8>(x, w, bias, r, mk, y, z, t, ntiles, *g, relu, accumulate, stream);
    case 111: return launch_hx32<256, 1, 11>(x, w, bias, r, mk, y, z, t, ntiles, *g, relu, accumulate, stream);
    case 132: return launch_hx32<256, 0, 32>(x, w, bias, r, mk, y, z, t, ntiles, *g, relu, accumulate, stream);
    case 116: return launch_hx32<256, 0, 16>(x, w, bias, r, mk, y, z, t, ntiles, *g, relu, accumulate, stream);
    case 126: return launch_hx32<128, 0, 16, 0, 8, 1>(x, w, bias, r, mk, y, z, t, ntiles, *g, relu, accumulate, stream);
    // bit 6: every 32x32x16 MFMA as two 16x16x32 on the same operands (same FLOPs; the shape's sustained clock)
    case 164: return launch_hx32<256, 0, 64>(x, w, bias, r, mk, y, z, t, ntiles, *g, relu, accumulate, stream);
    case 170: return launch_hx32<128, 0, 64, 0, 8, 1>(x, w, bias, r, mk, y, z, t, ntiles, *g, relu, accumulate, stream);
#endif
    default: return -6;
  }
}

void mxr_loss_finalize_launch(const float* partials, int n, const int* npos, float* out, hipStream_t stream);

// The classification final of the packed heads with the sigmoid-focal loss fused into its epilogue (variant 0's
// tiles: 256 output channels, two halo buffers): no logits are written; dpad (pixels x ld bf16, columns past A * 80
// untouched -- zero) receives d(loss)/d(logits) and *out the loss (sum / max(1, *npos), finalised from one partial
// per block in fixed order: partials must hold ceil(cout / 256) * ntiles floats).  State / label per anchor row
// (pixel * A + anchor), the Keras clip as logit bounds lo / hi; gamma == 2 and 80 classes (COCO) only.  variant: 0 or
// 10 (the same tiles on the 16x16x32 MFMA).
MXR_API int mxr_conv3x3_hx32_focal_v(const void* X, const void* Wt, const float* bias, const void* zpage,
                                     const ConvGeom* g, const void* tiles, int ntiles, const int8_t* state,
                                     const int32_t* label, const int* npos, void* dpad, int ld, int A, int C, float alpha,
                                     float gamma, float lo, float hi, float* partials, int nparts, float* out, int variant,
                                     hipStream_t stream) {
  if (g->cin % 32 != 0 || g->cout % 8 != 0) return -1;
  if (g->kh != 3 || g->kw != 3 || g->stride != 1 || g->pt != 1 || g->pl != 1 || g->ostride != 1) return -2;
  if (g->in_img != g->out_img || (g->M + 1) * (long long)std::max(g->cin, g->cout) >= (1LL << 31)) return -4;
  if ((long long)g->cout * 9 * g->cin * 2 >= (1LL << 31)) return -4;
  if (C != 80 || gamma != 2.0f || A * C != g->cout || ld < g->cout || ld % 8 != 0) return -8;
  const long long nwork = (long long)((g->cout + 255) / 256) * ntiles;
  if (nparts < nwork || (long long)g->M * ld >= (1LL << 31)) return -9;
  const FocalArgs fa{state, label, npos, (bf16_t*)dpad, partials, ld, A, alpha, gamma, lo, hi};
  if (variant != 0 && variant != 10) return -6;
  const int rc =
      variant == 10
          ? launch_hx32<256, 0, 0, 0, 8, 0, 0, 0, 80, 0, 1>((const bf16_t*)X, (const bf16_t*)Wt, bias, nullptr, nullptr,
                                                            nullptr, (const bf16_t*)zpage, (const HaloTile*)tiles,
                                                            ntiles, *g, 0, 0, stream, fa)
          : launch_hx32<256, 0, 0, 0, 8, 0, 0, 0, 80>((const bf16_t*)X, (const bf16_t*)Wt, bias, nullptr, nullptr,
                                                      nullptr, (const bf16_t*)zpage, (const HaloTile*)tiles,
                                                      ntiles, *g, 0, 0, stream, fa);
  if (rc) return rc;
  mxr_loss_finalize_launch(partials, (int)nwork, npos, out, stream);
  return (int)hipGetLastError();
}

// variant 0 (the 32x32x16 tiles): the original entry point
MXR_API int mxr_conv3x3_hx32_focal(const void* X, const void* Wt, const float* bias, const void* zpage,
                                   const ConvGeom* g, const void* tiles, int ntiles, const int8_t* state,
                                   const int32_t* label, const int* npos, void* dpad, int ld, int A, int C, float alpha,
                                   float gamma, float lo, float hi, float* partials, int nparts, float* out,
                                   hipStream_t stream) {
  return mxr_conv3x3_hx32_focal_v(X, Wt, bias, zpage, g, tiles, ntiles, state, label, npos, dpad, ld, A, C, alpha, gamma,
                                  lo, hi, partials, nparts, out, 0, stream);
}
