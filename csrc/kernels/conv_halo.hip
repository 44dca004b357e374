// Halo-staged 3x3 / stride-1 / pad-1 NHWC bf16 convolution (forward and stride-1 data-gradient) for gfx950.
//
// The hot 3x3 layers of the model -- the eight head-tower layers and the two head finals over the packed
// five-level pyramid (58.9 % of the forward MACs), the FPN P3-P5 smoothing convs and
// the backbone 3x3 convs (the conv layers the reference builds at /root/reference/train.py:91) -- are
// implicit GEMMs whose pixel operand is the 9-tap im2col of the input.  conv_pipe.hip streams that
// operand through LDS once per tap: every input pixel is fetched 9 times per 32-channel chunk, and the
// LDS-DMA issue cost of those pieces (~100-185 cycles per 1 KiB piece inside an MFMA phase,
// MI355X_MICROARCH.md) is what bounds that kernel (profiles/r1_ablate_head_fwd.log: the DMA + barrier
// skeleton alone runs at 70 % of the full kernel's time).
//
// Here a tile is a set of up to 4 rectangular "boxes" of output pixels (R rows x C columns of one image
// and pyramid level, <= 256 output slots in total, built on the host: ops/halo.py).  Per 32-channel input
// chunk the block stages the boxes' HALOS -- (R + 2) x (C + 2) input pixels, zero outside the level --
// ONCE into LDS, and every tap reads its B fragments from that image at a per-tap shifted address.
// Pixel traffic drops from 9 x 256 to <= 448 rows per chunk; only the weight operand is streamed.
//
// * tile = BCO output channels x 256 pixel slots, 8 waves as 2 (co) x 4 (pixels), MFMA 16x16x32 bf16;
// * a sub-stage is TPS taps (1, or 3 = one kernel row) of one 32-channel chunk: the weight pieces of a
//   sub-stage go into an NS-deep LDS ring; the halo has two buffers (448 x 64 B each), the next chunk's
//   halo is fetched during the current chunk;
// * halo rows are 64 B (32 channels); the 16-B chunk index is XOR-swizzled by the pixel's halo COLUMN
//   ((col / 4) mod 4 -> [0, 2, 3, 1]) so a fragment read (16 consecutive columns of one box row, aligned)
//   hits 16 distinct bank slots; the swizzle is applied to the DMA source address, the LDS image stays
//   lane-linear (LDS-DMA writes lane l at base + 16 l);
// * the pipeline never drains inside the loop: counted `s_waitcnt vmcnt(N)` (N a compile-time function of
//   the sub-stage, see hx_younger) + raw `s_barrier`; past the last chunk the DMA keeps its uniform shape
//   by loading the zero page into slots nobody reads any more, and the epilogue waits vmcnt(0) before it
//   reuses the LDS.
#include <type_traits>

#include "common.h"

#include "conv_common.h"
#include "halo_tile.h"

namespace {

constexpr int HX_NW = 8;                                      // waves per block
constexpr int HX_NQ = (HX_HMAX + 16 * HX_NW - 1) / (16 * HX_NW);   // halo pieces per wave per chunk (4)
constexpr int HX_HBYTES = HX_HMAX * 64;                       // one halo buffer

__device__ __forceinline__ int hx_swz(int col) { return (120 >> (2 * ((col >> 2) & 3))) & 3; }   // [0,2,3,1]

template <int N>
__device__ __forceinline__ void hx_vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// Halo piece q (of HX_NQ per wave and chunk) is issued at local sub-stage hx_pos(q) of the PREVIOUS chunk;
// positions stay <= SPC - NS so every piece is older than the weight DMA of the next chunk's first
// sub-stage (issued at local sub-stage SPC - NS + 1), whose counted wait therefore covers it.
template <int NS, int SPC>
constexpr int hx_pos(int q) { return (q * (SPC - NS + 1)) / HX_NQ; }
template <int NS, int SPC>
constexpr int hx_hq(int u) {
  int n = 0;
  for (int q = 0; q < HX_NQ; ++q) n += hx_pos<NS, SPC>(q) == u ? 1 : 0;
  return n;
}
// DMA instructions of this wave younger than the weight pieces of the sub-stage at local index t.
// Issue order per sub-stage: NWP weight pieces of sub-stage s + NS - 1, then the halo pieces placed at
// that sub-stage; prologue: the halo of chunk 0, then the weights of sub-stages 0 .. NS - 2 (consistent
// with the formula because no halo piece sits at a local index > SPC - NS).
template <int NS, int SPC, int NWP>
constexpr int hx_younger(int t) {
  int n = hx_hq<NS, SPC>((((t - NS + 1) % SPC) + SPC) % SPC);
  for (int k = 1; k <= NS - 2; ++k) n += NWP + hx_hq<NS, SPC>((((t - k) % SPC) + SPC) % SPC);
  return n;
}

template <int I, int N, typename F>
__device__ __forceinline__ void hx_static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    hx_static_for<I + 1, N>(f);
  }
}

// MINW: waves per SIMD the register budget must allow (4 = two 8-wave blocks per CU, <= 128 VGPRs)
// SCHED: 0 = compiler schedule, 1 = fragment reads pinned ahead of the MFMAs (sched_group_barrier),
// 2 = 1 + the sub-stage's MFMAs kept above the next barrier
// RF: the sub-stage's fragment reads are issued before its DMA pieces (the LDS read latency then
// overlaps the DMA issue instead of following it)
template <int BCO, int NS, int TPS, int MINW, bool PF, int SCHED, int RF = 0>
__global__ __launch_bounds__(HX_NW * 64, MINW) void conv3x3_halo_kernel(
    const bf16_t* __restrict__ X, const bf16_t* __restrict__ Wt, const float* __restrict__ bias,
    const bf16_t* __restrict__ Rs, const bf16_t* __restrict__ Mk, bf16_t* __restrict__ Y,
    const bf16_t* __restrict__ zpage, const HaloTile* __restrict__ tiles, ConvGeom g, int relu, int accumulate,
    int tiles_co) {
  constexpr int NW = HX_NW, WCO = 2, WPX = NW / WCO;
  constexpr int NSA = BCO / (16 * NW);          // weight pieces per wave per tap
  static_assert(NSA * 16 * NW == BCO, "weight rows must split evenly over the waves");
  constexpr int SPC = 9 / TPS;                  // sub-stages per chunk
  static_assert(SPC * TPS == 9, "taps per sub-stage");
  constexpr int NWP = NSA * TPS;                // weight pieces per wave per sub-stage
  constexpr int WT_CO = BCO / WCO, WT_PIX = HX_PB / WPX;
  constexpr int TI = WT_CO / 16, TJ = WT_PIX / 16;
  constexpr int WTAP = BCO * 64;                // bytes of one tap's weight tile
  constexpr int WST = TPS * WTAP;               // bytes per weight sub-stage
  constexpr int HOFF = NS * WST;                // halo buffers follow the ring
  static_assert(NS >= 2 && NS <= SPC, "ring depth");
  static_assert(NWP + 2 * HX_NQ <= 63, "vmcnt range");

  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // SGPR: every DMA base is scalar
  const int wid = xcd_remap(blockIdx.x, gridDim.x);
  const int tco = wid % tiles_co;
  const int tm = wid / tiles_co;
  const int co0 = tco * BCO;
  const HaloTile& T = tiles[tm];
  const int cin = g.cin;
  const int K = 9 * cin;
  const int nch = cin >> 5;
  const int rloc = lane >> 2;

  // ---- weight DMA descriptors: rows co0 + (s * NW + wave) * 16 + lane / 4, swizzled 16-B chunk
  const int clw = (lane & 3) ^ ((120 >> (2 * (rloc >> 2))) & 3);
  const bf16_t* wsrc[NSA];
#pragma unroll
  for (int s = 0; s < NSA; ++s) {
    const int co = co0 + (s * NW + wave) * 16 + rloc;
    wsrc[s] = co < g.cout ? Wt + (long long)co * K + clw * 8 : nullptr;
  }
  int wu_tap = 0, wu_c0 = 0, wu_slot = 0;       // next weight sub-stage to issue
  auto issue_w = [&]() {
    char* dst = smem + wu_slot * WST;
    const bool ok = wu_c0 < cin;
#pragma unroll
    for (int kk = 0; kk < TPS; ++kk) {
#pragma unroll
      for (int s = 0; s < NSA; ++s) {
        const uintptr_t a = (wsrc[s] && ok) ? (uintptr_t)(wsrc[s] + (wu_tap + kk) * cin + wu_c0) : (uintptr_t)zpage;
        glds16((const void*)a, dst + kk * WTAP + (s * NW + wave) * 1024);
      }
    }
    wu_tap += TPS;
    if (wu_tap == 9) { wu_tap = 0; wu_c0 += 32; }
    if (++wu_slot == NS) wu_slot = 0;
  };

  // ---- halo DMA descriptors: piece q of this wave = halo rows (q * NW + wave) * 16 .. + 15; a piece past
  // HX_HMAX repeats the previous piece (same source, same destination) so every wave issues HX_NQ
  auto hpiece = [&](int q) { return ((q * NW + wave) * 16 >= HX_HMAX) ? q - 1 : q; };   // wave-uniform
  int hsrc[HX_NQ];
#pragma unroll
  for (int q = 0; q < HX_NQ; ++q) {
    const int qe = hpiece(q);
    const int h = (qe * NW + wave) * 16 + rloc;
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
        off = (ib + y * W + x) * cin + (((lane & 3) ^ hx_swz(hc)) << 3);
    }
    hsrc[q] = off;
  }
  auto issue_halo = [&](int q, int c) {
    char* dst = smem + HOFF + (c & 1) * HX_HBYTES + (hpiece(q) * NW + wave) * 1024;
    const uintptr_t a =
        (hsrc[q] >= 0 && c < nch) ? (uintptr_t)(X + (long long)hsrc[q] + c * 32) : (uintptr_t)zpage;
    glds16((const void*)a, dst);
  };

  // ---- B-fragment addressing: lane's pixel slot p = wpx * 64 + j * 16 + lane % 16, chunk lane / 16;
  // slots past nslot read halo row 0 (finite data, results discarded)
  const int wco = wave / WPX, wpx = wave % WPX;
  // per fragment: byte offset of tap (0, 0), and packed {swizzle term of kx = 0, 1, 2 (6 bits each),
  // halo row pitch in pixels (bits 18+)}
  int hb64[TJ], swp[TJ];
#pragma unroll
  for (int j = 0; j < TJ; ++j) {
    const int p = wpx * WT_PIX + j * 16 + (lane & 15);
    HX_SELECT(sbeg, p)
    int sb = T.b[0].sbeg, ho = T.b[0].hoff, C = T.b[0].C;
#pragma unroll
    for (int t = 1; t < HX_BOX; ++t)
      if (sel == t) { sb = T.b[t].sbeg; ho = T.b[t].hoff; C = T.b[t].C; }
    int r = 0, c = 0;
    if (p < T.nslot) {
      const int loc = p - sb;
      r = fdiv(loc, C);
      c = loc - r * C;
    } else {
      ho = 0;
      C = 0;
    }
    const int pw = C + 2;
    hb64[j] = (ho + r * pw + c) * 64;
    const int ch = lane >> 4;
    swp[j] = (ch ^ hx_swz(c)) | ((ch ^ hx_swz(c + 1)) << 6) | ((ch ^ hx_swz(c + 2)) << 12) | (pw << 18);
  }
  // A fragment: row lane % 16 of a 16-row block, logical chunk lane / 16 (conv_pipe.hip layout)
  const int foff = (lane & 15) * 64 + (((lane >> 4) ^ ((120 >> (2 * ((lane & 15) >> 2))) & 3)) << 4);
  const int aoff = wco * WT_CO * 64 + foff;

  f32x4 acc[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto read_b = [&](bf16x8* bfr, const char* hbuf, int ky, int kx) {
#pragma unroll
    for (int j = 0; j < TJ; ++j)
      bfr[j] = *reinterpret_cast<const bf16x8*>(hbuf + hb64[j] + ky * ((swp[j] >> 18) << 6) +
                                                (((swp[j] >> (6 * kx)) & 3) << 4) + kx * 64);
  };
  auto read_a = [&](bf16x8* af, const char* wtap) {
#pragma unroll
    for (int i = 0; i < TI; ++i) af[i] = *reinterpret_cast<const bf16x8*>(wtap + aoff + i * 1024);
  };

  if constexpr (PF) {
    // ---- register-prefetch pipeline (TPS = 1): the fragments of sub-stage i + 1 are read right after
    // barrier i, behind the MFMAs of sub-stage i (whose operands are already in registers), so no MFMA
    // waits on an LDS read.  The DMA runs NS sub-stages ahead of the MFMAs (one more than the reads):
    // prologue = halo of chunk 0 + weights of sub-stages 0 .. NS - 1; iteration i issues sub-stage
    // i + NS into the slot of sub-stage i, whose fragments are in registers by then.  The counted waits
    // keep the hx_younger shape (the wait at iteration i retires the weights of sub-stage i + 1).
    static_assert(TPS == 1, "prefetch pipeline: one tap per sub-stage");
#pragma unroll
    for (int q = 0; q < HX_NQ; ++q) issue_halo(q, 0);
#pragma unroll
    for (int k = 0; k < NS; ++k) issue_w();
    hx_vm_wait<(NS - 1) * NWP>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    bf16x8 ca[TI], cb[TJ];
    read_a(ca, smem);
    read_b(cb, smem + HOFF, 0, 0);
    int rs = 0;
    for (int c = 0; c < nch; ++c) {
      const char* hb = smem + HOFF + (c & 1) * HX_HBYTES;
      const char* hbn = smem + HOFF + ((c + 1) & 1) * HX_HBYTES;
      hx_static_for<0, 9>([&](auto tc) {
        constexpr int t = decltype(tc)::value;
        hx_vm_wait<hx_younger<NS, 9, NWP>(t)>();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        auto dma = [&]() {
          issue_w();
          hx_static_for<0, HX_NQ>([&](auto qc) {
            constexpr int q = decltype(qc)::value;
            if constexpr (hx_pos<NS, 9>(q) == t) issue_halo(q, c + 1);
          });
        };
        if constexpr (!RF) dma();
        const int rn = (rs + 1 == NS) ? 0 : rs + 1;
        bf16x8 na[TI], nb[TJ];
        constexpr int tn = (t + 1) % 9;
        read_b(nb, t == 8 ? hbn : hb, tn / 3, tn % 3);   // past the last chunk: zero-page data, unused
        read_a(na, smem + rn * WST);
        if constexpr (RF) dma();
#pragma unroll
        for (int i = 0; i < TI; ++i)
#pragma unroll
          for (int j = 0; j < TJ; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ca[i], cb[j], acc[i][j], 0, 0, 0);
#pragma unroll
        for (int i = 0; i < TI; ++i) ca[i] = na[i];
#pragma unroll
        for (int j = 0; j < TJ; ++j) cb[j] = nb[j];
        rs = rn;
      });
    }
  } else {
  // ---- prologue: halo of chunk 0, then the weights of sub-stages 0 .. NS - 2
#pragma unroll
  for (int q = 0; q < HX_NQ; ++q) issue_halo(q, 0);
#pragma unroll
  for (int k = 0; k < NS - 1; ++k) issue_w();

  int rs = 0;   // ring slot of the sub-stage being consumed
  for (int c = 0; c < nch; ++c) {
    const char* hb = smem + HOFF + (c & 1) * HX_HBYTES;
    hx_static_for<0, SPC>([&](auto tc) {
      constexpr int t = decltype(tc)::value;
      hx_vm_wait<hx_younger<NS, SPC, NWP>(t)>();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      auto dma = [&]() {
        issue_w();
        hx_static_for<0, HX_NQ>([&](auto qc) {
          constexpr int q = decltype(qc)::value;
          if constexpr (hx_pos<NS, SPC>(q) == t) issue_halo(q, c + 1);
        });
      };
      if constexpr (!RF) dma();
      const char* ws = smem + rs * WST;
      // all fragment reads of a tap are issued before its MFMAs (and those of tap kk + 1 before the MFMAs
      // of tap kk): left alone, the scheduler keeps two A fragments live and waits lgkmcnt(0) every
      // 8 MFMAs, exposing the LDS latency four times per sub-stage
      if constexpr (SCHED == 3) {
        // one fragment set live (no next-tap prefetch): the partner wave on the SIMD covers the LDS
        // latency; keeps the 256-channel, 3-tap sub-stage inside 256 VGPRs
        if constexpr (RF) dma();
        hx_static_for<0, TPS>([&](auto kc) {
          constexpr int kk = decltype(kc)::value;
          constexpr int tt = t * TPS + kk;
          bf16x8 fa1[TI], fb1[TJ];
          read_b(fb1, hb, tt / 3, tt % 3);
          read_a(fa1, ws + kk * WTAP);
#pragma unroll
          for (int i = 0; i < TI; ++i)
#pragma unroll
            for (int j = 0; j < TJ; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa1[i], fb1[j], acc[i][j], 0, 0, 0);
        });
        rs = (rs + 1 == NS) ? 0 : rs + 1;
        return;
      }
      bf16x8 fa[2][TI], fb[2][TJ];
      read_b(fb[0], hb, (t * TPS) / 3, (t * TPS) % 3);
      read_a(fa[0], ws);
      if constexpr (SCHED >= 1) __builtin_amdgcn_sched_group_barrier(0x0100, TI + TJ, 0);
      if constexpr (RF) dma();
      hx_static_for<0, TPS>([&](auto kc) {
        constexpr int kk = decltype(kc)::value;
        if constexpr (kk + 1 < TPS) {
          constexpr int tn = t * TPS + kk + 1;
          read_b(fb[(kk + 1) & 1], hb, tn / 3, tn % 3);
          read_a(fa[(kk + 1) & 1], ws + (kk + 1) * WTAP);
          if constexpr (SCHED >= 1) __builtin_amdgcn_sched_group_barrier(0x0100, TI + TJ, 0);
        }
#pragma unroll
        for (int i = 0; i < TI; ++i)
#pragma unroll
          for (int j = 0; j < TJ; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[kk & 1][i], fb[kk & 1][j], acc[i][j], 0, 0, 0);
        if constexpr (SCHED >= 1) __builtin_amdgcn_sched_group_barrier(0x0008, TI * TJ, 0);
      });
      if constexpr (SCHED == 2) {
        // keep this sub-stage's MFMAs above the next wait + barrier (no sinking across it)
#pragma unroll
        for (int i = 0; i < TI; ++i)
#pragma unroll
          for (int j = 0; j < TJ; ++j) asm volatile("" ::"v"(acc[i][j]));
      }
      rs = (rs + 1 == NS) ? 0 : rs + 1;
    });
  }
  }

  // ---- epilogue (conv_pipe.hip's two passes): fragments -> LDS image [256 slots][BCO] -> 16-B sweeps
  constexpr int PITCH = BCO * 2 + 16;
  hx_vm_wait<0>();   // the tail's zero-page DMA must land before the LDS is reused
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __syncthreads();
  // the bias of this lane's TI channel groups, loaded together (a load per fragment, each waited on
  // before its use, cost ~0.5 us apiece)
  float4 bv[TI];
#pragma unroll
  for (int i = 0; i < TI; ++i) bv[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  if (bias) {                    // (channels past cout read a valid bias entry; their outputs are not stored)
#pragma unroll
    for (int i = 0; i < TI; ++i)
      bv[i] = *reinterpret_cast<const float4*>(bias + min(co0 + wco * WT_CO + i * 16 + 4 * (lane >> 4), g.cout - 4));
  }
#pragma unroll
  for (int j = 0; j < TJ; ++j) {
    const int pr = wpx * WT_PIX + j * 16 + (lane & 15);
#pragma unroll
    for (int i = 0; i < TI; ++i) {
      const int cl = wco * WT_CO + i * 16 + 4 * (lane >> 4);
      float v[4] = {acc[i][j][0] + bv[i].x, acc[i][j][1] + bv[i].y, acc[i][j][2] + bv[i].z, acc[i][j][3] + bv[i].w};
      uint2 o;
      o.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
      o.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
      *reinterpret_cast<uint2*>(smem + pr * PITCH + cl * 2) = o;
    }
  }
  __syncthreads();
  constexpr int CPR = BCO / 8;
  const int ncv = min(BCO, g.cout - co0) / 8;
  // the tile's box fields, read once outside the sweep's divergent loop (inside it hipcc turned every
  // field read into a vector load waited on with vmcnt(0), per 16-B chunk)
  int e_sb[HX_BOX], e_ob[HX_BOX], e_w[HX_BOX], e_y0[HX_BOX], e_x0[HX_BOX], e_c[HX_BOX];
#pragma unroll
  for (int t = 0; t < HX_BOX; ++t) {
    e_sb[t] = T.b[t].sbeg; e_ob[t] = T.b[t].out_base; e_w[t] = T.b[t].W;
    e_y0[t] = T.b[t].y0; e_x0[t] = T.b[t].x0; e_c[t] = T.b[t].C;
  }
  const int e_nbox = T.nbox, e_nslot = T.nslot;
  for (int e = threadIdx.x; e < HX_PB * CPR; e += NW * 64) {
    const int pr = e / CPR, ch = e - pr * CPR;
    if (pr >= e_nslot || ch >= ncv) continue;
    int sb = e_sb[0], ob = e_ob[0], W = e_w[0], y0 = e_y0[0], x0 = e_x0[0], C = e_c[0];
#pragma unroll
    for (int t = 1; t < HX_BOX; ++t) {
      const bool in = t < e_nbox && pr >= e_sb[t];
      sb = in ? e_sb[t] : sb; ob = in ? e_ob[t] : ob; W = in ? e_w[t] : W;
      y0 = in ? e_y0[t] : y0; x0 = in ? e_x0[t] : x0; C = in ? e_c[t] : C;
    }
    const int loc = pr - sb;
    const int r = fdiv(loc, C), c = loc - r * C;
    const long long m = (long long)ob + (long long)(y0 + r) * W + x0 + c;
    const long long off = m * g.cout + co0 + ch * 8;
    const uint4 raw = *reinterpret_cast<const uint4*>(smem + pr * PITCH + ch * 16);
    const uint32_t rw[4] = {raw.x, raw.y, raw.z, raw.w};
    float v[8];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      v[2 * q] = bf2f((bf16_t)(rw[q] & 0xffff));
      v[2 * q + 1] = bf2f((bf16_t)(rw[q] >> 16));
    }
    epi_sweep8(v, Rs, off, accumulate ? Y : nullptr, Mk, off, relu);
    uint4 o;
    o.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
    o.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
    o.z = (uint32_t)f2bf(v[4]) | ((uint32_t)f2bf(v[5]) << 16);
    o.w = (uint32_t)f2bf(v[6]) | ((uint32_t)f2bf(v[7]) << 16);
    *reinterpret_cast<uint4*>(Y + off) = o;
  }
}

template <int BCO, int NS, int TPS, int MINW, bool PF = false, int SCHED = 1, int RF = 0>
int launch_halo(const bf16_t* X, const bf16_t* Wt, const float* bias, const bf16_t* R, const bf16_t* Mk, bf16_t* Y,
                const bf16_t* zpage, const HaloTile* tiles, int ntiles, const ConvGeom& g, int relu, int accumulate,
                hipStream_t stream) {
  const int tiles_co = (g.cout + BCO - 1) / BCO;
  const long long nwg = (long long)tiles_co * ntiles;
  if (nwg > 0x7fffffffLL || nwg < 1) return -3;
  const size_t lds =
      std::max((size_t)NS * TPS * BCO * 64 + 2 * (size_t)HX_HBYTES, (size_t)HX_PB * (BCO * 2 + 16));
  auto kern = conv3x3_halo_kernel<BCO, NS, TPS, MINW, PF, SCHED, RF>;
  static bool attr_set = false;
  if (!attr_set) {
    hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr_set = true;
  }
  kern<<<(unsigned)nwg, HX_NW * 64, lds, stream>>>(X, Wt, bias, R, Mk, Y, zpage, tiles, g, relu, accumulate,
                                                   tiles_co);
  return (int)hipGetLastError();
}

}  // namespace

// variant (BCO co x 256 slots; NS-deep weight ring; TPS taps per sub-stage; LDS):
//   0 = 128, 3, 1 (80 KiB, <= 128 VGPRs: two blocks per CU)   1 = 256, 3, 1 (135 KiB)
//   2 = 128, 2, 3 (104 KiB)                                    3 = 128, 3, 3 (128 KiB)
// register-prefetch pipeline (next sub-stage's fragments read behind the current MFMAs):
//   4 = 256, 3, 1 (135 KiB)   5 = 128, 3, 1 (80 KiB)   6 = 256, 4, 1 (135 KiB)
// schedule variants (SCHED, see the kernel): 7 / 8 = variant 1 with SCHED 0 / 2, 9 / 10 = variant 2 with
// SCHED 0 / 2, 11 = variant 0 with SCHED 0; fragment reads ahead of the DMA pieces (RF): 12 / 13 = variants
// 7 / 8, 14 = variant 2, 15 = variant 4
// Requires a 3x3 / stride-1 / pad-1 geometry with equal input / output levels, cin % 32 == 0,
// cout % 8 == 0, the tile table of ops/halo.py for this geometry, and (pixels + 1) * cin < 2^31.
MXR_API int mxr_conv3x3_halo(const void* X, const void* Wt, const float* bias, const void* R, const void* Mk,
                             void* Y, const void* zpage, const ConvGeom* g, const void* tiles, int ntiles, int relu,
                             int accumulate, int variant, hipStream_t stream) {
  if (g->cin % 32 != 0 || g->cout % 8 != 0) return -1;
  if (g->kh != 3 || g->kw != 3 || g->stride != 1 || g->pt != 1 || g->pl != 1 || g->ostride != 1) return -2;
  if (g->in_img != g->out_img || (g->M + 1) * (long long)std::max(g->cin, g->cout) >= (1LL << 31)) return -4;
  const bf16_t *x = (const bf16_t*)X, *w = (const bf16_t*)Wt, *r = (const bf16_t*)R, *mk = (const bf16_t*)Mk;
  const bf16_t* z = (const bf16_t*)zpage;
  const HaloTile* t = (const HaloTile*)tiles;
  bf16_t* y = (bf16_t*)Y;
  switch (variant) {
    case 1: return launch_halo<256, 3, 1, 2>(x, w, bias, r, mk, y, z, t, ntiles, *g, relu, accumulate, stream);
    case 2: return launch_halo<128, 2, 3, 2>(x, w, bias, r, mk, y, z, t, ntiles, *g, relu, accumulate, stream);
    case 3: return launch_halo<128, 3, 3, 2>(x, w, bias, r, mk, y, z, t, ntiles, *g, relu, accumulate, stream);
    case 4: return launch_halo<256, 3, 1, 2, true>(x, w, bias, r, mk, y, z, t, ntiles, *g, relu, accumulate, stream);
    case 5: return launch_halo<128, 3, 1, 2, true>(x, w, bias, r, mk, y, z, t, ntiles, *g, relu, accumulate, stream);
    case 6: return launch_halo<256, 4, 1, 2, true>(x, w, bias, r, mk, y, z, t, ntiles, *g, relu, accumulate, stream);
    case 7: return launch_halo<256, 3, 1, 2, false, 0>(x, w, bias, r, mk, y, z, t, ntiles, *g, relu, accumulate, stream);
    case 8: return launch_halo<256, 3, 1, 2, false, 2>(x, w, bias, r, mk, y, z, t, ntiles, *g, relu, accumulate, stream);
    case 9: return launch_halo<128, 2, 3, 2, false, 0>(x, w, bias, r, mk, y, z, t, ntiles, *g, relu, accumulate, stream);
    case 10: return launch_halo<128, 2, 3, 2, false, 2>(x, w, bias, r, mk, y, z, t, ntiles, *g, relu, accumulate, stream);
    case 11: return launch_halo<128, 3, 1, 4, false, 0>(x, w, bias, r, mk, y, z, t, ntiles, *g, relu, accumulate, stream);
    case 12: return launch_halo<256, 3, 1, 2, false, 0, 1>(x, w, bias, r, mk, y, z, t, ntiles, *g, relu, accumulate, stream);
    case 13: return launch_halo<256, 3, 1, 2, false, 2, 1>(x, w, bias, r, mk, y, z, t, ntiles, *g, relu, accumulate, stream);
    case 14: return launch_halo<128, 2, 3, 2, false, 1, 1>(x, w, bias, r, mk, y, z, t, ntiles, *g, relu, accumulate, stream);
    case 15: return launch_halo<256, 3, 1, 2, true, 1, 1>(x, w, bias, r, mk, y, z, t, ntiles, *g, relu, accumulate, stream);
    default: return launch_halo<128, 3, 1, 4>(x, w, bias, r, mk, y, z, t, ntiles, *g, relu, accumulate, stream);
  }
}
