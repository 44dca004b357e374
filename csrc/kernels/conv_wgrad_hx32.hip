// Halo-staged WEIGHT gradient of the 3x3 / stride-1 / pad-1 convolutions on the 32x32x16 bf16 MFMA, for
// gfx950 (the head towers and finals over the packed pyramid, the FPN smoothing convs: SURVEY §2.6 K2, the
// layers built at /root/reference/train.py:91):
//
//   dW[co][ky][kx][ci] = sum_p dY[p][co] * X[p + (ky - 1, kx - 1)][ci]        (+ db[co] = sum_p dY[p][co])
//
// conv_wgrad_p8.hip stages an im2col tile per 64 pixels and 256 (tap, ci) columns, so every input pixel is
// fetched once per tap (128 FLOP per staged byte; 787 TF/s on the head towers, profiles/r3_conv_budget_final.txt).
// Here a block owns dW[256 co][9 taps][32 ci] (one 32-channel chunk) and walks the 256-slot tiles of
// conv_hx32.hip's tile table (ops/halo.py), split over the blocks:
//
// * per tile the chunk's input HALO (<= 448 pixels x 64 B) is staged ONCE by LDS-DMA and all 9 taps read it
//   shifted; its LDS image keeps whole 64-B pixel rows, so a 1-KiB DMA piece is 16 pixels x 64 B (the two-plane
//   image of conv_hx32.hip makes a piece 32 pixels x 32 B: a quarter of each cache line, and the halo DMA
//   then cost 29 % of the kernel against 18 % for the 4.5x larger dY stream -- profiles/r4_wgrad_hx32_ablation.txt); dY streams through a 5-slot ring of 32-slot sub-steps (4 in flight: ~1 us of DMA latency at the
//   MFMA pace of 0.5 us per sub-step) (32 x 512 B), so a
//   tile costs 28 KiB + 128 KiB of staging for 37.7 MFLOP (236 FLOP per staged byte);
// * 8 waves, wave w = co rows 32 w .. 32 w + 31 and all 9 taps (9 accumulators of 32 x 32 = 144 VGPRs):
//   per 16-slot K step one dY fragment and nine shifted halo fragments feed nine v_mfma_f32_32x32x16_bf16;
// * both operands are read TRANSPOSED (ds_read_b64_tr_b16: a lane supplies the LDS address of ITS row, so
//   a tap's shift is per-lane address arithmetic).  A 32-lane half of a halo read takes 4 consecutive 64-B
//   rows = 256 contiguous bytes (all 64 banks), and the dY rows are XOR-swizzled by (row & 3) << 2 on 16-B
//   chunks (applied at the DMA source): the reads are conflict-free;
// * per tile, a slot table (output row m, halo row of tap (0, 0) and the box pitch) is decoded once into
//   LDS for the NEXT tile while this one runs, and the next tile's halo is fetched during this tile:
//   the only vector-memory instructions in the loop are the LDS-DMA pieces, so the counted waits are exact;
// * fp32 split-K slabs part[split][co][tap][ci] (deterministic: reduced in fixed order by
//   mxr_wgrad_reduce_launch), blocks of one split on one XCD share the dY tiles in L2;
// * BIAS: the chunk-0 blocks multiply each dY fragment by a one-hot A fragment (row 0 all ones): column
//   sums of dY in one extra accumulator, bias partials per split -- no separate pass over dY.
#include "common.h"
#include "conv_common.h"
#include "halo_tile.h"

typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(4))) short s16x4;

void mxr_wgrad_reduce_launch(const float* part, int splits, long long n, int K, const float* scale, float* out,
                             int accumulate, hipStream_t stream);

namespace {

constexpr int WX_NW = 8;                         // waves per block
constexpr int WX_BCO = 32 * WX_NW;               // output channels per block
constexpr int WX_SUB = 32;                       // dY slots per sub-step
constexpr int WX_NSUB = HX_PB / WX_SUB;          // sub-steps per tile (8)
constexpr int WX_DROW = WX_BCO * 2;              // one dY row in LDS: 512 B
constexpr int WX_DSLOT = WX_SUB * WX_DROW;       // one ring slot: 16 KiB
constexpr int WX_LA = 5;                         // dY sub-steps in flight ahead of the one being computed
constexpr int WX_RING = WX_LA + 1;
constexpr int WX_DPW = WX_DSLOT / 1024 / WX_NW;  // dY DMA pieces per wave per sub-step (2)
constexpr int WX_HALO = HX_HMAX * 64;            // one halo buffer: 64-B pixel rows (the chunk's 32 channels)
constexpr int WX_HPC = 2 * HX_HMAX / 32;         // 1-KiB halo pieces per tile (28)
constexpr int WX_HQ = (WX_HPC + WX_NW - 1) / WX_NW;   // halo pieces per wave (4; the 29th-32nd repeat one)
constexpr int WX_OFF_H = WX_RING * WX_DSLOT;
constexpr int WX_OFF_T = WX_OFF_H + 2 * WX_HALO;
constexpr int WX_TBL = HX_PB * 8;                // slot table: int m[256], int hp[256]
constexpr int WX_LDS = WX_OFF_T + 2 * WX_TBL;
static_assert(WX_DPW * WX_NW * 1024 == WX_DSLOT, "dY pieces split evenly");
static_assert(WX_LA >= 2 && WX_LA <= WX_NSUB - 2, "the next tile's table is built at j = 0, visible from j = 1");
// the next tile's halo (issued at j = 2, after dY(2 + LA)) may stay in flight at the waits of j = 3 .. WX_HWIN;
// from j = 7 on it must have landed (the next tile's first halo fragments are read before its barrier)
constexpr int WX_HWIN = 2 + WX_LA < WX_NSUB - 2 ? 2 + WX_LA : WX_NSUB - 2;
static_assert(WX_LDS <= 160 * 1024, "LDS");
static_assert(WX_HALO % 16 == 0 && WX_OFF_T % 16 == 0, "16-B aligned LDS carve");

template <int N>
__device__ __forceinline__ void wx_vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// wx_vm_wait with a count that is a constant only after loop unrolling
__device__ __forceinline__ void wx_vm_wait_rt(int n) {
  switch (n) {
    case 0: wx_vm_wait<0>(); break;   case 1: wx_vm_wait<1>(); break;   case 2: wx_vm_wait<2>(); break;
    case 3: wx_vm_wait<3>(); break;   case 4: wx_vm_wait<4>(); break;   case 5: wx_vm_wait<5>(); break;
    case 6: wx_vm_wait<6>(); break;   case 7: wx_vm_wait<7>(); break;   case 8: wx_vm_wait<8>(); break;
    case 9: wx_vm_wait<9>(); break;   case 10: wx_vm_wait<10>(); break; case 11: wx_vm_wait<11>(); break;
    case 12: wx_vm_wait<12>(); break; case 13: wx_vm_wait<13>(); break; case 14: wx_vm_wait<14>(); break;
    default: wx_vm_wait<0>(); break;
  }
}

__device__ __forceinline__ void wx_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// a tile-table field, kept in an SGPR (a per-lane select of two loads becomes a load of a selected address --
// a VECTOR load whose wait drains the DMA pieces in flight)
__device__ __forceinline__ int U(int v) { return __builtin_amdgcn_readfirstlane(v); }

__device__ __forceinline__ s16x4 wx_tr(const char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(p));
}

// PIPE: software-pipelined main loop -- every fragment read is issued one 3-MFMA group (one kernel row ky of
// one K step) ahead of its MFMAs, the first group's halo fragments of the NEXT sub-step are read before the
// barrier (the halo is resident for the whole tile), the slot tables one sub-step ahead, and the dY DMA goes
// out right after the barrier; PIPE = 0: each K step reads all 20 fragments, then runs its 9 MFMAs
// DIAG (timing-only builds, wrong results; never raced by the tuner): bit 2 = halo pieces all from the zero
// page, bit 3 = dY pieces all from the zero page (same instructions and waits: isolates the source pattern),
// bits 5 / 6 = halo / dY sources folded into the first 1 MiB (same per-lane pattern, L2-resident); bit 7 = halo
// pieces of 8 pixels x 128 B (the chunk pair's channels: the source pattern of a 64-channel block); bit 8 = halo
// pieces of 1 KiB contiguous (random data, the dY / weight pattern);
// bit 0 = no dY DMA (the ring keeps stale
// data), bit 1 = no halo DMA (PIPE only)
// HSP (PIPE only): 1 = the next tile's halo pieces spread over sub-steps 1 .. WX_HQ (one per wave per sub-step)
// instead of all WX_HQ at j = 2; 2 = that, and a sub-step's DMA pieces spread between its MFMA groups -- the zero-page build (DIAG 4: same instructions and waits) ran 35 % faster,
// so the burst of 8 x 4 halo pieces (16 distinct 64-B segments each, mostly L2 misses) is what stalls
template <int BIAS, int PIPE = 1, int DIAG = 0, int HSP = 0, int PRIO = 0>
__global__ __launch_bounds__(WX_NW * 64, 2) void conv_wgrad_hx32_kernel(
    const bf16_t* __restrict__ X, const bf16_t* __restrict__ dY, int ldy, float* __restrict__ part,
    float* __restrict__ bpart, const bf16_t* __restrict__ zpage, const HaloTile* __restrict__ tiles, int ntiles,
    ConvGeom g, int tiles_co, int nch, int splits) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wid = xcd_remap(blockIdx.x, gridDim.x);
  const int c = wid % nch;            // the 8 chunks of one (co tile, split) are consecutive: one XCD
  const int rest = wid / nch;
  const int tco = rest % tiles_co;
  const int split = rest / tiles_co;
  const int co0 = tco * WX_BCO;
  const int cin = g.cin, cout = g.cout;
  const int K = 9 * cin;
  const int t_begin = (int)((long long)ntiles * split / splits);
  const int t_end = (int)((long long)ntiles * (split + 1) / splits);
  const uint32_t lds0 = __builtin_amdgcn_readfirstlane(lds_addr(smem));

  // slot tables of tile parity tb: m[256] then hp[256]
  auto tm = [&](int tb) { return reinterpret_cast<int*>(smem + WX_OFF_T + tb * WX_TBL); };
  auto th = [&](int tb) { return reinterpret_cast<int*>(smem + WX_OFF_T + tb * WX_TBL) + HX_PB; };

  // ---- slot table of tile t: m = output row (-1 empty), hp = halo row of tap (0, 0) | pitch << 16
  auto build_table = [&](int t, int tb) {
    {
      // every thread decodes (the tile record stays in scalar loads: no vector load in the loop), the
      // first 256 write
      const HaloTile& T = tiles[t];
      const int p = threadIdx.x & (HX_PB - 1);
      HX_SELECT(sbeg, p)
      int sb = T.b[0].sbeg, ho = T.b[0].hoff, C = T.b[0].C, ob = T.b[0].out_base, W = T.b[0].W, y0 = T.b[0].y0,
          x0 = T.b[0].x0;
#pragma unroll
      for (int u = 1; u < HX_BOX; ++u) {   // selects, not branches: the fields stay scalar loads
        const bool on = sel == u;
        sb = on ? U(T.b[u].sbeg) : sb; ho = on ? U(T.b[u].hoff) : ho; C = on ? U(T.b[u].C) : C;
        ob = on ? U(T.b[u].out_base) : ob; W = on ? U(T.b[u].W) : W; y0 = on ? U(T.b[u].y0) : y0;
        x0 = on ? U(T.b[u].x0) : x0;
      }
      int m = -1, hp = 0;
      if (p < T.nslot) {
        const int loc = p - sb;
        const int r = fdiv(loc, C), cc = loc - r * C;
        m = ob + (y0 + r) * W + x0 + cc;
        hp = (ho + r * (C + 2) + cc) | ((C + 2) << 16);
      }
      if (threadIdx.x < HX_PB) {
        tm(tb)[p] = m;
        th(tb)[p] = hp;
      }
    }
  };
  // ---- halo DMA sources of tile t for chunk c: piece k = 32 halo rows (k / 2) of plane k % 2; wave w
  // issues k = w + 8 q (k >= 28 repeats k - 8); -1 = outside the level (zero page)
  auto decode_halo = [&](int t, int* hs) {
    const HaloTile& T = tiles[t];
#pragma unroll
    for (int q = 0; q < WX_HQ; ++q) {
      int k = wave + WX_NW * q;
      if (k >= WX_HPC) k -= WX_NW;
      const int h = (DIAG & 128) ? k * 8 + (lane >> 3) : k * 16 + (lane >> 2);
      HX_SELECT(hoff, h)
      int hoff = T.b[0].hoff, ib = T.b[0].in_base, H = T.b[0].H, W = T.b[0].W, y0 = T.b[0].y0, x0 = T.b[0].x0,
          C = T.b[0].C;
#pragma unroll
      for (int u = 1; u < HX_BOX; ++u) {
        const bool on = sel == u;
        hoff = on ? U(T.b[u].hoff) : hoff; ib = on ? U(T.b[u].in_base) : ib; H = on ? U(T.b[u].H) : H;
        W = on ? U(T.b[u].W) : W; y0 = on ? U(T.b[u].y0) : y0; x0 = on ? U(T.b[u].x0) : x0;
        C = on ? U(T.b[u].C) : C;
      }
      int off = -1;
      if (h < T.nhalo) {
        const int pw = C + 2;
        const int loc = h - hoff;
        const int hr = fdiv(loc, pw), hc = loc - hr * pw;
        const int y = y0 - 1 + hr, x = x0 - 1 + hc;
        if ((unsigned)y < (unsigned)H && (unsigned)x < (unsigned)W)
          off = (DIAG & 128) ? (ib + y * W + x) * cin + (c & ~1) * 32 + (lane & 7) * 8
                             : (ib + y * W + x) * cin + c * 32 + (lane & 3) * 8;
      }
      hs[q] = off;
    }
  };
  auto issue_halo = [&](const int* hs, int buf, int q0 = 0, int q1 = WX_HQ) {
    if constexpr (DIAG & 2) return;
#pragma unroll
    for (int q = 0; q < WX_HQ; ++q) {
      if (q < q0 || q >= q1) continue;
      int k = wave + WX_NW * q;
      if (k >= WX_HPC) k -= WX_NW;
      const bf16_t* a = (hs[q] >= 0 && !(DIAG & 4)) ? X + ((DIAG & 32) ? ((unsigned)hs[q] & 0x7ffffu) : (unsigned)hs[q])
                                                     : zpage;
      if constexpr ((DIAG & 256) != 0) a = X + (unsigned)(c * 16384 + k * 512 + lane * 8);
      glds16_m0(a, lds0 + WX_OFF_H + buf * WX_HALO + k * 1024);
    }
  };
  // ---- dY sub-step j of the tile whose table is tb, into ring slot `slot`: piece s of wave w = rows
  // 2 (w + 8 s) + lane / 32, LDS chunk lane % 32 <- global chunk (lane % 32) ^ ((row & 3) << 2)
  int dcol[WX_DPW];
#pragma unroll
  for (int s = 0; s < WX_DPW; ++s) {
    const int row = 2 * (wave + WX_NW * s) + (lane >> 5);
    const int co = co0 + (((lane & 31) ^ ((row & 3) << 2)) << 3);
    dcol[s] = co < ldy ? co : -1;
  }
  auto issue_dy = [&](int tb, int j, int slot, bool live) {
#pragma unroll
    for (int s = 0; s < WX_DPW; ++s) {
      const int row = 2 * (wave + WX_NW * s) + (lane >> 5);
      const int m = live ? tm(tb)[j * WX_SUB + row] : -1;
      const bf16_t* a = (m >= 0 && dcol[s] >= 0) ? dY + (unsigned)(m * ldy + dcol[s]) : zpage;
      glds16_m0(a, lds0 + slot * WX_DSLOT + (wave + WX_NW * s) * 1024);
    }
  };

  // ---- fragment addressing.  Lane (h, g, q, p) = (lane / 32, lane / 16 % 2, lane / 4 % 4, lane % 4) reads
  // slot rows 8 h + q (lo) and 8 h + q + 4 (hi) of a 16-slot K step, columns 16 g + 4 p .. + 3 of its
  // 32-column block
  const int fh = lane >> 5, fg = (lane >> 4) & 1, fq = (lane >> 2) & 3, fp = lane & 3;
  const int dbyte = ((((wave * 4 + fg * 2 + (fp >> 1)) ^ (fq << 2))) << 4) + (fp & 1) * 8 + (8 * fh + fq) * WX_DROW;
  const int hbyte = WX_OFF_H + fg * 32 + fp * 8;

  f32x16 acc[9];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[t][e] = 0.f;
  f32x16 accb;
  if constexpr (!PIPE) {
#pragma unroll
    for (int e = 0; e < 16; ++e) accb[e] = 0.f;
  }
  float bacc = 0.f;      // PIPE bias: this lane's partial column sum (lanes l, l + 32 hold halves of one co)
  const bool bsum = BIAS && c == 0;

  // one 16-slot K step kk of sub-step j (ring slot `slot`, tile parity tb): fragment reads, then MFMAs.
  // (ds_read_b64_tr_b16 carries no alias information: a transposed read issued AFTER an LDS-DMA piece in
  // program order gets a compiler-inserted vmcnt(0), so every read of a sub-step is issued before its DMA.)
  struct Frags {
    bf16x8 b, a[9];
  };
  auto kread = [&](int tb, int j, int kk, int slot, Frags& f) {
    const int s_lo = j * WX_SUB + kk * 16 + 8 * fh + fq;
    const int* tht = th(tb);
    const int e_lo = tht[s_lo], e_hi = tht[s_lo + 4];
    const char* db = smem + slot * WX_DSLOT + kk * 16 * WX_DROW + dbyte;
    const s16x4 blo = wx_tr(db), bhi = wx_tr(db + 4 * WX_DROW);
    f.b = bf16x8{blo[0], blo[1], blo[2], blo[3], bhi[0], bhi[1], bhi[2], bhi[3]};
    const int hb_lo = e_lo & 0xffff, pi_lo = e_lo >> 16, hb_hi = e_hi & 0xffff, pi_hi = e_hi >> 16;
    const char* hbase = smem + hbyte + tb * WX_HALO;
#pragma unroll
    for (int ky = 0; ky < 3; ++ky) {
      const char* rlo = hbase + (hb_lo + ky * pi_lo) * 64;
      const char* rhi = hbase + (hb_hi + ky * pi_hi) * 64;
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        const s16x4 alo = wx_tr(rlo + kx * 64), ahi = wx_tr(rhi + kx * 64);
        f.a[ky * 3 + kx] = bf16x8{alo[0], alo[1], alo[2], alo[3], ahi[0], ahi[1], ahi[2], ahi[3]};
      }
    }
  };
  auto kmma = [&](const Frags& f) {
#pragma unroll
    for (int t = 0; t < 9; ++t) acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.a[t], f.b, acc[t], 0, 0, 0);
    if constexpr (BIAS) {
      if (bsum) {
        // one-hot A: row 0 (lanes 0 and 32, all 8 k) = 1.0 -> D[0][co] = sum_k dY[k][co]
        int v = (lane & 31) == 0 ? 0x3f803f80 : 0;
        asm volatile("" : "+v"(v));
        const bf16x8 a = __builtin_bit_cast(bf16x8, int4{v, v, v, v});
        accb = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, f.b, accb, 0, 0, 0);
      }
    }
  };

  // ---- prologue: tile t_begin's table + halo, its first two dY sub-steps
  int hs[WX_HQ];
  build_table(t_begin, 0);
  decode_halo(t_begin, hs);
  issue_halo(hs, 0);
  wx_sync();                       // table visible
#pragma unroll
  for (int j = 0; j < WX_LA; ++j) issue_dy(0, j, j, true);
  int slot = 0;                    // ring slot of the current sub-step (sub-step n lives in n % WX_RING)

  if constexpr (PIPE) {
    // byte offsets (LDS) of the halo rows of taps (ky, 0), ky = 0..2, for a K step's lo / hi slot rows
    auto rows = [&](int e_lo, int e_hi, int tb, int (&r)[2][3]) {
      const int hb_lo = e_lo & 0xffff, pi_lo = e_lo >> 16, hb_hi = e_hi & 0xffff, pi_hi = e_hi >> 16;
      const int base = hbyte + tb * WX_HALO;
#pragma unroll
      for (int ky = 0; ky < 3; ++ky) {
        r[0][ky] = base + (hb_lo + ky * pi_lo) * 64;
        r[1][ky] = base + (hb_hi + ky * pi_hi) * 64;
      }
    };
    auto ra = [&](const int (&r)[2][3], int ky, bf16x8 (&a)[3]) {
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        const s16x4 lo = wx_tr(smem + r[0][ky] + kx * 64), hi = wx_tr(smem + r[1][ky] + kx * 64);
        a[kx] = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
    };
    auto rb = [&](int slot, int kk) {
      const char* db = smem + slot * WX_DSLOT + kk * 16 * WX_DROW + dbyte;
      const s16x4 lo = wx_tr(db), hi = wx_tr(db + 4 * WX_DROW);
      return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    };
    auto mma3 = [&](int ky, const bf16x8 (&a)[3], const bf16x8& b) {
#pragma unroll
      for (int kx = 0; kx < 3; ++kx)
        acc[ky * 3 + kx] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[kx], b, acc[ky * 3 + kx], 0, 0, 0);
    };
    // bias: the dY fragment holds 8 slot values of ONE output channel (co = lane % 32) per lane; sum them on
    // the VALU (1 VGPR instead of a 16-VGPR one-hot accumulator: this loop sits at the register limit)
    auto bias1 = [&](const bf16x8& b) {
      if constexpr (BIAS) {
        if (bsum) {
#pragma unroll
          for (int e = 0; e < 8; ++e) bacc += bf2f((bf16_t)b[e]);
        }
      }
    };
    // table entries of sub-step j of parity tb: {kk 0 lo, kk 0 hi, kk 1 lo, kk 1 hi}
    auto tent = [&](int tb, int j, int (&e)[4]) {
      const int* tht = th(tb);
      const int s0 = j * WX_SUB + 8 * fh + fq;
      e[0] = tht[s0]; e[1] = tht[s0 + 4]; e[2] = tht[s0 + 16]; e[3] = tht[s0 + 20];
    };
    // m (output rows) of the lane's two dY DMA rows of sub-step j of parity tb (-1: zero page)
    auto mrows = [&](int tb, int j, bool live, int (&mm)[WX_DPW]) {
#pragma unroll
      for (int s = 0; s < WX_DPW; ++s) mm[s] = live ? tm(tb)[j * WX_SUB + 2 * (wave + WX_NW * s) + (lane >> 5)] : -1;
    };
    auto dma_dy = [&](const int (&mm)[WX_DPW], int slot, int s0 = 0, int s1 = WX_DPW) {
      if constexpr (DIAG & 1) return;
#pragma unroll
      for (int s = 0; s < WX_DPW; ++s) {
        if (s < s0 || s >= s1) continue;
        const unsigned o = (unsigned)(mm[s] * ldy + dcol[s]);
        const bf16_t* a = (mm[s] >= 0 && dcol[s] >= 0 && !(DIAG & 8)) ? dY + ((DIAG & 64) ? (o & 0x7ffffu) : o) : zpage;
        glds16_m0(a, lds0 + slot * WX_DSLOT + (wave + WX_NW * s) * 1024);
      }
    };

    int E[4], mm[WX_DPW];
    bf16x8 A0[3];
    {
      tent(0, 0, E);
      int r[2][3];
      rows(E[0], E[1], 0, r);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // prologue: the first halo has landed (own pieces)
      wx_sync();                                           // ... and every wave's
      ra(r, 0, A0);
      mrows(0, WX_LA, WX_LA < WX_NSUB, mm);
    }
    for (int t = t_begin; t < t_end; ++t) {
      const int tb = (t - t_begin) & 1;
      const bool has_next = t + 1 < t_end;
#pragma unroll
      for (int j = 0; j < WX_NSUB; ++j) {
        if constexpr (HSP) {
          // younger than dY(j): dY(j + 1 .. j + LA - 1) and the halo pieces of sub-steps s in
          // [max(1, j - LA), min(WX_HQ, j - 1)] (piece s goes out after dY(s + LA)); at j = 7 every halo
          // piece has landed (the next tile's first fragments are read in this sub-step): only the dY issued
          // after the last piece may stay in flight
          static_assert(WX_HQ + WX_LA >= WX_NSUB - 1 && WX_HQ + 1 <= WX_NSUB - 1, "halo spread window");
          const int lo = 1 > j - WX_LA ? 1 : j - WX_LA, hi = WX_HQ < j - 1 ? WX_HQ : j - 1;
          const int nh = hi >= lo ? hi - lo + 1 : 0;
          if (j == WX_NSUB - 1) wx_vm_wait<(WX_HQ + WX_LA - (WX_NSUB - 1)) * WX_DPW>();
          else wx_vm_wait_rt((WX_LA - 1) * WX_DPW + nh);
        } else {
          if (j >= 3 && j <= WX_HWIN) wx_vm_wait<(WX_LA - 1) * WX_DPW + WX_HQ>();
          else wx_vm_wait<(WX_LA - 1) * WX_DPW>();
        }
        wx_sync();
        // dY sub-step j + WX_LA into the slot sub-step j - 1 left (every wave is past it); HSP 2: its second
        // piece and the halo piece go out between the MFMA groups below
        const int dslot = slot == 0 ? WX_RING - 1 : slot - 1;
        dma_dy(mm, dslot, 0, HSP == 2 ? 1 : WX_DPW);
        if constexpr (HSP) {
          if (j == 0) {
            if (has_next) {
              build_table(t + 1, tb ^ 1);
              decode_halo(t + 1, hs);
            } else {
#pragma unroll
              for (int q = 0; q < WX_HQ; ++q) hs[q] = -1;
            }
          }
          if (HSP == 1 && j >= 1 && j <= WX_HQ) issue_halo(hs, tb ^ 1, j - 1, j);   // zero page without a next tile
        } else {
          if (j == 2) {
            if (!has_next) {
#pragma unroll
              for (int q = 0; q < WX_HQ; ++q) hs[q] = -1;
            }
            issue_halo(hs, tb ^ 1);      // zero page when there is no next tile: keeps the count
          }
          if (j == 0 && has_next) build_table(t + 1, tb ^ 1);
          if (j == 1 && has_next) decode_halo(t + 1, hs);
        }
        // one sub-step ahead: table entries of the next sub-step, DMA rows of the next iteration's DMA
        int En[4], mmn[WX_DPW];
        const int tbn = j + 1 < WX_NSUB ? tb : tb ^ 1;
        const bool nlive = j + 1 < WX_NSUB || has_next;
        if (nlive) tent(tbn, (j + 1) % WX_NSUB, En);
        else En[0] = En[1] = En[2] = En[3] = 0;
        {
          const int jd = j + 1 + WX_LA;   // sub-step whose DMA the next iteration issues
          if (jd < WX_NSUB) mrows(tb, jd, true, mmn);
          else mrows(tb ^ 1, jd - WX_NSUB, has_next && jd - WX_NSUB < WX_NSUB, mmn);
        }
        int r0[2][3], r1[2][3];
        rows(E[0], E[1], tb, r0);
        rows(E[2], E[3], tb, r1);
        bf16x8 A1[3], A2[3];
        if constexpr (PRIO) __builtin_amdgcn_s_setprio(1);   // the MFMA stream first while both waves have work
        const bf16x8 B0 = rb(slot, 0);
        ra(r0, 1, A1);
        mma3(0, A0, B0);
        ra(r0, 2, A2);
        mma3(1, A1, B0);
        if constexpr (HSP == 2) dma_dy(mm, dslot, 1, WX_DPW);
        const bf16x8 B1 = rb(slot, 1);
        ra(r1, 0, A1);
        mma3(2, A2, B0);
        bias1(B0);
        ra(r1, 1, A2);
        mma3(0, A1, B1);
        if constexpr (HSP == 2) {
          if (j >= 1 && j <= WX_HQ) issue_halo(hs, tb ^ 1, j - 1, j);
        }
        ra(r1, 2, A1);
        mma3(1, A2, B1);
        {
          int rn[2][3];
          rows(En[0], En[1], tbn, rn);
          ra(rn, 0, A0);               // the next sub-step's first halo fragments (resident halo)
        }
        mma3(2, A1, B1);
        if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);
        bias1(B1);
#pragma unroll
        for (int q = 0; q < 4; ++q) E[q] = En[q];
#pragma unroll
        for (int q = 0; q < WX_DPW; ++q) mm[q] = mmn[q];
        slot = slot == WX_RING - 1 ? 0 : slot + 1;
      }
    }
  } else {
  for (int t = t_begin; t < t_end; ++t) {
      const int tb = (t - t_begin) & 1;
      const bool has_next = t + 1 < t_end;
  #pragma unroll
      for (int j = 0; j < WX_NSUB; ++j) {
        // dY(j) landed (this wave's pieces; the barrier covers the others'): the WX_LA - 1 younger sub-steps
        // may stay in flight, plus the next tile's halo pieces (issued at j = 2 after dY(j + WX_LA)) while
        // they are younger than dY(j); they are older than dY(8) = the next tile's first sub-step
        if (j >= 3 && j <= WX_HWIN) wx_vm_wait<(WX_LA - 1) * WX_DPW + WX_HQ>();
        else wx_vm_wait<(WX_LA - 1) * WX_DPW>();
        wx_sync();
        if (j == 0 && has_next) build_table(t + 1, tb ^ 1);     // read from j = 8 - WX_LA (dY issue) on
        if (j == 1 && has_next) decode_halo(t + 1, hs);
        Frags f0, f1;
        kread(tb, j, 0, slot, f0);
        kmma(f0);
        kread(tb, j, 1, slot, f1);
        // sub-step j + WX_LA: this tile's, or the next tile's first ones (zero page when there is none); its
        // ring slot was last read by sub-step j - 1, which every wave has finished (barrier above)
        const int nslot = slot == 0 ? WX_RING - 1 : slot - 1;   // (slot + WX_LA) % WX_RING
        if (j + WX_LA < WX_NSUB) issue_dy(tb, j + WX_LA, nslot, true);
        else issue_dy(tb ^ 1, j + WX_LA - WX_NSUB, nslot, has_next);
        if (j == 2) {
          if (has_next) issue_halo(hs, tb ^ 1);
          else {
  #pragma unroll
            for (int q = 0; q < WX_HQ; ++q) hs[q] = -1;
            issue_halo(hs, tb ^ 1);    // keeps the count; nobody reads that buffer
          }
        }
        kmma(f1);
        slot = slot == WX_RING - 1 ? 0 : slot + 1;
      }
    }
  }
  wx_vm_wait<0>();

  // ---- slab: lane holds co = co0 + 32 wave + lane % 32 and, per tap, ci rows 8 q + 4 (lane / 32) + 0..3
  const int co = co0 + 32 * wave + (lane & 31);
  if (co < cout) {
    float* row = part + ((long long)split * cout + co) * K + c * 32 + 4 * fh;
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int q = 0; q < 4; ++q)
        *reinterpret_cast<f32x4*>(row + t * cin + 8 * q) =
            f32x4{acc[t][4 * q], acc[t][4 * q + 1], acc[t][4 * q + 2], acc[t][4 * q + 3]};
    if constexpr (BIAS) {
      if constexpr (PIPE) {
        const float tot = bacc + __shfl_xor(bacc, 32, 64);
        if (bsum && fh == 0) bpart[(long long)split * cout + co] = tot;
      } else {
        if (bsum && fh == 0) bpart[(long long)split * cout + co] = accb[0];
      }
    }
  }
}

template <int BIAS, int PIPE, int DIAG = 0, int HSP = 0, int PRIO = 0>
int launch_wx(const bf16_t* X, const bf16_t* dY, int ldy, float* part, float* bpart, int splits,
              const bf16_t* zpage, const HaloTile* tiles, int ntiles, const ConvGeom& g, hipStream_t stream) {
  const int tiles_co = (g.cout + WX_BCO - 1) / WX_BCO;
  const int nch = g.cin / 32;
  const long long nwg = (long long)tiles_co * nch * splits;
  if (nwg > 0x7fffffffLL || nwg < 1) return -3;
  auto kern = conv_wgrad_hx32_kernel<BIAS, PIPE, DIAG, HSP, PRIO>;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, WX_LDS);
    attr_set = true;
  }
  kern<<<(unsigned)nwg, WX_NW * 64, WX_LDS, stream>>>(X, dY, ldy, part, bpart, zpage, tiles, ntiles, g, tiles_co,
                                                       nch, splits);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------------------------------------
// 12-wave form (variant 2): three waves per SIMD instead of two, wave (cg, ky) = (wave % 4, wave / 4) owns co
// rows 64 cg .. 64 cg + 63 (two 32-row blocks) and the three taps (ky, 0..2): 6 accumulators (96 VGPRs),
// per K step 2 dY + 3 halo fragments (10 transposed reads) for 6 MFMAs -- 1.7 reads per MFMA instead of 2.2,
// and a third wave per SIMD to cover the read latency.  The SIMD holding waves s, s + 4, s + 8 runs one co
// group over all nine taps.  Same LDS images, tile walk, DMA ring and slabs as conv_wgrad_hx32_kernel.
constexpr int WY_NW = 12;
constexpr int WY_HQ = (WX_HPC + WY_NW - 1) / WY_NW;   // 3 halo pieces per wave (the 29th..36th repeat one)

template <int BIAS>
__global__ __launch_bounds__(WY_NW * 64, 3) void conv_wgrad_hx32w_kernel(
    const bf16_t* __restrict__ X, const bf16_t* __restrict__ dY, int ldy, float* __restrict__ part,
    float* __restrict__ bpart, const bf16_t* __restrict__ zpage, const HaloTile* __restrict__ tiles, int ntiles,
    ConvGeom g, int tiles_co, int nch, int splits) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int cg = wave & 3, wky = wave >> 2;
  const int wid = xcd_remap(blockIdx.x, gridDim.x);
  const int c = wid % nch;
  const int rest = wid / nch;
  const int tco = rest % tiles_co;
  const int split = rest / tiles_co;
  const int co0 = tco * WX_BCO;
  const int cin = g.cin, cout = g.cout;
  const int K = 9 * cin;
  const int t_begin = (int)((long long)ntiles * split / splits);
  const int t_end = (int)((long long)ntiles * (split + 1) / splits);
  const bool two = wave < 4;          // waves 0-3 issue two dY pieces per sub-step, the others one

  auto tm = [&](int tb) { return reinterpret_cast<int*>(smem + WX_OFF_T + tb * WX_TBL); };
  auto th = [&](int tb) { return reinterpret_cast<int*>(smem + WX_OFF_T + tb * WX_TBL) + HX_PB; };
  auto build_table = [&](int t, int tb) {
    const HaloTile& T = tiles[t];
    const int p = threadIdx.x & (HX_PB - 1);
    HX_SELECT(sbeg, p)
    int sb = T.b[0].sbeg, ho = T.b[0].hoff, C = T.b[0].C, ob = T.b[0].out_base, W = T.b[0].W, y0 = T.b[0].y0,
        x0 = T.b[0].x0;
#pragma unroll
    for (int u = 1; u < HX_BOX; ++u) {
      const bool on = sel == u;
      sb = on ? U(T.b[u].sbeg) : sb; ho = on ? U(T.b[u].hoff) : ho; C = on ? U(T.b[u].C) : C;
      ob = on ? U(T.b[u].out_base) : ob; W = on ? U(T.b[u].W) : W; y0 = on ? U(T.b[u].y0) : y0;
      x0 = on ? U(T.b[u].x0) : x0;
    }
    int m = -1, hp = 0;
    if (p < T.nslot) {
      const int loc = p - sb;
      const int r = fdiv(loc, C), cc = loc - r * C;
      m = ob + (y0 + r) * W + x0 + cc;
      hp = (ho + r * (C + 2) + cc) | ((C + 2) << 16);
    }
    if (threadIdx.x < HX_PB) {
      tm(tb)[p] = m;
      th(tb)[p] = hp;
    }
  };
  auto decode_halo = [&](int t, int* hs) {
    const HaloTile& T = tiles[t];
#pragma unroll
    for (int q = 0; q < WY_HQ; ++q) {
      int k = wave + WY_NW * q;
      if (k >= WX_HPC) k -= WY_NW;
      const int h = k * 16 + (lane >> 2);
      HX_SELECT(hoff, h)
      int hoff = T.b[0].hoff, ib = T.b[0].in_base, H = T.b[0].H, W = T.b[0].W, y0 = T.b[0].y0, x0 = T.b[0].x0,
          C = T.b[0].C;
#pragma unroll
      for (int u = 1; u < HX_BOX; ++u) {
        const bool on = sel == u;
        hoff = on ? U(T.b[u].hoff) : hoff; ib = on ? U(T.b[u].in_base) : ib; H = on ? U(T.b[u].H) : H;
        W = on ? U(T.b[u].W) : W; y0 = on ? U(T.b[u].y0) : y0; x0 = on ? U(T.b[u].x0) : x0;
        C = on ? U(T.b[u].C) : C;
      }
      int off = -1;
      if (h < T.nhalo) {
        const int pw = C + 2;
        const int loc = h - hoff;
        const int hr = fdiv(loc, pw), hc = loc - hr * pw;
        const int y = y0 - 1 + hr, x = x0 - 1 + hc;
        if ((unsigned)y < (unsigned)H && (unsigned)x < (unsigned)W)
          off = (ib + y * W + x) * cin + c * 32 + (lane & 3) * 8;
      }
      hs[q] = off;
    }
  };
  auto issue_halo = [&](const int* hs, int buf) {
#pragma unroll
    for (int q = 0; q < WY_HQ; ++q) {
      int k = wave + WY_NW * q;
      if (k >= WX_HPC) k -= WY_NW;
      char* dst = smem + WX_OFF_H + buf * WX_HALO + k * 1024;
      glds16_asm(hs[q] >= 0 ? X + (unsigned)hs[q] : zpage, dst);
    }
  };
  // dY pieces: piece p = rows 2 p + lane / 32; wave w issues p = w and (waves 0-3) p = w + 12
  int dcol[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const int row = 2 * (wave + WY_NW * s) + (lane >> 5);
    const int co = co0 + (((lane & 31) ^ ((row & 3) << 2)) << 3);
    dcol[s] = co < ldy ? co : -1;
  }
  auto mrows = [&](int tb, int j, bool live, int (&mm)[2]) {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int row = 2 * (wave + WY_NW * s) + (lane >> 5);
      mm[s] = (live && (s == 0 || two)) ? tm(tb)[j * WX_SUB + (row & 31)] : -1;
    }
  };
  auto dma_dy = [&](const int (&mm)[2], int slot) {
    glds16_asm((mm[0] >= 0 && dcol[0] >= 0) ? dY + (unsigned)(mm[0] * ldy + dcol[0]) : zpage,
               smem + slot * WX_DSLOT + wave * 1024);
    if (two)
      glds16_asm((mm[1] >= 0 && dcol[1] >= 0) ? dY + (unsigned)(mm[1] * ldy + dcol[1]) : zpage,
                 smem + slot * WX_DSLOT + (wave + WY_NW) * 1024);
  };
  // counted waits: this wave's own DMA count differs by role
  auto vm_wait_role = [&](bool halo_window) {
    if (two) {
      if (halo_window) wx_vm_wait<(WX_LA - 1) * 2 + WY_HQ>();
      else wx_vm_wait<(WX_LA - 1) * 2>();
    } else {
      if (halo_window) wx_vm_wait<(WX_LA - 1) + WY_HQ>();
      else wx_vm_wait<(WX_LA - 1)>();
    }
  };

  const int fh = lane >> 5, fg = (lane >> 4) & 1, fq = (lane >> 2) & 3, fp = lane & 3;
  int dbyte[2];
#pragma unroll
  for (int jj = 0; jj < 2; ++jj)
    dbyte[jj] = (((((2 * cg + jj) * 4 + fg * 2 + (fp >> 1)) ^ (fq << 2))) << 4) + (fp & 1) * 8 + (8 * fh + fq) * WX_DROW;
  const int hbyte = WX_OFF_H + fg * 32 + fp * 8;

  f32x16 acc[3][2];
#pragma unroll
  for (int kx = 0; kx < 3; ++kx)
#pragma unroll
    for (int jj = 0; jj < 2; ++jj)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[kx][jj][e] = 0.f;
  float bacc[2] = {0.f, 0.f};
  const bool bsum = BIAS && c == 0 && wky == 0;

  auto ra = [&](int e_lo, int e_hi, int tb, bf16x8 (&a)[3]) {
    const int base = hbyte + tb * WX_HALO;
    const int rlo = base + ((e_lo & 0xffff) + wky * (e_lo >> 16)) * 64;
    const int rhi = base + ((e_hi & 0xffff) + wky * (e_hi >> 16)) * 64;
#pragma unroll
    for (int kx = 0; kx < 3; ++kx) {
      const s16x4 lo = wx_tr(smem + rlo + kx * 64), hi = wx_tr(smem + rhi + kx * 64);
      a[kx] = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    }
  };
  auto rb = [&](int slot, int kk, bf16x8 (&b)[2]) {
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) {
      const char* db = smem + slot * WX_DSLOT + kk * 16 * WX_DROW + dbyte[jj];
      const s16x4 lo = wx_tr(db), hi = wx_tr(db + 4 * WX_DROW);
      b[jj] = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    }
  };
  auto mma6 = [&](const bf16x8 (&a)[3], const bf16x8 (&b)[2]) {
#pragma unroll
    for (int jj = 0; jj < 2; ++jj)
#pragma unroll
      for (int kx = 0; kx < 3; ++kx)
        acc[kx][jj] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[kx], b[jj], acc[kx][jj], 0, 0, 0);
    if constexpr (BIAS) {
      if (bsum) {
#pragma unroll
        for (int jj = 0; jj < 2; ++jj)
#pragma unroll
          for (int e = 0; e < 8; ++e) bacc[jj] += bf2f((bf16_t)b[jj][e]);
      }
    }
  };
  auto tent = [&](int tb, int j, int (&e)[4]) {
    const int* tht = th(tb);
    const int s0 = j * WX_SUB + 8 * fh + fq;
    e[0] = tht[s0]; e[1] = tht[s0 + 4]; e[2] = tht[s0 + 16]; e[3] = tht[s0 + 20];
  };

  // ---- prologue (as conv_wgrad_hx32_kernel): table + halo of the first tile, its first WX_LA sub-steps
  int hs[WY_HQ];
  build_table(t_begin, 0);
  decode_halo(t_begin, hs);
  issue_halo(hs, 0);
  wx_sync();
#pragma unroll
  for (int j = 0; j < WX_LA; ++j) {
    int mm0[2];
    mrows(0, j, true, mm0);
    dma_dy(mm0, j);
  }
  int slot = 0;
  int E[4], mm[2];
  tent(0, 0, E);
  mrows(0, WX_LA, WX_LA < WX_NSUB, mm);

  for (int t = t_begin; t < t_end; ++t) {
    const int tb = (t - t_begin) & 1;
    const bool has_next = t + 1 < t_end;
#pragma unroll
    for (int j = 0; j < WX_NSUB; ++j) {
      vm_wait_role(j >= 3 && j <= WX_HWIN);
      wx_sync();
      dma_dy(mm, slot == 0 ? WX_RING - 1 : slot - 1);
      if (j == 2) {
        if (!has_next) {
#pragma unroll
          for (int q = 0; q < WY_HQ; ++q) hs[q] = -1;
        }
        issue_halo(hs, tb ^ 1);
      }
      if (j == 0 && has_next) build_table(t + 1, tb ^ 1);
      if (j == 1 && has_next) decode_halo(t + 1, hs);
      int En[4], mmn[2];
      const int tbn = j + 1 < WX_NSUB ? tb : tb ^ 1;
      if (j + 1 < WX_NSUB || has_next) tent(tbn, (j + 1) % WX_NSUB, En);
      else En[0] = En[1] = En[2] = En[3] = 0;
      {
        const int jd = j + 1 + WX_LA;
        if (jd < WX_NSUB) mrows(tb, jd, true, mmn);
        else mrows(tb ^ 1, jd - WX_NSUB, has_next, mmn);
      }
      // per K step: the two dY fragments, then tap by tap one halo fragment (read one tap ahead) and its two
      // MFMAs -- 16-24 fragment VGPRs live, so the 96 accumulators fit the 168 VGPRs of three waves per SIMD
      // (the third wave per SIMD covers the read latency a deeper software pipeline would)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        bf16x8 B[2];
        rb(slot, kk, B);
        const int e_lo = E[2 * kk], e_hi = E[2 * kk + 1];
        const int base = hbyte + tb * WX_HALO;
        const int rlo = base + ((e_lo & 0xffff) + wky * (e_lo >> 16)) * 64;
        const int rhi = base + ((e_hi & 0xffff) + wky * (e_hi >> 16)) * 64;
        auto rd = [&](int kx) {
          const s16x4 lo = wx_tr(smem + rlo + kx * 64), hi = wx_tr(smem + rhi + kx * 64);
          return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        };
        bf16x8 a = rd(0);
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
          bf16x8 an;
          if (kx < 2) an = rd(kx + 1);
#pragma unroll
          for (int jj = 0; jj < 2; ++jj)
            acc[kx][jj] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, B[jj], acc[kx][jj], 0, 0, 0);
          if (kx < 2) a = an;
        }
        if constexpr (BIAS) {
          if (bsum) {
#pragma unroll
            for (int jj = 0; jj < 2; ++jj)
#pragma unroll
              for (int e = 0; e < 8; ++e) bacc[jj] += bf2f((bf16_t)B[jj][e]);
          }
        }
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) E[q] = En[q];
      mm[0] = mmn[0];
      mm[1] = mmn[1];
      slot = slot == WX_RING - 1 ? 0 : slot + 1;
    }
  }
  wx_vm_wait<0>();

#pragma unroll
  for (int jj = 0; jj < 2; ++jj) {
    const int co = co0 + 32 * (2 * cg + jj) + (lane & 31);
    if constexpr (BIAS) {
      const float tot = bacc[jj] + __shfl_xor(bacc[jj], 32, 64);
      if (bsum && fh == 0 && co < cout) bpart[(long long)split * cout + co] = tot;
    }
    if (co >= cout) continue;
    float* row = part + ((long long)split * cout + co) * K + c * 32 + 4 * fh;
#pragma unroll
    for (int kx = 0; kx < 3; ++kx)
#pragma unroll
      for (int q = 0; q < 4; ++q)
        *reinterpret_cast<f32x4*>(row + (wky * 3 + kx) * cin + 8 * q) =
            f32x4{acc[kx][jj][4 * q], acc[kx][jj][4 * q + 1], acc[kx][jj][4 * q + 2], acc[kx][jj][4 * q + 3]};
  }
}

template <int BIAS>
int launch_wy(const bf16_t* X, const bf16_t* dY, int ldy, float* part, float* bpart, int splits,
              const bf16_t* zpage, const HaloTile* tiles, int ntiles, const ConvGeom& g, hipStream_t stream) {
  const int tiles_co = (g.cout + WX_BCO - 1) / WX_BCO;
  const int nch = g.cin / 32;
  const long long nwg = (long long)tiles_co * nch * splits;
  if (nwg > 0x7fffffffLL || nwg < 1) return -3;
  auto kern = conv_wgrad_hx32w_kernel<BIAS>;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, WX_LDS);
    attr_set = true;
  }
  kern<<<(unsigned)nwg, WY_NW * 64, WX_LDS, stream>>>(X, dY, ldy, part, bpart, zpage, tiles, ntiles, g, tiles_co,
                                                       nch, splits);
  return (int)hipGetLastError();
}

}  // namespace

// dW (fp32 OHWI, scaled by `scale` when given, accumulated into `out` when `accumulate`) of a 3x3 / stride-1
// / pad-1 conv over conv_hx32's tile table; part: splits * cout * 9 * cin floats (+ splits * cout bias
// partials when bias_out is given: db = sum_m dY[m, :cout], unscaled).  Requires cin % 32 == 0, ldy % 8 == 0,
// 1 <= splits <= ntiles, equal input / output levels, (pixels + 1) * max(cin, ldy) < 2^31.  variant 0: each K
// step reads its 20 fragments then runs its 9 MFMAs; 1: the software-pipelined loop (PIPE); 2: the 12-wave
// form (three waves per SIMD, two co blocks x one kernel row per wave); 3: variant 1 with the next tile's halo
// spread over four sub-steps (HSP); 4: 3 with the second dY piece and the halo piece issued between the MFMA
// groups; 5: 4 with s_setprio 1 around the MFMA block.  (A 4-wave form -- one wave per SIMD,
// two co blocks x nine taps = 288 accumulator registers -- measured 0.71 ms against 0.50 on the head pyramid:
// past 256 AGPRs the compiler shuttles accumulators through v_accvgpr moves, ~190 per sub-step.)
MXR_API int mxr_conv_wgrad_hx32(const void* X, const void* dY, int ldy, float* part, int splits, float* out,
                                const float* scale, int accumulate, const void* zpage, const ConvGeom* g,
                                const void* tiles, int ntiles, float* bias_out, int bias_accumulate, int variant,
                                hipStream_t stream) {
  if (g->cin % 32 != 0 || ldy % 8 != 0 || g->cout < 1) return -1;
  if (g->kh != 3 || g->kw != 3 || g->stride != 1 || g->pt != 1 || g->pl != 1 || g->ostride != 1) return -2;
  if (g->in_img != g->out_img || (g->M + 1) * (long long)std::max(g->cin, ldy) >= (1LL << 31)) return -4;
  if (splits < 1 || splits > ntiles) return -5;
  const bf16_t *x = (const bf16_t*)X, *dy = (const bf16_t*)dY, *z = (const bf16_t*)zpage;
  const HaloTile* t = (const HaloTile*)tiles;
  const int K = 9 * g->cin;
  float* bpart = bias_out ? part + (long long)splits * g->cout * K : nullptr;
  int rc;
  if (variant >= 101 && variant <= 199) {   // timing-only builds of variant 1 (wrong results)
    if (variant == 101) rc = launch_wx<0, 1, 1>(x, dy, ldy, part, nullptr, splits, z, t, ntiles, *g, stream);
    else if (variant == 102) rc = launch_wx<0, 1, 2>(x, dy, ldy, part, nullptr, splits, z, t, ntiles, *g, stream);
    else if (variant == 104) rc = launch_wx<0, 1, 4>(x, dy, ldy, part, nullptr, splits, z, t, ntiles, *g, stream);
    else if (variant == 108) rc = launch_wx<0, 1, 8>(x, dy, ldy, part, nullptr, splits, z, t, ntiles, *g, stream);
    else if (variant == 112) rc = launch_wx<0, 1, 12>(x, dy, ldy, part, nullptr, splits, z, t, ntiles, *g, stream);
    else if (variant == 132) rc = launch_wx<0, 1, 32, 1>(x, dy, ldy, part, nullptr, splits, z, t, ntiles, *g, stream);
    else if (variant == 164) rc = launch_wx<0, 1, 64, 1>(x, dy, ldy, part, nullptr, splits, z, t, ntiles, *g, stream);
    else if (variant == 196) rc = launch_wx<0, 1, 96, 1>(x, dy, ldy, part, nullptr, splits, z, t, ntiles, *g, stream);
    else if (variant == 128) rc = launch_wx<0, 1, 128, 1>(x, dy, ldy, part, nullptr, splits, z, t, ntiles, *g, stream);
    else if (variant == 156) rc = launch_wx<0, 1, 256, 1>(x, dy, ldy, part, nullptr, splits, z, t, ntiles, *g, stream);
    else if (variant == 105) rc = launch_wx<0, 1, 4, 1>(x, dy, ldy, part, nullptr, splits, z, t, ntiles, *g, stream);
    else rc = launch_wx<0, 1, 3>(x, dy, ldy, part, nullptr, splits, z, t, ntiles, *g, stream);
  } else if (variant == 3) rc = bias_out ? launch_wx<1, 1, 0, 1>(x, dy, ldy, part, bpart, splits, z, t, ntiles, *g, stream)
                                  : launch_wx<0, 1, 0, 1>(x, dy, ldy, part, nullptr, splits, z, t, ntiles, *g, stream);
  else if (variant == 4) rc = bias_out ? launch_wx<1, 1, 0, 2>(x, dy, ldy, part, bpart, splits, z, t, ntiles, *g, stream)
                                  : launch_wx<0, 1, 0, 2>(x, dy, ldy, part, nullptr, splits, z, t, ntiles, *g, stream);
  else if (variant == 5) rc = bias_out ? launch_wx<1, 1, 0, 2, 1>(x, dy, ldy, part, bpart, splits, z, t, ntiles, *g, stream)
                                  : launch_wx<0, 1, 0, 2, 1>(x, dy, ldy, part, nullptr, splits, z, t, ntiles, *g, stream);
  else if (variant == 2) rc = bias_out ? launch_wy<1>(x, dy, ldy, part, bpart, splits, z, t, ntiles, *g, stream)
                                  : launch_wy<0>(x, dy, ldy, part, nullptr, splits, z, t, ntiles, *g, stream);
  else if (variant == 1) rc = bias_out ? launch_wx<1, 1>(x, dy, ldy, part, bpart, splits, z, t, ntiles, *g, stream)
                                  : launch_wx<0, 1>(x, dy, ldy, part, nullptr, splits, z, t, ntiles, *g, stream);
  else rc = bias_out ? launch_wx<1, 0>(x, dy, ldy, part, bpart, splits, z, t, ntiles, *g, stream)
                     : launch_wx<0, 0>(x, dy, ldy, part, nullptr, splits, z, t, ntiles, *g, stream);
  if (rc) return rc;
  mxr_wgrad_reduce_launch(part, splits, (long long)g->cout * K, K, scale, out, accumulate, stream);
  if (bias_out) mxr_wgrad_reduce_launch(bpart, splits, g->cout, 1 << 30, nullptr, bias_out, bias_accumulate, stream);
  return (int)hipGetLastError();
}
