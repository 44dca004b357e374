// Deep-pipelined NHWC bf16 implicit-GEMM convolution (forward / stride-1 data-gradient) for gfx950.
//
// Same GEMM as conv_igemm.hip (C^T = W . A^T, swapped orientation so each lane ends with 4
// consecutive output channels of one pixel; SURVEY §2.6 K1/K2, reached from the conv layers the
// reference builds at /root/reference/train.py:91), but shaped for ONE 8-wave block per CU:
//
// * tile = BCO output channels x 256 pixels, 8 waves as 2 (co) x 4 (pixels); per wave
//   (BCO/2) x 64 outputs = up to 8 x 4 MFMA 16x16x32 accumulators;
// * K is consumed in 32-deep sub-stages held in a 4-deep LDS ring (BCO=256: 4 x 32 KiB);
//   each sub-stage is filled by global_load_lds_dwordx4 (LDS-DMA, the im2col gather is the per-lane
//   source address) THREE sub-stages ahead, and the prefetch stays in flight across the barrier:
//   counted `s_waitcnt vmcnt(N)` + raw `s_barrier`, never `__syncthreads()` (which would drain
//   every outstanding DMA with vmcnt(0));
// * sub-stage rows are 64 B; the 16-B chunk index is XOR-swizzled with f(row/4 mod 4) = [0,2,3,1]
//   so each 16-lane group of the MFMA-fragment ds_read_b128 (lane groups per MI355X_MICROARCH.md
//   §LDS) hits 16 distinct 16-B bank slots: conflict-free; the swizzle is applied to the DMA
//   SOURCE address, the LDS image stays lane-linear;
// * per-lane fragment offsets are lane constants, so every ds_read uses an immediate offset.
//
// Protocol per sub-stage s (buffer s & 3):
//   wait own DMA of sub-stage s (vmcnt = loads of the <= 2 younger sub-stages)
//   s_waitcnt lgkmcnt(0); s_barrier          -> every wave's DMA for s has landed, and every wave
//                                               has finished reading s-1 (buffer of s+3)
//   issue DMA for s+3 into buffer (s+3) & 3
//   12 (BCO=256) ds_read_b128 + 32 MFMA on buffer s & 3
#include <algorithm>

#include "common.h"

#include "conv_common.h"

namespace {

constexpr int PBN = 256;   // pixels per tile (default; PB template parameter)
constexpr int PNST = 4;    // LDS ring depth (sub-stages; default of the NS template parameter)

__device__ __forceinline__ int pswz(int rq) { return (120 >> (2 * rq)) & 3; }  // [0, 2, 3, 1]

// ABL (diagnostics only, never used by the framework): 1 = no DMA, 2 = no MFMA, 3 = DMA + barriers only
// ILV: interleave the next sub-stage's DMA pieces between MFMA groups (steady state)
// NW / WCO: waves per block and wave-grid rows along Cout (8 / 2 by default; the narrow 64-channel
// variant runs 4 waves as 1 x 4 so two blocks share a CU)
template <int N>
__device__ __forceinline__ void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// PB: pixels per tile (256, or 128 for the small-K layers: half the LDS, two blocks per CU)
// NS: LDS ring depth; DMA runs NS - 1 sub-stages ahead (3: smaller ring -> more blocks per CU)
// SK: split-K form -- blockIdx.y is a split of the K sub-stages; the block writes its fp32 partial tile to
// part[split][m][co] and pipe_splitk_epilogue sums the splits and applies the epilogue (small-M, long-K
// layers: the FPN P6 / P7 convs have 35-70 tiles of 72-576 K sub-stages, a few CUs working serially)
// DS: dual-source 1x1 GEMM (a ResNet projection block's branch2c + branch1 as ONE GEMM over the concatenated K):
// Y = epi([X | X2(strided)] . [W2c | W1]^T + b).  K-sub-stages below ds.cin1 read row m of X (the 2b output,
// channel stride cin1); the rest read X2 (the block input) at pixel (b, oy*s, ox*s) of its H x W grid, channel
// stride cin2.  The shortcut tensor of the reference's ``Add([branch2c, branch1])`` is never written or re-read.
struct DualSrc {
  const bf16_t* x2;
  const bf16_t* w2;     // W1 [cout, cin2] (Wt = W2c [cout, cin1]): no concatenated weight copy
  int cin1, cin2, H, W, s;
};

// DD: dual-destination epilogue (a projection block's branch2c + branch1 DATA gradients as ONE GEMM over the
// block output gradient: [dH2 | dX] = dY . [W2c | W1]): output channels below dd.c1 go to Y ([M, c1], masked by Mk =
// the branch2b activation), the rest to dd.y2 ([.., ld2] channels: stride 1 row m, or the stride-2 scatter into an
// oH2 x oW2 grid writing the gaps' zeros), accumulated into it when dd.acc2 (a GradJoin buffer).  dY is read once.
struct DualDst {
  bf16_t* y2;
  const bf16_t* w2;     // the flipped W1 [c2, K] (Wt = the flipped W2c [c1, K])
  int c1, ld2, os2, oH2, oW2, acc2;
};

template <int BCO, int ABL = 0, int ILV = 0, int NW = 8, int WCO = 2, int PB = PBN, int NS = PNST, int SK = 0,
          int DS = 0, int DD = 0>
__global__ __launch_bounds__(NW * 64) void conv_fwd_pipe_kernel(
    const bf16_t* __restrict__ X, const bf16_t* __restrict__ Wt, const float* __restrict__ bias,
    const bf16_t* __restrict__ R, const bf16_t* __restrict__ Mk, bf16_t* __restrict__ Y,
    const bf16_t* __restrict__ zpage, ConvGeom g, int relu,
    int accumulate, int tiles_co, float* __restrict__ part, int nsplit, DualSrc ds, DualDst dd) {
  constexpr int NSA = BCO / (16 * NW);         // A (weight) wave-instructions per lane per sub-stage
  constexpr int NSB = PB / (16 * NW);         // B (pixel) wave-instructions per lane per sub-stage
  static_assert(NSA * 16 * NW == BCO && NSB * 16 * NW == PB, "rows must split evenly over the waves");
  constexpr int NTH = NW * 64;
  constexpr int STAGE = (BCO + PB) * 64;     // bytes per sub-stage
  constexpr int WPX = NW / WCO;
  constexpr int WT_CO = BCO / WCO, WT_PIX = PB / WPX;
  constexpr int TI = WT_CO / 16, TJ = WT_PIX / 16;

  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wid = xcd_remap(blockIdx.x, gridDim.x);
  const int tco = wid % tiles_co;
  const long long tm = wid / tiles_co;
  const int co0 = tco * BCO;
  const long long m0 = tm * PB;
  const int K = g.kh * g.kw * g.cin;
  const int split = SK ? (int)blockIdx.y : 0;
  const int ks0 = SK ? (int)((long long)(K >> 5) * split / nsplit) : 0;
  const int nks = SK ? (int)((long long)(K >> 5) * (split + 1) / nsplit) - ks0 : (K >> 5);

  // ---- per-lane DMA descriptors: lane writes row (q*16 + lane/4), physical chunk lane&3
  const int rloc = lane >> 2;
  const int cl = (lane & 3) ^ pswz(rloc >> 2);   // logical 16-B chunk this lane fetches
  const bf16_t* asrc[NSA];
  const bf16_t* asrc2[DS ? NSA : 1];    // DS: the row's W1 piece, offset so that + k (k >= cin1) addresses it
#pragma unroll
  for (int s = 0; s < NSA; ++s) {
    const int co = co0 + (s * NW + wave) * 16 + rloc;
    if constexpr (DS) {
      asrc[s] = co < g.cout ? Wt + (long long)co * ds.cin1 + cl * 8 : nullptr;
      asrc2[s] = co < g.cout ? ds.w2 + (long long)co * ds.cin2 - ds.cin1 + cl * 8 : nullptr;
    } else if constexpr (DD) {
      asrc[s] = co < g.cout ? (co < dd.c1 ? Wt + (long long)co * K : dd.w2 + (long long)(co - dd.c1) * K) + cl * 8
                            : nullptr;
    } else {
      asrc[s] = co < g.cout ? Wt + (long long)co * K + cl * 8 : nullptr;
    }
  }
  PixSlot<NSB> ps;
  int p2[DS ? NSB : 1];     // DS: the row's pixel in X2
#pragma unroll
  for (int s = 0; s < NSB; ++s) {
    const long long m = m0 + (s * NW + wave) * 16 + rloc;
    ps.base[s] = -1;
    ps.iy0[s] = ps.ix0[s] = ps.Hl[s] = ps.Wl[s] = 0;
    if constexpr (DS) p2[s] = 0;
    if (m < g.M) {
      int b, oy, ox;
      decode_row(g, m, ps.base[s], ps.iy0[s], ps.ix0[s], ps.Hl[s], ps.Wl[s], b, oy, ox);
      if constexpr (DS) p2[s] = (b * ds.H + oy * ds.s) * ds.W + ox * ds.s;
    }
  }

  // issue cursor (sub-stage ikt -> tap (iky, ikx), channel ic0), starting at the split's first sub-stage
  int ikt = ks0, ic0 = 0, iky = 0, ikx = 0;
  if (SK) {
    const int tap = (ks0 * 32) / g.cin;
    ic0 = ks0 * 32 - tap * g.cin;
    iky = tap / g.kw;
    ikx = tap - iky * g.kw;
  }
  // A-operand source of one 16-B piece at K-sub-stage ikt (uniform choice between the two DS weight matrices)
  auto asrc_at = [&](int s) -> uintptr_t {
    if (!asrc[s]) return (uintptr_t)zpage;
    if constexpr (DS) {
      if (ikt * 32 >= ds.cin1) return (uintptr_t)(asrc2[s] + ikt * 32);
    }
    return (uintptr_t)(asrc[s] + ikt * 32);
  };
  const int cstr = DS ? ds.cin1 : g.cin;     // channel stride of X
  // B-operand source of one 16-B piece (sub-stage channel ic0 of row slot sb)
  auto bsrc = [&](int sb) -> uintptr_t {
    const int iy = ps.iy0[sb] + iky, ix = ps.ix0[sb] + ikx;
    // branchless: invalid rows carry Hl = 0, so the unsigned compare fails for them too
    const bool ok = (unsigned)iy < (unsigned)ps.Hl[sb] && (unsigned)ix < (unsigned)ps.Wl[sb];
    if constexpr (DS) {
      if (ic0 >= ds.cin1) {     // uniform: the second source
        const long long off2 = (long long)p2[sb] * ds.cin2 + (ic0 - ds.cin1) + cl * 8;
        return ok ? (uintptr_t)(ds.x2 + off2) : (uintptr_t)zpage;
      }
    }
    const long long off = (long long)(ps.base[sb] + iy * ps.Wl[sb] + ix) * cstr + ic0 + cl * 8;
    return ok ? (uintptr_t)(X + off) : (uintptr_t)zpage;
  };
  auto issue = [&]() {
    char* base = smem + ((ikt - ks0) % NS) * STAGE;
#pragma unroll
    for (int s = 0; s < NSA; ++s) glds16((const void*)asrc_at(s), base + (s * NW + wave) * 1024);
#pragma unroll
    for (int s = 0; s < NSB; ++s) glds16((const void*)bsrc(s), base + BCO * 64 + (s * NW + wave) * 1024);
    ++ikt;
    ic0 += 32;
    if (ic0 == g.cin) {
      ic0 = 0;
      if (++ikx == g.kw) { ikx = 0; ++iky; }
    }
  };

  // slot-wise issue (steady state): slot q < NSA is a weight row piece, else a pixel row piece
  auto issue_slot = [&](int q) {
    char* base = smem + ((ikt - ks0) % NS) * STAGE;
    if (q < NSA) {
      glds16((const void*)asrc_at(q), base + (q * NW + wave) * 1024);
    } else {
      const int sb = q - NSA;
      glds16((const void*)bsrc(sb), base + BCO * 64 + (sb * NW + wave) * 1024);
    }
  };
  auto advance = [&]() {
    ++ikt;
    ic0 += 32;
    if (ic0 == g.cin) {
      ic0 = 0;
      if (++ikx == g.kw) { ikx = 0; ++iky; }
    }
  };

  f32x4 acc[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int wco = wave / WPX, wpx = wave % WPX;
  // fragment offset of this lane inside a 16-row x 64-B block: row lane&15, logical chunk lane>>4
  const int foff = (lane & 15) * 64 + (((lane >> 4) ^ pswz((lane & 15) >> 2)) << 4);
  const int aoff = wco * WT_CO * 64 + foff;
  const int boff = BCO * 64 + wpx * WT_PIX * 64 + foff;

  // iterations -3..-1 only prefetch (one issue path for prologue and steady state)
  for (int s = -(NS - 1); s < nks; ++s) {
    if (s >= 0) {
      const int rem = nks - 1 - s;
      constexpr int L = NSA + NSB;   // DMA pieces per wave per sub-stage
      static_assert(NS == 3 || NS == 4, "ring depth");
      if (rem >= NS - 2) vm_wait<(NS - 2) * L>();
      else if (rem == 1) vm_wait<L>();
      else vm_wait<0>();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    }
    if constexpr ((ILV == 1 || ILV == 2) && ABL == 0) {
      if (s >= 0) {
        const bool do_issue = s + NS - 1 < nks;
        // steady state: the DMA pieces of sub-stage s+3 are spread between this sub-stage's MFMA
        // groups, so one wave's DMA-issue stall overlaps MFMAs (its own queued ones and its SIMD
        // partner's) instead of idling the matrix core at the top of every sub-stage
        // DMA groups: one piece per MFMA group (4 pieces: BCO=256), {A, B0} + {B1} (3 pieces: BCO=128),
        // or {A} + {B} (2 pieces: 128 x 128 tiles)
        constexpr int L = NSA + NSB;
        static_assert(L >= 2 && L <= 4, "DMA grouping");
        constexpr int NG = (L == 4) ? 4 : 2;
        constexpr int IPQ = TI / NG;
        static_assert(TI % NG == 0, "MFMA groups must tile the wave's rows");
        const char* sb = smem + (s % NS) * STAGE;
        bf16x8 bfr[TJ];
#pragma unroll
        for (int j = 0; j < TJ; ++j) bfr[j] = *reinterpret_cast<const bf16x8*>(sb + boff + j * 1024);
#pragma unroll
        for (int q = 0; q < NG; ++q) {
          bf16x8 af[IPQ];
#pragma unroll
          for (int i = 0; i < IPQ; ++i) af[i] = *reinterpret_cast<const bf16x8*>(sb + aoff + (q * IPQ + i) * 1024);
          if (do_issue) {
            if constexpr (NG == 4 || L == 2) {
              issue_slot(q);
            } else {
              if (q == 0) { issue_slot(0); issue_slot(1); }
              else issue_slot(2);
            }
          }
          if constexpr (ILV == 2) __builtin_amdgcn_s_setprio(1);   // MFMA section wins issue arbitration
#pragma unroll
          for (int i = 0; i < IPQ; ++i)
#pragma unroll
            for (int j = 0; j < TJ; ++j)
              acc[q * IPQ + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[q * IPQ + i][j], 0, 0, 0);
          if constexpr (ILV == 2) __builtin_amdgcn_s_setprio(0);
          if (q == 0) __builtin_amdgcn_sched_group_barrier(0x0100, IPQ + TJ, 0);   // its fragment reads
          else __builtin_amdgcn_sched_group_barrier(0x0100, IPQ, 0);
          if (L == 3 && q == 0) __builtin_amdgcn_sched_group_barrier(0x0010, 2, 0);   // its DMA pieces
          else __builtin_amdgcn_sched_group_barrier(0x0010, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x0008, IPQ * TJ, 0);                // its MFMA group
        }
        if (do_issue) advance();
        continue;
      }
    }
    if (s + NS - 1 < nks) {
      if constexpr (ABL == 1) ++ikt;
      else issue();
    }
    if (s < 0) continue;
    if constexpr (ABL == 3) continue;
    const char* sb = smem + (s % NS) * STAGE;
    bf16x8 af[TI], bfr[TJ];
#pragma unroll
    for (int i = 0; i < TI; ++i) af[i] = *reinterpret_cast<const bf16x8*>(sb + aoff + i * 1024);
#pragma unroll
    for (int j = 0; j < TJ; ++j) bfr[j] = *reinterpret_cast<const bf16x8*>(sb + boff + j * 1024);
    if constexpr (ABL == 2) {
#pragma unroll
      for (int i = 0; i < TI; ++i) asm volatile("" ::"v"(af[i]));
#pragma unroll
      for (int j = 0; j < TJ; ++j) asm volatile("" ::"v"(bfr[j]));
      continue;
    }
    if constexpr (ILV == 3) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int j = 0; j < TJ; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    if constexpr (ILV == 3) __builtin_amdgcn_s_setprio(0);
  }

  // ---- epilogue, two passes through LDS so global traffic is full 16-B-per-lane rows:
  // (1) each lane writes its 4-channel fragments (acc + bias, bf16) into a [256 pix][BCO] LDS image
  //     (row pitch BCO*2 + 16 B: the 16 pixels of a fragment land on distinct banks);
  // (2) threads sweep the image in 16-B chunks along the channel axis and apply residual /
  //     accumulate / relu / mask with coalesced 16-B global loads and stores.
  // The residual / accumulate / mask loads of a thread's chunks are issued in groups of up to 4 ahead of
  // their use instead of one load-wait-store round trip per chunk (those round trips set the time of the
  // small-K residual layers, which are HBM-bound otherwise).  The groups start after pass (1): the
  // accumulators are dead by then, so the 48 VGPRs of a group do not raise the kernel's allocation.
  if constexpr (SK) {
    // fp32 partial tile straight from the accumulators: lane (j, i) holds 4 consecutive channels of a pixel
    float* P = part + (long long)split * g.M * g.cout;
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
      const long long m = m0 + wpx * WT_PIX + j * 16 + (lane & 15);
#pragma unroll
      for (int i = 0; i < TI; ++i) {
        const int co = co0 + wco * WT_CO + i * 16 + 4 * (lane >> 4);
        if (m < g.M && co < g.cout) *reinterpret_cast<f32x4*>(P + m * g.cout + co) = acc[i][j];
      }
    }
    return;
  }
  constexpr int PITCH = BCO * 2 + 16;
  constexpr int CPR = BCO / 8;                 // 16-B chunks per tile row
  constexpr int NIT = (PB * CPR + NTH - 1) / NTH;
  constexpr int EPG = NIT < 4 ? NIT : 4;
  static_assert(NIT % EPG == 0, "epilogue groups");
  const int ncv = min(BCO, g.cout - co0) / 8;  // valid chunks (cout % 8 == 0 on this path)
  const bf16_t* Yacc = accumulate ? Y : nullptr;
  const bool pre = R != nullptr || Yacc != nullptr || Mk != nullptr;   // uniform
  // chunk it of this thread -> (tile row, channel chunk, output offset); false = nothing to store
  auto chunk_at = [&](int it, int& pr, int& ch, long long& m, long long& off) -> bool {
    const int c = (int)threadIdx.x + it * NTH;
    if (c >= PB * CPR) return false;
    pr = c / CPR;
    ch = c - pr * CPR;
    m = m0 + pr;
    if (m >= g.M || ch >= ncv) return false;
    long long obase;
    if (g.ostride == 1) {
      obase = m * g.cout;
    } else {
      const int b = (int)(m / g.out_img);
      const int q = (int)(m - (long long)b * g.out_img);
      const int oy = q / g.Wo[0], ox = q - (q / g.Wo[0]) * g.Wo[0];
      obase = (((long long)b * g.oH + oy * g.ostride + g.ooy) * g.oW + ox * g.ostride + g.oox) * g.cout;
    }
    off = obase + co0 + ch * 8;
    return true;
  };
  Epi8 ep[EPG];
  auto load_group = [&](int g0) {
#pragma unroll
    for (int k = 0; k < EPG; ++k) {
      int pr, ch;
      long long m, off;
      if (chunk_at(g0 + k, pr, ch, m, off)) epi_load8(ep[k], R, m * g.cout + co0 + ch * 8, Yacc, Mk, off);
    }
  };
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __syncthreads();   // every wave is done reading the ring (all DMA retired by the last vmcnt(0))
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
  if constexpr (DD) {
    // chunk -> destination (dH2 row m, masked; or dX at stride 1 / 2, accumulated into for acc2); the mask /
    // accumulation loads of a group of EPG chunks are issued together, as in the single-destination epilogue
    auto dd_at = [&](int it, int& pr, int& ch, long long& off, bool& second, int& oy, int& ox) -> bool {
      const int c = (int)threadIdx.x + it * NTH;
      if (c >= PB * CPR) return false;
      pr = c / CPR;
      ch = c - pr * CPR;
      const long long m = m0 + pr;
      if (m >= g.M || ch >= ncv) return false;
      const int co = co0 + ch * 8;
      second = co >= dd.c1;
      oy = ox = 0;
      if (!second) {
        off = m * dd.c1 + co;
      } else if (dd.os2 == 1) {
        off = m * dd.ld2 + (co - dd.c1);
      } else {
        const int b = (int)(m / g.out_img);
        const int q = (int)(m - (long long)b * g.out_img);
        oy = q / g.Wo[0];
        ox = q - oy * g.Wo[0];
        off = (((long long)b * dd.oH2 + oy * dd.os2) * dd.oW2 + ox * dd.os2) * dd.ld2 + (co - dd.c1);
      }
      return true;
    };
    const bf16_t* acc2 = dd.acc2 ? dd.y2 : nullptr;
#pragma unroll
    for (int g0 = 0; g0 < NIT; g0 += EPG) {
#pragma unroll
      for (int k = 0; k < EPG; ++k) {
        int pr, ch, oy, ox;
        long long off;
        bool second;
        if (dd_at(g0 + k, pr, ch, off, second, oy, ox))
          epi_load8(ep[k], nullptr, 0, second ? acc2 : nullptr, second ? nullptr : Mk, off);
      }
#pragma unroll
      for (int k = 0; k < EPG; ++k) {
        int pr, ch, oy, ox;
        long long off;
        bool second;
        if (!dd_at(g0 + k, pr, ch, off, second, oy, ox)) continue;
        const uint4 raw = *reinterpret_cast<const uint4*>(smem + pr * PITCH + ch * 16);
        const uint32_t rw[4] = {raw.x, raw.y, raw.z, raw.w};
        float v[8];
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          v[2 * t] = bf2f((bf16_t)(rw[t] & 0xffff));
          v[2 * t + 1] = bf2f((bf16_t)(rw[t] >> 16));
        }
        epi_apply8(v, ep[k], nullptr, second ? acc2 : nullptr, second ? nullptr : Mk, false);
        uint4 o;
        o.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
        o.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
        o.z = (uint32_t)f2bf(v[4]) | ((uint32_t)f2bf(v[5]) << 16);
        o.w = (uint32_t)f2bf(v[6]) | ((uint32_t)f2bf(v[7]) << 16);
        bf16_t* dst = second ? dd.y2 : Y;
        *reinterpret_cast<uint4*>(dst + off) = o;
        if (second && dd.os2 == 2 && !dd.acc2) {     // the three positions no output pixel maps to
          const uint4 z = make_uint4(0u, 0u, 0u, 0u);
          const bool xr = 2 * ox + 1 < dd.oW2, yd = 2 * oy + 1 < dd.oH2;
          if (xr) *reinterpret_cast<uint4*>(dst + off + dd.ld2) = z;
          if (yd) *reinterpret_cast<uint4*>(dst + off + (long long)dd.oW2 * dd.ld2) = z;
          if (xr && yd) *reinterpret_cast<uint4*>(dst + off + (long long)(dd.oW2 + 1) * dd.ld2) = z;
        }
      }
    }
    return;
  }
#pragma unroll
  for (int g0 = 0; g0 < NIT; g0 += EPG) {
    if (pre) load_group(g0);
#pragma unroll
    for (int k = 0; k < EPG; ++k) {
      int pr, ch;
      long long m, off;
      if (!chunk_at(g0 + k, pr, ch, m, off)) continue;
      const uint4 raw = *reinterpret_cast<const uint4*>(smem + pr * PITCH + ch * 16);
      const uint32_t rw[4] = {raw.x, raw.y, raw.z, raw.w};
      float v[8];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        v[2 * t] = bf2f((bf16_t)(rw[t] & 0xffff));
        v[2 * t + 1] = bf2f((bf16_t)(rw[t] >> 16));
      }
      if (pre) {
        epi_apply8(v, ep[k], R, Yacc, Mk, relu);
      } else if (relu) {
#pragma unroll
        for (int t = 0; t < 8; ++t) v[t] = fmaxf(v[t], 0.f);
      }
      uint4 o;
      o.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
      o.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
      o.z = (uint32_t)f2bf(v[4]) | ((uint32_t)f2bf(v[5]) << 16);
      o.w = (uint32_t)f2bf(v[6]) | ((uint32_t)f2bf(v[7]) << 16);
      *reinterpret_cast<uint4*>(Y + off) = o;
      if (g.ostride == 2 && !accumulate && g.ooy == 0 && g.oox == 0) {
        // strided scatter (1x1/s2 data gradient): this kernel also writes the zeros of the three
        // positions no output pixel maps to, so the caller need not pre-fill dX
        const int b = (int)(m / g.out_img);
        const int q = (int)(m - (long long)b * g.out_img);
        const int oy = q / g.Wo[0], ox = q - oy * g.Wo[0];
        const uint4 z = make_uint4(0u, 0u, 0u, 0u);
        const bool xr = 2 * ox + 1 < g.oW, yd = 2 * oy + 1 < g.oH;
        if (xr) *reinterpret_cast<uint4*>(Y + off + g.cout) = z;
        if (yd) *reinterpret_cast<uint4*>(Y + off + (long long)g.oW * g.cout) = z;
        if (xr && yd) *reinterpret_cast<uint4*>(Y + off + (long long)(g.oW + 1) * g.cout) = z;
      }
    }
  }
}

template <int BCO, int ABL = 0, int ILV = 0, int NW = 8, int WCO = 2, int PB = PBN, int NS = PNST>
int launch_pipe(const bf16_t* X, const bf16_t* Wt, const float* bias, const bf16_t* R, const bf16_t* Mk, bf16_t* Y,
                const bf16_t* zpage, const ConvGeom& g, int relu, int accumulate, hipStream_t stream) {
  const int tiles_co = (g.cout + BCO - 1) / BCO;
  const long long tiles_m = (g.M + PB - 1) / PB;
  const long long nwg = tiles_co * tiles_m;
  if (nwg > 0x7fffffffLL) return -3;
  const size_t lds = std::max((size_t)NS * (BCO + PB) * 64, (size_t)PB * (BCO * 2 + 16));
  auto kern = conv_fwd_pipe_kernel<BCO, ABL, ILV, NW, WCO, PB, NS>;
  static bool attr_set = false;
  if (!attr_set) {
    hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr_set = true;
  }
  kern<<<(unsigned)nwg, NW * 64, lds, stream>>>(X, Wt, bias, R, Mk, Y, zpage, g, relu, accumulate, tiles_co, nullptr,
                                                  1, DualSrc{}, DualDst{});
  return (int)hipGetLastError();
}

template <int BCO, int ILV, int NW, int WCO, int PB, int NS>
int launch_pipe_dual(const bf16_t* X, const DualSrc& ds, const bf16_t* Wt, const float* bias, const bf16_t* Mk,
                     bf16_t* Y, const bf16_t* zpage, const ConvGeom& g, int relu, hipStream_t stream) {
  const int tiles_co = (g.cout + BCO - 1) / BCO;
  const long long tiles_m = (g.M + PB - 1) / PB;
  const long long nwg = tiles_co * tiles_m;
  if (nwg > 0x7fffffffLL) return -3;
  const size_t lds = std::max((size_t)NS * (BCO + PB) * 64, (size_t)PB * (BCO * 2 + 16));
  auto kern = conv_fwd_pipe_kernel<BCO, 0, ILV, NW, WCO, PB, NS, 0, 1>;
  static bool attr_set = false;
  if (!attr_set) {
    hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr_set = true;
  }
  kern<<<(unsigned)nwg, NW * 64, lds, stream>>>(X, Wt, bias, nullptr, Mk, Y, zpage, g, relu, 0, tiles_co, nullptr, 1,
                                                  ds, DualDst{});
  return (int)hipGetLastError();
}

template <int BCO, int ILV, int NW, int WCO, int PB, int NS>
int launch_pipe_dd(const bf16_t* X, const bf16_t* Wt, const bf16_t* Mk, bf16_t* Y, const DualDst& dd,
                   const bf16_t* zpage, const ConvGeom& g, hipStream_t stream) {
  const int tiles_co = (g.cout + BCO - 1) / BCO;
  const long long tiles_m = (g.M + PB - 1) / PB;
  const long long nwg = tiles_co * tiles_m;
  if (nwg > 0x7fffffffLL) return -3;
  const size_t lds = std::max((size_t)NS * (BCO + PB) * 64, (size_t)PB * (BCO * 2 + 16));
  auto kern = conv_fwd_pipe_kernel<BCO, 0, ILV, NW, WCO, PB, NS, 0, 0, 1>;
  static bool attr_set = false;
  if (!attr_set) {
    hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr_set = true;
  }
  kern<<<(unsigned)nwg, NW * 64, lds, stream>>>(X, Wt, nullptr, nullptr, Mk, Y, zpage, g, 0, 0, tiles_co, nullptr, 1,
                                                  DualSrc{}, dd);
  return (int)hipGetLastError();
}

// y[m, 8 c .. 8 c + 7] = epilogue(sum_s part[s][m][...] + bias): one thread per 16-B output chunk
__global__ __launch_bounds__(256) void pipe_splitk_epilogue(const float* __restrict__ part, int nsplit, long long M,
                                                            int cout, const float* __restrict__ bias,
                                                            const bf16_t* __restrict__ R, const bf16_t* __restrict__ Mk,
                                                            bf16_t* __restrict__ Y, int relu, int accumulate) {
  const int cv = cout >> 3;
  const long long t = (long long)blockIdx.x * 256 + threadIdx.x;
  if (t >= M * cv) return;
  const long long m = t / cv;
  const int c = (int)(t - m * cv) * 8;
  const long long off = m * cout + c;
  const long long stride = M * cout;
  f32x4 a = *reinterpret_cast<const f32x4*>(part + off), b = *reinterpret_cast<const f32x4*>(part + off + 4);
  for (int s = 1; s < nsplit; ++s) {
    a += *reinterpret_cast<const f32x4*>(part + s * stride + off);
    b += *reinterpret_cast<const f32x4*>(part + s * stride + off + 4);
  }
  float v[8] = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
  if (bias) {
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] += bias[c + q];
  }
  epi_sweep8(v, R, off, accumulate ? Y : nullptr, Mk, off, relu);
  uint4 o;
  o.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
  o.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
  o.z = (uint32_t)f2bf(v[4]) | ((uint32_t)f2bf(v[5]) << 16);
  o.w = (uint32_t)f2bf(v[6]) | ((uint32_t)f2bf(v[7]) << 16);
  *reinterpret_cast<uint4*>(Y + off) = o;
}

template <int BCO, int NW, int WCO, int PB, int NS>
int launch_pipe_sk(const bf16_t* X, const bf16_t* Wt, const float* bias, const bf16_t* R, const bf16_t* Mk, bf16_t* Y,
                   const bf16_t* zpage, const ConvGeom& g, int relu, int accumulate, int nsplit, float* part,
                   hipStream_t stream) {
  const int tiles_co = (g.cout + BCO - 1) / BCO;
  const long long tiles_m = (g.M + PB - 1) / PB;
  const long long nwg = tiles_co * tiles_m;
  if (nwg > 0x7fffffffLL || nsplit < 1 || nsplit > 64 || nsplit > (g.kh * g.kw * g.cin) / 32) return -3;
  const size_t lds = (size_t)NS * (BCO + PB) * 64;
  auto kern = conv_fwd_pipe_kernel<BCO, 0, 2, NW, WCO, PB, NS, 1>;
  static bool attr_set = false;
  if (!attr_set) {
    hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr_set = true;
  }
  kern<<<dim3((unsigned)nwg, (unsigned)nsplit), NW * 64, lds, stream>>>(X, Wt, bias, R, Mk, Y, zpage, g, relu, accumulate,
                                                                        tiles_co, part, nsplit, DualSrc{}, DualDst{});
  const long long n = g.M * (g.cout / 8);
  pipe_splitk_epilogue<<<(unsigned)((n + 255) / 256), 256, 0, stream>>>(part, nsplit, g.M, g.cout, bias, R, Mk, Y, relu,
                                                                        accumulate);
  return (int)hipGetLastError();
}

}  // namespace

// Split-K form of variants 11 (128 co x 128 px) / 12 (64 co x 128 px on 4 waves): part = nsplit * M * cout floats
// of scratch.  Requires ostride == 1 (no strided scatter), cin % 32 == 0, cout % 8 == 0, 1 <= nsplit <= 64.
MXR_API int mxr_conv_fwd_pipe_sk(const void* X, const void* Wt, const float* bias, const void* R, const void* Mk,
                                 void* Y, const void* zpage, const ConvGeom* g, int relu, int accumulate, int variant,
                                 int nsplit, float* part, hipStream_t stream) {
  if (g->cin % 32 != 0 || g->cout % 8 != 0 || g->ostride != 1) return -1;
  if (g->nlev < 1 || g->nlev > MXR_MAXLEV) return -2;
  const bf16_t *x = (const bf16_t*)X, *w = (const bf16_t*)Wt, *r = (const bf16_t*)R, *mk = (const bf16_t*)Mk;
  const bf16_t* z = (const bf16_t*)zpage;
  bf16_t* y = (bf16_t*)Y;
  switch (variant) {
    case 11: return launch_pipe_sk<128, 8, 2, 128, 3>(x, w, bias, r, mk, y, z, *g, relu, accumulate, nsplit, part, stream);
    case 12: return launch_pipe_sk<64, 4, 1, 128, 3>(x, w, bias, r, mk, y, z, *g, relu, accumulate, nsplit, part, stream);
    default: return -6;
  }
}

// variant: 0 = 256 co x 256 pixels, 1 = 128 co x 256 pixels (both 8 waves, 1 block per CU);
// 2 / 3 = the same tiles with the DMA pieces interleaved between MFMA groups, 4 / 5 = interleaved +
// s_setprio(1) around each MFMA group, 6 = 64 co x 256 pixels on 4 waves (two blocks per CU), 7 = 6 with
// s_setprio around the MFMA block; 128-pixel tiles for the small-K / big-epilogue 1x1 layers:
// 8 = 128 co (interleaved + setprio, two blocks per CU), 9 = 256 co (interleaved + setprio),
// 10 = 64 co on 4 waves (three blocks per CU); 3-deep rings (DMA two sub-stages ahead, smaller LDS):
// 11 = 128 co x 128 pix (three blocks per CU), 12 = 64 x 128 on 4 waves (four), 13 = 128 x 256 (two)
// cout % 8 == 0 (16-B epilogue chunks)
MXR_API int mxr_conv_fwd_pipe(const void* X, const void* Wt, const float* bias, const void* R, const void* Mk,
                              void* Y, const void* zpage, const ConvGeom* g, int relu, int accumulate, int variant,
                              hipStream_t stream) {
  if (g->cin % 32 != 0 || g->cout % 8 != 0) return -1;
  if (g->nlev < 1 || g->nlev > MXR_MAXLEV) return -2;
  const bf16_t *x = (const bf16_t*)X, *w = (const bf16_t*)Wt, *r = (const bf16_t*)R, *mk = (const bf16_t*)Mk;
  const bf16_t* z = (const bf16_t*)zpage;
  bf16_t* y = (bf16_t*)Y;
  switch (variant) {
    case 1: return launch_pipe<128>(x, w, bias, r, mk, y, z, *g, relu, accumulate, stream);
    case 2: return launch_pipe<256, 0, 1>(x, w, bias, r, mk, y, z, *g, relu, accumulate, stream);
    case 3: return launch_pipe<128, 0, 1>(x, w, bias, r, mk, y, z, *g, relu, accumulate, stream);
    case 4: return launch_pipe<256, 0, 2>(x, w, bias, r, mk, y, z, *g, relu, accumulate, stream);
    case 5: return launch_pipe<128, 0, 2>(x, w, bias, r, mk, y, z, *g, relu, accumulate, stream);
    case 6: return launch_pipe<64, 0, 0, 4, 1>(x, w, bias, r, mk, y, z, *g, relu, accumulate, stream);
    case 7: return launch_pipe<64, 0, 3, 4, 1>(x, w, bias, r, mk, y, z, *g, relu, accumulate, stream);
    case 8: return launch_pipe<128, 0, 2, 8, 2, 128>(x, w, bias, r, mk, y, z, *g, relu, accumulate, stream);
    case 9: return launch_pipe<256, 0, 2, 8, 2, 128>(x, w, bias, r, mk, y, z, *g, relu, accumulate, stream);
    case 10: return launch_pipe<64, 0, 0, 4, 1, 128>(x, w, bias, r, mk, y, z, *g, relu, accumulate, stream);
    case 11: return launch_pipe<128, 0, 2, 8, 2, 128, 3>(x, w, bias, r, mk, y, z, *g, relu, accumulate, stream);
    case 12: return launch_pipe<64, 0, 0, 4, 1, 128, 3>(x, w, bias, r, mk, y, z, *g, relu, accumulate, stream);
    case 13: return launch_pipe<128, 0, 2, 8, 2, 256, 3>(x, w, bias, r, mk, y, z, *g, relu, accumulate, stream);
    default: return launch_pipe<256>(x, w, bias, r, mk, y, z, *g, relu, accumulate, stream);
  }
}

// Dual-source 1x1 forward of a projection block (see DualSrc): X = branch2b output [M, cin1] (g describes the 1x1/s1
// conv over it, g.cin = cin1 + cin2 = the GEMM K, kh = kw = 1), X2 = the block input [N, H, W, cin2] read at stride s,
// Wt = W2c*s2c [cout, cin1], W1 = W1*s1 [cout, cin2], bias = the two frozen-BN shifts summed; no residual, no
// accumulate.
// variant: the pipe tiles of mxr_conv_fwd_pipe 8..13 (128-pixel tiles and the 3-deep rings) and 1 / 5.
MXR_API int mxr_conv_fwd_pipe_dual(const void* X, const void* X2, int cin1, int cin2, int H, int W, int s,
                                   const void* Wt, const void* W1, const float* bias, const void* Mk, void* Y,
                                   const void* zpage, const ConvGeom* g, int relu, int variant, hipStream_t stream) {
  if (cin1 % 32 != 0 || cin2 % 32 != 0 || g->cin != cin1 + cin2 || g->cout % 8 != 0) return -1;
  if (g->nlev != 1 || g->kh != 1 || g->kw != 1 || g->stride != 1 || g->ostride != 1 || g->pt != 0 || g->pl != 0)
    return -2;
  if (s < 1 || (g->Ho[0] - 1) * s >= H || (g->Wo[0] - 1) * s >= W || g->H[0] != g->Ho[0] || g->W[0] != g->Wo[0])
    return -4;
  const DualSrc ds{(const bf16_t*)X2, (const bf16_t*)W1, cin1, cin2, H, W, s};
  const bf16_t *x = (const bf16_t*)X, *w = (const bf16_t*)Wt, *mk = (const bf16_t*)Mk;
  const bf16_t* z = (const bf16_t*)zpage;
  bf16_t* y = (bf16_t*)Y;
  switch (variant) {
    case 1: return launch_pipe_dual<128, 0, 8, 2, 256, 4>(x, ds, w, bias, mk, y, z, *g, relu, stream);
    case 5: return launch_pipe_dual<128, 2, 8, 2, 256, 4>(x, ds, w, bias, mk, y, z, *g, relu, stream);
    case 8: return launch_pipe_dual<128, 2, 8, 2, 128, 4>(x, ds, w, bias, mk, y, z, *g, relu, stream);
    case 9: return launch_pipe_dual<256, 2, 8, 2, 128, 4>(x, ds, w, bias, mk, y, z, *g, relu, stream);
    case 10: return launch_pipe_dual<64, 0, 4, 1, 128, 4>(x, ds, w, bias, mk, y, z, *g, relu, stream);
    case 11: return launch_pipe_dual<128, 2, 8, 2, 128, 3>(x, ds, w, bias, mk, y, z, *g, relu, stream);
    case 12: return launch_pipe_dual<64, 0, 4, 1, 128, 3>(x, ds, w, bias, mk, y, z, *g, relu, stream);
    case 13: return launch_pipe_dual<128, 2, 8, 2, 256, 3>(x, ds, w, bias, mk, y, z, *g, relu, stream);
    default: return -6;
  }
}

// Dual-destination data gradient of a projection block (see DualDst): X = the block output gradient [M, K] over the
// output grid (g: 1x1/s1 GEMM, g.cin = K, g.cout = c1 + c2), Wt / W2 = the flipped W2c [c1, K] / W1 [c2, K],
// Mk = the branch2b activation (bf16 relu mask of dH2; null = none), Y = dH2 [M, c1], Y2 = dX [N, oH, oW, c2] written
// at stride os (1 or 2: the gaps' zeros too) or accumulated into (acc2, no gap writes).  variant: as the dual form.
MXR_API int mxr_conv_dgrad_pipe_dd(const void* X, const void* Wt, const void* W2, const void* Mk, void* Y, void* Y2,
                                   int c1, int c2, int os, int oH, int oW, int acc2, const void* zpage,
                                   const ConvGeom* g, int variant, hipStream_t stream) {
  if (g->cin % 32 != 0 || c1 % 8 != 0 || c2 % 8 != 0 || g->cout != c1 + c2) return -1;
  if (g->nlev != 1 || g->kh != 1 || g->kw != 1 || g->stride != 1 || g->ostride != 1 || g->pt != 0 || g->pl != 0)
    return -2;
  if ((os != 1 && os != 2) || (g->Ho[0] - 1) * os >= oH || (g->Wo[0] - 1) * os >= oW ||
      (os == 1 && (oH != g->Ho[0] || oW != g->Wo[0])))
    return -4;
  if (os == 2 && !acc2 && (((oH + 1) / 2 != g->Ho[0]) || ((oW + 1) / 2 != g->Wo[0]))) return -4;   // every gap covered
  if (((uintptr_t)Mk & 1) != 0) return -5;     // dH2's mask is the bf16 activation
  const DualDst dd{(bf16_t*)Y2, (const bf16_t*)W2, c1, c2, os, oH, oW, acc2};
  const bf16_t *x = (const bf16_t*)X, *w = (const bf16_t*)Wt, *mk = (const bf16_t*)Mk;
  const bf16_t* z = (const bf16_t*)zpage;
  bf16_t* y = (bf16_t*)Y;
  switch (variant) {
    case 1: return launch_pipe_dd<128, 0, 8, 2, 256, 4>(x, w, mk, y, dd, z, *g, stream);
    case 5: return launch_pipe_dd<128, 2, 8, 2, 256, 4>(x, w, mk, y, dd, z, *g, stream);
    case 8: return launch_pipe_dd<128, 2, 8, 2, 128, 4>(x, w, mk, y, dd, z, *g, stream);
    case 9: return launch_pipe_dd<256, 2, 8, 2, 128, 4>(x, w, mk, y, dd, z, *g, stream);
    case 10: return launch_pipe_dd<64, 0, 4, 1, 128, 4>(x, w, mk, y, dd, z, *g, stream);
    case 11: return launch_pipe_dd<128, 2, 8, 2, 128, 3>(x, w, mk, y, dd, z, *g, stream);
    case 12: return launch_pipe_dd<64, 0, 4, 1, 128, 3>(x, w, mk, y, dd, z, *g, stream);
    case 13: return launch_pipe_dd<128, 2, 8, 2, 256, 3>(x, w, mk, y, dd, z, *g, stream);
    default: return -6;
  }
}

// diagnostics: the 256x256 kernel with parts of its main loop removed (see ABL above)
MXR_API int mxr_conv_fwd_pipe_ablate(const void* X, const void* Wt, void* Y, const void* zpage, const ConvGeom* g,
                                     int abl, hipStream_t stream) {
  if (g->cin % 32 != 0 || g->cout % 8 != 0) return -1;
  const bf16_t *x = (const bf16_t*)X, *w = (const bf16_t*)Wt, *z = (const bf16_t*)zpage;
  bf16_t* y = (bf16_t*)Y;
  switch (abl) {
    case 1: return launch_pipe<256, 1>(x, w, nullptr, nullptr, nullptr, y, z, *g, 0, 0, stream);
    case 2: return launch_pipe<256, 2>(x, w, nullptr, nullptr, nullptr, y, z, *g, 0, 0, stream);
    case 3: return launch_pipe<256, 3>(x, w, nullptr, nullptr, nullptr, y, z, *g, 0, 0, stream);
    case 4: return launch_pipe<256, 0, 1>(x, w, nullptr, nullptr, nullptr, y, z, *g, 0, 0, stream);
    case 5: return launch_pipe<256, 0, 2>(x, w, nullptr, nullptr, nullptr, y, z, *g, 0, 0, stream);
    default: return launch_pipe<256, 0>(x, w, nullptr, nullptr, nullptr, y, z, *g, 0, 0, stream);
  }
}
