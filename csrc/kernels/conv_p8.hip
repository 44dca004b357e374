// Phase-pipelined 256 x 256 NHWC bf16 implicit-GEMM convolution (forward and stride-1 data gradient) for
// gfx950 -- the "8-phase" GEMM structure (cdna_hip_programming.md §5, 256² template) applied to the
// convolution's implicit GEMM.
//
//   Y[m, co] = sum_k X_im2col[m, k] * W[co, k]      k = (ky, kx, ci), OHWI weights, K-tile = 64 channels of one tap
//
// The head towers and finals (the conv layers built at /root/reference/train.py:91; SURVEY §2.6 K1: 58.9 % of
// the forward MACs) are GEMMs of M = B x 22,300 pyramid pixels, N = 256 (720) channels, K = 2,304: large
// enough that the kernel's steady state is all that matters.  The earlier kernels (conv_pipe.hip,
// conv_halo.hip) consume K in 32-deep sub-stages with one barrier each; here:
//
// * tile = 256 output channels (A operand = weight rows) x 256 pixels (B operand = im2col rows), 8 waves as
//   2 (co) x 4 (px), each wave 128 co x 64 px = 8 x 4 accumulators of mfma_f32_16x16x32_bf16 (128 VGPRs);
// * K advances in 64-deep K-tiles; each operand tile (256 rows x 128 B) lives in one of two LDS buffers (128
//   KiB) and is split into two HALVES by the rows the waves consume together: A-half h = the co fragments
//   4h..4h+3 of both co wave-rows, B-half h = the px fragments 2h, 2h+1 of the four px wave-columns;
// * a K-tile is 4 phases of 16 MFMAs per wave, each phase one quadrant (4 co x 2 px fragments x K 64):
//   (A0,B0) (A0,B1) (A1,B1) (A1,B0) -- fragment registers are reused across phases, so a K-tile costs
//   the minimal 24 ds_read_b128 per wave (16 A + 8 B) and at most 64 fragment VGPRs are live;
// * LDS-DMA (global_load_lds_dwordx4, 2 per wave per half) of the NEXT K-tile runs one half per phase in
//   the order the phases need them (A0, B0, B1, A1), so every counted wait is `vmcnt(4)`: two halves stay
//   in flight across each raw `s_barrier`; phase 3 reads nothing new and has no barrier;
// * LDS images are lane-linear 128-B rows (what LDS-DMA writes); the 16-B chunk index is XOR-swizzled
//   with (row >> 1) & 7 through the DMA SOURCE address, which makes every ds_read_b128 lane group of a
//   fragment read hit 16 distinct bank slots;
// * im2col rows are gathered per tap straight from the NHWC input (a row = 64 channels = 128 B): zero
//   page outside the image / level, multi-level packed pyramids (ConvGeom) supported;
// * epilogue: accumulators -> LDS image [256 px][256 co] -> 16-B stores with bias, residual, ReLU,
//   relu-gradient mask of the consumer's input, and accumulate (conv_halo.hip's epilogue).
#include "common.h"

#include "conv_common.h"

namespace {

constexpr int P8_NW = 8;
constexpr int P8_ROWB = 128;                  // bytes per LDS row (64 bf16)
constexpr int P8_OPB = 256 * P8_ROWB;         // one operand tile
constexpr int P8_BUF = 2 * P8_OPB;            // A + B of one K-tile
constexpr int P8_EPITCH = 256 * 2 + 16;       // epilogue row pitch (bytes)
constexpr int P8_LDS = (2 * P8_BUF > 256 * P8_EPITCH) ? 2 * P8_BUF : 256 * P8_EPITCH;

template <int N>
__device__ __forceinline__ void p8_vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ int p8_swz(int row) { return (row >> 1) & 7; }

// PRIO: s_setprio 1 around each phase's MFMA block.
// STAG: ping-pong schedule -- every phase is a LOAD segment (waits, DMA issue, fragment reads) and a
// COMPUTE segment (16 MFMAs), each closed by a barrier, and waves 4-7 run one barrier behind waves
// 0-3: on every SIMD one wave computes while its partner loads.  Data is retired one phase early
// (counted vmcnt(2): one half in flight) so that the half-phase skew never reads an unretired half.
// RF: 1 = fragment reads issued before the phase's DMA pieces (their LDS latency overlaps the DMA issue);
// 2 = fragment reads issued one phase ahead of their MFMAs (PF, see the loop)
// ABL: 1 = no epilogue (diagnostics), 2 = direct-store epilogue (DS, see there), 3 = no global store
// (diagnostics), 4 = non-temporal global stores
template <int PRIO, int STAG = 0, int RF = 0, int ABL = 0>
__global__ __launch_bounds__(P8_NW * 64, 2) void conv_p8_kernel(
    const bf16_t* __restrict__ X, const bf16_t* __restrict__ Wt, const float* __restrict__ bias,
    const bf16_t* __restrict__ Rs, const bf16_t* __restrict__ Mk, bf16_t* __restrict__ Y,
    const bf16_t* __restrict__ zpage, ConvGeom g, int relu, int accumulate, int tiles_co) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wid = xcd_remap(blockIdx.x, gridDim.x);
  const int tco = wid % tiles_co;
  const long long m0 = (long long)(wid / tiles_co) * 256;
  const int co0 = tco * 256;
  const int cin = g.cin;
  const int K = g.kh * g.kw * cin;
  const int cb = cin >> 6;                       // 64-channel blocks per tap
  const int T = g.kh * g.kw * cb;                // K-tiles

  // ---- DMA slots of this lane: rows r(h, s) of each half h, piece s (2 pieces per wave per half)
  //   A-half h piece s: row = s*128 + h*64 + wave*8 + lane/8;  B-half h piece s: row = (wave/4 + 2s)*64 + h*32 + (wave%4)*8 + lane/8
  const int lr = lane >> 3;
  // weight rows of (half h, piece s): s * 128 + h * 64 + wave * 8 + lane / 8 -> offset a_base + (128 s + 64 h) K
  const int a_row0 = wave * 8 + lr;
  const int a_base = (co0 + a_row0) * K + (((lane & 7) ^ p8_swz(a_row0)) << 3);   // swizzle period 16 rows
  const int a_rows = g.cout - co0;
  // im2col rows of (half h, piece s): (wave / 4 + 2 s) * 64 + h * 32 + (wave % 4) * 8 + lane / 8;
  // per row: element offset of tap (0, 0) + swizzled chunk, and valid-tap bits | level width << 16
  int b_off[2][2], b_mw[2][2];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int rb = (wave / 4 + 2 * s) * 64 + h * 32 + (wave % 4) * 8 + lr;
      const long long m = m0 + rb;
      int base = -1, iy0 = 0, ix0 = 0, Hl = 0, Wl = 0, bb, oy, ox;
      if (m < g.M) decode_row(g, m, base, iy0, ix0, Hl, Wl, bb, oy, ox);
      int mask = 0;
      if (base >= 0)
        for (int ky = 0; ky < g.kh; ++ky)
          for (int kx = 0; kx < g.kw; ++kx)
            if ((unsigned)(iy0 + ky) < (unsigned)Hl && (unsigned)(ix0 + kx) < (unsigned)Wl)
              mask |= 1 << (ky * g.kw + kx);
      b_mw[h][s] = mask | (Wl << 16);
      b_off[h][s] = base >= 0 ? (base + iy0 * Wl + ix0) * cin + (((lane & 7) ^ p8_swz(rb)) << 3) : 0;
    }

  // scalar state of the K-tile being issued (advanced once per K-tile: no divisions in the loop)
  int n_kt = 0, n_tap = 0, n_ky = 0, n_kx = 0, n_c0 = 0;
  // issue one half of K-tile n_kt into buffer n_kt & 1: hx = 0 A-half 0, 1 B-half 0, 2 B-half 1, 3 A-half 1
  auto issue_half = [&](int hx) {
    char* buf = smem + (n_kt & 1) * P8_BUF;
    const bool live = n_kt < T;
    if (hx == 0 || hx == 3) {
      const int h = hx == 0 ? 0 : 1;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int row = a_row0 + s * 128 + h * 64;
        const uintptr_t a = (live && row < a_rows) ? (uintptr_t)(Wt + a_base + (s * 128 + h * 64) * K + n_kt * 64)
                                                   : (uintptr_t)zpage;
        glds16((const void*)a, buf + (s * 128 + h * 64 + wave * 8) * P8_ROWB);
      }
    } else {
      const int h = hx - 1;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const bool ok = live && ((b_mw[h][s] >> n_tap) & 1);
        const int off = b_off[h][s] + (n_ky * (b_mw[h][s] >> 16) + n_kx) * cin + n_c0;
        const uintptr_t a = ok ? (uintptr_t)(X + off) : (uintptr_t)zpage;
        glds16((const void*)a, buf + P8_OPB + ((wave / 4 + 2 * s) * 64 + h * 32 + (wave % 4) * 8) * P8_ROWB);
      }
    }
    if (hx == 3) {
      ++n_kt;
      n_c0 += 64;
      if (n_c0 == cin) {
        n_c0 = 0;
        ++n_tap;
        if (++n_kx == g.kw) {
          n_kx = 0;
          ++n_ky;
        }
      }
    }
  };

  // ---- fragment read offsets (bytes inside an operand image), both K-halves
  const int wm = wave >> 2, wn = wave & 3;
  const int fr = lane & 15, fq = lane >> 4;
  int aro[8][2], bro[4][2];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int row = wm * 128 + i * 16 + fr;
#pragma unroll
    for (int k2 = 0; k2 < 2; ++k2) aro[i][k2] = row * P8_ROWB + (((k2 * 4 + fq) ^ p8_swz(row)) << 4);
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int row = wn * 64 + j * 16 + fr;
#pragma unroll
    for (int k2 = 0; k2 < 2; ++k2) bro[j][k2] = P8_OPB + row * P8_ROWB + (((k2 * 4 + fq) ^ p8_swz(row)) << 4);
  }

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto mma = [&](const bf16x8 (&fa)[4][2], const bf16x8 (&fb)[2][2], int i0, int j0) {
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int k2 = 0; k2 < 2; ++k2)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i0 + i][j0 + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][k2], fb[j][k2], acc[i0 + i][j0 + j], 0, 0, 0);
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);
  };
  auto read_a = [&](bf16x8 (&fa)[4][2], const char* buf, int i0) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int k2 = 0; k2 < 2; ++k2) fa[i][k2] = *reinterpret_cast<const bf16x8*>(buf + aro[i0 + i][k2]);
  };
  auto read_b = [&](bf16x8 (&fb)[2][2], const char* buf, int j0) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int k2 = 0; k2 < 2; ++k2) fb[j][k2] = *reinterpret_cast<const bf16x8*>(buf + bro[j0 + j][k2]);
  };
  auto sync = [&]() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };

  // ---- prologue: K-tile 0, halves in consumption order
#pragma unroll
  for (int hx = 0; hx < 4; ++hx) issue_half(hx);

  if constexpr (STAG) {
    auto bar = [&]() {
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    };
    p8_vm_wait<4>();          // A-half 0 and B-half 0 of K-tile 0
    sync();
    if (wave >= 4) bar();     // the stagger: waves 4-7 one barrier behind
    for (int t = 0; t < T; ++t) {
      const char* buf = smem + (t & 1) * P8_BUF;
      bf16x8 fa0[4][2], fa1[4][2], fb0[2][2], fb1[2][2];
      // phase 0: retire B-half 1 (phase 1), issue, read A0 + B0
      p8_vm_wait<2>();
      issue_half(0);
      read_a(fa0, buf, 0);
      read_b(fb0, buf, 0);
      sync();
      mma(fa0, fb0, 0, 0);
      bar();
      // phase 1: retire A-half 1 (phase 2), read B1
      p8_vm_wait<2>();
      issue_half(1);
      read_b(fb1, buf, 2);
      sync();
      mma(fa0, fb1, 0, 2);
      bar();
      // phase 2: read A1
      issue_half(2);
      read_a(fa1, buf, 4);
      sync();
      mma(fa1, fb1, 4, 2);
      bar();
      // phase 3: retire the next K-tile's A-half 0 / B-half 0 (its phase 0)
      p8_vm_wait<2>();
      issue_half(3);
      sync();
      mma(fa1, fb0, 4, 0);
      bar();
    }
    if (wave < 4) bar();      // equal barrier counts for both halves
  } else if constexpr (RF == 2) {
    // PF: every fragment read but one is issued a whole phase (16 MFMAs) before its MFMAs need it, and
    // no barrier waits on LDS reads (lgkmcnt is only counted by hipcc in front of the MFMAs).  Reads:
    // P0 B0 (its latency is the one exposed per K-tile) + B1, P1 A1, P3 the next tile's A0; the DMA
    // order (A0 B0 B1 A1 of the next K-tile, one half per phase) gives counted waits vmcnt(2) at P0 / P1
    // and vmcnt(4) at P3; P2 reads nothing and has no barrier.  Registers: the same four fragment sets.
    auto bar = [&]() {
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    };
    bf16x8 fa0[4][2], fa1[4][2], fb0[2][2], fb1[2][2];
    p8_vm_wait<6>();          // A-half 0 of K-tile 0
    sync();
    read_a(fa0, smem, 0);
    for (int t = 0; t < T; ++t) {
      const char* buf = smem + (t & 1) * P8_BUF;
      const char* nbuf = smem + ((t + 1) & 1) * P8_BUF;
      // P0: both B-halves of tile t landed
      p8_vm_wait<2>();
      bar();
      read_b(fb0, buf, 0);
      read_b(fb1, buf, 2);
      issue_half(0);
      mma(fa0, fb0, 0, 0);
      // P1: A-half 1 of tile t
      p8_vm_wait<2>();
      bar();
      read_a(fa1, buf, 4);
      issue_half(1);
      mma(fa0, fb1, 0, 2);
      // P2
      issue_half(2);
      mma(fa1, fb1, 4, 2);
      // P3: A-half 0 of tile t + 1 (zero-page rows past the last tile)
      p8_vm_wait<4>();
      bar();
      read_a(fa0, nbuf, 0);
      issue_half(3);
      mma(fa1, fb0, 4, 0);
    }
  } else {
  for (int t = 0; t < T; ++t) {
    const char* buf = smem + (t & 1) * P8_BUF;
    bf16x8 fa0[4][2], fa1[4][2], fb0[2][2], fb1[2][2];
    // phase 0: A-half 0 + B-half 0 of tile t
    p8_vm_wait<4>();
    sync();
    if constexpr (!RF) issue_half(0);
    read_a(fa0, buf, 0);
    read_b(fb0, buf, 0);
    if constexpr (RF) issue_half(0);
    mma(fa0, fb0, 0, 0);
    // phase 1: B-half 1
    p8_vm_wait<4>();
    sync();
    if constexpr (!RF) issue_half(1);
    read_b(fb1, buf, 2);
    if constexpr (RF) issue_half(1);
    mma(fa0, fb1, 0, 2);
    // phase 2: A-half 1
    p8_vm_wait<4>();
    sync();
    if constexpr (!RF) issue_half(2);
    read_a(fa1, buf, 4);
    if constexpr (RF) issue_half(2);
    mma(fa1, fb1, 4, 2);
    // phase 3: nothing new to read (no barrier needed: the half it refills was last read two phases ago)
    issue_half(3);
    mma(fa1, fb0, 4, 0);
  }
  }

  if constexpr (ABL == 1) {   // diagnostics: no epilogue (accumulators kept live, nothing stored)
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) asm volatile("" ::"v"(acc[i][j]));
    p8_vm_wait<0>();
    return;
  }
  if constexpr (ABL == 2) {
    // DS epilogue: straight from the accumulators, 8-B stores of 4 consecutive channels per lane (a wave's
    // 8 co fragments fill whole 256-B row pieces, merged in L2) -- no LDS image, no block barrier, so a
    // block's epilogue is its stores' issue time and the CU takes the next block while they drain.
    // (Loading every fragment's residual / accumulate / mask operands up front measured slower: 0.477 vs
    // 0.419 ms on the head layer.)
    p8_vm_wait<0>();   // the tail's zero-page DMA lands before the block (and its LDS) retires
    float4 bv[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) bv[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (bias) {
#pragma unroll
      for (int i = 0; i < 8; ++i)
        bv[i] = *reinterpret_cast<const float4*>(bias + min(co0 + wm * 128 + i * 16 + 4 * fq, g.cout - 4));
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const long long m = m0 + wn * 64 + j * 16 + fr;
      if (m >= g.M) continue;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int co = co0 + wm * 128 + i * 16 + 4 * fq;
        if (co >= g.cout) continue;
        const long long off = m * g.cout + co;
        float v[4] = {acc[i][j][0] + bv[i].x, acc[i][j][1] + bv[i].y, acc[i][j][2] + bv[i].z, acc[i][j][3] + bv[i].w};
        if (Rs) {
          const uint2 rr = *reinterpret_cast<const uint2*>(Rs + off);
          v[0] += bf2f((bf16_t)(rr.x & 0xffff)); v[1] += bf2f((bf16_t)(rr.x >> 16));
          v[2] += bf2f((bf16_t)(rr.y & 0xffff)); v[3] += bf2f((bf16_t)(rr.y >> 16));
        }
        if (accumulate) {
          const uint2 rr = *reinterpret_cast<const uint2*>(Y + off);
          v[0] += bf2f((bf16_t)(rr.x & 0xffff)); v[1] += bf2f((bf16_t)(rr.x >> 16));
          v[2] += bf2f((bf16_t)(rr.y & 0xffff)); v[3] += bf2f((bf16_t)(rr.y >> 16));
        }
        if (relu) {
#pragma unroll
          for (int q = 0; q < 4; ++q) v[q] = fmaxf(v[q], 0.f);
        }
        if (Mk) {
          const uint2 mm = *reinterpret_cast<const uint2*>(Mk + off);
          if (!(bf2f((bf16_t)(mm.x & 0xffff)) > 0.f)) v[0] = 0.f;
          if (!(bf2f((bf16_t)(mm.x >> 16)) > 0.f)) v[1] = 0.f;
          if (!(bf2f((bf16_t)(mm.y & 0xffff)) > 0.f)) v[2] = 0.f;
          if (!(bf2f((bf16_t)(mm.y >> 16)) > 0.f)) v[3] = 0.f;
        }
        uint2 o;
        o.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
        o.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
        *reinterpret_cast<uint2*>(Y + off) = o;
      }
    }
    return;
  }
  // ---- epilogue: fragments -> LDS image [256 px][256 co] -> 16-B sweeps (conv_halo.hip's two passes)
  p8_vm_wait<0>();   // the tail's zero-page DMA must land before the LDS is reused
  // the bias of this lane's 8 channel groups, loaded together (one per fragment, each waited on
  // before its use, cost ~0.5 us apiece: a quarter of the kernel)
  float4 bv[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) bv[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  if (bias) {                    // (channels past cout read a valid bias entry; their outputs are not stored)
#pragma unroll
    for (int i = 0; i < 8; ++i)
      bv[i] = *reinterpret_cast<const float4*>(bias + min(co0 + wm * 128 + i * 16 + 4 * fq, g.cout - 4));
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __syncthreads();
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int pr = wn * 64 + j * 16 + fr;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int cl = wm * 128 + i * 16 + 4 * fq;
      float v[4] = {acc[i][j][0] + bv[i].x, acc[i][j][1] + bv[i].y, acc[i][j][2] + bv[i].z, acc[i][j][3] + bv[i].w};
      uint2 o;
      o.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
      o.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
      *reinterpret_cast<uint2*>(smem + pr * P8_EPITCH + cl * 2) = o;
    }
  }
  __syncthreads();
  const int ncv = min(256, g.cout - co0) / 8;
  // residual / accumulate / mask operands loaded 4 chunks at a time ahead of their use (conv_pipe.hip)
  const bf16_t* Yacc = accumulate ? Y : nullptr;
  const bool pre = Rs != nullptr || Yacc != nullptr || Mk != nullptr;   // uniform
  constexpr int P8_NIT = 256 * 32 / (P8_NW * 64), P8_EPG = 4;
  static_assert(P8_NIT % P8_EPG == 0, "epilogue groups");
  Epi8 ep[P8_EPG];
#pragma unroll 1
  for (int g0 = 0; g0 < P8_NIT; g0 += P8_EPG) {
    if (pre) {
#pragma unroll
      for (int k = 0; k < P8_EPG; ++k) {
        const int e = threadIdx.x + (g0 + k) * P8_NW * 64;
        const int pr = e >> 5, ch = e & 31;
        const long long m = m0 + pr;
        if (m < g.M && ch < ncv) {
          const long long off = m * g.cout + co0 + ch * 8;
          epi_load8(ep[k], Rs, off, Yacc, Mk, off);
        }
      }
    }
#pragma unroll
  for (int k = 0; k < P8_EPG; ++k) {
    const int e = threadIdx.x + (g0 + k) * P8_NW * 64;
    const int pr = e >> 5, ch = e & 31;
    const long long m = m0 + pr;
    if (m >= g.M || ch >= ncv) continue;
    const long long off = m * g.cout + co0 + ch * 8;
    const uint4 raw = *reinterpret_cast<const uint4*>(smem + pr * P8_EPITCH + ch * 16);
    const uint32_t rw[4] = {raw.x, raw.y, raw.z, raw.w};
    float v[8];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      v[2 * q] = bf2f((bf16_t)(rw[q] & 0xffff));
      v[2 * q + 1] = bf2f((bf16_t)(rw[q] >> 16));
    }
    if (pre) {
      epi_apply8(v, ep[k], Rs, Yacc, Mk, relu);
    } else if (relu) {
#pragma unroll
      for (int t = 0; t < 8; ++t) v[t] = fmaxf(v[t], 0.f);
    }
    uint4 o;
    o.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
    o.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
    o.z = (uint32_t)f2bf(v[4]) | ((uint32_t)f2bf(v[5]) << 16);
    o.w = (uint32_t)f2bf(v[6]) | ((uint32_t)f2bf(v[7]) << 16);
    if constexpr (ABL == 3) {            // diagnostics: everything but the global store
      asm volatile("" ::"v"(o.x), "v"(o.y), "v"(o.z), "v"(o.w));
    } else if constexpr (ABL == 4) {     // non-temporal (streaming) stores
      typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
      __builtin_nontemporal_store(u32x4{o.x, o.y, o.z, o.w}, reinterpret_cast<u32x4*>(Y + off));
    } else {
      *reinterpret_cast<uint4*>(Y + off) = o;
    }
  }
  }
}

template <int PRIO, int STAG, int RF = 0, int ABL = 0>
int launch_p8(const bf16_t* X, const bf16_t* Wt, const float* bias, const bf16_t* R, const bf16_t* Mk, bf16_t* Y,
              const bf16_t* zpage, const ConvGeom& g, int relu, int accumulate, hipStream_t stream) {
  const int tiles_co = (g.cout + 255) / 256;
  const long long tiles_m = (g.M + 255) / 256;
  const long long nwg = tiles_m * tiles_co;
  if (nwg > 0x7fffffffLL || nwg < 1) return -3;
  auto kern = conv_p8_kernel<PRIO, STAG, RF, ABL>;
  static bool attr_set = false;
  if (!attr_set) {
    hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, P8_LDS);
    attr_set = true;
  }
  kern<<<(unsigned)nwg, P8_NW * 64, P8_LDS, stream>>>(X, Wt, bias, R, Mk, Y, zpage, g, relu, accumulate, tiles_co);
  return (int)hipGetLastError();
}

}  // namespace

// variant 0: plain; 1: s_setprio 1 around the MFMA blocks; 2 / 3: ping-pong stagger with / without s_setprio;
// 4 / 5: fragment reads ahead of the DMA pieces, with / without s_setprio; 6 / 7: fragment reads one phase
// ahead of their MFMAs, without / with s_setprio; 8 / 10: 6 / 7 with the direct-store epilogue (DS).
// Requires cin % 64 == 0, cout % 8 == 0, ostride == 1, kh * kw <= 16 and (pixels + 1) * cin, cout * K < 2^31.
MXR_API int mxr_conv_p8(const void* X, const void* Wt, const float* bias, const void* R, const void* Mk, void* Y,
                        const void* zpage, const ConvGeom* g, int relu, int accumulate, int variant,
                        hipStream_t stream) {
  if (g->cin % 64 != 0 || g->cout % 8 != 0 || g->kh * g->kw > 16) return -1;
  if (g->ostride != 1 || g->nlev < 1 || g->nlev > MXR_MAXLEV) return -2;
  const long long K = (long long)g->kh * g->kw * g->cin;
  if ((g->M + 1) * (long long)std::max(g->cin, g->cout) >= (1LL << 31) || g->cout * K >= (1LL << 31)) return -4;
  const bf16_t *x = (const bf16_t*)X, *w = (const bf16_t*)Wt, *r = (const bf16_t*)R, *mk = (const bf16_t*)Mk;
  const bf16_t* z = (const bf16_t*)zpage;
  bf16_t* y = (bf16_t*)Y;
  switch (variant) {
    case 1: return launch_p8<1, 0>(x, w, bias, r, mk, y, z, *g, relu, accumulate, stream);
    case 2: return launch_p8<1, 1>(x, w, bias, r, mk, y, z, *g, relu, accumulate, stream);
    case 3: return launch_p8<0, 1>(x, w, bias, r, mk, y, z, *g, relu, accumulate, stream);
    case 4: return launch_p8<1, 0, 1>(x, w, bias, r, mk, y, z, *g, relu, accumulate, stream);
    case 5: return launch_p8<0, 0, 1>(x, w, bias, r, mk, y, z, *g, relu, accumulate, stream);
    case 6: return launch_p8<0, 0, 2>(x, w, bias, r, mk, y, z, *g, relu, accumulate, stream);
    case 7: return launch_p8<1, 0, 2>(x, w, bias, r, mk, y, z, *g, relu, accumulate, stream);
    case 8: return launch_p8<0, 0, 2, 2>(x, w, bias, r, mk, y, z, *g, relu, accumulate, stream);
    case 9: return launch_p8<0, 0, 2, 1>(x, w, bias, r, mk, y, z, *g, relu, accumulate, stream);   // diagnostics
    case 10: return launch_p8<1, 0, 2, 2>(x, w, bias, r, mk, y, z, *g, relu, accumulate, stream);
    case 11: return launch_p8<0, 0, 2, 3>(x, w, bias, r, mk, y, z, *g, relu, accumulate, stream);   // diagnostics
    case 12: return launch_p8<0, 0, 2, 4>(x, w, bias, r, mk, y, z, *g, relu, accumulate, stream);
    default: return launch_p8<0, 0>(x, w, bias, r, mk, y, z, *g, relu, accumulate, stream);
  }
}
