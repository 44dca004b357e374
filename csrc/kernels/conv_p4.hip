// 4-wave 256 x 256 NHWC bf16 implicit-GEMM convolution (forward and stride-1 data gradient) for gfx950:
// ONE wave per SIMD, each wave a 128 x 128 output block.
//
//   Y[m, co] = sum_k X_im2col[m, k] * W[co, k]      k = (ky, kx, ci), OHWI weights, K-tile = 64 channels of one tap
//
// Why this shape (profiles/r2_pmc_p8_vs_hipblaslt.txt): the 8-wave 256² kernel (conv_p8.hip) shares each
// SIMD's matrix pipe between two waves that reach every barrier together, so 30-43 % of its wave-cycles
// are parked (SQ_WAIT_ANY), and it spends 7x hipBLASLt's scalar instructions on per-half address
// arithmetic.  hipBLASLt's 256² tile runs 4 waves (one per SIMD, 128 x 128 each, 256 accumulator VGPRs of
// the 512 a lone wave may use) and parks 5 %.  Here:
//
// * tile = 256 co (A = weight rows) x 256 px (B = im2col rows); waves 2 (co) x 2 (px); acc[8][8] of
//   mfma_f32_16x16x32_bf16;
// * K-tile = 64 channels of one tap; two LDS buffers of 64 KiB (A + B, 256 rows x 128 B each); the whole
//   next K-tile is fetched by LDS-DMA while the current one is multiplied (16 x 1 KiB pieces per wave),
//   one barrier per K-tile;
// * register pipeline: the fragments of K-half 1 are read behind the MFMAs of K-half 0, and those of the
//   next K-tile's K-half 0 right after the barrier, behind the second half of K-half 1's MFMAs, so no
//   MFMA waits on an LDS read and the pipe only drains for the barrier skew;
// * the im2col gather per row: a tap-validity bit mask, the row's element offset and its level width are
//   precomputed; per K-tile the tap / channel block advance in SGPRs (no divisions in the loop);
// * LDS rows are 128 B, 16-B chunks XOR-swizzled by (row >> 1) & 7 through the DMA source address
//   (conv_p8.hip), conflict-free fragment reads;
// * epilogue: conv_p8.hip's (LDS image [256 px][256 co], 16-B stores, bias / residual / ReLU / mask /
//   accumulate).
#include "common.h"

#include "conv_common.h"

namespace {

constexpr int P4_NW = 4;
constexpr int P4_ROWB = 128;
constexpr int P4_OPB = 256 * P4_ROWB;          // 32 KiB per operand tile
constexpr int P4_BUF = 2 * P4_OPB;             // A + B
constexpr int P4_EPITCH = 256 * 2 + 16;
constexpr int P4_LDS = (2 * P4_BUF > 256 * P4_EPITCH) ? 2 * P4_BUF : 256 * P4_EPITCH;

__device__ __forceinline__ int p4_swz(int row) { return (row >> 1) & 7; }

template <int N>
__device__ __forceinline__ void p4_vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// PRIO: s_setprio 1 over the MFMA stream.  (Pinning the accumulators to AGPRs with an asm MFMA removed
// hipcc's AGPR<->VGPR shuffles but reached only ~700 TF/s: profiles/r2_p4_agpr_microbench.txt.)
template <int PRIO>
__global__ __launch_bounds__(P4_NW * 64, 1) void conv_p4_kernel(
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
  const int T = K >> 6;

  // ---- DMA slots: piece q = wave + 4 s (s = 0..7) of each operand = rows 8q .. 8q + 7; lane row 8q + lane / 8.
  // The swizzled chunk depends on (row >> 1) & 7 = (4 (q & 1) + lane / 16) & 7 and q & 1 = wave & 1.
  const int chunk = ((lane & 7) ^ ((4 * (wave & 1) + (lane >> 4)) & 7)) << 3;
  // weight rows: row = wave * 8 + lane / 8 + 32 s -> offsets a_base + 32 s K (valid while row < cout - co0)
  const int a_row0 = wave * 8 + (lane >> 3);
  const int a_base = (co0 + a_row0) * K + chunk;
  const int a_rows = g.cout - co0;
  int b_off[8], b_mw[8];             // im2col row: element offset of tap (0, 0) + chunk; valid-tap bits | level width << 16
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    const int row = (wave + 4 * s) * 8 + (lane >> 3);
    const long long m = m0 + row;
    int base = -1, iy0 = 0, ix0 = 0, Hl = 0, Wl = 0, bb, oy, ox;
    if (m < g.M) decode_row(g, m, base, iy0, ix0, Hl, Wl, bb, oy, ox);
    int mask = 0;
    if (base >= 0)
      for (int ky = 0; ky < g.kh; ++ky)
        for (int kx = 0; kx < g.kw; ++kx)
          if ((unsigned)(iy0 + ky) < (unsigned)Hl && (unsigned)(ix0 + kx) < (unsigned)Wl) mask |= 1 << (ky * g.kw + kx);
    b_mw[s] = mask | (Wl << 16);
    b_off[s] = base >= 0 ? (base + iy0 * Wl + ix0) * cin + chunk : 0;   // may be negative: only used with a valid tap
  }

  // per K-tile scalar state of the NEXT tile to issue
  int n_kt = 0, n_tap = 0, n_ky = 0, n_kx = 0, n_c0 = 0;
  auto issue_tile = [&]() {
    char* buf = smem + (n_kt & 1) * P4_BUF;
    const bool live = n_kt < T;
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const uintptr_t a = (live && a_row0 + 32 * s < a_rows) ? (uintptr_t)(Wt + a_base + (32 * s) * K + n_kt * 64)
                                                             : (uintptr_t)zpage;
      glds16((const void*)a, buf + (wave + 4 * s) * 1024);
    }
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const bool ok = live && ((b_mw[s] >> n_tap) & 1);
      const int off = b_off[s] + (n_ky * (b_mw[s] >> 16) + n_kx) * cin + n_c0;
      const uintptr_t a = ok ? (uintptr_t)(X + off) : (uintptr_t)zpage;
      glds16((const void*)a, buf + P4_OPB + (wave + 4 * s) * 1024);
    }
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
  };

  // ---- fragment read offsets (bytes in an operand image), both K-halves
  const int wm = wave >> 1, wn = wave & 1;
  const int fr = lane & 15, fq = lane >> 4;
  int aro[2], bro[2];                 // row-independent parts: the swizzle only depends on fr
#pragma unroll
  for (int k2 = 0; k2 < 2; ++k2) {
    aro[k2] = (wm * 128 + fr) * P4_ROWB + (((k2 * 4 + fq) ^ p4_swz(fr)) << 4);
    bro[k2] = P4_OPB + (wn * 128 + fr) * P4_ROWB + (((k2 * 4 + fq) ^ p4_swz(fr)) << 4);
  }

  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // fragment i of a 128-row wave block sits 16 rows = 2048 B further (the swizzle repeats every 16 rows)
  auto read = [&](bf16x8 (&fa)[8], bf16x8 (&fb)[8], const char* buf, int k2) {
#pragma unroll
    for (int i = 0; i < 8; ++i) fa[i] = *reinterpret_cast<const bf16x8*>(buf + aro[k2] + i * 16 * P4_ROWB);
#pragma unroll
    for (int j = 0; j < 8; ++j) fb[j] = *reinterpret_cast<const bf16x8*>(buf + bro[k2] + j * 16 * P4_ROWB);
  };
  auto mma = [&](const bf16x8 (&fa)[8], const bf16x8 (&fb)[8], int i0, int i1) {
#pragma unroll
    for (int i = i0; i < i1; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
  };

  // ---- prologue: K-tile 0 landed, its K-half 0 in registers
  issue_tile();
  p4_vm_wait<0>();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  bf16x8 a0[8], b0[8], a1[8], b1[8];
  read(a0, b0, smem, 0);
  if constexpr (PRIO) __builtin_amdgcn_s_setprio(1);

  for (int t = 0; t < T; ++t) {
    const char* buf = smem + (t & 1) * P4_BUF;
    // next K-tile's DMA into the other buffer (its last readers passed the previous barrier)
    issue_tile();
    // K-half 1 fragments behind K-half 0's MFMAs
    read(a1, b1, buf, 1);
    mma(a0, b0, 0, 8);
    // first half of K-half 1, then the K-tile barrier, then the next K-half 0 reads behind the second half
    mma(a1, b1, 0, 4);
    p4_vm_wait<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (t + 1 < T) read(a0, b0, smem + ((t + 1) & 1) * P4_BUF, 0);
    mma(a1, b1, 4, 8);
  }
  if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);

  // ---- epilogue: fragments -> LDS image [256 px][256 co] -> 16-B sweeps
  p4_vm_wait<0>();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __syncthreads();
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int pr = wn * 128 + j * 16 + fr;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int cl = wm * 128 + i * 16 + 4 * fq;
      const int co = co0 + cl;
      float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
      if (bias && co < g.cout) {
        const float4 bb4 = *reinterpret_cast<const float4*>(bias + co);
        v[0] += bb4.x; v[1] += bb4.y; v[2] += bb4.z; v[3] += bb4.w;
      }
      uint2 o;
      o.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
      o.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
      *reinterpret_cast<uint2*>(smem + pr * P4_EPITCH + cl * 2) = o;
    }
  }
  __syncthreads();
  const int ncv = min(256, g.cout - co0) / 8;
  for (int e = threadIdx.x; e < 256 * 32; e += P4_NW * 64) {
    const int pr = e >> 5, ch = e & 31;
    const long long m = m0 + pr;
    if (m >= g.M || ch >= ncv) continue;
    const long long off = m * g.cout + co0 + ch * 8;
    const uint4 raw = *reinterpret_cast<const uint4*>(smem + pr * P4_EPITCH + ch * 16);
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

template <int PRIO>
int launch_p4(const bf16_t* X, const bf16_t* Wt, const float* bias, const bf16_t* R, const bf16_t* Mk, bf16_t* Y,
              const bf16_t* zpage, const ConvGeom& g, int relu, int accumulate, hipStream_t stream) {
  const int tiles_co = (g.cout + 255) / 256;
  const long long tiles_m = (g.M + 255) / 256;
  const long long nwg = tiles_m * tiles_co;
  if (nwg > 0x7fffffffLL || nwg < 1) return -3;
  auto kern = conv_p4_kernel<PRIO>;
  static bool attr_set = false;
  if (!attr_set) {
    hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, P4_LDS);
    attr_set = true;
  }
  kern<<<(unsigned)nwg, P4_NW * 64, P4_LDS, stream>>>(X, Wt, bias, R, Mk, Y, zpage, g, relu, accumulate, tiles_co);
  return (int)hipGetLastError();
}

}  // namespace

// variant 0: plain; 1: s_setprio 1 over the main loop.
// Requires cin % 64 == 0, cout % 8 == 0, ostride == 1, kh * kw <= 16 and (pixels + 1) * cin, cout * K < 2^31.
MXR_API int mxr_conv_p4(const void* X, const void* Wt, const float* bias, const void* R, const void* Mk, void* Y,
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
    case 1: return launch_p4<1>(x, w, bias, r, mk, y, z, *g, relu, accumulate, stream);
    default: return launch_p4<0>(x, w, bias, r, mk, y, z, *g, relu, accumulate, stream);
  }
}
