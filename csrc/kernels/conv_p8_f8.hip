// FP8 (e4m3 x e4m3) phase-pipelined 256 x 256 NHWC implicit-GEMM convolution for gfx950 -- conv_p8.hip's
// PF schedule with the operand bytes carrying twice the K (BASELINE config 5: fp8 weights + activations).
//
//   y[pix, co] = acc * inv_x * inv_w[co] + bias[co] (+ residual) (relu)  -> bf16 (+ fused fp8 copy)
//
// Everything that moves bytes is conv_p8.hip's: 128-B LDS rows (now 128 channels of one tap), the same
// two K-tile buffers, LDS-DMA halves issued one per phase (A0 B0 B1 A1), swizzled lane-linear images and
// the PF read schedule (fragment reads one phase ahead, counted vmcnt(2/2/4) waits, 3 barriers per
// K-tile).  Only the product changes: the two 16-B chunks a lane reads per fragment (chunks fq and 4 + fq
// of its row) form the 32-B operand of ONE v_mfma_scale_f32_16x16x128_f8f6f4 (unit block scales; the
// real per-tensor activation / per-channel weight scales are applied in the epilogue) instead of two
// bf16 16x16x32 MFMAs.  A and B lanes hold the same byte positions, so the contraction pairs identical
// k whatever the instruction's internal k order; the accumulator map is dtype-independent (as bf16).
// Per K-tile the MFMA cycles, LDS reads and DMA bytes equal the bf16 kernel's while the K-tile covers
// twice the reduction: half the K-tiles per output tile.
//
// Epilogue: conv_pipe_f8.hip's (scales + bias into an LDS image, then 16-B sweeps with residual / ReLU,
// the delayed-scaling fp8 copy for the next layer and one amax atomic per block).
#include <algorithm>

#include "common.h"

#include "conv_common.h"
#include "fp8_common.h"

typedef __attribute__((ext_vector_type(8))) int i32x8;
typedef __attribute__((ext_vector_type(4))) int i32x4;

namespace {

constexpr int Q8_NW = 8;
constexpr int Q8_ROWB = 128;                  // bytes per LDS row (128 fp8)
constexpr int Q8_OPB = 256 * Q8_ROWB;
constexpr int Q8_BUF = 2 * Q8_OPB;
constexpr int Q8_EPITCH = 256 * 2 + 16;
constexpr int Q8_LDS = (2 * Q8_BUF > 256 * Q8_EPITCH) ? 2 * Q8_BUF : 256 * Q8_EPITCH;

// Epilogue scales of a lane's 8 channel groups (co = co_lane + 16 i), loaded together: the combined
// dequantisation scale inv_x * inv_w[co] and the bias (channels past cout read a valid entry; their
// outputs are not stored).
__device__ __forceinline__ void q8_scales(const float* inv_x, const float* inv_w, const float* bias, int cout,
                                          int co_lane, float4 (&wv)[8], float4 (&bv)[8]) {
  const float sx = *inv_x;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const float4 w4 = *reinterpret_cast<const float4*>(inv_w + min(co_lane + 16 * i, cout - 4));
    wv[i] = make_float4(sx * w4.x, sx * w4.y, sx * w4.z, sx * w4.w);
    bv[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  if (bias) {
#pragma unroll
    for (int i = 0; i < 8; ++i) bv[i] = *reinterpret_cast<const float4*>(bias + min(co_lane + 16 * i, cout - 4));
  }
}

template <int N>
__device__ __forceinline__ void q8_vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ int q8_swz(int row) { return (row >> 1) & 7; }

__device__ __forceinline__ i32x8 q8_cat(const i32x4& lo, const i32x4& hi) {
  return i32x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

// ABL: 1 = no epilogue (diagnostics: accumulators kept live, nothing stored)
// BF: 1 = data-gradient form: the im2col operand (dY) and the fused fp8 copy of the output (dX, for the
// next data gradient) are e5m2 (gradients need the range), the weights stay e4m3
template <int PRIO, int ABL = 0, int BF = 0>
__global__ __launch_bounds__(Q8_NW * 64, 2) void conv_p8_f8_kernel(
    const uint8_t* __restrict__ X, const uint8_t* __restrict__ Wt, const float* __restrict__ inv_x,
    const float* __restrict__ inv_w, const float* __restrict__ bias, const bf16_t* __restrict__ Rs,
    const bf16_t* __restrict__ Mk, bf16_t* __restrict__ Y, const uint8_t* __restrict__ zpage, ConvGeom g, int relu,
    int accumulate, int tiles_co, F8Out fo) {
  constexpr float QMAX = BF ? 57344.f : 448.f;   // largest finite value of the emitted fp8 format
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wid = xcd_remap(blockIdx.x, gridDim.x);
  const int tco = wid % tiles_co;
  const long long m0 = (long long)(wid / tiles_co) * 256;
  const int co0 = tco * 256;
  const int cin = g.cin;
  const int K = g.kh * g.kw * cin;
  const int T = g.kh * g.kw * (cin >> 7);        // K-tiles of 128 channels

  const int lr = lane >> 3;
  const int a_row0 = wave * 8 + lr;
  const int a_base = (co0 + a_row0) * K + (((lane & 7) ^ q8_swz(a_row0)) << 4);
  const int a_rows = g.cout - co0;
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
      b_off[h][s] = base >= 0 ? (base + iy0 * Wl + ix0) * cin + (((lane & 7) ^ q8_swz(rb)) << 4) : 0;
    }

  int n_kt = 0, n_tap = 0, n_ky = 0, n_kx = 0, n_c0 = 0;
  auto issue_half = [&](int hx) {
    char* buf = smem + (n_kt & 1) * Q8_BUF;
    const bool live = n_kt < T;
    if (hx == 0 || hx == 3) {
      const int h = hx == 0 ? 0 : 1;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int row = a_row0 + s * 128 + h * 64;
        const uintptr_t a = (live && row < a_rows) ? (uintptr_t)(Wt + a_base + (s * 128 + h * 64) * K + n_kt * 128)
                                                   : (uintptr_t)zpage;
        glds16((const void*)a, buf + (s * 128 + h * 64 + wave * 8) * Q8_ROWB);
      }
    } else {
      const int h = hx - 1;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const bool ok = live && ((b_mw[h][s] >> n_tap) & 1);
        const int off = b_off[h][s] + (n_ky * (b_mw[h][s] >> 16) + n_kx) * cin + n_c0;
        const uintptr_t a = ok ? (uintptr_t)(X + off) : (uintptr_t)zpage;
        glds16((const void*)a, buf + Q8_OPB + ((wave / 4 + 2 * s) * 64 + h * 32 + (wave % 4) * 8) * Q8_ROWB);
      }
    }
    if (hx == 3) {
      ++n_kt;
      n_c0 += 128;
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

  const int wm = wave >> 2, wn = wave & 3;
  const int fr = lane & 15, fq = lane >> 4;
  // fragment i / j of a wave block is 16 rows = 2048 B further (the swizzle repeats every 16 rows)
  int aro[2], bro[2];
#pragma unroll
  for (int k2 = 0; k2 < 2; ++k2) {
    aro[k2] = (wm * 128 + fr) * Q8_ROWB + (((k2 * 4 + fq) ^ q8_swz(fr)) << 4);
    bro[k2] = Q8_OPB + (wn * 64 + fr) * Q8_ROWB + (((k2 * 4 + fq) ^ q8_swz(fr)) << 4);
  }

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto mma = [&](const i32x8 (&fa)[4], const i32x8 (&fb)[2], int i0, int j0) {
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        acc[i0 + i][j0 + j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(fa[i], fb[j], acc[i0 + i][j0 + j],
                                                                              0, BF, 0, 127, 0, 127);
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);
    // pin the phase's results here (an opaque use the barriers cannot pass): hipcc otherwise sinks all 32
    // MFMAs of a K-tile to the loop end, hoists every fragment read above them and spills
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) asm volatile("" : "+v"(acc[i0 + i][j0 + j]));
  };
  auto read_a = [&](i32x8 (&fa)[4], const char* buf, int i0) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
      fa[i] = q8_cat(*reinterpret_cast<const i32x4*>(buf + aro[0] + (i0 + i) * 16 * Q8_ROWB),
                     *reinterpret_cast<const i32x4*>(buf + aro[1] + (i0 + i) * 16 * Q8_ROWB));
  };
  auto read_b = [&](i32x8 (&fb)[2], const char* buf, int j0) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
      fb[j] = q8_cat(*reinterpret_cast<const i32x4*>(buf + bro[0] + (j0 + j) * 16 * Q8_ROWB),
                     *reinterpret_cast<const i32x4*>(buf + bro[1] + (j0 + j) * 16 * Q8_ROWB));
  };
  auto bar = [&]() {
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };

#pragma unroll
  for (int hx = 0; hx < 4; ++hx) issue_half(hx);
  i32x8 fa0[4], fa1[4], fb0[2], fb1[2];
  q8_vm_wait<6>();          // A-half 0 of K-tile 0
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  bar();
  read_a(fa0, smem, 0);
  for (int t = 0; t < T; ++t) {
    const char* buf = smem + (t & 1) * Q8_BUF;
    const char* nbuf = smem + ((t + 1) & 1) * Q8_BUF;
    q8_vm_wait<2>();
    bar();
    read_b(fb0, buf, 0);
    read_b(fb1, buf, 2);
    issue_half(0);
    mma(fa0, fb0, 0, 0);
    q8_vm_wait<2>();
    bar();
    read_a(fa1, buf, 4);
    issue_half(1);
    mma(fa0, fb1, 0, 2);
    issue_half(2);
    mma(fa1, fb1, 4, 2);
    q8_vm_wait<4>();
    bar();
    read_a(fa0, nbuf, 0);
    issue_half(3);
    mma(fa1, fb0, 4, 0);
  }

  if constexpr (ABL == 1) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) asm volatile("" ::"v"(acc[i][j]));
    q8_vm_wait<0>();
    return;
  }
  // ---- epilogue: scaled + biased bf16 into an LDS image [256 px][256 co], then 16-B sweeps
  q8_vm_wait<0>();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __syncthreads();
  float4 wv[8], bv[8];
  q8_scales(inv_x, inv_w, bias, g.cout, co0 + wm * 128 + 4 * fq, wv, bv);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int pr = wn * 64 + j * 16 + fr;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int cl = wm * 128 + i * 16 + 4 * fq;
      float v[4] = {acc[i][j][0] * wv[i].x + bv[i].x, acc[i][j][1] * wv[i].y + bv[i].y,
                    acc[i][j][2] * wv[i].z + bv[i].z, acc[i][j][3] * wv[i].w + bv[i].w};
      uint2 o;
      o.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
      o.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
      *reinterpret_cast<uint2*>(smem + pr * Q8_EPITCH + cl * 2) = o;
    }
  }
  __syncthreads();
  const int ncv = min(256, g.cout - co0) / 8;
  float qs = 0.f, tmax = 0.f;
  if (fo.amax3) {
    const float prev = fo.amax3[(fo.phase + 2) % 3];
    qs = prev > 0.f ? QMAX / (fo.margin * prev) : 0.f;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      fo.amax3[(fo.phase + 1) % 3] = 0.f;
      if (fo.inv_out) *fo.inv_out = fo.margin * prev / QMAX;
    }
  }
  for (int e = threadIdx.x; e < 256 * 32; e += Q8_NW * 64) {
    const int pr = e >> 5, ch = e & 31;
    const long long m = m0 + pr;
    if (m >= g.M || ch >= ncv) continue;
    const long long off = m * g.cout + co0 + ch * 8;
    const uint4 raw = *reinterpret_cast<const uint4*>(smem + pr * Q8_EPITCH + ch * 16);
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
    if (fo.amax3) {
#pragma unroll
      for (int q = 0; q < 8; ++q) tmax = fmaxf(tmax, fabsf(v[q]));
      if (fo.Yq) {
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
  if (fo.amax3) {   // block max -> one atomic per block (values >= 0: int order == float order)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) tmax = fmaxf(tmax, __shfl_xor(tmax, o));
    __syncthreads();
    float* red = reinterpret_cast<float*>(smem);
    if (lane == 0) red[wave] = tmax;
    __syncthreads();
    if (threadIdx.x == 0) {
      float mx = red[0];
#pragma unroll
      for (int w = 1; w < Q8_NW; ++w) mx = fmaxf(mx, red[w]);
      atomicMax(reinterpret_cast<int*>(fo.amax3 + fo.phase), __float_as_int(mx));
    }
  }
}

template <int PRIO, int ABL = 0, int BF = 0>
int launch_p8_f8(const uint8_t* X, const uint8_t* W, const float* ix, const float* iw, const float* bias,
                 const bf16_t* R, const bf16_t* Mk, bf16_t* Y, const uint8_t* z, const ConvGeom& g, int relu,
                 int accumulate, const F8Out& fo, hipStream_t stream) {
  const int tiles_co = (g.cout + 255) / 256;
  const long long tiles_m = (g.M + 255) / 256;
  const long long nwg = tiles_m * tiles_co;
  if (nwg > 0x7fffffffLL || nwg < 1) return -3;
  auto kern = conv_p8_f8_kernel<PRIO, ABL, BF>;
  static bool attr_set = false;
  if (!attr_set) {
    hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, Q8_LDS);
    attr_set = true;
  }
  kern<<<(unsigned)nwg, Q8_NW * 64, Q8_LDS, stream>>>(X, W, ix, iw, bias, R, Mk, Y, z, g, relu, accumulate, tiles_co,
                                                      fo);
  return (int)hipGetLastError();
}

}  // namespace

// X: fp8 NHWC activations (scale *inv_x), Wt: fp8 OHWI weights (row scale inv_w[co]), Y: bf16 (R residual, Mk
// relu-gradient mask, accumulate: Y += result); Yq / amax3 / inv_out / phase / margin: fused fp8 output for the
// next layer (F8Out; all null = off).
// variant 0: plain; 1: s_setprio 1 around the MFMA blocks; 4 / 5: 0 / 1 in the data-gradient form (BF: e5m2
// im2col operand and e5m2 fused output); 9: diagnostics (no epilogue).
// Requires cin % 128 == 0, cout % 8 == 0, ostride == 1, kh * kw <= 16, (pixels + 1) * cin and cout * K < 2^31.
MXR_API int mxr_conv_p8_f8(const void* X, const void* Wt, const float* inv_x, const float* inv_w, const float* bias,
                           const void* R, const void* Mk, void* Y, const void* zpage, const ConvGeom* g, int relu,
                           int accumulate, void* Yq, float* amax3, float* inv_out, int phase, float margin, int variant,
                           hipStream_t stream) {
  if (g->cin % 128 != 0 || g->cout % 8 != 0 || g->kh * g->kw > 16) return -1;
  if (g->ostride != 1 || g->nlev < 1 || g->nlev > MXR_MAXLEV) return -2;
  const long long K = (long long)g->kh * g->kw * g->cin;
  if ((g->M + 1) * (long long)std::max(g->cin, g->cout) >= (1LL << 31) || g->cout * K >= (1LL << 31)) return -4;
  if (Yq && !amax3) return -5;
  const uint8_t *x = (const uint8_t*)X, *w = (const uint8_t*)Wt, *z = (const uint8_t*)zpage;
  const bf16_t *r = (const bf16_t*)R, *mk = (const bf16_t*)Mk;
  bf16_t* y = (bf16_t*)Y;
  const F8Out fo{(uint8_t*)Yq, amax3, inv_out, phase % 3, margin};
  switch (variant) {
    case 1: return launch_p8_f8<1>(x, w, inv_x, inv_w, bias, r, mk, y, z, *g, relu, accumulate, fo, stream);
    case 4: return launch_p8_f8<0, 0, 1>(x, w, inv_x, inv_w, bias, r, mk, y, z, *g, relu, accumulate, fo, stream);
    case 5: return launch_p8_f8<1, 0, 1>(x, w, inv_x, inv_w, bias, r, mk, y, z, *g, relu, accumulate, fo, stream);
    case 9: return launch_p8_f8<0, 1>(x, w, inv_x, inv_w, bias, r, mk, y, z, *g, relu, accumulate, fo, stream);
    default: return launch_p8_f8<0>(x, w, inv_x, inv_w, bias, r, mk, y, z, *g, relu, accumulate, fo, stream);
  }
}
