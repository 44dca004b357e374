// FP8 (e4m3fn x e4m3fn) deep-pipelined NHWC implicit-GEMM convolution for gfx950 (BASELINE config 5:
// fp8 weights + activations on the CDNA4 block-scaled fp8 MFMA).
//
// The structure is conv_pipe.hip's (one 8-wave 256co x 256pix block per CU, 4-deep LDS ring filled by
// LDS-DMA three sub-stages ahead, counted vmcnt + raw s_barrier, chunk-swizzled 64-B rows), with the
// operand bytes halved: a 64-B row now carries 64 K-elements, so one sub-stage is K = 64 and feeds ONE
// v_mfma_scale_f32_32x32x64_f8f6f4 per 32x32 output tile (unit block scales: the real scales are a
// per-tensor activation scale and a per-output-channel weight scale applied in the epilogue):
//
//   y[pix, co] = acc * inv_x * inv_w[co] + bias[co] (+ residual) (relu)      -> bf16
//
// The scaled MFMA runs at twice the bf16 rate per clock, and each DMA byte carries twice the K, so the
// same pipeline does twice the work per sub-stage.
//
// * fragments (32x32x64): lane l holds row l & 31 and 32 consecutive bytes of K half (l >> 5), read as
//   the two logical 16-B chunks 2h, 2h+1 of the row with two ds_read_b128.  The chunk swizzle
//   f(row) = [0,2,3,1][(row >> 2) & 3] keeps every 16-lane ds_read_b128 group on 16 distinct bank
//   slots for this pattern too (rows r & 3 x f(r) cover all 16 slots).  A and B use the same lane ->
//   k assignment, so the contraction pairs identical k whatever the instruction's internal k order;
// * accumulator 32x32 (dtype-independent map): reg r of lane l is co = (r & 3) + 8 (r >> 2) + 4 (l >> 5),
//   pixel = l & 31 of the tile.
#include <algorithm>

#include "common.h"

#include "conv_common.h"
#include "fp8_common.h"

typedef __attribute__((ext_vector_type(8))) int i32x8;
typedef __attribute__((ext_vector_type(16))) float f32x16;

namespace {

constexpr int PBN = 256;   // pixels per tile
constexpr int PNST = 4;    // LDS ring depth (sub-stages)
constexpr int SUBK = 64;   // K elements per sub-stage (one 64-B row)

__device__ __forceinline__ int pswz(int rq) { return (120 >> (2 * rq)) & 3; }  // [0, 2, 3, 1]

template <int N>
__device__ __forceinline__ void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// SP: s_setprio(1) around the MFMA block; ILV: spread the next sub-stage's DMA pieces between the MFMA
// groups (steady state, as conv_pipe.hip ILV)
template <int BCO, int SP = 1, int ILV = 0>
__global__ __launch_bounds__(512) void conv_fwd_pipe_f8_kernel(
    const uint8_t* __restrict__ X, const uint8_t* __restrict__ Wt, const float* __restrict__ inv_x,
    const float* __restrict__ inv_w, const float* __restrict__ bias, const bf16_t* __restrict__ R,
    bf16_t* __restrict__ Y, const uint8_t* __restrict__ zpage, ConvGeom g, int relu, int tiles_co, F8Out fo) {
  constexpr int NW = 8, WCO = 2, WPX = NW / WCO;
  constexpr int NSA = BCO / (16 * NW);         // A (weight) wave-instructions per lane per sub-stage
  constexpr int NSB = PBN / (16 * NW);         // B (pixel) wave-instructions per lane per sub-stage
  static_assert(NSA * 16 * NW == BCO && NSB * 16 * NW == PBN, "rows must split evenly over the waves");
  constexpr int NTH = NW * 64;
  constexpr int STAGE = (BCO + PBN) * 64;
  constexpr int WT_CO = BCO / WCO, WT_PIX = PBN / WPX;
  constexpr int TI = WT_CO / 32, TJ = WT_PIX / 32;

  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wid = xcd_remap(blockIdx.x, gridDim.x);
  const int tco = wid % tiles_co;
  const long long tm = wid / tiles_co;
  const int co0 = tco * BCO;
  const long long m0 = tm * PBN;
  const int K = g.kh * g.kw * g.cin;
  const int nks = K / SUBK;

  // ---- per-lane DMA descriptors: lane writes row (q*16 + lane/4), physical chunk lane&3
  const int rloc = lane >> 2;
  const int cl = (lane & 3) ^ pswz(rloc >> 2);   // logical 16-B chunk this lane fetches
  const uint8_t* asrc[NSA];
#pragma unroll
  for (int s = 0; s < NSA; ++s) {
    const int co = co0 + (s * NW + wave) * 16 + rloc;
    asrc[s] = co < g.cout ? Wt + (long long)co * K + cl * 16 : nullptr;
  }
  PixSlot<NSB> ps;
#pragma unroll
  for (int s = 0; s < NSB; ++s) {
    const long long m = m0 + (s * NW + wave) * 16 + rloc;
    ps.base[s] = -1;
    ps.iy0[s] = ps.ix0[s] = ps.Hl[s] = ps.Wl[s] = 0;
    if (m < g.M) {
      int b, oy, ox;
      decode_row(g, m, ps.base[s], ps.iy0[s], ps.ix0[s], ps.Hl[s], ps.Wl[s], b, oy, ox);
    }
  }

  int iky = 0, ikx = 0, ic0 = 0, ikt = 0;   // issue cursor
  auto issue_slot = [&](int q) {
    char* base = smem + (ikt & (PNST - 1)) * STAGE;
    if (q < NSA) {
      const uintptr_t a = asrc[q] ? (uintptr_t)(asrc[q] + ikt * SUBK) : (uintptr_t)zpage;
      glds16((const void*)a, base + (q * NW + wave) * 1024);
    } else {
      const int sb = q - NSA;
      const int iy = ps.iy0[sb] + iky, ix = ps.ix0[sb] + ikx;
      const bool ok = (unsigned)iy < (unsigned)ps.Hl[sb] && (unsigned)ix < (unsigned)ps.Wl[sb];
      const long long off = (long long)(ps.base[sb] + iy * ps.Wl[sb] + ix) * g.cin + ic0 + cl * 16;
      const uintptr_t a = ok ? (uintptr_t)(X + off) : (uintptr_t)zpage;
      glds16((const void*)a, base + BCO * 64 + (sb * NW + wave) * 1024);
    }
  };
  auto advance = [&]() {
    ++ikt;
    ic0 += SUBK;
    if (ic0 == g.cin) {
      ic0 = 0;
      if (++ikx == g.kw) { ikx = 0; ++iky; }
    }
  };
  auto issue = [&]() {
    char* base = smem + (ikt & (PNST - 1)) * STAGE;
#pragma unroll
    for (int s = 0; s < NSA; ++s) {
      const uintptr_t a = asrc[s] ? (uintptr_t)(asrc[s] + ikt * SUBK) : (uintptr_t)zpage;
      glds16((const void*)a, base + (s * NW + wave) * 1024);
    }
#pragma unroll
    for (int s = 0; s < NSB; ++s) {
      const int iy = ps.iy0[s] + iky, ix = ps.ix0[s] + ikx;
      const bool ok = (unsigned)iy < (unsigned)ps.Hl[s] && (unsigned)ix < (unsigned)ps.Wl[s];
      const long long off = (long long)(ps.base[s] + iy * ps.Wl[s] + ix) * g.cin + ic0 + cl * 16;
      const uintptr_t a = ok ? (uintptr_t)(X + off) : (uintptr_t)zpage;
      glds16((const void*)a, base + BCO * 64 + (s * NW + wave) * 1024);
    }
    ++ikt;
    ic0 += SUBK;
    if (ic0 == g.cin) {
      ic0 = 0;
      if (++ikx == g.kw) { ikx = 0; ++iky; }
    }
  };

  f32x16 acc[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int wco = wave / WPX, wpx = wave % WPX;
  // fragment: row lane & 31, logical chunks 2h, 2h+1 (h = lane >> 5); (row >> 2) & 3 is a lane constant
  const int fr = lane & 31, fh = lane >> 5, fsw = pswz((fr >> 2) & 3);
  const int f0 = fr * 64 + (((2 * fh) ^ fsw) << 4);
  const int f1 = fr * 64 + (((2 * fh + 1) ^ fsw) << 4);
  const int abase = wco * WT_CO * 64, bbase = BCO * 64 + wpx * WT_PIX * 64;

  for (int s = -3; s < nks; ++s) {
    if (s >= 0) {
      const int rem = nks - 1 - s;
      constexpr int L = NSA + NSB;
      if (rem >= 2) vm_wait<2 * L>();
      else if (rem == 1) vm_wait<L>();
      else vm_wait<0>();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    }
    if constexpr (ILV) {
      if (s >= 0) {
        const bool do_issue = s + 3 < nks;
        constexpr int NG = (NSA + NSB == 4) ? 4 : 2;   // one DMA piece per MFMA group, or {A, B0} + {B1}
        constexpr int IPQ = TI / NG;
        static_assert(TI % NG == 0, "MFMA groups must tile the wave's rows");
        const char* sb = smem + (s & (PNST - 1)) * STAGE;
        i32x8 bfr[TJ];
#pragma unroll
        for (int j = 0; j < TJ; ++j) {
          const int4 lo = *reinterpret_cast<const int4*>(sb + bbase + j * 2048 + f0);
          const int4 hi = *reinterpret_cast<const int4*>(sb + bbase + j * 2048 + f1);
          bfr[j] = i32x8{lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
        }
#pragma unroll
        for (int q = 0; q < NG; ++q) {
          i32x8 af[IPQ];
#pragma unroll
          for (int i = 0; i < IPQ; ++i) {
            const int4 lo = *reinterpret_cast<const int4*>(sb + abase + (q * IPQ + i) * 2048 + f0);
            const int4 hi = *reinterpret_cast<const int4*>(sb + abase + (q * IPQ + i) * 2048 + f1);
            af[i] = i32x8{lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
          }
          if (do_issue) {
            if constexpr (NG == 4) {
              issue_slot(q);
            } else {
              if (q == 0) { issue_slot(0); issue_slot(1); }
              else issue_slot(2);
            }
          }
          if constexpr (SP) __builtin_amdgcn_s_setprio(1);
#pragma unroll
          for (int i = 0; i < IPQ; ++i)
#pragma unroll
            for (int j = 0; j < TJ; ++j)
              acc[q * IPQ + i][j] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(af[i], bfr[j], acc[q * IPQ + i][j],
                                                                                  0, 0, 0, 127, 0, 127);
          if constexpr (SP) __builtin_amdgcn_s_setprio(0);
          if (q == 0) __builtin_amdgcn_sched_group_barrier(0x0100, 2 * (IPQ + TJ), 0);
          else __builtin_amdgcn_sched_group_barrier(0x0100, 2 * IPQ, 0);
          if (NG == 2 && q == 0) __builtin_amdgcn_sched_group_barrier(0x0010, 2, 0);
          else __builtin_amdgcn_sched_group_barrier(0x0010, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x0008, IPQ * TJ, 0);
        }
        if (do_issue) advance();
        continue;
      }
    }
    if (s + 3 < nks) issue();
    if (s < 0) continue;
    const char* sb = smem + (s & (PNST - 1)) * STAGE;
    i32x8 af[TI], bfr[TJ];
#pragma unroll
    for (int i = 0; i < TI; ++i) {
      const int4 lo = *reinterpret_cast<const int4*>(sb + abase + i * 2048 + f0);
      const int4 hi = *reinterpret_cast<const int4*>(sb + abase + i * 2048 + f1);
      af[i] = i32x8{lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
    }
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
      const int4 lo = *reinterpret_cast<const int4*>(sb + bbase + j * 2048 + f0);
      const int4 hi = *reinterpret_cast<const int4*>(sb + bbase + j * 2048 + f1);
      bfr[j] = i32x8{lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
    }
    if constexpr (SP) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int j = 0; j < TJ; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(af[i], bfr[j], acc[i][j], 0, 0, 0, 127, 0, 127);
    if constexpr (SP) __builtin_amdgcn_s_setprio(0);
  }

  // ---- epilogue through LDS (as conv_pipe.hip): scaled + biased bf16 into a [256 pix][BCO] image,
  // then coalesced 16-B sweeps applying residual / relu
  constexpr int PITCH = BCO * 2 + 16;
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __syncthreads();
  const float sx = *inv_x;
#pragma unroll
  for (int j = 0; j < TJ; ++j) {
    const int pr = wpx * WT_PIX + j * 32 + fr;
#pragma unroll
    for (int i = 0; i < TI; ++i) {
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int cl4 = wco * WT_CO + i * 32 + 8 * t + 4 * fh;
        const int co = co0 + cl4;
        float v[4] = {acc[i][j][4 * t], acc[i][j][4 * t + 1], acc[i][j][4 * t + 2], acc[i][j][4 * t + 3]};
        if (co < g.cout) {
          const float4 w4 = *reinterpret_cast<const float4*>(inv_w + co);
          v[0] *= sx * w4.x; v[1] *= sx * w4.y; v[2] *= sx * w4.z; v[3] *= sx * w4.w;
          if (bias) {
            const float4 bb4 = *reinterpret_cast<const float4*>(bias + co);
            v[0] += bb4.x; v[1] += bb4.y; v[2] += bb4.z; v[3] += bb4.w;
          }
        }
        uint2 o;
        o.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
        o.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
        *reinterpret_cast<uint2*>(smem + pr * PITCH + cl4 * 2) = o;
      }
    }
  }
  __syncthreads();
  constexpr int CPR = BCO / 8;
  const int ncv = min(BCO, g.cout - co0) / 8;
  float qs = 0.f, tmax = 0.f;
  if (fo.amax3) {
    const float prev = fo.amax3[(fo.phase + 2) % 3];
    qs = prev > 0.f ? 448.f / (fo.margin * prev) : 0.f;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      fo.amax3[(fo.phase + 1) % 3] = 0.f;
      if (fo.inv_out) *fo.inv_out = fo.margin * prev / 448.f;
    }
  }
  for (int c = threadIdx.x; c < PBN * CPR; c += NTH) {
    const int pr = c / CPR, ch = c - pr * CPR;
    const long long m = m0 + pr;
    if (m >= g.M || ch >= ncv) continue;
    const long long off = m * g.cout + co0 + ch * 8;
    const uint4 raw = *reinterpret_cast<const uint4*>(smem + pr * PITCH + ch * 16);
    const uint32_t rw[4] = {raw.x, raw.y, raw.z, raw.w};
    float v[8];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      v[2 * t] = bf2f((bf16_t)(rw[t] & 0xffff));
      v[2 * t + 1] = bf2f((bf16_t)(rw[t] >> 16));
    }
    if (R) {
      const uint4 rr = *reinterpret_cast<const uint4*>(R + off);
      const uint32_t w[4] = {rr.x, rr.y, rr.z, rr.w};
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        v[2 * t] += bf2f((bf16_t)(w[t] & 0xffff));
        v[2 * t + 1] += bf2f((bf16_t)(w[t] >> 16));
      }
    }
    if (relu) {
#pragma unroll
      for (int t = 0; t < 8; ++t) v[t] = fmaxf(v[t], 0.f);
    }
    uint4 o;
    o.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
    o.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
    o.z = (uint32_t)f2bf(v[4]) | ((uint32_t)f2bf(v[5]) << 16);
    o.w = (uint32_t)f2bf(v[6]) | ((uint32_t)f2bf(v[7]) << 16);
    *reinterpret_cast<uint4*>(Y + off) = o;
    if (fo.amax3) {
#pragma unroll
      for (int t = 0; t < 8; ++t) tmax = fmaxf(tmax, fabsf(v[t]));
      if (fo.Yq) {
        uint2 q;
        q.x = pack4_e4m3(v[0] * qs, v[1] * qs, v[2] * qs, v[3] * qs);
        q.y = pack4_e4m3(v[4] * qs, v[5] * qs, v[6] * qs, v[7] * qs);
        *reinterpret_cast<uint2*>(fo.Yq + off) = q;
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
      float m = red[0];
#pragma unroll
      for (int w = 1; w < NW; ++w) m = fmaxf(m, red[w]);
      atomicMax(reinterpret_cast<int*>(fo.amax3 + fo.phase), __float_as_int(m));
    }
  }
}

template <int BCO, int SP, int ILV = 0>
int launch_f8(const uint8_t* X, const uint8_t* W, const float* ix, const float* iw, const float* bias, const bf16_t* R,
              bf16_t* Y, const uint8_t* z, const ConvGeom& g, int relu, const F8Out& fo, hipStream_t stream) {
  const int tiles_co = (g.cout + BCO - 1) / BCO;
  const long long tiles_m = (g.M + PBN - 1) / PBN;
  const long long nwg = tiles_co * tiles_m;
  if (nwg > 0x7fffffffLL) return -3;
  const size_t lds = std::max((size_t)PNST * (BCO + PBN) * 64, (size_t)PBN * (BCO * 2 + 16));
  auto kern = conv_fwd_pipe_f8_kernel<BCO, SP, ILV>;
  static bool attr_set = false;
  if (!attr_set) {
    hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr_set = true;
  }
  kern<<<(unsigned)nwg, 512, lds, stream>>>(X, W, ix, iw, bias, R, Y, z, g, relu, tiles_co, fo);
  return (int)hipGetLastError();
}

}  // namespace

// X: fp8 NHWC activations (scale *inv_x), Wt: fp8 OHWI weights (row scale inv_w[co]), Y: bf16.
// cin % 64 == 0, cout % 8 == 0, no strided output scatter.  variant: 0 = 256 co tile, 1 = 128 co tile,
// 2 / 3 = the same without s_setprio, 4 / 5 = DMA interleaved between MFMA groups (+ s_setprio).
// Yq / amax3 / inv_out / phase / margin: fused fp8 output for the next layer (F8Out above; all null = off).
MXR_API int mxr_conv_fwd_f8(const void* X, const void* Wt, const float* inv_x, const float* inv_w, const float* bias,
                            const void* R, void* Y, const void* zpage, const ConvGeom* g, int relu, void* Yq,
                            float* amax3, float* inv_out, int phase, float margin, int variant, hipStream_t stream) {
  if (g->cin % SUBK != 0 || g->cout % 8 != 0 || g->ostride != 1) return -1;
  if (g->nlev < 1 || g->nlev > MXR_MAXLEV) return -2;
  if (Yq && !amax3) return -5;
  const uint8_t *x = (const uint8_t*)X, *w = (const uint8_t*)Wt, *z = (const uint8_t*)zpage;
  const bf16_t* r = (const bf16_t*)R;
  bf16_t* y = (bf16_t*)Y;
  const F8Out fo{(uint8_t*)Yq, amax3, inv_out, phase % 3, margin};
  switch (variant) {
    case 1: return launch_f8<128, 1>(x, w, inv_x, inv_w, bias, r, y, z, *g, relu, fo, stream);
    case 2: return launch_f8<256, 0>(x, w, inv_x, inv_w, bias, r, y, z, *g, relu, fo, stream);
    case 3: return launch_f8<128, 0>(x, w, inv_x, inv_w, bias, r, y, z, *g, relu, fo, stream);
    case 4: return launch_f8<256, 1, 1>(x, w, inv_x, inv_w, bias, r, y, z, *g, relu, fo, stream);
    case 5: return launch_f8<128, 1, 1>(x, w, inv_x, inv_w, bias, r, y, z, *g, relu, fo, stream);
    default: return launch_f8<256, 1>(x, w, inv_x, inv_w, bias, r, y, z, *g, relu, fo, stream);
  }
}
