// Deep-pipelined NHWC bf16 implicit-GEMM WEIGHT gradient for gfx950 (one 8-wave block per CU).
//
//   dW[co, k] = sum_m dY[m, co] * A[m, k]      (A = im2col(X), k = (ky, kx, ci), OHWI layout)
//
// Same math and fp32 split-K slab protocol as conv_wgrad.hip (the reference's conv
// layers are built at /root/reference/train.py:91), re-shaped like conv_pipe.hip:
//
// * output tile TK (k) x TC (co); 8 waves as WK x WC; the reduction (pixels) is consumed in 32-row
//   sub-stages: a dY tile [32 m][TC] and an im2col tile [32 m][TK], both filled by LDS-DMA
//   (global_load_lds_dwordx4) into a 4-deep LDS ring, three sub-stages ahead of the MFMAs, with
//   counted `s_waitcnt vmcnt(N)` + raw `s_barrier` so the prefetch stays in flight;
// * both MFMA operands are read TRANSPOSED (ds_read_b64_tr_b16): a 32-lane half reads rows
//   {8h+q, 8h+8+q} x 16 columns; the 16-B chunk index is XOR-swizzled with
//   s(r) = ((r & 3) << 1) | (((r >> 3) & 1) << 3) (applied to the DMA source address, the LDS image
//   stays lane-linear) -> the 16 (row, chunk) slots of a half are distinct: conflict-free;
// * the per-step im2col gather needs the (image, level, oy, ox) of each staged pixel row: it is
//   advanced INCREMENTALLY (+32 pixels per sub-stage, a rare row / level / image carry) instead of
//   re-divided every step; the level geometry lives in registers and is reloaded from an LDS copy
//   of the tables on a level carry -- no vector-memory op besides the DMA inside the loop, so the
//   counted vmcnt is exact (a dynamically indexed kernel-argument array would become a global load).
#include "conv_common.h"

typedef __attribute__((ext_vector_type(4))) short s16x4;

namespace {

constexpr int WR = 32;     // pixel rows per sub-stage
constexpr int WNST = 4;    // LDS ring depth

__device__ __forceinline__ s16x4 tr_read(const char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(p));
}

__device__ __forceinline__ int wsw(int r) { return ((r & 3) << 1) | (((r >> 3) & 1) << 3); }
// swizzle for a tile with CPR 16-B chunks per row: wsw needs >= 16 chunks (values up to 14); 8-chunk
// rows (64-wide tiles) use swz8 (conv_common.h), conflict-free for the same transposed-read pattern
template <int CPR>
__device__ __forceinline__ int rsw(int r) {
  static_assert(CPR >= 8, "tile rows must be >= 8 chunks");
  if constexpr (CPR >= 16) return wsw(r);
  else return swz8(r);
}

// arr[l] for a per-lane level index with the table in SGPRs (no dynamic indexing -> no memory access)
__device__ __forceinline__ int lsel(const int* arr, int l) {
  int v = arr[0];
  v = l == 1 ? arr[1] : v;
  v = l == 2 ? arr[2] : v;
  v = l == 3 ? arr[3] : v;
  v = l == 4 ? arr[4] : v;
  return v;
}

// s_waitcnt vmcnt(N) with a compile-time N
template <int N>
__device__ __forceinline__ void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// NS: LDS ring depth (DMA runs NS - 1 sub-stages ahead); 3 shrinks the ring so two blocks share a CU
template <int TK, int TC, int WK, int WC, int ILV = 0, int NW = 8, int NS = WNST>
__global__ __launch_bounds__(NW * 64) void conv_wgrad_pipe_kernel(
    const bf16_t* __restrict__ X, const bf16_t* __restrict__ dY, int ldy, float* __restrict__ part,
    const bf16_t* __restrict__ zpage, ConvGeom g, int tiles_k, int tiles_co, int splits, int nsub) {
  static_assert(WK * WC == NW, "wave grid");
  constexpr int T_BYTES = WR * TC * 2, U_BYTES = WR * TK * 2, STAGE = T_BYTES + U_BYTES;
  constexpr int CPT = TC / 8, CPU = TK / 8;          // 16-B chunks per T / U row
  constexpr int RPT = 64 / CPT, RPU = 64 / CPU;      // rows per wave-instruction
  constexpr int NT = T_BYTES / 1024 / NW, NU = U_BYTES / 1024 / NW;   // instructions per wave per sub-stage
  static_assert(NT >= 1 && NU >= 1, "tile too small");
  constexpr int WT_K = TK / WK, WT_CO = TC / WC;
  constexpr int TI = WT_K / 16, TJ = WT_CO / 16;

  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wid = xcd_remap(blockIdx.x, gridDim.x);
  const int tk = wid % tiles_k;
  const int rest = wid / tiles_k;
  const int tco = rest % tiles_co;
  const int split = rest / tiles_co;
  const int co0 = tco * TC, k0 = tk * TK;
  const int K = g.kh * g.kw * g.cin;
  const int s_begin = (int)((long long)nsub * split / splits), s_end = (int)((long long)nsub * (split + 1) / splits);
  // level tables -> LDS (behind the ring): read only on the rare level carry, with ds_read
  // (lgkmcnt), so no vector-memory op other than the DMA ever enters the loop's vmcnt count
  int* lt = reinterpret_cast<int*>(smem + NS * STAGE);   // [H, W, Ho, Wo, in_off, mstart] x 5
  if (threadIdx.x < 6 * MXR_MAXLEV) {
    const int a = threadIdx.x / MXR_MAXLEV, t = threadIdx.x % MXR_MAXLEV;
    const int* src = a == 0 ? g.H : a == 1 ? g.W : a == 2 ? g.Ho : a == 3 ? g.Wo : a == 4 ? g.in_off : g.mstart;
    lt[threadIdx.x] = src[t];
  }
  __syncthreads();

  // ---- T (dY) slots: lane -> row, swizzled chunk
  const bf16_t* tptr[NT];
  int trow[NT];
#pragma unroll
  for (int s = 0; s < NT; ++s) {
    const int inst = s * NW + wave;
    trow[s] = inst * RPT + lane / CPT;
    const int c = (lane % CPT) ^ rsw<CPT>(trow[s]);
    const int co = co0 + c * 8;
    tptr[s] = co < ldy ? dY + ((long long)s_begin * WR + trow[s]) * ldy + co : nullptr;
  }
  // ---- U (im2col) slots: fixed (tap, ci) per lane; the pixel is advanced incrementally and its
  // level's geometry is cached in registers (reloaded from the LDS table only on a level carry)
  int u_dy[NU], u_dx[NU], u_ci[NU], u_kok[NU];
  int u_m[NU], u_oy[NU], u_ox[NU], u_l[NU], u_img[NU], u_H[NU], u_W[NU], u_Ho[NU], u_Wo[NU], u_off[NU];
#pragma unroll
  for (int s = 0; s < NU; ++s) {
    const int inst = s * NW + wave;
    const int row = inst * RPU + lane / CPU;
    const int c = (lane % CPU) ^ rsw<CPU>(row);
    const int k = k0 + c * 8;
    u_kok[s] = k < K;
    const int tap = k / g.cin;
    u_ci[s] = k - tap * g.cin;
    u_dy[s] = tap / g.kw;
    u_dx[s] = tap - u_dy[s] * g.kw;
    const long long m = (long long)s_begin * WR + row;
    u_m[s] = (int)m;
    int b = 0, q = 0, l = 0;
    if (m < g.M) {
      b = (int)(m / g.out_img);
      q = (int)(m - (long long)b * g.out_img);
      for (int t = 1; t < g.nlev; ++t)
        if (q >= lt[5 * MXR_MAXLEV + t]) l = t;
    }
    const int loc = q - lt[5 * MXR_MAXLEV + l];
    u_l[s] = l;
    u_img[s] = b * g.in_img;
    u_H[s] = lt[l];
    u_W[s] = lt[MXR_MAXLEV + l];
    u_Ho[s] = lt[2 * MXR_MAXLEV + l];
    u_Wo[s] = lt[3 * MXR_MAXLEV + l];
    u_off[s] = lt[4 * MXR_MAXLEV + l];
    u_oy[s] = loc / u_Wo[s];
    u_ox[s] = loc - u_oy[s] * u_Wo[s];
  }

  int it = s_begin;   // sub-stage being issued
  // DMA piece q of sub-stage `it`: q < NT -> dY rows, else im2col rows (advanced by WR pixels)
  auto issue_piece = [&](int q) {
    char* base = smem + (it % NS) * STAGE;
    if (q < NT) {
      const long long m = (long long)it * WR + trow[q];
      const uintptr_t a = (tptr[q] && m < g.M) ? (uintptr_t)tptr[q] : (uintptr_t)zpage;
      glds16_asm((const void*)a, base + (q * NW + wave) * 1024);
      if (tptr[q]) tptr[q] += (long long)WR * ldy;
      return;
    }
    const int s = q - NT;
    const int iy = u_oy[s] * g.stride - g.pt + u_dy[s];
    const int ix = u_ox[s] * g.stride - g.pl + u_dx[s];
    const bool ok = u_kok[s] && (long long)u_m[s] < g.M && (unsigned)iy < (unsigned)u_H[s] &&
                    (unsigned)ix < (unsigned)u_W[s];
    const long long off = (long long)(u_img[s] + u_off[s] + iy * u_W[s] + ix) * g.cin + u_ci[s];
    const uintptr_t a = ok ? (uintptr_t)(X + off) : (uintptr_t)zpage;
    glds16_asm((const void*)a, base + T_BYTES + (s * NW + wave) * 1024);
    // advance this row by WR pixels (carry over output rows / levels / images)
    u_m[s] += WR;
    u_ox[s] += WR;
    while (u_ox[s] >= u_Wo[s]) {
      u_ox[s] -= u_Wo[s];
      if (++u_oy[s] >= u_Ho[s]) {
        u_oy[s] = 0;
        int l = u_l[s] + 1;
        if (l >= g.nlev) { l = 0; u_img[s] += g.in_img; }
        u_l[s] = l;
        u_H[s] = lt[l];
        u_W[s] = lt[MXR_MAXLEV + l];
        u_Ho[s] = lt[2 * MXR_MAXLEV + l];
        u_Wo[s] = lt[3 * MXR_MAXLEV + l];
        u_off[s] = lt[4 * MXR_MAXLEV + l];
      }
    }
  };
  auto issue = [&]() {
#pragma unroll
    for (int q = 0; q < NT + NU; ++q) issue_piece(q);
    ++it;
  };

  f32x4 acc[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // ---- transposed-read addresses (lane constants): lane 4q+p of a 16-lane group reads row
  // kg*8 + q (+4 for the upper half of the fragment), columns 4p..4p+3 of a 16-column block
  const int kg = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
  const int r0 = kg * 8 + q;
  const int swu = rsw<CPU>(r0), swt = rsw<CPT>(r0);   // identical for r0 + 4
  const int wk = wave / WC, wc = wave % WC;
  int aoff[TI], boff[TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i) {
    const int c = ((wk * WT_K + i * 16) >> 3) + (p >> 1);
    aoff[i] = T_BYTES + r0 * (TK * 2) + ((c ^ swu) << 4) + (p & 1) * 8;
  }
#pragma unroll
  for (int j = 0; j < TJ; ++j) {
    const int c = ((wc * WT_CO + j * 16) >> 3) + (p >> 1);
    boff[j] = r0 * (TC * 2) + ((c ^ swt) << 4) + (p & 1) * 8;
  }

  const int n = s_end - s_begin;
  for (int s = -(NS - 1); s < n; ++s) {
    if (s >= 0) {
      const int rem = n - 1 - s;
      // own DMA of sub-stage s done: at most the NS - 2 younger sub-stages' loads still in flight
      static_assert(NS == 3 || NS == 4, "ring depth");
      static_assert((NS - 2) * (NT + NU) <= 63, "vmcnt range");
      if (rem >= NS - 2) vm_wait<(NS - 2) * (NT + NU)>();
      else if (rem == 1) vm_wait<NT + NU>();
      else vm_wait<0>();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    }
    if constexpr (ILV == 1 || ILV == 2) {
      if (s >= 0) {
        // DMA pieces of sub-stage s+3 spread between MFMA groups (see conv_pipe.hip ILV)
        const bool do_issue = s + NS - 1 < n;
        constexpr int NQ = NT + NU;
        static_assert(NQ >= 2 && NQ <= 4, "DMA grouping");
        constexpr int NG = NQ == 4 ? 4 : 2;   // one piece per group, {0, 1} + {2}, or {0} + {1}
        constexpr int IPQ = TI / NG;
        static_assert(TI % NG == 0, "MFMA groups must tile the wave's rows");
        const char* sb = smem + ((s_begin + s) % NS) * STAGE;
        bf16x8 bfr[TJ];
#pragma unroll
        for (int j = 0; j < TJ; ++j) {
          const s16x4 lo = tr_read(sb + boff[j]);
          const s16x4 hi = tr_read(sb + boff[j] + 4 * TC * 2);
          bfr[j] = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        }
#pragma unroll
        for (int q = 0; q < NG; ++q) {
          bf16x8 af[IPQ];
#pragma unroll
          for (int i = 0; i < IPQ; ++i) {
            const s16x4 lo = tr_read(sb + aoff[q * IPQ + i]);
            const s16x4 hi = tr_read(sb + aoff[q * IPQ + i] + 4 * TK * 2);
            af[i] = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          }
          if (do_issue) {
            if constexpr (NG == 4 || NQ == 2) {
              issue_piece(q);
            } else {
              if (q == 0) { issue_piece(0); issue_piece(1); }
              else issue_piece(2);
            }
          }
          if constexpr (ILV == 2) __builtin_amdgcn_s_setprio(1);
#pragma unroll
          for (int i = 0; i < IPQ; ++i)
#pragma unroll
            for (int j = 0; j < TJ; ++j)
              acc[q * IPQ + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[q * IPQ + i][j], 0, 0, 0);
          if constexpr (ILV == 2) __builtin_amdgcn_s_setprio(0);
          if (q == 0) __builtin_amdgcn_sched_group_barrier(0x0100, 2 * (IPQ + TJ), 0);
          else __builtin_amdgcn_sched_group_barrier(0x0100, 2 * IPQ, 0);
          if (NQ == 3 && q == 0) __builtin_amdgcn_sched_group_barrier(0x0010, 2, 0);
          else __builtin_amdgcn_sched_group_barrier(0x0010, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x0008, IPQ * TJ, 0);
        }
        if (do_issue) ++it;
        continue;
      }
    }
    if (s + NS - 1 < n) issue();
    if (s < 0) continue;
    const char* sb = smem + ((s_begin + s) % NS) * STAGE;
    bf16x8 af[TI], bfr[TJ];
#pragma unroll
    for (int i = 0; i < TI; ++i) {
      const s16x4 lo = tr_read(sb + aoff[i]);
      const s16x4 hi = tr_read(sb + aoff[i] + 4 * TK * 2);
      af[i] = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    }
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
      const s16x4 lo = tr_read(sb + boff[j]);
      const s16x4 hi = tr_read(sb + boff[j] + 4 * TC * 2);
      bfr[j] = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    }
    if constexpr (ILV == 3) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int j = 0; j < TJ; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    if constexpr (ILV == 3) __builtin_amdgcn_s_setprio(0);
  }

  // slab write: part[split][co][k]; lane holds k = 4*kg + e (e = 0..3) of co = lane & 15 per tile
  float* slab = part + (long long)split * g.cout * K;
#pragma unroll
  for (int j = 0; j < TJ; ++j) {
    const int co = co0 + wc * WT_CO + j * 16 + (lane & 15);
    if (co >= g.cout) continue;
#pragma unroll
    for (int i = 0; i < TI; ++i) {
      const int k = k0 + wk * WT_K + i * 16 + 4 * kg;
      if (k >= K) continue;
      *reinterpret_cast<f32x4*>(slab + (long long)co * K + k) = acc[i][j];
    }
  }
}

template <int TK, int TC, int WK, int WC, int ILV = 0, int NW = 8, int NS = WNST>
int launch_wgrad_pipe(const bf16_t* X, const bf16_t* dY, int ldy, float* part, int splits, const bf16_t* zpage,
                      const ConvGeom& g, hipStream_t stream) {
  const int K = g.kh * g.kw * g.cin;
  const int tiles_k = (K + TK - 1) / TK;
  const int tiles_co = (g.cout + TC - 1) / TC;
  const long long nsub = (g.M + WR - 1) / WR;
  if (nsub > 0x7fffffffLL) return -4;
  const long long nwg = (long long)tiles_k * tiles_co * splits;
  const size_t lds = (size_t)NS * WR * (TK + TC) * 2 + 6 * MXR_MAXLEV * sizeof(int);
  auto kern = conv_wgrad_pipe_kernel<TK, TC, WK, WC, ILV, NW, NS>;
  static bool attr_set = false;
  if (!attr_set) {
    hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr_set = true;
  }
  kern<<<(unsigned)nwg, NW * 64, lds, stream>>>(X, dY, ldy, part, zpage, g, tiles_k, tiles_co, splits, (int)nsub);
  return (int)hipGetLastError();
}

}  // namespace

void mxr_wgrad_reduce_launch(const float* part, int splits, long long n, int K, const float* scale, float* out,
                             int accumulate, hipStream_t stream);

// variant 0: 256 k x 256 co (waves 2 x 4), 1: 256 k x 128 co (waves 4 x 2); 2 / 3: the same with the DMA
// pieces interleaved between MFMA groups; 4: 256x256 interleaved + s_setprio; 5 / 6: 256x256 / 256x128 with
// s_setprio around the MFMA block; 7 / 8 / 9: narrow 4-wave tiles for 64-channel layers (256 k x 64 co,
// 128 x 64, 64 x 64; two or more blocks per CU); 10: 128 x 128 interleaved (two blocks per CU);
// 11 / 12: 256 x 128 / 128 x 256 interleaved on a 3-deep ring (two blocks per CU).
// part: splits * cout * K floats.
MXR_API int mxr_conv_wgrad_pipe(const void* X, const void* dY, int ldy, float* part, int splits, float* out,
                                const float* scale, int accumulate, const void* zpage, const ConvGeom* g, int variant,
                                hipStream_t stream) {
  if (g->cin % 8 != 0 || ldy % 8 != 0 || g->ostride != 1) return -1;
  if (g->nlev < 1 || g->nlev > MXR_MAXLEV) return -2;
  if (g->M + 64 >= (1LL << 31)) return -4;
  const bf16_t *x = (const bf16_t*)X, *dy = (const bf16_t*)dY, *z = (const bf16_t*)zpage;
  int rc;
  switch (variant) {
    case 1: rc = launch_wgrad_pipe<256, 128, 4, 2>(x, dy, ldy, part, splits, z, *g, stream); break;
    case 2: rc = launch_wgrad_pipe<256, 256, 2, 4, 1>(x, dy, ldy, part, splits, z, *g, stream); break;
    case 3: rc = launch_wgrad_pipe<256, 128, 4, 2, 1>(x, dy, ldy, part, splits, z, *g, stream); break;
    case 4: rc = launch_wgrad_pipe<256, 256, 2, 4, 2>(x, dy, ldy, part, splits, z, *g, stream); break;
    case 5: rc = launch_wgrad_pipe<256, 256, 2, 4, 3>(x, dy, ldy, part, splits, z, *g, stream); break;
    case 6: rc = launch_wgrad_pipe<256, 128, 4, 2, 3>(x, dy, ldy, part, splits, z, *g, stream); break;
    case 7: rc = launch_wgrad_pipe<256, 64, 4, 1, 0, 4>(x, dy, ldy, part, splits, z, *g, stream); break;
    case 8: rc = launch_wgrad_pipe<128, 64, 2, 2, 0, 4>(x, dy, ldy, part, splits, z, *g, stream); break;
    case 9: rc = launch_wgrad_pipe<64, 64, 2, 2, 0, 4>(x, dy, ldy, part, splits, z, *g, stream); break;
    case 10: rc = launch_wgrad_pipe<128, 128, 2, 4, 1, 8>(x, dy, ldy, part, splits, z, *g, stream); break;
    case 11: rc = launch_wgrad_pipe<256, 128, 4, 2, 1, 8, 3>(x, dy, ldy, part, splits, z, *g, stream); break;
    case 12: rc = launch_wgrad_pipe<128, 256, 2, 4, 1, 8, 3>(x, dy, ldy, part, splits, z, *g, stream); break;
    default: rc = launch_wgrad_pipe<256, 256, 2, 4>(x, dy, ldy, part, splits, z, *g, stream); break;
  }
  if (rc) return rc;
  const int K = g->kh * g->kw * g->cin;
  mxr_wgrad_reduce_launch(part, splits, (long long)g->cout * K, K, scale, out, accumulate, stream);
  return (int)hipGetLastError();
}
