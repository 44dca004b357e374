// NHWC bf16 implicit-GEMM convolution WEIGHT gradient (+ bias gradient) on CDNA4 MFMA.
//
//   dW[co, k] = sum_m dY[m, co] * A[m, k]      (A = im2col(X), k = (ky, kx, ci), OHWI layout)
//
// The reduction runs over m (pixels), which is the ROW index of both operands in memory, so both
// MFMA operands are read TRANSPOSED out of LDS with ds_read_b64_tr_b16 (gfx950): the dY tile is
// [64 m][BCO co] and the im2col tile [64 m][BK k] (BK/64 independent (tap, ci-block) chunks,
// gathered per lane by LDS-DMA exactly like the forward kernel, zero page for padding taps).
// Orientation C = A^T.dY -> each lane holds 4 consecutive k of one co -> 16-B fp32 stores.
// Huge M (up to 4.3M pixels at batch 16) is split over workgroups ("split-K" over pixels): each
// split writes an fp32 slab, a second kernel sums the slabs in a fixed order (deterministic),
// multiplies by the folded frozen-BN scale of the output channel and adds the result straight
// into the flat fp32 gradient buffer.  The pyramid (multi-level) geometry makes the shared head
// layers' weight gradient ONE reduction over all five levels.
#include <cstdlib>

#include "conv_common.h"

typedef __attribute__((ext_vector_type(4))) short s16x4;

namespace {

__device__ __forceinline__ s16x4 tr_read(const char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(p));
}

template <int BK, int BCO, int WK, int WCO>
__global__ __launch_bounds__(WK* WCO * 64) void conv_wgrad_kernel(
    const bf16_t* __restrict__ X, const bf16_t* __restrict__ dY, int ldy, float* __restrict__ part,
    const bf16_t* __restrict__ zpage, ConvGeom g, int tiles_k, int tiles_co, int splits, long long steps) {
  constexpr int NW = WK * WCO;
  constexpr int T_BYTES = 64 * BCO * 2;       // dY tile [64 m][BCO]
  constexpr int U_BYTES = 64 * BK * 2;        // im2col tile: BK/64 chunks of [64 m][64 k]
  constexpr int BUF = T_BYTES + U_BYTES;
  constexpr int T_ROWS_PER_INST = 1024 / (BCO * 2);
  constexpr int T_INST = 64 / T_ROWS_PER_INST;
  constexpr int U_INST = (BK / 64) * 8;
  static_assert(T_INST % NW == 0 && U_INST % NW == 0, "staging must divide among waves");
  constexpr int NT = T_INST / NW, NU = U_INST / NW;
  constexpr int WT_K = BK / WK, WT_CO = BCO / WCO;
  constexpr int TI = WT_K / 16, TJ = WT_CO / 16;
  constexpr int CPR = BCO / 8;                // 16-B chunks per dY row

  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wid = xcd_remap(blockIdx.x, gridDim.x);
  const int tk = wid % tiles_k;
  const int rest = wid / tiles_k;
  const int tco = rest % tiles_co;
  const int split = rest / tiles_co;
  const int co0 = tco * BCO;
  const int K = g.kh * g.kw * g.cin;
  const int cb = g.cin / 64;
  const long long s_begin = steps * split / splits, s_end = steps * (split + 1) / splits;

  // per-lane U-slot descriptors (chunk tap / ci block are fixed per block); the 16-B chunk a lane
  // loads is XOR-swizzled by its LDS row (linear LDS-DMA destination, swizzled source + read)
  int u_dy[NU], u_dx[NU], u_ci[NU], u_ok[NU], u_row[NU];
#pragma unroll
  for (int s = 0; s < NU; ++s) {
    const int gs = wave * NU + s;
    const int c = gs >> 3;                      // chunk within the tile
    const int kc = tk * (BK / 64) + c;          // global 64-chunk of K
    const int tap = kc / cb;
    u_ok[s] = (kc * 64 < K);
    u_dy[s] = tap / g.kw;
    u_dx[s] = tap - (tap / g.kw) * g.kw;
    u_row[s] = (gs & 7) * 8 + (lane >> 3);
    u_ci[s] = (kc - tap * cb) * 64 + (((lane & 7) ^ swz8(u_row[s])) * 8);
  }

  auto stage = [&](int buf, long long m0) {
    char* tb = smem + buf * BUF;
    char* ub = tb + T_BYTES;
#pragma unroll
    for (int s = 0; s < NT; ++s) {
      const int gs = wave * NT + s;
      const int row = gs * T_ROWS_PER_INST + lane / CPR;
      const int ch = (lane % CPR) ^ (CPR == 16 ? swz16(row) : swz8(row));
      const long long m = m0 + row;
      const int co = co0 + ch * 8;
      const void* src = (m < g.M && co < ldy) ? (const void*)(dY + m * ldy + co) : (const void*)zpage;
      glds16(src, tb + gs * 1024);
    }
#pragma unroll
    for (int s = 0; s < NU; ++s) {
      const int gs = wave * NU + s;
      const long long m = m0 + u_row[s];
      const void* src = zpage;
      if (u_ok[s] && m < g.M) {
        int base, iy0, ix0, Hl, Wl;
        decode_row_fast(g, (int)m, base, iy0, ix0, Hl, Wl);
        const int iy = iy0 + u_dy[s], ix = ix0 + u_dx[s];
        if (iy >= 0 && iy < Hl && ix >= 0 && ix < Wl)
          src = X + ((long long)(base + iy * Wl + ix)) * g.cin + u_ci[s];
      }
      glds16(src, ub + gs * 1024);
    }
  };

  f32x4 acc[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int wk = wave / WCO, wc = wave % WCO;
  const int grp = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
  if (s_begin < s_end) {
    stage(0, s_begin * 64);
    __syncthreads();
    int cur = 0;
    for (long long st = s_begin; st < s_end; ++st) {
      if (st + 1 < s_end) stage(cur ^ 1, (st + 1) * 64);
      const char* tb = smem + cur * BUF;
      const char* ub = tb + T_BYTES;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        bf16x8 af[TI], bfr[TJ];
        const int r0 = kk * 32 + grp * 8 + q;     // rows r0 (elements 0..3) and r0 + 4 (4..7)
        const int r1 = r0 + 4;
#pragma unroll
        for (int i = 0; i < TI; ++i) {
          const int col = wk * WT_K + i * 16;   // k column base within tile (multiple of 16)
          const char* base = ub + (col >> 6) * 8192;
          const int c = ((col & 63) >> 3) + (p >> 1);
          const s16x4 lo = tr_read(base + r0 * 128 + ((c ^ swz8(r0)) << 4) + (p & 1) * 8);
          const s16x4 hi = tr_read(base + r1 * 128 + ((c ^ swz8(r1)) << 4) + (p & 1) * 8);
          af[i] = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        }
#pragma unroll
        for (int j = 0; j < TJ; ++j) {
          const int c = ((wc * WT_CO + j * 16) >> 3) + (p >> 1);
          const int s0 = CPR == 16 ? swz16(r0) : swz8(r0), s1 = CPR == 16 ? swz16(r1) : swz8(r1);
          const s16x4 lo = tr_read(tb + r0 * (BCO * 2) + ((c ^ s0) << 4) + (p & 1) * 8);
          const s16x4 hi = tr_read(tb + r1 * (BCO * 2) + ((c ^ s1) << 4) + (p & 1) * 8);
          bfr[j] = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        }
#pragma unroll
        for (int i = 0; i < TI; ++i)
#pragma unroll
          for (int j = 0; j < TJ; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      }
      __syncthreads();
      cur ^= 1;
    }
  }
  // slab write: part[split][co][k]; lane holds k = 4*grp + r (r=0..3), co = li per 16x16 tile
  float* slab = part + (long long)split * g.cout * K;
#pragma unroll
  for (int j = 0; j < TJ; ++j) {
    const int co = co0 + wc * WT_CO + j * 16 + li;
    if (co >= g.cout) continue;
#pragma unroll
    for (int i = 0; i < TI; ++i) {
      const int k = tk * BK + wk * WT_K + i * 16 + 4 * grp;
      if (k >= K) continue;
      *reinterpret_cast<f32x4*>(slab + (long long)co * K + k) = acc[i][j];
    }
  }
}

// out[co, k] (+)= scale[co] * sum_s part[s, co, k]   (fixed summation order -> deterministic)
// A block owns CPB = 256 >> L consecutive float4 columns and splits the slab range over SPL = 1 << L
// thread rows (row r sums slabs r, r + SPL, ...; two loads in flight), then row 0 adds the SPL partial
// sums in row order out of LDS.  L is a function of (n, splits) only, so the order -- and the result --
// is fixed per shape.  Narrow layers need the split rows: a 64 x 256 1x1 gradient is 4096 float4
// columns over up to 1024 slabs, which one thread per column (16 blocks) summed as a latency-bound
// chain of 256 dependent rounds -- longer than the GEMM that produced the slabs.
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const float* __restrict__ part, int splits, int n, int K,
                                                           const float* __restrict__ scale, float* __restrict__ out,
                                                           int accumulate, int L) {
  __shared__ f32x4 red[256];
  const int cpb = 256 >> L, spl = 1 << L;
  const int col = threadIdx.x & (cpb - 1), r = threadIdx.x >> (8 - L);
  const int nv = n >> 2;
  const int i = blockIdx.x * cpb + col;
  f32x4 s0 = {0.f, 0.f, 0.f, 0.f}, s1 = s0;
  if (i < nv) {
    const float* p = part + 4 * (size_t)i;
    int t = r;
    for (; t + spl < splits; t += 2 * spl) {
      s0 += *reinterpret_cast<const f32x4*>(p + (size_t)t * n);
      s1 += *reinterpret_cast<const f32x4*>(p + (size_t)(t + spl) * n);
    }
    if (t < splits) s0 += *reinterpret_cast<const f32x4*>(p + (size_t)t * n);
  }
  red[threadIdx.x] = s0 + s1;
  __syncthreads();
  if (r == 0 && i < nv) {
    f32x4 s = red[col];
    for (int q = 1; q < spl; ++q) s += red[q * cpb + col];
    if (scale) s *= scale[(4 * i) / K];
    if (accumulate) s += *reinterpret_cast<const f32x4*>(out + 4 * (size_t)i);
    *reinterpret_cast<f32x4*>(out + 4 * (size_t)i) = s;
  }
}

void wgrad_reduce(const float* part, int splits, long long n, int K, const float* scale, float* out, int accumulate,
                  hipStream_t stream) {
#ifdef MXR_DIAG_KERNELS
  // timing-only diagnostic library: MXR_DIAG_NO_REDUCE=1 skips every split-K reduce (wrong gradients) to bound
  // what folding the reduce into the wgrad kernels could save
  static const bool skip = getenv("MXR_DIAG_NO_REDUCE") && getenv("MXR_DIAG_NO_REDUCE")[0] == '1';
  if (skip) return;
#endif
  // split rows until the grid has ~2 blocks per CU (or each row would sum fewer than 2 slabs)
  const long long nv = n / 4;
  int L = 0;
  while (L < 6 && (nv + (256 >> L) - 1) / (256 >> L) < 512 && (2 << L) <= splits / 2) ++L;
  const long long cpb = 256 >> L;
  wgrad_reduce_kernel<<<(unsigned)((nv + cpb - 1) / cpb), 256, 0, stream>>>(part, splits, (int)n, K, scale, out,
                                                                              accumulate, L);
}

// bias gradient: db[c] = sum_m dY[m, c]; stage 1 partial sums per block (8 channels per thread)
__global__ __launch_bounds__(256) void colsum_partial_kernel(const bf16_t* __restrict__ dy, long long M, int C, int ld,
                                                             float* __restrict__ part) {
  const int CV = C / 8;
  const int rows_per_pass = 256 / CV;   // C <= 2048 -> CV <= 256
  const int cv = threadIdx.x % CV, r = threadIdx.x / CV;
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (r < rows_per_pass) {
    const long long step = (long long)gridDim.x * rows_per_pass;
    long long m = (long long)blockIdx.x * rows_per_pass + r;
    // four rows in flight per iteration (same per-thread summation order as one at a time)
    for (; m + 3 * step < M; m += 4 * step) {
      uint4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = *reinterpret_cast<const uint4*>(dy + (m + u * step) * ld + cv * 8);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const uint32_t w[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          acc[2 * t] += bf2f((bf16_t)(w[t] & 0xffff));
          acc[2 * t + 1] += bf2f((bf16_t)(w[t] >> 16));
        }
      }
    }
    for (; m < M; m += step) {
      const uint4 v = *reinterpret_cast<const uint4*>(dy + m * ld + cv * 8);
      const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        acc[2 * t] += bf2f((bf16_t)(w[t] & 0xffff));
        acc[2 * t + 1] += bf2f((bf16_t)(w[t] >> 16));
      }
    }
  }
  __shared__ float red[256 * 8];
#pragma unroll
  for (int t = 0; t < 8; ++t) red[threadIdx.x * 8 + t] = acc[t];
  __syncthreads();
  if (threadIdx.x < CV) {
    float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int rr = 0; rr < rows_per_pass; ++rr)
#pragma unroll
      for (int t = 0; t < 8; ++t) s[t] += red[(rr * CV + threadIdx.x) * 8 + t];
#pragma unroll
    for (int t = 0; t < 8; ++t) part[(long long)blockIdx.x * C + threadIdx.x * 8 + t] = s[t];
  }
}

__global__ __launch_bounds__(256) void colsum_final_kernel(const float* __restrict__ part, int nblk, int C,
                                                           const float* __restrict__ scale, float* __restrict__ out,
                                                           int accumulate) {
  // one block per channel, threads stride over the partial rows (fixed order -> deterministic)
  __shared__ float red[16];
  const int c = blockIdx.x;
  float s = 0.f;
  for (int b = threadIdx.x; b < nblk; b += 256) s += part[(long long)b * C + c];
  s = block_sum(s, red);
  if (threadIdx.x == 0) {
    if (scale) s *= scale[c];
    out[c] = accumulate ? out[c] + s : s;
  }
}

template <int BK, int BCO, int WK, int WCO>
int launch_wgrad(const bf16_t* X, const bf16_t* dY, int ldy, float* part, int splits, const bf16_t* zpage,
                 const ConvGeom& g, hipStream_t stream) {
  const int K = g.kh * g.kw * g.cin;
  const int tiles_k = (K + BK - 1) / BK;
  const int tiles_co = (g.cout + BCO - 1) / BCO;
  const long long steps = (g.M + 63) / 64;
  const long long nwg = (long long)tiles_k * tiles_co * splits;
  const size_t lds = 2 * (64 * BCO * 2 + 64 * BK * 2);
  auto kern = conv_wgrad_kernel<BK, BCO, WK, WCO>;
  static bool attr_set = false;
  if (!attr_set) {
    hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr_set = true;
  }
  kern<<<(unsigned)nwg, WK * WCO * 64, lds, stream>>>(X, dY, ldy, part, zpage, g, tiles_k, tiles_co, splits, steps);
  return (int)hipGetLastError();
}

}  // namespace

// part: splits * cout * K floats of workspace. out: cout*K f32 (the flat-gradient slot).
// ldy: row stride of dY in elements (>= cout, multiple of 8). variant 0: 128k x 128co, 1: 128k x 64co,
// 2: 64k x 128co (K = 64 layers).
MXR_API int mxr_conv_wgrad(const void* X, const void* dY, int ldy, float* part, int splits, float* out,
                           const float* scale, int accumulate, const void* zpage, const ConvGeom* g, int variant,
                           hipStream_t stream) {
  if (g->cin % 64 != 0 || ldy % 8 != 0 || g->ostride != 1) return -1;
  if (g->M >= (1LL << 24)) return -4;   // decode_row_fast range
  int rc;
  if (variant == 1)
    rc = launch_wgrad<128, 64, 2, 2>((const bf16_t*)X, (const bf16_t*)dY, ldy, part, splits, (const bf16_t*)zpage, *g,
                                     stream);
  else if (variant == 2)
    rc = launch_wgrad<64, 128, 1, 4>((const bf16_t*)X, (const bf16_t*)dY, ldy, part, splits, (const bf16_t*)zpage, *g,
                                     stream);
  else
    rc = launch_wgrad<128, 128, 2, 2>((const bf16_t*)X, (const bf16_t*)dY, ldy, part, splits, (const bf16_t*)zpage, *g,
                                      stream);
  if (rc) return rc;
  const int K = g->kh * g->kw * g->cin;
  const long long n = (long long)g->cout * K;
  if (n >= 0x7fffffffLL) return -1;
  wgrad_reduce(part, splits, n, K, scale, out, accumulate, stream);
  return (int)hipGetLastError();
}

// shared by conv_wgrad_pipe.hip
void mxr_wgrad_reduce_launch(const float* part, int splits, long long n, int K, const float* scale, float* out,
                             int accumulate, hipStream_t stream) {
  wgrad_reduce(part, splits, n, K, scale, out, accumulate, stream);
}

// the split-K reduce of a dual-source slab [splits][cout][k1 + k2]: columns < k1 -> out1 (cout x k1, scale1[co]),
// the rest -> out2 (cout x k2, scale2[co]); 4 columns per thread (k1 % 4 == 0: a group never straddles), the splits
// shared by 2^L threads of a block and summed through LDS (wgrad_reduce_kernel's split-parallel layout)
__global__ __launch_bounds__(256) void wgrad_reduce_dual_kernel(const float* __restrict__ part, int splits, int cout,
                                                                int k1, int k2, const float* __restrict__ scale1,
                                                                const float* __restrict__ scale2, float* __restrict__ out1,
                                                                float* __restrict__ out2, int accumulate, int L) {
  __shared__ f32x4 red[256];
  const int Kt = k1 + k2;
  const long long n = (long long)cout * Kt;
  const int cpb = 256 >> L, spl = 1 << L;
  const int col = threadIdx.x & (cpb - 1), r = threadIdx.x >> (8 - L);
  const long long i = (long long)blockIdx.x * cpb + col;       // 4-column group
  const long long e = 4 * i;
  f32x4 s0 = {0.f, 0.f, 0.f, 0.f}, s1 = s0;
  if (e < n) {
    int t = r;
    for (; t + spl < splits; t += 2 * spl) {
      s0 += *reinterpret_cast<const f32x4*>(part + (size_t)t * n + e);
      s1 += *reinterpret_cast<const f32x4*>(part + (size_t)(t + spl) * n + e);
    }
    if (t < splits) s0 += *reinterpret_cast<const f32x4*>(part + (size_t)t * n + e);
  }
  red[threadIdx.x] = s0 + s1;
  __syncthreads();
  if (r != 0 || e >= n) return;
  f32x4 s = red[col];
  for (int q = 1; q < spl; ++q) s += red[q * cpb + col];
  const int co = (int)(e / Kt), k = (int)(e - (long long)co * Kt);
  float* o;
  if (k < k1) {
    if (scale1) s *= scale1[co];
    o = out1 + (size_t)co * k1 + k;
  } else {
    if (scale2) s *= scale2[co];
    o = out2 + (size_t)co * k2 + (k - k1);
  }
  if (accumulate) s += *reinterpret_cast<const f32x4*>(o);
  *reinterpret_cast<f32x4*>(o) = s;
}

void mxr_wgrad_reduce_dual_launch(const float* part, int splits, int cout, int k1, int k2, const float* scale1,
                                  const float* scale2, float* out1, float* out2, int accumulate, hipStream_t stream) {
  const long long nv = (long long)cout * (k1 + k2) / 4;
  int L = 0;     // as wgrad_reduce: split rows until ~2 blocks per CU (or < 2 slabs per thread)
  while (L < 6 && (nv + (256 >> L) - 1) / (256 >> L) < 512 && (2 << L) <= splits / 2) ++L;
  const long long cpb = 256 >> L;
  wgrad_reduce_dual_kernel<<<(unsigned)((nv + cpb - 1) / cpb), 256, 0, stream>>>(part, splits, cout, k1, k2, scale1,
                                                                                 scale2, out1, out2, accumulate, L);
}

// db[c] (+)= scale[c] * sum_m dY[m, c]; part: nblk * C floats (nblk = 512).
// nout <= C: only the first nout sums are written (a narrow layer's gradient in zero-padded rows: the
// column sums run over C = nout rounded up to 8, within the row pitch ld).
MXR_API int mxr_bias_grad(const void* dY, long long M, int C, int ld, int nout, float* part, float* out,
                          const float* scale, int accumulate, hipStream_t stream) {
  if (C % 8 != 0 || C / 8 > 256 || ld % 8 != 0 || C > ld || nout > C || nout < 1) return -1;
  const int nblk = 512;
  colsum_partial_kernel<<<nblk, 256, 0, stream>>>((const bf16_t*)dY, M, C, ld, part);
  colsum_final_kernel<<<nout, 256, 0, stream>>>(part, nblk, C, scale, out, accumulate);
  return (int)hipGetLastError();
}
