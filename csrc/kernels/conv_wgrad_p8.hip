// Phase-pipelined NHWC bf16 implicit-GEMM WEIGHT gradient for gfx950 (the conv_p8.hip structure applied to
// the wgrad GEMM):
//
//   dW[co, k] = sum_m dY[m, co] * A[m, k]      (A = im2col(X), k = (ky, kx, ci), OHWI layout)
//
// conv_wgrad_pipe.hip consumes the pixel reduction in 32-row sub-stages with a barrier each and reads
// every fragment after its barrier (690 TF/s on the head towers, profiles/r1_conv_budget_387ips.txt).
// Here, per 256 (k) x 256 (co) output tile and split of the pixel range:
//
// * K-tile = 64 pixel rows; each operand tile is held as two column HALVES of 128 columns (64 rows x 256 B,
//   lane-linear LDS images that LDS-DMA fills in 1 KiB pieces of 4 rows): U0 / U1 (im2col columns
//   k0 + [0, 128) / [128, 256)) and T0 / T1 (dY columns co0 + [0, 128) / [128, 256)); two buffers,
//   128 KiB;
// * 8 waves as 2 (k) x 4 (co); wave (wk, wc) owns k columns wk * 64 + [0, 64) of both U halves and co
//   columns wc * 32 + [0, 32) of both T halves, so a quadrant of its 8 x 4 accumulators reads exactly
//   one U half and one T half; 4 phases of 16 MFMAs per K-tile in the order (U0,T0) (U0,T1) (U1,T1)
//   (U1,T0) with fragment registers reused across phases; the NEXT K-tile's halves are fetched one per
//   phase in consumption order (U0, T0, T1, U1) so every counted wait is vmcnt(4);
// * both operands are read transposed (ds_read_b64_tr_b16, conv_wgrad_pipe.hip's fragment pattern);
//   the 16-B chunks of a 256-B row are XOR-swizzled by (r & 3) << 1 | ((r >> 3) & 1) << 3 through the
//   DMA source address -- conflict-free for the 8 rows a 32-lane half reads;
// * the im2col gather: each lane's (tap, channel) per half is fixed for the block; its two pixel rows
//   advance by 64 per K-tile incrementally (row / level / image carries, level geometry from an LDS copy
//   of the tables: the DMA is the only vector-memory op in the loop, so the counted waits are exact);
// * fp32 split-K slabs part[split][co][k], reduced (and scaled by the frozen-BN scale) in fixed order by
//   mxr_wgrad_reduce_launch (conv_wgrad.hip);
// * BIAS: the bias gradient db[co] = sum_m dY[m, co] rides along.  The k-tile-0 blocks already hold every
//   dY row of their split as T fragments: their wk = 0 waves multiply them by an all-ones A fragment
//   (8 extra MFMAs per 64 K-tile rows, against the 64 of the tile) and write a per-split partial
//   bpart[split][co], reduced like the weight slabs -- instead of a separate colsum pass that re-reads
//   all of dY from HBM (the head towers: 182 MB per layer).
#include "conv_common.h"

typedef __attribute__((ext_vector_type(4))) short s16x4;

void mxr_wgrad_reduce_launch(const float* part, int splits, long long n, int K, const float* scale, float* out,
                             int accumulate, hipStream_t stream);
void mxr_wgrad_reduce_dual_launch(const float* part, int splits, int cout, int k1, int k2, const float* scale1,
                                  const float* scale2, float* out1, float* out2, int accumulate, hipStream_t stream);

namespace {

constexpr int WQ_NW = 8;
constexpr int WQ_HB = 64 * 256;                 // one half image: 64 pixel rows x 256 B
constexpr int WQ_BUF = 4 * WQ_HB;               // U0 U1 T0 T1
constexpr int WQ_LDS = 2 * WQ_BUF + 6 * MXR_MAXLEV * 4;

__device__ __forceinline__ s16x4 wq_tr(const char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(p));
}

__device__ __forceinline__ int wq_swz(int r) { return ((r & 3) << 1) | (((r >> 3) & 1) << 3); }

template <int N>
__device__ __forceinline__ void wq_vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// RF: fragment reads issued before the phase's DMA pieces; OPQ: the DMA as inline asm (glds16_asm: no
// compiler-inserted vmcnt(0) in front of the phase-0 transposed reads -- the counted waits are the sync)
// DS: dual-source weight gradient of a projection block (branch2c + branch1 over ONE read of dY):
// dW[co, k] for k < k1 over X1 = the branch2b output [M, k1] (row m of the output grid), for k >= k1 over the 1x1
// stride-s im2col of X (g: the branch1 geometry, g.cin = K - k1); K = Kt; the slab row holds both weight matrices.
template <int PRIO, int RF = 0, int BIAS = 0, int OPQ = 0, int DS = 0>
__global__ __launch_bounds__(WQ_NW * 64, 2) void conv_wgrad_p8_kernel(
    const bf16_t* __restrict__ X, const bf16_t* __restrict__ dY, int ldy, float* __restrict__ part,
    float* __restrict__ bpart, const bf16_t* __restrict__ zpage, ConvGeom g, int tiles_k, int tiles_co, int splits,
    int ntm, const bf16_t* __restrict__ X1, int k1, int Kt) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wid = xcd_remap(blockIdx.x, gridDim.x);
  const int tk = wid % tiles_k;
  const int rest = wid / tiles_k;
  const int tco = rest % tiles_co;
  const int split = rest / tiles_co;
  const int co0 = tco * 256, k0 = tk * 256;
  const int K = DS ? Kt : g.kh * g.kw * g.cin;
  const int t_begin = (int)((long long)ntm * split / splits), t_end = (int)((long long)ntm * (split + 1) / splits);

  // level tables -> LDS behind the buffers (read on the rare level carry only)
  int* lt = reinterpret_cast<int*>(smem + 2 * WQ_BUF);   // [H, W, Ho, Wo, in_off, mstart] x MXR_MAXLEV
  if (threadIdx.x < 6 * MXR_MAXLEV) {
    const int a = threadIdx.x / MXR_MAXLEV, t = threadIdx.x % MXR_MAXLEV;
    const int* src = a == 0 ? g.H : a == 1 ? g.W : a == 2 ? g.Ho : a == 3 ? g.Wo : a == 4 ? g.in_off : g.mstart;
    lt[threadIdx.x] = src[t];
  }
  __syncthreads();

  // ---- DMA slots: piece s (0, 1) of every half = rows 4 (wave + 8 s) + lane / 16, LDS chunk lane % 16
  const int pos = lane & 15;
  int rrow[2];
  int u_ci[2][2], u_dy[2][2], u_dx[2][2], u_ok[2][2];   // [half][piece]: fixed im2col column of the lane
  int t_co[2][2];                                        // [half][piece]: dY column (-1 outside)
  bool u_x1[2][2];                                       // DS: the column reads X1
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    rrow[s] = 4 * (wave + 8 * s) + (lane >> 4);
    const int lc = pos ^ wq_swz(rrow[s]);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int k = k0 + h * 128 + lc * 8;
      u_ok[h][s] = k < K;
      if constexpr (DS) {
        u_x1[h][s] = k < k1;
        u_ci[h][s] = k < k1 ? k : k - k1;
        u_dy[h][s] = u_dx[h][s] = 0;
      } else {
        u_x1[h][s] = false;
        const int tap = k / g.cin;
        u_ci[h][s] = k - tap * g.cin;
        u_dy[h][s] = tap / g.kw;
        u_dx[h][s] = tap - u_dy[h][s] * g.kw;
      }
      const int co = co0 + h * 128 + lc * 8;
      t_co[h][s] = co < ldy ? co : -1;
    }
  }
  // the lane's two pixel rows, advanced by 64 per K-tile
  int p_m[2], p_oy[2], p_ox[2], p_l[2], p_img[2], p_H[2], p_W[2], p_Ho[2], p_Wo[2], p_off[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const long long m = (long long)t_begin * 64 + rrow[s];
    p_m[s] = (int)m;
    int b = 0, q = 0, l = 0;
    if (m < g.M) {
      b = (int)(m / g.out_img);
      q = (int)(m - (long long)b * g.out_img);
      for (int t = 1; t < g.nlev; ++t)
        if (q >= lt[5 * MXR_MAXLEV + t]) l = t;
    }
    const int loc = q - lt[5 * MXR_MAXLEV + l];
    p_l[s] = l;
    p_img[s] = b * g.in_img;
    p_H[s] = lt[l];
    p_W[s] = lt[MXR_MAXLEV + l];
    p_Ho[s] = lt[2 * MXR_MAXLEV + l];
    p_Wo[s] = lt[3 * MXR_MAXLEV + l];
    p_off[s] = lt[4 * MXR_MAXLEV + l];
    p_oy[s] = loc / p_Wo[s];
    p_ox[s] = loc - p_oy[s] * p_Wo[s];
  }

  int n_t = t_begin;   // K-tile being issued
  // hx = 0 U-half 0, 1 T-half 0, 2 T-half 1, 3 U-half 1 of K-tile n_t into buffer (n_t - t_begin) & 1
  auto issue_half = [&](int hx) {
    char* buf = smem + ((n_t - t_begin) & 1) * WQ_BUF;
    const bool live = n_t < t_end;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      char* dst;
      uintptr_t a = (uintptr_t)zpage;
      const bool mok = live && p_m[s] < g.M;
      if (hx == 1 || hx == 2) {
        const int h = hx - 1;
        dst = buf + (2 + h) * WQ_HB + (wave + 8 * s) * 1024;
        if (mok && t_co[h][s] >= 0) a = (uintptr_t)(dY + (long long)p_m[s] * ldy + t_co[h][s]);
      } else {
        const int h = hx == 0 ? 0 : 1;
        dst = buf + h * WQ_HB + (wave + 8 * s) * 1024;
        const int iy = p_oy[s] * g.stride - g.pt + u_dy[h][s];
        const int ix = p_ox[s] * g.stride - g.pl + u_dx[h][s];
        if (DS && u_x1[h][s]) {
          if (mok && u_ok[h][s]) a = (uintptr_t)(X1 + (long long)p_m[s] * k1 + u_ci[h][s]);
        } else if (mok && u_ok[h][s] && (unsigned)iy < (unsigned)p_H[s] && (unsigned)ix < (unsigned)p_W[s]) {
          a = (uintptr_t)(X + (long long)(p_img[s] + p_off[s] + iy * p_W[s] + ix) * g.cin + u_ci[h][s]);
        }
      }
      if constexpr (OPQ) glds16_asm((const void*)a, dst);
      else glds16((const void*)a, dst);
    }
    if (hx == 3) {
      ++n_t;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        p_m[s] += 64;
        p_ox[s] += 64;
        while (p_ox[s] >= p_Wo[s]) {
          p_ox[s] -= p_Wo[s];
          if (++p_oy[s] >= p_Ho[s]) {
            p_oy[s] = 0;
            int l = p_l[s] + 1;
            if (l >= g.nlev) { l = 0; p_img[s] += g.in_img; }
            p_l[s] = l;
            p_H[s] = lt[l];
            p_W[s] = lt[MXR_MAXLEV + l];
            p_Ho[s] = lt[2 * MXR_MAXLEV + l];
            p_Wo[s] = lt[3 * MXR_MAXLEV + l];
            p_off[s] = lt[4 * MXR_MAXLEV + l];
          }
        }
      }
    }
  };

  // ---- transposed fragment reads (conv_wgrad_pipe.hip's pattern): lane 4q + p of a 16-lane group reads
  // row kg * 8 + q (and + 4), columns 4p .. 4p + 3 of a 16-column block
  const int kg = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
  const int r0 = kg * 8 + q;
  const int sw = wq_swz(r0);            // identical for r0 + 4 and r0 + 32
  const int wk = wave >> 2, wc = wave & 3;
  int aro[4], bro[2];                   // byte offsets inside a half image (row r0), per fragment slot
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = ((wk * 64 + i * 16) >> 3) + (p >> 1);
    aro[i] = r0 * 256 + ((c ^ sw) << 4) + (p & 1) * 8;
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int c = ((wc * 32 + j * 16) >> 3) + (p >> 1);
    bro[j] = r0 * 256 + ((c ^ sw) << 4) + (p & 1) * 8;
  }
  auto frag = [&](const char* img, int off, int kk) {
    const char* a = img + off + kk * 32 * 256;
    const s16x4 lo = wq_tr(a), hi = wq_tr(a + 4 * 256);
    return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  };
  auto read_u = [&](bf16x8 (&fa)[4][2], const char* img) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) fa[i][kk] = frag(img, aro[i], kk);
  };
  auto read_t = [&](bf16x8 (&fb)[2][2], const char* img) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) fb[j][kk] = frag(img, bro[j], kk);
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // BIAS: column sums of this wave's four T fragments j (co as acc[.][j]) in ONE accumulator: fragment j is
  // multiplied by an A fragment whose row j is all ones and the other rows zero, so row j of accb (lanes
  // 0-15, element j) sums fragment j's columns (4 VGPRs instead of 16 + a ones fragment: the kernel
  // sits at 240 of its 256)
  f32x4 accb = {0.f, 0.f, 0.f, 0.f};
  const bool bsum = BIAS && tk == 0 && wk == 0;
  auto mma = [&](const bf16x8 (&fa)[4][2], const bf16x8 (&fb)[2][2], int i0, int j0) {
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i0 + i][j0 + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][kk], fb[j][kk], acc[i0 + i][j0 + j], 0, 0, 0);
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);
  };
  auto colsum = [&](const bf16x8 (&fb)[2][2], int j0) {
    if (bsum) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        // the one-hot row, rebuilt here (opaque: not hoisted out of the loop into 4 live fragments)
        int v = (lane & 15) == j0 + j ? 0x3f803f80 : 0;
        asm volatile("" : "+v"(v));
        const bf16x8 a = __builtin_bit_cast(bf16x8, int4{v, v, v, v});
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) accb = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, fb[j][kk], accb, 0, 0, 0);
      }
    }
  };
  auto sync = [&]() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };

#pragma unroll
  for (int hx = 0; hx < 4; ++hx) issue_half(hx);
  for (int t = t_begin; t < t_end; ++t) {
    const char* buf = smem + ((t - t_begin) & 1) * WQ_BUF;
    bf16x8 fa0[4][2], fa1[4][2], fb0[2][2], fb1[2][2];
    // phase 0: U-half 0 + T-half 0
    wq_vm_wait<4>();
    sync();
    if constexpr (!RF) issue_half(0);
    read_u(fa0, buf);
    read_t(fb0, buf + 2 * WQ_HB);
    if constexpr (RF) issue_half(0);
    mma(fa0, fb0, 0, 0);
    // phase 1: T-half 1
    wq_vm_wait<4>();
    sync();
    if constexpr (!RF) issue_half(1);
    read_t(fb1, buf + 3 * WQ_HB);
    if constexpr (RF) issue_half(1);
    mma(fa0, fb1, 0, 2);
    // phase 2: U-half 1
    wq_vm_wait<4>();
    sync();
    if constexpr (!RF) issue_half(2);
    read_u(fa1, buf + WQ_HB);
    if constexpr (RF) issue_half(2);
    mma(fa1, fb1, 4, 2);
    // (the bias sums of a T half right after its last use: no fragment lives longer than without them)
    if constexpr (BIAS) colsum(fb1, 2);
    // phase 3: nothing new to read
    issue_half(3);
    mma(fa1, fb0, 4, 0);
    if constexpr (BIAS) colsum(fb0, 0);
  }
  wq_vm_wait<0>();

  if constexpr (BIAS) {
    // row j of the one-hot products (lanes 0-15, element j) = the split's column sums of fragment j
    if (bsum && lane < 16) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int co = co0 + (j >> 1) * 128 + wc * 32 + (j & 1) * 16 + lane;
        if (co < g.cout) bpart[(long long)split * g.cout + co] = accb[j];
      }
    }
  }
  // slab write: part[split][co][k]; acc[i][j] holds k = base + 4 kg .. + 3 of co = base + lane % 16
  float* slab = part + (long long)split * g.cout * K;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int co = co0 + (j >> 1) * 128 + wc * 32 + (j & 1) * 16 + (lane & 15);
    if (co >= g.cout) continue;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int k = k0 + (i >> 2) * 128 + wk * 64 + (i & 3) * 16 + 4 * kg;
      if (k >= K) continue;
      *reinterpret_cast<f32x4*>(slab + (long long)co * K + k) = acc[i][j];
    }
  }
}

template <int PRIO, int RF = 0, int BIAS = 0, int OPQ = 0>
int launch_wq(const bf16_t* X, const bf16_t* dY, int ldy, float* part, float* bpart, int splits,
              const bf16_t* zpage, const ConvGeom& g, hipStream_t stream) {
  const int K = g.kh * g.kw * g.cin;
  const int tiles_k = (K + 255) / 256;
  const int tiles_co = (g.cout + 255) / 256;
  const long long ntm = (g.M + 63) / 64;
  if (ntm > 0x7fffffffLL) return -4;
  const long long nwg = (long long)tiles_k * tiles_co * splits;
  auto kern = conv_wgrad_p8_kernel<PRIO, RF, BIAS, OPQ>;
  static bool attr_set = false;
  if (!attr_set) {
    hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, WQ_LDS);
    attr_set = true;
  }
  kern<<<(unsigned)nwg, WQ_NW * 64, WQ_LDS, stream>>>(X, dY, ldy, part, bpart, zpage, g, tiles_k, tiles_co, splits,
                                                      (int)ntm, nullptr, 0, K);
  return (int)hipGetLastError();
}

template <int PRIO, int RF, int OPQ>
int launch_wq_dual(const bf16_t* X, const bf16_t* X1, int k1, const bf16_t* dY, int ldy, float* part, int splits,
                   const bf16_t* zpage, const ConvGeom& g, hipStream_t stream) {
  const int Kt = k1 + g.cin;
  const int tiles_k = (Kt + 255) / 256;
  const int tiles_co = (g.cout + 255) / 256;
  const long long ntm = (g.M + 63) / 64;
  if (ntm > 0x7fffffffLL) return -4;
  const long long nwg = (long long)tiles_k * tiles_co * splits;
  auto kern = conv_wgrad_p8_kernel<PRIO, RF, 0, OPQ, 1>;
  static bool attr_set = false;
  if (!attr_set) {
    hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, WQ_LDS);
    attr_set = true;
  }
  kern<<<(unsigned)nwg, WQ_NW * 64, WQ_LDS, stream>>>(X, dY, ldy, part, nullptr, zpage, g, tiles_k, tiles_co, splits,
                                                      (int)ntm, X1, k1, Kt);
  return (int)hipGetLastError();
}

}  // namespace

template <int BIAS>
int launch_wq_variant(const bf16_t* x, const bf16_t* dy, int ldy, float* part, float* bpart, int splits,
                      const bf16_t* z, const ConvGeom& g, int variant, hipStream_t stream) {
  switch (variant) {
    case 1: return launch_wq<1, 0, BIAS>(x, dy, ldy, part, bpart, splits, z, g, stream);
    case 2: return launch_wq<0, 1, BIAS>(x, dy, ldy, part, bpart, splits, z, g, stream);
    case 3: return launch_wq<1, 1, BIAS>(x, dy, ldy, part, bpart, splits, z, g, stream);
    case 4: return launch_wq<0, 0, BIAS, 1>(x, dy, ldy, part, bpart, splits, z, g, stream);
    case 5: return launch_wq<1, 1, BIAS, 1>(x, dy, ldy, part, bpart, splits, z, g, stream);
    default: return launch_wq<0, 0, BIAS>(x, dy, ldy, part, bpart, splits, z, g, stream);
  }
}

// variant 0: plain; 1: s_setprio 1 around the MFMA blocks; 2 / 3: fragment reads ahead of the DMA pieces
// (without / with s_setprio); 4 / 5: 0 / 3 with the DMA as inline asm (glds16_asm).  part: splits * cout * K floats (+ splits * cout for the bias partials when
// bias_out is given: db = sum_m dY[m, :cout], unscaled, into bias_out, accumulated when bias_accumulate).
// Requires cin % 8 == 0, ldy % 8 == 0, ostride == 1 (and cout % 4 == 0 with bias_out).
MXR_API int mxr_conv_wgrad_p8_bias(const void* X, const void* dY, int ldy, float* part, int splits, float* out,
                                   const float* scale, int accumulate, const void* zpage, const ConvGeom* g,
                                   int variant, float* bias_out, int bias_accumulate, hipStream_t stream) {
  if (g->cin % 8 != 0 || ldy % 8 != 0 || g->ostride != 1) return -1;
  if (g->nlev < 1 || g->nlev > MXR_MAXLEV) return -2;
  if (g->M + 128 >= (1LL << 31)) return -4;
  if (bias_out && g->cout % 4) return -1;
  const bf16_t *x = (const bf16_t*)X, *dy = (const bf16_t*)dY, *z = (const bf16_t*)zpage;
  const int K = g->kh * g->kw * g->cin;
  float* bpart = bias_out ? part + (long long)splits * g->cout * K : nullptr;
  const int rc = bias_out ? launch_wq_variant<1>(x, dy, ldy, part, bpart, splits, z, *g, variant, stream)
                          : launch_wq_variant<0>(x, dy, ldy, part, nullptr, splits, z, *g, variant, stream);
  if (rc) return rc;
  mxr_wgrad_reduce_launch(part, splits, (long long)g->cout * K, K, scale, out, accumulate, stream);
  // the bias partials: one "row" of cout values (K past any index -> no per-row scale lookup)
  if (bias_out) mxr_wgrad_reduce_launch(bpart, splits, g->cout, 1 << 30, nullptr, bias_out, bias_accumulate, stream);
  return (int)hipGetLastError();
}

MXR_API int mxr_conv_wgrad_p8(const void* X, const void* dY, int ldy, float* part, int splits, float* out,
                              const float* scale, int accumulate, const void* zpage, const ConvGeom* g, int variant,
                              hipStream_t stream) {
  return mxr_conv_wgrad_p8_bias(X, dY, ldy, part, splits, out, scale, accumulate, zpage, g, variant, nullptr, 0,
                                stream);
}

// Dual-source weight gradient of a projection block (DS above): X = the block input [N, H, W, cin] (g: the branch1
// 1x1 / stride-s geometry), X1 = the branch2b output [M, k1] on the output grid, dY [M, ldy]; out1 (cout x k1) (+)=
// scale1[co] * dW2c, out2 (cout x cin) (+)= scale2[co] * dW1 through one split-K slab [splits][cout][k1 + cin].
// variant: as mxr_conv_wgrad_p8.  Requires k1 % 8 == 0, cin % 8 == 0, ldy % 8 == 0, kh = kw = 1, pads 0.
MXR_API int mxr_conv_wgrad_p8_dual(const void* X, const void* X1, int k1, const void* dY, int ldy, float* part,
                                   int splits, float* out1, float* out2, const float* scale1, const float* scale2,
                                   int accumulate, const void* zpage, const ConvGeom* g, int variant,
                                   hipStream_t stream) {
  if (g->cin % 8 != 0 || k1 % 8 != 0 || k1 < 8 || ldy % 8 != 0 || g->ostride != 1 || g->nlev != 1) return -1;
  if (g->kh != 1 || g->kw != 1 || g->pt != 0 || g->pl != 0) return -2;
  if (g->M + 128 >= (1LL << 31)) return -4;
  const bf16_t *x = (const bf16_t*)X, *x1 = (const bf16_t*)X1, *dy = (const bf16_t*)dY, *z = (const bf16_t*)zpage;
  int rc;
  switch (variant) {
    case 1: rc = launch_wq_dual<1, 0, 0>(x, x1, k1, dy, ldy, part, splits, z, *g, stream); break;
    case 2: rc = launch_wq_dual<0, 1, 0>(x, x1, k1, dy, ldy, part, splits, z, *g, stream); break;
    case 4: rc = launch_wq_dual<0, 0, 1>(x, x1, k1, dy, ldy, part, splits, z, *g, stream); break;
    default: rc = launch_wq_dual<0, 0, 0>(x, x1, k1, dy, ldy, part, splits, z, *g, stream); break;
  }
  if (rc) return rc;
  mxr_wgrad_reduce_dual_launch(part, splits, g->cout, k1, g->cin, scale1, scale2, out1, out2, accumulate, stream);
  return (int)hipGetLastError();
}
