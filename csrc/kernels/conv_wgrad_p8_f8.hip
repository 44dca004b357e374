// FP8 weight gradient (e5m2 dY x e4m3 X, fp32 accumulation) of the packed head / FPN convs for gfx950 -- the
// phase-pipelined conv_wgrad_p8.hip schedule on v_mfma_scale_f32_16x16x128_f8f6f4 (BASELINE config 5: "fp8
// weights + activations"; the weight gradients of the layers built at /root/reference/train.py:91):
//
//   dW[co, k] = inv_x * inv_dy * sum_m dYq[m, co] * Aq[m, k]      (A = im2col(Xq), k = (ky, kx, ci), OHWI)
//
// * the operands are the fp8 copies the step already holds: Xq from the forward's fused epilogue (the
//   packed features / tower outputs, per-tensor e4m3 scale), dYq from the data-gradient path (per-tensor e5m2
//   scale, quantised once for the fp8 dgrad); both scales are device scalars multiplied into the slabs;
// * per 256 (k) x 256 (co) tile and split of the pixel range: K-tile = 128 pixel rows (twice conv_wgrad_p8's
//   64 -- one byte per value), each operand held as two column HALVES of 128 columns (128 rows x 128 B,
//   lane-linear LDS images filled by LDS-DMA in 1-KiB pieces of 8 rows); two buffers, 128 KiB;
// * 8 waves as 2 (k) x 4 (co), conv_wgrad_p8's phase order (U0,T0) (U0,T1) (U1,T1) (U1,T0), the next K-tile's
//   halves fetched one per phase, counted vmcnt(4) waits;
// * both operands are read transposed with ds_read_b64_tr_b8: per 16-lane group g (pixels 32 g .. 32 g + 31 of
//   the K-tile) four reads of 8 rows x 16 columns give each lane the 32 bytes of its column (channel) -- the
//   32-B operand of one 16x16x128 MFMA; A and B lanes hold the same pixels at the same byte positions, so the
//   contraction pairs identical k whatever the instruction's internal k order (conv_p8_f8.hip);
// * the 16-B chunks of a 128-B row are XOR-swizzled by f(r) = (r >> 1 & 3) | (r >> 5 & 1) << 2 through the
//   DMA source address: a 32-lane half's two 8-row blocks (rows 8 q + j and 32 + 8 q + j) hit 64 distinct banks;
// * fp32 split-K slabs part[split][co][k] (already scaled by inv_x * inv_dy), reduced in fixed order by
//   mxr_wgrad_reduce_launch (conv_wgrad.hip);
// * BIAS: the bias gradient db[co] = inv_dy * sum_m dYq[m, co] rides along (conv_wgrad_p8.hip's one-hot trick on
//   the scaled MFMA): the k-tile-0 blocks' wk = 0 waves multiply each T fragment they hold by an e4m3 A fragment
//   whose row j is all ones (4 extra MFMAs per 128 K-tile rows against 64), so the fp8 step needs no bf16 column-sum
//   pass over dY -- the sums are of the e5m2 values the weight gradient contracts.
#include "conv_common.h"

typedef __attribute__((ext_vector_type(8))) int i32x8;
typedef __attribute__((ext_vector_type(2))) int i32x2;

void mxr_wgrad_reduce_launch(const float* part, int splits, long long n, int K, const float* scale, float* out,
                             int accumulate, hipStream_t stream);

namespace {

constexpr int W8_NW = 8;
constexpr int W8_HB = 128 * 128;                // one half image: 128 pixel rows x 128 B
constexpr int W8_BUF = 4 * W8_HB;               // U0 U1 T0 T1
constexpr int W8_LDS = 2 * W8_BUF + 6 * MXR_MAXLEV * 4;

__device__ __forceinline__ i32x2 w8_tr(const char* p) {
  return __builtin_amdgcn_ds_read_tr8_b64_v2i32((__attribute__((address_space(3))) i32x2*)(p));
}

__device__ __forceinline__ int w8_swz(int r) { return ((r >> 1) & 3) | (((r >> 5) & 1) << 2); }

template <int N>
__device__ __forceinline__ void w8_vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <int PRIO, int BIAS>
__global__ __launch_bounds__(W8_NW * 64, 2) void conv_wgrad_p8_f8_kernel(
    const uint8_t* __restrict__ X, const uint8_t* __restrict__ dY, int ldy, const float* __restrict__ inv_x,
    const float* __restrict__ inv_dy, float* __restrict__ part, float* __restrict__ bpart,
    const uint8_t* __restrict__ zpage, ConvGeom g, int tiles_k, int tiles_co, int splits, int ntm) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wid = xcd_remap(blockIdx.x, gridDim.x);
  const int tk = wid % tiles_k;
  const int rest = wid / tiles_k;
  const int tco = rest % tiles_co;
  const int split = rest / tiles_co;
  const int co0 = tco * 256, k0 = tk * 256;
  const int K = g.kh * g.kw * g.cin;
  const int t_begin = (int)((long long)ntm * split / splits), t_end = (int)((long long)ntm * (split + 1) / splits);

  // level tables -> LDS behind the buffers (read on the rare level carry only)
  int* lt = reinterpret_cast<int*>(smem + 2 * W8_BUF);   // [H, W, Ho, Wo, in_off, mstart] x MXR_MAXLEV
  if (threadIdx.x < 6 * MXR_MAXLEV) {
    const int a = threadIdx.x / MXR_MAXLEV, t = threadIdx.x % MXR_MAXLEV;
    const int* src = a == 0 ? g.H : a == 1 ? g.W : a == 2 ? g.Ho : a == 3 ? g.Wo : a == 4 ? g.in_off : g.mstart;
    lt[threadIdx.x] = src[t];
  }
  __syncthreads();

  // ---- DMA slots: piece s (0, 1) of every half = rows 8 (wave + 8 s) + lane / 8, LDS chunk lane % 8
  const int pos = lane & 7;
  int rrow[2];
  int u_ci[2][2], u_dy[2][2], u_dx[2][2], u_ok[2][2];   // [half][piece]: fixed im2col column of the lane
  int t_co[2][2];                                        // [half][piece]: dY column (-1 outside)
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    rrow[s] = 8 * (wave + 8 * s) + (lane >> 3);
    const int lc = pos ^ w8_swz(rrow[s]);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int k = k0 + h * 128 + lc * 16;
      const int tap = k / g.cin;
      u_ok[h][s] = k < K;
      u_ci[h][s] = k - tap * g.cin;
      u_dy[h][s] = tap / g.kw;
      u_dx[h][s] = tap - u_dy[h][s] * g.kw;
      const int co = co0 + h * 128 + lc * 16;
      t_co[h][s] = co < ldy ? co : -1;
    }
  }
  // the lane's two pixel rows, advanced by 128 per K-tile
  int p_m[2], p_oy[2], p_ox[2], p_l[2], p_img[2], p_H[2], p_W[2], p_Ho[2], p_Wo[2], p_off[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const long long m = (long long)t_begin * 128 + rrow[s];
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
    char* buf = smem + ((n_t - t_begin) & 1) * W8_BUF;
    const bool live = n_t < t_end;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      char* dst;
      uintptr_t a = (uintptr_t)zpage;
      const bool mok = live && p_m[s] < g.M;
      if (hx == 1 || hx == 2) {
        const int h = hx - 1;
        dst = buf + (2 + h) * W8_HB + (wave + 8 * s) * 1024;
        if (mok && t_co[h][s] >= 0) a = (uintptr_t)(dY + (long long)p_m[s] * ldy + t_co[h][s]);
      } else {
        const int h = hx == 0 ? 0 : 1;
        dst = buf + h * W8_HB + (wave + 8 * s) * 1024;
        const int iy = p_oy[s] * g.stride - g.pt + u_dy[h][s];
        const int ix = p_ox[s] * g.stride - g.pl + u_dx[h][s];
        if (mok && u_ok[h][s] && (unsigned)iy < (unsigned)p_H[s] && (unsigned)ix < (unsigned)p_W[s])
          a = (uintptr_t)(X + (long long)(p_img[s] + p_off[s] + iy * p_W[s] + ix) * g.cin + u_ci[h][s]);
      }
      glds16_asm((const void*)a, dst);
    }
    if (hx == 3) {
      ++n_t;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        p_m[s] += 128;
        p_ox[s] += 128;
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

  // ---- transposed fragment reads: lane (2 j + p) of 16-lane group gq reads row 32 gq + 8 q + j, bytes 8 p .. 8 p + 7
  // of a 16-column block (q = 0..3 -> the 32 pixels of the group); the lane receives its column's 8 rows per read
  const int gq = lane >> 4, jj = (lane & 15) >> 1, pp = lane & 1;
  const int wk = wave >> 2, wc = wave & 3;
  int rowb[4];          // byte offset of row 32 gq + 8 q + jj
  int rsw[4];           // its swizzle
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int r = 32 * gq + 8 * q + jj;
    rowb[q] = r * 128 + pp * 8;
    rsw[q] = w8_swz(r);
  }
  auto frag = [&](const char* img, int cb) {
    i32x8 v;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const i32x2 t = w8_tr(img + rowb[q] + ((cb ^ rsw[q]) << 4));
      v[2 * q] = t[0];
      v[2 * q + 1] = t[1];
    }
    return v;
  };
  auto read_u = [&](i32x8 (&fa)[4], const char* img) {
#pragma unroll
    for (int i = 0; i < 4; ++i) fa[i] = frag(img, 4 * wk + i);
  };
  auto read_t = [&](i32x8 (&fb)[2], const char* img) {
#pragma unroll
    for (int j = 0; j < 2; ++j) fb[j] = frag(img, 2 * wc + j);
  };

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
                                                                              0, 1, 0, 127, 0, 127);
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);
    // pin the phase's results here (an opaque use the barriers cannot pass): conv_p8_f8.hip found hipcc otherwise
    // sinks the MFMAs to the loop end and hoists every fragment read above them
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) asm volatile("" : "+v"(acc[i0 + i][j0 + j]));
  };
  // BIAS: column sums of this wave's four T fragments j (co as acc[.][j]) in ONE accumulator -- fragment j times an
  // A fragment whose row j is e4m3 1.0 and the other rows zero puts fragment j's column sums in row j (lanes 0-15,
  // element j)
  f32x4 accb = {0.f, 0.f, 0.f, 0.f};
  const bool bsum = BIAS && tk == 0 && wk == 0;
  auto colsum = [&](const i32x8 (&fb)[2], int j0) {
    if (bsum) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        // the one-hot row, rebuilt here (opaque: not hoisted out of the loop into live fragments)
        int v = (lane & 15) == j0 + j ? 0x38383838 : 0;
        asm volatile("" : "+v"(v));
        const i32x8 a = {v, v, v, v, v, v, v, v};
        accb = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, fb[j], accb, 0, 1, 0, 127, 0, 127);
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
    const char* buf = smem + ((t - t_begin) & 1) * W8_BUF;
    i32x8 fa0[4], fa1[4], fb0[2], fb1[2];
    // phase 0: U-half 0 + T-half 0
    w8_vm_wait<4>();
    sync();
    issue_half(0);
    read_u(fa0, buf);
    read_t(fb0, buf + 2 * W8_HB);
    mma(fa0, fb0, 0, 0);
    // phase 1: T-half 1
    w8_vm_wait<4>();
    sync();
    issue_half(1);
    read_t(fb1, buf + 3 * W8_HB);
    mma(fa0, fb1, 0, 2);
    // phase 2: U-half 1
    w8_vm_wait<4>();
    sync();
    issue_half(2);
    read_u(fa1, buf + W8_HB);
    mma(fa1, fb1, 4, 2);
    // (the bias sums of a T half right after its last use: no fragment lives longer than without them)
    if constexpr (BIAS) colsum(fb1, 2);
    // phase 3: nothing new to read
    issue_half(3);
    mma(fa1, fb0, 4, 0);
    if constexpr (BIAS) colsum(fb0, 0);
  }
  w8_vm_wait<0>();

  if constexpr (BIAS) {
    // row j of the one-hot products (lanes 0-15, element j) = the split's column sums of fragment j
    if (bsum && lane < 16) {
      const float sb = *inv_dy;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int co = co0 + (j >> 1) * 128 + wc * 32 + (j & 1) * 16 + lane;
        if (co < g.cout) bpart[(long long)split * g.cout + co] = accb[j] * sb;
      }
    }
  }

  // slab write: part[split][co][k] (x inv_x * inv_dy); acc[i][j] holds k = base + 4 (lane / 16) .. + 3 of
  // co = base + lane % 16 (the 16x16 accumulator map, as in conv_wgrad_p8.hip)
  const float sc = (*inv_x) * (*inv_dy);
  float* slab = part + (long long)split * g.cout * K;
  const int kg = lane >> 4;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int co = co0 + (j >> 1) * 128 + wc * 32 + (j & 1) * 16 + (lane & 15);
    if (co >= g.cout) continue;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int k = k0 + (i >> 2) * 128 + wk * 64 + (i & 3) * 16 + 4 * kg;
      if (k >= K) continue;
      *reinterpret_cast<f32x4*>(slab + (long long)co * K + k) = acc[i][j] * sc;
    }
  }
}

template <int PRIO, int BIAS>
int launch_w8(const uint8_t* X, const uint8_t* dY, int ldy, const float* inv_x, const float* inv_dy, float* part,
              float* bpart, int splits, const uint8_t* zpage, const ConvGeom& g, hipStream_t stream) {
  const int K = g.kh * g.kw * g.cin;
  const int tiles_k = (K + 255) / 256;
  const int tiles_co = (g.cout + 255) / 256;
  const long long ntm = (g.M + 127) / 128;
  if (ntm > 0x7fffffffLL) return -4;
  const long long nwg = (long long)tiles_k * tiles_co * splits;
  auto kern = conv_wgrad_p8_f8_kernel<PRIO, BIAS>;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, W8_LDS);
    attr_set = true;
  }
  kern<<<(unsigned)nwg, W8_NW * 64, W8_LDS, stream>>>(X, dY, ldy, inv_x, inv_dy, part, bpart, zpage, g, tiles_k,
                                                      tiles_co, splits, (int)ntm);
  return (int)hipGetLastError();
}

}  // namespace

// dW (OHWI fp32) (+)= scale[co] * inv_x * inv_dy * sum_m dYq[m, co] Aq[m, k]: Xq e4m3 (M pixels x cin, the conv's
// input levels), dYq e5m2 (M x ldy, columns past cout ignored), inv_x / inv_dy device scalars.  part: splits * cout
// * K floats (+ splits * cout with bias_out: db = inv_dy * sum_m dYq[m, :cout] (+)= into bias_out).  variant 0:
// plain, 1: s_setprio around the MFMA blocks.  Requires cin % 16 == 0, ldy % 16 == 0, ostride == 1.
MXR_API int mxr_conv_wgrad_p8_f8_bias(const void* Xq, const void* dYq, int ldy, const float* inv_x, const float* inv_dy,
                                      float* part, int splits, float* out, const float* scale, int accumulate,
                                      const void* zpage, const ConvGeom* g, int variant, float* bias_out,
                                      int bias_accumulate, hipStream_t stream) {
  if (g->cin % 16 != 0 || ldy % 16 != 0 || g->ostride != 1 || splits < 1) return -1;
  if (g->nlev < 1 || g->nlev > MXR_MAXLEV) return -2;
  if (g->M + 256 >= (1LL << 31)) return -4;
  const uint8_t *x = (const uint8_t*)Xq, *dy = (const uint8_t*)dYq, *z = (const uint8_t*)zpage;
  const int K = g->kh * g->kw * g->cin;
  float* bpart = bias_out ? part + (long long)splits * g->cout * K : nullptr;
  int rc;
  if (bias_out)
    rc = variant == 1 ? launch_w8<1, 1>(x, dy, ldy, inv_x, inv_dy, part, bpart, splits, z, *g, stream)
                      : launch_w8<0, 1>(x, dy, ldy, inv_x, inv_dy, part, bpart, splits, z, *g, stream);
  else
    rc = variant == 1 ? launch_w8<1, 0>(x, dy, ldy, inv_x, inv_dy, part, nullptr, splits, z, *g, stream)
                      : launch_w8<0, 0>(x, dy, ldy, inv_x, inv_dy, part, nullptr, splits, z, *g, stream);
  if (rc) return rc;
  mxr_wgrad_reduce_launch(part, splits, (long long)g->cout * K, K, scale, out, accumulate, stream);
  // the bias partials: one "row" of cout values (K past any index -> no per-row scale lookup)
  if (bias_out) mxr_wgrad_reduce_launch(bpart, splits, g->cout, 1 << 30, nullptr, bias_out, bias_accumulate, stream);
  return (int)hipGetLastError();
}

MXR_API int mxr_conv_wgrad_p8_f8(const void* Xq, const void* dYq, int ldy, const float* inv_x, const float* inv_dy,
                                 float* part, int splits, float* out, const float* scale, int accumulate,
                                 const void* zpage, const ConvGeom* g, int variant, hipStream_t stream) {
  return mxr_conv_wgrad_p8_f8_bias(Xq, dYq, ldy, inv_x, inv_dy, part, splits, out, scale, accumulate, zpage, g, variant,
                                   nullptr, 0, stream);
}
