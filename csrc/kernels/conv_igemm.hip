// NHWC bf16 implicit-GEMM convolution on CDNA4 MFMA (gfx950), forward + data-gradient.
//
// Covers every conv of the reference model (keras-resnet backbone with frozen BN folded into the
// bias, FPN and the shared heads; /root/reference/train.py:91 -> SURVEY §2.6 K1-K5, K7, K10):
//
//   Y[m, co] = act( sum_k  W[co, k] * A[m, k]  + bias[co] (+ R[m, co]) )
//   k = (ky, kx, ci) (OHWI weights, K contiguous),  A[m, k] = X[pixel(m) shifted by tap, ci] or 0
//
// * GEMM orientation is swapped (C^T = W . A^T): the MFMA "A" operand is the weight tile (rows =
//   output channels), the "B" operand the gathered pixel tile (rows = pixels), so every lane ends
//   with 4 consecutive output channels of one pixel -> 8-byte NHWC stores, bias/residual loads.
// * Both tiles are [rows][64 k] bf16 (128-B rows) in LDS, filled by global_load_lds_dwordx4
//   (LDS-DMA): one wave instruction = 8 rows x 128 B; the per-lane SOURCE address does the im2col
//   gather and the XOR swizzle (chunk ^= row & 7, rule 21: linear LDS dest, swizzled source and
//   read); out-of-image taps and partial tiles read from a zero page.
// * 2-stage LDS double buffer, one barrier per 64-deep K-step, v_mfma_f32_16x16x32_bf16.
// * Multi-level "pyramid" geometry: the M axis may span several feature maps laid out batch-major
//   ([b][level][y][x]), so the 5 pyramid levels of a shared head layer run as ONE ragged GEMM.
// * XCD-aware block remap so blocks sharing a pixel tile run on the same XCD (L2 reuse).
// * Data-gradient = the same kernel on dY with flipped/transposed weights (stride 1), or a 1x1
//   GEMM scattered with output stride 2 into a zeroed dX (Caffe-style strided 1x1 convs).
#include "common.h"

#include "conv_common.h"

namespace {

template <int BCO, int BPIX, int WCO, int WPIX>
__global__ __launch_bounds__(WCO* WPIX * 64) void conv_fwd_kernel(
    const bf16_t* __restrict__ X, const bf16_t* __restrict__ Wt, const float* __restrict__ bias,
    const bf16_t* __restrict__ R, const bf16_t* __restrict__ Mk, bf16_t* __restrict__ Y,
    const bf16_t* __restrict__ zpage, ConvGeom g, int relu,
    int accumulate, int tiles_co) {
  constexpr int NW = WCO * WPIX;
  constexpr int WT_CO = BCO / WCO, WT_PIX = BPIX / WPIX;
  constexpr int TI = WT_CO / 16, TJ = WT_PIX / 16;
  constexpr int NSLOT = (BCO + BPIX) / 8;
  static_assert(NSLOT % NW == 0, "staging slots must divide among waves");
  constexpr int NS = NSLOT / NW;
  constexpr int BUF = (BCO + BPIX) * 128;

  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wid = xcd_remap(blockIdx.x, gridDim.x);
  const int tco = wid % tiles_co;
  const long long tm = wid / tiles_co;
  const int co0 = tco * BCO;
  const long long m0 = tm * BPIX;
  const int K = g.kh * g.kw * g.cin;

  // ---- per-lane staging descriptors
  const bf16_t* wsrc[NS];
  PixSlot<NS> ps;
  int lchunk[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const int gs = wave * NS + s;
    const int row = gs * 8 + (lane >> 3);
    const int pc = lane & 7;
    const int lc = pc ^ (row & 7);
    lchunk[s] = lc;
    wsrc[s] = nullptr;
    ps.base[s] = -1;
    ps.iy0[s] = ps.ix0[s] = ps.Hl[s] = ps.Wl[s] = 0;
    if (gs * 8 < BCO) {
      const int co = co0 + row;
      if (co < g.cout) wsrc[s] = Wt + (long long)co * K + lc * 8;
    } else {
      const long long m = m0 + (row - BCO);
      if (m < g.M) {
        int b, oy, ox;
        decode_row(g, m, ps.base[s], ps.iy0[s], ps.ix0[s], ps.Hl[s], ps.Wl[s], b, oy, ox);
      }
    }
  }

  auto stage = [&](int buf, int kt, int ky, int kx, int c0) {
    char* base = smem + buf * BUF;
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const int gs = wave * NS + s;
      char* dst = base + gs * 1024;   // 8 rows x 128 B, wave-uniform
      const void* src;
      if (gs * 8 < BCO) {
        src = wsrc[s] ? (const void*)(wsrc[s] + kt * 64) : (const void*)zpage;
      } else {
        const int iy = ps.iy0[s] + ky, ix = ps.ix0[s] + kx;
        const bool ok = ps.base[s] >= 0 && iy >= 0 && iy < ps.Hl[s] && ix >= 0 && ix < ps.Wl[s];
        src = ok ? (const void*)(X + ((long long)(ps.base[s] + iy * ps.Wl[s] + ix)) * g.cin + c0 + lchunk[s] * 8)
                 : (const void*)zpage;
      }
      glds16(src, dst);
    }
  };

  f32x4 acc[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int wco = wave / WPIX, wpx = wave % WPIX;
  const int nk = K / 64;
  int ky = 0, kx = 0, c0 = 0;
  stage(0, 0, 0, 0, 0);
  __syncthreads();
  int cur = 0;
  for (int kt = 0; kt < nk; ++kt) {
    // advance the tap / channel cursor for k-step kt+1
    c0 += 64;
    if (c0 == g.cin) { c0 = 0; if (++kx == g.kw) { kx = 0; ++ky; } }
    if (kt + 1 < nk) stage(cur ^ 1, kt + 1, ky, kx, c0);
    const char* ab = smem + cur * BUF;
    const char* bb = ab + BCO * 128;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int lc = kk * 4 + (lane >> 4);
      bf16x8 af[TI], bfr[TJ];
#pragma unroll
      for (int i = 0; i < TI; ++i) {
        const int r = wco * WT_CO + i * 16 + (lane & 15);
        af[i] = *reinterpret_cast<const bf16x8*>(ab + r * 128 + ((lc ^ (r & 7)) << 4));
      }
#pragma unroll
      for (int j = 0; j < TJ; ++j) {
        const int r = wpx * WT_PIX + j * 16 + (lane & 15);
        bfr[j] = *reinterpret_cast<const bf16x8*>(bb + r * 128 + ((lc ^ (r & 7)) << 4));
      }
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
    cur ^= 1;
  }

  // ---- epilogue: lane holds 4 consecutive channels of one pixel per (i, j)
#pragma unroll
  for (int j = 0; j < TJ; ++j) {
    const long long m = m0 + wpx * WT_PIX + j * 16 + (lane & 15);
    if (m >= g.M) continue;
    long long obase;
    if (g.ostride == 1) {
      obase = m * g.cout;
    } else {
      const int b = (int)(m / g.out_img);
      const int q = (int)(m - (long long)b * g.out_img);
      const int oy = q / g.Wo[0], ox = q - (q / g.Wo[0]) * g.Wo[0];
      obase = (((long long)b * g.oH + oy * g.ostride + g.ooy) * g.oW + ox * g.ostride + g.oox) * g.cout;
    }
#pragma unroll
    for (int i = 0; i < TI; ++i) {
      const int co = co0 + wco * WT_CO + i * 16 + 4 * (lane >> 4);
      if (co >= g.cout) continue;
      float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
      if (bias) {
        const float4 bb4 = *reinterpret_cast<const float4*>(bias + co);
        v[0] += bb4.x; v[1] += bb4.y; v[2] += bb4.z; v[3] += bb4.w;
      }
      if (R) {
        const uint2 rr = *reinterpret_cast<const uint2*>(R + m * g.cout + co);
        v[0] += bf2f((bf16_t)(rr.x & 0xffff)); v[1] += bf2f((bf16_t)(rr.x >> 16));
        v[2] += bf2f((bf16_t)(rr.y & 0xffff)); v[3] += bf2f((bf16_t)(rr.y >> 16));
      }
      if (accumulate) {
        const uint2 rr = *reinterpret_cast<const uint2*>(Y + obase + co);
        v[0] += bf2f((bf16_t)(rr.x & 0xffff)); v[1] += bf2f((bf16_t)(rr.x >> 16));
        v[2] += bf2f((bf16_t)(rr.y & 0xffff)); v[3] += bf2f((bf16_t)(rr.y >> 16));
      }
      if (relu) {
#pragma unroll
        for (int t = 0; t < 4; ++t) v[t] = fmaxf(v[t], 0.f);
      }
      if (Mk) {   // relu-gradient mask of the consumer's input (dgrad of a relu output): keep where Mk > 0
        const uint2 mm = *reinterpret_cast<const uint2*>(Mk + obase + co);
        if (!(bf2f((bf16_t)(mm.x & 0xffff)) > 0.f)) v[0] = 0.f;
        if (!(bf2f((bf16_t)(mm.x >> 16)) > 0.f)) v[1] = 0.f;
        if (!(bf2f((bf16_t)(mm.y & 0xffff)) > 0.f)) v[2] = 0.f;
        if (!(bf2f((bf16_t)(mm.y >> 16)) > 0.f)) v[3] = 0.f;
      }
      uint2 o;
      o.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
      o.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
      *reinterpret_cast<uint2*>(Y + obase + co) = o;
      if (g.ostride == 2 && !accumulate && g.ooy == 0 && g.oox == 0) {   // also zero the scatter gaps (see conv_pipe.hip)
        const int b = (int)(m / g.out_img);
        const int q = (int)(m - (long long)b * g.out_img);
        const int oy = q / g.Wo[0], ox = q - oy * g.Wo[0];
        const bool xr = 2 * ox + 1 < g.oW, yd = 2 * oy + 1 < g.oH;
        const uint2 z = make_uint2(0u, 0u);
        if (xr) *reinterpret_cast<uint2*>(Y + obase + g.cout + co) = z;
        if (yd) *reinterpret_cast<uint2*>(Y + obase + (long long)g.oW * g.cout + co) = z;
        if (xr && yd) *reinterpret_cast<uint2*>(Y + obase + (long long)(g.oW + 1) * g.cout + co) = z;
      }
    }
  }
}

// W[co][ky][kx][ci] -> Wd[ci][kh-1-ky][kw-1-kx][co]  (data-gradient weights for stride-1 convs)
__global__ void flip_transpose_kernel(const bf16_t* __restrict__ W, bf16_t* __restrict__ Wd, int cout, int kh, int kw,
                                      int cin) {
  // 32-bit index math (a weight tensor has < 2^31 elements; 64-bit division is emulated on CDNA)
  const int total = cout * kh * kw * cin;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < total; e += gridDim.x * blockDim.x) {
    int r = e;
    const int ci = r % cin; r /= cin;
    const int kx = r % kw; r /= kw;
    const int ky = r % kh;
    const int co = r / kh;
    Wd[((ci * kh + (kh - 1 - ky)) * kw + (kw - 1 - kx)) * cout + co] = W[e];
  }
}

template <int BCO, int BPIX, int WCO, int WPIX>
int launch_fwd(const bf16_t* X, const bf16_t* Wt, const float* bias, const bf16_t* R, const bf16_t* Mk, bf16_t* Y,
               const bf16_t* zpage, const ConvGeom& g, int relu, int accumulate, hipStream_t stream) {
  const int tiles_co = (g.cout + BCO - 1) / BCO;
  const long long tiles_m = (g.M + BPIX - 1) / BPIX;
  const long long nwg = tiles_co * tiles_m;
  if (nwg > 0x7fffffffLL) return -3;
  const size_t lds = 2 * (BCO + BPIX) * 128;
  auto kern = conv_fwd_kernel<BCO, BPIX, WCO, WPIX>;
  static bool attr_set = false;
  if (!attr_set) {
    hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr_set = true;
  }
  kern<<<(unsigned)nwg, WCO * WPIX * 64, lds, stream>>>(X, Wt, bias, R, Mk, Y, zpage, g, relu, accumulate, tiles_co);
  return (int)hipGetLastError();
}

}  // namespace

MXR_API int mxr_conv_geom_size() { return (int)sizeof(ConvGeom); }

// variant: 0 = 128co x 128pix (4 waves), 1 = 64co x 128pix (4 waves, small Cout), 2 = 256co x 128pix (8 waves)
// Mk (optional): output is zeroed where Mk <= 0 (fused relu backward of the producing layer).
MXR_API int mxr_conv_fwd(const void* X, const void* Wt, const float* bias, const void* R, const void* Mk, void* Y,
                         const void* zpage, const ConvGeom* g, int relu, int accumulate, int variant,
                         hipStream_t stream) {
  if (g->cin % 64 != 0 || g->cout % 4 != 0) return -1;
  if (g->nlev < 1 || g->nlev > MXR_MAXLEV) return -2;
  switch (variant) {
    case 1:
      return launch_fwd<64, 128, 2, 2>((const bf16_t*)X, (const bf16_t*)Wt, bias, (const bf16_t*)R, (const bf16_t*)Mk, (bf16_t*)Y,
                                       (const bf16_t*)zpage, *g, relu, accumulate, stream);
    case 2:
      return launch_fwd<256, 128, 4, 2>((const bf16_t*)X, (const bf16_t*)Wt, bias, (const bf16_t*)R, (const bf16_t*)Mk, (bf16_t*)Y,
                                        (const bf16_t*)zpage, *g, relu, accumulate, stream);
    default:
      return launch_fwd<128, 128, 2, 2>((const bf16_t*)X, (const bf16_t*)Wt, bias, (const bf16_t*)R, (const bf16_t*)Mk, (bf16_t*)Y,
                                        (const bf16_t*)zpage, *g, relu, accumulate, stream);
  }
}

// Batched flip-transpose of every conv weight in one launch (the data-gradient weights of a whole
// model, refreshed once per optimizer step).  Block = one 32 x 32 (co x ci) tile of one tap of one
// tensor: rows of ci are read and rows of co written as 64-B segments through an LDS transpose.
struct FlipSeg {
  long long src, dst;   // element offsets
  int cout, kh, kw, cin;
};

__global__ __launch_bounds__(256) void flip_batch_kernel(const bf16_t* __restrict__ src, bf16_t* __restrict__ dst,
                                                         const FlipSeg* __restrict__ segs,
                                                         const int4* __restrict__ tiles) {
  __shared__ bf16_t t[32][33];
  const int4 tl = tiles[blockIdx.x];   // (seg, tap, co0, ci0)
  const FlipSeg s = segs[tl.x];
  const int tap = tl.y, co0 = tl.z, ci0 = tl.w;
  const int taps = s.kh * s.kw;
  const int ky = tap / s.kw, kx = tap - ky * s.kw;
  const int ftap = (s.kh - 1 - ky) * s.kw + (s.kw - 1 - kx);
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;   // 32 x 8
#pragma unroll
  for (int r = ty; r < 32; r += 8) {
    const int co = co0 + r, ci = ci0 + tx;
    t[r][tx] = (co < s.cout && ci < s.cin) ? src[s.src + ((long long)co * taps + tap) * s.cin + ci] : (bf16_t)0;
  }
  __syncthreads();
#pragma unroll
  for (int r = ty; r < 32; r += 8) {
    const int ci = ci0 + r, co = co0 + tx;
    if (ci < s.cin && co < s.cout) dst[s.dst + ((long long)ci * taps + ftap) * s.cout + co] = t[tx][r];
  }
}

MXR_API int mxr_flip_batch(const void* src, void* dst, const void* segs, const void* tiles, int ntiles,
                           hipStream_t stream) {
  if (ntiles <= 0) return 0;
  flip_batch_kernel<<<ntiles, 256, 0, stream>>>((const bf16_t*)src, (bf16_t*)dst, (const FlipSeg*)segs,
                                                (const int4*)tiles);
  return (int)hipGetLastError();
}

MXR_API int mxr_flip_transpose(const void* W, void* Wd, int cout, int kh, int kw, int cin, hipStream_t stream) {
  const long long total = (long long)cout * kh * kw * cin;
  flip_transpose_kernel<<<mxr_grid(total, 256, 4096), 256, 0, stream>>>((const bf16_t*)W, (bf16_t*)Wd, cout, kh, kw, cin);
  return (int)hipGetLastError();
}
