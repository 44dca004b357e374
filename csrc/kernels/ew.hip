// Fused NHWC elementwise epilogues used around library (MIOpen) convolutions and in backward.
//
//   bias_res_act : y = act(y + bias[c] (+ r))   -- frozen-BN shift / conv bias + residual + ReLU in
//                  ONE pass (instead of three torch kernels) when a conv runs on MIOpen;
//   relu_bwd     : dx = dy * (y > 0)            -- one pass (torch needs compare + masked_fill);
//   s2_shuffle   : the sub-pixel phases of a stride-2 data gradient -> dX (+ mask, accumulate).
// 8 bf16 channels (16 B) per thread; C must be a multiple of 8.
#include "common.h"
#include "fp8_common.h"

namespace {
constexpr int kBlock = 256;

__global__ __launch_bounds__(kBlock) void bias_res_act_kernel(bf16_t* __restrict__ y, const float* __restrict__ bias,
                                                              const bf16_t* __restrict__ r, long long nvec, int CV,
                                                              int relu) {
  for (long long i = blockIdx.x * (long long)kBlock + threadIdx.x; i < nvec; i += (long long)gridDim.x * kBlock) {
    const int cv = (int)(i % CV);
    uint4 v = reinterpret_cast<uint4*>(y)[i];
    uint32_t* w = &v.x;
    uint4 rv = make_uint4(0, 0, 0, 0);
    if (r) rv = reinterpret_cast<const uint4*>(r)[i];
    const uint32_t* rw = &rv.x;
    float b[8];
    if (bias) {
      const float4 b0 = reinterpret_cast<const float4*>(bias)[2 * cv];
      const float4 b1 = reinterpret_cast<const float4*>(bias)[2 * cv + 1];
      b[0] = b0.x; b[1] = b0.y; b[2] = b0.z; b[3] = b0.w; b[4] = b1.x; b[5] = b1.y; b[6] = b1.z; b[7] = b1.w;
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) b[j] = 0.f;
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      float lo = bf2f((bf16_t)(w[t] & 0xffff)) + b[2 * t];
      float hi = bf2f((bf16_t)(w[t] >> 16)) + b[2 * t + 1];
      if (r) {
        lo += bf2f((bf16_t)(rw[t] & 0xffff));
        hi += bf2f((bf16_t)(rw[t] >> 16));
      }
      if (relu) {
        lo = fmaxf(lo, 0.f);
        hi = fmaxf(hi, 0.f);
      }
      w[t] = (uint32_t)f2bf(lo) | ((uint32_t)f2bf(hi) << 16);
    }
    reinterpret_cast<uint4*>(y)[i] = v;
  }
}

__global__ __launch_bounds__(kBlock) void relu_bwd_kernel(const bf16_t* dy, const bf16_t* __restrict__ y,
                                                          bf16_t* dx, long long nvec) {
  for (long long i = blockIdx.x * (long long)kBlock + threadIdx.x; i < nvec; i += (long long)gridDim.x * kBlock) {
    uint4 g = reinterpret_cast<const uint4*>(dy)[i];
    const uint4 v = reinterpret_cast<const uint4*>(y)[i];
    uint32_t* gw = &g.x;
    const uint32_t* vw = &v.x;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      // bf16 > 0  <=>  sign bit clear and value != +0 (NaN never occurs after a ReLU output)
      const uint32_t lo = vw[t] & 0xffff, hi = vw[t] >> 16;
      const uint32_t mlo = (!(lo & 0x8000) && lo) ? 0xffffu : 0u;
      const uint32_t mhi = (!(hi & 0x8000) && hi) ? 0xffff0000u : 0u;
      gw[t] &= (mlo | mhi);
    }
    reinterpret_cast<uint4*>(dx)[i] = g;
  }
}
}  // namespace

MXR_API int mxr_bias_res_act(void* y, const float* bias, const void* r, long long n, int C, int relu,
                             hipStream_t stream) {
  if (C % 8 || n % 8) return -1;
  const long long nvec = n / 8;
  bias_res_act_kernel<<<mxr_grid(nvec, kBlock, 16384), kBlock, 0, stream>>>((bf16_t*)y, bias, (const bf16_t*)r, nvec,
                                                                            C / 8, relu);
  return (int)hipGetLastError();
}

// Stride-2 data-gradient pixel shuffle: y4 [N, Hp, Wp, 4, C] holds the four sub-pixel phases of dX (phase
// 2 py + px at (a, b) is dX[2a + py, 2b + px]); writes dX [N, H, W, C] with the relu-gradient mask and
// optional accumulation.  8 channels (16 B) per thread; C % 8 == 0.
__global__ __launch_bounds__(kBlock) void s2_shuffle_kernel(const bf16_t* __restrict__ y4, bf16_t* __restrict__ dx,
                                                            const bf16_t* __restrict__ mask, int accumulate, int N,
                                                            int H, int W, int Hp, int Wp, int C) {
  const int CV = C >> 3;
  const long long total = (long long)N * H * W * CV;
  for (long long i = blockIdx.x * (long long)kBlock + threadIdx.x; i < total; i += (long long)gridDim.x * kBlock) {
    const int cv = (int)(i % CV);
    const long long pix = i / CV;
    const int x = (int)(pix % W);
    const long long t = pix / W;
    const int y = (int)(t % H);
    const int n = (int)(t / H);
    const int ph = 2 * (y & 1) + (x & 1);
    const long long src = ((((long long)n * Hp + (y >> 1)) * Wp + (x >> 1)) * 4 + ph) * C + cv * 8;
    const uint4 v = *reinterpret_cast<const uint4*>(y4 + src);
    uint4 a = make_uint4(0u, 0u, 0u, 0u), m = make_uint4(0u, 0u, 0u, 0u);
    if (accumulate) a = reinterpret_cast<const uint4*>(dx)[i];
    if (mask) m = reinterpret_cast<const uint4*>(mask)[i];
    const uint32_t vw[4] = {v.x, v.y, v.z, v.w}, aw[4] = {a.x, a.y, a.z, a.w}, mw[4] = {m.x, m.y, m.z, m.w};
    uint32_t o[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float lo = bf2f((bf16_t)(vw[q] & 0xffff)), hi = bf2f((bf16_t)(vw[q] >> 16));
      if (accumulate) {
        lo += bf2f((bf16_t)(aw[q] & 0xffff));
        hi += bf2f((bf16_t)(aw[q] >> 16));
      }
      if (mask) {
        if (!(bf2f((bf16_t)(mw[q] & 0xffff)) > 0.f)) lo = 0.f;
        if (!(bf2f((bf16_t)(mw[q] >> 16)) > 0.f)) hi = 0.f;
      }
      o[q] = (uint32_t)f2bf(lo) | ((uint32_t)f2bf(hi) << 16);
    }
    reinterpret_cast<uint4*>(dx)[i] = make_uint4(o[0], o[1], o[2], o[3]);
  }
}

MXR_API int mxr_s2_shuffle(const void* y4, void* dx, const void* mask, int accumulate, int N, int H, int W, int Hp,
                           int Wp, int C, hipStream_t stream) {
  if (C % 8 || Hp * 2 < H || Wp * 2 < W) return -1;
  const long long nvec = (long long)N * H * W * (C / 8);
  s2_shuffle_kernel<<<mxr_grid(nvec, kBlock, 16384), kBlock, 0, stream>>>((const bf16_t*)y4, (bf16_t*)dx,
                                                                          (const bf16_t*)mask, accumulate, N, H, W,
                                                                          Hp, Wp, C);
  return (int)hipGetLastError();
}

// Phase-stacked weights of the stride-2 data gradient (ops/native_conv._s2_stacked_weights):
// w4[p * cin + ci][slot][co] = w[co][tap(p, slot)][ci], zero where tap(p, slot) < 0 (16 entries: 4 phases x 2 x 2
// window slots, tap = ky * 3 + kx of the OHWI 3x3 weights).
struct S2Taps {
  int tap[16];
};

__global__ __launch_bounds__(kBlock) void s2_stack_kernel(const bf16_t* __restrict__ w, bf16_t* __restrict__ w4,
                                                          int cin, int cout, S2Taps t) {
  const long long total = 16LL * cin * cout;
  for (long long i = blockIdx.x * (long long)kBlock + threadIdx.x; i < total; i += (long long)gridDim.x * kBlock) {
    const int co = (int)(i % cout);
    const long long r = i / cout;           // (p * cin + ci) * 4 + slot
    const int slot = (int)(r & 3);
    const long long pc = r >> 2;
    const int p = (int)(pc / cin), ci = (int)(pc - (long long)p * cin);
    int tap = t.tap[0];
#pragma unroll
    for (int k = 1; k < 16; ++k) tap = (k == p * 4 + slot) ? t.tap[k] : tap;
    w4[i] = tap < 0 ? (bf16_t)0 : w[((long long)co * 9 + tap) * cin + ci];
  }
}

MXR_API int mxr_s2_stack(const void* w, void* w4, int cin, int cout, const int* taps16, hipStream_t stream) {
  S2Taps t;
  for (int k = 0; k < 16; ++k) t.tap[k] = taps16[k];
  const long long total = 16LL * cin * cout;
  s2_stack_kernel<<<mxr_grid(total, kBlock, 16384), kBlock, 0, stream>>>((const bf16_t*)w, (bf16_t*)w4, cin, cout, t);
  return (int)hipGetLastError();
}

// The same stacked weights from the flip-transposed copy wd[ci][ky][kx][co] (ComputeWeights' batched flip, already
// in hand for the data gradients): w4 row (p * cin + ci, slot) = wd row (ci, 8 - tap) -- a contiguous cout-wide row
// copy per output row, 16 B per thread (the gather above reads w with a 9 * cin stride: 60 us for P6's weights).
__global__ __launch_bounds__(kBlock) void s2_stack_flip_kernel(const uint4* __restrict__ wd, uint4* __restrict__ w4,
                                                               int cin, int cvec, S2Taps t) {
  const long long total = 16LL * cin * cvec;
  for (long long i = blockIdx.x * (long long)kBlock + threadIdx.x; i < total; i += (long long)gridDim.x * kBlock) {
    const int c = (int)(i % cvec);
    const long long r = i / cvec;           // (p * cin + ci) * 4 + slot
    const int slot = (int)(r & 3);
    const long long pc = r >> 2;
    const int p = (int)(pc / cin), ci = (int)(pc - (long long)p * cin);
    int tap = t.tap[0];
#pragma unroll
    for (int k = 1; k < 16; ++k) tap = (k == p * 4 + slot) ? t.tap[k] : tap;
    w4[i] = tap < 0 ? make_uint4(0u, 0u, 0u, 0u) : wd[((long long)ci * 9 + (8 - tap)) * cvec + c];
  }
}

MXR_API int mxr_s2_stack_flip(const void* wd, void* w4, int cin, int cout, const int* taps16, hipStream_t stream) {
  if (cout % 8) return -1;
  S2Taps t;
  for (int k = 0; k < 16; ++k) t.tap[k] = taps16[k];
  const int cvec = cout / 8;
  const long long total = 16LL * cin * cvec;
  s2_stack_flip_kernel<<<mxr_grid(total, kBlock, 16384), kBlock, 0, stream>>>((const uint4*)wd, (uint4*)w4, cin, cvec,
                                                                               t);
  return (int)hipGetLastError();
}

MXR_API int mxr_relu_bwd(const void* dy, const void* y, void* dx, long long n, hipStream_t stream) {
  if (n % 8) return -1;
  const long long nvec = n / 8;
  relu_bwd_kernel<<<mxr_grid(nvec, kBlock, 16384), kBlock, 0, stream>>>((const bf16_t*)dy, (const bf16_t*)y,
                                                                        (bf16_t*)dx, nvec);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------------------------------
// Packed pyramid <-> per-level tensors (the heads' [B, P, C] input, P = sum of the levels' h * w).
// One image's block of the packed tensor is the levels' [h_l * w_l * C] blocks back to back, so a 16-B
// chunk idx maps to image n = idx / per_img, level l by its offset inside the image (select chain over
// the statically indexed levels: no computed indexing into the kernel arguments) and the level tensor's
// chunk n * size_l + (r - off_l).  unpack = 0 gathers the levels into the packed tensor (forward,
// instead of torch.cat); unpack = 1 scatters the packed gradient into contiguous per-level gradients
// (backward: the FPN output convs otherwise copied each strided level slice with a generic
// TensorIterator kernel, ~0.7 ms per step for the four big levels).
namespace {
struct PyrLevels {
  uint4* ptr[5];
  int off[6];   // per-image chunk offset of level l (off[nlev] = per_img)
  int size[5];  // per-image chunks of level l
  int nlev;
};

__global__ __launch_bounds__(kBlock) void pyr_pack_kernel(uint4* __restrict__ packed, PyrLevels lv, int per_img,
                                                          long long total, int unpack) {
  for (long long idx = blockIdx.x * (long long)kBlock + threadIdx.x; idx < total;
       idx += (long long)gridDim.x * kBlock) {
    const int n = (int)(idx / per_img);
    const int r = (int)(idx - (long long)n * per_img);
    uint4* base = lv.ptr[0];
    int off = 0, size = lv.size[0];
#pragma unroll
    for (int t = 1; t < 5; ++t) {
      const bool in = t < lv.nlev && r >= lv.off[t];
      base = in ? lv.ptr[t] : base;
      off = in ? lv.off[t] : off;
      size = in ? lv.size[t] : size;
    }
    uint4* q = base + (long long)n * size + (r - off);
    if (unpack)
      *q = packed[idx];
    else
      packed[idx] = *q;
  }
}
// pack + the e4m3 copy of the packed features for the heads' fp8 first layers (delayed scaling, F8Out):
// Yq[i] = sat(x[i] * 448 / (margin * amax_prev)), this step's amax(|x|) max-reduced into amax3[phase]
__global__ __launch_bounds__(kBlock) void pyr_pack_f8_kernel(uint4* __restrict__ packed, PyrLevels lv, int per_img,
                                                             long long total, F8Out fo) {
  __shared__ float red[kBlock / 64];
  const float prev = fo.amax3[(fo.phase + 2) % 3];
  const float qs = prev > 0.f ? 448.f / (fo.margin * prev) : 0.f;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    fo.amax3[(fo.phase + 1) % 3] = 0.f;
    if (fo.inv_out) *fo.inv_out = fo.margin * prev / 448.f;
  }
  float tmax = 0.f;
  for (long long idx = blockIdx.x * (long long)kBlock + threadIdx.x; idx < total;
       idx += (long long)gridDim.x * kBlock) {
    const int n = (int)(idx / per_img);
    const int r = (int)(idx - (long long)n * per_img);
    uint4* base = lv.ptr[0];
    int off = 0, size = lv.size[0];
#pragma unroll
    for (int t = 1; t < 5; ++t) {
      const bool in = t < lv.nlev && r >= lv.off[t];
      base = in ? lv.ptr[t] : base;
      off = in ? lv.off[t] : off;
      size = in ? lv.size[t] : size;
    }
    const uint4 v = base[(long long)n * size + (r - off)];
    packed[idx] = v;
    const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
    float f[8];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      f[2 * e] = bf2f((bf16_t)(w4[e] & 0xffff));
      f[2 * e + 1] = bf2f((bf16_t)(w4[e] >> 16));
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) tmax = fmaxf(tmax, fabsf(f[e]));
    if (fo.Yq) {
      uint2 q;
      q.x = pack4_e4m3(f[0] * qs, f[1] * qs, f[2] * qs, f[3] * qs);
      q.y = pack4_e4m3(f[4] * qs, f[5] * qs, f[6] * qs, f[7] * qs);
      reinterpret_cast<uint2*>(fo.Yq)[idx] = q;
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) tmax = fmaxf(tmax, __shfl_xor(tmax, o));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = tmax;
  __syncthreads();
  if (threadIdx.x == 0) {
    float mx = red[0];
#pragma unroll
    for (int w = 1; w < kBlock / 64; ++w) mx = fmaxf(mx, red[w]);
    atomicMax(reinterpret_cast<int*>(fo.amax3 + fo.phase), __float_as_int(mx));
  }
}
}  // namespace

// the pack direction of mxr_pyr_pack plus the fused e4m3 copy (Yq may be null: only record the amax)
MXR_API int mxr_pyr_pack_f8(void* packed, void* const* levels, const int* hw, int nlev, int N, int C, void* Yq,
                            float* amax3, float* inv_out, int phase, float margin, hipStream_t stream) {
  if (nlev < 1 || nlev > 5 || C % 8 || amax3 == nullptr) return -1;
  PyrLevels lv;
  int off = 0;
  for (int l = 0; l < 5; ++l) {
    lv.ptr[l] = (uint4*)levels[l < nlev ? l : 0];
    lv.off[l] = off;
    lv.size[l] = l < nlev ? hw[l] * (C / 8) : 0;
    if (l < nlev) off += lv.size[l];
  }
  lv.off[5] = off;
  lv.nlev = nlev;
  const long long total = (long long)N * off;
  if (total >= (1LL << 31)) return -4;
  const F8Out fo{(uint8_t*)Yq, amax3, inv_out, phase % 3, margin};
  pyr_pack_f8_kernel<<<mxr_grid(total, kBlock, 16384), kBlock, 0, stream>>>((uint4*)packed, lv, off, total, fo);
  return (int)hipGetLastError();
}

// levels: nlev pointers to [N, h_l, w_l, C] bf16 tensors; hw: nlev pixel counts h_l * w_l.
MXR_API int mxr_pyr_pack(void* packed, void* const* levels, const int* hw, int nlev, int N, int C, int unpack,
                         hipStream_t stream) {
  if (nlev < 1 || nlev > 5 || C % 8) return -1;
  PyrLevels lv;
  int off = 0;
  for (int l = 0; l < 5; ++l) {
    lv.ptr[l] = (uint4*)levels[l < nlev ? l : 0];
    lv.off[l] = off;
    lv.size[l] = l < nlev ? hw[l] * (C / 8) : 0;
    if (l < nlev) off += lv.size[l];
  }
  lv.off[5] = off;
  lv.nlev = nlev;
  const long long total = (long long)N * off;
  if (total >= (1LL << 31)) return -4;
  pyr_pack_kernel<<<mxr_grid(total, kBlock, 16384), kBlock, 0, stream>>>((uint4*)packed, lv, off, total, unpack);
  return (int)hipGetLastError();
}

// A stream restricted to `num`/`den` of the device's CUs, the same share on every XCD (CU mask bit i enabled when
// (i / 8) % den < num: a whole multiple of the 8 XCDs per pattern period, whichever way the driver distributes the
// mask bits over the XCDs).  For the side-stream weight gradients (ops.side_stream, MXR_SIDE_CU_FRAC): the
// critical-path data gradients keep the remaining CUs to themselves.  Returns the stream handle, 0 on failure.
MXR_API void* mxr_stream_create_cumask(int num, int den, int priority) {
  int dev = 0, ncu = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0) return nullptr;
  if (den <= 0 || num <= 0 || num > den) return nullptr;
  const int words = (ncu + 31) / 32;
  uint32_t mask[64] = {0};
  if (words > 64) return nullptr;
  for (int i = 0; i < ncu; ++i)
    if ((i / 8) % den < num) mask[i / 32] |= 1u << (i % 32);
  hipStream_t s = nullptr;
  if (hipExtStreamCreateWithCUMask(&s, (uint32_t)words, mask) != hipSuccess) return nullptr;
  (void)priority;
  return s;
}
