// FP8 (OCP e4m3fn) quantisation for the fp8 convolution path (BASELINE config 5: fp8 weights and
// activations on the CDNA4 fp8 MFMA).  Per-tensor scaling for activations, per-output-channel for
// weights; the scales stay on the device (no host round trip):
//
//   amax  = max |x|                                  (mxr_fp8_amax: block max + atomicMax on the bits)
//   q     = sat(x * 448 / amax) as e4m3fn             (mxr_fp8_quant: reads amax from device memory)
//   inv   = amax / 448                                (written for the conv epilogue: y = acc * inv_x * inv_w)
//
// gfx950 converts with v_cvt_pk_fp8_f32 (OCP encoding on CDNA4); inputs are clamped to +-448 first
// so nothing overflows to NaN.
#include <algorithm>

#include "common.h"

namespace {

constexpr float FP8_MAX = 448.f;
constexpr float BF8_MAX = 57344.f;

__device__ __forceinline__ uint32_t pack4_fp8(float a, float b, float c, float d) {
  a = fminf(fmaxf(a, -FP8_MAX), FP8_MAX);
  b = fminf(fmaxf(b, -FP8_MAX), FP8_MAX);
  c = fminf(fmaxf(c, -FP8_MAX), FP8_MAX);
  d = fminf(fmaxf(d, -FP8_MAX), FP8_MAX);
  int v = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
  v = __builtin_amdgcn_cvt_pk_fp8_f32(c, d, v, true);
  return (uint32_t)v;
}

__device__ __forceinline__ float block_max(float v) {
  __shared__ float red[16];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  if (threadIdx.x < 64) {
    v = threadIdx.x < (blockDim.x >> 6) ? red[threadIdx.x] : 0.f;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  }
  return v;   // valid in wave 0
}

// n % 8 == 0; 8 bf16 per thread-iteration
__global__ __launch_bounds__(256) void amax_kernel(const bf16_t* __restrict__ x, long long n8, float* __restrict__ amax) {
  float m = 0.f;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n8; i += (long long)gridDim.x * blockDim.x) {
    const uint4 r = reinterpret_cast<const uint4*>(x)[i];
    const uint32_t w[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      m = fmaxf(m, fabsf(bf2f((bf16_t)(w[t] & 0xffff))));
      m = fmaxf(m, fabsf(bf2f((bf16_t)(w[t] >> 16))));
    }
  }
  m = block_max(m);
  if (threadIdx.x == 0) atomicMax(reinterpret_cast<int*>(amax), __float_as_int(m));   // m >= 0: int order
}

__device__ __forceinline__ uint32_t pack4_bf8(float a, float b, float c, float d) {
  a = fminf(fmaxf(a, -BF8_MAX), BF8_MAX);
  b = fminf(fmaxf(b, -BF8_MAX), BF8_MAX);
  c = fminf(fmaxf(c, -BF8_MAX), BF8_MAX);
  d = fminf(fmaxf(d, -BF8_MAX), BF8_MAX);
  int v = __builtin_amdgcn_cvt_pk_bf8_f32(a, b, 0, false);
  v = __builtin_amdgcn_cvt_pk_bf8_f32(c, d, v, true);
  return (uint32_t)v;
}

// 16 elements per thread-iteration (32 B in, 16 B out); BF8: e5m2 (gradients) instead of e4m3
template <int BF8>
__global__ __launch_bounds__(256) void quant_kernel(const bf16_t* __restrict__ x, long long n16, uint8_t* __restrict__ q,
                                                    const float* __restrict__ amax, float* __restrict__ inv_out) {
  constexpr float QMAX = BF8 ? BF8_MAX : FP8_MAX;
  const float a = fmaxf(*amax, 1e-12f);
  const float s = QMAX / a;
  if (inv_out && blockIdx.x == 0 && threadIdx.x == 0) *inv_out = a / QMAX;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n16; i += (long long)gridDim.x * blockDim.x) {
    const uint4 r0 = reinterpret_cast<const uint4*>(x)[2 * i];
    const uint4 r1 = reinterpret_cast<const uint4*>(x)[2 * i + 1];
    const uint32_t w[8] = {r0.x, r0.y, r0.z, r0.w, r1.x, r1.y, r1.z, r1.w};
    uint32_t o[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const float f0 = bf2f((bf16_t)(w[2 * t] & 0xffff)) * s, f1 = bf2f((bf16_t)(w[2 * t] >> 16)) * s;
      const float f2 = bf2f((bf16_t)(w[2 * t + 1] & 0xffff)) * s, f3 = bf2f((bf16_t)(w[2 * t + 1] >> 16)) * s;
      o[t] = BF8 ? pack4_bf8(f0, f1, f2, f3) : pack4_fp8(f0, f1, f2, f3);
    }
    reinterpret_cast<uint4*>(q)[i] = uint4{o[0], o[1], o[2], o[3]};
  }
}

// One pass with delayed scaling (the fused conv epilogues' AmaxState protocol, conv_hx32_f8.hip): the scale
// comes from the previous step's amax (amax3[(phase + 2) % 3], times margin), this tensor's amax is max-reduced
// into amax3[phase] and block 0 clears amax3[(phase + 1) % 3] for the next step.  One read of x instead of
// mxr_fp8_amax + quant_kernel's two.
template <int BF8>
__global__ __launch_bounds__(256) void quant_delayed_kernel(const bf16_t* __restrict__ x, long long n16,
                                                            uint8_t* __restrict__ q, float* __restrict__ amax3,
                                                            int phase, float margin, float* __restrict__ inv_out) {
  constexpr float QMAX = BF8 ? BF8_MAX : FP8_MAX;
  const float prev = fmaxf(amax3[(phase + 2) % 3], 1e-12f);
  const float s = QMAX / (margin * prev);
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    amax3[(phase + 1) % 3] = 0.f;
    if (inv_out) *inv_out = margin * prev / QMAX;
  }
  float m = 0.f;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n16; i += (long long)gridDim.x * blockDim.x) {
    const uint4 r0 = reinterpret_cast<const uint4*>(x)[2 * i];
    const uint4 r1 = reinterpret_cast<const uint4*>(x)[2 * i + 1];
    const uint32_t w[8] = {r0.x, r0.y, r0.z, r0.w, r1.x, r1.y, r1.z, r1.w};
    uint32_t o[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const float f0 = bf2f((bf16_t)(w[2 * t] & 0xffff)), f1 = bf2f((bf16_t)(w[2 * t] >> 16));
      const float f2 = bf2f((bf16_t)(w[2 * t + 1] & 0xffff)), f3 = bf2f((bf16_t)(w[2 * t + 1] >> 16));
      m = fmaxf(m, fmaxf(fmaxf(fabsf(f0), fabsf(f1)), fmaxf(fabsf(f2), fabsf(f3))));
      o[t] = BF8 ? pack4_bf8(f0 * s, f1 * s, f2 * s, f3 * s) : pack4_fp8(f0 * s, f1 * s, f2 * s, f3 * s);
    }
    reinterpret_cast<uint4*>(q)[i] = uint4{o[0], o[1], o[2], o[3]};
  }
  m = block_max(m);
  if (threadIdx.x == 0) atomicMax(reinterpret_cast<int*>(amax3 + phase), __float_as_int(m));   // m >= 0: int order
}

// one block per row (output channel): per-row amax, then quantise the row; K % 16 == 0
__global__ __launch_bounds__(256) void quant_rows_kernel(const bf16_t* __restrict__ w, int K, uint8_t* __restrict__ q,
                                                         float* __restrict__ inv) {
  const bf16_t* row = w + (long long)blockIdx.x * K;
  float m = 0.f;
  for (int k = threadIdx.x * 8; k < K; k += blockDim.x * 8) {
    const uint4 r = *reinterpret_cast<const uint4*>(row + k);
    const uint32_t v[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      m = fmaxf(m, fabsf(bf2f((bf16_t)(v[t] & 0xffff))));
      m = fmaxf(m, fabsf(bf2f((bf16_t)(v[t] >> 16))));
    }
  }
  __shared__ float rowmax;
  m = block_max(m);
  if (threadIdx.x == 0) rowmax = fmaxf(m, 1e-12f);
  __syncthreads();
  const float a = rowmax, s = FP8_MAX / a;
  if (threadIdx.x == 0) inv[blockIdx.x] = a / FP8_MAX;
  uint8_t* qr = q + (long long)blockIdx.x * K;
  for (int k = threadIdx.x * 16; k < K; k += blockDim.x * 16) {
    const uint4 r0 = *reinterpret_cast<const uint4*>(row + k);
    const uint4 r1 = *reinterpret_cast<const uint4*>(row + k + 8);
    const uint32_t v[8] = {r0.x, r0.y, r0.z, r0.w, r1.x, r1.y, r1.z, r1.w};
    uint32_t o[4];
#pragma unroll
    for (int t = 0; t < 4; ++t)
      o[t] = pack4_fp8(bf2f((bf16_t)(v[2 * t] & 0xffff)) * s, bf2f((bf16_t)(v[2 * t] >> 16)) * s,
                       bf2f((bf16_t)(v[2 * t + 1] & 0xffff)) * s, bf2f((bf16_t)(v[2 * t + 1] >> 16)) * s);
    *reinterpret_cast<uint4*>(qr + k) = uint4{o[0], o[1], o[2], o[3]};
  }
}

// quant_rows_kernel with the bytes stored straight in conv_hx32_f8's packed weight layout
// ([tap][cin / 64][plane][cout][32 B], 16-B half h of plane p at ((((tap nch + c) 2 + p) cout + co) 2 + h) 16):
// one launch per weight instead of a quantisation and a pack pass.  Row = output channel, K = 9 cin.
__device__ __forceinline__ void quant_row_hx8(const bf16_t* __restrict__ w, int cout, int cin, int co,
                                              uint8_t* __restrict__ qp, float* __restrict__ inv) {
  const int K = 9 * cin, nch = cin >> 6;
  const bf16_t* row = w + (long long)co * K;
  float m = 0.f;
  for (int k = threadIdx.x * 8; k < K; k += blockDim.x * 8) {
    const uint4 r = *reinterpret_cast<const uint4*>(row + k);
    const uint32_t v[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      m = fmaxf(m, fabsf(bf2f((bf16_t)(v[t] & 0xffff))));
      m = fmaxf(m, fabsf(bf2f((bf16_t)(v[t] >> 16))));
    }
  }
  __shared__ float rowmax;
  m = block_max(m);
  if (threadIdx.x == 0) rowmax = fmaxf(m, 1e-12f);
  __syncthreads();
  const float a = rowmax, s = FP8_MAX / a;
  if (threadIdx.x == 0) inv[co] = a / FP8_MAX;
  for (int k = threadIdx.x * 16; k < K; k += blockDim.x * 16) {
    const uint4 r0 = *reinterpret_cast<const uint4*>(row + k);
    const uint4 r1 = *reinterpret_cast<const uint4*>(row + k + 8);
    const uint32_t v[8] = {r0.x, r0.y, r0.z, r0.w, r1.x, r1.y, r1.z, r1.w};
    uint32_t o[4];
#pragma unroll
    for (int t = 0; t < 4; ++t)
      o[t] = pack4_fp8(bf2f((bf16_t)(v[2 * t] & 0xffff)) * s, bf2f((bf16_t)(v[2 * t] >> 16)) * s,
                       bf2f((bf16_t)(v[2 * t + 1] & 0xffff)) * s, bf2f((bf16_t)(v[2 * t + 1] >> 16)) * s);
    const int tap = k / cin, e = k - tap * cin;
    const int c = e >> 6, p = (e >> 5) & 1, h = (e >> 4) & 1;
    const long long unit = ((((long long)tap * nch + c) * 2 + p) * cout + co) * 2 + h;
    *reinterpret_cast<uint4*>(qp + unit * 16) = uint4{o[0], o[1], o[2], o[3]};
  }
}

__global__ __launch_bounds__(256) void quant_rows_hx8_kernel(const bf16_t* __restrict__ w, int cout, int cin,
                                                             uint8_t* __restrict__ qp, float* __restrict__ inv) {
  quant_row_hx8(w, cout, cin, blockIdx.x, qp, inv);
}

// several weights in one launch (the fp8 head layers' forward and flipped data-gradient copies, once per optimizer
// step: 18 launches of ~11 us, latency-bound at one row per block, become one)
struct Q8Seg {
  const bf16_t* src;
  uint8_t* dst;
  float* inv;
  int cout, cin, row0, pad;
};

__global__ __launch_bounds__(256) void quant_rows_hx8_batch_kernel(const Q8Seg* __restrict__ segs, int nseg) {
  const int b = blockIdx.x;
  int i = 0;
  while (i + 1 < nseg && segs[i + 1].row0 <= b) ++i;
  const Q8Seg sg = segs[i];
  quant_row_hx8(sg.src, sg.cout, sg.cin, b - sg.row0, sg.dst, sg.inv);
}

int grid_for(long long n, int per_thread) {
  const long long g = (n / per_thread + 255) / 256;
  return (int)std::min<long long>(std::max<long long>(g, 1), 4096);
}

}  // namespace

// amax (float, device) must be zeroed by the caller unless accumulating a running max
MXR_API int mxr_fp8_amax(const void* x, long long n, float* amax, hipStream_t stream) {
  if (n % 8) return -1;
  amax_kernel<<<grid_for(n, 8), 256, 0, stream>>>((const bf16_t*)x, n / 8, amax);
  return (int)hipGetLastError();
}

MXR_API int mxr_fp8_quant(const void* x, long long n, void* q, const float* amax, float* inv_out, hipStream_t stream) {
  if (n % 16) return -1;
  quant_kernel<0><<<grid_for(n, 16), 256, 0, stream>>>((const bf16_t*)x, n / 16, (uint8_t*)q, amax, inv_out);
  return (int)hipGetLastError();
}

// e5m2 ("bf8") per-tensor quantisation of gradients: q = sat(x * 57344 / amax), inv = amax / 57344
MXR_API int mxr_bf8_quant(const void* x, long long n, void* q, const float* amax, float* inv_out, hipStream_t stream) {
  if (n % 16) return -1;
  quant_kernel<1><<<grid_for(n, 16), 256, 0, stream>>>((const bf16_t*)x, n / 16, (uint8_t*)q, amax, inv_out);
  return (int)hipGetLastError();
}

// delayed-scaling quantisation in one pass (quant_delayed_kernel): bf8 = 1 -> e5m2, 0 -> e4m3; phase 0..2
MXR_API int mxr_quant_delayed(const void* x, long long n, void* q, float* amax3, int phase, float margin,
                              float* inv_out, int bf8, hipStream_t stream) {
  if (n % 16 || phase < 0 || phase > 2 || !(margin > 0.f)) return -1;
  if (bf8)
    quant_delayed_kernel<1><<<grid_for(n, 16), 256, 0, stream>>>((const bf16_t*)x, n / 16, (uint8_t*)q, amax3, phase,
                                                                  margin, inv_out);
  else
    quant_delayed_kernel<0><<<grid_for(n, 16), 256, 0, stream>>>((const bf16_t*)x, n / 16, (uint8_t*)q, amax3, phase,
                                                                  margin, inv_out);
  return (int)hipGetLastError();
}

MXR_API int mxr_fp8_quant_rows(const void* w, int rows, int K, void* q, float* inv, hipStream_t stream) {
  if (K % 16) return -1;
  quant_rows_kernel<<<rows, 256, 0, stream>>>((const bf16_t*)w, K, (uint8_t*)q, inv);
  return (int)hipGetLastError();
}

// conv_hx32_f8's weights in one pass: per-row e4m3 quantisation (inv[co] = amax / 448) written in its packed
// layout (mxr_hx8_pack_weights of mxr_fp8_quant_rows, bit for bit).  cin % 64 == 0.
// segs: nseg device records {src, dst, inv, cout, cin, row0, pad} (row0 = the segment's first row in the
// concatenation, ascending; rows = total rows), each as mxr_hx8_quant_pack (cin % 64 == 0, checked by the caller)
MXR_API int mxr_hx8_quant_pack_batch(const void* segs, int nseg, int rows, hipStream_t stream) {
  if (nseg < 1 || rows < 1) return -1;
  quant_rows_hx8_batch_kernel<<<rows, 256, 0, stream>>>((const Q8Seg*)segs, nseg);
  return (int)hipGetLastError();
}

MXR_API int mxr_hx8_quant_pack(const void* w, int cout, int cin, void* qp, float* inv, hipStream_t stream) {
  if (cin % 64 != 0 || cout < 1) return -1;
  quant_rows_hx8_kernel<<<cout, 256, 0, stream>>>((const bf16_t*)w, cout, cin, (uint8_t*)qp, inv);
  return (int)hipGetLastError();
}
