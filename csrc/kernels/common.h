// Shared helpers for the gfx950 (CDNA4) kernels of batchai_retinanet_horovod_coco_amd.
// Wave = 64 lanes; every block size is a multiple of 64.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define MXR_API extern "C" __attribute__((visibility("default")))

typedef uint16_t bf16_t;  // raw bf16 bits

__device__ __forceinline__ float bf2f(bf16_t h) { return __uint_as_float(((uint32_t)h) << 16); }

// Round-to-nearest-even f32 -> bf16 (NaN kept a NaN): gfx950's v_cvt_pk_bf16_f32.  (The integer
// rounding sequence with its NaN test compiled to a divergent branch per value: ~10 instructions and
// two exec-mask flips each, a large part of every conv epilogue.)
__device__ __forceinline__ bf16_t f2bf(float f) { return __builtin_bit_cast(bf16_t, (__bf16)f); }

template <typename T> struct Cvt;
template <> struct Cvt<float> {
  __device__ __forceinline__ static float to_f(float x) { return x; }
  __device__ __forceinline__ static float from_f(float x) { return x; }
};
template <> struct Cvt<bf16_t> {
  __device__ __forceinline__ static float to_f(bf16_t x) { return bf2f(x); }
  __device__ __forceinline__ static bf16_t from_f(float x) { return f2bf(x); }
};

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ int wave_sum_i(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Block-wide sum for blockDim.x <= 1024 (result valid in thread 0).
__device__ __forceinline__ float block_sum(float v, float* red /* >= 16 floats of LDS */) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float s = 0.f;
  if (threadIdx.x == 0) {
    const int nw = (blockDim.x + 63) >> 6;
    for (int i = 0; i < nw; ++i) s += red[i];
  }
  return s;
}

static inline int mxr_grid(long long n, int block, int cap = 8192) {
  long long g = (n + block - 1) / block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (int)g;
}
