// fp8 pieces shared by the fp8 convolution kernels (conv_pipe_f8.hip, conv_p8_f8.hip).
#pragma once
#include "common.h"

// Fused fp8 output for the NEXT fp8 conv (delayed scaling): Yq = sat(y * 448 / (margin * amax_prev)),
// amax_prev = amax3[(phase + 2) % 3] (the previous step's), this step's amax(|y|) is max-reduced into
// amax3[phase], amax3[(phase + 1) % 3] is cleared for the next step, inv_out = margin * amax_prev / 448.
// Yq == nullptr: only record the amax (first step of a layer: no previous amax yet).
struct F8Out {
  uint8_t* Yq;
  float* amax3;
  float* inv_out;
  int phase;
  float margin;
};

__device__ __forceinline__ uint32_t pack4_e4m3(float a, float b, float c, float d) {
  a = fminf(fmaxf(a, -448.f), 448.f);
  b = fminf(fmaxf(b, -448.f), 448.f);
  c = fminf(fmaxf(c, -448.f), 448.f);
  d = fminf(fmaxf(d, -448.f), 448.f);
  int v = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
  v = __builtin_amdgcn_cvt_pk_fp8_f32(c, d, v, true);
  return (uint32_t)v;
}


// e5m2 ("bf8") for gradients: largest finite value 57344
__device__ __forceinline__ uint32_t pack4_e5m2(float a, float b, float c, float d) {
  a = fminf(fmaxf(a, -57344.f), 57344.f);
  b = fminf(fmaxf(b, -57344.f), 57344.f);
  c = fminf(fmaxf(c, -57344.f), 57344.f);
  d = fminf(fmaxf(d, -57344.f), 57344.f);
  int v = __builtin_amdgcn_cvt_pk_bf8_f32(a, b, 0, false);
  v = __builtin_amdgcn_cvt_pk_bf8_f32(c, d, v, true);
  return (uint32_t)v;
}
