// Per-element sigmoid-focal loss and logit gradient (keras-retinanet losses.focal, alpha 0.25 / gamma 2, Keras'
// probability clip as a logit clip -- /root/reference/train.py:99-102), shared by the fused loss
// kernel (losses.hip) and the classification final's focal epilogue (conv_hx32.hip / conv_hx32_f8.hip), so the
// two paths compute the same bits per element.
#pragma once

#include "common.h"

__device__ __forceinline__ void focal_elem(float x, bool y, float alpha, float gamma, bool g2, float lo, float hi,
                                           float& loss, float& grad) {
  const float ax = fabsf(x);
  const float e = __expf(-ax);
  const float r = 1.0f / (1.0f + e);
  const float p = x >= 0.f ? r : e * r;        // sigmoid(x)
  const float q = x >= 0.f ? e * r : r;        // 1 - sigmoid(x)
  const float xc = fminf(fmaxf(x, lo), hi);
  const bool inr = (x > lo) && (x < hi);
  // softplus(xc); inside the clip range exp(-|xc|) is the e above
  const float sp_pos = fmaxf(xc, 0.f) + __logf(1.0f + (inr ? e : __expf(-fabsf(xc))));
  if (y) {
    const float qg = g2 ? q * q : __powf(q, gamma);
    const float w = alpha * qg;
    const float bce = sp_pos - xc;             // softplus(-xc)
    const float dw = -alpha * gamma * p * qg;  // d/dx alpha (1-p)^g
    const float dbce = inr ? -q : 0.f;
    loss = w * bce;
    grad = dw * bce + w * dbce;
  } else {
    const float pg = g2 ? p * p : __powf(p, gamma);
    const float w = (1.f - alpha) * pg;
    const float bce = sp_pos;
    const float dw = (1.f - alpha) * gamma * pg * q;
    const float dbce = inr ? p : 0.f;
    loss = w * bce;
    grad = dw * bce + w * dbce;
  }
}

// focal_elem for y = 0 (the background class of an anchor: 79 of 80 elements of a positive row, all of a
// negative one).  A clipped logit's exp(-|xc|) is the constant e_clip of its side (passed in), so this costs
// one exp, one rcp and one log: the second exp and the y = 1 branch focal_elem evaluates (and discards) for
// every element are gone.
__device__ __forceinline__ void focal_neg(float x, float alpha, float gamma, bool g2, float lo, float hi,
                                          float e_lo, float e_hi, float& loss, float& grad) {
  const float ax = fabsf(x);
  // raw v_exp_f32 / v_log_f32 (base 2): the argument of the exp is <= 0 and that of the log in [1, 2], so
  // the denormal scaling __expf / __logf wrap around them (ldexp + compare + select each) is dead weight
  const float e = __builtin_amdgcn_exp2f(-ax * 1.44269504f);
  const float r = __builtin_amdgcn_rcpf(1.0f + e);
  const float p = x >= 0.f ? r : e * r;        // sigmoid(x)
  const float q = x >= 0.f ? e * r : r;
  const bool inr = (x > lo) && (x < hi);
  const float xc = fminf(fmaxf(x, lo), hi);
  const float ec = inr ? e : (x <= lo ? e_lo : e_hi);
  const float sp_pos = fmaxf(xc, 0.f) + __builtin_amdgcn_logf(1.0f + ec) * 0.693147181f;
  const float pg = g2 ? p * p : __powf(p, gamma);
  const float w = (1.f - alpha) * pg;
  const float dw = (1.f - alpha) * gamma * pg * q;
  loss = w * sp_pos;
  grad = dw * sp_pos + (inr ? w * p : 0.f);
}

// focal_neg for gamma = 2 and a logit inside the clip range (lo < x < hi): xc = x, so the log
// reuses 1 + e, the clip selects and the (always-true) BCE-gradient mask go, and the weight folds into
// loss = c_loss p^2 sp, grad = c_grad p^2 (2 q sp + p)  (sp = softplus(x) = the BCE of y = 0; c_grad
// carries the 1 / #positives scale).  ~18 VALU operations per logit against ~45 for focal_neg.
__device__ __forceinline__ void focal_neg_g2_inr(float x, float c_loss, float c_grad, float& loss, float& grad) {
  const float e = __builtin_amdgcn_exp2f(-fabsf(x) * 1.44269504f);
  const float d = 1.0f + e;
  const float r = __builtin_amdgcn_rcpf(d);
  const float er = e * r;
  const bool pos = x >= 0.f;
  const float p = pos ? r : er;
  const float q = pos ? er : r;
  const float sp = (pos ? x : 0.f) + __builtin_amdgcn_logf(d) * 0.693147181f;
  const float p2 = p * p;
  loss = c_loss * p2 * sp;
  grad = c_grad * p2 * fmaf(q, sp + sp, p);
}

// One 8-logit chunk of an anchor row's 80 classes for gamma = 2 (focal_bf16_kernel's G2 body): the loss sum of the
// chunk and the gradients gv (already scaled by inv = 1 / #positives).  lb = the positive class's index inside the
// chunk (0..7), or anything else when the chunk holds none.
__device__ __forceinline__ float focal8_g2(const float (&x)[8], int lb, float alpha, float gamma, float lo, float hi,
                                          float e_lo, float e_hi, float inv, float (&gv)[8]) {
  bool oor = false;
  float accv = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    float l;
    oor |= !(x[j] > lo && x[j] < hi);
    focal_neg_g2_inr(x[j], 1.f - alpha, (1.f - alpha) * inv, l, gv[j]);
    accv += l;
  }
  if (oor) {
    accv = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float l, g;
      focal_neg(x[j], alpha, gamma, true, lo, hi, e_lo, e_hi, l, g);
      accv += l;
      gv[j] = g * inv;
    }
  }
  if (lb >= 0 && lb < 8) {                        // rare: one element takes the y = 1 branch
    float xl = x[0];
#pragma unroll
    for (int j = 1; j < 8; ++j) xl = j == lb ? x[j] : xl;
    float ln, gn, l, g;
    focal_neg(xl, alpha, gamma, true, lo, hi, e_lo, e_hi, ln, gn);
    focal_elem(xl, true, alpha, gamma, true, lo, hi, l, g);
    accv += l - ln;
#pragma unroll
    for (int j = 0; j < 8; ++j) gv[j] = j == lb ? g * inv : gv[j];
  }
  return accv;
}

// the classification final's fused focal epilogue (conv_hx32 / conv_hx32_f8 FOC forms): per anchor row
// (pixel * A + anchor) its state (-1 ignore / 0 negative / 1 positive) and label, the #positives, the padded
// gradient rows dpad[pixel][ld] (anchor a's C logits at a * C), one loss partial per block
struct FocalArgs {
  const int8_t* state;
  const int32_t* label;
  const int* npos;
  bf16_t* dpad;
  float* partials;
  int ld, A;
  float alpha, gamma, lo, hi;
};
