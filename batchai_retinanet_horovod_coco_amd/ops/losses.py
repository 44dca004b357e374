"""Focal and smooth-L1 losses.

Behavioural spec: keras-retinanet ``losses.focal(alpha=0.25, gamma=2.0)`` and
``losses.smooth_l1(sigma=3.0)`` compiled at ``/root/reference/train.py:99-102``
(SURVEY §2.8.6).  Both are normalised by max(1, #positive anchors in the *local* batch).

* ``focal_keras`` / ``smooth_l1_keras`` take the reference's dense ``y_true`` tensors
  (labels or regression targets with the anchor state as last column) and probabilities
  -- a literal fp32 re-statement used as the test oracle.
* ``focal_loss`` / ``smooth_l1_loss`` are the training path: logits in, compact targets
  (state int8, label int32, regression f32).  On the GPU they dispatch to one fused HIP
  kernel (``csrc/kernels/losses.hip``) that writes the loss partial sums *and* dlogits in
  a single pass over the 16M-logit/image classification tensor; the torch fallback is
  used on the CPU.
"""
from __future__ import annotations

import math

import torch

KERAS_EPSILON = 1e-7
# Keras' binary_crossentropy clips probabilities to [eps, 1-eps] (fp32) and converts back
# to logits; in logit space that is a clamp to [LOGIT_LO, LOGIT_HI].  1-eps rounds to
# 0.99999988 in fp32, hence the asymmetric bounds.
_P_HI = float(torch.tensor(1.0 - KERAS_EPSILON, dtype=torch.float32))
LOGIT_LO = math.log(KERAS_EPSILON / (1.0 - KERAS_EPSILON))
LOGIT_HI = math.log(_P_HI / (1.0 - _P_HI))


def focal_keras(y_true: torch.Tensor, y_pred: torch.Tensor, alpha: float = 0.25, gamma: float = 2.0) -> torch.Tensor:
    """Reference focal loss.  y_true (B, A, C+1) labels + state column; y_pred (B, A, C) probs."""
    labels = y_true[..., :-1]
    state = y_true[..., -1]
    keep = state != -1
    labels = labels[keep]
    cls = y_pred[keep]
    alpha_f = torch.where(labels == 1, torch.full_like(labels, alpha), torch.full_like(labels, 1 - alpha))
    fw = torch.where(labels == 1, 1 - cls, cls)
    fw = alpha_f * fw ** gamma
    out = cls.clamp(KERAS_EPSILON, _P_HI)
    logit = torch.log(out / (1 - out))
    bce = torch.clamp(logit, min=0) - logit * labels + torch.log1p(torch.exp(-logit.abs()))
    normalizer = torch.clamp((state == 1).sum().to(y_pred.dtype), min=1.0)
    return (fw * bce).sum() / normalizer


def smooth_l1_keras(y_true: torch.Tensor, y_pred: torch.Tensor, sigma: float = 3.0) -> torch.Tensor:
    """Reference smooth-L1.  y_true (B, A, 5) targets + state column; y_pred (B, A, 4)."""
    s2 = sigma ** 2
    tgt = y_true[..., :4]
    state = y_true[..., 4]
    pos = state == 1
    d = (y_pred[pos] - tgt[pos]).abs()
    loss = torch.where(d < 1.0 / s2, 0.5 * s2 * d ** 2, d - 0.5 / s2)
    normalizer = torch.clamp(pos.sum().to(y_pred.dtype), min=1.0)
    return loss.sum() / normalizer


# ----------------------------------------------------------------------------------------
# training path (compact targets, logits)
# ----------------------------------------------------------------------------------------

def num_positives(state: torch.Tensor) -> torch.Tensor:
    return (state == 1).sum()


def _focal_torch(logits, state, label, alpha, gamma):
    x = logits.float()
    B, A, C = x.shape
    keep = (state != -1)
    pos = (state == 1)
    y = torch.zeros_like(x)
    y.scatter_(2, label.clamp(0, C - 1).long()[..., None], pos[..., None].to(x.dtype))
    p = torch.sigmoid(x)
    alpha_t = torch.where(y == 1, torch.full_like(x, alpha), torch.full_like(x, 1 - alpha))
    fw = alpha_t * torch.where(y == 1, 1 - p, p) ** gamma
    xc = x.clamp(LOGIT_LO, LOGIT_HI)
    bce = torch.where(y == 1, torch.nn.functional.softplus(-xc), torch.nn.functional.softplus(xc))
    loss = (fw * bce * keep[..., None].to(x.dtype)).sum()
    return loss / torch.clamp(pos.sum().to(x.dtype), min=1.0)


def _smooth_l1_torch(reg, reg_t, state, sigma):
    s2 = sigma ** 2
    pos = (state == 1)
    d = (reg.float() - reg_t.float()).abs()
    l = torch.where(d < 1.0 / s2, 0.5 * s2 * d * d, d - 0.5 / s2)
    l = (l * pos[..., None].to(l.dtype)).sum()
    return l / torch.clamp(pos.sum().to(l.dtype), min=1.0)


def focal_loss(logits: torch.Tensor, state: torch.Tensor, label: torch.Tensor,
               alpha: float = 0.25, gamma: float = 2.0, backend: str = "auto") -> torch.Tensor:
    """Focal loss on logits (B, A, C) with compact targets; returns a scalar fp32."""
    from . import native
    if backend == "auto":
        backend = "hip" if (logits.is_cuda and native.available()) else "torch"
    if backend == "hip":
        return native.FocalLossFn.apply(logits, state, label, alpha, gamma)
    return _focal_torch(logits, state, label, alpha, gamma)


def smooth_l1_loss(reg: torch.Tensor, reg_t: torch.Tensor, state: torch.Tensor,
                   sigma: float = 3.0, backend: str = "auto") -> torch.Tensor:
    """Smooth-L1 over positive anchors; reg/reg_t (B, A, 4)."""
    from . import native
    if backend == "auto":
        backend = "hip" if (reg.is_cuda and native.available()) else "torch"
    if backend == "hip":
        return native.SmoothL1Fn.apply(reg, reg_t, state, sigma)
    return _smooth_l1_torch(reg, reg_t, state, sigma)
