"""Keras-semantics Adam with ``clipnorm`` over flat fp32 buffers.

Spec: ``keras.optimizers.adam(lr=1e-5, clipnorm=0.001)`` at ``/root/reference/train.py:104``
(SURVEY §2.8.7):

    g <- g * clipnorm / ||g||   if ||g|| >= clipnorm   (global L2 norm over ALL grads)
    t  = iterations + 1
    lr_t = lr * sqrt(1 - beta2^t) / (1 - beta1^t)
    m  = beta1 m + (1 - beta1) g
    v  = beta2 v + (1 - beta2) g^2
    p -= lr_t * m / (sqrt(v) + eps)          eps = K.epsilon() = 1e-7 (outside the bias fix)

The update runs as ONE fused multi-tensor HIP kernel over the flat buffers on the GPU
(``csrc/kernels/optim.hip``: gradient pre-scale (1/world, clip factor) + Adam + refresh of
the bf16 compute weights), and as the equivalent torch expression on the CPU.  The clip
factor and lr_t live on the device so a step never synchronises with the host.
"""
from __future__ import annotations

import math
from typing import Dict, Optional

import torch

from .flat import FlatParams


class KerasAdam:
    def __init__(self, flat: FlatParams, lr: float = 1e-5, beta_1: float = 0.9, beta_2: float = 0.999,
                 epsilon: float = 1e-7, decay: float = 0.0, clipnorm: Optional[float] = 0.001,
                 amsgrad: bool = False, backend: str = "auto"):
        if amsgrad:
            raise NotImplementedError("amsgrad is off in the reference optimizer")
        self.flat = flat
        self.lr = float(lr)
        self.initial_lr = float(lr)
        self.beta_1, self.beta_2, self.epsilon, self.decay = beta_1, beta_2, epsilon, decay
        self.clipnorm = clipnorm
        dev = flat.data.device
        self.m = torch.zeros_like(flat.data)
        self.v = torch.zeros_like(flat.data)
        self.iterations = 0                       # host mirror (the step count is deterministic)
        self.backend = backend
        self._dev = dev

    # -------------------------------------------------------------- keras-ish API
    def get_config(self) -> Dict:
        return {"lr": self.lr, "beta_1": self.beta_1, "beta_2": self.beta_2, "decay": self.decay,
                "epsilon": self.epsilon, "amsgrad": False, "clipnorm": self.clipnorm}

    def state_tensors(self):
        return {"m": self.m, "v": self.v}

    def _use_hip(self) -> bool:
        from ..ops import native
        if self.backend == "torch":
            return False
        return self.flat.data.is_cuda and native.available()

    # -------------------------------------------------------------- math
    def grad_norm(self, grad: Optional[torch.Tensor] = None) -> torch.Tensor:
        g = self.flat.grad if grad is None else grad
        if self._use_hip():
            from ..ops import native
            return native.l2norm(g)
        return torch.linalg.vector_norm(g.float())

    def norm_and_scale(self, norm_mul: float = 1.0, scale_mul: float = 1.0):
        """(norm * norm_mul, clip_factor(norm * norm_mul) * scale_mul) as 0-d device tensors; on the HIP
        path ONE fused reduction + finalize launch instead of the norm and five scalar torch ops."""
        if self._use_hip():
            from ..ops import native
            out = native.grad_norm_clip(self.flat.grad, norm_mul, float(self.clipnorm or 0.0), scale_mul)
            return out[0], out[1]
        norm = self.grad_norm() * norm_mul
        return norm, self.clip_factor(norm) * scale_mul

    def clip_factor(self, norm: torch.Tensor) -> torch.Tensor:
        if not self.clipnorm or self.clipnorm <= 0:
            return torch.ones((), device=norm.device)
        c = self.clipnorm
        return torch.where(norm >= c, c / norm.clamp_min(1e-30), torch.ones_like(norm))

    def lr_t(self, t: int) -> float:
        lr = self.lr
        if self.decay > 0:
            lr = lr * (1.0 / (1.0 + self.decay * (t - 1)))
        return lr * math.sqrt(1.0 - self.beta_2 ** t) / (1.0 - self.beta_1 ** t)

    def apply(self, grad_scale: torch.Tensor) -> None:
        """Adam step with ``g_eff = grad * grad_scale`` (grad_scale: 0-d device tensor)."""
        t = self.iterations + 1
        lr_t = self.lr_t(t)
        if self._use_hip():
            from ..ops import native
            lr = self.lr if self.decay <= 0 else self.lr * (1.0 / (1.0 + self.decay * (t - 1)))
            native.adam_step(self.flat, self.m, self.v, grad_scale, lr, self.iterations, self.beta_1, self.beta_2,
                             self.epsilon)
        else:
            g = self.flat.grad * grad_scale
            self.m.mul_(self.beta_1).add_(g, alpha=1 - self.beta_1)
            self.v.mul_(self.beta_2).addcmul_(g, g, value=1 - self.beta_2)
            self.flat.data.addcdiv_(self.m, self.v.sqrt().add_(self.epsilon), value=-lr_t)
        self.iterations = t

    def step(self, world_size: int = 1) -> torch.Tensor:
        """Local step (no communication): clip, then Adam.  Returns the pre-clip norm."""
        norm, scale = self.norm_and_scale(1.0, 1.0 / world_size)
        self.apply(scale)
        return norm

    def zero_grad(self) -> None:
        self.flat.zero_grad()
