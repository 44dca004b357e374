"""Keras-named building blocks: Conv2D (OHWI weights, optional frozen BN folded in) and
FrozenBatchNormalization.

Keras layers of the reference model (keras-resnet / keras-retinanet, imported by
``/root/reference/train.py:41-46``) map 1:1 onto these modules; every module carries its
Keras layer name so checkpoints (``io/keras_h5.py``) and ``--weights`` by-name loading
(``train.py:75-78``) line up.  BatchNormalization is frozen in the reference model
(inference-mode statistics, non-trainable), so it is a per-channel affine that is folded
into the preceding convolution: ``conv(x, W * s) + (beta - mean * s)`` with
``s = gamma / sqrt(var + eps)``.
"""
from __future__ import annotations

import math
from typing import Optional, Sequence, Tuple, Union

import torch
import torch.nn as nn

from ..ops import conv as conv_ops


def he_normal_(t: torch.Tensor, fan_in: int, gen: Optional[torch.Generator] = None) -> torch.Tensor:
    """Keras he_normal: truncated normal (2 sigma), std = sqrt(2 / fan_in)."""
    std = math.sqrt(2.0 / fan_in)
    with torch.no_grad():
        nn.init.trunc_normal_(t, mean=0.0, std=std / 0.87962566103423978, a=-2 * std / 0.87962566103423978,
                              b=2 * std / 0.87962566103423978, generator=gen)
    return t


def glorot_uniform_(t: torch.Tensor, fan_in: int, fan_out: int, gen: Optional[torch.Generator] = None) -> torch.Tensor:
    limit = math.sqrt(6.0 / (fan_in + fan_out))
    with torch.no_grad():
        t.uniform_(-limit, limit, generator=gen)
    return t


def prior_probability_bias(probability: float = 0.01) -> float:
    """keras-retinanet ``initializers.PriorProbability``: -log((1 - p) / p)."""
    return -math.log((1 - probability) / probability)


class FrozenBatchNormalization(nn.Module):
    """Inference-mode BN with non-trainable gamma/beta/moving stats (eps 1e-5)."""

    def __init__(self, name: str, channels: int, eps: float = 1e-5):
        super().__init__()
        self.keras_name = name
        self.eps = eps
        self.register_buffer("gamma", torch.ones(channels))
        self.register_buffer("beta", torch.zeros(channels))
        self.register_buffer("moving_mean", torch.zeros(channels))
        self.register_buffer("moving_variance", torch.ones(channels))

    def scale_shift(self) -> Tuple[torch.Tensor, torch.Tensor]:
        """(scale, shift) of the folded affine; cached until a buffer changes (frozen BN: ~never)."""
        key = (self.gamma.device, self.gamma._version, self.beta._version, self.moving_mean._version,
               self.moving_variance._version)
        c = self.__dict__.get("_ss_cache")
        if c is not None and c[0] == key:
            return c[1]
        s = self.gamma / torch.sqrt(self.moving_variance + self.eps)
        out = (s, self.beta - self.moving_mean * s)
        self.__dict__["_ss_cache"] = (key, out)
        return out

    def keras_weights(self):
        return [("gamma:0", self.gamma), ("beta:0", self.beta),
                ("moving_mean:0", self.moving_mean), ("moving_variance:0", self.moving_variance)]


class Conv2D(nn.Module):
    """Keras Conv2D with NHWC activations and OHWI weights.

    ``padding``: ``'same'`` (TF semantics, asymmetric at stride 2) or an int = explicit
    symmetric ZeroPadding2D in front of a ``'valid'`` conv (keras-resnet style).
    """

    def __init__(self, name: str, cin: int, cout: int, kernel_size: int, stride: int = 1,
                 padding: Union[str, int] = "same", use_bias: bool = True, relu: bool = False,
                 kernel_init: str = "glorot_uniform", bias_value: float = 0.0,
                 bn_name: Optional[str] = None, bn_eps: float = 1e-5):
        super().__init__()
        self.keras_name = name
        self.cin, self.cout, self.k, self.stride = cin, cout, kernel_size, stride
        self.padding = padding
        self.relu = relu
        self.kernel_init = kernel_init
        self.bias_value = bias_value
        self.weight = nn.Parameter(torch.empty(cout, kernel_size, kernel_size, cin))
        self.bias = nn.Parameter(torch.empty(cout)) if use_bias else None
        self.bn = FrozenBatchNormalization(bn_name, cout, bn_eps) if bn_name else None
        self.reset_parameters()

    def reset_parameters(self, gen: Optional[torch.Generator] = None) -> None:
        fan_in = self.k * self.k * self.cin
        fan_out = self.k * self.k * self.cout
        if self.kernel_init == "he_normal":
            he_normal_(self.weight.data, fan_in, gen)
        elif self.kernel_init == "normal001":
            with torch.no_grad():
                self.weight.normal_(0.0, 0.01, generator=gen)
        else:
            glorot_uniform_(self.weight.data, fan_in, fan_out, gen)
        if self.bias is not None:
            with torch.no_grad():
                self.bias.fill_(self.bias_value)

    def pads(self, in_hw: Sequence[int]) -> conv_ops.Pads:
        if self.padding == "same":
            return conv_ops.same_pads(in_hw, self.k, self.stride)
        p = int(self.padding)
        return (p, p, p, p)

    def out_hw(self, in_hw: Sequence[int]) -> Tuple[int, int]:
        return conv_ops.out_hw(in_hw, self.k, self.stride, self.pads(in_hw))

    def effective(self, dtype: torch.dtype) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
        """Weights/bias as seen by the conv kernel (frozen BN folded in), cast to ``dtype``."""
        w, b = self.weight, self.bias
        if self.bn is not None:
            s, t = self.bn.scale_shift()
            w = w * s.view(-1, 1, 1, 1)
            b = t if b is None else b * s + t
        w = w.to(dtype)
        if b is not None:
            b = b.float()
        return w, b

    def forward(self, x: torch.Tensor, residual: Optional[torch.Tensor] = None,
                relu: Optional[bool] = None, join=None) -> torch.Tensor:
        return conv_ops.conv_layer(x, self, residual=residual, relu=self.relu if relu is None else relu, join=join)

    def keras_weights(self):
        out = [("kernel:0", self.weight)]
        if self.bias is not None:
            out.append(("bias:0", self.bias))
        return out

    def extra_repr(self) -> str:
        return (f"{self.keras_name}: {self.cin}->{self.cout} k{self.k} s{self.stride} pad={self.padding}"
                f" bias={self.bias is not None} bn={self.bn.keras_name if self.bn else None} relu={self.relu}")
