"""NHWC convolution front-end.

All activations in this framework are contiguous NHWC tensors (Keras' layout, which keeps
the checkpoint mapping trivial) and all conv weights are OHWI (GEMM-K contiguous per output
channel).  Every conv in the model -- backbone (with frozen BN folded in), FPN and the shared
heads -- goes through :func:`conv2d` / :func:`pyramid_conv`, which pick a backend:

* ``"hip"``: the hand-written MFMA implicit-GEMM kernels (``csrc/kernels/conv_igemm.hip``)
  -- forward with fused bias/ReLU/residual epilogue, dgrad, split-K wgrad;
* ``"torch"``: ``F.conv2d`` on a channels-last view (MIOpen on ROCm, ATen on CPU).

Padding is explicit (top, bottom, left, right) so TensorFlow's asymmetric "same" padding at
stride 2 (P6, P7, pool1) is exact.
"""
from __future__ import annotations

import math
from typing import List, Optional, Sequence, Tuple

import torch
import torch.nn.functional as F

Pads = Tuple[int, int, int, int]

_BACKEND = {"conv": "auto"}
_CALIB = {"hook": None}     # models/calibrate.py: sees each BN conv's raw output before BN


def set_calibration_hook(fn) -> None:
    """``fn(layer, raw_conv_output)`` for every conv with a frozen BN (None = off)."""
    _CALIB["hook"] = fn


def set_conv_backend(name: str) -> None:
    """'auto' | 'hip' | 'torch'."""
    assert name in ("auto", "hip", "torch")
    _BACKEND["conv"] = name


def get_conv_backend() -> str:
    return _BACKEND["conv"]


def same_pads(in_hw: Sequence[int], k: int, s: int) -> Pads:
    """TensorFlow 'same' padding: extra row/col goes bottom/right."""
    out = []
    for n in in_hw:
        o = (n + s - 1) // s
        tot = max((o - 1) * s + k - n, 0)
        out.append((tot // 2, tot - tot // 2))
    return (out[0][0], out[0][1], out[1][0], out[1][1])


def out_hw(in_hw: Sequence[int], k: int, s: int, pads: Pads) -> Tuple[int, int]:
    h = (in_hw[0] + pads[0] + pads[1] - k) // s + 1
    w = (in_hw[1] + pads[2] + pads[3] - k) // s + 1
    return h, w


def _resolve_backend(x: torch.Tensor) -> str:
    b = _BACKEND["conv"]
    if b == "auto":
        from . import native
        return "hip" if (x.is_cuda and native.available() and native.conv_supported()) else "torch"
    return b


def _conv_torch(x, w, bias, stride, pads, relu, residual):
    pt, pb, pl, pr = pads
    xin = x
    if pt == pb and pl == pr:
        padding = (pt, pl)
    else:
        xin = F.pad(x, (0, 0, pl, pr, pt, pb))
        padding = (0, 0)
    if bias is not None and bias.dtype != x.dtype:
        bias = bias.to(x.dtype)
    y = F.conv2d(xin.permute(0, 3, 1, 2), w.permute(0, 3, 1, 2), bias, stride=stride, padding=padding)
    y = y.permute(0, 2, 3, 1)
    if residual is not None:
        y = y + residual
    if relu:
        y = F.relu(y)
    return y.contiguous()


def conv2d(x: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor], stride: int, pads: Pads,
           relu: bool = False, residual: Optional[torch.Tensor] = None, backend: Optional[str] = None) -> torch.Tensor:
    """y = act(conv(x, w) + bias [+ residual]).  x (N,H,W,Cin), w (Cout,kh,kw,Cin)."""
    be = backend or _resolve_backend(x)
    if be == "hip":
        from . import native
        return native.conv2d(x, w, bias, stride, pads, relu, residual)
    return _conv_torch(x, w, bias, stride, pads, relu, residual)


def conv_layer(x: torch.Tensor, layer, residual: Optional[torch.Tensor] = None, relu: bool = False,
               join=None) -> torch.Tensor:
    """Run a ``models.layers.Conv2D`` (fp32 master weights, optional frozen BN) on NHWC ``x``."""
    if _CALIB["hook"] is not None and getattr(layer, "bn", None) is not None:
        raw = _conv_torch(x, layer.weight.to(x.dtype), layer.bias, layer.stride, layer.pads(x.shape[1:3]),
                          False, None)
        _CALIB["hook"](layer, raw)
    if _resolve_backend(x) == "hip":
        from . import native_conv
        return native_conv.conv_layer(x, layer, residual, relu, join)
    if join is not None:
        raise RuntimeError("GradJoin needs the HIP conv backend")
    w, b = layer.effective(x.dtype)
    return _conv_torch(x, w, b, layer.stride, layer.pads(x.shape[1:3]), relu, residual)


def fused_blocks(x: torch.Tensor, convs) -> bool:
    """True when a ResNet block runs as one fused HIP autograd node (see native_conv.ResidualBlockFn)."""
    if _resolve_backend(x) != "hip":
        return False
    from . import native_conv
    return native_conv.fused_block_ok(x, convs)


def stem_fused(x: torch.Tensor, conv1) -> bool:
    """True when the ResNet stem (conv1 + BN + ReLU + pool1) runs as one HIP node (ops/stem.py)."""
    if _resolve_backend(x) != "hip" or _CALIB["hook"] is not None:
        return False
    from . import stem
    return stem.stem_ok(x, conv1)


def use_packed_heads(x: torch.Tensor) -> bool:
    """True when the heads run as packed ragged GEMMs (HIP backend, bf16, C % 64 == 0)."""
    return _resolve_backend(x) == "hip" and x.dtype == torch.bfloat16 and x.shape[-1] % 64 == 0


def pyramid_conv(xs: List[torch.Tensor], w: torch.Tensor, bias: Optional[torch.Tensor], relu: bool,
                 backend: Optional[str] = None) -> List[torch.Tensor]:
    """One 3x3/s1/'same' conv with shared weights applied to every pyramid level."""
    be = backend or _resolve_backend(xs[0])
    if be == "hip":
        from . import native
        return native.pyramid_conv(xs, w, bias, relu)
    k = w.shape[1]
    p = k // 2
    return [_conv_torch(x, w, bias, 1, (p, p, p, p), relu, None) for x in xs]


def maxpool_same(x: torch.Tensor, k: int = 3, s: int = 2) -> torch.Tensor:
    """MaxPool2D(k, s, padding='same') on NHWC with -inf padding (TF semantics)."""
    pads = same_pads(x.shape[1:3], k, s)
    from . import native
    if x.is_cuda and native.available() and _BACKEND["conv"] != "torch":
        return native.maxpool(x, k, s, pads)
    pt, pb, pl, pr = pads
    xp = F.pad(x.permute(0, 3, 1, 2), (pl, pr, pt, pb), value=float("-inf"))
    return F.max_pool2d(xp, k, s).permute(0, 2, 3, 1).contiguous()


def upsample_like(x: torch.Tensor, target_hw: Sequence[int]) -> torch.Tensor:
    """TF1 ``resize_images(NEAREST, align_corners=False)``: src = min(floor(dst*in/out), in-1)."""
    H, W = int(target_hw[0]), int(target_hw[1])
    h, w = x.shape[1], x.shape[2]
    iy = torch.clamp(torch.floor(torch.arange(H, device=x.device, dtype=torch.float32) * (h / H)).long(), max=h - 1)
    ix = torch.clamp(torch.floor(torch.arange(W, device=x.device, dtype=torch.float32) * (w / W)).long(), max=w - 1)
    return x[:, iy][:, :, ix]


def upsample_add(x: torch.Tensor, lateral: torch.Tensor) -> torch.Tensor:
    """lateral + UpsampleLike(x, lateral) -- the P4_merged / P3_merged adds."""
    from . import native
    if x.is_cuda and native.available() and _BACKEND["conv"] != "torch":
        return native.upsample_add(x, lateral)
    return lateral + upsample_like(x, lateral.shape[1:3])
