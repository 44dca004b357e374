"""ResNet stem on the HIP kernels: conv1 (7x7/s2, Cin 3) + frozen BN + ReLU + pool1 as ONE autograd node.

Spec: keras-resnet ``ZeroPadding2D(3)`` -> ``conv1`` -> ``bn_conv1`` -> ReLU -> ``pool1`` MaxPool 3x3 s2
'same' (the reference builds it through keras-retinanet at
``/root/reference/train.py:406-418``).

* forward: ``mxr_stem_pack`` folds the BN scale into a (64, 7, 8, 4) bf16 weight image,
  ``mxr_stem_pool_fwd`` (csrc/kernels/stem.hip) runs the conv on MFMA with shift + ReLU and pools its tile in
  LDS, marking windows whose max is 0 (:data:`POOL_FUSED`; else ``mxr_stem_fwd`` + ``mxr_maxpool_fwd(relu_in=1)``);
* backward: ``mxr_maxpool_bwd`` scatters the pooled gradient to the argmax pixels -- the ReLU backward
  is already in it (a window of zeros has no argmax) -- and ``mxr_stem_wgrad`` reduces the weight
  gradient over all output pixels on MFMA, returning ``scale * dW_eff`` in fp32.  The image needs
  no gradient, so there is no dgrad.
"""
from __future__ import annotations

import os

import torch

from . import native as _n
from .native import _chk, _p, _s, lib

_KP = 224           # packed K per output channel (7 ky x 8 kx x 4 ci)
_TR, _TC = 4, 64    # output tile of the kernels
_WS_COLS = 224


def stem_ok(x: torch.Tensor, conv1, pool_k: int = 3, pool_s: int = 2) -> bool:
    return (os.environ.get("MXR_STEM", "1") == "1" and x.is_cuda and x.dtype == torch.bfloat16
            and x.dim() == 4 and x.shape[-1] == 3 and conv1.k == 7 and conv1.stride == 2 and conv1.cout == 64
            and conv1.cin == 3 and conv1.bias is None and _n.available()
            and x.numel() < 2 ** 31 and x.shape[0] * x.shape[1] * x.shape[2] * 64 < 2 ** 31
            and x.data_ptr() % 4 == 0)   # the patch rows are fetched as 4-B words (stem.hip stem_fetch_rows)


def _ws_floats(N: int, Ho: int, Wo: int) -> int:
    nt = N * ((Wo + _TC - 1) // _TC) * ((Ho + _TR - 1) // _TR)
    return min(nt, 512) * 64 * _WS_COLS


def pack_weight(weight: torch.Tensor, scale) -> torch.Tensor:
    wpk = torch.empty((64, _KP), dtype=torch.bfloat16, device=weight.device)
    w = weight.detach().float().contiguous()
    sc = None if scale is None else scale.detach().float().contiguous()
    _chk(lib().mxr_stem_pack(_p(w), _p(sc), _p(wpk), _s()), "stem_pack")
    return wpk


def stem_conv_fwd(x, weight, scale, shift, pads, relu=True) -> torch.Tensor:
    """conv1 + BN + (ReLU) only, NHWC bf16 out (also the numerics-test entry)."""
    N, H, W, _ = x.shape
    pt, pb, pl, pr = pads
    Ho, Wo = (H + pt + pb - 7) // 2 + 1, (W + pl + pr - 7) // 2 + 1
    wpk = pack_weight(weight, scale)
    y = torch.empty((N, Ho, Wo, 64), dtype=torch.bfloat16, device=x.device)
    sh = None if shift is None else shift.detach().float().contiguous()
    _chk(lib().mxr_stem_fwd(_p(x), _p(wpk), _p(sh), _p(y), N, H, W, Ho, Wo, pt, pl, int(relu), _s()), "stem_fwd")
    return y


def stem_wgrad(x, dy, scale, pads, out=None, pool=None) -> torch.Tensor:
    """fp32 (64, 7, 7, 3) weight gradient ``scale * dW_eff`` of conv1 (accumulates into ``out``).

    ``pool = (arg, (Ho, Wo), pool_pads)``: ``dy`` is pool1's OUTPUT gradient and ``arg`` its relu-aware
    argmax; the conv-output gradient is gathered on the fly (never materialised)."""
    N, H, W, _ = x.shape
    if pool is None:
        Ho, Wo = dy.shape[1], dy.shape[2]
        parg, Hp, Wp, qt, ql = None, 0, 0, 0, 0
    else:
        parg, (Ho, Wo), qpads = pool
        Hp, Wp, qt, ql = dy.shape[1], dy.shape[2], qpads[0], qpads[2]
    ws = torch.empty(_ws_floats(N, Ho, Wo), dtype=torch.float32, device=x.device)
    dw = out if out is not None else torch.empty((64, 7, 7, 3), dtype=torch.float32, device=x.device)
    sc = None if scale is None else scale.detach().float().contiguous()
    _chk(lib().mxr_stem_wgrad(_p(x), _p(dy), _p(ws), _p(sc), _p(dw), N, H, W, Ho, Wo, pads[0], pads[2],
                              int(out is not None), _p(parg), Hp, Wp, qt, ql, _s()), "stem_wgrad")
    return dw


# conv1 + BN + ReLU + pool1 as ONE kernel (mxr_stem_pool_fwd): the conv output is never stored (a switch for
# same-process A/Bs; profiles/r6_stem_pool_fused.txt)
POOL_FUSED = True


def stem_pool_fwd(x, weight, scale, shift, conv_pads, pool_pads):
    """(pool1 output, its relu-aware argmax, conv-output shape) of the fused stem kernel."""
    N, H, W, _ = x.shape
    pt, pb, pl, pr = conv_pads
    Ho, Wo = (H + pt + pb - 7) // 2 + 1, (W + pl + pr - 7) // 2 + 1
    qt, qb, ql, qr = pool_pads
    Hp, Wp = (Ho + qt + qb - 3) // 2 + 1, (Wo + ql + qr - 3) // 2 + 1
    wpk = pack_weight(weight, scale)
    y = torch.empty((N, Hp, Wp, 64), dtype=torch.bfloat16, device=x.device)
    arg = torch.empty((N, Hp, Wp, 64), dtype=torch.uint8, device=x.device)
    sh = None if shift is None else shift.detach().float().contiguous()
    _chk(lib().mxr_stem_pool_fwd(_p(x), _p(wpk), _p(sh), _p(y), _p(arg), N, H, W, Ho, Wo, pt, pl, Hp, Wp, qt, ql, _s()),
         "stem_pool_fwd")
    return y, arg, (N, Ho, Wo, 64)


class StemFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, scale, shift, conv_pads, pool_pads):
        x = x.contiguous()
        if POOL_FUSED:
            y, arg, y1_shape = stem_pool_fwd(x, weight, scale, shift, conv_pads, pool_pads)
        else:
            y1 = stem_conv_fwd(x, weight, scale, shift, conv_pads, relu=True)
            y, arg = _n.maxpool_fwd_raw(y1, 3, 2, pool_pads, relu_in=True)
            y1_shape = tuple(y1.shape)
        ctx.save_for_backward(x, arg, scale if scale is not None else torch.empty(0))
        ctx.cfg = (y1_shape, conv_pads, pool_pads, scale is not None)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, arg, scale = ctx.saved_tensors
        y1_shape, conv_pads, pool_pads, has_scale = ctx.cfg
        dw = None
        if ctx.needs_input_grad[1]:
            dyp = dy.to(torch.bfloat16).contiguous()
            # (stem_wgrad's pool= form, gathering the conv-output gradient inside the staging, measured
            # slower: 0.84 vs 0.50 ms at B=16 -- the 4-window gather serialises the prefetch loads)
            dy1 = _n.maxpool_bwd_raw(dyp, arg, y1_shape, 3, 2, pool_pads)
            dw = stem_wgrad(x, dy1, scale if has_scale else None, conv_pads)
        return None, dw, None, None, None, None


def stem(x: torch.Tensor, conv1, pool_pads) -> torch.Tensor:
    """pool1(relu(bn_conv1(conv1(x)))) for a models.layers.Conv2D ``conv1`` (checked by :func:`stem_ok`)."""
    scale = shift = None
    if conv1.bn is not None:
        scale, shift = conv1.bn.scale_shift()
    return StemFn.apply(x, conv1.weight, scale, shift, tuple(conv1.pads(x.shape[1:3])), tuple(pool_pads))
