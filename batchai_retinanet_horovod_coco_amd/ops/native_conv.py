"""HIP implicit-GEMM convolution bindings: forward, data gradient, weight/bias gradient.

Kernels: ``csrc/kernels/conv_igemm.hip`` (fwd + dgrad) and ``csrc/kernels/conv_wgrad.hip``
(split-K wgrad over pixels, deterministic slab reduction, bias-gradient column sums).

The autograd functions take the layer's fp32 MASTER weight and (for backbone convs) the frozen-BN
scale/shift: the bf16 effective weight ``W * s`` is formed inside the op and the weight gradient
comes back as ``s * dW_eff`` in fp32 straight from the reduction kernel -- no bf16 gradients, no
extra rescaling pass.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional, Sequence, Tuple

import torch
import torch.nn.functional as F

from . import native as _n
from .native import ConvGeom, _chk, _p, _s, lib, zero_page, c_int, c_ll, c_vp
from .side_stream import SIDE

_SIGS = {
    "mxr_conv_wgrad": [c_vp, c_vp, c_int, c_vp, c_int, c_vp, c_vp, c_int, c_vp, ctypes.POINTER(ConvGeom), c_int, c_vp],
    "mxr_bias_grad": [c_vp, c_ll, c_int, c_int, c_int, c_vp, c_vp, c_vp, c_int, c_vp],
    "mxr_bias_res_act": [c_vp, c_vp, c_vp, c_ll, c_int, c_int, c_vp],
    "mxr_relu_bwd": [c_vp, c_vp, c_vp, c_ll, c_vp],
}
_BOUND = [False]


def _bind():
    if not _BOUND[0]:
        L = lib()
        for name, args in _SIGS.items():
            fn = getattr(L, name)
            fn.argtypes = args
            fn.restype = c_int
        _BOUND[0] = True
    return lib()


# ------------------------------------------------------------------------------- geometry
def geom_single(N, H, W, Ho, Wo, k, stride, pads, cin, cout, ostride=1, oH=0, oW=0) -> ConvGeom:
    g = ConvGeom()
    g.nlev = 1
    g.H[0], g.W[0], g.Ho[0], g.Wo[0] = H, W, Ho, Wo
    g.in_off[0] = 0
    g.mstart[0], g.mstart[1] = 0, Ho * Wo
    g.in_img, g.out_img = H * W, Ho * Wo
    g.stride, g.pt, g.pl, g.kh, g.kw = stride, pads[0], pads[2], k, k
    g.cin, g.cout = cin, cout
    g.M = N * Ho * Wo
    g.ostride, g.oH, g.oW = ostride, oH, oW
    return g


def geom_pyramid(N, shapes: Sequence[Tuple[int, int]], cin, cout) -> ConvGeom:
    g = ConvGeom()
    g.nlev = len(shapes)
    off = 0
    for l, (h, w) in enumerate(shapes):
        g.H[l] = g.Ho[l] = h
        g.W[l] = g.Wo[l] = w
        g.in_off[l] = off
        g.mstart[l] = off
        off += h * w
    g.mstart[len(shapes)] = off
    g.in_img = g.out_img = off
    g.stride, g.pt, g.pl, g.kh, g.kw = 1, 1, 1, 3, 3
    g.cin, g.cout = cin, cout
    g.M = N * off
    g.ostride, g.oH, g.oW = 1, 0, 0
    return g


def _variant(cout: int) -> int:
    v = os.environ.get("MXR_CONV_VARIANT")
    if v is not None:
        return int(v)
    return 1 if cout <= 64 else 0


def launch_fwd(x, w, bias, res, y, g: ConvGeom, relu: bool, accumulate: bool = False,
               variant: Optional[int] = None, mask: Optional[torch.Tensor] = None) -> None:
    """One implicit-GEMM launch.  ``mask``: zero the output where ``mask <= 0`` (fused relu backward
    of the layer that produced this conv's input); ``accumulate``: ``y += result``."""
    v = _variant(g.cout) if variant is None else variant
    zp = _p(zero_page(x.device))
    if isinstance(v, str) and v.startswith("c1x1_"):   # streaming narrow-K 1x1 kernel (conv1x1_stream.hip)
        launch_c1x1(x, w, bias, res, y, g, relu, accumulate, int(v[5:]), mask)
        return
    if isinstance(v, str) and v.startswith("hx32_"):   # 32x32x16-MFMA halo kernel (conv_hx32.hip)
        launch_hx32(x, w, bias, res, y, g, relu, accumulate, int(v[5:]), mask)
        return
    if isinstance(v, str) and v.startswith("p8_"):   # 256x256 kernels, 8-wave phases (conv_p8.hip)
        launch_p8(x, w, bias, res, y, g, relu, accumulate, int(v[3:]), mask)
        return
    if isinstance(v, str):      # "haloN": halo-staged 3x3/s1 kernel (conv_halo.hip, tile table ops/halo.py)
        launch_halo(x, w, bias, res, y, g, relu, accumulate, int(v[4:]), mask)
        return
    if v >= 3:   # deep-pipelined 8-wave kernels (conv_pipe.hip): 3 = 256co x 256pix, 4 = 128co x 256pix,
                 # 5 / 6 = the same with the next sub-stage's DMA interleaved between MFMA groups,
                 # 7 / 8 = interleaved + s_setprio around the MFMA groups,
                 # 9 / 10 = narrow 64co x 256pix on 4 waves (two blocks per CU; 64-channel layers),
                 # 10 with s_setprio; 11 / 12 / 13 = 128-pixel tiles (128 / 256 / 64 co) for the
                 # small-K 1x1 layers whose epilogue (residual / mask / accumulate) dominates;
                 # 14 / 15 / 16 = 3-deep LDS rings (128x128, 64x128, 128x256: 3 / 4 / 2 blocks per CU)
        _chk(lib().mxr_conv_fwd_pipe(_p(x), _p(w), _p(bias), _p(res), _p(mask), _p(y), zp, ctypes.byref(g),
                                     int(relu), int(accumulate), v - 3, _s()), "conv_fwd_pipe")
        return
    _chk(lib().mxr_conv_fwd(_p(x), _p(w), _p(bias), _p(res), _p(mask), _p(y), zp, ctypes.byref(g), int(relu),
                            int(accumulate), v, _s()), "conv_fwd")


HALO_VARIANTS = (0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15)
HX32_VARIANTS = (0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10)   # 2 / 3 / 6 / 7 / 9: persistent grid
C1X1_BN = (64, 128, 256)
P8_VARIANTS = (0, 1, 2, 3, 4, 5, 6, 7, 8, 10)
# raced by the tuner: the fragment-reads-first forms (the others never came within 3 % in situ).  (A
# 4-wave, one-wave-per-SIMD form measured 574-747 TF/s on the head shape vs 912 for p8_5 even with its
# accumulators pinned to AGPRs, profiles/r2_p4_agpr_microbench.txt, and was removed.)
P8_TUNED = (5, 6, 8)


def p8_covers(g: ConvGeom) -> bool:
    """conv_p8.hip: 64-channel K-tiles of one tap, 16-B output chunks, no strided output scatter, at most
    16 taps."""
    K = g.kh * g.kw * g.cin
    return (g.cin % 64 == 0 and g.cout % 8 == 0 and g.ostride == 1 and 1 <= g.nlev <= 5 and g.kh * g.kw <= 16
            and (int(g.M) + 1) * max(g.cin, g.cout) < 2 ** 31 and g.cout * K < 2 ** 31)


def big_tile_variants(g: ConvGeom):
    if not p8_covers(g):
        return []
    return ["p8_%d" % v for v in P8_TUNED]


def launch_p8(x, w, bias, res, y, g: ConvGeom, relu: bool, accumulate: bool = False, variant: int = 0,
              mask: Optional[torch.Tensor] = None) -> None:
    """256 co x 256 px implicit GEMM, 8-wave phase-pipelined (csrc/kernels/conv_p8.hip)."""
    if not p8_covers(g):
        raise RuntimeError("conv_p8: geometry not covered")
    K = g.kh * g.kw * g.cin
    if not (x.is_contiguous() and w.is_contiguous() and y.is_contiguous() and x.shape[-1] == g.cin
            and int(w.numel()) == g.cout * K and int(y.numel()) == int(g.M) * g.cout
            and (bias is None or bias.data_ptr() % 16 == 0)):
        raise RuntimeError("conv_p8: operand shapes do not match the geometry")
    _chk(lib().mxr_conv_p8(_p(x), _p(w), _p(bias), _p(res), _p(mask), _p(y), _p(zero_page(x.device)),
                           ctypes.byref(g), int(relu), int(accumulate), int(variant), _s()), "conv_p8")


def c1x1_variants(g: ConvGeom):
    """Streaming 1x1 kernel variants covering ``g`` (1x1, no padding, single level, K in 64/128/256)."""
    if not (g.kh == 1 and g.kw == 1 and g.nlev == 1 and g.ostride == 1 and g.pt == 0 and g.pl == 0
            and g.stride in (1, 2) and g.cin in (64, 128, 256) and g.cout % 8 == 0):
        return []
    if g.stride == 1 and (g.H[0] != g.Ho[0] or g.W[0] != g.Wo[0]):
        return []
    return ["c1x1_%d" % bn for bn in C1X1_BN if bn * g.cin <= 32768 and bn <= max(64, g.cout)]


def launch_c1x1(x, w, bias, res, y, g: ConvGeom, relu: bool, accumulate: bool = False, bn: int = 128,
                mask: Optional[torch.Tensor] = None) -> None:
    """1x1 conv with the weight slice resident in LDS and pixels streamed (csrc/kernels/conv1x1_stream.hip)."""
    if "c1x1_%d" % bn not in c1x1_variants(g):
        raise RuntimeError("conv1x1_stream: geometry not covered")
    nimg = int(g.M) // (g.Ho[0] * g.Wo[0])
    if not (x.is_contiguous() and w.is_contiguous() and y.is_contiguous() and x.shape[-1] == g.cin
            and int(x.numel()) == nimg * g.H[0] * g.W[0] * g.cin and int(y.numel()) == int(g.M) * g.cout
            and int(w.numel()) == g.cout * g.cin and (bias is None or bias.data_ptr() % 16 == 0)):
        raise RuntimeError("conv1x1_stream: operand shapes do not match the geometry")
    _chk(lib().mxr_conv1x1_stream(_p(x), _p(w), _p(bias), _p(res), _p(mask), _p(y), int(g.M), g.cout, g.cin,
                                  g.H[0], g.W[0], g.Ho[0], g.Wo[0], g.stride, int(relu), int(accumulate), bn, 0,
                                  _s()), "conv1x1_stream")


def launch_halo(x, w, bias, res, y, g: ConvGeom, relu: bool, accumulate: bool = False, variant: int = 0,
                mask: Optional[torch.Tensor] = None) -> None:
    """3x3 / stride-1 / pad-1 conv with halo-staged pixels (csrc/kernels/conv_halo.hip): per 32-channel
    chunk each tile's input halo is loaded into LDS once and shared by the 9 taps."""
    from . import halo as _hx
    if not _hx.covers(g):
        raise RuntimeError("conv3x3_halo: geometry not covered")
    tiles, nt = _hx.device_tiles(_hx.geom_batch(g), _hx.geom_shapes(g), x.device)
    _chk(lib().mxr_conv3x3_halo(_p(x), _p(w), _p(bias), _p(res), _p(mask), _p(y), _p(zero_page(x.device)),
                                ctypes.byref(g), _p(tiles), nt, int(relu), int(accumulate), int(variant), _s()),
         "conv3x3_halo")


def launch_hx32(x, w, bias, res, y, g: ConvGeom, relu: bool, accumulate: bool = False, variant: int = 0,
                mask: Optional[torch.Tensor] = None) -> None:
    """3x3 / stride-1 / pad-1 conv on the 32x32x16 MFMA with conflict-free plane-split LDS images
    (csrc/kernels/conv_hx32.hip; same tile table as :func:`launch_halo`)."""
    from . import halo as _hx
    if not hx32_covers(g):
        raise RuntimeError("conv3x3_hx32: geometry not covered")
    if not (x.is_contiguous() and w.is_contiguous() and y.is_contiguous() and x.shape[-1] == g.cin
            and int(w.numel()) == g.cout * 9 * g.cin and int(y.numel()) == int(g.M) * g.cout
            and int(x.numel()) == int(g.M) * g.cin and (bias is None or bias.data_ptr() % 16 == 0)):
        raise RuntimeError("conv3x3_hx32: operand shapes do not match the geometry")
    if (g.cin // 32) % 2:     # the persistent grid chains tiles over an even chunk count only
        variant = {2: 0, 3: 1, 6: 4, 7: 5, 9: 8}.get(variant, variant)
    tiles, nt = _hx.device_tiles(_hx.geom_batch(g), _hx.geom_shapes(g), x.device)
    wp = hx32_packed(w, g.cout, g.cin)
    _chk(lib().mxr_conv3x3_hx32(_p(x), _p(wp), _p(bias), _p(res), _p(mask), _p(y), _p(zero_page(x.device)),
                                ctypes.byref(g), _p(tiles), nt, int(relu), int(accumulate), int(variant), _s()),
         "conv3x3_hx32")


def hx32_packed(w: torch.Tensor, cout: int, cin: int) -> torch.Tensor:
    """``w`` (OHWI bf16) in conv_hx32's [tap][cin / 32][plane][cout][16] layout (a 1-KiB weight DMA piece
    is then contiguous).  Packed on every call (one small kernel, ~2 x the weight bytes): the weights are
    rewritten in place by HIP kernels every optimizer step, which a version-keyed cache cannot see."""
    wp = torch.empty(cout * 9 * cin, dtype=w.dtype, device=w.device)
    _chk(lib().mxr_hx32_pack_weights(_p(w), _p(wp), cout, cin, _s()), "hx32_pack")
    return wp


def hx32_covers(g: ConvGeom) -> bool:
    from . import halo as _hx
    return _hx.covers(g) and g.cout * 9 * g.cin * 2 < 2 ** 31


def relu_bwd_(dy: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
    """In-place ``dy *= (y > 0)`` (elementwise: reading and writing the same element is safe)."""
    assert dy.is_contiguous() and y.is_contiguous() and dy.shape == y.shape
    _chk(_bind().mxr_relu_bwd(_p(dy), _p(y), _p(dy), dy.numel(), _s()), "relu_bwd_")
    return dy


def relu_bwd(dy: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
    dx = torch.empty_like(dy)
    _chk(_bind().mxr_relu_bwd(_p(dy), _p(y), _p(dx), dy.numel(), _s()), "relu_bwd")
    return dx


def bias_res_act_(y: torch.Tensor, bias: Optional[torch.Tensor], res: Optional[torch.Tensor], relu: bool):
    if bias is None and res is None and not relu:
        return y
    _chk(_bind().mxr_bias_res_act(_p(y), _p(bias), _p(res), y.numel(), y.shape[-1], int(relu), _s()), "epilogue")
    return y


def miopen_fwd(x, w, bias, res, stride, pads, relu):
    """Library conv (MIOpen, channels-last) + ONE fused bias/residual/ReLU epilogue pass."""
    pt, pb, pl, pr = pads
    if pt == pb and pl == pr:
        xin, padding = x, (pt, pl)
    else:
        xin, padding = F.pad(x, (0, 0, pl, pr, pt, pb)), (0, 0)
    y = F.conv2d(xin.permute(0, 3, 1, 2), w.permute(0, 3, 1, 2), None, stride=stride, padding=padding)
    y = y.permute(0, 2, 3, 1)
    if not y.is_contiguous():
        y = y.contiguous()
    return bias_res_act_(y, bias, res, relu)


FWD_VARIANTS = (0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16)


def fwd_candidates(x, w, b, res, g: ConvGeom, stride, pads, relu, out_shape, allow_miopen=True, mask=None,
                   fp8_ok=False, out: Optional[torch.Tensor] = None, only: Optional[str] = None):
    """``fp8_ok``: a forward pass that may run in fp8 -- with fp8 enabled (ops.fp8) and a covered shape
    the fp8 kernel variants (quantisation of the input included) join the race; a backbone conv whose
    input quantisation costs more than fp8 saves stays bf16 (the packed head layers, which get their
    input's fp8 copy from the producing epilogue, always run fp8: ops.fp8.pyramid_forward).
    ``only``: build just that candidate (the tuned winner: the dispatch fast path, see :func:`_only`)."""
    from . import fp8 as _f8
    f8c = {}
    if (fp8_ok and mask is None and (only is None or only.startswith("f8")) and _f8.enabled()
            and _f8.eligible(g.cin, g.cout, g.ostride)):
        f8c = _f8.candidates(x, w, b, res, g, relu, out_shape)

    def hip(v):
        def f():
            if out is not None:        # accumulate into ``out`` (y += conv)
                launch_fwd(x, w, b, res, out, g, relu, accumulate=True, variant=v, mask=mask)
                return out
            y = torch.empty(out_shape, dtype=x.dtype, device=x.device)
            launch_fwd(x, w, b, res, y, g, relu, variant=v, mask=mask)
            return y
        return f
    if only is not None:
        return _only_fwd(only, hip, g, out, allow_miopen, f8c, x, w, b, res, stride, pads, relu, mask)
    cands = {"hip%d" % v: hip(v) for v in FWD_VARIANTS if v < 3 or g.cout % 8 == 0}
    from . import halo as _hx
    if _hx.covers(g):
        cands.update({"halo%d" % v: hip("halo%d" % v) for v in HALO_VARIANTS})
    if hx32_covers(g):
        cands.update({"hx32_%d" % v: hip("hx32_%d" % v) for v in HX32_VARIANTS})
    cands.update({v: hip(v) for v in c1x1_variants(g)})
    cands.update({v: hip(v) for v in big_tile_variants(g)})
    if out is not None:       # accumulating forms: HIP kernels only (their epilogue adds in place)
        allow_miopen = False
        f8c = {}
    if allow_miopen:
        if mask is None:
            cands["miopen"] = lambda: miopen_fwd(x, w, b, res, stride, pads, relu)
        else:
            cands["miopen"] = lambda: relu_bwd(miopen_fwd(x, w, b, res, stride, pads, relu), mask)
    cands.update(f8c)
    return cands


def _only_fwd(only, hip, g, out, allow_miopen, f8c, x, w, b, res, stride, pads, relu, mask):
    """fwd_candidates restricted to ``only`` (empty when it is not a candidate of this call: the caller
    then builds the full set)."""
    if only.startswith("hip"):
        v = int(only[3:])
        return {only: hip(v)} if v in FWD_VARIANTS and (v < 3 or g.cout % 8 == 0) else {}
    if only.startswith("hx32_"):
        return {only: hip(only)} if hx32_covers(g) and int(only[5:]) in HX32_VARIANTS else {}
    if only.startswith("halo"):
        from . import halo as _hx
        return {only: hip(only)} if _hx.covers(g) and int(only[4:]) in HALO_VARIANTS else {}
    if only.startswith("c1x1_"):
        return {only: hip(only)} if only in c1x1_variants(g) else {}
    if only.startswith("p8_"):
        return {only: hip(only)} if only in big_tile_variants(g) else {}
    if only == "miopen":
        if out is not None or not allow_miopen:
            return {}
        if mask is None:
            return {only: lambda: miopen_fwd(x, w, b, res, stride, pads, relu)}
        return {only: lambda: relu_bwd(miopen_fwd(x, w, b, res, stride, pads, relu), mask)}
    if out is None and only in f8c:
        return {only: f8c[only]}
    return {}


def _only(key: str) -> Optional[str]:
    """The tuned winner for ``key`` when dispatch can go straight to it (else None: build every candidate).
    Building the full candidate dict costs 15-40 us of host time per conv pass -- ~8 ms per training step
    over R50-FPN -- which left the GPU waiting for the host in the backbone's backward."""
    from .conv_tuner import TUNER
    return TUNER.winner(key)


def hip_conv_ok(cin: int, cout: int, dtype) -> bool:
    return dtype == torch.bfloat16 and cin % 64 == 0 and cout % 4 == 0


def flip(w: torch.Tensor) -> torch.Tensor:
    cw = _n.compute_weights()
    if cw is not None:
        f = cw.flipped(w)      # batched once per optimizer step for the whole model
        if f is not None:
            return f
    co, kh, kw, ci = w.shape
    wd = torch.empty((ci, kh, kw, co), dtype=w.dtype, device=w.device)
    _chk(lib().mxr_flip_transpose(_p(w), _p(wd), co, kh, kw, ci, _s()), "flip")
    return wd


def torch_conv_backward(x, w, dy, stride, pads, need_dx, need_dw):
    """MIOpen fallback for the shape classes the HIP kernels do not cover (stem, s2 3x3 dgrad)."""
    pt, pb, pl, pr = pads
    if pt == pb and pl == pr:
        xin, padding, padded = x, [pt, pl], False
    else:
        xin, padding, padded = F.pad(x, (0, 0, pl, pr, pt, pb)), [0, 0], True
    dx_in, dw, _ = torch.ops.aten.convolution_backward(
        dy.permute(0, 3, 1, 2), xin.permute(0, 3, 1, 2), w.permute(0, 3, 1, 2), None, [stride, stride], padding,
        [1, 1], False, [0, 0], 1, [need_dx, need_dw, False])
    dx = None
    if need_dx:
        dx = dx_in.permute(0, 2, 3, 1)
        if padded:
            dx = dx[:, pt:pt + x.shape[1], pl:pl + x.shape[2], :]
        dx = dx.contiguous()
    if need_dw:
        dw = dw.permute(0, 2, 3, 1).contiguous()
    return dx, dw


def conv_dgrad(dy, w, x_shape, stride, pads, variant: Optional[int] = None, mask: Optional[torch.Tensor] = None,
               out: Optional[torch.Tensor] = None, res: Optional[torch.Tensor] = None) -> Optional[torch.Tensor]:
    """dX via the forward kernel (stride 1: flipped weights; 1x1/s2: strided scatter); None if uncovered.

    ``mask``: fused relu backward (dX zeroed where mask <= 0); ``out``: accumulate into this tensor;
    ``res`` (stride 1): dX = dgrad + res into a fresh tensor (``out`` without touching ``res``).
    1x1/s2 with ``out``: only the strided positions are read, accumulated and masked -- the buffer it
    joins is the other 1x1/s2 branch's fresh dX, which already holds zeros at the gaps."""
    N, H, W, cin = x_shape
    cout, kh, kw, _ = w.shape
    Ho, Wo = dy.shape[1], dy.shape[2]
    if stride == 1 and hip_conv_ok(cout, cin, dy.dtype):
        wd = flip(w)
        dpads = (kh - 1 - pads[0], kh - 1 - pads[1], kw - 1 - pads[2], kw - 1 - pads[3])
        dx = out if out is not None else torch.empty((N, H, W, cin), dtype=dy.dtype, device=dy.device)
        launch_fwd(dy, wd, None, res, dx, geom_single(N, Ho, Wo, H, W, kh, 1, dpads, cout, cin), False,
                   accumulate=out is not None, variant=variant, mask=mask)
        return dx
    if res is not None:
        return None
    if kh == 1 and stride == 2 and tuple(pads) == (0, 0, 0, 0) and hip_conv_ok(cout, cin, dy.dtype):
        wd = flip(w)     # 1x1: the flip is the (cin, cout) transpose
        # the kernels write the zeros of the positions no output pixel maps to themselves (when not
        # accumulating), so a fresh dX needs no fill pass
        dx = out if out is not None else torch.empty((N, H, W, cin), dtype=dy.dtype, device=dy.device)
        g = geom_single(N, Ho, Wo, Ho, Wo, 1, 1, (0, 0, 0, 0), cout, cin, ostride=2, oH=H, oW=W)
        launch_fwd(dy, wd, None, None, dx, g, False, accumulate=out is not None, variant=variant, mask=mask)
        return dx
    if kh == 3 and kw == 3 and stride == 2 and hip_conv_ok(cout, cin, dy.dtype):
        return _dgrad_s2_subpixel(dy, w, x_shape, pads, variant, mask, out)
    return None


def _s2_phase_taps(p: int, pad: int):
    """Sub-pixel split of a 3-tap / stride-2 data gradient along one axis: input coordinate i = 2a + p
    receives dY[o] W[k] for every tap k with p + pad - k even, at o = a + (p + pad - k) / 2.  Returns the
    taps ordered by that offset (consecutive) and the stride-1 'pad' of the phase convolution."""
    ks = sorted((k for k in range(3) if (p + pad - k) % 2 == 0), key=lambda k: (p + pad - k) // 2)
    offs = [(p + pad - k) // 2 for k in ks]
    assert offs == list(range(offs[0], offs[0] + len(offs)))
    return ks, -offs[0]


def _pick_taps(t, dim, ks):
    """Taps ``ks`` (one tap, or (2, 0)) along ``dim`` by slicing -- no index tensor, so no host-to-device
    copy (the step may be under HIP-graph capture)."""
    if len(ks) == 1:
        return t.narrow(dim, ks[0], 1)
    assert list(ks) == [2, 0], ks
    return t.narrow(dim, 0, 3)[(slice(None),) * dim + (slice(0, 3, 2),)].flip(dim)


def _dgrad_s2_subpixel(dy, w, x_shape, pads, variant, mask, out):
    """dX of a 3x3 / stride-2 conv (FPN P6 / P7) in ONE implicit GEMM: the four sub-pixel phases (one per
    (row, column) parity of dX; 1-2 taps per axis) share a 2x2 tap window over dY, so their weights are
    stacked as 4 x cin output channels (zero where a phase has no tap) and one stride-1 2x2 conv produces
    all phases; ``mxr_s2_shuffle`` scatters them into dX with the mask / accumulation.  (1.8x the MACs of
    the exact phases, but one launch instead of four small ones.)"""
    N, H, W, cin = x_shape
    cout = w.shape[0]
    Ho, Wo = dy.shape[1], dy.shape[2]
    Hp, Wp = (H + 1) // 2, (W + 1) // 2
    w4, win = _s2_stacked_weights_hip(w, pads)
    g = geom_single(N, Ho, Wo, Hp, Wp, 2, 1, (win[0], 0, win[1], 0), cout, 4 * cin)
    y4 = torch.empty((N, Hp, Wp, 4 * cin), dtype=dy.dtype, device=dy.device)
    launch_fwd(dy, w4, None, None, y4, g, False, variant=variant)
    dx = out if out is not None else torch.empty((N, H, W, cin), dtype=dy.dtype, device=dy.device)
    _chk(lib().mxr_s2_shuffle(_p(y4), _p(dx), _p(mask), int(out is not None), N, H, W, Hp, Wp, cin, _s()),
         "s2_shuffle")
    return dx


def _s2_stack_taps(pads):
    """Per phase (2 py + px) and window slot (2 ty + tx): the 3x3 tap ky * 3 + kx, or -1; and the window's
    (top, left) pad."""
    axes = []
    for pad in (pads[0], pads[2]):
        ph = [_s2_phase_taps(p, pad) for p in (0, 1)]
        lo = min(-pd for _, pd in ph)
        slots = [{-pd - lo + i: k for i, k in enumerate(ks)} for ks, pd in ph]
        axes.append((slots, -lo))
    (sy, pty), (sx, ptx) = axes
    taps = []
    for py in (0, 1):
        for px in (0, 1):
            for ty in range(2):
                for tx in range(2):
                    ky, kx = sy[py].get(ty), sx[px].get(tx)
                    taps.append(-1 if ky is None or kx is None else ky * 3 + kx)
    return taps, (pty, ptx)


_S2_TAPS = {}


def _s2_stacked_weights_hip(w, pads):
    """_s2_stacked_weights in one kernel (mxr_s2_stack) instead of ~25 small torch ops."""
    cout, _, _, cin = w.shape
    key = (tuple(pads), w.device)
    ent = _S2_TAPS.get(key)
    if ent is None:
        taps, win = _s2_stack_taps(pads)
        ent = _S2_TAPS[key] = ((ctypes.c_int * 16)(*taps), win)
    w4 = torch.empty((4 * cin, 2, 2, cout), dtype=w.dtype, device=w.device)
    _chk(lib().mxr_s2_stack(_p(w.contiguous()), _p(w4), cin, cout, ent[0], _s()), "s2_stack")
    return w4, ent[1]


def _s2_stacked_weights(w, pads):
    """(4 cin, 2, 2, cout) bf16 weights of the phase-stacked 2x2 conv and its (top, left) pad.  Per axis the
    phases' tap offsets span one 2-wide window [lo, lo + 1]; window slot t of phase p holds the 3x3 tap
    k with offset lo + t (or zero)."""
    cout, _, _, cin = w.shape
    wt = w.permute(3, 1, 2, 0)                               # (cin, ky, kx, cout)
    axes = []
    for pad in (pads[0], pads[2]):
        ph = [_s2_phase_taps(p, pad) for p in (0, 1)]        # (taps ordered by offset, stride-1 pad)
        lo = min(-pd for _, pd in ph)
        slots = []
        for ks, pd in ph:
            first = -pd - lo                                 # window slot of the phase's first tap
            slots.append({first + i: k for i, k in enumerate(ks)})
        axes.append((slots, -lo))
    (sy, pty), (sx, ptx) = axes
    blocks = []
    for py in (0, 1):
        for px in (0, 1):
            rows = []
            for ty in range(2):
                cols = []
                for tx in range(2):
                    ky, kx = sy[py].get(ty), sx[px].get(tx)
                    if ky is None or kx is None:
                        cols.append(torch.zeros_like(wt[:, 0, 0]))
                    else:
                        cols.append(wt[:, ky, kx])
                rows.append(torch.stack(cols, 1))
            blocks.append(torch.stack(rows, 1))              # (cin, 2, 2, cout)
    return torch.cat(blocks, 0).contiguous(), (pty, ptx)


_WGRAD_TILE = {0: (128, 128), 1: (128, 64), 2: (64, 128)}   # variant -> (BK, BCO)


def _splits(g: ConvGeom, bk: int, bco: int) -> int:
    K = g.kh * g.kw * g.cin
    tiles = ((K + bk - 1) // bk) * ((g.cout + bco - 1) // bco)
    steps = (g.M + 63) // 64
    target = int(os.environ.get("MXR_WGRAD_BLOCKS", "1024"))
    s = max(1, -(-target // tiles))
    return int(max(1, min(s, steps // 4 if steps >= 4 else 1, 256)))


# variant -> (TK, TC) of conv_wgrad_pipe.hip (5 / 6: DMA interleaved between MFMA groups, 7: interleaved +
# s_setprio, 8 / 9: s_setprio around the MFMA block, 10-12: narrow 4-wave tiles for 64-channel layers,
# 13-15: two blocks per CU -- 128 x 128, and 256 x 128 / 128 x 256 on 3-deep rings)
_WGRAD_PIPE_TILE = {3: (256, 256), 4: (256, 128), 5: (256, 256), 6: (256, 128), 7: (256, 256), 8: (256, 256),
                    9: (256, 128), 10: (256, 64), 11: (128, 64), 12: (64, 64), 13: (128, 128), 14: (256, 128),
                    15: (128, 256)}
# phase-pipelined 256 k x 256 co wgrad (conv_wgrad_p8.hip): variant -> kernel variant (1 = s_setprio)
_WGRAD_P8 = {20: 0, 21: 1, 22: 2, 23: 3}
# resident blocks per CU the split count aims for (narrow / small-ring tiles run several per CU)
_WGRAD_PIPE_OCC = {10: 2, 11: 3, 12: 4, 13: 2, 14: 2, 15: 2}


def _splits_pipe(g: ConvGeom, tk: int, tc: int, occ: int = 1) -> int:
    """Pixel splits so the grid is ~192 x ``occ`` blocks (``occ`` blocks on three quarters of the 256 CUs),
    each split >= 8 sub-stages of 32 rows.  The weight gradients run on the side stream next to the data-gradient chain:
    a grid that leaves a quarter of the CUs to the concurrent dgrad kernels also halves the split-K slab
    traffic of a full-chip grid's extra splits (bench sweep: 128 / 160 / 192 / 224 / 256 / 384 blocks ->
    434 / 446 / 457-458 / 446 / 452 / 433 img/s)."""
    K = g.kh * g.kw * g.cin
    tiles = ((K + tk - 1) // tk) * ((g.cout + tc - 1) // tc)
    nsub = (g.M + 31) // 32
    target = int(os.environ.get("MXR_WGRAD_PIPE_BLOCKS", "192")) * occ
    if g.nlev > 1:      # packed head layers (A/B knob)
        target = int(os.environ.get("MXR_WGRAD_PIPE_BLOCKS_PYR", str(target // occ))) * occ
    s = max(1, round(target / tiles))
    return int(max(1, min(s, nsub // 8 if nsub >= 8 else 1, 512 * occ)))


def conv_wgrad(x, dy, g: ConvGeom, scale: Optional[torch.Tensor], out: Optional[torch.Tensor] = None,
               accumulate: bool = False, variant: Optional[int] = None) -> torch.Tensor:
    """fp32 dW (OHWI) = scale[co] * sum_m dY (x) im2col(X); dY may have cout % 8 != 0 (padded)."""
    cout = g.cout
    K = g.kh * g.kw * g.cin
    ldy = dy.shape[-1]
    if ldy % 8:
        dy = F.pad(dy, (0, 8 - ldy % 8))
        ldy = dy.shape[-1]
    dy = dy.contiguous()
    if variant is None:
        variant = 1 if cout <= 64 else (2 if K <= 64 else 0)
    if out is None:
        out = torch.empty((cout, g.kh, g.kw, g.cin), dtype=torch.float32, device=dy.device)
    sc = None if scale is None else scale.float().contiguous()
    if variant in _WGRAD_P8:
        splits = _splits_pipe(g, 256, 256)
        part = torch.empty(splits * cout * K, dtype=torch.float32, device=dy.device)
        _chk(lib().mxr_conv_wgrad_p8(_p(x), _p(dy), ldy, _p(part), splits, _p(out), _p(sc), int(accumulate),
                                     _p(zero_page(dy.device)), ctypes.byref(g), _WGRAD_P8[variant], _s()),
             "conv_wgrad_p8")
        return out
    if variant in _WGRAD_PIPE_TILE:
        tk, tc = _WGRAD_PIPE_TILE[variant]
        splits = _splits_pipe(g, tk, tc, _WGRAD_PIPE_OCC.get(variant, 1))
        part = torch.empty(splits * cout * K, dtype=torch.float32, device=dy.device)
        _chk(lib().mxr_conv_wgrad_pipe(_p(x), _p(dy), ldy, _p(part), splits, _p(out), _p(sc), int(accumulate),
                                       _p(zero_page(dy.device)), ctypes.byref(g), variant - 3, _s()),
             "conv_wgrad_pipe")
        return out
    bk, bco = _WGRAD_TILE[variant]
    splits = _splits(g, bk, bco)
    part = torch.empty(splits * cout * K, dtype=torch.float32, device=dy.device)
    _chk(_bind().mxr_conv_wgrad(_p(x), _p(dy), ldy, _p(part), splits, _p(out), _p(sc), int(accumulate),
                                _p(zero_page(dy.device)), ctypes.byref(g), variant, _s()), "conv_wgrad")
    return out


def wgrad_candidates(x, dy, g, scale, only: Optional[str] = None):
    if only is not None:
        return _only_wgrad(only, x, dy, g, scale, None)
    vs = list(_WGRAD_TILE) + list(_WGRAD_PIPE_TILE) + list(_WGRAD_P8)
    c = {"hip%d" % v: (lambda v=v: conv_wgrad(x, dy, g, scale, variant=v)) for v in vs}
    if w64_covers(g):
        c["w64"] = lambda: wgrad3x3_c64(x, dy, scale)
    if whalo_covers(g):
        c["whalo"] = lambda: halo_wgrad(x, dy, g, scale)
    return c


_WGRAD_VS = None


def _only_wgrad(only, x, dy, g, scale, sink):
    """The one wgrad candidate ``only`` (plain, or accumulating into ``sink``); {} if not a candidate here
    (the library form is added by the callers)."""
    global _WGRAD_VS
    if _WGRAD_VS is None:
        _WGRAD_VS = set(list(_WGRAD_TILE) + list(_WGRAD_PIPE_TILE) + list(_WGRAD_P8))
    if only.startswith("hip") and int(only[3:]) in _WGRAD_VS:
        v = int(only[3:])
        if sink is None:
            return {only: lambda: conv_wgrad(x, dy, g, scale, variant=v)}
        return {only: lambda: conv_wgrad(x, dy, g, scale, out=sink, accumulate=True, variant=v)}
    if only == "w64" and w64_covers(g):
        if sink is None:
            return {only: lambda: wgrad3x3_c64(x, dy, scale)}
        return {only: lambda: wgrad3x3_c64(x, dy, scale, out=sink.view(64, 3, 3, 64), accumulate=True)}
    if only == "whalo" and whalo_covers(g):
        if sink is None:
            return {only: lambda: halo_wgrad(x, dy, g, scale)}
        return {only: lambda: halo_wgrad(x, dy, g, scale, out=sink.view(g.cout, 3, 3, g.cin), accumulate=True)}
    return {}


def whalo_covers(g: ConvGeom) -> bool:
    """3x3 / stride 1 / pad 1 with Cin % 64 == 0 and Cout >= 64 (single level or packed pyramid):
    csrc/kernels/wgrad_halo.hip."""
    return (g.kh == 3 and g.kw == 3 and g.stride == 1 and g.pt == 1 and g.pl == 1 and g.ostride == 1
            and g.cin % 64 == 0 and g.cout >= 64
            and all(g.H[l] == g.Ho[l] and g.W[l] == g.Wo[l] for l in range(g.nlev)))


_WH_TILES = {}


def _wh_box(h: int, w: int):
    """R x C box for a level: 2 x 64 where the level is at least 64 wide, else full-width boxes of as
    many rows as fit 128 slots / 264 halo rows.  (Measured: boxes narrower than 64 columns that waste
    fewer slots are still slower -- the per-step slot -> row / col division and shorter halo rows.)"""
    if w >= 64:
        return 2, 64
    r = max(1, min(128 // w, h))
    while r > 1 and (r + 2) * (w + 2) > 264:
        r -= 1
    return r, w


def halo_wgrad_tiles(N: int, shapes, device):
    """(tile table int4 {image, level, oy0, ox0}, per-level (R, C) boxes, #leading 2 x 64 tiles): the
    tiles of levels >= 64 wide first (the kernel's compile-time box), then the narrow levels; image /
    level / row order within each so consecutive tiles share halo rows."""
    key = (N, tuple(shapes), str(device))
    t = _WH_TILES.get(key)
    if t is None:
        boxes = [_wh_box(h, w) for h, w in shapes]
        def rows(wide):
            return [(b, l, y, x) for b in range(N) for l, (h, w) in enumerate(shapes) if (boxes[l][1] == 64) == wide
                    for y in range(0, h, boxes[l][0]) for x in range(0, w, boxes[l][1])]
        wide = rows(True)
        t = (torch.tensor(wide + rows(False), dtype=torch.int32, device=device), boxes, len(wide))
        _WH_TILES[key] = t
    return t


def halo_wgrad(x, dy, g: ConvGeom, scale=None, out: Optional[torch.Tensor] = None, accumulate: bool = False,
               splits: Optional[int] = None) -> torch.Tensor:
    """fp32 (cout, 3, 3, cin) weight gradient from halo-staged tiles (``dy`` may be wider than cout)."""
    if not whalo_covers(g):
        raise RuntimeError("wgrad_halo: geometry not covered")
    shapes = [(g.H[l], g.W[l]) for l in range(g.nlev)]
    N = int(g.M) // g.out_img
    ldy = dy.shape[-1]
    if ldy % 8:
        dy = F.pad(dy, (0, 8 - ldy % 8))
        ldy = dy.shape[-1]
    x, dy = x.contiguous(), dy.contiguous()
    if not (x.dtype == torch.bfloat16 and dy.dtype == torch.bfloat16 and x.numel() == N * g.in_img * g.cin
            and dy.numel() == N * g.out_img * ldy and g.in_img == g.out_img):
        raise RuntimeError("wgrad_halo: operands do not match the geometry")
    tiles, boxes, nwide = halo_wgrad_tiles(N, shapes, x.device)
    n_co, n_ci = -(-g.cout // 128), g.cin // 64
    if splits is None:
        splits = max(1, min(int(tiles.shape[0]), round(int(os.environ.get("MXR_WHALO_BLOCKS", "256")) / (n_co * n_ci))))
    splits = max(splits, int(nwide > 0) + int(nwide < int(tiles.shape[0])))
    ws = torch.empty(splits * g.cout * 9 * g.cin, dtype=torch.float32, device=x.device)
    if out is None:
        out = torch.empty((g.cout, 3, 3, g.cin), dtype=torch.float32, device=x.device)
        accumulate = False
    sc = None if scale is None else scale.float().contiguous()
    Hs = (ctypes.c_int * 5)(*[g.H[l] for l in range(5)])
    Ws = (ctypes.c_int * 5)(*[g.W[l] for l in range(5)])
    Os = (ctypes.c_int * 5)(*[g.in_off[l] for l in range(5)])
    Rs = (ctypes.c_int * 5)(*([b[0] for b in boxes] + [1] * (5 - len(boxes))))
    Cs = (ctypes.c_int * 5)(*([b[1] for b in boxes] + [1] * (5 - len(boxes))))
    _chk(lib().mxr_wgrad_halo(_p(x), _p(dy), ldy, _p(tiles), int(tiles.shape[0]), nwide, splits, g.nlev, Hs, Ws, Os, Rs, Cs,
                              g.in_img, g.cin, g.cout, _p(ws), _p(sc), _p(out), int(accumulate), _s()), "wgrad_halo")
    return out


def w64_covers(g: ConvGeom) -> bool:
    """3x3 / stride 1 / pad 1, 64 -> 64 channels, one level: csrc/kernels/wgrad_narrow.hip."""
    return (g.nlev == 1 and g.kh == 3 and g.kw == 3 and g.stride == 1 and g.pt == 1 and g.pl == 1 and g.cin == 64
            and g.cout == 64 and g.H[0] == g.Ho[0] and g.W[0] == g.Wo[0] and g.ostride == 1)


def wgrad3x3_c64(x, dy, scale=None, out: Optional[torch.Tensor] = None, accumulate: bool = False) -> torch.Tensor:
    """fp32 (64, 3, 3, 64) weight gradient of a 64-channel 3x3/s1 conv, ``scale`` (frozen BN) folded in."""
    N, H, W, C = x.shape
    if not (C == 64 and tuple(dy.shape) == (N, H, W, 64) and x.is_contiguous() and dy.is_contiguous()
            and x.dtype == torch.bfloat16 and dy.dtype == torch.bfloat16):
        raise RuntimeError("wgrad3x3_c64: operands not covered")
    ntiles = N * ((H + 1) // 2) * ((W + 63) // 64)
    ws = torch.empty(min(ntiles, 256) * 64 * 576, dtype=torch.float32, device=x.device)
    if out is None:
        out = torch.empty((64, 3, 3, 64), dtype=torch.float32, device=x.device)
        accumulate = False
    sc = None if scale is None else scale.float().contiguous()
    _chk(lib().mxr_wgrad3x3_c64(_p(x), _p(dy), _p(ws), _p(sc), _p(out), N, H, W, int(accumulate), _s()),
         "wgrad3x3_c64")
    return out


def bias_grad(dy: torch.Tensor, scale: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None,
              accumulate: bool = False, channels: Optional[int] = None) -> torch.Tensor:
    """``channels``: the first ``channels`` of each (wider, zero-padded) row of ``dy``."""
    ld = dy.shape[-1]
    C = channels or ld
    M = dy.numel() // ld
    C8 = (C + 7) // 8 * 8          # padded rows: sum the zero columns up to the next 8 too, write C
    if C8 > ld or C8 // 8 > 256 or ld % 8:
        db = dy.float().reshape(M, ld)[:, :C].sum(0)
        db = db * scale if scale is not None else db
        if out is None:
            return db
        return out.add_(db) if accumulate else out.copy_(db)
    if out is None:
        out = torch.empty(C, dtype=torch.float32, device=dy.device)
    part = torch.empty(512 * C8, dtype=torch.float32, device=dy.device)
    sc = None if scale is None else scale.float().contiguous()
    _chk(_bind().mxr_bias_grad(_p(dy.contiguous()), M, C8, ld, C, _p(part), _p(out), _p(sc), int(accumulate), _s()),
         "bias_grad")
    return out


def _sink(param):
    gs = _n.grad_sinks()
    return gs.get(param) if gs is not None else None


def deliver_bias_grad(param, dy, scale=None, channels: Optional[int] = None):
    """Bias gradient for ``param``: straight into its flat-gradient slot when a sink is active
    (returns None so autograd does not add it again), else a tensor."""
    sink = _sink(param)
    if sink is None:
        return bias_grad(dy, scale, channels=channels)
    if SIDE.usable(dy):
        with SIDE.run(dy.device, dy, scale):
            bias_grad(dy, scale, out=sink, accumulate=True, channels=channels)
            _n.grad_sinks().notify(param)
        return None
    bias_grad(dy, scale, out=sink, accumulate=True, channels=channels)
    _n.grad_sinks().notify(param)
    return None


# ------------------------------------------------------------------------------- autograd
def _effective(weight, scale, bias, shift):
    cw = _n.compute_weights()
    w = cw.get(weight) if cw is not None else None
    if w is None:
        w = weight if scale is None else weight * scale.view(-1, 1, 1, 1)
        w = w.to(torch.bfloat16).contiguous()
    if scale is None:
        b = None if bias is None else bias.float().contiguous()
    else:
        b = shift.float() if bias is None else bias.float() * scale + shift.float()
        b = b.contiguous()
    return w, b


def _miopen_wgrad(x, w, dy, stride, pads, scale):
    _, dw = torch_conv_backward(x, w, dy, stride, pads, False, True)
    dw = dw.float()
    return dw * scale.view(-1, 1, 1, 1) if scale is not None else dw


def _miopen_pyramid_wgrad(x, w, dy, shapes):
    """Library wgrad per pyramid level, summed (candidate for the packed head layers)."""
    N = x.shape[0]
    dw, off = None, 0
    for (h, wd) in shapes:
        xl = x[:, off:off + h * wd].reshape(N, h, wd, x.shape[-1])
        dyl = dy[:, off:off + h * wd].reshape(N, h, wd, dy.shape[-1])
        d = _miopen_wgrad(xl, w, dyl, 1, (1, 1, 1, 1), None)
        dw = d if dw is None else dw.add_(d)
        off += h * wd
    return dw


def _out_hw(H, W, kh, stride, pads):
    return (H + pads[0] + pads[1] - kh) // stride + 1, (W + pads[2] + pads[3] - kh) // stride + 1


def run_fwd(x, w, b, res, stride, pads, relu) -> torch.Tensor:
    """Tuned forward (HIP tile variants vs MIOpen + fused epilogue) of one NHWC conv."""
    from .conv_tuner import TUNER
    N, H, W, cin = x.shape
    cout, kh = w.shape[0], w.shape[1]
    Ho, Wo = _out_hw(H, W, kh, stride, pads)
    g = geom_single(N, H, W, Ho, Wo, kh, stride, pads, cin, cout)
    from . import fp8 as _f8
    f8 = "|f8" if _f8.enabled() and _f8.eligible(cin, cout) else ""
    key = TUNER.key("fwd", N, H, W, cin, cout, kh, stride, tuple(pads), int(relu), int(res is not None)) + f8
    only = _only(key)
    if only is not None:
        c = fwd_candidates(x, w, b, res, g, stride, pads, relu, (N, Ho, Wo, cout), fp8_ok=True, only=only)
        if c:
            return TUNER.run(key, c)
    return TUNER.run(key, fwd_candidates(x, w, b, res, g, stride, pads, relu, (N, Ho, Wo, cout), fp8_ok=True))


def _dgrad_cands(dy, w, x, stride, pads, mask=None, out=None, res=None, only: Optional[str] = None):
    cands = {}
    cout, kh = w.shape[0], w.shape[1]
    cin = x.shape[-1]
    if res is not None:
        assert out is None and stride == 1
        kw = dict(mask=mask, res=res)
    else:
        kw = dict(mask=mask, out=out)
    if only is not None and (only.startswith("hip") or only.startswith("c1x1_") or only.startswith("p8_")
                             or only.startswith("halo") or only.startswith("hx32_")):
        # the tuned winner among the HIP forms: every one of them is conv_dgrad with that variant
        v = int(only[3:]) if only.startswith("hip") else only
        return {only: (lambda: conv_dgrad(dy, w, tuple(x.shape), stride, pads, v, **kw))}
    if (stride == 1 or (kh == 1 and stride == 2 and tuple(pads) == (0, 0, 0, 0))
            or (kh == 3 and w.shape[2] == 3 and stride == 2)) and hip_conv_ok(cout, cin, dy.dtype):
        for v in FWD_VARIANTS:
            if v < 3 or cin % 8 == 0:
                cands["hip%d" % v] = (lambda v=v: conv_dgrad(dy, w, tuple(x.shape), stride, pads, v, **kw))
        if stride == 1 and kh == 1 and tuple(pads) == (0, 0, 0, 0) and cout in (64, 128, 256) and cin % 8 == 0:
            for bn in C1X1_BN:
                if bn * cout <= 32768 and bn <= max(64, cin):
                    cands["c1x1_%d" % bn] = (lambda bn=bn: conv_dgrad(dy, w, tuple(x.shape), stride, pads,
                                                                      "c1x1_%d" % bn, **kw))
        if stride == 1 and cout % 64 == 0 and cin % 8 == 0 and kh * w.shape[2] <= 16:
            for v in ["p8_%d" % v for v in P8_TUNED]:
                cands[v] = (lambda v=v: conv_dgrad(dy, w, tuple(x.shape), stride, pads, v, **kw))
        if stride == 1 and kh == 3 and tuple(pads) == (1, 1, 1, 1) and cout % 32 == 0 and cin % 8 == 0:
            for v in HALO_VARIANTS:
                cands["halo%d" % v] = (lambda v=v: conv_dgrad(dy, w, tuple(x.shape), stride, pads, "halo%d" % v,
                                                              **kw))
            for v in HX32_VARIANTS:
                cands["hx32_%d" % v] = (lambda v=v: conv_dgrad(dy, w, tuple(x.shape), stride, pads, "hx32_%d" % v,
                                                               **kw))

    from . import fp8 as _f8
    if (_f8.enabled() and stride == 1 and res is None and _f8.dgrad_eligible(cout, cin)
            and w.shape[1] * w.shape[2] <= 16):
        # fp8 data gradient (conv_p8_f8's e5m2 x e4m3 form; quantisation of dY and of the flipped weights
        # included in the timed candidate, so the tuner keeps it only where it wins)
        N, H, W, _ = x.shape
        k_h, k_w = w.shape[1], w.shape[2]
        dpads = (k_h - 1 - pads[0], k_h - 1 - pads[1], k_w - 1 - pads[2], k_w - 1 - pads[3])
        g8 = geom_single(N, dy.shape[1], dy.shape[2], H, W, k_h, 1, dpads, cout, cin)
        g8.kw = k_w

        def f8_dgrad(v):
            dq, idq = _f8.quantize_bf8(dy)
            wq, iw = _f8.quantize_rows(flip(w))
            dx = out if out is not None else torch.empty((N, H, W, cin), dtype=dy.dtype, device=dy.device)
            return _f8.launch(dq, idq, wq, iw, None, None, dx, g8, False, v, mask=mask, accumulate=out is not None)
        for v in _f8.F8_DGRAD_VARIANTS:
            cands["f8d_%d" % v] = (lambda v=v: f8_dgrad(v))

    def lib_path():
        dx = torch_conv_backward(x, w, dy, stride, pads, True, False)[0]
        if res is not None:
            dx = dx + res
        if out is not None:     # in place: callers (GradJoin, fused blocks) rely on ``out`` holding the result
            dx = out.add_(dx)
            if mask is not None:
                dx.masked_fill_(~(mask > 0), 0)
            return dx
        return relu_bwd(dx, mask) if mask is not None else dx
    cands["miopen"] = lib_path
    if only is not None and only in cands:
        return {only: cands[only]}
    return cands


def run_dgrad(dy, w, x, stride, pads, mask: Optional[torch.Tensor] = None,
              out: Optional[torch.Tensor] = None, res: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Tuned data gradient; ``mask`` fuses the producer's relu backward, ``out`` accumulates, ``res``
    (stride 1) is added into a fresh dX."""
    from .conv_tuner import TUNER
    N, H, W, cin = x.shape
    cout, kh = w.shape[0], w.shape[1]
    # the fused forms (relu mask / accumulation) cost the library path extra passes and the HIP
    # kernels nothing, so they are tuned as their own keys
    # (``res`` costs what accumulation does -- one more dX-sized read -- and shares its key)
    key = TUNER.key("dgrad", N, H, W, cin, cout, kh, stride, tuple(pads)) + \
        ("|m" if mask is not None else "") + ("|a" if (out is not None or res is not None) else "")
    only = _only(key)
    cands = _dgrad_cands(dy, w, x, stride, pads, mask, out, res, only=only) if only is not None else None
    if not cands:
        cands = _dgrad_cands(dy, w, x, stride, pads, mask, out, res)
    if out is not None and TUNER.needs_tuning(key, cands):
        # time the accumulating candidates against a scratch copy, then run the winner for real
        TUNER.run(key, _dgrad_cands(dy, w, x, stride, pads, mask, out.clone()))
    return TUNER.run(key, cands)


def _deliver_wgrad(key, cands, sink_cands, param, reads=()):
    """Run the tuned wgrad; with a gradient sink for ``param`` accumulate into it and return None.
    Once the sink form is tuned it runs on the side stream (``ops.side_stream``), overlapped with the
    data gradients; ``reads`` = the compute-stream tensors it reads (x, dY, scale)."""
    from .conv_tuner import TUNER
    sink = _sink(param)
    if sink is None:
        return TUNER.run(key, cands() if callable(cands) else cands)
    key = key + "|s"        # accumulate-into-sink forms: the library path pays an extra add
    only = _only(key)
    c = sink_cands(sink, only) if only is not None else None
    if not c:
        c = sink_cands(sink)
        if TUNER.needs_tuning(key, c):
            TUNER.run(key, sink_cands(sink.clone()))    # time against a scratch copy of the slot
            c = sink_cands(sink)
            TUNER.run(key, c)
            _n.grad_sinks().notify(param)
            return None
    if SIDE.usable(sink):
        with SIDE.run(sink.device, *reads):
            TUNER.run(key, c)
            _n.grad_sinks().notify(param)
        return None
    TUNER.run(key, c)
    _n.grad_sinks().notify(param)
    return None


def _wgrad_sink_cands(x, dy, g, scale, lib_fn):
    def make(sink, only=None):
        if only is not None:
            if only == "miopen":
                return {only: lambda: sink.add_(lib_fn())}
            return _only_wgrad(only, x, dy, g, scale, sink)
        vs = list(_WGRAD_TILE) + list(_WGRAD_PIPE_TILE) + list(_WGRAD_P8)
        c = {"hip%d" % v: (lambda v=v: conv_wgrad(x, dy, g, scale, out=sink, accumulate=True, variant=v)) for v in vs}
        c["miopen"] = lambda: sink.add_(lib_fn())
        if w64_covers(g):
            c["w64"] = lambda: wgrad3x3_c64(x, dy, scale, out=sink.view(64, 3, 3, 64), accumulate=True)
        if whalo_covers(g):
            c["whalo"] = lambda: halo_wgrad(x, dy, g, scale, out=sink.view(g.cout, 3, 3, g.cin), accumulate=True)
        return c
    return make


def run_wgrad(x, dy, w, stride, pads, scale, param=None) -> Optional[torch.Tensor]:
    """Tuned fp32 weight gradient (OHWI), scaled by the folded frozen-BN scale.  With an active
    gradient sink for ``param`` it is accumulated into the flat gradient buffer (returns None)."""
    from .conv_tuner import TUNER
    N, H, W, cin = x.shape
    cout, kh = w.shape[0], w.shape[1]
    Ho, Wo = dy.shape[1], dy.shape[2]
    g = geom_single(N, H, W, Ho, Wo, kh, stride, pads, cin, cout)
    lib_fn = lambda: _miopen_wgrad(x, w, dy, stride, pads, scale)   # noqa: E731

    def cands():        # built only without a gradient sink (the training step always has one)
        c = wgrad_candidates(x, dy, g, scale)
        c["miopen"] = lib_fn
        return c
    key = TUNER.key("wgrad", N, H, W, cin, cout, kh, stride, tuple(pads))
    return _deliver_wgrad(key, cands, _wgrad_sink_cands(x, dy, g, scale, lib_fn), param, (x, dy, scale))


class GradJoin:
    """Input-gradient join for a ReLU output consumed by ``n`` HIP conv nodes (C3 / C4 / C5: the next
    ResNet stage and the FPN lateral / P6 convs).

    Autograd would hand each consumer's dX to a separate buffer, add them, and the producing block
    would then run a ReLU backward over the sum -- two activation-sized passes.  Instead the first
    consumer to run writes its dX (unmasked) and returns it; the others accumulate into that same
    buffer through their dgrad epilogues (and return None); the LAST one also applies the ReLU mask
    (accumulate-then-mask), so the producer skips its ReLU backward (``grad_premasked``).
    Autograd runs every consumer before the producer, so the buffer is complete when it is read.
    """

    def __init__(self, n: int):
        self.n = n
        self._buf = None
        self.seen = 0
        self._owner = None      # stream the buffer was written on (consumers may run on two streams:
        self._event = None      # the head towers, RetinaNet.forward)

    @property
    def buf(self):
        return self._buf

    @buf.setter
    def buf(self, t):
        self._buf = t
        if t is not None and t.is_cuda:
            self._owner = torch.cuda.current_stream(t.device)
            self._event = torch.cuda.Event()
            self._event.record(self._owner)

    def claim(self):
        """-> (buffer to accumulate into or None, whether this consumer is the last).  A consumer on
        another stream than the buffer's writer first waits for that write."""
        self.seen += 1
        if self._buf is not None and self._owner is not None:
            cur = torch.cuda.current_stream(self._buf.device)
            if cur.cuda_stream != self._owner.cuda_stream:
                cur.wait_event(self._event)
        return self._buf, self.seen == self.n

    def release(self):
        """After accumulating into the buffer: autograd hands it on from the writer's stream, so that
        stream waits for an accumulation made on another one (no-op on the same stream)."""
        if self._buf is not None and self._owner is not None:
            cur = torch.cuda.current_stream(self._buf.device)
            if cur.cuda_stream != self._owner.cuda_stream:
                self._owner.wait_stream(cur)


class ConvLayerFn(torch.autograd.Function):
    """y = act(conv(x, W*s) + (b*s + t) [+ residual]) with fp32 master W/b; NHWC bf16 x/y.

    Every pass (fwd / dgrad / wgrad) is dispatched per shape by :data:`conv_tuner.TUNER` between
    the HIP implicit-GEMM kernels and the MIOpen path (whichever measured faster on this GPU).
    """

    @staticmethod
    def forward(ctx, x, weight, bias, scale, shift, stride, pads, relu, residual, join=None):
        x = x.contiguous()
        w, b = _effective(weight, scale, bias, shift)
        res = None if residual is None else residual.contiguous()
        y = run_fwd(x, w, b, res, stride, pads, relu)
        ctx.params = (weight, bias)
        ctx.save_for_backward(x, w, y if relu else None, scale)
        ctx.cfg = (stride, tuple(pads), relu, bias is not None, residual is not None)
        ctx.join = join
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w, y, scale = ctx.saved_tensors
        stride, pads, relu, has_bias, has_res = ctx.cfg
        dy = dy.to(x.dtype).contiguous()
        if relu:
            dy = relu_bwd(dy, y)
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            if ctx.join is not None:
                buf, last = ctx.join.claim()
                r = run_dgrad(dy, w, x, stride, pads, mask=x if last else None, out=buf)
                if buf is None:
                    ctx.join.buf = dx = r
                else:
                    if r is not buf:
                        buf.copy_(r)
                    ctx.join.release()
            else:
                dx = run_dgrad(dy, w, x, stride, pads)
        if ctx.needs_input_grad[1]:
            dw = run_wgrad(x, dy, w, stride, pads, scale, param=ctx.params[0])
        if has_bias and ctx.needs_input_grad[2]:
            db = deliver_bias_grad(ctx.params[1], dy, scale)
        if has_res:
            # dy becomes the residual's gradient, which autograd may accumulate into in place when it holds
            # the only reference: keep one until the side-stream wgrad / bias grad reading it has run
            SIDE.keep(dy)
        return dx, dw, db, None, None, None, None, None, (dy if has_res else None), None


# A premasked block's incoming gradient is the next block's dX, which only this node consumes (the
# block chain inside a stage is linear), so the identity-shortcut dX may accumulate into it in place
# instead of into a copy (one activation-sized copy per identity block). MXR_INPLACE_BLOCK_GRAD=0 copies.
_INPLACE_GRAD = os.environ.get("MXR_INPLACE_BLOCK_GRAD", "1") == "1"


class ResidualBlockFn(torch.autograd.Function):
    """A whole ResNet block (bottleneck or basic) as ONE autograd node on the HIP path.

    Forward: h1 = relu(conv_0(x)), ..., out = relu(conv_last(h_L) + shortcut), shortcut = x or
    branch1(x) -- each conv a tuned fused-epilogue launch.  Backward, with the block's structure
    known: ONE relu backward (of ``out``); every inner relu backward is fused into the data-gradient
    epilogue that produces it (mask = the saved relu output, which is that conv's input); the data
    gradient of the first conv ACCUMULATES into the shortcut's gradient buffer (no separate add).
    Per-conv algorithm choice (HIP variants / MIOpen) stays with the tuner, keyed like ConvLayerFn.
    ``specs`` = ((stride, pads) for conv_0..conv_last, then branch1 or None).
    """

    @staticmethod
    def forward(ctx, x, specs, flags, join, *params):
        x = x.contiguous()
        nconv = len(specs) - 1
        ctx.mask_in, ctx.premasked = flags
        ctx.join = join
        ws, scales = [], []
        for i in range(nconv + 1):
            wt, sc, sh = params[3 * i:3 * i + 3]
            if wt is None:
                ws.append(None)
                scales.append(None)
                continue
            w, b = _effective(wt, sc, None, sh)
            ws.append((w, b))
            scales.append(sc)
        if specs[nconv] is not None:
            st, pd = specs[nconv]
            shortcut = run_fwd(x, ws[nconv][0], ws[nconv][1], None, st, pd, False)
        else:
            shortcut = x
        hs = [x]
        h = x
        for i in range(nconv):
            st, pd = specs[i]
            last = i == nconv - 1
            h = run_fwd(h, ws[i][0], ws[i][1], shortcut if last else None, st, pd, True)
            hs.append(h)
        ctx.specs = specs
        ctx.nconv = nconv
        ctx.has_b1 = specs[nconv] is not None
        ctx.wparams = [params[3 * i] for i in range(nconv + 1)]
        present = [i for i in range(nconv + 1) if ws[i] is not None]
        ctx.save_for_backward(*(hs + [ws[i][0] for i in present] + [scales[i] for i in present]))
        return h

    @staticmethod
    def backward(ctx, dout):
        specs, nconv = ctx.specs, ctx.nconv
        saved = ctx.saved_tensors
        hs = saved[:nconv + 1]
        nw = nconv + (1 if ctx.has_b1 else 0)
        ws = list(saved[nconv + 1:nconv + 1 + nw])
        scs = list(saved[nconv + 1 + nw:])
        out = hs[-1]
        g = dout.to(out.dtype).contiguous()
        if not ctx.premasked:       # else the next block already applied this relu's backward
            g = relu_bwd(g, out)
        elif g is dout and not ctx.has_b1 and ctx.needs_input_grad[0] and not _INPLACE_GRAD:
            g = g.clone()           # g becomes dX (identity-shortcut accumulation): own the buffer
        grads = [None] * (3 * (nconv + 1))
        need_x = ctx.needs_input_grad[0]
        # shortcut first: its gradient buffer becomes dX, which conv_0's dgrad accumulates into
        dx = None
        jbuf, jlast, mask_in, post_mask = None, False, ctx.mask_in, False
        if ctx.join is not None and need_x:
            # x has other consumers (GradJoin): accumulate into the shared buffer if one exists, mask
            # only if this is the last consumer.  A strided (1x1/s2) scatter dgrad only visits every
            # other pixel, so then the mask goes over the whole buffer after the accumulation.
            jbuf, jlast = ctx.join.claim()
            strided = specs[0][0] != 1 or (ctx.has_b1 and specs[nconv][0] != 1)
            mask_in = jlast and not strided
            post_mask = jlast and strided
        if ctx.has_b1:
            st, pd = specs[nconv]
            if ctx.needs_input_grad[4 + 3 * nconv]:
                grads[3 * nconv] = run_wgrad(hs[0], g, ws[nconv], st, pd, scs[nconv], param=ctx.wparams[nconv])
            if need_x:
                dx = run_dgrad(g, ws[nconv], hs[0], st, pd, out=jbuf)
        gi = g
        for i in range(nconv - 1, -1, -1):
            st, pd = specs[i]
            if ctx.needs_input_grad[4 + 3 * i]:
                grads[3 * i] = run_wgrad(hs[i], gi, ws[i], st, pd, scs[i], param=ctx.wparams[i])
            if i > 0:
                gi = run_dgrad(gi, ws[i], hs[i], st, pd, mask=hs[i])
            elif need_x:
                mk = hs[0] if mask_in else None
                if dx is None and jbuf is None and st == 1 and SIDE.usable(g):
                    # identity shortcut while side-stream wgrads may still read g: dX = dgrad + g into a
                    # fresh buffer (same traffic as accumulating into g, which is left untouched)
                    dx = run_dgrad(gi, ws[0], hs[0], st, pd, res=g, mask=mk)
                else:
                    if dx is None:
                        if jbuf is not None:             # identity shortcut into a joined buffer
                            dx = jbuf.add_(g)
                        else:
                            dx = g if gi is not g else g.clone()    # identity shortcut: g is ours, reuse it
                    # x is the previous block's relu output and we are its only consumer: fuse that
                    # relu backward into this (accumulating) dgrad epilogue
                    dx = run_dgrad(gi, ws[0], hs[0], st, pd, out=dx, mask=mk)
        if post_mask:
            relu_bwd_(dx, hs[0])
        if ctx.join is not None and need_x:
            if jbuf is None:
                ctx.join.buf = dx
            else:
                if dx is not jbuf:
                    jbuf.copy_(dx)
                ctx.join.release()
                dx = None                            # already accumulated into the first consumer's dX
        return (dx, None, None, None) + tuple(grads)


def residual_block(x, convs, branch1, mask_input_grad: bool = False, grad_premasked: bool = False,
                   join: Optional[GradJoin] = None) -> torch.Tensor:
    """Run ``convs`` (models.layers.Conv2D chain, the last one takes the residual) and the optional
    projection ``branch1`` as one :class:`ResidualBlockFn` node.

    ``mask_input_grad``: x is a relu output consumed only by this block (its relu backward is fused
    into this block's last dgrad); ``grad_premasked``: the next block does that for our output."""
    specs, params = [], []
    hw = tuple(x.shape[1:3])
    for c in convs:
        specs.append((c.stride, tuple(c.pads(hw))))
        hw = c.out_hw(hw)
    specs.append(None if branch1 is None else (branch1.stride, tuple(branch1.pads(tuple(x.shape[1:3])))))
    for c in list(convs) + [branch1]:
        if c is None:
            params += [None, None, None]
            continue
        sc, sh = c.bn.scale_shift() if c.bn is not None else (None, None)
        params += [c.weight, sc, sh]
    return ResidualBlockFn.apply(x, tuple(specs), (bool(mask_input_grad), bool(grad_premasked)), join, *params)


def fused_block_ok(x, convs) -> bool:
    return (os.environ.get("MXR_FUSED_BLOCKS", "1") == "1" and x.is_cuda and x.dtype == torch.bfloat16
            and all(c is None or (hip_conv_ok(c.cin, c.cout, x.dtype) and c.bias is None) for c in convs))


class PyramidConvFn(torch.autograd.Function):
    """Shared 3x3/s1/'same' conv over packed pyramid levels [B, P, C] (batch-major): all five
    levels as ONE ragged implicit GEMM per pass (the HIP kernel's multi-level geometry)."""

    @staticmethod
    def forward(ctx, x, weight, bias, shapes, relu, mask_input_grad=False, grad_premasked=False, pad_sink=None,
                join=None):
        from .conv_tuner import TUNER
        x = x.contiguous()
        N, P, cin = x.shape
        cout = weight.shape[0]
        w, b = _effective(weight, None, bias, None)
        ctx.wdt = weight.dtype
        g = geom_pyramid(N, shapes, cin, cout)
        from . import fp8 as _f8
        if _f8.enabled() and _f8.eligible(cin, cout):
            y = _f8.pyramid_forward(x, w, b, g, relu, (N, P, cout), id(weight),
                                    TUNER.key("pfwd", N, tuple(shapes), cin, cout, int(relu)) + "|f8")
        else:
            key = TUNER.key("pfwd", N, tuple(shapes), cin, cout, int(relu))
            cands = fwd_candidates(x, w, b, None, g, 1, (1, 1, 1, 1), relu, (N, P, cout), allow_miopen=False)
            if cout % 8 and cout < 64:
                cands["pad64"] = lambda: _pad64_pfwd(x, w, b, shapes, relu)
            y = TUNER.run(key, cands)
        ctx.save_for_backward(x, w, y if relu else None)
        ctx.params = (weight, bias)
        ctx.cfg = (tuple(shapes), relu, bias is not None, bool(mask_input_grad), bool(grad_premasked))
        ctx.pad_sink = pad_sink
        ctx.join = join
        return y

    @staticmethod
    def backward(ctx, dy):
        from .conv_tuner import TUNER
        x, w, y = ctx.saved_tensors
        shapes, relu, has_bias, mask_in, premasked = ctx.cfg
        N, P, cin = x.shape
        cout = w.shape[0]
        padded = ctx.pad_sink.pop("dy", None) if ctx.pad_sink is not None else None
        if padded is not None:
            # the loss kernel wrote this layer's gradient straight into zero-padded [N, P, 64k] rows
            # (Trainer._losses_backward); autograd only carried a placeholder
            dy = padded
        else:
            dy = dy.to(x.dtype).contiguous()
        if relu and not premasked:
            dy = relu_bwd(dy, y)
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            wd = flip(w)
            dyp = dy
            if cout % 64:
                # head final layers (720 / 36 outputs): pad the K dimension of the data-gradient GEMM
                cp = (cout + 63) // 64 * 64
                if dyp.shape[-1] != cp:
                    dyp = F.pad(dy, (0, cp - cout))
                wd = F.pad(wd, (0, cp - cout))
            wd = wd.contiguous()
            gd = geom_pyramid(N, shapes, dyp.shape[-1], cin)
            key = TUNER.key("pdgrad", N, tuple(shapes), cin, cout)
            buf = None
            if ctx.join is not None:
                # both head towers read the packed features: the second dgrad accumulates into the first's dX
                buf, _ = ctx.join.claim()
            from . import fp8 as _f8
            if _f8.enabled() and _f8.dgrad_eligible(dyp.shape[-1], cin):
                # fp8 data gradient (e5m2 dY x e4m3 W); a tower layer's dX is the next data gradient's dY, so
                # its e5m2 copy comes out of this epilogue (mask_in: x is a tower layer's relu output)
                r = _f8.pyramid_dgrad(dyp, wd, gd, x if mask_in else None, (N, P, cin), ("pdgrad", id(ctx.params[0])),
                                      key + ("|a" if buf is not None else "") + "|f8", emit=mask_in, out=buf)
                if buf is None:
                    dx = r
                    if ctx.join is not None:
                        ctx.join.buf = dx
                else:
                    ctx.join.release()
                    dx = None
            elif buf is None:
                dx = TUNER.run(key, fwd_candidates(dyp, wd, None, None, gd, 1, (1, 1, 1, 1), False, (N, P, cin),
                                                   allow_miopen=False, mask=x if mask_in else None))
                if ctx.join is not None:
                    ctx.join.buf = dx
            else:
                mk = x if mask_in else None
                cands = fwd_candidates(dyp, wd, None, None, gd, 1, (1, 1, 1, 1), False, (N, P, cin),
                                       allow_miopen=False, mask=mk, out=buf)
                if TUNER.needs_tuning(key + "|a", cands):
                    TUNER.run(key + "|a", fwd_candidates(dyp, wd, None, None, gd, 1, (1, 1, 1, 1), False,
                                                         (N, P, cin), allow_miopen=False, mask=mk, out=buf.clone()))
                TUNER.run(key + "|a", cands)
                ctx.join.release()
                dx = None
        if ctx.needs_input_grad[1]:
            gw = geom_pyramid(N, shapes, cin, cout)
            cands = wgrad_candidates(x, dy, gw, None)
            dyl = dy if dy.shape[-1] == cout else dy[..., :cout]
            lib_fn = lambda: _miopen_pyramid_wgrad(x, w, dyl, shapes)   # noqa: E731
            cands["miopen"] = lib_fn
            sink_make = _wgrad_sink_cands(x, dy, gw, None, lib_fn)
            if cout % 8 and cout < 64:
                # narrow regression final (36): the 64-wide pipelined wgrad on zero-padded dY rows
                pad_fn = lambda: _pad64_pwgrad(x, dy, shapes, cout)   # noqa: E731
                cands["pad64"] = pad_fn
                base_make = sink_make

                def sink_make(sink, only=None, base_make=base_make, pad_fn=pad_fn):
                    if only == "pad64":
                        return {only: lambda: sink.add_(pad_fn())}
                    c = base_make(sink, only)
                    if only is None:
                        c["pad64"] = lambda: sink.add_(pad_fn())
                    return c
            dw = _deliver_wgrad(TUNER.key("pwgrad", N, tuple(shapes), cin, cout), cands, sink_make, ctx.params[0],
                                (x, dy))
            if dw is not None:
                dw = dw.to(ctx.wdt)
        if has_bias and ctx.needs_input_grad[2]:
            db = deliver_bias_grad(ctx.params[1], dy, channels=cout)
        return dx, dw, db, None, None, None, None, None, None


def _pad64_pfwd(x, w, b, shapes, relu):
    """Narrow pyramid conv (cout < 64, e.g. the 36-output regression final) on the 64-wide kernels:
    zero weight rows, then the first ``cout`` channels copied out (a 25 MB copy vs a 2x faster GEMM)."""
    from .conv_tuner import TUNER
    N, P, cin = x.shape
    cout = w.shape[0]
    wp = F.pad(w, (0, 0, 0, 0, 0, 0, 0, 64 - cout)).contiguous()
    bp = None if b is None else F.pad(b, (0, 64 - cout)).contiguous()
    gp = geom_pyramid(N, shapes, cin, 64)
    yp = TUNER.run(TUNER.key("pfwd", N, tuple(shapes), cin, 64, int(relu), "pad"),
                   fwd_candidates(x, wp, bp, None, gp, 1, (1, 1, 1, 1), relu, (N, P, 64), allow_miopen=False))
    return yp[..., :cout].contiguous()


def _pad64_pwgrad(x, dy, shapes, cout):
    """fp32 (cout, 3, 3, cin) weight gradient of a narrow pyramid conv through the 64-wide kernels."""
    from .conv_tuner import TUNER
    N, P, cin = x.shape
    dyp = dy if dy.shape[-1] == 64 else F.pad(dy[..., :cout], (0, 64 - cout)).contiguous()
    gp = geom_pyramid(N, shapes, cin, 64)
    dw = TUNER.run(TUNER.key("pwgrad", N, tuple(shapes), cin, 64, "pad"), wgrad_candidates(x, dyp, gp, None))
    return dw[:cout]


def conv_layer(x, layer, residual=None, relu=None, join: Optional[GradJoin] = None) -> torch.Tensor:
    """Run a models.layers.Conv2D through the HIP kernels (falls back when uncovered)."""
    relu = layer.relu if relu is None else relu
    pads = layer.pads(x.shape[1:3])
    scale = shift = None
    if layer.bn is not None:
        scale, shift = layer.bn.scale_shift()
    if not hip_conv_ok(layer.cin, layer.cout, x.dtype):
        if join is not None:
            raise RuntimeError("GradJoin consumer %s is not on the HIP conv path" % layer.keras_name)
        from .conv import _conv_torch
        w, b = layer.effective(x.dtype)
        return _conv_torch(x, w, b, layer.stride, pads, relu, residual)
    return ConvLayerFn.apply(x, layer.weight, layer.bias, scale, shift, layer.stride, tuple(pads), bool(relu),
                             residual, join)


def _pyr_pack(packed: torch.Tensor, levels, shapes, unpack: bool) -> None:
    ptrs = (c_vp * 5)(*([t.data_ptr() for t in levels] + [None] * (5 - len(levels))))
    hw = (c_int * 5)(*([h * w for h, w in shapes] + [0] * (5 - len(shapes))))
    _chk(lib().mxr_pyr_pack(_p(packed), ptrs, hw, len(levels), packed.shape[0], packed.shape[-1], int(unpack), _s()),
         "pyr_pack")


class PyramidPackFn(torch.autograd.Function):
    """FPN outputs [N, h_l, w_l, C] -> the heads' packed [N, P, C] in one launch (``mxr_pyr_pack``); the
    backward scatters the packed gradient into CONTIGUOUS per-level gradients in one launch, so the
    P3-P7 output convs' backward reads them as is (torch.cat's backward hands them strided slices,
    which each cost a generic strided copy).  Reference: the heads run on every pyramid level,
    keras_retinanet/models/retinanet.py ``__build_pyramid`` (``/root/reference/train.py:91``)."""

    @staticmethod
    def forward(ctx, *xs):
        N, C = xs[0].shape[0], xs[0].shape[-1]
        shapes = tuple((int(x.shape[1]), int(x.shape[2])) for x in xs)
        ctx.shapes = shapes
        packed = torch.empty((N, sum(h * w for h, w in shapes), C), dtype=xs[0].dtype, device=xs[0].device)
        _pyr_pack(packed, [x.contiguous() for x in xs], shapes, False)
        return packed

    @staticmethod
    def backward(ctx, dp):
        dp = dp.contiguous()
        N, C = dp.shape[0], dp.shape[-1]
        outs = [torch.empty((N, h, w, C), dtype=dp.dtype, device=dp.device) for h, w in ctx.shapes]
        _pyr_pack(dp, outs, ctx.shapes, True)
        return tuple(outs)


def pyramid_pack(xs: Sequence[torch.Tensor]):
    N = xs[0].shape[0]
    C = xs[0].shape[-1]
    shapes = tuple((int(x.shape[1]), int(x.shape[2])) for x in xs)
    if (xs[0].is_cuda and xs[0].dtype == torch.bfloat16 and C % 8 == 0 and 1 <= len(xs) <= 5
            and all(x.dtype == xs[0].dtype and x.shape[0] == N and x.shape[-1] == C for x in xs)):
        return PyramidPackFn.apply(*xs), shapes
    packed = torch.cat([x.reshape(N, -1, C) for x in xs], dim=1)
    return packed, shapes


def pyramid_conv_layer(x, shapes, layer, relu, mask_input_grad=False, grad_premasked=False,
                       pad_sink=None, join=None) -> torch.Tensor:
    """``mask_input_grad``: x is a relu output whose only consumer is this layer -> its relu backward
    is fused into this layer's dgrad; ``grad_premasked``: the (sole) consumer of this layer's relu
    output does that, so skip the relu backward here."""
    return PyramidConvFn.apply(x, layer.weight, layer.bias, tuple(shapes), bool(relu), bool(mask_input_grad),
                               bool(grad_premasked), pad_sink, join)


def pyramid_unpack(y, shapes):
    out, off = [], 0
    N = y.shape[0]
    for (h, wd) in shapes:
        out.append(y[:, off:off + h * wd].reshape(N, h, wd, -1))
        off += h * wd
    return out


# ---------------------------------------------------------------- raw-weight helpers (tests)
class _RawConvFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, bias, stride, pads, relu, residual):
        ctx.wdt = w.dtype
        return ConvLayerFn.forward(ctx, x, w.float(), bias, None, None, stride, pads, relu, residual)

    @staticmethod
    def backward(ctx, dy):
        dx, dw, db, *_rest, dres = ConvLayerFn.backward(ctx, dy)
        return dx, (None if dw is None else dw.to(ctx.wdt)), db, None, None, None, dres


def conv2d(x, w, bias, stride, pads, relu, residual):
    """Functional conv with an explicit (bf16 or fp32) OHWI weight."""
    if not hip_conv_ok(x.shape[-1], w.shape[0], x.dtype):
        from .conv import _conv_torch
        return _conv_torch(x, w, bias, stride, pads, relu, residual)
    return _RawConvFn.apply(x, w, bias, stride, tuple(pads), bool(relu), residual)


def pyramid_conv_packed(x, shapes, w, bias, relu):
    return PyramidConvFn.apply(x, w, bias, tuple(shapes), bool(relu))


def pyramid_conv(xs, w, bias, relu):
    packed, shapes = pyramid_pack(xs)
    return pyramid_unpack(pyramid_conv_packed(packed, shapes, w, bias, relu), shapes)
