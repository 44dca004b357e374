"""Convolution kernel launchers, geometry and the forward candidate sets (split out of ``native_conv``).

One function per HIP kernel family -- ``conv_igemm.hip`` / ``conv_pipe.hip`` (``launch_fwd``),
``conv_p8.hip``, ``conv1x1_stream.hip``, ``conv_halo.hip``, ``conv_hx32.hip`` -- with the shape checks the
kernels assume, the library (MIOpen) forms, and ``fwd_candidates`` / ``run_fwd``: the tuned forward of the
conv layers the reference builds at /root/reference/train.py:91.
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
    return 1 if cout <= 64 else 0

class BitMask:
    """The ReLU mask of a bf16 NHWC activation as one bit per element (uint8 per 8 channels: 1/16 of the
    activation's bytes), for the data gradient that fuses that ReLU's backward.  It reaches the HIP kernels
    as their mask pointer with bit 0 set (csrc/kernels/conv_common.h, ``epi_mask8``): a forward epilogue
    with ReLU WRITES it for its own output, a data-gradient epilogue READS it instead of the activation.
    Only the kernels whose epilogues go through those helpers take it (:func:`bits_capable`).
    ``MXR_MASK_BITS=0`` keeps the bf16 activation as the mask everywhere."""
    __slots__ = ("bits", "shape", "device")
    is_cuda = True

    def __init__(self, like: Optional[torch.Tensor] = None, shape: Optional[Sequence[int]] = None, device=None):
        """The bitmask of an activation shaped like ``like`` (or of ``shape`` on ``device``)."""
        if like is not None:
            shape, device = like.shape, like.device
        shape = tuple(int(v) for v in shape)
        n = 1
        for v in shape:
            n *= v
        assert shape[-1] % 8 == 0 and torch.device(device).type == "cuda"
        self.bits = torch.empty(n // 8, dtype=torch.uint8, device=device)
        self.shape, self.device = shape, torch.device(device)

    def data_ptr(self) -> int:
        return self.bits.data_ptr() | 1

    def record_stream(self, s) -> None:
        self.bits.record_stream(s)

    @classmethod
    def of(cls, t: torch.Tensor) -> "BitMask":
        """The bitmask of ``t > 0`` built with torch ops (tests; the model's come from the epilogues)."""
        bm = cls(t)
        sh = torch.arange(8, device=t.device, dtype=torch.int32)
        bm.bits.copy_(((t.reshape(-1, 8) > 0).to(torch.int32) << sh).sum(1).to(torch.uint8))
        return bm

    def dense(self) -> torch.Tensor:
        """bool tensor of ``shape`` (tests / debugging)."""
        sh = torch.arange(8, device=self.bits.device, dtype=torch.uint8)
        return ((self.bits[:, None] >> sh) & 1).bool().reshape(self.shape)

MASK_BITS = os.environ.get("MXR_MASK_BITS", "1") == "1"

def bits_capable(name: str) -> bool:
    """Tuner candidates whose epilogue handles a :class:`BitMask` (conv_pipe, split-K pipe, streaming 1x1,
    halo and hx32 kernels; not the igemm hip0-2 / p8 direct epilogues, MIOpen or fp8)."""
    if name.startswith(("c1x1_", "sk", "halo", "hx32_")) or name == "c1p":
        return True
    return name.startswith("hip") and name[3:].isdigit() and int(name[3:]) >= 3

def _bits_filter(cands, mask):
    if not isinstance(mask, BitMask):
        return cands
    return {k: v for k, v in cands.items() if bits_capable(k)}

def launch_fwd(x, w, bias, res, y, g: ConvGeom, relu: bool, accumulate: bool = False,
               variant: Optional[int] = None, mask: Optional[torch.Tensor] = None) -> None:
    """One implicit-GEMM launch.  ``mask``: zero the output where ``mask <= 0`` (fused relu backward
    of the layer that produced this conv's input); ``accumulate``: ``y += result``."""
    v = _variant(g.cout) if variant is None else variant
    zp = _p(zero_page(x.device))
    if isinstance(v, str) and v.startswith("c1x1_"):   # streaming narrow-K 1x1 kernel (conv1x1_stream.hip)
        launch_c1x1(x, w, bias, res, y, g, relu, accumulate, int(v[5:]), mask)
        return
    if v == "c1p":      # persistent streaming 1x1 kernel (conv1x1_pers.hip)
        launch_c1p(x, w, bias, res, y, g, relu, accumulate, mask)
        return
    if isinstance(v, str) and v.startswith("hx32_"):   # 32x32x16-MFMA halo kernel (conv_hx32.hip)
        launch_hx32(x, w, bias, res, y, g, relu, accumulate, int(v[5:]), mask)
        return
    if isinstance(v, str) and v.startswith("sk"):    # split-K form of the 128-pixel pipe tiles (conv_pipe.hip)
        launch_splitk(x, w, bias, res, y, g, relu, accumulate, int(v[2:]), mask)
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

HX32_VARIANTS = (0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15)   # 2 / 3: persistent grid, 4 / 5: 64-B halo rows, 6: one halo buffer (2 blocks / CU), 7: 3-slot weight ring, 8 / 9: 64-channel tiles (9: one halo buffer), 10-15: 0 / 6 / 1 / 2 / 3 / 7 on the 16x16x32 MFMA
HX32_NARROW = (8, 9)     # the 64-channel tiles: offered only to layers with cout <= 64


NARROW_TILES = True      # (a switch for same-process A/Bs, scripts/bench_switch.py; not an environment knob)


def hx32_variants(g: ConvGeom):
    return tuple(v for v in HX32_VARIANTS if v not in HX32_NARROW or (g.cout <= 64 and NARROW_TILES))

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

SK_VARIANTS = (11, 12)     # conv_pipe variants 11 (128 co x 128 px) / 12 (64 co x 128 px) split over K


def splitk_splits(g: ConvGeom, v: int) -> int:
    """K splits of the split-K pipe form for ``g``: only grids under one round of the chip (the FPN P6 /
    P7 convs: 20-70 tiles of 72-576 K sub-stages), aiming at ~512 blocks with >= 8 sub-stages per split;
    0 = not a candidate."""
    if g.ostride != 1 or g.cin % 32 or g.cout % 8:
        return 0
    bco = 128 if v == 11 else 64
    tiles = -(-int(g.M) // 128) * -(-g.cout // bco)
    nks = g.kh * g.kw * g.cin // 32
    if tiles >= 256 or nks < 16:
        return 0
    s = min(64, max(2, round(512 / tiles)), nks // 8)
    return s if s >= 2 else 0


def launch_splitk(x, w, bias, res, y, g: ConvGeom, relu: bool, accumulate: bool = False, variant: int = 11,
                  mask: Optional[torch.Tensor] = None) -> None:
    """Split-K pipe conv: fp32 partial tiles per K split, then one epilogue pass (csrc/kernels/conv_pipe.hip)."""
    ns = splitk_splits(g, variant)
    if ns < 2:
        raise RuntimeError("conv_fwd_pipe_sk: geometry not covered")
    part = torch.empty(ns * int(g.M) * g.cout, dtype=torch.float32, device=y.device)
    _chk(lib().mxr_conv_fwd_pipe_sk(_p(x), _p(w), _p(bias), _p(res), _p(mask), _p(y), _p(zero_page(x.device)),
                                    ctypes.byref(g), int(relu), int(accumulate), int(variant), ns, _p(part), _s()),
         "conv_fwd_pipe_sk")


def c1x1_variants(g: ConvGeom):
    """Streaming 1x1 kernel variants covering ``g`` (1x1, no padding, single level, K in 64/128/256)."""
    if not (g.kh == 1 and g.kw == 1 and g.nlev == 1 and g.ostride == 1 and g.pt == 0 and g.pl == 0
            and g.stride in (1, 2) and g.cin in (64, 128, 256) and g.cout % 8 == 0):
        return []
    if g.stride == 1 and (g.H[0] != g.Ho[0] or g.W[0] != g.Wo[0]):
        return []
    # 65 = the 64-cout slice with its epilogue operands prefetched a tile ahead
    eff = lambda bn: 64 if bn == 65 else bn   # noqa: E731
    return ["c1x1_%d" % bn for bn in C1X1_BN + (65,) if eff(bn) * g.cin <= 32768 and eff(bn) <= max(64, g.cout)]

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

def c1p_covers(g: ConvGeom) -> bool:
    """The persistent 1x1 kernel (csrc/kernels/conv1x1_pers.hip): 1x1 / stride 1 / no padding, one level, no
    strided output scatter, K = cin % 32 == 0 and >= 96, cout % 8 == 0 (at least one 64-channel half tile)."""
    return (g.kh == 1 and g.kw == 1 and g.nlev == 1 and g.ostride == 1 and g.pt == 0 and g.pl == 0
            and g.stride == 1 and g.H[0] == g.Ho[0] and g.W[0] == g.Wo[0] and g.cin % 32 == 0 and g.cin >= 96
            and g.cout % 8 == 0 and g.cout >= 64 and int(g.M) < 2 ** 31)

def launch_c1p(x, w, bias, res, y, g: ConvGeom, relu: bool, accumulate: bool = False,
               mask: Optional[torch.Tensor] = None) -> None:
    """Persistent streaming 1x1 conv: one LDS-DMA stream per CU across tiles, epilogue operands prefetched
    (csrc/kernels/conv1x1_pers.hip)."""
    if not c1p_covers(g):
        raise RuntimeError("conv1x1_pers: geometry not covered")
    if not (x.is_contiguous() and w.is_contiguous() and y.is_contiguous() and x.shape[-1] == g.cin
            and int(x.numel()) == int(g.M) * g.cin and int(y.numel()) == int(g.M) * g.cout
            and int(w.numel()) == g.cout * g.cin and (bias is None or bias.data_ptr() % 16 == 0)
            and (res is None or (res.is_contiguous() and int(res.numel()) == int(g.M) * g.cout))):
        raise RuntimeError("conv1x1_pers: operand shapes do not match the geometry")
    _chk(lib().mxr_conv1x1_pers(_p(x), _p(w), _p(bias), _p(res), _p(mask), _p(y), _p(zero_page(x.device)),
                                _p(_n.trash_page(x.device)), int(g.M), g.cout, g.cin, int(relu), int(accumulate),
                                _s()), "conv1x1_pers")

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
    """3x3 / stride-1 / pad-1 conv on the 32x32x16 MFMA (variants 10-15: the 16x16x32 MFMA) with plane-split LDS
    images (csrc/kernels/conv_hx32.hip; same tile table as :func:`launch_halo`)."""
    from . import halo as _hx
    if not hx32_covers(g):
        raise RuntimeError("conv3x3_hx32: geometry not covered")
    if not (x.is_contiguous() and w.is_contiguous() and y.is_contiguous() and x.shape[-1] == g.cin
            and int(w.numel()) == g.cout * 9 * g.cin and int(y.numel()) == int(g.M) * g.cout
            and int(x.numel()) == int(g.M) * g.cin and (bias is None or bias.data_ptr() % 16 == 0)):
        raise RuntimeError("conv3x3_hx32: operand shapes do not match the geometry")
    if (g.cin // 32) % 2:     # the persistent grid chains tiles over an even chunk count only
        variant = {2: 0, 3: 1, 13: 10, 14: 12}.get(variant, variant)
    tiles, nt = _hx.device_tiles(_hx.geom_batch(g), _hx.geom_shapes(g), x.device)
    wp = hx32_packed(w, g.cout, g.cin)
    _chk(lib().mxr_conv3x3_hx32(_p(x), _p(wp), _p(bias), _p(res), _p(mask), _p(y), _p(zero_page(x.device)),
                                ctypes.byref(g), _p(tiles), nt, int(relu), int(accumulate), int(variant), _s()),
         "conv3x3_hx32")

class FocalRequest:
    """The classification final's fused sigmoid-focal loss (conv_hx32.hip FOC form; reference: the focal loss
    compiled at /root/reference/train.py:99-102).  The Trainer sets this step's anchor targets before the forward
    (``RetinaNet.forward`` hands the request to the final layer through its pad sink); when the layer's tuned
    kernel has the form, its forward writes no logits -- ``loss`` and the padded gradient rows come out of the
    epilogue -- else ``loss`` stays None and the loss kernel runs as before.  One object per Trainer: its
    zero-padded gradient buffer persists across steps (columns past A * C are never written)."""

    def __init__(self, alpha: float = 0.25, gamma: float = 2.0):
        self.alpha, self.gamma = alpha, gamma
        self._buf = None
        self.set(None, None, None, 0)

    def set(self, state, label, npos, A: int) -> None:
        self.state, self.label, self.npos, self.A = state, label, npos, int(A)
        self.loss = None

    def dpad(self, n: int, p: int, ld: int, device) -> torch.Tensor:
        key = (n, p, ld, str(device))
        if self._buf is None or self._buf[0] != key:
            self._buf = (key, torch.zeros((n, p, ld), dtype=torch.bfloat16, device=device))
        return self._buf[1]

    def dpad_q(self, n: int, p: int, ld: int, device) -> torch.Tensor:
        """The zero-padded e5m2 gradient rows of the fp8 FOCAL form (columns past A * C are never written)."""
        key = (n, p, ld, str(device))
        b = getattr(self, "_qbuf", None)
        if b is None or b[0] != key:
            self._qbuf = b = (key, torch.zeros((n, p, ld), dtype=torch.uint8, device=device))
        return b[1]


# the fused focal form on or off (a switch for the tests' same-process comparisons, not an environment knob)
FOCAL_FUSED = True
# the fused form's kernel is adopted when its race time is within this of the raced winner's (ConvTuner.prefer):
# fusing saves the logits store and the separate focal kernel, 0.28 ms/step on the R50 bench
# (profiles/r5_focal_fused_ab.txt), which the race of the bare convolutions does not see
FOCAL_PREFER_MS = 0.15
FOCAL_LAUNCHES = [0]        # fused focal launches (bf16 and fp8), reported by bench.py


FOCAL_VARIANTS = (0, 10)      # conv_hx32 tiles with the fused focal form (10: the 16x16x32 MFMA)


def launch_hx32_focal(x, w, bias, g: ConvGeom, req: "FocalRequest", ld: int, variant: int = 0) -> torch.Tensor:
    """conv_hx32 variant ``variant`` (:data:`FOCAL_VARIANTS`) with the focal loss in its epilogue: returns the padded
    gradient rows [N, P, ld] (also the loss into ``req.loss``)."""
    from . import halo as _hx
    from .losses import LOGIT_HI, LOGIT_LO
    N = int(g.M) // g.out_img
    C = g.cout // req.A
    if not (hx32_covers(g) and x.is_contiguous() and w.is_contiguous() and int(x.numel()) == int(g.M) * g.cin
            and int(w.numel()) == g.cout * 9 * g.cin and bias is not None and bias.data_ptr() % 16 == 0
            and C == 80 and req.gamma == 2.0 and ld % 8 == 0 and ld >= g.cout
            and int(req.state.numel()) == int(g.M) * req.A and int(req.label.numel()) == int(g.M) * req.A):
        raise RuntimeError("conv3x3_hx32_focal: operands do not match the geometry")
    tiles, nt = _hx.device_tiles(_hx.geom_batch(g), _hx.geom_shapes(g), x.device)
    wp = hx32_packed(w, g.cout, g.cin)
    nparts = -(-g.cout // 256) * nt
    parts = torch.empty(nparts, dtype=torch.float32, device=x.device)
    out = torch.empty(1, dtype=torch.float32, device=x.device)
    dpad = req.dpad(N, g.out_img, ld, x.device)
    if variant not in FOCAL_VARIANTS:
        raise RuntimeError("conv3x3_hx32_focal: no focal form of variant %r" % (variant,))
    _chk(lib().mxr_conv3x3_hx32_focal_v(_p(x), _p(wp), _p(bias), _p(zero_page(x.device)), ctypes.byref(g), _p(tiles),
                                        nt, _p(req.state.contiguous()), _p(req.label.contiguous()), _p(req.npos),
                                        _p(dpad), int(ld), req.A, C, float(req.alpha), float(req.gamma), LOGIT_LO,
                                        LOGIT_HI, _p(parts), nparts, _p(out), int(variant), _s()),
         "conv3x3_hx32_focal")
    req.loss = out.reshape(())
    FOCAL_LAUNCHES[0] += 1
    return dpad

def hx32_packed(w: torch.Tensor, cout: int, cin: int) -> torch.Tensor:
    """``w`` (OHWI bf16) in conv_hx32's [tap][cin / 32][plane][cout][16] layout (a 1-KiB weight DMA piece
    is then contiguous).  The model's compute weights come from ``ComputeWeights.hx32_packed`` (all of
    them packed by one launch per optimizer step: the weights are rewritten in place by the Adam kernel,
    which a version-keyed cache cannot see); any other weight (padded final layers, tests) is packed
    here, per call."""
    cw = _n.compute_weights()
    if cw is not None:
        wp = cw.hx32_packed(w)
        if wp is not None:
            return wp
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

# output target of the next forward launch (the HIP candidates write there instead of a fresh tensor): a chunk of a
# preallocated full-batch activation (ResidualBlockFn's image-chunked forward); see :func:`run_fwd_into`
_DST = [None]


def run_fwd_into(dst: torch.Tensor, x, w, b, res, stride, pads, relu, emit=None) -> torch.Tensor:
    """:func:`run_fwd` writing its output into ``dst`` (contiguous, the output's shape)."""
    _DST[0] = dst
    try:
        y = run_fwd(x, w, b, res, stride, pads, relu, emit=emit)
    finally:
        _DST[0] = None
    if y.data_ptr() != dst.data_ptr():
        dst.copy_(y)           # a candidate that allocates its own output (library / fp8)
    return dst

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

    dst = _DST[0]
    if dst is not None and (tuple(dst.shape) != tuple(out_shape) or dst.dtype != x.dtype or not dst.is_contiguous()):
        dst = None

    def hip(v):
        def f():
            if out is not None:        # accumulate into ``out`` (y += conv)
                launch_fwd(x, w, b, res, out, g, relu, accumulate=True, variant=v, mask=mask)
                return out
            y = dst if dst is not None else torch.empty(out_shape, dtype=x.dtype, device=x.device)
            launch_fwd(x, w, b, res, y, g, relu, variant=v, mask=mask)
            return y
        return f
    if only is not None:
        return _bits_filter(_only_fwd(only, hip, g, out, allow_miopen, f8c, x, w, b, res, stride, pads, relu, mask),
                            mask)
    cands = {"hip%d" % v: hip(v) for v in FWD_VARIANTS if v < 3 or g.cout % 8 == 0}
    from . import halo as _hx
    if _hx.covers(g):
        cands.update({"halo%d" % v: hip("halo%d" % v) for v in HALO_VARIANTS})
    if hx32_covers(g):
        cands.update({"hx32_%d" % v: hip("hx32_%d" % v) for v in hx32_variants(g)})
    cands.update({v: hip(v) for v in c1x1_variants(g)})
    if c1p_covers(g):
        cands["c1p"] = hip("c1p")
    cands.update({v: hip(v) for v in big_tile_variants(g)})
    cands.update({"sk%d" % v: hip("sk%d" % v) for v in SK_VARIANTS if splitk_splits(g, v)})
    if out is not None:       # accumulating forms: HIP kernels only (their epilogue adds in place)
        allow_miopen = False
        f8c = {}
    if allow_miopen:
        if mask is None:
            cands["miopen"] = lambda: miopen_fwd(x, w, b, res, stride, pads, relu)
        else:
            cands["miopen"] = lambda: relu_bwd(miopen_fwd(x, w, b, res, stride, pads, relu), mask)
    cands.update(f8c)
    return _bits_filter(cands, mask)

def _only_fwd(only, hip, g, out, allow_miopen, f8c, x, w, b, res, stride, pads, relu, mask):
    """fwd_candidates restricted to ``only`` (empty when it is not a candidate of this call: the caller
    then builds the full set)."""
    if only.startswith("hip"):
        v = int(only[3:])
        return {only: hip(v)} if v in FWD_VARIANTS and (v < 3 or g.cout % 8 == 0) else {}
    if only.startswith("hx32_"):
        return {only: hip(only)} if hx32_covers(g) and int(only[5:]) in hx32_variants(g) else {}
    if only.startswith("halo"):
        from . import halo as _hx
        return {only: hip(only)} if _hx.covers(g) and int(only[4:]) in HALO_VARIANTS else {}
    if only.startswith("c1x1_"):
        return {only: hip(only)} if only in c1x1_variants(g) else {}
    if only == "c1p":
        return {only: hip(only)} if c1p_covers(g) else {}
    if only.startswith("p8_"):
        return {only: hip(only)} if only in big_tile_variants(g) else {}
    if only.startswith("sk"):
        return {only: hip(only)} if int(only[2:]) in SK_VARIANTS and splitk_splits(g, int(only[2:])) else {}
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

# a ResNet projection block's branch2c + branch1 as ONE dual-source GEMM (conv_pipe.hip DualSrc): the shortcut
# tensor is never written nor re-read (a switch for same-process A/Bs, scripts/bench_switch.py)
PROJ_FUSED = True
DUAL_VARIANTS = (1, 5, 8, 9, 10, 11, 12, 13)


def proj_fusable(h: torch.Tensor, x: torch.Tensor, w2c: torch.Tensor, w1: torch.Tensor, stride: int) -> bool:
    """The dual-source kernel's contract: 1x1 convs, bf16, channel counts multiples of 32 (cout of 8), and the
    branch1 grid (stride ``stride`` over x) equal to h's."""
    if not (PROJ_FUSED and h.is_cuda and h.dtype == torch.bfloat16 and x.dtype == torch.bfloat16):
        return False
    if w2c.shape[1] != 1 or w2c.shape[2] != 1 or w1.shape[1] != 1 or w1.shape[2] != 1:
        return False
    N, Ho, Wo, c1 = h.shape
    return (c1 % 32 == 0 and x.shape[-1] % 32 == 0 and w2c.shape[0] % 8 == 0 and w1.shape[0] == w2c.shape[0]
            and x.shape[0] == N and (x.shape[1] - 1) // stride + 1 == Ho and (x.shape[2] - 1) // stride + 1 == Wo)


def run_fwd_proj(h: torch.Tensor, x: torch.Tensor, w2c: torch.Tensor, w1: torch.Tensor, b: torch.Tensor, stride: int,
                 emit: Optional[BitMask] = None) -> torch.Tensor:
    """y = relu([h | x(::stride)] . [w2c | w1]^T + b): branch2c (1x1 over h) + branch1 (1x1/``stride`` over the block
    input x) + the residual add + ReLU of a projection block (/root/reference/train.py:91 builds them as two convs and
    a keras ``Add``), one tuned launch.  ``w2c`` / ``w1`` = the effective (BN-scaled) 1x1 weights, read in place by
    the kernel (no concatenated copy); ``b`` the summed BN shifts; ``emit``: the output's ReLU bitmask for the next
    block's data gradient."""
    from .conv_tuner import TUNER
    N, Ho, Wo, c1 = h.shape
    c2 = x.shape[-1]
    cout = w2c.shape[0]
    w2c, w1 = w2c.contiguous(), w1.contiguous()
    g = geom_single(N, Ho, Wo, Ho, Wo, 1, 1, (0, 0, 0, 0), c1 + c2, cout)
    key = TUNER.key("fwdp", N, Ho, Wo, c1, c2, cout, stride, x.shape[1], x.shape[2]) + ("|eb" if emit is not None else "")
    zp = _p(zero_page(h.device))
    h, x = h.contiguous(), x.contiguous()

    def cand(v):
        def f():
            y = torch.empty((N, Ho, Wo, cout), dtype=h.dtype, device=h.device)
            _chk(lib().mxr_conv_fwd_pipe_dual(_p(h), _p(x), c1, c2, x.shape[1], x.shape[2], stride, _p(w2c), _p(w1),
                                              _p(b), _p(emit), _p(y), zp, ctypes.byref(g), 1, v, _s()),
                 "conv_fwd_pipe_dual")
            return y
        return f
    def c1p():
        # the persistent streaming 1x1 kernel's dual-source form (conv1x1_pers.hip QDual)
        y = torch.empty((N, Ho, Wo, cout), dtype=h.dtype, device=h.device)
        _chk(lib().mxr_conv1x1_pers_dual(_p(h), _p(x), _p(w2c), _p(w1), _p(b), _p(emit), _p(y), zp,
                                         _p(_n.trash_page(h.device)), int(g.M), cout, c1 + c2, c1, x.shape[1],
                                         x.shape[2], stride, Ho, Wo, _s()), "conv1x1_pers_dual")
        return y
    c1p_ok = c1 % 32 == 0 and c2 % 32 == 0 and b.data_ptr() % 16 == 0
    win = TUNER.winner(key)
    if win is not None and win.startswith("d") and int(win[1:]) in DUAL_VARIANTS:
        return TUNER.run(key, {win: cand(int(win[1:]))})
    if win == "c1p" and c1p_ok:
        return TUNER.run(key, {win: c1p})
    cands = {"d%d" % v: cand(v) for v in DUAL_VARIANTS}
    if c1p_ok:
        cands["c1p"] = c1p
    return TUNER.run(key, cands)


def run_fwd(x, w, b, res, stride, pads, relu, emit: Optional[BitMask] = None) -> torch.Tensor:
    """Tuned forward (HIP tile variants vs MIOpen + fused epilogue) of one NHWC conv.  ``emit`` (relu only):
    the epilogue also writes the output's ReLU mask into this :class:`BitMask`."""
    from .conv_tuner import TUNER
    N, H, W, cin = x.shape
    cout, kh = w.shape[0], w.shape[1]
    Ho, Wo = _out_hw(H, W, kh, stride, pads)
    g = geom_single(N, H, W, Ho, Wo, kh, stride, pads, cin, cout)
    from . import fp8 as _f8
    f8 = "|f8" if _f8.enabled() and _f8.eligible(cin, cout) and emit is None else ""
    key = TUNER.key("fwd", N, H, W, cin, cout, kh, stride, tuple(pads), int(relu), int(res is not None)) + f8
    if emit is not None:
        assert relu
        key += "|eb"
    only = _only(key)
    if only is not None:
        c = fwd_candidates(x, w, b, res, g, stride, pads, relu, (N, Ho, Wo, cout), fp8_ok=True, only=only, mask=emit)
        if c:
            return TUNER.run(key, c)
    return TUNER.run(key, fwd_candidates(x, w, b, res, g, stride, pads, relu, (N, Ho, Wo, cout), fp8_ok=True,
                                         mask=emit))
