"""Data gradients of the convolutions: stride-1 through the forward kernels on flipped
weights, 1x1 / stride-2 as a strided scatter, 3x3 / stride-2 as the four sub-pixel phases in one GEMM;
``run_dgrad`` races the candidates per shape (split out of ``native_conv``).
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
from . import conv_launch as _cl
from .conv_launch import (C1X1_BN, FWD_VARIANTS, HALO_VARIANTS, HX32_NARROW, HX32_VARIANTS, P8_TUNED, BitMask, _only, bits_capable, flip, geom_single, hip_conv_ok, launch_fwd, relu_bwd, torch_conv_backward)


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
        assert not isinstance(mask, BitMask), "mxr_s2_shuffle reads a bf16 mask"
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
# stacked stride-2 weights as row copies of the batched flip (a switch for same-process A/Bs)
S2_FROM_FLIP = True

def _s2_stacked_weights_hip(w, pads):
    """_s2_stacked_weights in one kernel (mxr_s2_stack) instead of ~25 small torch ops."""
    cout, _, _, cin = w.shape
    key = (tuple(pads), w.device)
    ent = _S2_TAPS.get(key)
    if ent is None:
        taps, win = _s2_stack_taps(pads)
        ent = _S2_TAPS[key] = ((ctypes.c_int * 16)(*taps), win)
    w4 = torch.empty((4 * cin, 2, 2, cout), dtype=w.dtype, device=w.device)
    cw = _n.compute_weights()
    wd = cw.flipped(w) if cw is not None else None
    if wd is not None and cout % 8 == 0 and S2_FROM_FLIP:
        # rows of the batched flip-transposed copy (coalesced), instead of the strided gather from w
        _chk(lib().mxr_s2_stack_flip(_p(wd), _p(w4), cin, cout, ent[0], _s()), "s2_stack_flip")
    else:
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
                             or only.startswith("halo") or only.startswith("hx32_") or only == "c1p"):
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
        if (stride == 1 and kh == 1 and tuple(pads) == (0, 0, 0, 0) and cout % 32 == 0 and cout >= 96
                and cin % 8 == 0 and cin >= 64):
            # the persistent streaming 1x1 kernel (conv1x1_pers.hip) on the transposed weights
            cands["c1p"] = lambda: conv_dgrad(dy, w, tuple(x.shape), stride, pads, "c1p", **kw)
        if stride == 1 and cout % 64 == 0 and cin % 8 == 0 and kh * w.shape[2] <= 16:
            for v in ["p8_%d" % v for v in P8_TUNED]:
                cands[v] = (lambda v=v: conv_dgrad(dy, w, tuple(x.shape), stride, pads, v, **kw))
        if stride == 1 and kh == 3 and tuple(pads) == (1, 1, 1, 1) and cout % 32 == 0 and cin % 8 == 0:
            for v in HALO_VARIANTS:
                cands["halo%d" % v] = (lambda v=v: conv_dgrad(dy, w, tuple(x.shape), stride, pads, "halo%d" % v,
                                                              **kw))
            for v in HX32_VARIANTS:
                if v in HX32_NARROW and (cin > 64 or not _cl.NARROW_TILES):   # 64-channel tiles: narrow outputs
                    continue
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
            # (lean: one delayed-scaling pass over dY, the flipped 3x3 weights from the per-step batched quantisation;
            # ops.fp8.LEAN_CANDIDATES)
            lean = _f8.LEAN_CANDIDATES
            dq, idq = _f8.quantize_delayed(dy, ("bbdy", w), bf8=True) if lean else _f8.quantize_bf8(dy)
            packed = lean and v in _f8.HX8_DGRAD_VARIANTS
            wq, iw = _f8.quantize_rows_hx8(flip(w)) if packed else _f8.quantize_rows(flip(w))
            dx = out if out is not None else torch.empty((N, H, W, cin), dtype=dy.dtype, device=dy.device)
            return _f8.launch(dq, idq, wq, iw, None, None, dx, g8, False, v, mask=mask, accumulate=out is not None,
                              packed=packed)
        for v in _f8.F8_DGRAD_VARIANTS + (_f8.HX8_DGRAD_VARIANTS if _f8.hx8_covers(g8) else ()):
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
    bits = isinstance(mask, BitMask)
    key = TUNER.key("dgrad", N, H, W, cin, cout, kh, stride, tuple(pads)) + \
        ("|mb" if bits else "|m" if mask is not None else "") + ("|a" if (out is not None or res is not None) else "")
    only = _only(key)
    cands = _dgrad_cands(dy, w, x, stride, pads, mask, out, res, only=only) if only is not None else None
    if bits and cands:
        cands = {k: v for k, v in cands.items() if bits_capable(k)}
    if not cands:
        cands = _dgrad_cands(dy, w, x, stride, pads, mask, out, res)
        if bits:
            cands = {k: v for k, v in cands.items() if bits_capable(k)}
    if out is not None and TUNER.needs_tuning(key, cands):
        # time the accumulating candidates against a scratch copy, then run the winner for real
        tc = _dgrad_cands(dy, w, x, stride, pads, mask, out.clone())
        TUNER.run(key, {k: v for k, v in tc.items() if bits_capable(k)} if bits else tc)
    return TUNER.run(key, cands)


# the dual-destination data gradient of the projection blocks (a switch for same-process A/Bs)
PROJ_DGRAD = True


def proj_dgrad_fusable(dy: torch.Tensor, w2c: torch.Tensor, w1: torch.Tensor, h2: torch.Tensor, x_shape,
                       stride: int) -> bool:
    """:func:`run_dgrad_proj`'s contract: 1x1 convs, bf16, K (the block's output channels) a multiple of 32, both
    output channel counts of 8, a bf16 mask, stride 1 or 2 over x."""
    if not (PROJ_DGRAD and _cl.PROJ_FUSED and dy.is_cuda and dy.dtype == torch.bfloat16 and stride in (1, 2)):
        return False
    if w2c.shape[1] != 1 or w2c.shape[2] != 1 or w1.shape[1] != 1 or w1.shape[2] != 1:
        return False
    K, c1, c2 = dy.shape[-1], h2.shape[-1], x_shape[-1]
    return (K % 32 == 0 and c1 % 8 == 0 and c2 % 8 == 0 and w2c.shape[0] == K and w1.shape[0] == K
            and (x_shape[1] - 1) // stride + 1 == dy.shape[1] and (x_shape[2] - 1) // stride + 1 == dy.shape[2]
            and tuple(h2.shape[:3]) == tuple(dy.shape[:3]))


def run_dgrad_proj(dy: torch.Tensor, w2c: torch.Tensor, w1: torch.Tensor, h2: torch.Tensor, x_shape, stride: int,
                   out: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """Both data gradients of a projection block from ONE read of its output gradient ``dy`` (conv_pipe.hip
    ``DualDst``): dH2 = relu'(h2) * (dy . W2c) and dX = dy . W1 (stride 1, or scattered at stride 2 with the gaps
    zeroed), or dX accumulated into ``out`` (a GradJoin buffer).  Returns (dH2, dX)."""
    from .conv_tuner import TUNER
    N, Ho, Wo, K = dy.shape
    c1, c2 = h2.shape[-1], x_shape[-1]
    H, W = x_shape[1], x_shape[2]
    wd1, wd2 = flip(w2c).contiguous(), flip(w1).contiguous()    # [c1 | c2, 1, 1, K]: read in place, no concat
    g = geom_single(N, Ho, Wo, Ho, Wo, 1, 1, (0, 0, 0, 0), K, c1 + c2)
    key = TUNER.key("dgradp", N, Ho, Wo, K, c1, c2, stride, H, W) + ("|a" if out is not None else "")
    zp = _p(zero_page(dy.device))
    dy, h2 = dy.contiguous(), h2.contiguous()

    def cand(v, dst):
        def f():
            dh2 = torch.empty((N, Ho, Wo, c1), dtype=dy.dtype, device=dy.device)
            dx = dst if dst is not None else torch.empty((N, H, W, c2), dtype=dy.dtype, device=dy.device)
            _chk(lib().mxr_conv_dgrad_pipe_dd(_p(dy), _p(wd1), _p(wd2), _p(h2), _p(dh2), _p(dx), c1, c2, stride, H, W,
                                              int(dst is not None), zp, ctypes.byref(g), v, _s()), "conv_dgrad_pipe_dd")
            return dh2, dx
        return f
    win = TUNER.winner(key)
    if win is not None and win.startswith("d") and int(win[1:]) in _cl.DUAL_VARIANTS:
        return TUNER.run(key, {win: cand(int(win[1:]), out)})
    cands = {"d%d" % v: cand(v, out) for v in _cl.DUAL_VARIANTS}
    if out is not None and TUNER.needs_tuning(key, cands):
        # race the accumulating form on a scratch copy, then run the winner for real
        TUNER.run(key, {"d%d" % v: cand(v, out.clone()) for v in _cl.DUAL_VARIANTS})
    return TUNER.run(key, cands)
