"""Weight and bias gradients of the convolutions: split-K implicit GEMMs with slab
reductions, the halo-staged 3x3 form, the 64-channel 3x3 kernel, column-sum bias gradients, and their
delivery into the flat gradient buffer (gradient sinks, side stream) -- split out of ``native_conv``.
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
from .conv_launch import (_bind, _miopen_wgrad, _only, geom_single)


_WGRAD_TILE = {0: (128, 128), 1: (128, 64), 2: (64, 128)}   # variant -> (BK, BCO)

def _splits(g: ConvGeom, bk: int, bco: int) -> int:
    K = g.kh * g.kw * g.cin
    tiles = ((K + bk - 1) // bk) * ((g.cout + bco - 1) // bco)
    steps = (g.M + 63) // 64
    target = 1024
    s = max(1, -(-target // tiles))
    return int(max(1, min(s, steps // 4 if steps >= 4 else 1, 256)))


# variant -> (TK, TC) of conv_wgrad_pipe.hip (5 / 6: DMA interleaved between MFMA groups, 7: interleaved +
# s_setprio, 8 / 9: s_setprio around the MFMA block, 10-12: narrow 4-wave tiles for 64-channel layers,
# 13-15: two blocks per CU -- 128 x 128, and 256 x 128 / 128 x 256 on 3-deep rings)

_WGRAD_PIPE_TILE = {3: (256, 256), 4: (256, 128), 5: (256, 256), 6: (256, 128), 7: (256, 256), 8: (256, 256),
                    9: (256, 128), 10: (256, 64), 11: (128, 64), 12: (64, 64), 13: (128, 128), 14: (256, 128),
                    15: (128, 256)}
# phase-pipelined 256 k x 256 co wgrad (conv_wgrad_p8.hip): variant -> kernel variant (1 = s_setprio)

_WGRAD_P8 = {20: 0, 21: 1, 22: 2, 23: 3, 24: 4, 25: 5}
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
    if g.nlev > 1:       # the packed head layers (a separate target only for the sweep, scripts/gpu_sweep_wgrad_blocks.sh)
        target = int(os.environ.get("MXR_WGRAD_HEAD_BLOCKS", str(target)))
    s = max(1, round(target / tiles))
    return int(max(1, min(s, nsub // 8 if nsub >= 8 else 1, 512 * occ)))

def conv_wgrad(x, dy, g: ConvGeom, scale: Optional[torch.Tensor], out: Optional[torch.Tensor] = None,
               accumulate: bool = False, variant: Optional[int] = None, bias_out: Optional[torch.Tensor] = None,
               bias_accumulate: bool = False) -> torch.Tensor:
    """fp32 dW (OHWI) = scale[co] * sum_m dY (x) im2col(X); dY may have cout % 8 != 0 (padded).
    ``bias_out`` (phase-pipelined variants, see :data:`_WGRAD_P8`, cout % 4 == 0): the unscaled bias
    gradient sum_m dY[m, :cout] is computed by the same kernel from the dY tiles it stages anyway."""
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
    if bias_out is not None and (variant not in _WGRAD_P8 or cout % 4 or bias_out.numel() != cout
                                 or bias_out.dtype != torch.float32 or not bias_out.is_contiguous()):
        raise RuntimeError("conv_wgrad: the fused bias gradient needs a phase-pipelined variant, cout % 4 == 0 "
                           "and a contiguous fp32 (cout,) output")
    if variant in _WGRAD_P8:
        splits = _splits_pipe(g, 256, 256)
        nb = 0 if bias_out is None else splits * cout
        part = torch.empty(splits * cout * K + nb, dtype=torch.float32, device=dy.device)
        _chk(lib().mxr_conv_wgrad_p8_bias(_p(x), _p(dy), ldy, _p(part), splits, _p(out), _p(sc), int(accumulate),
                                          _p(zero_page(dy.device)), ctypes.byref(g), _WGRAD_P8[variant],
                                          _p(bias_out), int(bias_accumulate), _s()),
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
        splits = max(1, min(int(tiles.shape[0]), round(256 / (n_co * n_ci))))
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



def _side(sink, param) -> bool:
    """Whether this weight gradient goes to the side stream: not for parameters tagged ``mxr_main_wgrad``
    (models.resnet: the last blocks of the backward, whose weight gradients would otherwise queue at the
    end of the side stream's backlog while the compute stream idles before the optimizer)."""
    return SIDE.usable(sink) and not getattr(param, "mxr_main_wgrad", False)

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
    if _side(sink, param):
        with SIDE.run(sink.device, *reads):
            TUNER.run(key, c)
            _n.grad_sinks().notify(param)
        return None
    TUNER.run(key, c)
    _n.grad_sinks().notify(param)
    return None

def _is_p8(name: str) -> bool:
    return name.startswith("hip") and name[3:].isdigit() and int(name[3:]) in _WGRAD_P8

def deliver_wgrad_bias_fused(key, x, dy, g: ConvGeom, wparam, bparam) -> bool:
    """Weight AND bias gradient of an unscaled conv in one kernel, when the tuned sink winner for ``key``
    is a phase-pipelined variant (conv_wgrad_p8.hip BIAS: the bias sums come from the dY tiles the wgrad
    stages anyway, instead of a separate colsum pass over all of dY) and both parameters have gradient
    sinks.  Accumulates into both sinks (on the side stream when usable) and returns True; False = not
    applicable, the caller runs the separate paths.  ``MXR_WGRAD_FUSED_BIAS=0`` disables it."""
    from .conv_tuner import TUNER
    if g.cout % 4 or os.environ.get("MXR_WGRAD_FUSED_BIAS", "1") == "0":
        return False
    gs = _n.grad_sinks()
    if gs is None:
        return False
    ws, bs = gs.get(wparam), gs.get(bparam)
    if ws is None or bs is None or bs.numel() != g.cout:
        return False
    key = key + "|s"
    win = TUNER.winner(key)
    if win is not None and not _is_p8(win):
        # a near-tie race winner without the fused bias form loses the separate bias pass over all of dY:
        # adopt the fastest phase-pipelined candidate within that pass's time (ConvTuner.prefer)
        t = TUNER.timings.get(TUNER.borrowed.get(key, key), {})
        p8 = sorted((v, n) for n, v in t.items() if isinstance(v, float) and _is_p8(n))
        if p8 and TUNER.prefer(key, p8[0][1], dy.numel() * dy.element_size() / 4.0e9):
            win = p8[0][1]
    if win is not None and _is_p8(win):
        v = int(win[3:])

        def run():
            conv_wgrad(x, dy, g, None, out=ws, accumulate=True, variant=v, bias_out=bs, bias_accumulate=True)
            gs.notify(wparam)
            gs.notify(bparam)
    else:
        return False
    TUNER.calls[key] = TUNER.calls.get(key, 0) + 1

    if _side(ws, wparam):
        with SIDE.run(ws.device, x, dy):
            run()
    else:
        run()
    return True

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

def run_wgrad_bias_fused(x, dy, w, stride, pads, scale, param, bias_param) -> bool:
    """:func:`deliver_wgrad_bias_fused` for a single-geometry conv (the FPN convs: biased, unscaled);
    True = both gradients delivered, False = the caller runs :func:`run_wgrad` and the bias pass."""
    if scale is not None:
        return False
    from .conv_tuner import TUNER
    N, H, W, cin = x.shape
    cout, kh = w.shape[0], w.shape[1]
    g = geom_single(N, H, W, dy.shape[1], dy.shape[2], kh, stride, pads, cin, cout)
    key = TUNER.key("wgrad", N, H, W, cin, cout, kh, stride, tuple(pads))
    return deliver_wgrad_bias_fused(key, x, dy, g, param, bias_param)


# the projection blocks' two weight gradients as ONE dual-source GEMM (a switch for same-process A/Bs)
PROJ_WGRAD = True
PROJ_WGRAD_MIN_PX = 40000
_WGRAD_DUAL = (0, 1, 2, 4)


def proj_wgrad_fusable(h2, x, dy, w2c, w1, stride) -> bool:
    """:func:`run_wgrad_proj`'s contract (1x1 convs, bf16, both channel counts multiples of 8) with gradient sinks
    for both weights (the training step)."""
    from . import conv_launch as _cl
    if not (PROJ_WGRAD and _cl.PROJ_FUSED and dy.is_cuda and dy.dtype == torch.bfloat16):
        return False
    if w2c.shape[1] != 1 or w2c.shape[2] != 1 or w1.shape[1] != 1 or w1.shape[2] != 1:
        return False
    # (res5a at B=16 -- 16,800 pixels, K = 512 + 1024 -- measured 0.150 ms fused vs 0.127 ms for the two separate
    # weight gradients: below ~40k pixels the split-K grid of the long-K fused GEMM loses, profiles/r6_conv_budget_dual.txt)
    return (h2.shape[-1] % 8 == 0 and x.shape[-1] % 8 == 0 and dy.shape[-1] % 8 == 0
            and dy.shape[0] * dy.shape[1] * dy.shape[2] >= PROJ_WGRAD_MIN_PX
            and tuple(h2.shape[:3]) == tuple(dy.shape[:3])
            and (x.shape[1] - 1) // stride + 1 == dy.shape[1] and (x.shape[2] - 1) // stride + 1 == dy.shape[2])


def run_wgrad_proj(h2, x, dy, stride, s2c, s1, p2c, p1) -> bool:
    """Both weight gradients of a projection block from ONE read of its output gradient ``dy``
    (conv_wgrad_p8.hip DS form): dW2c over the branch2b output ``h2`` and dW1 over the stride-``stride`` 1x1 im2col of
    the block input ``x`` as one split-K GEMM over the concatenated K, reduced straight into both gradient sinks
    (scaled by the two frozen-BN scales).  On the side stream like the single weight gradients.  False when a sink is
    missing (the caller runs the two separate weight gradients)."""
    from .conv_tuner import TUNER
    k1 = int(h2.shape[-1])
    gs = _n.grad_sinks()
    o1 = gs.get(p2c) if gs is not None else None
    o2 = gs.get(p1) if gs is not None else None
    if o1 is None or o2 is None:
        return False
    N, H, W, cin = x.shape
    cout = int(dy.shape[-1])
    Ho, Wo = int(dy.shape[1]), int(dy.shape[2])
    g = geom_single(N, H, W, Ho, Wo, 1, stride, (0, 0, 0, 0), cin, cout)
    K = k1 + cin
    splits = _splits_pipe(_kgeom(g, K), 256, 256)
    h2, x, dy = h2.contiguous(), x.contiguous(), dy.contiguous()
    sc1 = None if s2c is None else s2c.float().contiguous()
    sc2 = None if s1 is None else s1.float().contiguous()
    zp = _p(zero_page(dy.device))

    def cand(v, d1, d2):
        def f():
            part = torch.empty(splits * cout * K, dtype=torch.float32, device=dy.device)
            _chk(lib().mxr_conv_wgrad_p8_dual(_p(x), _p(h2), k1, _p(dy), cout, _p(part), splits, _p(d1), _p(d2),
                                              _p(sc1), _p(sc2), 1, zp, ctypes.byref(g), v, _s()), "conv_wgrad_p8_dual")
            return d1
        return f
    key = TUNER.key("wgradp", N, Ho, Wo, k1, cin, cout, stride, H, W) + "|s"
    win = TUNER.winner(key)
    if win is not None and win.startswith("p8d_") and int(win[4:]) in _WGRAD_DUAL:
        c = {win: cand(int(win[4:]), o1, o2)}
    else:
        c = {"p8d_%d" % v: cand(v, o1, o2) for v in _WGRAD_DUAL}
        if TUNER.needs_tuning(key, c):
            # race on scratch copies of the two slots, then run the winner for real (serially, like a first sight)
            a1, a2 = o1.clone(), o2.clone()
            TUNER.run(key, {"p8d_%d" % v: cand(v, a1, a2) for v in _WGRAD_DUAL})
            TUNER.run(key, c)
            gs.notify(p2c)
            gs.notify(p1)
            return True
    if _side(o1, p2c):
        with SIDE.run(o1.device, h2, x, dy, sc1, sc2):
            TUNER.run(key, c)
            gs.notify(p2c)
            gs.notify(p1)
        return True
    TUNER.run(key, c)
    gs.notify(p2c)
    gs.notify(p1)
    return True


def _kgeom(g: ConvGeom, K: int) -> ConvGeom:
    """``g`` with its K (kh * kw * cin) replaced by ``K`` -- for the split count of a dual-source GEMM."""
    h = ConvGeom.from_buffer_copy(g)
    h.cin = K
    return h
