"""FP8 convolutions of the packed head layers (BASELINE config 5: "RetinaNet-R50-FPN fp8 weights+activations (CDNA4
fp8 MFMA)").

Recipe:

* activations: one per-tensor e4m3 scale.  The head layers' inputs are quantised by the PRODUCING layer's epilogue with
  delayed scaling (:class:`AmaxState`: the previous step's amax x :data:`MARGIN`, this step's amax max-reduced for the
  next), so they cost no extra pass; a first sight falls back to the exact two-pass ``mxr_fp8_amax`` +
  ``mxr_fp8_quant`` (device scalars, no host sync);
* weights: one scale per output channel on the bf16 compute weight ``W * bn_scale``, re-quantised every step since Adam
  moves them -- straight into conv_hx32_f8's packed layout, all head weights (forward and flipped copies) by one
  batched launch per optimizer step (``ComputeWeights.hx8_quant``);
* forward: the halo-staged ``conv_hx32_f8`` (``v_mfma_scale_f32_32x32x64_f8f6f4``, unit block scales) with the
  epilogue applying ``inv_x * inv_w[co]``, bias and relu, emitting the next layer's e4m3 copy; a tower output whose
  only reader is the next fp8 layer is that copy + a 1-bit relu mask, no bf16 store (:func:`pyramid_forward`
  ``f8_only``); the classification final runs the focal loss in its epilogue (no logits);
* data gradients: e5m2 dY x e4m3 W on the same kernel (:func:`pyramid_dgrad`), masked by the producer's relu bits and
  emitting dX's e5m2 copy; a dX whose only reader is an fp8 tower layer's backward is that copy alone (``f8_only``);
* weight gradients: e5m2 dY x e4m3 X on the scaled 16x16x128 MFMA (``csrc/kernels/conv_wgrad_p8_f8.hip``,
  :func:`pyramid_wgrad`) from the fp8 copies the step already holds, fp32 accumulation, slabs and sink -- the
  optimizer still sees fp32 gradients; the bias gradients come out of the same kernel (sums of the e5m2 dY);
* backbone / FPN convs: ``conv_pipe_f8`` / ``conv_p8_f8`` compete in the per-shape tuner race and run where they win
  (they would need their own quantisation pass; the fused residual blocks stay bf16).

The encodings are OCP ``e4m3fn`` / ``e5m2`` (CDNA4), the same as ``torch.float8_e4m3fn`` / ``torch.float8_e5m2``.
Enable with ``set_enabled(True)`` / ``MXR_FP8=1`` (``bench.py --dtype fp8``, ``train --fp8``).
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional, Tuple

import torch

from .native import ConvGeom, _chk, _p, _s, lib, zero_page

FP8_MAX = 448.0
_STATE = {"enabled": os.environ.get("MXR_FP8", "0") == "1"}
# fp8 weight gradients of the packed head layers (conv_wgrad_p8_f8.hip); MXR_FP8_WGRAD=0 keeps them bf16 (A/B)
WGRAD = os.environ.get("MXR_FP8_WGRAD", "1") == "1"
# tower outputs whose reader is the next fp8 head layer exist only as their e4m3 copy + relu bitmask
# (:func:`pyramid_forward` f8_only); a switch for the tests' same-process A/B, not an environment knob
F8_ONLY_TOWERS = True
# an fp8-only tower output saves its 183 MB bf16 store and the next data gradient's mask read, ~0.05 ms per layer
# (profiles/r5_fp8_wgrad_ab.txt): the hx8 variant with that form is adopted within this of the raced winner
F8ONLY_PREFER_MS = 0.02
# the head layers' bias gradients from the fp8 weight gradient kernel (sums of the e5m2 dY copy it contracts) instead of
# a bf16 column-sum pass over dY (a switch for same-process A/Bs, scripts/bench_switch.py)
WGRAD_BIAS = True
# data gradients whose reader is an fp8 tower layer's backward exist only as their e5m2 copy (pyramid_dgrad f8_only;
# needs WGRAD_BIAS: the producer's bias then needs no bf16 column sum); a switch for same-process A/Bs
F8_ONLY_DGRAD = True
# the classification final's fused focal gradient rows as their e5m2 copy only (_focal_forward; a switch for A/Bs)
FOCAL_DQ = True
# conv_wgrad_p8_f8 kernel variant of the head weight gradients (1 = s_setprio around the MFMA blocks; an A/B switch)
WGRAD_VARIANT = 0
F8_VARIANTS = (0, 1, 2, 3, 4, 5, 6, 7)
# 0-5: conv_pipe_f8.hip (32x32x64 scaled MFMA, 4-deep ring); 6 / 7: conv_p8_f8.hip (conv_p8's PF phase
# schedule with one 16x16x128 scaled MFMA per fragment pair; needs cin % 128 == 0), 7 with s_setprio
P8F_VARIANTS = (6, 7)
# data-gradient form of conv_p8_f8 (e5m2 dY x e4m3 W, e5m2 fused output): kernel variants 4 / 5
F8_DGRAD_VARIANTS = (10, 11)
P8F_ABLATE = 15      # diagnostics only (scripts/bench_f8.py): conv_p8_f8 without its epilogue
# halo-staged 3x3 on the 32x32x64 scaled MFMA (conv_hx32_f8.hip): forward 256 / 128-channel tiles, and the
# data-gradient form (e5m2 dY, e5m2 fused output); kernel variant = v - 20
HX8_VARIANTS = (20, 21)
HX8_DGRAD_VARIANTS = (22, 23)


def variants_for(cin: int, g: Optional[ConvGeom] = None):
    vs = tuple(v for v in F8_VARIANTS if v not in P8F_VARIANTS or cin % 128 == 0)
    return vs + (HX8_VARIANTS if g is not None and hx8_covers(g) else ())


def hx8_covers(g: ConvGeom) -> bool:
    """conv_hx32_f8.hip: the halo tile table's 3x3 / s1 / pad-1 geometries with an even count of
    64-channel chunks."""
    from . import halo as _hx
    return g.cin % 128 == 0 and g.cout % 8 == 0 and _hx.covers(g) and g.cout * 9 * g.cin < 2 ** 31


def set_enabled(on: bool) -> None:
    _STATE["enabled"] = bool(on)


def enabled() -> bool:
    return _STATE["enabled"]


def eligible(cin: int, cout: int, ostride: int = 1) -> bool:
    """Shapes the fp8 kernel covers: 64-channel K sub-stages and 16-B output chunks."""
    return cin % 64 == 0 and cout % 8 == 0 and ostride == 1


def quantize(x: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """bf16 tensor -> (e4m3fn bytes as uint8, inv_scale float[1]); ``x ~= q * inv_scale``."""
    x = x.contiguous()
    n = x.numel()
    if n % 16:
        raise ValueError("fp8 quantize needs numel % 16 == 0")
    amax = torch.zeros(1, dtype=torch.float32, device=x.device)
    inv = torch.empty(1, dtype=torch.float32, device=x.device)
    q = torch.empty(x.shape, dtype=torch.uint8, device=x.device)
    _chk(lib().mxr_fp8_amax(_p(x), n, _p(amax), _s()), "fp8_amax")
    _chk(lib().mxr_fp8_quant(_p(x), n, _p(q), _p(amax), _p(inv), _s()), "fp8_quant")
    return q, inv


def quantize_rows(w: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """bf16 [rows, ...] -> (uint8 e4m3fn, per-row inv_scale float[rows])."""
    w = w.contiguous()
    rows = w.shape[0]
    K = w.numel() // rows
    q = torch.empty(w.shape, dtype=torch.uint8, device=w.device)
    inv = torch.empty(rows, dtype=torch.float32, device=w.device)
    _chk(lib().mxr_fp8_quant_rows(_p(w), rows, K, _p(q), _p(inv), _s()), "fp8_quant_rows")
    return q, inv


def quantize_rows_hx8(w: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """bf16 OHWI 3x3 weights -> (e4m3 bytes in conv_hx32_f8's packed layout, per-row inv_scale): the result of
    :func:`quantize_rows` followed by the hx8 pack, in one launch.  The model's compute weights (and their flipped
    copies) come from ``ComputeWeights.hx8_quant``: all of them requantised by one launch per optimizer step."""
    from . import native as _n
    cw = _n.compute_weights()
    if cw is not None:
        hit = cw.hx8_quant(w)
        if hit is not None:
            return hit
    w = w.contiguous()
    cout, cin = int(w.shape[0]), int(w.shape[-1])
    qp = torch.empty(w.numel(), dtype=torch.uint8, device=w.device)
    inv = torch.empty(cout, dtype=torch.float32, device=w.device)
    _chk(lib().mxr_hx8_quant_pack(_p(w), cout, cin, _p(qp), _p(inv), _s()), "hx8_quant_pack")
    return qp, inv


def quantize_bf8(x: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """bf16 gradient -> (e5m2 bytes as uint8, inv_scale float[1]); ``x ~= q * inv_scale``."""
    x = x.contiguous()
    n = x.numel()
    if n % 16:
        raise ValueError("bf8 quantize needs numel % 16 == 0")
    amax = torch.zeros(1, dtype=torch.float32, device=x.device)
    inv = torch.empty(1, dtype=torch.float32, device=x.device)
    q = torch.empty(x.shape, dtype=torch.uint8, device=x.device)
    _chk(lib().mxr_fp8_amax(_p(x), n, _p(amax), _s()), "fp8_amax")
    _chk(lib().mxr_bf8_quant(_p(x), n, _p(q), _p(amax), _p(inv), _s()), "bf8_quant")
    return q, inv


def dequantize_bf8(q: torch.Tensor, inv: torch.Tensor) -> torch.Tensor:
    return q.view(torch.float8_e5m2).float() * inv


def dequantize(q: torch.Tensor, inv: torch.Tensor) -> torch.Tensor:
    """Reference decode (tests): fp32 values of the e4m3fn bytes times their scale."""
    v = q.view(torch.float8_e4m3fn).float()
    if inv.numel() == 1:
        return v * inv
    return v * inv.view((-1,) + (1,) * (v.dim() - 1))


MARGIN = 2.0     # delayed scaling headroom: this step's activations may grow 2x over the last step's amax


class AmaxState:
    """Per-layer delayed-scaling state of a fused fp8 output: three device floats rotated by a host
    phase counter (previous step's amax -> this step's scale; this step's amax is max-reduced by the
    kernel; the third slot is cleared for the next step)."""

    def __init__(self, device):
        self.amax3 = torch.zeros(3, dtype=torch.float32, device=device)
        self.phase = 0

    @property
    def ready(self) -> bool:
        return self.phase > 0

    def advance(self) -> None:
        self.phase += 1


_AMAX: "dict[object, AmaxState]" = {}
_QCACHE: "list[tuple]" = []     # [(weakref(x), version, q, inv)], newest last
_QCACHE_MAX = 8     # both head towers interleave in the backward: two live copies each


def amax_state(key, device) -> AmaxState:
    """The delayed-scaling state of ``key``: a parameter tensor (or ``(tag, parameter)``) keeps its state on the
    tensor object itself -- an ``id()`` key outlived its model and a later model whose weight reused the id
    started from the stale amax (saturated fp8 copies on its first steps); other keys (strings) live in a
    process table that :func:`reset_state` clears (``Trainer`` does at construction)."""
    tag, obj = ("fwd", key) if isinstance(key, torch.Tensor) else (
        (key[0], key[1]) if isinstance(key, tuple) and len(key) == 2 and isinstance(key[1], torch.Tensor)
        else (None, None))
    if obj is not None:
        d = obj.__dict__.setdefault("_mxr_amax", {})
        st = d.get(tag)
        if st is None:
            st = d[tag] = AmaxState(device)
        return st
    st = _AMAX.get(key)
    if st is None:
        st = _AMAX[key] = AmaxState(device)
    return st


def cache_put(x: torch.Tensor, q: torch.Tensor, inv: torch.Tensor) -> None:
    """Remember the fp8 copy of ``x`` (produced by the fused epilogue) for its consumer."""
    import weakref
    _QCACHE.append((weakref.ref(x), x._version, q, inv))
    del _QCACHE[:-_QCACHE_MAX]


def cache_get(x: torch.Tensor):
    pinned = getattr(x, "_mxr_f8copy", None)     # an fp8-only tensor carries its copy (no LRU eviction)
    if pinned is not None:
        return pinned
    for ref, ver, q, inv in reversed(_QCACHE):
        if ref() is x and x._version == ver:
            return q, inv
    return None


def quantize_cached(x: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    hit = cache_get(x)
    if hit is not None:
        return hit
    q, inv = quantize(x)
    cache_put(x, q, inv)
    return q, inv


def reset_state() -> None:
    _AMAX.clear()
    _QCACHE.clear()


def hx8_tiles(g: ConvGeom, device):
    """conv_hx32_f8's (device tile table, ntiles) for ``g`` (ops/halo.py, cached)."""
    from . import halo as _hx
    return _hx.device_tiles(_hx.geom_batch(g), _hx.geom_shapes(g), device)


def launch(xq, inv_x, wq, inv_w, bias, res, y, g: ConvGeom, relu: bool, variant: int = 0, fo=None,
           mask=None, accumulate: bool = False, packed: bool = False, store_y: bool = True) -> torch.Tensor:
    """``fo = (yq or None, AmaxState, inv_out)``: also emit the fp8 copy of y for the next layer.
    ``mask`` / ``accumulate`` (conv_p8_f8 only): relu-gradient mask and y += result.  ``packed``: ``wq``
    is already in conv_hx32_f8's layout (:func:`quantize_rows_hx8`).  ``store_y=False`` (conv_hx32_f8, a relu
    layer writing its fp8 copy and a conv_launch.BitMask ``mask``): no bf16 output is written at all."""
    yq = amax3 = inv_out = None
    phase = 0
    if fo is not None:
        yq, st, inv_out = fo
        amax3, phase = st.amax3, st.phase
    if variant in HX8_VARIANTS or variant in HX8_DGRAD_VARIANTS:
        if not hx8_covers(g):
            raise RuntimeError("conv3x3_hx32_f8: geometry not covered")
        tiles, nt = hx8_tiles(g, y.device)
        wp = wq
        if not packed:
            wp = torch.empty(wq.numel(), dtype=torch.uint8, device=wq.device)
            _chk(lib().mxr_hx8_pack_weights(_p(wq), _p(wp), g.cout, g.cin, _s()), "hx8_pack")
        _chk(lib().mxr_conv3x3_hx32_f8(_p(xq), _p(wp), _p(inv_x), _p(inv_w), _p(bias), _p(res), _p(mask),
                                       _p(y) if store_y else None,
                                       _p(zero_page(y.device)), ctypes.byref(g), _p(tiles), nt, int(relu),
                                       int(accumulate), _p(yq), _p(amax3), _p(inv_out), int(phase), float(MARGIN),
                                       variant - 20, _s()),
             "conv3x3_hx32_f8")
        return y
    if variant in P8F_VARIANTS or variant in F8_DGRAD_VARIANTS or variant == P8F_ABLATE:
        kv = 9 if variant == P8F_ABLATE else variant - 6      # 6, 7 -> 0, 1 (forward); 10, 11 -> 4, 5 (dgrad)
        _chk(lib().mxr_conv_p8_f8(_p(xq), _p(wq), _p(inv_x), _p(inv_w), _p(bias), _p(res), _p(mask), _p(y),
                                  _p(zero_page(y.device)), ctypes.byref(g), int(relu), int(accumulate), _p(yq),
                                  _p(amax3), _p(inv_out), int(phase), float(MARGIN), kv, _s()),
             "conv_p8_f8")
        return y
    if not store_y:
        raise ValueError("fp8 variant %d always writes its bf16 output" % variant)
    if mask is not None or accumulate:
        raise ValueError("fp8 variant %d has no mask / accumulate epilogue" % variant)
    _chk(lib().mxr_conv_fwd_f8(_p(xq), _p(wq), _p(inv_x), _p(inv_w), _p(bias), _p(res), _p(y),
                               _p(zero_page(y.device)), ctypes.byref(g), int(relu), _p(yq), _p(amax3), _p(inv_out),
                               int(phase), float(MARGIN), int(variant), _s()),
         "conv_fwd_f8")
    return y


def pyramid_forward(x, w, b, g: ConvGeom, relu: bool, out_shape, key, tuner_key, f8_only: bool = False,
                    focal=None, focal_dq_ok: bool = False):
    """fp8 forward of one packed head layer: the input's fp8 copy comes from the producing layer's
    fused epilogue when it has one (else one quantisation pass, shared by both subnets); relu layers
    (the tower) emit their own fp8 copy for the next layer with the delayed scale of ``key``.

    ``f8_only`` (the only reader is the next fp8 head layer, with fp8 weight gradients): once the tuned hx8 kernel
    emits the fp8 copy, it writes the relu mask as bits (``y._mxr_bits``) INSTEAD of the bf16 output -- the 183 MB
    store and the next data gradient's 183 MB mask read become 11 MB each.  The returned bf16 tensor is then never
    written (``y._mxr_f8only``; every reader of it raises).

    ``focal`` (a conv_launch.FocalRequest, the classification final): with the tuned hx8 kernel the focal loss runs
    in its epilogue -- no logits; ``y._mxr_focal_dpad`` = the padded gradient rows, ``focal.loss`` the loss.
    ``focal_dq_ok``: the layer's backward takes an e5m2-only dY (its weight has a gradient, fp8 weight gradients,
    the bias from the same kernel through gradient sinks); otherwise the rows always come out in bf16."""
    from .conv_tuner import TUNER
    if getattr(x, "_mxr_f8only", False) and cache_get(x) is None:
        raise RuntimeError("fp8 head layer: the input is an fp8-only tower output without its fp8 copy")
    xq, ix = quantize_cached(x)
    # the fused-loss and no-bf16-output forms exist for the first hx8 variant only: adopt it over a near-tie
    # winner (ConvTuner.prefer; the race times the bare convolution, not the work the form removes)
    if focal is not None and not relu and b is not None and g.cout == 80 * focal.A:
        from .conv_launch import FOCAL_PREFER_MS
        TUNER.prefer(tuner_key, "f8_%d" % HX8_VARIANTS[0], FOCAL_PREFER_MS)
    elif f8_only and relu:
        TUNER.prefer(tuner_key, "f8_%d" % HX8_VARIANTS[0], F8ONLY_PREFER_MS)
    win = TUNER.winner(tuner_key)
    fused = win is not None and win.startswith("f8_") and int(win[3:]) in HX8_VARIANTS
    wq, iw = quantize_rows_hx8(w) if fused else quantize_rows(w)     # tuned hx8 winner: one fused launch
    fo = None
    if relu:
        st = amax_state(key, x.device)
        yq = torch.empty(out_shape, dtype=torch.uint8, device=x.device) if st.ready else None
        fo = (yq, st, torch.empty(1, dtype=torch.float32, device=x.device))

    if (focal is not None and fused and int(win[3:]) == HX8_VARIANTS[0] and not relu and fo is None
            and b is not None and g.cout == 80 * focal.A and focal.gamma == 2.0):
        return _focal_forward(xq, ix, wq, iw, b, g, focal, out_shape, x.device, key if focal_dq_ok else None)
    bits = None
    # (the no-bf16-output form is a compile-time epilogue of the 256-channel tiles only: conv_hx32_f8.hip launch_form)
    if f8_only and fused and int(win[3:]) == HX8_VARIANTS[0] and relu and fo is not None and fo[0] is not None:
        from .conv_launch import BitMask
        bits = BitMask(shape=out_shape, device=x.device)

    def run(v):
        y = torch.empty(out_shape, dtype=torch.bfloat16, device=x.device)
        return launch(xq, ix, wq, iw, b, None, y, g, relu, v, fo, packed=fused, mask=bits, store_y=bits is None)
    if fused:
        y = TUNER.run(tuner_key, {win: (lambda: run(int(win[3:])))})
        if bits is not None:
            y._mxr_bits = bits
            y._mxr_f8only = True
            y._mxr_f8copy = (fo[0], fo[2])
    else:
        y = TUNER.run(tuner_key, {"f8_%d" % v: (lambda v=v: run(v)) for v in variants_for(g.cin, g)})
    if fo is not None:
        if fo[0] is not None:
            cache_put(y, fo[0], fo[2])
        fo[1].advance()
    return y


# backbone / FPN fp8 candidates: the input in ONE delayed-scaling pass (per-layer AmaxState) and the 3x3 weights from
# the per-step batched quantisation instead of a two-pass quantize + per-call weight quantisation and packing (a
# switch for same-process A/Bs)
LEAN_CANDIDATES = True


def candidates(x, w, b, res, g: ConvGeom, relu: bool, out_shape) -> dict:
    """Tuner candidates of one fp8 forward (quantisation of x and W included in each).

    With :data:`LEAN_CANDIDATES` the input is quantised in one pass with the layer's delayed scale (state kept on the
    compute weight ``w``: ``("bbx", w)``) and the conv_hx32_f8 weights come from ``ComputeWeights.hx8_quant`` (every
    registered weight requantised by one launch per optimizer step) -- so an fp8 3x3 conv of the backbone / FPN costs
    one quantisation pass more than its MFMA work, and the race can pick it where that pays (round 6)."""
    lean = LEAN_CANDIDATES

    def run(v):
        xq, ix = quantize_delayed(x, ("bbx", w), bf8=False) if lean else quantize(x)
        packed = lean and v in HX8_VARIANTS
        wq, iw = quantize_rows_hx8(w) if packed else quantize_rows(w)
        y = torch.empty(out_shape, dtype=torch.bfloat16, device=x.device)
        return launch(xq, ix, wq, iw, b, res, y, g, relu, v, packed=packed)
    return {"f8_%d" % v: (lambda v=v: run(v)) for v in variants_for(g.cin, g)}


def conv2d_fp8(x: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor], stride: int, pads, relu: bool = False,
               residual: Optional[torch.Tensor] = None, variant: int = 0) -> torch.Tensor:
    """Forward-only fp8 NHWC conv of bf16 inputs (quantises both operands)."""
    from .native_conv import geom_single, _out_hw
    N, H, W, cin = x.shape
    cout, kh = w.shape[0], w.shape[1]
    Ho, Wo = _out_hw(H, W, kh, stride, pads)
    g = geom_single(N, H, W, Ho, Wo, kh, stride, pads, cin, cout)
    xq, ix = quantize(x)
    wq, iw = quantize_rows(w)
    y = torch.empty((N, Ho, Wo, cout), dtype=torch.bfloat16, device=x.device)
    b = None if bias is None else bias.float().contiguous()
    r = None if residual is None else residual.contiguous()
    return launch(xq, ix, wq, iw, b, r, y, g, relu, variant)


def dgrad_eligible(cin_dgrad: int, cout_dgrad: int) -> bool:
    """conv_p8_f8's data-gradient form: 128-channel K-tiles over dY's channels, 16-B output chunks."""
    return cin_dgrad % 128 == 0 and cout_dgrad % 8 == 0


def pyramid_dgrad(dy, wd, g: ConvGeom, mask, out_shape, key, tuner_key, emit: bool, out=None, f8_only: bool = False):
    """fp8 data gradient of one packed head layer: dX = conv(dY, flip(W)) with dY in e5m2 (the fp8 copy the
    layer above emitted from its own data-gradient epilogue, else one quantisation pass) and the flipped
    weights in e4m3 per row; ``mask`` fuses the producer's relu backward, ``out`` accumulates (the towers'
    shared input), ``emit`` writes dX's e5m2 copy for the next data gradient (delayed scaling of ``key``).

    ``f8_only`` (dX's only reader is an fp8 tower layer's backward, whose data / weight / bias gradients all take the
    e5m2 copy): once the tuned hx8 kernel emits the copy under a bitmask ``mask``, no bf16 dX is written --
    ``dx._mxr_f8only``; the 183 MB store per layer is gone (the forward's fp8-only outputs, mirrored)."""
    from .conv_tuner import TUNER
    dq, idq = quantize_bf8_cached(dy)
    if f8_only:
        TUNER.prefer(tuner_key, "f8d_%d" % HX8_DGRAD_VARIANTS[0], F8ONLY_PREFER_MS)
    win = TUNER.winner(tuner_key)
    fused = win is not None and win.startswith("f8d_") and int(win[4:]) in HX8_DGRAD_VARIANTS
    wq, iw = quantize_rows_hx8(wd) if fused else quantize_rows(wd)
    fo = None
    if emit:
        st = amax_state(key, dy.device)
        yq = torch.empty(out_shape, dtype=torch.uint8, device=dy.device) if st.ready else None
        fo = (yq, st, torch.empty(1, dtype=torch.float32, device=dy.device))

    from .conv_launch import BitMask
    noy = (f8_only and fused and int(win[4:]) == HX8_DGRAD_VARIANTS[0] and out is None and fo is not None
           and fo[0] is not None and isinstance(mask, BitMask))

    def run(v, dst):
        y = dst if dst is not None else torch.empty(out_shape, dtype=torch.bfloat16, device=dy.device)
        return launch(dq, idq, wq, iw, None, None, y, g, False, v, fo, mask=mask, accumulate=dst is not None,
                      packed=fused, store_y=not noy)
    dvs = F8_DGRAD_VARIANTS + (HX8_DGRAD_VARIANTS if hx8_covers(g) else ())
    if fused:
        dvs = (int(win[4:]),)
    cands = {"f8d_%d" % v: (lambda v=v: run(v, out)) for v in dvs}
    if out is not None and TUNER.needs_tuning(tuner_key, cands):
        TUNER.run(tuner_key, {"f8d_%d" % v: (lambda v=v: run(v, out.clone())) for v in dvs})
    y = TUNER.run(tuner_key, cands)
    if noy:
        y._mxr_f8only = True
        y._mxr_f8copy = (fo[0], fo[2])
    if fo is not None:
        if fo[0] is not None:
            cache_put(y, fo[0], fo[2])
        fo[1].advance()
    return y


def _focal_forward(xq, ix, wq, iw, b, g: ConvGeom, req, out_shape, device, key=None):
    """conv_hx32_f8's FOCAL form (the classification final, 256-channel tiles): returns the unwritten logits
    placeholder carrying the padded gradient rows (``_mxr_focal_dpad``); the loss goes to ``req.loss``.

    With ``key`` (the layer's weight) and :data:`FOCAL_DQ`, once the delayed scale of the layer's dY copy
    (``("dyq", key)``, the state the backward's quantisation seeds) has history, the rows leave the epilogue as their
    e5m2 copy only: ``_mxr_focal_dpad`` is then an fp8-only placeholder carrying that copy -- no 548 MB bf16 rows, no
    quantisation pass over them (the fp8 data / weight / bias gradients read nothing else)."""
    from . import halo as _hx
    from .losses import LOGIT_HI, LOGIT_LO
    if not (int(req.state.numel()) == int(g.M) * req.A and int(req.label.numel()) == int(g.M) * req.A
            and b.dtype == torch.float32 and b.data_ptr() % 16 == 0):
        raise RuntimeError("conv3x3_hx32_f8_focal: targets do not match the geometry")
    tiles, nt = _hx.device_tiles(_hx.geom_batch(g), _hx.geom_shapes(g), device)
    ld = (g.cout + 63) // 64 * 64
    nparts = -(-g.cout // 256) * nt
    parts = torch.empty(nparts, dtype=torch.float32, device=device)
    out = torch.empty(1, dtype=torch.float32, device=device)
    n, p = int(g.M) // g.out_img, g.out_img
    st = amax_state(("dyq", key), device) if (key is not None and FOCAL_DQ and WGRAD and WGRAD_BIAS) else None
    if st is not None and st.ready:
        dq = req.dpad_q(n, p, ld, device)
        inv = torch.empty(1, dtype=torch.float32, device=device)
        _chk(lib().mxr_conv3x3_hx32_f8_focal_q(_p(xq), _p(wq), _p(ix), _p(iw), _p(b), _p(zero_page(device)),
                                               ctypes.byref(g), _p(tiles), nt, _p(req.state.contiguous()),
                                               _p(req.label.contiguous()), _p(req.npos), None, ld, req.A, 80,
                                               float(req.alpha), float(req.gamma), LOGIT_LO, LOGIT_HI, _p(parts), nparts,
                                               _p(out), _p(dq), _p(st.amax3), _p(inv), st.phase % 3, float(MARGIN),
                                               _s()), "conv3x3_hx32_f8_focal_q")
        st.advance()
        dpad = torch.empty((n, p, ld), dtype=torch.bfloat16, device=device)     # never written
        dpad._mxr_f8only = True
        dpad._mxr_f8copy = (dq, inv)
    else:
        dpad = req.dpad(n, p, ld, device)
        _chk(lib().mxr_conv3x3_hx32_f8_focal(_p(xq), _p(wq), _p(ix), _p(iw), _p(b), _p(zero_page(device)),
                                             ctypes.byref(g), _p(tiles), nt, _p(req.state.contiguous()),
                                             _p(req.label.contiguous()), _p(req.npos), _p(dpad), ld, req.A, 80,
                                             float(req.alpha), float(req.gamma), LOGIT_LO, LOGIT_HI, _p(parts), nparts,
                                             _p(out), _s()), "conv3x3_hx32_f8_focal")
    req.loss = out.reshape(())
    y = torch.empty(out_shape, dtype=torch.bfloat16, device=device)
    y._mxr_unwritten = True
    y._mxr_focal_dpad = dpad
    from .conv_launch import FOCAL_LAUNCHES
    FOCAL_LAUNCHES[0] += 1
    return y


def quantize_delayed(x: torch.Tensor, key, bf8: bool = True) -> Tuple[torch.Tensor, torch.Tensor]:
    """``quantize_bf8`` (``quantize`` for ``bf8=False``) in ONE pass with delayed scaling (:class:`AmaxState` of
    ``key``): the scale is the previous step's amax times :data:`MARGIN`, this step's amax is recorded for the next
    (``mxr_quant_delayed``). The first step (no history) quantises with its own amax and seeds the state."""
    x = x.contiguous()
    n = x.numel()
    if n % 16:
        raise ValueError("fp8 quantize needs numel % 16 == 0")
    st = amax_state(key, x.device)
    if not st.ready:
        q, inv = quantize_bf8(x) if bf8 else quantize(x)
        st.amax3[0].copy_(inv[0] * (BF8_MAX if bf8 else FP8_MAX))     # amax of this step, slot of phase 0
        st.advance()
        return q, inv
    inv = torch.empty(1, dtype=torch.float32, device=x.device)
    q = torch.empty(x.shape, dtype=torch.uint8, device=x.device)
    _chk(lib().mxr_quant_delayed(_p(x), n, _p(q), _p(st.amax3), st.phase % 3, float(MARGIN), _p(inv), int(bf8), _s()),
         "quant_delayed")
    st.advance()
    return q, inv


BF8_MAX = 57344.0


def quantize_bf8_cached(x: torch.Tensor, key=None) -> Tuple[torch.Tensor, torch.Tensor]:
    """The e5m2 copy of ``x``: a producer epilogue's cached copy, else one quantisation pass (delayed scaling of
    ``key`` when given), remembered for the next consumer of ``x``."""
    hit = cache_get(x)
    if hit is not None:
        return hit
    q, inv = quantize_delayed(x, key) if key is not None else quantize_bf8(x)
    cache_put(x, q, inv)
    return q, inv


def wgrad_eligible(g: ConvGeom, ldy: int) -> bool:
    """conv_wgrad_p8_f8.hip: 16-channel fp8 chunks of the input and of dY's row pitch, no output scatter."""
    return g.cin % 16 == 0 and ldy % 16 == 0 and g.ostride == 1 and 1 <= g.nlev <= 5


def _wgrad_splits(g: ConvGeom) -> int:
    """Pixel splits of the fp8 wgrad grid: ~144 blocks (fewer than conv_wgrad_p8's 192: the fp8 kernels are shorter
    next to the concurrent fp8 data gradients), each split at least 4 K-tiles of 128 pixels."""
    K = g.kh * g.kw * g.cin
    tiles = ((K + 255) // 256) * ((g.cout + 255) // 256)
    ntm = (int(g.M) + 127) // 128
    # 144 blocks: the same-box sweep over 96 / 120 / 144 / 168 / 192 / 256 (profiles/r5_fp8_wgrad_blocks_sweep.txt)
    target = int(os.environ.get("MXR_WGRAD_HEAD_BLOCKS", "144"))
    return int(max(1, min(max(1, round(target / tiles)), max(1, ntm // 4))))


def pyramid_wgrad(xq, ix, dq, idq, g: ConvGeom, out: Optional[torch.Tensor] = None, accumulate: bool = False,
                  variant: int = 0, splits: Optional[int] = None, bias_out: Optional[torch.Tensor] = None,
                  bias_accumulate: bool = False) -> torch.Tensor:
    """fp32 (cout, kh, kw, cin) weight gradient from the e4m3 input copy ``xq`` (scale ``ix``) and the e5m2
    gradient copy ``dq`` (scale ``idq``, row pitch >= cout, columns past cout ignored) on
    ``conv_wgrad_p8_f8``; ``out`` (+)= the result.  ``bias_out`` (fp32 (cout,)): the bias gradient
    ``idq * sum_m dq[m, :cout]`` from the same kernel (the kernel's BIAS form), (+)= when ``bias_accumulate``."""
    ldy = int(dq.shape[-1])
    if not wgrad_eligible(g, ldy):
        raise RuntimeError("conv_wgrad_p8_f8: geometry not covered")
    if not (xq.dtype == torch.uint8 and dq.dtype == torch.uint8 and xq.is_contiguous() and dq.is_contiguous()
            and int(xq.numel()) == int(g.M) * g.cin and int(dq.numel()) == int(g.M) * ldy and ldy >= g.cout):
        raise RuntimeError("conv_wgrad_p8_f8: operands do not match the geometry")
    if bias_out is not None and not (bias_out.dtype == torch.float32 and bias_out.is_contiguous()
                                     and bias_out.numel() == g.cout):
        raise RuntimeError("conv_wgrad_p8_f8: the bias gradient needs a contiguous fp32 (cout,) output")
    K = g.kh * g.kw * g.cin
    s = splits or _wgrad_splits(g)
    part = torch.empty(s * g.cout * (K + (1 if bias_out is not None else 0)), dtype=torch.float32, device=dq.device)
    if out is None:
        out = torch.empty((g.cout, g.kh, g.kw, g.cin), dtype=torch.float32, device=dq.device)
        accumulate = False
    _chk(lib().mxr_conv_wgrad_p8_f8_bias(_p(xq), _p(dq), ldy, _p(ix), _p(idq), _p(part), s, _p(out), None,
                                         int(accumulate), _p(zero_page(dq.device)), ctypes.byref(g), int(variant),
                                         _p(bias_out), int(bias_accumulate), _s()),
         "conv_wgrad_p8_f8")
    return out


def deliver_pyramid_wgrad(f8x, f8dy, g: ConvGeom, param, reads=(), bias_param=None) -> Optional[torch.Tensor]:
    """The fp8 weight gradient of a packed head layer into ``param``'s gradient sink (on the side stream when
    usable, like the bf16 wgrads; returns None), or as a tensor when the parameter has no sink.  ``bias_param``
    (with a sink, :data:`WGRAD_BIAS`): its gradient comes out of the same kernel; callers check
    :func:`bias_fusable` first."""
    from . import native as _n
    from .side_stream import SIDE
    xq, ix = f8x
    dq, idq = f8dy
    gs = _n.grad_sinks()
    sink = gs.get(param) if gs is not None else None
    if sink is None:
        return pyramid_wgrad(xq, ix, dq, idq, g)
    out = sink.view(g.cout, g.kh, g.kw, g.cin)
    bsink = gs.get(bias_param) if bias_param is not None else None

    def run():
        pyramid_wgrad(xq, ix, dq, idq, g, out=out, accumulate=True, variant=WGRAD_VARIANT, bias_out=bsink,
                      bias_accumulate=True)
        gs.notify(param)
        if bsink is not None:
            gs.notify(bias_param)
    side = SIDE.usable(sink) and not getattr(param, "mxr_main_wgrad", False)
    if side:
        with SIDE.run(sink.device, xq, ix, dq, idq, *reads):
            run()
        return None
    run()
    return None


def bias_fusable(param, bias_param) -> bool:
    """Whether :func:`deliver_pyramid_wgrad` can take ``bias_param``'s gradient too: both parameters have gradient
    sinks (the training step) and the fused form is on."""
    from . import native as _n
    gs = _n.grad_sinks()
    return (WGRAD_BIAS and bias_param is not None and gs is not None and gs.get(param) is not None
            and gs.get(bias_param) is not None)
