"""HIP implicit-GEMM convolution layers: the autograd nodes over the kernel launchers.

Launchers / forward candidates: ``conv_launch``; data gradients: ``conv_dgrad``; weight / bias gradients:
``conv_wgrad`` (all re-exported here).  This module: ``GradJoin``, the conv / residual-block / pyramid
autograd functions and the pyramid pack.

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
from .conv_launch import (  # noqa: F401  (re-exported: the public surface of native_conv)
    MASK_BITS, BitMask, bits_capable, proj_fusable, run_fwd_proj, run_fwd_into, C1X1_BN, FWD_VARIANTS, HALO_VARIANTS, HX32_VARIANTS, P8_TUNED, P8_VARIANTS, _BOUND, _SIGS, _bind,
    _effective, _miopen_pyramid_wgrad, _miopen_wgrad, _only, _only_fwd, _out_hw, _variant, bias_res_act_,
    big_tile_variants, c1x1_variants, flip, fwd_candidates, geom_pyramid, geom_single, hip_conv_ok,
    hx32_covers, hx32_packed, launch_c1x1, launch_fwd, launch_halo, launch_hx32, launch_p8, miopen_fwd,
    p8_covers, relu_bwd, relu_bwd_, run_fwd, torch_conv_backward,)
from .conv_dgrad import (  # noqa: F401  (re-exported: the public surface of native_conv)
    proj_dgrad_fusable, run_dgrad_proj, _S2_TAPS, _dgrad_cands, _dgrad_s2_subpixel, _pick_taps, _s2_phase_taps, _s2_stack_taps,
    _s2_stacked_weights, _s2_stacked_weights_hip, conv_dgrad, run_dgrad,)
from .conv_wgrad import (  # noqa: F401  (re-exported: the public surface of native_conv)
    proj_wgrad_fusable, run_wgrad_proj, _WGRAD_P8, _WGRAD_PIPE_OCC, _WGRAD_PIPE_TILE, _WGRAD_TILE, _WGRAD_VS, _WH_TILES, _deliver_wgrad,
    _only_wgrad, _sink, _splits, _splits_pipe, _wgrad_sink_cands, _wh_box, bias_grad, conv_wgrad,
    deliver_bias_grad, deliver_wgrad_bias_fused, halo_wgrad, halo_wgrad_tiles, run_wgrad, run_wgrad_bias_fused,
    w64_covers, wgrad3x3_c64, wgrad_candidates, whalo_covers,)


class GradJoin:
    """Input-gradient join for a ReLU output consumed by ``n`` HIP conv nodes (C3 / C4 / C5: the next
    ResNet stage and the FPN lateral / P6 convs).

    Autograd would hand each consumer's dX to a separate buffer, add them, and the producing block
    would then run a ReLU backward over the sum -- two activation-sized passes.  Instead the first
    consumer to run writes its dX and returns it; the others accumulate into that same buffer through
    their dgrad epilogues (and return None).  EVERY consumer applies the ReLU mask in its epilogue
    (mask(a + b) = mask(a) + mask(b) for a 0/1 mask, and an accumulate-then-mask over an already masked
    buffer only masks the new term), so the producer skips its ReLU backward (``grad_premasked``) and
    no consumer order needs a separate pass -- a 1x1/s2 scatter dgrad that only visits the stride grid
    leaves the gaps to the other consumers' (masked) writes or to its own zeros.  One mask read per
    consumer instead of a read-read-write pass over the activation after the last one.
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
        # a GradJoin consumer (FPN lateral on C3 / C4 / C5) masks with the block output's bitmask when its
        # producer wrote one and this is a 1x1 (the 3x3/s2 P6 dgrad's shuffle reads a bf16 mask)
        ctx.bits_in = getattr(x, "_mxr_bits", None) if (join is not None and w.shape[1] == 1) else None
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
                buf, _ = ctx.join.claim()
                r = run_dgrad(dy, w, x, stride, pads, mask=ctx.bits_in if ctx.bits_in is not None else x, out=buf)
                if buf is None:
                    ctx.join.buf = dx = r
                else:
                    if r is not buf:
                        buf.copy_(r)
                    ctx.join.release()
            else:
                dx = run_dgrad(dy, w, x, stride, pads)
        fused_bias = (ctx.needs_input_grad[1] and has_bias and ctx.needs_input_grad[2]
                      and run_wgrad_bias_fused(x, dy, w, stride, pads, scale, ctx.params[0], ctx.params[1]))
        if ctx.needs_input_grad[1] and not fused_bias:
            dw = run_wgrad(x, dy, w, stride, pads, scale, param=ctx.params[0])
        if has_bias and ctx.needs_input_grad[2] and not fused_bias:
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
        # projection block: branch2c + branch1 + add + relu as ONE dual-source GEMM when the shapes allow it (the
        # shortcut is then never materialised: conv_launch.run_fwd_proj)
        proj = (specs[nconv] is not None and nconv >= 2 and specs[nconv - 1] == (1, (0, 0, 0, 0))
                and specs[nconv][1] == (0, 0, 0, 0))
        if specs[nconv] is not None and not proj:
            st, pd = specs[nconv]
            shortcut = run_fwd(x, ws[nconv][0], ws[nconv][1], None, st, pd, False)
        else:
            shortcut = x if specs[nconv] is None else None
        hs = [x]
        h = x
        cout = ws[nconv - 1][0].shape[0]
        # the output's ReLU mask as bits for the next block's 1x1 data gradient (conv_launch.BitMask); the mask
        # of our own input, if its producer wrote one
        # only when a backward will run (grad mode on and some input needs a gradient): under no_grad / eval
        # nothing reads the bits, and the plain forward key (fp8-capable, no bit emission) is kept
        bits_ok = MASK_BITS and x.is_cuda and any(ctx.needs_input_grad) and cout % 8 == 0
        emit = None
        ctx.bits_in = getattr(x, "_mxr_bits", None)
        # (the inner ReLU masks stay bf16 saved outputs: as bits they measured -0.2 %, profiles/r4_mask_bits_ab.txt)
        chunk = _block_chunk(x, specs)
        if chunk:
            # identity block, image by image in chunks: a chunk's input is read by conv_0 and again, as the
            # residual, by the last conv a few launches later -- small enough to still sit in the 256 MB
            # Infinity Cache then, instead of coming from HBM twice (stage 2: 547 MB per read at B=16)
            hs = [x] + _chunked_chain(x, ws, specs, nconv, cout, bits_ok, chunk)
            h = hs[-1]
            emit = getattr(h, "_mxr_bits", None)
        for i in (range(nconv) if not chunk else ()):
            st, pd = specs[i]
            last = i == nconv - 1
            if last and bits_ok:     # (the last conv is stride 1, 'same': the block output has h's grid)
                emit = BitMask(shape=tuple(h.shape[:3]) + (cout,), device=x.device)
            if last and specs[nconv] is not None and shortcut is None:
                w2c, b2c = ws[i]
                w1, b1 = ws[nconv]
                st1 = specs[nconv][0]
                if proj_fusable(h, x, w2c, w1, st1):
                    h = run_fwd_proj(h, x, w2c, w1, b2c + b1, st1, emit=emit)
                else:
                    shortcut = run_fwd(x, w1, b1, None, st1, specs[nconv][1], False)
                    h = run_fwd(h, w2c, b2c, shortcut, st, pd, True, emit=emit)
            else:
                h = run_fwd(h, ws[i][0], ws[i][1], shortcut if last else None, st, pd, True, emit=emit if last else None)
            hs.append(h)
        if emit is not None:
            h._mxr_bits = emit
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
        jbuf, mask_in = None, ctx.mask_in
        if ctx.join is not None and need_x:
            # x has other consumers (GradJoin): accumulate into the shared buffer if one exists and mask
            # our contribution (every consumer does; a 1x1/s2 block's scatter dgrads only touch the
            # stride grid, whose gaps hold the other consumers' masked terms or zeros)
            jbuf, _ = ctx.join.claim()
            mask_in = True
        dh_last = None
        wfused = False
        if ctx.has_b1:
            st, pd = specs[nconv]
            if (ctx.needs_input_grad[4 + 3 * nconv] and ctx.needs_input_grad[4 + 3 * (nconv - 1)] and nconv >= 2
                    and specs[nconv - 1] == (1, (0, 0, 0, 0)) and pd == (0, 0, 0, 0)
                    and proj_wgrad_fusable(hs[nconv - 1], hs[0], g, ws[nconv - 1], ws[nconv], st)):
                # branch2c's and branch1's weight gradients from one read of g, into both sinks (run_wgrad_proj)
                wfused = run_wgrad_proj(hs[nconv - 1], hs[0], g, st, scs[nconv - 1], scs[nconv],
                                        ctx.wparams[nconv - 1], ctx.wparams[nconv])
            if ctx.needs_input_grad[4 + 3 * nconv] and not wfused:
                grads[3 * nconv] = run_wgrad(hs[0], g, ws[nconv], st, pd, scs[nconv], param=ctx.wparams[nconv])
            if need_x:
                if (nconv >= 2 and specs[nconv - 1] == (1, (0, 0, 0, 0)) and pd == (0, 0, 0, 0) and
                        proj_dgrad_fusable(g, ws[nconv - 1], ws[nconv], hs[nconv - 1], tuple(hs[0].shape), st)):
                    # branch2c's and branch1's data gradients from one read of g (conv_dgrad.run_dgrad_proj)
                    dh_last, dx = run_dgrad_proj(g, ws[nconv - 1], ws[nconv], hs[nconv - 1], tuple(hs[0].shape), st,
                                                 out=jbuf)
                else:
                    dx = run_dgrad(g, ws[nconv], hs[0], st, pd, out=jbuf)
        gi = g
        for i in range(nconv - 1, -1, -1):
            st, pd = specs[i]
            if ctx.needs_input_grad[4 + 3 * i] and not (wfused and i == nconv - 1):
                grads[3 * i] = run_wgrad(hs[i], gi, ws[i], st, pd, scs[i], param=ctx.wparams[i])
            if i > 0:
                if i == nconv - 1 and dh_last is not None:
                    gi = dh_last
                    continue
                gi = run_dgrad(gi, ws[i], hs[i], st, pd, mask=hs[i])
            elif need_x:
                mk = hs[0] if mask_in else None
                if mk is not None and ctx.bits_in is not None and ws[0].shape[1] == 1:
                    mk = ctx.bits_in            # 1x1 conv_0: its epilogue reads the producer's bitmask
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
        if ctx.join is not None and need_x:
            if jbuf is None:
                ctx.join.buf = dx
            else:
                if dx is not jbuf:
                    jbuf.copy_(dx)
                ctx.join.release()
                dx = None                            # already accumulated into the first consumer's dX
        return (dx, None, None, None) + tuple(grads)

# images per chunk of an identity block's forward (MXR_BLOCK_CHUNK; 0 = whole batch) and the smallest per-image
# pixel count it applies to (stage 2 / 3 at 800x1333: 66,800 / 16,700)
_BLOCK_CHUNK = int(os.environ.get("MXR_BLOCK_CHUNK", "0"))
_BLOCK_CHUNK_MIN_PX = int(os.environ.get("MXR_BLOCK_CHUNK_MIN_PX", "10000"))


def _block_chunk(x, specs) -> int:
    if (_BLOCK_CHUNK <= 0 or specs[-1] is not None or x.shape[0] < 2 * _BLOCK_CHUNK
            or x.shape[1] * x.shape[2] < _BLOCK_CHUNK_MIN_PX or any(st != 1 for st, _ in specs[:-1])):
        return 0
    return _BLOCK_CHUNK


def _bits_view(full: BitMask, i0: int, i1: int) -> BitMask:
    """The images [i0, i1) of a bitmask (its bytes are image-major, like the activation)."""
    v = BitMask.__new__(BitMask)
    per = full.bits.numel() // full.shape[0]
    v.bits = full.bits[i0 * per:i1 * per]
    v.shape = (i1 - i0,) + tuple(full.shape[1:])
    v.device = full.device
    return v


def _chunked_chain(x, ws, specs, nconv, cout, bits_ok, chunk):
    """Conv outputs h_1..h_L of an identity block computed chunk by chunk into full-batch tensors (the saved
    activations of the backward are the same tensors as the whole-batch form's)."""
    N, H, W, _ = x.shape
    outs = [torch.empty((N, H, W, ws[i][0].shape[0]), dtype=x.dtype, device=x.device) for i in range(nconv)]
    emit = BitMask(shape=(N, H, W, cout), device=x.device) if bits_ok else None
    for i0 in range(0, N, chunk):
        i1 = min(N, i0 + chunk)
        xs = x[i0:i1]
        h = xs
        for i in range(nconv):
            st, pd = specs[i]
            last = i == nconv - 1
            em = _bits_view(emit, i0, i1) if (last and emit is not None) else None
            h = run_fwd_into(outs[i][i0:i1], h, ws[i][0], ws[i][1], xs if last else None, st, pd, True, emit=em)
    if emit is not None:
        outs[-1]._mxr_bits = emit
    return outs


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

# bf16 head towers pass relu bitmasks between layers (a switch for same-process A/Bs, not an environment knob)
HEAD_BITS = True

class PyramidConvFn(torch.autograd.Function):
    """Shared 3x3/s1/'same' conv over packed pyramid levels [B, P, C] (batch-major): all five
    levels as ONE ragged implicit GEMM per pass (the HIP kernel's multi-level geometry)."""

    @staticmethod
    def forward(ctx, x, weight, bias, shapes, relu, mask_input_grad=False, grad_premasked=False, pad_sink=None,
                join=None, out_f8=False):
        from .conv_tuner import TUNER
        x = x.contiguous()
        N, P, cin = x.shape
        cout = weight.shape[0]
        w, b = _effective(weight, None, bias, None)
        ctx.wdt = weight.dtype
        g = geom_pyramid(N, shapes, cin, cout)
        from . import fp8 as _f8
        ctx.f8x = None
        f8_only_in = getattr(x, "_mxr_f8only", False)
        # the input's relu mask as bits (an fp8-only tower output: its producer wrote no bf16 values)
        ctx.bits_in = getattr(x, "_mxr_bits", None) if mask_input_grad else None
        if f8_only_in and not (_f8.enabled() and _f8.eligible(cin, cout) and _f8.WGRAD and ctx.bits_in is not None):
            raise RuntimeError("PyramidConvFn: the input is an fp8-only tower output; this layer would read its bf16 "
                               "values")
        if _f8.enabled() and _f8.eligible(cin, cout):
            # out_f8: the only reader of this output is the next fp8 head layer (Submodel.forward_packed)
            from . import conv_launch as _cl
            req = pad_sink.get("focal") if pad_sink is not None else None
            if not (req is not None and req.state is not None and _cl.FOCAL_FUSED and req.A > 0):
                req = None
            y = _f8.pyramid_forward(x, w, b, g, relu, (N, P, cout), weight,
                                    TUNER.key("pfwd", N, tuple(shapes), cin, cout, int(relu)) + "|f8",
                                    f8_only=bool(out_f8) and _f8.WGRAD and _f8.F8_ONLY_TOWERS and MASK_BITS
                                    and relu and any(ctx.needs_input_grad), focal=req,
                                    # the focal rows may leave as an e5m2-only copy only when this layer's backward
                                    # reads nothing else: fp8 weight gradient, bias from the same kernel (sinks)
                                    focal_dq_ok=bool(weight.requires_grad and _f8.WGRAD
                                                     and (bias is None or _f8.bias_fusable(weight, bias))))
            if getattr(y, "_mxr_focal_dpad", None) is not None:
                pad_sink["dy"] = y._mxr_focal_dpad     # the fused focal loss's gradient rows (conv_launch.FocalRequest)
            if weight.requires_grad and _f8.WGRAD:
                # the input's e4m3 copy (the producer's fused copy, or this call's quantisation: a cache hit) stays
                # for the fp8 weight gradient
                ctx.f8x = _f8.quantize_cached(x)
                if getattr(y, "_mxr_f8only", False):
                    # this layer's backward can take its incoming gradient as an e5m2 copy only (fp8 data / weight
                    # gradients, the bias from the fp8 weight gradient): the reader's data gradient may skip bf16 dX
                    y._mxr_grad_f8ok = bias is None or _f8.bias_fusable(weight, bias)
        elif _focal_fused(pad_sink, relu, b, g, TUNER.key("pfwd", N, tuple(shapes), cin, cout, int(relu))):
            # the classification final with the focal loss in its epilogue (conv_launch.FocalRequest): no logits
            # are written -- the loss and the padded gradient rows the backward reads come out of the kernel
            from .conv_launch import launch_hx32_focal
            req = pad_sink["focal"]
            fv = 10 if TUNER.winner(TUNER.key("pfwd", N, tuple(shapes), cin, cout, int(relu))) == "hx32_10" else 0
            pad_sink["dy"] = launch_hx32_focal(x, w, b, g, req, (cout + 63) // 64 * 64, variant=fv)
            y = torch.empty((N, P, cout), dtype=x.dtype, device=x.device)
            y._mxr_unwritten = True
        else:
            # a bf16 tower layer's relu output also leaves its epilogue as a 1-bit mask (conv_launch.BitMask): the
            # next layer's data gradient reads 1/16 of the bytes (conv_hx32's MK = 2 / BW forms)
            emit = BitMask(shape=(N, P, cout), device=x.device) if (
                relu and MASK_BITS and HEAD_BITS and x.is_cuda and cout % 8 == 0 and any(ctx.needs_input_grad)) else None
            key = TUNER.key("pfwd", N, tuple(shapes), cin, cout, int(relu)) + ("|eb" if emit is not None else "")
            cands = fwd_candidates(x, w, b, None, g, 1, (1, 1, 1, 1), relu, (N, P, cout), allow_miopen=False,
                                   mask=emit)
            if cout % 8 and cout < 64:
                cands["pad64"] = lambda: _pad64_pfwd(x, w, b, shapes, relu)
            y = TUNER.run(key, cands)
            if emit is not None:
                y._mxr_bits = emit
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
        from . import fp8 as _f8
        dy_f8only = getattr(dy, "_mxr_f8only", False)
        if dy_f8only and not ((premasked or not relu) and ctx.f8x is not None and _f8.cache_get(dy) is not None
                              and (not has_bias or _f8.bias_fusable(ctx.params[0], ctx.params[1]))):
            raise RuntimeError("PyramidConvFn: the incoming gradient is an fp8-only data gradient; this layer would "
                               "read its bf16 values")
        if relu and not premasked:
            dy = relu_bwd(dy, y)
        dx = dw = db = None
        mk = None
        if mask_in:
            mk = ctx.bits_in if ctx.bits_in is not None else x
        f8_only_in = getattr(x, "_mxr_f8only", False)
        from . import fp8 as _f8
        f8dy = None
        if ctx.f8x is not None and ctx.needs_input_grad[1]:
            # one e5m2 copy of dY for both the fp8 weight gradient and (cache hit) the fp8 data gradient
            dq_src = dy
            if cout % 64 and dq_src.shape[-1] % 64:
                cp = (cout + 63) // 64 * 64
                dq_src = F.pad(dy, (0, cp - dy.shape[-1]))
            # (the layer above's epilogue copy, else one delayed-scaling pass: the loss gradient of the class final,
            # the tower top under the bf16 regression final)
            f8dy = _f8.quantize_bf8_cached(dq_src, key=("dyq", ctx.params[0]))
            if ctx.needs_input_grad[0] and cout % 64 and dq_src is not dy:
                dy = dq_src        # the data gradient's padded dY is this same tensor (its copy is cached)
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
            key = TUNER.key("pdgrad", N, tuple(shapes), cin, cout) + ("|mb" if isinstance(mk, BitMask) else "")
            buf = None
            if ctx.join is not None:
                # both head towers read the packed features: the second dgrad accumulates into the first's dX
                buf, _ = ctx.join.claim()
            from . import fp8 as _f8
            if _f8.enabled() and _f8.dgrad_eligible(dyp.shape[-1], cin):
                # fp8 data gradient (e5m2 dY x e4m3 W); a tower layer's dX is the next data gradient's dY, so
                # its e5m2 copy comes out of this epilogue (mask_in: x is a tower layer's relu output)
                # dX of an fp8-only tower output: its producer's backward reads only the e5m2 copy (premasked, fp8
                # data / weight gradients, the bias from the fp8 weight gradient) -> no bf16 dX (F8_ONLY_DGRAD)
                f8o = f8_only_in and _f8.F8_ONLY_DGRAD and getattr(x, "_mxr_grad_f8ok", False)
                r = _f8.pyramid_dgrad(dyp, wd, gd, mk, (N, P, cin), ("pdgrad", ctx.params[0]),
                                      key + ("|a" if buf is not None else "") + "|f8", emit=mask_in, out=buf,
                                      f8_only=f8o)
                if buf is None:
                    dx = r
                    if ctx.join is not None:
                        ctx.join.buf = dx
                else:
                    ctx.join.release()
                    dx = None
            elif buf is None:
                dx = TUNER.run(key, fwd_candidates(dyp, wd, None, None, gd, 1, (1, 1, 1, 1), False, (N, P, cin),
                                                   allow_miopen=False, mask=mk))
                if ctx.join is not None:
                    ctx.join.buf = dx
            else:
                cands = fwd_candidates(dyp, wd, None, None, gd, 1, (1, 1, 1, 1), False, (N, P, cin),
                                       allow_miopen=False, mask=mk, out=buf)
                if TUNER.needs_tuning(key + "|a", cands):
                    TUNER.run(key + "|a", fwd_candidates(dyp, wd, None, None, gd, 1, (1, 1, 1, 1), False,
                                                         (N, P, cin), allow_miopen=False, mask=mk, out=buf.clone()))
                TUNER.run(key + "|a", cands)
                ctx.join.release()
                dx = None
        fused_bias = False
        if ctx.needs_input_grad[1]:
            gw = geom_pyramid(N, shapes, cin, cout)
            wkey = TUNER.key("pwgrad", N, tuple(shapes), cin, cout)
            if f8dy is not None and _f8.wgrad_eligible(gw, int(f8dy[0].shape[-1])):
                # fp8 weight gradient (e5m2 dY x e4m3 X on the scaled MFMA); the bias gradient from the same kernel
                # (sums of the e5m2 dY) when both parameters have sinks, else a bf16 column sum
                fb = has_bias and ctx.needs_input_grad[2] and _f8.bias_fusable(ctx.params[0], ctx.params[1])
                dw = _f8.deliver_pyramid_wgrad(ctx.f8x, f8dy, gw, ctx.params[0], reads=(x, dy),
                                               bias_param=ctx.params[1] if fb else None)
                if dw is not None:
                    dw = dw.to(ctx.wdt)
                if has_bias and ctx.needs_input_grad[2] and not fb:
                    db = deliver_bias_grad(ctx.params[1], dy, channels=cout)
                return dx, dw, db, None, None, None, None, None, None, None
            fused_bias = (has_bias and ctx.needs_input_grad[2]
                          and deliver_wgrad_bias_fused(wkey, x, dy, gw, ctx.params[0], ctx.params[1]))
        if f8_only_in and ctx.needs_input_grad[1]:
            raise RuntimeError("PyramidConvFn: a bf16 weight gradient over an fp8-only tower output")
        if ctx.needs_input_grad[1] and not fused_bias:
            cands = wgrad_candidates(x, dy, gw, None)
            dyl = dy if dy.shape[-1] == cout else dy[..., :cout]
            lib_fn = lambda: _miopen_pyramid_wgrad(x, w, dyl, shapes)   # noqa: E731
            cands["miopen"] = lib_fn
            sink_make = _wgrad_sink_cands(x, dy, gw, None, lib_fn)
            if cout % 8 and cout < 64:
                # narrow regression final (36): the 64-wide pipelined wgrad on zero-padded dY rows
                # or the role-swapped GEMM (im2col over dY, X as the wide operand)
                narrow = {"pad64": lambda: _pad64_pwgrad(x, dy, shapes, cout)}
                if SWAP_NARROW_WGRAD:
                    narrow["swap"] = lambda: _swap_pwgrad(x, dy, shapes, cout)
                cands.update(narrow)
                base_make = sink_make

                def sink_make(sink, only=None, base_make=base_make, narrow=narrow):
                    if only in narrow:
                        return {only: lambda: sink.add_(narrow[only]())}
                    c = base_make(sink, only)
                    if only is None:
                        c.update({n: (lambda fn=fn: sink.add_(fn())) for n, fn in narrow.items()})
                    return c
            dw = _deliver_wgrad(wkey, cands, sink_make, ctx.params[0], (x, dy))
            if dw is not None:
                dw = dw.to(ctx.wdt)
        if has_bias and ctx.needs_input_grad[2] and not fused_bias:
            db = deliver_bias_grad(ctx.params[1], dy, channels=cout)
        return dx, dw, db, None, None, None, None, None, None, None

def _focal_fused(pad_sink, relu, b, g: ConvGeom, key: str) -> bool:
    """Whether this pyramid layer is the classification final with a focal request and a tuned conv_hx32 variant
    with the fused focal form (``conv_launch.FOCAL_VARIANTS``: 10, else 0) -- adopted over a raced winner that is
    at most ``FOCAL_PREFER_MS`` faster (``ConvTuner.prefer``)."""
    from . import conv_launch as _cl
    from .conv_tuner import TUNER
    req = pad_sink.get("focal") if pad_sink is not None else None
    return (req is not None and req.state is not None and _cl.FOCAL_FUSED and not relu and b is not None
            and req.A > 0 and g.cout == 80 * req.A and _cl.hx32_covers(g)
            and (TUNER.prefer(key, "hx32_10", _cl.FOCAL_PREFER_MS) or TUNER.prefer(key, "hx32_0", _cl.FOCAL_PREFER_MS)))

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

# the role-swapped narrow weight gradient in the race (a switch for same-process A/Bs, scripts/bench_switch.py)
SWAP_NARROW_WGRAD = True

def _swap_pwgrad(x, dy, shapes, cout):
    """fp32 (cout, 3, 3, cin) weight gradient of a narrow pyramid conv as the weight gradient of the ROLE-SWAPPED
    conv: with o_t the offset of tap t, dW[co, t, ci] = sum_p dY[p, co] X[p + o_t, ci] = sum_q dY[q - o_t, co] X[q, ci]
    -- the im2col runs over the 64-wide zero-padded dY rows (tap offsets negated = taps flipped) and the wide
    operand is X.  The GEMM is then cin (256) x 9 * 64 instead of 36 (padded to a 64- or 256-wide output tile)
    x 9 * cin: every 256-wide wgrad tile is full on the X side (the regression final, /root/reference/train.py:91's
    9 * 4 outputs)."""
    from .conv_tuner import TUNER
    N, P, cin = x.shape
    dyp = dy if dy.shape[-1] == 64 else F.pad(dy[..., :cout], (0, 64 - cout)).contiguous()
    gs = geom_pyramid(N, shapes, 64, cin)
    r = TUNER.run(TUNER.key("pwgrad", N, tuple(shapes), 64, cin, "swap"), wgrad_candidates(dyp, x, gs, None))
    # r[ci, ky', kx', co] belongs to tap (2 - ky', 2 - kx')
    return r[..., :cout].flip(1, 2).permute(3, 1, 2, 0)

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
        from . import fp8 as _f8
        if _f8.enabled():
            # fp8 heads: the e4m3 copy of the packed features comes out of this launch (delayed scaling), so the
            # towers' first layers need no amax + quantisation passes over them
            st = _f8.amax_state("pyr_features", packed.device)
            yq = torch.empty(packed.shape, dtype=torch.uint8, device=packed.device) if st.ready else None
            inv = torch.empty(1, dtype=torch.float32, device=packed.device)
            levels = [x.contiguous() for x in xs]
            ptrs = (c_vp * 5)(*([t.data_ptr() for t in levels] + [None] * (5 - len(levels))))
            hw = (c_int * 5)(*([h * w for h, w in shapes] + [0] * (5 - len(shapes))))
            _chk(lib().mxr_pyr_pack_f8(_p(packed), ptrs, hw, len(levels), N, C, _p(yq), _p(st.amax3), _p(inv),
                                       int(st.phase), float(_f8.MARGIN), _s()), "pyr_pack_f8")
            if yq is not None:
                _f8.cache_put(packed, yq, inv)
            st.advance()
            return packed
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
                       pad_sink=None, join=None, out_f8: bool = False) -> torch.Tensor:
    """``mask_input_grad``: x is a relu output whose only consumer is this layer -> its relu backward
    is fused into this layer's dgrad; ``grad_premasked``: the (sole) consumer of this layer's relu
    output does that, so skip the relu backward here; ``out_f8``: that consumer is an fp8 head layer (under fp8
    the output may then exist only as its fp8 copy and relu bitmask, ops.fp8.pyramid_forward)."""
    return PyramidConvFn.apply(x, layer.weight, layer.bias, tuple(shapes), bool(relu), bool(mask_input_grad),
                               bool(grad_premasked), pad_sink, join, bool(out_f8))

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
