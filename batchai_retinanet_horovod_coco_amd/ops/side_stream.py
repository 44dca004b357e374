"""Weight gradients on a second HIP stream, overlapped with the data-gradient chain.

A conv layer's weight gradient (wgrad GEMM + split-K reduce + bias column sums) and its data gradient
read the same dY but do not depend on each other, and only the data gradient is on the backward's
critical path (the next layer down needs it).  With the side stream on, every HIP weight gradient that
accumulates into a gradient sink (the flat fp32 buffer, ``ops.native.GradSinks``) is launched on a second
stream that first waits for the compute stream's current position, so the wgrad kernels fill the tail
rounds and launch gaps of the dgrad kernels instead of queueing behind them.  (The reference has no
such split: Keras/TF's executor schedules the backward ops itself, ``/root/reference/train.py:444-450``.)

Ordering rules kept here:

* the wgrad reads x / dY that live in compute-stream allocations -> ``record_stream`` so the caching
  allocator does not hand that memory out again before the side stream is done with it;
* no compute-stream kernel overwrites in place a tensor a side region reads: ``ResidualBlockFn``'s
  identity shortcut writes dX = dgrad + dY to a fresh buffer instead of accumulating into dY, and a
  dY handed on as a residual's gradient is referenced (:meth:`keep`) so autograd does not accumulate into it;
* a bucket's all-reduce readiness (``DistributedOptimizer._launch``) is recorded on the side stream after
  it waited for the compute stream (:meth:`SideStream.covering`), so the event covers both streams;
* the optimizer step (and any reset) makes the compute stream wait for the side stream (:meth:`join`)
  before anything reads or zeroes the gradients;
* while the conv tuner races candidates (first sight of a shape), the layer runs serially on the compute
  stream after a join, so every candidate is timed on an otherwise idle GPU;
* inside a HIP-graph capture the same fork / join events become the graph's edges (``MXR_SIDE_IN_GRAPH``).

``MXR_SIDE_WGRAD=0`` turns it off.
"""
from __future__ import annotations

import os
from typing import Dict, Optional

import torch


_RAW = getattr(torch._C, "_cuda_getCurrentRawStream", None)
_DEV = getattr(torch._C, "_cuda_getDevice", None)
_SET = getattr(torch._C, "_cuda_setStream", None)
_CAPTURING = getattr(torch._C, "_cuda_isCurrentStreamCapturing", None)


def _capturing() -> bool:
    return bool(_CAPTURING()) if _CAPTURING is not None else torch.cuda.is_current_stream_capturing()


def _set_stream(s: torch.cuda.Stream) -> None:
    if _SET is not None:
        _SET(stream_id=s.stream_id, device_index=s.device_index, device_type=s.device_type)
    else:
        torch.cuda.set_stream(s)


def _cu_masked_stream(idx: int, frac: str) -> torch.cuda.ExternalStream:
    """``MXR_SIDE_CU_FRAC=num/den``: the side stream on ``num/den`` of the CUs of every XCD
    (``hipExtStreamCreateWithCUMask``, csrc/kernels/ew.hip ``mxr_stream_create_cumask``), so the weight gradients
    cannot take CUs from the critical-path data gradients beyond that share (A/B: profiles/r6_side_cu_mask_ab.txt)."""
    import ctypes
    from . import native
    num, den = (int(v) for v in frac.split("/"))
    L = native.lib()
    L.mxr_stream_create_cumask.restype = ctypes.c_void_p
    with torch.cuda.device(idx):
        h = L.mxr_stream_create_cumask(num, den, 0)
    if not h:
        raise RuntimeError("MXR_SIDE_CU_FRAC=%s: hipExtStreamCreateWithCUMask failed" % frac)
    return torch.cuda.ExternalStream(h, device=torch.device("cuda", idx))


class _Dev:
    """Per-device state: the side stream, the compute-stream objects seen (by raw handle: the
    torch.cuda.current_stream() wrapper costs several us of device-index resolution per call, and the
    backward enters a side region per weight gradient), and two reusable fork / join events (a stream
    wait binds to the event's record at the time of the wait, so re-recording later is safe)."""

    def __init__(self, idx: int):
        self.idx = idx
        # normal priority (a high-priority compute stream measured 449 vs 460 img/s,
        # profiles/r2_stream_priority_ab.txt)
        frac = os.environ.get("MXR_SIDE_CU_FRAC", "")
        if frac:
            self.side = _cu_masked_stream(idx, frac)
        else:
            self.side = torch.cuda.Stream(torch.device("cuda", idx), priority=0)
        self.side_raw = self.side.cuda_stream
        self.streams: Dict[int, torch.cuda.Stream] = {}
        self.fork = torch.cuda.Event()
        self.back = torch.cuda.Event()

    def current(self) -> torch.cuda.Stream:
        raw = _RAW(self.idx) if _RAW is not None else torch.cuda.current_stream(self.idx).cuda_stream
        s = self.streams.get(raw)
        if s is None:
            s = torch.cuda.current_stream(self.idx)
            self.streams[raw] = s
        return s


class _Region:
    """Context object of :meth:`SideStream.run` (a plain class: the generator-based contextmanager
    costs more per entry than the region's own bookkeeping)."""
    __slots__ = ("owner", "d", "tensors", "prev")

    def __init__(self, owner, d, tensors):
        self.owner, self.d, self.tensors, self.prev = owner, d, tensors, None

    def __enter__(self):
        d = self.d
        main = d.current()
        if main.cuda_stream == d.side_raw:          # nested: already on the side stream
            return self
        d.fork.record(main)
        d.side.wait_event(d.fork)
        for t in self.tensors:
            if t is not None and t.is_cuda:
                t.record_stream(d.side)
        o = self.owner
        o._main = main
        o.launches += 1
        self.prev = main
        _set_stream(d.side)
        if o.delay_cycles:
            torch.cuda._sleep(o.delay_cycles)
        return self

    def __exit__(self, *exc):
        if self.prev is not None:
            _set_stream(self.prev)
        return False


class _Cover:
    __slots__ = ("owner", "prev")

    def __init__(self, owner):
        self.owner, self.prev = owner, None

    def __enter__(self):
        o = self.owner
        if o._main is None:
            return self
        d = o._dev(o._main.device_index)
        cur = d.current()
        if cur.cuda_stream != d.side_raw:
            d.fork.record(cur)
            d.side.wait_event(d.fork)
        if o._main.cuda_stream != cur.cuda_stream:
            d.back.record(o._main)
            d.side.wait_event(d.back)
        self.prev = cur
        _set_stream(d.side)
        return self

    def __exit__(self, *exc):
        if self.prev is not None:
            _set_stream(self.prev)
        return False


class _Null:
    def __enter__(self):
        return self

    def __exit__(self, *exc):
        return False


_NULL = _Null()


class SideStream:
    def __init__(self):
        self.enabled = os.environ.get("MXR_SIDE_WGRAD", "1") == "1"
        # inside a HIP-graph capture too: the fork / join events become graph edges, so a replay runs the weight
        # gradients as a parallel branch of the data-gradient chain, as the eager step does (MXR_SIDE_IN_GRAPH=0:
        # serial on the capture stream)
        self.in_graph = os.environ.get("MXR_SIDE_IN_GRAPH", "1") == "1"
        self._devs: Dict[int, _Dev] = {}
        self._main: Optional[torch.cuda.Stream] = None   # compute stream of the pending side work
        self._kept = []                                   # see keep()
        self.launches = 0                                 # side-stream regions entered (tests / stats)
        # ordering stress (tests): a spin kernel of this many cycles heads every side-stream region, so a
        # missing wait shows up as a wrong gradient instead of hiding behind the timing
        self.delay_cycles = int(os.environ.get("MXR_SIDE_DELAY", "0"))

    def _dev(self, idx: Optional[int]) -> _Dev:
        if idx is None:
            idx = _DEV() if _DEV is not None else torch.cuda.current_device()
        d = self._devs.get(idx)
        if d is None:
            d = self._devs[idx] = _Dev(idx)
        return d

    @property
    def _streams(self) -> Dict[int, torch.cuda.Stream]:
        return {i: d.side for i, d in self._devs.items()}

    def usable(self, t: torch.Tensor) -> bool:
        return self.enabled and t.is_cuda and (self.in_graph or not _capturing())

    @property
    def pending(self) -> bool:
        return self._main is not None

    def run(self, device: torch.device, *tensors):
        """Launches inside the block go to the side stream, ordered after everything the current
        (compute) stream has queued; ``tensors`` are compute-stream allocations the block reads."""
        return _Region(self, self._dev(device.index), tensors)

    def keep(self, t: torch.Tensor) -> None:
        """Hold a reference to ``t`` until the next :meth:`join` while side work is pending: autograd
        accumulates gradients in place only into tensors nobody else references."""
        if self._main is not None:
            self._kept.append(t)

    def join(self) -> None:
        """The current stream waits for all side-stream work queued so far (no host sync)."""
        if self._main is None:
            return
        d = self._dev(self._main.device_index)
        cur = d.current()
        if cur.cuda_stream != d.side_raw:
            d.back.record(d.side)
            cur.wait_event(d.back)
        if cur.cuda_stream == self._main.cuda_stream:
            self._main = None
            self._kept.clear()

    def covering(self):
        """Work launched inside the block (a bucket-ready event) is ordered after both the compute
        stream and the side stream: it goes to the side stream after that waited for the compute
        stream -- the compute stream itself is not held up."""
        if self._main is None:
            return _NULL
        return _Cover(self)


SIDE = SideStream()
