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
* never during HIP-graph capture (the step is then one graph launch anyway).

``MXR_SIDE_WGRAD=0`` turns it off.
"""
from __future__ import annotations

import contextlib
import os
from typing import Dict, Optional

import torch


class SideStream:
    def __init__(self):
        self.enabled = os.environ.get("MXR_SIDE_WGRAD", "1") == "1"
        self._streams: Dict[int, torch.cuda.Stream] = {}
        self._main: Optional[torch.cuda.Stream] = None   # compute stream of the pending side work
        self._kept = []                                   # see keep()
        self.launches = 0                                 # side-stream regions entered (tests / stats)
        # ordering stress (tests): a spin kernel of this many cycles heads every side-stream region, so a
        # missing wait shows up as a wrong gradient instead of hiding behind the timing
        self.delay_cycles = int(os.environ.get("MXR_SIDE_DELAY", "0"))
        self.towers = os.environ.get("MXR_TOWER_STREAM", "0") == "1"
        self._towers: Dict[int, torch.cuda.Stream] = {}

    def _side(self, device: torch.device) -> torch.cuda.Stream:
        idx = device.index if device.index is not None else torch.cuda.current_device()
        s = self._streams.get(idx)
        if s is None:
            s = torch.cuda.Stream(torch.device("cuda", idx))
            self._streams[idx] = s
        return s

    def tower_stream(self, t: torch.Tensor) -> Optional[torch.cuda.Stream]:
        """Second compute stream for the regression head tower (``RetinaNet.forward``): the two head
        towers are independent until the loss, so each fills the other's tail rounds (forward and,
        since autograd runs a node's backward on its forward stream, backward).  Off by default
        (``MXR_TOWER_STREAM=1`` turns it on): with the weight gradients already on the side stream it
        measured within run-to-run noise (433.1 / 431.4 / 430.3 img/s on, off, on).  None when off, on CPU
        or under graph capture."""
        if not (self.towers and t.is_cuda and not torch.cuda.is_current_stream_capturing()):
            return None
        idx = t.device.index if t.device.index is not None else torch.cuda.current_device()
        s = self._towers.get(idx)
        if s is None:
            s = torch.cuda.Stream(torch.device("cuda", idx))
            self._towers[idx] = s
        return s

    def usable(self, t: torch.Tensor) -> bool:
        return (self.enabled and t.is_cuda and not torch.cuda.is_current_stream_capturing())

    @property
    def pending(self) -> bool:
        return self._main is not None

    @contextlib.contextmanager
    def run(self, device: torch.device, *tensors):
        """Launches inside the block go to the side stream, ordered after everything the current
        (compute) stream has queued; ``tensors`` are compute-stream allocations the block reads."""
        main = torch.cuda.current_stream(device)
        side = self._side(device)
        if main.cuda_stream == side.cuda_stream:       # nested: already on the side stream
            yield
            return
        side.wait_stream(main)
        for t in tensors:
            if t is not None and t.is_cuda:
                t.record_stream(side)
        self._main = main
        self.launches += 1
        with torch.cuda.stream(side):
            if self.delay_cycles:
                torch.cuda._sleep(self.delay_cycles)
            yield

    def keep(self, t: torch.Tensor) -> None:
        """Hold a reference to ``t`` until the next :meth:`join` while side work is pending: autograd
        accumulates gradients in place only into tensors nobody else references."""
        if self._main is not None:
            self._kept.append(t)

    def join(self) -> None:
        """The current stream waits for all side-stream work queued so far (no host sync)."""
        if self._main is None:
            return
        cur = torch.cuda.current_stream(self._main.device)
        for s in self._streams.values():
            if s.device == cur.device and s.cuda_stream != cur.cuda_stream:
                cur.wait_stream(s)
        if cur.cuda_stream == self._main.cuda_stream:
            self._main = None
            self._kept.clear()

    @contextlib.contextmanager
    def covering(self):
        """Work launched inside the block (a bucket-ready event) is ordered after both the compute
        stream and the side stream: it goes to the side stream after that waited for the compute
        stream -- the compute stream itself is not held up."""
        if self._main is None:
            yield
            return
        side = self._side(self._main.device)
        cur = torch.cuda.current_stream(self._main.device)
        if cur.cuda_stream != side.cuda_stream:
            side.wait_stream(cur)
        if self._main.cuda_stream != cur.cuda_stream:
            side.wait_stream(self._main)
        with torch.cuda.stream(side):
            yield


SIDE = SideStream()
