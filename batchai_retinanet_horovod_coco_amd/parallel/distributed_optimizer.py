"""``hvd.DistributedOptimizer``: bucketed, overlapped gradient all-reduce over RCCL.

Reference: ``hvd.DistributedOptimizer(keras.optimizers.adam(lr=1e-5, clipnorm=0.001))``
(``/root/reference/train.py:103-104``).  Horovod wraps ``get_gradients`` -- Keras applies
``clipnorm`` per rank with the LOCAL global norm, then every gradient is all-reduced
(average) through a <=64 MiB fusion buffer after a rank-0 negotiation.

MI355X design:

* gradients already live in one flat fp32 buffer in backward order (``train.flat``), so a
  "fusion buffer" is a slice -- no pack/unpack copies;
* the buffer is cut into buckets of ``HOROVOD_FUSION_THRESHOLD`` bytes (default 25 MiB ->
  6 buckets for R50, each large enough to spread over RCCL's channels on the 7 xGMI links);
* ``clip_mode='global'`` (default for benchmarks): a bucket's in-place SUM all-reduce is
  launched as soon as its last gradient is accumulated (post-accumulate hooks, strictly in
  bucket order on every rank, so no negotiation is needed), overlapping the rest of the
  backward pass; after the wait the clip factor is computed from the *averaged* gradient and
  ``clip / world`` is folded into the fused Adam kernel;
* ``clip_mode='local'`` reproduces the reference exactly: local norm -> clip -> all-reduce
  average -> Adam.  The local norm is a barrier over the whole backward, so this mode cannot
  overlap (as in the reference).
* the native C++ comm core (``parallel.native_comm``) is the default gradient path for GPU runs with
  world > 1 (``MXR_COMM=auto``): readiness is an event on the compute stream, the in-order RCCL
  all-reduces run on its own high-priority stream, and the optimizer's stream waits on per-bucket
  events -- no Python work or host sync on the gradient path.  ``--allreduce-dtype bf16`` keeps a
  persistent bf16 mirror of the flat gradient: each bucket is cast on the compute stream right
  before it is handed over, and the reduced mirror is widened back once after the wait.
  ``MXR_COMM=torch`` selects the ProcessGroupNCCL path instead; ``MXR_COMM=native`` forces the
  native engine even at world 1 (a one-rank RCCL communicator -- tests and single-GPU profiling).
"""
from __future__ import annotations

import os
import warnings
from typing import Dict, List, Optional, Tuple

import torch

from . import collectives, runtime
from . import timeline as _timeline
from ..ops.side_stream import SIDE

DEFAULT_BUCKET_BYTES = 25 * 1024 * 1024


def _fusion_threshold() -> int:
    v = os.environ.get("HOROVOD_FUSION_THRESHOLD")
    return int(v) if v else DEFAULT_BUCKET_BYTES


class DistributedOptimizer:
    def __init__(self, optimizer, compression=collectives.Compression.none, clip_mode: str = "local",
                 bucket_bytes: Optional[int] = None, overlap: bool = True, backward_passes_per_step: int = 1):
        if clip_mode not in ("local", "global"):
            raise ValueError("clip_mode must be 'local' or 'global'")
        self.optimizer = optimizer
        self.flat = optimizer.flat
        self.compression = compression
        self.clip_mode = clip_mode
        self.overlap = overlap and clip_mode == "global"
        self.bucket_bytes = bucket_bytes or _fusion_threshold()
        self.buckets: List[Tuple[int, int]] = []
        self.bucket_of: Dict[int, int] = {}
        self._build_buckets()
        self._pending: List[int] = []
        self._handles: List[Optional[collectives.Handle]] = []
        self._next_launch = 0
        self._ready: List[bool] = []
        self._hooks = []
        self.native = None
        self._comm_buf: Optional[torch.Tensor] = None     # bf16 mirror of flat.grad (compressed native path)
        self._notified: set = set()
        self._fallback: Optional[str] = None      # why the agreed bring-up fell back to torch (all ranks)
        want = self._want_native()
        if want:
            self._init_native(compression, forced=(want == "native"))
        self.reset()
        for seg in self.flat.segments:
            self._hooks.append(seg.param.register_post_accumulate_grad_hook(self._on_grad))
        self.last_grad_norm: Optional[torch.Tensor] = None

    def _init_native(self, compression, forced: bool, make=None, new_uid=None) -> None:
        """Bring the native engine up on every rank or on none (``native_comm.bring_up``: load, init and a
        bucket-engine self-test, each closed by an all-rank agreement).  On an agreed failure every rank
        stays on torch.distributed (``MXR_COMM=auto``) or every rank raises (``MXR_COMM=native``)."""
        from .native_comm import bring_up, CommBringUpError
        dev = self.flat.grad.device.index or 0
        world = runtime.size() if runtime.is_initialized() else 1
        rank = runtime.rank() if runtime.is_initialized() else 0
        if compression is collectives.Compression.none:
            src = self.flat.grad
        else:
            self._comm_buf = torch.zeros(self.flat.total, dtype=compression.dtype, device=self.flat.grad.device)
            src = self._comm_buf

        def setup(comm):
            comm.set_buckets([src[a:e] for a, e in self.buckets], average=False)
            # collective watchdog: a bucket not reduced within MXR_COMM_TIMEOUT seconds
            # aborts the communicator and the next step raises, naming the bucket
            comm.watchdog(float(os.environ.get("MXR_COMM_TIMEOUT", "600")))

        comm, why = bring_up(rank, world, dev, setup=setup, make=make, new_uid=new_uid)
        if comm is None:
            self._comm_buf = None
            self._fallback = why
            if forced:
                raise CommBringUpError("MXR_COMM=native: native RCCL bucket engine unavailable: " + why)
            # MXR_COMM=auto: ProcessGroupNCCL (RCCL through torch.distributed) carries the same buckets --
            # on EVERY rank, since the decision was agreed
            warnings.warn("native RCCL bucket engine unavailable (%s); all ranks use torch.distributed" % why)
            return
        self.native = comm
        from . import ops as _ops
        _ops.set_native_comm(self.native)      # torch.ops.mxr.* collectives use it for GPU tensors

    def _want_native(self):
        """False, "native" (forced: failures raise) or "auto" (world > 1 on GPU: failures fall back).
        Decided from settings every rank shares (env, world size, device type) -- nothing rank-local like a
        file check, which now happens inside the agreed bring-up."""
        mode = os.environ.get("MXR_COMM", "auto")
        if mode not in ("auto", "native", "torch"):
            raise ValueError("MXR_COMM must be auto|native|torch, got %r" % mode)
        if mode == "torch" or not self.flat.grad.is_cuda:
            return False
        if mode == "native":
            return "native"
        return "auto" if runtime.distributed() else False

    @property
    def reducing(self) -> bool:
        """True when gradients go through a collective (world > 1, or the native engine is forced)."""
        return runtime.distributed() or self.native is not None

    # ------------------------------------------------------------------ buckets
    def _build_buckets(self) -> None:
        cap = max(1, self.bucket_bytes // 4)
        start = None
        cur = 0
        self._seg_count: List[int] = []
        count = 0
        for s in self.flat.segments:
            if start is None:
                start = s.offset
            end = s.offset + s.numel
            self.bucket_of[id(s.param)] = len(self.buckets)
            count += 1
            cur = end - start
            if cur >= cap:
                self.buckets.append((start, self._aligned_end(s)))
                self._seg_count.append(count)
                start, count = None, 0
        if start is not None:
            self.buckets.append((start, self.flat.total))
            self._seg_count.append(count)
        if self.buckets:
            # the last aligned end of each bucket = start of the next bucket
            fixed = []
            for i, (a, b) in enumerate(self.buckets):
                nb = self.buckets[i + 1][0] if i + 1 < len(self.buckets) else self.flat.total
                fixed.append((a, nb))
            self.buckets = fixed

    def _aligned_end(self, s) -> int:
        from ..train.flat import ALIGN
        return s.offset + (s.numel + ALIGN - 1) // ALIGN * ALIGN

    def bucket_sizes_bytes(self) -> List[int]:
        return [(b - a) * 4 for a, b in self.buckets]

    def reset(self) -> None:
        SIDE.join()
        for h in getattr(self, "_handles", ()):   # torch path: an abandoned step's in-flight all-reduces
            if h is not None and h.work is not None:   # write into flat.grad -- let them finish first
                h.work.wait()
        self._pending = list(self._seg_count)
        self._ready = [False] * len(self.buckets)
        self._handles = [None] * len(self.buckets)
        self._next_launch = 0
        self._notified = set()
        if self.native is not None and not self.native.aborted():
            self.native.reset()      # an abandoned step's launched buckets finish before grads are reused

    # ------------------------------------------------------------------ hooks
    def _on_grad(self, param) -> None:
        self.notify_grad_ready(param)

    def notify_grad_ready(self, param) -> None:
        """A parameter's gradient is complete for this step (post-accumulate hook, or a HIP gradient
        sink that accumulated straight into the flat buffer).  Idempotent per step: a parameter
        reported by both mechanisms counts once, so a bucket can neither launch early nor stall."""
        b = self.bucket_of.get(id(param))
        if b is None or id(param) in self._notified:
            return
        self._notified.add(id(param))
        self._pending[b] -= 1
        if self._pending[b] == 0:
            self._ready[b] = True
            tl = _timeline.get()
            if tl.enabled:
                tl.instant("bucket{}".format(b), "READY")
            if self.overlap and self.reducing:
                self._launch_ready_in_order()

    def _launch(self, b: int) -> None:
        # weight gradients may still be running on the side stream (ops.side_stream): the bucket's
        # readiness is ordered after both streams without holding up the compute stream
        with SIDE.covering():
            self._launch_one(b)

    def _launch_one(self, b: int) -> None:
        if self.native is not None:
            if self._comm_buf is not None:
                a, e = self.buckets[b]
                self._comm_buf[a:e].copy_(self.flat.grad[a:e])     # compress on the compute stream
            self.native.bucket_ready(b)
            return
        a, e = self.buckets[b]
        self._handles[b] = collectives.allreduce_async_(self.flat.grad[a:e], average=False,
                                                        name="bucket{}".format(b), compression=self.compression)

    def _launch_ready_in_order(self) -> None:
        while self._next_launch < len(self.buckets) and self._ready[self._next_launch]:
            self._launch(self._next_launch)
            self._next_launch += 1

    def _reduce_all(self) -> None:
        """Launch whatever is left (in order) and wait for every bucket."""
        while self._next_launch < len(self.buckets):
            self._launch(self._next_launch)
            self._next_launch += 1
        if self.native is not None:
            self.native.wait()
            if self._comm_buf is not None:
                self.flat.grad.copy_(self._comm_buf)               # widen the reduced bf16 mirror
            return
        for h in self._handles:
            if h is not None:
                collectives.synchronize(h)

    def comm_stats(self) -> Optional[dict]:
        """Per-step GPU comm timings of the native engine (None on the torch path)."""
        return self.native.step_stats() if self.native is not None else None

    # ------------------------------------------------------------------ public API
    def zero_grad(self) -> None:
        # reset FIRST: it joins the side stream (weight gradients still accumulating into flat.grad) and
        # makes the compute stream wait for an abandoned step's bucket all-reduces; only then is zeroing
        # the buffer ordered after every in-flight writer
        self.reset()
        self.flat.zero_grad()

    def step(self) -> torch.Tensor:
        """Reduce, clip and apply.  Returns the gradient norm the clip was computed from."""
        SIDE.join()                 # side-stream weight gradients land before anything reads flat.grad
        opt = self.optimizer
        world = runtime.size() if runtime.is_initialized() else 1
        if not self.reducing:
            norm, scale = opt.norm_and_scale()
        elif self.clip_mode == "local":
            norm = opt.grad_norm()
            self.flat.grad.mul_(opt.clip_factor(norm))
            self._reduce_all()
            scale = torch.full((), 1.0 / world, device=self.flat.grad.device)
        else:
            self._reduce_all()
            norm, scale = opt.norm_and_scale(1.0 / world, 1.0 / world)
        opt.apply(scale)
        self.last_grad_norm = norm
        self._pending = list(self._seg_count)       # next step: fresh counters (the engine was waited)
        self._ready = [False] * len(self.buckets)
        self._handles = [None] * len(self.buckets)
        self._next_launch = 0
        self._notified = set()
        return norm

    # keras-ish passthroughs
    @property
    def lr(self):
        return self.optimizer.lr

    @lr.setter
    def lr(self, v):
        self.optimizer.lr = v

    @property
    def iterations(self):
        return self.optimizer.iterations

    @iterations.setter
    def iterations(self, v):
        self.optimizer.iterations = v

    def state_tensors(self):
        return self.optimizer.state_tensors()

    def get_config(self):
        return self.optimizer.get_config()

    def remove_hooks(self) -> None:
        for h in self._hooks:
            h.remove()
        self._hooks = []
