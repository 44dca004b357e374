"""ctypes front-end of the native communication core (``csrc/comm/comm.hip`` -> ``_lib/libmxr_comm.so``).

Horovod's C++ core equivalent (``/root/reference/train.py:20-21,103-104``): an
RCCL communicator bootstrapped from a unique id that rank 0 creates and the process group
broadcasts, plain collectives ordered against the caller's HIP stream by events, and the gradient
bucket engine used by :class:`parallel.distributed_optimizer.DistributedOptimizer` with
``MXR_COMM=native``: buckets are registered once (slices of the flat gradient buffer), become ready
on the compute stream, and are all-reduced IN BUCKET ORDER on a dedicated high-priority stream.
A watchdog thread (``watchdog``, started by the DistributedOptimizer with ``MXR_COMM_TIMEOUT``
seconds) aborts the communicator when a launched bucket is not reduced in time or RCCL
reports an async error; the next ``bucket_ready``/``wait``/``check`` then raises with the bucket named.
The RCCL library is the one PyTorch already loaded (``torch/lib/librccl.so``), opened by path so the
process holds a single RCCL instance.
"""
from __future__ import annotations

import ctypes
import os
from typing import List, Optional

import torch

_LIB = None
_DT = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2, torch.int32: 3, torch.int64: 4, torch.uint8: 5,
       torch.float64: 6}
c_int, c_ll, c_vp, c_char_p = ctypes.c_int, ctypes.c_longlong, ctypes.c_void_p, ctypes.c_char_p

_SIGS = {
    "mxr_comm_load": ([c_char_p], c_int),
    "mxr_comm_unique_id": ([c_vp], c_int),
    "mxr_comm_init": ([c_vp, c_int, c_int, c_int], c_vp),
    "mxr_comm_destroy": ([c_vp], c_int),
    "mxr_comm_allreduce": ([c_vp, c_vp, c_vp, c_ll, c_int, c_int, c_vp], c_int),
    "mxr_comm_broadcast": ([c_vp, c_vp, c_ll, c_int, c_int, c_vp], c_int),
    "mxr_comm_allgather": ([c_vp, c_vp, c_vp, c_ll, c_int, c_vp], c_int),
    "mxr_comm_reduce_scatter": ([c_vp, c_vp, c_vp, c_ll, c_int, c_int, c_vp], c_int),
    "mxr_comm_set_buckets": ([c_vp, c_int, ctypes.POINTER(c_vp), ctypes.POINTER(c_ll), c_int, c_int], c_int),
    "mxr_comm_bucket_ready": ([c_vp, c_int, c_vp], c_int),
    "mxr_comm_wait": ([c_vp, c_vp], c_int),
    "mxr_comm_next_launch": ([c_vp], c_int),
    "mxr_comm_set_stream": ([c_vp, c_vp], c_int),
    "mxr_comm_info": ([c_vp, c_vp], c_int),
    "mxr_comm_reset": ([c_vp, c_vp], c_int),
    "mxr_comm_debug": ([c_vp, c_int, ctypes.c_float], c_int),
    "mxr_comm_step_stats": ([c_vp, ctypes.POINTER(ctypes.c_float), c_int], c_int),
    "mxr_comm_watchdog": ([c_vp, c_int, c_int, c_int], c_int),
    "mxr_comm_status": ([c_vp], c_int),
    "mxr_comm_timeline": ([c_vp, c_char_p], c_int),
    "mxr_comm_timeline_flush": ([c_vp], c_int),
    "mxr_comm_last_error": ([], c_char_p),
}


def lib_path() -> str:
    return os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "_lib", "libmxr_comm.so")


def rccl_path() -> str:
    """The librccl PyTorch ships (and loads for its nccl backend)."""
    p = os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")
    return p if os.path.exists(p) else "librccl.so.1"


def lib():
    global _LIB
    if _LIB is None:
        if not os.path.exists(lib_path()):
            raise RuntimeError("native comm library not built: {} (python -m batchai_retinanet_horovod_coco_amd.build)"
                               .format(lib_path()))
        L = ctypes.CDLL(lib_path())
        for name, (args, res) in _SIGS.items():
            fn = getattr(L, name)
            fn.argtypes = args
            fn.restype = res
        rc = L.mxr_comm_load(rccl_path().encode())
        if rc != 0:
            raise RuntimeError("loading RCCL failed: {}".format(L.mxr_comm_last_error().decode()))
        _LIB = L
    return _LIB


def _chk(rc: int, what: str) -> None:
    if rc != 0:
        raise RuntimeError("{} failed ({}): {}".format(what, rc, lib().mxr_comm_last_error().decode()))


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def unique_id() -> bytes:
    buf = ctypes.create_string_buffer(128)
    _chk(lib().mxr_comm_unique_id(buf), "ncclGetUniqueId")
    return buf.raw


class NativeComm:
    """One RCCL communicator + bucket engine.  ``uid`` must be the same 128 bytes on every rank."""

    def __init__(self, rank: int, world: int, device: int, uid: Optional[bytes] = None):
        if uid is None:
            if world != 1:
                raise ValueError("multi-rank NativeComm needs the rank-0 unique id (use NativeComm.create)")
            uid = unique_id()
        self.rank, self.world, self.device = rank, world, device
        buf = ctypes.create_string_buffer(uid, 128)
        self.h = lib().mxr_comm_init(buf, world, rank, device)
        if not self.h:
            raise RuntimeError("ncclCommInitRank failed: {}".format(lib().mxr_comm_last_error().decode()))
        self._buckets: List[torch.Tensor] = []
        # The collectives run on a stream taken from PyTorch's pool (high priority).  A stream the core
        # created itself after the RCCL init measured 13 ms/step slower at world 1 (every compute kernel
        # slowed while buckets crossed streams; profiles/r2_native_stream_ab.txt); a pool stream shows
        # none of it.
        self._stream = torch.cuda.Stream(torch.device("cuda", device), priority=-1)
        _chk(lib().mxr_comm_set_stream(self.h, self._stream.cuda_stream), "set_stream")

    @classmethod
    def create(cls, rank: int, world: int, device: int) -> "NativeComm":
        """Rank 0 makes the unique id; the default process group broadcasts it.  (No agreement: a
        failure on one rank hangs the others -- the training path uses :func:`bring_up`.)"""
        import torch.distributed as dist
        uid = unique_id() if rank == 0 else None
        if world > 1:
            box = [uid]
            dist.broadcast_object_list(box, src=0)
            uid = box[0]
        return cls(rank, world, device, uid)

    def self_test(self, timeout_s: float = 60.0) -> None:
        """Reduce a rank-valued probe THROUGH THE BUCKET ENGINE (set_buckets / bucket_ready / wait on
        the current stream) and check it equals sum(rank + 1) on this rank.  Bounded: the watchdog
        aborts the communicator if a peer never joins, and the host poll gives up after ``timeout_s``.
        Replaces the bucket list (the caller registers the real buckets afterwards)."""
        import time
        dev = torch.device("cuda", self.device)
        probe = torch.full((4096,), float(self.rank + 1), dtype=torch.float32, device=dev)
        self.set_buckets([probe])
        self.watchdog(timeout_s)
        self.bucket_ready(0)
        self.wait()
        ev = torch.cuda.Event()
        ev.record()
        t0 = time.time()
        while not ev.query():
            if self.aborted() or time.time() - t0 > timeout_s + 5:
                self.check()
                raise RuntimeError("comm self-test: the probe all-reduce did not complete in %.0f s" % timeout_s)
            time.sleep(0.001)
        self.check()
        self.watchdog(0)
        expect = self.world * (self.world + 1) / 2.0
        got = probe.cpu()
        if not bool((got == expect).all()):
            raise RuntimeError("comm self-test: probe reduced to {} (min) / {} (max), expected {}".format(
                float(got.min()), float(got.max()), expect))
        self._buckets = []

    def info(self) -> dict:
        """What RCCL reports for this communicator: ``nranks`` (ncclCommCount), ``device``
        (ncclCommCuDevice), ``rank`` (ncclCommUserRank); -1 where the library lacks the symbol."""
        out = (ctypes.c_int * 3)()
        lib().mxr_comm_info(self.h, out)
        return {"nranks": int(out[0]), "device": int(out[1]), "rank": int(out[2])}

    # ---------------------------------------------------------------- collectives
    def allreduce_(self, t: torch.Tensor, average: bool = False) -> torch.Tensor:
        _chk(lib().mxr_comm_allreduce(self.h, t.data_ptr(), t.data_ptr(), t.numel(), _DT[t.dtype], int(average),
                                      _stream()), "allreduce")
        return t

    def broadcast_(self, t: torch.Tensor, root: int = 0) -> torch.Tensor:
        _chk(lib().mxr_comm_broadcast(self.h, t.data_ptr(), t.numel(), _DT[t.dtype], root, _stream()), "broadcast")
        return t

    def allgather(self, t: torch.Tensor) -> torch.Tensor:
        out = torch.empty((self.world * t.numel(),), dtype=t.dtype, device=t.device)
        _chk(lib().mxr_comm_allgather(self.h, t.data_ptr(), out.data_ptr(), t.numel(), _DT[t.dtype], _stream()),
             "allgather")
        return out.view((self.world,) + tuple(t.shape))

    def reduce_scatter(self, t: torch.Tensor, average: bool = False) -> torch.Tensor:
        n = t.numel() // self.world
        out = torch.empty((n,), dtype=t.dtype, device=t.device)
        _chk(lib().mxr_comm_reduce_scatter(self.h, t.data_ptr(), out.data_ptr(), n, _DT[t.dtype], int(average),
                                           _stream()), "reduce_scatter")
        return out

    # ---------------------------------------------------------------- bucket engine
    def set_buckets(self, tensors: List[torch.Tensor], average: bool = False) -> None:
        dts = {t.dtype for t in tensors}
        if len(dts) != 1:
            raise ValueError("buckets must share one dtype")
        self._buckets = list(tensors)       # keep the views alive
        n = len(tensors)
        ptrs = (c_vp * n)(*[t.data_ptr() for t in tensors])
        counts = (c_ll * n)(*[t.numel() for t in tensors])
        _chk(lib().mxr_comm_set_buckets(self.h, n, ptrs, counts, _DT[tensors[0].dtype], int(average)), "set_buckets")

    def bucket_ready(self, b: int) -> None:
        _chk(lib().mxr_comm_bucket_ready(self.h, b, _stream()), "bucket_ready")

    def wait(self) -> None:
        _chk(lib().mxr_comm_wait(self.h, _stream()), "wait")

    def reset(self) -> None:
        """Abandon the current step: the current stream waits for the buckets already launched (no
        host sync), and the readiness flags clear, so the next step starts clean even after an
        exception mid-backward."""
        _chk(lib().mxr_comm_reset(self.h, _stream()), "reset")

    def step_stats(self) -> Optional[dict]:
        """GPU timings of the last completed step (blocks until its last bucket is done):
        ``comm_ms`` = summed all-reduce time, ``exposed_ms`` = time from the last bucket becoming
        ready (end of the backward) to the end of its all-reduce, ``bucket_ms`` per bucket."""
        n = max(1, len(self._buckets)) + 2
        out = (ctypes.c_float * n)()
        nb = lib().mxr_comm_step_stats(self.h, out, n)
        if nb <= 0:
            return None
        return {"comm_ms": float(out[0]), "exposed_ms": float(out[1]),
                "bucket_ms": [float(out[2 + b]) for b in range(nb)]}

    # ---------------------------------------------------------------- failure detection
    def watchdog(self, timeout_s: Optional[float], poll_ms: int = 100, inject_bucket: int = -1) -> None:
        """Start (``timeout_s`` > 0) or stop the watchdog.  ``inject_bucket`` is the fault-injection
        hook: that bucket never reports completion, so the timeout path runs without a dead peer."""
        ms = int(1000 * timeout_s) if timeout_s else 0
        _chk(lib().mxr_comm_watchdog(self.h, ms, int(poll_ms), int(inject_bucket)), "watchdog")

    def perturb(self, delay_us: int = 0, post_scale: float = 1.0) -> None:
        """Stream-ordering perturbation (tests): spin ``delay_us`` on the comm stream before, and
        multiply the bucket by ``post_scale`` after, every bucket all-reduce."""
        _chk(lib().mxr_comm_debug(self.h, int(delay_us), float(post_scale)), "debug")

    def aborted(self) -> bool:
        return bool(self.h) and lib().mxr_comm_status(self.h) == 1

    def check(self) -> None:
        """Raise if the watchdog aborted the communicator."""
        if self.aborted():
            raise RuntimeError("collective watchdog: " + lib().mxr_comm_last_error().decode())

    def launched(self) -> int:
        return lib().mxr_comm_next_launch(self.h)

    # ---------------------------------------------------------------- timeline
    def timeline(self, path: Optional[str]) -> None:
        _chk(lib().mxr_comm_timeline(self.h, (path or "").encode()), "timeline")

    def flush_timeline(self) -> None:
        _chk(lib().mxr_comm_timeline_flush(self.h), "timeline_flush")

    def close(self) -> None:
        if self.h:
            _chk(lib().mxr_comm_destroy(self.h), "destroy")
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass


# ---------------------------------------------------------------------------- agreed bring-up
def _fault(rank: int, stage: str) -> None:
    """``MXR_COMM_FAULT=rank:stage`` (stage: load | init | selftest | setup): raise at that stage on that
    rank -- the test hook for the agreed fallback."""
    spec = os.environ.get("MXR_COMM_FAULT")
    if not spec:
        return
    r, s = spec.split(":", 1)
    if int(r) == rank and s == stage:
        raise RuntimeError("injected comm fault at %s (MXR_COMM_FAULT)" % stage)


def _with_timeout(fn, timeout_s: float, on_late=None):
    """Run ``fn`` on a helper thread (ctypes releases the GIL) and give up after ``timeout_s``: a rank whose
    peers never join ncclCommInitRank must come back to the agreement instead of blocking forever.  The
    abandoned daemon thread may still finish later (a slow peer joined after all): ``on_late(result)``
    then disposes of what it made, so no communicator leaks."""
    import threading
    box = {}
    lock = threading.Lock()

    def run():
        try:
            v = fn()
        except BaseException as e:  # noqa: BLE001
            with lock:
                box["e"] = e
            return
        with lock:
            late = box.get("abandoned", False)
            box["v"] = v
        if late and on_late is not None:
            try:
                on_late(v)
            except Exception:  # noqa: BLE001
                pass
    t = threading.Thread(target=run, daemon=True, name="mxr-comm-init")
    t.start()
    t.join(timeout_s)
    with lock:
        if "v" not in box and "e" not in box:
            box["abandoned"] = True
            raise TimeoutError("no answer within %.0f s (a peer did not join)" % timeout_s)
    if "e" in box:
        raise box["e"]
    return box["v"]


def stage_timeouts(init_timeout: Optional[float] = None, pg_timeout: Optional[float] = None):
    """(init, self-test) bounds of :func:`bring_up`, clamped under the default process group's timeout.

    A rank that fails a stage at once enters the stage's agreement (a collective over the default group)
    while its peers may still sit in that stage for its whole bound: the bound must stay well under the
    group's timeout or the group's watchdog tears the job down before the agreed fallback."""
    if init_timeout is None:
        init_timeout = float(os.environ.get("MXR_COMM_INIT_TIMEOUT", "180"))
    if pg_timeout is None:
        from . import runtime
        pg_timeout = runtime.pg_timeout()
    cap = 0.4 * float(pg_timeout)
    return min(float(init_timeout), cap), min(60.0, cap)


class CommBringUpError(RuntimeError):
    pass


def bring_up(rank: int, world: int, device: int, setup=None, make=None, new_uid=None, self_test: bool = True,
             init_timeout: Optional[float] = None):
    """Create the native engine on EVERY rank or on none (VERDICT r3 Next #4).

    Three stages, each closed by a collective agreement over the default process group
    (``runtime.rank_flags``), so no rank can be left waiting on a peer that gave up, and no two ranks
    can end up on different gradient engines:

    1. load ``libmxr_comm`` + RCCL on every rank, rank 0 makes the unique id -> agree;
    2. broadcast the id, ``ncclCommInitRank`` (bounded by ``MXR_COMM_INIT_TIMEOUT``, default 180 s, and by
       0.4 x the default group's timeout: :func:`stage_timeouts`) -> agree;
    3. the bucket-engine self-test (a rank-valued probe must reduce to sum(rank + 1)), then ``setup(comm)``
       (the real buckets + watchdog) -> agree.

    Returns ``(comm, None)``, or ``(None, reason)`` on every rank after destroying any communicator this
    rank created.  ``make(rank, world, device, uid)`` and ``new_uid()`` replace the communicator factory and
    the id source (CPU tests without RCCL)."""
    from . import runtime
    import torch.distributed as dist
    init_timeout, test_timeout = stage_timeouts(init_timeout)
    make = make or (lambda r, w, d, u: NativeComm(r, w, d, u))

    def failed(stage, flags, err):
        bad = [r for r, ok in enumerate(flags) if not ok]
        return "{} failed on rank(s) {}{}".format(stage, bad, (" (this rank: %s)" % err) if err else "")

    err, uid = None, None
    try:
        _fault(rank, "load")
        if new_uid is None:
            lib()
        uid = (new_uid or unique_id)() if rank == 0 else None
    except Exception as e:  # noqa: BLE001
        err = "%s: %s" % (type(e).__name__, e)
    flags = runtime.rank_flags(err is None)
    if not all(flags):
        return None, failed("load", flags, err)
    if world > 1:
        box = [uid]
        dist.broadcast_object_list(box, src=0)
        uid = box[0]

    comm = None
    try:
        _fault(rank, "init")
        comm = _with_timeout(lambda: make(rank, world, device, uid), init_timeout, on_late=_close_quietly)
    except Exception as e:  # noqa: BLE001
        err = "%s: %s" % (type(e).__name__, e)
    flags = runtime.rank_flags(comm is not None)
    if not all(flags):
        _close_quietly(comm)
        return None, failed("ncclCommInitRank", flags, err)

    try:
        _fault(rank, "selftest")
        if self_test:
            comm.self_test(timeout_s=test_timeout)
        _fault(rank, "setup")
        if setup is not None:
            setup(comm)
    except Exception as e:  # noqa: BLE001
        err = "%s: %s" % (type(e).__name__, e)
    flags = runtime.rank_flags(err is None)
    if not all(flags):
        _close_quietly(comm)
        return None, failed("self-test / setup", flags, err)
    return comm, None


def _close_quietly(comm) -> None:
    if comm is None:
        return
    try:
        comm.close()
    except Exception:  # noqa: BLE001
        pass
