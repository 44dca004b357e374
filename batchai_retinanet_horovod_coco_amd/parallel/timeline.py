"""Chrome-trace timeline of collective activity (Horovod ``HOROVOD_TIMELINE`` equivalent).

Enabled by ``HOROVOD_TIMELINE=<path>`` or ``MXR_TIMELINE=<path>``; rank r writes
``<path>`` (rank 0) or ``<path>.<r>``.  Events follow Horovod's naming: one track per tensor /
bucket with ``NEGOTIATE``-free phases ``READY``, ``ALLREDUCE`` (enqueue -> completion seen by the
host), plus ``STEP`` spans from the training loop.  Open in chrome://tracing or Perfetto.
"""
from __future__ import annotations

import json
import os
import threading
import time
from typing import Optional


class Timeline:
    def __init__(self, path: Optional[str], rank: int = 0):
        self.path = None
        if path:
            self.path = path if rank == 0 else "{}.{}".format(path, rank)
        self.rank = rank
        self._lock = threading.Lock()
        self._f = None
        self._first = True
        self._t0 = time.perf_counter()
        self._tids = {}
        if self.path:
            d = os.path.dirname(os.path.abspath(self.path))
            os.makedirs(d, exist_ok=True)
            self._f = open(self.path, "w")
            self._f.write("[\n")

    @property
    def enabled(self) -> bool:
        return self._f is not None

    def _tid(self, name: str) -> int:
        t = self._tids.get(name)
        if t is None:
            t = len(self._tids) + 1
            self._tids[name] = t
            self._emit({"name": "thread_name", "ph": "M", "pid": self.rank, "tid": t, "args": {"name": name}})
        return t

    def _emit(self, ev) -> None:
        if not self._f:
            return
        with self._lock:
            if not self._first:
                self._f.write(",\n")
            self._first = False
            self._f.write(json.dumps(ev))

    def now_us(self) -> float:
        return (time.perf_counter() - self._t0) * 1e6

    def begin(self, track: str, phase: str, args=None) -> None:
        if self._f:
            self._emit({"name": phase, "ph": "B", "ts": self.now_us(), "pid": self.rank, "tid": self._tid(track),
                        "args": args or {}})

    def end(self, track: str, phase: str) -> None:
        if self._f:
            self._emit({"name": phase, "ph": "E", "ts": self.now_us(), "pid": self.rank, "tid": self._tid(track)})

    def instant(self, track: str, name: str, args=None) -> None:
        if self._f:
            self._emit({"name": name, "ph": "i", "s": "t", "ts": self.now_us(), "pid": self.rank,
                        "tid": self._tid(track), "args": args or {}})

    def close(self) -> None:
        if self._f:
            with self._lock:
                self._f.write("\n]\n")
                self._f.close()
                self._f = None


_TL: Optional[Timeline] = None


def get() -> Timeline:
    global _TL
    if _TL is None:
        from . import runtime
        path = os.environ.get("MXR_TIMELINE") or os.environ.get("HOROVOD_TIMELINE")
        _TL = Timeline(path, runtime.rank() if runtime.is_initialized() else 0)
        if _TL.enabled:
            import atexit
            atexit.register(_TL.close)     # valid JSON even without an explicit shutdown
    return _TL


def reset() -> None:
    global _TL
    if _TL is not None:
        _TL.close()
    _TL = None
