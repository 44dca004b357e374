"""Per-shape algorithm selection for every convolution pass ("measure, don't guess").

Each conv pass (forward / data-gradient / weight-gradient) of each distinct shape has several
implementations: the in-tree HIP implicit-GEMM kernels (tile variants) and the vendor library path
(MIOpen through ``aten.convolution*`` + our fused epilogue kernel).  The first time a shape is seen
-- outside HIP-graph capture -- every candidate is timed with HIP events and the fastest is
recorded; later calls dispatch straight to the winner.  The table can be persisted
(``MXR_SAVE_CONV_TABLE=path``) and loaded (``MXR_CONV_TABLE=path``; ``tuning/conv_table.json`` is
one measured on MI355X) so a job can start tuned; by default every process tunes on its own GPU.

``MXR_CONV_FORCE=hip|miopen`` pins one implementation family (A/B runs, tests);
``MXR_CONV_TUNE=0`` disables timing (first listed candidate wins); ``MXR_CONV_EXCLUDE=miopen`` drops a
family from the candidates wherever another remains (its host-side cost per call is not in the timing).
"""
from __future__ import annotations

import json
import os
import threading
from typing import Callable, Dict, Optional, Tuple

import torch

# hot-path environment reads (several per conv pass): the raw bytes mapping behind os.environ (kept in
# step with it by os.environ / monkeypatch writes), not the per-call key encode of os.environ.get
_ENVD = getattr(os.environ, "_data", None)
if _ENVD is not None and not all(isinstance(k, bytes) for k in list(_ENVD)[:1]):
    _ENVD = None


def _env(key: bytes, default: Optional[str] = None) -> Optional[str]:
    if _ENVD is None:
        return os.environ.get(key.decode(), default)
    v = _ENVD.get(key)
    return default if v is None else v.decode()


_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
DEFAULT_TABLE = os.path.join(_ROOT, "tuning", "conv_table.json")


class ConvTuner:
    def __init__(self):
        self.table: Dict[str, str] = {}
        self.timings: Dict[str, Dict[str, float]] = {}
        self.calls: Dict[str, int] = {}
        # timed work per candidate: enough repetitions to fill ~budget ms (2 reps of a 50 us kernel
        # are within launch noise of each other)
        self.budget_ms = float(os.environ.get("MXR_CONV_TUNE_MS", "2.0"))
        self.lock = threading.Lock()
        self.reps = int(os.environ.get("MXR_CONV_TUNE_REPS", "2"))
        # default: tune on this GPU at first sight (library timings drift between runs / boxes);
        # MXR_CONV_TABLE=path (e.g. tuning/conv_table.json) pins a saved table instead
        path = os.environ.get("MXR_CONV_TABLE", "")
        if path and os.path.exists(path):
            try:
                with open(path) as f:
                    self.table.update(json.load(f).get("table", {}))
            except (OSError, ValueError):
                pass

    @staticmethod
    def key(*parts) -> str:
        return "|".join(str(p) for p in parts)

    def _tuning_allowed(self) -> bool:
        if _env(b"MXR_CONV_TUNE", "1") != "1":
            return False
        try:
            return not torch.cuda.is_current_stream_capturing()
        except Exception:  # noqa: BLE001
            return False

    @staticmethod
    def _filter(names):
        ex = _env(b"MXR_CONV_EXCLUDE")
        if not ex:
            return names
        kept = [n for n in names if not n.startswith(ex)]
        return kept or names

    def needs_tuning(self, key: str, names) -> bool:
        """True when ``run(key, ...)`` would time the candidates (callers whose candidates have side
        effects -- accumulation into an output -- tune a pure version first)."""
        names = self._filter(list(names))
        force = _env(b"MXR_CONV_FORCE")
        if force and any(n.startswith(force) for n in names):
            return False
        if self.table.get(key) in names:
            return False
        return len(names) > 1 and self._tuning_allowed()

    def winner(self, key: str) -> Optional[str]:
        """The recorded choice for ``key`` when a call would dispatch straight to it (no family pinned by the
        environment, the choice itself not excluded), so callers can build that one candidate only; else None."""
        name = self.table.get(key)
        ex = _env(b"MXR_CONV_EXCLUDE")
        if name is None or _env(b"MXR_CONV_FORCE") or (ex and name.startswith(ex)):
            return None
        return name

    def run(self, key: str, cands: Dict[str, Callable[[], object]]):
        """Run the chosen candidate for ``key`` (tuning on first sight). Returns its result."""
        self.calls[key] = self.calls.get(key, 0) + 1
        if _env(b"MXR_CONV_EXCLUDE"):
            keep = self._filter(list(cands))
            cands = {n: cands[n] for n in keep}
        force = _env(b"MXR_CONV_FORCE")
        if force:
            for name, fn in cands.items():
                if name.startswith(force):
                    return fn()
        name = self.table.get(key)
        if name in cands:
            return cands[name]()
        if len(cands) == 1 or not self._tuning_allowed():
            return next(iter(cands.values()))()
        from .side_stream import SIDE
        SIDE.join()                               # race on an otherwise idle GPU: no side-stream wgrads,
        torch.cuda.synchronize()                  # nothing queued on another stream (first sight only)
        best, best_t, best_out, times = None, float("inf"), None, {}
        for name, fn in cands.items():
            try:
                out = fn()                        # warm-up (also JIT/heuristic setup of the library)
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                out = fn()
                e.record()
                e.synchronize()
                t1 = s.elapsed_time(e)
                reps = max(self.reps, min(32, int(self.budget_ms / max(t1, 1e-3))))
                s.record()
                for _ in range(reps):
                    out = fn()
                e.record()
                e.synchronize()
                t = s.elapsed_time(e) / reps
            except RuntimeError as exc:           # an unsupported configuration is simply not a candidate
                times[name] = str(exc)[:80]
                continue
            times[name] = t
            if t < best_t:
                best, best_t, best_out = name, t, out
        # near-ties (within MXR_CONV_TUNE_TIE of the best, 8 % by default) are re-timed round-robin with
        # a larger budget: single back-to-back timings of kernels a few % apart flip between runs
        tie = float(os.environ.get("MXR_CONV_TUNE_TIE", "0.08"))
        close = [n for n, t in times.items() if isinstance(t, float) and t <= best_t * (1 + tie)]
        if len(close) > 1:
            reps = max(self.reps, min(64, int(4 * self.budget_ms / max(best_t, 1e-3))))
            acc = {n: [] for n in close}
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            for _ in range(3):
                for n in close:
                    s.record()
                    for _ in range(reps):
                        out = cands[n]()
                    e.record()
                    e.synchronize()
                    acc[n].append(s.elapsed_time(e) / reps)
                    if n == close[-1]:
                        last_out = out
            med = {n: sorted(v)[1] for n, v in acc.items()}
            win = min(med, key=med.get)
            times.update({n + "~": t for n, t in med.items()})
            if win != best:
                best, best_t = win, med[win]
                best_out = last_out if win == close[-1] else cands[win]()
        with self.lock:
            self.table[key] = best
            self.timings[key] = times
        return best_out

    def save(self, path: Optional[str] = None) -> str:
        path = path or os.environ.get("MXR_CONV_TABLE", DEFAULT_TABLE)
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        with open(path, "w") as f:
            json.dump({"table": self.table, "timings_ms": self.timings, "calls": self.calls}, f, indent=1,
                      sort_keys=True)
        return path

    def sync(self, root: int = 0) -> int:
        """Multi-rank runs: adopt rank ``root``'s choices for every key it tuned.  Each rank times the
        candidates on its own GPU while the others' all-reduces share the chip, so near-tie choices can
        differ between ranks and the step then waits for the slowest rank's kernel mix; after the first
        (tuning) step every rank runs the same kernels.  Returns the number of keys changed here."""
        from ..parallel import collectives, runtime
        if not (runtime.is_initialized() and runtime.distributed()):
            return 0
        with self.lock:
            mine = dict(self.table)
        theirs = collectives.broadcast_object(mine, root)
        changed = 0
        with self.lock:
            for k, v in theirs.items():
                if self.table.get(k) != v:
                    self.table[k] = v
                    changed += 1
        return changed

    def sync_all(self) -> int:
        """Merge every rank's table, the lowest rank's choice winning per key: keys first seen by some
        other rank (COCO batches change H / W from step to step, so new shapes keep appearing after
        step 0) end up with one kernel everywhere.  Returns the number of keys changed here."""
        from ..parallel import collectives, runtime
        if not (runtime.is_initialized() and runtime.distributed()):
            return 0
        with self.lock:
            mine = dict(self.table)
        tables = collectives.allgather_object(mine)
        merged: Dict[str, str] = {}
        for t in reversed(tables):          # rank 0 written last: its choice wins
            merged.update(t)
        changed = 0
        with self.lock:
            for k, v in merged.items():
                if self.table.get(k) != v:
                    self.table[k] = v
                    changed += 1
        return changed

    @staticmethod
    def sync_due(step: int) -> bool:
        """Steps at which a multi-rank loop merges the tables (the same on every rank, no collective
        needed to decide): step 0, every power of two up to 4096, then every 2048 steps."""
        if step < 0:
            return False
        if step == 0 or (step <= 4096 and step & (step - 1) == 0):
            return True
        return step > 4096 and step % 2048 == 0

    def summary(self) -> Dict[str, int]:
        out: Dict[str, int] = {}
        for v in self.table.values():
            fam = "hip" if v and v.startswith("hip") else str(v)
            out[fam] = out.get(fam, 0) + 1
        return out


TUNER = ConvTuner()
