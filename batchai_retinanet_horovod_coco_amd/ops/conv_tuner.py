"""Per-shape algorithm selection for every convolution pass ("measure, don't guess").

Each conv pass (forward / data-gradient / weight-gradient) of each distinct shape has several
implementations: the in-tree HIP implicit-GEMM kernels (tile variants) and the vendor library path
(MIOpen through ``aten.convolution*`` + our fused epilogue kernel).  The first time a shape is seen
-- outside HIP-graph capture -- every candidate is timed with HIP events and the fastest is
recorded; later calls dispatch straight to the winner.  The table can be persisted
(``MXR_SAVE_CONV_TABLE=path``) and loaded (``MXR_CONV_TABLE=path``; ``tuning/conv_table.json`` is
one measured on MI355X) so a job can start tuned; by default every process tunes on its own GPU.

``MXR_CONV_FORCE=hip|miopen`` pins one implementation family (A/B runs, tests);
``MXR_CONV_TUNE=0`` disables timing (first listed candidate wins); ``MXR_CONV_EXCLUDE=<prefix>`` drops a
family from the candidates wherever another remains.  The default is ``miopen``: MIOpen's first-sight
find takes seconds per shape and never won a race on the HIP path (profiles/r4_*), so it only runs where
no in-tree kernel covers a shape (``MXR_CONV_EXCLUDE=none`` races it again).

Shape classes (real COCO batches change H x W from step to step; /root/reference/train.py:197-214,377-378):
a key first seen at a new spatial size reuses the winner of the NEAREST tuned key of the same layer
signature (every key field but the spatial ones) instead of re-racing, when the pixel counts differ by at
most ``MXR_CONV_NEAREST`` in log space (default 0.7, about 2x; 0 = always race).  ``borrowed`` records
which key each reused choice came from.
"""
from __future__ import annotations

import functools
import json
import math
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
        self.borrowed: Dict[str, str] = {}      # key -> the raced key whose winner it reuses (shape classes)
        self._near_memo: Dict[tuple, tuple] = {}
        self._gen = 0       # bumped by every table / borrowed write (prefer and sync included): the memo's clock
        self.calls: Dict[str, int] = {}
        self.preferred: Dict[str, str] = {}     # key -> the raced winner a prefer() call replaced
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
                    saved = json.load(f)
                self.table.update(saved.get("table", {}))
                self.borrowed.update(saved.get("borrowed", {}))
            except (OSError, ValueError):
                pass

    @staticmethod
    def key(*parts) -> str:
        return "|".join(str(p) for p in parts)

    # ------------------------------------------------------------------ shape classes
    @staticmethod
    @functools.lru_cache(maxsize=65536)
    def split_key(key: str):
        """(signature, pixels) of a conv key: the signature is the key with its spatial fields replaced by
        '*' (pyramid keys: the level tuple; plain keys: H and W), pixels = the spatial size it held (all
        levels summed).  None for keys of another form."""
        parts = key.split("|")
        if len(parts) < 4:
            return None
        try:
            if parts[0] in ("pfwd", "pdgrad", "pwgrad"):
                import ast
                shapes = ast.literal_eval(parts[2])
                px = sum(int(h) * int(w) for h, w in shapes)
                sig = "|".join(parts[:2] + ["*"] + parts[3:])
            elif parts[0] in ("fwd", "dgrad", "wgrad"):
                px = int(parts[2]) * int(parts[3])
                sig = "|".join(parts[:2] + ["*", "*"] + parts[4:])
            elif parts[0] in ("fwdp", "dgradp", "wgradp") and len(parts) >= 10:
                # projection-block GEMMs: kind|N|Ho|Wo|a|b|c|stride|H|W[|flags] -- both grids are spatial
                px = int(parts[2]) * int(parts[3])
                sig = "|".join(parts[:2] + ["*", "*"] + parts[4:8] + ["*", "*"] + parts[10:])
            else:
                return None
        except (ValueError, SyntaxError, TypeError):
            return None
        return sig, px

    def _nearest(self, key: str, names=None) -> Optional[Tuple[str, str]]:
        """(winner, source key) of the nearest raced (or loaded) key of ``key``'s signature whose winner is among
        ``names`` (any name when None), within the MXR_CONV_NEAREST log-pixel radius; else None."""
        radius = float(_env(b"MXR_CONV_NEAREST", "0.7"))
        if radius <= 0:
            return None
        sk = self.split_key(key)
        if sk is None:
            return None
        # memo per (key, candidate set) until the table changes: winner() runs on every conv pass, and a key
        # that only ever goes through winner() (the fused weight + bias gradient) must not rescan the table
        # each time (measured: ~25 ms per training step on real COCO batches before this memo)
        mkey = (key, None if names is None else frozenset(names))
        hit = self._near_memo.get(mkey)
        if hit is not None and hit[0] == self._table_gen():
            return hit[1]
        res = self._nearest_scan(key, names, sk, radius)
        self._near_memo[mkey] = (self._table_gen(), res)
        return res

    def _table_gen(self):
        # (direct edits of the dicts -- tests, a loaded table -- change the lengths at least)
        return (self._gen, len(self.table), len(self.borrowed))

    def _set(self, key: str, name: str, borrowed_from: Optional[str] = None) -> None:
        """Record ``name`` for ``key`` (caller holds the lock): a raced / preferred / synced choice drops the key's
        borrowed link (its timings are its own from now on), a borrowed one records its source key."""
        self.table[key] = name
        if borrowed_from is None:
            self.borrowed.pop(key, None)
        else:
            self.borrowed[key] = borrowed_from
        self._gen += 1

    def _nearest_scan(self, key, names, sk, radius):
        sig, px = sk
        best = None
        with self.lock:
            items = [(k, v) for k, v in self.table.items() if k not in self.borrowed]
        for k, v in items:
            if names is not None and v not in names:
                continue
            o = self.split_key(k)
            if o is None or o[0] != sig or o[1] <= 0 or px <= 0:
                continue
            d = abs(math.log(px / o[1]))
            if d <= radius and (best is None or d < best[0]):
                best = (d, v, k)
        return None if best is None else (best[1], best[2])

    def _borrow(self, key: str, names) -> Optional[str]:
        """Adopt the nearest shape class's winner for ``key`` (recorded in the table and ``borrowed``)."""
        hit = self._nearest(key, names)
        if hit is None:
            return None
        with self.lock:
            self._set(key, hit[0], hit[1])
        return hit[0]

    def _tuning_allowed(self) -> bool:
        if _env(b"MXR_CONV_TUNE", "1") != "1":
            return False
        try:
            return not torch.cuda.is_current_stream_capturing()
        except Exception:  # noqa: BLE001
            return False

    @staticmethod
    def _exclude() -> Optional[str]:
        ex = _env(b"MXR_CONV_EXCLUDE", "miopen")
        return None if (not ex or ex == "none") else ex

    @classmethod
    def _filter(cls, names):
        ex = cls._exclude()
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
        if len(names) <= 1 or not self._tuning_allowed():
            return False
        return self._nearest(key, set(names)) is None

    def winner(self, key: str) -> Optional[str]:
        """The recorded choice for ``key`` when a call would dispatch straight to it (no family pinned by the
        environment, the choice itself not excluded), so callers can build that one candidate only; else None."""
        name = self.table.get(key)
        if name is None:
            hit = self._nearest(key)
            name = hit[0] if hit is not None else None
            if hit is not None and self._tuning_allowed():
                # adopt it: the key's next calls dispatch from the table (a caller whose candidates do not
                # include it falls back to run(), which races, overwrites the entry and drops the borrowed link)
                with self.lock:
                    self._set(key, hit[0], hit[1])
        ex = self._exclude()
        if name is None or _env(b"MXR_CONV_FORCE") or (ex and name.startswith(ex)):
            return None
        return name

    def prefer(self, key: str, name: str, margin_ms: float) -> bool:
        """Adopt candidate ``name`` for the tuned ``key`` when its time is within ``margin_ms`` of the recorded
        winner's, and return whether ``name`` is now the choice.  For candidates that unlock work outside the
        timed call (a fused loss epilogue, an output that needs no bf16 store): the race cannot see that saving,
        and near-ties flip between runs (the 8 % re-timing resolves noise, not the caller's extra kernels).
        Compares the round-robin re-timed medians when both have one, else the first-pass times."""
        win = self.winner(key)
        if win is None:
            return False
        if win == name:
            return True
        t = self.timings.get(self.borrowed.get(key, key), {})

        def best(n, retimed):
            v = t.get(n + "~" if retimed else n)
            return v if isinstance(v, float) else None
        retimed = best(name, True) is not None and best(win, True) is not None
        a, b = best(name, retimed), best(win, retimed)
        if a is None or b is None or a > b + margin_ms:
            return False
        with self.lock:
            self.table[key] = name       # a preference keeps the borrowed link: its timings are the source's
            self._gen += 1
            self.preferred[key] = win
        return True

    def run(self, key: str, cands: Dict[str, Callable[[], object]]):
        """Run the chosen candidate for ``key`` (tuning on first sight). Returns its result."""
        self.calls[key] = self.calls.get(key, 0) + 1
        force = _env(b"MXR_CONV_FORCE")
        if force:
            for name, fn in cands.items():
                if name.startswith(force):
                    return fn()
        if self._exclude():
            keep = self._filter(list(cands))
            cands = {n: cands[n] for n in keep}
        name = self.table.get(key)
        if name in cands:
            return cands[name]()
        if len(cands) == 1 or not self._tuning_allowed():
            return next(iter(cands.values()))()
        name = self._borrow(key, set(cands))
        if name is not None:
            return cands[name]()
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
            self._set(key, best)
            self.timings[key] = times
        return best_out

    def save(self, path: Optional[str] = None) -> str:
        path = path or os.environ.get("MXR_CONV_TABLE", DEFAULT_TABLE)
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        with open(path, "w") as f:
            json.dump({"table": self.table, "timings_ms": self.timings, "calls": self.calls,
                       "borrowed": self.borrowed}, f, indent=1, sort_keys=True)
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
            self._gen += 1
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
            self._gen += 1
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
