"""Keras-compatible callbacks used by the reference training script.

``create_callbacks`` in the reference (``/root/reference/train.py:110-174``) builds, in order:
``BroadcastGlobalVariablesCallback(0)``, rank-0 ``ModelCheckpoint('checkpoint-{epoch:02d}.h5')``,
rank-0 ``TensorBoard``, optional ``RedirectModel(CocoEval | Evaluate, prediction_model)`` and
``ReduceLROnPlateau(monitor='loss', factor=0.1, patience=2, epsilon=1e-4, cooldown=0, min_lr=0)``.
This module provides those (plus ``ProgbarLogger``, ``TerminateOnNaN``, ``CSVLogger``,
``JSONLMetrics``); the Horovod ones live in :mod:`parallel.callbacks`.

The "model" a callback sees is the :class:`train.engine.Trainer` (it carries ``model``,
``optimizer``, ``lr``, ``stop_training``).
"""
from __future__ import annotations

import csv
import json
import math
import os
import sys
import time
import warnings
from typing import Dict, List, Optional

import numpy as np


def _f(v) -> float:
    try:
        return float(v)
    except Exception:  # noqa: BLE001
        return float("nan")


class Callback:
    def __init__(self):
        self.model = None
        self.params: Dict = {}

    def set_params(self, params: Dict) -> None:
        self.params = params

    def set_model(self, model) -> None:
        self.model = model

    def on_epoch_begin(self, epoch, logs=None): pass
    def on_epoch_end(self, epoch, logs=None): pass
    def on_batch_begin(self, batch, logs=None): pass
    def on_batch_end(self, batch, logs=None): pass
    def on_train_begin(self, logs=None): pass
    def on_train_end(self, logs=None): pass


class CallbackList:
    def __init__(self, callbacks: Optional[List[Callback]] = None):
        self.callbacks = [c for c in (callbacks or []) if c is not None]

    def append(self, cb: Callback) -> None:
        self.callbacks.append(cb)

    def set_params(self, params):
        for c in self.callbacks:
            c.set_params(params)

    def set_model(self, model):
        for c in self.callbacks:
            c.set_model(model)

    def _call(self, name, *args):
        for c in self.callbacks:
            getattr(c, name)(*args)

    def on_epoch_begin(self, epoch, logs=None): self._call("on_epoch_begin", epoch, logs if logs is not None else {})
    def on_epoch_end(self, epoch, logs=None): self._call("on_epoch_end", epoch, logs if logs is not None else {})
    def on_batch_begin(self, batch, logs=None): self._call("on_batch_begin", batch, logs if logs is not None else {})
    def on_batch_end(self, batch, logs=None): self._call("on_batch_end", batch, logs if logs is not None else {})
    def on_train_begin(self, logs=None): self._call("on_train_begin", logs if logs is not None else {})
    def on_train_end(self, logs=None): self._call("on_train_end", logs if logs is not None else {})


class ProgbarLogger(Callback):
    """Keras Progbar line: ``step/steps [====>....] - ETA: 1s - loss: x - regression_loss: ...``.

    ``log_every`` bounds how often device scalars are synced for printing (1 = every step, like
    the reference's verbose=1 on every rank).
    """

    def __init__(self, log_every: int = 1, stream=None, width: int = 30, prefix: str = ""):
        super().__init__()
        self.log_every = max(1, int(log_every))
        self.stream = stream or sys.stdout
        self.width = width
        self.prefix = prefix
        self.tty = hasattr(self.stream, "isatty") and self.stream.isatty()

    def on_epoch_begin(self, epoch, logs=None):
        self.steps = self.params.get("steps")
        self.t0 = time.time()
        self.seen = 0
        self.sums: Dict[str, float] = {}
        self.stream.write("{}Epoch {}/{}\n".format(self.prefix, epoch + 1, self.params.get("epochs")))
        self.stream.flush()

    def _line(self, current, values):
        n = self.steps or current
        frac = min(1.0, current / float(n))
        done = int(self.width * frac)
        bar = "=" * max(0, done - 1) + (">" if done < self.width else "=") + "." * (self.width - done)
        elapsed = time.time() - self.t0
        per = elapsed / max(current, 1)
        if current < n:
            info = " - ETA: {:.0f}s".format(per * (n - current))
        else:
            info = " - {:.0f}s {:.0f}ms/step".format(elapsed, per * 1000)
        for k, v in values.items():
            info += " - {}: {:.4f}".format(k, v)
        digits = len(str(n))
        return "{}{:>{d}}/{} [{}]{}".format(self.prefix, current, n, bar, info, d=digits)

    def on_batch_end(self, batch, logs=None):
        logs = logs or {}
        self.seen = batch + 1
        if (batch + 1) % self.log_every and (batch + 1) != self.steps:
            return
        vals = {}
        for k in self.params.get("metrics", []):
            if k in logs:
                vals[k] = _f(logs[k])
        line = self._line(batch + 1, vals)
        self.stream.write(("\r" + line) if self.tty else (line + "\n"))
        self.stream.flush()

    def on_epoch_end(self, epoch, logs=None):
        if self.tty:
            self.stream.write("\n")
            self.stream.flush()


class History(Callback):
    def on_train_begin(self, logs=None):
        self.epoch: List[int] = []
        self.history: Dict[str, List[float]] = {}

    def on_epoch_end(self, epoch, logs=None):
        self.epoch.append(epoch)
        for k, v in (logs or {}).items():
            self.history.setdefault(k, []).append(_f(v))


class ModelCheckpoint(Callback):
    """Rank-0 checkpointing; ``filepath`` may contain ``{epoch:02d}`` and log keys (1-based epoch)."""

    def __init__(self, filepath: str, monitor: str = "val_loss", verbose: int = 0, save_best_only: bool = False,
                 save_weights_only: bool = False, mode: str = "auto", period: int = 1, fmt: Optional[str] = None):
        super().__init__()
        self.filepath = filepath
        self.monitor = monitor
        self.verbose = verbose
        self.save_best_only = save_best_only
        self.save_weights_only = save_weights_only
        self.period = period
        self.fmt = fmt
        self.epochs_since_last_save = 0
        if mode == "min" or (mode == "auto" and "acc" not in monitor and "mAP" not in monitor):
            self.monitor_op, self.best = np.less, np.inf
        else:
            self.monitor_op, self.best = np.greater, -np.inf

    def on_epoch_end(self, epoch, logs=None):
        from ..io import checkpoint
        logs = logs or {}
        self.epochs_since_last_save += 1
        if self.epochs_since_last_save < self.period:
            return
        self.epochs_since_last_save = 0
        filepath = self.filepath.format(epoch=epoch + 1, **{k: _f(v) for k, v in logs.items()})
        if self.save_best_only:
            current = logs.get(self.monitor)
            if current is None:
                warnings.warn("Can save best model only with {} available, skipping.".format(self.monitor))
                return
            if not self.monitor_op(_f(current), self.best):
                return
            self.best = _f(current)
        opt = None if self.save_weights_only else self.model.base_optimizer
        fmt = self.fmt or ("safetensors" if filepath.endswith(".safetensors") else "h5")
        checkpoint.save_checkpoint(filepath, self.model.model, opt, epoch=epoch + 1, fmt=fmt)
        if self.verbose > 0:
            print("\nEpoch %05d: saving model to %s" % (epoch + 1, filepath))


class TensorBoard(Callback):
    """Rank-0 epoch scalars (loss, regression_loss, classification_loss, lr + eval metrics)."""

    def __init__(self, log_dir: str = "./logs", histogram_freq: int = 0, batch_size: int = 32, write_graph: bool = True,
                 write_grads: bool = False, write_images: bool = False, **kwargs):
        super().__init__()
        self.log_dir = log_dir
        self.write_graph = write_graph
        self.writer = None

    def _w(self):
        if self.writer is None:
            from ..io.tb_events import EventFileWriter
            self.writer = EventFileWriter(self.log_dir)
        return self.writer

    def on_train_begin(self, logs=None):
        self._w()

    def on_epoch_end(self, epoch, logs=None):
        scal = {k: _f(v) for k, v in (logs or {}).items() if isinstance(v, (int, float)) or hasattr(v, "item")}
        if self.model is not None and "lr" not in scal:
            scal["lr"] = float(self.model.lr)
        self._w().add_scalars(scal, epoch)

    def add_scalars(self, scalars: Dict[str, float], step: int) -> None:
        self._w().add_scalars(scalars, step)

    def on_train_end(self, logs=None):
        if self.writer is not None:
            self.writer.close()
            self.writer = None


class ReduceLROnPlateau(Callback):
    """Keras 2.2 ReduceLROnPlateau (``epsilon`` is the old name of ``min_delta``)."""

    def __init__(self, monitor: str = "val_loss", factor: float = 0.1, patience: int = 10, verbose: int = 0,
                 mode: str = "auto", epsilon: float = 1e-4, cooldown: int = 0, min_lr: float = 0, min_delta=None):
        super().__init__()
        if factor >= 1.0:
            raise ValueError("ReduceLROnPlateau does not support a factor >= 1.0.")
        self.monitor = monitor
        self.factor = factor
        self.min_lr = min_lr
        self.min_delta = epsilon if min_delta is None else min_delta
        self.patience = patience
        self.verbose = verbose
        self.cooldown = cooldown
        self.cooldown_counter = 0
        self.wait = 0
        self.mode = mode
        self._reset()

    def _reset(self):
        if self.mode == "min" or (self.mode == "auto" and "acc" not in self.monitor):
            self.monitor_op = lambda a, b: np.less(a, b - self.min_delta)
            self.best = np.inf
        else:
            self.monitor_op = lambda a, b: np.greater(a, b + self.min_delta)
            self.best = -np.inf
        self.cooldown_counter = 0
        self.wait = 0

    def on_train_begin(self, logs=None):
        self._reset()

    def in_cooldown(self):
        return self.cooldown_counter > 0

    def on_epoch_end(self, epoch, logs=None):
        logs = logs if logs is not None else {}
        logs["lr"] = float(self.model.lr)
        current = logs.get(self.monitor)
        if current is None:
            warnings.warn("Reduce LR on plateau conditioned on metric `{}` which is not available.".format(self.monitor))
            return
        current = _f(current)
        if self.in_cooldown():
            self.cooldown_counter -= 1
            self.wait = 0
        if self.monitor_op(current, self.best):
            self.best = current
            self.wait = 0
        elif not self.in_cooldown():
            self.wait += 1
            if self.wait >= self.patience:
                old_lr = float(self.model.lr)
                if old_lr > self.min_lr:
                    new_lr = max(old_lr * self.factor, self.min_lr)
                    self.model.lr = new_lr
                    if self.verbose > 0:
                        print("\nEpoch %05d: ReduceLROnPlateau reducing learning rate to %s." % (epoch + 1, new_lr))
                    self.cooldown_counter = self.cooldown
                    self.wait = 0


class TerminateOnNaN(Callback):
    stops_training = True     # fit_generator agrees on the stop across ranks every batch

    def on_batch_end(self, batch, logs=None):
        loss = (logs or {}).get("loss")
        if loss is not None and not math.isfinite(_f(loss)):
            print("Batch %d: Invalid loss, terminating training" % batch)
            self.model.stop_training = True


class RedirectModel(Callback):
    """Run ``callback`` against a different model (the prediction model), keras-retinanet style."""

    def __init__(self, callback: Callback, model):
        super().__init__()
        self.callback = callback
        self.redirect_model = model

    def set_params(self, params):
        super().set_params(params)
        self.callback.set_params(params)

    def on_epoch_begin(self, epoch, logs=None): self.callback.on_epoch_begin(epoch, logs)
    def on_epoch_end(self, epoch, logs=None): self.callback.on_epoch_end(epoch, logs)
    def on_batch_begin(self, batch, logs=None): self.callback.on_batch_begin(batch, logs)
    def on_batch_end(self, batch, logs=None): self.callback.on_batch_end(batch, logs)

    def on_train_begin(self, logs=None):
        self.callback.set_model(self.redirect_model)
        self.callback.on_train_begin(logs)

    def on_train_end(self, logs=None):
        self.callback.on_train_end(logs)


class CSVLogger(Callback):
    def __init__(self, filename: str, append: bool = False):
        super().__init__()
        self.filename = filename
        self.append = append
        self._f = None
        self._w = None

    def on_train_begin(self, logs=None):
        self._f = open(self.filename, "a" if self.append else "w", newline="")

    def on_epoch_end(self, epoch, logs=None):
        row = {"epoch": epoch}
        row.update({k: _f(v) for k, v in (logs or {}).items()})
        if self._w is None:
            self._w = csv.DictWriter(self._f, fieldnames=list(row.keys()))
            if not self.append:
                self._w.writeheader()
        self._w.writerow({k: row.get(k) for k in self._w.fieldnames})
        self._f.flush()

    def on_train_end(self, logs=None):
        if self._f:
            self._f.close()


class JSONLMetrics(Callback):
    """Per-step JSONL metrics: step, loss terms, lr, img/s, step_ms."""

    def __init__(self, path: str, every: int = 1, batch_size: int = 1, world: int = 1):
        super().__init__()
        self.path = path
        self.every = max(1, every)
        self.batch_size = batch_size
        self.world = world
        self._f = None
        self._t = None
        self.global_step = 0

    def on_train_begin(self, logs=None):
        os.makedirs(os.path.dirname(os.path.abspath(self.path)), exist_ok=True)
        self._f = open(self.path, "a")

    def on_epoch_begin(self, epoch, logs=None):
        self.epoch = epoch

    def on_batch_begin(self, batch, logs=None):
        if self._t is None:
            self._t = time.time()

    def on_batch_end(self, batch, logs=None):
        self.global_step += 1
        if self.global_step % self.every:
            return
        now = time.time()
        dt = (now - self._t) / self.every
        self._t = now
        rec = {"epoch": self.epoch, "step": self.global_step, "lr": float(self.model.lr), "step_ms": 1000 * dt,
               "img_per_sec": self.batch_size * self.world / max(dt, 1e-9)}
        rec.update({k: _f(v) for k, v in (logs or {}).items() if k in ("loss", "regression_loss",
                                                                         "classification_loss")})
        self._f.write(json.dumps(rec) + "\n")
        self._f.flush()

    def on_train_end(self, logs=None):
        if self._f:
            self._f.close()
