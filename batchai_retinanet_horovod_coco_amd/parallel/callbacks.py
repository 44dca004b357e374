"""``hvd.callbacks``: BroadcastGlobalVariablesCallback, MetricAverageCallback, LR warmup/schedule.

Reference: ``hvd.callbacks.BroadcastGlobalVariablesCallback(0)`` is the first callback
(``/root/reference/train.py:111``): in ``on_train_begin`` every global variable -- trainable
weights, frozen BN statistics and the optimizer slots -- is broadcast from the root rank
(SURVEY §2.7 C2).  Here that is one coalesced flat broadcast per dtype.

``MetricAverageCallback`` all-reduces the epoch logs so that ``ReduceLROnPlateau`` sees the
same (global) loss on every rank -- the fix for reference quirk #4 (per-rank LR divergence).
"""
from __future__ import annotations

from typing import Optional

import torch

from ..train.callbacks import Callback
from . import collectives, runtime


class BroadcastGlobalVariablesCallback(Callback):
    def __init__(self, root_rank: int = 0, device: Optional[str] = None):
        super().__init__()
        self.root_rank = root_rank
        self.broadcast_done = False

    def on_train_begin(self, logs=None):
        if self.broadcast_done:
            return
        tr = self.model
        collectives.broadcast_parameters(tr.state_for_broadcast(), self.root_rank)
        collectives.broadcast_optimizer_state(tr.base_optimizer, self.root_rank)
        if hasattr(tr, "on_weights_changed"):
            tr.on_weights_changed()
        self.broadcast_done = True


class MetricAverageCallback(Callback):
    """Average epoch-end logs over ranks (runs before checkpoint/TensorBoard/LR callbacks)."""

    def on_epoch_end(self, epoch, logs=None):
        if logs is None or not runtime.distributed():
            return
        keys = sorted(k for k, v in logs.items() if isinstance(v, (int, float)) or torch.is_tensor(v))
        if not keys:
            return
        dev = runtime.device() if runtime.backend() == "nccl" else torch.device("cpu")
        vals = torch.tensor([float(logs[k]) for k in keys], dtype=torch.float64, device=dev)
        collectives.allreduce_(vals, average=True, name="metric_average")
        for k, v in zip(keys, vals.tolist()):
            logs[k] = v


class LearningRateWarmupCallback(Callback):
    """Horovod-style gradual warmup: lr ramps from ``lr/size`` to ``lr`` over ``warmup_epochs``."""

    def __init__(self, warmup_epochs: float = 5, steps_per_epoch: Optional[int] = None, verbose: int = 0,
                 initial_lr: Optional[float] = None):
        super().__init__()
        self.warmup_epochs = warmup_epochs
        self.steps_per_epoch = steps_per_epoch
        self.verbose = verbose
        self.initial_lr = initial_lr
        self.current_epoch = 0

    def on_train_begin(self, logs=None):
        if self.initial_lr is None:
            self.initial_lr = float(self.model.lr)
        if self.steps_per_epoch is None:
            self.steps_per_epoch = self.params.get("steps") or 1

    def on_epoch_begin(self, epoch, logs=None):
        self.current_epoch = epoch

    def on_batch_begin(self, batch, logs=None):
        e = self.current_epoch + float(batch) / self.steps_per_epoch
        if e >= self.warmup_epochs:
            return
        size = runtime.size() if runtime.is_initialized() else 1
        mult = 1.0 / size * (e * (size - 1) / self.warmup_epochs + 1)
        self.model.lr = self.initial_lr * mult

    def on_epoch_end(self, epoch, logs=None):
        if epoch + 1 == int(self.warmup_epochs):
            self.model.lr = self.initial_lr
            if self.verbose and (not runtime.is_initialized() or runtime.rank() == 0):
                print("\nEpoch %d: finished gradual learning rate warmup to %g." % (epoch + 1, self.initial_lr))


class LearningRateScheduleCallback(Callback):
    """lr = initial_lr * multiplier(epoch) for start_epoch <= epoch < end_epoch."""

    def __init__(self, multiplier, start_epoch: int = 0, end_epoch: Optional[int] = None,
                 initial_lr: Optional[float] = None):
        super().__init__()
        self.multiplier = multiplier if callable(multiplier) else (lambda e, m=multiplier: m)
        self.start_epoch = start_epoch
        self.end_epoch = end_epoch
        self.initial_lr = initial_lr

    def on_train_begin(self, logs=None):
        if self.initial_lr is None:
            self.initial_lr = float(self.model.lr)

    def on_epoch_begin(self, epoch, logs=None):
        if epoch >= self.start_epoch and (self.end_epoch is None or epoch < self.end_epoch):
            self.model.lr = self.initial_lr * self.multiplier(epoch)
