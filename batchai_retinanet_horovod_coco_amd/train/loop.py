"""``fit_generator`` -- the Keras training loop the reference drives (``/root/reference/train.py:444-450``).

Semantics kept from Keras 2.x: ``steps_per_epoch`` steps per epoch (each rank pulls its own
batches; there is no epoch-over-dataset notion), epoch logs are the mean of the batch logs,
callbacks fire in list order (``on_train_begin`` -> per epoch ``on_epoch_begin`` / per batch
``on_batch_begin``/``on_batch_end`` / ``on_epoch_end``), ``stop_training`` ends the run, and a
``History`` is returned.  ``initial_epoch`` supports resume (fixing reference quirk #3).

Additions: batches are prefetched by a :class:`data.enqueuer.GeneratorEnqueuer` (H2D on a side
HIP stream), loss scalars stay on the device (synced only when a callback prints them), and
``MXR_FAULT=rank:step:kind`` injects failures (``exit`` | ``hang`` | ``nan`` | ``nanloss``) for tests
(SURVEY §5.3).
"""
from __future__ import annotations

import math
import os
import time
from typing import Dict, List, Optional

import torch

from ..parallel import runtime
from .callbacks import CallbackList, History, ProgbarLogger

METRICS = ["loss", "regression_loss", "classification_loss"]


def _parse_fault():
    spec = os.environ.get("MXR_FAULT")
    if not spec:
        return None
    r, s, kind = spec.split(":")
    return int(r), int(s), kind


def _inject(fault, step: int, trainer, logs=None) -> None:
    if fault is None:
        return
    r, s, kind = fault
    me = runtime.rank() if runtime.is_initialized() else 0
    if me != r or step != s:
        return
    if kind == "exit":
        os._exit(17)
    elif kind == "hang":
        time.sleep(10 ** 6)
    elif kind == "nan":
        with torch.no_grad():
            trainer.flat.data[0] = float("nan")
    elif kind == "nanloss" and logs is not None:
        # only THIS rank sees a non-finite loss (data-dependent NaN): the stop must still be collective
        logs["loss"] = torch.full_like(logs["loss"], float("nan"))


def _any_rank(flag: bool) -> bool:
    """MAX-reduce a stop flag over the ranks (host sync; only used with per-batch stop callbacks)."""
    import torch.distributed as dist
    dev = runtime.device() if runtime.backend() == "nccl" else torch.device("cpu")
    t = torch.tensor([1 if flag else 0], dtype=torch.int32, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return bool(t.item())


def fit_generator(trainer, generator, steps_per_epoch: int, epochs: int = 1, verbose: int = 1,
                  callbacks: Optional[List] = None, initial_epoch: int = 0, workers: int = 1,
                  max_queue_size: int = 10, log_every: int = 1, progbar: bool = True, loader: str = "auto") -> History:
    history = History()
    cbs = list(callbacks or [])
    if verbose and progbar:
        cbs.append(ProgbarLogger(log_every=log_every))
    cbs.append(history)
    cb = CallbackList(cbs)
    cb.set_model(trainer)
    cb.set_params({"epochs": epochs, "steps": steps_per_epoch, "verbose": verbose, "metrics": list(METRICS),
                   "do_validation": False})
    trainer.stop_training = False
    # a callback that can stop mid-epoch (TerminateOnNaN) decides on its rank's own loss: agree across
    # ranks every step, or a rank that stops alone leaves the others blocked in the next all-reduce
    sync_stop = runtime.distributed() and any(getattr(c, "stops_training", False) for c in cbs)
    fault = _parse_fault()
    from ..data.enqueuer import make_enqueuer
    enq = None
    if not isinstance(generator, (list, tuple)) and workers > 0:
        enq = make_enqueuer(generator, workers=workers, max_queue_size=max_queue_size, device=trainer.device,
                            loader=loader).start()
    cb.on_train_begin()
    global_step = 0
    try:
        for epoch in range(initial_epoch, epochs):
            cb.on_epoch_begin(epoch)
            sums: Dict[str, torch.Tensor] = {}
            n = 0
            for step in range(steps_per_epoch):
                batch = enq.get() if enq is not None else next(generator)
                B = int(batch["images"].shape[0])
                cb.on_batch_begin(step, {"batch": step, "size": B})
                logs = trainer.train_on_batch(batch["images"], batch["gt"], batch["gt_count"], batch["image_hw"])
                _inject(fault, global_step, trainer, logs)
                if runtime.distributed():
                    from ..ops.conv_tuner import TUNER
                    if TUNER.sync_due(global_step):
                        TUNER.sync_all()   # one kernel per shape on every rank, new shapes included
                for k in METRICS:
                    sums[k] = sums[k] + logs[k] if k in sums else logs[k].clone()
                n += 1
                global_step += 1
                if global_step == 2:
                    # model, optimizer state, tuner tables and kernel caches exist now: keep them out of the cyclic
                    # GC's generations (a full collection walking them pauses the host ~1 ms mid-step)
                    import gc
                    gc.collect()
                    gc.freeze()
                blogs = dict(logs)
                blogs.update({"batch": step, "size": B})
                cb.on_batch_end(step, blogs)
                if sync_stop:
                    trainer.stop_training = _any_rank(trainer.stop_training)
                if trainer.stop_training:
                    break
            epoch_logs = {k: float(v) / max(n, 1) for k, v in sums.items()}
            cb.on_epoch_end(epoch, epoch_logs)
            if trainer.stop_training:
                break
    finally:
        if enq is not None:
            enq.stop()
    cb.on_train_end()
    return history
