"""Background batch prefetching (Keras ``GeneratorEnqueuer`` semantics: worker threads + queue).

The reference's ``fit_generator`` pulls batches with 1 worker thread and a queue of 10
(``/root/reference/train.py:444-450``, Keras defaults).  Here workers are threads (image decode
in PIL and the native resize/warp release the GIL) and, when a device is given, each batch is
copied host->device on a dedicated HIP stream from pinned memory so the copy overlaps compute.
"""
from __future__ import annotations

import queue
import threading
from typing import Dict, Optional

import torch


class GeneratorEnqueuer:
    def __init__(self, generator, workers: int = 1, max_queue_size: int = 10, device: Optional[torch.device] = None):
        self.generator = generator
        self.workers = max(1, int(workers))
        self.queue: "queue.Queue" = queue.Queue(maxsize=max_queue_size)
        self.device = device
        self._stop = threading.Event()
        self._threads = []
        self._stream = torch.cuda.Stream(device) if (device is not None and device.type == "cuda") else None
        self._error = None

    def _to_device(self, batch: Dict[str, torch.Tensor]):
        if self._stream is None:
            return batch, None
        with torch.cuda.stream(self._stream):
            out = {k: (v if v.is_cuda else v.pin_memory().to(self.device, non_blocking=True)) for k, v in batch.items()}
            ev = torch.cuda.Event()
            ev.record(self._stream)
        return out, ev

    def _next(self):
        if self._stream is None:
            return next(self.generator)
        with torch.cuda.stream(self._stream):        # device-side preprocessing runs on the copy stream
            return next(self.generator)

    def _run(self):
        try:
            while not self._stop.is_set():
                batch = self._next()
                item = self._to_device(batch)
                while not self._stop.is_set():
                    try:
                        self.queue.put(item, timeout=0.1)
                        break
                    except queue.Full:
                        continue
        except Exception as e:  # noqa: BLE001
            self._error = e
            self._stop.set()

    def start(self):
        for _ in range(self.workers):
            t = threading.Thread(target=self._run, daemon=True)
            t.start()
            self._threads.append(t)
        return self

    def get(self) -> Dict[str, torch.Tensor]:
        while True:
            if self._error is not None:
                raise self._error
            try:
                batch, ev = self.queue.get(timeout=0.5)
            except queue.Empty:
                continue
            if ev is not None:
                cur = torch.cuda.current_stream(self.device)
                cur.wait_event(ev)
                for v in batch.values():      # allocated on the copy stream, consumed on this one
                    if v.is_cuda:
                        v.record_stream(cur)
            return batch

    def stop(self):
        self._stop.set()
        for t in self._threads:
            t.join(timeout=5)
        self._threads = []

    def __enter__(self):
        return self.start()

    def __exit__(self, *a):
        self.stop()


def make_enqueuer(generator, workers: int = 1, max_queue_size: int = 10, device: Optional[torch.device] = None,
                  loader: str = "auto"):
    """The batch prefetcher for ``generator``: worker PROCESSES (``data.process_loader``) for a generator
    with device preprocessing when ``loader`` is "process" or "auto" and they can be started safely,
    else worker threads (this module's :class:`GeneratorEnqueuer`)."""
    if loader not in ("auto", "thread", "process"):
        raise ValueError("loader must be auto|thread|process, got %r" % loader)
    if loader == "process" and getattr(generator, "device_preprocessor", None) is None:
        # the workers hand over raw uint8 pixels for the device preprocessing kernels; without it a request
        # for processes would silently run threads
        raise ValueError("--loader process needs device preprocessing (--device-preprocess)")
    if loader != "thread" and getattr(generator, "device_preprocessor", None) is not None:
        from . import process_loader
        if process_loader.usable():
            return process_loader.ProcessEnqueuer(generator, workers=workers, max_queue_size=max_queue_size,
                                                  device=device)
        if loader == "process":
            raise RuntimeError("--loader process: the GPU was initialised before process_loader.prestart(), or "
                               "its forkserver / resource tracker has exited (they cannot be restarted from a "
                               "process that initialised the GPU)")
    return GeneratorEnqueuer(generator, workers=workers, max_queue_size=max_queue_size, device=device)
