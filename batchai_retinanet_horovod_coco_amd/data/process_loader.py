"""Process-based batch loading for the device-preprocessing path.

The reference pulls batches through Keras ``fit_generator``'s enqueuer (worker threads, queue 10:
``/root/reference/train.py:444-450``).  Thread workers share the GIL with the training loop's dispatch
thread: with the JPEG decode and the per-image Python on loader threads the step measured 12 % slower
than with device-generated batches (``profiles/r2_host_pipeline_bench.txt``).

Here the host work moves into worker PROCESSES:

* the parent keeps the reference's batch order (aspect-ratio groups, group shuffle, one random transform
  drawn per image from ``transform_generator``, in the parent, in order) and hands ``(group, raw
  transforms)`` to the workers;
* a worker decodes the images (PIL), loads / filters / transforms the annotations (the same host box
  arithmetic as ``data/device_preprocess.py``, so annotations are bit-identical to the thread path) and
  writes the uint8 pixels into a slot of one shared-memory arena (``multiprocessing.shared_memory``), which
  the parent registers with the HIP runtime once (``hipHostRegister``: the host->device copy reads the
  arena directly, no staging copy);
* a collector thread in the parent turns each finished slot into the padded device batch (the HIP
  warp / normalise / resize kernels of ``DevicePreprocessor``) on a copy stream, waits for the copies, and
  recycles the slot; batches come out in submission order.

Workers are started from a ``forkserver`` started BEFORE the process touches the GPU (:func:`prestart`,
called at the top of ``bin/train.py``): no worker is ever forked from, or exec'd by, a process that has
initialised HIP.  If the GPU is already initialised and no forkserver is running, the caller falls back
to the thread enqueuer (:func:`usable`).
"""
from __future__ import annotations

import multiprocessing as mp
import queue
import threading
import warnings
from multiprocessing import shared_memory
from typing import Dict, List, Optional

import numpy as np
import torch

_CTX = None


def prestart() -> bool:
    """Start the forkserver the workers are forked from AND the resource tracker that shared-memory
    segments register with (call before anything initialises the GPU: both are started with fork + exec)."""
    global _CTX
    if _CTX is not None:
        return True
    try:
        ctx = mp.get_context("forkserver")
        from multiprocessing import forkserver, resource_tracker
        forkserver.ensure_running()
        resource_tracker.ensure_running()
        _CTX = ctx
        return True
    except Exception as exc:  # noqa: BLE001
        warnings.warn("process loader unavailable: %s" % exc)
        return False


def _child_alive(pid) -> bool:
    """``pid`` (a child of this process) has not exited; ``waitpid(WNOHANG)`` never blocks."""
    import os
    if not pid:
        return False
    try:
        done, _ = os.waitpid(pid, os.WNOHANG)
    except ChildProcessError:
        return False
    return done == 0


def helper_pids():
    """(forkserver pid, resource-tracker pid) as multiprocessing records them; None where this Python's
    private attribute names differ (unknown, NOT exited)."""
    from multiprocessing import forkserver, resource_tracker
    fs = getattr(forkserver, "_forkserver", None)
    rt = getattr(resource_tracker, "_resource_tracker", None)
    return getattr(fs, "_forkserver_pid", None), getattr(rt, "_pid", None)


_WARNED_UNKNOWN = [False]


def helpers_alive() -> bool:
    """The forkserver and the resource tracker are still running.  If either has exited, multiprocessing's
    next ``ensure_running()`` (``Process.start()``, ``SharedMemory(create=True)``) would relaunch it with
    fork + exec from THIS process -- after GPU init that is the exec this pool forbids.

    A helper whose pid this Python does not expose (renamed private attribute) is UNKNOWN, not dead: it was
    started by :func:`prestart` and is taken as alive, with a one-time warning."""
    alive = True
    for name, pid in zip(("forkserver", "resource tracker"), helper_pids()):
        if pid is None:
            if not _WARNED_UNKNOWN[0]:
                _WARNED_UNKNOWN[0] = True
                import warnings
                warnings.warn("process loader: cannot read the %s pid on this Python; assuming it is alive" % name)
            continue
        alive = alive and _child_alive(pid)
    return alive


def _gpu_initialised() -> bool:
    return torch.cuda.is_available() and torch.cuda.is_initialized()


def usable() -> bool:
    """Workers can be started safely: the GPU is still untouched, or prestart() ran before it was and its
    forkserver and resource tracker are both still alive (nothing would be re-exec'd from this process)."""
    if not _gpu_initialised():
        return prestart()
    return _CTX is not None and helpers_alive()


# ------------------------------------------------------------------------------------------ worker side
def _worker(gen, task_q, result_q, shm_name: str, nslots: int, slot_bytes: int) -> None:
    # one thread per worker: a decode worker with the default intra-op pool (OMP_NUM_THREADS, or every CPU
    # the host shows) keeps that many threads runnable; 8 such workers on a 16-CPU share starved the training
    # process -- 5.2 s per step instead of 28 ms on the GPU box (profiles/r4_jpeg_pipeline.txt)
    import os
    os.environ["OMP_NUM_THREADS"] = "1"
    torch.set_num_threads(1)
    try:
        import cv2  # noqa: F401  (absent in this image; if present, keep it single-threaded too)
        cv2.setNumThreads(1)
    except Exception:  # noqa: BLE001
        pass
    from .transform import adjust_transform_for_image, transform_aabb
    from .image import compute_resize_scale
    shm = shared_memory.SharedMemory(name=shm_name)
    # results the parent no longer reads (after stop()) must not hold this process at exit: without this its
    # queue feeder thread blocks the exit until the pipe drains, and stop() waited out a join timeout per worker
    result_q.cancel_join_thread()
    try:
        arena = np.ndarray((nslots, slot_bytes), dtype=np.uint8, buffer=shm.buf)
        while True:
            task = task_q.get()
            if task is None:
                break
            seq, slot, group, raws = task
            try:
                images = gen.load_image_group(group)
                anns = gen.load_annotations_group(group)
                images, anns = gen.filter_annotations(images, anns, group)
                metas = []
                off = 0
                for i, (im, ann) in enumerate(zip(images, anns)):
                    im = np.ascontiguousarray(im, dtype=np.uint8)
                    ann = ann.copy()
                    M = None
                    if raws[i] is not None:
                        M = adjust_transform_for_image(raws[i], im, gen.transform_parameters.relative_translation)
                        for j in range(ann.shape[0]):
                            ann[j, :4] = transform_aabb(M, ann[j, :4])
                    s = compute_resize_scale(im.shape[:2], min_side=gen.image_min_side, max_side=gen.image_max_side)
                    out_hw = (int(round(im.shape[0] * s)), int(round(im.shape[1] * s)))
                    ann[:, :4] *= s
                    nb = im.nbytes
                    if off + nb <= slot_bytes:
                        arena[slot, off:off + nb] = im.reshape(-1)
                        metas.append((im.shape, off, M, out_hw, ann, None))
                        off += (nb + 255) // 256 * 256
                    else:                        # does not fit the slot: goes through the pipe
                        metas.append((im.shape, -1, M, out_hw, ann, im))
                result_q.put((seq, slot, metas, None))
            except Exception as exc:  # noqa: BLE001
                result_q.put((seq, slot, None, "%s: %s" % (type(exc).__name__, exc)))
    finally:
        shm.close()


# ------------------------------------------------------------------------------------------ parent side
class ProcessEnqueuer:
    """``GeneratorEnqueuer``-compatible (``start`` / ``get`` / ``stop``) loader with worker processes.

    ``generator``: a ``data.generator.Generator`` with device preprocessing enabled; ``slot_mb``: shared
    memory per batch slot (a batch's decoded images; larger images travel through the result pipe)."""

    def __init__(self, generator, workers: int = 4, max_queue_size: int = 10, device: Optional[torch.device] = None,
                 slot_mb: float = 0.0):
        if generator.device_preprocessor is None:
            raise ValueError("ProcessEnqueuer needs a generator with device preprocessing enabled")
        if not usable():
            raise RuntimeError("process loader: GPU initialised before prestart(); use the thread enqueuer")
        self.gen = generator
        self.workers = max(1, int(workers))
        self.device = torch.device(device) if device is not None else generator.device_preprocessor.device
        self.nslots = max(2, int(max_queue_size)) + self.workers
        B = generator.batch_size
        per_image = int(slot_mb * 2 ** 20 / B) if slot_mb else 4 * 1024 * 1024   # 1333 x 1000 x 3 uint8
        self.slot_bytes = B * ((per_image + 255) // 256 * 256)
        self.shm = shared_memory.SharedMemory(create=True, size=self.nslots * self.slot_bytes)
        self.arena = torch.frombuffer(self.shm.buf, dtype=torch.uint8).view(self.nslots, self.slot_bytes)
        self._registered = False
        if self.device.type == "cuda":
            try:        # pin the arena: the H2D copies read it directly
                rc = torch.cuda.cudart().cudaHostRegister(self.arena.data_ptr(), self.arena.numel(), 0)
                self._registered = int(rc) == 0
            except Exception:  # noqa: BLE001
                self._registered = False
        self.out: "queue.Queue" = queue.Queue(maxsize=max(1, int(max_queue_size)))
        self.free: "queue.Queue" = queue.Queue()
        for s in range(self.nslots):
            self.free.put(s)
        self._stop = threading.Event()
        self._error: Optional[BaseException] = None
        self._threads: List[threading.Thread] = []
        self._procs = []
        self._stream = torch.cuda.Stream(self.device) if self.device.type == "cuda" else None
        self.stats = {"batches": 0, "images": 0, "inline_images": 0}

    # -------------------------------------------------------------- lifecycle
    def start(self) -> "ProcessEnqueuer":
        ctx = _CTX
        self.task_q = ctx.Queue()
        self.result_q = ctx.Queue()
        for _ in range(self.workers):
            p = ctx.Process(target=_worker, args=(self.gen, self.task_q, self.result_q, self.shm.name, self.nslots,
                                                  self.slot_bytes), daemon=True)
            p.start()
            self._procs.append(p)
        for fn in (self._feed, self._collect):
            t = threading.Thread(target=fn, daemon=True)
            t.start()
            self._threads.append(t)
        return self

    def stop(self) -> None:
        self._stop.set()
        for _ in self._procs:
            try:
                self.task_q.put(None)
            except Exception:  # noqa: BLE001
                pass
        for t in self._threads:
            t.join(timeout=5)
        # the workers finish the task in hand and read their sentinel; one shared deadline for all of them
        # (a per-worker join timeout made stop() cost seconds per worker), then terminate the stragglers
        import time as _time
        deadline = _time.monotonic() + 2.0
        for p in self._procs:
            p.join(timeout=max(0.0, deadline - _time.monotonic()))
        for p in self._procs:
            if p.is_alive():
                p.terminate()
        for p in self._procs:
            p.join(timeout=1.0)
        self._procs, self._threads = [], []
        if self._registered:
            try:
                torch.cuda.synchronize(self.device)
                torch.cuda.cudart().cudaHostUnregister(self.arena.data_ptr())
            except Exception:  # noqa: BLE001
                pass
            self._registered = False
        del self.arena
        try:
            self.shm.close()
        except Exception:  # noqa: BLE001 -- e.g. BufferError while a view of the arena is still exported
            pass
        try:
            self.shm.unlink()            # always: the segment must not outlive the loader in /dev/shm
        except Exception:  # noqa: BLE001
            pass

    def __enter__(self):
        return self.start()

    def __exit__(self, *a):
        self.stop()

    # -------------------------------------------------------------- parent threads
    def _next_task(self):
        """The reference's order: Generator.next's group walk and one raw transform per image."""
        gen = self.gen
        with gen.lock:
            if gen.group_index == 0 and gen.shuffle_groups:
                gen.rng.shuffle(gen.groups)
            group = gen.groups[gen.group_index]
            gen.group_index = (gen.group_index + 1) % len(gen.groups)
        raws = []
        for _ in group:
            if gen.transform_generator is not None:
                with gen._transform_lock:
                    raws.append(next(gen.transform_generator))
            else:
                raws.append(None)
        return group, raws

    def _feed(self) -> None:
        seq = 0
        try:
            while not self._stop.is_set():
                try:
                    slot = self.free.get(timeout=0.1)
                except queue.Empty:
                    continue
                group, raws = self._next_task()
                self.task_q.put((seq, slot, group, raws))
                seq += 1
        except Exception as exc:  # noqa: BLE001
            self._error = exc
            self._stop.set()

    def _dead_worker(self) -> Optional[str]:
        """A worker that exited while the loader runs (OOM kill, crash in native decode): its task's result
        never arrives, so the batch order would wait on it forever."""
        if self._stop.is_set():
            return None
        for i, p in enumerate(self._procs):
            code = p.exitcode
            if code is not None:
                return "loader worker %d (pid %s) exited with code %s" % (i, p.pid, code)
        return None

    def _collect(self) -> None:
        pending: Dict[int, tuple] = {}
        want = 0
        try:
            while not self._stop.is_set():
                dead = self._dead_worker()      # every round, not only on timeouts: live workers keep the
                if dead:                        # results flowing while a dead one's task never arrives
                    raise RuntimeError(dead)
                try:
                    seq, slot, metas, err = self.result_q.get(timeout=0.1)
                except queue.Empty:
                    continue
                if err is not None:
                    raise RuntimeError("loader worker: " + err)
                pending[seq] = (slot, metas)
                while want in pending:
                    slot, metas = pending.pop(want)
                    item = self._assemble(slot, metas)
                    while not self._stop.is_set():
                        try:
                            self.out.put(item, timeout=0.1)
                            break
                        except queue.Full:
                            continue
                    want += 1
        except Exception as exc:  # noqa: BLE001
            self._error = exc
            self._stop.set()

    def _assemble(self, slot: int, metas):
        """Device batch from one slot (on the copy stream); the slot is recycled once its copies are done."""
        if self.device.type != "cuda":
            return self._assemble_host(slot, metas)
        from ..ops import native
        from ..utils import cpu_native
        gen = self.gen
        pre = gen.device_preprocessor
        B = gen.batch_size
        from .generator import pad_shape
        H0 = max(m[3][0] for m in metas)
        W0 = max(m[3][1] for m in metas)
        # the batch canvas is the largest image rounded up to --pad-multiple (shape classes), exactly as the
        # thread path (Generator.compute_input_output) and DevicePreprocessor pad it
        Hm, Wm = pad_shape((H0, W0), getattr(gen, "pad_multiple", 0))
        params = gen.transform_parameters
        interp = cpu_native.INTERP[params.interpolation] if params is not None else 1
        border = cpu_native.BORDER[params.fill_mode] if params is not None else 1
        cval = float(params.cval) if params is not None else 0.0
        ctx = torch.cuda.stream(self._stream) if self._stream is not None else _Null()
        with ctx:
            batch = torch.zeros((B, Hm, Wm, 3), dtype=pre.dtype, device=self.device)
            for i, (shape, off, M, out_hw, ann, inline) in enumerate(metas):
                if off >= 0:
                    n = int(np.prod(shape))
                    host = self.arena[slot, off:off + n].view(*shape)
                    if not self._registered and self.device.type == "cuda":
                        host = host.pin_memory()
                else:
                    host = torch.from_numpy(inline)
                    self.stats["inline_images"] += 1
                    if self.device.type == "cuda":
                        host = host.pin_memory()
                src = host.to(self.device, non_blocking=True)
                f = native.image_warp_normalize(src, M, None, interp, border, cval, pre.scale, pre.mean)
                native.image_resize_into(f, batch, i, out_hw)
            ev = None
            if self._stream is not None:
                ev = torch.cuda.Event()
                ev.record(self._stream)
        if ev is not None:
            ev.synchronize()        # the copies out of this slot are done (GIL released while waiting)
        self.free.put(slot)
        G = max(1, max(m[4].shape[0] for m in metas))
        gt = np.full((B, G, 5), -1.0, dtype=np.float32)
        cnt = np.zeros((B,), dtype=np.int32)
        hw = np.zeros((B, 2), dtype=np.int32)
        for i, m in enumerate(metas):
            ann = m[4]
            gt[i, :ann.shape[0]] = ann
            cnt[i] = ann.shape[0]
            hw[i] = m[3]
        for i in range(len(metas), B):
            hw[i] = (Hm, Wm)         # as the host path's compute_inputs canvas
        self.stats["batches"] += 1
        self.stats["images"] += len(metas)
        out = {"images": batch, "gt": torch.from_numpy(gt), "gt_count": torch.from_numpy(cnt),
               "image_hw": torch.from_numpy(hw)}
        return out, ev

    def _assemble_host(self, slot: int, metas):
        """CPU device: the host pipeline's image work (normalise -> warp -> resize -> pad, the functions
        Generator.preprocess_group_entry calls) on the worker-decoded pixels -- the same batch the thread
        path makes on the host (tests/test_data_io.py)."""
        from .image import apply_transform, resize_image
        gen = self.gen
        imgs = []
        for shape, off, M, out_hw, ann, inline in metas:
            im = self.arena[slot, off:off + int(np.prod(shape))].view(*shape).numpy().copy() if off >= 0 else inline
            im = gen.preprocess_image(im)
            if M is not None:
                im = apply_transform(M, im, gen.transform_parameters)
            im, _ = resize_image(im, min_side=gen.image_min_side, max_side=gen.image_max_side)
            imgs.append(im)
        self.free.put(slot)
        B = gen.batch_size
        G = max(1, max(m[4].shape[0] for m in metas))
        gt = np.full((B, G, 5), -1.0, dtype=np.float32)
        cnt = np.zeros((B,), dtype=np.int32)
        hw = np.zeros((B, 2), dtype=np.int32)
        for i, (m, im) in enumerate(zip(metas, imgs)):
            gt[i, :m[4].shape[0]] = m[4]
            cnt[i] = m[4].shape[0]
            hw[i] = im.shape[:2]
        images = gen.compute_inputs(imgs)
        for i in range(len(metas), B):
            hw[i] = images.shape[1:3]
        self.stats["batches"] += 1
        self.stats["images"] += len(metas)
        return {"images": torch.from_numpy(images), "gt": torch.from_numpy(gt), "gt_count": torch.from_numpy(cnt),
                "image_hw": torch.from_numpy(hw)}, None

    # -------------------------------------------------------------- consumer
    def get(self) -> Dict[str, torch.Tensor]:
        while True:
            if self._error is not None:
                raise self._error
            try:
                batch, ev = self.out.get(timeout=0.5)
            except queue.Empty:
                dead = self._dead_worker()
                if dead and self._error is None:
                    self._error = RuntimeError(dead)
                continue
            if ev is not None:
                cur = torch.cuda.current_stream(self.device)
                cur.wait_event(ev)
                batch["images"].record_stream(cur)
            return batch


class _Null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False
