"""Process/rank runtime: the ``hvd.init()`` / ``rank()`` / ``local_rank()`` layer.

Reference: ``hvd.init()`` runs at import (``/root/reference/train.py:20-21``), the GPU is
pinned by local rank (``train.py:71``) and ranks come from ``mpirun`` (``training_job.json:7``).

Here one OS process drives one GPU.  Rank information is read from the environment in this
order: ``OMPI_COMM_WORLD_*`` (mpirun-compatible), ``RANK/WORLD_SIZE/LOCAL_RANK/LOCAL_WORLD_SIZE``
(torchrun / our ``mxrun`` launcher), else a single-process world.  Collectives run on
``torch.distributed``: backend ``nccl`` (= RCCL over xGMI on ROCm) when the process owns a GPU,
``gloo`` on the CPU (tests).  A world of one needs no process group at all (loopback).

``MXR_FAKE_LOCAL_SIZE=k`` splits the ranks into fake "nodes" of k ranks to exercise the
local/cross rank logic on one host.
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass
from typing import Optional

import torch
import torch.distributed as dist


@dataclass
class _State:
    initialized: bool = False
    rank: int = 0
    size: int = 1
    local_rank: int = 0
    local_size: int = 1
    backend: Optional[str] = None
    device: torch.device = torch.device("cpu")
    owns_pg: bool = False
    pg_timeout: Optional[float] = None


_S = _State()


def _env_int(*names, default=None):
    for n in names:
        v = os.environ.get(n)
        if v is not None and v != "":
            return int(v)
    return default


def init(backend: Optional[str] = None, device: Optional[str] = None, timeout_s: Optional[float] = None) -> None:
    """Initialise the world.  Idempotent."""
    if _S.initialized:
        return
    rank = _env_int("OMPI_COMM_WORLD_RANK", "PMI_RANK", "RANK", default=0)
    size = _env_int("OMPI_COMM_WORLD_SIZE", "PMI_SIZE", "WORLD_SIZE", default=1)
    local_rank = _env_int("OMPI_COMM_WORLD_LOCAL_RANK", "LOCAL_RANK", default=None)
    local_size = _env_int("OMPI_COMM_WORLD_LOCAL_SIZE", "LOCAL_WORLD_SIZE", default=None)
    fake = _env_int("MXR_FAKE_LOCAL_SIZE", default=None)
    if fake:
        local_size = fake
        local_rank = rank % fake
    if local_rank is None:
        local_rank = rank
    if local_size is None:
        local_size = size
    _S.rank, _S.size, _S.local_rank, _S.local_size = rank, size, local_rank, local_size

    want_gpu = device != "cpu" and torch.cuda.is_available()
    if device is not None and device != "cpu" and device != "cuda":
        _S.device = torch.device(device)
    elif want_gpu:
        n = torch.cuda.device_count()
        _S.device = torch.device("cuda", local_rank % max(n, 1))
    else:
        _S.device = torch.device("cpu")
    if _S.device.type == "cuda":
        torch.cuda.set_device(_S.device)

    if backend is None:
        backend = os.environ.get("MXR_DIST_BACKEND") or ("nccl" if _S.device.type == "cuda" else "gloo")
    _S.backend = backend
    if size > 1:
        if dist.is_initialized():
            _S.owns_pg = False
        else:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29500")
            t = timeout_s or float(os.environ.get("MXR_COMM_TIMEOUT", "600"))
            _S.pg_timeout = float(t)
            kw = dict(backend=backend, rank=rank, world_size=size, timeout=datetime.timedelta(seconds=t))
            if backend == "nccl":
                kw["device_id"] = _S.device
            dist.init_process_group(**kw)
            _S.owns_pg = True
    _S.initialized = True


def shutdown() -> None:
    from . import ops, timeline
    timeline.reset()              # flush + close the chrome-trace file
    ops.set_native_comm(None)
    from . import collectives
    collectives._GROUPS = None
    if _S.owns_pg and dist.is_initialized():
        dist.destroy_process_group()
    _S.initialized = False
    _S.owns_pg = False


def pg_timeout() -> float:
    """Timeout (s) of the default process group: any bounded wait that a peer may sit out inside a collective
    of that group (the native-comm bring-up stages) must stay well under it."""
    t = getattr(_S, "pg_timeout", None)
    if t is None:
        if dist.is_available() and dist.is_initialized():
            try:
                from torch.distributed.distributed_c10d import _get_default_group
                t = _get_default_group().options._timeout.total_seconds()   # noqa: SLF001
            except Exception:  # noqa: BLE001
                t = None
        if t is None:
            t = float(os.environ.get("MXR_COMM_TIMEOUT", "600"))
    return float(t)


def is_initialized() -> bool:
    return _S.initialized


def _check():
    if not _S.initialized:
        raise ValueError("Horovod-style runtime has not been initialized; use hvd.init().")


def rank() -> int:
    _check(); return _S.rank


def size() -> int:
    _check(); return _S.size


def local_rank() -> int:
    _check(); return _S.local_rank


def local_size() -> int:
    _check(); return _S.local_size


def cross_rank() -> int:
    _check(); return _S.rank // max(_S.local_size, 1)


def cross_size() -> int:
    _check(); return (_S.size + _S.local_size - 1) // max(_S.local_size, 1)


def device() -> torch.device:
    _check(); return _S.device


def backend() -> Optional[str]:
    return _S.backend


def distributed() -> bool:
    return _S.initialized and _S.size > 1


def mpi_threads_supported() -> bool:
    return True


def barrier() -> None:
    if distributed():
        if _S.backend == "nccl":
            dist.barrier(device_ids=[_S.device.index])
        else:
            dist.barrier()


def rank_flags(ok: bool) -> list:
    """Every rank's ``ok`` flag, on every rank (one SUM all-reduce of a one-hot vector over the default
    group).  A collective: every rank must call it the same number of times, whatever happened locally --
    it is how the ranks AGREE on a decision (e.g. native comm engine vs torch.distributed) instead of each
    rank deciding on its own."""
    if not distributed():
        return [bool(ok)]
    dev = _S.device if _S.backend == "nccl" else torch.device("cpu")
    v = torch.zeros(_S.size, dtype=torch.int32, device=dev)
    v[_S.rank] = 1 if ok else 0
    dist.all_reduce(v)
    return [bool(x) for x in v.tolist()]


def agree(ok: bool) -> bool:
    """True iff ``ok`` on EVERY rank (collective, see :func:`rank_flags`)."""
    return all(rank_flags(ok))
