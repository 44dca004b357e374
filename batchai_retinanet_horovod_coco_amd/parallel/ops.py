"""``torch.library`` collective ops: ``mxr::allreduce_``, ``mxr::broadcast_``, ``mxr::allgather``.

The reference reaches Horovod's TF custom ops (``HorovodAllreduce`` / ``HorovodBroadcast`` /
``HorovodAllgather``, SURVEY §2.2 E-HVD-tfop, §2.3 N2) through ``hvd.DistributedOptimizer``
(``/root/reference/train.py:103-104``) and ``BroadcastGlobalVariablesCallback``
(``train.py:111``).  Those ops were CPU-registered in the reference's MPI-only build, so every
gradient took a device->host copy.  Here the ops are registered with the PyTorch dispatcher and stay
on the device:

* on a GPU tensor, when a native communicator is installed (:func:`set_native_comm`, done by the
  ``DistributedOptimizer`` under ``MXR_COMM=native``), they call the C++ comm core
  (``csrc/comm/comm.hip``: RCCL on the current HIP stream);
* otherwise they go through :mod:`.collectives` (torch.distributed: RCCL over xGMI or gloo).

Being real dispatcher ops (with fake/meta kernels) they can be used from traced or captured code
and from TorchScript-free C++ callers via ``torch.ops.mxr.*``.
"""
from __future__ import annotations

from typing import Optional

import torch

from . import collectives, runtime

_NATIVE = None


def set_native_comm(comm) -> None:
    """Install (or clear with ``None``) the :class:`~.native_comm.NativeComm` used for GPU tensors."""
    global _NATIVE
    _NATIVE = comm


def native_comm():
    return _NATIVE


def _use_native(t: torch.Tensor) -> bool:
    return _NATIVE is not None and t.is_cuda


@torch.library.custom_op("mxr::allreduce_", mutates_args=("tensor",))
def allreduce_(tensor: torch.Tensor, average: bool = True) -> None:
    """In-place all-reduce (sum, or sum / size when ``average``)."""
    if _use_native(tensor):
        _NATIVE.allreduce_(tensor, average=average)
    else:
        collectives.allreduce_(tensor, average=average)


@allreduce_.register_fake
def _(tensor, average=True):
    return None


@torch.library.custom_op("mxr::broadcast_", mutates_args=("tensor",))
def broadcast_(tensor: torch.Tensor, root_rank: int = 0) -> None:
    """In-place broadcast from ``root_rank``."""
    if _use_native(tensor):
        _NATIVE.broadcast_(tensor, root=root_rank)
    else:
        collectives.broadcast_(tensor, root_rank)


@broadcast_.register_fake
def _(tensor, root_rank=0):
    return None


@torch.library.custom_op("mxr::allgather", mutates_args=())
def allgather(tensor: torch.Tensor) -> torch.Tensor:
    """Concatenate every rank's tensor along dim 0.  The native path needs equal shapes on every
    rank (one RCCL allgather); the torch path also accepts ragged first dimensions."""
    if _use_native(tensor) and tensor.dim() > 0:
        out = _NATIVE.allgather(tensor.contiguous())
        return out.reshape((-1,) + tuple(tensor.shape[1:]))
    return collectives.allgather(tensor)


@allgather.register_fake
def _(tensor):
    shape = list(tensor.shape) if tensor.dim() else [1]
    shape[0] = shape[0] * (runtime.size() if runtime.is_initialized() else 1)
    return tensor.new_empty(shape)


def allreduce(tensor: torch.Tensor, average: bool = True, name: Optional[str] = None) -> torch.Tensor:
    """Out-of-place convenience wrapper of ``torch.ops.mxr.allreduce_``."""
    out = tensor.clone()
    torch.ops.mxr.allreduce_(out, average)
    return out
