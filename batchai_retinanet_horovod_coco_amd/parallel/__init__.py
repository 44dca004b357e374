"""Horovod-compatible data-parallel API over torch.distributed (RCCL over xGMI / gloo).

``from batchai_retinanet_horovod_coco_amd import hvd`` gives the same names the reference
uses (``/root/reference/train.py:20-21,71,103,111-112,119``): ``init``, ``rank``, ``size``,
``local_rank``, ``DistributedOptimizer``, ``callbacks.BroadcastGlobalVariablesCallback`` ...
"""
from .runtime import (init, shutdown, is_initialized, rank, size, local_rank, local_size,  # noqa: F401
                      cross_rank, cross_size, device, distributed, barrier, mpi_threads_supported)
from .collectives import (Compression, allreduce, allreduce_, allreduce_async, allreduce_async_,  # noqa: F401
                          synchronize, poll, allgather, broadcast, broadcast_, broadcast_object,
                          broadcast_parameters, broadcast_optimizer_state, SignatureMismatch,
                          set_signature_check)
from .distributed_optimizer import DistributedOptimizer  # noqa: F401
from . import ops  # noqa: F401,E402  (registers torch.ops.mxr.allreduce_ / broadcast_ / allgather)
