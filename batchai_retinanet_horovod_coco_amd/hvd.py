"""``from batchai_retinanet_horovod_coco_amd import hvd`` -- Horovod-style API (see ``parallel``).

Mirrors the names the reference uses (``hvd.init``, ``hvd.rank``, ``hvd.local_rank``,
``hvd.DistributedOptimizer``, ``hvd.callbacks.BroadcastGlobalVariablesCallback``; reference
``/root/reference/train.py:20-21,71,103,111``).
"""
from .parallel import *  # noqa: F401,F403
from .parallel import callbacks  # noqa: F401
