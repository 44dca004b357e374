"""batchai_retinanet_horovod_coco_amd -- an MI355X-native RetinaNet + Horovod-style
data-parallel training framework (capabilities of msalvaris/batchai_retinanet_horovod_coco).

Subpackages: models, ops, parallel (hvd API), data, train, io, eval, utils, bin.
"""
import torch  # noqa: F401  (import first: binds the HIP runtime our kernels link against)

__version__ = "0.1.0"
