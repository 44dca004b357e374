"""``check_runtime``: the analogue of keras-retinanet's ``check_keras_version`` (train.py:52,393).

Verifies the PyTorch version and, when a GPU is visible, that it is a gfx950 (MI355X) device and
that the in-tree HIP kernel library loads (a missing build fails loudly instead of silently
falling back to PyTorch ops).
"""
from __future__ import annotations

import os
import warnings

MIN_TORCH = (2, 1)


def check_runtime(require_kernels: bool = None) -> dict:
    import torch
    ver = tuple(int(x) for x in torch.__version__.split("+")[0].split(".")[:2])
    if ver < MIN_TORCH:
        raise RuntimeError("PyTorch {} is too old; need >= {}.{}".format(torch.__version__, *MIN_TORCH))
    info = {"torch": torch.__version__, "hip": getattr(torch.version, "hip", None), "gpu": None, "kernels": False}
    if torch.cuda.is_available():
        props = torch.cuda.get_device_properties(torch.cuda.current_device())
        arch = getattr(props, "gcnArchName", "")
        info["gpu"] = arch
        if "gfx950" not in arch:
            warnings.warn("GPU arch {} is not gfx950 (MI355X); kernels are compiled for gfx950 only".format(arch))
        from ..ops import native
        req = require_kernels if require_kernels is not None else os.environ.get("MXR_REQUIRE_KERNELS", "1") == "1"
        info["kernels"] = native.load(required=req)
    return info
