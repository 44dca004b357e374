"""Microbench of the 64-channel 3x3 wgrad kernel at the res2 shape (B=16, 200x334) -- PMC target."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from batchai_retinanet_horovod_coco_amd.ops import native as N  # noqa: E402
from batchai_retinanet_horovod_coco_amd.ops import native_conv as NC  # noqa: E402

N.load(required=True)
dev = torch.device("cuda", 0)
x = torch.randn(16, 200, 334, 64, device=dev).to(torch.bfloat16)
dy = torch.randn(16, 200, 334, 64, device=dev).to(torch.bfloat16)
for _ in range(3):
    NC.wgrad3x3_c64(x, dy)
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(10):
    NC.wgrad3x3_c64(x, dy)
torch.cuda.synchronize()
print("w64 %.3f ms" % ((time.perf_counter() - t) / 10 * 1e3))
