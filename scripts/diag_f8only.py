#!/usr/bin/env python
"""Diagnostic: an fp8 training step with fp8-only tower outputs (ops.fp8.pyramid_forward f8_only) vs the same step
with bf16 tower outputs -- losses and the per-parameter relative gradient difference of the head layers (the step is
bitwise reproducible, so any non-zero difference is real).  Kernels pinned to the hx8 forms as in the tests."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from batchai_retinanet_horovod_coco_amd import models  # noqa: E402
from batchai_retinanet_horovod_coco_amd.data.synthetic import make_batch  # noqa: E402
from batchai_retinanet_horovod_coco_amd.models.calibrate import calibrate_from_synthetic  # noqa: E402
from batchai_retinanet_horovod_coco_amd.ops import fp8 as F8  # noqa: E402
from batchai_retinanet_horovod_coco_amd.ops.conv_tuner import TUNER  # noqa: E402
from batchai_retinanet_horovod_coco_amd.ops.side_stream import SIDE  # noqa: E402
from batchai_retinanet_horovod_coco_amd.train.engine import Trainer  # noqa: E402


def main():
    cuda = torch.device("cuda", 0)
    real = TUNER.winner
    TUNER.winner = lambda k: (("f8_20" if k.startswith("pfwd|") else "f8d_22")
                              if k.endswith("|f8") and k.startswith(("pfwd|", "pdgrad|")) else real(k))
    passes = int(os.environ.get("PASSES", "3"))

    def run(on):
        F8.F8_ONLY_TOWERS = on
        F8.set_enabled(True)
        F8.reset_state()
        torch.manual_seed(0)
        model = models.backbone("resnet50").retinanet(80)
        calibrate_from_synthetic(model, torch.device("cpu"), batch=1, height=256, width=320)
        tr = Trainer(model, compute_dtype=torch.bfloat16, clip_mode="global", device=cuda)
        b = make_batch(2, 256, 320, device=cuda, generator=torch.Generator(device=cuda).manual_seed(3))
        losses = []
        for _ in range(passes):
            tr.flat.zero_grad()
            loss = tr.forward_backward(b["images"], b["gt"], b["gt_count"], b["image_hw"])
            SIDE.join()
            torch.cuda.synchronize()
            losses.append([float(v) for v in loss])
        g = {n: p.grad.detach().clone() for n, p in model.named_parameters()
             if p.grad is not None and ("classification" in n or "regression" in n)}
        F8.set_enabled(False)
        return losses, g
    off, on = run(False), run(True)
    print("losses off", off[0])
    print("losses on ", on[0])
    for n in off[1]:
        a, b = on[1][n], off[1][n]
        print("%-40s rel %.3e  |off| %.3e  |on| %.3e" % (n, ((a - b).norm() / b.norm().clamp_min(1e-30)).item(),
                                                        b.norm().item(), a.norm().item()))


if __name__ == "__main__":
    main()
