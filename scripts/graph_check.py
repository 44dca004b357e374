"""Eager vs HIP-graph training-step losses (lr = 0) for R50 under different conv algorithm pins."""
import copy
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from batchai_retinanet_horovod_coco_amd import models  # noqa: E402
from batchai_retinanet_horovod_coco_amd.data.synthetic import make_batch  # noqa: E402
from batchai_retinanet_horovod_coco_amd.ops import native  # noqa: E402
from batchai_retinanet_horovod_coco_amd.train.engine import Trainer  # noqa: E402


def run(base, batches, graphed, H, W):
    native.set_grad_sinks(None)
    native.set_compute_weights(None)
    tr = Trainer(copy.deepcopy(base), lr=0.0, clipnorm=0.001, compute_dtype=torch.bfloat16,
                 device=torch.device("cuda"), clip_mode="global")
    b = batches[0]
    if graphed:
        step = tr.graph_step(b["images"], b["gt"], b["gt_count"], b["image_hw"], warmup=2)
    else:
        step = tr.train_on_batch
        for _ in range(2):
            step(b["images"], b["gt"], b["gt_count"], b["image_hw"])
    return [float(step(b["images"], b["gt"], b["gt_count"], b["image_hw"])["loss"]) for b in batches]


def main():
    native.load(required=True)
    H, W = int(os.environ.get("GC_H", "320")), int(os.environ.get("GC_W", "448"))
    torch.manual_seed(0)
    base = models.backbone(os.environ.get("GC_BACKBONE", "resnet50")).retinanet(80)
    g = torch.Generator(device="cuda").manual_seed(0)
    batches = [make_batch(4, H, W, 80, 8, "cuda", g) for _ in range(3)]
    for force in ("", "hip", "miopen"):
        if force:
            os.environ["MXR_CONV_FORCE"] = force
        else:
            os.environ.pop("MXR_CONV_FORCE", None)
        e = run(base, batches, False, H, W)
        gr = run(base, batches, True, H, W)
        print("force=%-7s eager %s graph %s" % (force or "-", ["%.4f" % v for v in e], ["%.4f" % v for v in gr]),
              flush=True)


if __name__ == "__main__":
    main()
