"""Gradient parity diagnostics: torch fp32 vs torch bf16 vs HIP bf16 (same weights, same batch)."""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from batchai_retinanet_horovod_coco_amd import models  # noqa: E402
from batchai_retinanet_horovod_coco_amd.data.synthetic import make_batch  # noqa: E402
from batchai_retinanet_horovod_coco_amd.models.calibrate import calibrate_from_synthetic  # noqa: E402
from batchai_retinanet_horovod_coco_amd.ops import conv as conv_ops  # noqa: E402
from batchai_retinanet_horovod_coco_amd.ops import native  # noqa: E402
from batchai_retinanet_horovod_coco_amd.train.engine import Trainer  # noqa: E402


def grads(state, cuda, mode, batch, backbone):
    env = {}
    if mode == "torch32" or mode == "torch16":
        native.disable()
        conv_ops.set_conv_backend("torch")
    else:
        native.enable()
        conv_ops.set_conv_backend("auto")
        if mode == "hip_miopen":
            os.environ["MXR_CONV_FORCE"] = "miopen"
        if mode == "hip_nosink":
            os.environ["MXR_NO_GRAD_SINKS"] = "1"
    dt = torch.float32 if mode == "torch32" else torch.bfloat16
    try:
        model = models.backbone(backbone).retinanet(80)
        model.load_state_dict(state)
        tr = Trainer(model, compute_dtype=dt, clip_mode="global", device=cuda)
        tr.optimizer.zero_grad()
        b = {k: v.to(cuda) for k, v in batch.items()}
        reg, cls = tr.forward_backward(b["images"], b["gt"], b["gt_count"], b["image_hw"])
        torch.cuda.synchronize()
        g = {s.name: tr.flat.grad[s.offset:s.offset + s.numel].double().clone() for s in tr.flat.segments}
        tr.optimizer.remove_hooks()
        return float(reg), float(cls), g
    finally:
        native.set_grad_sinks(None)
        native.set_compute_weights(None)
        native.enable()
        conv_ops.set_conv_backend("auto")
        os.environ.pop("MXR_CONV_FORCE", None)
        os.environ.pop("MXR_NO_GRAD_SINKS", None)


def cos(a, b):
    na, nb = a.norm().item(), b.norm().item()
    return float(torch.dot(a, b) / (na * nb)) if na > 0 and nb > 0 else 1.0


def main():
    cuda = torch.device("cuda", 0)
    backbone = sys.argv[1] if len(sys.argv) > 1 else "resnet50"
    torch.manual_seed(0)
    model = models.backbone(backbone).retinanet(80)
    calibrate_from_synthetic(model, torch.device("cpu"), batch=1, height=256, width=320)
    state = {k: v.clone() for k, v in model.state_dict().items()}
    batch = make_batch(2, 384, 640, generator=torch.Generator().manual_seed(7))
    modes = ["torch32", "torch32b", "torch16", "hip", "hip_nosink", "hip_miopen"]
    res = {}
    for m in modes:
        mm = "torch32" if m == "torch32b" else m
        res[m] = grads(state, cuda, mm, batch, backbone)
        print("%-10s reg %.6f cls %.6f" % (m, res[m][0], res[m][1]), flush=True)
    names = list(res["torch32"][2].keys())
    ref = res["torch32"][2]
    print("%-48s" % "param" + "".join("%11s" % m for m in modes[1:]))
    for n in names[:30] + names[-30:]:
        print("%-48s" % n[:48] + "".join("%11.5f" % cos(ref[n], res[m][2][n]) for m in modes[1:]))


if __name__ == "__main__":
    main()
