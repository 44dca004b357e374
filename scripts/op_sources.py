#!/usr/bin/env python
"""Where the step's remaining torch (at::native) kernels come from: profiles one training step of the
bench config (R50, 16 x 800 x 1333, bf16) with CPU stacks and prints, for each aten op that launched a
GPU kernel outside our extension (copy_, fill_, cat, add_, ...), the count per step and the innermost
frame of our package that issued it."""
import collections
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

OPS = ("aten::copy_", "aten::fill_", "aten::zero_", "aten::cat", "aten::add_", "aten::add", "aten::mul",
       "aten::mul_", "aten::sum", "aten::index", "aten::nonzero", "aten::sub", "aten::div", "aten::where",
       "aten::clamp", "aten::_foreach_", "aten::constant_pad_nd", "aten::flip", "aten::scatter", "aten::gather")


def main():
    from batchai_retinanet_horovod_coco_amd import models
    from batchai_retinanet_horovod_coco_amd.data.synthetic import SyntheticBatches
    from batchai_retinanet_horovod_coco_amd.models.calibrate import calibrate_from_synthetic
    from batchai_retinanet_horovod_coco_amd.train.engine import Trainer
    dev = torch.device("cuda", 0)
    torch.manual_seed(1234)
    model = models.backbone("resnet50").retinanet(80)
    calibrate_from_synthetic(model, torch.device("cpu"), batch=1, height=384, width=640)
    tr = Trainer(model, lr=1e-5, clipnorm=0.001, compute_dtype=torch.bfloat16, clip_mode="global", device=dev)
    data = SyntheticBatches(16, 800, 1333, pool=2, device=dev, seed=100, dtype=torch.bfloat16)
    for _ in range(4):
        b = next(data)
        tr.train_on_batch(b["images"], b["gt"], b["gt_count"], b["image_hw"])
    torch.cuda.synchronize()
    steps = 2
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU], with_stack=True, record_shapes=True, acc_events=True) as prof:
        for _ in range(steps):
            b = next(data)
            tr.train_on_batch(b["images"], b["gt"], b["gt_count"], b["image_hw"])
        torch.cuda.synchronize()
    cnt = collections.Counter()
    def has_op(ev):
        if any(ev.name.startswith(o) for o in OPS):
            return True
        return any(has_op(c) for c in ev.cpu_children)

    for ev in prof.events():
        # top-level aten ops (a contiguous / to / clone whose copy_ launches the kernel) with their shapes
        if not ev.name.startswith("aten::") or not has_op(ev):
            continue
        if ev.cpu_parent is not None and ev.cpu_parent.name.startswith("aten::"):
            continue
        frame = "?"
        for fr in ev.stack or []:
            if "batchai_retinanet_horovod_coco_amd" in fr or "bench" in fr:
                frame = fr.split("batchai_retinanet_horovod_coco_amd/")[-1]
                break
        par = ev.cpu_parent.name if ev.cpu_parent is not None else "-"
        cnt[(ev.name, str(ev.input_shapes)[:90], par[:40], frame)] += 1
    for (name, shapes, par, frame), n in sorted(cnt.items(), key=lambda kv: -kv[1]):
        print("%5.1f/step  %-22s %-40s %s  %s" % (n / steps, name, par, shapes, frame))


if __name__ == "__main__":
    main()
