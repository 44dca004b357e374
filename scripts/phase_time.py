#!/usr/bin/env python
"""Per-phase host vs GPU time of the bench training step (R50, 16 x 800 x 1333): for each phase (zero_grad +
targets, forward, losses + backward, optimizer) the host time to issue it and the GPU time between
events recorded at the phase boundaries.  A phase whose GPU time is far below the step's share while the
host lags shows where launch overhead / host syncs leave the GPU idle."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from batchai_retinanet_horovod_coco_amd import models
    from batchai_retinanet_horovod_coco_amd.data.synthetic import SyntheticBatches
    from batchai_retinanet_horovod_coco_amd.models.calibrate import calibrate_from_synthetic
    from batchai_retinanet_horovod_coco_amd.train.engine import Trainer
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    dev = torch.device("cuda", 0)
    torch.manual_seed(1234)
    model = models.backbone("resnet50").retinanet(80)
    calibrate_from_synthetic(model, torch.device("cpu"), batch=1, height=384, width=640)
    tr = Trainer(model, lr=1e-5, clipnorm=0.001, compute_dtype=torch.bfloat16, clip_mode="local", device=dev)
    data = SyntheticBatches(16, 800, 1333, pool=2, device=dev, seed=100, dtype=torch.bfloat16)
    for _ in range(4):
        b = next(data)
        tr.train_on_batch(b["images"], b["gt"], b["gt_count"], b["image_hw"])
    torch.cuda.synchronize()
    names = ("targets", "forward", "loss+backward", "optimizer")
    host = [[] for _ in names]
    evs = []
    for _ in range(steps):
        b = next(data)
        e = [torch.cuda.Event(enable_timing=True) for _ in range(len(names) + 1)]
        t = [time.perf_counter()]
        e[0].record()
        tr.model.train()
        tr.optimizer.zero_grad()
        state, label, reg_t, npos = tr.compute_targets(b["images"], b["gt"], b["gt_count"], b["image_hw"])
        t.append(time.perf_counter()); e[1].record()
        out = tr.model(b["images"].to(tr.compute_dtype))
        t.append(time.perf_counter()); e[2].record()
        tr._losses_backward(out, reg_t, state, label, npos)
        t.append(time.perf_counter()); e[3].record()
        tr.optimizer.step()
        t.append(time.perf_counter()); e[4].record()
        for i in range(len(names)):
            host[i].append((t[i + 1] - t[i]) * 1e3)
        evs.append(e)
    torch.cuda.synchronize()
    gpu = [[ev[i].elapsed_time(ev[i + 1]) for ev in evs] for i in range(len(names))]
    step_gpu = [ev[0].elapsed_time(ev[-1]) for ev in evs]
    gap = [evs[k][-1].elapsed_time(evs[k + 1][0]) for k in range(len(evs) - 1)]
    med = lambda v: sorted(v)[len(v) // 2]   # noqa: E731
    for i, n in enumerate(names):
        print("%-14s host %7.2f ms   gpu %7.2f ms" % (n, med(host[i]), med(gpu[i])))
    print("step: gpu %.2f ms (events), host issue %.2f ms, gpu gap between steps %.3f ms"
          % (med(step_gpu), sum(med(h) for h in host), med(gap) if gap else 0.0), flush=True)


if __name__ == "__main__":
    main()
