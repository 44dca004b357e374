#!/usr/bin/env python
"""Host cost of issuing one training step: after warm-up, a spin kernel holds the GPU while the host
issues N steps, so the host time per step is measured without waiting on the GPU; then the GPU-bound
time per step.  A host time near (or above) the step time means launch overhead shows up as GPU idle.

    python scripts/host_time.py [N] [--batch-size B] [--height H] [--width W]
"""
import argparse
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
    p = argparse.ArgumentParser()
    # (a handful: with ~1000 launches per step, more steps than the HIP launch queue holds make the host wait on
    # the GPU and the 'issue' time meaningless)
    p.add_argument("n", type=int, nargs="?", default=3)
    p.add_argument("--batch-size", type=int, default=16)
    p.add_argument("--height", type=int, default=800)
    p.add_argument("--width", type=int, default=1333)
    a = p.parse_args()
    n = a.n
    dev = torch.device("cuda", 0)
    torch.manual_seed(1234)
    model = models.backbone("resnet50").retinanet(80)
    calibrate_from_synthetic(model, torch.device("cpu"), batch=1, height=384, width=640)
    tr = Trainer(model, lr=1e-5, clipnorm=0.001, compute_dtype=torch.bfloat16, clip_mode="global", device=dev)
    data = SyntheticBatches(a.batch_size, a.height, a.width, pool=2, device=dev, seed=100, dtype=torch.bfloat16)

    def step():
        b = next(data)
        return tr.train_on_batch(b["images"], b["gt"], b["gt_count"], b["image_hw"])

    for _ in range(4):
        step()
    torch.cuda.synchronize()
    import gc
    gc.collect()
    gc.freeze()
    import cProfile
    import pstats
    torch.cuda._sleep(int(3e9))             # ~1.3 s of GPU spin: the host issues freely meanwhile
    prof = cProfile.Profile() if os.environ.get("HOST_PROFILE") == "1" else None
    t0 = time.perf_counter()
    if prof:
        prof.enable()
    for _ in range(n):
        step()
    if prof:
        prof.disable()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    t3 = time.perf_counter()
    for _ in range(n):
        step()
    torch.cuda.synchronize()
    t4 = time.perf_counter()
    print("B=%d %dx%d  host issue %.2f ms/step   (GPU spin covered %.0f ms)   steady %.2f ms/step"
          % (a.batch_size, a.height, a.width, (t1 - t0) / n * 1e3, (t2 - t0) * 1e3, (t4 - t3) / n * 1e3), flush=True)
    if prof:
        pstats.Stats(prof).sort_stats("tottime").print_stats(25)


if __name__ == "__main__":
    main()
