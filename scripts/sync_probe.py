#!/usr/bin/env python
"""Why does the GPU wait for the host at the start of each bench step?  Runs the bench config (R50,
16 x 800 x 1333, bf16) and reports (1) torch-level synchronising calls (``set_sync_debug_mode``) with the
frame that issued them, (2) device allocations / allocator retries during steady-state steps, and (3) per
step how far ahead of the GPU the host is when it finishes issuing the step (negative = the GPU had
already drained the previous step, i.e. the host was the bottleneck at that point)."""
import os
import sys
import time
import traceback
import warnings

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


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

    def step():
        b = next(data)
        return tr.train_on_batch(b["images"], b["gt"], b["gt_count"], b["image_hw"])

    for _ in range(4):
        step()
    torch.cuda.synchronize()

    # (1) synchronising torch calls
    seen = {}
    orig = warnings.showwarning

    def show(message, category, filename, lineno, file=None, line=None):
        stack = "".join(traceback.format_stack(limit=8)[:-1])
        key = str(message)[:80] + stack[-300:]
        seen[key] = seen.get(key, 0) + 1

    warnings.showwarning = show
    torch.cuda.set_sync_debug_mode("warn")
    for _ in range(2):
        step()
    torch.cuda.set_sync_debug_mode(0)
    warnings.showwarning = orig
    torch.cuda.synchronize()
    print("== synchronising calls in 2 steps: %d distinct" % len(seen))
    for k, n in seen.items():
        print("-- x%d\n%s" % (n, k))

    # (2) allocator activity in steady state
    s0 = torch.cuda.memory_stats(dev)
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    s1 = torch.cuda.memory_stats(dev)
    for k in ("num_alloc_retries", "num_device_alloc", "num_device_free", "num_sync_all_streams"):
        if k in s1:
            print("%-22s +%d over 3 steps" % (k, s1[k] - s0.get(k, 0)))

    # (3) host lead per step
    evs = []
    for k in range(8):
        t0 = time.perf_counter()
        step()
        e = torch.cuda.Event()
        e.record()
        t1 = time.perf_counter()
        prev_done = evs[-1].query() if evs else None
        evs.append(e)
        print("step %d: host issue %.2f ms, previous step already finished on the GPU: %s"
              % (k, (t1 - t0) * 1e3, prev_done), flush=True)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
