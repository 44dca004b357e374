#!/usr/bin/env python
"""Host-side (Python) cost of the bench step: cProfile over 3 steady-state steps of the bench config
(R50, 16 x 800 x 1333, bf16), with the autograd engine kept on the calling thread so the backward's
Python (custom Function backward, tuner dispatch, side-stream bookkeeping, ctypes launches) is seen.

usage: host_profile.py [N_LINES]"""
import cProfile
import os
import pstats
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from batchai_retinanet_horovod_coco_amd import models
    from batchai_retinanet_horovod_coco_amd.data.synthetic import SyntheticBatches
    from batchai_retinanet_horovod_coco_amd.models.calibrate import calibrate_from_synthetic
    from batchai_retinanet_horovod_coco_amd.train.engine import Trainer
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 45
    dev = torch.device("cuda", 0)
    torch.manual_seed(1234)
    model = models.backbone("resnet50").retinanet(80)
    calibrate_from_synthetic(model, torch.device("cpu"), batch=1, height=384, width=640)
    tr = Trainer(model, lr=1e-5, clipnorm=0.001, compute_dtype=torch.bfloat16, clip_mode="global", device=dev)
    data = SyntheticBatches(16, 800, 1333, pool=2, device=dev, seed=100, dtype=torch.bfloat16)

    def step():
        b = next(data)
        return tr.train_on_batch(b["images"], b["gt"], b["gt_count"], b["image_hw"])

    torch.autograd.set_multithreading_enabled(False)
    for _ in range(4):
        step()
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(3):
        step()
    pr.disable()
    torch.cuda.synchronize()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(n)
    st.sort_stats("cumulative").print_stats(n)


if __name__ == "__main__":
    main()
