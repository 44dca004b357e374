"""Isolated timing of the fused focal loss + gradient kernel at the bench shape (16 images x 200,700 anchors x
80 classes, bf16 logits written into the packed head's padded gradient rows):  python scripts/bench_focal.py
Prints ms per call and the HBM rate of its one read + one write of the logits."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from batchai_retinanet_horovod_coco_amd.ops import native as N  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    B, A, C = 16, 200700, 80
    for scale, bias, tag in ((0.3, -4.6, "prior-init logits"), (6.0, -8.0, "spread logits, some beyond +-16.1")):
        logits = (torch.randn(B, A, C, device=dev) * scale + bias).bfloat16()
        state = torch.randint(-1, 2, (B, A), device=dev).to(torch.int8)
        state[state == 1] = torch.where(torch.rand_like(state[state == 1].float()) < 0.01, 1, 0).to(torch.int8)
        label = torch.randint(0, C, (B, A), device=dev).to(torch.int32)
        out = torch.zeros(B * A // 9, 768, dtype=torch.bfloat16, device=dev)
        for _ in range(3):
            N.focal_fwd_bwd(logits, state, label, grad_out=out, group=9)
        torch.cuda.synchronize()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        n = 20
        ev[0].record()
        for _ in range(n):
            N.focal_fwd_bwd(logits, state, label, grad_out=out, group=9)
        ev[1].record()
        torch.cuda.synchronize()
        ms = ev[0].elapsed_time(ev[1]) / n
        gb = 2 * logits.numel() * 2 / 1e9
        print("focal %-36s %.3f ms/call  %.2f TB/s" % (tag, ms, gb / ms))


if __name__ == "__main__":
    main()
