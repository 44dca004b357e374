"""Run one conv kernel on a head-sized shape repeatedly (target for rocprofv3 --pmc counter runs)."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from batchai_retinanet_horovod_coco_amd.ops import native as N  # noqa: E402

PYR = [(100, 167), (50, 84), (25, 42), (13, 21), (7, 11)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--op", choices=["fwd", "wgrad"], default="fwd")
    ap.add_argument("--variant", type=int, default=2)
    ap.add_argument("--cout", type=int, default=256)
    ap.add_argument("--iters", type=int, default=5)
    a = ap.parse_args()
    N.load(required=True)
    dev = torch.device("cuda")
    B = 16
    xs = [torch.randn(B, h, w, 256, device=dev).bfloat16() for h, w in PYR]
    packed, sh = N.pyramid_pack(xs)
    w = (torch.randn(a.cout, 3, 3, 256, device=dev) * 0.05).bfloat16()
    if a.op == "fwd":
        g = N.geom_pyramid(B, sh, 256, a.cout)
        y = torch.empty(B, packed.shape[1], a.cout, device=dev, dtype=torch.bfloat16)
        for _ in range(a.iters):
            N.launch_fwd(packed, w, None, None, y, g, False, variant=a.variant)
    else:
        dy = torch.randn(B, packed.shape[1], a.cout, device=dev).bfloat16()
        g = N.geom_pyramid(B, sh, 256, a.cout)
        for _ in range(a.iters):
            N.conv_wgrad(packed, dy, g, None, variant=a.variant)
    torch.cuda.synchronize()
    print("done")


if __name__ == "__main__":
    main()
