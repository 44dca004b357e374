"""Microbench: halo-staged wgrad vs the pipelined implicit-GEMM wgrad (hip3 / hip6 / hip8) at B=16."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from batchai_retinanet_horovod_coco_amd.ops import native as N  # noqa: E402
from batchai_retinanet_horovod_coco_amd.ops import native_conv as NC  # noqa: E402

PYR = [(100, 167), (50, 84), (25, 42), (13, 21), (7, 11)]
CASES = [("head_256", PYR, 256, 256), ("cls_final_720", PYR, 256, 720), ("fpn_P3", [(100, 167)], 256, 256),
         ("s4_256", [(50, 84)], 256, 256), ("s3_128", [(100, 167)], 128, 128), ("s5_512", [(25, 42)], 512, 512)]


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e3


def main():
    N.load(required=True)
    dev = torch.device("cuda", 0)
    B = 16
    for name, shapes, cin, cout in CASES:
        P = sum(h * w for h, w in shapes)
        x = torch.randn(B, P, cin, device=dev).to(torch.bfloat16)
        ld = cout if cout % 8 == 0 else cout + 8 - cout % 8
        dy = torch.randn(B, P, ld, device=dev).to(torch.bfloat16)
        g = NC.geom_pyramid(B, shapes, cin, cout) if len(shapes) > 1 else \
            NC.geom_single(B, shapes[0][0], shapes[0][1], shapes[0][0], shapes[0][1], 3, 1, (1, 1, 1, 1), cin, cout)
        gf = 2.0 * B * P * 9 * cin * cout / 1e9
        out = []
        for splits in (None,):
            t = timeit(lambda: NC.halo_wgrad(x, dy, g, splits=splits))
            out.append("whalo %.3f ms %4.0f TF/s" % (t, gf / t))
        for v in (3, 6, 8):
            try:
                t = timeit(lambda: NC.conv_wgrad(x, dy, g, None, variant=v))
                out.append("hip%d %.3f" % (v, t))
            except RuntimeError as e:
                out.append("hip%d n/a" % v)
        print("%-14s %6.0f GF | %s" % (name, gf, " | ".join(out)))


if __name__ == "__main__":
    main()
