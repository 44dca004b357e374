#!/usr/bin/env python
"""Halo-staged 3x3 kernel (conv_halo.hip) vs the pipelined implicit GEMM (conv_pipe.hip) on every
3x3 / stride-1 shape of RetinaNet-R50-FPN at 800x1333, batch 16: forward and data gradient."""
import argparse
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from batchai_retinanet_horovod_coco_amd.ops import native as N  # noqa: E402

B = 16
PYR = [(100, 167), (50, 84), (25, 42), (13, 21), (7, 11)]


def timeit(fn, iters=10, warm=3):
    for _ in range(warm):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pipe", default="16,5")
    ap.add_argument("--halo", default="1,7,8,2,9,10,3,5")
    ap.add_argument("--hx32", default="0,1,2,3")
    ap.add_argument("--only", default="")
    ap.add_argument("--zero-x", action="store_true", help="all-zero input (operand values change the MFMA power, hence the clock)")
    args = ap.parse_args()
    N.load(required=True)
    dev = torch.device("cuda")
    cases = [("head_256_256", PYR, 256, 256), ("head_256_720", PYR, 256, 720), ("head_dgrad_768_256", PYR, 768, 256),
             ("head_256_512", PYR, 256, 512),
             ("fpn_P3", [(100, 167)], 256, 256), ("s2_3x3_64", [(200, 334)], 64, 64),
             ("s3_3x3_128", [(100, 167)], 128, 128), ("s4_3x3_256", [(50, 84)], 256, 256),
             ("s5_3x3_512", [(25, 42)], 512, 512)]
    for name, shapes, cin, cout in cases:
        if args.only and args.only not in name:
            continue
        P = sum(h * w for h, w in shapes)
        x = torch.randn(B, P, cin, device=dev).bfloat16()
        if args.zero_x:
            x.zero_()
        w = (torch.randn(cout, 3, 3, cin, device=dev) * 0.05).bfloat16()
        b = torch.randn(cout, device=dev)
        y = torch.empty(B, P, cout, device=dev, dtype=torch.bfloat16)
        g = N.geom_pyramid(B, shapes, cin, cout)
        gf = 2.0 * B * P * cout * 9 * cin / 1e9
        res = {}
        ref = None
        for v in [int(t) for t in args.pipe.split(",") if t] + ["halo%s" % t for t in args.halo.split(",") if t] + \
                ["hx32_%s" % t for t in args.hx32.split(",") if t]:
            try:
                ms = timeit(lambda: N.launch_fwd(x, w, b, None, y, g, True, variant=v))
                if ref is None:
                    ref = y.float().clone()
                    err = 0.0
                else:
                    err = ((y.float() - ref).abs().max() / (ref.abs().max() + 1e-3)).item()
                res[str(v)] = "%.3f ms %4.0f TF%s" % (ms, gf / ms, "" if err < 2e-2 else " MISMATCH %.3g" % err)
            except Exception as exc:  # noqa: BLE001
                res[str(v)] = "err %s" % str(exc)[:40]
        print("%-20s %7.1f GF | " % (name, gf) + " | ".join("%s: %s" % kv for kv in res.items()), flush=True)


if __name__ == "__main__":
    main()
