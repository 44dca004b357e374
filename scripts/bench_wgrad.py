#!/usr/bin/env python
"""Weight-gradient microbenchmark at the production shapes (R50-FPN, 16 x 800 x 1333): the head pyramid
(256 -> 256 / 720 / 64-padded) and the FPN / backbone 3x3 levels: the phase-pipelined conv_wgrad_p8 (hip23 /
hip24 / hip25) and the halo wgrad ("whalo").  Isolated kernel time (events, median of
repeats) and TF/s.

usage: bench_wgrad.py [--reps 20] [--only pyr|single] [--data randn|zeros|small|sparse]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from batchai_retinanet_horovod_coco_amd.ops import native as N  # noqa: E402


def timeit(fn, reps):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    ts.sort()
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--only", default="")
    ap.add_argument("--data", default="randn", help="randn | zeros | small (x0.01) | sparse (90 %% zeros): "
                    "operand values change the MFMA power draw, hence the clock")
    a = ap.parse_args()
    N.load(required=True)
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    pyr = [(100, 167), (50, 84), (25, 42), (13, 21), (7, 11)]
    cases = []
    if a.only in ("", "pyr"):
        for cout in (256, 720, 64):
            cases.append(("pyr", 16, pyr, 256, cout))
    if a.only in ("", "single"):
        for (h, w, c) in ((100, 167, 256), (50, 84, 256), (100, 167, 128), (50, 84, 256), (25, 42, 512)):
            cases.append(("single", 16, [(h, w)], c, c))
    for kind, n, shapes, cin, cout in cases:
        P = sum(h * w for h, w in shapes)
        ldy = (cout + 63) // 64 * 64 if kind == "pyr" else cout
        x = torch.randn(n, P, cin, device=dev).bfloat16()
        dy = (torch.randn(n, P, ldy, device=dev) * 0.1).bfloat16()
        if a.data == "zeros":
            x.zero_()
            dy.zero_()
        elif a.data == "small":
            x.mul_(0.01)
            dy.mul_(0.01)
        elif a.data == "sparse":
            x.mul_((torch.rand_like(x, dtype=torch.float32) < 0.1).bfloat16())
            dy.mul_((torch.rand_like(dy, dtype=torch.float32) < 0.1).bfloat16())
        g = N.geom_pyramid(n, shapes, cin, cout) if kind == "pyr" else \
            N.geom_single(n, shapes[0][0], shapes[0][1], shapes[0][0], shapes[0][1], 3, 1, (1, 1, 1, 1), cin, cout)
        flop = 2.0 * n * P * cout * 9 * cin
        out = torch.zeros(cout, 3, 3, cin, device=dev)
        res = {}
        res["hip23"] = timeit(lambda: N.conv_wgrad(x, dy, g, None, out=out, accumulate=True, variant=23), a.reps)
        res["hip25"] = timeit(lambda: N.conv_wgrad(x, dy, g, None, out=out, accumulate=True, variant=25), a.reps)
        res["hip24"] = timeit(lambda: N.conv_wgrad(x, dy, g, None, out=out, accumulate=True, variant=24), a.reps)
        if N.whalo_covers(g):
            res["whalo"] = timeit(lambda: N.halo_wgrad(x, dy, g, out=out, accumulate=True), a.reps)
        desc = "%s %s %d->%d" % (kind, shapes[0], cin, cout)
        print(desc + "  " + "  ".join("%s %.3f ms %.0f TF/s" % (k, v, flop / v / 1e9) for k, v in res.items()),
              flush=True)


if __name__ == "__main__":
    main()
