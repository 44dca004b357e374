#!/usr/bin/env python
"""The persistent 1x1 kernel (conv1x1_pers.hip, tuner name "c1p") against every other HIP candidate of the
R50-FPN 1x1 / stride-1 layers at 800 x 1333, batch 16, in the epilogue forms the training step uses (forward:
bias + relu, bias + residual + relu + bitmask write; data gradient: bf16 mask, bitmask + accumulate).
Isolated kernel time (events, median of repeats), TF/s and TB/s of the minimal HBM traffic.

usage: bench_c1p.py [--reps 20] [--only NAME]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from batchai_retinanet_horovod_coco_amd.ops import native_conv as NC  # noqa: E402
from batchai_retinanet_horovod_coco_amd.ops.conv_launch import BitMask, fwd_candidates  # noqa: E402

B = 16
# name, H, W, cin, cout, form ("f" forward bias+relu, "fr" + residual + bits, "d" dgrad + mask, "da" dgrad +
# bits + accumulate; dgrad rows: cin / cout of the FORWARD conv)
CASES = [
    ("s2 64->256 fr", 200, 334, 64, 256, "fr"), ("s2 256->64 f", 200, 334, 256, 64, "f"),
    ("s3 128->512 fr", 100, 167, 128, 512, "fr"), ("s3 512->128 f", 100, 167, 512, 128, "f"),
    ("s4 256->1024 fr", 50, 84, 256, 1024, "fr"), ("s4 1024->256 f", 50, 84, 1024, 256, "f"),
    ("s5 512->2048 fr", 25, 42, 512, 2048, "fr"), ("s5 2048->512 f", 25, 42, 2048, 512, "f"),
    ("fpn C3 512->256", 100, 167, 512, 256, "f0"),
    ("d s3 128<-512 m", 100, 167, 128, 512, "d"), ("d s3 512<-128 mb|a", 100, 167, 512, 128, "da"),
    ("d s4 256<-1024 m", 50, 84, 256, 1024, "d"), ("d s4 1024<-256 mb|a", 50, 84, 1024, 256, "da"),
    ("d s5 512<-2048 m", 25, 42, 512, 2048, "d"), ("d s5 2048<-512 mb|a", 25, 42, 2048, 512, "da"),
    ("d s2 64<-256 m", 200, 334, 64, 256, "d"),
]


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
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    for name, H, W, cin, cout, form in CASES:
        if a.only and a.only not in name:
            continue
        M = B * H * W
        if form.startswith("d"):
            ci, co = cout, cin                      # the data gradient as a 1x1 conv: dY (cout ch) -> dX (cin ch)
        else:
            ci, co = cin, cout
        x = torch.randn(B, H, W, ci, device=dev).to(torch.bfloat16)
        w = (torch.randn(co, 1, 1, ci, device=dev) / ci ** 0.5).to(torch.bfloat16)
        g = NC.geom_single(B, H, W, H, W, 1, 1, (0, 0, 0, 0), ci, co)
        b = torch.randn(co, device=dev) if form.startswith("f") and form != "f0" else None
        res = torch.randn(B, H, W, co, device=dev).to(torch.bfloat16) if form == "fr" else None
        act = torch.randn(B, H, W, co, device=dev).to(torch.bfloat16)
        relu = form in ("f", "fr")
        out = torch.randn(B, H, W, co, device=dev).to(torch.bfloat16) if form == "da" else None
        if form == "fr":
            mask = BitMask(shape=(B, H, W, co), device=dev)
        elif form == "da":
            mask = BitMask(act)
        elif form == "d":
            mask = act
        else:
            mask = None
        cands = fwd_candidates(x, w, b, res, g, 1, (0, 0, 0, 0), relu, (B, H, W, co), allow_miopen=False,
                               mask=mask, out=out)
        res_t = {}
        for cn, fn in cands.items():
            try:
                res_t[cn] = timeit(fn, a.reps)
            except RuntimeError:
                continue
        # minimal traffic: X once, Y written (+ read when accumulating), residual, mask (bf16 or 1/16 bits)
        byt = M * ci * 2 + M * co * 2 * (2 if out is not None else 1) + (M * co * 2 if res is not None else 0)
        byt += (M * co * 2 if form == "d" else (M * co // 8 if form in ("fr", "da") else 0))
        flop = 2.0 * M * ci * co
        best = sorted((t, n) for n, t in res_t.items() if n != "c1p")[:3]
        line = "  ".join("%s %.4f" % (n, t) for t, n in best)
        c = res_t.get("c1p")
        cs = ("c1p %.4f ms %.0f TF/s %.2f TB/s (x%.2f vs best)" % (c, flop / c / 1e9, byt / c / 1e9, best[0][0] / c)
              if c else "c1p n/a")
        print("%-22s %s | %s" % (name, cs, line), flush=True)


if __name__ == "__main__":
    main()
