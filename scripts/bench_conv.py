#!/usr/bin/env python
"""Per-shape-class conv timing: HIP implicit-GEMM kernels vs MIOpen (F.conv2d, channels-last bf16).

Shapes are every conv class of RetinaNet-R50-FPN at 800x1333, batch 16.
Prints one line per shape: ms and TFLOP/s for each variant, forward and data-gradient.
"""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from batchai_retinanet_horovod_coco_amd.ops import native as N  # noqa: E402
from batchai_retinanet_horovod_coco_amd.ops import conv as C  # noqa: E402
from batchai_retinanet_horovod_coco_amd.ops import fp8 as F8  # noqa: E402

B = 16
SHAPES = [
    # name, H, W, cin, cout, k, stride, pad
    ("s2_1x1_64_64", 200, 334, 64, 64, 1, 1, 0),
    ("s2_3x3_64", 200, 334, 64, 64, 3, 1, 1),
    ("s2_1x1_64_256", 200, 334, 64, 256, 1, 1, 0),
    ("s2_1x1_256_64", 200, 334, 256, 64, 1, 1, 0),
    ("s3_1x1s2_256_128", 200, 334, 256, 128, 1, 2, 0),
    ("s3_3x3_128", 100, 167, 128, 128, 3, 1, 1),
    ("s3_1x1_128_512", 100, 167, 128, 512, 1, 1, 0),
    ("s3_1x1_512_128", 100, 167, 512, 128, 1, 1, 0),
    ("s3_1x1s2_256_512", 200, 334, 256, 512, 1, 2, 0),
    ("s4_3x3_256", 50, 84, 256, 256, 3, 1, 1),
    ("s4_1x1_256_1024", 50, 84, 256, 1024, 1, 1, 0),
    ("s4_1x1_1024_256", 50, 84, 1024, 256, 1, 1, 0),
    ("s5_3x3_512", 25, 42, 512, 512, 3, 1, 1),
    ("s5_1x1_512_2048", 25, 42, 512, 2048, 1, 1, 0),
    ("s5_1x1_2048_512", 25, 42, 2048, 512, 1, 1, 0),
    ("fpn_P3_3x3", 100, 167, 256, 256, 3, 1, 1),
    ("fpn_C3red", 100, 167, 512, 256, 1, 1, 0),
    ("fpn_P6", 25, 42, 2048, 256, 3, 2, "same"),
]
PYR = [(100, 167), (50, 84), (25, 42), (13, 21), (7, 11)]
WGRAD_VARIANTS = tuple(range(16))


def timeit(fn, iters=10, warm=3):
    for _ in range(warm):
        fn()
    s = torch.cuda.Event(enable_timing=True)
    e = torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="0,1,2,3,4,5,6,7,8,9,10,11,12,13,14,15,16")
    ap.add_argument("--only", default="", help="substring filter on shape names")
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    N.load(required=True)
    torch.backends.cudnn.benchmark = True
    dev = torch.device("cuda")
    rows = []
    variants = [int(v) for v in args.variants.split(",")]
    for name, H, W, cin, cout, k, s, pad in SHAPES:
        if args.only and not any(o in name for o in args.only.split(",")):
            continue
        pads = C.same_pads((H, W), k, s) if pad == "same" else (pad, pad, pad, pad)
        Ho, Wo = C.out_hw((H, W), k, s, pads)
        x = torch.randn(B, H, W, cin, device=dev).bfloat16()
        w = (torch.randn(cout, k, k, cin, device=dev) * 0.05).bfloat16()
        b = torch.randn(cout, device=dev)
        flops = 2.0 * B * Ho * Wo * cout * k * k * cin
        r = {"name": name, "gflop": flops / 1e9}
        xin = x if pads[0] == pads[1] and pads[2] == pads[3] else F.pad(x, (0, 0, pads[2], pads[3], pads[0], pads[1]))
        pd = (pads[0], pads[2]) if xin is x else (0, 0)
        xc, wc, bc = xin.permute(0, 3, 1, 2), w.permute(0, 3, 1, 2), b.bfloat16()
        t = timeit(lambda: F.conv2d(xc, wc, bc, s, pd))
        r["miopen_fwd_ms"] = t
        g = N.geom_single(B, H, W, Ho, Wo, k, s, pads, cin, cout)
        y = torch.empty(B, Ho, Wo, cout, device=dev, dtype=torch.bfloat16)
        for v in variants:   # explicit launches (N.conv2d would run the tuner's pick for every v)
            try:
                r["hip_fwd_v%d_ms" % v] = timeit(lambda: N.launch_fwd(x, w, b, None, y, g, True, variant=v))
            except Exception as e:  # noqa: BLE001
                r["hip_fwd_v%d_ms" % v] = str(e)
        if F8.eligible(cin, cout):
            xq, ix = F8.quantize(x)
            wq, iw = F8.quantize_rows(w)
            bf = b.float()
            r["f8_quant_x_ms"] = timeit(lambda: F8.quantize(x))
            for v in F8.F8_VARIANTS:
                r["f8_fwd_v%d_ms" % v] = timeit(lambda: F8.launch(xq, ix, wq, iw, bf, None, y, g, True, v))
        # data gradient
        dy = torch.randn(B, Ho, Wo, cout, device=dev).bfloat16()
        dyc = dy.permute(0, 3, 1, 2)
        t = timeit(lambda: torch.ops.aten.convolution_backward(dyc, xc, wc, None, [s, s], list(pd), [1, 1], False,
                                                                [0, 0], 1, [True, False, False]))
        r["miopen_dgrad_ms"] = t
        t = timeit(lambda: torch.ops.aten.convolution_backward(dyc, xc, wc, None, [s, s], list(pd), [1, 1], False,
                                                                [0, 0], 1, [False, True, False]))
        r["miopen_wgrad_ms"] = t
        if N.conv_dgrad(dy, w, tuple(x.shape), s, pads) is not None:
            for v in variants:
                r["hip_dgrad_v%d_ms" % v] = timeit(lambda: N.conv_dgrad(dy, w, tuple(x.shape), s, pads, v))
        for v in WGRAD_VARIANTS:
            r["hip_wgrad_v%d_ms" % v] = timeit(lambda: N.conv_wgrad(x, dy, g, None, variant=v))
        rows.append(r)
        print(json.dumps({k2: (round(v2, 4) if isinstance(v2, float) else v2) for k2, v2 in r.items()}), flush=True)
    # heads: 5 levels as one ragged GEMM vs 5 MIOpen calls
    for cout in (256, 720, 36):
        if args.only and not any(o in "head_3x3_256_%d" % cout for o in args.only.split(",")):
            continue
        xs = [torch.randn(B, h, w_, 256, device=dev).bfloat16() for h, w_ in PYR]
        w = (torch.randn(cout, 3, 3, 256, device=dev) * 0.05).bfloat16()
        b = torch.randn(cout, device=dev)
        packed, sh = N.pyramid_pack(xs)
        flops = 2.0 * B * sum(h * w_ for h, w_ in PYR) * cout * 9 * 256
        r = {"name": "head_3x3_256_%d" % cout, "gflop": flops / 1e9}
        wc, bc = w.permute(0, 3, 1, 2), b.bfloat16()
        xcs = [x.permute(0, 3, 1, 2) for x in xs]
        r["miopen_fwd_ms"] = timeit(lambda: [F.conv2d(xc, wc, bc, 1, 1) for xc in xcs])
        # explicit variant launches (the pyramid autograd path would run the tuner's pick for every v)
        gf = N.geom_pyramid(B, sh, 256, cout)
        yf = torch.empty(B, packed.shape[1], cout, device=dev, dtype=torch.bfloat16)
        for v in variants:
            try:
                r["hip_fwd_v%d_ms" % v] = timeit(lambda: N.launch_fwd(packed, w, b, None, yf, gf, True, variant=v))
            except Exception as e:  # noqa: BLE001
                r["hip_fwd_v%d_ms" % v] = str(e)
        if F8.eligible(256, cout):
            xq, ix = F8.quantize(packed)
            wq, iw = F8.quantize_rows(w)
            r["f8_quant_x_ms"] = timeit(lambda: F8.quantize(packed))
            for v in F8.F8_VARIANTS:
                r["f8_fwd_v%d_ms" % v] = timeit(lambda: F8.launch(xq, ix, wq, iw, b, None, yf, gf, True, v))
        dy = torch.randn(B, packed.shape[1], cout, device=dev).bfloat16()
        cp = (cout + 63) // 64 * 64
        dyp = F.pad(dy, (0, cp - cout)).contiguous()
        wd = F.pad(N.flip(w), (0, cp - cout)).contiguous()
        gd = N.geom_pyramid(B, sh, cp, 256)
        dx = torch.empty(B, packed.shape[1], 256, device=dev, dtype=torch.bfloat16)
        for v in variants:
            r["hip_dgrad_v%d_ms" % v] = timeit(lambda: N.launch_fwd(dyp, wd, None, None, dx, gd, False, variant=v))
        for v in WGRAD_VARIANTS:
            r["hip_wgrad_v%d_ms" % v] = timeit(lambda: N.conv_wgrad(packed, dy, N.geom_pyramid(B, sh, 256, cout), None,
                                                                     variant=v))
        dyl = [dy[:, o:o + h * w_].reshape(B, h, w_, cout).permute(0, 3, 1, 2) for o, (h, w_) in
               zip([0, 16700, 20900, 21950, 22223], PYR)]
        r["miopen_wgrad_ms"] = timeit(lambda: [torch.ops.aten.convolution_backward(
            d, xc, wc, None, [1, 1], [1, 1], [1, 1], False, [0, 0], 1, [False, True, False]) for d, xc in zip(dyl, xcs)])
        r["miopen_dgrad_ms"] = timeit(lambda: [torch.ops.aten.convolution_backward(
            d, xc, wc, None, [1, 1], [1, 1], [1, 1], False, [0, 0], 1, [True, False, False]) for d, xc in zip(dyl, xcs)])
        rows.append(r)
        print(json.dumps({k2: (round(v2, 4) if isinstance(v2, float) else v2) for k2, v2 in r.items()}), flush=True)
    tot = {}
    for r in rows:
        for k2, v2 in r.items():
            if k2.endswith("_ms") and isinstance(v2, float):
                tot[k2] = tot.get(k2, 0.0) + v2
    print("TOTALS", json.dumps({k2: round(v2, 3) for k2, v2 in tot.items()}))
    if args.out:
        with open(args.out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
