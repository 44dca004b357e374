"""Microbench: fp8 (e4m3 x e4m3, scaled MFMA) head-layer forward vs the bf16 incumbents at the production
pyramid shape (quantisation passes excluded: in training they are fused into the producer's epilogue)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from batchai_retinanet_horovod_coco_amd.ops import fp8  # noqa: E402
from batchai_retinanet_horovod_coco_amd.ops import native as N  # noqa: E402
from bench_p8 import bench  # noqa: E402


def main():
    N.load(required=True)
    dev = torch.device("cuda", 0)
    shapes = [(100, 167), (50, 84), (25, 42), (13, 21), (7, 11)]
    n = 16
    P = sum(h * w for h, w in shapes)
    for cin, cout in ((256, 256), (256, 720)):
        x = torch.relu(torch.randn(n, P, cin, device=dev)).bfloat16()
        w = (torch.randn(cout, 3, 3, cin, device=dev) / (9 * cin) ** 0.5).bfloat16()
        b = torch.randn(cout, device=dev)
        y = torch.empty(n, P, cout, device=dev, dtype=torch.bfloat16)
        g = N.geom_pyramid(n, shapes, cin, cout)
        flops = 2.0 * n * P * cout * 9 * cin
        for v in ("hx32_0", "hx32_1", "p8_8"):
            ms = bench(lambda: N.launch_fwd(x, w, b, None, y, g, True, variant=v))
            print("pyramid %4d->%4d bf16 %-7s %7.3f ms %6.0f TF/s" % (cin, cout, v, ms, flops / ms / 1e9), flush=True)
        xq, ix = fp8.quantize(x)
        wq, iw = fp8.quantize_rows(w)
        for v in (3, 6, 7) + fp8.HX8_VARIANTS:
            ms = bench(lambda: fp8.launch(xq, ix, wq, iw, b, None, y, g, True, v))
            print("pyramid %4d->%4d fp8  f8_%-4d %7.3f ms %6.0f TF/s" % (cin, cout, v, ms, flops / ms / 1e9), flush=True)
        # data-gradient form (e5m2 dY x e4m3 flipped W; 720 -> 768-padded dY rows for the classification final)
        if cout == 256:
            dq, idq = fp8.quantize_bf8(x)
            for v in fp8.F8_DGRAD_VARIANTS + fp8.HX8_DGRAD_VARIANTS:
                ms = bench(lambda: fp8.launch(dq, idq, wq, iw, None, None, y, g, False, v, mask=x))
                print("pyramid %4d->%4d dgrad f8d_%-3d %7.3f ms %6.0f TF/s" % (cin, cout, v, ms, flops / ms / 1e9),
                      flush=True)


if __name__ == "__main__":
    main()
