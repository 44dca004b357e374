"""Run one head-layer conv pass at the production pyramid shape a few times (rocprofv3 --pmc target).
usage: pmc_pyr.py fwd|wgrad|wgradb|f8 VARIANT [cout]   (wgradb: with the fused bias gradient)"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from batchai_retinanet_horovod_coco_amd.ops import native as N  # noqa: E402


def main():
    N.load(required=True)
    dev = torch.device("cuda", 0)
    kind, v = sys.argv[1], sys.argv[2]
    cout = int(sys.argv[3]) if len(sys.argv) > 3 else 256
    shapes = [(100, 167), (50, 84), (25, 42), (13, 21), (7, 11)]
    n, cin = 16, 256
    P = sum(h * w for h, w in shapes)
    x = torch.randn(n, P, cin, device=dev).bfloat16()
    if os.environ.get("PMC_ZERO_X") == "1":   # operand values change the MFMA power draw, hence the clock
        x.zero_()
    g = N.geom_pyramid(n, shapes, cin, cout)
    if kind == "fwd":
        w = (torch.randn(cout, 3, 3, cin, device=dev) / 48).bfloat16()
        b = torch.randn(cout, device=dev)
        y = torch.empty(n, P, cout, device=dev, dtype=torch.bfloat16)
        for _ in range(4):
            N.launch_fwd(x, w, b, None, y, g, True, variant=v)
    elif kind == "f8":
        from batchai_retinanet_horovod_coco_amd.ops import fp8
        w = (torch.randn(cout, 3, 3, cin, device=dev) / 48).bfloat16()
        b = torch.randn(cout, device=dev)
        xq, ix = fp8.quantize(x)
        wq, iw = fp8.quantize_rows(w)
        y = torch.empty(n, P, cout, device=dev, dtype=torch.bfloat16)
        for _ in range(4):
            fp8.launch(xq, ix, wq, iw, b, None, y, g, True, int(v))
    else:
        dy = torch.randn(n, P, cout, device=dev).bfloat16()
        db = torch.zeros(cout, device=dev) if kind == "wgradb" else None
        for _ in range(4):
            N.conv_wgrad(x, dy, g, None, variant=int(v), bias_out=db)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
