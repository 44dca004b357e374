"""Microbench: conv_p8 vs the tuned incumbents at the production head shapes, and vs hipBLASLt GEMM."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from batchai_retinanet_horovod_coco_amd.ops import native as N  # noqa: E402


def bench(fn, reps=20):
    for _ in range(3):
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
    shapes = [(100, 167), (50, 84), (25, 42), (13, 21), (7, 11)]
    n = 16
    P = sum(h * w for h, w in shapes)
    for cin, cout in ((256, 256), (256, 720), (256, 768)):
        x = torch.randn(n, P, cin, device=dev).bfloat16()
        w = (torch.randn(cout, 3, 3, cin, device=dev) / (9 * cin) ** 0.5).bfloat16()
        b = torch.randn(cout, device=dev)
        y = torch.empty(n, P, cout, device=dev, dtype=torch.bfloat16)
        g = N.geom_pyramid(n, shapes, cin, cout)
        flops = 2.0 * n * P * cout * 9 * cin
        for v in ("halo12", "p8_5", "p8_6", "p8_7"):
            try:
                ms = bench(lambda: N.launch_fwd(x, w, b, None, y, g, True, variant=v))
                print("pyramid %4d->%4d %-6s %7.3f ms %6.0f TF/s" % (cin, cout, v, ms, flops / ms / 1e9), flush=True)
            except Exception as e:  # noqa: BLE001
                print("pyramid %4d->%4d %-6s failed: %s" % (cin, cout, v, str(e)[:80]), flush=True)
    # plain GEMM: 1x1 conv M x 2304 -> 256 vs torch.matmul (hipBLASLt)
    M, K, Nn = n * P, 2304, 256
    x = torch.randn(M, K, device=dev).bfloat16()
    w = torch.randn(Nn, K, device=dev).bfloat16()
    y = torch.empty(M, Nn, device=dev, dtype=torch.bfloat16)
    g = N.geom_single(1, M, 1, M, 1, 1, 1, (0, 0, 0, 0), K, Nn)
    flops = 2.0 * M * K * Nn
    for v in ("p8_5", "p8_6", "p8_7"):
        ms = bench(lambda: N.launch_fwd(x.view(1, M, 1, K), w.view(Nn, 1, 1, K), None, None, y, g, False, variant=v))
        print("gemm %d x %d x %d %-6s %7.3f ms %6.0f TF/s" % (M, Nn, K, v, ms, flops / ms / 1e9), flush=True)
    ms = bench(lambda: torch.matmul(x, w.t()))
    print("gemm %d x %d x %d hipblaslt %7.3f ms %6.0f TF/s" % (M, Nn, K, ms, flops / ms / 1e9), flush=True)
    x2 = torch.randn(8192, 8192, device=dev).bfloat16()
    w2 = torch.randn(8192, 8192, device=dev).bfloat16()
    ms = bench(lambda: torch.matmul(x2, w2.t()), reps=10)
    print("gemm 8192^3 hipblaslt %7.3f ms %6.0f TF/s" % (ms, 2 * 8192 ** 3 / ms / 1e9), flush=True)
    y2 = torch.empty(8192, 8192, device=dev, dtype=torch.bfloat16)
    g2 = N.geom_single(1, 8192, 1, 8192, 1, 1, 1, (0, 0, 0, 0), 8192, 8192)
    for v in ("p8_5", "p8_6", "p8_7"):
        ms = bench(lambda: N.launch_fwd(x2.view(1, 8192, 1, 8192), w2.view(8192, 1, 1, 8192), None, None, y2, g2,
                                        False, variant=v), reps=10)
        print("gemm 8192^3 %-6s %7.3f ms %6.0f TF/s" % (v, ms, 2 * 8192 ** 3 / ms / 1e9), flush=True)




def wgrad_main():
    N.load(required=True)
    dev = torch.device("cuda", 0)
    shapes = [(100, 167), (50, 84), (25, 42), (13, 21), (7, 11)]
    n = 16
    P = sum(h * w for h, w in shapes)
    for cin, cout in ((256, 256), (256, 720)):
        x = torch.randn(n, P, cin, device=dev).bfloat16()
        dy = torch.randn(n, P, cout, device=dev).bfloat16()
        g = N.geom_pyramid(n, shapes, cin, cout)
        flops = 2.0 * n * P * cout * 9 * cin
        for v in (3, 20, 21, 22, 23):
            ms = bench(lambda: N.conv_wgrad(x, dy, g, None, variant=v))
            print("pyramid wgrad %4d->%4d hip%-3d %7.3f ms %6.0f TF/s" % (cin, cout, v, ms, flops / ms / 1e9), flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "wgrad":
        wgrad_main()
    else:
        main()
