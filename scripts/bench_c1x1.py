"""Microbench: streaming 1x1 kernel variants vs the pipelined kernel on the backbone 1x1 shapes (B=16)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from batchai_retinanet_horovod_coco_amd.ops import native as N  # noqa: E402
from batchai_retinanet_horovod_coco_amd.ops import native_conv as NC  # noqa: E402

SHAPES = [  # name, H, W, cin, cout, residual+relu
    ("s2_64_256_res", 200, 334, 64, 256, True),
    ("s2_256_64", 200, 334, 256, 64, False),
    ("s2_64_64", 200, 334, 64, 64, False),
    ("s3_128_512_res", 100, 167, 128, 512, True),
    ("s4_256_1024_res", 50, 84, 256, 1024, True),
    ("dg_s2_K64_N256_mask_acc", 200, 334, 64, 256, "ma"),
]


def timeit(fn, reps=20):
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
    for name, H, W, cin, cout, epi in SHAPES:
        x = torch.randn(B, H, W, cin, device=dev).to(torch.bfloat16)
        w = (torch.randn(cout, 1, 1, cin, device=dev) / cin ** 0.5).to(torch.bfloat16)
        b = torch.randn(cout, device=dev)
        y = torch.empty(B, H, W, cout, device=dev, dtype=torch.bfloat16)
        res = torch.randn_like(y) if epi is True else None
        mask = torch.randn_like(y) if epi == "ma" else None
        g = NC.geom_single(B, H, W, H, W, 1, 1, (0, 0, 0, 0), cin, cout)
        nbytes = x.numel() * 2 + y.numel() * 2 * (2 if epi is True else (3 if epi == "ma" else 1))
        out = []
        for v in NC.c1x1_variants(g) + [14, 15, 16]:
            t = timeit(lambda: NC.launch_fwd(x, w, b, res, y, g, epi is True, accumulate=epi == "ma", variant=v,
                                             mask=mask))
            out.append("%s %.3f ms %.2f TB/s" % (v, t, nbytes / t / 1e9))
        print("%-26s %s" % (name, " | ".join(out)))
    # pure streaming reference: a bf16 copy of the biggest activation
    y = torch.empty(B, 200, 334, 256, device=dev, dtype=torch.bfloat16)
    z = torch.empty_like(y)
    t = timeit(lambda: z.copy_(y))
    print("copy 547MB: %.3f ms %.2f TB/s" % (t, 2 * y.numel() * 2 / t / 1e9))


if __name__ == "__main__":
    main()
