#!/usr/bin/env python
"""Practical HBM bandwidth of this MI355X through plain PyTorch elementwise kernels (copy: 1 read + 1 write;
``a += b``: 2 reads + 1 write), the yardstick for the memory-bound 1x1 convolutions' TB/s in the conv budgets.

usage: bw_probe.py [MB ...]   (default 256 1024; each size is warmed up before it is timed)"""
import sys

import torch


def _time(fn, reps=20):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps


def main():
    d = torch.device("cuda", 0)
    for mb in [int(v) for v in sys.argv[1:]] or [256, 1024]:
        n = mb * 2 ** 20 // 2
        a = torch.randn(n, device=d).bfloat16()
        b = torch.empty_like(a)
        t = _time(lambda: b.copy_(a))
        print("copy %5d MB: %.3f ms  %.2f TB/s (read + write)" % (mb, t, 2 * mb * 2 ** 20 / t / 1e9))
        t = _time(lambda: a.add_(b))
        print("a+=b %5d MB: %.3f ms  %.2f TB/s (2 reads + write)" % (mb, t, 3 * mb * 2 ** 20 / t / 1e9))


if __name__ == "__main__":
    main()
