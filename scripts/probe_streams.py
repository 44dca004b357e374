"""Does cross-stream event traffic slow the compute stream's kernels?  (native comm engine A/B)

Times a chain of L2/MALL-resident memory-bound kernels and a bf16 GEMM on the current stream while a
side stream (the comm stream's role) waits on events recorded between them, in several forms.
"""
import sys
import time

import torch


def chain(bufs, n):
    a, b, c = bufs
    for _ in range(n):
        torch.add(a, b, out=c)
        torch.mul(c, 0.5, out=a)


def gemm(x, w, n):
    for _ in range(n):
        torch.matmul(x, w)


def timeit(fn, reps=5):
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(reps):
        t = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t)
    return best * 1e3


def main():
    dev = torch.device("cuda", 0)
    n_el = 8 << 20     # 32 MB fp32 per buffer: L2/MALL resident
    bufs = [torch.randn(n_el, device=dev) for _ in range(3)]
    x = torch.randn(16384, 2304, device=dev, dtype=torch.bfloat16)
    w = torch.randn(2304, 256, device=dev, dtype=torch.bfloat16)
    lo, hi = torch.cuda.Stream.priority_range() if hasattr(torch.cuda.Stream, "priority_range") else (0, -1)
    side_hi = torch.cuda.Stream(dev, priority=-1)
    side_lo = torch.cuda.Stream(dev, priority=0)
    N = 50

    def plain():
        chain(bufs, N)

    def with_events(side, wait_back=False, every=1):
        def f():
            cur = torch.cuda.current_stream()
            evs = []
            for i in range(N):
                torch.add(bufs[0], bufs[1], out=bufs[2])
                torch.mul(bufs[2], 0.5, out=bufs[0])
                if side is not None and i % every == 0:
                    e = torch.cuda.Event()
                    e.record(cur)
                    side.wait_event(e)
                    evs.append(e)
            if side is not None and wait_back:
                e2 = torch.cuda.Event()
                e2.record(side)
                cur.wait_event(e2)
        return f

    def only_record():
        cur = torch.cuda.current_stream()
        for i in range(N):
            torch.add(bufs[0], bufs[1], out=bufs[2])
            torch.mul(bufs[2], 0.5, out=bufs[0])
            torch.cuda.Event().record(cur)

    res = {}
    res["plain"] = timeit(plain)
    res["record_only"] = timeit(only_record)
    res["side_hi_wait"] = timeit(with_events(side_hi))
    res["side_lo_wait"] = timeit(with_events(side_lo))
    res["side_hi_wait_back"] = timeit(with_events(side_hi, True))
    res["side_hi_every10"] = timeit(with_events(side_hi, True, 10))
    res["plain_again"] = timeit(plain)
    res["gemm_plain"] = timeit(lambda: gemm(x, w, 20))

    def gemm_side():
        cur = torch.cuda.current_stream()
        for i in range(20):
            torch.matmul(x, w)
            e = torch.cuda.Event()
            e.record(cur)
            side_hi.wait_event(e)
    res["gemm_side_hi"] = timeit(gemm_side)
    res["gemm_plain_again"] = timeit(lambda: gemm(x, w, 20))
    # side stream that once waited and is now idle: does its mere existence keep costing?
    res["plain_after_side"] = timeit(plain)
    for k, v in res.items():
        print("%-20s %8.3f ms" % (k, v), flush=True)


if __name__ == "__main__":
    sys.exit(main())
