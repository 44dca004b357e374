"""Which part of the bucket-engine event pattern slows the compute stream?  torch-API replicas."""
import time

import torch


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
    bufs = [torch.randn(8 << 20, device=dev) for _ in range(3)]
    side = torch.cuda.Stream(dev, priority=-1)
    NB = 5

    def chain():
        for _ in range(50):
            torch.add(bufs[0], bufs[1], out=bufs[2])
            torch.mul(bufs[2], 0.5, out=bufs[0])

    fixed = {k: [torch.cuda.Event(enable_timing=t) for _ in range(NB)] for k, t in
             (("ready", False), ("done", False), ("ready_t", True), ("done_t", True), ("start_t", True))}

    def engine(reuse, timing, back=True, markers=True):
        def f():
            chain()
            cur = torch.cuda.current_stream()
            dones = []
            for b in range(NB):
                r = fixed["ready_t" if timing else "ready"][b] if reuse else torch.cuda.Event(enable_timing=timing)
                r.record(cur)
                side.wait_event(r)
                if markers:
                    if timing:
                        (fixed["start_t"][b] if reuse else torch.cuda.Event(enable_timing=True)).record(side)
                    d = fixed["done_t" if timing else "done"][b] if reuse else torch.cuda.Event(enable_timing=timing)
                    d.record(side)
                    dones.append(d)
            if back:
                for d in dones:
                    cur.wait_event(d)
        return f

    res = {"chain": timeit(chain)}
    for reuse in (False, True):
        for timing in (False, True):
            res["reuse%d_timing%d" % (reuse, timing)] = timeit(engine(reuse, timing))
    res["fresh_noback"] = timeit(engine(False, False, back=False))
    res["fresh_nomarkers"] = timeit(engine(False, False, back=False, markers=False))
    res["chain_again"] = timeit(chain)
    for k, v in res.items():
        print("%-22s %8.3f ms" % (k, v), flush=True)


if __name__ == "__main__":
    main()
