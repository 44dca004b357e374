"""Does merely having an RCCL communicator (native core or torch ProcessGroupNCCL) slow kernels down?"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


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
    mode = sys.argv[1]
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    bufs = [torch.randn(8 << 20, device=dev) for _ in range(3)]
    x = torch.randn(16384, 2304, device=dev, dtype=torch.bfloat16)
    w = torch.randn(2304, 256, device=dev, dtype=torch.bfloat16)
    flat = torch.randn(40 << 20, device=dev)

    def chain():
        for _ in range(50):
            torch.add(bufs[0], bufs[1], out=bufs[2])
            torch.mul(bufs[2], 0.5, out=bufs[0])

    def gemm():
        for _ in range(20):
            torch.matmul(x, w)

    out = {}
    out["chain_before"] = timeit(chain)
    out["gemm_before"] = timeit(gemm)
    if mode == "native":
        from batchai_retinanet_horovod_coco_amd.parallel.native_comm import NativeComm
        c = NativeComm(0, 1, 0)
        out["chain_comm_exists"] = timeit(chain)
        c.set_buckets([flat[i * (8 << 20):(i + 1) * (8 << 20)] for i in range(5)])
        out["chain_buckets_set"] = timeit(chain)

        def step():
            chain()
            for b in range(5):
                c.bucket_ready(b)
            c.wait()
        out["chain_with_buckets"] = timeit(step)
        out["buckets_only"] = timeit(lambda: ([c.bucket_ready(b) for b in range(5)], c.wait()))
        st = c.step_stats()
        out["stats_comm_ms"] = st["comm_ms"] if st else -1
        out["stats_exposed_ms"] = st["exposed_ms"] if st else -1
        out["chain_after"] = timeit(chain)
        out["gemm_after"] = timeit(gemm)
        c.close()
        out["chain_after_close"] = timeit(chain)
    elif mode == "torchpg":
        import torch.distributed as dist
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT="29533")
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
        out["chain_pg_exists"] = timeit(chain)

        def step():
            chain()
            for b in range(5):
                dist.all_reduce(flat[b * (8 << 20):(b + 1) * (8 << 20)], async_op=True)
        out["chain_with_allreduce"] = timeit(step)
        out["chain_after"] = timeit(chain)
        out["gemm_after"] = timeit(gemm)
        dist.destroy_process_group()
    for k, v in out.items():
        print("%-8s %-22s %8.3f ms" % (mode, k, v), flush=True)


if __name__ == "__main__":
    main()
