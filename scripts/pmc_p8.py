"""Run one GEMM-shaped conv_p8 variant a few times (for rocprofv3 --pmc passes)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from batchai_retinanet_horovod_coco_amd.ops import native as N  # noqa: E402


def main():
    N.load(required=True)
    dev = torch.device("cuda", 0)
    M, Nn, K = (int(v) for v in sys.argv[2:5]) if len(sys.argv) > 4 else (8192, 8192, 8192)
    x = torch.randn(M, K, device=dev).bfloat16()
    w = torch.randn(Nn, K, device=dev).bfloat16()
    y = torch.empty(M, Nn, device=dev, dtype=torch.bfloat16)
    v = sys.argv[1]
    for _ in range(4):
        if v == "blas":
            torch.matmul(x, w.t())
        else:
            g = N.geom_single(1, M, 1, M, 1, 1, 1, (0, 0, 0, 0), K, Nn)
            N.launch_fwd(x.view(1, M, 1, K), w.view(Nn, 1, 1, K), None, None, y, g, False, variant=v)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
