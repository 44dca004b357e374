"""Main-loop ablation of the pipelined conv kernel on the head GEMM (what bounds it?)."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from batchai_retinanet_horovod_coco_amd.ops import native as N  # noqa: E402
from batchai_retinanet_horovod_coco_amd.ops.native import ConvGeom, _p, _s, zero_page  # noqa: E402

PYR = [(100, 167), (50, 84), (25, 42), (13, 21), (7, 11)]


def main():
    N.load(required=True)
    L = N.lib()
    L.mxr_conv_fwd_pipe_ablate.argtypes = [ctypes.c_void_p] * 4 + [ctypes.POINTER(ConvGeom), ctypes.c_int,
                                                                   ctypes.c_void_p]
    dev = torch.device("cuda")
    B = 16
    xs = [torch.randn(B, h, w, 256, device=dev).bfloat16() for h, w in PYR]
    packed, sh = N.pyramid_pack(xs)
    for cout in (256, 720):
        w = (torch.randn(cout, 3, 3, 256, device=dev) * 0.05).bfloat16()
        y = torch.empty(B, packed.shape[1], cout, device=dev, dtype=torch.bfloat16)
        g = N.geom_pyramid(B, sh, 256, cout)
        gf = 2.0 * B * packed.shape[1] * cout * 9 * 256 / 1e9
        for abl, name in ((0, "full"), (4, "full interleaved"), (5, "interleaved+setprio"), (1, "no-DMA"),
                          (2, "no-MFMA"),
                          (3, "DMA+barrier only")):
            def run():
                rc = L.mxr_conv_fwd_pipe_ablate(_p(packed), _p(w), _p(y), _p(zero_page(dev)), ctypes.byref(g), abl,
                                                _s())
                assert rc == 0, rc
            for _ in range(3):
                run()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(10):
                run()
            e.record()
            torch.cuda.synchronize()
            ms = s.elapsed_time(e) / 10
            print("cout %4d %-18s %.3f ms  (%.0f TF-equivalent)" % (cout, name, ms, gf / ms))


if __name__ == "__main__":
    main()
