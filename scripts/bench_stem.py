"""Microbench of the stem kernels at the headline shape (B=16, 800x1333): HIP conv1 fwd / wgrad and the
relu-aware max-pool vs the MIOpen library path."""
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from batchai_retinanet_horovod_coco_amd.ops import conv as C  # noqa: E402
from batchai_retinanet_horovod_coco_amd.ops import native as N  # noqa: E402
from batchai_retinanet_horovod_coco_amd.ops import stem as S  # noqa: E402


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
    B, H, W = int(os.environ.get("B", "16")), 800, 1333
    x = (torch.randn(B, H, W, 3, device=dev) * 50).to(torch.bfloat16)
    w = torch.randn(64, 7, 7, 3, device=dev) * 0.05
    scale = torch.rand(64, device=dev) + 0.5
    shift = torch.randn(64, device=dev) * 0.1
    pads = (3, 3, 3, 3)
    y1 = S.stem_conv_fwd(x, w, scale, shift, pads)
    Ho, Wo = y1.shape[1], y1.shape[2]
    pp = C.same_pads((Ho, Wo), 3, 2)
    yp, arg = N.maxpool_fwd_raw(y1, 3, 2, pp, relu_in=True)
    dyp = torch.randn_like(yp)
    dy1 = N.maxpool_bwd_raw(dyp, arg, tuple(y1.shape), 3, 2, pp)
    gflop = 2 * B * Ho * Wo * 64 * 147 / 1e9
    t_fwd = timeit(lambda: S.stem_conv_fwd(x, w, scale, shift, pads))
    t_fused = timeit(lambda: S.stem_pool_fwd(x, w, scale, shift, pads, pp))
    t_pf = timeit(lambda: N.maxpool_fwd_raw(y1, 3, 2, pp, relu_in=True))
    t_pb = timeit(lambda: N.maxpool_bwd_raw(dyp, arg, tuple(y1.shape), 3, 2, pp))
    t_wg = timeit(lambda: S.stem_wgrad(x, dy1, scale, pads))
    t_wgf = timeit(lambda: S.stem_wgrad(x, dyp, scale, pads, pool=(arg, (Ho, Wo), pp)))
    xc = x.permute(0, 3, 1, 2)
    wb = (w * scale.view(-1, 1, 1, 1)).to(torch.bfloat16).permute(0, 3, 1, 2)
    t_mf = timeit(lambda: torch.relu(F.conv2d(xc, wb, None, 2, 3) + shift.to(torch.bfloat16).view(1, -1, 1, 1)))
    dyc = dy1.permute(0, 3, 1, 2)
    t_mw = timeit(lambda: torch.ops.aten.convolution_backward(dyc, xc, wb, None, (2, 2), (3, 3), (1, 1), False,
                                                              (0, 0), 1, (False, True, False)))
    print("stem conv fwd  hip %.3f ms (%.0f TF/s) | miopen+bias+relu %.3f ms" % (t_fwd, gflop / t_fwd, t_mf))
    print("stem wgrad     hip %.3f ms (%.0f TF/s) | miopen %.3f ms" % (t_wg, gflop / t_wg, t_mw))
    print("maxpool fwd %.3f ms  bwd %.3f ms" % (t_pf, t_pb))
    print("stem conv + pool fused %.3f ms (vs conv + pool %.3f ms)" % (t_fused, t_fwd + t_pf))
    print("pool-fused stem wgrad %.3f ms (vs pool bwd + wgrad %.3f ms)" % (t_wgf, t_pb + t_wg))


if __name__ == "__main__":
    main()
