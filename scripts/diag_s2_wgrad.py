"""Every weight-gradient candidate of the FPN 3x3 / stride-2 convs at TF-same pads, against fp32 PyTorch:
prints the cosine and relative norm error per candidate (diagnostic for tests/test_backbone_grad_gpu.py)."""
import sys
import os

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from batchai_retinanet_horovod_coco_amd.ops import conv as C  # noqa: E402
from batchai_retinanet_horovod_coco_amd.ops import native  # noqa: E402
from batchai_retinanet_horovod_coco_amd.ops import native_conv  # noqa: E402,F401  (imports conv_wgrad in order)
from batchai_retinanet_horovod_coco_amd.ops import conv_wgrad as CW  # noqa: E402
from batchai_retinanet_horovod_coco_amd.ops.conv_launch import geom_single, _miopen_wgrad  # noqa: E402

native.load(required=True)
dev = torch.device("cuda", 0)
for (N, H, W, cin, cout) in [(2, 6, 8, 256, 256), (2, 12, 16, 2048, 256), (2, 13, 21, 256, 256), (2, 25, 42, 2048, 256),
                             (2, 7, 9, 256, 256)]:
    pads = C.same_pads((H, W), 3, 2)
    Ho, Wo = C.out_hw((H, W), 3, 2, pads)
    g = torch.Generator().manual_seed(0)
    x = torch.randn(N, H, W, cin, generator=g).relu().to(dev).bfloat16()
    dy = torch.randn(N, Ho, Wo, cout, generator=g).to(dev).bfloat16()
    w = torch.randn(cout, 3, 3, cin, generator=g).to(dev).bfloat16()
    xr = x.float().permute(0, 3, 1, 2).contiguous()
    wr = w.float().permute(0, 3, 1, 2).contiguous().requires_grad_()
    y = F.conv2d(F.pad(xr, (pads[2], pads[3], pads[0], pads[1])), wr, stride=2)
    y.backward(dy.float().permute(0, 3, 1, 2))
    ref = wr.grad.permute(0, 2, 3, 1).contiguous().double().flatten()
    geo = geom_single(N, H, W, Ho, Wo, 3, 2, pads, cin, cout)
    cands = CW.wgrad_candidates(x, dy, geo, None)
    cands["miopen"] = lambda: _miopen_wgrad(x, w, dy, 2, pads, None)
    print("== N%d %dx%d %d->%d pads %s out %dx%d" % (N, H, W, cin, cout, pads, Ho, Wo))
    for name, fn in cands.items():
        try:
            got = fn()
            torch.cuda.synchronize()
        except Exception as e:  # noqa: BLE001
            print("  %-8s error %s" % (name, str(e)[:80]))
            continue
        got = got.double().flatten().cpu()
        r = ref.cpu()
        cos = float(torch.dot(got, r) / (got.norm() * r.norm() + 1e-30))
        print("  %-8s cosine %.6f  norm err %.2e  max err %.2e" % (
            name, cos, float((got.norm() - r.norm()).abs() / r.norm()), float((got - r).abs().max() / r.abs().max())))
