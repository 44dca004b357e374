"""bf16 vs fp32 of a random-init, BN-calibrated RetinaNet-R50 on the PyTorch CPU path, per residual-branch scale
(branch2c BN gamma): cosine of the P3..P7 forward and the worst backbone / FPN parameter-gradient cosine for
fixed random gradients on P3..P7.  Shows the alpha = 1 network is chaotic under bf16 rounding (the reason
tests/test_backbone_grad_gpu.py scales its branches).  Usage: python scripts/bf16_conditioning.py 1.0 0.3 0.1"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from batchai_retinanet_horovod_coco_amd import models  # noqa: E402
from batchai_retinanet_horovod_coco_amd.models.calibrate import calibrate_from_synthetic  # noqa: E402
from batchai_retinanet_horovod_coco_amd.data.synthetic import make_batch  # noqa: E402
from batchai_retinanet_horovod_coco_amd.ops import conv as conv_ops  # noqa: E402

conv_ops.set_conv_backend("torch")
torch.manual_seed(0)
m = models.backbone("resnet50").retinanet(80)
calibrate_from_synthetic(m, torch.device("cpu"), batch=1, height=256, width=320)
x = make_batch(1, 256, 320, generator=torch.Generator().manual_seed(5))["images"]
for alpha in [float(a) for a in sys.argv[1:]]:
    st = {k: v.clone() for k, v in m.state_dict().items()}
    feats, grads = {}, {}
    for dt in (torch.float32, torch.bfloat16):
        mm = models.backbone("resnet50").retinanet(80)
        mm.load_state_dict(st)
        with torch.no_grad():
            for n, mod in mm.named_modules():
                if n.endswith("branch2c") and getattr(mod, "bn", None) is not None:
                    mod.bn.gamma.mul_(alpha)
        f = mm.features(x.to(dt))
        g = torch.Generator().manual_seed(9)
        torch.autograd.backward(f, [torch.randn(t.shape, generator=g).to(dt) for t in f])
        feats[dt] = [t.detach().float() for t in f]
        grads[dt] = {n: p.grad.double().flatten() for n, p in mm.named_parameters()
                     if p.grad is not None and not n.startswith(("classification", "regression"))}
    cs = [float(torch.nn.functional.cosine_similarity(a.flatten(), c.flatten(), 0))
          for a, c in zip(feats[torch.float32], feats[torch.bfloat16])]
    gc = sorted((float(torch.dot(a, grads[torch.bfloat16][n]) / (a.norm() * grads[torch.bfloat16][n].norm() + 1e-30)), n)
                for n, a in grads[torch.float32].items())
    print("alpha %.2f  P3..P7 %s  grad cosine worst %.4f (%s), 5th %.4f, median %.4f over %d" % (
        alpha, ["%.4f" % c for c in cs], gc[0][0], gc[0][1], gc[4][0], gc[len(gc) // 2][0], len(gc)), flush=True)
