"""Per-parameter gradient difference: GradJoin on vs off (and off vs off as the rounding baseline)."""
import copy
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from batchai_retinanet_horovod_coco_amd import models  # noqa: E402
from batchai_retinanet_horovod_coco_amd.data.synthetic import make_batch  # noqa: E402
from batchai_retinanet_horovod_coco_amd.train.engine import Trainer  # noqa: E402

os.environ["MXR_CONV_FORCE"] = "hip"
dev = torch.device("cuda", 0)
torch.manual_seed(0)
base = models.backbone(sys.argv[1] if len(sys.argv) > 1 else "resnet50").retinanet(8)
g = torch.Generator().manual_seed(0)
b = make_batch(2, 160, 224, num_classes=8, max_boxes=3, generator=g)
res = {}
for tag, join in (("join", "1"), ("plain", "0"), ("plain2", "0")):
    os.environ["MXR_GRAD_JOIN"] = join
    tr = Trainer(copy.deepcopy(base), lr=0.0, clipnorm=0.0, compute_dtype=torch.bfloat16, device=dev,
                 clip_mode="global")
    tr.train_on_batch(b["images"], b["gt"], b["gt_count"], b["image_hw"])
    res[tag] = (tr.flat.grad.clone(), [(s.param, s.offset, s.numel) for s in tr.flat.segments], tr)
names = {id(p): n for n, p in res["join"][2].model.named_parameters()}
gj, segs, _ = res["join"]
gp = res["plain"][0]
gp2 = res["plain2"][0]
rows = []
for p, o, n in segs:
    a, c, d = gj[o:o + n], gp[o:o + n], gp2[o:o + n]
    den = c.norm().item() + 1e-12
    rows.append(((a - c).norm().item() / den, (d - c).norm().item() / den, names.get(id(p), "?"), den))
rows.sort(reverse=True)
for r in rows[:25]:
    print("join-vs-plain %.2e  plain-vs-plain %.2e  |g| %.3e  %s" % (r[0], r[1], r[3], r[2]))
