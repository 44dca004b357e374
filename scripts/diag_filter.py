import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from batchai_retinanet_horovod_coco_amd import models
from batchai_retinanet_horovod_coco_amd.ops import anchors as anchor_ops, boxes as box_ops, native as N
cuda = torch.device("cuda", 0)
torch.manual_seed(0)
model = models.backbone("resnet18").retinanet(8).to(cuda).eval()
x = torch.randn(2, 128, 192, 3, device=cuda)
with torch.no_grad():
    model.classification_submodel.final.bias.add_(3.0)
    out = model(x)
    out2 = model(x)
print("deterministic outputs:", torch.equal(out["classification"], out2["classification"]), torch.equal(out["regression"], out2["regression"]))
anchors = anchor_ops.AnchorCache().get((128, 192), cuda, shapes_callback=anchor_ops.make_shapes_callback(model))
print("anchors", anchors.shape, "cls", out["classification"].shape, out["classification"].dtype, "reg", out["regression"].shape)
for cap in (4096, 8192):
    gb, gs, gl = N.filter_detections_batched(anchors, out["regression"], out["classification"], 128.0, 192.0, max_detections=100, cap=cap)
    boxes = box_ops.clip_boxes(box_ops.bbox_transform_inv(anchors[None], out["regression"].float()), 128, 192)
    cls = torch.sigmoid(out["classification"].float())
    for i in range(2):
        rb, rs, rl = box_ops.filter_detections(boxes[i], cls[i], True, True, 0.5, 0.05, 100, backend="torch")
        print("cap", cap, "img", i, "got", gs[i][:4].tolist(), gl[i][:4].tolist(), gb[i][0].tolist())
        print("               ref", rs[:4].tolist(), rl[:4].tolist(), rb[0].tolist())
