"""Experimental backbone registry (keras-retinanet vgg / mobilenet / densenet; SURVEY §2.2 E-KR-models)."""
import os

import pytest
import torch

from batchai_retinanet_horovod_coco_amd import models
from batchai_retinanet_horovod_coco_amd.io import checkpoint

# trainable parameter counts of the keras.applications notop models
NAMES = [("vgg16", 14714688), ("mobilenet128_0.5", 818592), ("densenet121", 6951808)]


@pytest.mark.parametrize("name,nparams", NAMES)
def test_backbone_shapes_and_h5_roundtrip(tmp_path, name, nparams):
    torch.manual_seed(0)
    m = models.backbone(name).retinanet(3)
    assert sum(p.numel() for p in m.backbone.parameters() if p.requires_grad) == nparams
    x = torch.randn(1, 96, 128, 3)
    m.eval()
    out = m(x)
    shapes = m.pyramid_shapes((96, 128))
    assert out["regression"].shape == (1, sum(h * w * 9 for h, w in shapes), 4)
    p = str(tmp_path / "w.h5")
    checkpoint.save_keras_h5(p, m)
    m2 = models.backbone(name).retinanet(3).eval()
    checkpoint.load_weights(m2, p)
    assert torch.equal(m(x)["classification"], m2(x)["classification"])


def test_registry_validation():
    with pytest.raises(ValueError):
        models.backbone("vgg11")
    with pytest.raises(ValueError):
        models.backbone("mobilenet100_1.0")
    assert models.backbone("mobilenet224_0.25").backbone == "mobilenet224_0.25"
    assert models.backbone("densenet169").imagenet_filename().startswith("densenet169")


@pytest.mark.parametrize("name", ["vgg16", "mobilenet128_0.25"])
def test_train_step_bf16(name):
    from batchai_retinanet_horovod_coco_amd.data.synthetic import make_batch
    from batchai_retinanet_horovod_coco_amd.ops.anchors import make_shapes_callback
    from batchai_retinanet_horovod_coco_amd.train.engine import Trainer
    torch.manual_seed(0)
    m = models.backbone(name).retinanet(3)
    tr = Trainer(m, lr=1e-4, compute_dtype=torch.bfloat16, device=torch.device("cpu"))
    tr.shapes_callback = make_shapes_callback(m)
    g = torch.Generator()
    g.manual_seed(0)
    b = make_batch(1, 64, 96, num_classes=3, max_boxes=2, generator=g)
    before = tr.flat.data.clone()
    logs = tr.train_on_batch(b["images"], b["gt"], b["gt_count"], b["image_hw"])
    assert all(float(v) == float(v) for v in logs.values())
    assert not torch.equal(before, tr.flat.data)


def test_calibrate_frozen_bn_normalises_activations():
    """Data-dependent frozen-BN init keeps a random-init ResNet's C3..C5 near unit scale and the
    classification logits near the prior-probability bias (identity BN: C5 std ~1e4)."""
    from batchai_retinanet_horovod_coco_amd.models.calibrate import calibrate_frozen_bn
    from batchai_retinanet_horovod_coco_amd.data.synthetic import make_batch
    torch.manual_seed(0)
    m = models.backbone("resnet50").retinanet(4)
    x = make_batch(1, 128, 160, device=torch.device("cpu"))["images"].float()
    with torch.no_grad():
        before = m.backbone(x)[-1].std().item()
    assert calibrate_frozen_bn(m, x) == 53
    with torch.no_grad():
        feats = m.backbone(x)
        out = m(x)
    assert before > 100
    for f in feats:
        assert 0.3 < f.std().item() < 5
    bn = m.backbone.conv1.bn
    assert torch.all(bn.gamma == 1) and torch.all(bn.moving_variance > 0)
    assert out["regression"].abs().max().item() < 1.0
