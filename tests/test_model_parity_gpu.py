"""Whole-model numerics on the GPU (the losses / optimizer of /root/reference/train.py:99-104).

* parity: RetinaNet-R50-FPN at 2 x 384 x 640 through the production path (bf16, every HIP kernel, fused
  losses, gradient sinks, compute-weight copies) against the plain PyTorch fp32 path (kernels off,
  MIOpen/torch convs, torch losses) on the same weights and batch: the two losses, and the gradient of every
  parameter (cosine similarity) and its norm per layer group.  The bar for the gradients is PyTorch's OWN
  bf16 path: for this random-init network the bf16 backward is intrinsically noisy (the backbone gradient
  is a near-cancelling sum -- PyTorch bf16 vs fp32 reaches a cosine of only ~0.03 there, while fp32 vs fp32
  reruns agree to 0.9999; profiles/r2_grad_parity_r50.txt), so a cosine >= 0.99 is reachable by no bf16
  implementation; the HIP path must be at least as close to fp32 as PyTorch bf16 is, per layer group;
* convergence: the HIP bf16 path overfits two fixed images (loss at least halves within 60 Adam steps at
  lr 3e-4).
"""
import math

import pytest
import torch

from batchai_retinanet_horovod_coco_amd import models
from batchai_retinanet_horovod_coco_amd.data.synthetic import make_batch
from batchai_retinanet_horovod_coco_amd.models.calibrate import calibrate_from_synthetic
from batchai_retinanet_horovod_coco_amd.ops import conv as conv_ops
from batchai_retinanet_horovod_coco_amd.ops import native
from batchai_retinanet_horovod_coco_amd.train.engine import Trainer

pytestmark = pytest.mark.gpu


def _group(name: str) -> str:
    if name.startswith("classification"):
        return "cls_head"
    if name.startswith("regression"):
        return "reg_head"
    if name.startswith("fpn"):
        return "fpn"
    return "backbone"


def _state():
    torch.manual_seed(0)
    model = models.backbone("resnet50").retinanet(80)
    calibrate_from_synthetic(model, torch.device("cpu"), batch=1, height=256, width=320)
    return {k: v.clone() for k, v in model.state_dict().items()}


def _grads(state, cuda, hip: bool, batch):
    if hip:
        native.enable()
        conv_ops.set_conv_backend("auto")
    else:
        native.disable()
        conv_ops.set_conv_backend("torch")
    try:
        model = models.backbone("resnet50").retinanet(80)
        model.load_state_dict(state)
        tr = Trainer(model, compute_dtype=torch.bfloat16 if hip else torch.float32, clip_mode="global", device=cuda)
        tr.optimizer.zero_grad()
        b = {k: v.to(cuda) for k, v in batch.items()}
        reg, cls = tr.forward_backward(b["images"], b["gt"], b["gt_count"], b["image_hw"])
        torch.cuda.synchronize()
        grads = {s.name: tr.flat.grad[s.offset:s.offset + s.numel].double().clone() for s in tr.flat.segments}
        tr.optimizer.remove_hooks()
        return float(reg), float(cls), grads
    finally:
        native.set_grad_sinks(None)
        native.set_compute_weights(None)
        native.enable()
        conv_ops.set_conv_backend("auto")


def _grads_torch_bf16(state, cuda, batch):
    native.disable()
    conv_ops.set_conv_backend("torch")
    try:
        model = models.backbone("resnet50").retinanet(80)
        model.load_state_dict(state)
        tr = Trainer(model, compute_dtype=torch.bfloat16, clip_mode="global", device=cuda)
        tr.optimizer.zero_grad()
        b = {k: v.to(cuda) for k, v in batch.items()}
        tr.forward_backward(b["images"], b["gt"], b["gt_count"], b["image_hw"])
        torch.cuda.synchronize()
        g = {s.name: tr.flat.grad[s.offset:s.offset + s.numel].double().clone() for s in tr.flat.segments}
        tr.optimizer.remove_hooks()
        return g
    finally:
        native.enable()
        conv_ops.set_conv_backend("auto")


def _group_cos(ref, g):
    out = {}
    for name, a in ref.items():
        b = g[name]
        acc = out.setdefault(_group(name), [0.0, 0.0, 0.0])
        acc[0] += float(torch.dot(a, b))
        acc[1] += float(a.norm()) ** 2
        acc[2] += float(b.norm()) ** 2
    return {k: (d / math.sqrt(aa * bb), abs(math.sqrt(bb) - math.sqrt(aa)) / math.sqrt(aa))
            for k, (d, aa, bb) in out.items()}


def test_r50_bf16_hip_matches_fp32_torch(cuda):
    state = _state()
    batch = make_batch(2, 384, 640, generator=torch.Generator().manual_seed(7))
    r32, c32, g32 = _grads(state, cuda, False, batch)
    r16, c16, g16 = _grads(state, cuda, True, batch)
    gt16 = _grads_torch_bf16(state, cuda, batch)
    print("\nlosses fp32 torch: reg %.5f cls %.5f | bf16 HIP: reg %.5f cls %.5f" % (r32, c32, r16, c16))
    assert abs(r16 - r32) <= 0.02 * abs(r32) and abs(c16 - c32) <= 0.02 * abs(c32)
    hip = _group_cos(g32, g16)
    tb = _group_cos(g32, gt16)
    for gname in sorted(hip):
        print("group %-9s cosine vs fp32: HIP bf16 %.4f  torch bf16 %.4f | norm error HIP %.4f torch bf16 %.4f" % (
            gname, hip[gname][0], tb[gname][0], hip[gname][1], tb[gname][1]))
    for gname in hip:
        assert hip[gname][0] >= tb[gname][0] - 0.05, gname
        assert hip[gname][1] <= max(0.10, tb[gname][1] + 0.05), gname
    # the layers next to the loss, where bf16 noise has not compounded yet, agree closely
    for name in ("classification_submodel.final.weight", "classification_submodel.final.bias",
                 "regression_submodel.final.weight", "regression_submodel.final.bias"):
        a, b = g32[name], g16[name]
        c = float(torch.dot(a, b) / (a.norm() * b.norm()))
        print("%-40s cosine %.5f" % (name, c))
        assert c >= 0.95, name


def test_r50_hip_overfits_two_images(cuda):
    native.enable()
    conv_ops.set_conv_backend("auto")
    state = _state()
    model = models.backbone("resnet50").retinanet(80)
    model.load_state_dict(state)
    tr = Trainer(model, lr=3e-4, clipnorm=0.001, compute_dtype=torch.bfloat16, clip_mode="global", device=cuda)
    try:
        b = {k: v.to(cuda) for k, v in make_batch(2, 256, 384, generator=torch.Generator().manual_seed(3)).items()}
        losses = []
        for _ in range(60):
            logs = tr.train_on_batch(b["images"], b["gt"], b["gt_count"], b["image_hw"])
            losses.append(float(logs["loss"]))
        print("\noverfit losses", ["%.3f" % v for v in losses[::5]], "%.3f" % losses[-1])
        assert all(math.isfinite(v) for v in losses)
        assert min(losses[-10:]) <= 0.5 * losses[0], losses
    finally:
        tr.optimizer.remove_hooks()
        native.set_grad_sinks(None)
        native.set_compute_weights(None)
