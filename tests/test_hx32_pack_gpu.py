"""Batched hx32 weight packing (ComputeWeights.hx32_packed -> mxr_hx32_pack_batch): every packed copy the
step serves equals the per-call pack (mxr_hx32_pack_weights) of the same compute weight -- forward and
flipped data-gradient copies -- and is refreshed after an optimizer step rewrote the weights."""
import pytest
import torch

from batchai_retinanet_horovod_coco_amd import models
from batchai_retinanet_horovod_coco_amd.data.synthetic import make_batch
from batchai_retinanet_horovod_coco_amd.ops import native
from batchai_retinanet_horovod_coco_amd.ops.native import _chk, _p, _s, lib
from batchai_retinanet_horovod_coco_amd.train.engine import Trainer

pytestmark = pytest.mark.gpu


def _per_call(w):
    co, _, _, ci = w.shape
    wp = torch.empty(w.numel(), dtype=w.dtype, device=w.device)
    _chk(lib().mxr_hx32_pack_weights(_p(w), _p(wp), co, ci, _s()), "hx32_pack")
    return wp


def _check_all(cw):
    checked = 0
    for seg in cw.flat.segments:
        if len(seg.shape) != 4 or tuple(seg.shape[1:3]) != (3, 3):
            continue
        fwd = cw.plan.copy[seg.offset:seg.offset + seg.numel].view(seg.shape)
        for w in (fwd, cw.flipped(fwd)):
            got = cw.hx32_packed(w)
            if got is None:
                continue
            torch.cuda.synchronize()
            assert torch.equal(got, _per_call(w)), tuple(w.shape)
            checked += 1
    return checked


def test_batched_pack_matches_per_call_and_follows_updates(cuda):
    native.load(required=True)
    torch.manual_seed(0)
    model = models.backbone("resnet18").retinanet(8)
    tr = Trainer(model, compute_dtype=torch.bfloat16, clip_mode="global", device=cuda, lr=1e-2)
    try:
        cw = tr.compute_weights
        assert cw is not None
        n0 = _check_all(cw)
        assert n0 >= 20          # heads, FPN and backbone 3x3 layers, both directions
        b = make_batch(2, 128, 160, device=cuda)
        tr.train_on_batch(b["images"], b["gt"], b["gt_count"], b["image_hw"])
        torch.cuda.synchronize()
        assert _check_all(cw) == n0
    finally:
        tr.optimizer.remove_hooks()
        native.set_grad_sinks(None)
        native.set_compute_weights(None)
