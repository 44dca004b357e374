"""Fused backward structure (ResidualBlockFn, masked head dgrads) vs the per-conv autograd path."""
import pytest
import torch

from batchai_retinanet_horovod_coco_amd.models.resnet import Block
from batchai_retinanet_horovod_coco_amd.models.retinanet import Submodel
from batchai_retinanet_horovod_coco_amd.ops import conv as C
from batchai_retinanet_horovod_coco_amd.ops import native as N

pytestmark = pytest.mark.gpu


def _randomize_bn(block):
    g = torch.Generator().manual_seed(3)
    for c in block.convs():
        if c.bn is not None:
            for t in c.bn.buffers():
                t.copy_(torch.rand(t.shape, generator=g) * 0.5 + 0.5)


def _run(block, x, gout):
    xx = x.detach().clone().requires_grad_()
    params = [p for p in block.parameters() if p.requires_grad]
    for p in params:
        p.grad = None
    y = block(xx)
    y.backward(gout)
    return y.detach().float(), xx.grad.float(), [p.grad.float().clone() for p in params]


@pytest.mark.parametrize("kind,cin,filters,stage,block", [("bottleneck", 256, 128, 1, 0), ("bottleneck", 256, 64, 0, 1),
                                                          ("basic", 64, 128, 1, 0), ("basic", 64, 64, 0, 1)])
def test_residual_block_fused_matches_unfused(cuda, monkeypatch, kind, cin, filters, stage, block):
    monkeypatch.setenv("MXR_CONV_FORCE", "hip")
    torch.manual_seed(0)
    blk = Block(kind, cin, filters, stage, block, False).to(cuda)
    with torch.no_grad():
        _randomize_bn(blk)
    x = torch.randn(2, 18, 27, cin, device=cuda).bfloat16()
    monkeypatch.setenv("MXR_FUSED_BLOCKS", "0")
    with torch.no_grad():
        y0 = blk(x)
    gout = torch.randn_like(y0)
    y0, dx0, g0 = _run(blk, x, gout)
    monkeypatch.setenv("MXR_FUSED_BLOCKS", "1")
    assert C.fused_blocks(x, blk.convs())
    y1, dx1, g1 = _run(blk, x, gout)
    assert torch.equal(y0, y1)
    assert (dx1 - dx0).abs().max() <= 2e-2 * dx0.abs().max()
    for a, b in zip(g1, g0):
        assert (a - b).abs().max() <= 2e-2 * b.abs().max() + 1e-6


def test_head_masked_dgrads_match_reference(cuda, monkeypatch):
    monkeypatch.setenv("MXR_CONV_FORCE", "hip")
    torch.manual_seed(1)
    sub = Submodel("classification_submodel", "pyramid_classification", 256, 256, 9 * 8, -4.59).to(cuda)
    shapes = [(10, 17), (5, 9), (3, 5), (2, 3), (1, 2)]
    xs = [torch.randn(2, h, w, 256, device=cuda).bfloat16() for (h, w) in shapes]
    packed, sh = N.pyramid_pack(xs)
    packed = packed.detach().requires_grad_()
    y = sub.forward_packed(packed, sh)
    g = torch.randn_like(y)
    y.backward(g)
    got_dx = packed.grad.float()
    got_dw = [c.weight.grad.float().clone() for c in sub.convs()]
    # fp32 reference: per-level torch convs with the same (bf16-rounded) weights
    import torch.nn.functional as F
    for c in sub.convs():
        c.weight.grad = None
    ref_in = packed.detach().float().requires_grad_()
    ws = [c.weight.detach().bfloat16().float().requires_grad_() for c in sub.convs()]
    bs = [c.bias.detach().float() for c in sub.convs()]
    outs, off = [], 0
    for (h, w) in sh:
        t = ref_in[:, off:off + h * w].reshape(2, h, w, 256).permute(0, 3, 1, 2)
        for i, (wt, b) in enumerate(zip(ws, bs)):
            t = F.conv2d(t, wt.permute(0, 3, 1, 2), b, padding=1)
            if i < 4:
                t = F.relu(t)
        outs.append(t.permute(0, 2, 3, 1).reshape(2, h * w, -1))
        off += h * w
    torch.cat(outs, 1).backward(g.float())
    assert (got_dx - ref_in.grad).abs().max() <= 3e-2 * ref_in.grad.abs().max()
    for a, wt in zip(got_dw, ws):
        assert (a - wt.grad).abs().max() <= 3e-2 * wt.grad.abs().max()
