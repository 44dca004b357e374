"""Stem kernels (csrc/kernels/stem.hip + relu-aware max-pool) vs plain PyTorch fp32 references."""
import pytest
import torch
import torch.nn.functional as F

from batchai_retinanet_horovod_coco_amd import models
from batchai_retinanet_horovod_coco_amd.ops import conv as C
from batchai_retinanet_horovod_coco_amd.ops import native as N
from batchai_retinanet_horovod_coco_amd.ops import stem as S

pytestmark = pytest.mark.gpu


def _ref_stem(x, w, scale, shift, pads, pool=True):
    """fp32: pool1(relu(conv1(x) * scale + shift)) with TF-'same' pooling."""
    pt, pb, pl, pr = pads
    xp = F.pad(x.float(), (0, 0, pl, pr, pt, pb))
    y = F.conv2d(xp.permute(0, 3, 1, 2), (w.float() * scale.view(-1, 1, 1, 1)).permute(0, 3, 1, 2), None, 2)
    y = torch.relu(y + shift.view(1, -1, 1, 1))
    if not pool:
        return y.permute(0, 2, 3, 1)
    H, W = y.shape[2], y.shape[3]
    q = C.same_pads((H, W), 3, 2)
    y = F.max_pool2d(F.pad(y, (q[2], q[3], q[0], q[1]), value=float("-inf")), 3, 2)
    return y.permute(0, 2, 3, 1)


def _params(dev, seed=0):
    g = torch.Generator().manual_seed(seed)
    w = (torch.randn(64, 7, 7, 3, generator=g) * 0.1).to(dev)
    scale = (torch.rand(64, generator=g) + 0.5).to(dev)
    shift = (torch.randn(64, generator=g) * 0.2).to(dev)
    return w, scale, shift


@pytest.mark.parametrize("shape", [(1, 21, 37), (2, 64, 150), (1, 131, 266), (2, 50, 333)])
def test_stem_conv_fwd(cuda, shape):
    n, h, w_ = shape
    x = torch.randn(n, h, w_, 3, device=cuda).to(torch.bfloat16)
    w, scale, shift = _params(cuda)
    pads = (3, 3, 3, 3)
    y = S.stem_conv_fwd(x, w, scale, shift, pads, relu=True)
    ref = _ref_stem(x, w, scale, shift, pads, pool=False)
    assert y.shape == ref.shape
    err = (y.float() - ref).abs().max().item()
    assert err < 2e-2 * ref.abs().max().item() + 1e-2, err


@pytest.mark.parametrize("shape", [(2, 45, 70), (1, 160, 267), (3, 33, 300), (2, 50, 333), (1, 17, 19), (2, 130, 260)])
def test_stem_pool_fused_matches_two_kernels(cuda, shape):
    """conv1 + BN + ReLU + pool1 in one kernel (mxr_stem_pool_fwd): the pooled output and the relu-aware argmax are
    bit-identical to the stem kernel followed by the max-pool kernel (tile edges, recomputed rows, image borders)."""
    n, h, w_ = shape
    torch.manual_seed(3)
    x = (torch.randn(n, h, w_, 3, device=cuda) * 50).to(torch.bfloat16)
    w, scale, shift = _params(cuda, 2)
    shift = shift - 0.3          # some all-zero pool windows (argmax 255)
    pads = (3, 3, 3, 3)
    y1 = S.stem_conv_fwd(x, w, scale, shift, pads, relu=True)
    pool_pads = C.same_pads((y1.shape[1], y1.shape[2]), 3, 2)
    y_ref, a_ref = N.maxpool_fwd_raw(y1, 3, 2, pool_pads, relu_in=True)
    y, a, y1_shape = S.stem_pool_fwd(x, w, scale, shift, pads, pool_pads)
    torch.cuda.synchronize()
    assert y1_shape == tuple(y1.shape)
    assert torch.equal(y, y_ref)
    assert torch.equal(a, a_ref)
    assert (a == 255).any()


def test_maxpool_relu_in_masks_zero_windows(cuda):
    x = torch.relu(torch.randn(2, 9, 11, 64, device=cuda)).to(torch.bfloat16)
    x[:, :3, :3] = 0                         # a window of zeros: no gradient may flow through it
    pads = C.same_pads((9, 11), 3, 2)
    y, arg = N.maxpool_fwd_raw(x, 3, 2, pads, relu_in=True)
    assert int((arg == 255).sum()) > 0
    xr = x.float().requires_grad_(True)
    yr = F.max_pool2d(F.pad(xr.permute(0, 3, 1, 2), (pads[2], pads[3], pads[0], pads[1]), value=float("-inf")), 3, 2)
    torch.testing.assert_close(y.float(), yr.permute(0, 2, 3, 1), rtol=0, atol=0)
    dy = torch.randn_like(y)
    dx = N.maxpool_bwd_raw(dy, arg, tuple(x.shape), 3, 2, pads)
    # reference: maxpool backward, then relu backward of the producer (x > 0)
    (yr.permute(0, 2, 3, 1) * dy.float()).sum().backward()
    ref = xr.grad * (x.float() > 0)
    torch.testing.assert_close(dx.float(), ref, rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("shape", [(2, 45, 70), (1, 160, 267)])
def test_stem_fn_fwd_bwd(cuda, shape):
    n, h, w_ = shape
    torch.manual_seed(0)
    x = (torch.randn(n, h, w_, 3, device=cuda) * 50).to(torch.bfloat16)
    w, scale, shift = _params(cuda, 1)
    conv1 = models.Conv2D("conv1", 3, 64, 7, 2, 3, False, True, "he_normal", bn_name="bn_conv1").to(cuda)
    with torch.no_grad():
        conv1.weight.copy_(w)
        conv1.bn.moving_variance.copy_(1.0 / scale ** 2 - conv1.bn.eps)
        conv1.bn.moving_mean.copy_(-shift / scale)
    s_, t_ = conv1.bn.scale_shift()
    assert S.stem_ok(x, conv1)
    pool_pads = C.same_pads(conv1.out_hw((h, w_)), 3, 2)
    y = S.stem(x, conv1, pool_pads)
    wr = w.clone().requires_grad_(True)
    ref = _ref_stem(x, wr, s_, t_, (3, 3, 3, 3))
    assert y.shape == ref.shape
    torch.testing.assert_close(y.float(), ref, rtol=3e-2, atol=3e-2 * ref.abs().max().item())
    dy = torch.randn_like(ref)
    y.backward(dy.to(torch.bfloat16))
    (ref * dy.to(torch.bfloat16).float()).sum().backward()
    g, gr = conv1.weight.grad, wr.grad
    # end to end the bf16 forward moves some argmax / relu decisions vs the fp32 reference
    rel = (g - gr).norm() / gr.norm()
    assert rel < 0.1, rel.item()


@pytest.mark.parametrize("shape", [(2, 45, 70), (1, 160, 267), (3, 33, 300), (2, 50, 333)])
def test_stem_wgrad_exact_dy(cuda, shape):
    """mxr_stem_wgrad vs the fp32 conv weight gradient for the same (bf16) dy."""
    n, h, w_ = shape
    torch.manual_seed(1)
    x = (torch.randn(n, h, w_, 3, device=cuda) * 20).to(torch.bfloat16)
    Ho, Wo = (h + 6 - 7) // 2 + 1, (w_ + 6 - 7) // 2 + 1
    dy = torch.randn(n, Ho, Wo, 64, device=cuda).to(torch.bfloat16)
    scale = torch.rand(64, device=cuda) + 0.5
    dw = S.stem_wgrad(x, dy, scale, (3, 3, 3, 3))
    xp = F.pad(x.float(), (0, 0, 3, 3, 3, 3)).permute(0, 3, 1, 2)
    ref = torch.nn.grad.conv2d_weight(xp, (64, 3, 7, 7), dy.float().permute(0, 3, 1, 2), stride=2)
    ref = ref.permute(0, 2, 3, 1) * scale.view(-1, 1, 1, 1)
    rel = (dw - ref).norm() / ref.norm()
    assert rel < 1e-3, rel.item()
    acc = S.stem_wgrad(x, dy, scale, (3, 3, 3, 3), out=dw.clone())
    torch.testing.assert_close(acc, 2 * dw, rtol=1e-5, atol=1e-5)


def test_resnet_uses_stem_node(cuda):
    torch.manual_seed(0)
    m = models.backbone("resnet50").retinanet(4).to(cuda)
    x = torch.randn(1, 96, 128, 3, device=cuda).to(torch.bfloat16)
    assert C.stem_fused(x, m.backbone.conv1)
    out = m.backbone(x)
    assert out[0].grad_fn is not None or not out[0].requires_grad


@pytest.mark.parametrize("shape", [(2, 45, 70), (1, 160, 267)])
def test_stem_wgrad_pool_fused(cuda, shape):
    """Pool-fused stem wgrad (conv-output gradient gathered from pool1's gradient + argmax inside the
    staging) equals maxpool backward followed by the plain stem wgrad."""
    n, h, w_ = shape
    torch.manual_seed(3)
    x = (torch.randn(n, h, w_, 3, device=cuda) * 30).to(torch.bfloat16)
    wt, scale, shift = _params(cuda, 2)
    y1 = S.stem_conv_fwd(x, wt, scale, shift, (3, 3, 3, 3))
    pp = C.same_pads(tuple(y1.shape[1:3]), 3, 2)
    yp, arg = N.maxpool_fwd_raw(y1, 3, 2, pp, relu_in=True)
    dyp = torch.randn_like(yp)
    dy1 = N.maxpool_bwd_raw(dyp, arg, tuple(y1.shape), 3, 2, pp)
    ref = S.stem_wgrad(x, dy1, scale, (3, 3, 3, 3))
    got = S.stem_wgrad(x, dyp, scale, (3, 3, 3, 3), pool=(arg, tuple(y1.shape[1:3]), pp))
    torch.testing.assert_close(got, ref, rtol=1e-4, atol=1e-4 * ref.abs().max().item())
