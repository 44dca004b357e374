"""Streaming 1x1 conv kernel (csrc/kernels/conv1x1_stream.hip) vs plain PyTorch fp32 references."""
import pytest
import torch
import torch.nn.functional as F

from batchai_retinanet_horovod_coco_amd.ops import native_conv as NC

pytestmark = pytest.mark.gpu


def _ref(x, w, b, stride, res=None, relu=False):
    y = F.conv2d(x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), None if b is None else b.float(),
                 stride)
    y = y.permute(0, 2, 3, 1)
    if res is not None:
        y = y + res.float()
    return torch.relu(y) if relu else y


@pytest.mark.parametrize("cin,cout,stride", [(64, 256, 1), (64, 64, 1), (128, 512, 1), (256, 64, 1), (256, 1024, 1),
                                             (256, 128, 2), (256, 512, 2), (128, 96, 1)])
@pytest.mark.parametrize("epi", ["plain", "res_relu", "mask_acc"])
def test_c1x1_fwd(cuda, cin, cout, stride, epi):
    torch.manual_seed(0)
    N, H, W = 2, 23, 37
    Ho, Wo = (H - 1) // stride + 1, (W - 1) // stride + 1
    x = torch.randn(N, H, W, cin, device=cuda).to(torch.bfloat16)
    w = (torch.randn(cout, 1, 1, cin, device=cuda) / cin ** 0.5).to(torch.bfloat16)
    b = torch.randn(cout, device=cuda)
    g = NC.geom_single(N, H, W, Ho, Wo, 1, stride, (0, 0, 0, 0), cin, cout)
    res = torch.randn(N, Ho, Wo, cout, device=cuda).to(torch.bfloat16) if epi == "res_relu" else None
    mask = torch.randn(N, Ho, Wo, cout, device=cuda).to(torch.bfloat16) if epi == "mask_acc" else None
    y0 = torch.randn(N, Ho, Wo, cout, device=cuda).to(torch.bfloat16)
    ref = _ref(x, w, b, stride, res, relu=epi == "res_relu")
    if epi == "mask_acc":
        ref = (ref + y0.float()) * (mask.float() > 0)
    variants = NC.c1x1_variants(g)
    assert variants
    for v in variants:
        y = y0.clone() if epi == "mask_acc" else torch.empty(N, Ho, Wo, cout, device=cuda, dtype=torch.bfloat16)
        NC.launch_fwd(x, w, b, res, y, g, epi == "res_relu", accumulate=epi == "mask_acc", variant=v, mask=mask)
        torch.testing.assert_close(y.float(), ref, rtol=2e-2, atol=2e-2 * max(1.0, ref.abs().max().item()),
                                   msg=lambda m: "%s: %s" % (v, m))


@pytest.mark.parametrize("cin,cout", [(256, 64), (512, 128), (1024, 256), (64, 64)])
def test_c1x1_dgrad(cuda, cin, cout):
    torch.manual_seed(1)
    N, H, W = 2, 19, 33
    x = torch.randn(N, H, W, cin, device=cuda).to(torch.bfloat16)
    w = (torch.randn(cout, 1, 1, cin, device=cuda) / cin ** 0.5).to(torch.bfloat16)
    dy = torch.randn(N, H, W, cout, device=cuda).to(torch.bfloat16)
    ref = torch.einsum("nhwo,oi->nhwi", dy.float(), w.float().reshape(cout, cin))
    n = 0
    for bn in NC.C1X1_BN + (65,):          # 65: the 64 slice with epilogue operands prefetched
        eb = 64 if bn == 65 else bn
        if eb * cout > 32768 or eb > max(64, cin):
            continue
        dx = NC.conv_dgrad(dy, w, tuple(x.shape), 1, (0, 0, 0, 0), "c1x1_%d" % bn)
        torch.testing.assert_close(dx.float(), ref, rtol=2e-2, atol=2e-2 * ref.abs().max().item())
        n += 1
    assert n > 0


@pytest.mark.parametrize("H,W", [(20, 34), (25, 41)])
def test_strided_dgrad_writes_gaps(cuda, H, W):
    """1x1/s2 data gradient (strided scatter): every variant writes the zeros of the unmapped positions
    itself, so a NaN-filled output comes back fully defined."""
    torch.manual_seed(2)
    N, cin, cout = 2, 128, 256
    Ho, Wo = (H - 1) // 2 + 1, (W - 1) // 2 + 1
    w = (torch.randn(cout, 1, 1, cin, device=cuda) / cin ** 0.5).to(torch.bfloat16)
    dy = torch.randn(N, Ho, Wo, cout, device=cuda).to(torch.bfloat16)
    ref = torch.nn.grad.conv2d_input((N, cin, H, W), w.float().permute(0, 3, 1, 2), dy.float().permute(0, 3, 1, 2),
                                     stride=2).permute(0, 2, 3, 1)
    wd = w.reshape(cout, cin).t().contiguous().reshape(cin, 1, 1, cout)
    g = NC.geom_single(N, Ho, Wo, Ho, Wo, 1, 1, (0, 0, 0, 0), cout, cin, ostride=2, oH=H, oW=W)
    for v in NC.FWD_VARIANTS:
        dx = torch.full((N, H, W, cin), float("nan"), device=cuda, dtype=torch.bfloat16)
        NC.launch_fwd(dy, wd, None, None, dx, g, False, variant=v)
        torch.testing.assert_close(dx.float(), ref, rtol=2e-2, atol=2e-2 * ref.abs().max().item(),
                                   msg=lambda m: "hip%d: %s" % (v, m))
