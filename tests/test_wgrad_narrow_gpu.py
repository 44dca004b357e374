"""64-channel 3x3 weight-gradient kernel (csrc/kernels/wgrad_narrow.hip) vs the fp32 PyTorch reference."""
import pytest
import torch
import torch.nn.functional as F

from batchai_retinanet_horovod_coco_amd.ops import native_conv as NC

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("shape", [(2, 37, 150), (1, 4, 64), (3, 9, 70)])
def test_wgrad3x3_c64(cuda, shape):
    n, h, w = shape
    torch.manual_seed(0)
    x = torch.randn(n, h, w, 64, device=cuda).to(torch.bfloat16)
    dy = torch.randn(n, h, w, 64, device=cuda).to(torch.bfloat16)
    scale = torch.rand(64, device=cuda) + 0.5
    dw = NC.wgrad3x3_c64(x, dy, scale)
    ref = torch.nn.grad.conv2d_weight(x.float().permute(0, 3, 1, 2), (64, 64, 3, 3), dy.float().permute(0, 3, 1, 2),
                                      padding=1)
    ref = ref.permute(0, 2, 3, 1) * scale.view(-1, 1, 1, 1)
    rel = (dw - ref).norm() / ref.norm()
    assert rel < 1e-3, rel.item()
    acc = NC.wgrad3x3_c64(x, dy, scale, out=dw.clone(), accumulate=True)
    torch.testing.assert_close(acc, 2 * dw, rtol=1e-5, atol=1e-4)
    g = NC.geom_single(n, h, w, h, w, 3, 1, (1, 1, 1, 1), 64, 64)
    assert NC.w64_covers(g) and "w64" in NC.wgrad_candidates(x, dy, g, scale)


@pytest.mark.parametrize("cin,cout,shapes", [(256, 256, [(20, 70), (10, 35), (5, 18), (3, 9), (2, 5)]),
                                             (128, 128, [(19, 131)]), (64, 720, [(9, 40), (5, 20)]),
                                             (256, 36, [(7, 66)])])
def test_halo_wgrad(cuda, cin, cout, shapes):
    """Halo-staged wgrad (csrc/kernels/wgrad_halo.hip) on single-level and packed-pyramid geometry."""
    torch.manual_seed(0)
    N = 2
    P = sum(h * w for h, w in shapes)
    x = torch.randn(N, P, cin, device=cuda).to(torch.bfloat16)
    dy = torch.randn(N, P, cout, device=cuda).to(torch.bfloat16)
    g = NC.geom_pyramid(N, shapes, cin, cout) if len(shapes) > 1 else \
        NC.geom_single(N, shapes[0][0], shapes[0][1], shapes[0][0], shapes[0][1], 3, 1, (1, 1, 1, 1), cin, cout)
    if cout < 64:
        assert not NC.whalo_covers(g)
        return
    dw = NC.halo_wgrad(x, dy, g)
    ref = torch.zeros(cout, cin, 3, 3, device=cuda)
    off = 0
    for h, w in shapes:
        xl = x[:, off:off + h * w].reshape(N, h, w, cin).float().permute(0, 3, 1, 2)
        dl = dy[:, off:off + h * w].reshape(N, h, w, cout).float().permute(0, 3, 1, 2)
        ref += torch.nn.grad.conv2d_weight(xl, (cout, cin, 3, 3), dl, padding=1)
        off += h * w
    ref = ref.permute(0, 2, 3, 1)
    rel = (dw - ref).norm() / ref.norm()
    assert rel < 2e-3, rel.item()
    acc = NC.halo_wgrad(x, dy, g, out=dw.clone(), accumulate=True)
    torch.testing.assert_close(acc, 2 * dw, rtol=1e-4, atol=1e-3)
