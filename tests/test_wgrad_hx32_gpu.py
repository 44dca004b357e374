"""conv_wgrad_hx32 (csrc/kernels/conv_wgrad_hx32.hip): halo-staged 3x3 weight gradient on the 32x32x16 MFMA
vs fp32 PyTorch references on MI355X -- single levels and the packed head pyramid, partial co tiles, padded
dY rows, the fused bias gradient, accumulation into an existing gradient and the frozen-BN scale."""
import pytest
import torch
import torch.nn.functional as F

from batchai_retinanet_horovod_coco_amd.ops import native as N

pytestmark = pytest.mark.gpu


def _ref_wgrad(x, dy, cout):
    """fp32 dW (cout, 3, 3, cin) of a 3x3 / s1 / p1 conv: x [n, h, w, cin], dy [n, h, w, >= cout]."""
    xr = x.float().permute(0, 3, 1, 2)
    w = torch.zeros(cout, x.shape[-1], 3, 3, device=x.device, requires_grad=True)
    F.conv2d(xr, w, padding=1).backward(dy[..., :cout].float().permute(0, 3, 1, 2))
    return w.grad.permute(0, 2, 3, 1)


def _rel(a, b):
    return ((a.float() - b).abs().max() / (b.abs().max() + 1e-6)).item()


@pytest.mark.parametrize("case", [(2, 17, 23, 64, 64), (2, 13, 19, 256, 256), (1, 9, 11, 256, 720),
                                  (2, 40, 170, 32, 136), (1, 3, 200, 96, 8), (3, 50, 84, 256, 256)])
@pytest.mark.parametrize("splits", [None, 1, 3])
@pytest.mark.parametrize("variant", [0, 1, 2, 3, 4, 5])
def test_wgrad_hx32_single_level(cuda, case, splits, variant):
    torch.manual_seed(5)
    n, H, W, cin, cout = case
    x = torch.randn(n, H, W, cin, device=cuda).bfloat16()
    dy = torch.randn(n, H, W, cout, device=cuda).bfloat16()
    g = N.geom_single(n, H, W, H, W, 3, 1, (1, 1, 1, 1), cin, cout)
    dw = N.hx32_wgrad(x, dy, g, splits=splits, variant=variant)
    assert _rel(dw, _ref_wgrad(x, dy, cout)) < 1e-2


@pytest.mark.parametrize("cout,ldy", [(256, 256), (720, 768), (64, 64), (36, 64)])
@pytest.mark.parametrize("variant", [0, 1, 2, 3, 4, 5])
def test_wgrad_hx32_pyramid_bias_accumulate(cuda, cout, ldy, variant):
    """The head layers: packed pyramid, zero-padded dY rows past cout, bias gradient from the one-hot MFMA,
    both accumulated onto existing values; the weight gradient equals the bias-free launch bit for bit."""
    torch.manual_seed(6)
    shapes = [(20, 34), (10, 17), (5, 9), (3, 5), (2, 3)]
    n, cin = 2, 256
    xs = [torch.randn(n, h, w, cin, device=cuda).bfloat16() for (h, w) in shapes]
    packed, sh = N.pyramid_pack(xs)
    dy = torch.randn(n, packed.shape[1], ldy, device=cuda).bfloat16()
    dy[..., cout:] = 0
    g = N.geom_pyramid(n, sh, cin, ldy if cout % 8 else cout)
    gco = g.cout
    dw_plain = N.hx32_wgrad(packed, dy, g, variant=variant)
    w0 = torch.randn(gco, 3, 3, cin, device=cuda)
    b0 = torch.randn(gco, device=cuda)
    dw, db = w0.clone(), b0.clone()
    N.hx32_wgrad(packed, dy, g, out=dw, accumulate=True, bias_out=db, bias_accumulate=True, variant=variant)
    torch.cuda.synchronize()
    off = 0
    ref = torch.zeros(gco, 3, 3, cin, device=cuda)
    for x, (h, w) in zip(xs, sh):
        ref += _ref_wgrad(x, dy[:, off:off + h * w].reshape(n, h, w, ldy), gco)
        off += h * w
    assert _rel(dw_plain, ref) < 1e-2
    assert torch.allclose(dw - w0, dw_plain, atol=1e-4 * float(ref.abs().max()), rtol=0)
    refb = dy[..., :gco].float().sum((0, 1))
    assert ((db - b0) - refb).abs().max() / refb.abs().max() < 1e-4


def test_wgrad_hx32_scale_matches_unscaled(cuda):
    """The frozen-BN scale (backbone 3x3 convs) multiplies row co of dW in the reduce."""
    torch.manual_seed(7)
    n, H, W, cin, cout = 2, 25, 42, 128, 128
    x = torch.randn(n, H, W, cin, device=cuda).bfloat16()
    dy = torch.randn(n, H, W, cout, device=cuda).bfloat16()
    sc = torch.rand(cout, device=cuda) + 0.5
    g = N.geom_single(n, H, W, H, W, 3, 1, (1, 1, 1, 1), cin, cout)
    dw = N.hx32_wgrad(x, dy, g, scale=sc)
    assert _rel(dw, _ref_wgrad(x, dy, cout) * sc.view(-1, 1, 1, 1)) < 1e-2


def test_wgrad_hx32_matches_p8_production_pyramid(cuda):
    """At the production head shape (16 x 800 x 1333 pyramid, 256 -> 256) the new kernel agrees with the
    tuned p8 kernel (both fp32-accumulated bf16 GEMMs; only the summation order differs)."""
    torch.manual_seed(8)
    shapes = [(100, 167), (50, 84), (25, 42), (13, 21), (7, 11)]
    n, cin, cout = 16, 256, 256
    P = sum(h * w for h, w in shapes)
    x = torch.randn(n, P, cin, device=cuda).bfloat16()
    dy = (torch.randn(n, P, cout, device=cuda) * 0.1).bfloat16()
    g = N.geom_pyramid(n, shapes, cin, cout)
    a = N.hx32_wgrad(x, dy, g)
    b = N.conv_wgrad(x, dy, g, None, variant=23)
    assert _rel(N.hx32_wgrad(x, dy, g, variant=0), b) < 2e-3
    assert _rel(a, b) < 2e-3
