"""Phase-pipelined 256x256 implicit-GEMM conv (csrc/kernels/conv_p8.hip) vs fp32 PyTorch references."""
import pytest
import torch
import torch.nn.functional as F

from batchai_retinanet_horovod_coco_amd.ops import native as N

pytestmark = pytest.mark.gpu

VARIANTS = ["p8_0", "p8_1", "p8_2", "p8_3", "p8_4", "p8_5", "p8_6", "p8_7", "p8_8", "p8_10"]


def _ref(x, w, b=None, stride=1, pad=1):
    y = F.conv2d(x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), None if b is None else b.float(),
                 stride=stride, padding=pad)
    return y.permute(0, 2, 3, 1)


def _rel(a, b):
    return ((a.float() - b).abs().max() / (b.abs().max() + 1e-3)).item()


@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("case", [(2, 17, 23, 64, 64, 3, 1), (2, 13, 19, 256, 256, 3, 1), (1, 9, 11, 256, 720, 3, 1),
                                  (1, 21, 30, 128, 512, 1, 1), (2, 16, 18, 512, 256, 3, 2), (1, 5, 7, 2048, 512, 1, 2),
                                  (3, 40, 70, 64, 136, 3, 1)])
def test_p8_fwd_epilogue(cuda, variant, case):
    torch.manual_seed(3)
    n, H, W, cin, cout, k, s = case
    p = k // 2
    Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    x = torch.randn(n, H, W, cin, device=cuda).bfloat16()
    w = (torch.randn(cout, k, k, cin, device=cuda) / (k * k * cin) ** 0.5).bfloat16()
    b = torch.randn(cout, device=cuda)
    res = torch.randn(n, Ho, Wo, cout, device=cuda).bfloat16()
    g = N.geom_single(n, H, W, Ho, Wo, k, s, (p, p, p, p), cin, cout)
    y = torch.empty(n, Ho, Wo, cout, device=cuda, dtype=torch.bfloat16)
    N.launch_fwd(x, w, b, res, y, g, True, variant=variant)
    assert _rel(y, torch.relu(_ref(x, w, b, s, p) + res.float())) < 2e-2
    y0 = torch.randn_like(y)
    mk = torch.randn_like(y)
    y2 = y0.clone()
    N.launch_fwd(x, w, None, None, y2, g, False, accumulate=True, variant=variant, mask=mk)
    assert _rel(y2, (y0.float() + _ref(x, w, None, s, p)) * (mk.float() > 0)) < 2e-2


@pytest.mark.parametrize("variant", VARIANTS)
def test_p8_pyramid_fwd_and_dgrad(cuda, variant):
    torch.manual_seed(4)
    shapes = [(10, 17), (5, 9), (3, 5), (2, 3), (1, 2)]
    n, cin, cout = 3, 256, 256
    xs = [torch.randn(n, h, w, cin, device=cuda).bfloat16() for (h, w) in shapes]
    packed, sh = N.pyramid_pack(xs)
    w = (torch.randn(cout, 3, 3, cin, device=cuda) / (9 * cin) ** 0.5).bfloat16()
    b = torch.randn(cout, device=cuda)
    g = N.geom_pyramid(n, sh, cin, cout)
    y = torch.empty(n, packed.shape[1], cout, device=cuda, dtype=torch.bfloat16)
    N.launch_fwd(packed, w, b, None, y, g, True, variant=variant)
    off = 0
    for x, (h, wd) in zip(xs, sh):
        yl = y[:, off:off + h * wd].reshape(n, h, wd, cout)
        assert _rel(yl, torch.relu(_ref(x, w, b))) < 2e-2
        off += h * wd


@pytest.mark.parametrize("variant", VARIANTS)
def test_p8_production_head_shape(cuda, variant):
    """The tuner's head-tower key at the bench's real shape (B = 16 at 800x1333: M = 356,800 pixels,
    256 -> 256, K = 2,304), checked on a strided sample of output rows against an fp32 reference."""
    torch.manual_seed(5)
    shapes = [(100, 167), (50, 84), (25, 42), (13, 21), (7, 11)]
    n, cin, cout = 16, 256, 256
    P = sum(h * w for h, w in shapes)
    packed = torch.randn(n, P, cin, device=cuda).bfloat16()
    w = (torch.randn(cout, 3, 3, cin, device=cuda) / (9 * cin) ** 0.5).bfloat16()
    g = N.geom_pyramid(n, shapes, cin, cout)
    y = torch.empty(n, P, cout, device=cuda, dtype=torch.bfloat16)
    N.launch_fwd(packed, w, None, None, y, g, False, variant=variant)
    for img in (0, 7, 15):
        off = 0
        for (h, wd) in shapes:
            x = packed[img:img + 1, off:off + h * wd].reshape(1, h, wd, cin)
            ref = _ref(x, w)
            assert _rel(y[img:img + 1, off:off + h * wd].reshape(1, h, wd, cout), ref) < 2e-2, (img, h, wd)
            off += h * wd
