"""Halo-staged 3x3 conv kernels (csrc/kernels/conv_halo.hip, conv_hx32.hip) vs fp32 PyTorch references on MI355X."""
import pytest
import torch
import torch.nn.functional as F

from batchai_retinanet_horovod_coco_amd.ops import native as N
from batchai_retinanet_horovod_coco_amd.ops import native_conv as NC

pytestmark = pytest.mark.gpu

VARIANTS = ["halo%d" % v for v in range(16)] + ["hx32_%d" % v for v in NC.HX32_VARIANTS]


def _ref(x, w, b=None):
    y = F.conv2d(x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), None if b is None else b.float(),
                 padding=1)
    return y.permute(0, 2, 3, 1)


def _rel(a, b):
    return ((a.float() - b).abs().max() / (b.abs().max() + 1e-3)).item()


@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("case", [(2, 17, 23, 64, 64), (2, 13, 19, 256, 256), (1, 9, 11, 256, 720),
                                  (2, 40, 170, 32, 136), (1, 3, 200, 96, 8)])
def test_halo_fwd_epilogue(cuda, variant, case):
    torch.manual_seed(3)
    n, H, W, cin, cout = case
    x = torch.randn(n, H, W, cin, device=cuda).bfloat16()
    w = (torch.randn(cout, 3, 3, cin, device=cuda) / (9 * cin) ** 0.5).bfloat16()
    b = torch.randn(cout, device=cuda)
    res = torch.randn(n, H, W, cout, device=cuda).bfloat16()
    g = N.geom_single(n, H, W, H, W, 3, 1, (1, 1, 1, 1), cin, cout)
    y = torch.empty(n, H, W, cout, device=cuda, dtype=torch.bfloat16)
    N.launch_fwd(x, w, b, res, y, g, True, variant=variant)
    assert _rel(y, torch.relu(_ref(x, w, b) + res.float())) < 2e-2
    # accumulate + relu-gradient mask (the fused dgrad epilogue)
    y0 = torch.randn_like(y)
    mk = torch.randn_like(y)
    y2 = y0.clone()
    N.launch_fwd(x, w, None, None, y2, g, False, accumulate=True, variant=variant, mask=mk)
    ref = (y0.float() + _ref(x, w)) * (mk.float() > 0)
    assert _rel(y2, ref) < 2e-2


@pytest.mark.parametrize("variant", VARIANTS)
def test_halo_pyramid_fwd_and_dgrad(cuda, variant):
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
    # data gradient through the same kernel (flipped weights), 720 -> padded 768 K like the head final
    co2 = 720
    w2 = (torch.randn(co2, 3, 3, cin, device=cuda) / (9 * co2) ** 0.5).bfloat16()
    dy = torch.randn(n, packed.shape[1], co2, device=cuda).bfloat16()
    dyp = F.pad(dy, (0, 48)).contiguous()
    wd_ = F.pad(N.flip(w2), (0, 48)).contiguous()
    gd = N.geom_pyramid(n, sh, 768, cin)
    dx = torch.empty(n, packed.shape[1], cin, device=cuda, dtype=torch.bfloat16)
    N.launch_fwd(dyp, wd_, None, None, dx, gd, False, variant=variant)
    off = 0
    for (h, wd) in sh:
        xr = torch.zeros(n, h, wd, cin, device=cuda, requires_grad=True)
        _ref(xr, w2).backward(dy[:, off:off + h * wd].reshape(n, h, wd, co2).float())
        assert _rel(dx[:, off:off + h * wd].reshape(n, h, wd, cin), xr.grad) < 3e-2
        off += h * wd


@pytest.mark.parametrize("variant", VARIANTS)
def test_halo_through_autograd(cuda, monkeypatch, variant):
    """The tuner candidate path: forced halo variant for fwd and dgrad of a 3x3 conv layer."""
    monkeypatch.setenv("MXR_CONV_FORCE", variant)
    torch.manual_seed(6)
    x = torch.randn(2, 21, 30, 128, device=cuda).bfloat16().requires_grad_()
    w = (torch.randn(64, 3, 3, 128, device=cuda) / (9 * 128) ** 0.5).bfloat16()
    y = N.conv2d(x, w, None, 1, (1, 1, 1, 1), False, None)
    g = torch.randn_like(y)
    y.backward(g)
    xr = x.detach().float().requires_grad_()
    yr = _ref(xr, w)
    yr.backward(g.float())
    assert _rel(y, yr.detach()) < 2e-2
    assert _rel(x.grad, xr.grad) < 3e-2


@pytest.mark.parametrize("variant", ["hx32_2", "hx32_3", "hx32_13", "hx32_14"])
@pytest.mark.parametrize("case", [(4, 100, 167, 256, 256), (2, 100, 167, 64, 720)])
def test_hx32_persistent_chains_many_tiles(cuda, variant, case):
    """More tiles than CUs: every block of the persistent grid walks several tiles, prefetching the next
    tile's halo / weights during the current one's last chunk (each tile's bias in its own buffer)."""
    torch.manual_seed(11)
    n, H, W, cin, cout = case
    x = torch.randn(n, H, W, cin, device=cuda).bfloat16()
    w = (torch.randn(cout, 3, 3, cin, device=cuda) / (9 * cin) ** 0.5).bfloat16()
    b = torch.randn(cout, device=cuda)
    g = N.geom_single(n, H, W, H, W, 3, 1, (1, 1, 1, 1), cin, cout)
    from batchai_retinanet_horovod_coco_amd.ops import halo as HX
    ntiles = HX.device_tiles(HX.geom_batch(g), HX.geom_shapes(g), x.device)[1]
    assert ntiles * ((cout + 255) // 256) > torch.cuda.get_device_properties(0).multi_processor_count
    y = torch.empty(n, H, W, cout, device=cuda, dtype=torch.bfloat16)
    N.launch_fwd(x, w, b, None, y, g, True, variant=variant)
    assert _rel(y, torch.relu(_ref(x, w, b))) < 2e-2
    res = torch.randn_like(y)
    y2 = torch.empty_like(y)
    N.launch_fwd(x, w, None, res, y2, g, False, variant=variant)
    assert _rel(y2, _ref(x, w) + res.float()) < 2e-2
