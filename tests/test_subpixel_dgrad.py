"""CPU check of the sub-pixel split behind the HIP stride-2 3x3 data gradient (native_conv._dgrad_s2_subpixel):
the four phase convolutions, built from the same tap / pad rule and scattered into the parity classes,
reproduce autograd's data gradient of a TF-'same' stride-2 3x3 conv (FPN P6 / P7 paddings)."""
import pytest
import torch
import torch.nn.functional as F

from batchai_retinanet_horovod_coco_amd.ops.native_conv import _s2_phase_taps


@pytest.mark.parametrize("H,W,pads", [(25, 42, (1, 1, 0, 1)), (13, 21, (1, 1, 1, 1)), (8, 9, (0, 1, 0, 1)),
                                      (7, 6, (1, 1, 0, 1))])
def test_subpixel_split_matches_autograd(H, W, pads):
    torch.manual_seed(0)
    N, cin, cout = 2, 3, 4
    x = torch.randn(N, cin, H, W, dtype=torch.float64, requires_grad=True)
    w = torch.randn(cout, cin, 3, 3, dtype=torch.float64)
    y = F.conv2d(F.pad(x, (pads[2], pads[3], pads[0], pads[1])), w, stride=2)
    dy = torch.randn_like(y)
    y.backward(dy)
    Ho, Wo = y.shape[2], y.shape[3]
    dx = torch.full((N, cin, H, W), float("nan"), dtype=torch.float64)
    for py in (0, 1):
        kys, pad_y = _s2_phase_taps(py, pads[0])
        Hp = (H - py + 1) // 2
        for px in (0, 1):
            kxs, pad_x = _s2_phase_taps(px, pads[2])
            Wp = (W - px + 1) // 2
            # phase conv: out[a, b] = sum_t dY[a - pad_y + ty, b - pad_x + tx] W[:, :, kys[ty], kxs[tx]]^T
            wp = w[:, :, kys][:, :, :, kxs].transpose(0, 1)          # (cin, cout, ty, tx)
            lo_y, lo_x = pad_y, pad_x
            hi_y = max(0, Hp - 1 - pad_y + len(kys) - Ho)
            hi_x = max(0, Wp - 1 - pad_x + len(kxs) - Wo)
            src = F.pad(dy, (lo_x, hi_x, lo_y, hi_y))
            ph = F.conv2d(src, wp)[:, :, :Hp, :Wp]
            dx[:, :, py::2, px::2] = ph
    torch.testing.assert_close(dx, x.grad, rtol=1e-10, atol=1e-10)


@pytest.mark.parametrize("H,W,pads", [(25, 42, (1, 1, 0, 1)), (13, 21, (1, 1, 1, 1)), (8, 9, (0, 1, 0, 1)),
                                      (7, 6, (1, 1, 0, 1))])
def test_phase_stacked_2x2_conv_matches_autograd(H, W, pads):
    """The HIP path's single launch: the phases stacked as 4 x cin output channels of one 2x2 conv over dY
    (native_conv._s2_stacked_weights), then the pixel shuffle of mxr_s2_shuffle."""
    from batchai_retinanet_horovod_coco_amd.ops.native_conv import _s2_stacked_weights
    torch.manual_seed(1)
    N, cin, cout = 2, 3, 4
    x = torch.randn(N, cin, H, W, dtype=torch.float64, requires_grad=True)
    w = torch.randn(cout, cin, 3, 3, dtype=torch.float64)
    y = F.conv2d(F.pad(x, (pads[2], pads[3], pads[0], pads[1])), w, stride=2)
    dy = torch.randn_like(y)
    y.backward(dy)
    w4, (pt, pl) = _s2_stacked_weights(w.permute(0, 2, 3, 1), pads)
    Hp, Wp = (H + 1) // 2, (W + 1) // 2
    Ho, Wo = y.shape[2], y.shape[3]
    dyp = F.pad(dy, (pl, max(0, Wp + 1 - pl - Wo), pt, max(0, Hp + 1 - pt - Ho)))
    y4 = F.conv2d(dyp, w4.permute(0, 3, 1, 2))[:, :, :Hp, :Wp]
    dx = torch.empty(N, cin, H, W, dtype=torch.float64)
    for py in (0, 1):
        for px in (0, 1):
            p = 2 * py + px
            d = dx[:, :, py::2, px::2]
            d.copy_(y4[:, p * cin:(p + 1) * cin, :d.shape[2], :d.shape[3]])
    torch.testing.assert_close(dx, x.grad)


@pytest.mark.parametrize("pads", [(1, 1, 0, 1), (1, 1, 1, 1), (0, 1, 0, 1), (0, 1, 1, 1)])
def test_stack_tap_table_matches_stacked_weights(pads):
    """mxr_s2_stack's 16-entry tap table (phase x window slot -> 3x3 tap) rebuilds _s2_stacked_weights."""
    from batchai_retinanet_horovod_coco_amd.ops.native_conv import _s2_stack_taps, _s2_stacked_weights
    torch.manual_seed(2)
    cout, cin = 4, 5
    w = torch.randn(cout, 3, 3, cin)
    taps, win = _s2_stack_taps(pads)
    w4, win_ref = _s2_stacked_weights(w, pads)
    assert win == win_ref
    emu = torch.zeros(4 * cin, 2, 2, cout)
    for p in range(4):
        for slot in range(4):
            t = taps[4 * p + slot]
            if t >= 0:
                emu[p * cin:(p + 1) * cin, slot // 2, slot % 2] = w[:, t // 3, t % 3].t()
    assert torch.equal(emu, w4)
