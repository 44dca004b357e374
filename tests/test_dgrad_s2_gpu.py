"""HIP data gradient of the FPN's 3x3 / stride-2 convs (P6: 2048 -> 256 on C5, P7: 256 -> 256 on P6) by
sub-pixel phases (native_conv._dgrad_s2_subpixel) against the fp32 PyTorch gradient of the same conv."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

SHAPES = [(2, 25, 42, 2048, 256, (1, 1, 0, 1)), (2, 13, 21, 256, 256, (1, 1, 1, 1)),
          (16, 25, 42, 2048, 256, (1, 1, 0, 1))]


def _ref(x, w, dy, pads):
    """fp32 dX (NHWC) of y = conv(pad(x), w, stride 2)."""
    xr = x.float().permute(0, 3, 1, 2).contiguous().requires_grad_()
    wr = w.float().permute(0, 3, 1, 2)
    y = F.conv2d(F.pad(xr, (pads[2], pads[3], pads[0], pads[1])), wr, stride=2)
    y.backward(dy.float().permute(0, 3, 1, 2))
    return xr.grad.permute(0, 2, 3, 1)


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("variant", [0, 1, 3, 8, 11, 13, 16])
def test_s2_dgrad_matches_fp32(cuda, shape, variant):
    from batchai_retinanet_horovod_coco_amd.ops import native_conv as NC
    N, H, W, cin, cout, pads = shape
    if N > 2 and variant not in (11, 13):
        pytest.skip("production batch: the tuner's usual winners only")
    g = torch.Generator(device="cpu").manual_seed(variant)
    x = torch.randn(N, H, W, cin, generator=g).to(cuda).bfloat16()
    w = (torch.randn(cout, 3, 3, cin, generator=g) / (9 * cin) ** 0.5).to(cuda).bfloat16()
    Ho = (H + pads[0] + pads[1] - 3) // 2 + 1
    Wo = (W + pads[2] + pads[3] - 3) // 2 + 1
    dy = torch.randn(N, Ho, Wo, cout, generator=g).to(cuda).bfloat16()
    ref = _ref(x, w, dy, pads)
    dx = NC.conv_dgrad(dy, w, tuple(x.shape), 2, pads, variant)
    torch.cuda.synchronize()
    err = (dx.float() - ref).abs().max() / ref.abs().max()
    assert err < 1e-2, float(err)
    # fused relu mask + accumulation into an existing buffer (the GradJoin form on C5)
    base = torch.randn(N, H, W, cin, generator=g).to(cuda).bfloat16()
    acc = base.clone()
    NC.conv_dgrad(dy, w, tuple(x.shape), 2, pads, variant, mask=x, out=acc)
    want = torch.where(x.float() > 0, base.float() + ref, torch.zeros_like(ref))
    err = (acc.float() - want).abs().max() / want.abs().max()
    assert err < 1e-2, float(err)


@pytest.mark.parametrize("pads", [(1, 1, 0, 1), (1, 1, 1, 1), (0, 1, 0, 1)])
def test_s2_stack_kernel_matches_torch(cuda, pads):
    from batchai_retinanet_horovod_coco_amd.ops import native_conv as NC
    w = torch.randn(96, 3, 3, 40, device=cuda).bfloat16()
    w4, win = NC._s2_stacked_weights_hip(w, pads)
    ref, win_ref = NC._s2_stacked_weights(w, pads)
    torch.cuda.synchronize()
    assert win == win_ref
    assert torch.equal(w4, ref)


@pytest.mark.parametrize("pads", [(1, 1, 0, 1), (1, 1, 1, 1), (0, 1, 0, 1)])
def test_s2_stack_from_flipped_copy_matches_torch(cuda, pads):
    """mxr_s2_stack_flip: the stacked weights as row copies of the flip-transposed weights (the batched flip the
    data gradients already use) equal the torch construction bit for bit."""
    import ctypes
    from batchai_retinanet_horovod_coco_amd.ops import native_conv as NC
    from batchai_retinanet_horovod_coco_amd.ops.native import _chk, _p, _s, lib
    cout, cin = 96, 40
    w = torch.randn(cout, 3, 3, cin, device=cuda).bfloat16()
    wd = w.flip(1, 2).permute(3, 1, 2, 0).contiguous()          # [ci][ky][kx][co] of the flipped kernel
    taps, win = NC._s2_stack_taps(pads)
    w4 = torch.empty((4 * cin, 2, 2, cout), dtype=w.dtype, device=cuda)
    _chk(lib().mxr_s2_stack_flip(_p(wd), _p(w4), cin, cout, (ctypes.c_int * 16)(*taps), _s()), "s2_stack_flip")
    ref, win_ref = NC._s2_stacked_weights(w, pads)
    torch.cuda.synchronize()
    assert tuple(win) == tuple(win_ref)
    assert torch.equal(w4, ref)
