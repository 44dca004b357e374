"""Persistent streaming 1x1 conv kernel (csrc/kernels/conv1x1_pers.hip) vs plain PyTorch fp32 references: every
epilogue form (bias, residual, relu, accumulate, bf16 mask, bitmask read and write), tails in both M and N, K from
96 to 2048, several tiles per block (the cross-tile DMA stream) and the data-gradient direction."""
import pytest
import torch
import torch.nn.functional as F

from batchai_retinanet_horovod_coco_amd.ops import native_conv as NC
from batchai_retinanet_horovod_coco_amd.ops.conv_launch import BitMask, c1p_covers

pytestmark = pytest.mark.gpu


def _ref(x, w, b, res=None, relu=False):
    y = F.conv2d(x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), None if b is None else b.float())
    y = y.permute(0, 2, 3, 1)
    if res is not None:
        y = y + res.float()
    return torch.relu(y) if relu else y


def _bits_of(t):
    """The reference BitMask bytes of a bf16 activation (bit j of byte i: element 8 i + j > 0)."""
    v = (t.reshape(-1, 8) > 0).to(torch.int32)
    return (v << torch.arange(8, device=t.device, dtype=torch.int32)).sum(1).to(torch.uint8)


@pytest.mark.parametrize("cin,cout,N,H,W", [(256, 1024, 2, 23, 37), (1024, 256, 3, 19, 40), (96, 200, 1, 17, 31),
                                            (512, 2048, 1, 9, 13), (128, 512, 2, 41, 50), (2048, 512, 1, 11, 17),
                                            (256, 64, 2, 13, 21)])
@pytest.mark.parametrize("epi", ["plain", "bias_relu", "res_relu", "res_relu_bits", "mask_acc", "bits_acc", "mask",
                                 "acc"])
def test_c1p_fwd_epilogues(cuda, cin, cout, N, H, W, epi):
    torch.manual_seed(0)
    x = torch.randn(N, H, W, cin, device=cuda).to(torch.bfloat16)
    w = (torch.randn(cout, 1, 1, cin, device=cuda) / cin ** 0.5).to(torch.bfloat16)
    b = torch.randn(cout, device=cuda) if epi in ("bias_relu", "res_relu", "res_relu_bits") else None
    g = NC.geom_single(N, H, W, H, W, 1, 1, (0, 0, 0, 0), cin, cout)
    assert c1p_covers(g)
    relu = epi.startswith(("bias_relu", "res_relu"))
    res = torch.randn(N, H, W, cout, device=cuda).to(torch.bfloat16) if epi.startswith("res") else None
    act = torch.randn(N, H, W, cout, device=cuda).to(torch.bfloat16)      # a relu output whose mask applies
    y0 = torch.randn(N, H, W, cout, device=cuda).to(torch.bfloat16)
    acc = epi in ("mask_acc", "bits_acc", "acc")
    ref = _ref(x, w, b, res, relu)
    if acc:
        ref = ref + y0.float()
    if epi in ("mask_acc", "bits_acc", "mask"):
        ref = ref * (act.float() > 0)
    mask = None
    if epi in ("mask_acc", "mask"):
        mask = act
    elif epi == "bits_acc":
        mask = BitMask(act)
        mask.bits.copy_(_bits_of(act))
    elif epi == "res_relu_bits":
        mask = BitMask(shape=(N, H, W, cout), device=cuda)
        mask.bits.fill_(0xA5)
    y = y0.clone() if acc else torch.full((N, H, W, cout), float("nan"), device=cuda, dtype=torch.bfloat16)
    NC.launch_fwd(x, w, b, res, y, g, relu, accumulate=acc, variant="c1p", mask=mask)
    torch.cuda.synchronize()
    tol = 2e-2 * max(1.0, ref.abs().max().item())
    torch.testing.assert_close(y.float(), ref, rtol=2e-2, atol=tol)
    if epi == "res_relu_bits":
        # the written mask bits are exactly those of the stored (bf16) output
        assert torch.equal(mask.bits, _bits_of(y))


@pytest.mark.parametrize("cin,cout", [(1024, 256), (512, 128), (256, 1024), (2048, 512), (512, 2048)])
@pytest.mark.parametrize("form", ["plain", "mask", "bits_acc"])
def test_c1p_dgrad(cuda, cin, cout, form):
    torch.manual_seed(1)
    N, H, W = 2, 19, 33
    x = torch.randn(N, H, W, cin, device=cuda).to(torch.bfloat16)     # the forward input (a relu output)
    w = (torch.randn(cout, 1, 1, cin, device=cuda) / cin ** 0.5).to(torch.bfloat16)
    dy = torch.randn(N, H, W, cout, device=cuda).to(torch.bfloat16)
    ref = torch.einsum("nhwo,oi->nhwi", dy.float(), w.float().reshape(cout, cin))
    out = None
    mask = None
    if form == "mask":
        mask = x
        ref = ref * (x.float() > 0)
    elif form == "bits_acc":
        out = torch.randn(N, H, W, cin, device=cuda).to(torch.bfloat16)
        ref = (ref + out.float()) * (x.float() > 0)
        mask = BitMask(x)
        mask.bits.copy_(_bits_of(x))
    dx = NC.conv_dgrad(dy, w, tuple(x.shape), 1, (0, 0, 0, 0), "c1p", mask=mask, out=out)
    torch.cuda.synchronize()
    torch.testing.assert_close(dx.float(), ref, rtol=2e-2, atol=2e-2 * max(1.0, ref.abs().max().item()))


def test_c1p_many_tiles_per_block(cuda):
    """More tiles than CUs (several tiles per persistent block) and an M tail: the DMA stream crosses tile
    boundaries, the epilogue operands of each tile are its own."""
    torch.manual_seed(2)
    N, H, W, cin, cout = 4, 100, 167, 256, 1024     # 66,800 pixels: 261 x 8 tiles
    x = torch.randn(N, H, W, cin, device=cuda).to(torch.bfloat16)
    w = (torch.randn(cout, 1, 1, cin, device=cuda) / cin ** 0.5).to(torch.bfloat16)
    b = torch.randn(cout, device=cuda)
    res = torch.randn(N, H, W, cout, device=cuda).to(torch.bfloat16)
    g = NC.geom_single(N, H, W, H, W, 1, 1, (0, 0, 0, 0), cin, cout)
    y = torch.empty(N, H, W, cout, device=cuda, dtype=torch.bfloat16)
    NC.launch_fwd(x, w, b, res, y, g, True, variant="c1p")
    torch.cuda.synchronize()
    ref = _ref(x, w, b, res, True)
    torch.testing.assert_close(y.float(), ref, rtol=2e-2, atol=2e-2 * ref.abs().max().item())
