"""ReLU masks as bits (ops.conv_launch.BitMask, csrc/kernels/conv_common.h epi_mask8).

* every bit-capable forward candidate, given a BitMask with relu on, stores exactly the output it stores
  without one and writes bits == (y > 0);
* every bit-capable data-gradient candidate gives bit-identical dX with the bitmask of x and with x itself
  as the mask (plain, accumulating, and the 1x1/s2 scatter of the GradJoin form);
* the fused ResNet block path (ResidualBlockFn) really hands the bitmask to the next block's 1x1 dgrad.
Numerics against fp32 PyTorch are covered by tests/test_winners_gpu.py for the tuned ``|eb`` / ``|mb`` keys."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _rand(*shape, dev, relu=False, scale=1.0):
    t = torch.randn(*shape, device=dev) * scale
    return (t.clamp_min(0) if relu else t).bfloat16()


@pytest.mark.parametrize("shape", [(2, 50, 84, 64, 256, 1, 1), (2, 25, 42, 128, 512, 1, 1), (2, 20, 34, 128, 128, 3, 1),
                                   (2, 40, 68, 256, 64, 1, 1)])
def test_forward_emits_bits(cuda, shape):
    from batchai_retinanet_horovod_coco_amd.ops import native_conv as NC
    N, H, W, cin, cout, kh, stride = shape
    pads = (kh // 2,) * 4
    torch.manual_seed(1)
    x = _rand(N, H, W, cin, dev=cuda, relu=True)
    w = _rand(cout, kh, kh, cin, dev=cuda, scale=(kh * kh * cin) ** -0.5)
    b = torch.randn(cout, device=cuda) * 0.1
    Ho, Wo = NC._out_hw(H, W, kh, stride, pads)
    res = _rand(N, Ho, Wo, cout, dev=cuda) if kh == 1 else None
    g = NC.geom_single(N, H, W, Ho, Wo, kh, stride, pads, cin, cout)
    plain = NC.fwd_candidates(x, w, b, res, g, stride, pads, True, (N, Ho, Wo, cout), allow_miopen=False)
    probe = NC.BitMask(torch.empty(N, Ho, Wo, cout, device=cuda))
    names = sorted(NC.fwd_candidates(x, w, b, res, g, stride, pads, True, (N, Ho, Wo, cout), allow_miopen=False,
                                     mask=probe))
    assert names and all(NC.bits_capable(n) for n in names)
    for name in names:
        y0 = plain[name]()
        bm = NC.BitMask(y0)
        bm.bits.fill_(0xA5)
        y1 = NC.fwd_candidates(x, w, b, res, g, stride, pads, True, (N, Ho, Wo, cout), allow_miopen=False,
                               mask=bm, only=name)[name]()
        torch.cuda.synchronize()
        assert torch.equal(y0, y1), name
        assert torch.equal(bm.dense(), y1 > 0), name


@pytest.mark.parametrize("shape,acc", [((2, 50, 84, 256, 64, 1, 1), False), ((2, 50, 84, 256, 64, 1, 1), True),
                                       ((2, 40, 68, 512, 128, 1, 2), True), ((2, 40, 68, 512, 128, 1, 2), False),
                                       ((2, 20, 34, 128, 128, 3, 1), False), ((2, 20, 34, 64, 64, 3, 1), False)])
def test_dgrad_reads_bits(cuda, shape, acc):
    from batchai_retinanet_horovod_coco_amd.ops import native_conv as NC
    from batchai_retinanet_horovod_coco_amd.ops.conv_dgrad import _dgrad_cands
    N, H, W, cin, cout, kh, stride = shape
    pads = (kh // 2,) * 4 if stride == 1 else (0, 0, 0, 0)
    torch.manual_seed(2)
    x = _rand(N, H, W, cin, dev=cuda, relu=True)
    w = _rand(cout, kh, kh, cin, dev=cuda, scale=(kh * kh * cin) ** -0.5)
    Ho, Wo = NC._out_hw(H, W, kh, stride, pads)
    dy = _rand(N, Ho, Wo, cout, dev=cuda)
    base = _rand(N, H, W, cin, dev=cuda) if acc else None
    if acc and stride == 2:
        base[:, 1::2] = 0
        base[:, :, 1::2] = 0
    bm = NC.BitMask.of(x)
    assert torch.equal(bm.dense(), x > 0)
    names = [n for n in _dgrad_cands(dy, w, x, stride, pads, mask=x, out=base) if NC.bits_capable(n)]
    assert names
    for name in names:
        o0 = base.clone() if acc else None
        o1 = base.clone() if acc else None
        d0 = _dgrad_cands(dy, w, x, stride, pads, mask=x, out=o0, only=name)[name]()
        d1 = _dgrad_cands(dy, w, x, stride, pads, mask=bm, out=o1, only=name)[name]()
        torch.cuda.synchronize()
        assert torch.equal(o0 if acc else d0, o1 if acc else d1), name


def test_block_path_uses_bits(cuda, monkeypatch):
    """Two chained bottleneck blocks: the second block's 1x1 conv_0 data gradient runs with the first
    block's bitmask (a '|mb' tuner key), and the input gradient matches the bf16-mask run."""
    from batchai_retinanet_horovod_coco_amd.models.resnet import Block
    from batchai_retinanet_horovod_coco_amd.ops import native_conv as NC
    from batchai_retinanet_horovod_coco_amd.ops.conv_tuner import TUNER
    torch.manual_seed(3)
    b1 = Block("bottleneck", 256, 64, 0, 1, False)
    b2 = Block("bottleneck", 256, 64, 0, 2, False)
    for c in b1.chain() + b2.chain():
        c.reset_parameters()
    b1, b2 = b1.to(cuda), b2.to(cuda)
    x0 = _rand(2, 40, 68, 256, dev=cuda, relu=True)

    def run(bits):
        monkeypatch.setattr(NC, "MASK_BITS", bits)
        x = x0.clone().requires_grad_()
        y = b2(b1(x, mask_input_grad=False, grad_premasked=True), mask_input_grad=True, grad_premasked=False)
        g = torch.randn(y.shape, generator=torch.Generator(cuda).manual_seed(4), device=cuda).bfloat16()
        y.backward(g)
        torch.cuda.synchronize()
        return x.grad.clone()

    ref = run(False)
    got = run(True)
    assert any(k.endswith("|mb") or "|mb|" in k for k in TUNER.table), "no bitmask dgrad key was tuned"
    assert any(k.endswith("|eb") for k in TUNER.table), "no bitmask-emitting forward key was tuned"
    # (the '|m' and '|mb' keys are tuned separately, so the winning kernels -- and the summation order -- may
    # differ between the two runs: bf16 rounding, not bit identity)
    # (a wrong mask would change whole rows, not round them: a relative-norm bound that a pick of other kernels for
    # the two key sets -- the stage-2 3x3s have ten hx32 candidates -- cannot trip)
    assert ((ref.float() - got.float()).norm() / ref.float().norm()).item() <= 2e-2


def test_head_tower_bits_bf16_chain_exact(cuda, monkeypatch):
    """bf16 packed head layers (relu, relu, final) on conv_hx32: with HEAD_BITS each relu output leaves its
    epilogue as a bitmask too (BW form) and the next data gradient masks with it (MK = 2 form); every gradient
    equals the bf16-mask run's bit for bit."""
    from batchai_retinanet_horovod_coco_amd.ops import native_conv as NC
    monkeypatch.setenv("MXR_CONV_FORCE", "hx32_0")
    shapes = ((20, 34), (10, 17), (5, 9), (3, 5), (2, 3))
    n, c = 2, 256
    P = sum(h * w for h, w in shapes)
    torch.manual_seed(4)
    ws = [(torch.randn(c, 3, 3, c, device=cuda) / 48).requires_grad_() for _ in range(3)]
    bs = [(torch.randn(c, device=cuda) * 0.1).requires_grad_() for _ in range(3)]
    x0 = torch.randn(n, P, c, device=cuda).bfloat16()
    gy = (torch.randn(n, P, c, device=cuda) * 1e-2).bfloat16()
    flags = []

    def run(on):
        monkeypatch.setattr(NC, "HEAD_BITS", on)
        flags.clear()
        x = x0.clone().requires_grad_()
        h = x
        for i in range(3):
            h = NC.PyramidConvFn.apply(h, ws[i].bfloat16(), bs[i], shapes, i < 2, i > 0, i < 2)
            flags.append(getattr(h, "_mxr_bits", None) is not None)
        h.backward(gy)
        torch.cuda.synchronize()
        out = [x.grad.clone()] + [t.grad.clone() for t in bs]
        for t in ws + bs:
            t.grad = None
        return out
    ref = run(False)
    assert flags == [False, False, False]
    got = run(True)
    assert flags == [True, True, False], flags
    for a, b in zip(got, ref):
        assert torch.equal(a, b)
