"""The projection block's branch2c + branch1 as ONE dual-source GEMM (csrc/kernels/conv_pipe.hip ``DualSrc``,
``mxr_conv_fwd_pipe_dual``; VERDICT r5 Next #1a): every tile variant against an fp32 PyTorch reference of
relu(conv1x1(h, W2c) + conv1x1_s(x, W1) + b) -- the block the reference builds with two convs and a keras ``Add``
(/root/reference/train.py:91) -- including the emitted ReLU bitmask, and the fused residual block
(forward and every gradient) against the two-launch form."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.fixture
def cuda():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


CASES = [  # (N, H, W of x, c_h, c_x, cout, stride)
    (2, 30, 46, 64, 64, 256, 1),
    (2, 27, 41, 128, 256, 512, 2),
    (1, 13, 21, 256, 512, 1024, 2),
    (1, 8, 11, 512, 1024, 2048, 2),
]


def _ref(h, x, w2c, w1, b, s):
    xs = x[:, ::s, ::s].float()
    y = F.linear(h.float(), w2c.float()) + F.linear(xs, w1.float()) + b
    return torch.relu(y)


@pytest.mark.parametrize("case", CASES)
def test_dual_source_kernel_matches_fp32(cuda, case):
    from batchai_retinanet_horovod_coco_amd.ops import conv_launch as CL
    from batchai_retinanet_horovod_coco_amd.ops.conv_tuner import TUNER
    N, H, W, c1, c2, cout, s = case
    Ho, Wo = (H - 1) // s + 1, (W - 1) // s + 1
    g = torch.Generator(device=cuda).manual_seed(1)
    h = torch.randn(N, Ho, Wo, c1, device=cuda, generator=g).relu().bfloat16()
    x = torch.randn(N, H, W, c2, device=cuda, generator=g).relu().bfloat16()
    w2c = (torch.randn(cout, c1, device=cuda, generator=g) / c1 ** 0.5).bfloat16()
    w1 = (torch.randn(cout, c2, device=cuda, generator=g) / c2 ** 0.5).bfloat16()
    b = torch.randn(cout, device=cuda, generator=g) * 0.1
    ref = _ref(h, x, w2c, w1, b, s)
    assert CL.proj_fusable(h, x, w2c.view(cout, 1, 1, c1), w1.view(cout, 1, 1, c2), s)
    for v in CL.DUAL_VARIANTS:
        emit = CL.BitMask(shape=(N, Ho, Wo, cout), device=cuda)
        key = "test_dual|%d|%s" % (v, case)
        TUNER.table[key] = "d%d" % v
        y = torch.empty_like(ref, dtype=torch.bfloat16)
        import ctypes
        from batchai_retinanet_horovod_coco_amd.ops.native import _chk, _p, _s, lib, zero_page
        gm = CL.geom_single(N, Ho, Wo, Ho, Wo, 1, 1, (0, 0, 0, 0), c1 + c2, cout)
        _chk(lib().mxr_conv_fwd_pipe_dual(_p(h), _p(x), c1, c2, H, W, s, _p(w2c), _p(w1), _p(b), _p(emit), _p(y),
                                          _p(zero_page(cuda)), ctypes.byref(gm), 1, v, _s()), "dual")
        torch.cuda.synchronize()
        err = (y.float() - ref).abs().max().item()
        assert err <= 2e-2 * ref.abs().max().item() + 1e-2, (v, err)
        assert torch.equal(emit.dense(), y > 0), v


def test_run_fwd_proj_tuned(cuda):
    from batchai_retinanet_horovod_coco_amd.ops import conv_launch as CL
    N, H, W, c1, c2, cout, s = CASES[1]
    Ho, Wo = (H - 1) // s + 1, (W - 1) // s + 1
    g = torch.Generator(device=cuda).manual_seed(2)
    h = torch.randn(N, Ho, Wo, c1, device=cuda, generator=g).relu().bfloat16()
    x = torch.randn(N, H, W, c2, device=cuda, generator=g).relu().bfloat16()
    w2c = (torch.randn(cout, c1, device=cuda, generator=g) / c1 ** 0.5).bfloat16()
    w1 = (torch.randn(cout, c2, device=cuda, generator=g) / c2 ** 0.5).bfloat16()
    b = torch.randn(cout, device=cuda, generator=g) * 0.1
    y = CL.run_fwd_proj(h, x, w2c, w1, b, s)
    ref = _ref(h, x, w2c, w1, b, s)
    assert (y.float() - ref).abs().max().item() <= 2e-2 * ref.abs().max().item() + 1e-2


@pytest.mark.parametrize("stage", [0, 1])
def test_fused_projection_block_matches_two_launch_form(cuda, monkeypatch, stage):
    """A bottleneck projection block (res2a: stride 1, res3a: stride 2) through ResidualBlockFn with the dual-source
    forward vs the branch1-then-residual form: same output (to bf16 rounding of the shortcut) and gradients."""
    from batchai_retinanet_horovod_coco_amd.models.resnet import Block
    from batchai_retinanet_horovod_coco_amd.ops import conv_launch as CL
    from batchai_retinanet_horovod_coco_amd.ops import native
    native.set_grad_sinks(None)
    native.set_compute_weights(None)
    torch.manual_seed(0)
    cin, filters = (64, 64) if stage == 0 else (256, 128)
    blk = Block("bottleneck", cin, filters, stage, 0, False).to(cuda)
    # every block output well above 0: the output relu takes the same side in both forms (an output within
    # rounding of 0 would flip its gradient entry -- the backward code is shared, only the forward rounding differs)
    blk.branch2c.bn.beta.fill_(24.0)
    x0 = torch.randn(2, 40, 58, cin, device=cuda).relu().bfloat16()
    res = []
    for fused in (True, False):
        monkeypatch.setattr(CL, "PROJ_FUSED", fused)
        for p in blk.parameters():
            p.grad = None
        x = x0.clone().requires_grad_(True)
        y = blk(x)
        gy = torch.randn_like(y.float(), generator=torch.Generator(device=cuda).manual_seed(5)).bfloat16()
        y.backward(gy)
        res.append((y.detach().float(), x.grad.float(), [p.grad.float().clone() for p in blk.parameters()
                                                          if p.grad is not None]))
    (ya, xa, ga), (yb, xb, gb) = res
    assert (ya - yb).abs().max().item() <= 2e-2 * yb.abs().max().item()
    assert (ya > 0).all() and (yb > 0).all()
    assert (xa - xb).norm().item() <= 1e-2 * xb.norm().item()
    assert len(ga) == len(gb) and len(ga) >= 4
    for a, b in zip(ga, gb):
        assert (a - b).norm().item() <= 1e-2 * b.norm().item()


@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("acc", [False, True])
def test_dual_destination_dgrad_matches_fp32(cuda, case, acc):
    """[dH2 | dX] = dY . [W2c | W1] in one launch (conv_pipe.hip DualDst): dH2 masked by the branch2b activation,
    dX at stride 1 or scattered at stride 2 (gap zeros written), or accumulated into a join buffer."""
    import ctypes
    from batchai_retinanet_horovod_coco_amd.ops import conv_launch as CL
    from batchai_retinanet_horovod_coco_amd.ops.native import _chk, _p, _s, lib, zero_page
    N, H, W, c1, c2, K, s = case
    Ho, Wo = (H - 1) // s + 1, (W - 1) // s + 1
    g = torch.Generator(device=cuda).manual_seed(4)
    dy = torch.randn(N, Ho, Wo, K, device=cuda, generator=g).bfloat16()
    h2 = torch.randn(N, Ho, Wo, c1, device=cuda, generator=g).relu().bfloat16()
    w2c = (torch.randn(K, c1, device=cuda, generator=g) / K ** 0.5).bfloat16()
    w1 = (torch.randn(K, c2, device=cuda, generator=g) / K ** 0.5).bfloat16()
    base = torch.randn(N, H, W, c2, device=cuda, generator=g).bfloat16()
    ref_dh = (dy.float() @ w2c.float()) * (h2.float() > 0)
    ref_dx = torch.zeros(N, H, W, c2, device=cuda)
    ref_dx[:, ::s, ::s] = dy.float() @ w1.float()
    if acc:
        ref_dx[:, ::s, ::s] += base.float()[:, ::s, ::s]
        if s == 2:      # accumulation touches the strided positions only
            keep = torch.ones(N, H, W, 1, device=cuda, dtype=torch.bool)
            keep[:, ::s, ::s] = False
            ref_dx = torch.where(keep, base.float(), ref_dx)
    wd1, wd2 = w2c.t().contiguous(), w1.t().contiguous()     # [c1, K], [c2, K]
    gm = CL.geom_single(N, Ho, Wo, Ho, Wo, 1, 1, (0, 0, 0, 0), K, c1 + c2)
    for v in CL.DUAL_VARIANTS:
        dh = torch.empty(N, Ho, Wo, c1, device=cuda, dtype=torch.bfloat16)
        dx = base.clone() if acc else torch.full((N, H, W, c2), float("nan"), device=cuda, dtype=torch.bfloat16)
        _chk(lib().mxr_conv_dgrad_pipe_dd(_p(dy), _p(wd1), _p(wd2), _p(h2), _p(dh), _p(dx), c1, c2, s, H, W, int(acc),
                                          _p(zero_page(cuda)), ctypes.byref(gm), v, _s()), "dd")
        torch.cuda.synchronize()
        for name, got, ref in (("dh2", dh, ref_dh), ("dx", dx, ref_dx)):
            assert not torch.isnan(got).any(), (v, name)
            err = (got.float() - ref).abs().max().item()
            assert err <= 2e-2 * ref.abs().max().item() + 1e-2, (v, name, err)


@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("bits", [False, True])
def test_persistent_dual_source_matches_fp32(cuda, case, bits):
    """The persistent streaming 1x1 kernel's dual-source form (conv1x1_pers.hip QDual) vs fp32 PyTorch."""
    from batchai_retinanet_horovod_coco_amd.ops import conv_launch as CL
    from batchai_retinanet_horovod_coco_amd.ops import native as NV
    from batchai_retinanet_horovod_coco_amd.ops.native import _chk, _p, _s, lib, zero_page
    N, H, W, c1, c2, cout, s = case
    Ho, Wo = (H - 1) // s + 1, (W - 1) // s + 1
    g = torch.Generator(device=cuda).manual_seed(7)
    h = torch.randn(N, Ho, Wo, c1, device=cuda, generator=g).relu().bfloat16()
    x = torch.randn(N, H, W, c2, device=cuda, generator=g).relu().bfloat16()
    w2c = (torch.randn(cout, c1, device=cuda, generator=g) / c1 ** 0.5).bfloat16()
    w1 = (torch.randn(cout, c2, device=cuda, generator=g) / c2 ** 0.5).bfloat16()
    b = torch.randn(cout, device=cuda, generator=g) * 0.1
    ref = _ref(h, x, w2c, w1, b, s)
    emit = CL.BitMask(shape=(N, Ho, Wo, cout), device=cuda) if bits else None
    y = torch.full((N, Ho, Wo, cout), float("nan"), device=cuda, dtype=torch.bfloat16)
    _chk(lib().mxr_conv1x1_pers_dual(_p(h), _p(x), _p(w2c), _p(w1), _p(b), _p(emit), _p(y), _p(zero_page(cuda)),
                                     _p(NV.trash_page(cuda)), N * Ho * Wo, cout, c1 + c2, c1, H, W, s, Ho, Wo, _s()),
         "c1p_dual")
    torch.cuda.synchronize()
    assert not torch.isnan(y).any()
    err = (y.float() - ref).abs().max().item()
    assert err <= 2e-2 * ref.abs().max().item() + 1e-2, err
    if bits:
        assert torch.equal(emit.dense(), y > 0)


def test_chunked_identity_block_matches_whole_batch(cuda, monkeypatch):
    """MXR_BLOCK_CHUNK: an identity block's forward image-chunk by image-chunk (into the same full-batch activations)
    gives the whole-batch output, bitmask and gradients."""
    from batchai_retinanet_horovod_coco_amd.models.resnet import Block
    from batchai_retinanet_horovod_coco_amd.ops import native
    from batchai_retinanet_horovod_coco_amd.ops import native_conv as NC
    native.set_grad_sinks(None)
    native.set_compute_weights(None)
    torch.manual_seed(0)
    blk = Block("bottleneck", 256, 64, 0, 1, False).to(cuda)
    blk.branch2c.bn.beta.fill_(24.0)          # outputs away from the relu kink (see above)
    x0 = torch.randn(8, 24, 40, 256, device=cuda).relu().bfloat16()
    res = []
    for chunk in (0, 2):
        monkeypatch.setattr(NC, "_BLOCK_CHUNK", chunk)
        monkeypatch.setattr(NC, "_BLOCK_CHUNK_MIN_PX", 1)
        for p in blk.parameters():
            p.grad = None
        x = x0.clone().requires_grad_(True)
        y = blk(x)
        bits = getattr(y, "_mxr_bits", None)
        gy = torch.randn(y.shape, device=cuda, generator=torch.Generator(device=cuda).manual_seed(5)).bfloat16()
        y.backward(gy)
        res.append((y.detach().float(), None if bits is None else bits.dense(), x.grad.float(),
                    [p.grad.float().clone() for p in blk.parameters() if p.grad is not None]))
    (ya, ba, xa, ga), (yb, bb, xb, gb) = res
    assert (ya - yb).abs().max().item() <= 1e-2 * yb.abs().max().item()
    if ba is not None:
        assert torch.equal(ba, bb) and torch.equal(bb, yb > 0)
    assert (xa - xb).norm().item() <= 1e-2 * xb.norm().item()
    for a, b in zip(ga, gb):
        assert (a - b).norm().item() <= 1e-2 * b.norm().item()


@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("variant", [0, 2, 4])
def test_dual_source_wgrad_matches_fp32(cuda, case, variant):
    """Both weight gradients of a projection block from one split-K GEMM over [h2 | x(::s)] (conv_wgrad_p8.hip DS,
    mxr_conv_wgrad_p8_dual), reduced into two outputs with the two BN scales, against fp32 PyTorch."""
    import ctypes
    from batchai_retinanet_horovod_coco_amd.ops import conv_launch as CL
    from batchai_retinanet_horovod_coco_amd.ops.native import _chk, _p, _s, lib, zero_page
    N, H, W, c1, c2, cout, s = case
    Ho, Wo = (H - 1) // s + 1, (W - 1) // s + 1
    g = torch.Generator(device=cuda).manual_seed(9)
    h2 = torch.randn(N, Ho, Wo, c1, device=cuda, generator=g).relu().bfloat16()
    x = torch.randn(N, H, W, c2, device=cuda, generator=g).relu().bfloat16()
    dy = torch.randn(N, Ho, Wo, cout, device=cuda, generator=g).bfloat16()
    s1c = torch.rand(cout, device=cuda, generator=g) + 0.5
    s1 = torch.rand(cout, device=cuda, generator=g) + 0.5
    dyf = dy.float().reshape(-1, cout)
    ref1 = (dyf.t() @ h2.float().reshape(-1, c1)) * s1c[:, None]
    ref2 = (dyf.t() @ x.float()[:, ::s, ::s].reshape(-1, c2)) * s1[:, None]
    gm = CL.geom_single(N, H, W, Ho, Wo, 1, s, (0, 0, 0, 0), c2, cout)
    splits = 3
    part = torch.empty(splits * cout * (c1 + c2), device=cuda)
    o1 = torch.zeros(cout, c1, device=cuda)
    o2 = torch.full((cout, c2), 1.0, device=cuda)          # accumulate: += onto existing values
    _chk(lib().mxr_conv_wgrad_p8_dual(_p(x), _p(h2), c1, _p(dy), cout, _p(part), splits, _p(o1), _p(o2), _p(s1c),
                                      _p(s1), 1, _p(zero_page(cuda)), ctypes.byref(gm), variant, _s()), "wgrad_dual")
    torch.cuda.synchronize()
    for got, ref in ((o1, ref1), (o2 - 1.0, ref2)):
        err = (got - ref).norm().item() / ref.norm().item()
        assert err < 1e-2, err


def test_projection_wgrad_through_sinks_matches_separate(cuda, monkeypatch):
    """In a training step (gradient sinks on) the fused projection weight gradients equal the two separate ones."""
    import copy
    from batchai_retinanet_horovod_coco_amd import models
    from batchai_retinanet_horovod_coco_amd.data.synthetic import make_batch
    from batchai_retinanet_horovod_coco_amd.ops import conv_wgrad as CW
    from batchai_retinanet_horovod_coco_amd.ops import native
    from batchai_retinanet_horovod_coco_amd.train.engine import Trainer
    torch.manual_seed(0)
    base = models.backbone("resnet50").retinanet(8)
    g = torch.Generator(device=cuda).manual_seed(0)
    b = make_batch(2, 256, 384, 8, device=cuda, generator=g, dtype=torch.bfloat16)
    grads = []
    monkeypatch.setattr(CW, "PROJ_WGRAD_MIN_PX", 0)       # every projection block of this small batch
    for fused in (True, False):
        monkeypatch.setattr(CW, "PROJ_WGRAD", fused)
        native.set_grad_sinks(None)
        native.set_compute_weights(None)
        tr = Trainer(copy.deepcopy(base), lr=0.0, compute_dtype=torch.bfloat16, device=cuda)
        tr.optimizer.zero_grad()
        tr.forward_backward(b["images"], b["gt"], b["gt_count"], b["image_hw"])
        from batchai_retinanet_horovod_coco_amd.ops.side_stream import SIDE
        SIDE.join()
        torch.cuda.synchronize()
        grads.append({s.name: tr.flat.grad[s.offset:s.offset + s.numel].clone()
                      for s in tr.flat.segments if "branch1" in s.name or "branch2c" in s.name})
        native.set_grad_sinks(None)
        native.set_compute_weights(None)
    assert grads[0].keys() == grads[1].keys() and len(grads[0]) >= 8
    for n in grads[0]:
        a, c = grads[0][n], grads[1][n]
        assert (a - c).norm().item() <= 1e-2 * c.norm().item() + 1e-12, n
