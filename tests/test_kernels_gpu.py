"""HIP kernel numerics vs plain PyTorch fp32 references (run on a real MI355X via gpurun)."""
import pytest
import torch
import torch.nn.functional as F

from batchai_retinanet_horovod_coco_amd.ops import anchors as A
from batchai_retinanet_horovod_coco_amd.ops import boxes as Bx
from batchai_retinanet_horovod_coco_amd.ops import conv as C
from batchai_retinanet_horovod_coco_amd.ops import losses as L
from batchai_retinanet_horovod_coco_amd.ops import native as N

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _force_hip(monkeypatch):
    # numerics of the HIP kernels themselves: never let the per-shape tuner pick the library path
    monkeypatch.setenv("MXR_CONV_FORCE", "hip")


def ref_conv(x, w, b, stride, pads, relu=False, res=None):
    """fp32 NHWC reference."""
    xf = x.float()
    pt, pb, pl, pr = pads
    xp = F.pad(xf, (0, 0, pl, pr, pt, pb))
    y = F.conv2d(xp.permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), None if b is None else b.float(), stride)
    y = y.permute(0, 2, 3, 1)
    if res is not None:
        y = y + res.float()
    if relu:
        y = F.relu(y)
    return y


CONV_CASES = [
    # N, H, W, cin, cout, k, stride, padmode
    (2, 20, 33, 64, 64, 1, 1, "valid"),
    (2, 20, 33, 64, 256, 1, 1, "valid"),
    (2, 21, 34, 256, 128, 1, 2, "valid"),
    (2, 17, 23, 64, 64, 3, 1, 1),
    (2, 13, 19, 256, 256, 3, 1, "same"),
    (1, 25, 42, 512, 256, 3, 2, "same"),      # P6-like (asymmetric TF-same)
    (2, 9, 11, 256, 36, 3, 1, "same"),        # regression final
    (2, 9, 11, 256, 720, 3, 1, "same"),       # classification final
    (1, 7, 9, 2048, 512, 1, 1, "valid"),
]


def _pads(H, W, k, s, mode):
    if mode == "same":
        return C.same_pads((H, W), k, s)
    if mode == "valid":
        return (0, 0, 0, 0)
    return (mode, mode, mode, mode)


@pytest.mark.parametrize("case", CONV_CASES)
@pytest.mark.parametrize("epi", ["plain", "bias_relu", "bias_res_relu"])
def test_conv_fwd(cuda, case, epi):
    torch.manual_seed(0)
    n, H, W, cin, cout, k, s, pm = case
    pads = _pads(H, W, k, s, pm)
    x = torch.randn(n, H, W, cin, device=cuda).bfloat16()
    w = (torch.randn(cout, k, k, cin, device=cuda) / (k * k * cin) ** 0.5).bfloat16()
    b = torch.randn(cout, device=cuda) if epi != "plain" else None
    Ho, Wo = C.out_hw((H, W), k, s, pads)
    res = torch.randn(n, Ho, Wo, cout, device=cuda).bfloat16() if epi == "bias_res_relu" else None
    relu = epi != "plain"
    y = N.conv2d(x, w, b, s, pads, relu, res)
    yr = ref_conv(x, w, b, s, pads, relu, res)
    assert y.shape == yr.shape
    err = (y.float() - yr).abs().max().item()
    scale = yr.abs().max().item() + 1e-3
    assert err / scale < 2e-2, (err, scale)


@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_backward(cuda, case):
    torch.manual_seed(1)
    n, H, W, cin, cout, k, s, pm = case
    pads = _pads(H, W, k, s, pm)
    x = torch.randn(n, H, W, cin, device=cuda).bfloat16().requires_grad_()
    w = (torch.randn(cout, k, k, cin, device=cuda) / (k * k * cin) ** 0.5).bfloat16().requires_grad_()
    b = torch.randn(cout, device=cuda).requires_grad_()
    y = N.conv2d(x, w, b, s, pads, True, None)
    g = torch.randn_like(y)
    y.backward(g)
    xr = x.detach().float().requires_grad_()
    wr = w.detach().float().requires_grad_()
    br = b.detach().clone().requires_grad_()
    yr = ref_conv(xr, wr, br, s, pads, True, None)
    # use the bf16 kernel's relu mask to avoid boundary disagreement
    yr.backward(g.float() * (y.detach().float() > 0) * (yr.detach() > 0) + 0 * yr.detach())
    for got, ref in ((x.grad, xr.grad), (w.grad, wr.grad), (b.grad, br.grad)):
        err = (got.float() - ref).abs().max().item()
        scale = ref.abs().max().item() + 1e-3
        assert err / scale < 3e-2, (err, scale)


def test_pyramid_conv(cuda):
    torch.manual_seed(2)
    shapes = [(10, 17), (5, 9), (3, 5), (2, 3), (1, 2)]
    n, cin, cout = 2, 256, 256
    xs = [torch.randn(n, h, w, cin, device=cuda).bfloat16() for (h, w) in shapes]
    w = (torch.randn(cout, 3, 3, cin, device=cuda) / (9 * cin) ** 0.5).bfloat16()
    b = torch.randn(cout, device=cuda)
    ys = N.pyramid_conv(xs, w, b, True)
    for x, y in zip(xs, ys):
        yr = ref_conv(x, w, b, 1, (1, 1, 1, 1), True)
        err = (y.float() - yr).abs().max().item()
        assert err / (yr.abs().max().item() + 1e-3) < 2e-2
    # backward through the packed path
    packed, sh = N.pyramid_pack(xs)
    packed = packed.detach().requires_grad_()
    wq = w.detach().clone().requires_grad_()
    y = N.pyramid_conv_packed(packed, sh, wq, b, True)
    g = torch.randn_like(y)
    y.backward(g)
    off = 0
    dws = torch.zeros_like(w, dtype=torch.float32)
    for (h, wd) in sh:
        xl = packed.detach()[:, off:off + h * wd].reshape(n, h, wd, cin).float().requires_grad_()
        wr = w.detach().float().requires_grad_()
        yl = ref_conv(xl, wr, b, 1, (1, 1, 1, 1), True)
        gl = g[:, off:off + h * wd].reshape(n, h, wd, cout).float() * (y.detach()[:, off:off + h * wd]
                                                                         .reshape(n, h, wd, cout).float() > 0)
        yl.backward(gl)
        dx = packed.grad[:, off:off + h * wd].reshape(n, h, wd, cin).float()
        assert (dx - xl.grad).abs().max() / (xl.grad.abs().max() + 1e-3) < 3e-2
        dws += wr.grad
        off += h * wd
    assert (wq.grad.float() - dws).abs().max() / (dws.abs().max() + 1e-3) < 3e-2


def test_focal_and_smooth_l1(cuda):
    torch.manual_seed(3)
    B, Anc, Cn = 2, 999, 80
    logits = (torch.randn(B, Anc, Cn, device=cuda) * 4).bfloat16()
    state = torch.randint(-1, 2, (B, Anc), device=cuda).to(torch.int8)
    label = torch.randint(0, Cn, (B, Anc), device=cuda).to(torch.int32)
    loss, grad = N.focal_fwd_bwd(logits, state, label)
    lr = logits.float().requires_grad_()
    ref = L._focal_torch(lr, state, label, 0.25, 2.0)
    ref.backward()
    assert abs(loss.item() - ref.item()) / ref.item() < 1e-3
    assert (grad.float() - lr.grad).abs().max() / lr.grad.abs().max() < 2e-2
    # keras-literal oracle on probabilities agrees with the logit-space loss
    onehot = torch.zeros(B, Anc, Cn + 1, device=cuda)
    onehot[..., :Cn].scatter_(2, label.long()[..., None], (state == 1).float()[..., None])
    onehot[..., :Cn] = torch.where((state == -1)[..., None], torch.full_like(onehot[..., :Cn], -1.0), onehot[..., :Cn])
    onehot[..., Cn] = state.float()
    kref = L.focal_keras(onehot, torch.sigmoid(logits.float()))
    assert abs(kref.item() - loss.item()) / kref.item() < 2e-3
    reg = torch.randn(B, Anc, 4, device=cuda).bfloat16()
    tgt = torch.randn(B, Anc, 4, device=cuda)
    l2, g2 = N.smooth_l1_fwd_bwd(reg, tgt, state)
    rr = reg.float().requires_grad_()
    r2 = L._smooth_l1_torch(rr, tgt, state, 3.0)
    r2.backward()
    assert abs(l2.item() - r2.item()) / r2.item() < 1e-3
    assert (g2.float() - rr.grad).abs().max() < 2e-2 * rr.grad.abs().max()


@pytest.mark.parametrize("scale,gamma", [(1.0, 2.0), (12.0, 2.0), (4.0, 1.5)])
def test_focal_paths(cuda, scale, gamma):
    """focal_bf16_kernel's three bodies against the fp32 reference: gamma 2 with every logit inside the
    clip range (focal_neg_g2_inr), gamma 2 with many logits beyond +-16.1 (the exact per-vector fallback),
    and a runtime gamma (focal_neg with __powf)."""
    torch.manual_seed(5)
    B, Anc, Cn = 2, 1501, 80
    logits = (torch.randn(B, Anc, Cn, device=cuda) * scale - 2).bfloat16()
    state = torch.randint(-1, 2, (B, Anc), device=cuda).to(torch.int8)
    label = torch.randint(0, Cn, (B, Anc), device=cuda).to(torch.int32)
    loss, grad = N.focal_fwd_bwd(logits, state, label, gamma=gamma)
    lr = logits.float().requires_grad_()
    ref = L._focal_torch(lr, state, label, 0.25, gamma)
    ref.backward()
    assert abs(loss.item() - ref.item()) / ref.item() < 1e-3
    assert (grad.float() - lr.grad).abs().max() / lr.grad.abs().max() < 2e-2


def test_anchor_targets(cuda):
    torch.manual_seed(4)
    from batchai_retinanet_horovod_coco_amd.data.synthetic import make_batch
    b = make_batch(3, 256, 320, device=cuda, max_boxes=12)
    b["gt_count"][1] = 0
    b["image_hw"][2] = torch.tensor([200, 300], device=cuda)
    cache = A.AnchorCache()
    anchors, centers = cache.get((256, 320), cuda), cache.centers((256, 320), cuda)
    s1, l1, r1, n1 = N.anchor_targets(anchors, b["gt"], b["gt_count"], b["image_hw"], centers=centers)
    s0, l0, r0 = A.anchor_targets_torch(anchors, b["gt"], b["gt_count"], b["image_hw"], centers=centers)
    mism = (s1 != s0).float().mean().item()
    assert mism < 1e-4
    pos = s0 == 1
    assert (l1[pos] == l0[pos]).all()
    assert torch.allclose(r1[pos], r0[pos], atol=1e-4)
    assert n1.item() == int(pos.sum().item())


def test_adam_fused_matches_torch(cuda):
    from batchai_retinanet_horovod_coco_amd.train.flat import FlatParams
    from batchai_retinanet_horovod_coco_amd.train.optimizer import KerasAdam
    torch.manual_seed(5)
    ps = [torch.nn.Parameter(torch.randn(s, device=cuda)) for s in [(7, 3, 3, 5), (13,), (64, 1, 1, 64)]]
    ps2 = [torch.nn.Parameter(p.detach().clone()) for p in ps]
    f1 = FlatParams([(str(i), p) for i, p in enumerate(ps)])
    f2 = FlatParams([(str(i), p) for i, p in enumerate(ps2)])
    o1 = KerasAdam(f1, lr=1e-3, clipnorm=0.5)
    o2 = KerasAdam(f2, lr=1e-3, clipnorm=0.5, backend="torch")
    for _ in range(3):
        g = torch.randn(f1.total, device=cuda)
        f1.grad.copy_(g)
        f2.grad.copy_(g)
        n1 = o1.step()
        n2 = o2.step()
        assert abs(n1.item() - n2.item()) < 1e-3 * n2.item()
    for s1, s2 in zip(f1.segments, f2.segments):   # alignment padding is not a parameter
        a, b = slice(s1.offset, s1.offset + s1.numel), slice(s2.offset, s2.offset + s2.numel)
        assert torch.allclose(f1.data[a], f2.data[b], atol=1e-6, rtol=1e-5)
        assert torch.allclose(o1.m[a], o2.m[b], atol=1e-7, rtol=1e-5)


def test_maxpool_upsample(cuda):
    torch.manual_seed(6)
    x = torch.randn(2, 40, 67, 64, device=cuda).bfloat16().requires_grad_()
    y = C.maxpool_same(x)
    xr = x.detach().float().requires_grad_()
    pads = C.same_pads((40, 67), 3, 2)
    yr = F.max_pool2d(F.pad(xr.permute(0, 3, 1, 2), (pads[2], pads[3], pads[0], pads[1]), value=float("-inf")), 3, 2)
    yr = yr.permute(0, 2, 3, 1)
    assert torch.equal(y.float(), yr)
    g = torch.randn_like(yr)
    y.backward(g.bfloat16())
    yr.backward(g)
    assert (x.grad.float() - xr.grad).abs().max() < 5e-2
    s = torch.randn(2, 50, 84, 256, device=cuda).bfloat16().requires_grad_()
    lat = torch.randn(2, 100, 167, 256, device=cuda).bfloat16().requires_grad_()
    out = N.upsample_add(s, lat)
    sr = s.detach().float().requires_grad_()
    lr_ = lat.detach().float().requires_grad_()
    outr = lr_ + C.upsample_like(sr, (100, 167))
    assert (out.float() - outr).abs().max() < 5e-2
    g = torch.randn_like(outr)
    out.backward(g.bfloat16())
    outr.backward(g)
    assert (s.grad.float() - sr.grad).abs().max() / sr.grad.abs().max() < 2e-2


def test_nms_and_decode(cuda):
    torch.manual_seed(7)
    n = 500
    xy = torch.rand(n, 2, device=cuda) * 200
    wh = torch.rand(n, 2, device=cuda) * 50 + 5
    boxes = torch.cat([xy, xy + wh], 1)
    scores = torch.rand(n, device=cuda)
    k1 = N.nms(boxes, scores, 0.5, 300)
    k0 = Bx.nms(boxes, scores, 0.5, 300)
    assert torch.equal(k1.cpu(), k0.cpu())
    anchors = A.AnchorCache().get((128, 160), cuda)
    deltas = torch.randn(2, anchors.shape[0], 4, device=cuda)
    d1 = N.decode_clip(anchors, deltas, 128, 160)
    d0 = Bx.clip_boxes(Bx.bbox_transform_inv(anchors[None], deltas), 128, 160)
    assert torch.allclose(d1, d0, atol=1e-3)


@pytest.mark.parametrize("variant", [0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 20, 21, 22, 23, 24])
@pytest.mark.parametrize("case", [(2, 17, 23, 64, 64, 3, 1, 1), (2, 21, 34, 256, 128, 1, 2, "valid"),
                                  (1, 13, 19, 128, 36, 3, 1, "same"), (2, 9, 11, 64, 256, 1, 1, "valid"),
                                  (2, 30, 41, 256, 256, 3, 1, "same"), (1, 7, 9, 512, 320, 3, 2, "same")])
def test_wgrad_variants(cuda, case, variant):
    torch.manual_seed(11)
    n, H, W, cin, cout, k, s, pm = case
    pads = _pads(H, W, k, s, pm)
    Ho, Wo = C.out_hw((H, W), k, s, pads)
    x = torch.randn(n, H, W, cin, device=cuda).bfloat16()
    dy = torch.randn(n, Ho, Wo, cout, device=cuda).bfloat16()
    scale = torch.rand(cout, device=cuda) + 0.5
    g = N.geom_single(n, H, W, Ho, Wo, k, s, pads, cin, cout)
    dw = N.conv_wgrad(x, dy, g, scale, variant=variant)
    xr = x.float().requires_grad_()
    wr = torch.zeros(cout, k, k, cin, device=cuda, requires_grad=True)
    ref_conv(xr, wr, None, s, pads).backward(dy.float())
    ref = wr.grad * scale.view(-1, 1, 1, 1)
    assert (dw - ref).abs().max() / ref.abs().max() < 1e-2


@pytest.mark.parametrize("variant", ["hip3", "hip4", "hip5", "hip6", "hip7", "hip8", "hip9", "hip10", "hip11",
                                     "hip12", "hip13", "hip14", "hip15", "hip16"])
@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_pipe_variants(cuda, monkeypatch, case, variant):
    """Deep-pipelined 8-wave kernels (conv_pipe.hip): fwd with the full epilogue, and dgrad."""
    monkeypatch.setenv("MXR_CONV_FORCE", variant)
    torch.manual_seed(5)
    n, H, W, cin, cout, k, s, pm = case
    pads = _pads(H, W, k, s, pm)
    x = torch.randn(n, H, W, cin, device=cuda).bfloat16().requires_grad_()
    w = (torch.randn(cout, k, k, cin, device=cuda) / (k * k * cin) ** 0.5).bfloat16()
    b = torch.randn(cout, device=cuda)
    Ho, Wo = C.out_hw((H, W), k, s, pads)
    res = torch.randn(n, Ho, Wo, cout, device=cuda).bfloat16()
    if cout % 8 == 0:      # the pipelined kernels' 16-B epilogue needs cout % 8 == 0
        y = N.conv2d(x, w, b, s, pads, True, res)
        yr = ref_conv(x.detach(), w, b, s, pads, True, res)
        assert (y.float() - yr).abs().max().item() / (yr.abs().max().item() + 1e-3) < 2e-2
    if s == 1 or (k == 1 and pm == "valid"):
        y2 = N.conv2d(x, w, None, s, pads, False, None)
        g = torch.randn_like(y2)
        y2.backward(g)
        xr = x.detach().float().requires_grad_()
        ref_conv(xr, w.float(), None, s, pads).backward(g.float())
        err = (x.grad.float() - xr.grad).abs().max().item()
        assert err / (xr.grad.abs().max().item() + 1e-3) < 3e-2


@pytest.mark.parametrize("variant", [0, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 20, 21, 22, 23, 24])
@pytest.mark.parametrize("cout", [256, 72])
def test_pyramid_wgrad_variants(cuda, variant, cout):
    """Head weight gradient over the packed ragged pyramid (level / image carries in the gather)."""
    torch.manual_seed(12)
    shapes = [(10, 17), (5, 9), (3, 5), (2, 3), (1, 2)]
    n, cin = 3, 256
    xs = [torch.randn(n, h, w, cin, device=cuda).bfloat16() for (h, w) in shapes]
    packed, sh = N.pyramid_pack(xs)
    dy = torch.randn(n, packed.shape[1], cout, device=cuda).bfloat16()
    g = N.geom_pyramid(n, sh, cin, cout)
    dw = N.conv_wgrad(packed, dy, g, None, variant=variant)
    ref = torch.zeros(cout, 3, 3, cin, device=cuda)
    off = 0
    for (h, w) in sh:
        xr = packed[:, off:off + h * w].reshape(n, h, w, cin).float()
        wr = torch.zeros(cout, 3, 3, cin, device=cuda, requires_grad=True)
        ref_conv(xr, wr, None, 1, (1, 1, 1, 1)).backward(dy[:, off:off + h * w].reshape(n, h, w, cout).float())
        ref += wr.grad
        off += h * w
    assert (dw - ref).abs().max() / ref.abs().max() < 1e-2


@pytest.mark.parametrize("variant", [20, 21, 22, 23, 24])
@pytest.mark.parametrize("cout,ldy", [(256, 256), (720, 720), (36, 64)])
def test_pyramid_wgrad_fused_bias(cuda, variant, cout, ldy):
    """conv_wgrad_p8 BIAS: the k-tile-0 blocks' one-hot-row MFMA column sums of the staged dY tiles equal
    the fp32 bias gradient sum_m dY[m, :cout] (3 co tiles with a partial one at 720; zero-padded dY rows at
    36 / 64), accumulated onto an existing value; the weight gradient is the same as without the bias."""
    torch.manual_seed(13)
    shapes = [(20, 34), (10, 17), (5, 9), (3, 5), (2, 3)]
    n, cin = 2, 256
    xs = [torch.randn(n, h, w, cin, device=cuda).bfloat16() for (h, w) in shapes]
    packed, sh = N.pyramid_pack(xs)
    dy = torch.randn(n, packed.shape[1], ldy, device=cuda).bfloat16()
    dy[..., cout:] = 0
    g = N.geom_pyramid(n, sh, cin, cout)
    dw_ref = N.conv_wgrad(packed, dy, g, None, variant=variant)
    db0 = torch.randn(cout, device=cuda)
    db = db0.clone()
    dw = N.conv_wgrad(packed, dy, g, None, variant=variant, bias_out=db, bias_accumulate=True)
    torch.cuda.synchronize()
    assert torch.equal(dw, dw_ref)
    ref = db0 + dy[..., :cout].float().sum((0, 1))
    assert (db - ref).abs().max() / ref.abs().max() < 1e-5, (db - ref).abs().max()
    db2 = torch.full((cout,), 7.0, device=cuda)
    N.conv_wgrad(packed, dy, g, None, variant=variant, bias_out=db2, bias_accumulate=False)
    ref2 = dy[..., :cout].float().sum((0, 1))
    assert (db2 - ref2).abs().max() / ref2.abs().max() < 1e-5


@pytest.mark.parametrize("shape", [(2, 17, 23, 64), (1, 16, 22, 64), (2, 400, 667, 64), (1, 9, 8, 16)])
@pytest.mark.parametrize("relu_in", [False, True])
def test_maxpool_k3s2_matches_generic(cuda, shape, relu_in):
    """maxpool_fwd_k3s2 (nine window loads issued together, clamped out-of-range taps masked to -inf)
    against the generic kernel: the same pooled values AND the same argmax bytes (first-max tie rule,
    relu_in's 255 marks, the TF-'same' border), on odd and even H / W, ties included."""
    from batchai_retinanet_horovod_coco_amd.ops import native as NN
    torch.manual_seed(2)
    N_, H, W, C_ = shape
    x = torch.randn(N_, H, W, C_, device=cuda).bfloat16()
    if relu_in:
        x = torch.relu(x)
    x[:, 1::2] = x[:, 0:H - 1:2].clone()       # every odd row repeats the one above it: ties in each window
    Ho, Wo = (H + 1) // 2, (W + 1) // 2
    pt, pl = max(0, (Ho - 1) * 2 + 3 - H) // 2, max(0, (Wo - 1) * 2 + 3 - W) // 2
    pads = (pt, max(0, (Ho - 1) * 2 + 3 - H) - pt, pl, max(0, (Wo - 1) * 2 + 3 - W) - pl)
    y0, a0 = NN.maxpool_fwd_raw(x, 3, 2, pads, relu_in=relu_in, impl=0)
    y1, a1 = NN.maxpool_fwd_raw(x, 3, 2, pads, relu_in=relu_in, impl=1)
    torch.cuda.synchronize()
    assert torch.equal(y0, y1)
    assert torch.equal(a0, a1)


@pytest.mark.parametrize("variant", ["sk11", "sk12"])
@pytest.mark.parametrize("case", [(2, 13, 21, 256, 256, 3, 2), (2, 25, 42, 512, 256, 3, 2), (1, 7, 9, 2048, 512, 1, 1)])
@pytest.mark.parametrize("epi", ["bias_relu", "bias_res_relu", "mask_acc"])
def test_conv_splitk_matches_fp32(cuda, variant, case, epi):
    """Split-K pipe form (conv_pipe.hip SK): fp32 partial tiles per K split + one epilogue pass, for the
    small-M long-K layers (FPN P6 / P7) -- every epilogue form against the fp32 reference."""
    from batchai_retinanet_horovod_coco_amd.ops import conv_launch as CL
    torch.manual_seed(5)
    n, H, W, cin, cout, k, s = case
    pads = C.same_pads((H, W), k, s) if k > 1 else (0, 0, 0, 0)
    Ho, Wo = C.out_hw((H, W), k, s, pads)
    g = CL.geom_single(n, H, W, Ho, Wo, k, s, pads, cin, cout)
    assert CL.splitk_splits(g, int(variant[2:])) >= 2
    x = torch.randn(n, H, W, cin, device=cuda).bfloat16()
    w = (torch.randn(cout, k, k, cin, device=cuda) / (k * k * cin) ** 0.5).bfloat16()
    b = torch.randn(cout, device=cuda)
    res = torch.randn(n, Ho, Wo, cout, device=cuda).bfloat16() if epi == "bias_res_relu" else None
    ref = ref_conv(x, w, b, s, pads, True, res) if epi != "mask_acc" else ref_conv(x, w, b, s, pads)
    y = torch.empty(n, Ho, Wo, cout, device=cuda, dtype=torch.bfloat16)
    if epi == "mask_acc":
        base = torch.randn_like(y)
        mask = torch.randn_like(y)
        y.copy_(base)
        CL.launch_fwd(x, w, b, None, y, g, False, accumulate=True, variant=variant, mask=mask)
        ref = torch.where(mask.float() > 0, ref + base.float(), torch.zeros_like(ref))
    else:
        CL.launch_fwd(x, w, b, res, y, g, True, variant=variant)
    err = (y.float() - ref).abs().max().item() / (ref.abs().max().item() + 1e-3)
    assert err < 2e-2, err
