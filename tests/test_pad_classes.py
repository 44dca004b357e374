"""CPU: padding a batch up to a multiple of the pyramid stride (``--pad-multiple``, VERDICT r4 Next #2a) changes
nothing inside the images: every anchor of the batch-max layout keeps its targets (state, label, regression),
every added anchor is ignored (state -1), and the focal + smooth-L1 losses over the padded layout equal the
batch-max ones whatever the network predicts on the added anchors.  (The reference pads to the batch max only:
keras-retinanet ``compute_inputs``, reached from /root/reference/train.py:197-214.)"""
import numpy as np
import pytest
import torch

from batchai_retinanet_horovod_coco_amd.data.generator import pad_shape
from batchai_retinanet_horovod_coco_amd.ops import anchors as AN
from batchai_retinanet_horovod_coco_amd.ops.losses import focal_loss, smooth_l1_loss

NA = AN.AnchorParameters.default.num_anchors()


def _index_map(shape, padded):
    """Index in the padded layout of every anchor of the batch-max layout (level by level)."""
    g0, g1 = AN.guess_shapes(shape), AN.guess_shapes(padded)
    out, o0, o1 = [], 0, 0
    for (h, w), (hp, wp) in zip(g0, g1):
        assert hp >= h and wp >= w
        y, x, a = np.meshgrid(np.arange(h), np.arange(w), np.arange(NA), indexing="ij")
        out.append(o1 + (y * wp + x) * NA + a)
        o0 += h * w * NA
        o1 += hp * wp * NA
    return np.concatenate([m.ravel() for m in out]), o1


def _boxes(rng, h, w, n):
    x1, y1 = rng.uniform(0, w - 40, n), rng.uniform(0, h - 40, n)
    bw, bh = rng.uniform(16, 400, n), rng.uniform(16, 400, n)
    b = np.stack([x1, y1, np.minimum(x1 + bw, w - 1), np.minimum(y1 + bh, h - 1), rng.integers(0, 80, n)], 1)
    b[0, :4] = [w - 120, h - 90, w - 1, h - 1]          # one box in the bottom-right corner: the padded border
    return b


@pytest.mark.parametrize("mult", [32, 128])
def test_targets_and_losses_identical_inside_images(mult):
    rng = np.random.default_rng(0)
    sizes = [(800, 1067), (800, 1201), (761, 1333)]      # one batch: the max is 800 x 1333
    H, W = max(s[0] for s in sizes), max(s[1] for s in sizes)
    Hp, Wp = pad_shape((H, W), mult)
    assert Hp % mult == 0 and Wp % mult == 0 and (Hp, Wp) != (H, W)
    idx, Ap = _index_map((H, W), (Hp, Wp))
    a0 = AN.anchors_for_shape((H, W))
    a1 = AN.anchors_for_shape((Hp, Wp))
    assert np.array_equal(a0, a1[idx])
    gts = [_boxes(rng, h, w, 9) for h, w in sizes]
    # numpy oracle (the reference's anchor_targets_bbox semantics)
    for (h, w), gt in zip(sizes, gts):
        l0, r0, s0 = AN.anchor_targets_bbox((H, W), gt, 80, mask_shape=(h, w))
        l1, r1, s1 = AN.anchor_targets_bbox((Hp, Wp), gt, 80, mask_shape=(h, w))
        assert np.array_equal(s0, s1[idx]) and np.array_equal(l0, l1[idx]) and np.array_equal(r0, r1[idx])
        extra = np.setdiff1d(np.arange(Ap), idx)
        assert (s1[extra] == -1).all()
    # the training path: batched torch targets + losses
    B, G = len(sizes), 9
    gt = torch.tensor(np.stack(gts), dtype=torch.float32)
    cnt = torch.full((B,), G, dtype=torch.int32)
    hw = torch.tensor(sizes, dtype=torch.int32)
    t0 = AN.anchor_targets_torch(torch.from_numpy(a0.astype(np.float32)), gt, cnt, hw,
                                 centers=torch.from_numpy(AN.centers_round_down(a0)))
    t1 = AN.anchor_targets_torch(torch.from_numpy(a1.astype(np.float32)), gt, cnt, hw,
                                 centers=torch.from_numpy(AN.centers_round_down(a1)))
    ti = torch.from_numpy(idx)
    for x0, x1 in zip(t0, t1):
        assert torch.equal(x0, x1[:, ti])
    assert int((t0[0] == 1).sum()) > 0
    g = torch.Generator().manual_seed(1)
    logits0 = torch.randn(B, a0.shape[0], 80, generator=g) * 3
    reg0 = torch.randn(B, a0.shape[0], 4, generator=g)
    logits1 = torch.randn(B, Ap, 80, generator=g) * 3           # anything on the added anchors
    reg1 = torch.randn(B, Ap, 4, generator=g)
    logits1[:, ti] = logits0
    reg1[:, ti] = reg0
    f0 = focal_loss(logits0, t0[0], t0[1], backend="torch")
    f1 = focal_loss(logits1, t1[0], t1[1], backend="torch")
    s0 = smooth_l1_loss(reg0, t0[2], t0[0], backend="torch")
    s1 = smooth_l1_loss(reg1, t1[2], t1[0], backend="torch")
    assert torch.allclose(f0, f1, rtol=1e-5, atol=0) and torch.allclose(s0, s1, rtol=1e-5, atol=0)


def test_generator_pads_to_multiple():
    from batchai_retinanet_horovod_coco_amd.data.synthetic import SyntheticGenerator
    g = SyntheticGenerator(num_images=4, height=150, width=210, batch_size=2, image_min_side=100,
                           image_max_side=180, cache_bytes=0, pad_multiple=32)
    b = g.compute_input_output(g.groups[0])
    H, W = b["images"].shape[1:3]
    assert H % 32 == 0 and W % 32 == 0
    hw = b["image_hw"]
    assert (hw[:, 0] <= H).all() and (hw[:, 1] <= W).all() and (hw[:, 0] > H - 32).any()
    img = b["images"]
    for i in range(2):
        h, w = int(hw[i, 0]), int(hw[i, 1])
        assert float(img[i, h:].abs().sum()) == 0 and float(img[i, :, w:].abs().sum()) == 0
    assert pad_shape((800, 1333, 3), 128) == (896, 1408, 3) and pad_shape((800, 1333), 0) == (800, 1333)


@pytest.mark.gpu
def test_device_preprocessor_pads_to_multiple_gpu():
    """The device batch assembly (HIP warp / resize into the padded batch) pads like the host path."""
    from batchai_retinanet_horovod_coco_amd.data.device_preprocess import DevicePreprocessor
    from batchai_retinanet_horovod_coco_amd.data.synthetic import SyntheticGenerator
    kw = dict(num_images=4, height=150, width=210, batch_size=2, image_min_side=100, image_max_side=180,
              cache_bytes=0)
    host = SyntheticGenerator(pad_multiple=32, **kw)
    want = host.compute_input_output(host.groups[0])
    g = SyntheticGenerator(pad_multiple=32, **kw)
    assert g.enable_device_preprocess(torch.device("cuda"))
    assert isinstance(g.device_preprocessor, DevicePreprocessor) and g.device_preprocessor.pad_multiple == 32
    got = g.compute_input_output(g.groups[0])
    assert got["images"].shape == want["images"].shape and got["images"].shape[1] % 32 == 0
    assert torch.equal(got["image_hw"], want["image_hw"])
    torch.testing.assert_close(got["images"].cpu(), want["images"], atol=2e-3, rtol=1e-5)


def _process_batches(device, pad, n=3):
    from batchai_retinanet_horovod_coco_amd.data import process_loader
    from batchai_retinanet_horovod_coco_amd.data.device_preprocess import DevicePreprocessor
    from batchai_retinanet_horovod_coco_amd.data.synthetic import SyntheticGenerator
    g = SyntheticGenerator(num_images=6, height=150, width=210, batch_size=2, image_min_side=100,
                           image_max_side=180, seed=4, cache_bytes=0, pad_multiple=pad)
    g.device_preprocessor = DevicePreprocessor(device, 100, 180, pad_multiple=pad)
    assert process_loader.prestart()
    enq = process_loader.ProcessEnqueuer(g, workers=2, max_queue_size=2, device=device).start()
    try:
        return [enq.get() for _ in range(n)]
    finally:
        enq.stop()


def test_process_loader_pads_to_multiple():
    """The process loader's batches are padded to --pad-multiple like the thread path (the GPU
    assembly used the plain batch max)."""
    for b in _process_batches(torch.device("cpu"), 32):
        assert b["images"].shape[1] % 32 == 0 and b["images"].shape[2] % 32 == 0


@pytest.mark.gpu
def test_process_loader_pads_to_multiple_gpu():
    """GPU assembly (HIP warp / resize into the canvas) pads to --pad-multiple and matches the host batch."""
    got = _process_batches(torch.device("cuda"), 32)
    want = _process_batches(torch.device("cpu"), 32)
    for g, w in zip(got, want):
        assert g["images"].shape[1] % 32 == 0 and g["images"].shape[2] % 32 == 0
        assert g["images"].shape == w["images"].shape
        assert torch.equal(g["image_hw"], w["image_hw"])
        torch.testing.assert_close(g["images"].float().cpu(), w["images"].float(), atol=2e-3, rtol=1e-5)


def test_pad_multiple_loss_tolerance_model():
    """Model-level effect of --pad-multiple 32 (GPU default) against the reference's batch-max padding
    (ADVICE r5): the targets are identical and the added anchors are ignored, but pixels at the largest
    image's right / bottom edge see the network's response to the zero canvas instead of the convs' own
    zero padding from the second layer on, so logits near that edge move.  The total loss of a random-init
    model stays within 2 % (measured 1.0 % here); README documents the deviation."""
    from batchai_retinanet_horovod_coco_amd import models
    torch.manual_seed(0)
    model = models.backbone("resnet50").retinanet(8).eval()
    rng = np.random.default_rng(1)
    H, W = 200, 290
    img = torch.from_numpy(rng.normal(0, 40, (2, H, W, 3)).astype(np.float32))
    hw = torch.tensor([[H, W], [H - 20, W - 30]], dtype=torch.int32)
    boxes = [_boxes(rng, int(h), int(w), 4) for h, w in hw.tolist()]
    for b in boxes:
        b[:, 4] %= 8
    gt = torch.full((2, 4, 5), -1.0)
    for i, b in enumerate(boxes):
        gt[i, :len(b)] = torch.from_numpy(b)
    cnt = torch.tensor([len(b) for b in boxes], dtype=torch.int32)
    losses = []
    for mult in (0, 32):
        Hp, Wp = pad_shape((H, W), mult)
        x = torch.zeros((2, Hp, Wp, 3))
        x[:, :H, :W] = img
        anchors = AN.anchors_for_shape((Hp, Wp))
        state, label, reg = AN.anchor_targets_torch(torch.from_numpy(anchors.astype(np.float32)), gt, cnt, hw,
                                                    centers=torch.from_numpy(AN.centers_round_down(anchors)))
        with torch.no_grad():
            out = model(x)
        losses.append(float(focal_loss(out["classification"], state, label, backend="torch") +
                            smooth_l1_loss(out["regression"], reg, state, backend="torch")))
    assert abs(losses[1] - losses[0]) <= 0.02 * abs(losses[0]), losses
