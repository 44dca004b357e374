"""Weight gradients on the side stream (ops/side_stream.py): same gradients as the serial step, with the side
stream slowed down by a spin kernel so that any missing wait (allocator reuse of x / dY, the towers' shared
input-gradient buffer, bucket readiness, optimizer join) would show up as a different result."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _grads(cuda, monkeypatch, comm, side, state, delay=0):
    """flat.grad after one step (the optimizer step ran: for the native engine that includes the
    in-place bucket all-reduces, which would corrupt a slot still being accumulated on the side stream)."""
    from batchai_retinanet_horovod_coco_amd import models
    from batchai_retinanet_horovod_coco_amd.data.synthetic import make_batch
    from batchai_retinanet_horovod_coco_amd.ops import native
    from batchai_retinanet_horovod_coco_amd.ops.side_stream import SIDE
    from batchai_retinanet_horovod_coco_amd.parallel import ops
    from batchai_retinanet_horovod_coco_amd.train.engine import Trainer
    monkeypatch.setenv("MXR_COMM", comm)
    model = models.backbone("resnet18").retinanet(8)
    model.load_state_dict(state)
    tr = Trainer(model, lr=1e-3, compute_dtype=torch.bfloat16, clip_mode="global", device=cuda,
                 bucket_bytes=4 << 20)
    g = torch.Generator().manual_seed(5)
    saved = (SIDE.enabled, SIDE.delay_cycles)
    SIDE.enabled, SIDE.delay_cycles, n0 = side, delay, SIDE.launches
    try:
        b = {k: v.to(cuda) for k, v in make_batch(2, 128, 192, num_classes=8, max_boxes=4, generator=g).items()}
        tr.train_on_batch(b["images"], b["gt"], b["gt_count"], b["image_hw"])
        torch.cuda.synchronize()
        segs = [(sg.offset, sg.numel) for sg in tr.flat.segments]
        return tr.flat.grad.clone(), SIDE.launches - n0, segs
    finally:
        SIDE.enabled, SIDE.delay_cycles = saved
        if tr.optimizer.native is not None:
            ops.set_native_comm(None)
            tr.optimizer.native.close()
        native.set_grad_sinks(None)
        native.set_compute_weights(None)


@pytest.mark.parametrize("comm", ["torch", "native"])
def test_side_stream_wgrad_matches_serial(cuda, monkeypatch, comm):
    from batchai_retinanet_horovod_coco_amd import models
    monkeypatch.setenv("MXR_CONV_FORCE", "hip")     # no tuner races: the side stream is used from step 0
    torch.manual_seed(0)
    state = {k: v.clone() for k, v in models.backbone("resnet18").retinanet(8).state_dict().items()}
    g_ser, n_ser, segs = _grads(cuda, monkeypatch, comm, False, state)
    g_ser2, _, _ = _grads(cuda, monkeypatch, comm, False, state)
    g_side, n_side, _ = _grads(cuda, monkeypatch, comm, True, state, delay=200000)
    assert n_ser == 0 and n_side > 20, (n_ser, n_side)

    def seg_err(a, b):
        # per parameter: max |a - b| / max |b| -- a lost, doubled or half-accumulated weight gradient
        # (a missing wait) is an O(1) error in its segment; bf16 run-to-run noise is ~1e-5
        out = []
        for off, n in segs:
            ref = b[off:off + n]
            out.append(float((a[off:off + n] - ref).abs().max() / ref.abs().max().clamp_min(1e-12)))
        return out

    noise = seg_err(g_ser2, g_ser)
    err = seg_err(g_side, g_ser)
    worst = max(range(len(err)), key=lambda i: err[i])
    assert err[worst] <= max(4 * noise[worst], 1e-2), (worst, err[worst], noise[worst], max(noise))


def test_side_stream_join_is_noop_without_work(cuda):
    from batchai_retinanet_horovod_coco_amd.ops.side_stream import SideStream
    s = SideStream()
    s.join()
    x = torch.ones(4, device=cuda)
    with s.run(x.device, x):
        y = x * 2
    assert s.pending
    s.join()
    assert not s.pending and float(y.sum()) == 8.0
