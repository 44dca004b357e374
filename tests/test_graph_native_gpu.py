"""A HIP-graph-captured training step through the native RCCL bucket engine (VERDICT r5 Next #2): the bucket
readiness events, the in-order all-reduces on the comm stream and the optimizer's waits on the done events are
captured with the step, and a replay reproduces the eager step BIT FOR BIT (world 1, ``MXR_COMM=native``: a
one-rank RCCL communicator; every kernel of the step is deterministic -- split-K slabs, no float atomics).
The reference's per-rank workload is a small batch (``--batch-size 1``, /root/reference/train.py:365), where
the eager step is bound by the host's kernel issue; the graph removes that."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture
def cuda():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


def _run(cuda, state, batches, graphed: bool):
    from batchai_retinanet_horovod_coco_amd import models
    from batchai_retinanet_horovod_coco_amd.ops import native
    from batchai_retinanet_horovod_coco_amd.parallel import ops
    from batchai_retinanet_horovod_coco_amd.train.engine import Trainer
    native.set_grad_sinks(None)
    native.set_compute_weights(None)
    model = models.backbone("resnet18").retinanet(8)
    model.load_state_dict(state)
    tr = Trainer(model, lr=1e-4, clipnorm=0.001, compute_dtype=torch.bfloat16, clip_mode="global", device=cuda,
                 bucket_bytes=4 << 20)
    try:
        assert tr.optimizer.native is not None and len(tr.optimizer.buckets) >= 3
        b = batches[0]
        if graphed:
            step = tr.graph_step(b["images"], b["gt"], b["gt_count"], b["image_hw"], warmup=2)
        else:
            step = tr.train_on_batch
            for _ in range(2):
                step(b["images"], b["gt"], b["gt_count"], b["image_hw"])
        losses = []
        for b in batches:
            logs = step(b["images"], b["gt"], b["gt_count"], b["image_hw"])
            losses.append(logs["loss"].clone())
        torch.cuda.synchronize()
        stats = tr.optimizer.comm_stats()
        return (torch.stack(losses), tr.flat.data.clone(), tr.base_optimizer.m.clone(), tr.base_optimizer.v.clone(),
                tr.base_optimizer.iterations, stats)
    finally:
        ops.set_native_comm(None)
        tr.optimizer.native.close()
        native.set_grad_sinks(None)
        native.set_compute_weights(None)


def test_graph_replay_through_native_engine_is_bit_exact(cuda, monkeypatch):
    from batchai_retinanet_horovod_coco_amd import models
    from batchai_retinanet_horovod_coco_amd.data.synthetic import make_batch
    monkeypatch.setenv("MXR_COMM", "native")
    torch.manual_seed(0)
    state = {k: v.clone() for k, v in models.backbone("resnet18").retinanet(8).state_dict().items()}
    g = torch.Generator().manual_seed(3)
    batches = [{k: v.to(cuda) for k, v in make_batch(2, 128, 192, num_classes=8, max_boxes=4, generator=g).items()}
               for _ in range(3)]
    _run(cuda, state, batches[:1], graphed=False)          # first sight: the conv tuner races here, not below
    eager = _run(cuda, state, batches, graphed=False)
    graph = _run(cuda, state, batches, graphed=True)
    assert eager[4] == graph[4] == 5
    for name, a, b in zip(("loss", "weights", "adam m", "adam v"), eager[:4], graph[:4]):
        assert torch.equal(a, b), (name, (a.float() - b.float()).abs().max().item())
    assert eager[5] is not None and graph[5] is None       # no per-step comm timings from a replay
