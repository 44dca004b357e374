"""Distributed semantics on CPU with gloo, world_size 2 (SURVEY §4.3 'distributed (no cluster)')."""
import os
import socket
import tempfile

import pytest
import torch
import torch.multiprocessing as mp


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init(rank, world, port):
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "RANK": str(rank),
                       "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank), "LOCAL_WORLD_SIZE": str(world)})
    from batchai_retinanet_horovod_coco_amd.parallel import runtime
    runtime.init(backend="gloo", device="cpu", timeout_s=60)
    return runtime


def _w_collectives(rank, world, port, out):
    rt = _init(rank, world, port)
    from batchai_retinanet_horovod_coco_amd import hvd
    res = {}
    t = torch.tensor([1.0, 2.0]) * (rank + 1)
    res["avg"] = hvd.allreduce(t, average=True).tolist()
    res["sum"] = hvd.allreduce(t, average=False).tolist()
    res["gather"] = hvd.allgather(torch.full((rank + 1, 2), float(rank))).tolist()
    b = torch.full((3,), float(rank))
    hvd.broadcast_(b, 1)
    res["bcast"] = b.tolist()
    res["obj"] = hvd.broadcast_object({"r": rank}, 0)
    res["ranks"] = (hvd.rank(), hvd.size(), hvd.local_rank(), hvd.local_size(), hvd.cross_rank())
    # dispatcher ops (torch.ops.mxr.*), SURVEY §2.3 N2
    t2 = torch.tensor([1.0, 2.0]) * (rank + 1)
    torch.ops.mxr.allreduce_(t2, True)
    res["op_avg"] = t2.tolist()
    b2 = torch.full((2,), float(rank))
    torch.ops.mxr.broadcast_(b2, 1)
    res["op_bcast"] = b2.tolist()
    res["op_gather"] = torch.ops.mxr.allgather(torch.full((1, 2), float(rank))).tolist()
    hvd.set_signature_check(True)
    try:
        hvd.allreduce(torch.zeros(2 + rank), name="bad")
        res["mismatch"] = "no error"
    except hvd.SignatureMismatch:
        res["mismatch"] = "raised"
    torch.save(res, os.path.join(out, "r{}.pt".format(rank)))
    rt.shutdown()


def test_collectives_world2():
    out = tempfile.mkdtemp()
    mp.spawn(_w_collectives, args=(2, _port(), out), nprocs=2, join=True)
    r0 = torch.load(os.path.join(out, "r0.pt"), weights_only=False)
    r1 = torch.load(os.path.join(out, "r1.pt"), weights_only=False)
    assert r0["avg"] == [1.5, 3.0] and r1["avg"] == [1.5, 3.0]
    assert r0["sum"] == [3.0, 6.0]
    assert r0["gather"] == [[0.0, 0.0], [1.0, 1.0], [1.0, 1.0]]
    assert r0["bcast"] == [1.0, 1.0, 1.0]
    assert r1["obj"] == {"r": 0}
    assert r1["ranks"] == (1, 2, 1, 2, 0)
    assert r0["mismatch"] == "raised" and r1["mismatch"] == "raised"
    assert r0["op_avg"] == [1.5, 3.0] and r1["op_avg"] == [1.5, 3.0]
    assert r0["op_bcast"] == [1.0, 1.0] and r0["op_gather"] == [[0.0, 0.0], [1.0, 1.0]]


def _linear_setup(seed=0):
    torch.manual_seed(seed)
    model = torch.nn.Sequential(torch.nn.Linear(6, 5), torch.nn.Linear(5, 3))
    X = torch.randn(8, 6)
    Y = torch.randn(8, 3)
    return model, X, Y


def _train(model, X, Y, clip_mode, world, rank, steps=3, clipnorm=0.5):
    from batchai_retinanet_horovod_coco_amd.parallel.distributed_optimizer import DistributedOptimizer
    from batchai_retinanet_horovod_coco_amd.train.flat import FlatParams, backward_order
    from batchai_retinanet_horovod_coco_amd.train.optimizer import KerasAdam
    flat = FlatParams(backward_order(model))
    opt = DistributedOptimizer(KerasAdam(flat, lr=0.05, clipnorm=clipnorm), clip_mode=clip_mode,
                               bucket_bytes=64)   # tiny buckets -> several, exercises ordering
    n = X.shape[0] // world
    xs, ys = X[rank * n:(rank + 1) * n], Y[rank * n:(rank + 1) * n]
    for _ in range(steps):
        opt.zero_grad()
        loss = ((model(xs) - ys) ** 2).mean()
        loss.backward()
        opt.step()
    return flat.data.clone(), len(opt.buckets)


def _w_dopt(rank, world, port, out, clip_mode):
    rt = _init(rank, world, port)
    model, X, Y = _linear_setup()
    w, nb = _train(model, X, Y, clip_mode, world, rank)
    torch.save({"w": w, "nb": nb}, os.path.join(out, "r{}.pt".format(rank)))
    rt.shutdown()


@pytest.mark.parametrize("clip_mode", ["global", "local"])
def test_distributed_optimizer_equivalence(clip_mode):
    out = tempfile.mkdtemp()
    mp.spawn(_w_dopt, args=(2, _port(), out, clip_mode), nprocs=2, join=True)
    r0 = torch.load(os.path.join(out, "r0.pt"))
    r1 = torch.load(os.path.join(out, "r1.pt"))
    assert torch.equal(r0["w"], r1["w"])          # replicas stay identical
    assert r0["nb"] > 1
    model, X, Y = _linear_setup()
    from batchai_retinanet_horovod_coco_amd.train.flat import FlatParams, backward_order
    from batchai_retinanet_horovod_coco_amd.train.optimizer import KerasAdam
    flat = FlatParams(backward_order(model))
    opt = KerasAdam(flat, lr=0.05, clipnorm=0.5)
    for _ in range(3):
        flat.zero_grad()
        if clip_mode == "global":
            # mean over the full batch == average of the two equal halves, clipped once
            ((model(X) - Y) ** 2).mean().backward()
            opt.step()
        else:
            # reference semantics: each half clipped with its own norm, then averaged
            gs = []
            for h in range(2):
                flat.zero_grad()
                ((model(X[4 * h:4 * h + 4]) - Y[4 * h:4 * h + 4]) ** 2).mean().backward()
                g = flat.grad.clone()
                gs.append(g * opt.clip_factor(torch.linalg.vector_norm(g)))
            flat.grad.copy_((gs[0] + gs[1]) / 2)
            opt.apply(torch.ones(()))
    assert torch.allclose(r0["w"], flat.data, atol=1e-6)


def _w_trainer(rank, world, port, out):
    rt = _init(rank, world, port)
    from batchai_retinanet_horovod_coco_amd import models
    from batchai_retinanet_horovod_coco_amd.data.synthetic import make_batch
    from batchai_retinanet_horovod_coco_amd.parallel.callbacks import BroadcastGlobalVariablesCallback
    from batchai_retinanet_horovod_coco_amd.train.engine import Trainer
    torch.manual_seed(100 + rank)          # different init per rank -> broadcast must unify
    model = models.backbone("resnet18").retinanet(4)
    tr = Trainer(model, lr=1e-4, clip_mode="global", device=torch.device("cpu"))
    cb = BroadcastGlobalVariablesCallback(0)
    cb.set_model(tr)
    cb.on_train_begin()
    g = torch.Generator()
    g.manual_seed(rank)
    for _ in range(2):
        b = make_batch(1, 64, 96, num_classes=4, max_boxes=3, generator=g)
        logs = tr.train_on_batch(b["images"], b["gt"], b["gt_count"], b["image_hw"])
    torch.save({"w": tr.flat.data.clone(), "loss": float(logs["loss"])}, os.path.join(out, "r{}.pt".format(rank)))
    rt.shutdown()


def test_trainer_replicas_stay_in_sync():
    out = tempfile.mkdtemp()
    mp.spawn(_w_trainer, args=(2, _port(), out), nprocs=2, join=True)
    r0 = torch.load(os.path.join(out, "r0.pt"))
    r1 = torch.load(os.path.join(out, "r1.pt"))
    assert torch.equal(r0["w"], r1["w"])
    assert r0["loss"] == r0["loss"]


def _w_metric_avg(rank, world, port, out):
    rt = _init(rank, world, port)
    from batchai_retinanet_horovod_coco_amd.parallel.callbacks import MetricAverageCallback
    cb = MetricAverageCallback()
    logs = {"loss": float(rank + 1), "regression_loss": 2.0 * rank}
    cb.on_epoch_end(0, logs)
    torch.save(logs, os.path.join(out, "r{}.pt".format(rank)))
    rt.shutdown()


def test_metric_average():
    out = tempfile.mkdtemp()
    mp.spawn(_w_metric_avg, args=(2, _port(), out), nprocs=2, join=True)
    for r in (0, 1):
        logs = torch.load(os.path.join(out, "r{}.pt".format(r)))
        assert logs == {"loss": 1.5, "regression_loss": 1.0}


def test_fake_local_size(monkeypatch):
    from batchai_retinanet_horovod_coco_amd.parallel import runtime
    runtime.shutdown()
    monkeypatch.setenv("RANK", "3")
    monkeypatch.setenv("WORLD_SIZE", "1")
    monkeypatch.setenv("MXR_FAKE_LOCAL_SIZE", "2")
    runtime._S.initialized = False
    runtime.init(device="cpu")
    assert runtime.local_rank() == 1 and runtime.local_size() == 2 and runtime.cross_rank() == 1
    runtime.shutdown()


def test_mxr_ops_fake_shapes():
    """The dispatcher ops have fake kernels (usable under FakeTensorMode / tracing)."""
    from torch._subclasses.fake_tensor import FakeTensorMode
    from batchai_retinanet_horovod_coco_amd.parallel import ops  # noqa: F401
    with FakeTensorMode():
        x = torch.empty(3, 4)
        y = torch.ops.mxr.allgather(x)
        torch.ops.mxr.allreduce_(x, True)
    assert tuple(y.shape) == (3, 4)       # world size 1 outside a process group


def _w_hier(rank, world, port, out):
    os.environ["MXR_FAKE_LOCAL_SIZE"] = "2"
    rt = _init(rank, world, port)
    from batchai_retinanet_horovod_coco_amd.parallel import collectives
    collectives.set_hierarchical(True)
    assert collectives._use_hier()
    t = torch.arange(7, dtype=torch.float32) * (rank + 1)
    res = {"hier": collectives.allreduce(t, average=True).tolist()}
    collectives.set_hierarchical(False)
    res["flat"] = collectives.allreduce(t, average=True).tolist()
    torch.save(res, os.path.join(out, "r{}.pt".format(rank)))
    rt.shutdown()


def test_hierarchical_allreduce_world4():
    """Two-level all-reduce over 2 fake nodes x 2 ranks equals the flat one."""
    out = tempfile.mkdtemp()
    mp.spawn(_w_hier, args=(4, _port(), out), nprocs=4, join=True)
    for r in range(4):
        res = torch.load(os.path.join(out, "r{}.pt".format(r)))
        assert res["hier"] == res["flat"] == [2.5 * i for i in range(7)]


def _w_tuner_sync(rank, world, port, out):
    rt = _init(rank, world, port)
    from batchai_retinanet_horovod_coco_amd.ops.conv_tuner import ConvTuner
    t = ConvTuner()
    t.table = {"k1": "hip%d" % rank, "k2": "halo7", "k%d" % (rank + 3): "x"}
    n = t.sync(0)
    torch.save({"table": t.table, "changed": n}, os.path.join(out, "r{}.pt".format(rank)))
    rt.shutdown()


def test_tuner_sync_adopts_rank0_choices():
    out = tempfile.mkdtemp()
    mp.spawn(_w_tuner_sync, args=(2, _port(), out), nprocs=2, join=True)
    r0 = torch.load(os.path.join(out, "r0.pt"))
    r1 = torch.load(os.path.join(out, "r1.pt"))
    assert r0["changed"] == 0 and r1["changed"] == 2
    assert r1["table"]["k1"] == "hip0" and r1["table"]["k2"] == "halo7" and r1["table"]["k3"] == "x"


def _w_tuner_sync_all(rank, world, port, out):
    rt = _init(rank, world, port)
    from batchai_retinanet_horovod_coco_amd.ops.conv_tuner import ConvTuner
    t = ConvTuner()
    # k1 tuned by both (rank 0 wins), k_r only by rank r (a shape first seen after step 0 on that rank)
    t.table = {"k1": "hip%d" % rank, "k_%d" % rank: "halo%d" % rank}
    n = t.sync_all()
    torch.save({"table": t.table, "changed": n}, os.path.join(out, "r{}.pt".format(rank)))
    rt.shutdown()


def test_tuner_sync_all_merges_new_keys_lowest_rank_wins():
    out = tempfile.mkdtemp()
    mp.spawn(_w_tuner_sync_all, args=(2, _port(), out), nprocs=2, join=True)
    r0 = torch.load(os.path.join(out, "r0.pt"))
    r1 = torch.load(os.path.join(out, "r1.pt"))
    want = {"k1": "hip0", "k_0": "halo0", "k_1": "halo1"}
    assert r0["table"] == want and r1["table"] == want
    assert r0["changed"] == 1 and r1["changed"] == 2


def test_tuner_sync_cadence():
    from batchai_retinanet_horovod_coco_amd.ops.conv_tuner import ConvTuner
    due = [s for s in range(0, 10000) if ConvTuner.sync_due(s)]
    assert due[:6] == [0, 1, 2, 4, 8, 16] and 4096 in due and 3000 not in due
    assert 6144 in due and 8192 in due and 5000 not in due


def _w_dopt_abandon(rank, world, port, out):
    """A step abandoned after its backward launched bucket all-reduces (no step()): zero_grad must wait
    for them before zeroing, so the next steps match a run that never saw the abandoned step."""
    rt = _init(rank, world, port)
    from batchai_retinanet_horovod_coco_amd.parallel.distributed_optimizer import DistributedOptimizer
    from batchai_retinanet_horovod_coco_amd.train.flat import FlatParams, backward_order
    from batchai_retinanet_horovod_coco_amd.train.optimizer import KerasAdam
    res = {}
    for abandon in (False, True):
        model, X, Y = _linear_setup()
        flat = FlatParams(backward_order(model))
        opt = DistributedOptimizer(KerasAdam(flat, lr=0.05, clipnorm=0.5), clip_mode="global", bucket_bytes=64)
        xs, ys = X[rank * 4:(rank + 1) * 4], Y[rank * 4:(rank + 1) * 4]
        if abandon:
            opt.zero_grad()
            ((model(xs) * 7.0 - ys) ** 2).mean().backward()   # buckets launch from the hooks, then: abandoned
        for _ in range(3):
            opt.zero_grad()
            ((model(xs) - ys) ** 2).mean().backward()
            opt.step()
        res[abandon] = flat.data.clone()
    torch.save(res, os.path.join(out, "r{}.pt".format(rank)))
    rt.shutdown()


def test_zero_grad_after_abandoned_step_matches_fresh_run():
    out = tempfile.mkdtemp()
    mp.spawn(_w_dopt_abandon, args=(2, _port(), out), nprocs=2, join=True)
    for r in range(2):
        res = torch.load(os.path.join(out, "r{}.pt".format(r)))
        assert torch.equal(res[False], res[True])


def test_xgmi_bucket_model():
    """parallel/xgmi.py: the default 25 MiB buckets fill every channel at world 8; smaller buckets under-fill
    the rings; the R50 gradient (151.7 MB fp32) models well under 1 ms at world 8."""
    from batchai_retinanet_horovod_coco_amd.parallel import xgmi
    assert xgmi.min_bucket_bytes(8) == 7 * 8 * 256 * 1024
    big = xgmi.estimate(25 * 2 ** 20, 8)
    small = xgmi.estimate(2 * 2 ** 20, 8)
    assert big.fill == 1.0 and small.fill < 1.0
    assert small.us / (2 * 2 ** 20) > big.us / (25 * 2 ** 20)      # per-byte cost rises below the floor
    p = xgmi.plan([25 * 2 ** 20] * 5 + [26 * 2 ** 20], 8)
    assert 200 < p["total_us"] < 1000 and p["min_fill"] == 1.0
    assert xgmi.plan([2 ** 20], 1)["total_us"] == 0.0          # one rank: nothing to reduce
