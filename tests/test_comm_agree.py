"""Agreed native-engine bring-up and the replica check (VERDICT r3 Next #4), CPU / gloo world 2.

The native RCCL engine is replaced by a fake communicator (no GPU here); what is under test is the
protocol around it: a failure on ONE rank -- at load, at ncclCommInitRank (error or a peer that never
answers), in the self-test or in setup -- must leave EVERY rank on torch.distributed (``MXR_COMM=auto``)
or make every rank raise (``MXR_COMM=native``), without a hang."""
import json
import os
import subprocess
import sys
import tempfile
import time

import pytest
import torch
import torch.multiprocessing as mp

from test_dist import _init, _port

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class FakeComm:
    """Stands in for NativeComm: the self-test reduces a rank-valued probe over its OWN gloo group (a
    separate communicator, as RCCL's is; its 5 s timeout plays the watchdog)."""
    group = None

    def __init__(self, rank, world, device, uid, hang=False):
        if hang:
            time.sleep(3600)
        assert uid == b"u" * 128
        self.rank, self.world, self.closed = rank, world, False
        self.buckets = None

    def self_test(self, timeout_s=60.0):
        import torch.distributed as dist
        FakeComm.test_timeout = timeout_s
        p = torch.full((4,), float(self.rank + 1))
        dist.all_reduce(p, group=FakeComm.group)
        assert float(p[0]) == self.world * (self.world + 1) / 2

    def set_buckets(self, ts, average=False):
        self.buckets = ts

    def watchdog(self, t):
        pass

    def close(self):
        self.closed = True


def _side_group():
    import datetime
    import torch.distributed as dist
    FakeComm.group = dist.new_group(backend="gloo", timeout=datetime.timedelta(seconds=5))


def _w_bringup(rank, world, port, out, fault, hang_rank, pg_timeout=None, init_timeout=3.0):
    if fault:
        os.environ["MXR_COMM_FAULT"] = fault
    if pg_timeout is None:
        rt = _init(rank, world, port)
    else:
        os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "RANK": str(rank),
                           "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank), "LOCAL_WORLD_SIZE": str(world),
                           "MXR_COMM_TIMEOUT": str(pg_timeout), "MXR_COMM_INIT_TIMEOUT": "180"})
        from batchai_retinanet_horovod_coco_amd.parallel import runtime as rt
        rt.init(backend="gloo", device="cpu")
    _side_group()
    from batchai_retinanet_horovod_coco_amd.parallel.native_comm import bring_up
    made = []

    def make(r, w, d, u):
        c = FakeComm(r, w, d, u, hang=(r == hang_rank))
        made.append(c)
        return c
    t0 = time.time()
    comm, why = bring_up(rank, world, 0, setup=lambda c: c.set_buckets([1]), make=make,
                         new_uid=lambda: b"u" * 128, init_timeout=init_timeout)
    res = {"ok": comm is not None, "why": why, "s": time.time() - t0, "test_timeout": FakeComm.__dict__.get("test_timeout"),
           "closed": [c.closed for c in made], "buckets": comm.buckets if comm is not None else None}
    with open(os.path.join(out, "r%d.json" % rank), "w") as f:
        json.dump(res, f)
    rt.shutdown()


def _run(fault=None, hang_rank=-1, pg_timeout=None, init_timeout=3.0):
    out = tempfile.mkdtemp()
    mp.spawn(_w_bringup, args=(2, _port(), out, fault, hang_rank, pg_timeout, init_timeout), nprocs=2, join=True)
    return [json.load(open(os.path.join(out, "r%d.json" % r))) for r in range(2)]


def test_bringup_all_ranks_succeed():
    r = _run()
    assert all(x["ok"] and x["why"] is None and x["buckets"] == [1] for x in r)


@pytest.mark.parametrize("stage", ["load", "init", "selftest", "setup"])
def test_one_rank_failure_every_rank_falls_back(stage):
    r = _run(fault="1:" + stage)
    for x in r:
        assert not x["ok"], x
        # rank 1 failed; in the self-test rank 0 also gives up (its probe never finds a partner)
        assert ("rank(s) [0, 1]" if stage == "selftest" else "rank(s) [1]") in x["why"], x["why"]
        assert x["s"] < 30
    if stage in ("selftest", "setup"):
        assert r[0]["closed"] == [True] and r[1]["closed"] == [True]   # communicators destroyed everywhere


def test_init_hang_on_one_rank_times_out_and_agrees():
    r = _run(hang_rank=1)
    for x in r:
        assert not x["ok"] and "ncclCommInitRank failed on rank(s) [1]" in x["why"], x["why"]
    assert r[0]["closed"] == [True]          # rank 0's communicator existed: destroyed before the fallback


def test_init_bound_stays_under_process_group_timeout():
    """MXR_COMM_TIMEOUT (the default group's) below MXR_COMM_INIT_TIMEOUT: a peer stuck in init must be given
    up on well before the group's watchdog fires, so every rank still reaches the agreed fallback."""
    r = _run(hang_rank=1, pg_timeout=10, init_timeout=None)
    for x in r:
        assert not x["ok"] and "ncclCommInitRank failed on rank(s) [1]" in x["why"], x["why"]
        assert x["s"] < 9, x["s"]
    r = _run(pg_timeout=10, init_timeout=None)
    assert all(x["ok"] and x["test_timeout"] <= 4.0 + 1e-9 for x in r), r


def test_stage_timeouts_clamp():
    from batchai_retinanet_horovod_coco_amd.parallel.native_comm import stage_timeouts
    assert stage_timeouts(180.0, 600.0) == (180.0, 60.0)
    assert stage_timeouts(180.0, 100.0) == (40.0, 40.0)
    assert stage_timeouts(5.0, 100.0) == (5.0, 40.0)


def _w_optimizer(rank, world, port, out, forced):
    os.environ["MXR_COMM_FAULT"] = "0:init"
    rt = _init(rank, world, port)
    _side_group()
    from batchai_retinanet_horovod_coco_amd.parallel.distributed_optimizer import DistributedOptimizer
    from batchai_retinanet_horovod_coco_amd.parallel.native_comm import CommBringUpError
    from batchai_retinanet_horovod_coco_amd.parallel.collectives import Compression
    from batchai_retinanet_horovod_coco_amd.train.flat import FlatParams
    from batchai_retinanet_horovod_coco_amd.train.optimizer import KerasAdam
    model = torch.nn.Linear(4, 3)
    flat = FlatParams(list(model.named_parameters()), torch.device("cpu"))
    dopt = DistributedOptimizer(KerasAdam(flat), clip_mode="global")
    assert dopt.native is None and dopt._fallback is None          # CPU tensors: no native engine wanted
    res = {}
    try:
        dopt._init_native(Compression.none, forced=forced, make=lambda r, w, d, u: FakeComm(r, w, d, u),
                          new_uid=lambda: b"u" * 128)
        res["raised"] = False
    except CommBringUpError as e:
        res["raised"] = True
        res["msg"] = str(e)
    res["native"] = dopt.native is not None
    res["fallback"] = dopt._fallback
    # the torch path still reduces the buckets after the agreed fallback
    t = torch.full((2,), float(rank + 1))
    from batchai_retinanet_horovod_coco_amd import hvd
    res["sum"] = hvd.allreduce(t, average=False).tolist()
    with open(os.path.join(out, "r%d.json" % rank), "w") as f:
        json.dump(res, f)
    rt.shutdown()


@pytest.mark.parametrize("forced", [False, True])
def test_distributed_optimizer_agreed_fallback(forced):
    out = tempfile.mkdtemp()
    mp.spawn(_w_optimizer, args=(2, _port(), out, forced), nprocs=2, join=True)
    for r in range(2):
        x = json.load(open(os.path.join(out, "r%d.json" % r)))
        assert not x["native"]
        assert x["raised"] == forced
        assert "rank(s) [0]" in x["fallback"]
        if forced:
            assert "MXR_COMM=native" in x["msg"]
        assert x["sum"] == [3.0, 3.0]


def _w_replicas(rank, world, port, out, break_rank):
    rt = _init(rank, world, port)
    from batchai_retinanet_horovod_coco_amd.parallel.collectives import replicas_consistent
    torch.manual_seed(0)
    a, b = torch.randn(5000), torch.randn(300)
    if rank == break_rank:
        a[1234] += 1e-6
    ok, bad = replicas_consistent([a, b])
    with open(os.path.join(out, "r%d.json" % rank), "w") as f:
        json.dump({"ok": ok, "bad": bad}, f)
    rt.shutdown()


@pytest.mark.parametrize("break_rank", [-1, 1])
def test_replicas_consistent(break_rank):
    out = tempfile.mkdtemp()
    mp.spawn(_w_replicas, args=(2, _port(), out, break_rank), nprocs=2, join=True)
    for r in range(2):
        x = json.load(open(os.path.join(out, "r%d.json" % r)))
        assert x["ok"] == (break_rank < 0) and x["bad"] == ([] if break_rank < 0 else [1])


def test_bench_exits_nonzero_on_replica_divergence():
    """bench.py at world 2 reports replicas_consistent and exits 4 when one replica was broken."""
    from test_bench_launch import TINY, _env
    for fault, rc_want, cons in ((None, 0, True), ("1", 4, False)):
        env = _env(**({"MXR_TEST_FAULT_REPLICA": fault} if fault else {}))
        r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"] + TINY, cwd=ROOT,
                           env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=300)
        assert r.returncode == rc_want, r.stderr[-3000:]
        line = [l for l in r.stdout.splitlines() if l.startswith("{")]
        assert len(line) == 1
        assert json.loads(line[0])["config"]["replicas_consistent"] is cons
        if fault:
            assert "replicas diverged" in r.stderr
