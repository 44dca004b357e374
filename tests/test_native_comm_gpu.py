"""Native comm core (csrc/comm/comm.hip) on one GPU: RCCL world-1 collectives and the bucket engine."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_native_comm_world1(cuda, tmp_path):
    from batchai_retinanet_horovod_coco_amd.parallel.native_comm import NativeComm
    c = NativeComm(0, 1, 0)
    t = torch.arange(1000, device=cuda, dtype=torch.float32)
    ref = t.clone()
    c.allreduce_(t)
    c.broadcast_(t, 0)
    assert torch.equal(t, ref)
    g = c.allgather(torch.ones(7, device=cuda, dtype=torch.bfloat16))
    assert g.shape == (1, 7) and float(g.float().sum()) == 7.0
    assert torch.equal(c.reduce_scatter(ref.clone()), ref)
    # bucket engine: out-of-order readiness still launches in order; wait() covers everything
    flat = torch.randn(4096, device=cuda)
    keep = flat.clone()
    c.set_buckets([flat[0:1024], flat[1024:3000], flat[3000:4096]])
    c.timeline(str(tmp_path / "tl.json"))
    for it in range(2):
        c.bucket_ready(1)
        assert c.launched() == 0
        c.bucket_ready(0)
        assert c.launched() == 2
        c.wait()
        assert c.launched() == 0
    torch.cuda.synchronize()
    assert torch.equal(flat, keep)
    c.flush_timeline()
    import json
    ev = json.load(open(tmp_path / "tl.json"))
    assert sum(e["ph"] == "B" for e in ev) == 6
    c.close()


def test_mxr_dispatcher_ops_use_native_core(cuda):
    """torch.ops.mxr.* route GPU tensors to the C++ comm core once one is installed."""
    from batchai_retinanet_horovod_coco_amd.parallel import ops
    from batchai_retinanet_horovod_coco_amd.parallel.native_comm import NativeComm
    c = NativeComm(0, 1, 0)
    ops.set_native_comm(c)
    try:
        assert ops.native_comm() is c
        t = torch.randn(513, device=cuda)
        ref = t.clone()
        torch.ops.mxr.allreduce_(t, True)
        torch.ops.mxr.broadcast_(t, 0)
        g = torch.ops.mxr.allgather(t.view(27, 19))
        torch.cuda.synchronize()
        assert torch.equal(t, ref) and g.shape == (27, 19) and torch.equal(g.flatten(), ref)
    finally:
        ops.set_native_comm(None)
        c.close()


def test_native_comm_watchdog_aborts_stalled_bucket(cuda):
    """Failure detection: a launched bucket that never completes (fault-injection hook)
    makes the watchdog abort the communicator; the next bucket call raises naming the bucket."""
    import time
    from batchai_retinanet_horovod_coco_amd.parallel.native_comm import NativeComm
    c = NativeComm(0, 1, 0)
    flat = torch.randn(2048, device=cuda)
    c.set_buckets([flat[:1024], flat[1024:]])
    c.watchdog(5.0, poll_ms=10)            # healthy buckets complete well inside the timeout
    for _ in range(3):
        c.bucket_ready(0)
        c.bucket_ready(1)
        c.wait()
    torch.cuda.synchronize()
    time.sleep(0.1)
    assert not c.aborted()
    c.watchdog(0.2, poll_ms=10, inject_bucket=1)
    c.bucket_ready(0)
    c.bucket_ready(1)
    deadline = time.time() + 10
    while not c.aborted() and time.time() < deadline:
        time.sleep(0.02)
    assert c.aborted()
    with pytest.raises(RuntimeError, match="bucket 1"):
        c.check()
    with pytest.raises(RuntimeError, match="bucket 1"):
        c.wait()
    with pytest.raises(RuntimeError, match="bucket 1"):
        c.allreduce_(flat)
    torch.cuda.synchronize()
    c.close()
