"""Failure detection, fault injection and timeline on CPU with gloo."""
import json
import os
import socket
import subprocess
import sys
import tempfile
import textwrap
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


WORKER = textwrap.dedent("""
    import os, sys, torch
    sys.path.insert(0, {root!r})
    from batchai_retinanet_horovod_coco_amd.parallel import runtime
    runtime.init(backend="gloo", device="cpu", timeout_s=20)
    from batchai_retinanet_horovod_coco_amd import models
    from batchai_retinanet_horovod_coco_amd.data.synthetic import SyntheticGenerator
    from batchai_retinanet_horovod_coco_amd.parallel.callbacks import BroadcastGlobalVariablesCallback
    from batchai_retinanet_horovod_coco_amd.train.callbacks import TerminateOnNaN
    from batchai_retinanet_horovod_coco_amd.train.engine import Trainer
    from batchai_retinanet_horovod_coco_amd.train.loop import fit_generator
    torch.manual_seed(0)
    tr = Trainer(models.backbone("resnet18").retinanet(3), lr=1e-4, clip_mode="global", device=torch.device("cpu"),
                 bucket_bytes=1 << 20)
    gen = SyntheticGenerator(num_images=2, height=64, width=96, num_classes=3, max_boxes=2, batch_size=1,
                             image_min_side=64, image_max_side=96)
    h = fit_generator(tr, gen, steps_per_epoch=int(os.environ.get("STEPS", "3")), epochs=1, verbose=0, workers=0,
                      callbacks=[BroadcastGlobalVariablesCallback(0), TerminateOnNaN()])
    print("DONE", runtime.rank(), tr.base_optimizer.iterations, flush=True)
    runtime.shutdown()
""")


def _launch(world, env_extra, steps=3, timeout=240):
    port = _port()
    script = os.path.join(tempfile.mkdtemp(), "w.py")
    with open(script, "w") as f:
        f.write(WORKER.format(root=ROOT))
    procs = []
    for r in range(world):
        env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(r), WORLD_SIZE=str(world),
                   LOCAL_RANK=str(r), LOCAL_WORLD_SIZE=str(world), STEPS=str(steps), OMP_NUM_THREADS="2")
        env.update(env_extra)
        procs.append(subprocess.Popen([sys.executable, script], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.STDOUT, text=True))
    t0 = time.time()
    outs = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=max(1, timeout - (time.time() - t0)))
        except subprocess.TimeoutExpired:
            p.kill()
            out, _ = p.communicate()
            out += "\nTIMEOUT"
        outs.append((p.returncode, out))
    return outs, time.time() - t0


def test_rank_exit_is_detected_not_hung():
    """Rank 1 dies mid-training (MXR_FAULT=1:1:exit): rank 0 must fail with an error, not hang."""
    outs, dt = _launch(2, {"MXR_FAULT": "1:1:exit"})
    (rc0, out0), (rc1, _) = outs
    assert rc1 == 17                       # the injected exit code
    assert rc0 != 0 and "TIMEOUT" not in out0, out0[-2000:]
    assert dt < 200


def test_nan_injection_stops_training():
    """MXR_FAULT=0:1:nan poisons a weight; TerminateOnNaN stops every rank after that step."""
    outs, _ = _launch(1, {"MXR_FAULT": "0:1:nan"}, steps=5)
    rc, out = outs[0]
    assert rc == 0, out[-2000:]
    done = [l for l in out.splitlines() if l.startswith("DONE")]
    assert done and int(done[0].split()[2]) < 5


def test_timeline_written_per_rank():
    path = os.path.join(tempfile.mkdtemp(), "tl.json")
    outs, _ = _launch(2, {"HOROVOD_TIMELINE": path}, steps=2)
    assert all(rc == 0 for rc, _ in outs), outs[0][1][-2000:]
    for p in (path, path + ".1"):
        ev = json.load(open(p))
        names = {e.get("name") for e in ev}
        assert "READY" in names and "ALLREDUCE" in names, names


def test_nan_loss_on_one_rank_stops_every_rank():
    """Only rank 1 sees a non-finite loss (MXR_FAULT=1:1:nanloss): TerminateOnNaN's decision is
    MAX-reduced across ranks each batch, so both ranks stop after the same step instead of rank 0
    blocking in the next all-reduce until the collective timeout."""
    outs, dt = _launch(2, {"MXR_FAULT": "1:1:nanloss"}, steps=5)
    for rc, out in outs:
        assert rc == 0 and "TIMEOUT" not in out, out[-2000:]
    its = [int([l for l in out.splitlines() if l.startswith("DONE")][0].split()[2]) for _, out in outs]
    assert its[0] == its[1] == 2, its
