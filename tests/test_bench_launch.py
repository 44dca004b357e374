"""bench.py's multi-rank contract on CPU (gloo): ``--gpus N`` starts N ranks itself and rank 0
prints ONE JSON line with ``n_gpus == N``; under a launcher the world size must match ``--gpus``."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TINY = ["--backbone", "resnet18", "--height", "64", "--width", "96", "--batch-size", "1", "--steps", "2",
        "--warmup", "1", "--no-calibrate-bn"]


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "OMPI_COMM_WORLD_SIZE", "PMI_SIZE")}
    env.update(OMP_NUM_THREADS="2", **kw)
    return env


def test_bench_spawns_ranks_gpus2():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"] + TINY, cwd=ROOT,
                       env=_env(), stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["config"]["parallelism"] == "dp2"
    assert res["config"]["global_batch"] == 2 and res["value"] > 0
    assert res["ms_per_step"] > 0 and res["steps"] == 2 and res["warmup"] == 1


def test_bench_rejects_world_mismatch():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"] + TINY, cwd=ROOT,
                       env=_env(WORLD_SIZE="1", RANK="0"), stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                       text=True, timeout=120)
    assert r.returncode == 2 and "launcher started 1" in r.stderr
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]
