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


def test_check_rccl_mismatch_and_debug_env(monkeypatch, tmp_path):
    """bench.py exits non-zero when RCCL's own rank count differs from --gpus; rank 0 of a multi-rank run
    logs RCCL's topology / channels (NCCL_DEBUG_FILE) unless the user configured NCCL_DEBUG."""
    sys.path.insert(0, ROOT)
    import bench
    assert bench.check_rccl(None, 8) is None                       # torch path: nothing to check
    assert bench.check_rccl({"nranks": 8, "device": 0, "rank": 0}, 8) is None
    assert bench.check_rccl({"nranks": -1, "device": -1, "rank": -1}, 8) is None   # query unavailable
    assert "has 1 rank(s), expected 8" in bench.check_rccl({"nranks": 1, "device": 0, "rank": 0}, 8)
    args = bench.parse(["--gpus", "2", "--rccl-debug-dir", str(tmp_path)])
    for k in ("NCCL_DEBUG", "NCCL_DEBUG_FILE", "NCCL_DEBUG_SUBSYS"):
        monkeypatch.delenv(k, raising=False)
    bench.rccl_debug_env(args, 1, 2)
    assert "NCCL_DEBUG" not in os.environ                          # rank 1 stays quiet
    bench.rccl_debug_env(args, 0, 1)
    assert "NCCL_DEBUG" not in os.environ                          # world 1: nothing to log
    bench.rccl_debug_env(args, 0, 2)
    assert os.environ["NCCL_DEBUG"] == "INFO"
    assert os.environ["NCCL_DEBUG_FILE"].startswith(str(tmp_path)) and "%p" in os.environ["NCCL_DEBUG_FILE"]
