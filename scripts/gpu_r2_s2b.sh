#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONFAULTHANDLER=1
echo "== tests"
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_dgrad_s2_gpu.py tests/test_p8_gpu.py tests/test_kernels_gpu.py > gpurun_out/pytest_s2.log 2>&1 || { tail -30 gpurun_out/pytest_s2.log; exit 1; }
tail -1 gpurun_out/pytest_s2.log
echo "== microbench"
timeout -k 10 300 python scripts/bench_f8.py > gpurun_out/bench_f8.log 2>&1 || { tail -20 gpurun_out/bench_f8.log; exit 1; }
grep -v amdgpu.ids gpurun_out/bench_f8.log | grep "bf16"
echo "== bench"
MXR_SAVE_CONV_TABLE=gpurun_out/conv_table.json timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1 || { tail -30 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log | cut -c1-250
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/conv_table.json"))
for k, v in d["table"].items():
    if "|3|2|" in k and k.startswith("dgrad"):
        t = d["timings_ms"][k]
        print(k, "->", v, sorted((round(x, 4), n) for n, x in t.items() if isinstance(x, float))[:4])
PY
