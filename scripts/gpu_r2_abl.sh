#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python scripts/bench_f8.py > gpurun_out/bench_f8.log 2>&1 || { tail -20 gpurun_out/bench_f8.log; exit 1; }
grep -v amdgpu.ids gpurun_out/bench_f8.log | grep "bf16\|f8_6\|f8_15"
