#!/bin/bash
# Driver-equivalent bench, then per-kernel hardware counters of the step (scripts/pmc_step.py).
#   BENCH_ARGS="--dtype fp8" NO_PMC=1 TOP=16 bash scripts/gpu_bench_pmc.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
echo "== bench"
MXR_SAVE_CONV_TABLE=gpurun_out/conv_table.json timeout -k 10 400 python -u bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
tail -1 gpurun_out/bench.log
[ -n "$NO_PMC" ] && exit 0
echo "== pmc"
MXR_CONV_TABLE=$PWD/gpurun_out/conv_table.json timeout -k 10 1000 python -u scripts/pmc_step.py run --out gpurun_out/pmc_step --top ${TOP:-16} -- ${BENCH_ARGS:-}
