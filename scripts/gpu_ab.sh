#!/bin/bash
# usage: gpu_ab.sh VAR[=VALUE] [test files...]: GPU tests, then bench A/B on one tuned table: default,
# VAR=VALUE (VALUE defaults to 0), default
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONFAULTHANDLER=1
VAR=$1; shift
case "$VAR" in *=*) ;; *) VAR="$VAR=0" ;; esac
if [ $# -gt 0 ]; then
  echo "== tests $*"
  timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread "$@" > gpurun_out/pytest_ab.log 2>&1 || { tail -40 gpurun_out/pytest_ab.log; exit 1; }
  grep -E "passed|failed" gpurun_out/pytest_ab.log | tail -2
fi
echo "== bench (tunes)"
MXR_SAVE_CONV_TABLE=gpurun_out/conv_table.json timeout -k 10 600 python bench.py --verbose > gpurun_out/bench_a1.log 2>&1 || { tail -30 gpurun_out/bench_a1.log; exit 1; }
tail -1 gpurun_out/bench_a1.log | cut -c1-300
echo "== bench $VAR"
env $VAR MXR_CONV_TABLE=gpurun_out/conv_table.json timeout -k 10 600 python bench.py > gpurun_out/bench_b.log 2>&1 || { tail -30 gpurun_out/bench_b.log; exit 1; }
tail -1 gpurun_out/bench_b.log | cut -c1-300
echo "== bench default again"
MXR_CONV_TABLE=gpurun_out/conv_table.json timeout -k 10 600 python bench.py > gpurun_out/bench_a2.log 2>&1 || { tail -30 gpurun_out/bench_a2.log; exit 1; }
tail -1 gpurun_out/bench_a2.log | cut -c1-300
