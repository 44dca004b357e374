#!/bin/bash
# selected GPU tests (TESTS, pytest args) -> driver-style bench (+ saved tuner table) -> rocprof kernel stats
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONFAULTHANDLER=1
if [ -n "$TESTS" ]; then
  echo "== pytest $TESTS"
  timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest $TESTS -m gpu -q -rA --timeout 120 --timeout-method thread > gpurun_out/pytest_sel.log 2>&1; rc=$?
  grep -E "passed|failed|FAILED|Error|worst|fp32 torch|bf16 HIP" gpurun_out/pytest_sel.log | tail -20
  if [ $rc -ne 0 ]; then echo "pytest rc=$rc -> stop"; exit $rc; fi
fi
echo "== bench"
MXR_SAVE_CONV_TABLE=gpurun_out/conv_table.json timeout -k 10 400 python -u bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2> gpurun_out/bench.err || { echo "bench rc=$?"; tail -30 gpurun_out/bench.err; exit 1; }
tail -1 gpurun_out/bench.log
python scripts/conv_budget.py gpurun_out/conv_table.json ${BUDGET_STEPS:-25} > gpurun_out/conv_budget.txt && head -25 gpurun_out/conv_budget.txt
if [ "${PROF:-1}" = "1" ]; then
  echo "== rocprof"
  R=$GRAFT_REPO_ROOT
  cd /tmp && export TMPDIR=/tmp
  MXR_CONV_TABLE=$R/gpurun_out/conv_table.json timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_hip -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 3 ${BENCH_ARGS:-} > $R/gpurun_out/prof_hip.log 2>&1 || { echo "rocprof rc=$?"; tail -20 $R/gpurun_out/prof_hip.log; exit 1; }
  python3 $R/scripts/prof_summary.py $R/gpurun_out/prof_hip/run_kernel_stats.csv --steps 6 > $R/gpurun_out/prof_summary.txt && head -40 $R/gpurun_out/prof_summary.txt
  KT=$(ls $R/gpurun_out/prof_hip/run_kernel_trace.csv $R/gpurun_out/prof_hip/*/run_kernel_trace.csv 2>/dev/null | head -1)
  if [ -n "$KT" ]; then
    TOPK=25 python3 $R/scripts/trace_overlap.py "$KT" 3 > $R/gpurun_out/overlap.txt && head -60 $R/gpurun_out/overlap.txt
    python3 $R/scripts/steady_kernels.py "$KT" 3 40 > $R/gpurun_out/steady_kernels.txt
    rm -f "$KT"
  fi
fi
