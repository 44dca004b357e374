#!/bin/bash
# Same-box A/B of module switches on the driver-equivalent bench, alternating (REPS rounds):
#   TESTS="tests/test_x_gpu.py" REPS=2 bash scripts/ab_switch.sh - "ops.conv_launch.PROJ_FUSED=0"
# ('-' = no switch; each spec is a space-separated list of mod.NAME=value for scripts/bench_switch.py;
#  BENCH_ARGS go to every run)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONFAULTHANDLER=1
if [ -n "$TESTS" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-700} python -u -m pytest $TESTS -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_ab.log 2>&1 \
    || { echo "pytest rc=$?"; grep -E "PASS|FAIL|Error|assert" gpurun_out/pytest_ab.log | tail -40; exit 1; }
  grep -E "passed|failed" gpurun_out/pytest_ab.log | tail -3
fi
for rep in $(seq 1 ${REPS:-2}); do
  i=0
  for spec in "$@"; do
    i=$((i+1))
    if [ "$spec" = "-" ]; then prog="bench.py"; else prog="scripts/bench_switch.py $spec --"; fi
    timeout -k 10 400 python -u $prog ${BENCH_ARGS:-} > gpurun_out/abs_${i}_$rep.log 2> gpurun_out/abs_${i}_$rep.err \
      || { echo "$spec rc=$?"; tail -20 gpurun_out/abs_${i}_$rep.err; exit 1; }
    echo "[$rep] $spec: $(tail -1 gpurun_out/abs_${i}_$rep.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], "img/s", r["ms_per_step"], "ms/step")')"
  done
done
