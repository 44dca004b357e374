#!/bin/bash
# driver-style bench that saves the tuner table -> every winner of THAT table re-checked at its production shape
# (tests/test_winners_gpu.py, incl. the projection-block fwdp/dgradp/wgradp keys) -> copy to tuning/ by hand after
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONFAULTHANDLER=1
echo "== bench"
MXR_SAVE_CONV_TABLE=gpurun_out/conv_table.json timeout -k 10 400 python -u bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2> gpurun_out/bench.err || { echo "bench rc=$?"; tail -30 gpurun_out/bench.err; exit 1; }
tail -1 gpurun_out/bench.log
python scripts/conv_budget.py gpurun_out/conv_table.json ${BUDGET_STEPS:-25} > gpurun_out/conv_budget.txt && head -25 gpurun_out/conv_budget.txt
echo "== winners at production shapes"
MXR_WINNER_TABLE=gpurun_out/conv_table.json timeout -k 10 ${TEST_TIMEOUT:-700} python -u -m pytest tests/test_winners_gpu.py -m gpu -q -rA --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_winners.log 2>&1 || { echo "pytest rc=$?"; grep -E "FAILED|Error" gpurun_out/pytest_winners.log | head -30; tail -5 gpurun_out/pytest_winners.log; exit 1; }
tail -2 gpurun_out/pytest_winners.log
grep -cE "PASSED.*(fwdp|dgradp|wgradp)" gpurun_out/pytest_winners.log || true
