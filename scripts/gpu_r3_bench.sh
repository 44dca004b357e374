#!/bin/bash
# full bench (the driver's command) + a kernel-trace profile of a short run
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
echo "== bench"
MXR_SAVE_CONV_TABLE=gpurun_out/conv_table.json timeout -k 10 400 python -u bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2> gpurun_out/bench.err; rc=$?
tail -2 gpurun_out/bench.log; tail -3 gpurun_out/bench.err
[ $rc -ne 0 ] && exit $rc
if [ -n "$PROFILE" ]; then
  echo "== profile"
  timeout -k 10 500 python -u bench.py --steps 5 --warmup 3 --profile stats --profile-dir gpurun_out/profile ${BENCH_ARGS:-} > gpurun_out/profile.log 2>&1; rc=$?
  tail -45 gpurun_out/profile.log
fi
exit $rc
