#!/bin/bash
# conv1x1_pers: GPU numerics tests, then the microbenchmark against the other 1x1 candidates
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_c1p_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/c1p_tests.log 2>&1; rc=$?
tail -15 gpurun_out/c1p_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/bench_c1p.py --reps 15 > gpurun_out/bench_c1p.log 2>&1 || { tail -20 gpurun_out/bench_c1p.log; exit 1; }
cat gpurun_out/bench_c1p.log
[ -n "$SHAPES" ] && MXR_BENCH_STEPS_DETAIL=1 PADS="32" STEPS=40 RUN_TIMEOUT=400 bash scripts/gpu_shape_classes.sh
exit 0
