#!/bin/bash
# conv_hx32.hip: numerics (hx32 variants of the halo tests), then the 3x3 microbench against conv_halo
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONFAULTHANDLER=1
echo "== pytest hx32"
timeout -k 10 300 python -u -m pytest tests/test_halo_gpu.py -x -q -k "hx32" --timeout 120 --timeout-method thread > gpurun_out/pytest_hx32.log 2>&1; rc=$?
tail -15 gpurun_out/pytest_hx32.log
if [ $rc -ne 0 ]; then echo "pytest rc=$rc -> stop"; exit $rc; fi
echo "== bench"
timeout -k 10 300 python -u scripts/bench_halo.py --pipe "" --halo "${HALO:-12,7}" --hx32 "${HX32:-0,1,2,3}" > gpurun_out/bench_hx32.log 2>&1; rc=$?
cat gpurun_out/bench_hx32.log
exit $rc
