#!/bin/bash
# isolate the fp8 one-step loss regression: default, hx8 excluded from the tuner, fp8 pack emission off
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for arm in "X=1" "MXR_CONV_EXCLUDE=f8_2" "MXR_FP8_PACK_EMIT=0"; do
  env $arm timeout -k 10 200 python -u -m pytest tests/test_fp8_gpu.py -m gpu -q -x --timeout 150 --timeout-method thread -k "retinanet_step" > gpurun_out/diag_fp8_step.log 2>&1
  echo "$arm rc=$? $(grep -o "AssertionError: {.*}" gpurun_out/diag_fp8_step.log | head -1) $(grep -o '[0-9]* passed' gpurun_out/diag_fp8_step.log)"
done
