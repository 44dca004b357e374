#!/bin/bash
# production-shape winners on the committed table + where the remaining torch kernels come from
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONFAULTHANDLER=1
echo "== winners"
timeout -k 10 500 python -u -m pytest tests/test_winners_gpu.py -q --timeout 120 --timeout-method thread > gpurun_out/winners.log 2>&1; rc=$?
tail -6 gpurun_out/winners.log
[ $rc -gt 1 ] && exit $rc
echo "== op sources"
MXR_CONV_TABLE=tuning/conv_table.json timeout -k 10 300 python scripts/op_sources.py > gpurun_out/op_sources.log 2>&1 || { tail -20 gpurun_out/op_sources.log; exit 1; }
grep -v Warning gpurun_out/op_sources.log | head -60
