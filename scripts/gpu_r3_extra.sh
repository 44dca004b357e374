#!/bin/bash
# round-3 evidence runs: new tests, default bench + profile table, fp8 bench, R101-FPN 1024 bench + winners,
# host pipeline (process loader) bench, JPEG decode rate
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONFAULTHANDLER=1
echo "== pytest ${TESTS}"
timeout -k 10 600 python -u -m pytest ${TESTS} -m gpu -q -rf --timeout 120 --timeout-method thread > gpurun_out/pytest_extra.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/pytest_extra.log; exit 1; }
tail -2 gpurun_out/pytest_extra.log
echo "== bench bf16"
MXR_SAVE_CONV_TABLE=gpurun_out/conv_table.json timeout -k 10 400 python -u bench.py > gpurun_out/bench.log 2> gpurun_out/bench.err || { echo "bench rc=$?"; tail -20 gpurun_out/bench.err; exit 1; }
tail -1 gpurun_out/bench.log
if [ -n "$FP8" ]; then
echo "== bench fp8"
timeout -k 10 400 python -u bench.py --dtype fp8 > gpurun_out/bench_fp8.log 2> gpurun_out/bench_fp8.err || { echo "fp8 rc=$?"; tail -20 gpurun_out/bench_fp8.err; exit 1; }
tail -1 gpurun_out/bench_fp8.log
fi
if [ -n "$R101" ]; then
echo "== bench R101 1024"
MXR_SAVE_CONV_TABLE=gpurun_out/conv_table_r101.json timeout -k 10 500 python -u bench.py --backbone resnet101 --height 1024 --width 1024 > gpurun_out/bench_r101.log 2> gpurun_out/bench_r101.err || { echo "r101 rc=$?"; tail -20 gpurun_out/bench_r101.err; exit 1; }
tail -1 gpurun_out/bench_r101.log
echo "== winners R101"
MXR_WINNER_TABLE=gpurun_out/conv_table_r101.json timeout -k 10 900 python -u -m pytest tests/test_winners_gpu.py -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/winners_r101.log 2>&1 || { echo "winners rc=$?"; tail -30 gpurun_out/winners_r101.log; exit 1; }
tail -2 gpurun_out/winners_r101.log
fi
if [ -n "$LOADER" ]; then
echo "== host pipeline"
for w in 2 4 8; do
  timeout -k 10 400 python -u -m batchai_retinanet_horovod_coco_amd.bin.train --bench 5 20 --workers $w --device-preprocess --loader process --batch-size 16 --no-weights --calibrate-bn --clip-mode global --no-evaluation synthetic --num-images 128 --height 800 --width 1333 > gpurun_out/pipe_w$w.log 2>&1 || { echo "pipeline rc=$?"; tail -20 gpurun_out/pipe_w$w.log; exit 1; }
  echo "workers $w: $(grep metric gpurun_out/pipe_w$w.log | tail -1)"
done
timeout -k 10 300 python -u scripts/bench_decode.py > gpurun_out/decode.log 2>&1 && cat gpurun_out/decode.log
fi
exit 0
