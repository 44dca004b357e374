#!/bin/bash
# one-halo-buffer hx32 variant (6): numerics on every hx32 geometry, then the per-shape race vs 1 / 3
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_halo_gpu.py -k "hx32_6 or hx32_1" > gpurun_out/hb1_test.log 2>&1 && \
timeout -k 10 300 python -u scripts/bench_halo.py --pipe "" --halo "" --hx32 0,1,3,6 > gpurun_out/hb1_bench.log 2>&1
