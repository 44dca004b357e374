#!/bin/bash
# round 6: graph-captured step through the native engine + side stream in the graph (tests), graph vs eager at
# B=1 / 16, and a kernel trace of the B=1 graph replay (GPU busy under replay).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONFAULTHANDLER=1
R=$GRAFT_REPO_ROOT
timeout -k 10 700 python -u -m pytest ${TESTS:-tests/test_graph_native_gpu.py tests/test_fused_gpu.py::test_graph_step_matches_eager tests/test_fp8_gpu.py::test_fp8_focal_without_grad_sinks tests/test_pad_classes.py tests/test_side_stream_gpu.py} \
    -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_r6.log 2>&1 \
    || { echo "pytest rc=$?"; tail -60 gpurun_out/pytest_r6.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" gpurun_out/pytest_r6.log | tail -30
for B in ${BATCHES:-1 16}; do
  for flag in "" "--graph"; do
    timeout -k 10 300 python -u bench.py --batch-size $B --steps 30 --warmup 5 $flag > gpurun_out/g.log 2> gpurun_out/g.err \
      || { echo "B=$B $flag rc=$?"; tail -20 gpurun_out/g.err; exit 1; }
    echo "B=$B ${flag:-eager}: $(tail -1 gpurun_out/g.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], "img/s", r["ms_per_step"], "ms/step")')" | tee -a gpurun_out/graph_ab.txt
  done
done
[ "${PROF:-1}" = "1" ] || exit 0
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d $R/gpurun_out/prof_g1 -o run --output-format csv -- python3 $R/bench.py --batch-size 1 --graph --steps 10 --warmup 5 > $R/gpurun_out/prof_g1.log 2>&1 || { echo "rocprof rc=$?"; tail -20 $R/gpurun_out/prof_g1.log; exit 1; }
KT=$(ls $R/gpurun_out/prof_g1/run_kernel_trace.csv $R/gpurun_out/prof_g1/*/run_kernel_trace.csv 2>/dev/null | head -1)
TOPK=10 python3 $R/scripts/trace_overlap.py "$KT" 5 > $R/gpurun_out/overlap_g1.txt && head -30 $R/gpurun_out/overlap_g1.txt
rm -f "$KT"
