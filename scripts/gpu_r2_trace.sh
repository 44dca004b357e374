#!/bin/bash
# tuned bench, then a kernel + HIP-runtime trace of 6 steps on that table: idle gaps and whether the host
# was behind at each; then where the remaining torch ops come from
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
if [ "$1" = "tests" ]; then
  echo "== tests"
  timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_side_stream_gpu.py tests/test_fused_gpu.py tests/test_model_parity_gpu.py tests/test_kernels_gpu.py tests/test_dgrad_s2_gpu.py tests/test_fp8_gpu.py > gpurun_out/pytest_tr.log 2>&1 || { tail -30 gpurun_out/pytest_tr.log; exit 1; }
  tail -1 gpurun_out/pytest_tr.log
fi
echo "== bench"
MXR_SAVE_CONV_TABLE=gpurun_out/conv_table.json timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1 || { tail -30 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log | cut -c1-200
echo "== trace"
cd /tmp && export TMPDIR=/tmp
MXR_CONV_TABLE=$R/gpurun_out/conv_table.json timeout -k 10 400 rocprofv3 --kernel-trace --hip-runtime-trace -d $R/gpurun_out/trace -o run --output-format csv -- python3 $R/bench.py --steps 6 --warmup 3 > $R/gpurun_out/trace.log 2>&1 || { echo "rocprof rc=$?"; tail -20 $R/gpurun_out/trace.log; exit 1; }
KT=$(ls $R/gpurun_out/trace/*kernel_trace.csv $R/gpurun_out/trace/*/*kernel_trace.csv 2>/dev/null | head -1)
HT=$(ls $R/gpurun_out/trace/*hip_api_trace.csv $R/gpurun_out/trace/*/*hip_api_trace.csv 2>/dev/null | head -1)
GAPS=40 python3 $R/scripts/trace_overlap.py $KT 5 adam $HT > $R/gpurun_out/overlap.txt; cat $R/gpurun_out/overlap.txt
python3 $R/scripts/host_lead.py $KT $HT > $R/gpurun_out/host_lead.txt; tail -45 $R/gpurun_out/host_lead.txt
gzip -f $HT
cd $R
exit 0
echo "== op sources"
timeout -k 10 300 python scripts/op_sources.py > gpurun_out/op_sources.log 2>&1 || { tail -20 gpurun_out/op_sources.log; exit 1; }
grep -v Warning gpurun_out/op_sources.log | head -50
