#!/bin/bash
# fp8 (BASELINE config 5) vs bf16, same box, alternating: bench.py bf16 / --dtype fp8 (fp8 weight gradients) /
# --dtype fp8 with MXR_FP8_WGRAD=0 (bf16 weight gradients), after the fp8 GPU tests (NO_TESTS=1 skips them);
# MODES picks the arms (bf16x / fp8x: with the XENV assignments; bf16s / fp8s, bf16t / fp8t: with the module switches in SWITCH, SWITCH2,
# scripts/bench_switch.py), REPS the repetitions
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_wgrad_f8_gpu.py tests/test_fp8_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/fp8_tests.log 2>&1; rc=$?
  tail -5 gpurun_out/fp8_tests.log
  [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" gpurun_out/fp8_tests.log | head -20; exit $rc; }
fi
for rep in ${REPS:-1 2}; do
  for mode in ${MODES:-bf16 fp8 fp8bw}; do
    case $mode in
      bf16) args=""; env="";;
      fp8) args="--dtype fp8"; env="";;
      fp8bw) args="--dtype fp8"; env="MXR_FP8_WGRAD=0";;
      bf16x) args=""; env="$XENV";;
      fp8x) args="--dtype fp8"; env="$XENV";;
      bf16s|bf16t) args=""; env="";;
      fp8s|fp8t) args="--dtype fp8"; env="";;
    esac
    prog="bench.py"
    case $mode in bf16s|fp8s) prog="scripts/bench_switch.py $SWITCH --";; bf16t|fp8t) prog="scripts/bench_switch.py $SWITCH2 --";; esac
    env $env timeout -k 10 400 python -u $prog $args > gpurun_out/ab_${mode}_$rep.log 2> gpurun_out/ab_${mode}_$rep.err || { echo "$mode rc=$?"; tail -20 gpurun_out/ab_${mode}_$rep.err; exit 1; }
    echo "$mode $rep: $(tail -1 gpurun_out/ab_${mode}_$rep.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], "img/s", r["ms_per_step"], "ms/step", r["dtype"])')"
  done
done
