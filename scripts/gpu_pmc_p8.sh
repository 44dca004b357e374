#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc_p8
cd /tmp && export TMPDIR=/tmp
G1="SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY"
G2="SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
for v in p8_0 p8_1 blas; do
  for gi in 1 2; do
    eval G=\$G$gi
    timeout -s KILL 90 rocprofv3 --pmc $G -d $R/gpurun_out/pmc_p8/${v}_$gi -o run --output-format csv -- python3 $R/scripts/pmc_p8.py $v > $R/gpurun_out/pmc_p8/${v}_$gi.log 2>&1 || { echo "pmc $v $gi failed"; tail -5 $R/gpurun_out/pmc_p8/${v}_$gi.log; exit 1; }
  done
done
python3 - <<'PY'
import csv, glob, collections, os
R = os.environ["GRAFT_REPO_ROOT"]
for v in ("p8_0", "p8_1", "blas"):
    acc = collections.defaultdict(float); disp = collections.defaultdict(set)
    for f in glob.glob(R + "/gpurun_out/pmc_p8/%s_*/**/run_counter_collection.csv" % v, recursive=True):
        for r in csv.DictReader(open(f)):
            kn = r["Kernel_Name"]
            if not ("conv_p8" in kn or "conv_p4" in kn or "Cijk" in kn or "gemm" in kn.lower()):
                continue
            acc[r["Counter_Name"]] += float(r["Counter_Value"]); disp[r["Counter_Name"]].add(r["Dispatch_Id"])
    print("==", v)
    for k in sorted(acc):
        print("  %-26s per-dispatch %.4g" % (k, acc[k] / max(1, len(disp[k]))))
PY
