#!/bin/bash
# Effective shader clock of one head conv pass with random vs all-zero input: GRBM_GUI_ACTIVE (summed over the
# 8 XCDs) over the kernel's duration from the same rocprofv3 run.  Usage: gpu_clock_probe.sh KIND VARIANT
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/clock
cd /tmp && export TMPDIR=/tmp
for z in 0 1; do
  PMC_ZERO_X=$z timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES --kernel-trace -d $R/gpurun_out/clock/z$z -o run --output-format csv -- python3 $R/scripts/pmc_pyr.py $1 $2 > $R/gpurun_out/clock/z$z.log 2>&1 || { echo "probe $z failed"; tail -5 $R/gpurun_out/clock/z$z.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, os
R = os.environ["GRAFT_REPO_ROOT"]
for z in (0, 1):
    rows = []
    for f in glob.glob(R + "/gpurun_out/clock/z%d/**/run_counter_collection.csv" % z, recursive=True):
        for r in csv.DictReader(open(f)):
            if "conv" in r["Kernel_Name"] and r["Counter_Name"] == "GRBM_GUI_ACTIVE":
                rows.append(r)
    durs = {}
    for f in glob.glob(R + "/gpurun_out/clock/z%d/**/run_kernel_trace.csv" % z, recursive=True):
        for r in csv.DictReader(open(f)):
            if "conv" in r["Kernel_Name"]:
                durs[r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    for r in rows:
        d = durs.get(r["Dispatch_Id"])
        if d:
            print("%s x: dispatch %s  %.3f ms  GRBM_GUI_ACTIVE %.4g  -> %.2f GHz per XCD" % (
                "zero" if z else "randn", r["Dispatch_Id"], d * 1e3, float(r["Counter_Value"]),
                float(r["Counter_Value"]) / 8 / d / 1e9))
PY
