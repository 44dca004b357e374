#!/usr/bin/env python
"""Steady-state per-kernel table from a rocprofv3 --kernel-trace csv: the last ``steps`` training steps
(a step ends at the fused Adam kernel), ms/step by family (prof_summary.FAMILIES) and the top kernels,
plus the library (MIOpen / CK / at::native) share the VERDICT asks to keep under 0.5 % of the step.

usage: steady_kernels.py run_kernel_trace.csv [steps=3] [top=30]
PER_CALL=<regex>: also list every call of the last step whose kernel name matches (grid, LDS, us)."""
import csv
import os
import re
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from prof_summary import FAMILIES  # noqa: E402

LIBRARY = r"at::native|igemm_|ck::|naive_conv|MIOpen|miopen|Cat|rocblas|Cijk_"


def main():
    path = sys.argv[1]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 30
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                         r.get("Grid_Size", r.get("Grid_Size_X", "?")), r.get("LDS_Block_Size", r.get("Lds_Size", "?"))))
    rows.sort()
    ends = [i for i, r in enumerate(rows) if "adam_kernel" in r[2]]
    if len(ends) < steps + 1:
        print("only %d step markers" % len(ends))
        return
    win = rows[ends[-steps - 1] + 1:ends[-1] + 1]
    wall = (max(r[1] for r in win) - win[0][0]) / steps / 1e6
    per = defaultdict(lambda: [0.0, 0])
    for s, e, n, _, _ in win:
        per[n][0] += (e - s) / steps / 1e6
        per[n][1] += 1
    ksum = sum(v[0] for v in per.values())
    print("last %d steps: wall %.2f ms/step, kernel time %.2f ms/step, %d launches/step"
          % (steps, wall, ksum, len(win) // steps))
    fam = defaultdict(float)
    for n, (t, _) in per.items():
        for name, pat in FAMILIES:
            if re.search(pat, n):
                fam[name] += t
                break
        else:
            fam["other"] += t
    for name, t in sorted(fam.items(), key=lambda kv: -kv[1]):
        print("  %-22s %7.3f ms/step  %5.1f%%" % (name, t, 100 * t / wall))
    lib = {n: v for n, v in per.items() if re.search(LIBRARY, n)}
    lt = sum(v[0] for v in lib.values())
    print("library kernels (MIOpen / CK / at::native / rocBLAS): %.3f ms/step = %.2f%% of the step"
          % (lt, 100 * lt / wall))
    for n, (t, c) in sorted(lib.items(), key=lambda kv: -kv[1][0]):
        print("    %7.3f ms/step  x%-4.0f %s" % (t, c / steps, n[:150]))
    print("top kernels:")
    for n, (t, c) in sorted(per.items(), key=lambda kv: -kv[1][0])[:top]:
        print("  %7.3f ms/step %5.1f%%  x%-4.0f %s" % (t, 100 * t / wall, c / steps, n[:140]))
    pc = os.environ.get("PER_CALL")
    if pc:
        last = rows[ends[-2] + 1:ends[-1] + 1]
        print("calls of the last step matching %r (start offset us, duration us, grid, LDS):" % pc)
        for s, e, n, grid, lds in last:
            if re.search(pc, n):
                print("  %9.1f %8.1f  grid %-9s lds %-7s %s" % ((s - last[0][0]) / 1e3, (e - s) / 1e3, grid, lds, n[:90]))


if __name__ == "__main__":
    main()
