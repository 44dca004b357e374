#!/usr/bin/env python
"""Stream overlap of the last steps of a rocprofv3 --kernel-trace run: wall time, GPU-busy time (union of
kernel intervals), kernel-time sum (> busy when streams overlap), idle gaps, and busy time per stream.

usage: trace_overlap.py run_kernel_trace.csv [steps=3] [step_marker=adam]
A step ends at the last kernel whose name contains ``step_marker`` (the fused Adam kernel)."""
import csv
import sys
from collections import defaultdict


def union(iv):
    tot, cur_s, cur_e = 0, None, None
    for s, e in sorted(iv):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def main():
    path = sys.argv[1]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    marker = sys.argv[3] if len(sys.argv) > 3 else "adam"
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r["Queue_Id"]))
    rows.sort()
    ends = [i for i, r in enumerate(rows) if marker in r[2].lower()]
    if len(ends) < steps + 1:
        print("only %d step markers" % len(ends))
        return
    a, b = ends[-steps - 1] + 1, ends[-1] + 1
    win = rows[a:b]
    t0, t1 = win[0][0], max(r[1] for r in win)
    wall = t1 - t0
    busy = union([(s, e) for s, e, _, _ in win])
    ksum = sum(e - s for s, e, _, _ in win)
    print("steps %d  wall %.2f ms/step  busy %.2f ms/step (%.1f %%)  kernel-sum %.2f ms/step  overlap x%.2f"
          % (steps, wall / steps / 1e6, busy / steps / 1e6, 100.0 * busy / wall, ksum / steps / 1e6, ksum / max(busy, 1)))
    per_q = defaultdict(list)
    for s, e, n, q in win:
        per_q[q].append((s, e))
    for q, iv in sorted(per_q.items()):
        print("  queue %s: %d kernels, busy %.2f ms/step" % (q, len(iv), union(iv) / steps / 1e6))
    gaps = []
    last_e = t0
    for s, e, n, q in win:
        if s > last_e:
            gaps.append((s - last_e, n))
        last_e = max(last_e, e)
    gaps.sort(reverse=True)
    print("  idle %.2f ms/step in %d gaps; largest before:" % (sum(g for g, _ in gaps) / steps / 1e6, len(gaps)))
    for g, n in gaps[:12]:
        print("    %7.1f us  %s" % (g / 1e3, n[:110]))


if __name__ == "__main__":
    main()
