"""Aggregate rocprofv3 counter_collection.csv per (kernel, counter) for kernels matching a pattern."""
import csv
import sys
from collections import defaultdict


def main():
    path, pat = sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "conv"
    agg = defaultdict(float)
    disp = defaultdict(set)
    dur = {}
    for r in csv.DictReader(open(path)):
        if pat not in r["Kernel_Name"]:
            continue
        key = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0][-60:]
        agg[(key, r["Counter_Name"])] += float(r["Counter_Value"])
        disp[key].add(r["Dispatch_Id"])
        dur[(key, r["Dispatch_Id"])] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    for (k, c), v in sorted(agg.items()):
        n = len(disp[k])
        print("{:60s} {:28s} {:16.4g} per-dispatch {:14.4g}".format(k, c, v, v / n))
    for k in disp:
        ds = [dur[(k, d)] for d in disp[k]]
        print("{:60s} dispatches {} mean dur {:.1f} us".format(k, len(ds), sum(ds) / len(ds) / 1e3))


if __name__ == "__main__":
    main()
