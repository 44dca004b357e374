#!/usr/bin/env python
"""Per-step conv time budget from a saved tuner table (MXR_SAVE_CONV_TABLE): for every key, calls per
step x the chosen candidate's tuned time, sorted -- where the conv milliseconds of a step go, and
what the runner-up would cost."""
import json
import sys


def main():
    path = sys.argv[1]
    steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
    d = json.load(open(path))
    table, tim, calls = d["table"], d.get("timings_ms", {}), d.get("calls", {})
    rows, tot = [], 0.0
    for k, choice in table.items():
        t = tim.get(k, {})
        best = t.get(choice)
        if not isinstance(best, float):
            continue
        n = calls.get(k, 0) / steps
        ms = n * best
        tot += ms
        others = sorted((v, c) for c, v in t.items() if isinstance(v, float) and c != choice)
        ru = "%s %.3f" % (others[0][1], others[0][0]) if others else ""
        rows.append((ms, k, choice, best, n, ru))
    rows.sort(reverse=True)
    print("conv total %.2f ms/step over %d keys" % (tot, len(rows)))
    for ms, k, c, b, n, ru in rows:
        print("%7.3f ms  x%.1f  %-8s %.4f  (next: %s)  %s" % (ms, n, c, b, ru, k))


if __name__ == "__main__":
    main()
