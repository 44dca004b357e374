#!/usr/bin/env python
"""Per-step conv time budget from a saved tuner table (MXR_SAVE_CONV_TABLE): for every key, calls per
step x the chosen candidate's tuned time, sorted -- where the conv milliseconds of a step go, and
what the runner-up would cost."""
import ast
import json
import sys


def flops(key: str) -> float:
    """2 * MACs of the pass named by a tuner key (0 if the key is not understood)."""
    try:
        parts = key.split("|")
        kind = parts[0]
        if kind in ("fwd", "dgrad", "wgrad"):
            n, h, w, cin, cout, kh, s = (int(v) for v in parts[1:8])
            pt, pb, pl, pr = ast.literal_eval(parts[8])
            ho = (h + pt + pb - kh) // s + 1
            wo = (w + pl + pr - kh) // s + 1
            return 2.0 * n * ho * wo * cout * kh * kh * cin
        if kind in ("pfwd", "pdgrad", "pwgrad"):
            n = int(parts[1])
            shapes = ast.literal_eval(parts[2])
            cin, cout = int(parts[3]), int(parts[4])
            return 2.0 * n * sum(a * b for a, b in shapes) * cout * 9 * cin
    except (ValueError, SyntaxError, IndexError):
        pass
    return 0.0


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
        tf = flops(k) / (best * 1e-3) / 1e12 if best > 0 else 0.0
        rows.append((ms, k, choice, best, n, ru, tf))
    rows.sort(reverse=True)
    print("conv total %.2f ms/step over %d keys" % (tot, len(rows)))
    for ms, k, c, b, n, ru, tf in rows:
        print("%7.3f ms  x%.1f  %-8s %.4f %5.0f TF/s (next: %s)  %s" % (ms, n, c, b, tf, ru, k))


if __name__ == "__main__":
    main()
