#!/usr/bin/env python3
"""Per-launch duration of a kernel from a rocprofv3 kernel trace, two ways: the mean start-to-end span
(what --stats reports) and the union of all launches' intervals divided by the launch count (the
basis of bench.py's roofline with frames in flight, where launches on several streams overlap).

  python scripts/trace_union.py gpurun_out/prof/run_kernel_trace.csv stitch_tiled [skip_first [count]]

skip_first / count select the launches of a bench.py run's timed region (bench.py: one setup stitch per
frame set, the warmup steps, the timed steps, then the one-in-flight supplement).
"""
import csv
import json
import sys


def main():
    path, pat = sys.argv[1], sys.argv[2]
    skip = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    count = int(sys.argv[4]) if len(sys.argv) > 4 else None
    rows = [r for r in csv.DictReader(open(path)) if pat in r["Kernel_Name"]]
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows)[skip:]
    if count is not None:
        iv = iv[:count]
    span = sum(b - a for a, b in iv)
    union, ca, cb = 0, None, None
    for a, b in iv:
        if cb is None or a > cb:
            if cb is not None:
                union += cb - ca
            ca, cb = a, b
        else:
            cb = max(cb, b)
    if cb is not None:
        union += cb - ca
    n = max(len(iv), 1)
    print(json.dumps({"kernel": pat, "skip_first": skip, "launches": len(iv), "span_us_per_launch": round(span / n / 1e3, 2),
                      "union_us_per_launch": round(union / n / 1e3, 2),
                      "window_us": round((iv[-1][1] - iv[0][0]) / 1e3, 1) if iv else 0}))


if __name__ == "__main__":
    main()
