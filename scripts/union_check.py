#!/usr/bin/env python3
"""Recompute a bench line's roofline from the rocprofv3 kernel trace of the same run (scripts/evidence.sh
kt_<tag>_<cfg>_if<k>: `rocprofv3 --kernel-trace --stats -- python3 bench.py ...`, whose log ends with the
bench line).  The timed region is bench.py's launches [skip, skip + count) of the anchor kernel (one per
frame: one setup stitch per frame set, then the warmup, then the timed steps); the union of the intervals
of every kernel matching `pattern` that starts inside that window, per frame, is the trace's counterpart
of the line's kernel_us (the union of the HIP-event intervals with frames in flight), and
bytes_per_launch / union is its achieved rate.  The line's own preroll steps (bench.py --preroll) are added to
`skip`, and `count` defaults to the line's timed steps.

    python scripts/union_check.py <kt dir> <pattern regex> <anchor regex> [skip [count]] > out.json
"""
import csv
import json
import os
import re
import sys


def main():
    d, pat, anchor = sys.argv[1], re.compile(sys.argv[2]), re.compile(sys.argv[3])
    line = [l for l in open(d + ".log").read().splitlines() if l.startswith("{")][-1]
    bl = json.loads(line)
    # the untimed preroll's steps (bench.py --preroll) come after the setup and warmup launches
    pre = bl.get("preroll", {}).get("steps", 0)
    skip = (int(sys.argv[4]) if len(sys.argv) > 4 else 13) + pre
    # frames per launch (octvr_mapper_stitch_batch): the anchor launches and the preroll's steps are calls,
    # each of nb frames
    nb = bl["config"].get("frames_per_launch", 1)
    count = int(sys.argv[5]) if len(sys.argv) > 5 else bl["steps"] // nb
    rows = list(csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv"))))
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    anchors = [a for a, b, n in iv if anchor.search(n)]
    t0 = anchors[skip]
    t1 = anchors[skip + count] if skip + count < len(anchors) else float("inf")
    sel = [(a, b) for a, b, n in iv if pat.search(n) and t0 <= a < t1]
    union, ca, cb = 0, None, None
    for a, b in sel:
        if cb is None or a > cb:
            if cb is not None:
                union += cb - ca
            ca, cb = a, b
        else:
            cb = max(cb, b)
    if cb is not None:
        union += cb - ca
    b = bl
    r = b["roofline"]
    u_us = union / (count * nb) / 1e3
    out = {"trace": os.path.basename(d), "pattern": sys.argv[2], "anchor": sys.argv[3], "frames": count * nb,
           "frames_per_launch": nb,
           "skip_first": skip, "preroll_steps": pre, "launches": len(sel), "union_us_per_frame": round(u_us, 2),
           "line_kernel_us": r["kernel_us"], "line_kernel_us_basis": r.get("kernel_us_basis"),
           "bytes_per_launch": r["bytes_per_launch"], "line_frac": r["frac"],
           "frac_from_trace": round(r["bytes_per_launch"] / (u_us * 1e-6) / 1e9 / r["peak"], 4),
           "trace_over_line": round(u_us / r["kernel_us"], 3), "ms_per_step": b["ms_per_step"],
           "frames_in_flight": b["config"].get("frames_in_flight"), "value": b["value"]}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
