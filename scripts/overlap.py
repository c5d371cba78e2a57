#!/usr/bin/env python3
"""Frames-in-flight anatomy from a rocprofv3 kernel trace (csv): over the last N frames, the wall time per
frame, the composite's own spans, how many composites run at once (time-weighted), and how long the
gain feed runs and how much of it overlaps a composite.

  python scripts/overlap.py gpurun_out/<dir> [frames=20] [tail=26]

tail: composites after the timed region to leave out (bench.py's one-in-flight measurement runs 2 + 8 + 16
serial stitches after it).
"""
import csv
import glob
import json
import sys


def load(d):
    f = glob.glob(d + "/**/*kernel_trace.csv", recursive=True)[0]
    rows = [r for r in csv.DictReader(open(f)) if "octvr" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    return rows


def coverage(iv, lo, hi):
    """time-weighted histogram of how many intervals are open, within [lo, hi)"""
    ev = []
    for a, b in iv:
        a, b = max(a, lo), min(b, hi)
        if b > a:
            ev += [(a, 1), (b, -1)]
    ev.sort()
    hist, cur, t = {}, 0, lo
    for x, d in ev:
        hist[cur] = hist.get(cur, 0) + (x - t)
        cur += d
        t = x
    hist[cur] = hist.get(cur, 0) + (hi - t)
    tot = sum(hist.values()) or 1
    return {k: round(v / tot, 3) for k, v in sorted(hist.items())}


def main():
    d = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    tail = int(sys.argv[3]) if len(sys.argv) > 3 else 26
    rows = load(d)
    comp = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows if "stitch_tiled" in r["Kernel_Name"]]
    feed = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows if "gain_feed" in r["Kernel_Name"]]
    comp = comp[:len(comp) - tail][-n:]
    lo, hi = comp[0][0], comp[-1][1]
    per_frame = (comp[-1][0] - comp[0][0]) / (len(comp) - 1) / 1e3
    feed = [f for f in feed if f[1] > lo and f[0] < hi]
    spans = sorted((b - a) / 1e3 for a, b in comp)
    fsp = sorted((b - a) / 1e3 for a, b in feed)

    def overlap(a, b, iv):
        return sum(max(0, min(b, y) - max(a, x)) for x, y in iv)
    f_ov = [overlap(a, b, comp) / max(b - a, 1) for a, b in feed]
    print(json.dumps({
        "dir": d, "frames": len(comp), "us_per_frame": round(per_frame, 1),
        "composite_span_us": {"min": round(spans[0], 1), "median": round(spans[len(spans) // 2], 1), "max": round(spans[-1], 1)},
        "composites_running": coverage(comp, lo, hi),
        "feed_span_us": {"median": round(fsp[len(fsp) // 2], 1), "max": round(fsp[-1], 1)} if fsp else None,
        "feed_share_beside_a_composite": round(sum(f_ov) / len(f_ov), 3) if f_ov else None,
        "feeds_running": coverage(feed, lo, hi) if feed else None}))


if __name__ == "__main__":
    main()
