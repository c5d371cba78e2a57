#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (scripts/pmc.sh) into profiles/<tag>_pmc_<cfg>.json.

Correction per /opt/skills/guides/MI355X_MICROARCH.md "HBM": on gfx950 FETCH_SIZE reports half the
bytes of wide (16 B/lane) coalesced reads -> doubled; WRITE_SIZE is exact.  Counter unit: KiB.
The summary carries the sha256 of the profiled liboctvr_hip.so (pmc.sh writes it on the GPU box):
bench.py uses a summary only for that exact binary.
    python scripts/pmc_summary.py C2 r03v1
"""
import csv
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    cfg, tag = sys.argv[1], sys.argv[2]
    g = os.path.join(ROOT, "gpurun_out")
    sha = open(os.path.join(g, "pmc_%s_so.sha" % cfg)).read().strip()
    frames = int(open(os.path.join(g, "pmc_%s_frames" % cfg)).read().strip())
    out = {"config": cfg, "so_sha256": sha, "frames": frames, "unit": "bytes",
           "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes (bench.py --pmc-child, "
                     "%d frames); traffic = 2 x FETCH_SIZE (gfx950 half-count of 16 B/lane reads) + WRITE_SIZE, "
                     "KiB -> bytes" % frames}
    totals = {}
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        rows = list(csv.DictReader(open(os.path.join(g, "pmc_%s_%s" % (cfg, c), "run_counter_collection.csv"))))
        by_kernel = {}
        for r in rows:
            by_kernel.setdefault(r["Kernel_Name"], []).append(float(r["Counter_Value"]))
        out[c] = {k: {"launches": len(v), "kib_median": statistics.median(v), "kib_total": sum(v)}
                  for k, v in by_kernel.items()}
        totals[c] = sum(sum(v) for v in by_kernel.values())
    traffic = {}
    for k in out["FETCH_SIZE"]:
        f = out["FETCH_SIZE"][k]["kib_median"]
        w = out["WRITE_SIZE"].get(k, {"kib_median": 0.0})["kib_median"]
        traffic[k] = (2.0 * f + w) * 1024.0
    out["traffic_bytes"] = traffic  # per launch, per kernel
    out["traffic_per_frame_bytes"] = (2.0 * totals["FETCH_SIZE"] + totals["WRITE_SIZE"]) * 1024.0 / frames
    dst = os.path.join(ROOT, "profiles", "%s_pmc_%s.json" % (tag, cfg))
    json.dump(out, open(dst, "w"), indent=1)
    print(dst, json.dumps({"per_launch": traffic, "per_frame": out["traffic_per_frame_bytes"]}))


if __name__ == "__main__":
    main()
