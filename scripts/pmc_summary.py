#!/usr/bin/env python3
"""Summarise the rocprofv3 --pmc passes of scripts/pmc.sh into profiles/<tag>_pmc_<cfg>.json (the streams and
frames per launch of the run inside: rocprofv3 --pmc serialises the dispatches, so one summary per config).

Per kernel and grid size (the multi-band sequence launches mb_down / mb_blend once per level, with a
different grid each) and per counter: launches, median and total.  HBM traffic per the MI355X guide's
"HBM" section: on gfx950 FETCH_SIZE reports half the bytes of wide (16 B/lane) coalesced reads, so it is
doubled; WRITE_SIZE is exact; unit KiB.  (The doubling is calibrated for 16 B/lane streaming reads; the
composite's staging loads are 8- and 4-byte gathers, so `traffic` is approximate for it.)
The summary carries the sha256 of the profiled liboctvr_hip.so: bench.py uses a summary only for that
exact binary.
    python scripts/pmc_summary.py C2 r04a [INFLIGHT]
"""
import csv
import glob
import json
import os
import re
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name):
    m = re.search(r"octvr(\d+)(\w+?_kernel)", name)
    base = m.group(2) if m else name.split("(")[0][:60]
    t = re.search(r"_kernelIL(b\d)ELi(\d)ELb(\d)E", name)  # stitch_tiled_kernel<DW, MODE, VIG(, QPL)>
    if t:
        base += "<mode%s>" % t.group(2)
    return base


def main():
    cfg, tag = sys.argv[1], sys.argv[2]
    inflight = sys.argv[3] if len(sys.argv) > 3 else "3"
    g = os.path.join(ROOT, "gpurun_out")
    d = "pmc_%s_if%s" % (cfg, inflight)
    sha = open(os.path.join(g, d + "_so.sha")).read().strip()
    frames = int(open(os.path.join(g, d + "_frames")).read().strip())
    bpath = os.path.join(g, d + "_batch")
    batch = int(open(bpath).read().strip()) if os.path.exists(bpath) else 1
    out = {"config": cfg, "frames_in_flight": int(inflight), "frames_per_launch": batch, "so_sha256": sha, "frames": frames,
           "method": "rocprofv3 --pmc, one pass per counter set (scripts/pmc.sh), bench.py --pmc-child --steps %d "
                     "--inflight %s; traffic = 2 x FETCH_SIZE (gfx950 half count of 16 B/lane reads) + WRITE_SIZE, "
                     "KiB -> bytes; keys: kernel@grid size" % (frames, inflight)}
    counters = {}
    for f in sorted(glob.glob(os.path.join(g, d + "_*", "run_counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            key = "%s@%s" % (short(r["Kernel_Name"]), r.get("Grid_Size", r.get("Grid_Size_X", "?")))
            counters.setdefault(key, {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    out["counters"] = {k: {c: {"launches": len(v), "median": statistics.median(v), "total": sum(v)} for c, v in cs.items()}
                       for k, cs in sorted(counters.items())}
    traffic, per_frame = {}, 0.0
    for k, cs in counters.items():
        if "FETCH_SIZE" in cs:
            f = statistics.median(cs["FETCH_SIZE"])
            w = statistics.median(cs.get("WRITE_SIZE", [0.0]))
            traffic[k] = (2.0 * f + w) * 1024.0
            if not k.startswith("gain_feed"):  # the stitch / blend sequence (the gain feed is reported apart)
                per_frame += (2.0 * sum(cs["FETCH_SIZE"]) + sum(cs.get("WRITE_SIZE", [0.0]))) * 1024.0
    if traffic:
        out["traffic_bytes"] = traffic  # per launch, per kernel@grid
        out["traffic_per_frame_bytes"] = per_frame / (frames * batch)
    sq = {}
    for k, cs in counters.items():
        if "SQ_INSTS_VALU" in cs or "SQ_WAVES" in cs:
            m = {c: statistics.median(v) for c, v in cs.items()}
            s = {c: m[c] for c in ("SQ_INSTS_VALU", "SQ_WAVES", "SQ_LDS_BANK_CONFLICT", "SQ_INSTS_LDS", "SQ_WAVE_CYCLES",
                                    "SQ_BUSY_CYCLES", "GRBM_GUI_ACTIVE") if c in m}
            if "SQ_WAVE_CYCLES" in m and m["SQ_WAVE_CYCLES"]:
                for c in ("SQ_WAIT_INST_ANY", "SQ_WAIT_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS"):
                    if c in m:
                        s[c + "_frac_of_wave_cycles"] = round(m[c] / m["SQ_WAVE_CYCLES"], 4)
            if "TCC_HIT_sum" in m and (m["TCC_HIT_sum"] + m.get("TCC_MISS_sum", 0)):
                s["tcc_hit_rate"] = round(m["TCC_HIT_sum"] / (m["TCC_HIT_sum"] + m.get("TCC_MISS_sum", 0)), 4)
            sq[k] = s
    if sq:
        out["sq_summary"] = sq
    suffix = ""
    dst = os.path.join(ROOT, "profiles", "%s_pmc_%s%s.json" % (tag, cfg, suffix))
    json.dump(out, open(dst, "w"), indent=1)
    print(dst, json.dumps({"traffic": traffic, "per_frame": out.get("traffic_per_frame_bytes")}))


if __name__ == "__main__":
    main()
