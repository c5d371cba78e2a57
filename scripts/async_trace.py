#!/usr/bin/env python3
"""AsyncMultiMapper end to end on one config (bench.async_e2e), for a rocprofv3 kernel + memory-copy
trace showing how H2D, stitch and D2H overlap across the 3 pipeline slots (async.cpp:32-172):
    rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/async -o run -- \
        python3 scripts/async_trace.py --config C2 --frames 12
then  python3 scripts/async_trace.py --analyze gpurun_out/async  (prints the overlap summary)."""
import argparse
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "opencv-octvr_amd"))


def run(cfg, frames):
    import bench
    import octvr_amd as ox
    from octvr_amd import synthetic
    rig, W, H, sizes = synthetic.CONFIGS[cfg]()
    blend = synthetic.BLEND[cfg]
    mt = ox.MapperTemplate.from_json(json.dumps(rig), W, H, use_roi=True, device=0)
    if blend > 0:
        mt.create_masks(0)
    frames_np = [synthetic.yuv_frame(w, h, bench.frame_seed(0, 0, i)) for i, (w, h) in enumerate(sizes)]
    print(json.dumps(bench.async_e2e(ox, mt, sizes, W, H, blend, frames_np, 0, frames=frames)))


def analyze(d):
    def rows(name):
        p = os.path.join(d, name)
        return list(csv.DictReader(open(p))) if os.path.exists(p) else []
    ker = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows("run_kernel_trace.csv")]
    cpy = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Direction", r.get("Operation", "")), int(r.get("Bytes", r.get("Size", 0)) or 0))
           for r in rows("run_memory_copy_trace.csv")]
    stitch = sorted((s, e) for s, e, n in ker if "stitch_tiled" in n or "mb_blend" in n)
    h2d = sorted((s, e, b) for s, e, k, b in cpy if "HOST_TO_DEVICE" in k.upper() and b >= 1 << 20)
    d2h = sorted((s, e, b) for s, e, k, b in cpy if "DEVICE_TO_HOST" in k.upper() and b >= 1 << 20)

    def union(iv):
        iv = sorted(iv)
        tot, cs, ce = 0, None, None
        for s, e in iv:
            if cs is None or s > ce:
                if cs is not None:
                    tot += ce - cs
                cs, ce = s, e
            else:
                ce = max(ce, e)
        return tot + (ce - cs if cs is not None else 0)

    def overlap(a, b):
        return union(a) + union(b) - union(a + b)
    h = [(s, e) for s, e, _ in h2d]
    o = [(s, e) for s, e, _ in d2h]
    t0 = min(x[0] for x in stitch + h + o)
    t1 = max(x[1] for x in stitch + h + o)
    out = {"window_us": (t1 - t0) / 1e3, "stitch_busy_us": union(stitch) / 1e3, "h2d_busy_us": union(h) / 1e3,
           "d2h_busy_us": union(o) / 1e3, "h2d_copies": len(h), "d2h_copies": len(o),
           "h2d_GBps": sum(b for _, _, b in h2d) / max(union(h), 1), "d2h_GBps": sum(b for _, _, b in d2h) / max(union(o), 1),
           "stitch_under_h2d_us": overlap(stitch, h) / 1e3, "stitch_under_d2h_us": overlap(stitch, o) / 1e3,
           "h2d_under_d2h_us": overlap(h, o) / 1e3}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C2")
    ap.add_argument("--frames", type=int, default=12)
    ap.add_argument("--analyze")
    a = ap.parse_args()
    if a.analyze:
        analyze(a.analyze)
    else:
        run(a.config, a.frames)
