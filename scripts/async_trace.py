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
    """Busy time (interval union) per copy direction and of the stitch kernels, and their pairwise
    overlaps.  Uploads appear as HOST_TO_DEVICE copies (SDMA); the downloads into pinned host memory
    run as `__amd_rocclr_copyBuffer` blit kernels on the download stream."""
    def rows(name):
        p = os.path.join(d, name)
        return list(csv.DictReader(open(p))) if os.path.exists(p) else []
    ker = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows("run_kernel_trace.csv")]
    cpy = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Direction"].replace("MEMORY_COPY_", ""))
           for r in rows("run_memory_copy_trace.csv")]

    def union(iv):
        tot, cs, ce = 0, None, None
        for s, e in sorted(iv):
            if cs is None or s > ce:
                if cs is not None:
                    tot += ce - cs
                cs, ce = s, e
            else:
                ce = max(ce, e)
        return tot + (ce - cs if cs is not None else 0)

    def overlap(a, b):
        return union(a) + union(b) - union(a + b)
    stitch = [(s, e) for s, e, n in ker if "stitch" in n or "mb_" in n]
    t_first = min(s for s, _ in stitch)  # the pipeline's window: from the first stitch on
    groups = {"stitch": stitch}
    for s, e, k in cpy:
        if e >= t_first:
            groups.setdefault(k, []).append((s, e))
    groups["DEVICE_TO_HOST (blit kernel)"] = [(s, e) for s, e, n in ker if "copyBuffer" in n and e >= t_first]
    t0 = min(s for v in groups.values() for s, _ in v)
    t1 = max(e for v in groups.values() for _, e in v)
    out = {"window_us": round((t1 - t0) / 1e3, 1),
           "busy_us": {k: round(union(v) / 1e3, 1) for k, v in groups.items()},
           "count": {k: len(v) for k, v in groups.items()},
           "overlap_us": {}}
    keys = sorted(groups)
    for i in range(len(keys)):
        for j in range(i + 1, len(keys)):
            out["overlap_us"][keys[i] + "|" + keys[j]] = round(overlap(groups[keys[i]], groups[keys[j]]) / 1e3, 1)
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
