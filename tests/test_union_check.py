"""scripts/union_check.py on a synthetic kernel trace (CPU): the timed window starts after the setup
launches and the line's own preroll steps (bench.py --preroll), and its union of intervals per frame is
set against the line's kernel_us."""
import csv
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_union_check_skips_setup_and_preroll(tmp_path):
    d = tmp_path / "kt_x_C2_if3"
    d.mkdir()
    setup, pre, steps = 13, 7, 5
    rows, t = [], 0
    for k in range(setup + pre + steps + 2):
        # setup and preroll frames take 100 ns of composite, timed ones 40 ns (+ an overlapping 20 ns launch of
        # another kernel the pattern counts, the anchor does not)
        dur = 40 if setup + pre <= k < setup + pre + steps else 100
        rows.append({"Kernel_Name": "stitch_tiled_kernel", "Start_Timestamp": t, "End_Timestamp": t + dur})
        rows.append({"Kernel_Name": "gain_feed_kernel", "Start_Timestamp": t + 1000, "End_Timestamp": t + 1500})
        if dur == 40:
            rows.append({"Kernel_Name": "stitch_wide_kernel", "Start_Timestamp": t + 30, "End_Timestamp": t + 50})
        t += 10000
    with open(d / "run_kernel_trace.csv", "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Kernel_Name", "Start_Timestamp", "End_Timestamp"])
        w.writeheader()
        w.writerows(rows)
    line = {"value": 1.0, "ms_per_step": 0.01, "steps": steps, "preroll": {"s": 0.5, "steps": pre},
            "config": {"frames_in_flight": 3},
            "roofline": {"kernel_us": 0.05, "kernel_us_basis": "x", "bytes_per_launch": 1e6, "frac": 0.1,
                         "peak": 8000.0}}
    (tmp_path / "kt_x_C2_if3.log").write_text("noise\n" + json.dumps(line) + "\n")
    out = subprocess.check_output([sys.executable, os.path.join(ROOT, "scripts", "union_check.py"), str(d),
                                   "stitch_", "stitch_tiled"], text=True)
    r = json.loads(out)
    assert r["skip_first"] == setup + pre and r["preroll_steps"] == pre and r["frames"] == steps
    assert r["launches"] == 2 * steps
    assert abs(r["union_us_per_frame"] - 0.05) < 1e-9  # [0, 40) U [30, 50) = 50 ns per frame
    assert abs(r["trace_over_line"] - 1.0) < 1e-9
