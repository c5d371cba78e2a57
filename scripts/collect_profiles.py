#!/usr/bin/env python3
"""Copy one evidence session's results (scripts/evidence.sh, TAG=<tag>) from gpurun_out/ into profiles/:
bench lines, rocprofv3 kernel stats per config / frames in flight, the last frames of the C3 one-in-flight
kernel trace, and the PMC summaries (scripts/pmc_summary.py).
    python scripts/collect_profiles.py r04d
"""
import csv
import glob
import json
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
G = os.path.join(ROOT, "gpurun_out")
P = os.path.join(ROOT, "profiles")


def last_json_line(path):
    lines = [l for l in open(path).read().splitlines() if l.strip().startswith("{")]
    return lines[-1] if lines else None


def main():
    tag = sys.argv[1]
    for f in sorted(glob.glob(os.path.join(G, "%s_bench_*.json" % tag))):
        cfg = os.path.basename(f)[len(tag) + 7:-5]
        line = last_json_line(f)
        if line:
            json.loads(line)
            open(os.path.join(P, "%s_%s_bench.json" % (tag, cfg)), "w").write(line + "\n")
    for d in sorted(glob.glob(os.path.join(G, "kt_%s_*_if*" % tag))):
        if not os.path.isdir(d):
            continue
        cfg, inf = os.path.basename(d)[len(tag) + 4:].split("_if")  # inf: "<streams>b<frames per launch>"
        st = os.path.join(d, "run_kernel_stats.csv")
        # --stats averages are per-kernel durations only with one frame in flight: with several, launches
        # on different streams overlap and a launch's span exceeds the step time (the trace union,
        # scripts/union_check.py, is that run's evidence instead)
        if os.path.exists(st) and inf.startswith("1b"):
            shutil.copy(st, os.path.join(P, "%s_%s_inflight%s_kernel_stats.csv" % (tag, cfg, inf)))
        tr = os.path.join(d, "run_kernel_trace.csv")
        if cfg == "C3" and inf == "1b1" and os.path.exists(tr):
            rows = [r for r in csv.DictReader(open(tr)) if "octvr" in r["Kernel_Name"]]
            rows.sort(key=lambda r: int(r["Start_Timestamp"]))
            rows = rows[-90:]
            t0 = int(rows[0]["Start_Timestamp"])
            with open(os.path.join(P, "%s_C3_inflight1_last_frames_trace.csv" % tag), "w", newline="") as o:
                w = csv.writer(o)
                w.writerow(["kernel", "grid", "start_us", "dur_us"])
                for r in rows:
                    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
                    w.writerow([r["Kernel_Name"].split("(")[0], r["Grid_Size_X"], round((s - t0) / 1e3, 2),
                                round((e - s) / 1e3, 2)])
    tests_log = os.path.join(G, "%s_tests.log" % tag)
    if not os.path.exists(tests_log):  # a bench-only session (PART=B): its PMC summaries are an earlier tag's
        return
    t_session = os.path.getmtime(tests_log)
    for d in sorted(glob.glob(os.path.join(G, "pmc_*_if*_so.sha"))):
        if os.path.getmtime(d) < t_session - 60:  # an older session's passes
            continue
        cfg, inf = os.path.basename(d)[4:-7].split("_if")
        subprocess.check_call([sys.executable, os.path.join(ROOT, "scripts", "pmc_summary.py"), cfg, tag, inf])


if __name__ == "__main__":
    main()
