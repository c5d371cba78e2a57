#!/usr/bin/env python3
"""AsyncMultiMapper end to end on the C2 rig (bench.async_e2e) with the library OCTVR_HIP_LIB selects:
  OCTVR_HIP_LIB=... python scripts/async_ab.py [frames]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "opencv-octvr_amd"))
import bench  # noqa: E402
import octvr_amd as ox  # noqa: E402
from octvr_amd import synthetic  # noqa: E402

rig, W, H, sizes = synthetic.CONFIGS["C2"]()
mt = ox.MapperTemplate.from_json(json.dumps(rig), W, H, use_roi=True, device=0)
frames = [synthetic.yuv_frame(w, h, bench.frame_seed(0, 0, i)) for i, (w, h) in enumerate(sizes)]
n = int(sys.argv[1]) if len(sys.argv) > 1 else 24
for rep in range(2):
    r = bench.async_e2e(ox, mt, sizes, W, H, 0, frames, 0, frames=n)
    print(os.path.basename(os.environ.get("OCTVR_HIP_LIB", "cur")), rep, r["value"], r["ms_per_frame"], flush=True)
