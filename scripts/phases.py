#!/usr/bin/env python3
"""Per-wave phase breakdown of the stitch kernel's item loop (diagnostic build only).

  bash scripts/build_variant.sh phases -DOCTVR_PHASES=1
  OCTVR_HIP_LIB=$PWD/opencv-octvr_amd/lib/variants/phases.so python scripts/phases.py [--config C2]

Phases (shader cycles, s_memtime): 0 barrier before staging, 1 staging stores (+ extra chunks),
2 barrier after staging, 3 output stores + next-item loads/claim issue, 4 LDS taps + colour math,
5 back edge (waits for the next item's loads).
"""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "opencv-octvr_amd"))
NAMES = ["bar1", "stage", "bar2", "issue", "compute", "backedge"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C2")
    args = ap.parse_args()
    import torch
    import octvr_amd as ox
    from octvr_amd import synthetic
    rig, W, H, sizes = synthetic.CONFIGS[args.config]()
    mt = ox.MapperTemplate.from_json(json.dumps(rig), W, H, use_roi=True, device=0)
    m = ox.Mapper(mt, sizes, blend=0, enable_gain=True, device=0)
    frames = [torch.from_numpy(synthetic.yuv_frame(w, h, 1000 + i)).cuda() for i, (w, h) in enumerate(sizes)]
    out = torch.empty((H * 3 // 2, W), dtype=torch.uint8, device="cuda")
    lib = ox._lib
    lib.octvr_debug_stamps.argtypes = [C.c_void_p, C.c_int]
    rows = 2 * 8192
    for rep in range(3):
        m.set_timing(True)
        m.stitch(frames, out)
        torch.cuda.synchronize()
        ms, _ = m.kernel_time()
        m.set_timing(False)
        buf = np.zeros((rows, 4), np.uint64)
        assert lib.octvr_debug_stamps(buf.ctypes.data, rows) == rows
        w = buf.reshape(-1, 8)[:6144].astype(np.float64)
        w = w[w[:, 7] > 0]
        tot = w[:, :6].sum(1)
        print("rep %d: stitch %.1f us, %d waves, mean wave loop %.0f cycles (max %.0f)" % (
            rep, ms * 1e3, len(w), tot.mean(), tot.max()))
        for k, n in enumerate(NAMES):
            print("  %-9s mean %8.0f  (%.1f %%)" % (n, w[:, k].mean(), 100 * w[:, k].sum() / tot.sum()))


if __name__ == "__main__":
    main()
