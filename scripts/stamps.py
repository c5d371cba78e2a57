#!/usr/bin/env python3
"""Per-workgroup timing of the stitch and gain-feed kernels (diagnostic builds only).

  bash scripts/build_variant.sh stamps -DOCTVR_STAMPS=1
  OCTVR_HIP_LIB=$PWD/opencv-octvr_amd/lib/variants/stamps.so python scripts/stamps.py [--config C2]

Prints, per XCD band (blockIdx % 8), the spread of workgroup end times relative to the first start,
items / staging chunks per workgroup, and the gain feed's arrival span + last-workgroup solve time.
"""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "opencv-octvr_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C2")
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    import torch
    import octvr_amd as ox
    from octvr_amd import synthetic
    rig, W, H, sizes = synthetic.CONFIGS[args.config]()
    mt = ox.MapperTemplate.from_json(json.dumps(rig), W, H, use_roi=True, device=0)
    m = ox.Mapper(mt, sizes, blend=0, enable_gain=True, device=0)
    print(json.dumps(m.info()))
    frames = [torch.from_numpy(synthetic.yuv_frame(w, h, 1000 + i)).cuda() for i, (w, h) in enumerate(sizes)]
    out = torch.empty((H * 3 // 2, W), dtype=torch.uint8, device="cuda")
    lib = ox._lib
    lib.octvr_debug_stamps.argtypes = [C.c_void_p, C.c_int]
    rows = 2 * 8192
    buf = np.zeros((rows, 4), np.uint64)
    for rep in range(args.reps):
        for _ in range(3):  # back to back, as in bench.py: the stamps are the last launch's
            m.stitch(frames, out)
        torch.cuda.synchronize()
        assert lib.octvr_debug_stamps(buf.ctypes.data, rows) == rows
        st = buf[:8192].astype(np.int64)
        gf = buf[8192:].astype(np.int64)
        live = st[:, 1] > 0
        st = st[live]
        nb = len(st)
        t0 = st[:, 0].min()
        print("rep %d: stitch %d workgroups, span %.2f us (start spread %.2f us)" % (
            rep, nb, (st[:, 1].max() - t0) / 100.0, (st[:, 0].max() - t0) / 100.0))
        idx = np.nonzero(live)[0]
        for g in range(8):
            sel = (idx % 8) == g
            e = (st[sel, 1] - t0) / 100.0
            print("  band %d: end min %.1f med %.1f max %.1f us; items %d chunks %d (per wg max %d / %d)" % (
                g, e.min(), np.median(e), e.max(), st[sel, 2].sum(), st[sel, 3].sum(), st[sel, 2].max(), st[sel, 3].max()))
        f = buf.reshape(-1)[4 * 8192:4 * 8192 + 2048 * 8].reshape(-1, 8).astype(np.int64)
        f = f[f[:, 4] > 0]
        if len(f):
            ft0 = f[:, 0].min()
            rel = (f - ft0) / 100.0
            print("  gain feed: %d wgs; start spread %.2f; per-wg (median) gathered %.2f, reduced %.2f, adds done %.2f, "
                  "ticket %.2f us after its start; last ticket at %.2f" % (
                      len(f), rel[:, 0].max(), np.median(rel[:, 1] - rel[:, 0]), np.median(rel[:, 2] - rel[:, 0]),
                      np.median(rel[:, 3] - rel[:, 0]), np.median(rel[:, 4] - rel[:, 0]), rel[:, 4].max()))
            last = f[f[:, 5] == 1]
            if len(last):
                L = (last[0] - ft0) / 100.0
                X = (buf.reshape(-1)[4 * 8192 + 2048 * 8:4 * 8192 + 2048 * 8 + 2].astype(np.int64) - ft0) / 100.0
                print("  last workgroup: totals read %.2f, A/b built %.2f, solved %.2f, written %.2f; stitch starts %.2f us "
                      "after feed start; start times by 8-quantile %s" % (
                          L[6], X[0], X[1], L[7], (t0 - ft0) / 100.0,
                          np.round(np.quantile(rel[:, 0], np.linspace(0, 1, 9)), 2).tolist()))
        buf[:] = 0
        # clear the device copy too: the next rep overwrites every live row anyway


if __name__ == "__main__":
    main()
