#!/usr/bin/env python3
"""Line-traffic model of the gain feed ("The gain feed's bytes"), on the CPU.

Builds the C2 rig's LUT with the oracle, lays out the gain feed's samples exactly as octvr_mapper_create does
(octvr_debug_gain_plan, host only) and counts, for the six 8-byte tap-row loads of every sample (Y rows y0,
y1; U and V rows of y0 / 2, y1 / 2): the 64-B / 128-B requests per wave-instruction, the distinct 128-B
lines per wave and per workgroup, the distinct lines and 64-B segments of the whole frame, per-XCD distinct
lines for round-robin and contiguous chunk dealing, and the same under re-sorted sample orders.

    python scripts/gain_feed_model.py
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "opencv-octvr_amd"))


def addrs(e, W0, H0):
    P = int(W0)
    x0 = (e[:, 0] & 0xFFFF).astype(np.int64)
    x0 = np.where(x0 >= 32768, x0 - 65536, x0)
    y0 = (e[:, 0] >> 16).astype(np.int64)
    y0 = np.where(y0 >= 32768, y0 - 65536, y0)
    cam = (e[:, 1] >> 10) & 31
    valid = (e[:, 1] >> 15) & 1
    x0c, y0c = np.clip(x0, 0, W0 - 1), np.clip(y0, 0, H0 - 1)
    y1c = np.clip(y0 + 1, 0, H0 - 1)
    xa = x0c & ~3
    ca = (x0c >> 1) & ~3
    uo = H0 * P
    vo = uo + W0 // 2
    fb = cam.astype(np.int64) << 32  # frames apart
    A = [fb + y0c * P + xa, fb + y1c * P + xa, fb + uo + (y0c >> 1) * P + ca, fb + uo + (y1c >> 1) * P + ca,
         fb + vo + (y0c >> 1) * P + ca, fb + vo + (y1c >> 1) * P + ca]
    return np.stack(A, 1), valid, x0, y0, cam


def model(e, W0, H0, name):
    A, _, _, _, _ = addrs(e, W0, H0)
    n = len(e)
    req64 = wave_lines = wg_lines = 0
    for w in range(n // 192):
        blk = A[w * 192:(w + 1) * 192]
        for u in range(3):
            for c in range(6):
                a = blk[u * 64:(u + 1) * 64, c]
                req64 += len(set((a >> 6).tolist()) | set(((a + 7) >> 6).tolist()))
        wave_lines += len(set((blk.reshape(-1) >> 7).tolist()))
    for g in range(n // 768):
        a = A[g * 768:(g + 1) * 768].reshape(-1)
        wg_lines += len(set((a >> 7).tolist()) | set(((a + 7) >> 7).tolist()))
    uniq = len(set((A.reshape(-1) >> 7).tolist()))
    return {"order": name, "req64_per_sample": round(req64 / n, 2), "wave_unique_B_per_sample": round(wave_lines * 128 / n, 1),
            "wg_unique_B_per_sample": round(wg_lines * 128 / n, 1), "frame_unique_128B_MB": round(uniq * 128 / 1e6, 1)}


def main():
    import octvr_amd as ox
    import oracle_py as O
    from octvr_amd import synthetic
    rig, W, H, sizes = synthetic.CONFIGS["C2"]()
    text = json.dumps(rig)
    want = O.lut_build(O.json_loads_rj(text), W, H, threads=8)
    mt = ox.MapperTemplate.from_arrays(W, H, [list(r[0]) for r in want], [r[1] for r in want], [r[2] for r in want],
                                       [r[3] for r in want])
    e, _ = ox.debug_gain_plan(mt, sizes)
    W0, H0 = sizes[0]
    out = {"samples": len(e), "orders": [model(e, W0, H0, "shipped (camera, source row, column)")]}
    A, valid, x0, y0, cam = addrs(e, W0, H0)
    for TX, TY in [(64, 8), (128, 16), (256, 32), (512, 16)]:
        order, i = [], 0
        while i < len(e):  # per camera run: valid samples re-sorted into source tiles, padding kept last
            j = i
            while j < len(e) and cam[j] == cam[i]:
                j += 1
            seg = np.arange(i, j)
            v, iv = seg[valid[seg] == 1], seg[valid[seg] == 0]
            v = v[np.lexsort((x0[v], y0[v], x0[v] // TX, y0[v] // TY))]
            order += v.tolist() + iv.tolist()
            i = j
        out["orders"].append(model(e[np.array(order)], W0, H0, "tiles %dx%d" % (TX, TY)))
    u64 = len(set((A.reshape(-1) >> 6).tolist()) | set(((A.reshape(-1) + 7) >> 6).tolist()))
    out["frame_unique_64B_MB"] = round(u64 * 64 / 1e6, 1)
    for nm, cols in (("Y", [0, 1]), ("U", [2, 3]), ("V", [4, 5])):
        a = A[:, cols].reshape(-1)
        out["frame_unique_64B_MB_" + nm] = round(len(set((a >> 6).tolist())) * 64 / 1e6, 1)
    nch = len(e) // 768
    Ach = A.reshape(nch, -1)

    def xcd_lines(assign):
        tot = 0
        for x in range(8):
            idx = [c for c in range(nch) if assign(c) == x]
            if idx:
                tot += len(set((Ach[idx].reshape(-1) >> 7).tolist()))
        return round(tot * 128 / 1e6, 1)

    starts, s0 = [], 0
    for x in range(8):
        starts.append(s0)
        s0 += (nch - x + 7) >> 3
    out["per_xcd_unique_MB_round_robin"] = xcd_lines(lambda c: c % 8)
    out["per_xcd_unique_MB_contiguous"] = xcd_lines(lambda c: sum(1 for st in starts[1:] if c >= st))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
