#!/usr/bin/env python3
"""Pack the raw outputs of gen_golden.cpp into tests/golden/*.npz (TEST INFRASTRUCTURE ONLY).

The numbers come from the reference implementation (see gen_golden.cpp); this script only moves
them into compressed numpy archives (no pickles) plus a JSON manifest.
"""
import glob
import hashlib
import json
import os
import shutil
import sys

import numpy as np

CV_DT = {0: np.uint8, 1: np.int8, 2: np.uint16, 3: np.int16, 4: np.int32, 5: np.float32, 6: np.float64}


def load_mat(path):
    with open(path + ".meta") as f:
        typ, rows, cols = map(int, f.read().split())
    depth, cn = typ & 7, (typ >> 3) + 1
    a = np.fromfile(path, dtype=CV_DT[depth])
    shape = (rows, cols) if cn == 1 else (rows, cols, cn)
    return a.reshape(shape)


def main(raw, dst):
    os.makedirs(dst, exist_ok=True)
    manifest = {"source": "reference CPU build (SURVEY.md §8c) via oracle/golden_gen/gen_golden.cpp",
                "rigs": {}}
    for js in sorted(glob.glob(os.path.join(raw, "rig*.json"))):
        name = os.path.basename(js)[:-5]
        shutil.copy(js, os.path.join(dst, name + ".json"))
        hdr = np.fromfile(os.path.join(raw, name + "_rois.i64"), dtype=np.int64)
        out_w, out_h, n = (int(v) for v in hdr[:3])
        rois = hdr[3:].reshape(n, 4)
        arrs = {"rois": rois, "out_size": np.array([out_w, out_h], np.int64),
                "gains": np.fromfile(os.path.join(raw, name + "_gains.f64"), dtype=np.float64)}
        for i in range(n):
            for key in ("map1", "map2", "mask", "seam", "remap_c1", "remap_c3", "remap_c4"):
                p = os.path.join(raw, f"{name}_{i}_{key}")
                if os.path.exists(p):
                    arrs[f"{key}_{i}"] = load_mat(p)
        np.savez_compressed(os.path.join(dst, name + ".npz"), **arrs)
        with open(os.path.join(raw, name + ".dat"), "rb") as f:
            dat = f.read()
        manifest["rigs"][name] = {"n_inputs": n, "out_size": [out_w, out_h],
                                  "dat_sha256": hashlib.sha256(dat).hexdigest(), "dat_bytes": len(dat)}
    kats = {
        "remap_kat_src": load_mat(os.path.join(raw, "remap_kat_src")),
        "remap_kat_out": load_mat(os.path.join(raw, "remap_kat_out")),
        "rotation_kat": np.fromfile(os.path.join(raw, "rotation_kat.f64"), dtype=np.float64),
        "solve_kat": np.fromfile(os.path.join(raw, "solve_kat.f64"), dtype=np.float64),
        "dt_src": load_mat(os.path.join(raw, "dt_src")),
        "dt_out": load_mat(os.path.join(raw, "dt_out")),
        "rs_src": load_mat(os.path.join(raw, "rs_src")),
        "rs_up": load_mat(os.path.join(raw, "rs_up")),
        "rs_down": load_mat(os.path.join(raw, "rs_down")),
    }
    np.savez_compressed(os.path.join(dst, "kats.npz"), **kats)
    with open(os.path.join(dst, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
