"""Debug helper: stitch a golden rig on the GPU and the oracle, report where they differ (test infra)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "opencv-octvr_amd"))
import torch  # noqa: E402

import octvr_amd as ox  # noqa: E402
import oracle_py as O  # noqa: E402

for name in sys.argv[1:] or ["rigA"]:
    rig, z = O.load_rig(name)
    W, H = (int(v) for v in z["out_size"])
    n = len(z["rois"])
    sizes = [(rig["inputs"][i]["options"]["width"], rig["inputs"][i]["options"]["height"]) for i in range(n)]
    frames = [O.rand_img(w, h * 3 // 2, 1, 1000 + i) for i, (w, h) in enumerate(sizes)]
    maps1 = [z[f"map1_{i}"] for i in range(n)]
    maps2 = [z[f"map2_{i}"] for i in range(n)]
    masks = [z[f"mask_{i}"] for i in range(n)]
    seams = [z[f"seam_{i}"] for i in range(n)]
    for gains in ([1.0] * n, [1.0 + 0.013 * k * (-1) ** k for k in range(n)]):
        mt = ox.MapperTemplate.from_arrays(W, H, z["rois"].tolist(), maps1, maps2, masks, seams)
        m = ox.Mapper(mt, sizes, blend=0, enable_gain=True)
        out = torch.zeros((H * 3 // 2, W), dtype=torch.uint8, device="cuda")
        m.stitch([torch.from_numpy(f).cuda() for f in frames], out, gains=gains)
        torch.cuda.synchronize()
        got = out.cpu().numpy()
        want, _ = O.stitch_frame(frames, sizes, z["rois"].tolist(), maps1, maps2, masks, W, H, enable_gain=True,
                                 gains=gains, threads=8)
        d = np.argwhere(got[:H] != want[:H])
        print(name, "gains", gains[:3], "Y mismatches", len(d), "of", W * H, "UV mismatches",
              int((got[H:] != want[H:]).sum()))
        for y, x in d[:12]:
            # owning camera and its fractional code at this pixel
            info = []
            for i in range(n):
                rx, ry, rw, rh = z["rois"][i]
                if rx <= x < rx + rw and ry <= y < ry + rh and masks[i][y - ry, x - rx]:
                    w_, h_ = sizes[i]
                    X = np.float32(maps1[i][y - ry, x - rx]) * np.float32(w_)
                    Y = np.float32(maps2[i][y - ry, x - rx]) * np.float32(h_)
                    ix, iy = int(np.rint(np.float32(X) * 32)), int(np.rint(np.float32(Y) * 32))
                    info.append((i, ix & 31, iy & 31))
            print("  ", x, y, int(got[y, x]), int(want[y, x]), info)
