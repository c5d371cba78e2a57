import json, os, sys
import numpy as np
import torch
sys.path.insert(0, "opencv-octvr_amd"); sys.path.insert(0, "tests")
import octvr_amd as ox
import oracle_py as O
from octvr_amd import synthetic
rig, z = O.load_rig("rigA")
W, H = (int(v) for v in z["out_size"])
n = len(z["rois"])
sizes = [(rig["inputs"][i]["options"]["width"], rig["inputs"][i]["options"]["height"]) for i in range(n)]
mt = ox.MapperTemplate.from_arrays(W, H, z["rois"].tolist(), [z[f"map1_{i}"] for i in range(n)],
                                   [z[f"map2_{i}"] for i in range(n)], [z[f"mask_{i}"] for i in range(n)],
                                   [z[f"seam_{i}"] for i in range(n)])
frames = [synthetic.smooth_yuv_frame(w, h, 900 + i) for i, (w, h) in enumerate(sizes)]
dev = [torch.from_numpy(f).cuda() for f in frames]
for blend in (-5, 16):
    m = ox.Mapper(mt, sizes, blend=blend, enable_gain=False)
    out = torch.zeros((H * 3 // 2, W), dtype=torch.uint8, device="cuda")
    m.stitch(dev, out)
    torch.cuda.synchronize()
    np.save("gpurun_out/dbg_%s_%d.npy" % (os.environ.get("TAG", "x"), blend), out.cpu().numpy())
print("ok", W, H, [r for r in z["rois"].tolist()])
