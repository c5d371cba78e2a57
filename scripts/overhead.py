#!/usr/bin/env python3
"""Per-step time of back-to-back C2 stitches with and without the HIP-event kernel timing (the
bench's roofline timing) — what the timing itself costs on the GPU timeline."""
import json, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "opencv-octvr_amd"))
import torch
import octvr_amd as ox
from octvr_amd import synthetic
rig, W, H, sizes = synthetic.CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "C2"]()
mt = ox.MapperTemplate.from_json(json.dumps(rig), W, H, use_roi=True, device=0)
m = ox.Mapper(mt, sizes, blend=0, enable_gain=True, device=0)
frames = [torch.from_numpy(synthetic.yuv_frame(w, h, 1000 + i)).cuda() for i, (w, h) in enumerate(sizes)]
out = torch.empty((H * 3 // 2, W), dtype=torch.uint8, device="cuda")
s = torch.cuda.current_stream()
for timing in (False, True, False, True):
    m.set_timing(timing)
    for _ in range(5):
        m.stitch(frames, out, stream=s)
    torch.cuda.synchronize()
    m.kernel_time()
    t0 = time.perf_counter()
    for _ in range(100):
        m.stitch(frames, out, stream=s)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / 100
    k = m.kernel_time()
    print("timing=%d: %.2f us/step (%.1f k MP/s), stitch kernel %.2f us" % (timing, dt * 1e6, W * H / dt / 1e9,
                                                                          k[0] * 1e3 / max(k[1], 1)))
