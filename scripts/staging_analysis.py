"""How much of the composite's staging is redundant, and which scheme would remove it (CPU only, from the
oracle LUT): per 128x16 item and camera the staged box, the distinct taps, the 8-aligned row spans of the
taps, the union over vertical item strips, and the distinct taps per frame.
  python scripts/staging_analysis.py [C2|C4]   (C2: about 2 minutes)"""
import sys, time
sys.path.insert(0, '/root/repo/opencv-octvr_amd'); sys.path.insert(0, '/root/repo/tests')
import numpy as np
import oracle_py as O
from octvr_amd import synthetic
cfg = sys.argv[1] if len(sys.argv) > 1 else "C2"
rig, W, H, sizes = synthetic.CONFIGS[cfg]()
t = time.time()
luts = O.lut_build(rig, W, H, use_roi=True, threads=8)
print("lut", time.time() - t, flush=True)
cam = np.full((H, W), -1, np.int8)
sx = np.zeros((H, W), np.int32); sy = np.zeros((H, W), np.int32)
for i, ((x, y, w, h), m1, m2, mk) in enumerate(luts):
    iw, ih = sizes[i]
    ix = np.rint(m1.astype(np.float32) * np.float32(iw) * np.float32(32)).astype(np.int64)
    iy = np.rint(m2.astype(np.float32) * np.float32(ih) * np.float32(32)).astype(np.int64)
    sel = mk > 0
    sub_c = cam[y:y+h, x:x+w]; sub_x = sx[y:y+h, x:x+w]; sub_y = sy[y:y+h, x:x+w]
    sub_c[sel] = i; sub_x[sel] = (ix >> 5)[sel]; sub_y[sel] = (iy >> 5)[sel]
del luts
print("composite built", flush=True)
IW, IH = 128, 16
ny, nx = H // IH, W // IW
# per item per camera: box (8-aligned cols, even rows, +1 halo), exact tap set, row spans
staged = 0; exact = 0; spans8 = 0
distinct = [np.zeros((ih + 2, iw + 8), np.bool_) for iw, ih in sizes]
tapmap_rows = {}  # (cam, row) -> for ring analysis per column strip
colstrip_rows = 0  # vertical-walk: union of rows per (item column, camera), counting row spans
per_strip = {}
for ty in range(ny):
    for tx in range(nx):
        c = cam[ty*IH:(ty+1)*IH, tx*IW:(tx+1)*IW].ravel()
        xs = sx[ty*IH:(ty+1)*IH, tx*IW:(tx+1)*IW].ravel(); ys = sy[ty*IH:(ty+1)*IH, tx*IW:(tx+1)*IW].ravel()
        for k in np.unique(c[c >= 0]):
            s = c == k
            x0 = xs[s]; y0 = ys[s]
            bx0 = x0.min() & ~7; by0 = y0.min() & ~1
            bx1 = (x0.max() + 2 + 7) & ~7; by1 = (y0.max() + 2 + 1) & ~1
            staged += (bx1 - bx0) * (by1 - by0)
            # exact taps
            tx_ = np.concatenate([x0, x0 + 1, x0, x0 + 1]); ty_ = np.concatenate([y0, y0, y0 + 1, y0 + 1])
            key = np.unique(ty_.astype(np.int64) * 65536 + tx_)
            exact += key.size
            rr = key // 65536; cc = key % 65536
            # per row 8-aligned span
            for r in np.unique(rr):
                cs = cc[rr == r]
                spans8 += ((cs.max() + 8) & ~7) - (cs.min() & ~7)
            distinct[k][np.clip(ty_, 0, sizes[k][1]+1), np.clip(tx_, 0, sizes[k][0]+7)] = True
            # vertical strips: union of exact taps over the strip (items of one column, one camera)
            d = per_strip.setdefault((tx, k), set())
            d.update(key.tolist())
    if ty % 40 == 0: print(ty, flush=True)
strip = sum(len(v) for v in per_strip.values())
dist = sum(int(d.sum()) for d in distinct)
print(dict(items=ny*nx, staged_boxes=staged, exact_taps_per_item=exact, row_spans8_per_item=spans8,
           column_strip_union=strip, distinct=dist))
