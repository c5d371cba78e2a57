"""morph_controlpoints oracle (oracle/octvr_oracle_morph.c, template_morph.cpp:69-237) — CPU only.

Parity unpinned: no reference fixture covers morph_controlpoints, so the restatement of cv::Subdiv2D
is checked against the properties a Delaunay triangulation must have, and the morph against what its
definition fixes (which pixels may change, how many control points survive the filter)."""
import numpy as np
import pytest

import camera_rigs as R
import oracle_py as O


def _circumcircle_violations(tris, pts, tol=1e-9):
    bad = 0
    for t in tris.astype(np.float64):
        a, b, c = t[0:2], t[2:4], t[4:6]
        d = 2 * (a[0] * (b[1] - c[1]) + b[0] * (c[1] - a[1]) + c[0] * (a[1] - b[1]))
        ux = ((a @ a) * (b[1] - c[1]) + (b @ b) * (c[1] - a[1]) + (c @ c) * (a[1] - b[1])) / d
        uy = ((a @ a) * (c[0] - b[0]) + (b @ b) * (a[0] - c[0]) + (c @ c) * (b[0] - a[0])) / d
        r2 = (a[0] - ux) ** 2 + (a[1] - uy) ** 2
        dd = (pts[:, 0] - ux) ** 2 + (pts[:, 1] - uy) ** 2
        bad += int((dd < r2 * (1 - 1e-7) - tol).sum())
    return bad


def _hull_area(p):
    p = sorted(map(tuple, p))
    def half(seq):
        h = []
        for q in seq:
            while len(h) >= 2 and (h[-1][0] - h[-2][0]) * (q[1] - h[-2][1]) - (h[-1][1] - h[-2][1]) * (q[0] - h[-2][0]) <= 0:
                h.pop()
            h.append(q)
        return h
    hull = half(p)[:-1] + half(p[::-1])[:-1]
    x, y = np.array(hull).T
    return 0.5 * abs(np.dot(x, np.roll(y, 1)) - np.dot(y, np.roll(x, 1))), len(hull)


def _areas(tris):
    t = tris.astype(np.float64)
    return 0.5 * np.abs((t[:, 2] - t[:, 0]) * (t[:, 5] - t[:, 1]) - (t[:, 3] - t[:, 1]) * (t[:, 4] - t[:, 0]))


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_delaunay_random_points(seed):
    pts = np.random.default_rng(seed).uniform(0.05, 0.95, (80, 2)).astype(np.float32)
    tris = O.delaunay(pts)
    area, h = _hull_area(pts.astype(np.float64))
    # Delaunay of the points plus Subdiv2D's three far vertices, restricted to the real triangles: the
    # far vertices are finite (3, 0), (0, 3), (-3, -3), so a few hull slivers can go to them instead
    assert 2 * len(pts) - 2 - h - 4 <= len(tris) <= 2 * len(pts) - 2 - h
    assert area - 0.02 < _areas(tris).sum() <= area + 1e-6
    assert _circumcircle_violations(tris, pts.astype(np.float64)) == 0
    corners = {tuple(c) for c in tris.reshape(-1, 2)}
    assert corners == {tuple(p) for p in pts}


def test_delaunay_morph_frame_collinear():
    """The morph's frame (11 x 2 points on horizontal edges, 9 x 2 on vertical ones) puts many points
    on existing edges: Subdiv2D's PTLOC_ON_EDGE path (edge deletion, subdivision2d.cpp:420-425)."""
    L, R_, T, B = 0.1, 0.8, 0.2, 0.7
    pts = [(0.4, 0.45), (0.42, 0.5), (0.6, 0.38)]
    x = np.float32(L)
    while x < R_ + 1e-3:
        pts += [(x, T), (x, B)]
        x = np.float32(x + np.float32(R_ - L) / np.float32(10))
    for k in range(1, 10):
        y = T + (B - T) * k / 10
        pts += [(L, y), (R_, y)]
    pts = np.array(pts, np.float32)
    tris = O.delaunay(pts)
    assert abs(_areas(tris).sum() - (np.float32(R_) - np.float32(L)) * (np.float32(B) - np.float32(T))) < 2e-3
    assert _circumcircle_violations(tris, pts.astype(np.float64), tol=1e-7) == 0


def test_delaunay_duplicate_and_vertex_snapping():
    pts = np.array([(0.3, 0.3), (0.7, 0.3), (0.5, 0.8), (0.3, 0.3), (0.5, 0.4)], np.float32)
    tris = O.delaunay(pts)
    assert len(tris) == 3  # the duplicate is PTLOC_VERTEX: not inserted twice


def test_project_roundtrip():
    """_translate's projection (input image_to_obj, output obj_to_image) inverts the LUT."""
    rig = R.morph_rig(True)
    W, H = 512, 256
    luts = O.lut_build(rig, W, H)
    rng = np.random.default_rng(3)
    for i, ((x0, y0, w, h), m1, m2, mk) in enumerate(luts):
        ys, xs = np.nonzero(mk)
        for k in rng.choice(len(ys), 20, replace=False):
            u, v = O.project(rig["inputs"][i], rig["output"], float(m1[ys[k], xs[k]]), float(m2[ys[k], xs[k]]))
            assert abs(u - (xs[k] + x0) / W) < 1e-5 and abs(v - (ys[k] + y0) / H) < 1e-5


def _expected_kept(rig, cps):
    """The |dst0 - dst1|_1 > 0.1 filter in float (template_morph.cpp:123-124): jittered pairs stay,
    pairs split by the +-180 degree seam of the output go."""
    k = 0
    for n0, n1, x0, y0, x1, y1 in cps:
        f = np.float32
        d0 = [f(v) for v in O.project(rig["inputs"][n0], rig["output"], float(f(x0)), float(f(y0)))]
        d1 = [f(v) for v in O.project(rig["inputs"][n1], rig["output"], float(f(x1)), float(f(y1)))]
        k += float(f(abs(d0[0] - d1[0])) + f(abs(d0[1] - d1[1]))) <= 0.1
    return k


def test_morph_oracle_changes_only_triangles():
    rig = R.morph_rig(True)
    W, H = 512, 256
    luts = O.lut_build(rig, W, H)
    cps = R.morph_points(luts)
    rc, new, tris = O.morph_controlpoints(rig, luts, W, H, cps)
    assert rc == _expected_kept(rig, cps) > 0.8 * len(cps)
    moved = 0
    for i, ((x0, y0, w, h), m1, m2, mk) in enumerate(luts):
        st, dt = tris[i]
        assert len(st) > 0 and st.shape == dt.shape
        assert ((st >= 0) & (st <= 1)).all()
        cover = np.zeros((h, w), np.uint8)
        for t in dt:
            q = []
            for c in range(3):  # std::round: halves away from zero
                for v in (np.float32(t[2 * c]) * np.float32(W) - np.float32(x0),
                          np.float32(t[2 * c + 1]) * np.float32(H) - np.float32(y0)):
                    q.append(int(np.sign(v) * np.floor(abs(v) + np.float32(0.5))))
            O.fill_poly(cover, q, 1)
        _, n1, n2, nm = new[i]
        changed = (n1 != m1) | (n2 != m2) | (nm != mk)
        assert not (changed & (cover == 0)).any()
        moved += int(changed.sum())
    assert moved > 1000


def test_morph_oracle_far_points_dropped_and_errors():
    rig = R.morph_rig()
    W, H = 512, 256
    luts = O.lut_build(rig, W, H)
    cps = R.morph_points(luts, per_pair=3)
    far = [[0, 1, 0.2, 0.2, 0.8, 0.8]]  # projections far apart: skipped, not an error
    rc, _, _ = O.morph_controlpoints(rig, luts, W, H, cps + far)
    assert rc == _expected_kept(rig, cps + far) == _expected_kept(rig, cps)
    rc, _, _ = O.morph_controlpoints(rig, luts, W, H, [[1, 0] + cps[0][2:]])
    assert rc == -1  # CV_Assert(n0 < n1)
    fish = {"output": rig["output"], "inputs": [
        {"type": "fisheye", "options": {"width": 640, "height": 480, "fx": 300.0, "fy": 300.0, "cx": 320.0,
                                        "cy": 240.0, "dist_coeffs": [0, 0, 0, 0]}}] + rig["inputs"][1:]}
    rc, _, _ = O.morph_controlpoints(fish, O.lut_build(fish, W, H), W, H, [[0, 1, 0.5, 0.5, 0.5, 0.5]])
    assert rc == -2  # no image_to_obj_single (camera.hpp:101-103)
