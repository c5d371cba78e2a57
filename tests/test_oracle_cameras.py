"""CPU checks of the oracle's camera models (no reference fixture exists for them: parity unpinned).
Round trip: a rig whose output and input are the same camera (same parameters, no rotation) maps
every covered output pixel onto itself; pinhole without distortion matches the pinhole formula."""
import math

import numpy as np
import pytest

import camera_rigs as R
import oracle_py as O


@pytest.mark.parametrize("t", ["normal", "perspective", "stupidoval", "eqareanorthpole", "eqareasouthpole", "cubic",
                               "fullframe_fisheye"])
def test_oracle_camera_round_trip(t):
    o = R.OUTPUT_MODELS[t]
    rig = {"output": {"type": t, "options": o}, "inputs": [{"type": t, "options": o}]}
    W, H = 96, 64
    _, m1, m2, mk = O.lut_build(rig, W, H, use_roi=False)[0]
    xs = (np.arange(W) / W)[None, :]
    ys = (np.arange(H) / H)[:, None]
    v = mk > 0
    assert v.mean() > 0.5
    ok = (np.abs(m1 - xs) < 1e-6) & (np.abs(m2 - ys) < 1e-6)
    # cube edges belong to two faces: obj_to_image may pick the other one (cubic.hpp:53-81)
    assert ok[v].mean() >= (0.97 if t == "cubic" else 1.0), (t, ok[v].mean())


def test_oracle_pinhole_without_distortion_is_the_pinhole_formula():
    rig = R.input_rigs()["pinhole_nodist"]
    W, H = 128, 64
    _, m1, m2, mk = O.lut_build(rig, W, H, use_roi=False)[0]
    o = rig["inputs"][0]["options"]
    out = O.camera_from_json(rig["output"])
    cam = O.camera_from_json(rig["inputs"][0])
    Rin = np.array(cam.R[:]).reshape(3, 3)
    Rout_inv = np.array(out.Rinv[:]).reshape(3, 3)
    u, v = np.meshgrid(np.arange(W) / W, np.arange(H) / H)
    lon, lat = (u - 0.5) * 2 * math.pi, -(v - 0.5) * math.pi
    p = np.stack([np.cos(lon) * np.cos(lat), np.sin(lat), -np.sin(lon) * np.cos(lat)], -1)
    q = p @ Rout_inv.T @ Rin.T
    with np.errstate(divide="ignore", invalid="ignore"):
        x = (o["fx"] * q[..., 0] / q[..., 2] + o["cx"]) / o["width"]
        y = 1.0 - (o["fy"] * q[..., 1] / q[..., 2] + o["cy"]) / o["height"]
    want = (q[..., 2] > 0) & (x >= 0) & (x < 1) & (y >= 0) & (y < 1)
    inner = want & (x > 1e-4) & (x < 1 - 1e-4) & (y > 1e-4) & (y < 1 - 1e-4)
    assert (mk[inner] > 0).all() and ((mk > 0) <= want | ~inner).all()
    assert np.abs(m1[inner] - x[inner]).max() < 1e-5 and np.abs(m2[inner] - y[inner]).max() < 1e-5


def test_oracle_selection_excludes_outside_rectangle():
    rig = R.input_rigs()["fullframe_selection"]
    W, H = 256, 128
    base = {"output": rig["output"], "inputs": [dict(c, options={k: v for k, v in c["options"].items() if k != "selection"})
                                                 for c in rig["inputs"]]}
    with_sel = O.lut_build(rig, W, H, use_roi=False)
    without = O.lut_build(base, W, H, use_roi=False)
    for c, a, b in zip(rig["inputs"], with_sel, without):
        l, r, t, btm = c["options"]["selection"]
        _, m1, m2, mk = b
        px, py = (m1 * c["options"]["width"]).astype(int), (m2 * c["options"]["height"]).astype(int)
        inside = (mk > 0) & (px >= l) & (px <= r - 1) & (py >= t) & (py <= btm - 1)
        assert np.array_equal(a[3] > 0, inside)


def test_oracle_fullframe_output_without_distortion_round_trip():
    """radial [0,0,0]: solvePoly trims the quartic to degree 1 (mathfuncs.cpp:2091-2095)."""
    o = dict(R.OUTPUT_MODELS["fullframe_fisheye"], radial=[0.0, 0.0, 0.0], center_dx=0.0, center_dy=0.0)
    rig = {"output": {"type": "fullframe_fisheye", "options": o}, "inputs": [{"type": "fullframe_fisheye", "options": o}]}
    W, H = 96, 64
    _, m1, m2, mk = O.lut_build(rig, W, H, use_roi=False)[0]
    xs = (np.arange(W) / W)[None, :]
    ys = (np.arange(H) / H)[:, None]
    v = mk > 0
    assert v.mean() > 0.9
    # the centre row is mirrored by the reference itself: y == 0 gives alpha = atan2(-0., x) = -pi or -0,
    # |sin(alpha)| < 1e-3 selects theta = -x / distance / cos(alpha), whose sign is flipped against the
    # forward model (fullframe_fisheye_cam.cpp:242-248)
    quirk = np.zeros_like(v)
    quirk[H // 2, 1:] = True
    quirk[H // 2, W // 2] = False
    ok = (np.abs(m1 - xs) < 1e-6) & (np.abs(m2 - ys) < 1e-6)
    assert ok[v & ~quirk].all()
    assert np.allclose(m1[quirk], 1.0 - xs[0][quirk[H // 2]], atol=1e-6)
