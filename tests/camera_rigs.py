"""Synthetic rigs exercising every camera model of modules/octvr/src/cameras/ (SURVEY.md §8f row 3).
No reference fixtures exist for these models (parity unpinned): the oracle restatement is checked by
round-trip / analytic properties (test_oracle_cameras.py) and the GPU LUT against the oracle."""
import math

OCAM = {"pol": [-180.0, 0.0, 0.0018, -1.2e-6, 3e-9], "invpol": [260.0, 150.0, -12.0, 20.0, 9.0, -3.0, 1.0],
        "xc": 240.5, "yc": 320.25, "c": 1.0003, "d": 0.0002, "e": -0.0001, "width": 640, "height": 480}

# models usable as the output camera (they implement image_to_obj_single)
OUTPUT_MODELS = {
    "normal": {"aspect_ratio": 1.5, "cam_opt": 0.8},
    "perspective": {"aspect_ratio": 1.25, "sf": 1.3},
    "stupidoval": {},
    "cubic": {},
    "eqareanorthpole": {},
    "eqareasouthpole": {"antarctic_circle": -0.9},
    "ocam_fisheye": OCAM,
    # no crop: the output fisheye's crop must be the whole image (fullframe_fisheye_cam.cpp:224)
    "fullframe_fisheye": {"width": 480, "height": 320, "hfov": 3.0, "center_dx": 2.0, "center_dy": -1.5,
                          "radial": [0.02, -0.05, 0.01]},
}


def _rot(yaw, pitch=0.0, roll=0.0):
    return {"rotation": {"roll": roll, "yaw": yaw, "pitch": pitch}}


def input_rigs():
    """name -> rig with an equirectangular output and the model under test as inputs."""
    eq = {"type": "equirectangular", "options": _rot(0.1, 0.05)}
    ff = {"width": 640, "height": 360, "hfov": 3.4906585, "center_dx": 3.0, "center_dy": -2.0,
          "radial": [0.01, -0.02, 0.005], "crop": {"rect": [140, 500, 0, 360], "is_circular": True}}
    pin = {"width": 640, "height": 480, "fx": 380.0, "fy": 372.0, "cx": 318.5, "cy": 241.0}
    rigs = {
        "pinhole_k5": [dict(pin, dist_coeffs=[0.08, -0.03, 0.001, -0.002, 0.004], **_rot(0.0)),
                       dict(pin, dist_coeffs=[0.08, -0.03, 0.001, -0.002, 0.004], **_rot(2.0, 0.2))],
        "pinhole_k14_tilt": [dict(pin, dist_coeffs=[0.05, -0.01, 0.0005, 0.0003, 0.001, 0.01, -0.002, 0.0004,
                                                    0.001, -0.0004, 0.0006, 0.0002, 0.012, -0.018], **_rot(-1.0, -0.3))],
        "pinhole_nodist": [dict(pin, **_rot(0.5))],
        "normal": [dict(OUTPUT_MODELS["normal"], **_rot(0.3, 0.1)), dict(OUTPUT_MODELS["normal"], **_rot(-2.5))],
        "perspective": [dict(OUTPUT_MODELS["perspective"], **_rot(1.2, -0.4))],
        "ocam_fisheye": [dict(OCAM, **_rot(0.0, 0.3)), dict(OCAM, **_rot(math.pi, -0.2, 0.1))],
        "stupidoval": [dict(_rot(0.7, 0.2))],
        "cubic": [dict(_rot(0.4, 0.3, 0.2))],
        "eqarea": [dict(_rot(0.2, 0.1)), dict(antarctic_circle=-0.8, **_rot(-0.3))],
        "fullframe_selection": [dict(ff, selection=[180, 470, 20, 330], **_rot(0.0)),
                                dict(ff, selection=[0, 640, 40, 300], **_rot(math.pi))],
    }
    types = {"pinhole_k5": "pinhole", "pinhole_k14_tilt": "pinhole", "pinhole_nodist": "pinhole",
             "eqarea": ["eqareanorthpole", "eqareasouthpole"], "fullframe_selection": "fullframe_fisheye"}
    out = {}
    for name, opts in rigs.items():
        t = types.get(name, name)
        ts = t if isinstance(t, list) else [t] * len(opts)
        out[name] = {"output": eq, "inputs": [{"type": tt, "options": o} for tt, o in zip(ts, opts)]}
    return out


def output_rigs():
    """name -> rig with the model under test as the output camera and two fisheye + one equirect input."""
    ff = {"width": 640, "height": 360, "hfov": 3.4906585, "center_dx": 0.0, "center_dy": 0.0,
          "radial": [0.0, 0.0, 0.0], "crop": {"rect": [140, 500, 0, 360], "is_circular": True}}
    inputs = [{"type": "fullframe_fisheye", "options": dict(ff, **_rot(0.0))},
              {"type": "fullframe_fisheye", "options": dict(ff, **_rot(0.9, 0.1))},
              {"type": "equirectangular", "options": _rot(0.5, 0.2)}]
    return {t: {"output": {"type": t, "options": dict(o, **_rot(0.2, -0.1))}, "inputs": inputs}
            for t, o in OUTPUT_MODELS.items()}


def mask_rigs():
    """name -> rig exercising the camera masks of camera.cpp:96-187 on 640x360 fullframe fisheyes, and
    the include-mask visibility arbitration of template.cpp:86-116.  PNG areas register their decoded
    ground truth with the oracle (oracle_py.PNG_TRUTH)."""
    import numpy as np

    import oracle_py
    import png_fixture

    ff = {"width": 640, "height": 360, "hfov": 3.4906585, "center_dx": 0.0, "center_dy": 0.0,
          "radial": [0.0, 0.0, 0.0], "crop": {"rect": [140, 500, 0, 360], "is_circular": True}}

    def poly(*pts):
        return {"type": "polygonal", "args": [float(v) + 0.25 for v in pts]}  # int() truncation of args

    concave = poly(200, 50, 400, 80, 300, 180, 420, 300, 180, 320, 250, 180)
    outside = poly(600, -20, 700, 100, 560, 200)
    # PNG: red block (exclude) and a green band (include), blocky so it compresses
    img = np.zeros((360, 640, 3), np.int64)
    img[40:140, 150:260, 0] = 255
    img[200:330, 300:480, 1] = 200
    img[100:220, 380:420, :] = 90
    png, rgb = png_fixture.encode(img, 2, 8, seed=3)
    oracle_py.PNG_TRUTH[png] = rgb
    rigs = {
        "exclude_poly": [dict(ff, exclude_masks=[concave, outside], **_rot(0.0)),
                         dict(ff, selection=[150, 500, 10, 350], exclude_masks=[poly(300, 100, 340, 250, 260, 250)],
                              **_rot(2.0, 0.1))],
        "include_arbitration": [dict(ff, **_rot(0.0)),
                                dict(ff, exclude_masks=[], include_masks=[poly(150, 20, 480, 20, 480, 340, 150, 340)],
                                     **_rot(1.2)),
                                dict(ff, exclude_masks=[poly(10, 10, 60, 10, 35, 80)],
                                     include_masks=[poly(140, 60, 500, 100, 320, 330)], **_rot(2.4, -0.1)),
                                dict(ff, **_rot(-1.5))],
        "include_without_exclude": [dict(ff, include_masks=[poly(150, 20, 480, 20, 480, 340)], **_rot(0.5)),
                                    dict(ff, **_rot(1.5))],
        "png": [dict(ff, exclude_masks=[{"type": "png", "args": list(png)}], **_rot(0.3)),
                dict(ff, exclude_masks=[], include_masks=[concave], **_rot(-0.9))],
    }
    out = {name: {"output": {"type": "equirectangular", "options": _rot(0.1, 0.05)},
                  "inputs": [{"type": "fullframe_fisheye", "options": o} for o in opts]}
           for name, opts in rigs.items()}
    # an overlay whose include mask claims pixels: the inputs' masks lose them (template.cpp:102-116)
    ov = dict(out["exclude_poly"])
    ov["overlays"] = [{"type": "fullframe_fisheye", "options": dict(
        ff, exclude_masks=[], include_masks=[poly(200, 40, 440, 40, 440, 320, 200, 320)], **_rot(1.0))}]
    out["overlay_include"] = ov
    return out


# ---- morph_controlpoints (template_morph.cpp:69-237) --------------------------------------------
def morph_rig(with_equirect=False):
    """Three full-frame fisheyes 120 degrees apart (crop = whole image, as image_to_obj requires,
    fullframe_fisheye_cam.cpp:224), optionally a fourth, equirectangular input."""
    ff = {"width": 480, "height": 320, "hfov": 3.4906585, "center_dx": 1.5, "center_dy": -1.0,
          "radial": [0.01, -0.02, 0.005]}
    ins = [{"type": "fullframe_fisheye", "options": dict(ff, **_rot(k * 2.0943951, 0.05 * k, 0.02 * k))}
           for k in range(3)]
    if with_equirect:
        ins.append({"type": "equirectangular", "options": _rot(0.7, 0.1)})
    return {"output": {"type": "equirectangular", "options": {}}, "inputs": ins}


def morph_points(luts, per_pair=5, seed=0, jitter=0.003):
    """Control points [n0, n1, x0, y0, x1, y1]: output pixels seen by both cameras of a pair, camera
    n0's point read from its map, camera n1's jittered by up to `jitter` (normalized input units)."""
    import numpy as np
    rng = np.random.default_rng(seed)
    n = len(luts)
    cps = []
    for a in range(n):
        for b in range(a + 1, n):
            (ax, ay, aw, ah), a1, a2, am = luts[a]
            (bx, by, bw, bh), b1, b2, bm = luts[b]
            x0, y0 = max(ax, bx), max(ay, by)
            x1, y1 = min(ax + aw, bx + bw), min(ay + ah, by + bh)
            if x0 >= x1 or y0 >= y1:
                continue
            both = (am[y0 - ay:y1 - ay, x0 - ax:x1 - ax] > 0) & (bm[y0 - by:y1 - by, x0 - bx:x1 - bx] > 0)
            ys, xs = np.nonzero(both)
            if len(ys) < per_pair:
                continue
            for k in rng.choice(len(ys), per_pair, replace=False):
                X, Y = xs[k] + x0, ys[k] + y0
                j = rng.uniform(-jitter, jitter, 2)
                cps.append([a, b, float(a1[Y - ay, X - ax]), float(a2[Y - ay, X - ax]),
                            float(b1[Y - by, X - bx] + j[0]), float(b2[Y - by, X - bx] + j[1])])
    return cps
