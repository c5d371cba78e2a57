"""ctypes bindings to oracle/liboctvr_oracle.so (TEST INFRASTRUCTURE ONLY).

The oracle is the CPU restatement of the reference arithmetic; tests use it as the checker for the
HIP product path.  Rig JSON follows the reference schema.
"""
import ctypes as C
import json
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
_LIB = None


class OrcCamera(C.Structure):
    _fields_ = [
        ("type", C.c_int),
        ("R", C.c_double * 9),
        ("Rinv", C.c_double * 9),
        ("min_lon", C.c_double), ("max_lon", C.c_double),
        ("min_lat", C.c_double), ("max_lat", C.c_double), ("scale_lon", C.c_double),
        ("width", C.c_int), ("height", C.c_int),
        ("crop_x", C.c_int), ("crop_y", C.c_int), ("crop_w", C.c_int), ("crop_h", C.c_int),
        ("crop_circular", C.c_int),
        ("hfov", C.c_double), ("center_dx", C.c_double), ("center_dy", C.c_double),
        ("rad", C.c_double * 6),
        ("fx", C.c_double), ("fy", C.c_double), ("cx", C.c_double), ("cy", C.c_double),
        ("k", C.c_double * 4),
        ("sel", C.c_int), ("sel_l", C.c_int), ("sel_r", C.c_int), ("sel_t", C.c_int), ("sel_b", C.c_int),
        ("dist", C.c_double * 14), ("tilt", C.c_double * 9),
        ("aspect", C.c_double), ("cam_x", C.c_double), ("cam_y", C.c_double), ("cam_z", C.c_double),
        ("sf", C.c_double), ("circle", C.c_double),
        ("len_pol", C.c_int), ("len_invpol", C.c_int),
        ("xc", C.c_double), ("yc", C.c_double), ("oc", C.c_double), ("od", C.c_double), ("oe", C.c_double),
        ("pol", C.c_double * 64), ("invpol", C.c_double * 64),
        ("excl", C.c_void_p), ("incl", C.c_void_p),
    ]


class OrcFrame(C.Structure):
    _fields_ = [
        ("n", C.c_int),
        ("in_w", C.POINTER(C.c_int)),
        ("in_h", C.POINTER(C.c_int)),
        ("in_yuv", C.POINTER(C.c_void_p)),
        ("in_pitch", C.POINTER(C.c_size_t)),
        ("rois", C.POINTER(C.c_int)),
        ("map1", C.POINTER(C.c_void_p)),
        ("map2", C.POINTER(C.c_void_p)),
        ("masks", C.POINTER(C.c_void_p)),
        ("out_w", C.c_int), ("out_h", C.c_int),
        ("out_yuv", C.c_void_p),
        ("out_pitch", C.c_size_t),
        ("enable_gain", C.c_int),
        ("gains_in", C.POINTER(C.c_double)),
        ("gains_out", C.POINTER(C.c_double)),
        ("threads", C.c_int),
        ("row_begin", C.c_int), ("row_end", C.c_int),
        ("blend", C.c_int),
        ("seams", C.POINTER(C.c_void_p)),
        ("vig", C.POINTER(C.c_void_p)),
        ("scale_w", C.c_int), ("scale_h", C.c_int),
        ("preview", C.c_void_p),
        ("preview_w", C.c_int), ("preview_h", C.c_int),
        ("preview_pitch", C.c_size_t),
        ("remap_tex", C.c_int),
    ]


def lib():
    global _LIB
    if _LIB is None:
        so = os.path.join(ORACLE_DIR, "liboctvr_oracle.so")
        srcs = [os.path.join(ORACLE_DIR, f) for f in os.listdir(ORACLE_DIR) if f.endswith((".c", ".h"))]
        if not os.path.exists(so) or os.path.getmtime(so) < max(os.path.getmtime(f) for f in srcs):
            subprocess.check_call(["make", "-s", "-C", ORACLE_DIR])
        L = C.CDLL(so)
        L.orc_lut_build.restype = C.c_int
        L.orc_solve.restype = C.c_int
        L.orc_gain_feed.restype = C.c_int
        L.orc_stitch_frame.restype = C.c_int
        _LIB = L
    return _LIB


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


def rotation_rpy(roll, yaw, pitch):
    R = (C.c_double * 9)()
    lib().orc_rotation_rpy(C.c_double(roll), C.c_double(yaw), C.c_double(pitch), R)
    return np.array(R[:]).reshape(3, 3)


def invert3(R):
    a = np.ascontiguousarray(R, dtype=np.float64).reshape(9)
    out = np.zeros(9)
    lib().orc_invert3(_p(a), _p(out))
    return out.reshape(3, 3)


def camera_from_json(cam):
    """Build an orc_camera from one {type, options} entry (camera.cpp:27-136)."""
    t, o = cam["type"], cam.get("options", {})
    c = OrcCamera()
    L = lib()
    if t == "equirectangular":
        import math
        L.orc_camera_equirect(C.byref(c), C.c_double(o.get("min_lat", -math.pi / 2)),
                              C.c_double(o.get("max_lat", math.pi / 2)), C.c_double(o.get("scale_lon", 1.0)))
    elif t == "fullframe_fisheye":
        crop = o.get("crop")
        rect = crop["rect"] if crop else [0, 0, 0, 0]
        rad = (C.c_double * 3)(*o["radial"])
        L.orc_camera_fullframe_fisheye(C.byref(c), o["width"], o["height"], rect[0], rect[1], rect[2], rect[3],
                                       1 if crop else 0, 1 if (crop and crop["is_circular"]) else 0,
                                       C.c_double(o["hfov"]), C.c_double(o["center_dx"]), C.c_double(o["center_dy"]),
                                       rad)
    elif t == "fisheye":
        k = (C.c_double * 4)(*o["dist_coeffs"][:4])
        L.orc_camera_fisheye(C.byref(c), o["width"], o["height"], C.c_double(o["fx"]), C.c_double(o["fy"]),
                             C.c_double(o["cx"]), C.c_double(o["cy"]), k)
    elif t == "pinhole":
        d = o.get("dist_coeffs", [])
        L.orc_camera_pinhole(C.byref(c), o["width"], o["height"], C.c_double(o["fx"]), C.c_double(o["fy"]),
                             C.c_double(o["cx"]), C.c_double(o["cy"]), (C.c_double * max(1, len(d)))(*d), len(d))
    elif t == "normal":
        L.orc_camera_normal(C.byref(c), C.c_double(o["aspect_ratio"]), C.c_double(o["cam_opt"]))
    elif t == "perspective":
        L.orc_camera_perspective(C.byref(c), C.c_double(o["aspect_ratio"]), C.c_double(o["sf"]))
    elif t == "ocam_fisheye":
        pol, inv = o["pol"], o["invpol"]
        L.orc_camera_ocam(C.byref(c), (C.c_double * len(pol))(*pol), len(pol), (C.c_double * len(inv))(*inv), len(inv),
                          C.c_double(o["xc"]), C.c_double(o["yc"]), C.c_double(o["c"]), C.c_double(o["d"]),
                          C.c_double(o["e"]), o["width"], o["height"])
    elif t in ("stupidoval", "cubic", "eqareanorthpole", "eqareasouthpole"):
        import math
        typ = {"stupidoval": 7, "cubic": 8, "eqareanorthpole": 9, "eqareasouthpole": 10}[t]
        circle = o.get("arctic_circle", math.pi / 3) if t == "eqareanorthpole" else o.get("antarctic_circle", -math.pi / 3)
        L.orc_camera_simple(C.byref(c), typ, C.c_double(circle))
    else:
        raise ValueError("camera type not in the oracle: " + t)
    if "selection" in o:
        l, r, tt, b = o["selection"]
        L.orc_camera_set_selection(C.byref(c), o["width"], o["height"], l, r, tt, b)
    if "rotation" in o:
        r = o["rotation"]
        R = rotation_rpy(r["roll"], r["yaw"], r["pitch"])
    else:
        R = rotation_rpy(0, 0, 0)
    if "rotation_matrix" in o:
        R = np.array(o["rotation_matrix"], dtype=np.float64).reshape(3, 3)
    Rc = (C.c_double * 9)(*R.reshape(9))
    L.orc_camera_set_rotation(C.byref(c), Rc)
    if "longitude_selection" in o:
        c.min_lon, c.max_lon = o["longitude_selection"]
    excl, incl = camera_masks(o)
    c._masks = (excl, incl)  # keep the arrays alive while the struct points at them
    if excl is not None:
        c.sel = 0
        c.width, c.height = o["width"], o["height"]
        c.excl = excl.ctypes.data
        if incl is not None:
            c.incl = incl.ctypes.data
    return c


# PNG mask areas: tests register the RGB image each PNG byte string encodes (tests/png_fixture.py); the
# oracle takes that ground truth instead of decoding (libpng is a third-party dependency).
PNG_TRUTH = {}


def fill_poly(img, pts, color):
    """cv::fillPoly(img, {pts}, color) restatement (oracle/octvr_oracle_masks.c)."""
    flat = np.ascontiguousarray(np.asarray(pts, np.int32).reshape(-1))
    lib().orc_fill_poly(_p(img), img.shape[1], img.shape[0], _p(flat), len(flat) // 2, C.c_uint8(color))


def camera_masks(o):
    """Camera ctor mask part (camera.cpp:72-123) + draw_mask (:146-187) -> (exclude, include) or None."""
    if not any(k in o for k in ("selection", "exclude_masks", "include_masks")):
        return None, None
    w, h = o["width"], o["height"]
    m = {"excl": None, "incl": None}

    def prepare(k, v):
        if m[k] is None:
            m[k] = np.full((h, w), v, np.uint8)

    def draw(areas, include):
        for a in areas:
            if a["type"] == "polygonal":
                pts = [int(v) for v in a["args"]]
                fill_poly(m["incl" if include else "excl"], pts, 255)
            elif a["type"] == "png":
                rgb = PNG_TRUTH[bytes(a["args"])]
                if m["excl"] is None or rgb.shape[:2] != (h, w):
                    raise ValueError("png mask size differs from the exclude mask (camera.cpp:170)")
                m["excl"][rgb[..., 0] != 0] = 255
                m["incl"][rgb[..., 1] != 0] = 255
            else:
                raise ValueError(a["type"])
    if "selection" in o:
        prepare("excl", 255)
        l, r, t, b = o["selection"]
        fill_poly(m["excl"], [l, t, l, b - 1, r - 1, b - 1, r - 1, t], 0)
    if "exclude_masks" in o:
        prepare("excl", 0)
        prepare("incl", 0)
        draw(o["exclude_masks"], False)
    if "include_masks" in o:
        prepare("incl", 0)
        draw(o["include_masks"], True)
    return m["excl"], m["incl"]


def lut_build(rig, out_w, out_h, use_roi=True, threads=1):
    """Per input, then per overlay: (roi, map1, map2, mask) cropped to the ROI, as
    MapperTemplate::add_input, including the include-mask visible_mask arbitration across inputs and
    overlays (template.cpp:86-116).  threads > 1: row bands on that many threads (same result)."""
    out = camera_from_json(rig["output"])
    res = []
    visible = None
    n_inputs = len(rig["inputs"])
    for k, cam in enumerate(rig["inputs"] + rig.get("overlays", [])):
        c = camera_from_json(cam)
        m1 = np.empty((out_h, out_w), np.float32)
        m2 = np.empty((out_h, out_w), np.float32)
        mk = np.empty((out_h, out_w), np.uint8)
        roi = (C.c_int * 4)()
        if visible is None and c.incl:
            visible = np.zeros((out_h, out_w), np.uint8)
        vp = _p(visible) if visible is not None else None
        rc = lib().orc_lut_build_vis_mt(C.byref(out), C.byref(c), out_w, out_h, _p(m1), _p(m2), _p(mk), int(use_roi),
                                        roi, vp, int(threads))
        assert rc == 0
        if visible is not None and c.incl:
            for (px, py, pw, ph), _, _, pm in res[:n_inputs]:  # only this->inputs (template.cpp:106)
                pm[visible[py:py + ph, px:px + pw] == 2] = 0
            visible[visible == 2] = 1
        x, y, w, h = roi[:]
        res.append(((x, y, w, h), m1[y:y + h, x:x + w].copy(), m2[y:y + h, x:x + w].copy(), mk[y:y + h, x:x + w].copy()))
    return res


def project(cam_from, cam_to, u, v):
    """Camera::image_to_obj of cam_from, then obj_to_image of cam_to (JSON cameras); None where the
    reference throws (no image_to_obj)."""
    a, b = camera_from_json(cam_from), camera_from_json(cam_to)
    x, y = C.c_double(), C.c_double()
    if lib().orc_project(C.byref(a), C.byref(b), C.c_double(u), C.c_double(v), C.byref(x), C.byref(y)):
        return None
    return x.value, y.value


def morph_controlpoints(rig, luts, out_w, out_h, control_points, tri_cap=4096):
    """MapperTemplate::morph_controlpoints on lut_build()'s per-input (roi, map1, map2, mask) (inputs
    only).  Returns (kept or negative error, new luts, [(src_tris, dst_tris)] per input)."""
    out = camera_from_json(rig["output"])
    cams = [camera_from_json(c) for c in rig["inputs"]]
    n = len(cams)
    cam_arr = (C.c_void_p * n)(*[C.addressof(c) for c in cams])
    rois = (C.c_int * (4 * n))(*[v for (roi, _, _, _) in luts[:n] for v in roi])
    m1 = [np.ascontiguousarray(l[1], np.float32).copy() for l in luts[:n]]
    m2 = [np.ascontiguousarray(l[2], np.float32).copy() for l in luts[:n]]
    mk = [np.ascontiguousarray(l[3], np.uint8).copy() for l in luts[:n]]
    cps = np.ascontiguousarray(np.asarray(control_points, np.float64).reshape(-1, 6))
    st = [np.zeros((tri_cap, 6), np.float32) for _ in range(n)]
    dt = [np.zeros((tri_cap, 6), np.float32) for _ in range(n)]
    nt = (C.c_int * n)()
    P = lambda arrs: (C.c_void_p * n)(*[a.ctypes.data for a in arrs])
    L = lib()
    L.orc_morph_controlpoints.restype = C.c_int
    rc = L.orc_morph_controlpoints(C.byref(out), cam_arr, n, out_w, out_h, rois, P(m1), P(m2), P(mk), _p(cps),
                                   len(cps), P(st), P(dt), tri_cap, nt)
    new = [(luts[i][0], m1[i], m2[i], mk[i]) for i in range(n)]
    return rc, new, [(st[i][:nt[i]].copy(), dt[i][:nt[i]].copy()) for i in range(n)]


def delaunay(points, cap=8192):
    """cv::Subdiv2D(Rect(0,0,1,1)) + insert + getTriangleList, triangles inside [0,1]^2 kept."""
    pts = np.ascontiguousarray(np.asarray(points, np.float32).reshape(-1))
    out = np.zeros((cap, 6), np.float32)
    L = lib()
    L.orc_delaunay_triangles.restype = C.c_int
    k = L.orc_delaunay_triangles(_p(pts), len(pts) // 2, _p(out), cap)
    assert k >= 0, k
    return out[:k].copy()


def project_f64(rig_cam_out, rig_cam_in, W, H, y0=0, y1=None, threads=8):
    """FP64 (x, y) of output rows [y0, y1) through rig_cam_out's image_to_obj and rig_cam_in's
    obj_to_image (template.cpp:70-83), before the f32 rounding."""
    y1 = H if y1 is None else y1
    out = camera_from_json(rig_cam_out)
    c = camera_from_json(rig_cam_in)
    x = np.empty((y1 - y0, W), np.float64)
    y = np.empty((y1 - y0, W), np.float64)
    lib().orc_project_f64(C.byref(out), C.byref(c), W, H, y0, y1, _p(x), _p(y), int(threads))
    return x, y


def lut_rows(rig_cam_out, rig_cam_in, W, H, y0, y1):
    """Oracle LUT for output rows [y0, y1) of one input camera (full width, no ROI crop)."""
    out = camera_from_json(rig_cam_out)
    c = camera_from_json(rig_cam_in)
    m1 = np.empty((y1 - y0, W), np.float32)
    m2 = np.empty((y1 - y0, W), np.float32)
    mk = np.empty((y1 - y0, W), np.uint8)
    lib().orc_lut_rows(C.byref(out), C.byref(c), W, H, y0, y1, _p(m1), _p(m2), _p(mk))
    return m1, m2, mk


def remap_u8(src, map1, map2, scale_x, scale_y):
    src = np.ascontiguousarray(src)
    cn = 1 if src.ndim == 2 else src.shape[2]
    h, w = src.shape[:2]
    mh, mw = map1.shape
    m1 = np.ascontiguousarray(map1, np.float32)
    m2 = np.ascontiguousarray(map2, np.float32)
    dst = np.zeros((mh, mw, cn) if cn > 1 else (mh, mw), np.uint8)
    lib().orc_remap_u8(_p(src), w, h, C.c_size_t(w * cn), cn, _p(m1), _p(m2), mw, mh, C.c_size_t(mw),
                       C.c_float(scale_x), C.c_float(scale_y), _p(dst), C.c_size_t(mw * cn))
    return dst


def fast_remap_tex_rgba(rgba, map1, map2):
    """A12: CUDA fastRemap texture bilinear (normalized maps) -> u8x4 (oracle model, parity unpinned)."""
    rgba = np.ascontiguousarray(rgba)
    h, w = rgba.shape[:2]
    m1 = np.ascontiguousarray(map1, np.float32)
    m2 = np.ascontiguousarray(map2, np.float32)
    mh, mw = m1.shape
    out = np.zeros((mh, mw, 4), np.uint8)
    lib().orc_fast_remap_tex_rgba(_p(rgba), w, h, C.c_size_t(w * 4), _p(m1), _p(m2), mw, mh, C.c_size_t(mw), _p(out),
                                  C.c_size_t(mw * 4))
    return out


def bilinear_tab():
    t = np.zeros(4096, np.int16)
    lib().orc_bilinear_tab(_p(t))
    return t.reshape(1024, 4)


def solve(A, b):
    A = np.ascontiguousarray(A, np.float64)
    b = np.ascontiguousarray(b, np.float64)
    x = np.zeros_like(b)
    ok = lib().orc_solve(_p(A), _p(b), len(b), _p(x))
    return x if ok else None


def yuv420_to_rgba(yuv, w, h):
    out = np.zeros((h, w, 4), np.uint8)
    yuv = np.ascontiguousarray(yuv)
    lib().orc_yuv420_to_rgba(_p(yuv), w, h, C.c_size_t(yuv.shape[1]), _p(out), C.c_size_t(w * 4))
    return out


def _pyr(fn, src, dshape, dtype, threads=1):
    src = np.ascontiguousarray(src)
    out = np.zeros(dshape, dtype)
    getattr(lib(), fn)(_p(src), src.shape[1], src.shape[0], _p(out), threads)
    return out


def fast_pyr_down_u8x4(src, threads=1):
    h, w = src.shape[:2]
    return _pyr("orc_fast_pyr_down_u8x4", src, ((h + 1) // 2, (w + 1) // 2, 4), np.uint8, threads)


def pyr_up_u8x4(src, threads=1):
    h, w = src.shape[:2]
    return _pyr("orc_pyr_up_u8x4", src, (2 * h, 2 * w, 4), np.uint8, threads)


def pyr_up_s16x3(src, threads=1):
    h, w = src.shape[:2]
    return _pyr("orc_pyr_up_s16x3", src.astype(np.int16), (2 * h, 2 * w, 3), np.int16, threads)


def pyr_down_f32(src, threads=1):
    h, w = src.shape[:2]
    return _pyr("orc_pyr_down_f32", src.astype(np.float32), ((h + 1) // 2, (w + 1) // 2), np.float32, threads)


def vignette_map(opts, w=512, h=512):
    """Vignette(options).getMap(w, h) (vignette.cpp:18-54); None without a "vignette" option."""
    if "vignette" not in opts:
        return None
    a, b, c, d = (float(v) for v in opts["vignette"])
    if "exposure" in opts:
        ev = float(np.float32(2.0 ** float(opts["exposure"])))
        a, b, c, d = a / ev, b / ev, c / ev, d / ev
    out = np.zeros((h, w), np.float32)
    lib().orc_vignette_map(C.c_double(a), C.c_double(b), C.c_double(c), C.c_double(d), w, h, _p(out))
    return out


def resize_linear_cuda_f32(src, dw, dh):
    src = np.ascontiguousarray(src, np.float32)
    out = np.zeros((dh, dw), np.float32)
    lib().orc_resize_linear_cuda_f32(_p(src), src.shape[1], src.shape[0], _p(out), dw, dh)
    return out


def blend_bands(blend):
    return lib().orc_blend_bands(int(blend))


def resize_linear(src, dw, dh):
    """cv::resize INTER_LINEAR u8 on the CPU (oracle/octvr_oracle_seam.c)."""
    src = np.ascontiguousarray(src)
    sh, sw = src.shape[:2]
    cn = 1 if src.ndim == 2 else src.shape[2]
    out = np.zeros((dh, dw) + (() if cn == 1 else (cn,)), np.uint8)
    lib().orc_resize_linear_u8(_p(src), sw, sh, C.c_size_t(sw * cn), cn, _p(out), dw, dh, C.c_size_t(dw * cn))
    return out


def distance_transform(src):
    src = np.ascontiguousarray(src, dtype=np.uint8)
    h, w = src.shape
    out = np.zeros((h, w), np.float32)
    lib().orc_distance_transform_l2_3x3(_p(src), w, h, C.c_size_t(w), _p(out), C.c_size_t(w))
    return out


def create_masks(rois, masks, out_w):
    """MapperTemplate::create_masks() (DistanceSeamFinder): ROI-sized u8 seam masks."""
    n = len(masks)
    masks = [np.ascontiguousarray(m, dtype=np.uint8) for m in masks]
    seams = [np.zeros_like(m) for m in masks]
    r = np.ascontiguousarray(np.asarray(rois, dtype=np.int32).reshape(-1))
    arr = C.c_void_p * n
    rc = lib().orc_create_masks(n, _p(r), arr(*[m.ctypes.data for m in masks]), int(out_w),
                                arr(*[s.ctypes.data for s in seams]))
    assert rc == 0
    return seams


def rgb_to_yuv420(rgb):
    h, w, cn = rgb.shape
    out = np.zeros((h * 3 // 2, w), np.uint8)
    rgb = np.ascontiguousarray(rgb)
    lib().orc_rgb_to_yuv420(_p(rgb), w, h, C.c_size_t(w * cn), cn, _p(out), C.c_size_t(w))
    return out


def gain_feed(rois, warped, masks, out_w, out_h):
    n = len(rois)
    r = np.ascontiguousarray(np.array(rois, np.int32).reshape(-1))
    warped = [np.ascontiguousarray(a) for a in warped]
    masks = [np.ascontiguousarray(a) for a in masks]
    wp = (C.c_void_p * n)(*[a.ctypes.data for a in warped])
    mp = (C.c_void_p * n)(*[a.ctypes.data for a in masks])
    g = np.zeros(n)
    rc = lib().orc_gain_feed(n, r.ctypes.data_as(C.POINTER(C.c_int)), wp, mp, out_w, out_h, _p(g))
    assert rc == 0
    return g


def stitch_frame(in_yuv, in_sizes, rois, map1s, map2s, masks, out_w, out_h, enable_gain=True, gains=None,
                 threads=1, row_band=None, blend=0, seams=None, vig=None, scale=None, preview=None, remap_tex=False):
    """One Mapper::stitch -> (YUV420P output, gains); preview=(w, h): also the preview_output image,
    returned as a third value.  remap_tex: warp as the reference's CUDA fastRemap texture path
    (orc_fast_remap_tex_rgba; the library's OCTVR_REMAP_TEXTURE mode)."""
    n = len(in_yuv)
    keep = []

    def arr(t, vals):
        a = (t * len(vals))(*vals)
        keep.append(a)
        return a

    in_yuv = [np.ascontiguousarray(a) for a in in_yuv]
    map1s = [np.ascontiguousarray(a, np.float32) for a in map1s]
    map2s = [np.ascontiguousarray(a, np.float32) for a in map2s]
    masks = [np.ascontiguousarray(a, np.uint8) for a in masks]
    ow, oh = scale if scale else (out_w, out_h)
    out = np.zeros((oh * 3 // 2, ow), np.uint8)
    gout = np.zeros(n)
    f = OrcFrame()
    if scale:
        f.scale_w, f.scale_h = scale
    f.n = n
    f.in_w = arr(C.c_int, [s[0] for s in in_sizes])
    f.in_h = arr(C.c_int, [s[1] for s in in_sizes])
    f.in_yuv = arr(C.c_void_p, [a.ctypes.data for a in in_yuv])
    f.in_pitch = arr(C.c_size_t, [a.shape[1] for a in in_yuv])
    f.rois = arr(C.c_int, [v for r in rois for v in r])
    f.map1 = arr(C.c_void_p, [a.ctypes.data for a in map1s])
    f.map2 = arr(C.c_void_p, [a.ctypes.data for a in map2s])
    f.masks = arr(C.c_void_p, [a.ctypes.data for a in masks])
    f.out_w, f.out_h = out_w, out_h
    f.out_yuv = out.ctypes.data
    f.out_pitch = ow
    f.enable_gain = int(enable_gain)
    f.remap_tex = int(remap_tex)
    gin = None
    if gains is not None:
        gin = np.ascontiguousarray(gains, np.float64)
        f.gains_in = gin.ctypes.data_as(C.POINTER(C.c_double))
    f.gains_out = gout.ctypes.data_as(C.POINTER(C.c_double))
    f.threads = threads
    if row_band:
        f.row_begin, f.row_end = row_band
    f.blend = blend
    if seams is not None:
        seams = [np.ascontiguousarray(a, np.uint8) for a in seams]
        keep.append(seams)
        f.seams = arr(C.c_void_p, [a.ctypes.data for a in seams])
    if vig is not None:
        vig = [None if v is None else np.ascontiguousarray(v, np.float32) for v in vig]
        keep.append(vig)
        f.vig = arr(C.c_void_p, [None if v is None else v.ctypes.data for v in vig])
    pv = None
    if preview:
        pv = np.zeros((preview[1], preview[0], 3), np.uint8)
        f.preview = pv.ctypes.data
        f.preview_w, f.preview_h = preview
        f.preview_pitch = preview[0] * 3
    rc = lib().orc_stitch_frame(C.byref(f))
    assert rc == 0
    return (out, gout, pv) if preview else (out, gout)


def fastmapper_nv12(in_nv12, in_sizes, map1s, map2s, masks, out_w, out_h):
    """vr::FastMapper::stitch_nv12 (full-frame maps / masks): W x 1.5H output, chroma rows V, U."""
    n = len(in_nv12)
    in_nv12 = [np.ascontiguousarray(a) for a in in_nv12]
    m1 = [np.ascontiguousarray(a, np.float32) for a in map1s]
    m2 = [np.ascontiguousarray(a, np.float32) for a in map2s]
    mk = [np.ascontiguousarray(a, np.uint8) for a in masks]
    out = np.zeros((out_h * 3 // 2, out_w), np.uint8)
    P = C.c_void_p * n
    rc = lib().orc_fastmapper_nv12(n, (C.c_int * n)(*[s[0] for s in in_sizes]), (C.c_int * n)(*[s[1] for s in in_sizes]),
                                   P(*[a.ctypes.data for a in m1]), P(*[a.ctypes.data for a in m2]),
                                   P(*[a.ctypes.data for a in mk]), out_w, out_h, P(*[a.ctypes.data for a in in_nv12]),
                                   (C.c_size_t * n)(*[a.shape[1] for a in in_nv12]), _p(out), C.c_size_t(out_w))
    assert rc == 0
    return out


# ---------------------------------------------------------------------------------------------
# synthetic data (same generator as oracle/golden_gen/gen_golden.cpp)
# ---------------------------------------------------------------------------------------------
def splitmix64(seed, k):
    """k-th output (k = 0, 1, ...) of splitmix64 seeded with `seed`, vectorised over k."""
    k = np.asarray(k, dtype=np.uint64) + np.uint64(1)
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + k * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def splitmix_bytes(seed, n):
    k = np.arange(1, n + 1, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + k * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return (z & np.uint64(0xFF)).astype(np.uint8)


def rand_img(w, h, cn, seed):
    a = splitmix_bytes(seed, w * h * cn)
    return a.reshape((h, w, cn) if cn > 1 else (h, w))


def remap_kat_maps(per=256):
    """Maps of gen_golden.cpp remap_code_kat(): 256 random integer positions per fractional code."""
    k = np.arange(1024 * per, dtype=np.uint64)
    h = splitmix64(2718, k)
    sx = (h % np.uint64(63)).astype(np.float32)
    sy = ((h >> np.uint64(16)) % np.uint64(63)).astype(np.float32)
    code = (k // np.uint64(per)).astype(np.int64)
    m1 = sx + (code & 31).astype(np.float32) / np.float32(32)
    m2 = sy + (code >> 5).astype(np.float32) / np.float32(32)
    return m1.reshape(1, -1).astype(np.float32), m2.reshape(1, -1).astype(np.float32)


def rj_number(txt):
    """rapidjson 1.0.2 default-flag number parsing (reader.h:1090-1276, strtod.h:26-44), so the oracle
    sees the same doubles the reference sees."""
    s, i, n = txt, 0, len(txt)
    minus = s[0] == "-"
    if minus:
        i += 1
    M64 = (1 << 64) - 1
    iv, i64, use64, sig = 0, 0, False, 0
    if s[i] == "0":
        i += 1
    else:
        iv = ord(s[i]) - 48
        i += 1
        lim, lastd = (214748364, "8") if minus else (429496729, "5")
        while i < n and s[i].isdigit():
            if iv >= lim and (iv != lim or s[i] > lastd):
                i64, use64 = iv, True
                break
            iv = iv * 10 + ord(s[i]) - 48
            i += 1
            sig += 1
    use_d, d = False, 0.0
    if use64:
        lim, lastd = (0x0CCCCCCCCCCCCCCC, "8") if minus else (0x1999999999999999, "5")
        while i < n and s[i].isdigit():
            if i64 >= lim and (i64 != lim or s[i] > lastd):
                d, use_d = float(i64), True
                break
            i64 = (i64 * 10 + ord(s[i]) - 48) & M64
            i += 1
            sig += 1
    if use_d:
        while i < n and s[i].isdigit():
            d = d * 10 + (ord(s[i]) - 48)
            i += 1
    exp_frac = 0
    if i < n and s[i] == ".":
        i += 1
        if not use_d:
            if not use64:
                i64 = iv
            while i < n and s[i].isdigit():
                if i64 > 0x1FFFFFFFFFFFFF:
                    break
                i64 = i64 * 10 + ord(s[i]) - 48
                i += 1
                exp_frac -= 1
                if i64 != 0:
                    sig += 1
            d, use_d = float(i64), True
        while i < n and s[i].isdigit():
            if sig < 17:
                d = d * 10.0 + (ord(s[i]) - 48)
                exp_frac -= 1
                if d > 0.0:
                    sig += 1
            i += 1
    exp = 0
    if i < n and s[i] in "eE":
        i += 1
        if not use_d:
            d, use_d = float(i64 if use64 else iv), True
        em = False
        if s[i] == "+":
            i += 1
        elif s[i] == "-":
            em, i = True, i + 1
        exp = int(s[i:])
        if em:
            exp = -exp
    if use_d:
        p = exp + exp_frac
        def fast(v, e):
            return 0.0 if e < -308 else (v * float("1e%d" % e) if e >= 0 else v / float("1e%d" % -e))
        d = fast(fast(d, -308), p + 308) if p < -308 else fast(d, p)
        return -d if minus else d
    v = i64 if use64 else iv
    return float(-v if minus else v)


def json_loads_rj(text):
    """json.loads with rapidjson's (not always correctly rounded) number conversion."""
    return json.loads(text, parse_float=rj_number)


def load_rig(name):
    gdir = os.path.join(ROOT, "tests", "golden")
    with open(os.path.join(gdir, name + ".json")) as f:
        rig = json_loads_rj(f.read())
    z = np.load(os.path.join(gdir, name + ".npz"))
    return rig, z
