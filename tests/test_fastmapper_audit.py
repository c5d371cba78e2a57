"""FastMapper index audit on the CPU (no GPU): octvr_debug_fastmapper_audit builds the FastMapper plan
exactly as octvr_fastmapper_create does (modules/octvr/src/mapper_fast.cpp:27-109) and replays on the host
every index fast_y_kernel / fast_uv_kernel derive (opencv-octvr_amd/csrc/fastmapper.hip fast_plane; the
reference kernel is imgproc/src/opencl/remap_weighted.cl:20-78): the run table per workgroup, the block of
every camera slot of every group (dead slots included), the entry / weight / header index of every lane in
both entry formats, the camera, the 8-byte tap-row loads against the NV12 frame, the byte each in-image tap
takes from its load, and the output bytes.

Round 4 recorded an illegal-address fault in the wide-entry kernel of an uncommitted build
("The round-4 FastMapper fault"); these tests pin that every access of the shipped kernels
lies inside its allocation on the golden rigs, on the full C2 rig (the F2 bench workload), on random maps
whose luma blocks force the wide fallback, and on a frame whose taps sit on every edge."""
import json

import numpy as np
import pytest

import oracle_py as O


def _full_frame_template(ox, rig, W, H):
    luts = O.lut_build(rig, W, H, use_roi=False, threads=8)
    assert all(l[0] == (0, 0, W, H) for l in luts)
    return ox.MapperTemplate.from_arrays(W, H, [l[0] for l in luts], [l[1] for l in luts], [l[2] for l in luts],
                                         [l[3] for l in luts])


def _check(rep, blocks_live=True):
    for plane in ("y", "uv"):
        p = rep[plane]
        assert p["violations"] == 0, (plane, p["first"])
        # every live slot is a block of the plane, and the highest block any slot loads is the last one
        assert p["live_slots"] == p["blocks"]
        if blocks_live:
            assert p["max_block"] == p["blocks"] - 1
        assert p["slot_loads"] == 4 * p["groups"]


@pytest.mark.parametrize("wide", [False, True], ids=["compact", "wide"])
@pytest.mark.parametrize("name", ["rigA", "rigB", "rigC", "rigD"])
def test_fastmapper_audit_golden_rigs(product_lib, name, wide):
    ox = product_lib
    rig, z = O.load_rig(name)
    W, H = (int(v) for v in z["out_size"])
    mt = _full_frame_template(ox, rig, W, H)
    sizes = [(c["options"]["width"], c["options"]["height"]) for c in rig["inputs"]]
    for pad in (0, 64):
        ok, rep = ox.debug_fastmapper_audit(mt, sizes, wide=wide, pitch_pad=pad)
        assert ok, rep
        _check(rep)
        assert rep["y"]["compact"] == (0 if wide else 1) and rep["uv"]["compact"] == (0 if wide else 1)
        assert rep["y"]["taps_in_image"] > 0


@pytest.mark.parametrize("wide", [False, True], ids=["compact", "wide"])
def test_fastmapper_audit_c2_full_frame(product_lib, wide):
    """The F2 bench workload: the C2 rig (6 x 3840x2160 fisheyes -> 7680x3840) without ROI."""
    ox = product_lib
    from octvr_amd import synthetic
    rig, W, H, sizes = synthetic.CONFIGS["F2"]()
    mt = _full_frame_template(ox, rig, W, H)
    ok, rep = ox.debug_fastmapper_audit(mt, sizes, wide=wide)
    assert ok, rep
    _check(rep)
    # ~4 of the 6 fisheyes have feather weight in a C2 run: some runs need a second group
    assert rep["y"]["groups"] > rep["y"]["runs"]
    assert rep["y"]["blocks"] > 3 * rep["y"]["runs"]


def test_fastmapper_audit_wide_fallback_and_edges(product_lib):
    """Random maps over a 4000-pixel-wide source (a luma block spans >= 2048 px: the Y plane falls back to
    the 8-byte entries, the chroma plane stays compact), and maps onto every edge of a 42x26 frame (taps at
    -1, 0, w-1, w; the last chroma row's 8-byte loads start at size - 8)."""
    ox = product_lib
    W, H = 96, 32
    rng = np.random.default_rng(9)
    sizes = [(4000, 24), (64, 20)]
    m1 = [rng.uniform(0.0, 1.0, (H, W)).astype(np.float32) for _ in sizes]
    m2 = [rng.uniform(0.0, 1.0, (H, W)).astype(np.float32) for _ in sizes]
    mk = [np.full((H, W), 255, np.uint8) for _ in sizes]
    mk[1][:, W // 2:] = 0
    mt = ox.MapperTemplate.from_arrays(W, H, [[0, 0, W, H]] * 2, m1, m2, mk)
    ok, rep = ox.debug_fastmapper_audit(mt, sizes)
    assert ok, rep
    _check(rep, blocks_live=False)
    assert rep["y"]["compact"] == 0 and rep["uv"]["compact"] == 1
    # edge taps: map values on the border of the source, 1/2 pixel in and out
    w, h = 42, 26
    xs = np.array([-0.5, 0.0, 0.49, 1.0, w - 1.5, w - 1.0, w - 0.51, w - 0.0, w + 0.4]) / w
    ys = np.array([-0.5, 0.0, 0.49, 1.0, h - 1.5, h - 1.0, h - 0.51, h - 0.0, h + 0.4]) / h
    gx, gy = np.meshgrid(xs, ys)
    m1 = np.resize(gx.ravel(), (H, W)).astype(np.float32)
    m2 = np.resize(gy.ravel(), (H, W)).astype(np.float32)
    mt = ox.MapperTemplate.from_arrays(W, H, [[0, 0, W, H]], [m1], [m2], [np.full((H, W), 255, np.uint8)])
    for wide in (False, True):
        for pad in (0, 1, 2, 3):
            ok, rep = ox.debug_fastmapper_audit(mt, [(w, h)], wide=wide, pitch_pad=pad)
            assert ok, (wide, pad, json.dumps(rep))
            _check(rep, blocks_live=False)
