"""GPU LUT build (lut_build_kernel, FP64, with the host recompute of the pixels its guard defers) for
every camera model against the oracle restatement (parity unpinned: no reference fixture exists for
these models).  Bit-exact, as the pinned rigs of test_gpu_parity.py."""
import json

import numpy as np
import pytest

import camera_rigs as R
import oracle_py as O

pytestmark = pytest.mark.gpu

ASPECT = {"normal": 1.5, "perspective": 1.25, "stupidoval": 2.0, "cubic": 1.5, "eqareanorthpole": 1.0,
          "eqareasouthpole": 1.0, "ocam_fisheye": 640 / 480,
          "fullframe_fisheye": 1.5}


def _same(g1, g2, gm, w1, w2, wm):
    return (np.array_equal(gm, wm) and np.array_equal(g1.view(np.int32), w1.view(np.int32)) and
            np.array_equal(g2.view(np.int32), w2.view(np.int32)))


def _compare(ox, rig, W, H, use_roi=False):
    text = json.dumps(rig)
    mt = ox.MapperTemplate.from_json(text, W, H, use_roi=use_roi)
    W, H = mt.out_size
    # the oracle gets the doubles the product parses (rapidjson's rules, json_lite.hpp)
    want = O.lut_build(O.json_loads_rj(text), W, H, use_roi=use_roi)[:len(rig["inputs"])]
    assert len(mt) == len(want)
    for i, (roi, w1, w2, wm) in enumerate(want):
        groi, g1, g2, gm, _ = mt.input(i)
        assert groi == tuple(roi)
        assert _same(g1, g2, gm, w1, w2, wm), (i, int((gm != wm).sum()), int((g1 != w1).sum()), int((g2 != w2).sum()))
        assert (wm > 0).any()
    return mt


@pytest.mark.parametrize("name", sorted(R.input_rigs()))
def test_gpu_input_camera_models_vs_oracle(product_lib, name):
    _compare(product_lib, R.input_rigs()[name], 512, 256)


@pytest.mark.parametrize("name", sorted(R.output_rigs()))
def test_gpu_output_camera_models_vs_oracle(product_lib, name):
    # out_h = 0: derived from the output camera's aspect ratio (template.cpp:32-38)
    mt = _compare(product_lib, R.output_rigs()[name], 384, 0)
    assert mt.out_size == (384, int(384 / ASPECT[name]))


def test_gpu_unsupported_camera_options_fail_loudly(product_lib):
    ox = product_lib
    rig = R.input_rigs()["normal"]
    bad = json.loads(json.dumps(rig))
    bad["inputs"][0]["options"]["exclude_masks"] = [{"type": "polygonal", "args": [0, 0, 10, 0, 10, 10]}]
    with pytest.raises(ox.OctvrError):  # masks need the camera's width / height (camera.cpp:73-74)
        ox.MapperTemplate.from_json(json.dumps(bad), 256, 128)
    bad = json.loads(json.dumps(R.input_rigs()["pinhole_nodist"]))
    bad["inputs"][0]["options"]["exclude_masks"] = [{"type": "polygonal", "args": [0, 0, 10, 0, 10, 10]}]
    with pytest.raises(ox.OctvrError):  # PinholeCamera never consults the masks (pinhole_cam.cpp:32-50)
        ox.MapperTemplate.from_json(json.dumps(bad), 256, 128)
    bad = json.loads(json.dumps(R.mask_rigs()["png"]))
    bad["inputs"][0]["options"]["include_masks"] = bad["inputs"][0]["options"].pop("exclude_masks")
    with pytest.raises(ox.OctvrError):  # PNG area without an exclude mask (camera.cpp:170)
        ox.MapperTemplate.from_json(json.dumps(bad), 256, 128)
    bad = json.loads(json.dumps(rig))
    bad["output"] = {"type": "pinhole", "options": {"width": 64, "height": 48, "fx": 1, "fy": 1, "cx": 0, "cy": 0}}
    with pytest.raises(ox.OctvrError):
        ox.MapperTemplate.from_json(json.dumps(bad), 256, 128)


@pytest.mark.parametrize("name", sorted(R.mask_rigs()))
@pytest.mark.parametrize("use_roi", [False, True])
def test_gpu_camera_masks_vs_oracle(product_lib, name, use_roi):
    """selection / exclude_masks / include_masks (polygons and PNG) and the include-mask visibility
    arbitration across inputs (camera.cpp:96-187, 212-294; template.cpp:86-116)."""
    _compare(product_lib, R.mask_rigs()[name], 512, 256, use_roi=use_roi)


def test_gpu_selection_equals_its_polygon(product_lib):
    """`selection` = exclude everything, then clear the rectangle polygon: the same LUT as an
    exclude_masks polygon ring around it (independent of the oracle)."""
    import copy
    ox = product_lib
    rig = R.input_rigs()["fullframe_selection"]
    alt = copy.deepcopy(rig)
    for cam in alt["inputs"]:
        o = cam["options"]
        l, r, t, b = o.pop("selection")
        w, h = o["width"], o["height"]
        o["exclude_masks"] = [{"type": "polygonal", "args": a} for a in (
            [0, 0, w - 1, 0, w - 1, t - 1, 0, t - 1] if t > 0 else None,
            [0, b, w - 1, b, w - 1, h - 1, 0, h - 1] if b < h else None,
            [0, 0, l - 1, 0, l - 1, h - 1, 0, h - 1] if l > 0 else None,
            [r, 0, w - 1, 0, w - 1, h - 1, r, h - 1] if r < w else None) if a]
    a = ox.MapperTemplate.from_json(json.dumps(rig), 512, 256, use_roi=False)
    b = ox.MapperTemplate.from_json(json.dumps(alt), 512, 256, use_roi=False)
    for i in range(len(a)):
        ia, ib = a.input(i), b.input(i)
        assert ia[0] == ib[0]
        for k in (1, 2, 3):
            assert np.array_equal(ia[k], ib[k])


@pytest.mark.parametrize("use_roi", [False, True])
def test_gpu_overlay_luts_vs_oracle(product_lib, tmp_path, use_roi):
    """The overlays' own LUTs (maps, mask, ROI) against the oracle's add_input(overlay = true)
    restatement (template.cpp:46-153), and their .dat round trip (template.cpp:248-255, 306-311)."""
    ox = product_lib
    rig = R.mask_rigs()["overlay_include"]
    text = json.dumps(rig)
    mt = ox.MapperTemplate.from_json(text, 512, 256, use_roi=use_roi)
    n_in = len(rig["inputs"])
    want = O.lut_build(O.json_loads_rj(text), 512, 256, use_roi=use_roi)[n_in:]
    assert mt.num_overlays == len(want) == len(rig["overlays"])
    for i, (roi, w1, w2, wm) in enumerate(want):
        groi, g1, g2, gm, gs = mt.overlay(i)
        assert groi == tuple(roi) and gs is None
        assert _same(g1, g2, gm, w1, w2, wm), i
        assert (wm > 0).any()
    p = tmp_path / "ov.dat"
    mt.dump(str(p))
    back = ox.MapperTemplate.load(str(p))
    assert back.num_overlays == mt.num_overlays
    for i in range(mt.num_overlays):
        a, b = mt.overlay(i), back.overlay(i)
        assert a[0] == b[0] and all(np.array_equal(a[k], b[k]) for k in (1, 2, 3))
    with pytest.raises(ox.OctvrError) as e:  # overlays reach the mapper: unsupported, with the real reason
        ox.Mapper(back, [(256, 256)] * len(back), blend=0, enable_gain=False)
    assert "overlay" in str(e.value)
