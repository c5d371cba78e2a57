"""octvr_rig_morph_controlpoints (MapperTemplate::morph_controlpoints, template_morph.cpp:69-237)
against the oracle restatement (oracle/octvr_oracle_morph.c) — parity unpinned (no reference fixture
covers the morph), bit-exact product vs oracle: the same triangles (cv::Subdiv2D), and the same
warped map1 / map2 / mask bits (cv::warpAffine on the GPU vs the oracle's literal per-triangle warp).
The oracle morphs the product's own pre-morph LUT, so the comparison isolates the morph."""
import json

import numpy as np
import pytest

import camera_rigs as R
import oracle_py as O

pytestmark = pytest.mark.gpu

W, H = 512, 256


def _luts(mt):
    return [mt.input(i)[:4] for i in range(len(mt))]


@pytest.mark.parametrize("with_equirect,per_pair,seed", [(False, 5, 0), (True, 5, 1), (True, 12, 2)])
def test_gpu_morph_vs_oracle(product_lib, tmp_path, with_equirect, per_pair, seed):
    ox = product_lib
    rig = R.morph_rig(with_equirect)
    mt = ox.MapperTemplate.from_json(json.dumps(rig), W, H)
    before = _luts(mt)
    cps = R.morph_points(before, per_pair=per_pair, seed=seed)
    want_rc, want, want_tris = O.morph_controlpoints(rig, before, W, H, cps)
    assert want_rc > 0
    assert mt.morph_controlpoints(cps) == want_rc
    changed = 0
    for i in range(len(mt)):
        st, dt = mt.triangles(i)
        np.testing.assert_array_equal(st, want_tris[i][0])
        np.testing.assert_array_equal(dt, want_tris[i][1])
        roi, g1, g2, gm, _ = mt.input(i)
        assert roi == tuple(want[i][0])
        assert np.array_equal(g1.view(np.uint32), want[i][1].view(np.uint32)), i
        assert np.array_equal(g2.view(np.uint32), want[i][2].view(np.uint32)), i
        assert np.array_equal(gm, want[i][3]), i
        changed += int((g1 != before[i][1]).sum())
    assert changed > 1000
    # the morphed LUT is what .dat persists (the triangles are not: template.cpp:206-256)
    p = tmp_path / "morph.dat"
    mt.dump(str(p))
    back = ox.MapperTemplate.load(str(p))
    for i in range(len(mt)):
        a, b = mt.input(i), back.input(i)
        assert a[0] == b[0] and all(np.array_equal(a[k], b[k]) for k in (1, 2, 3))
    # morphing a .dat rig: the reference has no camera models there (input_cams empty)
    with pytest.raises(ox.OctvrError) as e:
        back.morph_controlpoints(cps)
    assert e.value.code == ox.E_UNSUPPORTED


def test_gpu_morph_stitch_uses_morphed_lut(product_lib):
    """A morphed rig stitches like any LUT: product composite vs the oracle frame on the morphed maps."""
    ox = product_lib
    import torch
    rig = R.morph_rig()
    mt = ox.MapperTemplate.from_json(json.dumps(rig), W, H)
    cps = R.morph_points(_luts(mt), per_pair=6, seed=5)
    assert mt.morph_controlpoints(cps) > 0
    sizes = [(480, 320)] * 3
    frames = [O.rand_img(w, h * 3 // 2, 1, 40 + i).reshape(h * 3 // 2, w) for i, (w, h) in enumerate(sizes)]
    m = ox.Mapper(mt, sizes, blend=0, enable_gain=False)
    out = torch.empty((H * 3 // 2, W), dtype=torch.uint8, device="cuda")
    m.stitch([torch.from_numpy(f).cuda() for f in frames], out)
    torch.cuda.synchronize()
    luts = _luts(mt)
    want, _ = O.stitch_frame(frames, sizes, [l[0] for l in luts], [l[1] for l in luts], [l[2] for l in luts],
                          [l[3] for l in luts], W, H, enable_gain=False)
    np.testing.assert_array_equal(out.cpu().numpy(), want)


def test_gpu_morph_errors(product_lib):
    ox = product_lib
    rig = R.morph_rig()
    mt = ox.MapperTemplate.from_json(json.dumps(rig), W, H)
    cps = R.morph_points(_luts(mt), per_pair=2)
    for bad in ([[1, 0] + cps[0][2:]], [[0, 7] + cps[0][2:]], [[0, 1, 0.5]]):
        with pytest.raises(ox.OctvrError) as e:
            mt.morph_controlpoints(bad)
        assert e.value.code == ox.E_INVALID
    fish = {"output": rig["output"], "inputs": [
        {"type": "fisheye", "options": {"width": 640, "height": 480, "fx": 300.0, "fy": 300.0, "cx": 320.0,
                                        "cy": 240.0, "dist_coeffs": [0, 0, 0, 0]}}] + rig["inputs"][1:]}
    mf = ox.MapperTemplate.from_json(json.dumps(fish), W, H)
    with pytest.raises(ox.OctvrError) as e:
        mf.morph_controlpoints([[0, 1, 0.5, 0.5, 0.5, 0.5]])
    assert e.value.code == ox.E_UNSUPPORTED
    assert mt.morph_controlpoints([]) == 0  # nothing kept: every LUT unchanged


@pytest.mark.parametrize("blend", [0, 16, -8])
def test_gpu_stitch_out_of_range_maps(product_lib, blend):
    """Claimed pixels whose map leaves [0, 1) — what a morph leaves near the mask edges, and what a
    .dat from elsewhere may hold: cells straddling the image edge, wholly outside, NaN.  remap's rule
    (per-tap BORDER_CONSTANT 0, s16 cell) for the composite, the gain feed and the multi-band path."""
    ox = product_lib
    import torch
    rng = np.random.default_rng(11 + blend)
    Wo, Ho = 256, 128
    sizes = [(64, 48), (96, 64)]
    rois, m1s, m2s, mks = [], [], [], []
    for i, (w, h) in enumerate(sizes):
        roi = (0, 0, Wo, Ho) if i == 0 else (32, 16, 160, 96)
        m1 = rng.uniform(-0.08, 1.08, (roi[3], roi[2])).astype(np.float32)
        m2 = rng.uniform(-0.08, 1.08, (roi[3], roi[2])).astype(np.float32)
        m1[rng.random(m1.shape) < 0.01] = np.nan
        m2[rng.random(m2.shape) < 0.01] = -5.0
        # a morph-like seam: exactly -1 / 32 of a pixel left of the image, cells at sx = -1
        m1[::7, ::5] = np.float32(-0.5 / w)
        mk = np.where(rng.random(m1.shape) < 0.9, 255, 0).astype(np.uint8)
        rois.append(roi); m1s.append(m1); m2s.append(m2); mks.append(mk)
    mt = ox.MapperTemplate.from_arrays(Wo, Ho, rois, m1s, m2s, mks)
    frames = [O.rand_img(w, h * 3 // 2, 1, 70 + i).reshape(h * 3 // 2, w) for i, (w, h) in enumerate(sizes)]
    seams = None
    if blend:
        mt.create_masks()
        seams = [mt.input(i)[4] for i in range(len(sizes))]
    m = ox.Mapper(mt, sizes, blend=blend, enable_gain=True)
    out = torch.empty((Ho * 3 // 2, Wo), dtype=torch.uint8, device="cuda")
    m.stitch([torch.from_numpy(f).cuda() for f in frames], out)
    torch.cuda.synchronize()
    want, g_orc = O.stitch_frame(frames, sizes, rois, m1s, m2s, mks, Wo, Ho, enable_gain=True, blend=blend,
                                 seams=seams)
    np.testing.assert_array_equal(np.array(m.gains()), g_orc)
    np.testing.assert_array_equal(out.cpu().numpy(), want)
