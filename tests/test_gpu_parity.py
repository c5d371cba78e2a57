"""GPU parity: the HIP path (through the C ABI) against the oracle and the reference goldens.

Bar: bit-exact everywhere — integer / byte outputs, and the FP64 LUT build too (the
device defers every pixel a last-ulp OCML / glibc difference could change to the host, which
recomputes it with glibc: tests/test_gpu_lut_exact.py).
"""
import json
import math
import os

import numpy as np
import pytest

import oracle_py as O

pytestmark = pytest.mark.gpu
RIGS = ["rigA", "rigB", "rigC", "rigD"]


@pytest.fixture(scope="module")
def ox(product_lib):
    import torch
    assert torch.cuda.is_available(), "gpu tests need a HIP device"
    return product_lib


def _cuda(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def _rig_text(name):
    with open(os.path.join(O.ROOT, "tests", "golden", name + ".json")) as f:
        return f.read()


@pytest.mark.parametrize("name", RIGS)
def test_gpu_lut_build_vs_reference(ox, name):
    rig, z = O.load_rig(name)
    W, H = (int(v) for v in z["out_size"])
    mt = ox.MapperTemplate.from_json(_rig_text(name), W, H, use_roi=(name != "rigD"))
    assert mt.out_size == (W, H) and len(mt) == len(z["rois"])
    for i in range(len(mt)):
        roi, m1, m2, mk, _ = mt.input(i)
        assert roi == tuple(z["rois"][i])
        g1, g2, gm = z[f"map1_{i}"], z[f"map2_{i}"], z[f"mask_{i}"]
        # the reference's own LUT, bit for bit (no mask flips, no ulp differences)
        assert np.array_equal(mk, gm), (i, int((mk != gm).sum()))
        assert np.array_equal(m1.view(np.int32), g1.view(np.int32)), (i, int((m1.view(np.int32) != g1.view(np.int32)).sum()))
        assert np.array_equal(m2.view(np.int32), g2.view(np.int32)), (i, int((m2.view(np.int32) != g2.view(np.int32)).sum()))


@pytest.mark.parametrize("name", RIGS)
def test_gpu_remap_vs_reference(ox, name):
    rig, z = O.load_rig(name)
    tag = ord(name[3])
    for i in range(len(z["rois"])):
        o = rig["inputs"][i]["options"]
        W, H = o["width"], o["height"]
        m1, m2 = _cuda(z[f"map1_{i}"]), _cuda(z[f"map2_{i}"])
        for cn, seed, key in ((1, 1000 * tag + i, "remap_c1"), (3, 5000 + 31 * tag + i, "remap_c3"),
                              (4, 9000 + 17 * tag, "remap_c4")):
            if f"{key}_{i}" not in z:
                continue
            img = _cuda(O.rand_img(W, H, cn, seed))
            out = ox.remap_u8(img, m1, m2, float(W), float(H)).cpu().numpy()
            assert np.array_equal(out.reshape(z[f"{key}_{i}"].shape), z[f"{key}_{i}"]), (i, key)


def test_gpu_remap_all_fractional_codes(ox):
    k = np.load(os.path.join(O.ROOT, "tests", "golden", "kats.npz"))
    m1, m2 = O.remap_kat_maps()
    out = ox.remap_u8(_cuda(k["remap_kat_src"]), _cuda(m1), _cuda(m2), 1.0, 1.0).cpu().numpy()
    assert np.array_equal(out, k["remap_kat_out"])


def test_gpu_remap_edges(ox):
    # NaN / huge / negative coordinates and partially-outside taps (BORDER_CONSTANT, imgwarp.cpp:3931-3970)
    src = O.rand_img(37, 23, 3, 99)
    m1 = np.array([[np.nan, 1e30, -1e30, -0.5, 36.5, 36.99, -1.0, 0.0, 17.03125]], np.float32)
    m2 = np.array([[3.0, 3.0, 3.0, 22.5, 22.5, -0.99, 5.0, 0.0, 11.96875]], np.float32)
    want = O.remap_u8(src, m1, m2, 1.0, 1.0)
    got = ox.remap_u8(_cuda(src), _cuda(m1), _cuda(m2), 1.0, 1.0).cpu().numpy()
    assert np.array_equal(got, want)


def _stitch_case(ox, name, frames_fn, gains, blend=0, info=None):
    rig, z = O.load_rig(name)
    W, H = (int(v) for v in z["out_size"])
    n = len(z["rois"])
    sizes = [(rig["inputs"][i]["options"]["width"], rig["inputs"][i]["options"]["height"]) for i in range(n)]
    frames = [frames_fn(w, h, 1000 * ord(name[3]) + i) for i, (w, h) in enumerate(sizes)]
    maps1 = [z[f"map1_{i}"] for i in range(n)]
    maps2 = [z[f"map2_{i}"] for i in range(n)]
    masks = [z[f"mask_{i}"] for i in range(n)]
    seams = [z[f"seam_{i}"] for i in range(n)]
    mt = ox.MapperTemplate.from_arrays(W, H, z["rois"].tolist(), maps1, maps2, masks, seams)
    m = ox.Mapper(mt, sizes, blend=blend, enable_gain=True)
    if info is not None:
        info.append(m.info())
    import torch
    out = torch.zeros((H * 3 // 2, W), dtype=torch.uint8, device="cuda")
    m.stitch([_cuda(f) for f in frames], out, gains=gains)
    torch.cuda.synchronize()
    g_gpu = m.gains()
    want, g_orc = O.stitch_frame(frames, sizes, z["rois"].tolist(), maps1, maps2, masks, W, H, enable_gain=True,
                                 gains=gains, blend=blend, seams=seams, threads=8)
    return out.cpu().numpy(), want, np.array(g_gpu), g_orc


@pytest.mark.parametrize("name", RIGS)
def test_gpu_stitch_fixed_gains_bit_exact(ox, name):
    n = len(O.load_rig(name)[1]["rois"])
    gains = [1.0 + 0.013 * k * (-1) ** k for k in range(n)]
    got, want, g_gpu, _ = _stitch_case(ox, name, lambda w, h, s: O.rand_img(w, h * 3 // 2, 1, s), gains)
    if n > 1:
        np.testing.assert_array_equal(g_gpu, np.array(gains))
    assert np.array_equal(got, want)


@pytest.mark.parametrize("name", RIGS)
def test_gpu_stitch_estimated_gains(ox, name):
    from octvr_amd import synthetic
    got, want, g_gpu, g_orc = _stitch_case(ox, name, synthetic.smooth_yuv_frame, None)
    # the pair sums are exact (u64 fixed point on the GPU, exact f64 in the oracle): gains bit-exact
    np.testing.assert_array_equal(g_gpu, g_orc)
    assert np.array_equal(got, want)


def _ring_rig(n, in_w=320, in_h=240):
    from octvr_amd import synthetic
    yaws = [2 * math.pi * k / n for k in range(n)]
    pitches = [0.35 * (-1) ** k for k in range(n)]
    return synthetic.fisheye_rig(in_w, in_h, yaws, pitches)


@pytest.mark.parametrize("n", [4, 7, 9, 12, 16])
def test_gpu_ring_estimated_gains_bit_exact(ox, n):
    """n cameras in a ring: the register LU (n <= 8) and the workgroup LU (9..16) of the fused feed,
    two frames in a row (the feed's totals and tickets must reset), gains and output vs the oracle."""
    import torch
    from octvr_amd import synthetic
    rig = _ring_rig(n)
    W, H = 512, 256
    mt = ox.MapperTemplate.from_json(json.dumps(rig), W, H)
    sizes = [(320, 240)] * n
    rois, maps1, maps2, masks = [], [], [], []
    for i in range(n):
        roi, m1, m2, mk, _ = mt.input(i)
        rois.append(roi); maps1.append(m1); maps2.append(m2); masks.append(mk)
    m = ox.Mapper(mt, sizes, blend=0, enable_gain=True)
    out = torch.zeros((H * 3 // 2, W), dtype=torch.uint8, device="cuda")
    for frame_no in range(2):
        frames = [synthetic.smooth_yuv_frame(w, h, 100 * n + 10 * frame_no + i) for i, (w, h) in enumerate(sizes)]
        m.stitch([_cuda(f) for f in frames], out)
        torch.cuda.synchronize()
        g = np.array(m.gains())
        want, g_orc = O.stitch_frame(frames, sizes, rois, maps1, maps2, masks, W, H, enable_gain=True, gains=None)
        np.testing.assert_array_equal(g, np.array(g_orc))
        assert not np.all(g == 1.0)
        assert np.array_equal(out.cpu().numpy(), want), frame_no


def test_gpu_stitch_is_deterministic_and_stream_ordered(ox):
    import torch
    name = "rigB"
    rig, z = O.load_rig(name)
    n = len(z["rois"])
    W, H = (int(v) for v in z["out_size"])
    mt = ox.MapperTemplate.from_arrays(W, H, z["rois"].tolist(), [z[f"map1_{i}"] for i in range(n)],
                                       [z[f"map2_{i}"] for i in range(n)], [z[f"mask_{i}"] for i in range(n)])
    m = ox.Mapper(mt, [(192, 108)] * n)
    frames = [_cuda(O.rand_img(192, 162, 1, 7 + i)) for i in range(n)]
    s = torch.cuda.Stream()
    outs = []
    for _ in range(3):
        o = torch.empty((H * 3 // 2, W), dtype=torch.uint8, device="cuda")
        with torch.cuda.stream(s):
            m.stitch(frames, o, stream=s)
        outs.append(o)
    s.synchronize()
    assert all(torch.equal(outs[0], o) for o in outs[1:])


@pytest.mark.parametrize("k,blend,n", [(2, 0, 6), (3, 0, 6), (2, 0, 3), (2, 0, 12), (2, 16, 6), (3, -10, 6),
                                         (4, 0, 6), (4, 16, 6)])
def test_gpu_frames_in_flight_vs_oracle(ox, k, blend, n):
    """octvr_mapper_set_frames_in_flight(k): 2k frames with their own inputs and outputs issued
    round-robin on k streams (no host sync in between) -> every output and the last frame's gains
    equal the oracle's for that frame, as if stitched one after another (no-blend composite,
    multi-band and feather: each slot has its own pyramids).  With frames in flight the mapper uses
    the lean gain feed (closed forms for n <= 3, the workgroup LU above)."""
    import torch
    from octvr_amd import synthetic
    rig = _ring_rig(n)
    W, H = 512, 256
    mt = ox.MapperTemplate.from_json(json.dumps(rig), W, H)
    if blend:
        mt.create_masks(0)
    sizes = [(320, 240)] * n
    rois, maps1, maps2, masks, seams = [], [], [], [], []
    for i in range(n):
        roi, m1, m2, mk, sm = mt.input(i)
        rois.append(roi); maps1.append(m1); maps2.append(m2); masks.append(mk); seams.append(sm)
    m = ox.Mapper(mt, sizes, blend=blend, enable_gain=True)
    m.set_frames_in_flight(k)
    streams = [torch.cuda.Stream() for _ in range(k)]
    frames = [[synthetic.smooth_yuv_frame(w, h, 500 + 10 * f + i) for i, (w, h) in enumerate(sizes)]
              for f in range(2 * k)]
    dev_frames = [[_cuda(x) for x in fr] for fr in frames]
    torch.cuda.synchronize()
    outs = [torch.zeros((H * 3 // 2, W), dtype=torch.uint8, device="cuda") for _ in range(2 * k)]
    for f in range(2 * k):
        m.stitch(dev_frames[f], outs[f], stream=streams[f % k])
    g_last = np.array(m.gains())
    torch.cuda.synchronize()
    for f in range(2 * k):
        want, g_orc = O.stitch_frame(frames[f], sizes, rois, maps1, maps2, masks, W, H, enable_gain=True, gains=None,
                                     blend=blend, seams=seams if blend else None, threads=8)
        assert np.array_equal(outs[f].cpu().numpy(), want), f
        if f == 2 * k - 1:
            np.testing.assert_array_equal(g_last, np.array(g_orc))
    # back to one slot: the next stitch on a new stream is ordered after the last one again
    m.set_frames_in_flight(1)
    np.testing.assert_array_equal(np.array(m.gains()), g_last)
    o = torch.zeros_like(outs[0])
    m.stitch(dev_frames[0], o, stream=torch.cuda.Stream())
    torch.cuda.synchronize()
    assert torch.equal(o, outs[0])


def test_gpu_frames_in_flight_rejected_for_scaled_output(ox):
    rig, z = O.load_rig("rigA")
    seams = [z["seam_0"], z["seam_1"]]
    mt = ox.MapperTemplate.from_arrays(512, 256, z["rois"].tolist(), [z["map1_0"], z["map1_1"]],
                                       [z["map2_0"], z["map2_1"]], [z["mask_0"], z["mask_1"]], seams)
    for blend in (0, 16):
        m = ox.Mapper(mt, [(256, 144)] * 2, blend=blend, scale_output=(256, 128))
        with pytest.raises(ox.OctvrError) as e:
            m.set_frames_in_flight(2)
        assert e.value.code == -4
        m.set_frames_in_flight(1)
    m0 = ox.Mapper(mt, [(256, 144)] * 2, blend=0)
    for bad in (0, 17):
        with pytest.raises(ox.OctvrError):
            m0.set_frames_in_flight(bad)


def test_gpu_mapper_argument_errors(ox):
    rig, z = O.load_rig("rigA")
    mt = ox.MapperTemplate.from_arrays(512, 256, z["rois"].tolist(), [z["map1_0"], z["map1_1"]],
                                       [z["map2_0"], z["map2_1"]], [z["mask_0"], z["mask_1"]])
    with pytest.raises(ox.OctvrError):
        ox.Mapper(mt, [(256, 144)])  # wrong input count
    with pytest.raises(ox.OctvrError) as e:
        ox.Mapper(mt, [(256, 144)] * 2, blend=16)  # multi-band needs seam masks
    assert e.value.code == -1 and "seam" in str(e.value)
    seams = [np.full(z["mask_0"].shape, 255, np.uint8)] * 2
    mt2 = ox.MapperTemplate.from_arrays(512, 256, z["rois"].tolist(), [z["map1_0"], z["map1_1"]],
                                        [z["map2_0"], z["map2_1"]], [z["mask_0"], z["mask_1"]], seams)
    with pytest.raises(ox.OctvrError) as e:
        ox.Mapper(mt2, [(256, 144)] * 2, blend=2)  # ceil(log2 2) - 1 = 0 bands (blenders.cpp:594)
    assert e.value.code == -1
    with pytest.raises(ox.OctvrError):
        ox.Mapper(mt, [(255, 144)] * 2)  # odd size: not YUV420


def test_gpu_single_input_disables_gain(ox):
    # mapper.cpp:78-82
    import torch
    rig, z = O.load_rig("rigD")
    mt = ox.MapperTemplate.from_arrays(256, 128, [z["rois"][0].tolist()], [z["map1_0"]], [z["map2_0"]], [z["mask_0"]])
    m = ox.Mapper(mt, [(320, 240)], enable_gain=True)
    f = O.rand_img(320, 360, 1, 5)
    out = torch.zeros((192, 256), dtype=torch.uint8, device="cuda")
    m.stitch([_cuda(f)], out)
    want, _ = O.stitch_frame([f], [(320, 240)], [z["rois"][0].tolist()], [z["map1_0"]], [z["map2_0"]], [z["mask_0"]],
                             256, 128, enable_gain=True)
    assert m.gains() == [1.0]
    assert np.array_equal(out.cpu().numpy(), want)


# ------------------------------------------------------------------------------------------------
# Full benchmark size (config C2: 6 x 3840x2160 -> 7680x3840): LUT rows vs the oracle, and the
# stitched output on row bands (poles, equator, seams) vs the oracle fed the GPU's gains.
# ------------------------------------------------------------------------------------------------
@pytest.fixture(scope="module")
def c2(ox):
    from octvr_amd import synthetic
    rig, W, H, sizes = synthetic.CONFIGS["C2"]()
    mt = ox.MapperTemplate.from_json(json.dumps(rig), W, H)
    return rig, W, H, sizes, mt


def test_gpu_c2_lut_rows_vs_oracle(ox, c2):
    rig, W, H, sizes, mt = c2
    rig = O.json_loads_rj(json.dumps(rig))
    for i in (0, 3):
        roi, m1, m2, mk, _ = mt.input(i)
        for y0 in (0, 1237, 1919, 3830):
            r1, r2, rk = O.lut_rows(rig["output"], rig["inputs"][i], W, H, y0, y0 + 8)
            sl = slice(y0 - roi[1], y0 - roi[1] + 8)
            g1 = np.zeros_like(r1) - 1
            g1[:, roi[0]:roi[0] + roi[2]] = m1[sl]
            g2 = np.zeros_like(r2) - 1
            g2[:, roi[0]:roi[0] + roi[2]] = m2[sl]
            assert np.array_equal(g1.view(np.int32), r1.view(np.int32)), (i, y0)
            assert np.array_equal(g2.view(np.int32), r2.view(np.int32)), (i, y0)


def test_gpu_c2_stitch_row_bands_vs_oracle(ox, c2):
    import torch
    from octvr_amd import synthetic
    rig, W, H, sizes, mt = c2
    n = len(sizes)
    m = ox.Mapper(mt, sizes, blend=0, enable_gain=True)
    frames = [synthetic.smooth_yuv_frame(w, h, 2000 + i) for i, (w, h) in enumerate(sizes)]
    out = torch.zeros((H * 3 // 2, W), dtype=torch.uint8, device="cuda")
    m.stitch([_cuda(f) for f in frames], out)
    torch.cuda.synchronize()
    g = m.gains()
    assert all(0.5 < x < 2.0 for x in g)
    got = out.cpu().numpy()
    rois, maps1, maps2, masks = [], [], [], []
    for i in range(n):
        roi, m1, m2, mk, _ = mt.input(i)
        rois.append(roi); maps1.append(m1); maps2.append(m2); masks.append(mk)
    for band in ((0, 16), (1904, 1936), (3824, 3840)):
        want, _ = O.stitch_frame(frames, sizes, rois, maps1, maps2, masks, W, H, enable_gain=True, gains=g,
                                 threads=8, row_band=band)
        y0, y1 = band
        assert np.array_equal(got[y0:y1], want[y0:y1]), band
        assert np.array_equal(got[H + y0 // 2:H + y1 // 2], want[H + y0 // 2:H + y1 // 2]), band


def test_gpu_saturating_conversion_kat(ox):
    # saturate_cast<uchar>(float) = round half to even, then clamp to [0, 255]; NaN -> 0
    vals = [-1e9, -256.0, -1.0, -0.5, -0.49, -0.0, 0.0, 0.25, 0.5, 0.5000001, 1.5, 2.5, 3.49999, 3.5, 126.5, 127.5,
            254.4, 254.5, 254.5001, 255.0, 255.49, 255.5, 256.0, 1e9, float("inf"), float("-inf"), float("nan")]
    want = np.array([0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 2, 2, 3, 4, 126, 128, 254, 254, 255, 255, 255, 255, 255, 255, 255,
                     0, 0], np.uint8)
    rng = np.random.default_rng(5)
    extra = rng.uniform(-10, 270, 100000).astype(np.float32)
    extra = np.concatenate([extra, (np.arange(-20, 560) / 2).astype(np.float32)])
    ref = np.clip(np.rint(extra), 0, 255).astype(np.uint8)
    for method in (0, 1):
        got = ox.selftest_sat_u8(vals, method).cpu().numpy()
        assert np.array_equal(got, want), (method, got)
        got2 = ox.selftest_sat_u8(torch_tensor(extra), method).cpu().numpy()
        assert np.array_equal(got2, ref), method


def torch_tensor(a):
    import torch
    return torch.from_numpy(a)


# ---- seam masks (MapperTemplate::create_masks) ----------------------------------
@pytest.mark.parametrize("name", RIGS)
def test_gpu_create_masks_vs_reference(ox, name, tmp_path):
    import hashlib
    rig, z = O.load_rig(name)
    n = len(z["rois"])
    W, H = (int(v) for v in z["out_size"])
    mt = ox.MapperTemplate.from_arrays(W, H, z["rois"].tolist(), [z[f"map1_{i}"] for i in range(n)],
                                       [z[f"map2_{i}"] for i in range(n)], [z[f"mask_{i}"] for i in range(n)])
    # dump without seams creates them (template.cpp:209-210): byte-identical to the reference's file
    p = tmp_path / "rig.dat"
    mt.dump(str(p))
    man = json.load(open(os.path.join(O.ROOT, "tests", "golden", "manifest.json")))["rigs"][name]
    assert hashlib.sha256(p.read_bytes()).hexdigest() == man["dat_sha256"]
    for i in range(n):
        assert np.array_equal(mt.input(i)[4], z[f"seam_{i}"]), i


@pytest.mark.parametrize("out_w", [1920, 2048])
def test_gpu_create_masks_scaled_vs_oracle(ox, out_w):
    # out_w > 960: masks go through the 1/2 area path (1920) or the generic linear path (2048) both
    # ways; oracle = CPU restatement pinned by the resize / distance KATs and the rig seams
    rig, _ = O.load_rig("rigB")
    for c in rig["inputs"]:
        c["options"]["width"], c["options"]["height"] = 640, 360
        c["options"]["crop"]["rect"] = [140, 500, 0, 360]
    H = out_w // 2
    res = O.lut_build(rig, out_w, H, use_roi=True)
    rois = [list(r[0]) for r in res]
    masks = [r[3] for r in res]
    mt = ox.MapperTemplate.from_arrays(out_w, H, rois, [r[1] for r in res], [r[2] for r in res], masks)
    mt.create_masks(0)
    want = O.create_masks(rois, masks, out_w)
    for i in range(len(res)):
        got = mt.input(i)[4]
        assert np.array_equal(got, want[i]), (i, int((got != want[i]).sum()))


# ---- multi-band blend (MultiBandGPUBlender): bit-exact against the oracle -----------
@pytest.mark.parametrize("blend", [4, 16, 128, -5, -20])
@pytest.mark.parametrize("name", RIGS)
def test_gpu_multiband_bit_exact(ox, name, blend):
    # blend > 0: MultiBandGPUBlender; blend < 0: FeatherGPUBlender
    from octvr_amd import synthetic
    n = len(O.load_rig(name)[1]["rois"])
    gains = [1.0 + 0.011 * k * (-1) ** k for k in range(n)]
    for frames_fn, g in ((lambda w, h, s: O.rand_img(w, h * 3 // 2, 1, s), gains), (synthetic.smooth_yuv_frame, None)):
        got, want, g_gpu, g_orc = _stitch_case(ox, name, frames_fn, g, blend=blend)
        np.testing.assert_array_equal(g_gpu, g_orc)
        d = got != want
        assert not d.any(), (int(d.sum()), np.argwhere(d)[:5].tolist())


def test_gpu_multiband_entry_widths(ox, monkeypatch):
    """The multi-band remap's 24-bit entries (tiled_entry24, LUTs without "no gain" pixels) and the 32-bit
    layout (OCTVR_ENTRY32=1, and every LUT with such pixels) give the same bit-exact outputs; both occur."""
    from octvr_amd import synthetic
    seen = set()
    for e32 in (False, True):
        if e32:
            monkeypatch.setenv("OCTVR_ENTRY32", "1")
        for name in RIGS:
            info = []
            got, want, _, _ = _stitch_case(ox, name, synthetic.smooth_yuv_frame, None, blend=4, info=info)
            bits = info[0]["remap_entry_bits"]
            assert bits == 32 or not e32
            seen.add(bits)
            d = got != want
            assert not d.any(), (name, bits, int(d.sum()), np.argwhere(d)[:5].tolist())
    assert seen == {24, 32}, seen


def test_gpu_multiband_deep_tiles(ox):
    """Deep tiles (R = G at their level, no pyrUp taps; multiband_host.cpp) occur on the golden rigs and
    the output stays bit-exact with them."""
    from octvr_amd import synthetic
    deep = {}
    for name in RIGS:
        for blend in (4, 16):
            info = []
            got, want, _, _ = _stitch_case(ox, name, synthetic.smooth_yuv_frame, None, blend=blend, info=info)
            lv = info[0]["level_tiles"]
            deep[(name, blend)] = [t.get("deep_subtiles", 0) for t in lv]
            assert all(t["deep_subtiles"] <= t["owned_subtiles"] for t in lv)
            d = got != want
            assert not d.any(), (name, blend, int(d.sum()), np.argwhere(d)[:5].tolist())
    print(deep)
    assert sum(v[0] for v in deep.values()) > 0, deep


@pytest.mark.parametrize("k", [1, 2])
def test_gpu_gain_feed_tight_pitch_last_chroma_cell(ox, k):
    """the gain feed reads 8-byte row segments through a frame-sized buffer resource whose
    range check drops whole dwords; with a tight pitch (pitch == w) and w/2 not a multiple of 4 the
    last V row ends mid-dword.  Width 100 (w/2 = 50), 4 cameras whose samples reach the bottom-right
    chroma cell: gains (full feed, k = 1; lean feed, k = 2) and output bit-exact vs the oracle."""
    import torch
    from octvr_amd import synthetic
    n, w, h = 4, 100, 76
    rig = synthetic.fisheye_rig(w, h, [2 * math.pi * i / n for i in range(n)], [0.2 * (-1) ** i for i in range(n)],
                                circular=False)
    W, H = 256, 128
    mt = ox.MapperTemplate.from_json(json.dumps(rig), W, H)
    rois, maps1, maps2, masks = [], [], [], []
    for i in range(n):
        roi, m1, m2, mk, _ = mt.input(i)
        rois.append(roi); maps1.append(m1); maps2.append(m2); masks.append(mk)
    # at this output size the working scale is 1: every pixel of a pairwise intersection is a sample;
    # make sure some sample's taps touch the last chroma row's last cell (x >= w - 2, y >= h - 2)
    hit = False
    for i in range(n):
        for j in range(n):
            if i == j:
                continue
            (xi, yi, wi, hi), (xj, yj, wj, hj) = rois[i], rois[j]
            x0, y0, x1, y1 = max(xi, xj), max(yi, yj), min(xi + wi, xj + wj), min(yi + hi, yj + hj)
            if x0 >= x1 or y0 >= y1:
                continue
            both = (masks[i][y0 - yi:y1 - yi, x0 - xi:x1 - xi] > 0) & (masks[j][y0 - yj:y1 - yj, x0 - xj:x1 - xj] > 0)
            mx = maps1[i][y0 - yi:y1 - yi, x0 - xi:x1 - xi] * w
            my = maps2[i][y0 - yi:y1 - yi, x0 - xi:x1 - xi] * h
            hit |= bool((both & (mx >= w - 2) & (my >= h - 2)).any())
    assert hit
    m = ox.Mapper(mt, [(w, h)] * n, blend=0, enable_gain=True)
    m.set_frames_in_flight(k)
    frames = [synthetic.smooth_yuv_frame(w, h, 40 + i) for i in range(n)]
    for f in frames:  # a distinctive last V byte: a zeroed dword would change the norm
        f[-1, -1] = 250
        f[-1, w // 2 - 1] = 3
    out = torch.zeros((H * 3 // 2, W), dtype=torch.uint8, device="cuda")
    dev = [torch.from_numpy(np.ascontiguousarray(f)).cuda() for f in frames]
    assert all(t.stride(0) == w for t in dev)
    m.stitch(dev, out)
    torch.cuda.synchronize()
    want, g_orc = O.stitch_frame(frames, [(w, h)] * n, rois, maps1, maps2, masks, W, H, enable_gain=True, gains=None)
    np.testing.assert_array_equal(np.array(m.gains()), np.array(g_orc))
    assert np.array_equal(out.cpu().numpy(), want)


def test_gpu_kernel_busy_log(ox):
    """octvr_mapper_kernel_busy (the bench's roofline timing): busy <= span, one logged launch per
    timed stitch, and the log resets."""
    import torch
    from octvr_amd import synthetic
    rig = _ring_rig(6)
    mt = ox.MapperTemplate.from_json(json.dumps(rig), 512, 256)
    m = ox.Mapper(mt, [(320, 240)] * 6, blend=0, enable_gain=True)
    m.set_frames_in_flight(2)
    frames = [_cuda(synthetic.yuv_frame(320, 240, 9 + i)) for i in range(6)]
    outs = [torch.zeros((384, 512), dtype=torch.uint8, device="cuda") for _ in range(2)]
    streams = [torch.cuda.Stream() for _ in range(2)]
    assert m.kernel_busy()[2] == 0  # empty log
    m.set_timing(1)
    for f in range(6):
        m.stitch(frames, outs[f % 2], stream=streams[f % 2])
    span, busy, launches = m.kernel_busy()
    assert launches == 6 and 0 < busy <= span + 1e-9
    assert m.kernel_busy() == (0.0, 0.0, 0)  # reset
    m.set_timing(2)  # every 2nd stitch
    for f in range(6):
        m.stitch(frames, outs[f % 2], stream=streams[f % 2])
    assert m.kernel_busy()[2] == 3
    # the launches themselves (octvr_mapper_kernel_intervals), relative to the first one's start, in issue
    # order; the event pairs come from the pool set_timing fills (1,024), reused across logs
    m.set_timing(1)
    for f in range(4):
        m.stitch(frames, outs[f % 2], stream=streams[f % 2])
    iv = m.kernel_intervals()
    assert len(iv) == 4 and iv[0][0] == 0.0 and all(0 <= a <= b for a, b in iv)
    sp, bu = ox.interval_union([a for a, _ in iv], [b for _, b in iv])
    assert 0 < bu <= sp + 1e-9
    assert m.kernel_intervals() == []
    for f in range(1100):  # more timed stitches than the pool holds: further pairs are created as needed
        m.stitch(frames, outs[f % 2], stream=streams[f % 2])
    assert m.kernel_busy()[2] == 1100
    m.set_timing(0)
