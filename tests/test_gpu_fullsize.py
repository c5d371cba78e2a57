"""The benchmark configurations at their full BASELINE size, on the code path bench.py times
(BASELINE.json configs[1..3]): the rig built by the GPU LUT build, three frames in
flight on three streams (the lean gain feed), gains estimated per frame — every output byte and the
gains against the oracle, which builds its own LUT (threads) and stitches each frame independently.
  C1: 2 x 1920x1080 fullframe_fisheye (yaw 0 / pi) -> 4096x2048, no blend (the reference's CPU plumbing case)
  C2: 6 x 3840x2160 fullframe_fisheye -> 7680x3840, no blend (copy chain)
  C3: C2 + multi-band blend = 16 (3 bands), seams from create_masks
  C4: 12 x 3840x2160 (pitch +-35 deg, hfov 150 deg) -> 15360x7680, no blend
Reference: mapper.cpp:193-312, exposure_compensate.cpp:223-297, blenders.cpp:670-735, template.cpp:46-204."""
import json

import numpy as np
import pytest

import oracle_py as O

pytestmark = pytest.mark.gpu
THREADS = 16


def _frames(sizes, seed):
    """Frame set `seed`: one smooth image per camera (gain-estimation realistic), later sets derived
    by cheap byte transforms (distinct content, fast to make at 4K)."""
    from octvr_amd import synthetic
    base = [synthetic.smooth_yuv_frame(w, h, 7000 + i) for i, (w, h) in enumerate(sizes)]
    out = []
    for f in base:
        g = f.copy()
        if seed:
            h = f.shape[0] * 2 // 3
            g[:h] = (f[:h].astype(np.int32) * (9 + seed) // 10 + 7 * seed).clip(0, 255).astype(np.uint8)
            g[h:] = np.roll(f[h:], 3 * seed, axis=1)
        out.append(g)
    return out


_LUTS = {}


def _oracle_lut(cfg):
    """(rig, W, H, sizes, text, rois, maps1, maps2, masks) of a BASELINE config, the LUT built by the
    oracle (cached per module: the 8K builds take seconds each)."""
    from octvr_amd import synthetic
    rig, W, H, sizes = synthetic.CONFIGS[cfg]()
    text = json.dumps(rig)
    key = (text, W, H)  # C3 shares C2's rig
    if key not in _LUTS:
        want = O.lut_build(O.json_loads_rj(text), W, H, threads=THREADS)
        _LUTS[key] = ([list(r[0]) for r in want], [r[1] for r in want], [r[2] for r in want], [r[3] for r in want])
    return (rig, W, H, sizes, text) + tuple(_LUTS[key])


def _bench_frames(sizes, j):
    """Frame set j as bench.py makes it (splitmix64 frames, the later sets derived from set 0)."""
    from octvr_amd import synthetic
    base = [synthetic.yuv_frame(w, h, 1000 + i) for i, (w, h) in enumerate(sizes)]
    return base if j == 0 else [synthetic.derived_frame(f, 1000 + 100 * j + i) for i, f in enumerate(base)]


@pytest.mark.parametrize("cfg", ["C1", "C2", "C3", "C4"])
def test_gpu_fullsize_bit_exact(product_lib, cfg):
    import torch
    from octvr_amd import synthetic
    ox = product_lib
    rig, W, H, sizes, text, rois, maps1, maps2, masks = _oracle_lut(cfg)
    blend = synthetic.BLEND[cfg]
    n = len(sizes)
    # the LUT: GPU build (with its host recompute of deferred pixels) == oracle, bit for bit
    mt = ox.MapperTemplate.from_json(text, W, H)
    for i in range(n):
        roi, g1, g2, gm, _ = mt.input(i)
        assert roi == tuple(rois[i]), (i, roi, rois[i])
        assert np.array_equal(gm, masks[i]), (i, int((gm != masks[i]).sum()))
        assert np.array_equal(g1.view(np.int32), maps1[i].view(np.int32)), i
        assert np.array_equal(g2.view(np.int32), maps2[i].view(np.int32)), i
    del g1, g2, gm
    seams = None
    if blend:
        mt.create_masks(0)
        seams = O.create_masks(rois, masks, W)
        for i in range(n):
            assert np.array_equal(mt.input(i)[4], seams[i]), i
    # three frames in flight on three streams, gains estimated (the bench's loop)
    m = ox.Mapper(mt, sizes, blend=blend, enable_gain=True)
    k = 3
    m.set_frames_in_flight(k)
    sets = [_frames(sizes, s) for s in range(k)]
    dev = [[torch.from_numpy(f).cuda() for f in fs] for fs in sets]
    outs = [torch.zeros((H * 3 // 2, W), dtype=torch.uint8, device="cuda") for _ in range(k)]
    streams = [torch.cuda.Stream() for _ in range(k)]
    torch.cuda.synchronize()
    for f in range(k):
        m.stitch(dev[f], outs[f], stream=streams[f])
    g_last = np.array(m.gains())
    torch.cuda.synchronize()
    exps = []
    for f in range(k):
        exp, g_orc = O.stitch_frame(sets[f], sizes, rois, maps1, maps2, masks, W, H, enable_gain=True, gains=None,
                                    blend=blend, seams=seams, threads=THREADS)
        exps.append(exp)
        got = outs[f].cpu().numpy()
        d = got != exp
        assert not d.any(), (cfg, f, int(d.sum()), np.argwhere(d)[:4].tolist())
        assert all(0.5 < x < 2.0 for x in g_orc) and not np.all(np.array(g_orc) == 1.0)
        if f == k - 1:
            np.testing.assert_array_equal(g_last, np.array(g_orc))
    # the AsyncMultiMapper from host planes (async.cpp): only each mapper's source footprint is uploaded,
    # the rest of the device frames hold a fixed pattern — every byte still equal to the oracle's frame
    if cfg in ("C1", "C2", "C3"):
        del dev
        am = ox.AsyncMultiMapper([mt], sizes, (W, H), [blend], [0], [(0.0, 0.0, 1.0, 1.0)])
        aouts = []
        for f in range(k):
            o = (np.zeros((H, W), np.uint8), np.zeros((H // 2, W // 2), np.uint8), np.zeros((H // 2, W // 2), np.uint8))
            am.push([(x[:h], x[h:, :w // 2], x[h:, w // 2:]) for x, (w, h) in zip(sets[f], sizes)], o)
            aouts.append(o)
        for f in range(k):
            am.pop()
            exp = exps[f]
            assert np.array_equal(aouts[f][0], exp[:H]), (cfg, f, "Y")
            assert np.array_equal(aouts[f][1], exp[H:, :W // 2]) and np.array_equal(aouts[f][2], exp[H:, W // 2:]), (cfg, f)
        am.close()
        dev = [[torch.from_numpy(f).cuda() for f in fs] for fs in sets]
    # and each frame's gains, stitched one at a time on one stream
    m.set_frames_in_flight(1)
    for f in range(k):
        m.stitch(dev[f], outs[0])
        _, g_orc = O.stitch_frame(sets[f], sizes, rois, maps1, maps2, masks, W, H, enable_gain=True, gains=None,
                                  blend=0, threads=THREADS, row_band=(0, 2))
        np.testing.assert_array_equal(np.array(m.gains()), np.array(g_orc))


@pytest.mark.parametrize("scale", [None, (3840, 1920)])
def test_gpu_c3_deep_tiles_equal_pyrup_path(product_lib, monkeypatch, scale):
    """C3 at full size, on noise frames (every level's Laplacian non-zero), three builds of the same
    mapper, bit-identical: the default (deep tiles' R = G, the deep level-0 tiles' result written by the
    remap itself: kItemResult / owned 4, multiband_host.cpp), the result left to the level-0 blend
    (OCTVR_MB_NO_REMAP_RESULT), and no deep shortcut at all (OCTVR_MB_NO_DEEP: every owned tile through
    both pyrUps).  With a scaled output the remap writes the RGBA result image instead of YUV420P."""
    import torch
    from octvr_amd import synthetic
    ox = product_lib
    rig, W, H, sizes = synthetic.CONFIGS["C3"]()
    mt = ox.MapperTemplate.from_json(json.dumps(rig), W, H)
    mt.create_masks(0)
    rng = np.random.default_rng(11)
    frames = [torch.from_numpy(rng.integers(0, 256, size=(h * 3 // 2, w), dtype=np.uint8)).cuda() for w, h in sizes]
    OW, OH = scale or (W, H)
    outs, deep, res = [], [], []
    for knob in (None, "OCTVR_MB_NO_REMAP_RESULT", "OCTVR_MB_NO_DEEP"):
        if knob:
            monkeypatch.setenv(knob, "1")
        m = ox.Mapper(mt, sizes, blend=synthetic.BLEND["C3"], enable_gain=True, scale_output=scale)
        info = m.info()
        deep.append([t["deep_subtiles"] for t in info["level_tiles"]])
        res.append(info["remap_result_subtiles"])
        out = torch.zeros((OH * 3 // 2, OW), dtype=torch.uint8, device="cuda")
        m.stitch(frames, out, gains=[1.0] * len(sizes))
        torch.cuda.synchronize()
        outs.append(out.cpu().numpy())
        del m
        if knob:
            monkeypatch.delenv(knob)
    print(deep, res)
    assert deep[0][0] > 0 and res[0] > 0.7 * 4 * 28800  # C3: 28,800 level-0 tiles of 4 sub-tiles each
    assert res[1] == 0 and deep[1][0] == deep[0][0]
    assert sum(deep[2]) == 0 and res[2] == 0
    for k in (1, 2):
        d = outs[0] != outs[k]
        assert not d.any(), (k, int(d.sum()), np.argwhere(d)[:4].tolist())


_F2_ORACLE = {}


def _nv12(yuv420p):
    """bench.py nv12_of: the same frame with interleaved U, V chroma rows, as FastMapper takes it."""
    h, w = yuv420p.shape[0] * 2 // 3, yuv420p.shape[1]
    m = np.empty_like(yuv420p)
    m[:h] = yuv420p[:h]
    m[h:, 0::2] = yuv420p[h:, : w // 2]
    m[h:, 1::2] = yuv420p[h:, w // 2:]
    return m


@pytest.mark.parametrize("wide", [False, True], ids=["compact", "wide"])
def test_gpu_fullsize_f2_fastmapper(product_lib, monkeypatch, wide):
    """F2 at the size it is benched: the C2 rig built by the GPU LUT build without ROI (octvr_dump -n), a
    vr::FastMapper in the compact (default) or the 8-byte entry format (OCTVR_FAST_WIDE=1), three
    stitch_nv12 calls in flight on three streams with their own outputs and the bench's splitmix frame
    sets (bench.py fast_rank) — every output byte against the oracle's FastMapper
    (mapper_fast.cpp:27-195, remap_weighted.cl:20-78)."""
    import torch
    from octvr_amd import synthetic
    ox = product_lib
    rig, W, H, sizes = synthetic.CONFIGS["F2"]()
    text = json.dumps(rig)
    monkeypatch.setenv("OCTVR_FAST_WIDE", "1" if wide else "0")
    mt = ox.MapperTemplate.from_json(text, W, H, use_roi=False)
    k = 3
    if "sets" not in _F2_ORACLE:
        want = O.lut_build(O.json_loads_rj(text), W, H, use_roi=False, threads=THREADS)
        _F2_ORACLE["luts"] = [(r[1], r[2], r[3]) for r in want]
        # bench.py fast_rank's sets: frame_seed(rank 0, set j, camera i) = 1000 + 100 j + i, set 0 splitmix64
        # frames, the others derived from it (bench.derive_set = synthetic.derived_frame)
        base = [_nv12(synthetic.yuv_frame(w, h, 1000 + i)) for i, (w, h) in enumerate(sizes)]
        _F2_ORACLE["sets"] = [base] + [[synthetic.derived_frame(f, 1000 + 100 * j + i) for i, f in enumerate(base)]
                                       for j in range(1, k)]
        _F2_ORACLE["want"] = [O.fastmapper_nv12(s, sizes, [l[0] for l in _F2_ORACLE["luts"]],
                                                [l[1] for l in _F2_ORACLE["luts"]], [l[2] for l in _F2_ORACLE["luts"]],
                                                W, H) for s in _F2_ORACLE["sets"]]
    for i, (m1, m2, mk) in enumerate(_F2_ORACLE["luts"]):
        roi, g1, g2, gm, _ = mt.input(i)
        assert roi == (0, 0, W, H)
        assert np.array_equal(gm, mk) and np.array_equal(g1.view(np.int32), m1.view(np.int32)) and \
            np.array_equal(g2.view(np.int32), m2.view(np.int32)), i
    fm = ox.FastMapper(mt, sizes)
    ok, rep = ox.debug_fastmapper_audit(mt, sizes, wide=wide)  # the same plan, replayed on the host
    assert ok, rep
    assert rep["y"]["compact"] == (0 if wide else 1)
    dev = [[torch.from_numpy(f).cuda() for f in s] for s in _F2_ORACLE["sets"]]
    outs = [torch.zeros((H * 3 // 2, W), dtype=torch.uint8, device="cuda") for _ in range(k)]
    streams = [torch.cuda.Stream() for _ in range(k)]
    torch.cuda.synchronize()
    for rep_ in range(2):  # twice round the streams: each stream's second call overlaps the others' first
        for j in range(k):
            fm.stitch_nv12(dev[j], outs[j], stream=streams[j])
    torch.cuda.synchronize()
    for j in range(k):
        got = outs[j].cpu().numpy()
        d = got != _F2_ORACLE["want"][j]
        assert not d.any(), (wide, j, int(d.sum()), np.argwhere(d)[:4].tolist())
        assert got[:H].std() > 10


@pytest.mark.parametrize("cfg", ["C2", "C3"])
def test_gpu_fullsize_texture_mode(product_lib, cfg):
    """The texture-convention mode (OCTVR_REMAP_TEXTURE: the reference's live CUDA sampling,
    fast_remap.cu:21-44) at the size its rate is quoted on: the staged instance (stitch_tiled_tex_kernel,
    12-bit LDS dword offsets, interior tiles) and the gather kernel for border tiles, the multi-band remap
    (C3) and the texture gain samples — three frames in flight on three streams, gains estimated, the
    bench's splitmix frame sets and one smooth set, every byte and the gains against the oracle's
    Mapper::stitch with the texture warp (orc_fast_remap_tex_rgba)."""
    import torch
    from octvr_amd import synthetic
    ox = product_lib
    rig, W, H, sizes, text, rois, maps1, maps2, masks = _oracle_lut(cfg)
    blend = synthetic.BLEND[cfg]
    mt = ox.MapperTemplate.from_json(text, W, H)
    seams = None
    if blend:
        mt.create_masks(0)
        seams = O.create_masks(rois, masks, W)
    m = ox.Mapper(mt, sizes, blend=blend, enable_gain=True, remap="texture")
    info = m.info()
    if not blend:  # most tiles are staged (interior), the fisheye circles' borders gather
        assert info["tiles"] > 0 and info["wide_tiles"] < info["tiles"], info
    k = 3
    m.set_frames_in_flight(k)
    sets = [_bench_frames(sizes, 0), _frames(sizes, 1), _bench_frames(sizes, 2)]
    dev = [[torch.from_numpy(f).cuda() for f in fs] for fs in sets]
    outs = [torch.zeros((H * 3 // 2, W), dtype=torch.uint8, device="cuda") for _ in range(k)]
    streams = [torch.cuda.Stream() for _ in range(k)]
    torch.cuda.synchronize()
    for f in range(k):
        m.stitch(dev[f], outs[f], stream=streams[f])
    g_last = np.array(m.gains())
    torch.cuda.synchronize()
    for f in range(k):
        exp, g_orc = O.stitch_frame(sets[f], sizes, rois, maps1, maps2, masks, W, H, enable_gain=True, gains=None,
                                    blend=blend, seams=seams, threads=THREADS, remap_tex=True)
        got = outs[f].cpu().numpy()
        d = got != exp
        assert not d.any(), (cfg, f, int(d.sum()), np.argwhere(d)[:4].tolist())
        if f == k - 1:
            np.testing.assert_array_equal(g_last, np.array(g_orc))
    if cfg == "C2":  # the AsyncMultiMapper in texture mode (the reference's AsyncMultiMapper runs vr::Mapper)
        del dev
        am = ox.AsyncMultiMapper([mt], sizes, (W, H), [0], [0], [(0.0, 0.0, 1.0, 1.0)], remap="texture")
        aouts = []
        for f in range(k):
            o = (np.zeros((H, W), np.uint8), np.zeros((H // 2, W // 2), np.uint8), np.zeros((H // 2, W // 2), np.uint8))
            am.push([(x[:h], x[h:, :w // 2], x[h:, w // 2:]) for x, (w, h) in zip(sets[f], sizes)], o)
            aouts.append(o)
        for f in range(k):
            am.pop()
            exp, _ = O.stitch_frame(sets[f], sizes, rois, maps1, maps2, masks, W, H, enable_gain=True,
                                    threads=THREADS, remap_tex=True)
            assert np.array_equal(aouts[f][0], exp[:H]), (f, "Y")
            assert np.array_equal(aouts[f][1], exp[H:, :W // 2]) and np.array_equal(aouts[f][2], exp[H:, W // 2:]), f
        am.close()


def test_gpu_fullsize_async_preview_c2(product_lib):
    """AsyncMultiMapper::New(..., preview_size) on the C2 rig at full size with two regions (top and bottom
    halves of the 8K output, each a scaled vr::Mapper): every preview byte (each region's Mapper preview
    resize into its rectangle, async.cpp:73-90) and every output byte against the oracle, frames pipelined."""
    import test_gpu_async as A
    ox = product_lib
    rig, W, H, sizes, text, rois, maps1, maps2, masks = _oracle_lut("C2")
    mt = ox.MapperTemplate.from_json(text, W, H)
    regions = [(0.0, 0.0, 1.0, 0.5), (0.0, 0.5, 1.0, 0.5)]
    pv_size = (1920, 961)
    am = ox.AsyncMultiMapper([mt, mt], sizes, (W, H), [0, 0], [0, 0], regions, preview_size=pv_size)
    sunk = []
    am.set_preview_sink(lambda a, h: sunk.append(a))
    sets = [_frames(sizes, 0), _bench_frames(sizes, 1)]
    outs = []
    for fs in sets:
        o = (np.zeros((H, W), np.uint8), np.zeros((H // 2, W // 2), np.uint8), np.zeros((H // 2, W // 2), np.uint8))
        am.push([(x[:h], x[h:, :w // 2], x[h:, w // 2:]) for x, (w, h) in zip(fs, sizes)], o)
        outs.append(o)
    for _ in sets:
        am.pop()
    assert len(sunk) == len(sets)
    for f, fs in enumerate(sets):
        want_out, want_pv = A.preview_oracle(fs, sizes, rois, maps1, maps2, masks, W, H, [0, 0], [0, 0], regions,
                                             (W, H), pv_size, threads=THREADS)
        for p in range(3):
            assert np.array_equal(outs[f][p], want_out[p]), (f, p)
        d = sunk[f] != want_pv
        assert not d.any(), (f, int(d.sum()), np.argwhere(d)[:4].tolist())
        assert sunk[f].std() > 5
    am.close()


@pytest.mark.parametrize("cfg,nb", [("C2", 2), ("C2", 4), ("C4", 4)])
def test_gpu_fullsize_batch(product_lib, cfg, nb):
    """Frame batches at the benched size (octvr_mapper_stitch_batch, one composite launch over (item, frame)
    units): two batches of nb frames on two streams, the bench's splitmix frame sets and smooth ones, gains
    estimated per frame — every output byte and the last frame's gains against the oracle."""
    import torch
    ox = product_lib
    rig, W, H, sizes, text, rois, maps1, maps2, masks = _oracle_lut(cfg)
    mt = ox.MapperTemplate.from_json(text, W, H)
    m = ox.Mapper(mt, sizes, blend=0, enable_gain=True)
    m.set_frames_in_flight(2 * nb)
    sets = [_bench_frames(sizes, j) if j % 2 == 0 else _frames(sizes, j) for j in range(2 * nb)]
    dev = [[torch.from_numpy(f).cuda() for f in fs] for fs in sets]
    outs = [torch.zeros((H * 3 // 2, W), dtype=torch.uint8, device="cuda") for _ in range(2 * nb)]
    streams = [torch.cuda.Stream() for _ in range(2)]
    torch.cuda.synchronize()
    for b in range(2):
        m.stitch_batch(dev[b * nb:(b + 1) * nb], outs[b * nb:(b + 1) * nb], stream=streams[b])
    g_last = np.array(m.gains())
    torch.cuda.synchronize()
    for f in range(2 * nb):
        exp, g_orc = O.stitch_frame(sets[f], sizes, rois, maps1, maps2, masks, W, H, enable_gain=True, gains=None,
                                    threads=THREADS)
        got = outs[f].cpu().numpy()
        d = got != exp
        assert not d.any(), (cfg, f, int(d.sum()), np.argwhere(d)[:4].tolist())
        if f == 2 * nb - 1:
            np.testing.assert_array_equal(g_last, np.array(g_orc))


@pytest.mark.parametrize("nb", [2, 4])
def test_gpu_fullsize_f2_batch(product_lib, nb):
    """FastMapper frame batches at the F2 size (octvr_fastmapper_stitch_nv12_batch: each run's entries loaded
    once for nb frames): the bench's frame sets, every byte against the oracle's FastMapper."""
    import torch
    from octvr_amd import synthetic
    ox = product_lib
    rig, W, H, sizes = synthetic.CONFIGS["F2"]()
    text = json.dumps(rig)
    mt = ox.MapperTemplate.from_json(text, W, H, use_roi=False)
    k = 3
    if "sets" not in _F2_ORACLE:  # (shared with test_gpu_fullsize_f2_fastmapper)
        want = O.lut_build(O.json_loads_rj(text), W, H, use_roi=False, threads=THREADS)
        _F2_ORACLE["luts"] = [(r[1], r[2], r[3]) for r in want]
        base = [_nv12(synthetic.yuv_frame(w, h, 1000 + i)) for i, (w, h) in enumerate(sizes)]
        _F2_ORACLE["sets"] = [base] + [[synthetic.derived_frame(f, 1000 + 100 * j + i) for i, f in enumerate(base)]
                                       for j in range(1, k)]
        _F2_ORACLE["want"] = [O.fastmapper_nv12(s, sizes, [l[0] for l in _F2_ORACLE["luts"]],
                                                [l[1] for l in _F2_ORACLE["luts"]], [l[2] for l in _F2_ORACLE["luts"]],
                                                W, H) for s in _F2_ORACLE["sets"]]
    fm = ox.FastMapper(mt, sizes)
    idx = [f % k for f in range(nb)]
    dev = [[torch.from_numpy(f).cuda() for f in _F2_ORACLE["sets"][j]] for j in idx]
    outs = [torch.zeros((H * 3 // 2, W), dtype=torch.uint8, device="cuda") for _ in range(nb)]
    torch.cuda.synchronize()
    fm.stitch_nv12_batch(dev, outs)
    torch.cuda.synchronize()
    for f, j in enumerate(idx):
        got = outs[f].cpu().numpy()
        d = got != _F2_ORACLE["want"][j]
        assert not d.any(), (nb, f, int(d.sum()), np.argwhere(d)[:4].tolist())
