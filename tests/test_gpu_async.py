"""AsyncMultiMapper (modules/octvr/src/async.cpp): several mappers over the same
camera frames writing regions of one merged output, gain chaining, scaled regions, frames pipelined
(several pushes before the first pop) — every region bit-exact against the oracle's Mapper::stitch."""
import numpy as np
import pytest

import oracle_py as O

pytestmark = pytest.mark.gpu


def _planes(f, w, h):
    return f[:h], f[h:, :w // 2], f[h:, w // 2:]


@pytest.mark.parametrize("out_size,blends,gain_modes", [
    ((768, 768), [0, 16], [0, 0]),        # two regions at template size; region 1 reuses mapper 0's gains
    ((1024, 1024), [-5, 0], [0, -1]),     # scaled regions (768x384 -> 1024x512); region 1 without gain
    ((768, 768), [16, 0], [-1, 1]),
])
def test_gpu_async_multimapper_bit_exact(product_lib, out_size, blends, gain_modes):
    import torch
    from octvr_amd import synthetic
    ox = product_lib
    assert torch.cuda.is_available(), "gpu tests need a HIP device"
    rig, z = O.load_rig("rigB")
    W, H = (int(v) for v in z["out_size"])
    n = len(z["rois"])
    sizes = [(rig["inputs"][i]["options"]["width"], rig["inputs"][i]["options"]["height"]) for i in range(n)]
    maps1 = [z[f"map1_{i}"] for i in range(n)]
    maps2 = [z[f"map2_{i}"] for i in range(n)]
    masks = [z[f"mask_{i}"] for i in range(n)]
    seams = [z[f"seam_{i}"] for i in range(n)]
    mts = [ox.MapperTemplate.from_arrays(W, H, z["rois"].tolist(), maps1, maps2, masks, seams) for _ in blends]
    regions = [(0.0, 0.0, 1.0, 0.5), (0.0, 0.5, 1.0, 0.5)]
    am = ox.AsyncMultiMapper(mts, sizes, out_size, blends, gain_modes, regions)
    OW, OH = out_size
    frames, outs = [], []
    for f in range(5):  # more frames than pipeline slots, all pushed before the first pop
        fr = [synthetic.smooth_yuv_frame(w, h, 700 + 10 * f + i) for i, (w, h) in enumerate(sizes)]
        out = (np.zeros((OH, OW), np.uint8), np.zeros((OH // 2, OW // 2), np.uint8), np.zeros((OH // 2, OW // 2), np.uint8))
        am.push([_planes(x, w, h) for x, (w, h) in zip(fr, sizes)], out)
        frames.append(fr)
        outs.append(out)
    assert am.pending() == 5
    for f in range(5):
        got = am.pop()
        assert got is outs[f]
        gains_of = []
        for k, (bl, gm) in enumerate(zip(blends, gain_modes)):
            rw, rh = OW, OH // 2
            chained = gains_of[gm] if 0 <= gm < k else None
            want, g = O.stitch_frame(frames[f], sizes, z["rois"].tolist(), maps1, maps2, masks, W, H,
                                     enable_gain=gm >= 0, gains=chained, blend=bl, seams=seams, threads=8,
                                     scale=None if (rw, rh) == (W, H) else (rw, rh))
            gains_of.append(g)
            y0 = k * rh
            assert np.array_equal(got[0][y0:y0 + rh], want[:rh]), (f, k, "Y")
            assert np.array_equal(got[1][y0 // 2:(y0 + rh) // 2], want[rh:, :rw // 2]), (f, k, "U")
            assert np.array_equal(got[2][y0 // 2:(y0 + rh) // 2], want[rh:, rw // 2:]), (f, k, "V")
    with pytest.raises(ox.OctvrError):
        am.pop()  # nothing pending
    am.close()


def test_gpu_async_side_by_side_regions(product_lib):
    """Regions split horizontally (x offsets, pitched output rows): the copy-out stage's row ranges
    over its helper threads (async.cpp RowPool) write each region's rows at its own column offset."""
    import torch
    from octvr_amd import synthetic
    ox = product_lib
    assert torch.cuda.is_available(), "gpu tests need a HIP device"
    rig, z = O.load_rig("rigB")
    W, H = (int(v) for v in z["out_size"])
    n = len(z["rois"])
    sizes = [(rig["inputs"][i]["options"]["width"], rig["inputs"][i]["options"]["height"]) for i in range(n)]
    maps1 = [z[f"map1_{i}"] for i in range(n)]
    maps2 = [z[f"map2_{i}"] for i in range(n)]
    masks = [z[f"mask_{i}"] for i in range(n)]
    mts = [ox.MapperTemplate.from_arrays(W, H, z["rois"].tolist(), maps1, maps2, masks) for _ in range(2)]
    OW, OH = 2 * W, H  # two template-size regions side by side
    am = ox.AsyncMultiMapper(mts, sizes, (OW, OH), [0, 0], [0, 0], [(0.0, 0.0, 0.5, 1.0), (0.5, 0.0, 0.5, 1.0)])
    frames, outs = [], []
    for f in range(7):
        fr = [synthetic.smooth_yuv_frame(w, h, 300 + 10 * f + i) for i, (w, h) in enumerate(sizes)]
        out = (np.zeros((OH, OW), np.uint8), np.zeros((OH // 2, OW // 2), np.uint8), np.zeros((OH // 2, OW // 2), np.uint8))
        am.push([_planes(x, w, h) for x, (w, h) in zip(fr, sizes)], out)
        frames.append(fr)
        outs.append(out)
        if am.pending() >= 3:
            am.pop()
    while am.pending():
        am.pop()
    for f in range(7):
        want, _ = O.stitch_frame(frames[f], sizes, z["rois"].tolist(), maps1, maps2, masks, W, H,
                                 enable_gain=True, threads=8)
        for k in range(2):
            x0 = k * W
            assert np.array_equal(outs[f][0][:, x0:x0 + W], want[:H]), (f, k, "Y")
            assert np.array_equal(outs[f][1][:, x0 // 2:(x0 + W) // 2], want[H:, :W // 2]), (f, k, "U")
            assert np.array_equal(outs[f][2][:, x0 // 2:(x0 + W) // 2], want[H:, W // 2:]), (f, k, "V")
    am.close()


def test_gpu_async_rejects_bad_regions(product_lib):
    ox = product_lib
    rig, z = O.load_rig("rigA")
    mt = ox.MapperTemplate.from_arrays(512, 256, z["rois"].tolist(), [z["map1_0"], z["map1_1"]],
                                       [z["map2_0"], z["map2_1"]], [z["mask_0"], z["mask_1"]])
    with pytest.raises(ox.OctvrError):  # odd region height
        ox.AsyncMultiMapper([mt], [(256, 144)] * 2, (512, 258), [0], [0], [(0.0, 0.0, 1.0, 0.5)])


@pytest.mark.parametrize("name", ["rigC", "rigD", "rigA"])
def test_gpu_async_footprint_upload(product_lib, name):
    """Only the input bytes some kernel reads are uploaded (async.cpp footprint runs; the rest of each
    device frame holds a fixed pattern): rigs with wide tiles (gathered taps), with taps on the image
    edges, and a two-mapper set with the gain feed and multi-band, every frame bit-exact."""
    import torch
    from octvr_amd import synthetic
    ox = product_lib
    assert torch.cuda.is_available(), "gpu tests need a HIP device"
    rig, z = O.load_rig(name)
    W, H = (int(v) for v in z["out_size"])
    n = len(z["rois"])
    sizes = [(rig["inputs"][i]["options"]["width"], rig["inputs"][i]["options"]["height"]) for i in range(n)]
    maps1 = [z[f"map1_{i}"] for i in range(n)]
    maps2 = [z[f"map2_{i}"] for i in range(n)]
    masks = [z[f"mask_{i}"] for i in range(n)]
    seams = [z[f"seam_{i}"] for i in range(n)]
    blends = [0, 16] if name == "rigA" else [0]
    mts = [ox.MapperTemplate.from_arrays(W, H, z["rois"].tolist(), maps1, maps2, masks, seams) for _ in blends]
    info = ox.Mapper(mts[0], sizes, blend=0, enable_gain=True).info()
    assert 0 < info["footprint_bytes"] <= sum(w * h * 3 // 2 for w, h in sizes)
    regions = [(0.0, 0.0, 1.0, 1.0)] if len(blends) == 1 else [(0.0, 0.0, 1.0, 0.5), (0.0, 0.5, 1.0, 0.5)]
    OW, OH = W, H * len(blends)
    am = ox.AsyncMultiMapper(mts, sizes, (OW, OH), blends, [0] * len(blends), regions)
    frames, outs = [], []
    for f in range(4):
        fr = [synthetic.smooth_yuv_frame(w, h, 900 + 10 * f + i) for i, (w, h) in enumerate(sizes)]
        out = (np.zeros((OH, OW), np.uint8), np.zeros((OH // 2, OW // 2), np.uint8), np.zeros((OH // 2, OW // 2), np.uint8))
        am.push([_planes(x, w, h) for x, (w, h) in zip(fr, sizes)], out)
        frames.append(fr)
        outs.append(out)
    for f in range(4):
        am.pop()
        for k, bl in enumerate(blends):
            want, _ = O.stitch_frame(frames[f], sizes, z["rois"].tolist(), maps1, maps2, masks, W, H,
                                     enable_gain=True, blend=bl, seams=seams, threads=8)
            y0 = k * H
            assert np.array_equal(outs[f][0][y0:y0 + H], want[:H]), (f, k, "Y")
            assert np.array_equal(outs[f][1][y0 // 2:(y0 + H) // 2], want[H:, :W // 2]), (f, k, "U")
            assert np.array_equal(outs[f][2][y0 // 2:(y0 + H) // 2], want[H:, W // 2:]), (f, k, "V")
    am.close()


def _rect_mul_size(r, w, h):
    """_rect_mul_size (async.cpp:20-30) with std::round (half away from zero)."""
    import math
    rnd = lambda v: int(math.floor(v + 0.5)) if v >= 0 else -int(math.floor(-v + 0.5))
    x, y, rw, rh = rnd(r[0] * w), rnd(r[1] * h), rnd(r[2] * w), rnd(r[3] * h)
    if x + rw >= w:
        rw = w - x
    if y + rh >= h:
        rh = h - y
    return x, y, rw, rh


def preview_oracle(frames, sizes, rois, maps1, maps2, masks, W, H, blends, gain_modes, regions, out_size,
                   preview_size, seams=None, remap_tex=False, threads=8):
    """The merged output and the preview image of one AsyncMultiMapper frame through the oracle: per region
    Mapper::stitch with preview_output = the region's view of a black preview_size RGB image (async.cpp:73-90)."""
    OW, OH = out_size
    PW, PH = preview_size
    y = np.zeros((OH, OW), np.uint8)
    u = np.zeros((OH // 2, OW // 2), np.uint8)
    v = np.zeros((OH // 2, OW // 2), np.uint8)
    pv = np.zeros((PH, PW, 3), np.uint8)
    gains_of = []
    for k, (bl, gm, reg) in enumerate(zip(blends, gain_modes, regions)):
        rx, ry, rw, rh = _rect_mul_size(reg, OW, OH)
        px, py, pw, ph = _rect_mul_size(reg, PW, PH)
        chained = gains_of[gm] if 0 <= gm < k else None
        res = O.stitch_frame(frames, sizes, rois, maps1, maps2, masks, W, H, enable_gain=gm >= 0, gains=chained,
                             blend=bl, seams=seams, threads=threads, remap_tex=remap_tex,
                             scale=None if (rw, rh) == (W, H) else (rw, rh),
                             preview=(pw, ph) if pw > 0 and ph > 0 else None)
        want, g = res[0], res[1]
        if pw > 0 and ph > 0:
            pv[py:py + ph, px:px + pw] = res[2]
        gains_of.append(g)
        y[ry:ry + rh, rx:rx + rw] = want[:rh]
        u[ry // 2:(ry + rh) // 2, rx // 2:(rx + rw) // 2] = want[rh:, :rw // 2]
        v[ry // 2:(ry + rh) // 2, rx // 2:(rx + rw) // 2] = want[rh:, rw // 2:]
    return (y, u, v), pv


@pytest.mark.parametrize("blends,gain_modes,preview_size,remap", [
    ([0, 16], [0, 0], (300, 201), "remap"),      # regions split the preview at an odd row (round(100.5) = 101)
    ([-5, 0], [0, -1], (256, 128), "remap"),     # feather + no gain
    ([0, 0], [0, 1], (321, 161), "texture"),     # the CUDA sampling; the second region estimates its own gains
])
def test_gpu_async_preview_bit_exact(product_lib, blends, gain_modes, preview_size, remap):
    """AsyncMultiMapper::New(..., preview_size) (async.cpp:73-110, 141-171): every frame, each region's
    Mapper::stitch also writes the RGB result resized into its rectangle of one preview image, downloaded
    with the outputs and published with a PreviewDataHeader — every preview byte equal to the oracle's
    (Mapper preview resize per region), the outputs still bit-exact, the sink called once per frame in
    order, the header's fps 0 until a block of 10 frames completes (async.cpp:141-147)."""
    import torch
    from octvr_amd import synthetic
    ox = product_lib
    assert torch.cuda.is_available(), "gpu tests need a HIP device"
    rig, z = O.load_rig("rigB")
    W, H = (int(v) for v in z["out_size"])
    n = len(z["rois"])
    sizes = [(rig["inputs"][i]["options"]["width"], rig["inputs"][i]["options"]["height"]) for i in range(n)]
    maps1 = [z[f"map1_{i}"] for i in range(n)]
    maps2 = [z[f"map2_{i}"] for i in range(n)]
    masks = [z[f"mask_{i}"] for i in range(n)]
    seams = [z[f"seam_{i}"] for i in range(n)]
    mts = [ox.MapperTemplate.from_arrays(W, H, z["rois"].tolist(), maps1, maps2, masks, seams) for _ in blends]
    regions = [(0.0, 0.0, 1.0, 0.5), (0.0, 0.5, 1.0, 0.5)]
    out_size = (W, H) if blends[0] == 0 else (1024, 1024)
    am = ox.AsyncMultiMapper(mts, sizes, out_size, blends, gain_modes, regions, remap=remap, preview_size=preview_size)
    assert am.preview_size == preview_size
    rgb, hdr = am.preview()
    assert rgb is None and hdr.width == 0 and hdr.height == 0  # nothing published yet
    sunk = []
    am.set_preview_sink(lambda a, h: sunk.append((a, h.width, h.height, h.step, h.fps)))
    OW, OH = out_size
    nf = 12
    frames, outs = [], []
    for f in range(nf):
        fr = [synthetic.smooth_yuv_frame(w, h, 1300 + 10 * f + i) for i, (w, h) in enumerate(sizes)]
        out = (np.zeros((OH, OW), np.uint8), np.zeros((OH // 2, OW // 2), np.uint8), np.zeros((OH // 2, OW // 2), np.uint8))
        am.push([_planes(x, w, h) for x, (w, h) in zip(fr, sizes)], out)
        frames.append(fr)
        outs.append(out)
        if am.pending() >= 3:
            am.pop()
    while am.pending():
        am.pop()
    rgb, hdr = am.preview()  # the last frame's
    assert (hdr.width, hdr.height, hdr.step) == preview_size + (0,)
    assert len(sunk) == nf
    for f in range(nf):
        want_out, want_pv = preview_oracle(frames[f], sizes, z["rois"].tolist(), maps1, maps2, masks, W, H, blends,
                                           gain_modes, regions, out_size, preview_size, seams=seams,
                                           remap_tex=remap == "texture")
        for p in range(3):
            assert np.array_equal(outs[f][p], want_out[p]), (f, p)
        a, w, h, st, fps = sunk[f]
        assert (w, h, st) == preview_size + (0,)
        assert np.array_equal(a, want_pv), (f, int((a != want_pv).sum()))
        assert (fps == 0.0) == (f < 9), (f, fps)  # the first block of 10 frames completes at frame 9
        if f == nf - 1:
            assert np.array_equal(rgb, want_pv)
            assert hdr.fps == fps
    info = am.info()
    assert info["preview"] == list(preview_size) and info["mappers"] == 2
    am.set_preview_sink(None)
    am.close()


def test_gpu_async_preview_rejects_bad_size(product_lib):
    ox = product_lib
    rig, z = O.load_rig("rigA")
    mt = ox.MapperTemplate.from_arrays(512, 256, z["rois"].tolist(), [z["map1_0"], z["map1_1"]],
                                       [z["map2_0"], z["map2_1"]], [z["mask_0"], z["mask_1"]])
    with pytest.raises(ox.OctvrError):
        ox.AsyncMultiMapper([mt], [(256, 144)] * 2, (512, 256), [0], [0], [(0.0, 0.0, 1.0, 1.0)],
                            preview_size=(-4, 10))
    am = ox.AsyncMultiMapper([mt], [(256, 144)] * 2, (512, 256), [0], [0], [(0.0, 0.0, 1.0, 1.0)])
    with pytest.raises(ox.OctvrError):  # no preview configured
        am.preview()
    am.close()


def test_gpu_async_registered_outputs(product_lib):
    """Output plane sets the caller registers (octvr_async_register_output) are downloaded straight into
    (2-D D2H copies at the caller's pitch, no staging, no copy-out); pushes mixing registered and
    unregistered sets, two regions side by side, padded pitches — every frame bit-exact; unregistering
    with frames pending is refused."""
    import torch
    from octvr_amd import synthetic
    ox = product_lib
    assert torch.cuda.is_available(), "gpu tests need a HIP device"
    rig, z = O.load_rig("rigB")
    W, H = (int(v) for v in z["out_size"])
    n = len(z["rois"])
    sizes = [(rig["inputs"][i]["options"]["width"], rig["inputs"][i]["options"]["height"]) for i in range(n)]
    maps1 = [z[f"map1_{i}"] for i in range(n)]
    maps2 = [z[f"map2_{i}"] for i in range(n)]
    masks = [z[f"mask_{i}"] for i in range(n)]
    mts = [ox.MapperTemplate.from_arrays(W, H, z["rois"].tolist(), maps1, maps2, masks) for _ in range(2)]
    OW, OH = 2 * W, H
    am = ox.AsyncMultiMapper(mts, sizes, (OW, OH), [0, 0], [0, 0], [(0.0, 0.0, 0.5, 1.0), (0.5, 0.0, 0.5, 1.0)])

    def planes(pad):  # views into padded buffers: pitch > width
        y = np.zeros((OH, OW + pad), np.uint8)[:, :OW]
        u = np.zeros((OH // 2, OW // 2 + pad), np.uint8)[:, :OW // 2]
        v = np.zeros((OH // 2, OW // 2 + pad), np.uint8)[:, :OW // 2]
        return (y, u, v)

    ring = [planes(64 * k) for k in range(3)]
    for r in ring[:2]:
        am.register_output(r)
    am.register_output(ring[0])  # again: a no-op
    frames, outs = [], []
    for f in range(6):
        fr = [synthetic.smooth_yuv_frame(w, h, 1700 + 10 * f + i) for i, (w, h) in enumerate(sizes)]
        out = ring[f % 3]  # ring[2] is not registered: staging path
        am.push([_planes(x, w, h) for x, (w, h) in zip(fr, sizes)], out)
        if f == 1:
            with pytest.raises(ox.OctvrError):
                am.unregister_output(ring[0])
        am.pop()
        want, _ = O.stitch_frame(fr, sizes, z["rois"].tolist(), maps1, maps2, masks, W, H, enable_gain=True,
                                 threads=8)
        for k in range(2):
            x0 = k * W
            assert np.array_equal(out[0][:, x0:x0 + W], want[:H]), (f, k, "Y")
            assert np.array_equal(out[1][:, x0 // 2:(x0 + W) // 2], want[H:, :W // 2]), (f, k, "U")
            assert np.array_equal(out[2][:, x0 // 2:(x0 + W) // 2], want[H:, W // 2:]), (f, k, "V")
    am.unregister_output(ring[1])
    am.close()
