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
