"""The blend = 0 composite's tiled LUT on the CPU (no GPU): octvr_debug_tiled_lut_info picks the copy chain's
winner per output pixel (the last camera whose ROI holds it and whose mask is set — the reference's
copy-mode chain, modules/octvr/src/mapper.cpp) and builds the tiled LUT exactly as octvr_mapper_create
does (opencv-octvr_amd/csrc/tiling.cpp build_tiled_lut).  build_tiled_lut REQUIREs that every tap of every
pixel lies in a staged row-span group of its camera slot ("staging groups"), so a build
that passes here is one whose stitch_tiled_kernel reads only staged LDS.  The checks below pin the
round-5 staging numbers DESIGN.md quotes for C2 (boxes 17.37 M pixels, spans 10.06 M)."""
import numpy as np
import pytest

import oracle_py as O


@pytest.mark.parametrize("name", ["rigA", "rigB", "rigC", "rigD"])
def test_tiled_lut_golden_rigs(product_lib, name):
    ox = product_lib
    rig, z = O.load_rig(name)
    W, H = (int(v) for v in z["out_size"])
    n = len(z["rois"])
    mt = ox.MapperTemplate.from_arrays(W, H, z["rois"].tolist(), [z[f"map1_{i}"] for i in range(n)],
                                       [z[f"map2_{i}"] for i in range(n)], [z[f"mask_{i}"] for i in range(n)])
    sizes = [(c["options"]["width"], c["options"]["height"]) for c in rig["inputs"]]
    info = ox.debug_tiled_lut_info(mt, sizes)
    assert info["items"] > 0
    # spans stage at most the bounding boxes, in u16 pixels (2 bytes each)
    assert 0 < info["staged_px"] <= info["box_px"]
    assert info["staged_bytes"] == 2 * info["staged_px"]
    assert sum(info["items_by_chunks"].values()) == info["items"]
    assert sum(info["items_by_lds_kib"]) == info["items"]


@pytest.mark.parametrize("name", ["rigA", "rigB", "rigC", "rigD"])
def test_tiled_lut_texture_convention(product_lib, name):
    """OCTVR_REMAP_TEXTURE entries (make_entry_tex): pixels whose four clamped taps lie inside the image are
    staged (16-bit fraction codes, tiled_entry_tex) under the same staged-group check; tiles with a border
    pixel take the gather path."""
    ox = product_lib
    rig, z = O.load_rig(name)
    W, H = (int(v) for v in z["out_size"])
    n = len(z["rois"])
    mt = ox.MapperTemplate.from_arrays(W, H, z["rois"].tolist(), [z[f"map1_{i}"] for i in range(n)],
                                       [z[f"map2_{i}"] for i in range(n)], [z[f"mask_{i}"] for i in range(n)])
    sizes = [(c["options"]["width"], c["options"]["height"]) for c in rig["inputs"]]
    base = ox.debug_tiled_lut_info(mt, sizes)
    info = ox.debug_tiled_lut_info(mt, sizes, remap="texture")
    assert base["tex"] == 0
    assert info["items"] + info["wide_tiles"] // 2 >= 1
    if info["items"]:
        assert info["tex"] == 1 and 0 < info["staged_px"] <= info["box_px"]
    # border taps move tiles to the gather path, never the other way
    assert info["wide_tiles"] >= base["wide_tiles"]


def test_tiled_lut_rejects_short_sizes(product_lib):
    ox = product_lib
    rig, z = O.load_rig("rigA")
    mt = ox.MapperTemplate.from_arrays(512, 256, z["rois"].tolist(), [z["map1_0"], z["map1_1"]],
                                       [z["map2_0"], z["map2_1"]], [z["mask_0"], z["mask_1"]])
    with pytest.raises(ox.OctvrError):
        ox.debug_tiled_lut_info(mt, [(64, 64)])


def test_tiled_lut_c2(product_lib):
    """The C2 bench workload (6 x 3840x2160 fisheyes -> 7680x3840 with ROIs)."""
    ox = product_lib
    from octvr_amd import synthetic
    rig, W, H, sizes = synthetic.CONFIGS["C2"]()
    luts = O.lut_build(rig, W, H, use_roi=True, threads=8)
    mt = ox.MapperTemplate.from_arrays(W, H, [l[0] for l in luts], [l[1] for l in luts], [l[2] for l in luts],
                                       [l[3] for l in luts])
    info = ox.debug_tiled_lut_info(mt, sizes)
    assert info["items"] == (W // 128) * (H // 16)
    assert info["wide_tiles"] == 0
    assert info["box_px"] == pytest.approx(17.37e6, rel=0.01)
    assert info["staged_px"] == pytest.approx(10.06e6, rel=0.01)
    # the composite's source footprint (what the AsyncMultiMapper uploads, gain samples aside): the union
    # of the staged groups, 13 % of the frames' YUV
    assert info["footprint_bytes"] == pytest.approx(info["source_bytes"], rel=0.01)
    assert info["footprint_bytes"] < 0.15 * info["frame_bytes"]
    # every item fits the 16 KiB tile LDS; no item needs more than 4 staging chunks
    assert info["items_by_lds_kib"][5:] == [0, 0]
    assert sum(v for k, v in info["items_by_chunks"].items() if int(k) > 4) == 0
    # the texture convention stages the same rig with one more column / row of taps per cell at most
    tex = ox.debug_tiled_lut_info(mt, sizes, remap="texture")
    assert tex["tex"] == 1 and tex["items"] + tex["wide_tiles"] // 2 == info["items"]
    assert tex["wide_tiles"] < 0.05 * info["items"]


@pytest.mark.parametrize("name", ["rigA", "rigB", "rigC", "rigD"])
def test_gain_plan_layout(product_lib, name):
    """The gain feed's sample layout on the host (octvr_debug_gain_plan, as octvr_mapper_create builds it):
    whole workgroups of 768 samples, one camera per wave run of 192 (kGainWaveRun: the wave's frame is
    uniform), no sample partnered with its own camera, padding samples invalid with no partner."""
    ox = product_lib
    rig, z = O.load_rig(name)
    W, H = (int(v) for v in z["out_size"])
    n = len(z["rois"])
    mt = ox.MapperTemplate.from_arrays(W, H, z["rois"].tolist(), [z[f"map1_{i}"] for i in range(n)],
                                       [z[f"map2_{i}"] for i in range(n)], [z[f"mask_{i}"] for i in range(n)])
    sizes = [(c["options"]["width"], c["options"]["height"]) for c in rig["inputs"]]
    e, p = ox.debug_gain_plan(mt, sizes)
    assert len(e) % 768 == 0 and len(e) == len(p)
    cam = (e[:, 1] >> 10) & 31
    valid = (e[:, 1] >> 15) & 1
    runs = cam.reshape(-1, 192)
    assert (runs == runs[:, :1]).all()  # one camera per wave run
    assert not ((p.astype(np.uint32) >> cam) & 1).any()  # never its own partner
    assert (valid[p != 0] <= 1).all()  # (mask-0 samples keep their partners: they add a zero norm)
    if name != "rigD":  # rigD's inputs do not overlap at the working scale
        assert (p != 0).sum() > 0
