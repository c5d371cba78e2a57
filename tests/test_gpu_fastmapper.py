"""vr::FastMapper::stitch_nv12 on the GPU against the oracle
restatement (oracle/octvr_oracle_fast.c): bit-exact NV12 output (chroma rows V,U) on full-frame
templates of every golden rig.  The reference runs this path on OpenCL only; no fixture exists
(parity unpinned)."""
import json

import numpy as np
import pytest

import oracle_py as O

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("wide", [False, True], ids=["compact", "wide"])
@pytest.mark.parametrize("name", ["rigA", "rigB", "rigC", "rigD"])
def test_gpu_fastmapper_nv12_bit_exact(product_lib, name, wide, monkeypatch):
    """Both entry formats: the compact 5-byte entries (default) and the 8-byte ones (OCTVR_FAST_WIDE=1)."""
    import torch
    ox = product_lib
    monkeypatch.setenv("OCTVR_FAST_WIDE", "1" if wide else "0")
    rig, z = O.load_rig(name)
    W, H = (int(v) for v in z["out_size"])
    mt = ox.MapperTemplate.from_json(json.dumps(rig), W, H, use_roi=False)  # octvr_dump without ROI
    n = len(mt)
    sizes = [(c["options"]["width"], c["options"]["height"]) for c in rig["inputs"]]
    maps1, maps2, masks = [], [], []
    for i in range(n):
        roi, m1, m2, mk, _ = mt.input(i)
        assert roi == (0, 0, W, H)
        maps1.append(m1); maps2.append(m2); masks.append(mk)
    fm = ox.FastMapper(mt, sizes)
    for seed in (11, 12):
        frames = [O.rand_img(w, h * 3 // 2, 1, 100 * seed + i) for i, (w, h) in enumerate(sizes)]
        out = torch.zeros((H * 3 // 2, W), dtype=torch.uint8, device="cuda")
        fm.stitch_nv12([torch.from_numpy(f).cuda() for f in frames], out)
        torch.cuda.synchronize()
        want = O.fastmapper_nv12(frames, sizes, maps1, maps2, masks, W, H)
        got = out.cpu().numpy()
        d = got != want
        assert not d.any(), (seed, int(d.sum()), np.argwhere(d)[:5].tolist())


def test_gpu_fastmapper_needs_full_frame_templates(product_lib):
    """mapper_fast.cpp:50-51: a template dumped with ROIs is refused (camera 0 cropped to its left half)."""
    ox = product_lib
    rig, z = O.load_rig("rigA")
    W, H = (int(v) for v in z["out_size"])
    n = len(z["rois"])
    rois = z["rois"].tolist()
    m1 = [z[f"map1_{i}"] for i in range(n)]
    m2 = [z[f"map2_{i}"] for i in range(n)]
    mk = [z[f"mask_{i}"] for i in range(n)]
    rois[0] = [0, 0, W // 2, H]
    m1[0], m2[0], mk[0] = (np.ascontiguousarray(a[:, : W // 2]) for a in (m1[0], m2[0], mk[0]))
    mt = ox.MapperTemplate.from_arrays(W, H, rois, m1, m2, mk)
    sizes = [(c["options"]["width"], c["options"]["height"]) for c in rig["inputs"]]
    with pytest.raises(ox.OctvrError):
        ox.FastMapper(mt, sizes)


def test_gpu_fastmapper_edge_taps(product_lib):
    """Maps scattered over [-0.06, 1.06] of small frames: taps at x / y = -1, 0, w - 1, w and beyond on
    both planes, where the kernel's 8-byte row loads start at the clamped column (and within 8 bytes of
    a frame that ends mid-dword, at size - 8) and the taps outside the image read 0 (remap_weighted
    BORDER_CONSTANT); bit-exact vs the oracle, full-frame masks."""
    import torch
    ox = product_lib
    W, H = 96, 48
    sizes = [(40, 24), (42, 26)]  # 42 x 39 = 1638 bytes: the frame ends mid-dword
    rng = np.random.default_rng(7)
    m1 = [rng.uniform(-0.06, 1.06, (H, W)).astype(np.float32) for _ in sizes]
    m2 = [rng.uniform(-0.06, 1.06, (H, W)).astype(np.float32) for _ in sizes]
    mk = [np.full((H, W), 255, np.uint8) for _ in sizes]
    mk[1][:, : W // 3] = 0
    mt = ox.MapperTemplate.from_arrays(W, H, [[0, 0, W, H]] * 2, m1, m2, mk)
    fm = ox.FastMapper(mt, sizes)
    for seed in (3, 4):
        frames = [O.rand_img(w, h * 3 // 2, 1, 50 * seed + i) for i, (w, h) in enumerate(sizes)]
        out = torch.zeros((H * 3 // 2, W), dtype=torch.uint8, device="cuda")
        fm.stitch_nv12([torch.from_numpy(f).cuda() for f in frames], out)
        torch.cuda.synchronize()
        want = O.fastmapper_nv12(frames, sizes, m1, m2, mk, W, H)
        got = out.cpu().numpy()
        d = got != want
        assert not d.any(), (seed, int(d.sum()), np.argwhere(d)[:5].tolist())
        assert want.any()


def test_gpu_fastmapper_wide_blocks(product_lib):
    """A 4000-pixel-wide source sampled at random over a 96-pixel output: a luma block's taps span more
    than 2048 pixels, so the Y plane falls back to the 8-byte entries, while the half-size chroma plane
    (spans < 2000) stays compact; both bit-exact vs the oracle."""
    import torch
    ox = product_lib
    W, H = 96, 32
    sizes = [(4000, 24), (64, 20)]
    rng = np.random.default_rng(9)
    m1 = [rng.uniform(0.0, 1.0, (H, W)).astype(np.float32) for _ in sizes]
    m2 = [rng.uniform(0.0, 1.0, (H, W)).astype(np.float32) for _ in sizes]
    mk = [np.full((H, W), 255, np.uint8) for _ in sizes]
    mk[1][:, W // 2:] = 0
    mt = ox.MapperTemplate.from_arrays(W, H, [[0, 0, W, H]] * 2, m1, m2, mk)
    fm = ox.FastMapper(mt, sizes)
    frames = [O.rand_img(w, h * 3 // 2, 1, 70 + i) for i, (w, h) in enumerate(sizes)]
    out = torch.zeros((H * 3 // 2, W), dtype=torch.uint8, device="cuda")
    fm.stitch_nv12([torch.from_numpy(f).cuda() for f in frames], out)
    torch.cuda.synchronize()
    want = O.fastmapper_nv12(frames, sizes, m1, m2, mk, W, H)
    got = out.cpu().numpy()
    d = got != want
    assert not d.any(), (int(d.sum()), np.argwhere(d)[:5].tolist())
    assert want.any()


@pytest.mark.parametrize("wide", [False, True], ids=["compact", "wide"])
@pytest.mark.parametrize("name", ["rigA", "rigB", "rigC", "rigD"])
@pytest.mark.parametrize("nb", [2, 4])
def test_gpu_fastmapper_batch_bit_exact(product_lib, name, wide, nb, monkeypatch):
    """octvr_fastmapper_stitch_nv12_batch: nb frames per launch (each run's entries loaded once), both entry
    formats, the general and the interior paths — every frame equal to the oracle's stitch of that frame."""
    import torch
    ox = product_lib
    monkeypatch.setenv("OCTVR_FAST_WIDE", "1" if wide else "0")
    rig, z = O.load_rig(name)
    W, H = (int(v) for v in z["out_size"])
    mt = ox.MapperTemplate.from_json(json.dumps(rig), W, H, use_roi=False)
    n = len(mt)
    sizes = [(c["options"]["width"], c["options"]["height"]) for c in rig["inputs"]]
    maps1, maps2, masks = [], [], []
    for i in range(n):
        _, m1, m2, mk, _ = mt.input(i)
        maps1.append(m1); maps2.append(m2); masks.append(mk)
    fm = ox.FastMapper(mt, sizes)
    frames = [[O.rand_img(w, h * 3 // 2, 1, 700 + 37 * f + i) for i, (w, h) in enumerate(sizes)] for f in range(nb)]
    outs = [torch.zeros((H * 3 // 2, W), dtype=torch.uint8, device="cuda") for _ in range(nb)]
    fm.stitch_nv12_batch([[torch.from_numpy(x).cuda() for x in fr] for fr in frames], outs)
    torch.cuda.synchronize()
    for f in range(nb):
        want = O.fastmapper_nv12(frames[f], sizes, maps1, maps2, masks, W, H)
        got = outs[f].cpu().numpy()
        d = got != want
        assert not d.any(), (f, int(d.sum()), np.argwhere(d)[:5].tolist())
