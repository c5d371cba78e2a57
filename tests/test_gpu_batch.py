"""Frame batches (octvr_mapper_stitch_batch): 2 or 4 frames of one rig through ONE composite launch whose
work runs over (item, frame) pairs (kernels.hpp FrameBatch) — each frame with its own gain feed, gains,
staging and output.  Every output and every frame's gains must equal the oracle's Mapper::stitch of that
frame alone (mapper.cpp:193-323), bit for bit: batches on several streams, rigs with wide (gathered) tiles,
vignetting, the texture convention, caller gains, and the 32- / 16-camera frame tables."""
import json
import math

import numpy as np
import pytest

import oracle_py as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ox(product_lib):
    import torch
    assert torch.cuda.is_available(), "gpu tests need a HIP device"
    return product_lib


def _cuda(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def _ring_rig(n, in_w=320, in_h=240):
    from octvr_amd import synthetic
    yaws = [2 * math.pi * k / n for k in range(n)]
    pitches = [0.35 * (-1) ** k for k in range(n)]
    return synthetic.fisheye_rig(in_w, in_h, yaws, pitches)


def _template(mt, n):
    rois, maps1, maps2, masks = [], [], [], []
    for i in range(n):
        roi, m1, m2, mk, _ = mt.input(i)
        rois.append(roi); maps1.append(m1); maps2.append(m2); masks.append(mk)
    return rois, maps1, maps2, masks


@pytest.mark.parametrize("nb,streams,n,gain", [(2, 1, 6, True), (2, 3, 6, True), (4, 2, 6, True), (2, 2, 3, True),
                                               (4, 1, 12, True), (4, 2, 16, True), (2, 2, 20, False)])
def test_gpu_batch_vs_oracle(ox, nb, streams, n, gain):
    """Batches of nb frames issued round-robin on `streams` streams (nb * streams frames in flight), two
    rounds: every output equals the oracle's stitch of that frame, the last frame's gains the oracle's."""
    import torch
    from octvr_amd import synthetic
    rig = _ring_rig(n)
    W, H = 512, 256
    mt = ox.MapperTemplate.from_json(json.dumps(rig), W, H)
    sizes = [(320, 240)] * n
    rois, maps1, maps2, masks = _template(mt, n)
    m = ox.Mapper(mt, sizes, blend=0, enable_gain=gain)
    m.set_frames_in_flight(nb * streams)
    st = [torch.cuda.Stream() for _ in range(streams)]
    nfr = 2 * nb * streams
    frames = [[synthetic.smooth_yuv_frame(w, h, 900 + 13 * f + i) for i, (w, h) in enumerate(sizes)]
              for f in range(nfr)]
    dev = [[_cuda(x) for x in fr] for fr in frames]
    outs = [torch.zeros((H * 3 // 2, W), dtype=torch.uint8, device="cuda") for _ in range(nfr)]
    torch.cuda.synchronize()
    for b in range(nfr // nb):
        m.stitch_batch(dev[b * nb:(b + 1) * nb], outs[b * nb:(b + 1) * nb], stream=st[b % streams])
    g_last = np.array(m.gains())
    torch.cuda.synchronize()
    for f in range(nfr):
        want, g_orc = O.stitch_frame(frames[f], sizes, rois, maps1, maps2, masks, W, H, enable_gain=gain, gains=None,
                                     threads=8)
        got = outs[f].cpu().numpy()
        assert np.array_equal(got, want), (f, int((got != want).sum()))
        if f == nfr - 1:
            np.testing.assert_array_equal(g_last, np.array(g_orc))


@pytest.mark.parametrize("name", ["rigA", "rigB", "rigC", "rigD"])
@pytest.mark.parametrize("remap", ["remap", "texture"])
def test_gpu_batch_golden_rigs(ox, name, remap):
    """The golden rigs (wide tiles: one wide-kernel launch per frame of the batch; partial ROIs; no overlap in
    rigD), both sampling conventions, a batch of 2 and one of 4, with the caller's gains for the second."""
    import torch
    from octvr_amd import synthetic
    rig, z = O.load_rig(name)
    W, H = (int(v) for v in z["out_size"])
    n = len(z["rois"])
    sizes = [(rig["inputs"][i]["options"]["width"], rig["inputs"][i]["options"]["height"]) for i in range(n)]
    maps1 = [z[f"map1_{i}"] for i in range(n)]
    maps2 = [z[f"map2_{i}"] for i in range(n)]
    masks = [z[f"mask_{i}"] for i in range(n)]
    rois = z["rois"].tolist()
    mt = ox.MapperTemplate.from_arrays(W, H, rois, maps1, maps2, masks)
    m = ox.Mapper(mt, sizes, blend=0, enable_gain=True, remap=remap)
    m.set_frames_in_flight(4)
    tex = remap == "texture"
    for nb, given in ((2, False), (4, True)):
        frames = [[synthetic.smooth_yuv_frame(w, h, 40 * nb + 7 * f + i) for i, (w, h) in enumerate(sizes)]
                  for f in range(nb)]
        gains = [[0.8 + 0.05 * ((f + i) % 7) for i in range(n)] for f in range(nb)] if given else None
        outs = [torch.zeros((H * 3 // 2, W), dtype=torch.uint8, device="cuda") for _ in range(nb)]
        m.stitch_batch([[_cuda(x) for x in fr] for fr in frames], outs, gains=gains)
        torch.cuda.synchronize()
        for f in range(nb):
            want, _ = O.stitch_frame(frames[f], sizes, rois, maps1, maps2, masks, W, H, enable_gain=True,
                                     gains=gains[f] if given else None, threads=8, remap_tex=tex)
            got = outs[f].cpu().numpy()
            assert np.array_equal(got, want), (name, nb, f, int((got != want).sum()))


def test_gpu_batch_vignette(ox):
    """Vignetted inputs (the VIG instance of the batched composite and the lean feed's vignette gathers)."""
    import torch
    from octvr_amd import synthetic
    import test_gpu_vignette as V
    rig = V._vignette_rig()
    W, H = 768, 384
    mt = ox.MapperTemplate.from_json(json.dumps(rig), W, H)
    n = len(mt)
    sizes = [(c["options"]["width"], c["options"]["height"]) for c in rig["inputs"]]
    vig = []
    for i, c in enumerate(rig["inputs"]):
        want = O.vignette_map(c["options"])
        vig.append(None if want is None else O.resize_linear_cuda_f32(want, sizes[i][0], sizes[i][1]))
    rois, maps1, maps2, masks = _template(mt, n)
    m = ox.Mapper(mt, sizes, blend=0, enable_gain=True)
    m.set_frames_in_flight(2)
    frames = [[synthetic.smooth_yuv_frame(w, h, 60 + 5 * f + i) for i, (w, h) in enumerate(sizes)] for f in range(2)]
    outs = [torch.zeros((H * 3 // 2, W), dtype=torch.uint8, device="cuda") for _ in range(2)]
    m.stitch_batch([[_cuda(x) for x in fr] for fr in frames], outs)
    torch.cuda.synchronize()
    for f in range(2):
        want, _ = O.stitch_frame(frames[f], sizes, rois, maps1, maps2, masks, W, H, enable_gain=True, vig=vig,
                                 threads=8)
        assert np.array_equal(outs[f].cpu().numpy(), want), f


def test_gpu_batch_rejects(ox):
    import torch
    rig = _ring_rig(20)
    mt = ox.MapperTemplate.from_json(json.dumps(rig), 512, 256)
    sizes = [(320, 240)] * 20
    m = ox.Mapper(mt, sizes, blend=0, enable_gain=False)
    fr = [torch.zeros((360, 320), dtype=torch.uint8, device="cuda") for _ in range(20)]
    outs = [torch.zeros((384, 512), dtype=torch.uint8, device="cuda") for _ in range(4)]
    with pytest.raises(ox.OctvrError):  # two frames need two frame slots
        m.stitch_batch([fr, fr], outs[:2])
    m.set_frames_in_flight(4)
    with pytest.raises(ox.OctvrError):  # four frames hold 16 cameras each
        m.stitch_batch([fr] * 4, outs)
    with pytest.raises(ox.OctvrError):  # 3 is not a batch size
        m.stitch_batch([fr] * 3, outs[:3])
    m.stitch_batch([fr] * 2, outs[:2])
    torch.cuda.synchronize()
