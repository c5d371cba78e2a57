"""GPU parity of vignette correction: Vignette::getMap (vignette.cpp:18-54) at
512x512, cuda::resize to the input size (mapper.cpp:108-112) and the per-source-pixel multiply
before the remap (mapper.cpp:230-231), through the whole stitch, bit-exact against the oracle."""
import json

import numpy as np
import pytest

import oracle_py as O

pytestmark = pytest.mark.gpu


def _vignette_rig():
    rig, _ = O.load_rig("rigB")
    rig = json.loads(json.dumps(rig))
    for k, c in enumerate(rig["inputs"]):
        o = c["options"]
        if k % 3 == 2:
            continue  # some cameras without a vignette: their frames are used as they are
        o["vignette"] = [1.0 + 0.05 * k, -0.35, 0.12 - 0.01 * k, -0.04]
        if k % 2:
            o["exposure"] = 0.25 * k - 0.5
    return rig


@pytest.mark.parametrize("blend,inflight", [(0, 1), (16, 1), (-5, 1), (0, 2), (16, 3)])
def test_gpu_vignette_bit_exact(product_lib, blend, inflight):
    import torch
    from octvr_amd import synthetic
    ox = product_lib
    assert torch.cuda.is_available(), "gpu tests need a HIP device"
    rig = _vignette_rig()
    W, H = 768, 384
    mt = ox.MapperTemplate.from_json(json.dumps(rig), W, H)
    n = len(mt)
    sizes = [(c["options"]["width"], c["options"]["height"]) for c in rig["inputs"]]
    vig = []
    for i, c in enumerate(rig["inputs"]):
        want = O.vignette_map(c["options"])
        got = mt.vignette(i)
        if want is None:
            assert got is None
            vig.append(None)
            continue
        assert np.array_equal(got.view(np.int32), want.view(np.int32)), i
        vig.append(O.resize_linear_cuda_f32(want, sizes[i][0], sizes[i][1]))
    mt.create_masks(0)
    rois, maps1, maps2, masks, seams = [], [], [], [], []
    for i in range(n):
        roi, m1, m2, mk, sm = mt.input(i)
        rois.append(roi); maps1.append(m1); maps2.append(m2); masks.append(mk); seams.append(sm)
    frames = [synthetic.smooth_yuv_frame(w, h, 300 + i) for i, (w, h) in enumerate(sizes)]
    m = ox.Mapper(mt, sizes, blend=blend, enable_gain=True)
    m.set_frames_in_flight(inflight)  # > 1: the lean gain feed (vignette gathers) and per-slot state
    dev_frames = [torch.from_numpy(f).cuda() for f in frames]
    outs = [torch.zeros((H * 3 // 2, W), dtype=torch.uint8, device="cuda") for _ in range(inflight)]
    streams = [torch.cuda.Stream() for _ in range(inflight)]
    torch.cuda.synchronize()
    for k in range(inflight):  # every slot in turn stitches the same frame, each on its own stream
        m.stitch(dev_frames, outs[k], stream=streams[k])
    torch.cuda.synchronize()
    g = np.array(m.gains())
    want, g_orc = O.stitch_frame(frames, sizes, rois, maps1, maps2, masks, W, H, enable_gain=True, blend=blend,
                                 seams=seams, vig=vig, threads=8)
    np.testing.assert_array_equal(g, g_orc)
    for out in outs:
        got = out.cpu().numpy()
        d = got != want
        assert not d.any(), (int(d.sum()), np.argwhere(d)[:5].tolist())
