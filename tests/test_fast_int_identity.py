"""The FastMapper kernels (opencv-octvr_amd/csrc/fastmapper.hip, weighted_sum_int) evaluate remap_weighted's
per-camera sum (imgproc/src/opencl/remap_weighted.cl:46-75)

    v = t0 (1 - ux) (1 - uy) + t1 ux (1 - uy) + t2 (1 - ux) uy + t3 ux uy;  v *= w;  convert_ushort_sat_rte(v)

in f32 (each product and sum rounded as written, ux = fx / 32, uy = fy / 32) as the integer
N = (32 - fy)(t0 (32 - fx) + t1 fx) + fy (t2 (32 - fx) + t3 fx) followed by rint(fl(N * (w / 1024))).
This checks the identity on the CPU for every fraction code and weight, with random and extreme taps."""
import numpy as np


def f32_reference(t, fx, fy, w):
    f = np.float32
    ux = fx.astype(f) / f(32)
    uy = fy.astype(f) / f(32)
    one = f(1)
    v = t[0] * (one - ux) * (one - uy)
    v = v + t[1] * ux * (one - uy)
    v = v + t[2] * (one - ux) * uy
    v = v + t[3] * ux * uy
    v = v * w.astype(f)
    return np.clip(np.rint(v), 0, 65535).astype(np.int64)


def integer_form(t, fx, fy, w):
    ti = t.astype(np.int64)
    n = (32 - fy) * (ti[0] * (32 - fx) + ti[1] * fx) + fy * (ti[2] * (32 - fx) + ti[3] * fx)
    wf = w.astype(np.float32) * np.float32(1.0 / 1024.0)
    return np.rint(n.astype(np.float32) * wf).astype(np.int64)


def test_fast_int_matches_f32_sum():
    rng = np.random.default_rng(5)
    code = np.arange(1024, dtype=np.int64)
    fx, fy = code & 31, code >> 5
    w = np.arange(256, dtype=np.int64)
    FX, W = np.meshgrid(fx, w, indexing="ij")
    FY, _ = np.meshgrid(fy, w, indexing="ij")
    FX, FY, W = FX.ravel(), FY.ravel(), W.ravel()
    tap_sets = [np.full((4, 1), 255), np.zeros((4, 1)), np.array([[255], [0], [0], [255]]), np.array([[0], [255], [255], [0]])]
    tap_sets += [rng.integers(0, 256, (4, 1)) for _ in range(24)]
    for taps in tap_sets:
        t = np.broadcast_to(taps, (4, FX.size)).astype(np.float32)
        want = f32_reference(t, FX, FY, W)
        got = integer_form(t, FX, FY, W)
        assert np.array_equal(want, got), (taps.ravel().tolist(), int((want != got).sum()))
    # per-pixel random taps over the whole code x weight grid
    t = rng.integers(0, 256, (4, FX.size)).astype(np.float32)
    assert np.array_equal(f32_reference(t, FX, FY, W), integer_form(t, FX, FY, W))
