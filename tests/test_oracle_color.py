"""The library's own RGB -> YUV420P (NPP's documented BT.601 matrix in fixed point; it stands in for NPP's
closed nppiRGBToYUV420, cudaimgproc/src/color.cpp:2306, so it is parity-unpinned against the reference):
the oracle (oracle/octvr_oracle.c rgb_quad_to_yuv) against a numpy statement of the definition in
DESIGN.md, its properties, and the YUV -> RGB -> YUV round trip through the staging conversion (the
inverse NPP documents, oracle yuv_px_to_rgb).  The GPU kernels (device_common.hpp quad_yuv) are checked
against the oracle by every -m gpu stitch test."""
import numpy as np

import oracle_py as O


def _numpy_yuv420(rgb):
    h, w, _ = rgb.shape
    x = rgb.astype(np.int64)
    R, G, B = x[..., 0], x[..., 1], x[..., 2]
    Y = (77 * R + 150 * G + 29 * B + 128) >> 8
    q = lambda a: a[0::2, 0::2] + a[0::2, 1::2] + a[1::2, 0::2] + a[1::2, 1::2]  # noqa: E731
    U = (q(-38 * R - 74 * G + 112 * B) + 131584) >> 10
    V = np.clip((q(79 * R - 66 * G - 13 * B) + 65792) >> 9, 0, 255)
    out = np.zeros((h * 3 // 2, w), np.uint8)
    out[:h] = Y
    out[h:, : w // 2] = U
    out[h:, w // 2:] = V
    return out


def test_rgb_to_yuv420_matches_definition():
    rng = np.random.default_rng(7)
    rgb = rng.integers(0, 256, size=(64, 96, 3), dtype=np.uint8)
    assert np.array_equal(O.rgb_to_yuv420(rgb), _numpy_yuv420(rgb))


def test_rgb_to_yuv420_within_one_of_npp_documented_matrix():
    """U = 0.492 (B - Y) + 128, V = 0.877 (R - Y) + 128 (NPP's documented RGBToYUV,
    the matrix its YUVToRGB inverts), chroma as the quad's mean: the fixed point is within +-1."""
    rng = np.random.default_rng(11)
    rgb = rng.integers(0, 256, size=(256, 512, 3), dtype=np.uint8)
    out = O.rgb_to_yuv420(rgb).astype(np.int64)
    x = rgb.astype(np.float64)
    Y = 0.299 * x[..., 0] + 0.587 * x[..., 1] + 0.114 * x[..., 2]
    q = lambda a: (a[0::2, 0::2] + a[0::2, 1::2] + a[1::2, 0::2] + a[1::2, 1::2]) / 4  # noqa: E731
    U = np.clip(np.floor(q(0.492 * (x[..., 2] - Y)) + 128.5), 0, 255)
    V = np.clip(np.floor(q(0.877 * (x[..., 0] - Y)) + 128.5), 0, 255)
    h = rgb.shape[0]
    assert np.abs(out[:h] - np.floor(Y + 0.5)).max() <= 1
    assert np.abs(out[h:, :256] - U).max() <= 1
    assert np.abs(out[h:, 256:] - V).max() <= 1


def test_yuv_rgb_yuv_round_trip_keeps_chroma():
    """Every in-gamut (Y, U, V) with the quad's chroma shared, as 4:2:0 staging delivers it: YUV ->
    RGB (staging) -> YUV420P returns U and V within +-1 and Y within +-1 (no camera blend: a single
    camera passed through the no-blend composite keeps its colours)."""
    rng = np.random.default_rng(5)
    n = 1 << 16
    yq = np.clip(rng.integers(0, 256, size=(n, 1)) + rng.integers(-12, 13, size=(n, 4)), 0, 255)
    u = rng.integers(0, 256, size=n)
    v = rng.integers(0, 256, size=n)
    # a YUV420P frame of n quads: 2 rows x 2n columns
    w, h = 2 * n, 2
    yuv = np.zeros((3, w), np.uint8)
    yuv[0, 0::2], yuv[0, 1::2], yuv[1, 0::2], yuv[1, 1::2] = yq[:, 0], yq[:, 1], yq[:, 2], yq[:, 3]
    yuv[2, : n] = u
    yuv[2, n:] = v
    rgba = O.yuv420_to_rgba(yuv, w, h)
    # in gamut: no channel of the quad saturated in the exact inverse
    Uf, Vf = (u - 128.0)[:, None], (v - 128.0)[:, None]
    Yf = yq.astype(np.float64)
    chans = [Yf + 1.140 * Vf, Yf - 0.394 * Uf - 0.581 * Vf, Yf + 2.032 * Uf]
    ing = np.all([(c > 0.5) & (c < 254.5) for c in chans], axis=(0, 2))
    assert ing.sum() > n // 16
    back = O.rgb_to_yuv420(rgba[..., :3]).astype(np.int64)
    assert np.abs(back[2, :n][ing] - u[ing]).max() <= 1
    assert np.abs(back[2, n:][ing] - v[ing]).max() <= 1
    yb = np.stack([back[0, 0::2], back[0, 1::2], back[1, 0::2], back[1, 1::2]], 1)
    assert np.abs(yb[ing] - yq[ing]).max() <= 1


def test_rgb_to_yuv420_gray_is_exact():
    # the Y coefficients sum to 256 and the chroma coefficients to 0: grey v -> (v, 128, 128) exactly
    v = np.arange(256, dtype=np.uint8)
    rgb = np.repeat(np.repeat(v[None, :, None], 2, axis=0), 3, axis=2)  # 2 x 256 greys
    out = O.rgb_to_yuv420(rgb)
    assert np.array_equal(out[0], v) and np.array_equal(out[1], v)
    assert (out[2] == 128).all()


def test_rgb_to_yuv420_extremes_saturate():
    # pure primaries and their complements: U stays in 16..240, V saturates at 0 / 255 (NPP's
    # 0.877 (R - Y) reaches +-157)
    cols = np.array([[255, 0, 0], [0, 255, 0], [0, 0, 255], [0, 255, 255], [255, 0, 255], [255, 255, 0],
                     [0, 0, 0], [255, 255, 255]], np.uint8)
    rgb = np.repeat(np.repeat(cols[None, :, :], 2, axis=0), 2, axis=1)  # 2 x 16, each colour a quad
    out = O.rgb_to_yuv420(rgb)
    assert np.array_equal(out, _numpy_yuv420(rgb))
    u, v = out[2, :8].astype(int), out[2, 8:].astype(int)
    assert u.min() >= 16 and u.max() <= 240
    assert v[0] == 255 and v[3] == 0  # red, cyan
