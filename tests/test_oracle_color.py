"""The library's own RGB -> YUV420P (full-range BT.601 in 8-bit fixed point; it stands in for NPP's closed
nppiRGBToYUV420, so it is parity-unpinned against the reference): the oracle (oracle/octvr_oracle.c
rgb_quad_to_yuv) against a numpy statement of the definition in DESIGN.md, and its properties.  The GPU
kernels (device_common.hpp quad_yuv) are checked against the oracle by every -m gpu stitch test."""
import numpy as np

import oracle_py as O


def _numpy_yuv420(rgb):
    h, w, _ = rgb.shape
    x = rgb.astype(np.int64)
    R, G, B = x[..., 0], x[..., 1], x[..., 2]
    Y = (77 * R + 150 * G + 29 * B + 128) >> 8
    q = lambda a: a[0::2, 0::2] + a[0::2, 1::2] + a[1::2, 0::2] + a[1::2, 1::2]  # noqa: E731
    U = (q(-43 * R - 84 * G + 127 * B) + 131584) >> 10
    V = (q(127 * R - 106 * G - 21 * B) + 131584) >> 10
    out = np.zeros((h * 3 // 2, w), np.uint8)
    out[:h] = Y
    out[h:, : w // 2] = U
    out[h:, w // 2:] = V
    return out


def test_rgb_to_yuv420_matches_definition():
    rng = np.random.default_rng(7)
    rgb = rng.integers(0, 256, size=(64, 96, 3), dtype=np.uint8)
    assert np.array_equal(O.rgb_to_yuv420(rgb), _numpy_yuv420(rgb))


def test_rgb_to_yuv420_gray_is_exact():
    # the Y coefficients sum to 256 and the chroma coefficients to 0: grey v -> (v, 128, 128) exactly
    v = np.arange(256, dtype=np.uint8)
    rgb = np.repeat(np.repeat(v[None, :, None], 2, axis=0), 3, axis=2)  # 2 x 256 greys
    out = O.rgb_to_yuv420(rgb)
    assert np.array_equal(out[0], v) and np.array_equal(out[1], v)
    assert (out[2] == 128).all()


def test_rgb_to_yuv420_extremes_stay_in_range():
    # U, V land in 1..255 without clamping for every quad (pure primaries and their complements)
    cols = np.array([[255, 0, 0], [0, 255, 0], [0, 0, 255], [0, 255, 255], [255, 0, 255], [255, 255, 0],
                     [0, 0, 0], [255, 255, 255]], np.uint8)
    rgb = np.repeat(np.repeat(cols[None, :, :], 2, axis=0), 2, axis=1)  # 2 x 16, each colour a quad
    out = O.rgb_to_yuv420(rgb)
    assert np.array_equal(out, _numpy_yuv420(rgb))
    assert out[2:].min() >= 1
