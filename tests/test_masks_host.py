"""Camera mask rasterisation on the host (no GPU): the product's cv::fillPoly and PNG decoding used by
octvr_rig_create_json for `selection`, `exclude_masks` and `include_masks` (camera.cpp:96-187).

fillPoly parity: product (opencv-octvr_amd/csrc/masks.cpp) vs the oracle restatement
(oracle/octvr_oracle_masks.c) on random concave / self-intersecting / clipped polygons, bit-exact, plus
a known-answer check that is independent of both: the reference's `selection` polygon
(camera.cpp:104-111) fills exactly the rectangle [l, r-1] x [t, b-1].  No fillPoly golden image exists
in the reference tree (its drawing tests compare against opencv_extra data that is not vendored), so
polygon parity beyond rectangles is pinned to the restatement only.

PNG: decoded RGB vs the ground truth each fixture was encoded from (tests/png_fixture.py)."""
import numpy as np
import pytest

import oracle_py as O
import png_fixture as P


def _random_polys(rng, n):
    for k in range(n):
        w, h = int(rng.integers(1, 80)), int(rng.integers(1, 60))
        npts = int(rng.integers(1, 9))
        span = 1.6 if k % 3 == 0 else 1.0  # every third polygon reaches outside the image
        xs = rng.integers(int(-0.3 * w * (span - 1)) - 1, int(w * span) + 1, npts)
        ys = rng.integers(int(-0.3 * h * (span - 1)) - 1, int(h * span) + 1, npts)
        if k % 5 == 0 and npts > 2:
            ys[1] = ys[0]  # horizontal edge
        yield w, h, np.stack([xs, ys], 1).reshape(-1).tolist(), int(rng.integers(1, 256))


def test_fill_poly_matches_oracle_random(product_lib):
    rng = np.random.default_rng(1234)
    for w, h, pts, color in _random_polys(rng, 600):
        base = rng.integers(0, 2, (h, w)).astype(np.uint8) * 7
        got = product_lib.fill_poly(base.copy(), pts, color)
        want = base.copy()
        O.fill_poly(want, pts, color)
        assert np.array_equal(got, want), (w, h, pts)


@pytest.mark.parametrize("rect", [(180, 470, 20, 330), (0, 640, 40, 300), (-20, 100, -5, 400), (600, 700, 350, 360),
                                  (5, 6, 7, 8)])
def test_selection_polygon_is_the_rectangle(product_lib, rect):
    """Independent KAT: the rectangle Camera builds for `selection` fills [l, r-1] x [t, b-1]."""
    l, r, t, b = rect
    w, h = 640, 360
    img = np.full((h, w), 255, np.uint8)
    product_lib.fill_poly(img, [l, t, l, b - 1, r - 1, b - 1, r - 1, t], 0)
    want = np.full((h, w), 255, np.uint8)
    want[max(t, 0):max(min(b, h), 0), max(l, 0):max(min(r, w), 0)] = 0
    assert np.array_equal(img, want)


def test_fill_poly_degenerate(product_lib):
    img = np.zeros((9, 9), np.uint8)
    product_lib.fill_poly(img, [4, 4], 9)  # one point: the single-pixel line from CollectPolyEdges
    assert img[4, 4] == 9 and img.sum() == 9
    img = np.zeros((9, 9), np.uint8)
    product_lib.fill_poly(img, [1, 2, 7, 2], 3)  # horizontal segment: lines only, no edges
    assert (img[2, 1:8] == 3).all() and img.sum() == 21
    img = np.zeros((9, 9), np.uint8)
    product_lib.fill_poly(img, [100, 100, 120, 130, 90, 140], 5)  # entirely outside
    assert img.sum() == 0


CASES = [  # (colour type, bit depth, interlaced)
    (2, 8, False), (2, 8, True), (2, 16, False), (6, 8, False), (6, 16, True), (0, 8, False), (0, 1, False),
    (0, 2, True), (0, 4, False), (0, 16, False), (4, 8, True), (3, 8, False), (3, 4, True), (3, 1, False),
]


@pytest.mark.parametrize("ctype,depth,interlace", CASES)
def test_png_decode_matches_ground_truth(product_lib, ctype, depth, interlace):
    rng = np.random.default_rng(ctype * 100 + depth + interlace)
    h, w = 13, 21
    chans = {0: 1, 2: 3, 3: 1, 4: 2, 6: 4}[ctype]
    top = (1 << depth) - 1
    samples = rng.integers(0, top + 1, (h, w, chans))
    samples[rng.random((h, w)) < 0.3] = 0  # plenty of zero pixels, as in a mask
    palette = rng.integers(0, 256, (1 << depth, 3)) if ctype == 3 else None
    if palette is not None:
        palette[0] = 0
    png, rgb = P.encode(samples, ctype, depth, palette, interlace, seed=depth)
    assert np.array_equal(product_lib.png_decode_rgb(png), rgb)


def test_png_decode_rejects_garbage(product_lib):
    with pytest.raises(product_lib.OctvrError):
        product_lib.png_decode_rgb(b"GIF89a" + bytes(40))
    png, _ = P.encode(np.zeros((4, 4, 3), np.int64), 2)
    with pytest.raises(product_lib.OctvrError):
        product_lib.png_decode_rgb(png[:-30])


@pytest.mark.parametrize("ctype,depth", [(2, 4), (2, 1), (6, 2), (4, 4), (3, 16)])
def test_png_decode_rejects_illegal_depth(product_lib, ctype, depth):
    """colour type / bit depth pairs the PNG spec forbids (libpng, hence cv::imdecode at
    camera.cpp:175-176, rejects them) fail instead of decoding to garbage."""
    chans = {0: 1, 2: 3, 3: 1, 4: 2, 6: 4}[ctype]
    samples = np.zeros((3, 5, chans), np.int64)
    palette = np.zeros((256, 3), np.int64) if ctype == 3 else None
    png, _ = P.encode(samples, ctype, depth, palette, False, seed=1)
    with pytest.raises(product_lib.OctvrError) as e:
        product_lib.png_decode_rgb(png)
    assert "depth" in str(e.value)
