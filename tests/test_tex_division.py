"""The texture-convention filter (device_common.hpp div255, tex_bilerp_f) replaces the correctly rounded
f32 quotient t / 255 of the oracle's texture model (oracle/octvr_oracle.c orc_fast_remap_tex_rgba) by
q = t * fl(1/255) corrected by one residual step, fma(fma(-q, 255, t), fl(1/255), q).  Checked here for
every byte value: the fused multiply-adds are evaluated exactly in f64 (a product of two f32 is exact in
f64, and these sums stay exact) and rounded once to f32, as an FMA rounds."""
import numpy as np


def _fma32(a, b, c):
    return np.float32(np.float64(a) * np.float64(b) + np.float64(c))


def test_div255_is_the_correctly_rounded_quotient():
    r = np.float32(1) / np.float32(255)
    naive = 0
    for t in range(256):
        x = np.float32(t)
        exact = x / np.float32(255)
        q = np.float32(x * r)
        naive += int(q != exact)
        assert _fma32(_fma32(-q, np.float32(255), x), r, q) == exact, t
    assert naive > 100  # the plain product alone is off in about half the cases
