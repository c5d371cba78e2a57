"""The texture-convention filter (device_common.hpp div255, tex_bilerp_f) replaces the correctly rounded
f32 quotient t / 255 of the oracle's texture model (oracle/octvr_oracle.c orc_fast_remap_tex_rgba) by
q = t * fl(1/255) corrected by one residual step, fma(fma(-q, 255, t), fl(1/255), q).  Checked here for
every byte value with the fused multiply-adds emulated exactly: a * b + c is computed as a rational
(fractions.Fraction, no intermediate rounding) and rounded once to the nearest f32, ties to even, as an
FMA rounds.  (The device's own texture-mode outputs are pinned against the oracle separately,
tests/test_gpu_texture_mode.py.)"""
from fractions import Fraction

import numpy as np


def _round_f32(x):
    """The f32 nearest to the rational x, ties to even (x finite and well inside the f32 range)."""
    c = np.float32(float(x))  # within one f32 ulp of the answer (f64 then f32: at most a double rounding)
    best = None
    for cand in (np.nextafter(c, np.float32(-np.inf)), c, np.nextafter(c, np.float32(np.inf))):
        d = abs(Fraction(float(cand)) - x)
        even = (int(np.array(cand, np.float32).view(np.uint32)) & 1) == 0
        if best is None or d < best[0] or (d == best[0] and even and not best[2]):
            best = (d, cand, even)
    return best[1]


def _fma32(a, b, c):
    return _round_f32(Fraction(float(a)) * Fraction(float(b)) + Fraction(float(c)))


def test_round_f32_ties_to_even():
    one = Fraction(1)
    ulp = Fraction(2) ** -23
    assert _round_f32(one + ulp / 2) == np.float32(1)            # tie -> even (1.0)
    assert _round_f32(one + ulp + ulp / 2) == np.float32(1) + np.float32(2) * np.float32(ulp)  # tie -> even
    assert _round_f32(one + ulp / 2 + Fraction(1, 2 ** 60)) == np.nextafter(np.float32(1), np.float32(2))


def test_div255_is_the_correctly_rounded_quotient():
    r = np.float32(1) / np.float32(255)
    naive = 0
    for t in range(256):
        x = np.float32(t)
        exact = _round_f32(Fraction(t, 255))
        assert exact == x / np.float32(255), t  # IEEE division is correctly rounded
        q = np.float32(x * r)
        naive += int(q != exact)
        assert _fma32(_fma32(-q, np.float32(255), x), r, q) == exact, t
    assert naive > 100  # the plain product alone is off in about half the cases
