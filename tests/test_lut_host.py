"""The host half of the bit-exact LUT build (no GPU): pixels the GPU's LUT guard defers are recomputed
on the host with glibc by the product's own camera_math.hpp (octvr_hip.cpp build_input).  That host
projection must equal the oracle's FP64 projection bit for bit (the oracle is pinned to the reference's
LUT goldens, tests/test_oracle_golden.py), for every camera model and mask kind the guard covers."""
import json
import os

import numpy as np
import pytest

import camera_rigs as R
import oracle_py as O

GOLDEN = ["rigA", "rigB", "rigC", "rigD"]


def _same_f64(a, b):
    """bitwise equal, NaN == NaN"""
    return np.array_equal(a.view(np.int64), b.view(np.int64)) or (
        np.array_equal(np.isnan(a), np.isnan(b)) and np.array_equal(a[~np.isnan(a)], b[~np.isnan(b)]))


def _check_rig(ox, rig, W, H, inputs=None, text=None):
    # the product parses numbers as rapidjson does (json_lite.hpp): the oracle gets the same doubles
    text = json.dumps(rig) if text is None else text
    rig = O.json_loads_rj(text)
    for i in (range(len(rig["inputs"])) if inputs is None else inputs):
        hx, hy, _ = ox.debug_project_f64(text, W, H, i, where=1)
        ox_, oy_ = O.project_f64(rig["output"], rig["inputs"][i], W, H)
        assert _same_f64(hx, ox_) and _same_f64(hy, oy_), (i, int((hx != ox_).sum()), int((hy != oy_).sum()))


@pytest.mark.parametrize("name", GOLDEN)
def test_host_projection_equals_oracle_golden_rigs(product_lib, name):
    rig, z = O.load_rig(name)
    W, H = (int(v) for v in z["out_size"])
    with open(os.path.join(O.ROOT, "tests", "golden", name + ".json")) as f:
        _check_rig(product_lib, rig, W, H, text=f.read())


@pytest.mark.parametrize("name", sorted(R.input_rigs()))
def test_host_projection_equals_oracle_input_models(product_lib, name):
    _check_rig(product_lib, R.input_rigs()[name], 512, 256)


@pytest.mark.parametrize("name", sorted(R.output_rigs()))
def test_host_projection_equals_oracle_output_models(product_lib, name):
    _check_rig(product_lib, R.output_rigs()[name], 384, 200)


@pytest.mark.parametrize("name", ["exclude_poly", "png"])
def test_host_projection_equals_oracle_masks(product_lib, name):
    _check_rig(product_lib, R.mask_rigs()[name], 512, 256)


@pytest.mark.parametrize("cfg", ["C2", "C4"])
def test_host_projection_equals_oracle_bench_rigs(product_lib, cfg):
    from octvr_amd import synthetic
    rig, W, H, _ = synthetic.CONFIGS[cfg]()
    _check_rig(product_lib, rig, 1536, 768, inputs=[0, len(rig["inputs"]) - 1])


def test_interval_union(product_lib):
    """octvr_interval_union (the arithmetic of Mapper.kernel_busy): overlapping, nested,
    touching, disjoint and unordered intervals, the empty log, and a bad interval."""
    U = product_lib.interval_union
    assert U([], []) == (0.0, 0.0)
    assert U([1.0], [3.0]) == (2.0, 2.0)
    assert U([0.0, 2.0], [3.0, 5.0]) == (6.0, 5.0)           # overlapping
    assert U([0.0, 1.0], [10.0, 2.0]) == (11.0, 10.0)        # nested
    assert U([0.0, 3.0], [3.0, 4.0]) == (4.0, 4.0)           # touching
    assert U([5.0, 0.0], [6.0, 1.0]) == (2.0, 2.0)           # disjoint, unordered
    assert U([4.0, 0.0, 1.0, 9.0], [5.0, 2.0, 3.0, 9.0]) == (5.0, 4.0)  # a chain, a zero-length one
    rng = np.random.default_rng(3)
    a = rng.uniform(0, 100, 200)
    b = a + rng.uniform(0, 5, 200)
    grid = np.zeros(100 * 64 + 5 * 64 + 64, bool)
    for s, e in zip(np.round(a * 64).astype(int), np.round(b * 64).astype(int)):
        grid[s:e] = True
    sp, bu = U(np.round(a * 64) / 64, np.round(b * 64) / 64)
    assert abs(bu - grid.sum() / 64) < 1e-9 and abs(sp - (np.round(b * 64) - np.round(a * 64)).sum() / 64) < 1e-9
    with pytest.raises(product_lib.OctvrError):
        U([2.0], [1.0])
