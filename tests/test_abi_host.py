"""Host-side checks of the product library (no GPU needed): every symbol declared in include/*.h is
exported, and the VRv11 .dat writer/reader is byte-compatible with the reference's dump
(template.cpp:206-314) — checked against the SHA-256 of the reference's own .dat files."""
import glob
import hashlib
import json
import os
import re

import numpy as np
import pytest

import oracle_py as O

ROOT = O.ROOT
RIGS = ["rigA", "rigB", "rigC", "rigD"]


def declared_symbols():
    names = set()
    for h in glob.glob(os.path.join(ROOT, "include", "*.h")):
        txt = open(h).read()
        for m in re.finditer(r"^\s*(?:const\s+)?[\w\s\*]+?\b(octvr_\w+)\s*\(", txt, re.M):
            names.add(m.group(1))
    return names


def test_library_exports_every_declared_symbol(product_lib):
    names = declared_symbols()
    assert len(names) >= 20
    lib = product_lib.lib()
    missing = [n for n in sorted(names) if not hasattr(lib, n)]
    assert not missing, missing
    assert product_lib.abi_version() == 1


@pytest.mark.parametrize("name", RIGS)
def test_dat_writer_matches_reference_bytes(product_lib, name, tmp_path):
    rig, z = O.load_rig(name)
    man = json.load(open(os.path.join(ROOT, "tests", "golden", "manifest.json")))["rigs"][name]
    n = len(z["rois"])
    W, H = (int(v) for v in z["out_size"])
    mt = product_lib.MapperTemplate.from_arrays(W, H, z["rois"].tolist(), [z[f"map1_{i}"] for i in range(n)],
                                               [z[f"map2_{i}"] for i in range(n)], [z[f"mask_{i}"] for i in range(n)],
                                               [z[f"seam_{i}"] for i in range(n)])
    p = tmp_path / (name + ".dat")
    mt.dump(str(p))
    data = p.read_bytes()
    assert len(data) == man["dat_bytes"]
    assert hashlib.sha256(data).hexdigest() == man["dat_sha256"]
    # reader round trip
    mt2 = product_lib.MapperTemplate.load(str(p))
    assert mt2.out_size == (W, H) and len(mt2) == n
    for i in range(n):
        roi, m1, m2, mk, seam = mt2.input(i)
        assert roi == tuple(z["rois"][i])
        assert np.array_equal(m1, z[f"map1_{i}"]) and np.array_equal(m2, z[f"map2_{i}"])
        assert np.array_equal(mk, z[f"mask_{i}"]) and np.array_equal(seam, z[f"seam_{i}"])


def test_dat_reader_rejects_bad_magic(product_lib, tmp_path):
    p = tmp_path / "bad.dat"
    p.write_bytes(b"VRv10" + b"\0" * 64)
    with pytest.raises(product_lib.OctvrError) as e:
        product_lib.MapperTemplate.load(str(p))
    assert "version" in str(e.value)


def test_dat_reader_rejects_truncated(product_lib, tmp_path):
    p = tmp_path / "trunc.dat"
    p.write_bytes(b"VRv11" + np.array([512, 256, 2], np.int64).tobytes())
    with pytest.raises(product_lib.OctvrError):
        product_lib.MapperTemplate.load(str(p))


def test_dump_without_seams_is_an_error(product_lib, tmp_path):
    rig, z = O.load_rig("rigA")
    mt = product_lib.MapperTemplate.from_arrays(512, 256, z["rois"].tolist(), [z["map1_0"], z["map1_1"]],
                                               [z["map2_0"], z["map2_1"]], [z["mask_0"], z["mask_1"]])
    with pytest.raises(product_lib.OctvrError):
        mt.dump(str(tmp_path / "x.dat"))
