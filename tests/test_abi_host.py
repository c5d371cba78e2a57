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


def _dat(out=(8, 4), rois=((0, 0, 4, 2),), mats=None, seams=None, n_ov=0, raw_inputs=None):
    """A small VRv11 file (template.cpp:206-256 layout): W, H, n, per input ROI + map1 + map2 + mask +
    vignette (empty), seam masks, overlay count.  `mats` / `seams` override the (type, rows, cols,
    payload) of each Mat."""
    i64 = lambda *v: np.array(v, np.int64).tobytes()
    b = b"VRv11" + i64(out[0], out[1], len(rois))
    for k, roi in enumerate(rois):
        w, h = roi[2], roi[3]
        b += i64(*roi)
        ms = (mats or {}).get(k) or [(5, h, w, np.zeros(w * h, np.float32).tobytes()),
                                      (5, h, w, np.zeros(w * h, np.float32).tobytes()),
                                      (0, h, w, np.zeros(w * h, np.uint8).tobytes()),
                                      (0, 0, 0, b"")]
        for t, r, c, payload in ms:
            b += i64(t, r, c) + payload
    for k, roi in enumerate(rois):
        t, r, c, payload = (seams or {}).get(k) or (0, roi[3], roi[2], np.zeros(roi[2] * roi[3], np.uint8).tobytes())
        b += i64(t, r, c) + payload
    return b + i64(n_ov)


def test_dat_reader_accepts_minimal_file(product_lib, tmp_path):
    p = tmp_path / "ok.dat"
    p.write_bytes(_dat())
    mt = product_lib.MapperTemplate.load(str(p))
    assert mt.out_size == (8, 4) and len(mt) == 1


@pytest.mark.parametrize("case", ["rows_cols_minus1", "map2_short", "seam_mismatch", "roi_outside", "roi_negative",
                                  "roi_empty", "out_zero", "negative_count", "truncated_map", "truncated_seam",
                                  "roi_x_int64_max", "roi_y_int64_max", "roi_w_int64_max"])
def test_dat_reader_rejects_malformed(product_lib, tmp_path, case):
    """every Mat must match its input's ROI and every ROI must lie inside the output frame,
    so a malformed .dat fails in the reader instead of reaching the mapper's ROI indexing."""
    z4 = lambda n, dt: np.zeros(n, dt).tobytes()
    if case == "rows_cols_minus1":  # (size_t)-1 * (size_t)-1 == 1 == 1 x 1 ROI
        data = _dat(rois=((0, 0, 1, 1),), mats={0: [(5, -1, -1, z4(1, np.float32)), (5, 1, 1, z4(1, np.float32)),
                                                    (0, 1, 1, z4(1, np.uint8)), (0, 0, 0, b"")]})
    elif case == "map2_short":
        data = _dat(mats={0: [(5, 2, 4, z4(8, np.float32)), (5, 1, 4, z4(4, np.float32)),
                              (0, 2, 4, z4(8, np.uint8)), (0, 0, 0, b"")]})
    elif case == "seam_mismatch":
        data = _dat(seams={0: (0, 1, 4, z4(4, np.uint8))})
    elif case == "roi_outside":
        data = _dat(rois=((6, 0, 4, 2),))
    elif case == "roi_negative":
        data = _dat(rois=((-1, 0, 4, 2),))
    elif case == "roi_empty":
        data = _dat(rois=((0, 0, 0, 2),))
    elif case == "roi_x_int64_max":  # x + w wraps negative and would pass `> out_w`
        data = _dat(rois=((2 ** 63 - 1, 0, 1, 2),), mats={0: [(5, 2, 1, z4(2, np.float32)), (5, 2, 1, z4(2, np.float32)),
                                                            (0, 2, 1, z4(2, np.uint8)), (0, 0, 0, b"")]})
    elif case == "roi_y_int64_max":
        data = _dat(rois=((0, 2 ** 63 - 1, 4, 1),), mats={0: [(5, 1, 4, z4(4, np.float32)), (5, 1, 4, z4(4, np.float32)),
                                                            (0, 1, 4, z4(4, np.uint8)), (0, 0, 0, b"")]})
    elif case == "roi_w_int64_max":
        data = _dat(rois=((1, 0, 2 ** 63 - 1, 2),), mats={0: [(5, 2, 4, z4(8, np.float32)), (5, 2, 4, z4(8, np.float32)),
                                                            (0, 2, 4, z4(8, np.uint8)), (0, 0, 0, b"")]},
                    seams={0: (0, 2, 4, z4(8, np.uint8))})
    elif case == "out_zero":
        data = _dat(out=(0, 4))
    elif case == "negative_count":
        data = b"VRv11" + np.array([8, 4, -1], np.int64).tobytes()
    elif case == "truncated_map":
        data = _dat()[:5 + 24 + 32 + 24 + 10]
    else:
        data = _dat()[:-20]
    p = tmp_path / ("bad_%s.dat" % case)
    p.write_bytes(data)
    with pytest.raises(product_lib.OctvrError):
        product_lib.MapperTemplate.load(str(p))


@pytest.mark.parametrize("roi", [(2 ** 31 - 1, 0, 1, 1), (0, 2 ** 31 - 1, 1, 1), (1, 0, 2 ** 31 - 1, 1)])
def test_from_arrays_rejects_overflowing_roi(product_lib, roi):
    """octvr_rig_create_from_arrays compares x <= out_w - w (no int overflow), so an
    ROI at INT_MAX is rejected instead of wrapping negative and passing."""
    one_f = np.zeros(1, np.float32)
    with pytest.raises(product_lib.OctvrError):
        product_lib.MapperTemplate.from_arrays(8, 4, [roi], [one_f], [one_f], [np.zeros(1, np.uint8)])


def test_mapper_create_ex_rejects_unknown_flags(product_lib):
    """octvr_mapper_create_ex validates its flags before any device work (OCTVR_REMAP_TEXTURE = 1 is the only
    one)."""
    import ctypes as C
    rig, z = O.load_rig("rigA")
    mt = product_lib.MapperTemplate.from_arrays(512, 256, z["rois"].tolist(), [z["map1_0"], z["map1_1"]],
                                               [z["map2_0"], z["map2_1"]], [z["mask_0"], z["mask_1"]])
    lib = product_lib.lib()
    w = (C.c_int * 2)(256, 256)
    h = (C.c_int * 2)(144, 144)
    out = C.c_void_p()
    rc = lib.octvr_mapper_create_ex(mt._h, 0, 2, w, h, 0, 1, 0, 0, 2, C.byref(out))
    assert rc == product_lib.E_INVALID and not out.value
    assert b"flags" in lib.octvr_last_error()


@pytest.mark.parametrize("failing", [0, 3, 15])
def test_worker_thread_error_becomes_a_status(product_lib, failing):
    """A REQUIRE inside a host worker thread (the tiler's staged-group check, the seam finder, the audits)
    reaches the caller as OCTVR_E_INVALID with the worker's message, and the process keeps running
    (an exception leaving a std::thread would std::terminate it, Python included)."""
    with pytest.raises(product_lib.OctvrError, match="worker %d failed" % failing):
        product_lib.debug_worker_failure(16, failing)
    product_lib.debug_worker_failure(16, -1)  # none fails: OK
    with pytest.raises(product_lib.OctvrError):  # the library is still usable after the error
        product_lib.debug_worker_failure(0, -1)
