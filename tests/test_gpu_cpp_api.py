"""The vr:: C++ API (include/octvr.hpp over the C ABI) driven by a reference-style C++ caller
(tests/cpp/vr_api_test.cpp, built by build() as opencv-octvr_amd/lib/vr_api_test): the dump.cpp flow
(MapperTemplate + add_input + dump) must write the reference's own .dat bytes for the golden rigs, and
vr::Mapper (with preview_output), AsyncMultiMapper push/pop and FastMapper::stitch_nv12 must equal the
oracle bit for bit.  Reference: octvr.hpp:48-144, mapper.hpp:72-90, dump.cpp:76-113, async.cpp:174-193,
map.cpp:91-129."""
import hashlib
import json
import os
import subprocess

import numpy as np
import pytest

import oracle_py as O

pytestmark = pytest.mark.gpu
BIN = os.path.join(O.ROOT, "opencv-octvr_amd", "lib", "vr_api_test")


def _spans(text):
    """(start, end) of every JSON value in `text`, keyed by its path (tuple of keys / indices)."""
    out = {}

    def ws(i):
        while i < len(text) and text[i] in " \t\r\n":
            i += 1
        return i

    def value(i, path):
        i = ws(i)
        start = i
        c = text[i]
        if c == "{":
            i = ws(i + 1)
            if text[i] == "}":
                i += 1
            else:
                while True:
                    i = ws(i)
                    j = text.index('"', i + 1)
                    key = json.loads(text[i:j + 1])
                    i = ws(j + 1) + 1  # ':'
                    i = ws(value(i, path + (key,)))
                    if text[i] == ",":
                        i += 1
                        continue
                    i += 1  # '}'
                    break
        elif c == "[":
            i = ws(i + 1)
            k = 0
            if text[i] == "]":
                i += 1
            else:
                while True:
                    i = ws(value(i, path + (k,)))
                    k += 1
                    if text[i] == ",":
                        i += 1
                        continue
                    i += 1
                    break
        elif c == '"':
            j = i + 1
            while text[j] != '"':
                j += 2 if text[j] == "\\" else 1
            i = j + 1
        else:
            while i < len(text) and text[i] not in ",]} \t\r\n":
                i += 1
        out[path] = (start, i)
        return i

    value(0, ())
    return out


@pytest.mark.parametrize("name,blend", [("rigA", 0), ("rigB", 16), ("rigC", -5), ("rigD", 0)])
def test_gpu_cpp_api_drop_in(product_lib, tmp_path, name, blend):
    assert os.path.exists(BIN), "build() builds opencv-octvr_amd/lib/vr_api_test"
    text = open(os.path.join(O.ROOT, "tests", "golden", name + ".json")).read()
    rig, z = O.load_rig(name)
    W, H = (int(v) for v in z["out_size"])
    n = len(rig["inputs"])
    use_roi = name != "rigD"  # rigD's golden .dat was dumped with -n (template.cpp:126-133)
    sp = _spans(text)
    d = str(tmp_path)
    pw, ph = 200, 100
    with open(os.path.join(d, "case.txt"), "w") as f:
        f.write("%s %d %d %d %d %d %d %d\n" % (rig["output"]["type"], W, H, n, blend, pw, ph, int(use_roi)))
    a, b = sp[("output", "options")]
    open(os.path.join(d, "out_opts.json"), "w").write(text[a:b])
    sizes = []
    frames = []
    from octvr_amd import synthetic
    for i, cam in enumerate(rig["inputs"]):
        w, h = cam["options"]["width"], cam["options"]["height"]
        sizes.append((w, h))
        a, b = sp[("inputs", i, "options")]
        open(os.path.join(d, "in%d_opts.json" % i), "w").write(text[a:b])
        open(os.path.join(d, "in%d.txt" % i), "w").write("%s %d %d\n" % (cam["type"], w, h))
        fr = synthetic.smooth_yuv_frame(w, h, 600 + i)
        frames.append(fr)
        fr.tofile(os.path.join(d, "frame%d.yuv" % i))
    r = subprocess.run([BIN, d], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and os.path.exists(os.path.join(d, "ok")), r.stderr[-3000:]

    # dump.cpp flow: the reference's own bytes
    man = json.load(open(os.path.join(O.ROOT, "tests", "golden", "manifest.json")))["rigs"][name]
    dat = open(os.path.join(d, "rig.dat"), "rb").read()
    assert len(dat) == man["dat_bytes"] and hashlib.sha256(dat).hexdigest() == man["dat_sha256"]

    rois = z["rois"].tolist()
    maps1 = [z[f"map1_{i}"] for i in range(n)]
    maps2 = [z[f"map2_{i}"] for i in range(n)]
    masks = [z[f"mask_{i}"] for i in range(n)]
    seams = [z[f"seam_{i}"] for i in range(n)]
    # vr::Mapper::stitch with preview_output (estimated gains)
    want, g_orc, want_pv = O.stitch_frame(frames, sizes, rois, maps1, maps2, masks, W, H, enable_gain=True, blend=blend,
                                          seams=seams, threads=8, preview=(pw, ph))
    got = np.fromfile(os.path.join(d, "out_mapper.yuv"), np.uint8).reshape(H * 3 // 2, W)
    assert np.array_equal(got, want)
    assert np.array_equal(np.fromfile(os.path.join(d, "out_preview.rgb"), np.uint8).reshape(ph, pw, 3), want_pv)
    g = [float(v) for v in open(os.path.join(d, "gains_mapper.txt")).read().split()]
    np.testing.assert_array_equal(np.array(g), np.array(g_orc))
    # AsyncMultiMapper push / pop: frame f = luma + 11 f (mod 256)
    for f in range(3):
        fr = [x.copy() for x in frames]
        for x, (w, h) in zip(fr, sizes):
            x[:h] = (x[:h].astype(np.int32) + 11 * f).astype(np.uint8)
        want, _ = O.stitch_frame(fr, sizes, rois, maps1, maps2, masks, W, H, enable_gain=True, blend=blend, seams=seams,
                                 threads=8)
        y = np.fromfile(os.path.join(d, "out_async%d_y" % f), np.uint8).reshape(H, W)
        u = np.fromfile(os.path.join(d, "out_async%d_u" % f), np.uint8).reshape(H // 2, W // 2)
        v = np.fromfile(os.path.join(d, "out_async%d_v" % f), np.uint8).reshape(H // 2, W // 2)
        assert np.array_equal(y, want[:H]), f
        assert np.array_equal(u, want[H:, :W // 2]) and np.array_equal(v, want[H:, W // 2:]), f
    # AsyncMultiMapper::New(..., preview_size): the last frame's preview and its header
    _, _, want_pv = O.stitch_frame(fr, sizes, rois, maps1, maps2, masks, W, H, enable_gain=True, blend=blend,
                                   seams=seams, threads=8, preview=(pw, ph))
    assert np.array_equal(np.fromfile(os.path.join(d, "out_async_preview.rgb"), np.uint8).reshape(ph, pw, 3), want_pv)
    assert open(os.path.join(d, "preview_hdr.txt")).read().split() == [str(pw), str(ph), "0"]
    # FastMapper::stitch_nv12 on the template without ROI
    luts = O.lut_build(O.json_loads_rj(text), W, H, use_roi=False)
    nv12 = []
    for x, (w, h) in zip(frames, sizes):
        m = np.empty((h * 3 // 2, w), np.uint8)
        m[:h] = x[:h]
        m[h:, 0::2] = x[h:, :w // 2]
        m[h:, 1::2] = x[h:, w // 2:]
        nv12.append(m)
    want = O.fastmapper_nv12(nv12, sizes, [l[1] for l in luts], [l[2] for l in luts], [l[3] for l in luts], W, H)
    assert np.array_equal(np.fromfile(os.path.join(d, "out_fast.nv12"), np.uint8).reshape(H * 3 // 2, W), want)


RJ_BIN = os.path.join(O.ROOT, "opencv-octvr_amd", "lib", "vr_dump_rj")


@pytest.mark.parametrize("name", ["rigA", "rigB", "rigC", "rigD"])
def test_gpu_rapidjson_dump_flow(tmp_path, name):
    """apps/octvr/dump.cpp:71-113 verbatim in shape (rapidjson::Document -> MapperTemplate(type,
    options["output"]["options"], w, h) -> add_input(type, (*i)["options"], false, roi) -> dump) through
    the rapidjson::Value overloads (OCTVR_JSON_EXACT): the .dat equals the reference's own bytes, also
    with a comma-decimal locale active in the caller (a Qt caller's setlocale(LC_ALL, ""))."""
    if not os.path.exists(RJ_BIN):
        pytest.skip("vr_dump_rj is built only where rapidjson's headers exist (build container)")
    import test_json_locale as L
    rig, z = O.load_rig(name)
    W, H = (int(v) for v in z["out_size"])
    man = json.load(open(os.path.join(O.ROOT, "tests", "golden", "manifest.json")))["rigs"][name]
    cfg = os.path.join(O.ROOT, "tests", "golden", name + ".json")
    envs = [{"LC_ALL": "C"}]
    loc = L.comma_locale(tmp_path)
    if loc:
        envs.append(loc)
    for k, env in enumerate(envs):
        out = str(tmp_path / ("rig%d.dat" % k))
        args = [RJ_BIN, "-w", str(W), "-h", str(H), "-o", out, cfg]
        if name == "rigD":
            args.insert(1, "-n")  # rigD's golden .dat was dumped with -n (template.cpp:126-133)
        r = subprocess.run(args, capture_output=True, text=True, timeout=300, env=dict(os.environ, **env))
        assert r.returncode == 0, r.stderr[-2000:]
        dat = open(out, "rb").read()
        assert len(dat) == man["dat_bytes"] and hashlib.sha256(dat).hexdigest() == man["dat_sha256"], env
