"""bench.py's roofline bookkeeping on the CPU: `roofline.traffic` comes only from a PMC summary whose
so_sha256 is the running library's (a summary of another binary is never used), and the committed
summaries under profiles/ have the shape bench.pmc_traffic reads."""
import glob
import json
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNEL = "void octvr::stitch_tiled_kernel<false, 0, false, 2>(octvr::FrameSet, ...)"


def _write(d, name, sha, per_launch=1000.0, per_frame=5000.0):
    os.makedirs(d / "profiles", exist_ok=True)
    (d / "profiles" / name).write_text(json.dumps({
        "so_sha256": sha, "traffic_per_frame_bytes": per_frame,
        "traffic_bytes": {"octvr::gain_feed_lean_kernel(...)": 7.0, KERNEL: per_launch}}))


@pytest.fixture
def bench_at(tmp_path, monkeypatch):
    import bench
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    monkeypatch.setattr(bench, "lib_sha256", lambda: "a" * 64)
    return bench, tmp_path


def test_pmc_traffic_keyed_to_library(bench_at):
    bench, d = bench_at
    _write(d, "r01_pmc_C2.json", "b" * 64, per_launch=1.0)  # another binary: skipped
    _write(d, "r02_pmc_C2.json", "a" * 64, per_launch=1234.4, per_frame=99.6)
    assert bench.pmc_traffic("C2", 0) == (1234, "r02_pmc_C2.json")  # the composite launch
    # blend > 0: the blend sequence per frame, every kernel but the gain feed (outside the timed events)
    (d / "profiles" / "r03_pmc_C3.json").write_text(json.dumps({
        "so_sha256": "a" * 64, "traffic_per_frame_bytes": 1e9,
        "traffic_bytes": {"octvr::gain_feed_lean_kernel(...)": 500.0, KERNEL: 1000.4, "octvr::mb_down_kernel@1": 200.2,
                          "octvr::mb_blend_kernel@2": 30.0}}))
    assert bench.pmc_traffic("C3", 3) == (1231, "r03_pmc_C3.json")


def test_pmc_traffic_absent_for_other_binaries(bench_at):
    bench, d = bench_at
    _write(d, "r01_pmc_C3.json", "b" * 64)
    v, why = bench.pmc_traffic("C3", 3)
    assert v is None and "no PMC summary" in why and "aaaaaaaaaaaa" in why
    assert bench.pmc_traffic("C4", 0)[0] is None  # no summary of that config at all


def test_committed_pmc_summaries_are_well_formed():
    # (round 1-2 summaries predate the sha256 key; bench.pmc_traffic skips them)
    paths = [p for p in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc_*.json")))
             if "so_sha256" in json.load(open(p))]
    assert len(paths) >= 3
    for p in paths:
        d = json.load(open(p))
        assert len(d["so_sha256"]) == 64, p
        assert d["traffic_per_frame_bytes"] > 0, p
        # the composite (C1-C4) or the FastMapper's two plane kernels (F2)
        want_k = ("fast_y_kernel", "fast_uv_kernel") if d.get("config") == "F2" else ("stitch_tiled_kernel",)
        assert all(any(w in k for k in d["traffic_bytes"]) for w in want_k), p
        # per launch: 2 x FETCH_SIZE + WRITE_SIZE, the medians over the profiled launches, KiB -> bytes
        if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
            for k, t in d["traffic_bytes"].items():
                f, w = d["FETCH_SIZE"].get(k), d["WRITE_SIZE"].get(k)
                if f and w:
                    want = (2 * f["kib_median"] + w["kib_median"]) * 1024
                    assert t == pytest.approx(want, rel=1e-6), (p, k)


def _kfd_tree(root, simds):
    for i, s in enumerate(simds):
        d = root / str(i)
        d.mkdir(parents=True)
        (d / "properties").write_text("cpu_cores_count %d\nsimd_count %d\nmax_waves_per_simd 8\n" % (0 if s else 64, s))


def test_visible_gpus_without_hip(tmp_path, monkeypatch):
    """The launcher parent counts GPUs from the KFD topology only: any HIP device query (which would
    initialise the runtime before the rank processes start) fails the test."""
    import torch
    import bench

    def no_hip(*a, **k):
        raise AssertionError("HIP queried by the launcher parent")
    monkeypatch.setattr(torch._C, "_cuda_getDeviceCount", no_hip, raising=False)
    monkeypatch.setattr(torch.cuda, "device_count", no_hip)
    monkeypatch.setattr(torch.cuda, "is_available", no_hip)
    nodes = tmp_path / "nodes"
    _kfd_tree(nodes, [0, 1024, 1024, 0, 1024])  # two CPU agents, three GPUs
    assert bench.visible_gpus(str(nodes), env={}) == 3
    assert bench.visible_gpus(str(nodes), env={"HIP_VISIBLE_DEVICES": "0,2"}) == 2
    assert bench.visible_gpus(str(nodes), env={"ROCR_VISIBLE_DEVICES": "1", "HIP_VISIBLE_DEVICES": "0,1"}) == 1
    assert bench.visible_gpus(str(nodes), env={"CUDA_VISIBLE_DEVICES": ""}) == 0
    with pytest.raises(RuntimeError):
        bench.visible_gpus(str(tmp_path / "absent"), env={})


def test_frame_sets_default_and_floor():
    """The timed steps rotate through at least 8 distinct source frame sets (more than the Infinity Cache
    holds for C2 / C4), never fewer than the frames in flight."""
    import argparse
    import bench
    a = argparse.Namespace(frame_sets=None)
    assert bench.frame_sets_of(a, 3) == 8 and bench.frame_sets_of(a, 12) == 12
    a.frame_sets = 2
    assert bench.frame_sets_of(a, 3) == 3


def test_derived_frame_sets_match_on_device_and_host():
    """bench.derive_set (torch, on the device in the bench) == synthetic.derived_frame (numpy, the tests'
    oracle inputs) byte for byte, and a derived set differs from its base."""
    import numpy as np
    import torch
    import bench
    from octvr_amd import synthetic
    base = [torch.from_numpy(synthetic.yuv_frame(w, h, 5 + i)) for i, (w, h) in enumerate([(64, 36), (300, 20)])]
    got = bench.derive_set(base, [1107, 1108])
    for i, t in enumerate(base):
        want = synthetic.derived_frame(t.numpy(), 1107 + i)
        assert np.array_equal(got[i].numpy(), want)
        assert (want != t.numpy()).mean() > 0.9


def test_preroll_runs_untimed_chunks_until_the_time_passes():
    """bench.preroll (the clock-settling steps before the timed region): whole
    synchronised chunks until `seconds` have passed, step indices consecutive from 0; none for 0 s."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import time
    import bench
    seen, syncs = [], []

    def step(k):
        seen.append(k)
        time.sleep(0.0005)

    n = bench.preroll(step, 0.05, lambda: syncs.append(len(seen)), chunk=16)
    assert n == len(seen) and n % 16 == 0 and n >= 16
    assert seen == list(range(n)) and syncs[-1] == n and all(s % 16 == 0 for s in syncs)
    assert bench.preroll(step, 0.0, lambda: None) == 0
