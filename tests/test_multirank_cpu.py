"""Multi-rank harness of bench.py on the CPU (gloo, world_size 2): one process per "GPU", each
stitching its own independent rig instance with no data-path collective, the timed
region bracketed by barriers and reduced with MAX over ranks, the value aggregated over ranks.

The per-rank stitch here is the oracle's (this container has no GPU); on the GPU box bench.py runs
the same harness around the HIP path under torch.distributed.run."""
import json
import os
import socket

import numpy as np
import pytest

import oracle_py as O


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank, world, port, out_dir):
    import time

    import torch.distributed as dist

    import bench
    from octvr_amd import synthetic

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rig, z = O.load_rig("rigA")
    W, H = (int(v) for v in z["out_size"])
    n = len(z["rois"])
    sizes = [(rig["inputs"][i]["options"]["width"], rig["inputs"][i]["options"]["height"]) for i in range(n)]
    frames = [synthetic.yuv_frame(w, h, bench.frame_seed(rank, 0, i)) for i, (w, h) in enumerate(sizes)]
    maps1 = [z[f"map1_{i}"] for i in range(n)]
    maps2 = [z[f"map2_{i}"] for i in range(n)]
    masks = [z[f"mask_{i}"] for i in range(n)]
    outs = []

    def step(k):
        out, g = O.stitch_frame(frames, sizes, z["rois"].tolist(), maps1, maps2, masks, W, H, enable_gain=True,
                                gains=None)
        outs.append((out, g))
        if rank == 1:
            time.sleep(0.05)  # the slower rank sets the job time

    steps = 3
    elapsed = bench.timed_region(step, steps, lambda: None, dist)
    digest = [int(np.frombuffer(outs[-1][0].tobytes(), np.uint8).astype(np.uint64).sum()), list(outs[-1][1])]
    with open(os.path.join(out_dir, "rank%d.json" % rank), "w") as f:
        json.dump({"elapsed": elapsed, "digest": digest, "steps": len(outs), "px": W * H,
                   "value": bench.aggregate_mps(world, steps, W * H, elapsed)}, f)
    dist.destroy_process_group()


def test_bench_harness_two_ranks_gloo(tmp_path):
    import torch.multiprocessing as mp
    world = 2
    mp.spawn(_rank_main, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    r = [json.load(open(tmp_path / ("rank%d.json" % k))) for k in range(world)]
    # the timed region is reduced with MAX: every rank reports the slowest rank's time
    assert r[0]["elapsed"] == r[1]["elapsed"]
    assert r[0]["elapsed"] >= 3 * 0.05
    assert all(x["steps"] == 3 for x in r)
    # independent rigs: frames seeded per rank, so the stitched outputs and the gains differ
    assert r[0]["digest"] != r[1]["digest"]
    # whole-job throughput counts every rank's frames
    assert r[0]["value"] == pytest.approx(world * 3 * r[0]["px"] / 1e6 / r[0]["elapsed"])


@pytest.mark.parametrize("n", [2, 8])
def test_bench_entry_point_standin(n):
    """bench.py's own `--gpus N` path (no WORLD_SIZE: bench.launch_ranks starts the ranks itself),
    with the oracle standing in for the HIP stitch: one JSON line, n_gpus N, every rank's frames, one
    local rank (device) per rank.  N = 8 is the driver's scaling run on a full node (SCALE_rNN), which
    this pool never lets a builder launch on GPUs: here it runs as 8 CPU ranks over gloo."""
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["OMP_NUM_THREADS"] = "1"
    p = subprocess.run([sys.executable, os.path.join(here, "bench_standin.py"), "--gpus", str(n), "--steps", "2",
                        "--warmup", "1"], env=env, capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == n and d["steps"] == 2
    assert sorted(r["rank"] for r in d["ranks"]) == list(range(n))
    assert sorted(r["local_rank"] for r in d["ranks"]) == list(range(n))
    assert all(r["frames"] == 2 for r in d["ranks"])
    assert len({r["digest"] for r in d["ranks"]}) == n  # independent rigs (rank-seeded frames)
    assert d["value"] == pytest.approx(n * 2 * d["frame_px"] / 1e6 / d["elapsed"])


def test_bench_entry_point_rejects_mismatch():
    """--gpus that disagrees with a launcher's WORLD_SIZE is an error, not a silent 1-GPU run."""
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(here, "bench_standin.py"), "--gpus", "2", "--steps", "1",
                        "--warmup", "0"], env=env, capture_output=True, text=True, timeout=120)
    assert p.returncode == 2 and "WORLD_SIZE=1" in p.stderr


def test_frame_seeds_are_distinct():
    import bench
    seeds = {bench.frame_seed(r, j, i) for r in range(8) for j in range(4) for i in range(16)}
    assert len(seeds) == 8 * 4 * 16


def test_bench_refuses_more_ranks_than_gpus():
    """bench.py --gpus N with fewer visible GPUs fails with a clear error before touching any GPU
    (this container has none, and no KFD topology: bench.visible_gpus says it cannot count them)."""
    import subprocess
    import sys
    import torch
    if torch.cuda.device_count() >= 2:
        pytest.skip("needs a host with fewer than 2 GPUs")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--steps", "1"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 2 and ("GPU(s) visible" in p.stderr or "cannot count GPUs" in p.stderr), p.stderr
