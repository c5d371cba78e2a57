"""bench.py's own entry point with a CPU stand-in for the per-rank GPU stitch (test infrastructure).

`python tests/bench_standin.py --gpus 2 --steps K --warmup W` goes through bench.main exactly as the
driver's `python bench.py --gpus N` does: with no WORLD_SIZE in the environment bench.launch_ranks
starts N copies of THIS script (sys.argv[0]) as ranks, each of which runs the harness (gloo barrier,
timed region, MAX over ranks, whole-job value) around the oracle's stitch of the rigA golden rig with
rank-seeded frames instead of the HIP mapper.  Rank 0 prints bench's one JSON line; the stand-in adds
what every rank did (frames stitched, output digest) so the test can see both ranks' work.
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "opencv-octvr_amd"))

import numpy as np  # noqa: E402

import bench  # noqa: E402


def standin_rank(args, world, rank, local_rank, dist):
    import torch

    import oracle_py as O
    from octvr_amd import synthetic

    rig, z = O.load_rig("rigA")
    W, H = (int(v) for v in z["out_size"])
    n = len(z["rois"])
    sizes = [(rig["inputs"][i]["options"]["width"], rig["inputs"][i]["options"]["height"]) for i in range(n)]
    frames = [synthetic.yuv_frame(w, h, bench.frame_seed(rank, 0, i)) for i, (w, h) in enumerate(sizes)]
    maps = [(z["map1_%d" % i], z["map2_%d" % i], z["mask_%d" % i]) for i in range(n)]
    done = []

    def step(k):
        out, g = O.stitch_frame(frames, sizes, z["rois"].tolist(), [m[0] for m in maps], [m[1] for m in maps],
                                [m[2] for m in maps], W, H, enable_gain=True, gains=None)
        done.append(int(np.frombuffer(out.tobytes(), np.uint8).astype(np.uint64).sum()))

    for k in range(args.warmup):
        step(k)
    del done[:]
    elapsed = bench.timed_region(step, args.steps, lambda: None, dist)
    # the stand-in's own record of every rank's work (bench itself moves no data between ranks)
    per_rank = [None] * world
    mine = {"rank": rank, "local_rank": local_rank, "frames": len(done), "digest": done[-1]}
    if dist:
        dist.all_gather_object(per_rank, mine)
    else:
        per_rank = [mine]
    return {"metric": "stitched megapixels/sec (stand-in)", "value": bench.aggregate_mps(world, args.steps, W * H, elapsed),
            "unit": "MP/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": elapsed * 1e3 / args.steps, "frame_px": W * H, "elapsed": elapsed,
            "ranks": per_rank, "torch": torch.__version__}


if __name__ == "__main__":
    bench.main(rank_body=standin_rank, check_devices=False)
