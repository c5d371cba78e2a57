#!/usr/bin/env python3
"""bench.py — stitched megapixels/s of the octVR remap + gain + composite path on MI355X.

Workload (BASELINE.json configs[1], SURVEY.md §8d "C2"): 6 x 3840x2160 fullframe_fisheye YUV420P
frames -> 7680x3840 equirectangular YUV420P, per-frame gain estimation (GainCompensatorGPU::feed +
apply) and the no-blend composite (mapper.cpp:193-312).  A step = one Mapper::stitch of one frame
set, inputs and outputs resident in HBM.  Multi-GPU: one process per GPU, each stitches its own
independent rig (rigs shard with no collective) -> "scaling": "weak".

Prints ONE JSON line on rank 0.  Extra objects: "roofline" (the composite kernel, HIP-event timed
live over the timed region) and "cpu_baseline" (the oracle restatement of the reference CPU path,
timed on this host).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config C2] [--no-cpu-baseline] [--preroll S]

K timed steps (default 1,000) follow W warmup steps and S seconds (default 0.5) of untimed preroll steps,
so that the timed region runs at the GPU's settled clock.

Diagnostics (Mapper configs; DESIGN.md §4 Round 6, "The 20-step region"): OCTVR_BENCH_STEP_MARKS=<file> appends
the host time at which each timed step returned, the GPU span between markers at the region's ends and every
composite's event interval; OCTVR_BENCH_NO_TIMING=1 times the region without the composites' event pairs (its
kernel_us is then the wall time, not a roofline figure).
"""
import argparse
import json
import math
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "opencv-octvr_amd"))

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one GPU each); without a launcher's WORLD_SIZE, bench.py starts them itself")
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="C2")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--inflight", type=int, default=None,
                    help="frames in flight: independent frame sets stitched round-robin on this many streams "
                         "(octvr_mapper_set_frames_in_flight); default per config, DEFAULT_INFLIGHT")
    ap.add_argument("--frame-sets", type=int, default=None,
                    help="distinct source frame sets rotated through the timed region (default 8, at least the "
                         "frames in flight): 8 C2 sets are 600 MB, more than the 256 MB Infinity Cache, so every "
                         "step reads its sources from HBM as a live pipeline's fresh frames would be")
    ap.add_argument("--no-async-e2e", action="store_true",
                    help="skip the AsyncMultiMapper end-to-end (PCIe-inclusive) measurement")
    ap.add_argument("--pmc-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--no-gain", action="store_true", help=argparse.SUPPRESS)  # diagnostic: composite alone
    ap.add_argument("--preroll", type=float, default=0.5,
                    help="seconds of untimed steps after the warmup steps, so that the timed steps run at the "
                         "GPU's settled clock (it idles during setup and takes ~0.1 s to ramp, DESIGN.md §4)")
    ap.add_argument("--batch", type=int, default=None, choices=[1, 2, 4],
                    help="frames per composite launch (octvr_mapper_stitch_batch: each frame its own gain feed, one "
                         "pass over the tiled LUT for all of them); a step is still one frame (default per config, "
                         "DEFAULT_BATCH)")
    ap.add_argument("--remap", default="remap", choices=["remap", "texture"],
                    help="sampling: cv::remap's fixed point (default) or the CUDA texture convention (OCTVR_REMAP_TEXTURE)")
    return ap.parse_args()


def preroll(step, seconds, sync, chunk=256):
    """Untimed steps until `seconds` have passed (in chunks, each synchronised, so the host never queues
    more than a chunk ahead): the GPU's shader clock falls while the host sets up and ramps back over ~0.1 s
    of load, which a timed region of a few milliseconds would otherwise partly measure.  Returns the
    steps run."""
    n = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        for _ in range(chunk):
            step(n)
            n += 1
        sync()
    return n


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def host_threads():
    n = os.environ.get("OMP_NUM_THREADS")
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count() or 1
    return max(1, min(int(n) if n else avail, avail, 64))


def frame_seed(rank, slot, cam):
    """Seed of camera `cam`'s synthetic frame for in-flight slot `slot` on rank `rank`: every rank
    stitches its own independent rig instance."""
    return 1000 * (rank + 1) + 100 * slot + cam


def derive_set(base, seeds):
    """Frame set from a base set on the device: camera i's frame XOR synthetic.frame_key(seeds[i]) repeated
    over its bytes (synthetic.derived_frame, byte for byte) — distinct uniform-random content in milliseconds
    instead of a host splitmix pass per 4K frame."""
    import torch
    from octvr_amd import synthetic
    out = []
    for t, sd in zip(base, seeds):
        key = torch.from_numpy(synthetic.frame_key(sd)).to(t.device)
        flat = t.reshape(-1)
        reps = (flat.numel() + key.numel() - 1) // key.numel()
        out.append(torch.bitwise_xor(flat, key.repeat(reps)[:flat.numel()]).reshape(t.shape))
    return out


ISSUE_S = [0.0]  # host time the last timed_region spent issuing its steps (before the final sync)


def timed_region(step, steps, sync, dist=None):
    """Exactly `steps` calls of step(k), bracketed by a barrier + device sync on both sides; returns
    the MAX over ranks of the elapsed wall time (the job is as slow as its slowest rank).  The host time
    spent issuing the steps is left in ISSUE_S[0]: close to the elapsed time means the host, not the
    GPU, set the pace."""
    if dist:
        dist.barrier()
    sync()
    marks = os.environ.get("OCTVR_BENCH_STEP_MARKS")  # diagnostic: the host time at which each step returned
    if marks:
        tk = [0.0] * steps
        t0 = time.perf_counter()
        for k in range(steps):
            step(k)
            tk[k] = time.perf_counter()
    else:
        t0 = time.perf_counter()
        for k in range(steps):
            step(k)
    ISSUE_S[0] = time.perf_counter() - t0
    sync()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if marks:
        with open(marks, "a") as f:
            f.write(json.dumps({"steps": steps, "elapsed_us": elapsed * 1e6,
                                "step_end_us": [round((t - t0) * 1e6, 1) for t in tk]}) + "\n")
    if dist:
        import torch
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t[0])
    return elapsed


def aggregate_mps(world, steps, frame_px, elapsed):
    """Whole-job throughput: every rank stitched `steps` frames of `frame_px` output pixels."""
    return world * steps * frame_px / 1e6 / elapsed


def lib_sha256():
    import hashlib
    p = os.path.join(ROOT, "opencv-octvr_amd", "lib", "liboctvr_hip.so")
    with open(p, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


def pmc_traffic(config, blend, nb=1):
    """(bytes, source) — per composite launch (blend 0) or per frame over the blend sequence (blend > 0:
    the remap, pyrDown and blend launches, i.e. what bytes_per_launch models and kernel_us times; the gain
    feed runs before the sequence and is excluded as for blend 0) — from the profiles/*_pmc_<config>.json
    whose so_sha256 is the running library's and whose launches stitched nb frames each (per frame: / nb);
    (None, reason) when no summary of this binary exists."""
    import glob
    sha = lib_sha256()
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc_%s.json" % config))):
        d = json.load(open(path))
        if d.get("so_sha256") != sha or d.get("frames_per_launch", 1) != nb:
            continue
        if blend > 0:
            seq = [v for k, v in d.get("traffic_bytes", {}).items() if "gain_feed" not in k]
            if seq:
                return round(sum(seq) / nb), os.path.basename(path)
            continue
        hit = [v for k, v in d.get("traffic_bytes", {}).items() if "stitch_tiled_kernel" in k]
        if hit:
            return round(hit[0] / nb), os.path.basename(path)
        if config == "F2":
            fast = [v for k, v in d.get("traffic_bytes", {}).items() if "fast_" in k]
            if fast:
                return round(sum(fast) / nb), os.path.basename(path)
    return None, "no PMC summary of this liboctvr_hip.so (sha256 %s...)" % sha[:12]


def pmc_valu_busy(config):
    """Bounds on the composite's VALU issue share from the PMC summary of this binary (one launch alone
    under rocprofv3, which serialises dispatches).  SIMD cycles of the launch = GRBM_GUI_ACTIVE / 8 XCDs x
    1,024 SIMDs.  Upper bound: SQ_ACTIVE_INST_VALU (quad-cycles) x 4 — the counter charges about one
    quad-cycle per VALU instruction, the issue cost of one wave alone; lower bound: SQ_INSTS_VALU x 2, the
    SIMD-32's cost of a wave64 instruction when two or more waves share the SIMD (MI355X_MICROARCH.md,
    Execution model and the per-instruction table).  Slow opcodes of this loop (v_perm, v_dot2, the packed
    forms) sit between the two.  None without such a summary."""
    import glob
    sha = lib_sha256()
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc_%s.json" % config))):
        d = json.load(open(path))
        if d.get("so_sha256") != sha:
            continue
        for k, cs in d.get("counters", {}).items():
            if "stitch_tiled_kernel" in k and "SQ_ACTIVE_INST_VALU" in cs and "GRBM_GUI_ACTIVE" in cs:
                a, g = cs["SQ_ACTIVE_INST_VALU"]["median"], cs["GRBM_GUI_ACTIVE"]["median"]
                simd_cycles = g / 8.0 * 1024.0
                r = {"upper": round(a * 4.0 / simd_cycles, 3), "source": os.path.basename(path),
                     "note": "share of the launch's SIMD cycles spent issuing VALU, bounded: upper = "
                             "SQ_ACTIVE_INST_VALU quad-cycles x 4 (4 cycles per instruction), lower = SQ_INSTS_VALU x 2 "
                             "(2 cycles per wave64 instruction on a shared SIMD-32)"}
                if "SQ_INSTS_VALU" in cs:
                    r["lower"] = round(cs["SQ_INSTS_VALU"]["median"] * 2.0 / simd_cycles, 3)
                return r
    return None


def async_e2e(ox, mt, sizes, W, H, blend, frames_np, dev, frames=64, gain=True, remap="remap"):
    """AsyncMultiMapper end to end (async.cpp:32-193): host YUV420P planes pushed, the bytes the mapper
    reads (its source footprint) copied into pinned staging and uploaded, stitched, downloaded and copied
    out, 3 frames in flight (the reference's BUF_SIZE, async.cpp:261-310), with the line's own sampling
    and gain mode.  PCIe-inclusive: reported beside `value`, never as it."""
    import numpy as np
    am = ox.AsyncMultiMapper([mt], sizes, (W, H), [blend], [0 if gain else -1], [(0.0, 0.0, 1.0, 1.0)], device=dev,
                             remap=remap)
    info = am.info()
    ins = [(f[:h], f[h:, :w // 2], f[h:, w // 2:]) for f, (w, h) in zip(frames_np, sizes)]
    outs = [(np.empty((H, W), np.uint8), np.empty((H // 2, W // 2), np.uint8), np.empty((H // 2, W // 2), np.uint8))
            for _ in range(4)]
    for o in outs:  # a ring of output frames the caller reuses: downloaded straight into (no copy-out)
        am.register_output(o)

    def run(n):
        for k in range(n):
            am.push(ins, outs[k % 4])
            if am.pending() >= 3:
                am.pop()
        while am.pending():
            am.pop()

    run(4)  # warm-up: pinned buffers, first-touch
    t0 = time.perf_counter()
    run(frames)
    dt = time.perf_counter() - t0
    am.close()
    in_b = sum(w * h * 3 // 2 for w, h in sizes)
    return {"value": round(frames * W * H / 1e6 / dt, 1), "unit": "MP/s", "ms_per_frame": round(dt * 1e3 / frames, 3),
            "frames": frames, "input_bytes_per_frame": in_b,
            "h2d_bytes_per_frame": int(info["packed_bytes"]), "d2h_bytes_per_frame": info["output_bytes"],
            "gain": "estimated" if gain else "none", "remap": remap,
            "note": "AsyncMultiMapper push->pop of host YUV420P planes: copy-in of the mapper's source footprint to "
                    "pinned staging, H2D, unpack, stitch, D2H straight into the caller's registered output ring "
                    "(octvr_async_register_output), 3 frames in flight; PCIe- and host-copy-inclusive, not the "
                    "roofline basis"}


# frames in flight per config, from interleaved sweeps on one box (scripts/r4_inflight_sweep.sh): C2 2 / 3 / 4 =
# 496k / 607k / 550k MP/s, C3 172k / 178k / 184k, C4 564k / 585k / 578k, C1 371k / 483k / 485k (3 kept: the
# two 4s were 511k and 459k), F2 (stitch_nv12 on 1 / 2 / 3 streams) 85k / 91k / 93k
DEFAULT_INFLIGHT = {"C3": 4, "F2": 3}
DEFAULT_INFLIGHT_BATCHED = {"F2": 1}  # streams when frames are batched (default 2)
# frames per composite launch (octvr_mapper_stitch_batch), no-blend configs only; interleaved on one box at
# 1,000 steps: C1 1 x 3 streams / 2 x 2 / 4 x 2 = 548k-568k / 573k-614k / 809k-813k MP/s,
# C4 739k-742k / 792k-794k / 819k-820k, C2 707k / 636k / 654k (C2 stays one frame per launch)
# F2 (FastMapper, one launch per plane): 1 x 3 streams 112k, 2 x 2 111k, 4 x 1 134k, 4 x 2 126k MP/s
DEFAULT_BATCH = {"C1": 4, "C4": 4, "F2": 4}
CPU_BASELINE_S = float(os.environ.get("OCTVR_CPU_BASELINE_S", "10"))
DEFAULT_FRAME_SETS = 8


def frame_sets_of(args, inflight):
    """Distinct source frame sets the timed steps rotate through: --frame-sets, default 8, never fewer
    than the frames in flight (a set is in use by one in-flight stitch at a time)."""
    return max(inflight, args.frame_sets if args.frame_sets is not None else DEFAULT_FRAME_SETS)


def cpu_baseline(mt, frames_np, sizes, W, H, blend=0, gain=True):
    """The reference CPU path restated by the oracle (YUV->RGBA, fixed-point cv::remap of every
    camera over its full ROI, gain feed + apply, copyTo(mask) or the multi-band blender,
    RGB->YUV420P) on this host.  gain=False: the C1 plumbing case (cv::remap + the seam-mask copy)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_py as O  # test infrastructure: used only as the timed CPU baseline
    rois, m1s, m2s, masks, seams = [], [], [], [], []
    for i in range(len(sizes)):
        roi, m1, m2, mk, sm = mt.input(i)
        rois.append(roi); m1s.append(m1); m2s.append(m2); masks.append(mk); seams.append(sm)
    T = host_threads()
    # whole frames back to back until about CPU_BASELINE_S seconds of CPU work (at least one frame)
    n, t0 = 0, time.perf_counter()
    while True:
        O.stitch_frame(frames_np, sizes, rois, m1s, m2s, masks, W, H, enable_gain=gain, gains=None, threads=T,
                       blend=blend, seams=seams if blend > 0 else None)
        n += 1
        dt = time.perf_counter() - t0
        if dt >= CPU_BASELINE_S or n >= 1000:
            break
    r = {"value": round(n * W * H / 1e6 / dt, 3), "unit": "MP/s", "cores": T, "kind": "port",
         "sample": "%d full %dx%d frames (%d cameras, %s%s) through the oracle (oracle/*.c), "
                   "%.2f s, host CPU: %s" % (n, W, H, len(sizes), "gain estimated" if gain else "no gain",
                                              ", multi-band blend=%d" % blend if blend else "", dt, cpu_model())}
    if not gain and blend == 0 and len(sizes) == 2:
        r["survey_reference"] = ("SURVEY.md §6: the reference's own CPU cv::remap + seam copy at this geometry, "
                                 "192-204 MP/s on 8 threads of an 8-core Xeon VM (YUV<->RGB not included there)")
    return r


def visible_gpus(kfd_nodes="/sys/class/kfd/kfd/topology/nodes", env=None):
    """Number of GPUs this process may use, counted without any HIP call: the parent of a multi-rank
    launch must not touch the GPU before it starts its ranks (torch.cuda.device_count() falls back to
    hipGetDeviceCount when amdsmi cannot enumerate).  GPU agents are the KFD topology nodes with SIMDs
    (simd_count > 0), narrowed by ROCR_VISIBLE_DEVICES / HIP_VISIBLE_DEVICES / CUDA_VISIBLE_DEVICES as
    the runtime narrows them.  Raises RuntimeError when the topology is unreadable."""
    env = os.environ if env is None else env
    try:
        names = sorted(os.listdir(kfd_nodes), key=lambda x: int(x) if x.isdigit() else -1)
    except OSError as e:
        raise RuntimeError("bench.py: cannot count GPUs without HIP: %s unreadable (%s)" % (kfd_nodes, e))
    n = 0
    for name in names:
        try:
            with open(os.path.join(kfd_nodes, name, "properties")) as f:
                props = dict(line.split()[:2] for line in f if len(line.split()) >= 2)
        except OSError:
            continue
        if int(props.get("simd_count", "0")) > 0:
            n += 1
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = env.get(var)
        if v is not None:  # each narrows the list the previous one left
            ids = [x for x in v.split(",") if x.strip() != ""]
            n = min(n, len(ids)) if v.strip() else 0
    return n


def launch_ranks(n, argv, check_devices=True):
    """`bench.py --gpus N` without a launcher: start N rank processes of this same script (one per
    GPU, SURVEY.md §8e: independent rigs, no data-path collective), each with RANK / LOCAL_RANK /
    WORLD_SIZE / MASTER_ADDR / MASTER_PORT in its environment, and wait for them.  Rank 0 prints the
    one JSON line.  Runs before anything touches the GPU; returns the worst child exit status."""
    import socket
    if check_devices:
        try:
            have = visible_gpus()
        except RuntimeError as e:
            sys.stderr.write("%s\n" % e)
            return 2
        if n > have:
            sys.stderr.write("bench.py: --gpus %d but only %d GPU(s) visible\n" % (n, have))
            return 2
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(argv[0])] + list(argv[1:]), env=env))
    # a rank that fails leaves the others waiting in a barrier: stop them, and report its status
    while True:
        rcs = [p.poll() for p in procs]
        bad = [c for c in rcs if c not in (None, 0)]
        if bad or all(c is not None for c in rcs):
            break
        time.sleep(0.2)
    for p in procs:
        if p.poll() is None:
            p.terminate()
    for p in procs:
        try:
            p.wait(timeout=30)
        except subprocess.TimeoutExpired:
            p.kill()
            p.wait()
    return bad[0] if bad else 0


def main(rank_body=None, check_devices=True):
    """rank_body(args, world, rank, local_rank, dist) -> result dict (rank 0) — the GPU stitch by
    default; tests/bench_standin.py passes a CPU stand-in to exercise the launcher and the harness."""
    args = parse()
    if "WORLD_SIZE" not in os.environ and (args.gpus or 1) > 1:
        sys.exit(launch_ranks(args.gpus, sys.argv, check_devices))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus is not None and world != args.gpus:
        sys.stderr.write("bench.py: --gpus %d but WORLD_SIZE=%d\n" % (args.gpus, world))
        sys.exit(2)
    dist = None
    if world > 1:
        import torch.distributed as dist
        # no data-path collective: gloo carries only the barrier and the max-over-ranks time
        dist.init_process_group("gloo")
    result = (rank_body or gpu_rank)(args, world, rank, local_rank, dist)
    if rank == 0:
        assert result["n_gpus"] == world
        print(json.dumps(result), flush=True)
    if dist:
        dist.destroy_process_group()


def nv12_of(yuv420p):
    """The same frame as NV12 (interleaved U, V rows), as FastMapper takes it."""
    import numpy as np
    h = yuv420p.shape[0] * 2 // 3
    w = yuv420p.shape[1]
    m = np.empty_like(yuv420p)
    m[:h] = yuv420p[:h]
    m[h:, 0::2] = yuv420p[h:, : w // 2]
    m[h:, 1::2] = yuv420p[h:, w // 2:]
    return m


def fast_rank(args, world, rank, local_rank, dist):
    """--config F2: vr::FastMapper::stitch_nv12 (mapper_fast.cpp:153-195) on the C2 rig built without ROI
    (octvr_dump -n), NV12 in / out, feather weights; a step = one stitch_nv12 of one frame set."""
    import torch
    import octvr_amd as ox
    from octvr_amd import synthetic

    torch.cuda.set_device(local_rank)
    dev = local_rank
    rig, W, H, sizes = synthetic.CONFIGS[args.config]()
    mt = ox.MapperTemplate.from_json(json.dumps(rig), W, H, use_roi=False, device=dev)
    fm = ox.FastMapper(mt, sizes, device=dev)
    # stitch_nv12 keeps no per-call device state, so a caller may run several at once on their own
    # streams and outputs (frames in flight, as the Mapper configs do through set_frames_in_flight)
    nb = args.batch if args.batch is not None else DEFAULT_BATCH.get(args.config, 1)
    if args.steps % nb:
        raise SystemExit("bench.py: --steps must be a multiple of --batch")
    inflight = max(1, args.inflight if args.inflight is not None else
                   (DEFAULT_INFLIGHT_BATCHED.get(args.config, 2) if nb > 1 else DEFAULT_INFLIGHT.get(args.config, 1)))
    nsets = frame_sets_of(args, inflight * nb)
    # distinct frame sets (seeded by rank, set, camera), rotated through the steps as the Mapper configs do
    frame_sets = [[torch.from_numpy(nv12_of(synthetic.yuv_frame(w, h, frame_seed(rank, 0, i)))).to(f"cuda:{dev}")
                   for i, (w, h) in enumerate(sizes)]]
    for j in range(1, nsets):
        frame_sets.append(derive_set(frame_sets[0], [frame_seed(rank, j, i) for i in range(len(sizes))]))
    frames = frame_sets[0]
    outs = [torch.empty((H * 3 // 2, W), dtype=torch.uint8, device=f"cuda:{dev}") for _ in range(inflight * nb)]
    streams = [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(dev) for _ in range(inflight - 1)]
    stream, out = streams[0], outs[0]

    refs = [ox.Mapper.frame_refs(fs) for fs in frame_sets]
    import ctypes
    raw_streams = [ctypes.c_void_p(st.cuda_stream) for st in streams]
    ncalls = nsets * inflight
    brefs = [ox.Mapper.batch_refs([refs[(c * nb + f) % nsets] for f in range(nb)],
                                  outs[(c % inflight) * nb:(c % inflight + 1) * nb]) for c in range(ncalls)] if nb > 1 else None

    def step(k):  # one call: one frame (nb = 1) or a batch of nb frames
        if nb == 1:
            fm.stitch_nv12(refs[k % nsets], outs[k % inflight], stream=raw_streams[k % inflight])
        else:
            fm.stitch_nv12_batch(brefs[k % ncalls], stream=raw_streams[k % inflight])

    if args.pmc_child:
        for k in range(max(args.steps // nb, 1)):  # calls of nb frames
            step(k)
        torch.cuda.synchronize(dev)
        sys.exit(0)
    for k in range(max(args.warmup, inflight, nsets)):  # every stream and frame set once outside the timed region
        step(k)
    torch.cuda.synchronize(dev)
    n_pre = preroll(step, args.preroll, lambda: torch.cuda.synchronize(dev))
    elapsed = timed_region(step, args.steps // nb, lambda: torch.cuda.synchronize(dev), dist)
    # kernel time: events around 16 back-to-back stitches (both plane launches) on one stream, after the
    # timed region (one frame per launch)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for k in range(16 // nb):  # 16 frames, nb per launch
        if nb == 1:
            fm.stitch_nv12(frames, out, stream=stream)
        else:
            fm.stitch_nv12_batch(brefs[(k * inflight) % ncalls], stream=stream)
    e1.record(stream)
    torch.cuda.synchronize(dev)
    kern_s = e0.elapsed_time(e1) / 1e3 / 16
    lut_b, frame_b = fm.traffic_parts()
    b = lut_b / nb + frame_b  # per frame: the entries are read once per launch of nb frames
    traffic, traffic_src = pmc_traffic(args.config, 1, nb)
    result = {
        "metric": "stitched megapixels/sec (6x4K->8K equirect, FastMapper NV12)",
        "value": round(aggregate_mps(world, args.steps, W * H, elapsed), 1), "unit": "MP/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "preroll": {"s": args.preroll, "steps": n_pre}, "ms_per_step": round(elapsed * 1e3 / args.steps, 4),
        "host_issue_ms_per_step": round(ISSUE_S[0] * 1e3 / args.steps, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic (splitmix64 frames as NV12, further sets derived by a splitmix64 key, SURVEY.md §8d rig)",
        "config": {"workload": "F2: %d x %dx%d fullframe_fisheye -> %dx%d, vr::FastMapper::stitch_nv12 (feather, "
                               "template without ROI), NV12 in/out" % (len(sizes), sizes[0][0], sizes[0][1], W, H),
                   "rigs_per_gpu": 1, "frames_in_flight": inflight * nb, "streams": inflight, "frames_per_launch": nb,
                   "frame_sets": nsets, "parallelism": "independent rig per GPU"},
        "roofline": {"bound": "hbm", "achieved": round(b / kern_s / 1e9, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": round(b / kern_s / 1e9 / HBM_PEAK_GBPS, 4), "traffic": traffic, "traffic_source": traffic_src,
                     "kernel": "fast_y_kernel + fast_uv_kernel", "kernel_us": round(kern_s * 1e6, 2),
                     "kernel_us_basis": "torch events around 16 back-to-back frames (%d per launch) on one stream, per frame" % nb,
                     "bytes_per_launch": b,
                     "bytes_basis": "per (camera, 256-px run) entry block pixel 5 B (compact entry + weight; 8 B per "
                                    "block header) or 8 B (wide planes), read once per launch of %d frames; 1.5 B out "
                                    "per px, source bytes the weighted taps reach (octvr_fastmapper_traffic_parts)" % nb,
                     "frac_at_step_time": round(b / (elapsed / args.steps) / 1e9 / HBM_PEAK_GBPS, 4),
                     "frac_traffic": round(traffic / kern_s / 1e9 / HBM_PEAK_GBPS, 4) if traffic else None},
    }
    # (no cpu_baseline: F2 is not a BASELINE configuration, and the oracle's FastMapper restatement
    # rebuilds the per-rig feather weights inside every call)
    return result


def gpu_rank(args, world, rank, local_rank, dist):
    import numpy as np  # noqa: F401
    import torch
    import octvr_amd as ox
    from octvr_amd import synthetic

    if args.config == "F2":
        return fast_rank(args, world, rank, local_rank, dist)
    torch.cuda.set_device(local_rank)
    dev = local_rank

    rig, W, H, sizes = synthetic.CONFIGS[args.config]()
    blend = synthetic.BLEND[args.config]
    mt = ox.MapperTemplate.from_json(json.dumps(rig), W, H, use_roi=True, device=dev)
    if blend > 0:
        mt.create_masks(dev)  # MapperTemplate::create_masks (DistanceSeamFinder), as octvr_dump does
    use_gain = synthetic.GAIN[args.config] and not args.no_gain
    m = ox.Mapper(mt, sizes, blend=blend, enable_gain=use_gain, device=dev, remap=args.remap)
    # frames in flight: like a capture pipeline, frame k+1 (its own buffers, its own stream) is issued
    # while frame k is still stitching, so frame k+1's gain feed overlaps frame k's composite
    # frames per composite launch: a batch of nb frames per call on each of the `inflight` streams
    nb = args.batch if args.batch is not None else (DEFAULT_BATCH.get(args.config, 1) if blend == 0 else 1)
    inflight = max(1, args.inflight if args.inflight is not None else
                   (DEFAULT_INFLIGHT_BATCHED.get(args.config, 2) if nb > 1 else DEFAULT_INFLIGHT.get(args.config, 3)))
    if blend != 0 and nb != 1:
        raise SystemExit("bench.py: --batch needs the no-blend composite (multi-band / feather stitch frame by frame)")
    if args.steps % nb:
        raise SystemExit("bench.py: --steps must be a multiple of --batch")
    m.set_frames_in_flight(inflight * nb)
    # each rank stitches an independent rig instance: frames seeded by (rank, frame set, camera); the
    # steps rotate through nsets distinct sets (> 256 MB of sources for C2 / C4 at the default 8, so the
    # Infinity Cache cannot keep them between steps)
    nsets = frame_sets_of(args, inflight * nb)
    frames_np = [synthetic.yuv_frame(w, h, frame_seed(rank, 0, i)) for i, (w, h) in enumerate(sizes)]
    frame_sets = [[torch.from_numpy(f).to(f"cuda:{dev}") for f in frames_np]]
    for j in range(1, nsets):
        frame_sets.append(derive_set(frame_sets[0], [frame_seed(rank, j, i) for i in range(len(sizes))]))
    outs = [torch.empty((H * 3 // 2, W), dtype=torch.uint8, device=f"cuda:{dev}") for _ in range(inflight * nb)]
    streams = [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(dev) for _ in range(inflight - 1)]
    # the frame sets' pointers marshalled once, raw stream handles (a capture ring reuses its buffers)
    refs = [ox.Mapper.frame_refs(fs) for fs in frame_sets]
    import ctypes
    raw_streams = [ctypes.c_void_p(st.cuda_stream) for st in streams]
    # batches: call c takes frame sets c nb .. c nb + nb - 1 (mod nsets) and the outputs of its stream
    ncalls = nsets * inflight
    brefs = [ox.Mapper.batch_refs([refs[(c * nb + f) % nsets] for f in range(nb)],
                                  outs[(c % inflight) * nb:(c % inflight + 1) * nb]) for c in range(ncalls)] if nb > 1 else None

    def step(k):  # one call: one frame (nb = 1) or a batch of nb frames
        j = k % inflight
        if nb == 1:
            m.stitch(refs[k % nsets], outs[j], stream=raw_streams[j])
        else:
            m.stitch_batch(brefs[k % ncalls], stream=raw_streams[j])

    if args.pmc_child:  # a few launches for rocprofv3 --pmc passes
        for k in range(max(args.steps // nb, 1)):  # calls of nb frames
            step(k)
        torch.cuda.synchronize(dev)
        sys.exit(0)

    # setup: one stitch per stream first, so every stream's hardware queue exists before the W warmup
    # steps (the first launch on a new stream costs ~8 ms: with W < inflight it used to land inside the
    # timed region — the "four in flight" cliff of round 2, profiles/r03_kt_inflight_cliff.md)
    for j in range(max(inflight, nsets)):  # (and every frame set once: no first touch in the timed region)
        step(j)
    torch.cuda.synchronize(dev)
    for k in range(args.warmup):
        step(k)
    torch.cuda.synchronize(dev)
    n_pre = preroll(step, args.preroll, lambda: torch.cuda.synchronize(dev))
    m.kernel_time()  # drop anything recorded before the timed region
    # HIP events around the composite.  One frame in flight: every 4th step (an event pair costs ~5 us
    # of that stream's timeline).  Several: every step on every stream, so the union of the launches'
    # intervals (the wall time some composite was running) is known; a launch's own start-to-end
    # span then also covers the other streams' kernels beside it.
    if not os.environ.get("OCTVR_BENCH_NO_TIMING"):  # diagnostic: the timed region without the event pairs
        m.set_timing(1 if inflight > 1 or nb > 1 else 4)
    marks = os.environ.get("OCTVR_BENCH_STEP_MARKS")
    if marks:  # diagnostic: GPU markers at the region's first step (stream 0) and after its last (every stream)
        ev_a = torch.cuda.Event(enable_timing=True)
        ev_z = [torch.cuda.Event(enable_timing=True) for _ in streams]
        syncs = [0]

        def step_m(k):
            if k == 0:
                ev_a.record(streams[0])
            step(k)

        def sync_m():
            if syncs[0] == 1:
                for e, st in zip(ev_z, streams):
                    e.record(st)
            syncs[0] += 1
            torch.cuda.synchronize(dev)
        elapsed = timed_region(step_m, args.steps // nb, sync_m, dist)
        with open(marks, "a") as f:
            f.write(json.dumps({"gpu_region_us": max(ev_a.elapsed_time(e) for e in ev_z) * 1e3}) + "\n")
    else:
        elapsed = timed_region(step, args.steps // nb, lambda: torch.cuda.synchronize(dev), dist)
    m.set_timing(False)
    if marks:  # diagnostic: every timed launch's GPU interval beside the host marks
        iv = m.kernel_intervals()
        with open(marks, "a") as f:
            f.write(json.dumps({"kernel_ms": [[round(a, 4), round(b, 4)] for a, b in iv]}) + "\n")
        span_ms, busy_ms = ox.interval_union([a for a, _ in iv], [b for _, b in iv])
        launches = len(iv)
    else:
        span_ms, busy_ms, launches = m.kernel_busy()
    kern_ms = busy_ms if inflight > 1 else span_ms
    if launches == 0:  # (OCTVR_BENCH_NO_TIMING) no events: the wall time stands in
        kern_ms, launches = elapsed * 1e3, args.steps // nb
    launches *= nb  # per frame: a batched launch stitches nb frames
    serial = serial_step = None
    if inflight > 1 and not dist:
        # supplementary, after the timed region: the composite kernel's duration with one frame in
        # flight (with two, the events on a stream also span the other stream's kernels).  The mapper
        # goes back to one slot, so no next frame's gain feed runs beside the measured composites.
        m.set_frames_in_flight(1)
        for k in range(2):
            m.stitch(frame_sets[0], outs[0], stream=streams[0])
        torch.cuda.synchronize(dev)
        m.kernel_time()
        m.set_timing(1)
        for k in range(8):
            m.stitch(frame_sets[0], outs[0], stream=streams[0])
        torch.cuda.synchronize(dev)
        s_ms, s_n = m.kernel_time()
        m.set_timing(False)
        serial = s_ms / 1e3 / max(s_n, 1)
        t0 = time.perf_counter()  # and the wall time per frame of serial stitches (feed + composite)
        for k in range(16):
            m.stitch(frame_sets[0], outs[0], stream=streams[0])
        torch.cuda.synchronize(dev)
        serial_step = (time.perf_counter() - t0) / 16

    gains = m.gains()
    frame_px = W * H
    value = aggregate_mps(world, args.steps, frame_px, elapsed)
    lut_b, frame_b = m.traffic_parts()
    bytes_per_launch = lut_b / nb + frame_b  # per frame: the tiled LUT is read once per launch of nb frames
    avg_kernel_s = kern_ms / 1e3 / max(launches, 1)
    achieved = bytes_per_launch / avg_kernel_s / 1e9
    n_valid = 0
    for i in range(len(sizes)):
        n_valid += int((mt.input(i)[3] > 0).sum())
    survey_b_alg = 1.5 * sum(w * h for w, h in sizes) + 9.0 * n_valid + 1.5 * frame_px
    if blend > 0:  # SURVEY.md §8d multi-band term: s16x3 Laplacian levels 1..B + f32 weight pyramids
        f = sum(4.0 ** -l for l in range(1, int(math.ceil(math.log(blend) / math.log(2.)) - 1) + 1))
        survey_b_alg += 12.0 * f * frame_px + 4.0 * f * n_valid

    # HBM traffic of the dominant kernel(s) from the committed PMC summary of THIS binary and config
    # (scripts/pmc.sh + scripts/pmc_summary.py record the sha256 of the profiled liboctvr_hip.so;
    # rocprofv3 cannot wrap the process that reads the counters)
    traffic, traffic_src = pmc_traffic(args.config, blend, nb)
    ncam = len(sizes)
    result = {
        "metric": "stitched megapixels/sec (6x4K->8K equirect)" if args.config in ("C2", "C3") else
                  "stitched megapixels/sec (%dx%dx%d->%dx%d equirect)" % (ncam, sizes[0][0], sizes[0][1], W, H),
        "value": round(value, 1),
        "unit": "MP/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "preroll": {"s": args.preroll, "steps": n_pre},
        "ms_per_step": round(elapsed * 1e3 / args.steps, 4),
        "host_issue_ms_per_step": round(ISSUE_S[0] * 1e3 / args.steps, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (splitmix64 YUV420P frames, further sets derived by a splitmix64 key, SURVEY.md §8d rig)",
        "config": {"workload": "%s: %d x %dx%d fullframe_fisheye -> %dx%d equirect, remap + %s + %s, YUV420P in/out" % (
                                   args.config, len(sizes), sizes[0][0], sizes[0][1], W, H,
                                   "gain (estimated per frame)" if use_gain else "no gain",
                                   "multi-band blend=%d (%d bands)" % (blend, int(math.ceil(math.log(blend) / math.log(2.)) - 1))
                                   if blend > 0 else "no-blend composite"),
                   "rigs_per_gpu": 1, "frames_in_flight": inflight * nb, "streams": inflight,
                   "frames_per_launch": nb, "frame_sets": nsets,
                   **({"remap": "texture (OCTVR_REMAP_TEXTURE)"} if args.remap == "texture" else {}),
                   "parallelism": "independent rig per GPU"},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": traffic, "traffic_source": traffic_src,
                     "kernel": "multiband sequence (remap, pyrDown, blend levels)" if blend > 0 else "stitch_kernel",
                     "kernel_us": round(avg_kernel_s * 1e6, 2),
                     "kernel_us_basis": ("union of the launches' HIP-event intervals over %d in-flight streams, per frame "
                                         "(%d frames per launch)" % (inflight, nb)) if inflight > 1 or nb > 1 else
                                        "HIP-event start-to-end, every 4th launch",
                     "kernel_us_span": round(span_ms / 1e3 / max(launches, 1) * 1e6, 2),
                     "bytes_per_launch": bytes_per_launch,
                     "bytes_basis": ("algorithmic: what each launch must move, each byte once (DESIGN.md §4; "
                                     "octvr_mapper_traffic_parts), per frame") + (
                                        "; the tiled LUT (%.1f MB) once per launch of %d frames" % (lut_b / 1e6, nb)
                                        if nb > 1 else "") + ("; per launch of the sequence in bytes_parts" if blend > 0 else ""),
                     **({"bytes_parts": m.info().get("traffic_parts")} if blend > 0 else {}),
                     "frac_at_step_time": round(bytes_per_launch / (elapsed / args.steps) / 1e9 / HBM_PEAK_GBPS, 4),
                     # the counter-based fraction: PMC HBM bytes of the same binary over the same kernel time
                     "frac_traffic": round(traffic / avg_kernel_s / 1e9 / HBM_PEAK_GBPS, 4) if traffic else None,
                     "traffic_over_bytes": round(traffic / bytes_per_launch, 3) if traffic else None,
                     **({"valu_busy": pmc_valu_busy(args.config)} if blend == 0 else {})},
        "survey_b_alg": {"bytes": survey_b_alg,
                         "gbps_at_step_time": round(survey_b_alg / (elapsed / args.steps) / 1e9, 1),
                         "note": "SURVEY.md §8(d) B_alg (per-camera maps re-read for every valid (camera, pixel)); "
                                 "this design moves fewer bytes for the same output, so this is a rate of the survey's "
                                 "model, not a fraction of HBM peak"},
        "gains": [round(g, 6) for g in gains],
        **({"roofline_one_in_flight": {"kernel_us": round(serial * 1e6, 2),
                                        "achieved": round(bytes_per_launch / serial / 1e9, 1),
                                        "frac": round(bytes_per_launch / serial / 1e9 / HBM_PEAK_GBPS, 4),
                                        "step_us": round(serial_step * 1e6, 1),
                                        "note": "after the timed region with set_frames_in_flight(1): kernel_us = the "
                                                "composite's packet-attached HIP events over 8 stitches (they read "
                                                "~10 us above rocprof's kernel duration here, profiles/r03_*_inflight1_"
                                                "kernel_stats.csv); step_us = wall time per frame of 16 serial stitches "
                                                "(gain feed + composite)"}}
           if serial else {}),
        "mapper": m.info(),
    }
    if rank == 0 and world == 1 and not args.no_async_e2e:
        result["async_e2e"] = async_e2e(ox, mt, sizes, W, H, blend, frames_np, dev, gain=use_gain, remap=args.remap)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(mt, frames_np, sizes, W, H, blend, gain=use_gain)
    return result


if __name__ == "__main__":
    main()
