"""Synthetic rigs and frames of the benchmark configurations (BASELINE.json configs).

Rig JSON follows the reference schema (producer modules/octvr/tools/ptx2json.py):
`fullframe_fisheye` inputs with a centred circular crop, 200 deg hfov, no radial distortion.
Frames are uniform-random bytes from splitmix64 (seed = 1000*rig + cam) in the "Y over [U|V]"
YUV420P layout of mapper.hpp:75-83.
"""
import math

import numpy as np

HFOV_200 = 3.490658503988659


def fisheye_rig(in_w, in_h, yaws, pitches=None, hfov=HFOV_200, circular=True):
    pitches = pitches or [0.0] * len(yaws)
    crop = [(in_w - in_h) // 2, (in_w + in_h) // 2, 0, in_h] if in_w >= in_h else [0, in_w, (in_h - in_w) // 2, (in_h + in_w) // 2]
    inputs = []
    for yaw, pitch in zip(yaws, pitches):
        inputs.append({"type": "fullframe_fisheye", "options": {
            "width": in_w, "height": in_h, "crop": {"rect": crop, "is_circular": circular},
            "hfov": hfov, "center_dx": 0.0, "center_dy": 0.0, "radial": [0.0, 0.0, 0.0],
            "rotation": {"roll": 0.0, "yaw": yaw, "pitch": pitch}}})
    return {"output": {"type": "equirectangular", "options": {}}, "inputs": inputs}


CONFIGS = {
    # name: (rig json, out_w, out_h, in sizes)
    "C1": lambda: (fisheye_rig(1920, 1080, [0.0, math.pi]), 4096, 2048, [(1920, 1080)] * 2),
    "C2": lambda: (fisheye_rig(3840, 2160, [k * math.pi / 3 for k in range(6)]), 7680, 3840, [(3840, 2160)] * 6),
    # C3 = C2 + multi-band blend=16 (3 bands), seams from the L2 distance seam finder
    "C3": lambda: (fisheye_rig(3840, 2160, [k * math.pi / 3 for k in range(6)]), 7680, 3840, [(3840, 2160)] * 6),
    "C4": lambda: (fisheye_rig(3840, 2160, [k * math.pi / 3 for k in range(6)] + [k * math.pi / 3 + math.pi / 6 for k in range(6)],
                               [0.6108652381980153] * 6 + [-0.6108652381980153] * 6, hfov=2.6179938779914944),
                   15360, 7680, [(3840, 2160)] * 12),
}


# F2: the C2 rig through vr::FastMapper::stitch_nv12 (feather-weighted NV12, template without ROI as
# octvr_dump -n writes it; mapper_fast.cpp:27-195) — the second drop-in entry point, not a BASELINE config
CONFIGS["F2"] = CONFIGS["C2"]

# Mapper blend mode per configuration (mapper.cpp:171-184: 0 copy chain, > 0 multi-band)
BLEND = {"C1": 0, "C2": 0, "C3": 16, "C4": 0, "F2": 0}

# Gain compensation per configuration: C1 is the reference's CPU plumbing case (BASELINE configs[0]:
# cv::remap + the seam-mask copy, no gain; SURVEY.md §6 measured it at 192-204 MP/s on 8 threads)
GAIN = {"C1": False, "C2": True, "C3": True, "C4": True, "F2": False}


def splitmix_bytes(seed, n):
    k = np.arange(1, n + 1, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + k * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return (z & np.uint64(0xFF)).astype(np.uint8)


def yuv_frame(w, h, seed):
    """(3h/2) x w uint8 YUV420P frame, Y over [U|V]."""
    return splitmix_bytes(seed, w * h * 3 // 2).reshape(h * 3 // 2, w)


FRAME_KEY_BYTES = 1 << 16


def frame_key(seed):
    """The 64 KiB byte key of a derived frame set (derived_frame)."""
    return splitmix_bytes(seed, FRAME_KEY_BYTES)


def derived_frame(base, seed):
    """Another frame of the same shape: base XOR frame_key(seed) repeated over its bytes (still uniform
    random bytes, distinct content).  The bench derives its extra frame sets this way on the device
    (bench.py derive_set), the same bytes as this."""
    flat = base.reshape(-1)
    key = np.resize(frame_key(seed), flat.size)
    return (flat ^ key).reshape(base.shape)


def smooth_yuv_frame(w, h, seed):
    """A frame with image-like structure (gradients + texture) — exercises gain estimation with
    realistic overlaps rather than white noise."""
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float32)
    base = 128 + 60 * np.sin(xx / (17 + seed % 7)) * np.cos(yy / 23.0) + 0.02 * (xx - yy)
    y = np.clip(base + rng.normal(0, 8, (h, w)), 0, 255).astype(np.uint8)
    u = np.clip(128 + 30 * np.sin(xx[::2, ::2] / 41.0) + rng.normal(0, 4, (h // 2, w // 2)), 0, 255).astype(np.uint8)
    v = np.clip(128 + 30 * np.cos(yy[::2, ::2] / 37.0) + rng.normal(0, 4, (h // 2, w // 2)), 0, 255).astype(np.uint8)
    out = np.empty((h * 3 // 2, w), np.uint8)
    out[:h] = y
    out[h:, : w // 2] = u
    out[h:, w // 2:] = v
    return out
