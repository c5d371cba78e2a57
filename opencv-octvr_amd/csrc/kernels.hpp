// kernels.hpp — launch interface of the gfx950 kernels (internal; the public boundary is
// include/octvr_hip.h).  All launchers are stream-ordered and never synchronize.
#pragma once

#include <hip/hip_runtime.h>
#include <cstdint>

#include "camera_math.hpp"

namespace octvr {

constexpr int kMaxCams = 32;

// Composite-LUT entry (8 bytes per output pixel), built once per rig by composite_lut:
//   x = sx | sy << 16                      integer source pixel of the top-left tap
//   y = fx | fy << 5 | cam << 10 | 1 << 15  5-bit fractions, winning camera, valid flag
// An entry with the valid bit clear produces black (no camera covers the pixel).
struct CompositeEntry {
    uint32_t xy;
    uint32_t code;
};

// Fixed-point source coordinate of a normalized map value, as RemapInvoker derives it from the
// caller's `map * W` (template.cpp:174-176): X = fl32(m * W); ix = round_half_even(X * 32).
__host__ __device__ inline int quantize_coord(float m, float scale) {
    float X = m * scale;
    return (int)rintf(X * 32.0f);
}

// Entry for a valid map value (mask != 0 guarantees 0 <= m < 1, so 0 <= sx <= W).
__host__ __device__ inline CompositeEntry make_entry(float m1, float m2, float w, float h, int cam) {
    int ix = quantize_coord(m1, w), iy = quantize_coord(m2, h);
    CompositeEntry e;
    e.xy = (uint32_t)(ix >> 5) | ((uint32_t)(iy >> 5) << 16);
    e.code = (uint32_t)(ix & 31) | ((uint32_t)(iy & 31) << 5) | ((uint32_t)cam << 10) | (1u << 15);
    return e;
}

// One input camera as the per-frame kernels see it: a YUV420P frame in "Y over [U|V]" layout.
struct SourceFrame {
    const uint8_t* yuv;
    int32_t w, h;
    int64_t pitch;
};

// All camera frames of one stitch call, passed by value as a kernel argument (no per-frame H2D copy).
struct FrameSet {
    SourceFrame f[kMaxCams];
};

// ROI-sized per-camera template data resident on the device.
struct CamTemplate {
    const float* map1;
    const float* map2;
    const uint8_t* mask;
    int32_t roi_x, roi_y, roi_w, roi_h;
    int32_t in_w, in_h;
};

// Gain-feed work description (built on the host once per rig, GainCompensatorGPU ctor
// exposure_compensate.cpp:174-221 + Mapper ctor mapper.cpp:94-114).
struct GainChunk {
    int32_t pair;     // index into the i<j pair list
    int32_t begin;    // [begin, end) into the flat sample-pair arrays
    int32_t end;
    int32_t pad_;
};

// initInterTab2D(INTER_LINEAR, fixpt=true) replica (imgproc/src/imgwarp.cpp:211-280), 1024 x 4.
void bilinear_table(int16_t tab[1024 * 4]);

hipError_t launch_lut_build(const CameraParams& out, const CameraParams& in, int W, int H, float* map1, float* map2,
                            uint8_t* mask, int32_t* bbox, hipStream_t s);

hipError_t launch_composite_lut(const CamTemplate* cams_dev, int n, int W, int H, CompositeEntry* lut,
                                hipStream_t s);

hipError_t launch_gain_feed(const FrameSet& frames_dev, const int16_t* tab, const CompositeEntry* samples_a,
                            const CompositeEntry* samples_b, const GainChunk* chunks, int n_chunks,
                            double* partials, hipStream_t s);

hipError_t launch_gain_solve(const double* partials, const GainChunk* chunks, int n_chunks, const int32_t* pair_ij,
                             const int32_t* N, int n, double* gains, hipStream_t s);

hipError_t launch_set_gains(const double* host_gains, int n, double* gains_dev, hipStream_t s);

hipError_t launch_stitch(const FrameSet& frames_dev, const int16_t* tab, const CompositeEntry* lut, int W, int H,
                         const double* gains,
                         int use_gain, uint8_t* out, int64_t out_pitch, hipStream_t s);

hipError_t launch_remap_u8(const int16_t* tab, const uint8_t* src, int sw, int sh, int64_t spitch, int cn, const float* map1,
                           const float* map2, int mw, int mh, int64_t mpitch, float scale_x, float scale_y,
                           uint8_t* dst, int64_t dpitch, hipStream_t s);

}  // namespace octvr
