// fastmapper.hip — vr::FastMapper::stitch_nv12 (modules/octvr/src/mapper_fast.cpp:153-195) on gfx950.
//
// The reference runs, per camera, three cv::remap_weighted OpenCL launches (Y; V; U) that add
// convert_ushort_sat_rte(bilinear * feather_weight) into u16 accumulators
// (imgproc/src/opencl/remap_weighted.cl:20-78), then converts the accumulators with 1/255.
// Here one launch per plane visits, per output pixel, only the cameras whose feather weight is non-zero
// somewhere in the pixel's 256-pixel run (a per-run camera bit mask built once per rig), accumulates in
// a register (u16 adds wrap, so the camera order does not matter) and writes the final u8 directly:
// no u16 accumulator planes in HBM, no separate convert pass.
//
// Per (camera, pixel) entry (uint2, built on the host from convertMaps + the feather weights; stored only
// for the (camera, 256-pixel run) pairs where the camera has a non-zero weight somewhere in the run):
//   x = sx | sy << 16 (s16 each, convertMaps' integer tap), y = code (10-bit fractions) | weight << 16.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "device_common.hpp"
#include "kernels.hpp"

namespace octvr {

namespace {

__device__ __forceinline__ uint32_t sat_u16_rte(float v) {
    return (uint32_t)__builtin_amdgcn_fmed3f(__builtin_rintf(v), 0.f, 65535.f);  // v >= 0 here
}

// remap_weighted.cl:46-75 for one pixel of one camera: taps outside the source are 0.
__device__ __forceinline__ uint32_t weighted_tap(const uint8_t* plane, int sw, int sh, int64_t pitch, int step,
                                                 uint2 e) {
    const int sx = (int)(int16_t)(e.x & 0xFFFFu), sy = (int)(int16_t)(e.x >> 16);
    const uint32_t code = e.y & 1023u, w = e.y >> 16;
    const float ux = (float)(code & 31u) / 32.f, uy = (float)(code >> 5) / 32.f;
    float t[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int x = sx + (k & 1), y = sy + (k >> 1);
        const bool out = x >= sw || y >= sh || x < 0 || y < 0;
        t[k] = out ? 0.f : (float)plane[(int64_t)y * pitch + (int64_t)x * step];
    }
    float v = t[0] * (1 - ux) * (1 - uy) + t[1] * (ux) * (1 - uy) + t[2] * (1 - ux) * (uy) + t[3] * (ux) * (uy);
    v *= (float)w;
    return sat_u16_rte(v);
}

__device__ __forceinline__ uint8_t convert_out(uint32_t acc) {  // convertTo(CV_8U, 1/255.) (convert.cl:77)
    return (uint8_t)__builtin_amdgcn_fmed3f(__builtin_rintf(__builtin_fmaf((float)(acc & 0xFFFFu), (float)(1.0 / 255.0), 0.f)),
                                            0.f, 255.f);
}

}  // namespace

// runs[r] = {camera mask, first block}: run r's cameras (ascending) own blocks first, first + 1, ... of
// 256 entries (fastmapper.cpp)
__global__ void __launch_bounds__(256) fast_y_kernel(FrameSet frames, const uint2* __restrict__ ent,
                                                     const uint2* __restrict__ runs, int W, int H, uint8_t* out,
                                                     int64_t out_pitch) {
    const int64_t npx = (int64_t)W * H;
    const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const uint2 rr = runs[blockIdx.x];
    uint32_t m = (uint32_t)uniform((int)rr.x);
    uint32_t blk = (uint32_t)uniform((int)rr.y);
    if (idx >= npx) return;
    uint32_t acc = 0;
    while (m) {
        const int c = __builtin_ctz(m);
        m &= m - 1;
        const uint2 e = ent[(int64_t)(blk++) * 256 + threadIdx.x];
        if ((e.y >> 16) == 0) continue;
        const SourceFrame& f = frames.f[c];
        acc += weighted_tap(f.yuv, f.w, f.h, f.pitch, 1, e);
    }
    const int y = (int)(idx / W), x = (int)(idx - (int64_t)y * W);
    out[(int64_t)y * out_pitch + x] = convert_out(acc);
}

__global__ void __launch_bounds__(256) fast_uv_kernel(FrameSet frames, const uint2* __restrict__ ent,
                                                      const uint2* __restrict__ runs, int W, int H, uint8_t* out,
                                                      int64_t out_pitch) {
    const int hw = W / 2, hh = H / 2;
    const int64_t npx = (int64_t)hw * hh;
    const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const uint2 rr = runs[blockIdx.x];
    uint32_t m = (uint32_t)uniform((int)rr.x);
    uint32_t blk = (uint32_t)uniform((int)rr.y);
    if (idx >= npx) return;
    uint32_t accV = 0, accU = 0;
    while (m) {
        const int c = __builtin_ctz(m);
        m &= m - 1;
        const uint2 e = ent[(int64_t)(blk++) * 256 + threadIdx.x];
        if ((e.y >> 16) == 0) continue;
        const SourceFrame& f = frames.f[c];
        const uint8_t* uv = f.yuv + (int64_t)f.h * f.pitch;  // interleaved U, V rows (NV12)
        accV += weighted_tap(uv + 1, f.w / 2, f.h / 2, f.pitch, 2, e);
        accU += weighted_tap(uv, f.w / 2, f.h / 2, f.pitch, 2, e);
    }
    const int y = (int)(idx / hw), x = (int)(idx - (int64_t)y * hw);
    uint8_t* o = out + (int64_t)(H + y) * out_pitch + 2 * x;  // merge(c1c2): V first, then U
    o[0] = convert_out(accV);
    o[1] = convert_out(accU);
}

hipError_t launch_fastmapper_nv12(const FrameSet& frames, const uint2* ent_y, const uint2* runs_y,
                                  const uint2* ent_uv, const uint2* runs_uv, int W, int H, uint8_t* out,
                                  int64_t out_pitch, hipStream_t s) {
    const int64_t ny = (int64_t)W * H, nuv = (int64_t)(W / 2) * (H / 2);
    hipLaunchKernelGGL(fast_y_kernel, dim3((unsigned)((ny + 255) / 256)), dim3(256), 0, s, frames, ent_y, runs_y, W, H,
                       out, out_pitch);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(fast_uv_kernel, dim3((unsigned)((nuv + 255) / 256)), dim3(256), 0, s, frames, ent_uv, runs_uv, W,
                       H, out, out_pitch);
    return hipGetLastError();
}

}  // namespace octvr
