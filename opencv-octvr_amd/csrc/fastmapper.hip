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
// Per (camera, pixel) entry, built on the host from convertMaps + the feather weights and stored only
// for the (camera, 256-pixel run) pairs where the camera has a non-zero weight somewhere in the run.
// Compact format (5 B per entry, the default): per 256-entry block a header {bsx | bsy << 16 (s16)},
// per entry a u32 dx | dy << 11 | code << 22 (tap = (bsx + dx, bsy + dy), 11-bit offsets, 10-bit
// fractions) and a u8 feather weight in a plane of its own.  Wide format (8 B, used for a plane when
// one of its blocks spans 2048 source pixels or more): uint2 {sx | sy << 16 (s16), code | weight << 16}.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "device_common.hpp"
#include "kernels.hpp"

namespace octvr {

namespace {

__device__ __forceinline__ uint32_t sat_u16_rte(float v) {
    return (uint32_t)__builtin_amdgcn_fmed3f(__builtin_rintf(v), 0.f, 65535.f);  // v >= 0 here
}

__device__ __forceinline__ uint8_t convert_out(uint32_t acc) {  // convertTo(CV_8U, 1/255.) (convert.cl:77)
    return (uint8_t)__builtin_amdgcn_fmed3f(__builtin_rintf(__builtin_fmaf((float)(acc & 0xFFFFu), (float)(1.0 / 255.0), 0.f)),
                                            0.f, 255.f);
}

}  // namespace

// remap_weighted.cl:46-75 for one pixel of one camera from its four taps (0 outside the source)
__device__ __forceinline__ uint32_t weighted_sum(const float (&t)[4], uint32_t code, uint32_t w) {
    const float ux = (float)(code & 31u) / 32.f, uy = (float)(code >> 5) / 32.f;
    float v = t[0] * (1 - ux) * (1 - uy) + t[1] * (ux) * (1 - uy) + t[2] * (1 - ux) * (uy) + t[3] * (ux) * (uy);
    v *= (float)w;
    return sat_u16_rte(v);
}

// A run's cameras in groups of kFastGroup: every entry load of the group, then every tap gather, then
// the arithmetic, so a pixel costs two memory round trips per group instead of two per camera (the
// plain per-camera loop, 920 us for a C2 frame, was a chain of dependent loads).  A tap row is one
// 8-byte load through the camera's frame as a buffer resource (32-bit offsets; addresses clamped into
// the image, taps outside it zeroed by mask, as BORDER_CONSTANT), instead of 2 (Y) or 4 (chroma) byte
// loads.  PLANE 0: Y; 1: the interleaved
// NV12 chroma, V and U (merge order c1, c2: V first, mapper_fast.cpp:181-187).
constexpr int kFastGroup = 4;

struct FastPlane {
    const uint2* ent;     // wide entries
    const uint32_t* off;  // compact entries
    const uint8_t* wgt;   // compact weights
    const uint2* hdr;     // compact block headers
    const uint2* runs;    // per run: camera mask, first block
};

template <int PLANE, bool COMPACT>
__device__ __forceinline__ void fast_plane(const FrameSet& frames, const FastPlane& fp, int W, int H, uint8_t* out,
                                           int64_t out_pitch) {
    typedef __attribute__((address_space(4))) const uint64_t kU64;
    const int pw = PLANE ? W / 2 : W, ph = PLANE ? H / 2 : H;
    const int64_t npx = (int64_t)pw * ph;
    const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const uint2 rr = fp.runs[blockIdx.x];
    uint32_t m = (uint32_t)uniform((int)rr.x);
    uint32_t blk = (uint32_t)uniform((int)rr.y);
    uint32_t acc0 = 0, acc1 = 0;  // Y (or V), U
    while (m) {
        int sxk[kFastGroup], syk[kFastGroup];
        uint32_t code[kFastGroup], wk[kFastGroup];
        int cam[kFastGroup];
        bool live[kFastGroup];
#pragma unroll
        for (int k = 0; k < kFastGroup; k++) {  // uniform: the group's cameras and their entry blocks
            live[k] = m != 0u;
            cam[k] = live[k] ? __builtin_ctz(m) : 0;
            m &= m - 1u;
            const uint32_t b = live[k] ? blk + k : blk;  // dead slots reload the group's first block
            if (COMPACT) {
                const uint64_t h = *(kU64*)(uintptr_t)(fp.hdr + b);
                const uint32_t c = fp.off[(int64_t)b * 256 + threadIdx.x];
                wk[k] = fp.wgt[(int64_t)b * 256 + threadIdx.x];
                sxk[k] = (int)(int16_t)(uint32_t)h + (int)(c & 2047u);
                syk[k] = (int)(int16_t)(uint32_t)(h >> 16) + (int)((c >> 11) & 2047u);
                code[k] = c >> 22;
            } else {
                const uint2 e = fp.ent[(int64_t)b * 256 + threadIdx.x];
                sxk[k] = (int)(int16_t)(e.x & 0xFFFFu);
                syk[k] = (int)(int16_t)(e.x >> 16);
                code[k] = e.y & 1023u;
                wk[k] = e.y >> 16;
            }
        }
        blk += live[3] ? 4u : live[2] ? 3u : live[1] ? 2u : 1u;
        // per camera and tap row one 8-byte load from the 4-byte aligned start at or below the row's
        // first in-image tap byte: it holds both taps' bytes (Y: x, x + 1; chroma: the V, U pairs of x, x + 1)
        uint2 rw[kFastGroup][2];
        uint32_t sel[kFastGroup][2];
#pragma unroll
        for (int k = 0; k < kFastGroup; k++) {
            const SourceFrame f = frames.f[cam[k]];
            const int sw = PLANE ? f.w / 2 : f.w, sh = PLANE ? f.h / 2 : f.h;
            const uint32_t base = PLANE ? (uint32_t)f.h * (uint32_t)f.pitch : 0u;
            const uint32_t size = (uint32_t)f.pitch * (uint32_t)(f.h + f.h / 2);  // >= 8 (host check)
            const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(f.yuv), 0, (int)size, 0x00020000);
            const int sx = sxk[k], sy = syk[k];
            const int xa = min(max(sx, 0), sw - 1);
            const uint32_t bx = (uint32_t)xa * (PLANE ? 2u : 1u) & ~3u;  // 4-byte aligned row start
#pragma unroll
            for (int r = 0; r < 2; r++) {
                const int y = min(max(sy + r, 0), sh - 1);
                const uint32_t row = base + (uint32_t)y * (uint32_t)f.pitch;
                // the buffer range-checks whole dwords: a start within 8 bytes of the frame's end (its last
                // chroma row, a pitch not a multiple of 4) is clamped to size - 8 and the taps taken from there
                const uint32_t st = min(row + bx, size - 8u);
                // byte index of taps x = sx, sx + 1 in the 8 loaded bytes (exact for taps inside the image,
                // any byte for the ones outside, which are masked below); an in-image chroma pair starts
                // at most at byte 6, so its second byte is i + 1 <= 7
                const uint32_t i0 = (row + (uint32_t)(sx * (PLANE ? 2 : 1)) - st) & 7u;
                const uint32_t i1 = (row + (uint32_t)((sx + 1) * (PLANE ? 2 : 1)) - st) & 7u;
                sel[k][r] = PLANE ? (i0 | (i0 + 1u) << 8 | i1 << 16 | (i1 + 1u) << 24) : (i0 | i1 << 8 | 0x0C0C0000u);
                typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
                const u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(rs, st, 0, 0);
                rw[k][r] = make_uint2(v.x, v.y);
            }
        }
#pragma unroll
        for (int k = 0; k < kFastGroup; k++) {
            if (!live[k] || wk[k] == 0) continue;
            const SourceFrame f = frames.f[cam[k]];
            const int sw = PLANE ? f.w / 2 : f.w, sh = PLANE ? f.h / 2 : f.h;
            const int sx = sxk[k], sy = syk[k];
            float t0[4], t1[4];
#pragma unroll
            for (int r = 0; r < 2; r++) {
                // row r's taps: Y bytes {x, x + 1}, or chroma bytes {U x, V x, U x+1, V x+1}
                const uint32_t b = __builtin_amdgcn_perm(rw[k][r].y, rw[k][r].x, sel[k][r]);
                const int y = sy + r;
#pragma unroll
                for (int c = 0; c < 2; c++) {
                    const int x = sx + c;
                    const bool in = x >= 0 && y >= 0 && x < sw && y < sh;
                    const int j = 2 * r + c;
                    if (PLANE) {
                        t0[j] = in ? (float)((b >> (16 * c + 8)) & 255u) : 0.f;  // V
                        t1[j] = in ? (float)((b >> (16 * c)) & 255u) : 0.f;      // U
                    } else {
                        t0[j] = in ? (float)((b >> (8 * c)) & 255u) : 0.f;
                    }
                }
            }
            acc0 += weighted_sum(t0, code[k], wk[k]);
            if (PLANE) acc1 += weighted_sum(t1, code[k], wk[k]);
        }
    }
    if (idx >= npx) return;
    const int y = (int)(idx / pw), x = (int)(idx - (int64_t)y * pw);
    if (PLANE) {
        uint8_t* o = out + (int64_t)(H + y) * out_pitch + 2 * x;  // merge(c1c2): V first, then U
        o[0] = convert_out(acc0);
        o[1] = convert_out(acc1);
    } else {
        out[(int64_t)y * out_pitch + x] = convert_out(acc0);
    }
}

// runs[r] = {camera mask, first block}: run r's cameras (ascending) own blocks first, first + 1, ... of
// 256 entries (fastmapper.cpp)
template <bool COMPACT>
__global__ void __launch_bounds__(256) fast_y_kernel(FrameSet frames, FastPlane fp, int W, int H, uint8_t* out,
                                                     int64_t out_pitch) {
    fast_plane<0, COMPACT>(frames, fp, W, H, out, out_pitch);
}

template <bool COMPACT>
__global__ void __launch_bounds__(256) fast_uv_kernel(FrameSet frames, FastPlane fp, int W, int H, uint8_t* out,
                                                      int64_t out_pitch) {
    fast_plane<1, COMPACT>(frames, fp, W, H, out, out_pitch);
}

template <int PLANE, bool COMPACT>
static void launch_plane_kernel(dim3 grid, const FrameSet& frames, const FastPlane& fp, int W, int H, uint8_t* out,
                                int64_t out_pitch, hipStream_t s) {
    if (PLANE)
        hipLaunchKernelGGL((fast_uv_kernel<COMPACT>), grid, dim3(256), 0, s, frames, fp, W, H, out, out_pitch);
    else
        hipLaunchKernelGGL((fast_y_kernel<COMPACT>), grid, dim3(256), 0, s, frames, fp, W, H, out, out_pitch);
}

template <int PLANE>
static hipError_t launch_plane(const FrameSet& frames, const FastMapperPlane& p, int W, int H, uint8_t* out,
                               int64_t out_pitch, hipStream_t s) {
    const int64_t n = PLANE ? (int64_t)(W / 2) * (H / 2) : (int64_t)W * H;
    const dim3 grid((unsigned)((n + 255) / 256));
    const FastPlane fp{p.ent, p.off, p.wgt, p.hdr, p.runs};
    if (p.compact)
        launch_plane_kernel<PLANE, true>(grid, frames, fp, W, H, out, out_pitch, s);
    else
        launch_plane_kernel<PLANE, false>(grid, frames, fp, W, H, out, out_pitch, s);
    return hipGetLastError();
}

hipError_t launch_fastmapper_nv12(const FrameSet& frames, const FastMapperPlane& y, const FastMapperPlane& uv, int W,
                                  int H, uint8_t* out, int64_t out_pitch, hipStream_t s) {
    const hipError_t e = launch_plane<0>(frames, y, W, H, out, out_pitch, s);
    if (e != hipSuccess) return e;
    return launch_plane<1>(frames, uv, W, H, out, out_pitch, s);
}

}  // namespace octvr
