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
#include <cstring>

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

// remap_weighted.cl:46-75 for one pixel of one camera, ((t0 (1 - ux)) (1 - uy) + (t1 ux) (1 - uy)) +
// (t2 (1 - ux)) uy + (t3 ux) uy in f32 with every product and sum rounded as written, computed in
// integers: with ux = fx / 32, uy = fy / 32 and integer taps t <= 255 every product and partial sum is
// exact in f32 (t (32 - fx) (32 - fy) <= 255 * 1024 < 2^24, and the four terms add up to at most
// 255 * 1024 / 1024): v = N / 1024 with
//   N = (32 - fy) (t0 (32 - fx) + t1 fx) + fy (t2 (32 - fx) + t3 fx),
// two v_dot2_u32_u16 for the rows and one for the column.  The only rounding is v * w: fl(N / 1024 * w) =
// fl(N * (w / 1024)), w / 1024 exact; then round half to even (<= 65,025, no saturation).  Taps outside
// the image are zeroed through the weights: column c's weight is 0 when x + c is outside, row r's when
// y + r is (tap (c, r) is inside exactly when both are).
typedef unsigned short fast_u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t weighted_sum_int(uint32_t row0, uint32_t row1, uint32_t wx, uint32_t wy, float wf) {
    const uint32_t h0 = __builtin_amdgcn_udot2(__builtin_bit_cast(fast_u16x2, row0), __builtin_bit_cast(fast_u16x2, wx), 0u, false);
    const uint32_t h1 = __builtin_amdgcn_udot2(__builtin_bit_cast(fast_u16x2, row1), __builtin_bit_cast(fast_u16x2, wx), 0u, false);
    const uint32_t n = __builtin_amdgcn_udot2(__builtin_bit_cast(fast_u16x2, h0 | h1 << 16), __builtin_bit_cast(fast_u16x2, wy), 0u, false);
    return (uint32_t)__builtin_rintf((float)n * wf);
}

// A run's cameras in groups of kFastGroup: every entry load of the group, then every tap gather, then
// the arithmetic, so a pixel costs two memory round trips per group instead of two per camera (the
// plain per-camera loop, 920 us for a C2 frame, was a chain of dependent loads).  A tap row is one
// 8-byte load through the camera's frame as a buffer resource (32-bit offsets; addresses clamped into
// the image, taps outside it zeroed by mask, as BORDER_CONSTANT), instead of 2 (Y) or 4 (chroma) byte
// loads.  Slots past the run's cameras are skipped by uniform branches (a C2 run has about 4 cameras,
// i.e. a second group of 4 is mostly empty; the kernels issue VALU in every SIMD cycle and keep the
// texture data path 94 % busy, so work done for empty slots cost its full share).  PLANE 0: Y; 1: the
// interleaved NV12 chroma, V and U (merge order c1, c2: V first, mapper_fast.cpp:181-187).
constexpr int kFastGroup = 4;  // (groups of 2, 3 or 6 measured 1-6 % slower)

struct FastPlane {
    const uint2* ent;     // wide entries
    const uint32_t* off;  // compact entries
    const uint8_t* wgt;   // compact weights
    const uint2* hdr;     // compact block headers
    const uint2* runs;    // per run: camera mask, first block
    uint32_t nblk;        // blocks allocated (>= 1)
};
// compact block header bit (y word): every weighted entry of the block is interior (fastmapper.cpp)
constexpr uint32_t kFastInterior = 1u;

// The frames of one launch (FastBatch, the FIRST kernel argument): camera c of frame f at src[fbase + c],
// fbase = f << cam_log2; read through the kernarg segment with the camera uniform (scalar loads).
typedef __attribute__((address_space(4))) const SourceFrame kFastSource;
static_assert(offsetof(FastBatch<1>, src) == 0 && offsetof(FastBatch<4>, src) == 0, "FastBatch layout");
__device__ __forceinline__ SourceFrame fast_frame(uint32_t idx) {
    const kFastSource* kf = (const kFastSource*)__builtin_amdgcn_kernarg_segment_ptr();
    SourceFrame s;
    s.yuv = kf[idx].yuv;
    s.w = kf[idx].w;
    s.h = kf[idx].h;
    s.pitch = kf[idx].pitch;
    s.vig = nullptr;
    return s;
}

// One group of up to kFastGroup cameras of a run, after the entry loads: per camera and tap row one 8-byte
// load from the 4-byte aligned start at or below the row's first in-image tap byte (it holds both taps'
// bytes: Y x, x + 1; chroma the V, U pairs of x, x + 1), then remap_weighted's sum in integers.
// INNER: every tap of the group's weighted entries lies inside the plane, at least two rows above its
// last (host-checked per block, kFastInterior), so the address clamps, the end-of-frame clamp and the
// in-image masks are identities and are left out.
template <int PLANE, bool INNER>
__device__ __forceinline__ void fast_group(uint32_t fbase, const bool (&live)[kFastGroup], const int (&cam)[kFastGroup],
                                           const int (&sxk)[kFastGroup], const int (&syk)[kFastGroup],
                                           const uint32_t (&code)[kFastGroup], const uint32_t (&wk)[kFastGroup],
                                           uint32_t& acc0, uint32_t& acc1) {
    constexpr uint32_t bpp = PLANE ? 2u : 1u;  // bytes per source pixel of the plane
    uint2 rw[kFastGroup][2];
    uint32_t sel[kFastGroup][2];
#pragma unroll
    for (int k = 0; k < kFastGroup; k++) {
        rw[k][0] = rw[k][1] = make_uint2(0u, 0u);
        sel[k][0] = sel[k][1] = 0u;
        if (!live[k]) continue;
        const SourceFrame f = fast_frame(fbase + (uint32_t)cam[k]);
        const int sw = PLANE ? f.w / 2 : f.w, sh = PLANE ? f.h / 2 : f.h;
        const uint32_t base = PLANE ? (uint32_t)f.h * (uint32_t)f.pitch : 0u;
        const uint32_t size = (uint32_t)f.pitch * (uint32_t)(f.h + f.h / 2);  // >= 8 (host check)
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(f.yuv), 0, (int)size, 0x00020000);
        const int sx = sxk[k], sy = syk[k];
        const int xa = INNER ? sx : min(max(sx, 0), sw - 1);
        const uint32_t bx = (uint32_t)xa * bpp & ~3u;  // 4-byte aligned row start
#pragma unroll
        for (int r = 0; r < 2; r++) {
            const int y = INNER ? sy + r : min(max(sy + r, 0), sh - 1);
            // y < 2^15, pitch < 2^24 (host check): a 24-bit multiply
            const uint32_t row = base + __umul24((uint32_t)y, (uint32_t)f.pitch);
            // the buffer range-checks whole dwords: a start within 8 bytes of the frame's end (its last
            // chroma row, a pitch not a multiple of 4) is clamped to size - 8 and the taps taken from there
            const uint32_t st = INNER ? row + bx : min(row + bx, size - 8u);
            // byte index of taps x = sx, sx + 1 in the 8 loaded bytes (exact for taps inside the image,
            // any byte for the ones outside, which are masked below); an in-image chroma pair starts
            // at most at byte 6, so its second byte is i + 1 <= 7
            const uint32_t d = INNER ? (uint32_t)sx * bpp & 3u : row + (uint32_t)sx * bpp - st;
            const uint32_t i0 = d & 7u, i1 = (d + bpp) & 7u;
            // u16 pairs {tap x, tap x + 1} (chroma: of U; V is the next byte of each)
            sel[k][r] = i0 | i1 << 16 | 0x0C000C00u;
            typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
            const u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(rs, st, 0, 0);
            rw[k][r] = make_uint2(v.x, v.y);
        }
    }
#pragma unroll
    for (int k = 0; k < kFastGroup; k++) {
        if (!live[k]) continue;
        if (wk[k] == 0) continue;
        const uint32_t fx = code[k] & 31u, fy = code[k] >> 5;
        uint32_t wx = 32u + fx * 0xFFFFu, wy = 32u + fy * 0xFFFFu;  // {32 - f, f} as u16 pairs
        if (!INNER) {  // taps outside the image weigh 0: column / row masks
            const SourceFrame f = fast_frame(fbase + (uint32_t)cam[k]);
            const uint32_t sw = (uint32_t)(PLANE ? f.w / 2 : f.w), sh = (uint32_t)(PLANE ? f.h / 2 : f.h);
            const int sx = sxk[k], sy = syk[k];
            const bool ix0 = (uint32_t)sx < sw, ix1 = (uint32_t)(sx + 1) < sw;
            const bool iy0 = (uint32_t)sy < sh, iy1 = (uint32_t)(sy + 1) < sh;
            wx &= (ix0 ? 0xFFFFu : 0u) | (ix1 ? 0xFFFF0000u : 0u);
            wy &= (iy0 ? 0xFFFFu : 0u) | (iy1 ? 0xFFFF0000u : 0u);
        }
        const float wf = (float)wk[k] * (1.f / 1024.f);
        const uint2 q0 = rw[k][0], q1 = rw[k][1];
        acc0 += weighted_sum_int(__builtin_amdgcn_perm(q0.y, q0.x, sel[k][0] + (PLANE ? 0x00010001u : 0u)),
                                 __builtin_amdgcn_perm(q1.y, q1.x, sel[k][1] + (PLANE ? 0x00010001u : 0u)), wx, wy, wf);
        if (PLANE)
            acc1 += weighted_sum_int(__builtin_amdgcn_perm(q0.y, q0.x, sel[k][0]), __builtin_amdgcn_perm(q1.y, q1.x, sel[k][1]),
                                     wx, wy, wf);
    }
}

// LG: 1 << LG frames per launch — each group's entries are loaded once and applied to every frame (FastBatch)
template <int PLANE, bool COMPACT, int LG>
__device__ __forceinline__ void fast_plane(const FastPlane& fp, int W, int H, int64_t out_pitch) {
    constexpr int NF = 1 << LG, cam_lg = LG <= 1 ? 5 : 4;
    typedef __attribute__((address_space(4))) const uint64_t kU64;
    const int pw = PLANE ? W / 2 : W, ph = PLANE ? H / 2 : H;
    const uint32_t npx = (uint32_t)pw * (uint32_t)ph;  // < 2^31 (host check)
    const uint2 rr = fp.runs[blockIdx.x];
    uint32_t m = (uint32_t)uniform((int)rr.x);
    uint32_t blk = (uint32_t)uniform((int)rr.y);
    uint32_t acc0[NF], acc1[NF];  // per frame: Y (or V), U
#pragma unroll
    for (int f = 0; f < NF; f++) acc0[f] = acc1[f] = 0u;
    while (m) {
        int sxk[kFastGroup], syk[kFastGroup];
        uint32_t code[kFastGroup], wk[kFastGroup];
        int cam[kFastGroup];
        bool live[kFastGroup];
        uint2 en[kFastGroup];  // compact: {offsets, weight}; wide: the entry
        uint64_t hd[kFastGroup];
#pragma unroll
        for (int k = 0; k < kFastGroup; k++) {  // uniform: the group's cameras and their entry blocks
            live[k] = m != 0u;
            cam[k] = live[k] ? __builtin_ctz(m) : 0;
            m &= m - 1u;
            // every slot loads (dead ones the group's first block) so that no load waits on a branch.  The
            // block is clamped into the plane's allocation (one scalar min): the host's index replay
            // (octvr_debug_fastmapper_audit) shows it never engages, but no entry, weight or header
            // address can then leave the buffers whatever the run table holds.
            const uint32_t b = min(live[k] ? blk + k : blk, fp.nblk - 1u);
            const uint32_t e = b * 256u + threadIdx.x;  // < 2^32 (host check)
            if (COMPACT) {
                hd[k] = *(kU64*)(uintptr_t)(fp.hdr + b);
                en[k] = make_uint2(fp.off[e], fp.wgt[e]);
            } else {
                hd[k] = 0;
                en[k] = fp.ent[e];
            }
        }
#pragma unroll
        for (int k = 0; k < kFastGroup; k++) {
            if (COMPACT) {
                sxk[k] = (int)(int16_t)(uint32_t)hd[k] + (int)(en[k].x & 2047u);
                syk[k] = (int)(int16_t)(uint32_t)(hd[k] >> 16) + (int)((en[k].x >> 11) & 2047u);
                code[k] = en[k].x >> 22;
                wk[k] = en[k].y;
            } else {
                sxk[k] = (int)(int16_t)(en[k].x & 0xFFFFu);
                syk[k] = (int)(int16_t)(en[k].x >> 16);
                code[k] = en[k].y & 1023u;
                wk[k] = en[k].y >> 16;
            }
        }
#pragma unroll
        for (int k = 0; k < kFastGroup; k++) blk += live[k] ? 1u : 0u;
        // Interior groups (compact blocks flagged by the host: every weighted entry's taps at x <= w - 2,
        // y <= h - 3 of the plane, so no tap is outside the image and no 8-byte row load reaches the frame's
        // end) take the taps without clamps, end-of-frame clamp or in-image masks; the rest the general path.
        bool inner = COMPACT;
#pragma unroll
        for (int k = 0; k < kFastGroup; k++) inner = inner && (!live[k] || ((hd[k] >> 32) & kFastInterior) != 0);
#pragma unroll
        for (int f = 0; f < NF; f++) {
            if (inner)
                fast_group<PLANE, true>((uint32_t)f << cam_lg, live, cam, sxk, syk, code, wk, acc0[f], acc1[f]);
            else
                fast_group<PLANE, false>((uint32_t)f << cam_lg, live, cam, sxk, syk, code, wk, acc0[f], acc1[f]);
        }
    }
    // pixel index -> (x, y): the run's first row by one scalar division, then at most 256 / pw row steps
    const uint32_t idx0 = blockIdx.x * 256u;
    uint32_t y = (uint32_t)uniform((int)(idx0 / (uint32_t)pw));
    uint32_t x = idx0 - y * (uint32_t)pw + threadIdx.x;
    if (idx0 + threadIdx.x >= npx) return;
    while (x >= (uint32_t)pw) {
        x -= (uint32_t)pw;
        y++;
    }
    typedef __attribute__((address_space(4))) const FastBatch<NF> kFastBatch;
    const kFastBatch* kb = (const kFastBatch*)__builtin_amdgcn_kernarg_segment_ptr();
#pragma unroll
    for (int f = 0; f < NF; f++) {
        uint8_t* out = kb->out[f];
        if (PLANE) {
            uint8_t* o = out + (int64_t)(H + (int)y) * out_pitch + 2 * x;  // merge(c1c2): V first, then U
            o[0] = convert_out(acc0[f]);
            o[1] = convert_out(acc1[f]);
        } else {
            out[(int64_t)y * out_pitch + x] = convert_out(acc0[f]);
        }
    }
}

// runs[r] = {camera mask, first block}: run r's cameras (ascending) own blocks first, first + 1, ... of
// 256 entries (fastmapper.cpp)
template <bool COMPACT, int LG>
__global__ void __launch_bounds__(256) fast_y_kernel(FastBatch<1 << LG> batch, FastPlane fp, int W, int H, int64_t out_pitch) {
    (void)batch;  // read through the kernarg segment (kFastBatch)
    fast_plane<0, COMPACT, LG>(fp, W, H, out_pitch);
}

template <bool COMPACT, int LG>
__global__ void __launch_bounds__(256) fast_uv_kernel(FastBatch<1 << LG> batch, FastPlane fp, int W, int H, int64_t out_pitch) {
    (void)batch;
    fast_plane<1, COMPACT, LG>(fp, W, H, out_pitch);
}

template <int PLANE, bool COMPACT, int LG>
static void launch_plane_kernel(dim3 grid, const FastBatch<1 << LG>& b, const FastPlane& fp, int W, int H, int64_t out_pitch,
                                hipStream_t s) {
    if (PLANE)
        hipLaunchKernelGGL((fast_uv_kernel<COMPACT, LG>), grid, dim3(256), 0, s, b, fp, W, H, out_pitch);
    else
        hipLaunchKernelGGL((fast_y_kernel<COMPACT, LG>), grid, dim3(256), 0, s, b, fp, W, H, out_pitch);
}

template <int PLANE, int LG>
static hipError_t launch_plane(const FastBatch<1 << LG>& b, const FastMapperPlane& p, int W, int H, int64_t out_pitch,
                               hipStream_t s) {
    const int64_t n = PLANE ? (int64_t)(W / 2) * (H / 2) : (int64_t)W * H;
    const dim3 grid((unsigned)((n + 255) / 256));
    const FastPlane fp{p.ent, p.off, p.wgt, p.hdr, p.runs, p.nblk};
    if (p.compact)
        launch_plane_kernel<PLANE, true, LG>(grid, b, fp, W, H, out_pitch, s);
    else
        launch_plane_kernel<PLANE, false, LG>(grid, b, fp, W, H, out_pitch, s);
    return hipGetLastError();
}

// both planes of 1 << LG frames, the frames as the kernels' kernarg table (FastBatch<1 << LG>)
template <int LG>
static hipError_t launch_nv12(const FrameSet* frames, const FastMapperPlane& y, const FastMapperPlane& uv, int W, int H,
                              uint8_t* const* out, int64_t out_pitch, hipStream_t s) {
    constexpr int cam_lg = LG <= 1 ? 5 : 4;
    FastBatch<1 << LG> b;
    memset(&b, 0, sizeof b);
    for (int f = 0; f < (1 << LG); f++) {
        for (int i = 0; i < (1 << cam_lg); i++) b.src[(f << cam_lg) + i] = frames[f].f[i];
        b.out[f] = out[f];
    }
    const hipError_t e = launch_plane<0, LG>(b, y, W, H, out_pitch, s);
    if (e != hipSuccess) return e;
    return launch_plane<1, LG>(b, uv, W, H, out_pitch, s);
}

hipError_t launch_fastmapper_nv12_batch(const FrameSet* frames, int nf, const FastMapperPlane& y,
                                        const FastMapperPlane& uv, int W, int H, uint8_t* const* out, int64_t out_pitch,
                                        hipStream_t s) {
    const int lg = nf == 1 ? 0 : nf == 2 ? 1 : nf == 4 ? 2 : -1;
    if (lg < 0) return hipErrorInvalidValue;
    const int cam_lg = lg <= 1 ? 5 : 4;
    for (int f = 0; f < nf; f++)
        for (int i = 1 << cam_lg; i < kMaxCams; i++)
            if (frames[f].f[i].yuv) return hipErrorInvalidValue;  // more cameras than a 4-frame batch holds
    if (lg == 2) return launch_nv12<2>(frames, y, uv, W, H, out, out_pitch, s);
    if (lg == 1) return launch_nv12<1>(frames, y, uv, W, H, out, out_pitch, s);
    return launch_nv12<0>(frames, y, uv, W, H, out, out_pitch, s);
}

hipError_t launch_fastmapper_nv12(const FrameSet& frames, const FastMapperPlane& y, const FastMapperPlane& uv, int W,
                                  int H, uint8_t* out, int64_t out_pitch, hipStream_t s) {
    return launch_fastmapper_nv12_batch(&frames, 1, y, uv, W, H, &out, out_pitch, s);
}

}  // namespace octvr
