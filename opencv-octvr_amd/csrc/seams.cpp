// seams.cpp — MapperTemplate::create_masks() for a rig without images (template.cpp:155-204):
// the L2 distance seam finder (DistanceSeamFinder, stitching/src/seam_finders.cpp:97-133).
//
// Work split: the two full-resolution resizes (each camera's LUT mask down to <= 960 px wide, and
// the seam mask back up to its ROI — 6 x 29.5 Mpx at 8K) run on the GPU (resize_u8_kernel,
// integer-only with host-built coefficient tables); the chamfer distance transform and the
// per-pixel arbitration work on the <= 960 px working images on host threads (two sequential
// raster passes per camera, as distransform.cpp:48-139 defines them).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstring>
#include <thread>
#include <vector>

#include "host_common.hpp"
#include "kernels.hpp"

namespace octvr {
namespace {

// Coefficient tables of cv::resize INTER_LINEAR (imgwarp.cpp:3290-3480), host side.
struct ResizePlan {
    std::vector<int32_t> xofs, rows;
    std::vector<int16_t> ax, by;
    int xmax = 0, area2 = 0;
};

int16_t coef(float v) {  // saturate_cast<short>(v * INTER_RESIZE_COEF_SCALE), round half even
    const long i = lrintf(v * 2048.f);
    return (int16_t)std::min(32767L, std::max(-32768L, i));
}

int floor_to_int(float v) {  // cvFloor(float)
    const int i = (int)v;
    return i - (i > v);
}

ResizePlan plan_resize(int sw, int sh, int dw, int dh) {
    ResizePlan p;
    const double scale_x = 1. / ((double)dw / sw), scale_y = 1. / ((double)dh / sh);
    const int isx = (int)std::lrint(scale_x), isy = (int)std::lrint(scale_y);
    // INTER_LINEAR at exactly 1/2 is INTER_AREA's fast path (imgwarp.cpp:3309-3312)
    if (std::fabs(scale_x - isx) < DBL_EPSILON && std::fabs(scale_y - isy) < DBL_EPSILON && isx == 2 && isy == 2) {
        p.area2 = 1;
        return p;
    }
    p.xofs.resize(dw);
    p.ax.resize(2 * (size_t)dw);
    p.xmax = dw;
    for (int dx = 0; dx < dw; dx++) {
        float fx = (float)((dx + 0.5) * scale_x - 0.5);
        int sx = floor_to_int(fx);
        fx -= sx;
        if (sx < 0) fx = 0, sx = 0;
        if (sx + 1 >= sw) {
            p.xmax = std::min(p.xmax, dx);
            if (sx >= sw - 1) fx = 0, sx = sw - 1;
        }
        p.xofs[dx] = sx;
        p.ax[2 * dx] = coef(1.f - fx);
        p.ax[2 * dx + 1] = coef(fx);
    }
    p.rows.resize(2 * (size_t)dh);
    p.by.resize(2 * (size_t)dh);
    for (int dy = 0; dy < dh; dy++) {
        float fy = (float)((dy + 0.5) * scale_y - 0.5);
        const int sy = floor_to_int(fy);
        fy -= sy;
        p.rows[2 * dy] = std::min(std::max(sy, 0), sh - 1);
        p.rows[2 * dy + 1] = std::min(std::max(sy + 1, 0), sh - 1);
        p.by[2 * dy] = coef(1.f - fy);
        p.by[2 * dy + 1] = coef(fy);
    }
    return p;
}

// Resize a host u8 image through the GPU (same size: plain copy, imgwarp.cpp:3264-3268).
std::vector<uint8_t> resize_on_device(const uint8_t* src, int sw, int sh, int dw, int dh) {
    std::vector<uint8_t> out((size_t)dw * dh);
    if (sw == dw && sh == dh) {
        memcpy(out.data(), src, out.size());
        return out;
    }
    const ResizePlan p = plan_resize(sw, sh, dw, dh);
    DevBuf<uint8_t> s, d;
    DevBuf<int32_t> xofs, rows;
    DevBuf<int16_t> ax, by;
    s.upload(src, (size_t)sw * sh);
    d.alloc(out.size());
    ResizeTables t{};
    t.area2 = p.area2;
    if (!p.area2) {
        xofs.upload(p.xofs.data(), p.xofs.size());
        ax.upload(p.ax.data(), p.ax.size());
        rows.upload(p.rows.data(), p.rows.size());
        by.upload(p.by.data(), p.by.size());
        t = ResizeTables{xofs.p, ax.p, rows.p, by.p, p.xmax, 0};
    }
    HIP_CHECK(launch_resize_u8(s.p, sw, sh, sw, d.p, dw, dh, dw, t, nullptr));
    HIP_CHECK(hipMemcpy(out.data(), d.p, out.size(), hipMemcpyDeviceToHost));
    return out;
}

}  // namespace

// distanceTransform(DIST_L2, 3x3) -> f32 (distransform.cpp:48-139): integer chamfer distances in
// 16.16 fixed point, metrics a = 0.955, b = 1.3693 (:402-420), one forward and one backward pass.
void chamfer_l2_3x3(const uint8_t* src, int w, int h, float* dist) {
    constexpr int kFar = 0x7FFFFFFF >> 2;
    const int a = (int)std::lrint(0.955f * 65536.0), b = (int)std::lrint(1.3693f * 65536.0);
    const int stride = w + 2;
    std::vector<int> t((size_t)stride * (h + 2), kFar);  // one-pixel frame at "infinity"
    auto row = [&](int y) { return t.data() + (size_t)(y + 1) * stride + 1; };
    for (int y = 0; y < h; y++) {
        const uint8_t* s = src + (size_t)y * w;
        int* r = row(y);
        const int* u = row(y - 1);
        for (int x = 0; x < w; x++)
            r[x] = s[x] ? std::min(std::min(u[x - 1] + b, u[x] + a), std::min(u[x + 1] + b, r[x - 1] + a)) : 0;
    }
    for (int y = h - 1; y >= 0; y--) {
        int* r = row(y);
        const int* d = row(y + 1);
        float* o = dist + (size_t)y * w;
        for (int x = w - 1; x >= 0; x--) {
            int v = r[x];
            if (v > a) {
                // same comparison order as the reference (ties cannot change a min)
                v = std::min(v, d[x + 1] + b);
                v = std::min(v, d[x] + a);
                v = std::min(v, d[x - 1] + b);
                v = std::min(v, r[x + 1] + a);
                r[x] = v;
            }
            o[x] = (float)(v * (1.f / 65536));
        }
    }
}


void rig_create_masks(octvr_rig& rig) {
    const int n = (int)rig.inputs.size();
    REQUIRE(n > 0, "rig has no inputs");
    REQUIRE(n <= 16, "seam arbitration is defined for at most 16 inputs (std::sort is stable only up to 16)");
    DeviceGuard dg(rig.device);
    const double scale = std::min(1.0, 960.0 / rig.out_w);
    struct Work {
        int x, y, w, h;  // scaled ROI (cv::Rect from doubles: truncation)
        std::vector<uint8_t> mask;
        std::vector<float> dist;
    };
    std::vector<Work> wk(n);
    int rx0 = 0, ry0 = 0, rx1 = 0, ry1 = 0;
    for (int i = 0; i < n; i++) {
        const RigInput& in = rig.inputs[i];
        Work& k = wk[i];
        k.x = (int)(in.roi[0] * scale);
        k.y = (int)(in.roi[1] * scale);
        k.w = (int)(in.roi[2] * scale);
        k.h = (int)(in.roi[3] * scale);
        REQUIRE(k.w > 0 && k.h > 0, "scaled ROI is empty");
        k.mask = resize_on_device(in.mask.data(), in.roi[2], in.roi[3], k.w, k.h);
        rx0 = i ? std::min(rx0, k.x) : k.x;
        ry0 = i ? std::min(ry0, k.y) : k.y;
        rx1 = i ? std::max(rx1, k.x + k.w) : k.x + k.w;
        ry1 = i ? std::max(ry1, k.y + k.h) : k.y + k.h;
    }
    // distances, one host thread per camera; a camera spanning the whole width (and starting at
    // column 0) is transformed as three side-by-side copies so the seam wraps at +-180 degrees
    // (warpedDistanceTransform, seam_finders.cpp:86-95)
    run_threads((size_t)n, [&](size_t i) {
        Work& k = wk[i];
        k.dist.resize((size_t)k.w * k.h);
        if (k.x == 0 && k.w == rx1 - rx0) {
            std::vector<uint8_t> tri((size_t)3 * k.w * k.h);
            for (int y = 0; y < k.h; y++)
                for (int c = 0; c < 3; c++)
                    memcpy(&tri[((size_t)y * 3 + c) * k.w], &k.mask[(size_t)y * k.w], k.w);
            std::vector<float> d3(tri.size());
            chamfer_l2_3x3(tri.data(), 3 * k.w, k.h, d3.data());
            for (int y = 0; y < k.h; y++)
                memcpy(&k.dist[(size_t)y * k.w], &d3[((size_t)y * 3 + 1) * k.w], sizeof(float) * k.w);
        } else {
            chamfer_l2_3x3(k.mask.data(), k.w, k.h, k.dist.data());
        }
    });
    // arbitration: each working pixel keeps only the camera with the largest distance (first
    // camera on ties); the masks are read-only here except for the zeroing of losers, and the
    // distances were fixed beforehand, so rows are independent
    const int T = (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    run_threads((size_t)T, [&](size_t t) {
        const int tid = (int)t;
        for (int y = ry0 + tid; y < ry1; y += T)
            for (int x = rx0; x < rx1; x++) {
                int best = -1;
                float bd = -1.f;
                for (int i = 0; i < n; i++) {
                    const Work& k = wk[i];
                    if (y < k.y || x < k.x || y - k.y >= k.h || x - k.x >= k.w) continue;
                    const float d = k.dist[(size_t)(y - k.y) * k.w + (x - k.x)];
                    if (best < 0 || d > bd) best = i, bd = d;
                }
                for (int i = 0; i < n; i++) {
                    Work& k = wk[i];
                    if (i == best || y < k.y || x < k.x || y - k.y >= k.h || x - k.x >= k.w) continue;
                    k.mask[(size_t)(y - k.y) * k.w + (x - k.x)] = 0;
                }
            }
    });
    rig.seam_masks.resize(n);
    for (int i = 0; i < n; i++) {
        const RigInput& in = rig.inputs[i];
        rig.seam_masks[i] = resize_on_device(wk[i].mask.data(), wk[i].w, wk[i].h, in.roi[2], in.roi[3]);
    }
}

}  // namespace octvr
