// fastmapper.cpp — vr::FastMapper (modules/octvr/src/mapper_fast.cpp:27-109): per-rig setup of the NV12
// feather stitch (fastmapper.hip).  Everything here runs once per rig on host threads:
//   convertMaps(map * in_size, CV_16SC2) for the luma maps and for the half-size chroma maps
//     (cv::resize of the f32 maps, 2x area fast path), imgwarp.cpp:4831-5044, 2284-2460;
//   feather weights w_i = max(distanceTransform(mask_i) - 5, 0), u8 = sat(rne(255 * w_i / (1e-5 + sum w))),
//     half-size weights by the u8 area fast path (mapper_fast.cpp:75-94);
//   per 256-pixel run, the bit mask of cameras with a non-zero weight, and the entries of exactly those
//   (camera, run) pairs as consecutive 256-entry blocks (camera order), so the per-frame kernels read no
//   entry of a camera that has zero weight on the whole run (C2 full frame: about 4 blocks per run instead
//   of one per camera: the fisheyes' feather weights overlap widely).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "host_common.hpp"

using namespace octvr;

namespace octvr {
hipError_t launch_fastmapper_nv12(const FrameSet& frames, const FastMapperPlane& y, const FastMapperPlane& uv, int W,
                                  int H, uint8_t* out, int64_t out_pitch, hipStream_t s);
hipError_t launch_fastmapper_nv12_batch(const FrameSet* frames, int nf, const FastMapperPlane& y,
                                        const FastMapperPlane& uv, int W, int H, uint8_t* const* out, int64_t out_pitch,
                                        hipStream_t s);
}

// One plane's entries: per (run, camera with weight in the run) a block of 256, on the host (FastPlaneHost,
// built once per rig without touching the GPU) and on the device (FastPlaneDev).
struct FastPlaneHost {
    bool compact = true;
    std::vector<uint2> ent;    // wide entries (kept for the audit in both formats)
    std::vector<uint32_t> off; // compact: dx | dy << 11 | code << 22
    std::vector<uint8_t> wgt;  // compact: feather weight
    std::vector<uint2> hdr;    // compact: per block {bsx | bsy << 16, 0}
    std::vector<uint2> runs;   // per run: camera mask, first block
    size_t nblk = 0;           // blocks in use (the arrays hold max(nblk, 1))
};

struct FastPlaneDev {
    bool compact = true;
    uint32_t nblk = 0;
    DevBuf<uint2> ent;
    DevBuf<uint32_t> off;
    DevBuf<uint8_t> wgt;
    DevBuf<uint2> hdr;
    DevBuf<uint2> runs;
    FastMapperPlane view() const {
        return FastMapperPlane{compact, ent.p, off.p, wgt.p, hdr.p, runs.p, std::max<uint32_t>(nblk, 1u)};
    }
};

// Everything FastMapper's constructor computes (mapper_fast.cpp:27-109), host side.
struct FastPlan {
    int n = 0, W = 0, H = 0;
    std::vector<int> in_w, in_h;
    FastPlaneHost y, uv;
    double bytes = 0;  // algorithmic bytes per stitch (octvr_fastmapper_traffic)
    double lut_bytes = 0;  // of which the entries, weights and block headers (read once per launch)
};

struct octvr_fastmapper {
    int device = 0, n = 0, W = 0, H = 0;
    std::vector<int> in_w, in_h;
    FastPlaneDev y, uv;
    double bytes = 0, lut_bytes = 0;
    size_t blocks = 0;  // 256-entry (camera, run) blocks, Y + UV
};

namespace {

int sat_int_rne(float v) {  // saturate_cast<int>(float)
    if (v != v) return INT32_MIN;
    if (v >= 2147483648.f) return INT32_MAX;
    if (v < -2147483648.f) return INT32_MIN;
    return (int)lrintf(v);
}
uint32_t sat_s16(int v) { return (uint32_t)(uint16_t)(int16_t)std::min(32767, std::max(-32768, v)); }
uint8_t sat_u8_rte(float v) { return !(v > 0.f) ? 0 : v >= 255.f ? 255 : (uint8_t)lrintf(v); }

// convertMaps of one element (imgwarp.cpp:5039-5043) with the MatExpr scale m * s in f32, packed with
// the weight into the kernel's entry.
uint2 make_entry(float m1, float m2, float sx, float sy, uint8_t w) {
    const float X = m1 * sx + 0.f, Y = m2 * sy + 0.f;
    const int ix = sat_int_rne(X * 32), iy = sat_int_rne(Y * 32);
    uint2 e;
    e.x = sat_s16(ix >> 5) | (sat_s16(iy >> 5) << 16);
    e.y = (uint32_t)((iy & 31) * 32 + (ix & 31)) | ((uint32_t)w << 16);
    return e;
}

// The compact form of a plane's wide entries: per block the smallest in-use tap (entries of weight 0
// are never used; their offsets stay 0, i.e. that tap) as the header, per entry the 11-bit offsets from
// it, the fractions and the weight.  Header word y, bit kFastInterior (fastmapper.hip): every in-use entry
// has its taps at x <= pw - 2, y <= ph - 3 of its camera's plane (blk_cam), so the kernel may take them
// without clamps or masks.  Returns false when some block's in-use taps span 2048 pixels or more.
constexpr uint32_t kFastInterior = 1u;
bool compact_entries(const std::vector<uint2>& e, size_t nblk, const std::vector<uint8_t>& blk_cam,
                     const std::vector<int>& plane_w, const std::vector<int>& plane_h, std::vector<uint32_t>& off,
                     std::vector<uint8_t>& wgt, std::vector<uint2>& hdr) {
    off.assign(e.size(), 0u);
    wgt.assign(e.size(), 0u);
    hdr.assign(std::max<size_t>(nblk, 1), make_uint2(0u, 0u));
    std::vector<uint8_t> fits(std::max<size_t>(nblk, 1), 1);
    parallel_for(nblk, [&](size_t b) {
        int x0 = 32767, y0 = 32767, x1 = -32768, y1 = -32768;
        for (size_t k = b * 256; k < b * 256 + 256; k++) {
            if (!(e[k].y >> 16)) continue;
            const int sx = (int)(int16_t)(e[k].x & 0xFFFFu), sy = (int)(int16_t)(e[k].x >> 16);
            x0 = std::min(x0, sx), x1 = std::max(x1, sx), y0 = std::min(y0, sy), y1 = std::max(y1, sy);
        }
        if (x1 < x0) x0 = x1 = y0 = y1 = 0;
        if (x1 - x0 >= 2048 || y1 - y0 >= 2048) {
            fits[b] = 0;
            return;
        }
        const int cw = plane_w[blk_cam[b]], ch = plane_h[blk_cam[b]];
        const bool interior = x1 >= x0 && x0 >= 0 && y0 >= 0 && x1 <= cw - 2 && y1 <= ch - 3;
        hdr[b] = make_uint2((uint32_t)(uint16_t)x0 | (uint32_t)(uint16_t)y0 << 16, interior ? kFastInterior : 0u);
        for (size_t k = b * 256; k < b * 256 + 256; k++) {
            const uint32_t w = e[k].y >> 16;
            wgt[k] = (uint8_t)w;
            if (!w) continue;
            const int sx = (int)(int16_t)(e[k].x & 0xFFFFu), sy = (int)(int16_t)(e[k].x >> 16);
            off[k] = (uint32_t)(sx - x0) | (uint32_t)(sy - y0) << 11 | (e[k].y & 1023u) << 22;
        }
    });
    for (size_t b = 0; b < nblk; b++)
        if (!fits[b]) return false;
    return true;
}

// cv::resize(f32 map, half size): resizeAreaFast with the SSE grouping (imgwarp.cpp:2284-2337, 2441-2454).
float half_f32(const float* s0, const float* s1, int x, int vec) {
    const float a = s0[2 * x], b = s0[2 * x + 1], c = s1[2 * x], d = s1[2 * x + 1];
    const float sum = x < vec ? (a + b) + (c + d) : 0.f + (((a + b) + c) + d);
    return sum * 0.25f;
}

}  // namespace

// FastMapper(mt, in_sizes) on the host: feather weights, per-run camera masks, convertMaps entries of
// both planes and their compact form; force_wide keeps the 8-byte entries (OCTVR_FAST_WIDE=1, tests).
static FastPlan fast_plan(const octvr_rig* rig, int n_inputs, const int* in_w, const int* in_h, bool force_wide) {
    REQUIRE(rig && in_w && in_h, "NULL argument");
    REQUIRE(rig->overlays.empty(), "FastMapper does not support overlays (mapper_fast.cpp:31)");
    const int n = (int)rig->inputs.size();
    REQUIRE(n_inputs == n && n > 0 && n <= kMaxCams && n <= 32, "in_sizes must cover the inputs (<= 32)");
    const int W = rig->out_w, H = rig->out_h;
    REQUIRE(W % 2 == 0 && H % 2 == 0, "NV12 output needs even width/height");
    REQUIRE((int64_t)W * H < ((int64_t)1 << 31), "output of 2^31 pixels or more");
    for (int i = 0; i < n; i++) {
        const RigInput& in = rig->inputs[i];
        // "does not support ROI yet" (mapper_fast.cpp:50-51): every map covers the whole output
        REQUIRE(in.roi[0] == 0 && in.roi[1] == 0 && in.roi[2] == W && in.roi[3] == H,
                "FastMapper needs full-frame templates (dump without ROI)");
        REQUIRE(in_w[i] > 0 && in_h[i] > 0 && in_w[i] % 2 == 0 && in_h[i] % 2 == 0 && in_w[i] < 32768 && in_h[i] < 32768,
                "input sizes must be even and < 32768");
    }
    FastPlan P;
    P.n = n;
    P.W = W;
    P.H = H;
    P.in_w.assign(in_w, in_w + n);
    P.in_h.assign(in_h, in_h + n);
    const size_t npx = (size_t)W * H, hw = (size_t)W / 2, hh = (size_t)H / 2, nh = hw * hh;
    // feather weights (mapper_fast.cpp:75-94): dst_weight_map = 1e-5 + sum_i max(DT_i - 5, 0)
    std::vector<std::vector<float>> wt(n);
    std::vector<float> total(npx, 1e-5f);
    for (int i = 0; i < n; i++) {
        wt[i].resize(npx);
        chamfer_l2_3x3(rig->inputs[i].mask.data(), W, H, wt[i].data());
    }
    parallel_for(npx, [&](size_t k) {
        float t = 1e-5f;
        for (int i = 0; i < n; i++) {
            const float v = wt[i][k] - 5.f;
            wt[i][k] = v > 0.f ? v : 0.f;
            t = wt[i][k] + t;
        }
        total[k] = t;
    });
    const size_t runs_y = (npx + 255) / 256, runs_uv = (nh + 255) / 256;
    std::vector<uint32_t> my(runs_y, 0u), muv(runs_uv, 0u);
    std::vector<std::vector<uint8_t>> fmask(n, std::vector<uint8_t>(npx)), hmask(n, std::vector<uint8_t>(nh));
    for (int i = 0; i < n; i++) {
        // divide(weight_i, dst_weight_map) then convertTo(CV_8U, 255): fma(r, 255, 0), rne, saturate
        uint8_t* fm_i = fmask[i].data();
        parallel_for(npx, [&](size_t k) {
            const float e2 = total[k];
            const float r = e2 != 0.f ? wt[i][k] / e2 : 0.f;
            fm_i[k] = sat_u8_rte(fmaf(r, 255.f, 0.f));
        });
        // cv::resize(feather_mask, half): u8 area fast path (a + b + c + d + 2) >> 2
        uint8_t* hm_i = hmask[i].data();
        parallel_for(hh, [&](size_t y) {
            for (size_t x = 0; x < hw; x++) {
                const uint8_t* s = fm_i + (2 * y) * W + 2 * x;
                hm_i[y * hw + x] = (uint8_t)((s[0] + s[1] + s[W] + s[W + 1] + 2) >> 2);
            }
        });
        for (size_t k = 0; k < npx; k++)
            if (fm_i[k]) my[k / 256] |= 1u << i;
        for (size_t k = 0; k < nh; k++)
            if (hm_i[k]) muv[k / 256] |= 1u << i;
    }
    // blocks: run r's cameras (ascending) at first[r], first[r] + 1, ...
    auto blocks = [](const std::vector<uint32_t>& m, std::vector<uint2>& runs) {
        runs.resize(m.size());
        uint32_t b = 0;
        for (size_t r = 0; r < m.size(); r++) {
            runs[r] = make_uint2(m[r], b);
            b += (uint32_t)__builtin_popcount(m[r]);
        }
        return (size_t)b;
    };
    std::vector<uint2> ry, ruv;
    const size_t by = blocks(my, ry), buv = blocks(muv, ruv);
    REQUIRE(std::max(by, buv) * 256 < ((size_t)1 << 32), "FastMapper entries exceed 2^32");
    std::vector<uint2> ey(std::max<size_t>(by, 1) * 256, make_uint2(0u, 0u)), euv(std::max<size_t>(buv, 1) * 256, make_uint2(0u, 0u));
    std::vector<float> h1(nh), h2(nh);
    for (int i = 0; i < n; i++) {
        const RigInput& in = rig->inputs[i];
        const float sx = (float)in_w[i], sy = (float)in_h[i];
        const uint8_t* fm_i = fmask[i].data();
        parallel_for(runs_y, [&](size_t r) {
            if (!(my[r] >> i & 1u)) return;
            const size_t blk = ry[r].y + (size_t)__builtin_popcount(my[r] & ((1u << i) - 1u));
            for (size_t k = r * 256; k < std::min(npx, (r + 1) * 256); k++)
                ey[blk * 256 + (k - r * 256)] = make_entry(in.map1[k], in.map2[k], sx, sy, fm_i[k]);
        });
        const int vec = (int)(hw / 4 * 4);
        parallel_for(hh, [&](size_t y) {
            const float* a0 = in.map1.data() + (2 * y) * W;
            const float* b0 = in.map2.data() + (2 * y) * W;
            for (size_t x = 0; x < hw; x++) {
                h1[y * hw + x] = half_f32(a0, a0 + W, (int)x, vec);
                h2[y * hw + x] = half_f32(b0, b0 + W, (int)x, vec);
            }
        });
        // r_map * (in_size / 2): integer halving first (mapper_fast.cpp:62-64)
        const float hx = (float)(in_w[i] / 2), hy = (float)(in_h[i] / 2);
        const uint8_t* hm_i = hmask[i].data();
        parallel_for(runs_uv, [&](size_t r) {
            if (!(muv[r] >> i & 1u)) return;
            const size_t blk = ruv[r].y + (size_t)__builtin_popcount(muv[r] & ((1u << i) - 1u));
            for (size_t k = r * 256; k < std::min(nh, (r + 1) * 256); k++)
                euv[blk * 256 + (k - r * 256)] = make_entry(h1[k], h2[k], hx, hy, hm_i[k]);
        });
    }
    // the camera of every block (run r's cameras in ascending order from its first block)
    auto block_cams = [](const std::vector<uint32_t>& m, size_t nb) {
        std::vector<uint8_t> c(std::max<size_t>(nb, 1), 0);
        size_t b = 0;
        for (uint32_t mr : m)
            for (uint32_t x = mr; x; x &= x - 1) c[b++] = (uint8_t)__builtin_ctz(x);
        return c;
    };
    std::vector<int> pw_y(in_w, in_w + n), ph_y(in_h, in_h + n), pw_uv(n), ph_uv(n);
    for (int i = 0; i < n; i++) pw_uv[i] = in_w[i] / 2, ph_uv[i] = in_h[i] / 2;
    P.y.compact = !force_wide && compact_entries(ey, by, block_cams(my, by), pw_y, ph_y, P.y.off, P.y.wgt, P.y.hdr);
    P.uv.compact = !force_wide && compact_entries(euv, buv, block_cams(muv, buv), pw_uv, ph_uv, P.uv.off, P.uv.wgt, P.uv.hdr);
    for (FastPlaneHost* pl : {&P.y, &P.uv})
        if (!pl->compact) pl->off.clear(), pl->wgt.clear(), pl->hdr.clear();
    // per stitch: the entries read (compact: 5 B per entry and 8 B per block header; wide: 8 B per
    // entry), 1.5 B per output pixel written, and the source bytes the weighted taps reach (each once:
    // luma pixels 1 B, interleaved chroma pairs 2 B)
    auto ent_bytes = [](bool compact, size_t blocks) { return compact ? (5.0 * 256 + 8.0) * blocks : 8.0 * 256 * blocks; };
    P.lut_bytes = ent_bytes(P.y.compact, by) + ent_bytes(P.uv.compact, buv);
    P.bytes = P.lut_bytes + 1.5 * (double)npx;
    for (int i = 0; i < n; i++) {
        const int w = in_w[i], h = in_h[i];
        std::vector<uint8_t> ty((size_t)w * h, 0), tuv((size_t)(w / 2) * (h / 2), 0);
        auto touch = [](std::vector<uint8_t>& t, int tw, int th, uint2 e) {
            const int sx = (int)(int16_t)(e.x & 0xFFFFu), sy = (int)(int16_t)(e.x >> 16);
            for (int k = 0; k < 4; k++) {
                const int x = sx + (k & 1), y = sy + (k >> 1);
                if (x >= 0 && y >= 0 && x < tw && y < th) t[(size_t)y * tw + x] = 1;
            }
        };
        for (size_t r = 0; r < runs_y; r++) {
            if (!(my[r] >> i & 1u)) continue;
            const size_t blk = ry[r].y + (size_t)__builtin_popcount(my[r] & ((1u << i) - 1u));
            for (size_t k = 0; k < 256; k++)
                if (ey[blk * 256 + k].y >> 16) touch(ty, w, h, ey[blk * 256 + k]);
        }
        for (size_t r = 0; r < runs_uv; r++) {
            if (!(muv[r] >> i & 1u)) continue;
            const size_t blk = ruv[r].y + (size_t)__builtin_popcount(muv[r] & ((1u << i) - 1u));
            for (size_t k = 0; k < 256; k++)
                if (euv[blk * 256 + k].y >> 16) touch(tuv, w / 2, h / 2, euv[blk * 256 + k]);
        }
        double c = 0;
        for (uint8_t v : ty) c += v;
        for (uint8_t v : tuv) c += 2.0 * v;
        P.bytes += c;
    }
    P.y.nblk = by;
    P.uv.nblk = buv;
    P.y.runs = std::move(ry);
    P.uv.runs = std::move(ruv);
    P.y.ent = std::move(ey);
    P.uv.ent = std::move(euv);
    return P;
}

static bool force_wide_env() {  // OCTVR_FAST_WIDE=1 keeps the 8-byte entries (tests of the wide kernels)
    const char* e = getenv("OCTVR_FAST_WIDE");
    return e && e[0] == '1';
}

// Replays, on the host, every index fast_y_kernel / fast_uv_kernel derive (fastmapper.hip fast_plane) for
// every run, camera group, slot and lane of one plane, and checks each against the allocation the plan
// uploads: runs[blockIdx], the block b = (live ? blk + k : blk) against nblk (the kernel also clamps it),
// the entry / weight index b * 256 + lane and the header b against the arrays of the plane's format, the
// camera against the frame set, the 8-byte tap-row load start st against the frame (NV12 of pitch
// w + pitch_pad: st + 8 <= size), the byte selectors of in-image taps (inside the 8 loaded bytes and
// equal to the tap's own byte), and the last output byte of each run.  Counts go to `c`.
struct AuditCounts {
    uint64_t groups = 0, slot_loads = 0, live_slots = 0, taps_in = 0, violations = 0, interior_slots = 0;
    int64_t max_block = -1;
    std::string first;
};
static void audit_plane(const FastPlan& P, const FastPlaneHost& pl, int plane, size_t pitch_pad, AuditCounts& c) {
    const uint32_t bpp = plane ? 2u : 1u;
    const uint32_t pw = plane ? P.W / 2 : P.W, ph = plane ? P.H / 2 : P.H;
    const uint64_t npx = (uint64_t)pw * ph;
    const size_t nruns = (size_t)((npx + 255) / 256);
    const size_t cap_e = pl.compact ? std::min(pl.off.size(), pl.wgt.size()) : pl.ent.size();
    const size_t cap_h = pl.compact ? pl.hdr.size() : (size_t)-1;
    std::mutex mu;
    auto bad = [&](const char* what, size_t r, int k, uint32_t lane) {
        std::lock_guard<std::mutex> lk(mu);
        if (c.violations++ == 0) {
            char b[200];
            snprintf(b, sizeof b, "plane %d run %zu slot %d lane %u: %s", plane, r, k, lane, what);
            c.first = b;
        }
    };
    if (pl.runs.size() != nruns) bad("runs[] does not match the grid", 0, -1, 0);
    std::vector<AuditCounts> part(16);
    const size_t T = part.size();
    run_threads(T, [&](size_t t) {
        AuditCounts& a = part[t];
        for (size_t r = nruns * t / T; r < std::min(nruns * (t + 1) / T, pl.runs.size()); r++) {
            uint32_t m = pl.runs[r].x, blk = pl.runs[r].y;
            while (m) {
                a.groups++;
                bool live[4];
                int cam[4];
                uint32_t b[4];
                for (int k = 0; k < 4; k++) {
                    live[k] = m != 0u;
                    cam[k] = live[k] ? __builtin_ctz(m) : 0;
                    m &= m - 1u;
                    b[k] = live[k] ? blk + (uint32_t)k : blk;
                    a.slot_loads++;
                    a.max_block = std::max<int64_t>(a.max_block, b[k]);
                    if (b[k] >= std::max<size_t>(pl.nblk, 1)) bad("block index past the plane's blocks", r, k, 0);
                    if (pl.compact && b[k] >= cap_h) bad("header index past the headers", r, k, 0);
                    if ((uint64_t)b[k] * 256 + 255 >= cap_e) bad("entry index past the entries", r, k, 255);
                    if (live[k] && cam[k] >= P.n) bad("camera past the frame set", r, k, 0);
                }
                for (int k = 0; k < 4; k++) blk += live[k] ? 1u : 0u;
                for (int k = 0; k < 4; k++) {
                    if (!live[k] || b[k] >= pl.nblk) continue;
                    a.live_slots++;
                    if (pl.compact && (pl.hdr[b[k]].y & kFastInterior)) a.interior_slots++;
                    const int fw = P.in_w[cam[k]], fh = P.in_h[cam[k]];
                    const uint32_t pitch = (uint32_t)(fw + pitch_pad);
                    const uint32_t size = pitch * (uint32_t)(fh + fh / 2);
                    const int sw = plane ? fw / 2 : fw, sh = plane ? fh / 2 : fh;
                    const uint32_t base = plane ? (uint32_t)fh * pitch : 0u;
                    const bool interior = pl.compact && (pl.hdr[b[k]].y & kFastInterior) != 0;
                    for (uint32_t lane = 0; lane < 256; lane++) {
                        const size_t e = (size_t)b[k] * 256 + lane;
                        int sx, sy;
                        uint32_t w;
                        if (pl.compact) {
                            const uint32_t o = pl.off[e], h = pl.hdr[b[k]].x;
                            sx = (int)(int16_t)(h & 0xFFFFu) + (int)(o & 2047u);
                            sy = (int)(int16_t)(h >> 16) + (int)((o >> 11) & 2047u);
                            w = pl.wgt[e];
                            if (w) {  // the compact form holds the same tap as the wide entry
                                const uint2 we = pl.ent[e];
                                if (sx != (int)(int16_t)(we.x & 0xFFFFu) || sy != (int)(int16_t)(we.x >> 16) ||
                                    (o >> 22) != (we.y & 1023u) || w != (we.y >> 16))
                                    bad("compact entry differs from the wide one", r, k, lane);
                            }
                        } else {
                            const uint2 we = pl.ent[e];
                            sx = (int)(int16_t)(we.x & 0xFFFFu);
                            sy = (int)(int16_t)(we.x >> 16);
                            w = we.y >> 16;
                        }
                        // interior blocks (fast_group<INNER>): no clamps — the claim itself is checked
                        if (interior && w && !(sx >= 0 && sy >= 0 && sx <= sw - 2 && sy <= sh - 3))
                            bad("interior block with a tap near or past the plane's edge", r, k, lane);
                        if (interior && !w && (sx < 0 || sy < 0 || sx > sw - 2 || sy > sh - 3))
                            bad("interior block with an unused entry off the interior", r, k, lane);
                        const int xa = interior ? sx : std::min(std::max(sx, 0), sw - 1);
                        const uint32_t bx = (uint32_t)xa * bpp & ~3u;
                        for (int rr = 0; rr < 2; rr++) {
                            const int y = interior ? sy + rr : std::min(std::max(sy + rr, 0), sh - 1);
                            const uint32_t row = base + (uint32_t)y * pitch;
                            if (size < 8u) { bad("frame under 8 bytes", r, k, lane); continue; }
                            const uint32_t st = interior ? row + bx : std::min(row + bx, size - 8u);
                            if ((uint64_t)st + 8 > size) bad("tap-row load past the frame", r, k, lane);
                            if (!w) continue;
                            const uint32_t d = interior ? ((uint32_t)sx * bpp & 3u) : row + (uint32_t)sx * bpp - st;
                            for (int cc = 0; cc < 2; cc++) {  // in-image taps: their bytes in the loaded 8
                                const int tx = sx + cc, ty = sy + rr;
                                if (tx < 0 || ty < 0 || tx >= sw || ty >= sh) continue;
                                a.taps_in++;
                                const uint32_t i = (d + (uint32_t)cc * bpp) & 7u;
                                const uint64_t want = (uint64_t)base + (uint64_t)ty * pitch + (uint64_t)tx * bpp;
                                if (i + bpp - 1 > 7u || (uint64_t)st + i != want) bad("tap byte outside the loaded row", r, k, lane);
                            }
                        }
                    }
                }
            }
            // the output bytes of the run's lanes (y * pitch + x, chroma (H + y) * pitch + 2x + 1)
            const uint64_t i0 = (uint64_t)r * 256, i1 = std::min<uint64_t>(i0 + 256, npx);
            if (i1 > i0) {
                const uint64_t yl = (i1 - 1) / pw, xl = (i1 - 1) % pw;
                const uint64_t last = plane ? ((uint64_t)P.H + yl) * P.W + 2 * xl + 1 : yl * P.W + xl;
                if (last >= (uint64_t)P.W * (P.H + P.H / 2)) bad("output byte past the frame", r, -1, 0);
            }
        }
    });
    for (auto& a : part) {
        c.groups += a.groups;
        c.slot_loads += a.slot_loads;
        c.live_slots += a.live_slots;
        c.taps_in += a.taps_in;
        c.interior_slots += a.interior_slots;
        c.max_block = std::max(c.max_block, a.max_block);
    }
}

extern "C" {

int octvr_debug_fastmapper_audit(const octvr_rig* rig, int n_inputs, const int* in_w, const int* in_h, int force_wide,
                                 int pitch_pad, char* json, size_t len) {
    try {
        REQUIRE(json && len > 0 && pitch_pad >= 0 && pitch_pad < 4096, "bad arguments");
        const FastPlan P = fast_plan(rig, n_inputs, in_w, in_h, force_wide != 0);
        std::string js = "{";
        uint64_t viol = 0;
        for (int plane = 0; plane < 2; plane++) {
            const FastPlaneHost& pl = plane ? P.uv : P.y;
            AuditCounts c;
            audit_plane(P, pl, plane, (size_t)pitch_pad, c);
            viol += c.violations;
            char b[512];
            snprintf(b, sizeof b,
                     "%s\"%s\": {\"compact\": %d, \"runs\": %zu, \"blocks\": %zu, \"groups\": %llu, "
                     "\"slot_loads\": %llu, \"live_slots\": %llu, \"interior_slots\": %llu, \"taps_in_image\": %llu, \"max_block\": %lld, "
                     "\"violations\": %llu, \"first\": \"%s\"}",
                     plane ? ", " : "", plane ? "uv" : "y", pl.compact ? 1 : 0, pl.runs.size(), pl.nblk,
                     (unsigned long long)c.groups, (unsigned long long)c.slot_loads, (unsigned long long)c.live_slots,
                     (unsigned long long)c.interior_slots, (unsigned long long)c.taps_in, (long long)c.max_block, (unsigned long long)c.violations,
                     c.first.c_str());
            js += b;
        }
        js += "}";
        REQUIRE(js.size() < len, "buffer too small");
        memcpy(json, js.c_str(), js.size() + 1);
        return viol ? OCTVR_E_INVALID : OCTVR_OK;
    } catch (const OctvrError& e) {
        set_last_error(e.what());
        return e.code;
    } catch (const std::exception& e) {
        set_last_error(e.what());
        return OCTVR_E_INVALID;
    }
}

int octvr_fastmapper_create(const octvr_rig* rig, int device, int n_inputs, const int* in_w, const int* in_h,
                            octvr_fastmapper** out) {
    try {
        REQUIRE(rig && in_w && in_h && out, "NULL argument");
        FastPlan P = fast_plan(rig, n_inputs, in_w, in_h, force_wide_env());
        auto fm = std::make_unique<octvr_fastmapper>();
        fm->device = device;
        fm->n = P.n;
        fm->W = P.W;
        fm->H = P.H;
        fm->in_w = P.in_w;
        fm->in_h = P.in_h;
        fm->bytes = P.bytes;
        fm->lut_bytes = P.lut_bytes;
        fm->blocks = P.y.nblk + P.uv.nblk;
        DeviceGuard dg(device);
        auto upload = [](FastPlaneDev& d, const FastPlaneHost& h) {
            d.compact = h.compact;
            d.nblk = (uint32_t)h.nblk;
            if (h.compact) {
                d.off.upload(h.off.data(), h.off.size());
                d.wgt.upload(h.wgt.data(), h.wgt.size());
                d.hdr.upload(h.hdr.data(), h.hdr.size());
            } else {
                d.ent.upload(h.ent.data(), h.ent.size());
            }
            d.runs.upload(h.runs.data(), h.runs.size());
        };
        upload(fm->y, P.y);
        upload(fm->uv, P.uv);
        *out = fm.release();
        return OCTVR_OK;
    } catch (const OctvrError& e) {
        set_last_error(e.what());
        return e.code;
    } catch (const std::exception& e) {
        set_last_error(e.what());
        return OCTVR_E_HIP;
    }
}

int octvr_fastmapper_stitch_nv12_batch(octvr_fastmapper* fm, int n_frames, const uint8_t* const* in_dev,
                                       const size_t* in_pitch, uint8_t* const* out_dev, size_t out_pitch, void* stream) {
    try {
        REQUIRE(fm && in_dev && in_pitch && out_dev, "NULL argument");
        REQUIRE(n_frames == 1 || n_frames == 2 || n_frames == 4, "a batch holds 1, 2 or 4 frames");
        REQUIRE(n_frames <= 2 || fm->n <= 16, "a batch of 4 frames holds 16 cameras per frame");
        REQUIRE(out_pitch >= (size_t)fm->W, "output pitch smaller than width");
        DeviceGuard dg(fm->device);
        FrameSet fs[kMaxBatch];
        for (int f = 0; f < n_frames; f++) {
            REQUIRE(out_dev[f], "NULL output");
            memset(&fs[f], 0, sizeof fs[f]);
            for (int i = 0; i < fm->n; i++) {
                const uint8_t* p = in_dev[(size_t)f * fm->n + i];
                const size_t pitch = in_pitch[(size_t)f * fm->n + i];
                REQUIRE(p && pitch >= (size_t)fm->in_w[i] && pitch < ((size_t)1 << 24), "bad input frame");
                REQUIRE(pitch * (size_t)(fm->in_h[i] + fm->in_h[i] / 2) >= 8 &&
                            pitch * (size_t)(fm->in_h[i] + fm->in_h[i] / 2) < 0x7FFFFFFFull,
                        "input frame of fewer than 8 or more than 2^31 bytes");
                fs[f].f[i] = SourceFrame{p, fm->in_w[i], fm->in_h[i], (int64_t)pitch, nullptr};
            }
        }
        HIP_CHECK(launch_fastmapper_nv12_batch(fs, n_frames, fm->y.view(), fm->uv.view(), fm->W, fm->H, out_dev,
                                               (int64_t)out_pitch, (hipStream_t)stream));
        return OCTVR_OK;
    } catch (const OctvrError& e) {
        set_last_error(e.what());
        return e.code;
    }
}

int octvr_fastmapper_stitch_nv12(octvr_fastmapper* fm, const uint8_t* const* in_dev, const size_t* in_pitch,
                                 uint8_t* out_dev, size_t out_pitch, void* stream) {
    return octvr_fastmapper_stitch_nv12_batch(fm, 1, in_dev, in_pitch, &out_dev, out_pitch, stream);
}

int octvr_fastmapper_traffic(const octvr_fastmapper* fm, double* bytes) {
    if (!fm || !bytes) {
        set_last_error("NULL argument");
        return OCTVR_E_INVALID;
    }
    *bytes = fm->bytes;
    return OCTVR_OK;
}

int octvr_fastmapper_traffic_parts(const octvr_fastmapper* fm, double* lut_bytes, double* frame_bytes) {
    if (!fm || !lut_bytes || !frame_bytes) {
        set_last_error("NULL argument");
        return OCTVR_E_INVALID;
    }
    *lut_bytes = fm->lut_bytes;
    *frame_bytes = fm->bytes - fm->lut_bytes;
    return OCTVR_OK;
}

void octvr_fastmapper_destroy(octvr_fastmapper* fm) {
    if (!fm) return;
    int prev = -1;
    if (hipGetDevice(&prev) == hipSuccess && prev != fm->device) (void)hipSetDevice(fm->device);
    delete fm;
    if (prev >= 0) (void)hipSetDevice(prev);
}

}  // extern "C"
