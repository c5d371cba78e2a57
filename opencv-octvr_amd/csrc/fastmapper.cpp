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
#include <thread>
#include <vector>

#include "host_common.hpp"

using namespace octvr;

namespace octvr {
hipError_t launch_fastmapper_nv12(const FrameSet& frames, const FastMapperPlane& y, const FastMapperPlane& uv, int W,
                                  int H, uint8_t* out, int64_t out_pitch, hipStream_t s);
}

// one plane's entries on the device: per (run, camera with weight in the run) a block of 256
struct FastPlaneDev {
    bool compact = true;
    DevBuf<uint2> ent;    // wide entries
    DevBuf<uint32_t> off; // compact: dx | dy << 11 | code << 22
    DevBuf<uint8_t> wgt;  // compact: feather weight
    DevBuf<uint2> hdr;    // compact: per block {bsx | bsy << 16, 0}
    DevBuf<uint2> runs;   // per run: camera mask, first block
    FastMapperPlane view() const { return FastMapperPlane{compact, ent.p, off.p, wgt.p, hdr.p, runs.p}; }
};

struct octvr_fastmapper {
    int device = 0, n = 0, W = 0, H = 0;
    std::vector<int> in_w, in_h;
    FastPlaneDev y, uv;
    double bytes = 0;                // algorithmic bytes per stitch (octvr_fastmapper_traffic)
    size_t blocks = 0;               // 256-entry (camera, run) blocks, Y + UV
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
// are never used) as the header, per entry the 11-bit offsets from it, the fractions and the weight.
// Returns false (nothing written) when some block's in-use taps span 2048 pixels or more.
bool compact_entries(const std::vector<uint2>& e, size_t nblk, std::vector<uint32_t>& off, std::vector<uint8_t>& wgt,
                     std::vector<uint2>& hdr) {
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
        hdr[b] = make_uint2((uint32_t)(uint16_t)x0 | (uint32_t)(uint16_t)y0 << 16, 0u);
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

extern "C" {

int octvr_fastmapper_create(const octvr_rig* rig, int device, int n_inputs, const int* in_w, const int* in_h,
                            octvr_fastmapper** out) {
    try {
        REQUIRE(rig && in_w && in_h && out, "NULL argument");
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
        auto fm = std::make_unique<octvr_fastmapper>();
        fm->device = device;
        fm->n = n;
        fm->W = W;
        fm->H = H;
        fm->in_w.assign(in_w, in_w + n);
        fm->in_h.assign(in_h, in_h + n);
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
        // OCTVR_FAST_WIDE=1 keeps the 8-byte entries (tests of the wide kernels)
        const char* wide_env = getenv("OCTVR_FAST_WIDE");
        const bool force_wide = wide_env && wide_env[0] == '1';
        std::vector<uint32_t> oy, ouv;
        std::vector<uint8_t> wy, wuv;
        std::vector<uint2> hy, huv;
        fm->y.compact = !force_wide && compact_entries(ey, by, oy, wy, hy);
        fm->uv.compact = !force_wide && compact_entries(euv, buv, ouv, wuv, huv);
        // per stitch: the entries read (compact: 5 B per entry and 8 B per block header; wide: 8 B per
        // entry), 1.5 B per output pixel written, and the source bytes the weighted taps reach (each once:
        // luma pixels 1 B, interleaved chroma pairs 2 B)
        auto ent_bytes = [](bool compact, size_t blocks) { return compact ? (5.0 * 256 + 8.0) * blocks : 8.0 * 256 * blocks; };
        fm->bytes = ent_bytes(fm->y.compact, by) + ent_bytes(fm->uv.compact, buv) + 1.5 * (double)npx;
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
            fm->bytes += c;
        }
        fm->blocks = by + buv;
        DeviceGuard dg(device);
        auto upload = [](FastPlaneDev& d, const std::vector<uint2>& e, const std::vector<uint32_t>& o,
                         const std::vector<uint8_t>& w, const std::vector<uint2>& h, const std::vector<uint2>& runs) {
            if (d.compact) {
                d.off.upload(o.data(), o.size());
                d.wgt.upload(w.data(), w.size());
                d.hdr.upload(h.data(), h.size());
            } else {
                d.ent.upload(e.data(), e.size());
            }
            d.runs.upload(runs.data(), runs.size());
        };
        upload(fm->y, ey, oy, wy, hy, ry);
        upload(fm->uv, euv, ouv, wuv, huv, ruv);
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

int octvr_fastmapper_stitch_nv12(octvr_fastmapper* fm, const uint8_t* const* in_dev, const size_t* in_pitch,
                                 uint8_t* out_dev, size_t out_pitch, void* stream) {
    try {
        REQUIRE(fm && in_dev && in_pitch && out_dev, "NULL argument");
        REQUIRE(out_pitch >= (size_t)fm->W, "output pitch smaller than width");
        DeviceGuard dg(fm->device);
        FrameSet fs;
        memset(&fs, 0, sizeof fs);
        for (int i = 0; i < fm->n; i++) {
            REQUIRE(in_dev[i] && in_pitch[i] >= (size_t)fm->in_w[i] && in_pitch[i] < ((size_t)1 << 24), "bad input frame");
            REQUIRE(in_pitch[i] * (size_t)(fm->in_h[i] + fm->in_h[i] / 2) >= 8 &&
                        in_pitch[i] * (size_t)(fm->in_h[i] + fm->in_h[i] / 2) < 0x7FFFFFFFull,
                    "input frame of fewer than 8 or more than 2^31 bytes");
            fs.f[i] = SourceFrame{in_dev[i], fm->in_w[i], fm->in_h[i], (int64_t)in_pitch[i], nullptr};
        }
        HIP_CHECK(launch_fastmapper_nv12(fs, fm->y.view(), fm->uv.view(), fm->W, fm->H, out_dev, (int64_t)out_pitch,
                                         (hipStream_t)stream));
        return OCTVR_OK;
    } catch (const OctvrError& e) {
        set_last_error(e.what());
        return e.code;
    }
}

int octvr_fastmapper_traffic(const octvr_fastmapper* fm, double* bytes) {
    if (!fm || !bytes) {
        set_last_error("NULL argument");
        return OCTVR_E_INVALID;
    }
    *bytes = fm->bytes;
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
