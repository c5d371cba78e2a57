// multiband_host.cpp — host orchestration of the multi-band blend (Mapper blend > 0):
// MultiBandGPUBlender (stitching/src/blenders.cpp:589-735) laid out for the MI355X.
//
// Build (once per rig, all on `device`):
//   * rectangles exactly as the reference: result ROI, align_result_roi (multiples of 2^B), per
//     camera align_rois with the 5 * 2^B gap (blenders.cpp:595-618);
//   * weights: level 0 = seam / 255 (kept as the u8 seam, converted in-kernel bit-exactly), levels
//     1..B = K4 pyrDown in f32 (multiband.hip); per level and tile the set of cameras with a non-zero
//     weight (tile_cams);
//   * pyrUp tap tables (UpQuad) per camera and level, and for the collapse;
//   * "required" tile sets per camera and level: a camera's Gaussian level is computed only on the
//     tiles that its blend reads (its weight tiles, the pyrUp support of its finer level's weight
//     tiles) and, transitively, the pyrDown support of its coarser required tiles.  For a rig whose
//     seams split the panorama, this is ~1.2-1.5 cameras per pixel instead of every camera
//     everywhere (the reference computes all pyramids over every align_roi);
//   * the level-0 remap as a tiled composite LUT over (camera, required tile) jobs (tiling.cpp).
// Per frame: remap (+gain) -> pyrDown levels -> blend + collapse from the top level to level 0.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "host_common.hpp"
#include "kernels.hpp"

namespace octvr {

namespace {
struct Rect {
    int x = 0, y = 0, w = 0, h = 0;
};
}  // namespace

class MultiBand {
   public:
    int n = 0, B = 0, device = 0;
    int out_w = 0, out_h = 0;
    Rect arr;
    std::vector<Rect> ar;
    struct Level {
        int W = 0, H = 0, tx_n = 0, ty_n = 0;
        DevBuf<uint8_t> g;              // all cameras' Gaussian level (u8x4)
        size_t g_bytes = 0;
        std::vector<MbCamLevel> cams_h;
        DevBuf<MbCamLevel> cams;
        DevBuf<uint8_t> seam0;          // level 0: u8 seams over each align_roi
        DevBuf<float> wts;              // level > 0: f32 weights over each align_roi >> l
        DevBuf<uint32_t> tile_cams;
        std::vector<uint32_t> tile_cams_h;
        // multi-band, per 32 x 8 sub-tile (tile * kSubs + quarter): the cameras with a non-zero weight there,
        // and its kind: 1 owned (one camera of weight exactly 1 throughout), 2 deep (R = G on every pixel,
        // the deep pass), 3 read by no collapse, 4 (level 0) deep with its result written by the remap
        std::vector<uint32_t> sub_cams_h;
        std::vector<uint8_t> sub_own_h;
        int n_owned = 0;
        int n_deep = 0;                 // sub-tiles with R = G at this level (owned = 2 or 4)
        int n_skip = 0;                 // sub-tiles no collapse reads (owned = 3)
        DevBuf<uint2> work;             // multi-band: the sub-tiles mb_blend computes (kinds 0-2), MbBlendArgs::work
        int n_work = -1;                // their count, padded to a multiple of 4 (-1: every tile, no list)
        DevBuf<UpQuad> up;              // per camera: rows then cols (level < B)
        DevBuf<UpQuad> rup;             // collapse: rows then cols (level < B)
        int rup_rows = 0;
        DevBuf<int32_t> up_org;         // per camera: staged-patch origins per tile row, then per tile col
        DevBuf<int32_t> rup_org;        // collapse: the same
        DevBuf<uint2> down_items;       // level > 0
        int n_down = 0;
        DevBuf<int16_t> R;              // level > 0: collapsed level, s16x4
        size_t req_tiles = 0;           // sum over cameras of required tiles
    };
    std::vector<Level> lv;
    TiledLutDev remap;
    // frames in flight (octvr_mapper_set_frames_in_flight): slot k > 0 has its own Gaussian levels,
    // collapsed levels and remap work queue; everything else above is per rig and read-only per frame
    struct FrameBufs {
        std::vector<DevBuf<uint8_t>> g;
        std::vector<DevBuf<int16_t>> R;
        DevBuf<uint32_t> queue;
    };
    std::vector<std::unique_ptr<FrameBufs>> extra;
    bool feather = false;  // FeatherGPUBlender instead of MultiBandGPUBlender
    bool deep_in_remap = false;  // deep level-0 tiles are written by the remap (kItemResult, owned 4)
    int n_result = 0;            // level-0 tiles the remap writes
    bool full_cover = true;
    int crop_w = 0, crop_h = 0;
};

void MultiBandDeleter::operator()(MultiBand* p) const { delete p; }

namespace {

int round_down(int x, int b) { return (x >> b) << b; }
int round_up(int x, int b) {
    const int m = 1 << b;
    return x + (m - (x % m)) % m;
}

// pyrUp (pyr_up.cu:55-166) source taps of one output row (col) `o` of a level of size n_out, from a
// source of size n_src: unclamped indices + weights (1,6,1 | 4,4), the 8-row block quirk for rows.
int up_taps(int o, bool rows, int* u, int* w) {
    if (!(o & 1)) {
        const int q = o >> 1;
        u[0] = q - 1;
        u[1] = q;
        u[2] = (rows && (o & 7) == 6) ? q + 2 : q + 1;
        w[0] = 1, w[1] = 6, w[2] = 1;
        return 3;
    }
    u[0] = (o - 1) >> 1;
    u[1] = (rows && (o & 7) == 7) ? ((o + 1) >> 1) + 1 : (o + 1) >> 1;
    w[0] = 4, w[1] = 4;
    return 2;
}

// The sub-tile (tile * kSubs + quarter) holding 8 x 8 block (bx, by) of a level grid tx_n tiles wide.
constexpr int kBlkPx = 8;
static_assert(kBlkPx == kTileH && kSubW % kBlkPx == 0, "blocks tile the sub-tiles");
size_t sub_of_block(int tx_n, int bx, int by) {
    return ((size_t)by * tx_n + (size_t)(bx * kBlkPx / kTileW)) * kSubs + (size_t)((bx * kBlkPx % kTileW) / kSubW);
}

// Tap table over the level grid's quad rows (cols): grid index g -> local index g - off, valid in
// [0, n_local); sources clamped to [0, n_src) after abs (pyr_up.cu:72-79).
std::vector<UpQuad> up_table(int n_grid, int off, int n_local, int n_src, bool rows) {
    std::vector<UpQuad> t((n_grid + 1) / 2);
    for (size_t q = 0; q < t.size(); q++) {
        int uni[6], nu = 0;
        int us[2][3], ws[2][3], nt[2] = {0, 0};
        for (int p = 0; p < 2; p++) {
            const int o = (int)(2 * q) + p - off;
            if (o < 0 || o >= n_local) continue;
            nt[p] = up_taps(o, rows, us[p], ws[p]);
            for (int k = 0; k < nt[p]; k++) {
                bool seen = false;
                for (int j = 0; j < nu; j++) seen |= uni[j] == us[p][k];
                if (!seen) uni[nu++] = us[p][k];
            }
        }
        UpQuad& e = t[q];
        memset(&e, 0, sizeof e);
        REQUIRE(nu <= 3, "pyrUp quad needs more than 3 source rows");
        std::sort(uni, uni + nu);
        for (int j = nu; j < 3; j++) uni[j] = nu ? uni[0] : 0;
        for (int j = 0; j < 3; j++) e.idx[j] = (uint16_t)std::min(n_src - 1, std::abs(uni[j]));
        for (int p = 0; p < 2; p++) {
            uint8_t* w = p ? e.w1 : e.w0;
            for (int k = 0; k < nt[p]; k++)
                for (int j = 0; j < nu; j++)
                    if (uni[j] == us[p][k]) w[j] = (uint8_t)ws[p][k];
        }
    }
    return t;
}

// mb_blend computes its taps in registers (up_arith, kernels.hpp); check once per rig that they weigh
// the same sources as the tables: per quad pixel, the summed weight of every source index.
void check_up_arith(const std::vector<UpQuad>& t, int off, int n_local, int n_src, bool rows) {
    for (size_t q = 0; q < t.size(); q++) {
        const UpArith e = up_arith((int)(2 * q), off, n_local, n_src, rows);
        for (int p = 0; p < 2; p++) {
            int wt[6] = {0}, we[6] = {0}, it[6], ie[6];
            for (int j = 0; j < 3; j++) {
                it[j] = t[q].idx[j], wt[j] = p ? t[q].w1[j] : t[q].w0[j];
                ie[j] = e.idx[j], we[j] = p ? e.w1[j] : e.w0[j];
                REQUIRE(ie[j] >= 0 && ie[j] < n_src, "pyrUp tap outside the source");
            }
            auto weight_of = [](const int* idx, const int* w, int v) {
                int s = 0;
                for (int j = 0; j < 3; j++) s += idx[j] == v ? w[j] : 0;
                return s;
            };
            for (int j = 0; j < 3; j++)
                REQUIRE(weight_of(it, wt, it[j]) == weight_of(ie, we, it[j]) &&
                            weight_of(it, wt, ie[j]) == weight_of(ie, we, ie[j]),
                        "pyrUp register taps differ from the tap table");
        }
    }
}

// Origin of each tile's staged pyrUp patch (kernels.hpp kUpPatchRows x kUpPatchCols): the smallest
// source index any weighted tap of the tile's quads reads; the span must fit the patch.
std::vector<int32_t> patch_origins(const std::vector<UpQuad>& t, int quads_per_tile, int n_tiles, int limit) {
    std::vector<int32_t> o(n_tiles, 0);
    for (int k = 0; k < n_tiles; k++) {
        int lo = INT32_MAX, hi = -1;
        for (int q = k * quads_per_tile; q < std::min((k + 1) * quads_per_tile, (int)t.size()); q++)
            for (int j = 0; j < 3; j++)
                if (t[q].w0[j] | t[q].w1[j]) lo = std::min(lo, (int)t[q].idx[j]), hi = std::max(hi, (int)t[q].idx[j]);
        if (hi < 0) continue;
        REQUIRE(hi - lo < limit, "pyrUp patch of a tile exceeds the staged size");
        o[k] = lo;
    }
    return o;
}

struct Bitmap {
    int tx_n = 0, ty_n = 0;
    std::vector<uint8_t> b;
    void init(int tx, int ty) {
        tx_n = tx, ty_n = ty;
        b.assign((size_t)tx * ty, 0);
    }
    // mark every tile overlapping grid rectangle [x0, x1] x [y0, y1] (inclusive)
    void mark(int x0, int y0, int x1, int y1) {
        x0 = std::max(x0, 0), y0 = std::max(y0, 0);
        x1 = std::min(x1, tx_n * kTileW - 1), y1 = std::min(y1, ty_n * kTileH - 1);
        for (int ty = y0 / kTileH; ty <= y1 / kTileH; ty++)
            for (int tx = x0 / kTileW; tx <= x1 / kTileW; tx++) b[(size_t)ty * tx_n + tx] = 1;
    }
};

}  // namespace

MultiBand* multiband_create(const octvr_rig& rig, int device, int bands, const std::vector<int>& in_w,
                            const std::vector<int>& in_h, int feather_border, SourceFootprint* foot, int tex) {
    auto mb = std::unique_ptr<MultiBand>(new MultiBand);
    MultiBand& M = *mb;
    const int n = (int)rig.inputs.size();
    M.n = n;
    M.B = bands;
    M.device = device;
    M.out_w = rig.out_w;
    M.out_h = rig.out_h;
    M.feather = feather_border > 0;
    if (M.feather) M.B = bands = 0;
    const int B = bands;
    // tile camera sets are 32-bit masks, and the blend's f32 Laplacian sum is exact only while
    // |D| <= 255 * sum(w) stays below 2^15 (sum(w) <= n <= 32, multiband.hip)
    REQUIRE(n >= 1 && n <= 32, "multi-band / feather blend: 1..32 inputs");
    if (!M.feather) {
        REQUIRE(B >= 1 && B <= kMbMaxBands, "multi-band blend: band count out of range (blend must be >= 3)");
        REQUIRE(rig.seam_masks.size() == (size_t)n,
                "multi-band blend needs seam masks (octvr_rig_create_masks or a .dat with seams)");
    }
    // ---- rectangles (blenders.cpp:479-486, 595-618) ------------------------------------------
    int x0 = INT32_MAX, y0 = INT32_MAX, x1 = INT32_MIN, y1 = INT32_MIN;
    for (auto& in : rig.inputs) {
        x0 = std::min(x0, in.roi[0]);
        y0 = std::min(y0, in.roi[1]);
        x1 = std::max(x1, in.roi[0] + in.roi[2]);
        y1 = std::max(y1, in.roi[1] + in.roi[3]);
    }
    M.arr = Rect{round_down(x0, B), round_down(y0, B), 0, 0};
    M.arr.w = round_up(x1, B) - M.arr.x;
    M.arr.h = round_up(y1, B) - M.arr.y;
    const int gap = M.feather ? 0 : 5 * (1 << B);  // feather: the ROIs themselves
    for (auto& in : rig.inputs) {
        const int l = std::max(M.arr.x, round_down(in.roi[0], B) - gap);
        const int t = std::max(M.arr.y, round_down(in.roi[1], B) - gap);
        const int r = std::min(M.arr.x + M.arr.w, round_up(in.roi[0] + in.roi[2], B) + gap);
        const int b = std::min(M.arr.y + M.arr.h, round_up(in.roi[1] + in.roi[3], B) + gap);
        REQUIRE(((r - l) >> B) > 0 && ((b - t) >> B) > 0, "multi-band: aligned ROI too small (blenders.cpp:614-615)");
        M.ar.push_back(Rect{l, t, r - l, b - t});
    }
    const double max_len = std::max(M.arr.w, M.arr.h);
    REQUIRE(M.feather || B <= (int)std::ceil(std::log(max_len) / std::log(2.0)),
            "multi-band: too many bands (blenders.cpp:621)");
    M.crop_w = std::min(M.arr.w, rig.out_w);
    M.crop_h = std::min(M.arr.h, rig.out_h);
    REQUIRE(M.arr.x + M.crop_w <= rig.out_w && M.arr.y + M.crop_h <= rig.out_h,
            "multi-band: aligned result ROI leaves the output frame (blenders.cpp:727-729)");
    M.full_cover = M.arr.x == 0 && M.arr.y == 0 && M.crop_w == rig.out_w && M.crop_h == rig.out_h;

    DeviceGuard dg(device);
    M.lv.resize(B + 1);
    for (int l = 0; l <= B; l++) {
        auto& L = M.lv[l];
        L.W = M.arr.w >> l;
        L.H = M.arr.h >> l;
        L.tx_n = (L.W + kTileW - 1) / kTileW;
        L.ty_n = (L.H + kTileH - 1) / kTileH;
        L.cams_h.resize(n);
        size_t off = 0;
        for (int i = 0; i < n; i++) {
            MbCamLevel& c = L.cams_h[i];
            memset(&c, 0, sizeof c);
            c.ox = (M.ar[i].x - M.arr.x) >> l;
            c.oy = (M.ar[i].y - M.arr.y) >> l;
            c.w = M.ar[i].w >> l;
            c.h = M.ar[i].h >> l;
            c.g_pitch = (uint32_t)c.w * 4;
            c.g_off = (uint32_t)off;
            off += ((size_t)c.g_pitch * c.h + 255) & ~(size_t)255;
        }
        REQUIRE(off < 0x7FFFFF00u, "multi-band: pyramid level larger than 2 GiB");
        L.g_bytes = off;
        L.g.alloc(off);
    }
    // ---- feather weights (FeatherGPUBlender ctor, blenders.cpp:531-568) -----------------------
    //   w_i = max(distanceTransform(mask_i, L2, 3) - border, 0); W = 1e-5f + sum_i w_i (camera order);
    //   w_i = n * w_i / W (DivScaleOp, div_mat.cu:82-91; plain a / b when n == 1)
    if (M.feather) {
        auto& L0 = M.lv[0];
        std::vector<std::vector<float>> w(n);
        run_threads((size_t)n, [&](size_t i) {
            const RigInput& in = rig.inputs[i];
            w[i].resize((size_t)in.roi[2] * in.roi[3]);
            chamfer_l2_3x3(in.mask.data(), in.roi[2], in.roi[3], w[i].data());
            for (float& v : w[i]) {
                const float d = v - (float)feather_border;
                v = d > 0.f ? d : 0.f;  // threshold(THRESH_TOZERO, 0)
            }
        });
        std::vector<float> W((size_t)M.arr.w * M.arr.h, 1e-5f);
        for (int i = 0; i < n; i++) {
            const RigInput& in = rig.inputs[i];
            for (int y = 0; y < in.roi[3]; y++)
                for (int x = 0; x < in.roi[2]; x++) {
                    float& d = W[(size_t)(in.roi[1] - M.arr.y + y) * M.arr.w + (in.roi[0] - M.arr.x + x)];
                    d = w[i][(size_t)y * in.roi[2] + x] + d;
                }
        }
        size_t tot = 0;
        std::vector<size_t> woff(n);
        for (int i = 0; i < n; i++) woff[i] = tot, tot += w[i].size();
        std::vector<float> all(tot);
        const float sc = (float)n;
        for (int i = 0; i < n; i++) {
            const RigInput& in = rig.inputs[i];
            for (int y = 0; y < in.roi[3]; y++)
                for (int x = 0; x < in.roi[2]; x++) {
                    const float a = w[i][(size_t)y * in.roi[2] + x];
                    const float b = W[(size_t)(in.roi[1] - M.arr.y + y) * M.arr.w + (in.roi[0] - M.arr.x + x)];
                    all[woff[i] + (size_t)y * in.roi[2] + x] = b != 0 ? (n == 1 ? a / b : sc * a / b) : 0.f;
                }
        }
        L0.wts.upload(all.data(), all.size());
        for (int i = 0; i < n; i++) L0.cams_h[i].weight = L0.wts.p + woff[i];
    }
    // ---- weights: level 0 = seam (u8), levels >= 1 = K4 pyrDown of seam/255 ------------------
    std::vector<uint8_t> seam_h;      // level-0 seams over each align_roi (host copy, for tile_owned)
    std::vector<size_t> seam_off;
    if (!M.feather) {
        auto& L0 = M.lv[0];
        size_t tot = 0;
        std::vector<size_t> woff(n);
        for (int i = 0; i < n; i++) woff[i] = tot, tot += (size_t)L0.cams_h[i].w * L0.cams_h[i].h;
        std::vector<uint8_t> s0(tot, 0);
        std::vector<float> f0(tot, 0.f);
        const float inv255 = (float)(1. / 255);
        for (int i = 0; i < n; i++) {
            const RigInput& in = rig.inputs[i];
            const Rect& a = M.ar[i];
            for (int y = 0; y < in.roi[3]; y++)
                for (int x = 0; x < in.roi[2]; x++) {
                    const uint8_t v = rig.seam_masks[i][(size_t)y * in.roi[2] + x];
                    const size_t d = woff[i] + (size_t)(in.roi[1] - a.y + y) * a.w + (in.roi[0] - a.x + x);
                    s0[d] = v;
                    f0[d] = inv255 * (float)v;
                }
        }
        L0.seam0.upload(s0.data(), s0.size());
        seam_h = s0;
        seam_off = woff;
        for (int i = 0; i < n; i++) L0.cams_h[i].weight = L0.seam0.p + woff[i];
        DevBuf<float> prev;
        prev.upload(f0.data(), f0.size());
        std::vector<size_t> poff = woff;
        for (int l = 1; l <= B; l++) {
            auto& L = M.lv[l];
            size_t t2 = 0;
            std::vector<size_t> o2(n);
            for (int i = 0; i < n; i++) o2[i] = t2, t2 += (size_t)L.cams_h[i].w * L.cams_h[i].h;
            L.wts.alloc(t2);
            for (int i = 0; i < n; i++) {
                const auto& pc = M.lv[l - 1].cams_h[i];
                HIP_CHECK(launch_pyr_down_f32(prev.p + poff[i], pc.w, pc.h, L.wts.p + o2[i], L.cams_h[i].w,
                                              L.cams_h[i].h, nullptr));
                L.cams_h[i].weight = L.wts.p + o2[i];
            }
            HIP_CHECK(hipDeviceSynchronize());
            if (l < B) {  // next level's source: a copy (L.wts stays owned by the level)
                prev.alloc(t2);
                HIP_CHECK(hipMemcpy(prev.p, L.wts.p, t2 * sizeof(float), hipMemcpyDeviceToDevice));
                poff = o2;
            }
        }
    }
    // ---- weight activity per 8x8 block, then per tile (bit n: camera n) -------------------------
    constexpr int kBlk = 8;
    std::vector<std::vector<std::vector<uint8_t>>> act(B + 1);  // [level][camera][block]
    // per level: the owner of each level-grid pixel (the one camera with a non-zero weight, that weight
    // exactly 1; -1 otherwise) and the tiles' owned flags (uploaded after the deep pass below)
    std::vector<std::vector<int8_t>> own_map(B + 1);
    std::vector<std::vector<uint8_t>> owned_h(B + 1);
    for (int l = 0; l <= B; l++) {
        auto& L = M.lv[l];
        const int bx_n = (L.W + kBlk - 1) / kBlk, by_n = (L.H + kBlk - 1) / kBlk;
        DevBuf<uint8_t> blk;
        blk.alloc((size_t)bx_n * by_n);
        act[l].resize(n);
        L.tile_cams_h.assign((size_t)L.tx_n * L.ty_n, 0u);
        for (int i = 0; i < n; i++) {
            const auto& c = L.cams_h[i];
            HIP_CHECK(hipMemset(blk.p, 0, blk.n));
            HIP_CHECK(launch_block_activity(c.weight, l == 0 && !M.feather, c.w, c.h, c.ox, c.oy, bx_n, blk.p, nullptr));
            act[l][i].resize(blk.n);
            HIP_CHECK(hipMemcpy(act[l][i].data(), blk.p, blk.n, hipMemcpyDeviceToHost));
            for (int by = 0; by < by_n; by++)
                for (int bx = 0; bx < bx_n; bx++)
                    if (act[l][i][(size_t)by * bx_n + bx])
                        L.tile_cams_h[(size_t)(by * kBlk / kTileH) * L.tx_n + bx * kBlk / kTileW] |= 1u << i;
        }
        L.tile_cams.upload(L.tile_cams_h.data(), L.tile_cams_h.size());
        if (!M.feather) {
            // tile_owned: one camera with a non-zero weight in the tile, and its weight is exactly 1 on
            // every tile pixel of the level grid (level 0: seam 255; above: the f32 pyramid's 1.0f), so
            // each pixel's Laplacian is that camera's alone with weight 1 (mb_blend's fast path)
            std::vector<float> wl;  // level l > 0: the f32 weights of every camera (host copy)
            if (l > 0) {
                wl.resize(L.wts.n);
                HIP_CHECK(hipMemcpy(wl.data(), L.wts.p, wl.size() * sizeof(float), hipMemcpyDeviceToHost));
            }
            auto& om = own_map[l];
            om.assign((size_t)L.W * L.H, (int8_t)-2);
            for (int i = 0; i < n; i++) {
                const auto& c = L.cams_h[i];
                const size_t woff = l == 0 ? seam_off[i] : (size_t)(static_cast<const float*>(c.weight) - L.wts.p);
                for (int yl = 0; yl < c.h; yl++) {
                    const int y = yl + c.oy;
                    if (y < 0 || y >= L.H) continue;
                    for (int xl = 0; xl < c.w; xl++) {
                        const int x = xl + c.ox;
                        if (x < 0 || x >= L.W) continue;
                        const size_t k = woff + (size_t)yl * c.w + xl;
                        const bool nz = l == 0 ? seam_h[k] != 0 : wl[k] != 0.f;
                        const bool one = l == 0 ? seam_h[k] == 255 : wl[k] == 1.0f;
                        if (!nz) continue;
                        int8_t& o = om[(size_t)y * L.W + x];
                        o = (o == -2 && one) ? (int8_t)i : (int8_t)-1;
                    }
                }
            }
            for (int8_t& o : om) o = o < 0 ? (int8_t)-1 : o;
            // per sub-tile: its cameras (8 x 8 blocks lie in one sub-tile each) and whether it is owned
            L.sub_cams_h.assign((size_t)L.tx_n * L.ty_n * kSubs, 0u);
            for (int i = 0; i < n; i++)
                for (int by = 0; by < by_n; by++)
                    for (int bx = 0; bx < bx_n; bx++)
                        if (act[l][i][(size_t)by * bx_n + bx]) L.sub_cams_h[sub_of_block(L.tx_n, bx, by)] |= 1u << i;
            std::vector<uint8_t> owned(L.sub_cams_h.size(), 0);
            for (int ty = 0; ty < L.ty_n; ty++)
                for (int tx = 0; tx < L.tx_n; tx++)
                    for (int q = 0; q < kSubs; q++) {
                        const size_t sidx = ((size_t)ty * L.tx_n + tx) * kSubs + q;
                        const uint32_t msk = L.sub_cams_h[sidx];
                        if (__builtin_popcount(msk) != 1) continue;
                        const int i = __builtin_ctz(msk);
                        const auto& c = L.cams_h[i];
                        const size_t woff = l == 0 ? seam_off[i] : (size_t)(static_cast<const float*>(c.weight) - L.wts.p);
                        bool all = c.w >= 2;  // the fast path reads pixel pairs
                        const int x0 = tx * kTileW + q * kSubW;
                        for (int y = ty * kTileH; all && y < std::min((ty + 1) * kTileH, L.H); y++)
                            for (int x = x0; x < std::min(x0 + kSubW, L.W); x++) {
                                const int xl = x - c.ox, yl = y - c.oy;
                                const size_t k = woff + (size_t)yl * c.w + xl;
                                if (xl < 0 || yl < 0 || xl >= c.w || yl >= c.h ||
                                    (l == 0 ? seam_h[k] != 255 : wl[k] != 1.0f)) {
                                    all = false;
                                    break;
                                }
                            }
                        owned[sidx] = all ? 1 : 0;
                        L.n_owned += all ? 1 : 0;
                    }
            owned_h[l] = std::move(owned);
        }
    }
    // ---- pyrUp tap tables -------------------------------------------------------------------
    std::vector<std::vector<std::vector<UpQuad>>> ur(B), uc(B);  // [level][camera]
    std::vector<std::vector<UpQuad>> rup_r(B), rup_c(B);             // [level]: the collapse's
    for (int l = 0; l < B; l++) {
        auto& L = M.lv[l];
        const auto& Ln = M.lv[l + 1];
        std::vector<UpQuad> all;
        ur[l].resize(n);
        uc[l].resize(n);
        std::vector<size_t> ro(n), co(n);
        for (int i = 0; i < n; i++) {
            const auto& c = L.cams_h[i];
            // tables cover the whole tile grid: lanes of the last tile row / column past the level
            // size index them too (their weights are 0, their taps clamped in range)
            ur[l][i] = up_table(L.ty_n * kTileH, c.oy, c.h, Ln.cams_h[i].h, true);
            uc[l][i] = up_table(L.tx_n * kTileW, c.ox, c.w, Ln.cams_h[i].w, false);
            check_up_arith(ur[l][i], c.oy, c.h, Ln.cams_h[i].h, true);
            check_up_arith(uc[l][i], c.ox, c.w, Ln.cams_h[i].w, false);
            ro[i] = all.size();
            all.insert(all.end(), ur[l][i].begin(), ur[l][i].end());
            co[i] = all.size();
            all.insert(all.end(), uc[l][i].begin(), uc[l][i].end());
        }
        L.up.upload(all.data(), all.size());
        std::vector<int32_t> org;
        std::vector<size_t> oo(n);
        for (int i = 0; i < n; i++) {
            L.cams_h[i].up_rows = L.up.p + ro[i];
            L.cams_h[i].up_cols = L.up.p + co[i];
            oo[i] = org.size();
            auto r0 = patch_origins(ur[l][i], kTileH / 2, L.ty_n, kUpPatchRows);
            auto c0 = patch_origins(uc[l][i], kTileW / 2, L.tx_n, kUpPatchCols);
            org.insert(org.end(), r0.begin(), r0.end());
            org.insert(org.end(), c0.begin(), c0.end());
        }
        L.up_org.upload(org.data(), org.size());
        for (int i = 0; i < n; i++) {
            L.cams_h[i].up_r0 = L.up_org.p + oo[i];
            L.cams_h[i].up_c0 = L.up_org.p + oo[i] + L.ty_n;
        }
        std::vector<UpQuad> rr = up_table(L.ty_n * kTileH, 0, L.H, Ln.H, true),
                            rc = up_table(L.tx_n * kTileW, 0, L.W, Ln.W, false);
        check_up_arith(rr, 0, L.H, Ln.H, true);
        check_up_arith(rc, 0, L.W, Ln.W, false);
        {
            auto r0 = patch_origins(rr, kTileH / 2, L.ty_n, kUpPatchRows);
            auto c0 = patch_origins(rc, kTileW / 2, L.tx_n, kUpPatchCols);
            r0.insert(r0.end(), c0.begin(), c0.end());
            L.rup_org.upload(r0.data(), r0.size());
        }
        L.rup_rows = (int)rr.size();
        rup_r[l] = rr;
        rup_c[l] = rc;
        rr.insert(rr.end(), rc.begin(), rc.end());
        L.rup.upload(rr.data(), rr.size());
    }
    // ---- deep tiles: R = G (mb_blend skips the pyrUps) -------------------------------------------
    // A pixel of level l is deep for camera n when n owns it (one camera of weight exactly 1), the
    // camera's pyrUp of G_{l+1} there reads the same sources with the same weights as the collapse's
    // pyrUp of R_{l+1}, and every such source is deep for n at level l + 1 (at the top level: owned).
    // Then R_l = G_l exactly, by induction from the top: L_l = G_l - up(G_{l+1}) (weight 1, the
    // normalisation exact for |D| <= 255), R_l = L_l + up(R_{l+1}) with R_{l+1} = G_{l+1} on every tap,
    // and the two pyrUps round identically (the u8 and s16 saturations are no-ops for 0..255).  A tile
    // whose pixels are all deep (owned = 2) takes R = G at its level: no taps, no collapse.
    // (OCTVR_MB_NO_DEEP=1: measurement / cross-check knob, every owned tile takes the pyrUp path)
    const bool deep_on = std::getenv("OCTVR_MB_NO_DEEP") == nullptr;
    if (!M.feather) {
        // nonzero-weight (source, weight) pairs of grid pixel 2q + p, sources shifted by `sh`, merged
        auto taps_of = [](const UpQuad& u, int p, int sh, int (&src)[3], int (&wt)[3]) {
            int k = 0;
            for (int j = 0; j < 3; j++) {
                const int w = p ? u.w1[j] : u.w0[j];
                if (!w) continue;
                const int v = (int)u.idx[j] + sh;
                int m = 0;
                while (m < k && src[m] != v) m++;
                if (m == k) src[k] = v, wt[k++] = 0;
                wt[m] += w;
            }
            for (int a = 1; a < k; a++)  // sorted by source
                for (int b = a; b > 0 && src[b - 1] > src[b]; b--) std::swap(src[b], src[b - 1]), std::swap(wt[b], wt[b - 1]);
            return k;
        };
        auto same_taps = [&](const UpQuad& cu, int sh, const UpQuad& gu, int p) {
            int s1[3], w1[3], s2[3], w2[3];
            const int k1 = taps_of(cu, p, sh, s1, w1), k2 = taps_of(gu, p, 0, s2, w2);
            if (k1 != k2 || k1 == 0) return false;
            for (int j = 0; j < k1; j++)
                if (s1[j] != s2[j] || w1[j] != w2[j]) return false;
            return true;
        };
        std::vector<int8_t> deep_next = own_map[B];
        for (int l = B - 1; l >= 0; l--) {
            auto& L = M.lv[l];
            const auto& Ln = M.lv[l + 1];
            std::vector<std::vector<uint8_t>> rok(n), cok(n);
            for (int i = 0; i < n; i++) {
                rok[i].resize(L.H);
                cok[i].resize(L.W);
                for (int y = 0; y < L.H; y++)
                    rok[i][y] = same_taps(ur[l][i][y >> 1], Ln.cams_h[i].oy, rup_r[l][y >> 1], y & 1);
                for (int x = 0; x < L.W; x++)
                    cok[i][x] = same_taps(uc[l][i][x >> 1], Ln.cams_h[i].ox, rup_c[l][x >> 1], x & 1);
            }
            auto deep_px = [&](int x, int y) -> bool {
                const int c = own_map[l][(size_t)y * L.W + x];
                if (c < 0 || !rok[c][y] || !cok[c][x]) return false;
                int rs[3], rw[3], cs[3], cw[3];
                const int kr = taps_of(rup_r[l][y >> 1], y & 1, 0, rs, rw), kc = taps_of(rup_c[l][x >> 1], x & 1, 0, cs, cw);
                for (int a = 0; a < kr; a++)
                    for (int b = 0; b < kc; b++)
                        if (deep_next[(size_t)rs[a] * Ln.W + cs[b]] != c) return false;
                return true;
            };
            std::vector<int8_t> deep;
            if (l > 0) {  // every pixel (the finer level's test reads them)
                deep.assign((size_t)L.W * L.H, (int8_t)-1);
                for (int y = 0; y < L.H; y++)
                    for (int x = 0; x < L.W; x++)
                        if (deep_px(x, y)) deep[(size_t)y * L.W + x] = own_map[l][(size_t)y * L.W + x];
            }
            for (int ty = 0; ty < L.ty_n; ty++)
                for (int tx = 0; tx < L.tx_n; tx++)
                    for (int q = 0; q < kSubs; q++) {
                        uint8_t& t = owned_h[l][((size_t)ty * L.tx_n + tx) * kSubs + q];
                        if (!t) continue;
                        bool all = true;
                        const int x0 = tx * kTileW + q * kSubW;
                        for (int y = ty * kTileH; all && y < std::min((ty + 1) * kTileH, L.H); y++)
                            for (int x = x0; x < std::min(x0 + kSubW, L.W); x++)
                                if (l > 0 ? deep[(size_t)y * L.W + x] < 0 : !deep_px(x, y)) {
                                    all = false;
                                    break;
                                }
                        if (all && deep_on) t = 2, L.n_deep++;
                    }
            deep_next = std::move(deep);
        }
        // Sub-tiles of level l >= 1 that no collapse reads (every level-(l-1) sub-tile whose pyrUp taps reach
        // them is deep or itself unread): owned = 3, mb_blend skips them, and their Gaussian blocks are not
        // required for them (below).
        for (int l = 1; deep_on && l <= B; l++) {
            auto& L = M.lv[l];
            const auto& Lf = M.lv[l - 1];
            std::vector<uint8_t> read(owned_h[l].size(), 0);
            for (int ty = 0; ty < Lf.ty_n; ty++)
                for (int tx = 0; tx < Lf.tx_n; tx++)
                    for (int sq = 0; sq < kSubs; sq++) {
                        const uint8_t t = owned_h[l - 1][((size_t)ty * Lf.tx_n + tx) * kSubs + sq];
                        if (t >= 2) continue;  // deep (2, 4) or unread (3): no collapse reads level l there
                        int r0 = INT32_MAX, r1 = -1, c0 = INT32_MAX, c1 = -1;
                        for (int q = ty * kTileH / 2; q < (ty + 1) * kTileH / 2; q++)
                            for (int j = 0; j < 3; j++)
                                if (rup_r[l - 1][q].w0[j] | rup_r[l - 1][q].w1[j])
                                    r0 = std::min(r0, (int)rup_r[l - 1][q].idx[j]), r1 = std::max(r1, (int)rup_r[l - 1][q].idx[j]);
                        const int qc = (tx * kTileW + sq * kSubW) / 2;
                        for (int q = qc; q < qc + kSubW / 2; q++)
                            for (int j = 0; j < 3; j++)
                                if (rup_c[l - 1][q].w0[j] | rup_c[l - 1][q].w1[j])
                                    c0 = std::min(c0, (int)rup_c[l - 1][q].idx[j]), c1 = std::max(c1, (int)rup_c[l - 1][q].idx[j]);
                        if (r1 < 0 || c1 < 0) continue;
                        const int cmax = L.tx_n * kTileW - 1;
                        for (int y = r0 / kTileH; y <= std::min(r1 / kTileH, L.ty_n - 1); y++)
                            for (int x = c0 / kSubW; x <= std::min(c1, cmax) / kSubW; x++)
                                read[(size_t)y * L.tx_n * kSubs + x] = 1;  // a tile row's sub-tiles are consecutive
                    }
            for (size_t t = 0; t < read.size(); t++)
                if (!read[t]) {
                    L.n_deep -= owned_h[l][t] == 2 ? 1 : 0;
                    owned_h[l][t] = 3;
                    L.n_skip++;
                }
        }
    }
    // ---- deep level-0 sub-tiles: the remap writes their result (item_result_bit) --------------------
    // A deep level-0 sub-tile's result is its one camera's G0 (R = G, above), so the MODE-1 remap item of that
    // camera converts it to YUV420P (or the RGBA result) right away and mb_blend skips it (owned 4): its
    // G0 is then needed only where a level-1 pyrDown reads it.  Only sub-tiles wholly inside the crop and the
    // output frame qualify (the remap's result stores take no bounds).  (OCTVR_MB_NO_REMAP_RESULT=1:
    // measurement / cross-check knob, the level-0 blend writes every sub-tile.)
    std::vector<int8_t> deep0_owner;  // per level-0 sub-tile: the camera of a remap-result sub-tile, else -1
    if (!M.feather && deep_on && std::getenv("OCTVR_MB_NO_REMAP_RESULT") == nullptr) {
        auto& L0 = M.lv[0];
        deep0_owner.assign(owned_h[0].size(), (int8_t)-1);
        for (int ty = 0; ty < L0.ty_n; ty++)
            for (int tx = 0; tx < L0.tx_n; tx++)
                for (int q = 0; q < kSubs; q++) {
                    const size_t t = ((size_t)ty * L0.tx_n + tx) * kSubs + q;
                    const int x1 = tx * kTileW + (q + 1) * kSubW, y1 = (ty + 1) * kTileH;
                    if (owned_h[0][t] != 2 || x1 > M.crop_w || y1 > M.crop_h || M.arr.x + x1 > rig.out_w ||
                        M.arr.y + y1 > rig.out_h)
                        continue;
                    deep0_owner[t] = (int8_t)__builtin_ctz(L0.sub_cams_h[t]);
                    owned_h[0][t] = 4;
                    M.n_result++;
                }
        M.deep_in_remap = M.n_result > 0;
    }
    // ---- per level, the sub-tiles mb_blend has work on (kinds 0-2), 4 per workgroup: it is launched over
    // this list only, so sub-tiles that need nothing (unread: 3, written by the remap: 4) cost no dispatch
    if (!M.feather) {
        for (int l = 0; l <= B; l++) {
            auto& L = M.lv[l];
            L.sub_own_h = owned_h[l];
            REQUIRE((size_t)L.tx_n * L.ty_n < (1u << 24), "multi-band: level grid too large");
            std::vector<uint2> work;
            for (size_t t = 0; t < owned_h[l].size(); t++)
                if (owned_h[l][t] < 3)
                    work.push_back(make_uint2((uint32_t)(t / kSubs) | (uint32_t)(t % kSubs) << 24 |
                                                  (uint32_t)owned_h[l][t] << 27,
                                              L.sub_cams_h[t]));
            while (work.size() % 4) work.push_back(make_uint2(3u << 27, 0u));
            L.n_work = (int)work.size();
            if (!work.empty()) L.work.upload(work.data(), work.size());
        }
    }
    // ---- required 8x8 blocks per camera and level, then tiles ------------------------------------
    // need(l) = weight blocks(l) + pyrUp support of weight blocks(l-1) + pyrDown support of need(l+1)
    // (level 0 with deep tiles written by the remap: their weight blocks need no G0)
    std::vector<std::vector<Bitmap>> req(B + 1, std::vector<Bitmap>(n));  // tiles
    std::vector<std::vector<uint8_t>> need_next(n);                       // blocks of level l + 1
    std::vector<std::vector<uint8_t>> req0_sub(n);                        // level 0, per sub-tile
    for (int l = B; l >= 0; l--) {
        auto& L = M.lv[l];
        const int bx_n = (L.W + kBlk - 1) / kBlk, by_n = (L.H + kBlk - 1) / kBlk;
        for (int i = 0; i < n; i++) {
            const auto& c = L.cams_h[i];
            std::vector<uint8_t> need = act[l][i];
            auto tile_of = [&](int lv_, int bx, int by) {  // kind of the sub-tile holding block (bx, by)
                return owned_h[lv_].empty() ? 0 : (int)owned_h[lv_][sub_of_block(M.lv[lv_].tx_n, bx, by)];
            };
            for (int by = 0; by < by_n; by++)  // blocks of unread / remap-result sub-tiles: no blend reads G there
                for (int bx = 0; bx < bx_n; bx++)
                    if (tile_of(l, bx, by) == 3 || tile_of(l, bx, by) == 4) need[(size_t)by * bx_n + bx] = 0;
            auto mark = [&](int x0, int y0, int x1, int y1) {  // level-grid pixel rectangle, inclusive
                x0 = std::max(x0, 0), y0 = std::max(y0, 0);
                x1 = std::min(x1, bx_n * kBlk - 1), y1 = std::min(y1, by_n * kBlk - 1);
                for (int by = y0 / kBlk; by <= y1 / kBlk; by++)
                    for (int bx = x0 / kBlk; bx <= x1 / kBlk; bx++) need[(size_t)by * bx_n + bx] = 1;
            };
            if (l >= 1) {  // pyrUp support of the finer level's weight blocks (8x8 px = 4x4 quads)
                const auto& Lf = M.lv[l - 1];
                const int fbx = (Lf.W + kBlk - 1) / kBlk, fby = (Lf.H + kBlk - 1) / kBlk;
                for (int by = 0; by < fby; by++)
                    for (int bx = 0; bx < fbx; bx++) {
                        if (!act[l - 1][i][(size_t)by * fbx + bx]) continue;
                        if (tile_of(l - 1, bx, by) >= 2) continue;  // deep / unread / result: no pyrUp of G_l there
                        int r0 = INT32_MAX, r1 = -1, c0 = INT32_MAX, c1 = -1;
                        for (int q = by * kBlk / 2; q < (by + 1) * kBlk / 2; q++) {
                            const UpQuad& u = ur[l - 1][i][q];
                            for (int j = 0; j < 3; j++)
                                if (u.w0[j] | u.w1[j]) r0 = std::min(r0, (int)u.idx[j]), r1 = std::max(r1, (int)u.idx[j]);
                        }
                        for (int q = bx * kBlk / 2; q < (bx + 1) * kBlk / 2; q++) {
                            const UpQuad& u = uc[l - 1][i][q];
                            for (int j = 0; j < 3; j++)
                                if (u.w0[j] | u.w1[j]) c0 = std::min(c0, (int)u.idx[j]), c1 = std::max(c1, (int)u.idx[j]);
                        }
                        if (r1 >= 0 && c1 >= 0) mark(c0 + c.ox, r0 + c.oy, c1 + c.ox, r1 + c.oy);
                    }
            }
            if (l < B) {  // pyrDown support of the coarser level's required blocks
                const auto& Lc = M.lv[l + 1];
                const auto& cc = Lc.cams_h[i];
                const int cbx = (Lc.W + kBlk - 1) / kBlk, cby = (Lc.H + kBlk - 1) / kBlk;
                for (int by = 0; by < cby; by++)
                    for (int bx = 0; bx < cbx; bx++) {
                        if (!need_next[i][(size_t)by * cbx + bx]) continue;
                        const int xa = std::max(bx * kBlk - cc.ox, 0), xb = std::min((bx + 1) * kBlk - 1 - cc.ox, cc.w - 1);
                        const int ya = std::max(by * kBlk - cc.oy, 0), yb = std::min((by + 1) * kBlk - 1 - cc.oy, cc.h - 1);
                        if (xa > xb || ya > yb) continue;
                        const int sx0 = std::max(2 * xa - 2, 0), sx1 = std::min(2 * xb + 2, c.w - 1);
                        const int sy0 = std::max(2 * ya - 2, 0), sy1 = std::min(2 * yb + 2, c.h - 1);
                        mark(sx0 + c.ox, sy0 + c.oy, sx1 + c.ox, sy1 + c.oy);
                    }
            }
            // blocks outside the camera's aligned ROI hold nothing of it
            for (int by = 0; by < by_n; by++)
                for (int bx = 0; bx < bx_n; bx++) {
                    uint8_t& v = need[(size_t)by * bx_n + bx];
                    if (v && !(bx * kBlk < c.ox + c.w && (bx + 1) * kBlk > c.ox && by * kBlk < c.oy + c.h &&
                               (by + 1) * kBlk > c.oy))
                        v = 0;
                }
            if (l == 0) {  // the remap writes G0 per sub-tile (item_g0_bit)
                req0_sub[i].assign((size_t)L.tx_n * L.ty_n * kSubs, 0);
                for (int by = 0; by < by_n; by++)
                    for (int bx = 0; bx < bx_n; bx++)
                        if (need[(size_t)by * bx_n + bx]) req0_sub[i][sub_of_block(L.tx_n, bx, by)] = 1;
            }
            Bitmap& R = req[l][i];
            R.init(L.tx_n, L.ty_n);
            for (int by = 0; by < by_n; by++)
                for (int bx = 0; bx < bx_n; bx++)
                    if (need[(size_t)by * bx_n + bx]) R.b[(size_t)(by * kBlk / kTileH) * L.tx_n + bx * kBlk / kTileW] = 1;
            for (uint8_t v : R.b) L.req_tiles += v;
            need_next[i] = std::move(need);
        }
    }
    // ---- per-level device tables, down items, collapse buffers ----------------------------------
    for (int l = 0; l <= B; l++) {
        auto& L = M.lv[l];
        L.cams.upload(L.cams_h.data(), n);
        if (l >= 1) {
            std::vector<uint2> items;
            for (int i = 0; i < n; i++)
                for (int ty = 0; ty < L.ty_n; ty++)
                    for (int tx = 0; tx < L.tx_n; tx++)
                        if (req[l][i].b[(size_t)ty * L.tx_n + tx])
                            items.push_back(make_uint2((uint32_t)i, (uint32_t)tx | ((uint32_t)ty << 16)));
            L.n_down = (int)items.size();
            L.down_items.upload(items.data(), items.size());
            L.R.alloc((size_t)L.W * L.H * 4);
        }
    }
    // ---- level-0 remap jobs (camera, required tile) -------------------------------------------
    {
        auto& L0 = M.lv[0];
        // items of qpl vertically adjacent tiles (128 x 8 qpl), kept when any of them is required
        const int qpl = composite_qpl();
        REQUIRE(qpl <= 2, "multi-band remap: items of at most 2 tiles (item flags)");
        // per half and sub-tile: G0 written where required (item_g0_bit), the result where the sub-tile is
        // deep and this camera owns it (item_result_bit)
        std::vector<TileJob> jobs;
        for (int i = 0; i < n; i++)
            for (int ty = 0; ty < (L0.ty_n + qpl - 1) / qpl; ty++)
                for (int tx = 0; tx < L0.tx_n; tx++) {
                    uint32_t fl = 0;
                    for (int h = 0; h < qpl; h++) {
                        if (ty * qpl + h >= L0.ty_n) continue;
                        for (int q = 0; q < kSubs; q++) {
                            const size_t t = ((size_t)(ty * qpl + h) * L0.tx_n + tx) * kSubs + q;
                            if (req0_sub[i][t]) fl |= item_g0_bit(h, q);
                            if (!deep0_owner.empty() && deep0_owner[t] == i) fl |= item_result_bit(h, q);
                        }
                    }
                    if (fl) jobs.push_back(TileJob{tx, ty, i, fl});
                }
        const Rect arr = M.arr;
        auto entry = [&](int job, int x, int y) -> CompositeEntry {
            const int i = jobs[job].cam;
            const RigInput& in = rig.inputs[i];
            const int X = x + arr.x, Y = y + arr.y;
            const int rx = X - in.roi[0], ry = Y - in.roi[1];
            if (rx < 0 || ry < 0 || rx >= in.roi[2] || ry >= in.roi[3]) return CompositeEntry{0u, 0u};
            const size_t k = (size_t)ry * in.roi[2] + rx;
            const float m1 = in.map1[k], m2 = in.map2[k];
            auto mk = [&]() {
                return tex ? make_entry_tex(m1, m2, (float)in_w[i], (float)in_h[i], i)
                           : make_entry(m1, m2, (float)in_w[i], (float)in_h[i], i);
            };
            if (in.mask[k]) return mk();
            // LUT mask 0: the remap still runs there, without gain (mul_scalar_with_mask); a template's
            // -1 maps put every tap outside the image (black; fastRemap's fill_zero in the texture
            // convention), other values follow the remap's rule
            CompositeEntry e = mk();
            e.code |= kCodeNoGain;
            return e;
        };
        TiledLutBuild tb = build_tiled_lut(jobs, entry, in_w, in_h, qpl);
        if (foot) footprint_add_tiles(*foot, tb);
        M.remap.upload(tb, true);
    }
    return mb.release();
}

void multiband_set_slots(MultiBand& M, int k) {
    M.extra.clear();
    for (int i = 1; i < k; i++) {
        auto f = std::make_unique<MultiBand::FrameBufs>();
        f->g.resize(M.lv.size());
        f->R.resize(M.lv.size());
        for (size_t l = 0; l < M.lv.size(); l++) {
            f->g[l].alloc(M.lv[l].g.n);
            f->R[l].alloc(M.lv[l].R.n);
        }
        f->queue.alloc(M.remap.queue.n);
        HIP_CHECK(hipMemset(f->queue.p, 0, f->queue.n * sizeof(uint32_t)));
        M.extra.push_back(std::move(f));
    }
}

void multiband_run(MultiBand& M, int slot, const FrameSet& frames, const double* gains_dev, int use_gain, uint8_t* out,
                   int64_t out_pitch, hipStream_t s, uint8_t* rgba, int64_t rgba_pitch) {
    REQUIRE(slot >= 0 && slot <= (int)M.extra.size(), "bad frame slot");
    MultiBand::FrameBufs* fb = slot ? M.extra[slot - 1].get() : nullptr;
    auto G = [&](int l) { return fb ? fb->g[l].p : M.lv[l].g.p; };
    auto Rl = [&](int l) { return fb ? fb->R[l].p : M.lv[l].R.p; };
    auto& L0 = M.lv[0];
    TiledLut view = M.remap.view;
    if (fb) view.queue = fb->queue.p;
    // (first: the remap writes the deep tiles' results into the output)
    if (!M.full_cover) {  // result pixels outside the blended ROI stay 0 (mapper.cpp:155): Y 0, U = V = 128
        if (rgba) {
            HIP_CHECK(hipMemset2DAsync(rgba, rgba_pitch, 0, (size_t)M.out_w * 4, M.out_h, s));
        } else {
            HIP_CHECK(hipMemset2DAsync(out, out_pitch, 0, M.out_w, M.out_h, s));
            HIP_CHECK(hipMemset2DAsync(out + (int64_t)M.out_h * out_pitch, out_pitch, 128, M.out_w, M.out_h / 2, s));
        }
    }
    RgbaOut ro{};
    ro.base = G(0);
    ro.bytes = (uint32_t)L0.g_bytes;
    ro.cams = L0.cams.p;
    if (M.deep_in_remap) {  // the result frame from the level-0 grid origin (align_result_roi's top-left)
        if (rgba) {
            const int64_t o = (int64_t)M.arr.y * rgba_pitch + (int64_t)M.arr.x * 4;
            const int64_t total = rgba_pitch * M.out_h;
            REQUIRE(total < ((int64_t)1 << 31) - 64 && rgba_pitch < ((int64_t)1 << 31), "result image exceeds 2 GiB");
            ro.res = rgba + o;
            ro.res_bytes = (uint32_t)(total - o);
            ro.res_pitch = (uint32_t)rgba_pitch;
            ro.res_rgba = 1;
        } else {
            const int64_t o = (int64_t)M.arr.y * out_pitch + M.arr.x;
            const int64_t total = out_pitch * (M.out_h + M.out_h / 2);
            REQUIRE(total < ((int64_t)1 << 31) - 64, "output frame exceeds 2 GiB");
            const int64_t u = (int64_t)M.out_h * out_pitch + (int64_t)(M.arr.y / 2) * out_pitch + M.arr.x / 2;
            ro.res = out + o;
            ro.res_bytes = (uint32_t)(total - o);
            ro.res_pitch = (uint32_t)out_pitch;
            ro.res_u_off = (uint32_t)(u - o);
            ro.res_v_off = (uint32_t)(u - o + M.out_w / 2);
        }
    }
    HIP_CHECK(launch_mb_remap(frames, view, gains_dev, use_gain, ro, s));
    for (int l = 1; l <= M.B; l++) {
        auto& L = M.lv[l];
        HIP_CHECK(launch_mb_down(L.down_items.p, L.n_down, L.cams.p, M.lv[l - 1].cams.p, G(l - 1), G(l), s));
    }
    for (int l = M.B; l >= 0; l--) {
        auto& L = M.lv[l];
        MbBlendArgs a{};
        a.level = l;
        a.bands = M.B;
        a.n_cams = M.n;
        a.w_u8 = l == 0 && !M.feather;
        a.feather = M.feather;
        a.out_scale = (float)(1.0 / M.n);
        a.W = L.W;
        a.H = L.H;
        a.tiles_x = L.tx_n;
        a.tile_cams = L.tile_cams.p;
        a.owned = nullptr;  // (the tile kinds travel in the work list)
        a.work = L.n_work >= 0 ? L.work.p : nullptr;
        a.n_work = L.n_work;
        a.cams = L.cams.p;
        a.g = G(l);
        if (l < M.B) {
            auto& Ln = M.lv[l + 1];
            a.cams_next = Ln.cams.p;
            a.g_next = G(l + 1);
            a.r_next = Rl(l + 1);
            a.W_next = Ln.W;
            a.H_next = Ln.H;
            a.rup_rows = L.rup.p;
            a.rup_cols = L.rup.p + L.rup_rows;
            a.rup_r0 = L.rup_org.p;
            a.rup_c0 = L.rup_org.p + L.ty_n;
        }
        if (l > 0) {
            a.r_out = Rl(l);
        } else {
            a.out = out;
            a.out_pitch = out_pitch;
            a.out_w = M.out_w;
            a.out_h = M.out_h;
            a.ax = M.arr.x;
            a.ay = M.arr.y;
            a.crop_w = M.crop_w;
            a.crop_h = M.crop_h;
            a.rgba = rgba;
            a.rgba_pitch = rgba_pitch;
        }
        HIP_CHECK(launch_mb_blend(a, s));
    }
}

// Algorithmic bytes per frame, per launch of the sequence: what each launch must move, every byte
// counted once per launch that needs it (re-reads of a neighbour's halo from L2 are not counted).
//   remap:   4 B tiled entry per item pixel (8 B wide), the G0 halves it writes (4 B / px), the deep
//            tiles' results (1.5 B / px YUV420P), the unique source bytes of its staged boxes, metadata;
//   down l:  4 B written per level-l item pixel, its level-(l-1) source window with the 5 x 5 halo
//            (20 x 260 pixels of 4 B per 128 x 8 item);
//   blend l: per sub-tile by kind — unread (owned 3): nothing; deep (2): G 4 B + R 8 B (level 0: nothing
//            when the remap wrote it, else 1.5 B out); owned (1): G 4 B + coarser G taps 1 B + collapsed
//            coarser level 2 B + R 8 B / out 1.5 B; general: per weighted camera G 4 B + weight (1 B u8
//            seam at level 0, else 4 B f32) + coarser G 1 B, then coarser R 2 B + R 8 B / out 1.5 B.
std::vector<std::pair<std::string, double>> multiband_traffic_parts(const MultiBand& M) {
    std::vector<std::pair<std::string, double>> parts;
    const TiledLut& t = M.remap.view;
    const TiledLutDev& r = M.remap;
    parts.emplace_back("remap", (t.e24 ? 3.0 : 4.0) * t.n_items * kTilePx * t.qpl + 8.0 * t.n_wide * kTilePx + r.g0_bytes +
                                    1.5 * r.result_bytes + r.source_bytes +
                                    (double)t.n_items * (sizeof(TileHdr) + kTileSlots * sizeof(TileSlot)));
    // down l: per item its (2 kTileH + 4) x (2 kTileW + 4) source window (the 5 x 5 support's halo) and the
    // tile it writes
    for (int l = 1; l <= M.B; l++)
        parts.emplace_back("down" + std::to_string(l),
                           (double)M.lv[l].n_down * (4.0 * (2 * kTileH + 4) * (2 * kTileW + 4) + 4.0 * kTilePx));
    for (int l = M.B; l >= 0; l--) {
        const auto& L = M.lv[l];
        const bool up = l < M.B;
        const double out_b = l ? 8.0 : 1.5;
        // per sub-tile (multi-band) or per tile (feather: every tile general)
        const bool sub = !L.sub_own_h.empty();
        const std::vector<uint32_t>& cams = sub ? L.sub_cams_h : L.tile_cams_h;
        const double unit_px = sub ? (double)kSubW * kTileH : (double)kTilePx;
        double b = 0;
        for (size_t k = 0; k < cams.size(); k++) {
            const uint32_t m = cams[k];
            const int o = sub ? L.sub_own_h[k] : 0;
            double px_b = 0;
            if (o == 3) {
                px_b = 0;
            } else if (o == 4) {
                px_b = 0;  // level 0: the remap wrote the result
            } else if (o == 2) {
                px_b = 4.0 + out_b;
            } else if (o == 1) {
                px_b = 4.0 + (up ? 1.0 + 2.0 : 0.0) + out_b;
            } else if (m) {
                px_b = __builtin_popcount(m) * (4.0 + ((l == 0 && !M.feather) ? 1.0 : 4.0) + (up ? 1.0 : 0.0)) +
                       (up ? 2.0 : 0.0) + out_b;
            } else {
                px_b = (up ? 2.0 : 0.0) + out_b;  // no camera: the collapse alone
            }
            b += px_b * unit_px;
        }
        parts.emplace_back("blend" + std::to_string(l), b);
    }
    return parts;
}

double multiband_traffic(const MultiBand& M) {
    double b = 0;
    for (const auto& p : multiband_traffic_parts(M)) b += p.second;
    return b;
}

std::string multiband_info(const MultiBand& M) {
    std::string s = std::string(M.feather ? "\"feather\": 1, " : "") + "\"bands\": " + std::to_string(M.B) + ", \"align_result_roi\": [" + std::to_string(M.arr.x) + ", " +
                    std::to_string(M.arr.y) + ", " + std::to_string(M.arr.w) + ", " + std::to_string(M.arr.h) +
                    "], \"remap_items\": " + std::to_string(M.remap.view.n_items) +
                    ", \"remap_wide\": " + std::to_string(M.remap.view.n_wide) +
                    ", \"remap_entry_bits\": " + std::to_string(M.remap.view.e24 ? 24 : 32) +
                    ", \"remap_result_subtiles\": " + std::to_string(M.n_result) + ", \"traffic_parts\": {";
    {
        bool first = true;
        for (const auto& p : multiband_traffic_parts(M)) {
            char buf[96];
            snprintf(buf, sizeof buf, "%s\"%s\": %.0f", first ? "" : ", ", p.first.c_str(), p.second);
            s += buf;
            first = false;
        }
    }
    s += "}, \"level_tiles\": [";
    for (int l = 0; l <= M.B; l++) {
        const auto& L = M.lv[l];
        size_t cam_tiles = 0;
        for (uint32_t m : L.tile_cams_h) cam_tiles += (size_t)__builtin_popcount(m);
        char buf[512];
        snprintf(buf, sizeof buf, "%s{\"tiles\": %d, \"required\": %zu, \"weight_cam_tiles\": %zu, \"down_items\": %d%s}",
                 l ? ", " : "", L.tx_n * L.ty_n, L.req_tiles, cam_tiles, L.n_down,
                 !L.sub_own_h.empty() ? (", \"blend_subtiles\": " + std::to_string(L.n_work) + ", \"owned_subtiles\": " +
                              std::to_string(L.n_owned) + ", \"deep_subtiles\": " + std::to_string(L.n_deep) +
                              ", \"unread_subtiles\": " + std::to_string(L.n_skip)).c_str() : "");
        s += buf;
    }
    return s + "]";
}

}  // namespace octvr
