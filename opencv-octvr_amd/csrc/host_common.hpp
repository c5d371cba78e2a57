// host_common.hpp — host-side helpers shared by the library's translation units (internal):
// error model of the C ABI (status codes, never exceptions across the boundary), device buffers,
// and the rig (vr::MapperTemplate) representation.
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <exception>
#include <functional>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "kernels.hpp"
#include "octvr_hip.h"

namespace octvr {

struct OctvrError : std::runtime_error {
    int code;
    OctvrError(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

#define HIP_CHECK(expr)                                                                                \
    do {                                                                                               \
        hipError_t e_ = (expr);                                                                        \
        if (e_ != hipSuccess)                                                                          \
            throw ::octvr::OctvrError(OCTVR_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

#define REQUIRE(cond, msg)                                                  \
    do {                                                                    \
        if (!(cond)) throw ::octvr::OctvrError(OCTVR_E_INVALID, (msg));     \
    } while (0)

// f(t) for t in [0, T) on T host threads.  An exception thrown by f (a REQUIRE, a HIP_CHECK, bad_alloc)
// never leaves its thread — that would std::terminate the host process, Python caller included: the
// first one is kept and rethrown on the calling thread after every thread has joined, so the C ABI's
// guard turns it into a status code.
template <class F>
void run_threads(size_t T, F f) {
    std::exception_ptr first;
    std::mutex mu;
    std::vector<std::thread> th;
    th.reserve(T);
    for (size_t t = 0; t < T; t++)
        th.emplace_back([&, t] {
            try {
                f(t);
            } catch (...) {
                std::lock_guard<std::mutex> g(mu);
                if (!first) first = std::current_exception();
            }
        });
    for (auto& x : th) x.join();
    if (first) std::rethrow_exception(first);
}

// f(k) for k in [0, n) on up to 16 host threads (contiguous ranges; build-time work only).
template <class F>
void parallel_for(size_t n, F f) {
    const size_t T = std::max<size_t>(1, std::min<size_t>({16, (size_t)std::thread::hardware_concurrency(), n}));
    if (T <= 1) {
        for (size_t k = 0; k < n; k++) f(k);
        return;
    }
    run_threads(T, [&](size_t t) {
        for (size_t k = n * t / T; k < n * (t + 1) / T; k++) f(k);
    });
}

// octvr_last_error() text of the calling thread (octvr_hip.cpp).
void set_last_error(const std::string& msg);

// Scoped device selection: restores the caller's current device.
struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        HIP_CHECK(hipGetDevice(&prev));
        if (dev != prev) HIP_CHECK(hipSetDevice(dev));
    }
    ~DeviceGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

template <class T>
struct DevBuf {
    T* p = nullptr;
    size_t n = 0;
    DevBuf() = default;
    DevBuf(const DevBuf&) = delete;
    DevBuf& operator=(const DevBuf&) = delete;
    DevBuf(DevBuf&& o) noexcept : p(o.p), n(o.n) { o.p = nullptr; o.n = 0; }
    ~DevBuf() { reset(); }
    void alloc(size_t count) {
        reset();
        if (count == 0) return;
        HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&p), count * sizeof(T)));
        n = count;
    }
    void upload(const T* h, size_t count) {
        alloc(count);
        if (count) HIP_CHECK(hipMemcpy(p, h, count * sizeof(T), hipMemcpyHostToDevice));
    }
    void reset() {
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
    }
};

}  // namespace octvr

// =================================================================================================
// Rig (vr::MapperTemplate, octvr.hpp:47-91): host-resident, like the reference's cv::Mat members.
// =================================================================================================
struct RigInput {
    int roi[4] = {0, 0, 0, 0};
    int in_w = 0, in_h = 0;  // input image size when known (JSON rigs)
    std::vector<float> map1, map2;
    std::vector<uint8_t> mask;
    std::vector<float> vignette;
    int vig_w = 0, vig_h = 0;
    // morph_controlpoints' triangles (octvr.hpp:60 src_triangles / dst_triangles), 6 floats each
    std::vector<float> src_tris, dst_tris;
    size_t n_fragile = 0;  // LUT pixels the GPU build left to the host (LutGuard, camera_math.hpp)
};

struct octvr_rig {
    int out_w = 0, out_h = 0;
    int device = 0;  // device used for GPU-side template work (LUT build, seam resizes)
    std::vector<RigInput> inputs;
    std::vector<RigInput> overlays;
    std::vector<std::vector<uint8_t>> seam_masks;
    // camera models of a JSON-built rig (MapperTemplate::output_cam / input_cams, octvr.hpp:69-70);
    // a rig loaded from .dat has none, like the reference's
    bool has_cameras = false;
    bool out_cam_masks = false;  // the output camera has exclude / include masks (not kept)
    octvr::CameraParams out_cam{};
    std::vector<octvr::CameraParams> cams;
    // MapperTemplate::visible_mask (octvr.hpp:67) on the device, allocated once an include mask appears
    octvr::DevBuf<uint8_t> visible;
};

namespace octvr {
// MapperTemplate::create_masks() (template.cpp:155-204) — seams.cpp
void rig_create_masks(octvr_rig& rig);
// MapperTemplate::morph_controlpoints (template_morph.cpp:69-237) — morph.cpp; returns the number of
// control points kept
struct JsonValue;
int rig_morph_controlpoints(octvr_rig& rig, const JsonValue& control_points);
// cv::distanceTransform(src, dst, DIST_L2, 3) on the host (distransform.cpp:48-139); w x h, packed
void chamfer_l2_3x3(const uint8_t* src, int w, int h, float* dist);

// ---- mapper internals used by the AsyncMultiMapper pipeline (octvr_hip.cpp, async.cpp) -----------
// preview_output of Mapper::stitch (mapper.cpp:308-312): a CV_8UC3 device image
struct PreviewOut {
    uint8_t* dev;
    int w, h;
    size_t pitch;
};
void mapper_stitch(octvr_mapper* m, const uint8_t* const* in_dev, const size_t* in_pitch, uint8_t* out_dev,
                   size_t out_pitch, const double* gains, int n_gains, const double* gains_dev, hipStream_t s,
                   const PreviewOut* preview = nullptr);
int mapper_num_inputs(const octvr_mapper* m);
bool mapper_has_gain(const octvr_mapper* m);
const double* mapper_gains_dev(const octvr_mapper* m);
void mapper_out_size(const octvr_mapper* m, int* w, int* h);

// ---- tiled composite LUT builder (tiling.cpp) ----------------------------------------------------
struct TileJob {
    int tx, ty;  // 128 x (8 qpl) item of the output (or level-0) grid
    int cam;     // RGBA mode: the camera whose pyramid image the tile is written to
    // RGBA mode: item_result_bit / item_g0_bit per half and quarter (kernels.hpp); by default every
    // sub-tile's G0 (the scaled output's result image) and no result
    uint32_t flags = kItemAllG0;
};
// entry(job, x, y): the 8-byte CompositeEntry of grid pixel (x, y) for that job ({0,0} = black)
using EntryFn = std::function<CompositeEntry(int job, int x, int y)>;
struct TiledLutBuild {
    std::vector<TileHdr> hdr;
    std::vector<TileSlot> slots;
    std::vector<uint32_t> entries;
    std::vector<CompositeEntry> wide;
    std::vector<uint32_t> wide_tiles;
    std::vector<uint16_t> wide_cams;  // camera | the half's flags (quarters' result bits, G0 bits << 4) << 8
    std::vector<uint16_t> item_flags;  // per staged item: its job's flags (RGBA mode)
    std::vector<uint16_t> grp0, grp1;  // staging groups (kernels.hpp TiledLut::grp0 / grp1)
    std::vector<int32_t> bands;  // kStitchBands + 1 item boundaries, balanced by estimated cost
    int n_items = 0, n_wide = 0;
    int qpl = 1;  // 128x8 halves per item (kernels.hpp TiledLut::qpl)
    int tex = 0;  // the staged items' entries are texture-convention ones (tiled_entry_tex)
    double staged_bytes = 0;  // YUV bytes staged, summed over items (groups of neighbouring items overlap)
    double source_bytes = 0;  // unique source bytes: the union of the staged groups (+ wide tiles' taps)
    std::string stats;  // JSON fragment: staged items by staging chunks / LDS bytes, per-band chunk sums
};
TiledLutBuild build_tiled_lut(const std::vector<TileJob>& jobs, const EntryFn& entry, const std::vector<int>& in_w,
                              const std::vector<int>& in_h, int qpl = 1);
struct TiledLutDev {
    DevBuf<TileHdr> meta;  // kMetaWords 16-byte words per staged item (kernels.hpp TiledLut::meta)
    DevBuf<uint32_t> entries;
    DevBuf<CompositeEntry> wide;
    DevBuf<uint32_t> wide_tiles;
    DevBuf<uint16_t> wide_cams;
    DevBuf<int32_t> bands;
    DevBuf<uint32_t> queue;
    DevBuf<uint16_t> grp0, grp1;
    double staged_bytes = 0;
    double source_bytes = 0;
    double g0_bytes = 0;      // RGBA mode: G0 bytes the items write (halves without kItemNoG0)
    double result_bytes = 0;  // RGBA mode: result pixels the items write (kItemResult halves)
    std::string stats;
    TiledLut view{};
    // e24: pack the entries to 24 bits when no entry carries "no gain" (tiled_entry24)
    void upload(const TiledLutBuild& b, bool e24 = false);
};

// ---- source footprint: the input bytes a mapper's kernels may read (tiling.cpp) ------------------------
// Per camera one bit per (luma row pair r, 8-pixel group g): luma rows 2r, 2r + 1 x columns [8g, 8g + 8)
// and chroma row r x columns [4g, 4g + 4) of U and V.  Built with the mapper from what drives its source
// reads: every staged group of its tiled LUTs (stitch_tiled_kernel's staging loads), the in-image taps of
// every wide-tile entry (stitch_wide_kernel) and gain sample (the gain feed).  Loads outside it are only
// the clamped addresses of out-of-image taps and invalid staging groups, whose bytes no result uses.  The
// AsyncMultiMapper uploads only these bytes (async.cpp).
struct SourceFootprint {
    std::vector<int> w, h;
    std::vector<std::vector<uint64_t>> bits;  // per camera: row_pairs x words
    void init(const std::vector<int>& in_w, const std::vector<int>& in_h);
    int groups(int i) const { return (w[i] + 7) / 8; }
    int words(int i) const { return (groups(i) + 63) / 64; }
    int row_pairs(int i) const { return (h[i] + 1) / 2; }
    bool test(int cam, int r, int g) const { return (bits[cam][(size_t)r * words(cam) + g / 64] >> (g % 64)) & 1u; }
    void mark(int cam, int y, int g) { bits[cam][(size_t)(y >> 1) * words(cam) + g / 64] |= 1ull << (g % 64); }
    void mark_taps(const CompositeEntry& e);  // the in-image taps of a valid entry
    void merge(const SourceFootprint& o);
    double bytes() const;  // YUV420P bytes under the set bits
};
void footprint_add_tiles(SourceFootprint& f, const TiledLutBuild& b);
const SourceFootprint& mapper_footprint(const octvr_mapper* m);

// ---- multi-band blend (multiband_host.cpp) ---------------------------------------------------------
class MultiBand;
struct MultiBandDeleter {
    void operator()(MultiBand* p) const;
};
// MultiBandGPUBlender(seam_masks, rois, bands) for a mapper: everything per rig (weights, tile lists,
// pyramid buffers) on `device`.  in_w / in_h: input frame sizes.
// feather_border > 0 instead builds FeatherGPUBlender(masks, rois, border) (blenders.cpp:531-586):
// a single level whose weights are the normalised feather weights.
// foot: when given, the remap's source reads are added to it.  tex: texture-convention remap entries
// (make_entry_tex, OCTVR_REMAP_TEXTURE).
MultiBand* multiband_create(const octvr_rig& rig, int device, int bands, const std::vector<int>& in_w,
                            const std::vector<int>& in_h, int feather_border = 0, SourceFootprint* foot = nullptr,
                            int tex = 0);
// One frame: camera level-0 images (remap + gain), Gaussian levels, blend + collapse -> YUV420P
// (or, with `rgba`, the RGB result as RGBA for a scaled output).
// slot: frame slot (0 = the buffers built with the rig, 1..k-1 after multiband_set_slots(k)).
void multiband_run(MultiBand& mb, int slot, const FrameSet& frames, const double* gains_dev, int use_gain, uint8_t* out,
                   int64_t out_pitch, hipStream_t s, uint8_t* rgba = nullptr, int64_t rgba_pitch = 0);
// Per-frame buffers (pyramid levels, collapsed levels, remap work queue) for k frames in flight.
void multiband_set_slots(MultiBand& mb, int k);
// Algorithmic bytes of one frame and a JSON fragment of build statistics.
double multiband_traffic(const MultiBand& mb);
std::string multiband_info(const MultiBand& mb);
}  // namespace octvr
