// kernels.hpp — launch interface of the gfx950 kernels (internal; the public boundary is
// include/octvr_hip.h).  All launchers are stream-ordered and never synchronize.
#pragma once

#include <hip/hip_runtime.h>
#include <cstdint>

#include "camera_math.hpp"

namespace octvr {

constexpr int kMaxCams = 32;

// Composite-LUT entry (8 bytes per output pixel), built once per rig by composite_lut:
//   x = sx | sy << 16                      integer source pixel of the top-left tap, s16 each
//   y = fx | fy << 5 | cam << 10 | 1 << 15  5-bit fractions, winning camera, valid flag
// An entry with the valid bit clear produces black (no camera covers the pixel).
struct CompositeEntry {
    uint32_t xy;
    uint32_t code;
};

// Fixed-point source coordinate of a normalized map value, as RemapInvoker derives it from the
// caller's `map * W` (template.cpp:174-176): X = fl32(m * W); ix = round_half_even(X * 32), NaN and
// out-of-int-range values INT_MIN (_mm_cvtps_epi32, imgwarp.cpp:4385-4420).
__host__ __device__ inline int quantize_coord(float m, float scale) {
    float X = m * scale;
    float f = X * 32.0f;
    if (!(f >= -2147483648.f && f < 2147483648.f)) return INT32_MIN;
    return (int)rintf(f);
}

// Entry for a claimed pixel.  Template-built LUTs keep 0 <= m < 1 where the mask is set, but
// morphed or externally made ones (.dat, from_arrays) need not: the tap cell saturates to s16 like
// remap's (short) conversion and every tap outside the image reads 0 (BORDER_CONSTANT).
__host__ __device__ inline CompositeEntry make_entry(float m1, float m2, float w, float h, int cam) {
    int ix = quantize_coord(m1, w), iy = quantize_coord(m2, h);
    const int sx = min(max(ix >> 5, -32768), 32767), sy = min(max(iy >> 5, -32768), 32767);
    CompositeEntry e;
    e.xy = (uint32_t)(uint16_t)sx | ((uint32_t)(uint16_t)sy << 16);
    e.code = (uint32_t)(ix & 31) | ((uint32_t)(iy & 31) << 5) | ((uint32_t)cam << 10) | (1u << 15);
    return e;
}

// Texture-convention entry (mapper flag OCTVR_REMAP_TEXTURE): the sampling of the reference's live CUDA
// path, cv::cuda::fastRemap through a linear-filtered, clamp-addressed texture with normalized coordinates
// (cudawarping/src/cuda/fast_remap.cu:21-44, texture.hpp:124-160), as oracle/octvr_oracle.c
// orc_fast_remap_tex_rgba models NVIDIA's filter: X = fl32(u W) - 0.5, i0 = floor(X), alpha =
// floor(frac(X) 256) / 256 (8 fractional bits), taps (i0, i0 + 1) x (j0, j0 + 1) clamped to the image and
// all four used.  xy: (i0, j0) kept in [-1, size - 1] (the same taps under the clamp); code: alpha | cam <<
// 10 | valid << 15 | beta << 17 | kCodeTex.  u < 0, NaN or infinite coordinates: invalid (black).  Tiles holding
// such entries always take the gather path (tiling.cpp), whose taps and weights test kCodeTex.
constexpr uint32_t kCodeTex = 1u << 31;
__host__ __device__ inline CompositeEntry make_entry_tex(float m1, float m2, float w, float h, int cam) {
    CompositeEntry e{0u, 0u};
    const float xb = m1 * w - 0.5f, yb = m2 * h - 0.5f;
    // u < 0: fill_zero; NaN or an infinite coordinate: the model's weights are NaN and every channel
    // saturates to 0 — the same black
    if (!(m1 >= 0.f) || !(fabsf(xb) <= 3.0e38f) || !(fabsf(yb) <= 3.0e38f)) return e;
    const float fx = floorf(xb), fy = floorf(yb);
    const uint32_t a = (uint32_t)floorf((xb - fx) * 256.f), b = (uint32_t)floorf((yb - fy) * 256.f);
    const int i0 = (int)fminf(fmaxf(fx, -1.f), w - 1.f), j0 = (int)fminf(fmaxf(fy, -1.f), h - 1.f);
    e.xy = (uint32_t)(uint16_t)(int16_t)i0 | ((uint32_t)(uint16_t)(int16_t)j0 << 16);
    e.code = (a & 255u) | ((uint32_t)cam << 10) | (1u << 15) | ((b & 255u) << 17) | kCodeTex;
    return e;
}

// The 2 x 2 taps of an entry's cell (sx, sy) in a w x h image: clamped addresses and in-image flags.
struct TapCell {
    int x0, x1, y0, y1;
    bool ix0, ix1, iy0, iy1;
};
__host__ __device__ inline TapCell tap_cell(uint32_t xy, int w, int h) {
    const int sx = (int)(int16_t)(xy & 0xFFFFu), sy = (int)(int16_t)(xy >> 16);
    TapCell c;
    c.ix0 = (unsigned)sx < (unsigned)w;
    c.ix1 = (unsigned)(sx + 1) < (unsigned)w;
    c.iy0 = (unsigned)sy < (unsigned)h;
    c.iy1 = (unsigned)(sy + 1) < (unsigned)h;
    c.x0 = min(max(sx, 0), w - 1);
    c.x1 = min(max(sx + 1, 0), w - 1);
    c.y0 = min(max(sy, 0), h - 1);
    c.y1 = min(max(sy + 1, 0), h - 1);
    return c;
}

// ---- tiled composite (the per-frame hot path) -------------------------------------------------
// The output is cut into 128 x 8 pixel tiles (one 256-lane workgroup per tile, one 2x2 quad per
// lane).  Per tile the host pre-computes, once per rig, which cameras win inside it (<= 4 "slots")
// and the luma bounding box of every in-image bilinear tap of each slot.  A staged tile converts
// those boxes from YUV420P (8-byte Y + 4-byte U/V loads per 8 pixels) into packed RGBA in LDS — every source pixel
// converted once, as NPP's full-frame pass does in the reference — at a tile-uniform row stride.
// Staging work is cut into chunks of 64 eight-pixel groups, each chunk inside one slot, so a wave's
// chunk has wave-uniform slot parameters (scalar registers, no per-lane slot search).
// LDS dwords 0-3 of the tile area are zero: a black pixel's entry (0) reads its tap (x, y) there.
// Each slot's box reaches one column / row past its taps (x0 + 1, y0 + 1), including taps outside
// the source image: staging writes RGBA 0 for box pixels outside the image (BORDER_CONSTANT), so
// every tap is read from LDS at off, off + 4, off + 4 S, off + 4 S + 4 (S = row stride) unmasked.
// The LUT is tile-major (quad-major inside the tile), 4 bytes per pixel:
//   bit 0 "no gain" (RGBA mode); bits 1-2 zero; 3-12 the fraction code fx | fy << 5, so e & 0x1FF8 is
//   the byte offset of the code's two packed weight pairs in the workgroup's 8 KiB LDS weight table;
//   13-26 LDS byte offset of tap (x, y) (one v_bfe_u32); 27-29 zero; 30-31 slot (the slot's gain
//   sits at byte offset e >> 27 of a 4-slot table of f32 pairs).  Three VALU decode a pixel's entry.
// A pixel with no camera, or with every tap outside, is entry 0 and comes out black.
constexpr int kTileW = 128, kTileH = 8, kTilePx = kTileW * kTileH;
constexpr int kTileSlots = 4;
// Items of the tiled composite: two vertically adjacent 128 x 8 tiles (128 x 16 pixels, 8 quads per lane).
constexpr int kItemHalves = 2;
// Staging LDS: 16 KiB less the composite's 176 bytes of other LDS, so its static LDS is exactly 16 KiB
// and the 8 KiB weight table starts at LDS address 0x4000 (every C2 / C4 item stages < 16 KiB; 6
// workgroups per CU by LDS)
constexpr int kTileLdsBytes = 16 * 1024 - 176;
static_assert(kTileLdsBytes <= (1 << 14), "the tiled entry's LDS byte offset field");
constexpr uint32_t kWtabBytes = 1024u * 8u;
constexpr int kTileZeroDwords = 4;
// Staging stores: 2 x 16 bytes per 8-pixel group, so a row stride is a multiple of 4 dwords.
constexpr int kStageAlignDwords = 4;
// The tiler pads an item's row stride by up to this many dwords (tiling.cpp: the stride whose tap reads
// conflict least in the LDS banks)
constexpr uint32_t kStridePadMax = 28;

struct TileSlot {
    uint16_t cam;
    uint16_t bw, bh;   // luma box size (bw a multiple of 8, bh even)
    uint16_t lds;      // dword offset of the slot's RGBA box in the tile's LDS area
    uint16_t bx0, by0; // luma box origin (bx0 multiple of 8, by0 even)
    uint16_t chunk0;   // first 64-group staging chunk of this slot (slots are chunk-aligned)
    uint16_t pad1;
};

struct TileHdr {           // one staged item
    uint32_t tile;          // item column | item row << 16 (items of 128 x 8 qpl pixels)
    uint32_t nslots;        // bits 0-7: slots used (0..4); bits 8-15: 64-group staging chunks
    uint32_t stage_groups;  // 4-pixel groups to convert into LDS (host; the device word: TiledLutDev::upload)
    uint32_t stride;        // bits 0-8: LDS row stride in dwords (max box width of the item + a bank pad); bits 9-31:
                            // the item's first chunk in the group overflow table (TiledLut::grp1)
};
constexpr int kStrideBits = 9;
static_assert(256 + kStridePadMax < (1u << kStrideBits), "a padded stride fits its field");
// Staging groups: an item stages, per slot and box row, only the 8-pixel groups between the row's leftmost
// and rightmost tap (the box layout in LDS is kept: the entries' tap offsets do not change).  One u16 per
// group: bit 15 valid, bits 8-12 the group's column in the box (x = bx0 + 8 col), bits 0-7 its row.  A
// slot's groups fill whole 64-group chunks (the last one padded with invalid groups); chunk c of an item:
// grp0[(t kGroupFirst + c) 64 + lane] for c < kGroupFirst (each wave's first chunk, loaded one iteration
// ahead by item index alone), grp1[(ovf + c - kGroupFirst) 64 + lane] after (ovf: TileHdr::stride >> 9).
constexpr int kGroupFirst = 4;
constexpr uint32_t kGroupValid = 0x8000u;

// One input camera as the per-frame kernels see it: a YUV420P frame in "Y over [U|V]" layout.
struct SourceFrame {
    const uint8_t* yuv;
    int32_t w, h;
    int64_t pitch;
    const float* vig;  // vignette gain per source pixel (w x h, packed) or NULL (mapper.cpp:108-112,230-231)
};

// All camera frames of one stitch call, passed by value as a kernel argument (no per-frame H2D copy).
struct FrameSet {
    SourceFrame f[kMaxCams];
};

// The frames of one composite launch (launch_stitch, octvr_mapper_stitch_batch): 1 << nf_log2 frame sets
// (at most kMaxBatch) stitched in one pass over the tiled LUT.  The item sequence runs over (item, frame)
// pairs — unit v = item << nf_log2 | frame — so the units of one item are dealt to neighbouring workgroups
// of one XCD band at the same time: the item's entries, metadata and staging groups come from HBM (or the
// Infinity Cache) once for all the frames and from L2 for the others, while each unit stages and computes
// its own frame.  Camera c of frame f: src[(f << cam_log2) + c], cam_log2 = 5 (32 cameras) for one or two
// frames, 4 (16 cameras) for four.  The FIRST argument of the composite kernels (kernarg_frame), sized for
// its frame count (one frame: 1,040 B of kernarg, as the round-5 FrameSet + pointers).
constexpr int kMaxBatch = 4;
template <int NF>
struct FrameBatch {
    static constexpr int kCamLog2 = NF <= 2 ? 5 : 4;
    SourceFrame src[NF << kCamLog2];
    uint8_t* out[NF];        // MODE 0: the frames' YUV420P outputs (one pitch)
    const double* gains[NF]; // the frames' gains (device)
};


// One NV12 plane of a FastMapper (fastmapper.cpp / fastmapper.hip): per run {camera mask, first block},
// and per (camera, run) block either the compact entries (header + u32 offsets/fractions + u8 weights)
// or the wide uint2 entries; nblk: the blocks allocated (>= 1).
struct FastMapperPlane {
    bool compact;
    const uint2* ent;
    const uint32_t* off;
    const uint8_t* wgt;
    const uint2* hdr;
    const uint2* runs;
    uint32_t nblk;
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
// exposure_compensate.cpp:174-221 + Mapper ctor mapper.cpp:94-114).  Every working-scale pixel of
// camera i that lies in the bitwise-AND intersection with some camera j becomes one sample: its
// 8-byte entry plus a partner mask (bit j).  Samples are sorted by (camera, source row, column); each
// camera's run is padded with invalid samples (partner mask 0) to whole runs of kGainWaveRun (one
// wave each, so a wave's frame is uniform), the whole array to chunks of kGainChunk (one workgroup,
// about one workgroup per CU on C2).
constexpr int kGainMaxCams = 16;
constexpr int kGainPer = 3;  // samples per lane of the gain feed
constexpr int kGainWaveRun = 64 * kGainPer;  // one wave's samples: contiguous, one camera
constexpr int kGainChunk = 4 * kGainWaveRun;  // one workgroup's samples (4 waves)
constexpr int kGainTotalStride = 32;  // u64 words between pair totals: one 256-B line each

// cams_dev: {output camera, input camera} in device memory (CameraParams holds the ocam polynomials).
// fragile (optional, cap + 1 words, fragile[0] zero): indices of the pixels the host must recompute
// (LutGuard, camera_math.hpp); fragile[0] receives their count (entries past cap are dropped).
hipError_t launch_lut_build(const CameraParams* cams_dev, int W, int H, float* map1, float* map2, uint8_t* mask,
                            int32_t* bbox, uint8_t* visible, uint32_t* fragile, uint32_t cap, hipStream_t s);

hipError_t launch_project_f64(const CameraParams* cams_dev, int W, int H, double* x, double* y, uint8_t* fragile,
                              hipStream_t s);

// tex: texture-convention entries (make_entry_tex) instead of cv::remap's (make_entry)
hipError_t launch_composite_lut(const CamTemplate* cams_dev, int n, int W, int H, CompositeEntry* lut,
                                hipStream_t s, int tex = 0);

// Gain feed in ONE launch (no host sync): each workgroup gathers its chunk's warped samples, takes
// the f32 RGB norm (elementNorm) and adds it per partner camera into exact u64 fixed-point totals
// (units of 2^-23, see kernels.hip); the last workgroup (per-XCD then global ticket) reads and
// resets the totals, assembles I(i,j), A, b and solves.  `totals` (kGainMaxCams^2) and `tickets`
// (9) must be zero before the first launch; the last workgroup leaves them zero.  tex: the samples are
// texture-convention entries (make_entry_tex).
hipError_t launch_gain_feed(const FrameSet& frames, const CompositeEntry* samples, const uint16_t* partners, int tex,
                            int n_chunks, const int32_t* N, int n,
                            unsigned long long* totals, uint32_t* tickets, double* gains, hipStream_t s,
                            bool lean = false);  // lean: <= 80 VGPRs (73 used), runs beside a composite (kernels.hip)

// FastMapper frames of one launch (octvr_fastmapper_stitch_nv12_batch): camera c of frame f at
// src[(f << cam_log2) + c] (cam_log2 5 for up to 2 frames, 4 for 4), the frames' NV12 outputs.
template <int NF>
struct FastBatch {
    SourceFrame src[NF << (NF <= 2 ? 5 : 4)];
    uint8_t* out[NF];
};

// The feeds of nf frames (1, 2 or 4) of a batch in one launch: workgroup b feeds frame b / n_chunks into its
// own totals / tickets / gains (FeedBatch, the kernel's first argument; one frame: 536 B of kernarg).
template <int NF>
struct FeedBatch {
    SourceFrame src[NF * kGainMaxCams];  // camera c of frame f at f * kGainMaxCams + c
    unsigned long long* totals[NF];
    uint32_t* tickets[NF];
    double* gains[NF];
};
hipError_t launch_gain_feed_batch(const FrameSet* frames, int nf, const CompositeEntry* samples, const uint16_t* partners,
                                  int tex, int n_chunks, const int32_t* N, int n, unsigned long long* const* totals,
                                  uint32_t* const* tickets, double* const* gains, hipStream_t s, bool lean);

hipError_t launch_set_gains(const double* host_gains, int n, double* gains_dev, hipStream_t s);

// AsyncMultiMapper footprint upload (async.cpp): a run is `ng` consecutive 8-pixel groups from group g0 of
// row pair r of camera `cam` (host_common.hpp SourceFootprint), packed at `off` as luma row 2r, luma row
// 2r + 1, then its chroma row of U and of V; the frames are "Y over [U | V]" with pitch = width.
struct FootRun {
    uint32_t cam;  // camera | row pair << 8
    uint32_t g0, ng;
    uint32_t off;
};
struct FootFrames {
    uint8_t* f[kMaxCams];
    int w[kMaxCams], h[kMaxCams];
};
hipError_t launch_unpack_runs(const uint8_t* packed, const FootRun* runs, int n_runs, const FootFrames& frames,
                              hipStream_t s);

struct TiledLut {
    const TileHdr* meta;          // per staged item kMetaWords 16-byte words: the TileHdr, then kTileSlots TileSlots
    const uint32_t* entries;      // kTilePx per staged item, quad-major inside the tile
    int n_items;
    const uint32_t* wide_tiles;   // tile column | row << 16 of each wide tile
    const CompositeEntry* wide;   // kTilePx per wide tile
    int n_wide;
    const uint16_t* wide_cams;    // RGBA mode: output camera of each wide tile | its half's item flags << 8
    const int32_t* bands;         // kStitchBands + 1 staged-item boundaries (one band per XCD)
    uint32_t* queue;              // per band a work counter, then a done ticket, kQueueStride apart;
                                  // zero before a launch, left zero by its last workgroup
    int qpl;                      // quads per lane: an item is 128 x (8 qpl) pixels, qpl * kTilePx entries
    const uint16_t* grp0;         // staging groups of each item's first kGroupFirst chunks (kGroupFirst * 64 per item)
    const uint16_t* grp1;         // the items' further chunks
    uint32_t n_grp1;              // entries of grp1
    int tex;                      // staged entries are texture-convention ones (tiled_entry_tex)
    int e24;                      // entries packed to 24 bits (tiled_entry24): 12 bytes per lane and half
};
constexpr int kMetaWords = 1 + kTileSlots;
constexpr int kQueueStride = 32;  // u32 words: one 128-B line per counter
// The staged items are cut into one contiguous band per XCD (locality: neighbouring tiles share
// source boxes in that XCD's L2) of equal item counts.  Measured on the C2 rig (r01 v10): equal counts
// beat every split weighted by staging chunks tried (base 16 / 8 / 4 / 2 per chunk: +2 % / +4 % / +10 % /
// +19 % stitch time) — the large pole boxes are re-read from L2 by many tiles, so staging chunks do not
// predict a tile's cost.
constexpr int kStitchBands = 8;
// 4-byte tiled entries: bit 0 = "no gain" (a pixel the gain does not touch: LUT mask 0 with an
// in-image map value; mul_scalar_with_mask, exposure_compensate.cu:15-30).  8-byte CompositeEntry
// records carry the same flag in code bit 16.  TileHdr.nslots bits 16-20: output camera (RGBA mode).
constexpr uint32_t kEntryNoGain = 1u;
constexpr int kEntrySlotShift = 30;
constexpr uint32_t kCodeNoGain = 1u << 16;

// One staged pixel's 4-byte entry (layout above): off = LDS byte offset of tap (x, y) in the item's
// staging area, fxy = fx | fy << 5.
__host__ __device__ constexpr uint32_t tiled_entry(uint32_t off, uint32_t fxy, uint32_t slot, bool nogain) {
    return (nogain ? kEntryNoGain : 0u) | (fxy & 1023u) << 3 | off << 13 | slot << kEntrySlotShift;
}

// The same entry in 24 bits, for LUTs without "no gain" pixels (TiledLutDev::upload packs them): bits 0-1
// the slot, 2-11 fxy, 12-23 the tap's LDS dword offset.  A lane's four entries of a half are packed into
// three dwords (c0 | c1 << 24, c1 >> 8 | c2 << 16, c2 >> 16 | c3 << 8): 3 instead of 4 bytes per pixel.
__host__ __device__ constexpr uint32_t tiled_entry24(uint32_t e) {
    return (e >> 30) | ((e >> 3) & 1023u) << 2 | ((e >> 15) & 4095u) << 12;
}

// A staged texture-convention pixel (make_entry_tex with all four taps inside the image): bit 0 "no gain",
// bits 1-8 alpha, 9-16 beta (8-bit fractions), 17-28 the tap's LDS dword offset, 30-31 the slot.
__host__ __device__ constexpr uint32_t tiled_entry_tex(uint32_t off, uint32_t ab, uint32_t slot, bool nogain) {
    return (nogain ? kEntryNoGain : 0u) | (ab & 0xFFFFu) << 1 | (off >> 2) << 17 | slot << kEntrySlotShift;
}

// 128 x 8 halves per item of the tiled composite (kItemHalves): the tiler's qpl.
int composite_qpl();

// ev0 / ev1 (optional): timing events around the composite (carried by the dispatch packet when it
// is a single launch)
hipError_t launch_stitch(const FrameSet& frames_dev, const TiledLut& lut, int W, int H,
                         const double* gains, int use_gain, uint8_t* out, int64_t out_pitch, hipStream_t s,
                         hipEvent_t ev0 = nullptr, hipEvent_t ev1 = nullptr);
// nf frames (1, 2 or 4; frame f = frames[f], gains[f], out[f], all outputs of pitch out_pitch) in one
// composite launch (FrameBatch); more than 16 cameras need nf <= 2
hipError_t launch_stitch_batch(const FrameSet* frames, int nf, const TiledLut& lut, int W, int H,
                               const double* const* gains, int use_gain, uint8_t* const* out, int64_t out_pitch,
                               hipStream_t s, hipEvent_t ev0 = nullptr, hipEvent_t ev1 = nullptr);

// ---- multi-band blend (blend > 0): MultiBandGPUBlender (blenders.cpp:589-735) ------------------
// Level l of the blend lives on the "level grid": align_result_roi >> l.  Each camera keeps its
// Gaussian pyramid G (u8x4, camera-local, dense over align_roi >> l) but only the 128x8 tiles some
// blend step reads are ever computed (tile lists built once per rig).  pyrUp is evaluated on the
// fly from 3x3 source taps per output quad through per-row / per-column tap tables (UpQuad), which
// encode pyr_up.cu's borders (abs, then clamp) and its 8-row-block quirk.
constexpr int kMbMaxBands = 10;
// pyrUp source patch of one 128x8 tile: <= 8 rows (4 quad rows, the row quirk, any block phase)
// by <= 72 columns (64 quad columns + borders), staged in LDS
constexpr int kUpPatchRows = 8, kUpPatchCols = 72;
struct alignas(16) UpQuad {  // one quad row (or column) of a pyrUp output; 16 B: one load per lane
    uint16_t idx[3];      // source rows (cols) of the 3 union taps, clamped, local to the coarser level
    uint16_t pad0;
    uint8_t w0[3], w1[3]; // integer weights of the quad's first / second row (col) over them
    uint8_t pad1[2];
};
static_assert(sizeof(UpQuad) == 16, "UpQuad layout");

// The same taps computed in registers instead of read from the UpQuad tables (no dependent table
// load between the camera record and the tap loads).  For the quad at even level-grid index g, local
// pixels o0 = g - off and o0 + 1 (up_taps / up_table in multiband_host.cpp, pyr_up.cu:55-166):
//   o0 even (o0 = 2h):   sources h-1, h, h+1+k   w0 = 1 6 1, w1 = 0 4 4    k: rows, o0 % 8 == 6
//   o0 odd  (o0 = 2h+1): sources h, h+1, h+2+k'  w0 = 4 4 0, w1 = 1 6 1    k': rows, o0 % 8 == 5
//                                   (rows, o0 % 8 == 7: the odd pixel reads h, h+2: w0 = 4 0 4)
// A pixel outside [0, n_local) weighs 0; sources are |u| clamped to n_src - 1.  Zero-weight slots
// may hold a different (in-range) source than the table's, so the weighted sums are identical.
__host__ __device__ inline int up_clamp(int u, int n_src) {
    u = u < 0 ? -u : u;
    return u < n_src - 1 ? u : n_src - 1;
}
struct UpArith {
    int idx[3];
    int w0[3], w1[3];
};
__host__ __device__ inline UpArith up_arith(int g, int off, int n_local, int n_src, bool rows) {
    UpArith e;
    const int o0 = g - off;
    const int h = o0 >> 1;  // floor
    const bool odd = (o0 & 1) != 0;
    const int m8 = o0 & 7;
    const bool v0 = o0 >= 0 && o0 < n_local, v1 = o0 + 1 >= 0 && o0 + 1 < n_local;
    int u0, u2;
    if (!odd) {
        u0 = h - 1;
        u2 = h + 1 + ((rows && m8 == 6) ? 1 : 0);
        e.w0[0] = 1, e.w0[1] = 6, e.w0[2] = 1;
        e.w1[0] = 0, e.w1[1] = 4, e.w1[2] = 4;
    } else {
        u0 = h;
        u2 = h + 2 + ((rows && m8 == 5) ? 1 : 0);
        const bool q7 = rows && m8 == 7;
        e.w0[0] = 4, e.w0[1] = q7 ? 0 : 4, e.w0[2] = q7 ? 4 : 0;
        e.w1[0] = 1, e.w1[1] = 6, e.w1[2] = 1;
    }
    e.idx[0] = up_clamp(u0, n_src);
    e.idx[1] = up_clamp(u0 + 1, n_src);
    e.idx[2] = up_clamp(u2, n_src);
#pragma unroll
    for (int j = 0; j < 3; j++) {
        e.w0[j] = v0 ? e.w0[j] : 0;
        e.w1[j] = v1 ? e.w1[j] : 0;
    }
    return e;
}

struct MbCamLevel {       // one camera at one level
    uint32_t g_off;        // byte offset of the camera's G in the level's pyramid allocation
    uint32_t g_pitch;      // bytes per row of G (4 * w)
    int32_t ox, oy, w, h;  // camera's aligned ROI on the level grid: origin and size
    const void* weight;    // level 0: u8 seam mask (pitch w), else f32 Gaussian weight (pitch w)
    const UpQuad* up_rows; // pyrUp taps into this camera's next level, by level-grid quad row
    const UpQuad* up_cols; // ... by level-grid quad column
    const int32_t* up_r0;  // per tile row / column: origin of the tile's staged source patch
    const int32_t* up_c0;
};

// Level-0 pyramid images as the composite kernels' RGBA sink.
struct RgbaOut {
    uint8_t* base;
    uint32_t bytes;        // allocation size (< 2^31)
    const MbCamLevel* cams;
    // Deep level-0 tiles (multi-band, owned = 4 on the host: the result there is exactly the owner
    // camera's G0): items flagged kItemResult write their halves' final result from the remap itself,
    // so the level-0 blend skips those tiles; items flagged kItemNoG0 write no G0 for that half (nothing
    // reads it).  The result frame is addressed from the level-0 grid origin (align_result_roi's
    // top-left): `res` points there, YUV420P with the U / V planes at res_u_off / res_v_off bytes
    // (res_rgba = 0), or the RGBA result image of a scaled output (res_rgba = 1).  Flagged tiles lie
    // wholly inside the crop and the frame (multiband_create), so the stores need no bounds.
    uint8_t* res;
    uint32_t res_bytes;    // addressable bytes from `res` (< 2^31)
    uint32_t res_pitch, res_u_off, res_v_off;
    int res_rgba;
};
// Sub-tiles: 32 x 8 quarters of a 128 x 8 tile (one mb_blend wave each; lane = quad).  The multi-band
// classification (owned / deep / unread / result, multiband_host.cpp) is per sub-tile, so a seam that
// crosses a tile leaves its other quarters on the cheap paths.
constexpr int kSubW = 32, kSubs = kTileW / kSubW;
// Per-item flags of the MODE-1 remap (bits 8-23 of the item header's device word 2, see
// TiledLutDev::upload; bits 8-15 of a wide tile's camera word, for its one half): for half h and quarter q,
// bit 4h + q: that sub-tile's final result is written by the remap (its one deep camera's G0 converted),
// bit 8 + 4h + q: its G0 is written (some pyrDown or blend reads it).  Items of <= 2 halves.
__host__ __device__ constexpr uint32_t item_result_bit(int h, int q) { return 1u << (4 * h + q); }
__host__ __device__ constexpr uint32_t item_g0_bit(int h, int q) { return 1u << (8 + 4 * h + q); }
constexpr uint32_t kItemAllG0 = 0xFF00u;

hipError_t launch_mb_remap(const FrameSet& frames, const TiledLut& lut, const double* gains, int use_gain,
                           const RgbaOut& out, hipStream_t s);
// fastPyrDown<uchar4> (fast_pyr_down.cu:17-76) of every listed (camera, tile) of level l from l - 1.
hipError_t launch_mb_down(const uint2* items, int n_items, const MbCamLevel* cams_l, const MbCamLevel* cams_prev,
                          const uint8_t* g_prev, uint8_t* g_l, hipStream_t s);
struct MbBlendArgs {
    int level, bands, n_cams;
    int w_u8;                       // weights are the u8 seam mask (multi-band level 0), else f32
    int feather;                    // FeatherGPUBlender: out = sat_u8(out_scale * D), no normalisation
    float out_scale;                // (float)(1.0 / n) (convertTo alpha, blenders.cpp:579)
    int W, H;                       // level grid
    int tiles_x;
    const uint32_t* tile_cams;      // bit n: camera n has a non-zero weight in the tile
    const uint8_t* owned;           // multi-band (or NULL): the tile's one camera has weight 1 on every tile pixel
    const uint2* work;              // multi-band (or NULL): the sub-tiles to blend, 4 per workgroup (wave w of
                                    // block b takes work[4 b + w]): x = tile | quarter << 24 | owned << 27,
                                    // y = the sub-tile's cameras; padded with owned = 3 (nothing to do)
    int n_work;                     // their count (a multiple of 4, when work is set)
    const MbCamLevel* cams;         // this level
    const MbCamLevel* cams_next;    // level + 1 (NULL at the top)
    const uint8_t* g;               // this level's pyramid allocation
    const uint8_t* g_next;          // level + 1 allocation
    const int16_t* r_next;          // collapsed level + 1 (s16x4, W_next x H_next)
    int W_next, H_next;
    const UpQuad* rup_rows;         // pyrUp taps of the collapse (level grid, camera independent)
    const UpQuad* rup_cols;
    const int32_t* rup_r0;          // per tile row / column: origin of the staged collapse patch
    const int32_t* rup_c0;
    int16_t* r_out;                 // level > 0: collapsed level (s16x4, pitch 4 * W shorts)
    uint8_t* out;                   // level 0: YUV420P output frame
    int64_t out_pitch;
    int out_w, out_h;
    int ax, ay, crop_w, crop_h;     // align_result_roi origin in the output frame, crop size
    uint8_t* rgba;                  // level 0, scaled output: the RGB result as RGBA (out_w x out_h) instead of YUV
    int64_t rgba_pitch;
    // level 0, multi-band: owned = 4 marks deep tiles whose result the remap wrote (kItemResult)
};
hipError_t launch_mb_blend(const MbBlendArgs& a, hipStream_t s);
// Build time: K4 pyrDown<float, BrdReflect101> with nvcc's FMA contraction (pyr_down.cu:55-192).
hipError_t launch_pyr_down_f32(const float* src, int sw, int sh, float* dst, int dw, int dh, hipStream_t s);
// Build time: blocks[by * bx_n + bx] = 1 for every 8x8 block of the level grid where the camera's
// weight is non-zero (level 0: u8 seam, else f32).
hipError_t launch_block_activity(const void* weight, int is_u8, int w, int h, int ox, int oy, int bx_n, uint8_t* blocks,
                                 hipStream_t s);

hipError_t launch_remap_u8(const uint8_t* src, int sw, int sh, int64_t spitch, int cn, const float* map1,
                           const float* map2, int mw, int mh, int64_t mpitch, float scale_x, float scale_y,
                           uint8_t* dst, int64_t dpitch, hipStream_t s);

// morph_controlpoints' warps (template_morph.cpp:207-231): pixel i of the w x h ROI takes the
// cv::warpAffine (INTER_LINEAR, BORDER_CONSTANT 0) of map1 / map2 / mask by triangle owner[i]'s
// matrix M[6 owner[i] ..] (already inverted as warpAffine inverts it), or is copied (owner < 0).
hipError_t launch_morph_warp(const float* map1, const float* map2, const uint8_t* mask, int w, int h,
                             const int16_t* owner, const double* M, float* out1, float* out2, uint8_t* out_mask,
                             hipStream_t s);

// cv::resize INTER_LINEAR, u8, one channel, with the CPU path's fixed-point rule
// (imgwarp.cpp:1391-1500): per output column the source column and 11-bit weights, per output row
// the two clipped source rows and weights — tables built on the host (seams.cpp), so the kernel
// does integer arithmetic only.  area2: exact 1/2 downscale, (a + b + c + d + 2) >> 2 (:2349-2400).
struct ResizeTables {
    const int32_t* xofs;  // dw
    const int16_t* ax;    // 2 * dw
    const int32_t* rows;  // 2 * dh
    const int16_t* by;    // 2 * dh
    int32_t xmax;
    int32_t area2;
};
hipError_t launch_resize_u8(const uint8_t* src, int sw, int sh, int64_t spitch, uint8_t* dst, int dw, int dh,
                            int64_t dpitch, const ResizeTables& t, hipStream_t s);

// Scaled output (mapper.cpp:290-306): cuda::resize INTER_LINEAR of the RGB(A) result (sw x sh,
// pitch spitch bytes, 4 bytes per pixel) to dw x dh (even), then RGB -> YUV420P into `out`.
hipError_t launch_resize_rgba_yuv420(const uint8_t* rgba, int sw, int sh, int64_t spitch, uint8_t* out, int dw, int dh,
                                     int64_t out_pitch, hipStream_t s);

// Preview output (mapper.cpp:308-312): cuda::resize INTER_LINEAR of the RGB(A) result to a dw x dh
// CV_8UC3 image (3 bytes per pixel, pitch out_pitch).
hipError_t launch_resize_rgba_rgb(const uint8_t* rgba, int sw, int sh, int64_t spitch, uint8_t* out, int dw, int dh,
                                  int64_t out_pitch, hipStream_t s);

hipError_t launch_selftest_sat(const float* in, uint8_t* out, int n, int method, hipStream_t s);

}  // namespace octvr
