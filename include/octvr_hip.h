/*
 * octvr_hip.h — C ABI of the MI355X-native octVR stitching path (remap + gain + seam composite).
 *
 * This is the drop-in boundary for the reference's octvr per-frame path.  Each entry point names
 * the reference interface it replaces (paths relative to the blahgeek/OpenCV-octVR root):
 *
 *   octvr_rig_*      <- vr::MapperTemplate           modules/octvr/include/octvr.hpp:47-91,
 *                                                     modules/octvr/src/template.cpp:23-322
 *   octvr_mapper_*   <- vr::Mapper                   modules/octvr/src/mapper.hpp:29-95,
 *                                                     modules/octvr/src/mapper.cpp:47-323
 *   octvr_async_*    <- vr::AsyncMultiMapper         modules/octvr/include/octvr.hpp:103-121,
 *                                                     modules/octvr/src/async.cpp:32-350
 *   octvr_fastmapper_* <- vr::FastMapper           modules/octvr/src/mapper_fast.cpp:27-195
 *   octvr_remap_*    <- cv::remap INTER_LINEAR u8    modules/imgproc/src/imgwarp.cpp:4689-4828
 *
 * Conventions: no exceptions cross the boundary; every call returns an int status
 * (OCTVR_OK = 0, negative = error, message via octvr_last_error()).  Pointers named *_dev are HIP
 * device pointers; `stream` is a hipStream_t (NULL = the legacy default stream).  A rig owns host
 * memory; a mapper owns device memory on one device and is not thread-safe.  Separate mappers on
 * separate devices are independent (the multi-GPU model: one rig per GPU).
 */
#ifndef OCTVR_HIP_H
#define OCTVR_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OCTVR_HIP_ABI_VERSION 1

enum {
    OCTVR_OK = 0,
    OCTVR_E_INVALID = -1,   /* bad argument / shape (reference: CV_Assert) */
    OCTVR_E_PARSE = -2,     /* bad JSON or .dat (reference: throw std::string) */
    OCTVR_E_HIP = -3,       /* HIP runtime failure */
    OCTVR_E_UNSUPPORTED = -4,
    OCTVR_E_IO = -5
};

typedef struct octvr_rig octvr_rig;
typedef struct octvr_mapper octvr_mapper;

/* One input of a MapperTemplate (octvr.hpp:55-61): ROI in output pixels, ROI-sized maps
 * (normalized x/W_in, y/H_in, or -1), ROI-sized LUT mask {0,255} and seam mask (may be NULL). */
typedef struct {
    int roi_x, roi_y, roi_w, roi_h;
    const float* map1;
    const float* map2;
    const uint8_t* mask;
    const uint8_t* seam_mask;
    const float* vignette;     /* 512x512 f32 or NULL (vignette.cpp:39-54) */
    int vignette_w, vignette_h;
} octvr_input_view;

int octvr_abi_version(void);
const char* octvr_last_error(void);
int octvr_device_count(int* count);

/* ---- device memory helpers (for C/C++ callers without their own allocator) ------------------- */
int octvr_dev_malloc(int device, size_t bytes, void** ptr);
int octvr_dev_free(void* ptr);
int octvr_memcpy_h2d(void* dst_dev, const void* src_host, size_t bytes);
int octvr_memcpy_d2h(void* dst_host, const void* src_dev, size_t bytes);
int octvr_stream_sync(void* stream);

/* ---- vr::MapperTemplate -------------------------------------------------------------------- */
/* MapperTemplate(to, to_opts, w, h) + add_input(..., use_roi) for every entry of `inputs`
 * (template.cpp:23-153, apps/octvr/dump.cpp:76-93).  The projection LUT is built on `device`
 * by a gfx950 FP64 kernel.  out_w/out_h <= 0 derive from the output aspect ratio (template.cpp:32-38).
 * Seam masks are NOT built here (see octvr_rig_create_masks). */
int octvr_rig_create_json(const char* json, int out_w, int out_h, int use_roi, int device, octvr_rig** rig);
/* MapperTemplate(to, to_opts, width, height) (template.cpp:23-44): an empty template with the output
 * camera `out_type` and its options object (JSON text); width / height <= 0 derive from the output
 * aspect ratio.  flags: OCTVR_JSON_EXACT = numbers are correctly rounded (text printed from doubles with
 * 17 digits); 0 = rapidjson 1.0.2's own number rules, as the reference parses a config file. */
#define OCTVR_JSON_EXACT 1
int octvr_rig_create(const char* out_type, const char* out_opts_json, int out_w, int out_h, int device, int flags,
                     octvr_rig** rig);
/* MapperTemplate::add_input(from, from_opts, overlay, use_roi) (template.cpp:46-153): builds input (or
 * overlay) LUT on the rig's device; include masks clear earlier inputs' masks (visible_mask).  Existing
 * seam masks are dropped (create_masks again). */
int octvr_rig_add_input(octvr_rig* rig, const char* type, const char* opts_json, int overlay, int use_roi, int flags);
/* MapperTemplate(std::ifstream&) — VRv11 reader (template.cpp:258-314). */
int octvr_rig_load_dat(const char* path, octvr_rig** rig);
/* The same reader / MapperTemplate::dump writer over caller streams: read(ctx, buf, n) returns the bytes
 * read (0 = end), write(ctx, data, n) returns n on success. */
typedef size_t (*octvr_read_fn)(void* ctx, void* buf, size_t n);
typedef size_t (*octvr_write_fn)(void* ctx, const void* data, size_t n);
int octvr_rig_load_stream(octvr_read_fn read, void* ctx, octvr_rig** rig);
int octvr_rig_dump_stream(octvr_rig* rig, octvr_write_fn write, void* ctx);
/* MapperTemplate::dump — VRv11 writer, byte-compatible (template.cpp:206-256).  Like the reference,
 * creates the seam masks first when the rig has none (template.cpp:209-210). */
int octvr_rig_dump_dat(octvr_rig* rig, const char* path);
/* MapperTemplate::create_masks() without images (template.cpp:155-204): the L2 distance seam finder
 * (DistanceSeamFinder, stitching/src/seam_finders.cpp:97-133) on masks resized to <= 960 px wide,
 * seams resized back to each ROI.  Resizes run on `device`; replaces existing seam masks. */
int octvr_rig_create_masks(octvr_rig* rig, int device);
/* Build a rig from caller arrays (ROI-sized maps/masks, row-major, tightly packed). */
int octvr_rig_create_from_arrays(int out_w, int out_h, int n_inputs, const int* rois, const float* const* map1,
                                 const float* const* map2, const uint8_t* const* masks,
                                 const uint8_t* const* seam_masks_or_null, octvr_rig** rig);
/* inputs[i].vignette (overlay = 0) or overlay_inputs[i].vignette: a w x h f32 gain map, or none
 * (map NULL, w = h = 0).  Overlay i of a rig made from arrays: */
int octvr_rig_set_vignette(octvr_rig* rig, int i, int overlay, const float* map, int w, int h);
int octvr_rig_add_overlay_arrays(octvr_rig* rig, const int* roi, const float* map1, const float* map2,
                                 const uint8_t* mask);
int octvr_rig_num_inputs(const octvr_rig* rig, int* n);
int octvr_rig_out_size(const octvr_rig* rig, int* w, int* h);
int octvr_rig_get_input(const octvr_rig* rig, int i, octvr_input_view* view);

/* Overlay inputs of the rig (MapperTemplate::overlay_inputs, octvr.hpp:62; built like the inputs by
 * add_input(..., overlay = true), template.cpp:46-153, written to .dat at template.cpp:248-255). */
int octvr_rig_num_overlays(const octvr_rig* rig, int* n);
/* ROI, maps, mask (and vignette) of overlay i; seam_mask is NULL (overlays have none). */
int octvr_rig_get_overlay(const octvr_rig* rig, int i, octvr_input_view* view);
/* MapperTemplate::morph_controlpoints(control_points) (modules/octvr/src/template_morph.cpp:69-237,
 * called by octvr_dump -c, apps/octvr/dump.cpp:98-99): control_points_json is the rig JSON's
 * "control_points" array, [[n0, n1, x0, y0, x1, y1], ...] (n0 < n1, normalized input coordinates).
 * Warps every input's map1 / map2 / mask piecewise-affinely (Delaunay triangles of the control
 * points' output positions -> their distance-weighted midpoints); seam masks are left as they are.
 * Needs a rig built by octvr_rig_create_json (camera models): OCTVR_E_UNSUPPORTED otherwise, and for
 * fisheye / pinhole control-point cameras (no image_to_obj in the reference).  Points that the
 * reference would index out of bounds (NaN projection, outside the camera's ROI) give
 * OCTVR_E_INVALID.  n_used (optional): control points kept after the 0.1 distance filter. */
int octvr_rig_morph_controlpoints(octvr_rig* rig, const char* control_points_json, int* n_used);
/* inputs[i].src_triangles / dst_triangles (octvr.hpp:60) of the last morph: 6 floats (x0 y0 x1 y1 x2
 * y2, normalized output coordinates) per triangle.  *n = count; src / dst may be NULL (count only). */
int octvr_rig_get_triangles(const octvr_rig* rig, int i, float* src, float* dst, int cap, int* n);
void octvr_rig_destroy(octvr_rig* rig);
/* An independent deep copy of a rig (camera models, LUTs, seams, include-mask visibility state): what
 * copying a vr::MapperTemplate copies (its Input vectors, octvr.hpp:56-64), so add_input / morph on
 * one copy leave the other unchanged. */
int octvr_rig_clone(const octvr_rig* rig, octvr_rig** out);

/* ---- vr::Mapper ---------------------------------------------------------------------------- */
/* Mapper(mt, in_sizes, blend, enable_gain, scale_output) (mapper.cpp:47-191).
 * blend: 0 = no blend (composite by LUT mask, later input wins; mapper.cpp:268-277), > 0 multi-band
 * with ceil(log2(blend)) - 1 bands (MultiBandGPUBlender), < 0 feather with border -blend
 * (FeatherGPUBlender); blend != 0 needs seam masks (octvr_rig_create_masks or a .dat).
 * scale_w/scale_h: 0 = output at template size, else the output is resized (mapper.cpp:290-306). */
int octvr_mapper_create(const octvr_rig* rig, int device, int n_inputs, const int* in_w, const int* in_h, int blend,
                        int enable_gain, int scale_w, int scale_h, octvr_mapper** mapper);
/* The same with creation flags (no reference counterpart; 0 = octvr_mapper_create).
 * OCTVR_REMAP_TEXTURE: sample the camera frames as the reference's live CUDA path does —
 * cv::cuda::fastRemap through a linear-filtered, clamp-addressed texture (cudawarping/src/cuda/
 * fast_remap.cu:21-44): x = u W - 0.5, 8-bit fractions, taps clamped to the image, u < 0 -> 0 — instead
 * of cv::remap's fixed point (imgwarp.cpp; the default, which the CPU and OpenCL paths share).  The
 * texture filter is NVIDIA hardware behaviour; this mode follows the oracle's model of it
 * (oracle/octvr_oracle.c orc_fast_remap_tex_rgba) bit for bit, gain samples included.  Tiles whose taps
 * all lie inside their camera's image are staged in LDS like the default's (stitch_tiled_tex_kernel, a
 * 16-bit fraction code per pixel); tiles with a tap the clamp moves take the gather kernel.  The f32
 * filter model costs about twice the default's VALU per pixel, so the mode is slower.  Other bits:
 * OCTVR_E_INVALID. */
#define OCTVR_REMAP_TEXTURE 1
int octvr_mapper_create_ex(const octvr_rig* rig, int device, int n_inputs, const int* in_w, const int* in_h, int blend,
                           int enable_gain, int scale_w, int scale_h, int flags, octvr_mapper** mapper);
/* Mapper::stitch (mapper.cpp:193-323) on device-resident YUV420P frames in the "Y over [U|V]"
 * layout of mapper.hpp:75-83: rows [0,H) = Y (W bytes), rows [H, 3H/2) = U in bytes [0, W/2) and
 * V in bytes [W/2, W) of each row; `pitch` = bytes per row (>= W).  gains: NULL = estimate
 * (GainCompensatorGPU::feed), else set_gains (n_gains == n_inputs).  Stream-ordered, no host sync. */
int octvr_mapper_stitch_yuv420p(octvr_mapper* mapper, const uint8_t* const* in_dev, const size_t* in_pitch,
                                uint8_t* out_dev, size_t out_pitch, const double* gains, int n_gains, void* stream);
/* n_frames (1, 2 or 4) consecutive frames of the same rig in one call (no reference counterpart; the
 * reference stitches a frame per Mapper::stitch): frame f's inputs are in_dev[f * n_inputs + i] /
 * in_pitch[...], its output out_dev[f] (all outputs of pitch out_pitch); gains NULL = estimate every frame's
 * own gains, else n_frames * n_inputs values.  Each frame gets its own gain feed into its own frame slot, then
 * ONE composite launch stitches all of them: its work runs over (item, frame) pairs, so an item's LUT entries,
 * metadata and staging groups are fetched once for the batch.  Every output equals a separate stitch of its
 * frame, bit for bit.  Needs n_frames frames in flight (octvr_mapper_set_frames_in_flight) and, for 4, at
 * most 16 inputs; scaled-output and multi-band / feather mappers stitch the frames one by one. */
int octvr_mapper_stitch_batch(octvr_mapper* mapper, int n_frames, const uint8_t* const* in_dev, const size_t* in_pitch,
                              uint8_t* const* out_dev, size_t out_pitch, const double* gains, void* stream);
/* The same with Mapper::stitch's preview_output (mapper.cpp:308-312): the RGB result resized
 * (cuda::resize INTER_LINEAR) into a preview_w x preview_h CV_8UC3 device image (3 bytes per pixel,
 * row pitch preview_pitch); preview_dev NULL = none.  Needs one frame in flight. */
int octvr_mapper_stitch_preview(octvr_mapper* mapper, const uint8_t* const* in_dev, const size_t* in_pitch,
                                uint8_t* out_dev, size_t out_pitch, uint8_t* preview_dev, int preview_w, int preview_h,
                                size_t preview_pitch, const double* gains, int n_gains, void* stream);
/* Mapper::gains() (mapper.hpp:88-90): gains used by the last stitch (synchronizes the stream). */
int octvr_mapper_gains(octvr_mapper* mapper, double* gains, int n);
/* Frames in flight (no reference counterpart: vr::Mapper is not re-entrant, and AsyncMultiMapper
 * serialises its stitches on one compute stream, async.cpp:78-92).  k slots of per-frame device state
 * (gains, gain-feed totals, composite work queue); consecutive stitches take the slots in turn, so
 * stitches issued on different streams overlap (frame k+1's gain feed under frame k's composite).
 * A stitch waits (through an event) only for its slot's previous stitch.
 * k > 1 needs the output at template size (no scaled output; OCTVR_E_UNSUPPORTED otherwise);
 * multi-band / feather mappers get per-slot pyramids.  Synchronizes. */
#define OCTVR_MAX_FRAMES_IN_FLIGHT 16
int octvr_mapper_set_frames_in_flight(octvr_mapper* mapper, int k);
/* Algorithmic device bytes read+written by one launch of the composite (stitch) kernel: 4 B tiled
 * LUT entry (8 B in wide tiles) + 1.5 B YUV420 out per output pixel + 1.5 B per input pixel (each
 * source frame read once) + the per-item headers (multi-band / feather: the whole blend sequence). */
int octvr_mapper_traffic(const octvr_mapper* mapper, double* bytes_per_frame);
/* The same split into the rig constants the composite reads once per launch (tiled-LUT entries, item headers,
 * wide-tile entries: read once for a whole frame batch, octvr_mapper_stitch_batch) and the per-frame bytes
 * (output, source); lut + frame = octvr_mapper_traffic.  Multi-band / feather: lut 0. */
int octvr_mapper_traffic_parts(const octvr_mapper* mapper, double* lut_bytes, double* frame_bytes);
/* Live per-kernel timing for roofline accounting: with enable = k > 0, every k-th stitch brackets
 * its main (composite) kernel with HIP events on the caller's stream (0 = off).  kernel_time
 * synchronizes on the recorded events, returns the summed device time and launch count, and resets
 * the log. */
int octvr_mapper_set_timing(octvr_mapper* mapper, int enable);
int octvr_mapper_kernel_time(octvr_mapper* mapper, double* total_ms, int* launches);
/* The same log with frames in flight (launches on several streams overlap): span_ms = summed
 * start-to-end times, busy_ms = length of the union of the launches' intervals (the wall time some
 * composite was running).  Synchronizes and resets the log. */
int octvr_mapper_kernel_busy(octvr_mapper* mapper, double* span_ms, double* busy_ms, int* launches);
/* The logged launches themselves: [start_ms[k], end_ms[k]] relative to the first launch's start, in issue
 * order, at most `cap` of them (*n: how many were logged); the log is then cleared as by kernel_busy. */
int octvr_mapper_kernel_intervals(octvr_mapper* mapper, double* start_ms, double* end_ms, int cap, int* n);
/* The arithmetic behind kernel_busy, on host arrays: span = sum of (end - start), busy = length of the
 * union of the n intervals [start[k], end[k]] (overlapping, nested, touching or disjoint, any order). */
int octvr_interval_union(const double* start, const double* end, int n, double* span, double* busy);
/* Build-time statistics of a mapper as a JSON object (tiles, wide tiles, staged bytes, gain samples). */
int octvr_mapper_info(const octvr_mapper* mapper, char* buf, size_t len);
void octvr_mapper_destroy(octvr_mapper* mapper);

/* ---- vr::AsyncMultiMapper -------------------------------------------------------------------- */
/* AsyncMultiMapper::New(mts, in_sizes, out_size, blend_modes, gain_modes, output_regions, preview)
 * (modules/octvr/src/async.cpp:195-350, octvr.hpp:103-121): one vr::Mapper per rig, all fed the same
 * n_inputs camera frames, each writing the region output_regions[4*i .. 4*i+3] = (x, y, w, h) (fractions
 * of out_w x out_h, async.cpp:20-30) of one merged YUV420P output.  gain_modes[i]: -1 = no gain, i = estimate,
 * j in [0, i) = use mapper j's gains of the same frame (async.cpp:78-86).  A 3-deep pipeline of pinned host
 * and device buffers overlaps the host copies, the H2D upload, the stitch and the D2H download of
 * consecutive frames (async.cpp:32-172).  No preview: octvr_async_create_preview adds it. */
typedef struct octvr_async octvr_async;
int octvr_async_create(const octvr_rig* const* rigs, int n_rigs, int device, int n_inputs, const int* in_w,
                       const int* in_h, int out_w, int out_h, const int* blend_modes, const int* gain_modes,
                       const double* output_regions, octvr_async** async);
/* The same with mapper creation flags for every mapper (octvr_mapper_create_ex; OCTVR_REMAP_TEXTURE keeps
 * the reference's CUDA sampling, which its AsyncMultiMapper runs through vr::Mapper). */
int octvr_async_create_ex(const octvr_rig* const* rigs, int n_rigs, int device, int n_inputs, const int* in_w,
                          const int* in_h, int out_w, int out_h, const int* blend_modes, const int* gain_modes,
                          const double* output_regions, int flags, octvr_async** async);
/* The same with AsyncMultiMapper::New's preview_size (async.cpp:73-110, 141-171): every frame, each mapper
 * also writes Mapper::stitch's preview_output (its RGB result resized, cuda::resize INTER_LINEAR,
 * mapper.cpp:308-312) into its region _rect_mul_size(output_regions[i], preview) of one preview_w x
 * preview_h RGB image (CV_8UC3, black where no region writes; a region whose rectangle is empty writes
 * none), which is downloaded with the outputs and published when the frame's outputs are written:
 * octvr_async_pop_preview reads the latest, a sink receives every one.  preview_w = preview_h = 0: none
 * (= octvr_async_create_ex).  Mappers with a preview stitch through their RGB result frame
 * (mapper.cpp:266-312 order: composite, then RGB -> YUV420P and the preview resize). */
int octvr_async_create_preview(const octvr_rig* const* rigs, int n_rigs, int device, int n_inputs, const int* in_w,
                               const int* in_h, int out_w, int out_h, const int* blend_modes, const int* gain_modes,
                               const double* output_regions, int flags, int preview_w, int preview_h,
                               octvr_async** async);
/* vr::PreviewDataHeader (octvr.hpp:97-101): what the reference writes in front of the RGB bytes of each
 * Qt shared-memory zone (async.cpp:163-167): width, height, step = 0, fps = 1 / (mean frame interval over
 * the last completed block of 10 frames, in s), 0 until 10 frames have completed (async.cpp:141-147). */
typedef struct octvr_preview_header {
    int width, height;
    int step;
    double fps;
} octvr_preview_header;
/* The latest published preview: rgb (host, preview_h rows of preview_w * 3 bytes, row pitch `pitch`) and
 * its header.  Before the first frame completes, hdr->width = hdr->height = 0 and rgb is untouched (the
 * reference's zones start with a zeroed header, preview_video.cpp:62-66).  OCTVR_E_INVALID without a
 * preview.  After pop() of frame k with no later frame pushed, this is frame k's preview. */
int octvr_async_pop_preview(octvr_async* async, uint8_t* rgb, size_t pitch, octvr_preview_header* hdr);
/* Called on the pipeline's copy-out thread for every frame's preview, after that frame's outputs are written
 * and before its pop() returns (the reference's Qt shared-memory write, async.cpp:149-171): rgb = the
 * downloaded preview (host, valid during the call only), pitch = preview_w * 3.  A Qt caller writes it into
 * zone *meta of its two QSharedMemory zones.  NULL removes the sink. */
typedef void (*octvr_preview_sink)(void* user, const uint8_t* rgb, size_t pitch, const octvr_preview_header* hdr);
int octvr_async_set_preview_sink(octvr_async* async, octvr_preview_sink sink, void* user);
/* Build-time facts of the pipeline as a JSON object: packed_bytes (the footprint bytes uploaded per frame,
 * run gaps included), runs, frame bytes, preview size, the mappers' creation flags. */
int octvr_async_info(const octvr_async* async, char* buf, size_t len);
/* push(inputs, output) (async.cpp:174-189): in_planes[3*i+0/1/2] = Y, U, V host planes of input i
 * (W x H, W/2 x H/2, W/2 x H/2) with row pitches in_pitches[3*i+k]; out_planes[0/1/2] / out_pitches: the
 * merged output's Y (out_w x out_h), U and V (out_w/2 x out_h/2) planes.  Returns once the frame is queued;
 * all planes must stay valid until the matching pop. */
int octvr_async_push(octvr_async* async, const uint8_t* const* in_planes, const size_t* in_pitches,
                     uint8_t* const* out_planes, const size_t* out_pitches);
/* pop() (async.cpp:191-193): blocks until the oldest pushed frame has been written to its output planes;
 * returns that frame's status (OCTVR_E_INVALID if nothing is pending). */
int octvr_async_pop(octvr_async* async);
/* Register an output plane set (Y, U, V of out_w x out_h, out_w/2 x out_h/2, ...) that the caller reuses
 * (a ring of output frames, as the reference reuses its output Mats, async.cpp:113-138): the planes are
 * page-locked (hipHostRegister) and every later push with exactly these pointers and pitches is downloaded
 * straight into them — no pinned staging, no host copy-out.  The planes must stay allocated until
 * octvr_async_unregister_output or octvr_async_destroy.  OCTVR_E_HIP if the memory cannot be locked (the
 * planes then keep the staging path). */
int octvr_async_register_output(octvr_async* async, uint8_t* const* planes, const size_t* pitches);
/* Undo octvr_async_register_output (no frame may be pending). */
int octvr_async_unregister_output(octvr_async* async, uint8_t* const* planes);
/* Frames pushed and not yet popped. */
int octvr_async_pending(const octvr_async* async, int* n);
/* Drains the frames in flight and joins the pipeline's worker threads (the reference leaves its five
 * threads running forever, async.cpp:337-349). */
void octvr_async_destroy(octvr_async* async);

/* ---- vr::FastMapper ------------------------------------------------------------------------- */
/* FastMapper(mt, in_sizes) (modules/octvr/src/mapper_fast.cpp:27-109): feather-weighted NV12 stitch
 * (weights 255 * max(DT_i - 5, 0) / (1e-5 + sum), half-size chroma maps); the rig's inputs must cover
 * the whole output (no ROI, mapper_fast.cpp:50-51) and have no overlays. */
typedef struct octvr_fastmapper octvr_fastmapper;
int octvr_fastmapper_create(const octvr_rig* rig, int device, int n_inputs, const int* in_w, const int* in_h,
                            octvr_fastmapper** fastmapper);
/* FastMapper::stitch_nv12 (mapper_fast.cpp:153-195) on device NV12 frames (H rows of Y, then H/2 rows
 * of interleaved U,V; W <= pitch < 2^24).  Output: W x 3H/2, chroma rows interleaved V,U — the reference's
 * channel order (merge of the V-then-U accumulators).  Stream-ordered; the FastMapper keeps no per-call
 * device state, so calls with their own outputs may run concurrently on different streams. */
int octvr_fastmapper_stitch_nv12(octvr_fastmapper* fastmapper, const uint8_t* const* in_dev, const size_t* in_pitch,
                                 uint8_t* out_dev, size_t out_pitch, void* stream);
/* Algorithmic bytes one stitch_nv12 moves (entries read, output written, source bytes its weighted taps
 * reach): the roofline basis of bench.py --config F2. */
/* n_frames (1, 2 or 4) frames in one launch per plane (no reference counterpart): frame f's inputs are
 * in_dev[f * n_inputs + i], its output out_dev[f] (one pitch); each run's entries and feather weights are
 * loaded once and applied to every frame.  Every output equals stitch_nv12 of its frame, bit for bit.  4
 * frames hold at most 16 inputs. */
int octvr_fastmapper_stitch_nv12_batch(octvr_fastmapper* fastmapper, int n_frames, const uint8_t* const* in_dev,
                                       const size_t* in_pitch, uint8_t* const* out_dev, size_t out_pitch, void* stream);
int octvr_fastmapper_traffic(const octvr_fastmapper* fastmapper, double* bytes);
/* The same split into entries / weights / block headers (once per launch) and per-frame bytes (taps, output). */
int octvr_fastmapper_traffic_parts(const octvr_fastmapper* fastmapper, double* lut_bytes, double* frame_bytes);
void octvr_fastmapper_destroy(octvr_fastmapper* fastmapper);

/* ---- standalone kernels --------------------------------------------------------------------- */
/* cv::remap(src, dst, map1*sx, map2*sy, INTER_LINEAR, BORDER_CONSTANT) on u8 with cn in {1,3,4}
 * channels: 5-bit coordinates, 15-bit weights (imgwarp.cpp:211-280, 3812-4030, 4246-4497). */
int octvr_remap_u8(const uint8_t* src_dev, int sw, int sh, size_t spitch, int cn, const float* map1_dev,
                   const float* map2_dev, int mw, int mh, size_t mpitch_elems, float scale_x, float scale_y,
                   uint8_t* dst_dev, size_t dpitch, void* stream);

/* ---- camera mask rasterisation (host; what octvr_rig_create_json uses for `selection`,
 *      `exclude_masks`, `include_masks`, camera.cpp:96-187) ------------------------------------ */
/* cv::fillPoly(img, {pts}, color), lineType 8, shift 0, on a w x h u8 image (row pitch w);
 * pts = x0,y0,x1,y1,... (imgproc/src/drawing.cpp:1196-1405, 1894-1917). */
int octvr_fill_poly_u8(uint8_t* img, int w, int h, const int* pts, int npts, uint8_t color);
/* cv::imdecode(png, IMREAD_COLOR) for PNG data (imgcodecs/src/grfmt_png.cpp:240-286), written as
 * R,G,B bytes into rgb (capacity rgb_cap bytes); *w, *h receive the size.  rgb may be NULL to query. */
int octvr_png_decode_rgb(const uint8_t* png, size_t n, uint8_t* rgb, size_t rgb_cap, int* w, int* h);

/* ---- self-test hooks (used by tests/, not by the stitching path) ---------------------------------- */
/* LUT-build bookkeeping of a JSON rig: the number of input i's output pixels whose projection the GPU
 * build left to the host because a last-ulp device / glibc libm difference could change them
 * (LutGuard, camera_math.hpp); 0 for rigs from .dat / arrays. */
int octvr_rig_lut_recomputed(const octvr_rig* rig, int i, uint64_t* n);
/* The FP64 projection (MapperTemplate::add_input's (x, y) before the f32 rounding, template.cpp:70-95)
 * of every pixel of an out_w x out_h output for input `input` of a JSON rig, on `device` (where = 0;
 * fragile[k] = 1 where the guard defers the pixel to the host) or on the host with glibc (where = 1,
 * fragile unused).  x, y, fragile: host arrays of out_w * out_h.  Include masks are not evaluated. */
int octvr_debug_project_f64(const char* json, int out_w, int out_h, int input, int device, int where, double* x,
                            double* y, uint8_t* fragile);
/* FastMapper index audit (host only, no GPU): builds the FastMapper plan of `rig` for these input sizes
 * (8-byte entries when force_wide) exactly as octvr_fastmapper_create does, and replays on the host every
 * index fast_y_kernel / fast_uv_kernel derive for every run, camera group, slot and lane — block, entry,
 * weight and header indices against the uploaded arrays, camera against the frame set, each 8-byte tap-row
 * load against an NV12 frame of pitch w + pitch_pad, the in-image taps' bytes inside the loaded 8, the
 * output bytes.  Writes per-plane counts as JSON; returns OCTVR_E_INVALID if any access is out of range. */
int octvr_debug_fastmapper_audit(const octvr_rig* rig, int n_inputs, const int* in_w, const int* in_h, int force_wide,
                                 int pitch_pad, char* json, size_t len);
/* The blend = 0 composite's tiling on the host only (no GPU): the copy chain's winner per output pixel,
 * then the tiled LUT exactly as octvr_mapper_create builds it — including its check that every tap of
 * every pixel lies in a staged group of its slot (OCTVR_E_INVALID otherwise) — reported as JSON (items,
 * wide tiles, staged pixels against the boxes' pixels, bytes, chunk histogram).  flags: the mapper's
 * creation flags (OCTVR_REMAP_TEXTURE: texture-convention entries, interior ones staged, border tiles wide). */
int octvr_debug_tiled_lut_info(const octvr_rig* rig, int n_inputs, const int* in_w, const int* in_h, int flags,
                               char* json, size_t len);
/* The gain feed's samples as octvr_mapper_create lays them out (host only, no GPU): per sample its entry
 * (samples[2k] = xy, samples[2k+1] = code, kernels.hpp CompositeEntry) and partner mask, in the order the
 * feed's waves take them (padding included).  count receives the number of samples; samples / partners
 * NULL = count only. */
int octvr_debug_gain_plan(const octvr_rig* rig, int n_inputs, const int* in_w, const int* in_h, int flags,
                          uint32_t* samples, uint16_t* partners, size_t cap, size_t* count);
/* The rig-config JSON reader on one document: the first number of `json` (a number, or the first element
 * of an array), parsed with rapidjson's rules (flags 0, as the reference reads its configs) or correctly
 * rounded (OCTVR_JSON_EXACT; out-of-range literals give +-HUGE_VAL / the subnormal / 0 as strtod). */
int octvr_debug_json_number(const char* json, int flags, double* value);
/* The host build's worker threads (tiler, seam finder, blender weights, audits) on n_threads threads of
 * which thread `failing` raises an error (test hook, no GPU): the error reaches the caller as a status
 * (OCTVR_E_INVALID + octvr_last_error) instead of terminating the process; failing < 0 = none fails. */
int octvr_debug_worker_failure(int n_threads, int failing);
/* Saturating float -> u8 conversion as the kernels implement it (method 0: rint + clamp in VALU,
 * method 1: v_cvt_pk_u8_f32), for a known-answer test of round-half-even and clamping on device. */
int octvr_selftest_sat_u8(const float* in_dev, uint8_t* out_dev, int n, int method, void* stream);

#ifdef __cplusplus
}
#endif
#endif
