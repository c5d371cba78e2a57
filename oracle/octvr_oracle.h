/*
 * octvr_oracle.h — CPU restatement of the reference octVR hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This library is the checker for the HIP product path
 * (opencv-octvr_amd/) and the timed "cpu_baseline" leg of bench.py.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline may load it; the product never links it.
 *
 * Every function cites the reference file:line (paths relative to the blahgeek/OpenCV-octVR root)
 * whose arithmetic it restates.  Parity pinning: tests/golden/ (generated from the reference by
 * oracle/golden_gen/) — see DESIGN.md "Oracle".
 */
#ifndef OCTVR_ORACLE_H
#define OCTVR_ORACLE_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
    ORC_EQUIRECT = 0, ORC_FULLFRAME_FISHEYE = 1, ORC_FISHEYE = 2, ORC_PINHOLE = 3, ORC_NORMAL = 4,
    ORC_PERSPECTIVE = 5, ORC_OCAM = 6, ORC_STUPIDOVAL = 7, ORC_CUBIC = 8, ORC_EQAREA_NORTH = 9, ORC_EQAREA_SOUTH = 10
};

typedef struct {
    int type;
    double R[9];      /* rotate_matrix, camera.cpp:57-70 */
    double Rinv[9];   /* rotate_matrix.inv(), camera.cpp:205 */
    double min_lon, max_lon;           /* longitude_selection, camera.cpp:125-135 */
    /* equirectangular.hpp:61-62 */
    double min_lat, max_lat, scale_lon;
    /* fullframe_fisheye_cam.cpp:105-140 */
    int width, height;
    int crop_x, crop_y, crop_w, crop_h, crop_circular;
    double hfov, center_dx, center_dy;
    double rad[6];
    /* pinhole_cam.cpp:13-30 (OpenCV fisheye model) */
    double fx, fy, cx, cy, k[4];
    /* camera.cpp:96-112 `selection` rectangle (an exclude mask that is 255 outside it) */
    int sel, sel_l, sel_r, sel_t, sel_b;
    /* cv::projectPoints distortion k1..tauY (calibration.cpp:644-665) and the tilt matrix */
    double dist[14], tilt[9];
    double aspect, cam_x, cam_y, cam_z; /* normal.cpp:13-19 */
    double sf;                          /* perspective.cpp:16 */
    double circle;                      /* eqarea{north,south}pole.hpp arctic / antarctic circle */
    int len_pol, len_invpol;            /* ocam_fisheye.hpp:23-35 */
    double xc, yc, oc, od, oe;
    double pol[64], invpol[64];
    /* exclude_mask / include_mask (camera.cpp:72-123), width x height, or NULL */
    const uint8_t* excl;
    const uint8_t* incl;
} orc_camera;

/* Type initialisers reset rotation to identity and longitude range to [-pi, pi]; call
 * orc_camera_set_rotation / set min_lon,max_lon afterwards.
 * Camera::Camera rotation part (camera.cpp:49-70): R = (Rx*Rz)*Ry from (roll, -yaw, -pitch)
 * via Rodrigues (calib3d/src/calibration.cpp:252-345); Rinv by lapack.cpp invert 3x3 closed form. */
void orc_rotation_rpy(double roll, double yaw, double pitch, double R[9]);
void orc_invert3(const double* A, double* out);
void orc_camera_set_rotation(orc_camera* c, const double R[9]);

void orc_camera_equirect(orc_camera* c, double min_lat, double max_lat, double scale_lon);
void orc_camera_fullframe_fisheye(orc_camera* c, int width, int height, int crop_l, int crop_r, int crop_t,
                                  int crop_b, int has_crop, int crop_circular, double hfov, double center_dx,
                                  double center_dy, const double radial[3]);
void orc_camera_fisheye(orc_camera* c, int width, int height, double fx, double fy, double cx, double cy,
                        const double k[4]);

/* PinholeCamera (pinhole_cam.cpp:13-30): nd in {0,4,5,8,12,14} distortion coefficients. */
void orc_camera_pinhole(orc_camera* c, int width, int height, double fx, double fy, double cx, double cy,
                        const double* dist, int nd);
void orc_camera_normal(orc_camera* c, double aspect_ratio, double cam_opt);           /* normal.cpp:13-22 */
void orc_camera_perspective(orc_camera* c, double aspect_ratio, double sf);           /* perspective.cpp:14-19 */
void orc_camera_ocam(orc_camera* c, const double* pol, int len_pol, const double* invpol, int len_invpol, double xc,
                     double yc, double cc, double d, double e, int width, int height); /* ocam_fisheye.cpp:82-110 */
/* stupidoval / cubic / eqareanorthpole / eqareasouthpole (circle: arctic / antarctic latitude) */
void orc_camera_simple(orc_camera* c, int type, double circle);
void orc_camera_set_selection(orc_camera* c, int width, int height, int l, int r, int t, int b);

/* MapperTemplate::add_input LUT loop (template.cpp:46-133) for one input camera.
 * map1/map2/mask are FULL output-size buffers (W*H); roi[4] = x,y,w,h (±8 pad, or full if !use_roi). */
int orc_lut_build(const orc_camera* out, const orc_camera* in, int W, int H, float* map1, float* map2,
                  uint8_t* mask, int use_roi, int roi[4]);
/* The same with the include-mask arbitration (template.cpp:86-116): visible is W*H, 1 = claimed by an
 * earlier camera (rejected here); pixels this camera claims first are set to 2. */
int orc_lut_build_vis(const orc_camera* out, const orc_camera* in, int W, int H, float* map1, float* map2,
                      uint8_t* mask, int use_roi, int roi[4], uint8_t* visible);
/* cv::fillPoly(img, {pts}, color), lineType 8, shift 0 (octvr_oracle_masks.c) */
void orc_fill_poly(uint8_t* img, int w, int h, const int* pts, int count, uint8_t color);

/* Camera::image_to_obj of `from`, then obj_to_image of `to`; nonzero where the reference throws. */
int orc_project(const orc_camera* from, const orc_camera* to, double u, double v, double* x, double* y);
/* orc_lut_build_vis on `threads` threads (identical result). */
int orc_lut_build_vis_mt(const orc_camera* out, const orc_camera* in, int W, int H, float* map1, float* map2,
                         uint8_t* mask, int use_roi, int roi[4], uint8_t* visible, int threads);
/* FP64 projection (before the f32 rounding) of output rows [y0, y1), full width. */
void orc_project_f64(const orc_camera* out, const orc_camera* in, int W, int H, int y0, int y1, double* x, double* y,
                     int threads);
/* MapperTemplate::morph_controlpoints (template_morph.cpp:69-237) on ROI-sized LUT planes, in place
 * (octvr_oracle_morph.c).  cps: n_cps x {n0, n1, x0, y0, x1, y1}; src_tris[i] / dst_tris[i] receive
 * camera i's triangles (6 floats each, at most tri_cap), n_tris[i] their count.  Returns the number
 * of control points kept, or < 0: -1 bad / out-of-bounds point, -2 camera without image_to_obj,
 * -3 frame loop does not advance, -4 triangulation failure. */
int orc_morph_controlpoints(const orc_camera* out, const orc_camera* const* cams, int n, int W, int H,
                            const int* rois, float* const* map1, float* const* map2, uint8_t* const* masks,
                            const double* cps, int n_cps, float* const* src_tris, float* const* dst_tris,
                            int tri_cap, int* n_tris);

/* cv::Subdiv2D(Rect(0,0,1,1)) + insert + getTriangleList, triangles with all corners in [0,1]^2. */
int orc_delaunay_triangles(const float* pts, int n, float* out, int cap);

/* The same per-pixel LUT rule for output rows [y0, y1) only (no ROI); buffers are (y1-y0) x W. */
void orc_lut_rows(const orc_camera* out, const orc_camera* in, int W, int H, int y0, int y1, float* map1,
                  float* map2, uint8_t* mask);

/* initInterTab2D(INTER_LINEAR, fixpt) incl. its sum fix-up quirk (imgproc/src/imgwarp.cpp:211-280). */
void orc_bilinear_tab(int16_t tab[1024 * 4]);

/* cv::remap INTER_LINEAR, BORDER_CONSTANT 0, u8 with cn channels (imgwarp.cpp:3812-4030, 4246-4497).
 * X = fl32(map1 * scale_x), Y = fl32(map2 * scale_y) (the caller's `map*W`, template.cpp:174-176). */
void orc_remap_u8(const uint8_t* src, int sw, int sh, size_t spitch, int cn, const float* map1, const float* map2,
                  int mw, int mh, size_t mpitch_elems, float scale_x, float scale_y, uint8_t* dst, size_t dpitch);

/* Own BT.601 definitions standing in for NPP nppiYUV420ToRGB / nppiRGBToYUV420 (parity unpinned,
 * cudaimgproc/src/color.cpp:2269,2306).  Layout "Y over [U|V]" of mapper.hpp:75-83. */
void orc_yuv420_to_rgba(const uint8_t* yuv, int w, int h, size_t pitch, uint8_t* rgba, size_t rgba_pitch);
void orc_rgb_to_yuv420(const uint8_t* rgb, int w, int h, size_t rgb_pitch, int rgb_cn, uint8_t* yuv, size_t pitch);

/* cv::solve DECOMP_LU for doubles (core/src/lapack.cpp:1050-1275, matrix_decomp.cpp:50-110). */
int orc_solve(const double* A, const double* b, int n, double* x);

/* Gain compensator feed (GainCompensatorGPU, stitching/src/exposure_compensate.cpp:174-297 + mapper.cpp:94-114,
 * 234-237).  warped[i]: ROI-sized u8x4 (pitch = roi_w*4), masks[i]: ROI-sized u8 LUT masks. */
int orc_gain_feed(int n, const int* rois, const uint8_t* const* warped, const uint8_t* const* masks, int out_w,
                  int out_h, double* gains_out);

/* One Mapper::stitch frame, blend=0 (mapper.cpp:193-312): YUV420 in -> YUV420 out, optional gain.
 * gains_in may be NULL (estimate) ; gains_out receives the gains used (may be NULL). */
typedef struct {
    int n;
    const int* in_w;
    const int* in_h;
    const uint8_t* const* in_yuv;
    const size_t* in_pitch;
    const int* rois;                 /* n*4 */
    const float* const* map1;        /* ROI-sized, normalized */
    const float* const* map2;
    const uint8_t* const* masks;     /* ROI-sized LUT masks */
    int out_w, out_h;
    uint8_t* out_yuv;
    size_t out_pitch;
    int enable_gain;
    const double* gains_in;
    double* gains_out;
    int threads;
    int row_begin, row_end;          /* restrict composite+output to a row band (cpu_baseline sample); 0,0 = all */
    int blend;                       /* Mapper blend: 0 copy chain, > 0 multi-band (bands = ceil(log2 blend) - 1), < 0 feather */
    const uint8_t* const* seams;     /* ROI-sized seam masks (multi-band weights); NULL unless blend > 0 */
    const float* const* vig;         /* per camera: vignette gains at input size (in_w x in_h) or NULL; may be NULL */
    int scale_w, scale_h;            /* scaled output size (mapper.cpp:69, 290-306); 0,0 = out_w x out_h.  When
                                        set, out_yuv / out_pitch describe the scaled frame and row_begin/end are ignored */
    uint8_t* preview;                /* preview_output (mapper.cpp:308-312): cuda::resize INTER_LINEAR of the RGB result
                                        to preview_w x preview_h, u8x3 rows of preview_pitch bytes; NULL = none */
    int preview_w, preview_h;
    size_t preview_pitch;
    int remap_tex;                   /* 1: warp with orc_fast_remap_tex_rgba (the CUDA fastRemap texture model,
                                        OCTVR_REMAP_TEXTURE) instead of orc_remap_u8 */
} orc_frame;
int orc_stitch_frame(const orc_frame* f);
/* A12 CUDA fastRemap texture bilinear on RGBA (for the documented A12-vs-A13 tolerance only). */
void orc_fast_remap_tex_rgba(const uint8_t* src, int w, int h, size_t spitch, const float* map1, const float* map2,
                             int mw, int mh, size_t mpitch, uint8_t* dst, size_t dpitch);

/* ---- GPU blenders (octvr_oracle_blend.c) ----------------------------------- */
void orc_fast_pyr_down_u8x4(const uint8_t* src, int sw, int sh, uint8_t* dst, int threads);           /* K2 */
void orc_pyr_up_u8x4(const uint8_t* src, int sw, int sh, uint8_t* dst, int threads);                  /* K3 */
void orc_pyr_up_s16x3(const int16_t* src, int sw, int sh, int16_t* dst, int threads);                 /* K3 */
void orc_pyr_down_f32(const float* src, int sw, int sh, float* dst, int threads);                     /* K4 */
/* MultiBandGPUBlender(seams, rois, bands).blend(warped u8x4 ROI images, result u8x3): writes the
 * aligned result ROI of `result` (out_w x out_h, pitch bytes).  Returns 0, or < 0 on a failed
 * reference assertion. */
int orc_multiband_blend(int n, const int* rois, const uint8_t* const* seams, const uint8_t* const* warped, int bands,
                        uint8_t* result, int out_w, int out_h, size_t result_pitch, int threads);
/* FeatherGPUBlender(masks, rois, border).blend(warped, result): blend < 0 with border = -blend. */
int orc_feather_blend(int n, const int* rois, const uint8_t* const* masks, const uint8_t* const* warped, int border,
                      uint8_t* result, int out_w, int out_h, size_t result_pitch);
/* Mapper's band count for blend > 0: int(ceil(log(blend) / log(2.)) - 1.) (mapper.cpp:172). */
int orc_blend_bands(int blend);

/* Vignette::getMap (vignette.cpp:39-54): w x h f32 map of 1 / (a + r^2 (b + r^2 (c + d r^2))); the
 * coefficients already divided by 2^exposure in float (vignette.cpp:26-33) by the caller. */
void orc_vignette_map(double a, double b, double c, double d, int w, int h, float* out);
/* cuda::resize INTER_LINEAR on f32 (texture LinearFilter path, filters.hpp:79-117; FMA-contracted). */
void orc_resize_linear_cuda_f32(const float* src, int sw, int sh, float* dst, int dw, int dh);

/* K13/K14 CUDA resize semantics used by the gain path (cudawarping/src/cuda/resize.cu:57-103). */
void orc_resize_nearest_u8(const uint8_t* src, int sw, int sh, size_t spitch, int cn, uint8_t* dst, int dw, int dh,
                           size_t dpitch);
void orc_resize_linear_cuda_u8(const uint8_t* src, int sw, int sh, size_t spitch, uint8_t* dst, int dw, int dh,
                               size_t dpitch);
/* The same kernel on cn interleaved u8 channels (resize_linear<uchar3>, the scaled output's resize). */
void orc_resize_linear_cuda_u8c(const uint8_t* src, int sw, int sh, size_t spitch, int cn, uint8_t* dst, int dw,
                                int dh, size_t dpitch);

/* ---- seam masks (octvr_oracle_seam.c) ------------------------------------------ */
/* cv::resize INTER_LINEAR u8 on the CPU (imgwarp.cpp:3120-3480; fixed point, 11-bit coefficients). */
void orc_resize_linear_u8(const uint8_t* src, int sw, int sh, size_t spitch, int cn, uint8_t* dst, int dw, int dh,
                          size_t dpitch);
/* cv::distanceTransform(src, dst, DIST_L2, 3) -> f32 (distransform.cpp:48-139). */
void orc_distance_transform_l2_3x3(const uint8_t* src, int w, int h, size_t spitch, float* dist, size_t dpitch_elems);
/* MapperTemplate::create_masks() without images (template.cpp:155-204 -> DistanceSeamFinder,
 * seam_finders.cpp:97-133).  masks / seams: ROI-sized u8 (tightly packed); seams are written. */
int orc_create_masks(int n, const int* rois, const uint8_t* const* masks, int out_w, uint8_t* const* seams);

/* ---- vr::FastMapper (octvr_oracle_fast.c) --------------------------------- */
/* convertMaps(map1 * sx, map2 * sy, CV_16SC2): s16 (x, y) pairs + u16 fraction codes (imgwarp.cpp:5039-5043). */
void orc_convert_maps(const float* m1, const float* m2, size_t n, float sx, float sy, int16_t* xy, uint16_t* a);
/* cv::resize of a f32 map to half size (area fast path, SSE grouping of imgwarp.cpp:2284-2337). */
void orc_resize_half_f32(const float* src, int w, int h, float* dst);
/* FastMapper(mt, in_sizes) + stitch_nv12 (mapper_fast.cpp:27-195): maps / masks are FULL output size
 * (the reference asserts ROI = whole frame); inputs NV12 (Y rows, then interleaved UV rows); the output
 * is W x 1.5H with the chroma rows interleaved V, U (the reference's channel order). */
int orc_fastmapper_nv12(int n, const int* in_w, const int* in_h, const float* const* map1, const float* const* map2,
                        const uint8_t* const* masks, int W, int H, const uint8_t* const* in_nv12,
                        const size_t* in_pitch, uint8_t* out, size_t out_pitch);

#ifdef __cplusplus
}
#endif
#endif
