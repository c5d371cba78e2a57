/*
 * octvr_oracle_fast.c — CPU restatement of vr::FastMapper (TEST INFRASTRUCTURE ONLY; see octvr_oracle.h).
 *
 *   constructor  modules/octvr/src/mapper_fast.cpp:27-109
 *   stitch_nv12  mapper_fast.cpp:153-195
 *   remap_weighted (OpenCL)  imgproc/src/opencl/remap_weighted.cl:20-78, host imgwarp.cpp:4635-4687
 *   convertMaps f32 -> 16SC2/16UC1  imgwarp.cpp:4831-5044 (scalar rule :5039-5043)
 *   resize 2x INTER_LINEAR -> INTER_AREA fast path, f32 (imgwarp.cpp:2284-2337 SSE, 2403-2460 tail)
 *
 * The reference evaluates the feather weights on its OpenCL device: division there need not be
 * correctly rounded; this restatement uses IEEE division (parity unpinned, no fixture exists).
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "octvr_oracle.h"

static inline int sat_int_rne(float v) { /* saturate_cast<int>(float) = cvRound */
    if (v != v) return INT32_MIN;
    if (v >= 2147483648.f) return INT32_MAX;
    if (v < -2147483648.f) return INT32_MIN;
    return (int)lrintf(v);
}
static inline short sat_s16(int v) { return (short)(v < -32768 ? -32768 : v > 32767 ? 32767 : v); }
static inline uint8_t sat_u8_rte(float v) {
    if (!(v > 0.f)) return 0;
    if (v >= 255.f) return 255;
    return (uint8_t)lrintf(v);
}
static inline uint16_t sat_u16_rte(float v) {
    if (!(v > 0.f)) return 0;
    if (v >= 65535.f) return 65535;
    return (uint16_t)lrintf(v);
}

/* convertMaps(map1 * sx, map2 * sy, CV_16SC2): MatExpr scale = convertTo(-1, s) in f32 (cvtScale32f). */
void orc_convert_maps(const float* m1, const float* m2, size_t n, float sx, float sy, int16_t* xy, uint16_t* a) {
    for (size_t k = 0; k < n; k++) {
        float X = m1[k] * sx + 0.f, Y = m2[k] * sy + 0.f;
        int ix = sat_int_rne(X * 32), iy = sat_int_rne(Y * 32);
        xy[2 * k] = sat_s16(ix >> 5);
        xy[2 * k + 1] = sat_s16(iy >> 5);
        a[k] = (uint16_t)((iy & 31) * 32 + (ix & 31));
    }
}

/* cv::resize(f32, (w/2, h/2)) = resizeAreaFast with ResizeAreaFastVec_SIMD_32f: columns in groups
 * of 4 as ((a + b) + (c + d)) * 0.25f, the rest as (0 + (((a + b) + c) + d)) * 0.25f. */
void orc_resize_half_f32(const float* src, int w, int h, float* dst) {
    int dw = w / 2, dh = h / 2, vec = dw / 4 * 4;
    for (int y = 0; y < dh; y++) {
        const float* s0 = src + (size_t)(2 * y) * w;
        const float* s1 = s0 + w;
        float* d = dst + (size_t)y * dw;
        for (int x = 0; x < dw; x++) {
            float a = s0[2 * x], b = s0[2 * x + 1], c = s1[2 * x], e = s1[2 * x + 1];
            float sum = x < vec ? (a + b) + (c + e) : 0.f + (((a + b) + c) + e);
            d[x] = sum * 0.25f;
        }
    }
}

/* cv::resize(u8, (w/2, h/2)): the 8u area fast path, (a + b + c + d + 2) >> 2. */
static void resize_half_u8(const uint8_t* src, int w, int h, uint8_t* dst) {
    int dw = w / 2, dh = h / 2;
    for (int y = 0; y < dh; y++)
        for (int x = 0; x < dw; x++) {
            const uint8_t* s = src + (size_t)(2 * y) * w + 2 * x;
            dst[(size_t)y * dw + x] = (uint8_t)((s[0] + s[1] + s[w] + s[w + 1] + 2) >> 2);
        }
}

/* remap_weighted.cl for one output pixel: bilinear in f32 with u = code / 32, taps outside -> 0,
 * times the u8 weight, convert_ushort_sat_rte, added to the u16 accumulator (wraps). */
static inline uint16_t remap_weighted_px(const uint8_t* src, int sw, int sh, size_t spitch, size_t sstep, int16_t sx,
                                         int16_t sy, uint16_t code, uint8_t w) {
    int m = code & (32 * 32 - 1);
    float ux = (float)(m & 31) / 32.f, uy = (float)(m >> 5) / 32.f;
    int X[4] = {sx, sx + 1, sx, sx + 1}, Y[4] = {sy, sy, sy + 1, sy + 1};
    float t[4];
    for (int k = 0; k < 4; k++)
        t[k] = (X[k] >= sw || Y[k] >= sh || X[k] < 0 || Y[k] < 0) ? 0.f : (float)src[(size_t)Y[k] * spitch + (size_t)X[k] * sstep];
    float v = t[0] * (1 - ux) * (1 - uy) + t[1] * (ux) * (1 - uy) + t[2] * (1 - ux) * (uy) + t[3] * (ux) * (uy);
    v *= (float)w;
    return sat_u16_rte(v);
}

int orc_fastmapper_nv12(int n, const int* in_w, const int* in_h, const float* const* map1, const float* const* map2,
                        const uint8_t* const* masks, int W, int H, const uint8_t* const* in_nv12,
                        const size_t* in_pitch, uint8_t* out, size_t out_pitch) {
    if (n <= 0 || W <= 0 || H <= 0 || (W & 1) || (H & 1)) return -1;
    const size_t npx = (size_t)W * H, nh = (size_t)(W / 2) * (H / 2);
    /* feather weights (mapper_fast.cpp:75-94) */
    float** wt = (float**)calloc(n, sizeof(float*));
    float* total = (float*)malloc(sizeof(float) * npx);
    for (size_t k = 0; k < npx; k++) total[k] = 1e-5f;
    for (int i = 0; i < n; i++) {
        wt[i] = (float*)malloc(sizeof(float) * npx);
        orc_distance_transform_l2_3x3(masks[i], W, H, (size_t)W, wt[i], (size_t)W);
        for (size_t k = 0; k < npx; k++) {
            float v = wt[i][k] - 5.f;        /* subtract(weight_map, 5) */
            wt[i][k] = v > 0.f ? v : 0.f;    /* threshold(THRESH_TOZERO, 0) */
            total[k] = wt[i][k] + total[k];  /* add(weight_map, dst_weight_map, dst_weight_map) */
        }
    }
    uint16_t* accY = (uint16_t*)calloc(npx, sizeof(uint16_t));
    uint16_t* accV = (uint16_t*)calloc(nh, sizeof(uint16_t));
    uint16_t* accU = (uint16_t*)calloc(nh, sizeof(uint16_t));
    uint8_t* fm = (uint8_t*)malloc(npx);
    uint8_t* hfm = (uint8_t*)malloc(nh);
    int16_t* xy = (int16_t*)malloc(sizeof(int16_t) * 2 * npx);
    uint16_t* a = (uint16_t*)malloc(sizeof(uint16_t) * npx);
    float* hm1 = (float*)malloc(sizeof(float) * nh);
    float* hm2 = (float*)malloc(sizeof(float) * nh);
    for (int i = 0; i < n; i++) {
        for (size_t k = 0; k < npx; k++) {
            float e2 = total[k];
            float r = e2 != 0.f ? wt[i][k] / e2 : 0.f; /* divide(weight_maps[i], dst_weight_map) */
            fm[k] = sat_u8_rte(fmaf(r, 255.f, 0.f));    /* convertTo(CV_8U, 255.0) */
        }
        resize_half_u8(fm, W, H, hfm);
        const int w = in_w[i], h = in_h[i];
        const size_t p = in_pitch[i];
        const uint8_t* Yp = in_nv12[i];
        const uint8_t* UV = Yp + (size_t)h * p;
        orc_convert_maps(map1[i], map2[i], npx, (float)w, (float)h, xy, a);
        for (size_t k = 0; k < npx; k++)
            accY[k] = (uint16_t)(accY[k] + remap_weighted_px(Yp, w, h, p, 1, xy[2 * k], xy[2 * k + 1], a[k], fm[k]));
        orc_resize_half_f32(map1[i], W, H, hm1);
        orc_resize_half_f32(map2[i], W, H, hm2);
        orc_convert_maps(hm1, hm2, nh, (float)(w / 2), (float)(h / 2), xy, a);
        for (size_t k = 0; k < nh; k++) {
            /* split(UV.reshape(2)): c1c2[0] = U (even bytes), c1c2[1] = V; V -> output channel 0 */
            accV[k] = (uint16_t)(accV[k] + remap_weighted_px(UV + 1, w / 2, h / 2, p, 2, xy[2 * k], xy[2 * k + 1], a[k], hfm[k]));
            accU[k] = (uint16_t)(accU[k] + remap_weighted_px(UV, w / 2, h / 2, p, 2, xy[2 * k], xy[2 * k + 1], a[k], hfm[k]));
        }
    }
    /* convertTo(CV_8U, 1/255.) = convert_uchar_sat_rte(fma(v, (float)(1/255.), 0)) */
    const float alpha = (float)(1.0 / 255.0);
    for (int y = 0; y < H; y++)
        for (int x = 0; x < W; x++) out[(size_t)y * out_pitch + x] = sat_u8_rte(fmaf((float)accY[(size_t)y * W + x], alpha, 0.f));
    for (int y = 0; y < H / 2; y++)
        for (int x = 0; x < W / 2; x++) {
            uint8_t* o = out + (size_t)(H + y) * out_pitch + 2 * x;
            o[0] = sat_u8_rte(fmaf((float)accV[(size_t)y * (W / 2) + x], alpha, 0.f));
            o[1] = sat_u8_rte(fmaf((float)accU[(size_t)y * (W / 2) + x], alpha, 0.f));
        }
    for (int i = 0; i < n; i++) free(wt[i]);
    free(wt); free(total); free(accY); free(accV); free(accU); free(fm); free(hfm); free(xy); free(a); free(hm1); free(hm2);
    return 0;
}
