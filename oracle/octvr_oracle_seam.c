/*
 * octvr_oracle_seam.c — CPU restatement of the seam-mask builder.
 *
 * TEST INFRASTRUCTURE ONLY (see octvr_oracle.h).  Restates, from the reference sources:
 *   cv::resize INTER_LINEAR u8, CPU path     modules/imgproc/src/imgwarp.cpp:3120-3480 (coefficients),
 *                                            HResizeLinear :1391-1443, VResizeLinear<uchar,int,short> :1477-1500,
 *                                            2x2 area-fast path :2349-2400 (taken for exact 2x INTER_LINEAR, :3309-3312)
 *   cv::distanceTransform DIST_L2, mask 3    modules/imgproc/src/distransform.cpp:48-139 (distanceTransform_3x3),
 *                                            metrics {0.955, 1.3693} :402-420
 *   warpedDistanceTransform                  modules/stitching/src/seam_finders.cpp:86-95
 *   DistanceSeamFinder::find (max_n = 1)     modules/stitching/src/seam_finders.cpp:97-133
 *   MapperTemplate::create_masks             modules/octvr/src/template.cpp:155-204 (no images -> DistanceSeamFinder)
 * Pinned by tests/golden (rs_up / rs_down / dt_out KATs and every rig's seam masks).
 */
#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "octvr_oracle.h"

static int sat_s16_rne(float v) {
    int i = (int)lrintf(v);
    return i < -32768 ? -32768 : i > 32767 ? 32767 : i;
}

static int floor_f(float v) { /* cvFloor(float) */
    int i = (int)v;
    return i - (i > v);
}

void orc_resize_linear_u8(const uint8_t* src, int sw, int sh, size_t spitch, int cn, uint8_t* dst, int dw, int dh,
                          size_t dpitch) {
    if (dw == sw && dh == sh) { /* imgwarp.cpp:3264-3268: same size -> copy */
        for (int y = 0; y < dh; y++) memcpy(dst + (size_t)y * dpitch, src + (size_t)y * spitch, (size_t)dw * cn);
        return;
    }
    const double inv_x = (double)dw / sw, inv_y = (double)dh / sh;
    const double scale_x = 1. / inv_x, scale_y = 1. / inv_y;
    const int isx = (int)lrint(scale_x), isy = (int)lrint(scale_y);
    const int area_fast = fabs(scale_x - isx) < DBL_EPSILON && fabs(scale_y - isy) < DBL_EPSILON;
    if (area_fast && isx == 2 && isy == 2) { /* INTER_LINEAR at exactly 1/2 == INTER_AREA fast: (a+b+c+d+2)>>2 */
        for (int y = 0; y < dh; y++) {
            const uint8_t* s0 = src + (size_t)(2 * y) * spitch;
            const uint8_t* s1 = s0 + spitch;
            for (int x = 0; x < dw; x++)
                for (int c = 0; c < cn; c++) {
                    int i = 2 * x * cn + c;
                    dst[(size_t)y * dpitch + (size_t)x * cn + c] = (uint8_t)((s0[i] + s0[i + cn] + s1[i] + s1[i + cn] + 2) >> 2);
                }
        }
        return;
    }
    int* xofs = (int*)malloc(sizeof(int) * dw);
    short* ax = (short*)malloc(sizeof(short) * 2 * dw);
    int xmax = dw;
    for (int dx = 0; dx < dw; dx++) {
        float fx = (float)((dx + 0.5) * scale_x - 0.5);
        int sx = floor_f(fx);
        fx -= sx;
        if (sx < 0) fx = 0, sx = 0;
        if (sx + 1 >= sw) {
            if (dx < xmax) xmax = dx;
            if (sx >= sw - 1) fx = 0, sx = sw - 1;
        }
        xofs[dx] = sx;
        ax[2 * dx] = (short)sat_s16_rne((1.f - fx) * 2048);
        ax[2 * dx + 1] = (short)sat_s16_rne(fx * 2048);
    }
    int* h0 = (int*)malloc(sizeof(int) * dw * cn);
    int* h1 = (int*)malloc(sizeof(int) * dw * cn);
    for (int dy = 0; dy < dh; dy++) {
        float fy = (float)((dy + 0.5) * scale_y - 0.5);
        int sy = floor_f(fy);
        fy -= sy;
        const int b0 = sat_s16_rne((1.f - fy) * 2048), b1 = sat_s16_rne(fy * 2048);
        int rows[2];
        for (int k = 0; k < 2; k++) {
            int r = sy + k;
            rows[k] = r < 0 ? 0 : r >= sh ? sh - 1 : r; /* clip(sy, 0, ssize.height) */
        }
        int* hb[2] = {h0, h1};
        for (int k = 0; k < 2; k++) {
            const uint8_t* S = src + (size_t)rows[k] * spitch;
            for (int dx = 0; dx < dw; dx++)
                for (int c = 0; c < cn; c++) {
                    int sx = xofs[dx] * cn + c;
                    hb[k][dx * cn + c] = dx < xmax ? S[sx] * ax[2 * dx] + S[sx + cn] * ax[2 * dx + 1] : S[sx] * 2048;
                }
        }
        uint8_t* D = dst + (size_t)dy * dpitch;
        for (int i = 0; i < dw * cn; i++)
            D[i] = (uint8_t)((((b0 * (h0[i] >> 4)) >> 16) + ((b1 * (h1[i] >> 4)) >> 16) + 2) >> 2);
    }
    free(xofs); free(ax); free(h0); free(h1);
}

void orc_distance_transform_l2_3x3(const uint8_t* src, int w, int h, size_t spitch, float* dist, size_t dpitch_elems) {
    const int INIT = 0x7FFFFFFF >> 2;
    const int HV = (int)lrint(0.955f * 65536.0), DIAG = (int)lrint(1.3693f * 65536.0); /* CV_FLT_TO_FIX, float x int */
    const float scale = 1.f / 65536;
    const int tw = w + 2;
    int* t = (int*)malloc(sizeof(int) * (size_t)tw * (h + 2));
    for (int j = 0; j < tw; j++) t[j] = t[(size_t)(h + 1) * tw + j] = INIT;
    for (int i = 0; i < h; i++) {
        const uint8_t* s = src + (size_t)i * spitch;
        int* r = t + (size_t)(i + 1) * tw + 1;
        r[-1] = r[w] = INIT;
        for (int j = 0; j < w; j++) {
            if (!s[j]) { r[j] = 0; continue; }
            int t0 = r[j - tw - 1] + DIAG, v = r[j - tw] + HV;
            if (t0 > v) t0 = v;
            v = r[j - tw + 1] + DIAG;
            if (t0 > v) t0 = v;
            v = r[j - 1] + HV;
            if (t0 > v) t0 = v;
            r[j] = t0;
        }
    }
    for (int i = h - 1; i >= 0; i--) {
        int* r = t + (size_t)(i + 1) * tw + 1;
        float* d = dist + (size_t)i * dpitch_elems;
        for (int j = w - 1; j >= 0; j--) {
            int t0 = r[j];
            if (t0 > HV) {
                int v = r[j + tw + 1] + DIAG;
                if (t0 > v) t0 = v;
                v = r[j + tw] + HV;
                if (t0 > v) t0 = v;
                v = r[j + tw - 1] + DIAG;
                if (t0 > v) t0 = v;
                v = r[j + 1] + HV;
                if (t0 > v) t0 = v;
                r[j] = t0;
            }
            d[j] = (float)(t0 * scale);
        }
    }
    free(t);
}

int orc_create_masks(int n, const int* rois, const uint8_t* const* masks, int out_w, uint8_t* const* seams) {
    const double scale = fmin(1.0, 960.0 / out_w);
    int* sr = (int*)malloc(sizeof(int) * 4 * n);
    uint8_t** um = (uint8_t**)malloc(sizeof(void*) * n);
    float** dist = (float**)malloc(sizeof(void*) * n);
    int rx0 = 0, ry0 = 0, rx1 = 0, ry1 = 0;
    for (int i = 0; i < n; i++) {
        const int* r = rois + 4 * i;
        int* s = sr + 4 * i;
        s[0] = (int)(r[0] * scale);
        s[1] = (int)(r[1] * scale);
        s[2] = (int)(r[2] * scale);
        s[3] = (int)(r[3] * scale);
        um[i] = (uint8_t*)malloc((size_t)s[2] * s[3] + 1);
        orc_resize_linear_u8(masks[i], r[2], r[3], (size_t)r[2], 1, um[i], s[2], s[3], (size_t)s[2]);
        /* resultRoi (seam_finders.cpp:99): union of the scaled rectangles */
        if (i == 0 || s[0] < rx0) rx0 = s[0];
        if (i == 0 || s[1] < ry0) ry0 = s[1];
        if (i == 0 || s[0] + s[2] > rx1) rx1 = s[0] + s[2];
        if (i == 0 || s[1] + s[3] > ry1) ry1 = s[1] + s[3];
    }
    for (int i = 0; i < n; i++) {
        const int w = sr[4 * i + 2], h = sr[4 * i + 3];
        dist[i] = (float*)malloc(sizeof(float) * ((size_t)w * h + 1));
        if (sr[4 * i] == 0 && w == rx1 - rx0) { /* warpedDistanceTransform: 3 copies side by side, keep the middle */
            uint8_t* w3 = (uint8_t*)malloc((size_t)3 * w * h);
            float* d3 = (float*)malloc(sizeof(float) * (size_t)3 * w * h);
            for (int y = 0; y < h; y++)
                for (int k = 0; k < 3; k++) memcpy(w3 + (size_t)y * 3 * w + (size_t)k * w, um[i] + (size_t)y * w, w);
            orc_distance_transform_l2_3x3(w3, 3 * w, h, (size_t)3 * w, d3, (size_t)3 * w);
            for (int y = 0; y < h; y++) memcpy(dist[i] + (size_t)y * w, d3 + (size_t)y * 3 * w + w, sizeof(float) * w);
            free(w3);
            free(d3);
        } else {
            orc_distance_transform_l2_3x3(um[i], w, h, (size_t)w, dist[i], (size_t)w);
        }
    }
    /* per pixel: keep only the camera with the largest distance; std::sort of <= 16 entries is an
     * insertion sort (stable), so ties go to the lowest camera index */
    for (int y = ry0; y < ry1; y++)
        for (int x = rx0; x < rx1; x++) {
            int best = -1;
            float bd = 0.f;
            for (int i = 0; i < n; i++) {
                const int* s = sr + 4 * i;
                float d = -1.f;
                if (y >= s[1] && x >= s[0] && y - s[1] < s[3] && x - s[0] < s[2])
                    d = dist[i][(size_t)(y - s[1]) * s[2] + (x - s[0])];
                if (best < 0 || d > bd) best = i, bd = d;
            }
            for (int i = 0; i < n; i++) {
                const int* s = sr + 4 * i;
                if (i == best) continue;
                if (!(y >= s[1] && x >= s[0] && y - s[1] < s[3] && x - s[0] < s[2])) continue; /* distance -1 */
                um[i][(size_t)(y - s[1]) * s[2] + (x - s[0])] = 0;
            }
        }
    for (int i = 0; i < n; i++) {
        const int* r = rois + 4 * i;
        orc_resize_linear_u8(um[i], sr[4 * i + 2], sr[4 * i + 3], (size_t)sr[4 * i + 2], 1, seams[i], r[2], r[3], (size_t)r[2]);
        free(um[i]);
        free(dist[i]);
    }
    free(sr); free(um); free(dist);
    return 0;
}
