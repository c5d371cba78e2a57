/*
 * octvr_oracle_blend.c — CPU restatement of the GPU blenders of Mapper::stitch.
 *
 * TEST INFRASTRUCTURE ONLY (see octvr_oracle.h).  Restated from the reference CUDA sources (no CUDA
 * device exists here, so these rows are pinned by restatement + known-answer tests, not fixtures):
 *   MultiBandGPUBlender ctor / do_blend        modules/stitching/src/blenders.cpp:589-735
 *   GPUStaticBlender (result ROI, checks)      modules/stitching/src/blenders.cpp:479-506
 *   fastPyrDown<uchar4> (K2, clamp texture)    modules/cudawarping/src/cuda/fast_pyr_down.cu:17-76
 *   pyrUp<T> (K3, abs + clamp border)          modules/cudawarping/src/cuda/pyr_up.cu:55-166
 *   pyrDown<float, BrdReflect101> (K4)         modules/cudawarping/src/cuda/pyr_down.cu:55-192
 *   vr_add_sub_and_multiply / vr_add_multiply  modules/stitching/src/cuda/blender.cu:15-98 (K5, K6)
 *   DivOpSpecial<short3> (K11)                 modules/cudaarithm/src/cuda/div_mat.cu:232-249
 *   GpuMat::convertTo u8 -> f32 (alpha 1/255)   modules/core/src/cuda/gpu_mat.cu:458-480
 *   FeatherGPUBlender ctor / do_blend          modules/stitching/src/blenders.cpp:531-586
 *
 * Arithmetic notes (why the integer forms below are exact restatements):
 *  - fastPyrDown on u8 and pyrUp on u8 / s16 sum products of small integers with the weights
 *    1/16, 1/4, 3/8 in f32; every partial sum is a multiple of 2^-8 below 2^16 (u8) or 2^23 (s16),
 *    so f32 (with or without nvcc's FMA contraction) is exact and the result is
 *    saturate(round_half_even(S / 256)) resp. saturate(round_half_even(S / 64)) of an integer S.
 *  - pyrUp's vertical pass reads the 6 rows of its s_dstPatch with a block-of-8 quirk: patch row 5 is
 *    filled from source row by/2 + 5 instead of by/2 + 4 (pyr_up.cu:104-118), so output rows
 *    y = 6, 7 (mod 8) take their last tap one source row further down.  Restated literally.
 *  - pyrDown on f32 (weights, build time only): nvcc contracts `sum + w * v` into fmaf (default
 *    -fmad=true); restated with fmaf.  Parity for this step is "unpinned" (no CUDA fixture).
 */
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "octvr_oracle.h"

/* ---- small parallel-for over rows ---------------------------------------------------------- */
typedef void (*band_fn)(void* ctx, int y0, int y1);
typedef struct { band_fn fn; void* ctx; int y0, y1; } band_job;
static void* band_worker(void* a) { band_job* j = (band_job*)a; j->fn(j->ctx, j->y0, j->y1); return NULL; }
static void par_rows(int T, int rows, band_fn fn, void* ctx) {
    if (rows <= 0) return;
    if (T > 64) T = 64;
    if (T > rows) T = rows;
    if (T <= 1) { fn(ctx, 0, rows); return; }
    pthread_t th[64];
    band_job jb[64];
    for (int t = 0; t < T; t++) {
        jb[t].fn = fn; jb[t].ctx = ctx;
        jb[t].y0 = (int)((long)rows * t / T);
        jb[t].y1 = (int)((long)rows * (t + 1) / T);
        pthread_create(&th[t], NULL, band_worker, &jb[t]);
    }
    for (int t = 0; t < T; t++) pthread_join(th[t], NULL);
}

static inline int clampi(int v, int lo, int hi) { return v < lo ? lo : v > hi ? hi : v; }
static inline int iabs(int v) { return v < 0 ? -v : v; }

/* round_half_even(S / 2^sh) for an integer S (any sign) */
static inline int rne_shift(int S, int sh) {
    int q = S >> sh;  /* floor */
    int r = S - (q << sh);
    int half = 1 << (sh - 1);
    if (r > half || (r == half && (q & 1))) q++;
    return q;
}

/* ---- K2 fastPyrDown<uchar4>: 5x5 [1 4 6 4 1]^2 / 256, clamp border, RGB channels (alpha unused) */
typedef struct { const uint8_t* s; int sw, sh; uint8_t* d; int dw; } pd_ctx;
static void pyr_down_u8x4_rows(void* c, int y0, int y1) {
    const pd_ctx* p = (const pd_ctx*)c;
    static const int w[5] = {1, 4, 6, 4, 1};
    for (int y = y0; y < y1; y++)
        for (int x = 0; x < p->dw; x++)
            for (int ch = 0; ch < 3; ch++) {
                int S = 0;
                for (int j = 0; j < 5; j++) {
                    const uint8_t* row = p->s + (size_t)clampi(2 * y + j - 2, 0, p->sh - 1) * p->sw * 4;
                    int h = 0;
                    for (int k = 0; k < 5; k++) h += w[k] * row[(size_t)clampi(2 * x + k - 2, 0, p->sw - 1) * 4 + ch];
                    S += w[j] * h;
                }
                int v = rne_shift(S, 8);
                p->d[((size_t)y * p->dw + x) * 4 + ch] = (uint8_t)clampi(v, 0, 255);
            }
}
void orc_fast_pyr_down_u8x4(const uint8_t* src, int sw, int sh, uint8_t* dst, int threads) {
    pd_ctx c = {src, sw, sh, dst, (sw + 1) / 2};
    par_rows(threads, (sh + 1) / 2, pyr_down_u8x4_rows, &c);
}

/* ---- K3 pyrUp (u8x4 or s16x3): dst = 2x src; horizontal taps floor((x+k)/2) with
 * min(cols-1, |.|); vertical rows through the 8-row block patch (see header note). */
static inline int up_row(int y, int t_sel, int rows) {
    /* source row of s_dstPatch entry t_sel (0..5) for the 8-row block containing y */
    int by2 = (y & ~7) >> 1;
    int r = t_sel < 5 ? by2 - 1 + t_sel : by2 + 5;
    r = iabs(r);
    return r < rows - 1 ? r : rows - 1;
}
typedef struct { const void* s; int sw, sh, cn_s, cn_d, is16; void* d; int dw; } pu_ctx;
static void pyr_up_rows(void* c, int y0, int y1) {
    const pu_ctx* p = (const pu_ctx*)c;
    for (int y = y0; y < y1; y++) {
        const int t = y & 7;
        int rows[2][3], nr, vw[3];
        if (!(t & 1)) {
            nr = 3; vw[0] = 1; vw[1] = 6; vw[2] = 1;
            for (int j = 0; j < 3; j++) rows[0][j] = up_row(y, (t >> 1) + j, p->sh);
        } else {
            nr = 2; vw[0] = 4; vw[1] = 4;
            rows[0][0] = up_row(y, ((t - 1) >> 1) + 1, p->sh);
            rows[0][1] = up_row(y, ((t + 1) >> 1) + 1, p->sh);
        }
        for (int x = 0; x < p->dw; x++) {
            int cols[3], nc, hw[3];
            if (!(x & 1)) {
                nc = 3; hw[0] = 1; hw[1] = 6; hw[2] = 1;
                for (int k = 0; k < 3; k++) {
                    int v = iabs((x >> 1) - 1 + k);
                    cols[k] = v < p->sw - 1 ? v : p->sw - 1;
                }
            } else {
                nc = 2; hw[0] = 4; hw[1] = 4;
                for (int k = 0; k < 2; k++) {
                    int v = ((x - 1) >> 1) + k;
                    cols[k] = v < p->sw - 1 ? v : p->sw - 1;
                }
            }
            for (int ch = 0; ch < 3; ch++) {
                int S = 0;
                for (int j = 0; j < nr; j++) {
                    int h = 0;
                    for (int k = 0; k < nc; k++) {
                        size_t o = ((size_t)rows[0][j] * p->sw + cols[k]) * p->cn_s + ch;
                        int v = p->is16 ? ((const int16_t*)p->s)[o] : ((const uint8_t*)p->s)[o];
                        h += hw[k] * v;
                    }
                    S += vw[j] * h;
                }
                int v = rne_shift(S, 6);
                size_t o = ((size_t)y * p->dw + x) * p->cn_d + ch;
                if (p->is16) ((int16_t*)p->d)[o] = (int16_t)clampi(v, -32768, 32767);
                else ((uint8_t*)p->d)[o] = (uint8_t)clampi(v, 0, 255);
            }
        }
    }
}
void orc_pyr_up_u8x4(const uint8_t* src, int sw, int sh, uint8_t* dst, int threads) {
    pu_ctx c = {src, sw, sh, 4, 4, 0, dst, 2 * sw};
    par_rows(threads, 2 * sh, pyr_up_rows, &c);
}
void orc_pyr_up_s16x3(const int16_t* src, int sw, int sh, int16_t* dst, int threads) {
    pu_ctx c = {src, sw, sh, 3, 3, 1, dst, 2 * sw};
    par_rows(threads, 2 * sh, pyr_up_rows, &c);
}

/* ---- K4 pyrDown<float, BrdReflect101> with nvcc's FMA contraction ----------------------------- */
static inline int refl101(int v, int last) {
    /* BrdReflect101 idx_*_low(idx_*_high(v)) (border_interpolate.hpp:351-386) */
    v = iabs(last - iabs(last - v)) % (last + 1);
    return iabs(v) % (last + 1);
}
static inline float sum5(float a, float b, float c, float d, float e) {
    float s = 0.0625f * a;
    s = fmaf(0.25f, b, s);
    s = fmaf(0.375f, c, s);
    s = fmaf(0.25f, d, s);
    return fmaf(0.0625f, e, s);
}
typedef struct { const float* s; int sw, sh; float* d; int dw; } pf_ctx;
static void pyr_down_f32_rows(void* c, int y0, int y1) {
    const pf_ctx* p = (const pf_ctx*)c;
    float* col = (float*)malloc(sizeof(float) * (p->sw + 4));
    for (int y = y0; y < y1; y++) {
        const int sy = 2 * y;
        const float* r[5];
        for (int j = 0; j < 5; j++) r[j] = p->s + (size_t)refl101(sy + j - 2, p->sh - 1) * p->sw;
        for (int x = -2; x < p->sw + 2; x++) {
            int cx = refl101(x, p->sw - 1);
            col[x + 2] = sum5(r[0][cx], r[1][cx], r[2][cx], r[3][cx], r[4][cx]);
        }
        for (int x = 0; x < p->dw; x++) {
            const float* v = col + 2 * x;  /* columns 2x-2 .. 2x+2 */
            p->d[(size_t)y * p->dw + x] = sum5(v[0], v[1], v[2], v[3], v[4]);
        }
    }
    free(col);
}
void orc_pyr_down_f32(const float* src, int sw, int sh, float* dst, int threads) {
    pf_ctx c = {src, sw, sh, dst, (sw + 1) / 2};
    par_rows(threads, (sh + 1) / 2, pyr_down_f32_rows, &c);
}

/* ---- MultiBandGPUBlender -------------------------------------------------------------------- */
typedef struct { int x, y, w, h; } rect;

static int round_down(int x, int b) { return (x >> b) << b; }
static int round_up(int x, int b) { int m = 1 << b; return x + (m - (x % m)) % m; }

typedef struct {
    int n, B, T;
    rect arr;           /* align_result_roi */
    rect* ar;           /* align_rois */
    const int* rois;
    float** w;          /* [n * (B+1)] weight pyramids (over align_rois >> level) */
    float** bw;         /* [B+1] dst_band_weights (over arr >> level) */
    uint8_t** g;        /* [n * (B+1)] src_pyr_laplaces (u8x4) */
    uint8_t** up;       /* [n * B] tmps = pyrUp(g[n][i+1]) */
    int16_t** lap;      /* [B+1] dst_pyr_laplace (s16x3) */
    int level, cam;
} mb_ctx;

static void mb_accum_rows(void* c, int y0, int y1) {
    /* vr_add_sub_and_multiply / vr_add_multiply of camera `cam` at `level` into lap[level](scale_roi) */
    const mb_ctx* m = (const mb_ctx*)c;
    const int i = m->level, n = m->cam, B = m->B;
    const rect a = m->ar[n];
    const int ox = (a.x - m->arr.x) >> i, oy = (a.y - m->arr.y) >> i, cw = a.w >> i;
    const int LW = m->arr.w >> i;
    const uint8_t* A = m->g[n * (B + 1) + i];
    const uint8_t* Tm = i < B ? m->up[n * B + i] : NULL;
    const float* W = m->w[n * (B + 1) + i];
    int16_t* D = m->lap[i];
    for (int y = y0; y < y1; y++)
        for (int x = 0; x < cw; x++) {
            const size_t k = (size_t)y * cw + x;
            const float we = W[k];
            if (we == 0) continue;
            int16_t* d = D + ((size_t)(oy + y) * LW + ox + x) * 3;
            for (int ch = 0; ch < 3; ch++) {
                int diff = Tm ? (int)A[4 * k + ch] - (int)Tm[4 * k + ch] : (int)A[4 * k + ch];
                float prod = (float)diff * we;
                int16_t sub = (int16_t)(int)truncf(prod);       /* float -> short: truncation */
                d[ch] = (int16_t)(d[ch] + sub);                  /* short += short: wraps */
            }
        }
}

static void mb_divide_rows(void* c, int y0, int y1) {
    /* DivOpSpecial<short3>: b != 0 ? sat_s16(a * (1.0f / b)) : 0 */
    const mb_ctx* m = (const mb_ctx*)c;
    const int i = m->level, LW = m->arr.w >> i;
    for (int y = y0; y < y1; y++)
        for (int x = 0; x < LW; x++) {
            const size_t k = (size_t)y * LW + x;
            float b = m->bw[i][k];
            int16_t* d = m->lap[i] + 3 * k;
            if (b != 0) {
                b = 1.0f / b;
                for (int ch = 0; ch < 3; ch++) d[ch] = (int16_t)clampi((int)lrintf((float)d[ch] * b), -32768, 32767);
            } else {
                d[0] = d[1] = d[2] = 0;
            }
        }
}

int orc_multiband_blend(int n, const int* rois, const uint8_t* const* seams, const uint8_t* const* warped, int bands,
                        uint8_t* result, int out_w, int out_h, size_t result_pitch, int threads) {
    const int B = bands;
    const int T = threads > 0 ? threads : 1;
    if (n < 1 || B < 1) return -1;
    /* result_roi = union of rois (GPUStaticBlender ctor, blenders.cpp:484-486) */
    int x0 = rois[0], y0 = rois[1], x1 = rois[0] + rois[2], y1 = rois[1] + rois[3];
    for (int i = 1; i < n; i++) {
        const int* r = rois + 4 * i;
        if (r[0] < x0) x0 = r[0];
        if (r[1] < y0) y0 = r[1];
        if (r[0] + r[2] > x1) x1 = r[0] + r[2];
        if (r[1] + r[3] > y1) y1 = r[1] + r[3];
    }
    mb_ctx m;
    memset(&m, 0, sizeof m);
    m.n = n; m.B = B; m.T = T; m.rois = rois;
    m.arr.x = round_down(x0, B); m.arr.y = round_down(y0, B);
    m.arr.w = round_up(x1, B) - m.arr.x; m.arr.h = round_up(y1, B) - m.arr.y;
    m.ar = (rect*)calloc(n, sizeof(rect));
    const int gap = 5 * (1 << B);
    for (int i = 0; i < n; i++) {
        const int* r = rois + 4 * i;
        int l = round_down(r[0], B) - gap, t = round_down(r[1], B) - gap;
        int rr = round_up(r[0] + r[2], B) + gap, bb = round_up(r[1] + r[3], B) + gap;
        if (l < m.arr.x) l = m.arr.x;
        if (t < m.arr.y) t = m.arr.y;
        if (rr > m.arr.x + m.arr.w) rr = m.arr.x + m.arr.w;
        if (bb > m.arr.y + m.arr.h) bb = m.arr.y + m.arr.h;
        m.ar[i].x = l; m.ar[i].y = t; m.ar[i].w = rr - l; m.ar[i].h = bb - t;
        if ((m.ar[i].w >> B) <= 0 || (m.ar[i].h >> B) <= 0) { free(m.ar); return -2; }
    }
    m.w = (float**)calloc((size_t)n * (B + 1), sizeof(void*));
    m.bw = (float**)calloc(B + 1, sizeof(void*));
    m.g = (uint8_t**)calloc((size_t)n * (B + 1), sizeof(void*));
    m.up = (uint8_t**)calloc((size_t)n * B, sizeof(void*));
    m.lap = (int16_t**)calloc(B + 1, sizeof(void*));
    for (int i = 0; i <= B; i++) {
        size_t k = (size_t)(m.arr.w >> i) * (m.arr.h >> i);
        m.bw[i] = (float*)malloc(sizeof(float) * k);
        for (size_t q = 0; q < k; q++) m.bw[i][q] = 1e-5f;
        m.lap[i] = (int16_t*)calloc(3 * k, sizeof(int16_t));
    }
    const float inv255 = (float)(1. / 255);
    for (int c = 0; c < n; c++) {
        const rect a = m.ar[c];
        const int* r = rois + 4 * c;
        float* w0 = (float*)calloc((size_t)a.w * a.h, sizeof(float));
        uint8_t* g0 = (uint8_t*)calloc((size_t)a.w * a.h * 4, 1);
        for (int y = 0; y < r[3]; y++)
            for (int x = 0; x < r[2]; x++) {
                size_t d = (size_t)(r[1] - a.y + y) * a.w + (r[0] - a.x + x);
                w0[d] = inv255 * (float)seams[c][(size_t)y * r[2] + x] + 0.0f;
                memcpy(g0 + 4 * d, warped[c] + 4 * ((size_t)y * r[2] + x), 4);
            }
        m.w[c * (B + 1)] = w0;
        m.g[c * (B + 1)] = g0;
        for (int i = 0; i < B; i++) {
            int sw = a.w >> i, sh = a.h >> i;
            m.w[c * (B + 1) + i + 1] = (float*)malloc(sizeof(float) * (size_t)(sw / 2) * (sh / 2));
            orc_pyr_down_f32(m.w[c * (B + 1) + i], sw, sh, m.w[c * (B + 1) + i + 1], T);
            m.g[c * (B + 1) + i + 1] = (uint8_t*)malloc((size_t)(sw / 2) * (sh / 2) * 4);
            orc_fast_pyr_down_u8x4(m.g[c * (B + 1) + i], sw, sh, m.g[c * (B + 1) + i + 1], T);
        }
        for (int i = 0; i < B; i++) {
            int sw = a.w >> (i + 1), sh = a.h >> (i + 1);
            m.up[c * B + i] = (uint8_t*)malloc((size_t)(2 * sw) * (2 * sh) * 4);
            orc_pyr_up_u8x4(m.g[c * (B + 1) + i + 1], sw, sh, m.up[c * B + i], T);
        }
        for (int i = 0; i <= B; i++) { /* dst_band_weights[i](scale_roi) += weight pyramid */
            const int ox = (a.x - m.arr.x) >> i, oy = (a.y - m.arr.y) >> i, cw = a.w >> i, ch = a.h >> i;
            const int LW = m.arr.w >> i;
            const float* wl = m.w[c * (B + 1) + i];
            for (int y = 0; y < ch; y++)
                for (int x = 0; x < cw; x++) m.bw[i][(size_t)(oy + y) * LW + ox + x] += wl[(size_t)y * cw + x];
        }
    }
    for (int i = 0; i <= B; i++) {
        m.level = i;
        for (int c = 0; c < n; c++) {
            m.cam = c;
            par_rows(T, m.ar[c].h >> i, mb_accum_rows, &m);
        }
        par_rows(T, m.arr.h >> i, mb_divide_rows, &m);
    }
    for (int i = B; i > 0; i--) { /* collapse: lap[i-1] = sat_s16(pyrUp(lap[i]) + lap[i-1]) */
        const int sw = m.arr.w >> i, sh = m.arr.h >> i;
        size_t k = (size_t)(2 * sw) * (2 * sh) * 3;
        int16_t* up = (int16_t*)malloc(sizeof(int16_t) * k);
        orc_pyr_up_s16x3(m.lap[i], sw, sh, up, T);
        for (size_t q = 0; q < k; q++) m.lap[i - 1][q] = (int16_t)clampi(up[q] + m.lap[i - 1][q], -32768, 32767);
        free(up);
    }
    {
        const int cw = m.arr.w < out_w ? m.arr.w : out_w, ch = m.arr.h < out_h ? m.arr.h : out_h;
        for (int y = 0; y < ch; y++)
            for (int x = 0; x < cw; x++) {
                if (m.arr.y + y >= out_h || m.arr.x + x >= out_w) continue;
                uint8_t* o = result + (size_t)(m.arr.y + y) * result_pitch + (size_t)(m.arr.x + x) * 3;
                const int16_t* s = m.lap[0] + ((size_t)y * m.arr.w + x) * 3;
                for (int q = 0; q < 3; q++) o[q] = (uint8_t)clampi(s[q], 0, 255);
            }
    }
    for (int i = 0; i < n * (B + 1); i++) { free(m.w[i]); free(m.g[i]); }
    for (int i = 0; i < n * B; i++) free(m.up[i]);
    for (int i = 0; i <= B; i++) { free(m.bw[i]); free(m.lap[i]); }
    free(m.w); free(m.g); free(m.up); free(m.bw); free(m.lap); free(m.ar);
    return 0;
}

/* ---- FeatherGPUBlender (blenders.cpp:531-586) ------------------------------------------------- */
/* ctor: w_i = threshold_tozero(distanceTransform(mask_i, L2, 3) - border), W = 1e-5f + sum_i w_i
 * over the result ROI (camera order), w_i = N * w_i / W (DivScaleOp, div_mat.cu:82-91);
 * do_blend: D = sum_i (short)(A_i * w_i) where w_i != 0 (K6, short wrap), result(result_roi) =
 * saturate_cast<uchar>((float)(1.0 / N) * D) (convertTo with alpha). */
int orc_feather_blend(int n, const int* rois, const uint8_t* const* masks, const uint8_t* const* warped, int border,
                      uint8_t* result, int out_w, int out_h, size_t result_pitch) {
    int x0 = rois[0], y0 = rois[1], x1 = rois[0] + rois[2], y1 = rois[1] + rois[3];
    for (int i = 1; i < n; i++) {
        const int* r = rois + 4 * i;
        if (r[0] < x0) x0 = r[0];
        if (r[1] < y0) y0 = r[1];
        if (r[0] + r[2] > x1) x1 = r[0] + r[2];
        if (r[1] + r[3] > y1) y1 = r[1] + r[3];
    }
    const int RW = x1 - x0, RH = y1 - y0;
    float* W = (float*)malloc(sizeof(float) * (size_t)RW * RH);
    for (size_t k = 0; k < (size_t)RW * RH; k++) W[k] = 1e-5f;
    float** w = (float**)calloc(n, sizeof(void*));
    for (int i = 0; i < n; i++) {
        const int* r = rois + 4 * i;
        w[i] = (float*)malloc(sizeof(float) * (size_t)r[2] * r[3]);
        orc_distance_transform_l2_3x3(masks[i], r[2], r[3], (size_t)r[2], w[i], (size_t)r[2]);
        for (size_t k = 0; k < (size_t)r[2] * r[3]; k++) {
            float v = w[i][k] - (float)border;
            w[i][k] = v > 0.f ? v : 0.f;
        }
        for (int y = 0; y < r[3]; y++)
            for (int x = 0; x < r[2]; x++) {
                float* d = &W[(size_t)(r[1] - y0 + y) * RW + (r[0] - x0 + x)];
                *d = w[i][(size_t)y * r[2] + x] + *d;
            }
    }
    const float sc = (float)n;
    for (int i = 0; i < n; i++) {
        const int* r = rois + 4 * i;
        for (int y = 0; y < r[3]; y++)
            for (int x = 0; x < r[2]; x++) {
                float* a = &w[i][(size_t)y * r[2] + x];
                float b = W[(size_t)(r[1] - y0 + y) * RW + (r[0] - x0 + x)];
                *a = b != 0 ? (n == 1 ? *a / b : sc * *a / b) : 0.f;
            }
    }
    int16_t* D = (int16_t*)calloc((size_t)RW * RH * 3, sizeof(int16_t));
    for (int i = 0; i < n; i++) {
        const int* r = rois + 4 * i;
        for (int y = 0; y < r[3]; y++)
            for (int x = 0; x < r[2]; x++) {
                const size_t k = (size_t)y * r[2] + x;
                const float we = w[i][k];
                if (we == 0) continue;
                int16_t* d = D + ((size_t)(r[1] - y0 + y) * RW + (r[0] - x0 + x)) * 3;
                for (int ch = 0; ch < 3; ch++) {
                    int16_t sub = (int16_t)(int)truncf((float)warped[i][4 * k + ch] * we);
                    d[ch] = (int16_t)(d[ch] + sub);
                }
            }
    }
    const float alpha = (float)(1.0 / n);
    for (int y = 0; y < RH; y++)
        for (int x = 0; x < RW; x++) {
            if (y0 + y >= out_h || x0 + x >= out_w) continue;
            uint8_t* o = result + (size_t)(y0 + y) * result_pitch + (size_t)(x0 + x) * 3;
            const int16_t* s = D + ((size_t)y * RW + x) * 3;
            for (int q = 0; q < 3; q++) o[q] = (uint8_t)clampi((int)lrintf(alpha * (float)s[q]), 0, 255);
        }
    for (int i = 0; i < n; i++) free(w[i]);
    free(w); free(W); free(D);
    return 0;
}
