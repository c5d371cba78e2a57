/* octvr_oracle_masks.c — TEST INFRASTRUCTURE ONLY (the checker, never shipped or measured).
 * Restatement of cv::fillPoly as vr::Camera uses it for `selection`, `exclude_masks` and
 * `include_masks` polygons (modules/octvr/src/camera.cpp:96-112, 146-163): lineType 8, shift 0, no
 * offset.  Follows modules/imgproc/src/drawing.cpp: fillPoly :1894-1917, CollectPolyEdges
 * :1196-1248, FillEdgeCollection :1262-1405 (pointer-linked active edge list), Line :239-265 with
 * LineIterator :153-236 (+ operator++ in imgproc.hpp) and clipLine :80-137. */
#include <limits.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "octvr_oracle.h"

#define XY_SHIFT 16
#define XY_ONE (1 << XY_SHIFT)

static int clip_line(int w, int h, int* p1x, int* p1y, int* p2x, int* p2y) {
    int64_t x1 = *p1x, y1 = *p1y, x2 = *p2x, y2 = *p2y, right = w - 1, bottom = h - 1;
    int c1, c2;
    if (w <= 0 || h <= 0) return 0;
    c1 = (x1 < 0) + (x1 > right) * 2 + (y1 < 0) * 4 + (y1 > bottom) * 8;
    c2 = (x2 < 0) + (x2 > right) * 2 + (y2 < 0) * 4 + (y2 > bottom) * 8;
    if ((c1 & c2) == 0 && (c1 | c2) != 0) {
        int64_t a;
        if (c1 & 12) { a = c1 < 8 ? 0 : bottom; x1 += (a - y1) * (x2 - x1) / (y2 - y1); y1 = a; c1 = (x1 < 0) + (x1 > right) * 2; }
        if (c2 & 12) { a = c2 < 8 ? 0 : bottom; x2 += (a - y2) * (x2 - x1) / (y2 - y1); y2 = a; c2 = (x2 < 0) + (x2 > right) * 2; }
        if ((c1 & c2) == 0 && (c1 | c2) != 0) {
            if (c1) { a = c1 == 1 ? 0 : right; y1 += (a - x1) * (y2 - y1) / (x2 - x1); x1 = a; c1 = 0; }
            if (c2) { a = c2 == 1 ? 0 : right; y2 += (a - x2) * (y2 - y1) / (x2 - x1); x2 = a; c2 = 0; }
        }
        *p1x = (int)x1; *p1y = (int)y1; *p2x = (int)x2; *p2y = (int)y2;
    }
    return (c1 | c2) == 0;
}

/* LineIterator(img, pt1, pt2, 8, left_to_right=true) walking byte offsets, as the reference does */
static void line8(uint8_t* img, int w, int h, int p1x, int p1y, int p2x, int p2y, uint8_t color) {
    if ((unsigned)p1x >= (unsigned)w || (unsigned)p2x >= (unsigned)w || (unsigned)p1y >= (unsigned)h ||
        (unsigned)p2y >= (unsigned)h)
        if (!clip_line(w, h, &p1x, &p1y, &p2x, &p2y)) return;
    int bt_pix = 1, istep = w;
    int dx = p2x - p1x, dy = p2y - p1y;
    int s = dx < 0 ? -1 : 0;
    dx = (dx ^ s) - s;
    dy = (dy ^ s) - s;
    p1x ^= (p1x ^ p2x) & s;
    p1y ^= (p1y ^ p2y) & s;
    ptrdiff_t off = (ptrdiff_t)p1y * w + p1x;
    s = dy < 0 ? -1 : 0;
    dy = (dy ^ s) - s;
    istep = (istep ^ s) - s;
    s = dy > dx ? -1 : 0;
    dx ^= dy & s; dy ^= dx & s; dx ^= dy & s;
    bt_pix ^= istep & s; istep ^= bt_pix & s; bt_pix ^= istep & s;
    int err = dx - (dy + dy), plusDelta = dx + dx, minusDelta = -(dy + dy);
    int plusStep = istep, minusStep = bt_pix, count = dx + 1;
    for (int i = 0; i < count; i++) {
        img[off] = color;
        int mask = err < 0 ? -1 : 0;
        err += minusDelta + (plusDelta & mask);
        off += minusStep + (plusStep & mask);
    }
}

typedef struct PolyEdge {
    int y0, y1, x, dx;
    struct PolyEdge* next;
} PolyEdge;

static int cmp_edges(const void* pa, const void* pb) {
    const PolyEdge *e1 = (const PolyEdge*)pa, *e2 = (const PolyEdge*)pb;
    if (e1->y0 != e2->y0) return e1->y0 < e2->y0 ? -1 : 1;
    if (e1->x != e2->x) return e1->x < e2->x ? -1 : 1;
    if (e1->dx != e2->dx) return e1->dx < e2->dx ? -1 : 1;
    return 0;
}

void orc_fill_poly(uint8_t* img, int w, int h, const int* pts, int count, uint8_t color) {
    if (count <= 0) return;
    PolyEdge* edges = (PolyEdge*)calloc((size_t)count + 1, sizeof(PolyEdge));
    int total = 0;
    int pt0x = pts[2 * (count - 1)] << XY_SHIFT, pt0y = pts[2 * (count - 1) + 1];
    for (int i = 0; i < count; i++) {
        int pt1x = pts[2 * i] << XY_SHIFT, pt1y = pts[2 * i + 1];
        line8(img, w, h, (pt0x + (XY_ONE >> 1)) >> XY_SHIFT, pt0y, (pt1x + (XY_ONE >> 1)) >> XY_SHIFT, pt1y, color);
        if (pt0y != pt1y) {
            PolyEdge* e = &edges[total++];
            if (pt0y < pt1y) { e->y0 = pt0y; e->y1 = pt1y; e->x = pt0x; }
            else { e->y0 = pt1y; e->y1 = pt0y; e->x = pt1x; }
            e->dx = (pt1x - pt0x) / (pt1y - pt0y);
        }
        pt0x = pt1x; pt0y = pt1y;
    }
    /* FillEdgeCollection */
    PolyEdge tmp;
    int y_max = INT_MIN, x_max = INT_MIN, y_min = INT_MAX, x_min = INT_MAX;
    if (total < 2) { free(edges); return; }
    for (int i = 0; i < total; i++) {
        PolyEdge* e1 = &edges[i];
        int x1 = e1->x + (e1->y1 - e1->y0) * e1->dx;
        if (e1->y0 < y_min) y_min = e1->y0;
        if (e1->y1 > y_max) y_max = e1->y1;
        if (e1->x < x_min) x_min = e1->x;
        if (e1->x > x_max) x_max = e1->x;
        if (x1 < x_min) x_min = x1;
        if (x1 > x_max) x_max = x1;
    }
    if (y_max < 0 || y_min >= h || x_max < 0 || x_min >= (w << XY_SHIFT)) { free(edges); return; }
    qsort(edges, (size_t)total, sizeof(PolyEdge), cmp_edges);
    edges[total].y0 = INT_MAX; /* sentinel */
    int i = 0;
    tmp.next = 0;
    PolyEdge* e = &edges[i];
    if (y_max > h) y_max = h;
    for (int y = e->y0; y < y_max; y++) {
        PolyEdge *last, *prelast, *keep_prelast;
        int sort_flag = 0, draw = 0, clipline = y < 0;
        prelast = &tmp;
        last = tmp.next;
        while (last || e->y0 == y) {
            if (last && last->y1 == y) {
                prelast->next = last->next;
                last = last->next;
                continue;
            }
            keep_prelast = prelast;
            if (last && (e->y0 > y || last->x < e->x)) {
                prelast = last;
                last = last->next;
            } else if (i < total) {
                prelast->next = e;
                e->next = last;
                prelast = e;
                e = &edges[++i];
            } else
                break;
            if (draw) {
                if (!clipline) {
                    int x1 = keep_prelast->x, x2 = prelast->x;
                    if (x1 > x2) { int t = x1; x1 = x2; x2 = t; }
                    x1 = (x1 + XY_ONE - 1) >> XY_SHIFT;
                    x2 = x2 >> XY_SHIFT;
                    if (x1 < w && x2 >= 0) {
                        if (x1 < 0) x1 = 0;
                        if (x2 >= w) x2 = w - 1;
                        for (int x = x1; x <= x2; x++) img[(size_t)y * w + x] = color;
                    }
                }
                keep_prelast->x += keep_prelast->dx;
                prelast->x += prelast->dx;
            }
            draw ^= 1;
        }
        keep_prelast = 0;
        do {
            prelast = &tmp;
            last = tmp.next;
            while (last != keep_prelast && last->next != 0) {
                PolyEdge* te = last->next;
                if (last->x > te->x) {
                    prelast->next = te;
                    last->next = te->next;
                    te->next = last;
                    prelast = te;
                    sort_flag = 1;
                } else {
                    prelast = last;
                    last = te;
                }
            }
            keep_prelast = prelast;
        } while (sort_flag && keep_prelast != tmp.next && keep_prelast != &tmp);
    }
    free(edges);
}
