/*
 * octvr_oracle_morph.c — MapperTemplate::morph_controlpoints (modules/octvr/src/template_morph.cpp:69-237).
 *
 * TEST INFRASTRUCTURE ONLY (see octvr_oracle.h): the checker for octvr_rig_morph_controlpoints.
 * Restated literally: cv::Subdiv2D (imgproc/src/subdivision2d.cpp), getAffineTransform + cv::solve
 * (imgwarp.cpp:6340-6361, lapack.cpp), and per triangle a fillPoly'd mask, cv::warpAffine of the three
 * LUT planes (imgwarp.cpp:5627-5745, WarpAffineInvoker :5282-5470, remapBilinear :3812-4030) and the
 * masked copy — computed only where the triangle's mask is set, which is what copyTo keeps.
 * Parity unpinned: no reference fixture exercises morph_controlpoints (the survey's dump runs had no
 * control points); the pieces it is built from (cv::solve, fillPoly, the bilinear tables, the
 * distance transform, the camera projections) are pinned elsewhere.
 */
#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "octvr_oracle.h"

/* ------------------------------------------------------------------------------------------ */
/* cv::Subdiv2D                                                                                */
/* ------------------------------------------------------------------------------------------ */
typedef struct { int next[4]; int pt[4]; } sd_qedge;            /* Subdiv2D::QuadEdge */
typedef struct { float x, y; int first_edge; int type; } sd_vtx; /* Subdiv2D::Vertex */
typedef struct {
    sd_qedge* qe; int nqe, cap_qe;
    sd_vtx* vt; int nvt, cap_vt;
    int free_qedge, free_point, recent_edge;
    float tl_x, tl_y, br_x, br_y;
    int failed;
} sd_subdiv;

#define SD_NEXT_AROUND_LEFT 0x13
#define SD_PREV_AROUND_ORG 0x11
#define SD_PREV_AROUND_DST 0x33
#define SD_PREV_AROUND_LEFT 0x20
#define SD_PTLOC_ERROR (-2)
#define SD_PTLOC_INSIDE 0
#define SD_PTLOC_VERTEX 1
#define SD_PTLOC_ON_EDGE 2

static void sd_push_qedge(sd_subdiv* s) {
    if (s->nqe == s->cap_qe) {
        s->cap_qe = s->cap_qe ? 2 * s->cap_qe : 64;
        s->qe = (sd_qedge*)realloc(s->qe, sizeof(sd_qedge) * s->cap_qe);
    }
    memset(&s->qe[s->nqe++], 0, sizeof(sd_qedge));
}
static void sd_push_vtx(sd_subdiv* s) {
    if (s->nvt == s->cap_vt) {
        s->cap_vt = s->cap_vt ? 2 * s->cap_vt : 64;
        s->vt = (sd_vtx*)realloc(s->vt, sizeof(sd_vtx) * s->cap_vt);
    }
    sd_vtx v = {0.f, 0.f, 0, -1};
    s->vt[s->nvt++] = v;
}
/* bounds-checked accessors: a corrupt index flags the subdivision instead of reading wild memory */
static sd_qedge* sd_q(sd_subdiv* s, int edge) {
    int i = edge >> 2;
    if (i < 0 || i >= s->nqe) { s->failed = 1; return &s->qe[0]; }
    return &s->qe[i];
}
static sd_vtx* sd_v(sd_subdiv* s, int i) {
    if (i < 0 || i >= s->nvt) { s->failed = 1; return &s->vt[0]; }
    return &s->vt[i];
}
static int sd_next_edge(sd_subdiv* s, int e) { return sd_q(s, e)->next[e & 3]; }         /* :46-50 */
static int sd_rotate(int e, int r) { return (e & ~3) + ((e + r) & 3); }                   /* :52-55 */
static int sd_sym(int e) { return e ^ 2; }                                                 /* :57-60 */
static int sd_get_edge(sd_subdiv* s, int e, int type) {                                    /* :62-68 */
    e = sd_q(s, e)->next[(e + type) & 3];
    return (e & ~3) + ((e + (type >> 4)) & 3);
}
static int sd_org(sd_subdiv* s, int e) { return sd_q(s, e)->pt[e & 3]; }                  /* :70-80 */
static int sd_dst(sd_subdiv* s, int e) { return sd_q(s, e)->pt[(e + 2) & 3]; }            /* :82-92 */

static void sd_splice(sd_subdiv* s, int a, int b) {                                       /* :160-170 */
    int* an = &sd_q(s, a)->next[a & 3];
    int* bn = &sd_q(s, b)->next[b & 3];
    int ar = sd_rotate(*an, 1), br = sd_rotate(*bn, 1);
    int* arn = &sd_q(s, ar)->next[ar & 3];
    int* brn = &sd_q(s, br)->next[br & 3];
    int t = *an; *an = *bn; *bn = t;
    t = *arn; *arn = *brn; *brn = t;
}
static void sd_set_edge_points(sd_subdiv* s, int e, int o, int d) {                      /* :172-178 */
    sd_q(s, e)->pt[e & 3] = o;
    sd_q(s, e)->pt[(e + 2) & 3] = d;
    sd_v(s, o)->first_edge = e;
    sd_v(s, d)->first_edge = e ^ 2;
}
static int sd_new_edge(sd_subdiv* s) {                                                    /* :221-233 */
    if (s->free_qedge <= 0) {
        sd_push_qedge(s);
        s->free_qedge = s->nqe - 1;
    }
    int e = s->free_qedge * 4;
    s->free_qedge = s->qe[e >> 2].next[1];
    sd_qedge* q = &s->qe[e >> 2];                  /* QuadEdge(edgeidx) (:118-127) */
    q->next[0] = e; q->next[1] = e + 3; q->next[2] = e + 2; q->next[3] = e + 1;
    q->pt[0] = q->pt[1] = q->pt[2] = q->pt[3] = 0;
    return e;
}
static void sd_delete_edge(sd_subdiv* s, int e) {                                         /* :235-247 */
    sd_splice(s, e, sd_get_edge(s, e, SD_PREV_AROUND_ORG));
    int se = sd_sym(e);
    sd_splice(s, se, sd_get_edge(s, se, SD_PREV_AROUND_ORG));
    e >>= 2;
    s->qe[e].next[0] = 0;
    s->qe[e].next[1] = s->free_qedge;
    s->free_qedge = e;
}
static int sd_new_point(sd_subdiv* s, float x, float y, int is_virtual) {                /* :249-262 */
    if (s->free_point == 0) {
        sd_push_vtx(s);
        s->free_point = s->nvt - 1;
    }
    int v = s->free_point;
    s->free_point = s->vt[v].first_edge;
    s->vt[v].x = x; s->vt[v].y = y; s->vt[v].first_edge = 0; s->vt[v].type = is_virtual;
    return v;
}
static int sd_connect_edges(sd_subdiv* s, int a, int b) {                                 /* :180-189 */
    int e = sd_new_edge(s);
    sd_splice(s, e, sd_get_edge(s, a, SD_NEXT_AROUND_LEFT));
    sd_splice(s, sd_sym(e), b);
    sd_set_edge_points(s, e, sd_dst(s, a), sd_org(s, b));
    return e;
}
static void sd_swap_edges(sd_subdiv* s, int e) {                                          /* :191-204 */
    int se = sd_sym(e);
    int a = sd_get_edge(s, e, SD_PREV_AROUND_ORG);
    int b = sd_get_edge(s, se, SD_PREV_AROUND_ORG);
    sd_splice(s, e, a);
    sd_splice(s, se, b);
    sd_set_edge_points(s, e, sd_dst(s, a), sd_dst(s, b));
    sd_splice(s, e, sd_get_edge(s, a, SD_NEXT_AROUND_LEFT));
    sd_splice(s, se, sd_get_edge(s, b, SD_NEXT_AROUND_LEFT));
}
static double sd_tri_area(float ax, float ay, float bx, float by, float cx, float cy) { /* :206-209 */
    return ((double)bx - ax) * ((double)cy - ay) - ((double)by - ay) * ((double)cx - ax);
}
static int sd_is_right_of(sd_subdiv* s, float px, float py, int e) {                      /* :211-219 */
    sd_vtx* o = sd_v(s, sd_org(s, e));
    sd_vtx* d = sd_v(s, sd_dst(s, e));
    double cw = sd_tri_area(px, py, d->x, d->y, o->x, o->y);
    return (cw > 0) - (cw < 0);
}
static int sd_in_circle(sd_vtx* pt, sd_vtx* a, sd_vtx* b, sd_vtx* c) {                   /* :386-397 */
    const double eps = FLT_EPSILON * 0.125;
    double val = ((double)a->x * a->x + (double)a->y * a->y) * sd_tri_area(b->x, b->y, c->x, c->y, pt->x, pt->y);
    val -= ((double)b->x * b->x + (double)b->y * b->y) * sd_tri_area(a->x, a->y, c->x, c->y, pt->x, pt->y);
    val += ((double)c->x * c->x + (double)c->y * c->y) * sd_tri_area(a->x, a->y, b->x, b->y, pt->x, pt->y);
    val -= ((double)pt->x * pt->x + (double)pt->y * pt->y) * sd_tri_area(a->x, a->y, b->x, b->y, c->x, c->y);
    return val > eps ? 1 : val < -eps ? -1 : 0;
}

static void sd_init(sd_subdiv* s) {                                                       /* initDelaunay :560-600 */
    memset(s, 0, sizeof *s);
    float big = 3.f * 1;  /* 3 * MAX(rect.width, rect.height), rect (0, 0, 1, 1) */
    s->tl_x = 0.f; s->tl_y = 0.f; s->br_x = 1.f; s->br_y = 1.f;
    sd_push_vtx(s);
    sd_push_qedge(s);
    s->free_qedge = 0; s->free_point = 0;
    int pA = sd_new_point(s, 0.f + big, 0.f, 0);
    int pB = sd_new_point(s, 0.f, 0.f + big, 0);
    int pC = sd_new_point(s, 0.f - big, 0.f - big, 0);
    int eAB = sd_new_edge(s), eBC = sd_new_edge(s), eCA = sd_new_edge(s);
    sd_set_edge_points(s, eAB, pA, pB);
    sd_set_edge_points(s, eBC, pB, pC);
    sd_set_edge_points(s, eCA, pC, pA);
    sd_splice(s, eAB, sd_sym(eCA));
    sd_splice(s, eBC, sd_sym(eAB));
    sd_splice(s, eCA, sd_sym(eBC));
    s->recent_edge = eAB;
}
static void sd_free(sd_subdiv* s) { free(s->qe); free(s->vt); }

static int sd_locate(sd_subdiv* s, float px, float py, int* out_edge, int* out_vertex) {  /* :272-383 */
    int vertex = 0, i, max_edges = s->nqe * 4;
    if (s->nqe < 4) return -100;
    if (px < s->tl_x || py < s->tl_y || px >= s->br_x || py >= s->br_y) return -101;  /* CV_StsOutOfRange */
    int edge = s->recent_edge;
    if (edge <= 0) return -100;
    int location = SD_PTLOC_ERROR;
    int right_of_curr = sd_is_right_of(s, px, py, edge);
    if (right_of_curr > 0) { edge = sd_sym(edge); right_of_curr = -right_of_curr; }
    for (i = 0; i < max_edges; i++) {
        int onext_edge = sd_next_edge(s, edge);
        int dprev_edge = sd_get_edge(s, edge, SD_PREV_AROUND_DST);
        int right_of_onext = sd_is_right_of(s, px, py, onext_edge);
        int right_of_dprev = sd_is_right_of(s, px, py, dprev_edge);
        if (right_of_dprev > 0) {
            if (right_of_onext > 0 || (right_of_onext == 0 && right_of_curr == 0)) { location = SD_PTLOC_INSIDE; break; }
            right_of_curr = right_of_onext; edge = onext_edge;
        } else {
            if (right_of_onext > 0) {
                if (right_of_dprev == 0 && right_of_curr == 0) { location = SD_PTLOC_INSIDE; break; }
                right_of_curr = right_of_dprev; edge = dprev_edge;
            } else if (right_of_curr == 0 &&
                       sd_is_right_of(s, sd_v(s, sd_dst(s, onext_edge))->x, sd_v(s, sd_dst(s, onext_edge))->y, edge) >= 0) {
                edge = sd_sym(edge);
            } else {
                right_of_curr = right_of_onext; edge = onext_edge;
            }
        }
    }
    s->recent_edge = edge;
    if (location == SD_PTLOC_INSIDE) {
        sd_vtx o = *sd_v(s, sd_org(s, edge)), d = *sd_v(s, sd_dst(s, edge));
        float dx1 = px - o.x, dy1 = py - o.y, dx2 = px - d.x, dy2 = py - d.y, dx3 = o.x - d.x, dy3 = o.y - d.y;
        double t1 = fabsf(dx1); t1 += fabsf(dy1);
        double t2 = fabsf(dx2); t2 += fabsf(dy2);
        double t3 = fabsf(dx3); t3 += fabsf(dy3);
        if (t1 < FLT_EPSILON) { location = SD_PTLOC_VERTEX; vertex = sd_org(s, edge); edge = 0; }
        else if (t2 < FLT_EPSILON) { location = SD_PTLOC_VERTEX; vertex = sd_dst(s, edge); edge = 0; }
        else if ((t1 < t3 || t2 < t3) && fabs(sd_tri_area(px, py, o.x, o.y, d.x, d.y)) < FLT_EPSILON) {
            location = SD_PTLOC_ON_EDGE; vertex = 0;
        }
    }
    if (location == SD_PTLOC_ERROR) { edge = 0; vertex = 0; }
    *out_edge = edge;
    *out_vertex = vertex;
    return location;
}

static int sd_insert(sd_subdiv* s, float px, float py) {                                 /* :399-480 */
    int curr_point = 0, curr_edge = 0, deleted_edge;
    int location = sd_locate(s, px, py, &curr_edge, &curr_point);
    if (location < SD_PTLOC_ERROR || location == SD_PTLOC_ERROR) return -1;
    if (location == SD_PTLOC_VERTEX) return curr_point;
    if (location == SD_PTLOC_ON_EDGE) {
        deleted_edge = curr_edge;
        s->recent_edge = curr_edge = sd_get_edge(s, curr_edge, SD_PREV_AROUND_ORG);
        sd_delete_edge(s, deleted_edge);
    }
    curr_point = sd_new_point(s, px, py, 0);
    int base_edge = sd_new_edge(s);
    int first_point = sd_org(s, curr_edge);
    sd_set_edge_points(s, base_edge, first_point, curr_point);
    sd_splice(s, base_edge, curr_edge);
    do {
        base_edge = sd_connect_edges(s, curr_edge, sd_sym(base_edge));
        curr_edge = sd_get_edge(s, base_edge, SD_PREV_AROUND_ORG);
        if (s->failed) return -1;
    } while (sd_dst(s, curr_edge) != first_point);
    curr_edge = sd_get_edge(s, base_edge, SD_PREV_AROUND_ORG);
    int i, max_edges = s->nqe * 4;
    for (i = 0; i < max_edges; i++) {
        int temp_edge = sd_get_edge(s, curr_edge, SD_PREV_AROUND_ORG);
        int temp_dst = sd_dst(s, temp_edge), curr_org = sd_org(s, curr_edge), curr_dst = sd_dst(s, curr_edge);
        if (sd_is_right_of(s, sd_v(s, temp_dst)->x, sd_v(s, temp_dst)->y, curr_edge) > 0 &&
            sd_in_circle(sd_v(s, curr_org), sd_v(s, temp_dst), sd_v(s, curr_dst), sd_v(s, curr_point)) < 0) {
            sd_swap_edges(s, curr_edge);
            curr_edge = sd_get_edge(s, curr_edge, SD_PREV_AROUND_ORG);
        } else if (curr_org == first_point) {
            break;
        } else {
            curr_edge = sd_get_edge(s, sd_next_edge(s, curr_edge), SD_PREV_AROUND_LEFT);
        }
    }
    return s->failed ? -1 : curr_point;
}

/* getTriangleList (:735-760) followed by getTriangleList's [0,1] filter (template_morph.cpp:22-41).
 * Writes at most cap triangles (6 floats each); returns the count kept, or -1. */
static int sd_triangles_in_unit_square(sd_subdiv* s, float* out, int cap) {
    int total = s->nqe * 4, kept = 0;
    char* mask = (char*)calloc((size_t)total, 1);
    for (int i = 4; i < total; i += 2) {
        if (mask[i]) continue;
        float t[6];
        int edge = i;
        sd_vtx* a = sd_v(s, sd_org(s, edge));
        t[0] = a->x; t[1] = a->y;
        if (edge < 0 || edge >= total) { s->failed = 1; break; }
        mask[edge] = 1;
        edge = sd_get_edge(s, edge, SD_NEXT_AROUND_LEFT);
        sd_vtx* b = sd_v(s, sd_org(s, edge));
        t[2] = b->x; t[3] = b->y;
        if (edge < 0 || edge >= total) { s->failed = 1; break; }
        mask[edge] = 1;
        edge = sd_get_edge(s, edge, SD_NEXT_AROUND_LEFT);
        sd_vtx* c = sd_v(s, sd_org(s, edge));
        t[4] = c->x; t[5] = c->y;
        if (edge < 0 || edge >= total) { s->failed = 1; break; }
        mask[edge] = 1;
        int ok = 1;
        for (int k = 0; k < 6; k++) ok = ok && t[k] >= 0.0 && t[k] <= 1.0;
        if (!ok) continue;
        if (kept >= cap) { s->failed = 1; break; }
        memcpy(out + 6 * kept, t, sizeof t);
        kept++;
    }
    free(mask);
    return s->failed ? -1 : kept;
}

/* Subdiv2D(Rect(0, 0, 1, 1)), insert(points), getTriangleList + the [0,1] filter; -1 on failure. */
int orc_delaunay_triangles(const float* pts, int n, float* out, int cap) {
    sd_subdiv s;
    sd_init(&s);
    int rc = 0;
    for (int k = 0; k < n && rc == 0; k++)
        if (sd_insert(&s, pts[2 * k], pts[2 * k + 1]) < 0) rc = -1;
    if (rc == 0) rc = sd_triangles_in_unit_square(&s, out, cap);
    sd_free(&s);
    return rc;
}

/* ------------------------------------------------------------------------------------------ */
/* cv::warpAffine INTER_LINEAR BORDER_CONSTANT 0, evaluated at one destination pixel            */
/* ------------------------------------------------------------------------------------------ */
static int round_sse2(double v) { /* cvRound = _mm_cvtsd_si32: ties to even, out of range -> INT_MIN */
    double r = nearbyint(v);
    if (!(r >= -2147483648.0 && r <= 2147483647.0)) return (int)0x80000000u;
    return (int)r;
}
static short sat_short(int v) { return (short)(v < -32768 ? -32768 : v > 32767 ? 32767 : v); }

/* WarpAffineInvoker (:5296-5380) for pixel (x, y): source cell and 5+5-bit fraction code */
static void warp_coords(const double* M, int x, int y, int* sx, int* sy, int* alpha) {
    const int AB_BITS = 10, AB_SCALE = 1 << AB_BITS, INTER_BITS = 5, INTER_TAB_SIZE = 32;
    const int round_delta = AB_SCALE / INTER_TAB_SIZE / 2;
    int adelta = round_sse2(M[0] * x * AB_SCALE), bdelta = round_sse2(M[3] * x * AB_SCALE); /* :5732-5736 */
    int X0 = round_sse2((M[1] * y + M[2]) * AB_SCALE) + round_delta;
    int Y0 = round_sse2((M[4] * y + M[5]) * AB_SCALE) + round_delta;
    int X = (int)((unsigned)X0 + (unsigned)adelta) >> (AB_BITS - INTER_BITS);
    int Y = (int)((unsigned)Y0 + (unsigned)bdelta) >> (AB_BITS - INTER_BITS);
    *sx = sat_short(X >> INTER_BITS);
    *sy = sat_short(Y >> INTER_BITS);
    *alpha = (Y & (INTER_TAB_SIZE - 1)) * INTER_TAB_SIZE + (X & (INTER_TAB_SIZE - 1));
}

/* remapBilinear (:3812-4030), one channel, for one destination pixel: the inlier expression when all
 * four taps are inside, else BORDER_CONSTANT's per-tap border value 0 */
static float remap_f32(const float* S0, int w, int h, int sx, int sy, const float* wt) {
    unsigned width1 = (unsigned)(w - 1 > 0 ? w - 1 : 0), height1 = (unsigned)(h - 1 > 0 ? h - 1 : 0);
    if ((unsigned)sx < width1 && (unsigned)sy < height1) {
        const float* S = S0 + (size_t)sy * w + sx;
        return S[0] * wt[0] + S[1] * wt[1] + S[w] * wt[2] + S[w + 1] * wt[3];
    }
    if (sx >= w || sx + 1 < 0 || sy >= h || sy + 1 < 0) return 0.f;
    int sx1 = sx + 1, sy1 = sy + 1;
    float v0 = (sx >= 0 && sx < w && sy >= 0 && sy < h) ? S0[(size_t)sy * w + sx] : 0.f;
    float v1 = (sx1 >= 0 && sx1 < w && sy >= 0 && sy < h) ? S0[(size_t)sy * w + sx1] : 0.f;
    float v2 = (sx >= 0 && sx < w && sy1 >= 0 && sy1 < h) ? S0[(size_t)sy1 * w + sx] : 0.f;
    float v3 = (sx1 >= 0 && sx1 < w && sy1 >= 0 && sy1 < h) ? S0[(size_t)sy1 * w + sx1] : 0.f;
    return v0 * wt[0] + v1 * wt[1] + v2 * wt[2] + v3 * wt[3];
}
static uint8_t remap_u8(const uint8_t* S0, int w, int h, int sx, int sy, const int16_t* wt) {
    int v[4];
    for (int t = 0; t < 4; t++) {
        int tx = sx + (t & 1), ty = sy + (t >> 1);
        v[t] = (tx >= 0 && tx < w && ty >= 0 && ty < h) ? S0[(size_t)ty * w + tx] : 0;
    }
    int acc = v[0] * wt[0] + v[1] * wt[1] + v[2] * wt[2] + v[3] * wt[3];
    acc = (acc + (1 << 14)) >> 15; /* FixedPtCast<int, uchar, 15> */
    return (uint8_t)(acc < 0 ? 0 : acc > 255 ? 255 : acc);
}

/* ------------------------------------------------------------------------------------------ */
/* morph_controlpoints                                                                         */
/* ------------------------------------------------------------------------------------------ */
int orc_project(const orc_camera* from, const orc_camera* to, double u, double v, double* x, double* y);

static float fmin_std(float a, float b) { return b < a ? b : a; } /* std::min */
static float fmax_std(float a, float b) { return a < b ? b : a; } /* std::max */

int orc_morph_controlpoints(const orc_camera* out, const orc_camera* const* cams, int n, int W, int H,
                            const int* rois, float* const* map1, float* const* map2, uint8_t* const* masks,
                            const double* cps_in, int n_cps, float* const* src_tris, float* const* dst_tris,
                            int tri_cap, int* n_tris) {
    typedef struct { int n0, n1; float s0x, s0y, s1x, s1y, d0x, d0y, d1x, d1y, mx, my; int l0x, l0y, l1x, l1y; } cp_t;
    cp_t* cps = (cp_t*)calloc((size_t)(n_cps > 0 ? n_cps : 1), sizeof(cp_t));
    int kept = 0, rc = 0;
    for (int k = 0; k < n_cps; k++) {
        cp_t cp;
        const double* a = cps_in + 6 * k;
        cp.n0 = (int)a[0]; cp.n1 = (int)a[1];
        cp.s0x = (float)a[2]; cp.s0y = (float)a[3]; cp.s1x = (float)a[4]; cp.s1y = (float)a[5];
        if (!(cp.n0 < cp.n1) || cp.n0 < 0 || cp.n1 >= n) { rc = -1; goto done; }
        double x, y;
        if (orc_project(cams[cp.n0], out, cp.s0x, cp.s0y, &x, &y)) { rc = -2; goto done; }
        cp.d0x = (float)x; cp.d0y = (float)y;
        if (orc_project(cams[cp.n1], out, cp.s1x, cp.s1y, &x, &y)) { rc = -2; goto done; }
        cp.d1x = (float)x; cp.d1y = (float)y;
        float l1 = fabsf(cp.d0x - cp.d1x) + fabsf(cp.d0y - cp.d1y); /* :123-124 */
        if ((double)l1 > 0.1) continue;
        if (isnan(cp.d0x) || isnan(cp.d0y) || isnan(cp.d1x) || isnan(cp.d1y)) { rc = -1; goto done; }
        const int* r0 = rois + 4 * cp.n0;
        const int* r1 = rois + 4 * cp.n1;
        cp.l0x = (int)(cp.d0x * W - r0[0]); cp.l0y = (int)(cp.d0y * H - r0[1]); /* :107-110 */
        cp.l1x = (int)(cp.d1x * W - r1[0]); cp.l1y = (int)(cp.d1y * H - r1[1]);
        if (cp.l0x < 0 || cp.l0x >= r0[2] || cp.l0y < 0 || cp.l0y >= r0[3] || cp.l1x < 0 || cp.l1x >= r1[2] ||
            cp.l1y < 0 || cp.l1y >= r1[3]) { rc = -1; goto done; }
        cps[kept++] = cp;
    }
    {
        /* DistanceSeamFinder::find's distances (seam_finders.cpp:97-110; resultRoi over all inputs) */
        int ux0 = rois[0], ux1 = rois[0] + rois[2];
        for (int i = 1; i < n; i++) {
            if (rois[4 * i] < ux0) ux0 = rois[4 * i];
            if (rois[4 * i] + rois[4 * i + 2] > ux1) ux1 = rois[4 * i] + rois[4 * i + 2];
        }
        for (int k = 0; k < kept; k++) {
            float wgt[2];
            for (int s = 0; s < 2; s++) {
                int cam = s ? cps[k].n1 : cps[k].n0;
                int lx = s ? cps[k].l1x : cps[k].l0x, ly = s ? cps[k].l1y : cps[k].l0y;
                const int* r = rois + 4 * cam;
                int w = r[2], h = r[3], wrap = r[0] == 0 && w == ux1 - ux0;
                int tw = wrap ? 3 * w : w;
                uint8_t* src = (uint8_t*)malloc((size_t)tw * h);
                float* dist = (float*)malloc(sizeof(float) * (size_t)tw * h);
                for (int yy = 0; yy < h; yy++)
                    for (int c = 0; c < (wrap ? 3 : 1); c++) memcpy(src + (size_t)yy * tw + c * w, masks[cam] + (size_t)yy * w, w);
                orc_distance_transform_l2_3x3(src, tw, h, (size_t)tw, dist, (size_t)tw);
                wgt[s] = dist[(size_t)ly * tw + lx + (wrap ? w : 0)];
                free(src);
                free(dist);
            }
            float w0 = wgt[0], w1 = wgt[1];
            if ((double)(w0 + w1) < 1e-3) w0 = w1 = 1.0f;
            cps[k].mx = (cps[k].d0x * w0 + cps[k].d1x * w1) / (w0 + w1);
            cps[k].my = (cps[k].d0y * w0 + cps[k].d1y * w1) / (w0 + w1);
        }
    }

    int16_t itab[1024 * 4];
    orc_bilinear_tab(itab);
    for (int i = 0; i < n; i++) {
        const int* r = rois + 4 * i;
        const int rw = r[2], rh = r[3];
        int cap = kept + 64, nv = 0;
        float *sv = (float*)malloc(sizeof(float) * 2 * cap), *dv = (float*)malloc(sizeof(float) * 2 * cap);
#define PUSH(SX, SY, DX, DY) do { if (nv == cap) { cap *= 2; sv = (float*)realloc(sv, sizeof(float) * 2 * cap); \
        dv = (float*)realloc(dv, sizeof(float) * 2 * cap); } sv[2 * nv] = (SX); sv[2 * nv + 1] = (SY); \
        dv[2 * nv] = (DX); dv[2 * nv + 1] = (DY); nv++; } while (0)
        for (int k = 0; k < kept; k++) {
            if (cps[k].n0 == i) PUSH(cps[k].d0x, cps[k].d0y, cps[k].mx, cps[k].my);
            if (cps[k].n1 == i) PUSH(cps[k].d1x, cps[k].d1y, cps[k].mx, cps[k].my);
        }
        float bl = 1.f, br = 0.f, bt = 1.f, bb = 0.f; /* :153-169 */
        for (int k = 0; k < nv; k++) {
            bl = fmin_std(bl, sv[2 * k]); br = fmax_std(br, sv[2 * k]);
            bt = fmin_std(bt, sv[2 * k + 1]); bb = fmax_std(bb, sv[2 * k + 1]);
        }
        for (int k = 0; k < nv; k++) {
            bl = fmin_std(bl, dv[2 * k]); br = fmax_std(br, dv[2 * k]);
            bt = fmin_std(bt, dv[2 * k + 1]); bb = fmax_std(bb, dv[2 * k + 1]);
        }
        { double t = (double)bl - 0.05; bl = (float)(1e-3 < t ? t : 1e-3); }
        { double t = (double)bt - 0.05; bt = (float)(1e-3 < t ? t : 1e-3); }
        { double t = (double)br + 0.05; br = (float)(t < 1 - 1e-3 ? t : 1 - 1e-3); }
        { double t = (double)bb + 0.05; bb = (float)(t < 1 - 1e-3 ? t : 1 - 1e-3); }
        int guard = 0;
        for (float x = bl; x < br + 1e-3; x += (br - bl) / 10) { /* :171-176 */
            if (++guard > 100000) { rc = -3; break; }
            PUSH(x, bt, x, bt);
            PUSH(x, bb, x, bb);
        }
        for (float y = bt + (bb - bt) / 10; y < bb - (bb - bt) / 10 + 1e-3; y += (bb - bt) / 10) { /* :177-182 */
            if (++guard > 100000) { rc = -3; break; }
            PUSH(bl, y, bl, y);
            PUSH(br, y, br, y);
        }
#undef PUSH
        int nt = 0;
        if (rc == 0) {
            sd_subdiv sd;
            sd_init(&sd);
            for (int k = 0; k < nv && rc == 0; k++)
                if (sd_insert(&sd, sv[2 * k], sv[2 * k + 1]) < 0) rc = -4;
            if (rc == 0) {
                nt = sd_triangles_in_unit_square(&sd, src_tris[i], tri_cap);
                if (nt < 0) rc = -4;
            }
            sd_free(&sd);
        }
        /* getTriangleListIndexes / FromIndexes (:43-67) */
        for (int t = 0; t < nt && rc == 0; t++)
            for (int c = 0; c < 3; c++) {
                float px = src_tris[i][6 * t + 2 * c], py = src_tris[i][6 * t + 2 * c + 1];
                int j = 0;
                while (j < nv && !(sv[2 * j] == px && sv[2 * j + 1] == py)) j++;
                if (j == nv) { rc = -4; break; }
                dst_tris[i][6 * t + 2 * c] = dv[2 * j];
                dst_tris[i][6 * t + 2 * c + 1] = dv[2 * j + 1];
            }
        free(sv);
        free(dv);
        if (rc) goto done;
        n_tris[i] = nt;
        if (nt == 0) continue;

        /* per triangle (:202-231): warpAffine of the ORIGINAL planes, copied where the triangle's
         * fillPoly mask is set; later triangles overwrite earlier ones */
        size_t px_n = (size_t)rw * rh;
        float* o1 = (float*)malloc(sizeof(float) * px_n);
        float* o2 = (float*)malloc(sizeof(float) * px_n);
        uint8_t* om = (uint8_t*)malloc(px_n);
        uint8_t* tri = (uint8_t*)malloc(px_n);
        memcpy(o1, map1[i], sizeof(float) * px_n);
        memcpy(o2, map2[i], sizeof(float) * px_n);
        memcpy(om, masks[i], px_n);
        for (int t = 0; t < nt; t++) {
            float s[6], d[6];
            for (int c = 0; c < 3; c++) { /* T(x, y) (:202-203) */
                s[2 * c] = src_tris[i][6 * t + 2 * c] * W - r[0];
                s[2 * c + 1] = src_tris[i][6 * t + 2 * c + 1] * H - r[1];
                d[2 * c] = dst_tris[i][6 * t + 2 * c] * W - r[0];
                d[2 * c + 1] = dst_tris[i][6 * t + 2 * c + 1] * H - r[1];
            }
            /* getAffineTransform (imgwarp.cpp:6340-6361) */
            double A[36], b[6], M[6];
            for (int k = 0; k < 3; k++) {
                int j = k * 12, kk = k * 12 + 6;
                A[j] = A[kk + 3] = s[2 * k];
                A[j + 1] = A[kk + 4] = s[2 * k + 1];
                A[j + 2] = A[kk + 5] = 1;
                A[j + 3] = A[j + 4] = A[j + 5] = 0;
                A[kk] = A[kk + 1] = A[kk + 2] = 0;
                b[k * 2] = d[2 * k];
                b[k * 2 + 1] = d[2 * k + 1];
            }
            if (!orc_solve(A, b, 6, M)) memset(M, 0, sizeof M); /* lapack.cpp:1317-1318 */
            /* warpAffine without WARP_INVERSE_MAP inverts M (imgwarp.cpp:5655-5666) */
            double D = M[0] * M[4] - M[1] * M[3];
            D = D != 0 ? 1. / D : 0;
            double A11 = M[4] * D, A22 = M[0] * D;
            M[0] = A11; M[1] *= -D;
            M[3] *= -D; M[4] = A22;
            double b1 = -M[0] * M[2] - M[1] * M[5];
            double b2 = -M[3] * M[2] - M[4] * M[5];
            M[2] = b1; M[5] = b2;

            int pts[6];
            for (int k = 0; k < 6; k++) pts[k] = (int)roundf(d[k]);
            memset(tri, 0, px_n);
            orc_fill_poly(tri, rw, rh, pts, 3, 255);
            for (int y = 0; y < rh; y++)
                for (int x = 0; x < rw; x++) {
                    size_t o = (size_t)y * rw + x;
                    if (!tri[o]) continue;
                    int sx, sy, alpha;
                    warp_coords(M, x, y, &sx, &sy, &alpha);
                    float fy = (float)(alpha >> 5) * (1.f / 32), fx = (float)(alpha & 31) * (1.f / 32);
                    float wt[4] = {(1.f - fy) * (1.f - fx), (1.f - fy) * fx, fy * (1.f - fx), fy * fx}; /* BilinearTab_f */
                    o1[o] = remap_f32(map1[i], rw, rh, sx, sy, wt);
                    o2[o] = remap_f32(map2[i], rw, rh, sx, sy, wt);
                    om[o] = remap_u8(masks[i], rw, rh, sx, sy, itab + 4 * alpha);
                }
        }
        memcpy(map1[i], o1, sizeof(float) * px_n);
        memcpy(map2[i], o2, sizeof(float) * px_n);
        memcpy(masks[i], om, px_n);
        free(o1); free(o2); free(om); free(tri);
    }
done:
    free(cps);
    return rc ? rc : kept;
}
