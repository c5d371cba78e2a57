/*
 * octvr_oracle.c — CPU restatement of the reference octVR hot path (TEST INFRASTRUCTURE ONLY).
 * See octvr_oracle.h.  Compiled with -ffp-contract=off so every float/double expression rounds
 * exactly as written (the reference x86-64 build has no FMA contraction).
 */
#include "octvr_oracle.h"

#include <float.h>
#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#ifndef M_PI
#define M_PI 3.14159265358979323846
#endif

/* ------------------------------------------------------------------------------------------ */
/* Rotation: Camera::Camera (octvr/src/camera.cpp:49-70)                                       */
/* ------------------------------------------------------------------------------------------ */

/* cvRodrigues2 vector -> matrix (calib3d/src/calibration.cpp:300-345). */
static void rodrigues(double rx, double ry, double rz, double R[9]) {
    double theta = sqrt(rx * rx + ry * ry + rz * rz);
    if (theta < DBL_EPSILON) {
        for (int k = 0; k < 9; k++) R[k] = (k % 4 == 0) ? 1.0 : 0.0;
        return;
    }
    static const double I[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
    double c = cos(theta), s = sin(theta), c1 = 1. - c;
    double itheta = theta ? 1. / theta : 0.;
    rx *= itheta; ry *= itheta; rz *= itheta;
    double rrt[9] = {rx * rx, rx * ry, rx * rz, rx * ry, ry * ry, ry * rz, rx * rz, ry * rz, rz * rz};
    double rx_[9] = {0, -rz, ry, rz, 0, -rx, -ry, rx, 0};
    for (int k = 0; k < 9; k++) R[k] = c * I[k] + c1 * rrt[k] + s * rx_[k];
}

/* 3x3 product through cv::gemm's len==3 fast path (core/src/matmul.cpp:934-1000):
 * t = a0*b0 + a1*b1 + a2*b2 ; d = t*alpha + c*beta with alpha=1, beta=0, c=zero. */
static void mul33(const double* a, const double* b, double* d) {
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
            double t = a[i * 3 + 0] * b[0 * 3 + j] + a[i * 3 + 1] * b[1 * 3 + j] + a[i * 3 + 2] * b[2 * 3 + j];
            d[i * 3 + j] = t * 1.0 + 0.0 * 0.0;
        }
}

void orc_rotation_rpy(double roll, double yaw, double pitch, double R[9]) {
    double v0 = roll, v1 = -yaw, v2 = -pitch;
    double Rx[9], Ry[9], Rz[9], T[9];
    rodrigues(v0, 0, 0, Rx);
    rodrigues(0, v1, 0, Ry);
    rodrigues(0, 0, v2, Rz);
    mul33(Rx, Rz, T);
    mul33(T, Ry, R);
}

/* cv::invert 3x3 double closed form (core/src/lapack.cpp:709-712 det3, :970-990). */
void orc_invert3(const double* S, double* D) {
#define Sd(y, x) S[(y) * 3 + (x)]
    double d = Sd(0, 0) * ((double)Sd(1, 1) * Sd(2, 2) - (double)Sd(1, 2) * Sd(2, 1)) -
               Sd(0, 1) * ((double)Sd(1, 0) * Sd(2, 2) - (double)Sd(1, 2) * Sd(2, 0)) +
               Sd(0, 2) * ((double)Sd(1, 0) * Sd(2, 1) - (double)Sd(1, 1) * Sd(2, 0));
    if (d == 0.) {
        for (int k = 0; k < 9; k++) D[k] = 0;
        return;
    }
    d = 1. / d;
    D[0] = (Sd(1, 1) * Sd(2, 2) - Sd(1, 2) * Sd(2, 1)) * d;
    D[1] = (Sd(0, 2) * Sd(2, 1) - Sd(0, 1) * Sd(2, 2)) * d;
    D[2] = (Sd(0, 1) * Sd(1, 2) - Sd(0, 2) * Sd(1, 1)) * d;
    D[3] = (Sd(1, 2) * Sd(2, 0) - Sd(1, 0) * Sd(2, 2)) * d;
    D[4] = (Sd(0, 0) * Sd(2, 2) - Sd(0, 2) * Sd(2, 0)) * d;
    D[5] = (Sd(0, 2) * Sd(1, 0) - Sd(0, 0) * Sd(1, 2)) * d;
    D[6] = (Sd(1, 0) * Sd(2, 1) - Sd(1, 1) * Sd(2, 0)) * d;
    D[7] = (Sd(0, 1) * Sd(2, 0) - Sd(0, 0) * Sd(2, 1)) * d;
    D[8] = (Sd(0, 0) * Sd(1, 1) - Sd(0, 1) * Sd(1, 0)) * d;
#undef Sd
}

void orc_camera_set_rotation(orc_camera* c, const double R[9]) {
    memcpy(c->R, R, sizeof(c->R));
    orc_invert3(R, c->Rinv);
}

static void camera_defaults(orc_camera* c, int type) {
    memset(c, 0, sizeof(*c));
    c->type = type;
    double R[9];
    orc_rotation_rpy(0, 0, 0, R);
    orc_camera_set_rotation(c, R);
    c->min_lon = -M_PI;
    c->max_lon = M_PI;
}

void orc_camera_equirect(orc_camera* c, double min_lat, double max_lat, double scale_lon) {
    camera_defaults(c, ORC_EQUIRECT);
    c->min_lat = min_lat;
    c->max_lat = max_lat;
    c->scale_lon = scale_lon;
}

/* CalcCorrectionRadius_copy and helpers (octvr/src/cameras/fullframe_fisheye_cam.cpp:20-103). */
static double cube_root(double x) {
    if (x == 0.0) return 0.0;
    if (x > 0.0) return pow(x, 1.0 / 3.0);
    return -pow(-x, 1.0 / 3.0);
}
static void square_zero(double* a, int* n, double* root) {
    if (a[2] == 0.0) {
        if (a[1] == 0.0) {
            if (a[0] == 0.0) { *n = 1; root[0] = 0.0; }
            else *n = 0;
        } else { *n = 1; root[0] = -a[0] / a[1]; }
    } else {
        if (4.0 * a[2] * a[0] > a[1] * a[1]) *n = 0;
        else {
            *n = 2;
            root[0] = (-a[1] + sqrt(a[1] * a[1] - 4.0 * a[2] * a[0])) / (2.0 * a[2]);
            root[1] = (-a[1] - sqrt(a[1] * a[1] - 4.0 * a[2] * a[0])) / (2.0 * a[2]);
        }
    }
}
static void cube_zero(double* a, int* n, double* root) {
    if (a[3] == 0.0) {
        square_zero(a, n, root);
    } else {
        double p = ((-1.0 / 3.0) * (a[2] / a[3]) * (a[2] / a[3]) + a[1] / a[3]) / 3.0;
        double q = ((2.0 / 27.0) * (a[2] / a[3]) * (a[2] / a[3]) * (a[2] / a[3]) - (1.0 / 3.0) * (a[2] / a[3]) * (a[1] / a[3]) +
                    a[0] / a[3]) / 2.0;
        if (q * q + p * p * p >= 0.0) {
            *n = 1;
            root[0] = cube_root(-q + sqrt(q * q + p * p * p)) + cube_root(-q - sqrt(q * q + p * p * p)) - a[2] / (3.0 * a[3]);
        } else {
            double phi = acos(-q / sqrt(-p * p * p));
            *n = 3;
            root[0] = 2.0 * sqrt(-p) * cos(phi / 3.0) - a[2] / (3.0 * a[3]);
            root[1] = -2.0 * sqrt(-p) * cos(phi / 3.0 + M_PI / 3.0) - a[2] / (3.0 * a[3]);
            root[2] = -2.0 * sqrt(-p) * cos(phi / 3.0 - M_PI / 3.0) - a[2] / (3.0 * a[3]);
        }
    }
}
static double correction_radius(const double* coeff) {
    double a[4];
    for (int k = 0; k < 4; k++) {
        a[k] = 0.0;
        if (coeff[k] != 0.0) a[k] = (k + 1) * coeff[k];
    }
    int n, i;
    double root[3], sroot = 1000.0;
    cube_zero(a, &n, root);
    for (i = 0; i < n; i++)
        if (root[i] > 0.0 && root[i] < sroot) sroot = root[i];
    return sroot;
}

void orc_camera_fullframe_fisheye(orc_camera* c, int width, int height, int crop_l, int crop_r, int crop_t,
                                  int crop_b, int has_crop, int crop_circular, double hfov, double center_dx,
                                  double center_dy, const double radial[3]) {
    camera_defaults(c, ORC_FULLFRAME_FISHEYE);
    c->width = width;
    c->height = height;
    if (has_crop) {
        c->crop_x = crop_l;
        c->crop_y = crop_t;
        c->crop_w = crop_r - crop_l;
        c->crop_h = crop_b - crop_t;
        c->crop_circular = crop_circular;
    }
    if (c->crop_w * c->crop_h == 0) { /* crop.area() == 0 (fullframe_fisheye_cam.cpp:122-125) */
        c->crop_x = c->crop_y = 0;
        c->crop_w = width;
        c->crop_h = height;
        c->crop_circular = 0;
    }
    c->hfov = hfov;
    c->center_dx = center_dx;
    c->center_dy = center_dy;
    c->rad[3] = radial[0];
    c->rad[2] = radial[1];
    c->rad[1] = radial[2];
    c->rad[0] = 1.0 - radial[0] - radial[1] - radial[2];
    c->rad[4] = (c->crop_w < c->crop_h ? c->crop_w : c->crop_h) / 2.0;
    c->rad[5] = correction_radius(c->rad);
}

void orc_camera_fisheye(orc_camera* c, int width, int height, double fx, double fy, double cx, double cy,
                        const double k[4]) {
    camera_defaults(c, ORC_FISHEYE);
    c->width = width;
    c->height = height;
    c->fx = fx; c->fy = fy; c->cx = cx; c->cy = cy;
    for (int i = 0; i < 4; i++) c->k[i] = k[i];
}

/* computeTiltProjectionMatrix (imgproc/include/opencv2/imgproc/detail/distortion_model.hpp:74-94);
 * Matx products accumulate s = 0; s += a(i,k) * b(k,j). */
static void matx33_mul(const double* a, const double* b, double* d) {
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
            double s = 0;
            for (int k = 0; k < 3; k++) s += a[i * 3 + k] * b[k * 3 + j];
            d[i * 3 + j] = s;
        }
}
static void tilt_projection(double tauX, double tauY, double* T) {
    double cTauX = cos(tauX), sTauX = sin(tauX), cTauY = cos(tauY), sTauY = sin(tauY);
    double rotX[9] = {1, 0, 0, 0, cTauX, sTauX, 0, -sTauX, cTauX};
    double rotY[9] = {cTauY, 0, -sTauY, 0, 1, 0, sTauY, 0, cTauY};
    double rotXY[9];
    matx33_mul(rotY, rotX, rotXY);
    double projZ[9] = {rotXY[8], 0, -rotXY[2], 0, rotXY[8], -rotXY[5], 0, 0, 1};
    matx33_mul(projZ, rotXY, T);
}

void orc_camera_pinhole(orc_camera* c, int width, int height, double fx, double fy, double cx, double cy,
                        const double* dist, int nd) {
    camera_defaults(c, ORC_PINHOLE);
    c->width = width;
    c->height = height;
    c->fx = fx; c->fy = fy; c->cx = cx; c->cy = cy;
    for (int i = 0; i < nd && i < 14; i++) c->dist[i] = dist[i];
    for (int i = 0; i < 9; i++) c->tilt[i] = (i % 4 == 0) ? 1.0 : 0.0;
    if (c->dist[12] != 0 || c->dist[13] != 0) tilt_projection(c->dist[12], c->dist[13], c->tilt);
}

void orc_camera_normal(orc_camera* c, double aspect_ratio, double cam_opt) {
    camera_defaults(c, ORC_NORMAL);
    c->aspect = aspect_ratio;
    c->cam_x = cam_opt;
    c->cam_z = sqrt((1.0 - c->cam_x * c->cam_x) / (1.0 + 1.0 / c->aspect / c->aspect));
    c->cam_y = c->cam_z / c->aspect;
}

void orc_camera_perspective(orc_camera* c, double aspect_ratio, double sf) {
    camera_defaults(c, ORC_PERSPECTIVE);
    c->aspect = aspect_ratio;
    c->sf = sf;
}

void orc_camera_ocam(orc_camera* c, const double* pol, int len_pol, const double* invpol, int len_invpol, double xc,
                     double yc, double cc, double d, double e, int width, int height) {
    camera_defaults(c, ORC_OCAM);
    c->len_pol = len_pol;
    c->len_invpol = len_invpol;
    for (int i = 0; i < len_pol && i < 64; i++) c->pol[i] = pol[i];
    for (int i = 0; i < len_invpol && i < 64; i++) c->invpol[i] = invpol[i];
    c->xc = xc; c->yc = yc; c->oc = cc; c->od = d; c->oe = e;
    c->width = width;
    c->height = height;
}

void orc_camera_simple(orc_camera* c, int type, double circle) {
    camera_defaults(c, type);
    c->circle = circle;
}

void orc_camera_set_selection(orc_camera* c, int width, int height, int l, int r, int t, int b) {
    c->sel = 1;
    c->width = width;
    c->height = height;
    c->sel_l = l; c->sel_r = r; c->sel_t = t; c->sel_b = b;
}

/* ------------------------------------------------------------------------------------------ */
/* Sphere helpers (camera.cpp:189-210)                                                         */
/* ------------------------------------------------------------------------------------------ */
/* noinline (and below): gcc merges the sin / cos of one argument within a function into one sincos
 * call, so the oracle keeps the reference's function boundaries (the reference model methods are separate
 * functions there) instead of letting inlining pair values the reference never pairs (camera.cpp, cameras/ sources). */
__attribute__((noinline)) static void lonlat_to_xyz(double lon, double lat, double* p) {
    p[0] = cos(lon) * cos(lat);
    p[1] = sin(lat);
    p[2] = -sin(lon) * cos(lat);
}
/* rotated = m * r.t() through GEMMSingleMul's A*Bt loop (matmul.cpp:234-262): s = ((0+a0b0)+a1b1)+a2b2. */
static void rotate(const double* r, const double* p, double* q) {
    for (int k = 0; k < 3; k++) {
        double s0 = 0;
        s0 += p[0] * r[k * 3 + 0];
        s0 += p[1] * r[k * 3 + 1];
        s0 += p[2] * r[k * 3 + 2];
        double s1 = 0, s2 = 0, s3 = 0;
        q[k] = (s0 + s1 + s2 + s3) * 1.0;
    }
}
static void xyz_to_lonlat(const double* xyz, double* lon, double* lat) {
    double n = sqrt(xyz[0] * xyz[0] + xyz[1] * xyz[1] + xyz[2] * xyz[2]);
    double inv = 1.0 / n;
    double px = xyz[0] * inv, py = xyz[1] * inv, pz = xyz[2] * inv;
    *lon = atan2(-pz, px);
    *lat = asin(py);
}
static int valid_longitude(const orc_camera* c, double l) {
#define BETWEEN(x) ((x) >= c->min_lon && (x) <= c->max_lon)
    return BETWEEN(l) || BETWEEN(l + 2 * M_PI) || BETWEEN(l - 2 * M_PI) || BETWEEN(l + 4 * M_PI) ||
           BETWEEN(l - 4 * M_PI);
#undef BETWEEN
}

/* Equirectangular::image_to_obj_single / obj_to_image_single (cameras/equirectangular.cpp:25-35). */
static void equirect_i2o(const orc_camera* c, double x, double y, double* lon, double* lat) {
    *lon = (x - 0.5) * M_PI * 2.0;
    *lat = (c->min_lat - c->max_lat) * y + c->max_lat;
}
static void equirect_o2i(const orc_camera* c, double lon, double lat, double* x, double* y) {
    *x = lon / (M_PI * 2.0) + 0.5;
    *y = (lat - c->max_lat) / (c->min_lat - c->max_lat);
}

/* FullFrameFisheyeCamera::obj_to_image_single (fullframe_fisheye_cam.cpp:146-221). */
__attribute__((noinline)) static void ffisheye_o2i(const orc_camera* c, double lon, double lat, double* ox, double* oy) {
    double s = cos(lat) * cos(lon);
    double v1 = sin(lat);
    double v0 = -cos(lat) * sin(lon);
    double r = sqrt(v0 * v0 + v1 * v1);
    double theta = atan2(r, s);
    double distance = (double)(c->crop_w) / (c->hfov);
    double x = -(theta * v0 / r) * distance;
    double y = -(theta * v1 / r) * distance;
    if (fabs(lon) < 1e-5 && fabs(lat) < 1e-5) x = y = 0;
    /* do_radial_distort */
    double rr = (sqrt(x * x + y * y)) / c->rad[4];
    double scale;
    if (rr < c->rad[5])
        scale = ((c->rad[3] * rr + c->rad[2]) * rr + c->rad[1]) * rr + c->rad[0];
    else
        scale = 1000.0;
    double rx = x * scale, ry = y * scale;
    rx += c->center_dx;
    ry += c->center_dy;
    rx /= (double)c->crop_w;
    ry /= (double)c->crop_h;
    rx += 0.5;
    ry += 0.5;
    if (c->crop_circular && (rx - 0.5) * (rx - 0.5) + (ry - 0.5) * (ry - 0.5) > 0.25) {
        *ox = NAN;
        *oy = NAN;
        return;
    }
    rx = (rx * c->crop_w) + c->crop_x;
    ry = (ry * c->crop_h) + c->crop_y;
    rx /= (double)c->width;
    ry /= (double)c->height;
    *ox = rx;
    *oy = ry;
}

/* PinholeCamera::obj_to_image + cv::fisheye::projectPoints (pinhole_cam.cpp:32-50, calib3d/src/fisheye.cpp:95-146).
 * Input: the rotated xyz (sphere_rotate(xyzs, false) output). */
static void fisheye_project(const orc_camera* c, const double* Y, double* ox, double* oy) {
    if (Y[2] <= 0) { *ox = NAN; *oy = NAN; return; }
    double x0 = Y[0] / Y[2], x1 = Y[1] / Y[2];
    double r2 = x0 * x0 + x1 * x1;
    double r = sqrt(r2);
    double theta = atan(r);
    double theta2 = theta * theta, theta3 = theta2 * theta, theta4 = theta2 * theta2, theta5 = theta4 * theta,
           theta6 = theta3 * theta3, theta7 = theta6 * theta, theta8 = theta4 * theta4, theta9 = theta8 * theta;
    double theta_d = theta + c->k[0] * theta3 + c->k[1] * theta5 + c->k[2] * theta7 + c->k[3] * theta9;
    double inv_r = r > 1e-8 ? 1.0 / r : 1;
    double cdist = r > 1e-8 ? theta_d * inv_r : 1;
    double xd0 = x0 * cdist, xd1 = x1 * cdist;
    double alpha = 0;
    double xd3_0 = xd0 + alpha * xd1, xd3_1 = xd1;
    double u = xd3_0 * c->fx + c->cx, v = xd3_1 * c->fy + c->cy;
    *ox = u / c->width;
    *oy = 1.0 - v / c->height;
}

/* cv::projectPoints (calibration.cpp:759-793) of one rotated point with rvec = tvec = 0 (R = I). */
static void pinhole_project(const orc_camera* c, const double* P, double* ox, double* oy) {
    double X = P[0], Y = P[1], Z = P[2];
    if (Z <= 0) X = Y = Z = NAN; /* pinhole_cam.cpp:38-40 */
    const double* k = c->dist;
    const double R[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1}, t[3] = {0, 0, 0};
    double x = R[0] * X + R[1] * Y + R[2] * Z + t[0];
    double y = R[3] * X + R[4] * Y + R[5] * Z + t[1];
    double z = R[6] * X + R[7] * Y + R[8] * Z + t[2];
    z = z ? 1. / z : 1;
    x *= z; y *= z;
    double r2 = x * x + y * y, r4 = r2 * r2, r6 = r4 * r2;
    double a1 = 2 * x * y, a2 = r2 + 2 * x * x, a3 = r2 + 2 * y * y;
    double cdist = 1 + k[0] * r2 + k[1] * r4 + k[4] * r6;
    double icdist2 = 1. / (1 + k[5] * r2 + k[6] * r4 + k[7] * r6);
    double xd0 = x * cdist * icdist2 + k[2] * a1 + k[3] * a2 + k[8] * r2 + k[9] * r4;
    double yd0 = y * cdist * icdist2 + k[2] * a3 + k[3] * a1 + k[10] * r2 + k[11] * r4;
    double vec[3] = {xd0, yd0, 1}, vt[3];
    for (int i = 0; i < 3; i++) {
        double s = 0;
        for (int j = 0; j < 3; j++) s += c->tilt[i * 3 + j] * vec[j];
        vt[i] = s;
    }
    double invProj = vt[2] ? 1. / vt[2] : 1;
    double xd = invProj * vt[0], yd = invProj * vt[1];
    double u = xd * c->fx + c->cx, v = yd * c->fy + c->cy;
    *ox = u / c->width;           /* pinhole_cam.cpp:48 */
    *oy = 1.0 - v / c->height;
}

/* OCamCalib cam2world / world2cam (ocam_fisheye.cpp:135-225). */
static void ocam_cam2world(const orc_camera* m, const double* p2, double* p3) {
    double invdet = 1 / (m->oc - m->od * m->oe);
    double xp = invdet * ((p2[0] - m->xc) - m->od * (p2[1] - m->yc));
    double yp = invdet * (-m->oe * (p2[0] - m->xc) + m->oc * (p2[1] - m->yc));
    double r = sqrt(xp * xp + yp * yp);
    double zp = m->pol[0], r_i = 1;
    for (int i = 1; i < m->len_pol; i++) { r_i *= r; zp += r_i * m->pol[i]; }
    double invnorm = 1 / sqrt(xp * xp + yp * yp + zp * zp);
    p3[0] = invnorm * xp; p3[1] = invnorm * yp; p3[2] = invnorm * zp;
}
static void ocam_world2cam(const orc_camera* m, const double* p3, double* p2) {
    double norm = sqrt(p3[0] * p3[0] + p3[1] * p3[1]);
    double theta = atan(p3[2] / norm);
    if (norm != 0) {
        double invnorm = 1 / norm, t = theta, rho = m->invpol[0], t_i = 1;
        for (int i = 1; i < m->len_invpol; i++) { t_i *= t; rho += t_i * m->invpol[i]; }
        double x = p3[0] * invnorm * rho, y = p3[1] * invnorm * rho;
        p2[0] = x * m->oc + y * m->od + m->xc;
        p2[1] = x * m->oe + y + m->yc;
    } else {
        p2[0] = m->xc;
        p2[1] = m->yc;
    }
}

static void lonlat_of(double x, double y, double z, double* lon, double* lat) {
    double p[3] = {x, y, z};
    xyz_to_lonlat(p, lon, lat);
}

/* image_to_obj_single of the output camera types (the cameras/ files cited in octvr_oracle.h). */
/* cv::solvePoly (core/src/mathfuncs.cpp:2063-2182, maxIters 300) for real coefficients, written with
 * cv::Complex<double> semantics (core/types.hpp:960-1029).  Returns the trimmed degree; only roots
 * [0, n) are defined (the reference copies uninitialised memory into rows n..n0-1).  The
 * num_same_root > 1 branch (:2119-2157) needs bit-identical iterates and is not restated. */
typedef struct { double re, im; } cplx;
static cplx c_mul(cplx a, cplx b) { cplx r = {a.re * b.re - a.im * b.im, a.re * b.im + a.im * b.re}; return r; }
static cplx c_add(cplx a, cplx b) { cplx r = {a.re + b.re, a.im + b.im}; return r; }
static cplx c_sub(cplx a, cplx b) { cplx r = {a.re - b.re, a.im - b.im}; return r; }
static cplx c_div(cplx a, cplx b) {
    double t = 1. / ((double)b.re * b.re + (double)b.im * b.im);
    cplx r = {(a.re * b.re + a.im * b.im) * t, (-a.re * b.im + a.im * b.re) * t};
    return r;
}
static int solve_poly(const double* a, int n0, cplx* roots) {
    cplx coeffs[16];
    int n = n0;
    for (int i = 0; i <= n0; i++) { coeffs[i].re = a[i]; coeffs[i].im = 0; }
    for (; n > 1; n--)
        if (fabs(coeffs[n].re) + fabs(coeffs[n].im) > DBL_EPSILON) break;
    cplx p = {1, 0}, r = {1, 1};
    for (int i = 0; i < n; i++) { roots[i] = p; p = c_mul(p, r); }
    for (int iter = 0; iter < 300; iter++) {
        double maxDiff = 0;
        for (int i = 0; i < n; i++) {
            p = roots[i];
            cplx num = coeffs[n], denom = coeffs[n];
            for (int j = 0; j < n; j++) {
                num = c_add(c_mul(num, p), coeffs[n - j - 1]);
                if (j != i) {
                    cplx d = c_sub(p, roots[j]);
                    if (d.re != 0 || d.im != 0) denom = c_mul(denom, d);
                }
            }
            num = c_div(num, denom);
            roots[i] = c_sub(p, num);
            double ad = sqrt((double)num.re * num.re + (double)num.im * num.im);
            if (ad > maxDiff) maxDiff = ad;
        }
        if (maxDiff <= 0) break;
    }
    for (int i = 0; i < n; i++)
        if (fabs(roots[i].im) < 1e-100) roots[i].im = 0;
    return n;
}

/* FullFrameFisheyeCamera::image_to_obj_single + do_reverse_radial_distort
 * (cameras/fullframe_fisheye_cam.cpp:160-185, 223-253) */
__attribute__((noinline)) static void fullframe_image_to_obj(const orc_camera* c, double x, double y, double* lon, double* lat) {
    x = (x - 0.5) * (double)c->crop_w - c->center_dx;
    y = (y - 0.5) * (double)c->crop_h - c->center_dy;
    if (fabs(x) < 1e-5 && fabs(y) < 1e-5) { *lon = 0; *lat = 0; return; }
    double sq = sqrt(x * x + y * y);
    double coeffs[5] = {-sq / c->rad[4], c->rad[0], c->rad[1], c->rad[2], c->rad[3]};
    cplx roots[4];
    double r = -1;
    int n = solve_poly(coeffs, 4, roots);
    for (int i = 0; i < n; i++)
        if (fabs(roots[i].im) < 1e-3 && roots[i].re > 0 && (roots[i].re < r || r < 0)) r = roots[i].re;
    double scale = (r < c->rad[5] && r > 0) ? sq / c->rad[4] / r : 1000.0;
    x /= scale;
    y /= scale;
    double distance = (double)c->crop_w / c->hfov;
    double alpha = atan2(-y, x);
    double theta = -y / distance / sin(alpha);
    if (fabs(sin(alpha)) < 1e-3) theta = -x / distance / cos(alpha);
    *lon = atan2(sin(theta) * cos(alpha), cos(theta));
    *lat = atan(tan(alpha) * sin(*lon));
}

__attribute__((noinline)) static void image_to_obj_single(const orc_camera* c, double x, double y, double* lon, double* lat) {
    switch (c->type) {
    case ORC_FULLFRAME_FISHEYE: fullframe_image_to_obj(c, x, y, lon, lat); return;
    case ORC_NORMAL: /* normal.cpp:24-30 */
        lonlat_of(c->cam_x, c->cam_y - y * 2.0 * c->cam_y, c->cam_z - x * 2.0 * c->cam_z, lon, lat);
        return;
    case ORC_PERSPECTIVE: /* perspective.cpp:21-26 */
        lonlat_of(1.0 / c->sf, 0.5 - y, (0.5 - x) * c->aspect, lon, lat);
        return;
    case ORC_OCAM: { /* ocam_fisheye.cpp:237-244 */
        double p2[2] = {y * c->height, x * c->width}, p3[3];
        ocam_cam2world(c, p2, p3);
        lonlat_of(-p3[2], -p3[0], -p3[1], lon, lat);
        return;
    }
    case ORC_STUPIDOVAL: { /* stupidoval.hpp:30-36 */
        double la = (0.5 - y) * M_PI;
        double lo = (x - 0.5) * M_PI * 2.0 / cos(la);
        if (lo < -M_PI || lo > M_PI) { *lon = *lat = NAN; return; }
        *lon = lo; *lat = la;
        return;
    }
    case ORC_CUBIC: { /* cubic.hpp:26-37, 86-103 */
        int index_x = 0, index_y = 0;
        if (y >= 0.5) index_y = 1;
        if (x >= 2.0 / 3.0) index_x = 2;
        else if (x >= 1.0 / 3.0) index_x = 1;
        double fx = (x - index_x * 1.0 / 3.0) * 3.0 * 2.0 - 1.0;
        double fy = (y - index_y * 1.0 / 2.0) * 2.0 * 2.0 - 1.0;
        int face = index_y * 3 + index_x;
        if (face == 0) lonlat_of(1.0, fy, fx, lon, lat);
        else if (face == 1) lonlat_of(-1., fy, -fx, lon, lat);
        else if (face == 2) lonlat_of(fx, -1., -fy, lon, lat);
        else if (face == 3) lonlat_of(fx, 1.0, fy, lon, lat);
        else if (face == 4) lonlat_of(fx, fy, -1.0, lon, lat);
        else lonlat_of(-fx, fy, 1.0, lon, lat);
        return;
    }
    case ORC_EQAREA_NORTH: { /* eqareanorthpole.hpp:35-41 */
        double dx = x - 0.5, dy = y - 0.5;
        double rho = sqrt(dx * dx + dy * dy) * 2;
        *lat = M_PI / 2 - (M_PI / 2 - c->circle) * rho;
        *lon = atan2(-dx, -dy);
        return;
    }
    case ORC_EQAREA_SOUTH: { /* eqareasouthpole.hpp:34-40 */
        double dx = x - 0.5, dy = y - 0.5;
        double rho = sqrt(dx * dx + dy * dy) * 2;
        *lat = -M_PI / 2 + (c->circle + M_PI / 2) * rho;
        *lon = atan2(dx, -dy);
        return;
    }
    default:
        equirect_i2o(c, x, y, lon, lat);
    }
}

static void cubic_face_to_img(int index, double x, double y, double* ox, double* oy) {
    double rx = (index % 3) * 1.0 / 3.0, ry = (index / 3) * 1.0 / 2.0;
    rx += (x + 1.0) / 2.0 / 3.0;
    ry += (y + 1.0) / 2.0 / 2.0;
    *ox = rx; *oy = ry;
}

/* The eqarea models' obj_to_image_single, each its own function as in the reference (one sin / cos
 * pair of one argument per function: gcc builds each pair as one sincos call there). */
__attribute__((noinline)) static void eqarea_north_o2i(const orc_camera* c, double lon, double lat, double* ox,
                                                       double* oy) { /* eqareanorthpole.hpp:24-33 */
    if (lat < c->circle) { *ox = *oy = NAN; return; }
    double rho = (M_PI / 2 - lat) / (M_PI / 2 - c->circle);
    *ox = -rho * sin(lon) / 2 + 0.5;
    *oy = -rho * cos(lon) / 2 + 0.5;
}
__attribute__((noinline)) static void eqarea_south_o2i(const orc_camera* c, double lon, double lat, double* ox,
                                                       double* oy) { /* eqareasouthpole.hpp:23-32 */
    if (lat > c->circle) { *ox = *oy = NAN; return; }
    double rho = (lat + M_PI / 2) / (c->circle + M_PI / 2);
    *ox = rho * sin(lon) / 2 + 0.5;
    *oy = -rho * cos(lon) / 2 + 0.5;
}

/* obj_to_image_single of the non-fisheye input camera types. */
__attribute__((noinline)) static void obj_to_image_single(const orc_camera* c, double lon, double lat, double* ox, double* oy) {
    double p[3];
    switch (c->type) {
    case ORC_FULLFRAME_FISHEYE:
        ffisheye_o2i(c, lon, lat, ox, oy);
        return;
    case ORC_NORMAL: { /* normal.cpp:32-39 */
        lonlat_to_xyz(lon, lat, p);
        if (p[0] < 0) { *ox = *oy = NAN; return; }
        double div = p[0] / c->cam_x;
        p[0] = p[0] / div; p[1] = p[1] / div; p[2] = p[2] / div;
        *ox = (c->cam_z - p[2]) / 2.0 / c->cam_z;
        *oy = (c->cam_y - p[1]) / 2.0 / c->cam_y;
        return;
    }
    case ORC_PERSPECTIVE: { /* perspective.cpp:28-33 */
        lonlat_to_xyz(lon, lat, p);
        double y_ = p[1] * (1.0 / c->sf / p[0]);
        double z_ = p[2] * (1.0 / c->sf / p[0]);
        *ox = 0.5 - z_ / c->aspect;
        *oy = 0.5 - y_;
        return;
    }
    case ORC_OCAM: { /* ocam_fisheye.cpp:227-235 */
        lonlat_to_xyz(lon, lat, p);
        double p3[3] = {-p[1], -p[2], -p[0]}, p2[2];
        ocam_world2cam(c, p3, p2);
        *ox = p2[1] / c->width;
        *oy = p2[0] / c->height;
        return;
    }
    case ORC_STUPIDOVAL: /* stupidoval.hpp:24-29 */
        *ox = cos(lat) * lon / (M_PI * 2.0) + 0.5;
        *oy = -lat / M_PI + 0.5;
        return;
    case ORC_CUBIC: { /* cubic.hpp:47-84 */
        lonlat_to_xyz(lon, lat, p);
        double sp[3], f;
#define WITHIN(a, b) ((a) >= -1.0 && (a) <= 1.0 && (b) >= -1.0 && (b) <= 1.0)
        if (fabs(p[0]) > 1e-2) {
            f = fabs(p[0]);
            sp[0] = p[0] / f; sp[1] = p[1] / f; sp[2] = p[2] / f;
            if (WITHIN(sp[1], sp[2])) {
                if (sp[0] < 0) cubic_face_to_img(1, -sp[2], sp[1], ox, oy);
                else cubic_face_to_img(0, sp[2], sp[1], ox, oy);
                return;
            }
        }
        if (fabs(p[2]) > 1e-2) {
            f = fabs(p[2]);
            sp[0] = p[0] / f; sp[1] = p[1] / f; sp[2] = p[2] / f;
            if (WITHIN(sp[0], sp[1])) {
                if (sp[2] < 0) cubic_face_to_img(4, sp[0], sp[1], ox, oy);
                else cubic_face_to_img(5, -sp[0], sp[1], ox, oy);
                return;
            }
        }
        if (fabs(p[1]) > 1e-2) {
            f = fabs(p[1]);
            sp[0] = p[0] / f; sp[1] = p[1] / f; sp[2] = p[2] / f;
            if (WITHIN(sp[0], sp[2])) {
                if (sp[1] < 0) cubic_face_to_img(2, sp[0], -sp[2], ox, oy);
                else cubic_face_to_img(3, sp[0], sp[2], ox, oy);
                return;
            }
        }
#undef WITHIN
        *ox = *oy = NAN;
        return;
    }
    case ORC_EQAREA_NORTH:
        eqarea_north_o2i(c, lon, lat, ox, oy);
        return;
    case ORC_EQAREA_SOUTH:
        eqarea_south_o2i(c, lon, lat, ox, oy);
        return;
    default:
        equirect_o2i(c, lon, lat, ox, oy);
    }
}

/* One output pixel through out->image_to_obj then in->obj_to_image (camera.cpp:212-253, 296-315). */
/* vis (optional): Camera::get_include_mask for the pixel (camera.cpp:255-294) -- the same projection
 * without the longitude / exclude tests, then include_mask.at(int(y*rows), int(x*cols)); it is only
 * consulted when exclude_mask is non-empty too (camera.cpp:281). */
static void project_pixel_vis(const orc_camera* out, const orc_camera* in, double u, double v, double* x, double* y,
                              int* vis);
static void project_pixel(const orc_camera* out, const orc_camera* in, double u, double v, double* x, double* y) {
    project_pixel_vis(out, in, u, v, x, y, NULL);
}
static void project_pixel_vis(const orc_camera* out, const orc_camera* in, double u, double v, double* x, double* y,
                              int* vis) {
    if (vis) *vis = 0;
    double lon, lat, p[3], q[3];
    /* output: image_to_obj */
    image_to_obj_single(out, u, v, &lon, &lat);
    lonlat_to_xyz(lon, lat, p);
    rotate(out->Rinv, p, q);
    xyz_to_lonlat(q, &lon, &lat);
    /* input: obj_to_image */
    lonlat_to_xyz(lon, lat, p);
    int lon_ok = valid_longitude(in, lon);
    rotate(in->R, p, q);
    if (in->type == ORC_FISHEYE) { /* PinholeCamera::obj_to_image overrides the base (no lon/excl masks) */
        fisheye_project(in, q, x, y);
        return;
    }
    if (in->type == ORC_PINHOLE) {
        pinhole_project(in, q, x, y);
        return;
    }
    double ll, la;
    xyz_to_lonlat(q, &ll, &la);
    double px = NAN, py = NAN;
    if (vis && in->excl && in->incl) {
        double qx = NAN, qy = NAN;
        obj_to_image_single(in, ll, la, &qx, &qy);
        if (qx >= 0 && qx < 1 && qy >= 0 && qy < 1)
            *vis = in->incl[(size_t)(int)(qy * in->height) * in->width + (int)(qx * in->width)] != 0;
    }
    if (lon_ok) obj_to_image_single(in, ll, la, &px, &py);
    if (px >= 0 && px < 1 && py >= 0 && py < 1 && in->excl) {  /* camera.cpp:239-246 */
        if (in->excl[(size_t)(int)(py * in->height) * in->width + (int)(px * in->width)]) px = py = NAN;
    } else if (px >= 0 && px < 1 && py >= 0 && py < 1 && in->sel) {
        /* exclude_mask.at(int(p.y * rows), int(p.x * cols)) (camera.cpp:239-246): 255 outside the
         * fillPoly'd selection rectangle [l, r-1] x [t, b-1] (camera.cpp:96-112) */
        int W = (int)(px * in->width), H = (int)(py * in->height);
        if (!(W >= in->sel_l && W <= in->sel_r - 1 && H >= in->sel_t && H <= in->sel_b - 1)) px = py = NAN;
    }
    *x = px;
    *y = py;
}

/* Camera::image_to_obj of `from` then Camera::obj_to_image of `to` (camera.cpp:212-253, 296-315), as
 * morph_controlpoints' _translate uses it (template_morph.cpp:86-90).  Returns nonzero where the
 * reference throws: fisheye / pinhole have no image_to_obj_single (camera.hpp:101-103), and
 * fullframe_fisheye's asserts a crop covering the image (fullframe_fisheye_cam.cpp:224). */
int orc_project(const orc_camera* from, const orc_camera* to, double u, double v, double* x, double* y) {
    if (from->type == ORC_FISHEYE || from->type == ORC_PINHOLE) return 1;
    if (from->type == ORC_FULLFRAME_FISHEYE &&
        !(from->crop_x == 0 && from->crop_y == 0 && from->crop_w == from->width && from->crop_h == from->height))
        return 1;
    project_pixel(from, to, u, v, x, y);
    return 0;
}

void orc_lut_rows(const orc_camera* out, const orc_camera* in, int W, int H, int y0, int y1, float* map1,
                  float* map2, uint8_t* mask) {
    for (int h = y0; h < y1; h++)
        for (int w = 0; w < W; w++) {
            double dx, dy;
            project_pixel(out, in, (double)w / W, (double)h / H, &dx, &dy);
            float x = (float)dx, y = (float)dy;
            size_t idx = (size_t)(h - y0) * W + w;
            if (isnan(x) || isnan(y) || x < 0 || x >= 1.0f || y < 0 || y >= 1.0f) {
                mask[idx] = 0;
                map1[idx] = map2[idx] = -1.0f;
            } else {
                mask[idx] = 255;
                map1[idx] = x;
                map2[idx] = y;
            }
        }
}

int orc_lut_build(const orc_camera* out, const orc_camera* in, int W, int H, float* map1, float* map2,
                  uint8_t* mask, int use_roi, int roi[4]) {
    return orc_lut_build_vis(out, in, W, H, map1, map2, mask, use_roi, roi, NULL);
}

int orc_lut_build_vis(const orc_camera* out, const orc_camera* in, int W, int H, float* map1, float* map2,
                      uint8_t* mask, int use_roi, int roi[4], uint8_t* visible) {
    int min_h = H, max_h = 0, min_w = W, max_w = 0;
    for (int h = 0; h < H; h++)
        for (int w = 0; w < W; w++) {
            double dx, dy;
            int vis = 0;
            project_pixel_vis(out, in, (double)w / W, (double)h / H, &dx, &dy, visible ? &vis : NULL);
            float x = (float)dx, y = (float)dy;
            size_t idx = (size_t)h * W + w;
            /* template.cpp:86-116: visible_mask[index] before this camera's update rejects the pixel;
             * a first claim is marked 2 for the caller to clear from the earlier cameras' masks */
            int claimed = visible && visible[idx] == 1;
            if (visible && vis && !claimed) visible[idx] = 2;
            if (isnan(x) || isnan(y) || x < 0 || x >= 1.0f || y < 0 || y >= 1.0f || claimed) {
                mask[idx] = 0;
                map1[idx] = map2[idx] = -1.0f;
            } else {
                mask[idx] = 255;
                map1[idx] = x;
                map2[idx] = y;
                if (h < min_h) min_h = h;
                if (h > max_h) max_h = h;
                if (w < min_w) min_w = w;
                if (w > max_w) max_w = w;
            }
        }
    if (!(min_h <= max_h && min_w <= max_w)) return -1; /* CV_Assert, template.cpp:124 */
    min_w = min_w - 8 > 0 ? min_w - 8 : 0;
    min_h = min_h - 8 > 0 ? min_h - 8 : 0;
    max_w = max_w + 8 < W - 1 ? max_w + 8 : W - 1;
    max_h = max_h + 8 < H - 1 ? max_h + 8 : H - 1;
    if (use_roi) {
        roi[0] = min_w; roi[1] = min_h; roi[2] = max_w + 1 - min_w; roi[3] = max_h + 1 - min_h;
    } else {
        roi[0] = 0; roi[1] = 0; roi[2] = W; roi[3] = H;
    }
    return 0;
}

/* ------------------------------------------------------------------------------------------ */
/* Fixed-point bilinear remap (imgproc/src/imgwarp.cpp)                                        */
/* ------------------------------------------------------------------------------------------ */
static short sat_s16_f(float v) {
    int iv = (int)lrintf(v);
    return (short)(iv < -32768 ? -32768 : iv > 32767 ? 32767 : iv);
}

void orc_bilinear_tab(int16_t out[1024 * 4]) {
    /* initInterTab1D(INTER_LINEAR): coeffs {1-x, x}, x = i*(1/32) (imgwarp.cpp:146-150, 188-195) */
    float tab1[32 * 2];
    float scale = 1.f / 32;
    for (int i = 0; i < 32; i++) { tab1[i * 2] = 1.f - i * scale; tab1[i * 2 + 1] = i * scale; }
    /* flat table with slack: the sum fix-up of the last cell reads past the end (imgwarp.cpp:249-264) */
    static short itab_buf[1024 * 4 + 8];
    short* itab = itab_buf;
    memset(itab_buf, 0, sizeof itab_buf);
    const int ksize = 2;
    for (int i = 0; i < 32; i++)
        for (int j = 0; j < 32; j++, itab += ksize * ksize) {
            int isum = 0;
            for (int k1 = 0; k1 < ksize; k1++) {
                float vy = tab1[i * ksize + k1];
                for (int k2 = 0; k2 < ksize; k2++) {
                    float v = vy * tab1[j * ksize + k2];
                    isum += itab[k1 * ksize + k2] = sat_s16_f(v * 32768);
                }
            }
            if (isum != 32768) {
                int diff = isum - 32768;
                int ksize2 = ksize / 2, Mk1 = ksize2, Mk2 = ksize2, mk1 = ksize2, mk2 = ksize2;
                for (int k1 = ksize2; k1 < ksize2 + 2; k1++)
                    for (int k2 = ksize2; k2 < ksize2 + 2; k2++) {
                        if (itab[k1 * ksize + k2] < itab[mk1 * ksize + mk2]) mk1 = k1, mk2 = k2;
                        else if (itab[k1 * ksize + k2] > itab[Mk1 * ksize + Mk2]) Mk1 = k1, Mk2 = k2;
                    }
                if (diff < 0) itab[Mk1 * ksize + Mk2] = (short)(itab[Mk1 * ksize + Mk2] - diff);
                else itab[mk1 * ksize + mk2] = (short)(itab[mk1 * ksize + mk2] - diff);
            }
        }
    memcpy(out, itab_buf, 1024 * 4 * sizeof(short));
}

static int16_t g_tab[1024 * 4];
static pthread_once_t g_tab_once = PTHREAD_ONCE_INIT;
static void init_tab(void) { orc_bilinear_tab(g_tab); }

static inline int round_half_even_f(float v) { return (int)lrintf(v); }
static inline short sat_s16_i(int v) { return (short)(v < -32768 ? -32768 : v > 32767 ? 32767 : v); }

void orc_remap_u8(const uint8_t* src, int sw, int sh, size_t spitch, int cn, const float* map1, const float* map2,
                  int mw, int mh, size_t mpitch, float scale_x, float scale_y, uint8_t* dst, size_t dpitch) {
    pthread_once(&g_tab_once, init_tab);
    for (int y = 0; y < mh; y++) {
        const float* m1 = map1 + (size_t)y * mpitch;
        const float* m2 = map2 + (size_t)y * mpitch;
        uint8_t* d = dst + (size_t)y * dpitch;
        for (int x = 0; x < mw; x++) {
            float X = m1[x] * scale_x, Y = m2[x] * scale_y;
            /* _mm_cvtps_epi32: out-of-range / NaN -> INT_MIN (RemapInvoker, imgwarp.cpp:4385-4420) */
            float fx32 = X * 32.0f, fy32 = Y * 32.0f;
            int ix = (fx32 != fx32 || fx32 >= 2147483648.f || fx32 < -2147483648.f) ? INT32_MIN : round_half_even_f(fx32);
            int iy = (fy32 != fy32 || fy32 >= 2147483648.f || fy32 < -2147483648.f) ? INT32_MIN : round_half_even_f(fy32);
            int sx = sat_s16_i(ix >> 5), sy = sat_s16_i(iy >> 5);
            int a = ((iy & 31) << 5) | (ix & 31);
            const int16_t* w = g_tab + a * 4;
            for (int k = 0; k < cn; k++) {
                int v[4];
                for (int t = 0; t < 4; t++) {
                    int tx = sx + (t & 1), ty = sy + (t >> 1);
                    v[t] = (tx >= 0 && tx < sw && ty >= 0 && ty < sh) ? src[(size_t)ty * spitch + (size_t)tx * cn + k] : 0;
                }
                int acc = v[0] * w[0] + v[1] * w[1] + v[2] * w[2] + v[3] * w[3];
                int r = (acc + (1 << 14)) >> 15;
                d[(size_t)x * cn + k] = (uint8_t)(r < 0 ? 0 : r > 255 ? 255 : r);
            }
        }
    }
}

/* ------------------------------------------------------------------------------------------ */
/* YUV420 <-> RGB (own BT.601 definition; NPP's arithmetic is closed and unpinned)             */
/* ------------------------------------------------------------------------------------------ */
static inline uint8_t sat_u8_rne(float v) {
    if (!(v > 0.f)) return 0; /* also NaN */
    if (v >= 255.f) return 255;
    return (uint8_t)lrintf(v);
}

/* The library's own BT.601 colour definitions (they stand in for NPP's closed arithmetic; parity
 * with NPP is unpinned).  Fused multiply-adds, round half to even, saturate — kernels.hip uses the
 * identical operation sequence. */
static inline void yuv_px_to_rgb(int y, int u, int v, uint8_t* o) {
    float Yf = (float)y, Uf = (float)u - 128.f, Vf = (float)v - 128.f;
    o[0] = sat_u8_rne(fmaf(1.140f, Vf, Yf));
    o[1] = sat_u8_rne(fmaf(-0.581f, Vf, fmaf(-0.394f, Uf, Yf)));
    o[2] = sat_u8_rne(fmaf(2.032f, Uf, Yf));
}

/* 2x2 RGB quad -> 4 Y + 1 U + 1 V (the library's own definition, device_common.hpp quad_yuv; it
 * stands in for NPP's closed nppiRGBToYUV420, color.cpp:2306): NPP's documented BT.601 matrix,
 * Y = 0.299 R + 0.587 G + 0.114 B, U = 0.492 (B - Y) + 128, V = 0.877 (R - Y) + 128 (the inverse of
 * yuv_px_to_rgb above), in fixed point with the chroma as the quad's mean:
 *   Y = (77 R + 150 G + 29 B + 128) >> 8,
 *   U = (sum over the quad of -38 R - 74 G + 112 B, + 131584) >> 10             (16..240),
 *   V = clamp((sum over the quad of 79 R - 66 G - 13 B, + 65792) >> 9, 0, 255)
 * (each chroma vector sums to 0, so R - 128 etc. may replace R in the sums). */
static inline void rgb_quad_to_yuv(const uint8_t* const p[4], uint8_t Y[4], uint8_t* U, uint8_t* V) {
    int au = 0, av = 0;
    for (int k = 0; k < 4; k++) {
        const int R = p[k][0], G = p[k][1], B = p[k][2];
        Y[k] = (uint8_t)((77 * R + 150 * G + 29 * B + 128) >> 8);
        au += -38 * R - 74 * G + 112 * B;
        av += 79 * R - 66 * G - 13 * B;
    }
    const int v = (av + 65792) >> 9;
    *U = (uint8_t)((au + 131584) >> 10);
    *V = (uint8_t)(v < 0 ? 0 : v > 255 ? 255 : v);
}

void orc_yuv420_to_rgba(const uint8_t* yuv, int w, int h, size_t pitch, uint8_t* rgba, size_t rgba_pitch) {
    const uint8_t* U = yuv + (size_t)h * pitch;
    const uint8_t* V = U + w / 2;
    for (int y = 0; y < h; y++)
        for (int x = 0; x < w; x++) {
            uint8_t* o = rgba + (size_t)y * rgba_pitch + (size_t)x * 4;
            yuv_px_to_rgb(yuv[(size_t)y * pitch + x], U[(size_t)(y >> 1) * pitch + (x >> 1)],
                          V[(size_t)(y >> 1) * pitch + (x >> 1)], o);
            o[3] = 255;
        }
}

void orc_rgb_to_yuv420(const uint8_t* rgb, int w, int h, size_t rgb_pitch, int cn, uint8_t* yuv, size_t pitch) {
    uint8_t* Uo = yuv + (size_t)h * pitch;
    uint8_t* Vo = Uo + w / 2;
    for (int y = 0; y < h; y += 2)
        for (int x = 0; x < w; x += 2) {
            const uint8_t* p[4];
            uint8_t Yq[4];
            for (int k = 0; k < 4; k++) p[k] = rgb + (size_t)(y + (k >> 1)) * rgb_pitch + (size_t)(x + (k & 1)) * cn;
            rgb_quad_to_yuv(p, Yq, &Uo[(size_t)(y >> 1) * pitch + (x >> 1)], &Vo[(size_t)(y >> 1) * pitch + (x >> 1)]);
            for (int k = 0; k < 4; k++) yuv[(size_t)(y + (k >> 1)) * pitch + x + (k & 1)] = Yq[k];
        }
}

/* ------------------------------------------------------------------------------------------ */
/* cv::solve (core/src/lapack.cpp:1050-1275; LUImpl core/src/matrix_decomp.cpp:50-110)        */
/* ------------------------------------------------------------------------------------------ */
int orc_solve(const double* Ain, const double* bin, int n, double* x) {
#define Sd(y, xx) Ain[(y) * n + (xx)]
#define bd(y) bin[y]
    if (n == 1) {
        double d = Sd(0, 0);
        if (d == 0.) return 0;
        x[0] = bd(0) / d;
        return 1;
    }
    if (n == 2) {
        double d = (double)Sd(0, 0) * Sd(1, 1) - (double)Sd(0, 1) * Sd(1, 0);
        if (d == 0.) return 0;
        double t;
        d = 1. / d;
        t = (bd(0) * Sd(1, 1) - bd(1) * Sd(0, 1)) * d;
        x[1] = (bd(1) * Sd(0, 0) - bd(0) * Sd(1, 0)) * d;
        x[0] = t;
        return 1;
    }
    if (n == 3) {
        double d = Sd(0, 0) * ((double)Sd(1, 1) * Sd(2, 2) - (double)Sd(1, 2) * Sd(2, 1)) -
                   Sd(0, 1) * ((double)Sd(1, 0) * Sd(2, 2) - (double)Sd(1, 2) * Sd(2, 0)) +
                   Sd(0, 2) * ((double)Sd(1, 0) * Sd(2, 1) - (double)Sd(1, 1) * Sd(2, 0));
        if (d == 0.) return 0;
        d = 1. / d;
        double t0 = ((Sd(1, 1) * Sd(2, 2) - Sd(1, 2) * Sd(2, 1)) * bd(0) + (Sd(0, 2) * Sd(2, 1) - Sd(0, 1) * Sd(2, 2)) * bd(1) +
                     (Sd(0, 1) * Sd(1, 2) - Sd(0, 2) * Sd(1, 1)) * bd(2)) * d;
        double t1 = ((Sd(1, 2) * Sd(2, 0) - Sd(1, 0) * Sd(2, 2)) * bd(0) + (Sd(0, 0) * Sd(2, 2) - Sd(0, 2) * Sd(2, 0)) * bd(1) +
                     (Sd(0, 2) * Sd(1, 0) - Sd(0, 0) * Sd(1, 2)) * bd(2)) * d;
        double t2 = ((Sd(1, 0) * Sd(2, 1) - Sd(1, 1) * Sd(2, 0)) * bd(0) + (Sd(0, 1) * Sd(2, 0) - Sd(0, 0) * Sd(2, 1)) * bd(1) +
                     (Sd(0, 0) * Sd(1, 1) - Sd(0, 1) * Sd(1, 0)) * bd(2)) * d;
        x[0] = t0; x[1] = t1; x[2] = t2;
        return 1;
    }
#undef Sd
#undef bd
    double* A = (double*)malloc(sizeof(double) * n * n);
    memcpy(A, Ain, sizeof(double) * n * n);
    memcpy(x, bin, sizeof(double) * n);
    double* b = x;
    int i, j, k, m = n;
    const double eps = DBL_EPSILON * 100;
    for (i = 0; i < m; i++) {
        k = i;
        for (j = i + 1; j < m; j++)
            if (fabs(A[j * m + i]) > fabs(A[k * m + i])) k = j;
        if (fabs(A[k * m + i]) < eps) { free(A); return 0; }
        if (k != i) {
            for (j = i; j < m; j++) { double t = A[i * m + j]; A[i * m + j] = A[k * m + j]; A[k * m + j] = t; }
            double t = b[i]; b[i] = b[k]; b[k] = t;
        }
        double d = -1 / A[i * m + i];
        for (j = i + 1; j < m; j++) {
            double alpha = A[j * m + i] * d;
            for (k = i + 1; k < m; k++) A[j * m + k] += alpha * A[i * m + k];
            b[j] += alpha * b[i];
        }
        A[i * m + i] = -d;
    }
    for (i = m - 1; i >= 0; i--) {
        double s = b[i];
        for (k = i + 1; k < m; k++) s -= A[i * m + k] * b[k];
        b[i] = s * A[i * m + i];
    }
    free(A);
    return 1;
}

/* ------------------------------------------------------------------------------------------ */
/* CUDA resize kernels used on the gain path (cudawarping/src/cuda/resize.cu:57-103)            */
/* ------------------------------------------------------------------------------------------ */
static float resize_inv_scale(int d, int s) {
    /* resize.cpp:82-83,105: fx = double(dsize)/src ; kernel gets (float)(1.0/fx) */
    double f = (double)d / s;
    return (float)(1.0 / f);
}

void orc_resize_nearest_u8(const uint8_t* src, int sw, int sh, size_t spitch, int cn, uint8_t* dst, int dw, int dh,
                           size_t dpitch) {
    float fx = resize_inv_scale(dw, sw), fy = resize_inv_scale(dh, sh);
    (void)sh;
    for (int y = 0; y < dh; y++)
        for (int x = 0; x < dw; x++) {
            float sxf = x * fx, syf = y * fy;
            int sx = (int)sxf, sy = (int)syf; /* __float2int_rz */
            memcpy(dst + (size_t)y * dpitch + (size_t)x * cn, src + (size_t)sy * spitch + (size_t)sx * cn, cn);
        }
}

/* resize_linear (resize.cu:71-103). nvcc contracts `out + src*w` into fmaf by default (-fmad=true);
 * restated with explicit fmaf. */
void orc_resize_linear_cuda_u8(const uint8_t* src, int sw, int sh, size_t spitch, uint8_t* dst, int dw, int dh,
                               size_t dpitch) {
    float fx = resize_inv_scale(dw, sw), fy = resize_inv_scale(dh, sh);
    for (int y = 0; y < dh; y++)
        for (int x = 0; x < dw; x++) {
            float src_x = x * fx, src_y = y * fy;
            int x1 = (int)floorf(src_x), y1 = (int)floorf(src_y);
            int x2 = x1 + 1, y2 = y1 + 1;
            int x2r = x2 < sw - 1 ? x2 : sw - 1, y2r = y2 < sh - 1 ? y2 : sh - 1;
            float out = 0.f;
            out = fmaf((float)src[(size_t)y1 * spitch + x1], (x2 - src_x) * (y2 - src_y), out);
            out = fmaf((float)src[(size_t)y1 * spitch + x2r], (src_x - x1) * (y2 - src_y), out);
            out = fmaf((float)src[(size_t)y2r * spitch + x1], (x2 - src_x) * (src_y - y1), out);
            out = fmaf((float)src[(size_t)y2r * spitch + x2r], (src_x - x1) * (src_y - y1), out);
            dst[(size_t)y * dpitch + x] = sat_u8_rne(out);
        }
}

void orc_resize_linear_cuda_u8c(const uint8_t* src, int sw, int sh, size_t spitch, int cn, uint8_t* dst, int dw,
                                int dh, size_t dpitch) {
    float fx = resize_inv_scale(dw, sw), fy = resize_inv_scale(dh, sh);
    for (int y = 0; y < dh; y++)
        for (int x = 0; x < dw; x++) {
            float src_x = x * fx, src_y = y * fy;
            int x1 = (int)floorf(src_x), y1 = (int)floorf(src_y);
            int x2 = x1 + 1, y2 = y1 + 1;
            int x2r = x2 < sw - 1 ? x2 : sw - 1, y2r = y2 < sh - 1 ? y2 : sh - 1;
            float w00 = (x2 - src_x) * (y2 - src_y), w01 = (src_x - x1) * (y2 - src_y);
            float w10 = (x2 - src_x) * (src_y - y1), w11 = (src_x - x1) * (src_y - y1);
            for (int c = 0; c < cn; c++) {
                float out = 0.f;
                out = fmaf((float)src[(size_t)y1 * spitch + (size_t)x1 * cn + c], w00, out);
                out = fmaf((float)src[(size_t)y1 * spitch + (size_t)x2r * cn + c], w01, out);
                out = fmaf((float)src[(size_t)y2r * spitch + (size_t)x1 * cn + c], w10, out);
                out = fmaf((float)src[(size_t)y2r * spitch + (size_t)x2r * cn + c], w11, out);
                dst[(size_t)y * dpitch + (size_t)x * cn + c] = sat_u8_rne(out);
            }
        }
}

/* ------------------------------------------------------------------------------------------ */
/* Gain compensator (stitching/src/exposure_compensate.cpp:174-297; mapper.cpp:94-114)         */
/* ------------------------------------------------------------------------------------------ */
static void working_scale(int out_w, int out_h, double* ws) {
    double s = sqrt(0.1 * 1e6 / ((double)out_w * out_h)); /* WORKING_MEGAPIX, mapper.cpp:43,94 */
    *ws = s < 1.0 ? s : 1.0;
}

int orc_gain_feed(int n, const int* rois, const uint8_t* const* warped, const uint8_t* const* masks, int out_w,
                  int out_h, double* gains) {
    double ws;
    working_scale(out_w, out_h, &ws);
    int* wr = (int*)malloc(sizeof(int) * 4 * n);
    uint8_t** smask = (uint8_t**)malloc(sizeof(void*) * n);
    uint8_t** simg = (uint8_t**)malloc(sizeof(void*) * n);
    float** norm = (float**)malloc(sizeof(void*) * n);
    for (int i = 0; i < n; i++) {
        const int* r = rois + 4 * i;
        wr[4 * i + 0] = (int)(r[0] * ws);
        wr[4 * i + 1] = (int)(r[1] * ws);
        wr[4 * i + 2] = (int)(r[2] * ws);
        wr[4 * i + 3] = (int)(r[3] * ws);
        int w = wr[4 * i + 2], h = wr[4 * i + 3];
        smask[i] = (uint8_t*)malloc((size_t)w * h + 1);
        simg[i] = (uint8_t*)malloc((size_t)w * h * 4 + 1);
        norm[i] = (float*)malloc(sizeof(float) * ((size_t)w * h + 1));
        orc_resize_linear_cuda_u8(masks[i], r[2], r[3], r[2], smask[i], w, h, w);
        orc_resize_nearest_u8(warped[i], r[2], r[3], (size_t)r[2] * 4, 4, simg[i], w, h, (size_t)w * 4);
        for (size_t k = 0; k < (size_t)w * h; k++) {
            const uint8_t* p = simg[i] + 4 * k;
            int s = p[0] * p[0] + p[1] * p[1] + p[2] * p[2];
            norm[i][k] = sqrtf((float)s);
        }
    }
    int* N = (int*)calloc((size_t)n * n, sizeof(int));
    double* I = (double*)calloc((size_t)n * n, sizeof(double));
    for (int i = 0; i < n; i++) {
        int w = wr[4 * i + 2], h = wr[4 * i + 3], nz = 0;
        for (size_t k = 0; k < (size_t)w * h; k++) nz += smask[i][k] != 0;
        N[i * n + i] = nz > 1 ? nz : 1;
    }
    for (int i = 0; i < n; i++)
        for (int j = i + 1; j < n; j++) {
            const int *a = wr + 4 * i, *b = wr + 4 * j;
            int x0 = a[0] > b[0] ? a[0] : b[0], y0 = a[1] > b[1] ? a[1] : b[1];
            int x1 = (a[0] + a[2]) < (b[0] + b[2]) ? (a[0] + a[2]) : (b[0] + b[2]);
            int y1 = (a[1] + a[3]) < (b[1] + b[3]) ? (a[1] + a[3]) : (b[1] + b[3]);
            int ow = x1 - x0, oh = y1 - y0;
            if (ow <= 0 || oh <= 0) { /* cv::Rect & -> empty */
                N[i * n + j] = N[j * n + i] = 1;
                I[i * n + j] = I[j * n + i] = 0;
                continue;
            }
            int nz = 0;
            double s1 = 0, s2 = 0;
            for (int yy = 0; yy < oh; yy++)
                for (int xx = 0; xx < ow; xx++) {
                    size_t ka = (size_t)(y0 + yy - a[1]) * a[2] + (x0 + xx - a[0]);
                    size_t kb = (size_t)(y0 + yy - b[1]) * b[2] + (x0 + xx - b[0]);
                    if ((smask[i][ka] & smask[j][kb]) != 0) {
                        nz++;
                        s1 += norm[i][ka];
                        s2 += norm[j][kb];
                    }
                }
            int nn = nz > 1 ? nz : 1;
            N[i * n + j] = N[j * n + i] = nn;
            I[i * n + j] = s1 / nn;
            I[j * n + i] = s2 / nn;
        }
    double alpha = 0.01, beta = 100;
    double* A = (double*)calloc((size_t)n * n, sizeof(double));
    double* bb = (double*)calloc((size_t)n, sizeof(double));
    for (int i = 0; i < n; i++)
        for (int j = 0; j < n; j++) {
            bb[i] += beta * N[i * n + j];
            A[i * n + i] += beta * N[i * n + j];
            if (j == i) continue;
            A[i * n + i] += 2 * alpha * I[i * n + j] * I[i * n + j] * N[i * n + j];
            A[i * n + j] -= 2 * alpha * I[i * n + j] * I[j * n + i] * N[i * n + j];
        }
    int ok = orc_solve(A, bb, n, gains);
    for (int i = 0; i < n; i++) { free(smask[i]); free(simg[i]); free(norm[i]); }
    free(smask); free(simg); free(norm); free(wr); free(N); free(I); free(A); free(bb);
    return ok ? 0 : -1;
}

/* ------------------------------------------------------------------------------------------ */
/* One Mapper::stitch frame, blend = 0 (mapper.cpp:193-312)                                    */
/* ------------------------------------------------------------------------------------------ */
/* Minimal row-parallel helper: fn(ctx, y0, y1) over [0, rows) split into T contiguous bands. */
typedef void (*row_fn)(void* ctx, int y0, int y1);
typedef struct { row_fn fn; void* ctx; int y0, y1; } row_job;
static void* row_worker(void* a) { row_job* j = (row_job*)a; j->fn(j->ctx, j->y0, j->y1); return NULL; }
static void parallel_rows(int T, int y0, int y1, row_fn fn, void* ctx) {
    int rows = y1 - y0;
    if (rows <= 0) return;
    if (T > 64) T = 64;
    if (T > rows) T = rows;
    if (T <= 1) { fn(ctx, y0, y1); return; }
    pthread_t th[64];
    row_job jobs[64];
    for (int t = 0; t < T; t++) {
        jobs[t].fn = fn; jobs[t].ctx = ctx;
        jobs[t].y0 = y0 + (int)((long)rows * t / T);
        jobs[t].y1 = y0 + (int)((long)rows * (t + 1) / T);
        pthread_create(&th[t], NULL, row_worker, &jobs[t]);
    }
    for (int t = 0; t < T; t++) pthread_join(th[t], NULL);
}

/* orc_lut_build_vis on T threads (row bands): every pixel's computation and the visible_mask update
 * are per pixel, so the result equals the serial build's; the bands' bounding boxes are merged. */
typedef struct {
    const orc_camera *out, *in;
    int W, H;
    float *map1, *map2;
    uint8_t *mask, *visible;
    int bb[64][4];
    int next;
    pthread_mutex_t mu;
} lut_mt_ctx;

static void lut_mt_rows(void* a, int y0, int y1) {
    lut_mt_ctx* c = (lut_mt_ctx*)a;
    int min_h = c->H, max_h = 0, min_w = c->W, max_w = 0;
    for (int h = y0; h < y1; h++)
        for (int w = 0; w < c->W; w++) {
            double dx, dy;
            int vis = 0;
            project_pixel_vis(c->out, c->in, (double)w / c->W, (double)h / c->H, &dx, &dy, c->visible ? &vis : NULL);
            float x = (float)dx, y = (float)dy;
            size_t idx = (size_t)h * c->W + w;
            int claimed = c->visible && c->visible[idx] == 1;
            if (c->visible && vis && !claimed) c->visible[idx] = 2;
            if (isnan(x) || isnan(y) || x < 0 || x >= 1.0f || y < 0 || y >= 1.0f || claimed) {
                c->mask[idx] = 0;
                c->map1[idx] = c->map2[idx] = -1.0f;
            } else {
                c->mask[idx] = 255;
                c->map1[idx] = x;
                c->map2[idx] = y;
                if (h < min_h) min_h = h;
                if (h > max_h) max_h = h;
                if (w < min_w) min_w = w;
                if (w > max_w) max_w = w;
            }
        }
    pthread_mutex_lock(&c->mu);
    int k = c->next++;
    c->bb[k][0] = min_w; c->bb[k][1] = min_h; c->bb[k][2] = max_w; c->bb[k][3] = max_h;
    pthread_mutex_unlock(&c->mu);
}

int orc_lut_build_vis_mt(const orc_camera* out, const orc_camera* in, int W, int H, float* map1, float* map2,
                         uint8_t* mask, int use_roi, int roi[4], uint8_t* visible, int threads) {
    lut_mt_ctx c;
    memset(&c, 0, sizeof c);
    c.out = out; c.in = in; c.W = W; c.H = H;
    c.map1 = map1; c.map2 = map2; c.mask = mask; c.visible = visible;
    pthread_mutex_init(&c.mu, NULL);
    parallel_rows(threads, 0, H, lut_mt_rows, &c);
    pthread_mutex_destroy(&c.mu);
    int min_h = H, max_h = 0, min_w = W, max_w = 0;
    for (int k = 0; k < c.next; k++) {
        if (c.bb[k][1] > c.bb[k][3] || c.bb[k][0] > c.bb[k][2]) continue;  /* a band without valid pixels */
        if (c.bb[k][0] < min_w) min_w = c.bb[k][0];
        if (c.bb[k][1] < min_h) min_h = c.bb[k][1];
        if (c.bb[k][2] > max_w) max_w = c.bb[k][2];
        if (c.bb[k][3] > max_h) max_h = c.bb[k][3];
    }
    if (!(min_h <= max_h && min_w <= max_w)) return -1; /* CV_Assert, template.cpp:124 */
    min_w = min_w - 8 > 0 ? min_w - 8 : 0;
    min_h = min_h - 8 > 0 ? min_h - 8 : 0;
    max_w = max_w + 8 < W - 1 ? max_w + 8 : W - 1;
    max_h = max_h + 8 < H - 1 ? max_h + 8 : H - 1;
    if (use_roi) {
        roi[0] = min_w; roi[1] = min_h; roi[2] = max_w + 1 - min_w; roi[3] = max_h + 1 - min_h;
    } else {
        roi[0] = 0; roi[1] = 0; roi[2] = W; roi[3] = H;
    }
    return 0;
}

/* The FP64 (x, y) of Camera::obj_to_image for output rows [y0, y1) (template.cpp:70-83), before the
 * f32 rounding; T threads. */
typedef struct {
    const orc_camera *out, *in;
    int W, H, y0;
    double *x, *y;
} proj_ctx;
static void proj_rows(void* a, int y0, int y1) {
    proj_ctx* c = (proj_ctx*)a;
    for (int h = y0; h < y1; h++)
        for (int w = 0; w < c->W; w++) {
            size_t idx = (size_t)(h - c->y0) * c->W + w;
            project_pixel(c->out, c->in, (double)w / c->W, (double)h / c->H, &c->x[idx], &c->y[idx]);
        }
}
void orc_project_f64(const orc_camera* out, const orc_camera* in, int W, int H, int y0, int y1, double* x, double* y,
                     int threads) {
    proj_ctx c = {out, in, W, H, y0, x, y};
    parallel_rows(threads, y0, y1, proj_rows, &c);
}

typedef struct {
    const orc_frame* f;
    int cam;
    uint8_t* rgba;
    uint8_t* warped;
    float gain;
    uint8_t* result;
    int rb, re;
} stage_ctx;

static void yuv_rows(void* c, int y0, int y1) {
    stage_ctx* s = (stage_ctx*)c;
    const orc_frame* f = s->f;
    int i = s->cam, w = f->in_w[i], h = f->in_h[i];
    size_t pitch = f->in_pitch[i];
    const uint8_t* yuv = f->in_yuv[i];
    const uint8_t* U = yuv + (size_t)h * pitch;
    const uint8_t* V = U + w / 2;
    for (int y = y0; y < y1; y++)
        for (int x = 0; x < w; x++) {
            uint8_t* o = s->rgba + ((size_t)y * w + x) * 4;
            yuv_px_to_rgb(yuv[(size_t)y * pitch + x], U[(size_t)(y >> 1) * pitch + (x >> 1)],
                          V[(size_t)(y >> 1) * pitch + (x >> 1)], o);
            o[3] = 255;
            if (f->vig && f->vig[i]) { /* multiply(rgba, vignette) = MulOpSpecial_c4 (mul_mat.cu:198-214) */
                const float g = f->vig[i][(size_t)y * w + x];
                for (int ch = 0; ch < 4; ch++) o[ch] = sat_u8_rne((float)o[ch] * g);
            }
        }
}

static void remap_rows(void* c, int y0, int y1) {
    stage_ctx* s = (stage_ctx*)c;
    const orc_frame* f = s->f;
    int i = s->cam;
    const int* r = f->rois + 4 * i;
    if (f->remap_tex) { /* the reference's live CUDA path: fastRemap through the texture (A12 model) */
        orc_fast_remap_tex_rgba(s->rgba, f->in_w[i], f->in_h[i], (size_t)f->in_w[i] * 4, f->map1[i] + (size_t)y0 * r[2],
                                f->map2[i] + (size_t)y0 * r[2], r[2], y1 - y0, r[2],
                                s->warped + (size_t)y0 * r[2] * 4, (size_t)r[2] * 4);
        return;
    }
    orc_remap_u8(s->rgba, f->in_w[i], f->in_h[i], (size_t)f->in_w[i] * 4, 4, f->map1[i] + (size_t)y0 * r[2],
                 f->map2[i] + (size_t)y0 * r[2], r[2], y1 - y0, r[2], (float)f->in_w[i], (float)f->in_h[i],
                 s->warped + (size_t)y0 * r[2] * 4, (size_t)r[2] * 4);
}

/* mul_scalar_with_mask (stitching/src/cuda/exposure_compensate.cu:15-30) */
static void gain_rows(void* c, int y0, int y1) {
    stage_ctx* s = (stage_ctx*)c;
    const orc_frame* f = s->f;
    const int* r = f->rois + 4 * s->cam;
    for (size_t k = (size_t)y0 * r[2]; k < (size_t)y1 * r[2]; k++) {
        if (f->masks[s->cam][k] == 0) continue;
        uint8_t* p = s->warped + 4 * k;
        for (int ch = 0; ch < 4; ch++) p[ch] = sat_u8_rne((float)p[ch] * s->gain);
    }
}

/* RGBA2RGB + copyTo(result(roi), mask) (mapper.cpp:268-277) */
static void copy_rows(void* c, int y0, int y1) {
    stage_ctx* s = (stage_ctx*)c;
    const orc_frame* f = s->f;
    const int* r = f->rois + 4 * s->cam;
    size_t W = (size_t)f->out_w;
    for (int y = y0; y < y1; y++) {
        int oy = r[1] + y;
        if (oy < s->rb || oy >= s->re) continue;
        for (int x = 0; x < r[2]; x++) {
            size_t k = (size_t)y * r[2] + x;
            if (f->masks[s->cam][k] == 0) continue;
            uint8_t* o = s->result + ((size_t)oy * W + r[0] + x) * 3;
            const uint8_t* p = s->warped + 4 * k;
            o[0] = p[0]; o[1] = p[1]; o[2] = p[2];
        }
    }
}

/* own RGB -> YUV420P definition; rows [y0, y1) are quad rows (2 output rows each) */
static void out_rows(void* c, int q0, int q1) {
    stage_ctx* s = (stage_ctx*)c;
    const orc_frame* f = s->f;
    size_t W = (size_t)f->out_w;
    uint8_t* Uo = f->out_yuv + (size_t)f->out_h * f->out_pitch;
    uint8_t* Vo = Uo + f->out_w / 2;
    for (int q = q0; q < q1; q++) {
        int y = 2 * q;
        for (int x = 0; x < f->out_w; x += 2) {
            const uint8_t* p[4];
            uint8_t Yq[4];
            for (int k = 0; k < 4; k++) p[k] = s->result + ((size_t)(y + (k >> 1)) * W + x + (k & 1)) * 3;
            rgb_quad_to_yuv(p, Yq, &Uo[(size_t)q * f->out_pitch + (x >> 1)], &Vo[(size_t)q * f->out_pitch + (x >> 1)]);
            for (int k = 0; k < 4; k++) f->out_yuv[(size_t)(y + (k >> 1)) * f->out_pitch + x + (k & 1)] = Yq[k];
        }
    }
}

int orc_stitch_frame(const orc_frame* f) {
    int n = f->n;
    int T = f->threads > 0 ? f->threads : 1;
    int rb = f->row_begin, re = f->row_end;
    if (re <= rb) { rb = 0; re = f->out_h; }
    rb &= ~1;
    re = (re + 1) & ~1;
    if (re > f->out_h) re = f->out_h;
    uint8_t** warped = (uint8_t**)calloc(n, sizeof(void*));
    int estimate = f->enable_gain && !f->gains_in && n > 1;
    for (int i = 0; i < n; i++) {
        const int* r = f->rois + 4 * i;
        stage_ctx c = {f, i, NULL, NULL, 1.f, NULL, rb, re};
        c.rgba = (uint8_t*)malloc((size_t)f->in_w[i] * f->in_h[i] * 4);
        warped[i] = c.warped = (uint8_t*)calloc((size_t)r[2] * r[3] * 4, 1);
        parallel_rows(T, 0, f->in_h[i], yuv_rows, &c);
        /* ROI rows the output band needs (all rows when the feed needs whole warped images) */
        int y0 = 0, y1 = r[3];
        if (!estimate && f->blend == 0) {
            y0 = rb - r[1]; y1 = re - r[1];
            if (y0 < 0) y0 = 0;
            if (y1 > r[3]) y1 = r[3];
            if (y1 < y0) y1 = y0;
        }
        parallel_rows(T, y0, y1, remap_rows, &c);
        free(c.rgba);
    }
    double* gains = (double*)malloc(sizeof(double) * n);
    int use_gain = f->enable_gain && n > 1; /* mapper.cpp:78-82 */
    if (use_gain) {
        if (f->gains_in) memcpy(gains, f->gains_in, sizeof(double) * n);
        else if (orc_gain_feed(n, f->rois, (const uint8_t* const*)warped, f->masks, f->out_w, f->out_h, gains) != 0)
            for (int i = 0; i < n; i++) gains[i] = 1.0; /* cv::solve failure leaves gains_ undefined; use 1 */
        for (int i = 0; i < n; i++) {
            const int* r = f->rois + 4 * i;
            stage_ctx c = {f, i, NULL, warped[i], (float)gains[i], NULL, rb, re};
            parallel_rows(T, 0, r[3], gain_rows, &c);
        }
    } else {
        for (int i = 0; i < n; i++) gains[i] = 1.0;
    }
    if (f->gains_out) memcpy(f->gains_out, gains, sizeof(double) * n);
    /* result = 0 (mapper.cpp:153-156); blend (mapper.cpp:266-278): a blender over the warped
     * images, or the copy chain in camera order */
    uint8_t* result = (uint8_t*)calloc((size_t)f->out_w * f->out_h * 3, 1);
    const int blend = n > 1 ? f->blend : 0; /* mapper.cpp:78-82 */
    int rc = 0;
    if (blend > 0) {
        rc = orc_multiband_blend(n, f->rois, f->seams, (const uint8_t* const*)warped, orc_blend_bands(blend), result,
                                 f->out_w, f->out_h, (size_t)f->out_w * 3, T);
    } else if (blend < 0) {
        rc = orc_feather_blend(n, f->rois, f->masks, (const uint8_t* const*)warped, -blend, result, f->out_w, f->out_h,
                               (size_t)f->out_w * 3);
    } else {
        for (int i = 0; i < n; i++) {
            const int* r = f->rois + 4 * i;
            stage_ctx c = {f, i, NULL, warped[i], 1.f, result, rb, re};
            parallel_rows(T, 0, r[3], copy_rows, &c);
        }
    }
    if (f->scale_w > 0 && (f->scale_w != f->out_w || f->scale_h != f->out_h)) {
        /* cuda::resize(result, result_scaled, scaled_output_size, INTER_LINEAR) + RGB -> YUV420P (mapper.cpp:290-306) */
        uint8_t* scaled = (uint8_t*)malloc((size_t)f->scale_w * f->scale_h * 3);
        orc_resize_linear_cuda_u8c(result, f->out_w, f->out_h, (size_t)f->out_w * 3, 3, scaled, f->scale_w, f->scale_h,
                                   (size_t)f->scale_w * 3);
        orc_frame g = *f;
        g.out_w = f->scale_w;
        g.out_h = f->scale_h;
        stage_ctx c = {&g, 0, NULL, NULL, 1.f, scaled, 0, f->scale_h};
        parallel_rows(T, 0, f->scale_h / 2, out_rows, &c);
        free(scaled);
    } else {
        stage_ctx c = {f, 0, NULL, NULL, 1.f, result, rb, re};
        parallel_rows(T, rb / 2, re / 2, out_rows, &c);
    }
    if (f->preview && f->preview_w > 0 && f->preview_h > 0)  /* mapper.cpp:308-312 */
        orc_resize_linear_cuda_u8c(result, f->out_w, f->out_h, (size_t)f->out_w * 3, 3, f->preview, f->preview_w,
                                   f->preview_h, f->preview_pitch);
    for (int i = 0; i < n; i++) free(warped[i]);
    free(warped); free(gains); free(result);
    return rc;
}

int orc_blend_bands(int blend) { return (int)(ceil(log((double)blend) / log(2.)) - 1.); }

void orc_vignette_map(double a, double b, double c, double d, int width, int height, float* out) {
    for (int j = 0; j < height; j++)
        for (int i = 0; i < width; i++) {
            float dx = (float)(i - width / 2), dy = (float)(j - height / 2);
            float hx = (float)(width / 2), hy = (float)(height / 2);
            float r = sqrtf(dx * dx + dy * dy) / sqrtf(hx * hx + hy * hy);
            out[(size_t)j * width + i] = (float)(1.0 / (a + r * r * (b + r * r * (c + d * r * r))));
        }
}

void orc_resize_linear_cuda_f32(const float* src, int sw, int sh, float* dst, int dw, int dh) {
    float fx = resize_inv_scale(dw, sw), fy = resize_inv_scale(dh, sh);
    for (int y = 0; y < dh; y++)
        for (int x = 0; x < dw; x++) {
            float src_x = x * fx, src_y = y * fy;
            int x1 = (int)floorf(src_x), y1 = (int)floorf(src_y);
            int x2 = x1 + 1, y2 = y1 + 1;
            int x2r = x2 < sw - 1 ? x2 : sw - 1, y2r = y2 < sh - 1 ? y2 : sh - 1;
            float o = 0.f;
            o = fmaf(src[(size_t)y1 * sw + x1], (x2 - src_x) * (y2 - src_y), o);
            o = fmaf(src[(size_t)y1 * sw + x2r], (src_x - x1) * (y2 - src_y), o);
            o = fmaf(src[(size_t)y2r * sw + x1], (x2 - src_x) * (src_y - y1), o);
            o = fmaf(src[(size_t)y2r * sw + x2r], (src_x - x1) * (src_y - y1), o);
            dst[(size_t)y * dw + x] = o;
        }
}

/* ------------------------------------------------------------------------------------------ */
/* A12: CUDA fastRemap's texture bilinear (the OCTVR_REMAP_TEXTURE checker; A12 vs A13)      */
/* ------------------------------------------------------------------------------------------ */
/* fast_remap<uchar4> (cudawarping/src/cuda/fast_remap.cu:21-44) through a texture object with
 * normalized coordinates, clamp addressing, linear filtering and cudaReadModeNormalizedFloat
 * (cudev/ptr2d/texture.hpp:124-160).  The filtering is CUDA hardware behaviour, not in the reference
 * repository; modelled after the CUDA Programming Guide's "Texture Fetching" appendix: x = u W - 0.5,
 * i = floor(x), alpha = frac(x) held with 8 fractional bits (truncated here), taps clamped to the
 * image, the weighted sum of the normalized texels in f32, then saturate_cast<uchar>(v * 255) (round
 * half to even).  map1 < 0 -> 0 (fill_zero).  Test infrastructure: the checker of the product's
 * opt-in OCTVR_REMAP_TEXTURE mode (stitch_tiled_tex_kernel / tex_bilerp_f follow these semantics bit for
 * bit, tests/test_gpu_texture_mode.py, test_gpu_fullsize.py) and the measure of the default A13 path's
 * documented A12 tolerance (arithmetic contract). */
void orc_fast_remap_tex_rgba(const uint8_t* src, int w, int h, size_t spitch, const float* map1, const float* map2,
                             int mw, int mh, size_t mpitch, uint8_t* dst, size_t dpitch) {
    for (int y = 0; y < mh; y++)
        for (int x = 0; x < mw; x++) {
            float u = map1[(size_t)y * mpitch + x], v = map2[(size_t)y * mpitch + x];
            uint8_t* o = dst + (size_t)y * dpitch + (size_t)x * 4;
            float xb = u * (float)w - 0.5f, yb = v * (float)h - 0.5f;
            /* u < 0: fill_zero; NaN / infinite coordinates give NaN weights, i.e. 0 in every channel */
            if (!(u >= 0) || !(fabsf(xb) <= 3.0e38f) || !(fabsf(yb) <= 3.0e38f)) { o[0] = o[1] = o[2] = o[3] = 0; continue; }
            float fx = floorf(xb), fy = floorf(yb);
            float a = floorf((xb - fx) * 256.f) / 256.f, b = floorf((yb - fy) * 256.f) / 256.f;
            /* the cell index, limited to [-1, size - 1] first (the same taps after the clamps below) */
            int i0 = (int)fminf(fmaxf(fx, -1.f), (float)w - 1.f), j0 = (int)fminf(fmaxf(fy, -1.f), (float)h - 1.f);
            int i1 = i0 + 1, j1 = j0 + 1;
            i0 = i0 < 0 ? 0 : i0 > w - 1 ? w - 1 : i0;
            i1 = i1 < 0 ? 0 : i1 > w - 1 ? w - 1 : i1;
            j0 = j0 < 0 ? 0 : j0 > h - 1 ? h - 1 : j0;
            j1 = j1 < 0 ? 0 : j1 > h - 1 ? h - 1 : j1;
            const uint8_t* t00 = src + (size_t)j0 * spitch + (size_t)i0 * 4;
            const uint8_t* t10 = src + (size_t)j0 * spitch + (size_t)i1 * 4;
            const uint8_t* t01 = src + (size_t)j1 * spitch + (size_t)i0 * 4;
            const uint8_t* t11 = src + (size_t)j1 * spitch + (size_t)i1 * 4;
            for (int c = 0; c < 4; c++) {
                float val = (1.f - a) * (1.f - b) * (t00[c] / 255.f) + a * (1.f - b) * (t10[c] / 255.f) +
                            (1.f - a) * b * (t01[c] / 255.f) + a * b * (t11[c] / 255.f);
                o[c] = (uint8_t)sat_u8_rne(val * 255.f);
            }
        }
}
