// camera_math.hpp — camera projection models for the LUT build, evaluated per output pixel in FP64.
//
// __host__ __device__ so the same arithmetic runs in the gfx950 LUT kernel and in host-side setup.
// The order of every floating-point operation follows the reference so results agree bit-for-bit
// with it wherever the libm calls agree (the translation unit is built with -ffp-contract=off):
//   sphere helpers            modules/octvr/src/camera.cpp:189-210
//   obj_to_image/image_to_obj camera.cpp:212-253, 296-315
//   equirectangular           modules/octvr/src/cameras/equirectangular.cpp:25-35
//   fullframe_fisheye         modules/octvr/src/cameras/fullframe_fisheye_cam.cpp:146-221
//   fisheye (OpenCV KB)       modules/octvr/src/cameras/pinhole_cam.cpp:32-50 + calib3d/src/fisheye.cpp:95-146
//   pinhole (projectPoints)   pinhole_cam.cpp:32-57 + calib3d/src/calibration.cpp:759-793
//   normal                    modules/octvr/src/cameras/normal.cpp:24-39
//   perspective               modules/octvr/src/cameras/perspective.cpp:21-33
//   ocam_fisheye              modules/octvr/src/cameras/ocam_fisheye.cpp:135-244
//   stupidoval                modules/octvr/src/cameras/stupidoval.hpp:24-36
//   cubic                     modules/octvr/src/cameras/cubic.hpp:19-103
//   eqareanorthpole / -south  modules/octvr/src/cameras/eqareanorthpole.hpp:24-41, eqareasouthpole.hpp:23-40
#pragma once

#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdint>

namespace octvr {

enum CameraType : int32_t {
    CAM_EQUIRECT = 0,
    CAM_FULLFRAME_FISHEYE = 1,
    CAM_FISHEYE = 2,
    CAM_PINHOLE = 3,
    CAM_NORMAL = 4,
    CAM_PERSPECTIVE = 5,
    CAM_OCAM = 6,
    CAM_STUPIDOVAL = 7,
    CAM_CUBIC = 8,
    CAM_EQAREA_NORTH = 9,
    CAM_EQAREA_SOUTH = 10,
};

constexpr int kOcamMaxPol = 64;  // MAX_POL_LENGTH (ocam_fisheye.hpp:21)

// Plain-old-data camera description; the LUT kernel reads it from device memory.
struct CameraParams {
    int32_t type;
    int32_t width, height;                      // input image size (fisheye / pinhole / ocam / masks)
    int32_t crop_x, crop_y, crop_w, crop_h;     // fullframe_fisheye crop rect
    int32_t crop_circular;
    int32_t sel;                                // `selection` present: exclude everything outside sel_*
    int32_t sel_l, sel_r, sel_t, sel_b;         // selection rectangle (camera.cpp:96-112)
    int32_t len_pol, len_invpol;                // ocam polynomial lengths
    double R[9];                                // rotate_matrix (camera.cpp:57-70)
    double Rinv[9];                             // rotate_matrix.inv() (camera.cpp:205)
    double min_lon, max_lon;                    // longitude_selection (camera.cpp:125-135)
    double min_lat, max_lat, scale_lon;         // equirectangular.hpp:26-27
    double hfov, center_dx, center_dy;          // fullframe_fisheye_cam.cpp:128-130
    double rad[6];                              // radial_distortion[0..5] (fullframe_fisheye_cam.cpp:133-138)
    double fx, fy, cx, cy, k[4];                // fisheye / pinhole intrinsics (pinhole_cam.cpp:13-30)
    double dist[14];                            // pinhole: projectPoints distortion k1..tauY (zero padded)
    double tilt[9];                             // pinhole: matTilt (identity unless tauX / tauY != 0)
    double aspect;                              // normal / perspective aspect_ratio
    double cam_x, cam_y, cam_z;                 // normal.cpp:16-19
    double sf;                                  // perspective.cpp:16
    double circle;                              // eqarea: arctic_circle / antarctic_circle
    double xc, yc, oc, od, oe;                  // ocam: center and affine parameters c, d, e
    double pol[kOcamMaxPol], invpol[kOcamMaxPol];
    // exclude_mask / include_mask (camera.cpp:72-123), width x height u8 in device memory, or null.
    // `incl` is only set when both exist: get_include_mask tests exclude_mask.empty() (camera.cpp:281).
    const uint8_t* excl;
    const uint8_t* incl;
};

#define OCTVR_HD __host__ __device__ inline
constexpr double kPi = 3.14159265358979323846;

// sin(x) and cos(x) of one argument.  The reference is built by gcc, whose sincos pass turns every
// sin(x) / cos(x) pair of one function into ONE glibc sincos() call, and glibc's sincos differs in the
// last bit from its (FMA-dispatched) sin and cos at some arguments.  So the host evaluation calls
// sincos exactly where a reference function computes both (camera.cpp:197-199, fullframe_fisheye_cam.cpp:
// 191-193 and 244-248, eqarea*.hpp, cvRodrigues2) and plain sin / cos everywhere else (clang never merges
// them); the device uses OCML's sin and cos (its results are only trusted away from every decision
// boundary, see LutGuard).
OCTVR_HD void sin_cos(double x, double* s, double* c) {
#if defined(__HIP_DEVICE_COMPILE__)
    *s = sin(x);
    *c = cos(x);
#else
    ::sincos(x, s, c);
#endif
}

// ---- decision guard of the GPU LUT build ---------------------------------------------------------
// Device libm (OCML) and glibc may differ in the last ulps of sin / cos / atan2 / asin / atan / tan,
// and so may every quantity derived from them.  The LUT kernel therefore passes a guard through the
// projection: every comparison whose outcome such a difference could flip (a branch threshold, the
// [0, 1) image test, a mask pixel index) marks the pixel fragile when its two sides are within
// kLutGuardTol of each other, and so does a final f64 -> f32 rounding that lies that close to a
// rounding boundary.  The host then recomputes the fragile pixels with glibc, i.e. with exactly the
// reference's arithmetic (octvr_hip.cpp build_input), so the LUT is bit-exact.  The host
// evaluation passes no guard.  Measured device-vs-glibc deviations of the final coordinates in and
// next to the image: <= 1e-13 on every model but the tilted k1-k4 pinhole (6.9e-13), at least 20x
// inside the tolerance (tests/test_gpu_lut_exact.py).
constexpr double kLutGuardTol = 0x1p-36;  // ~1.5e-11 on O(1) quantities
struct LutGuard {
    bool hit;
};
// a and b (finite) closer than tol: the comparison of a with b may differ between device and host
OCTVR_HD void guard_near(LutGuard* g, double a, double b, double tol = kLutGuardTol) {
    if (g && fabs(a - b) <= tol) g->hit = true;
}
// v compared with both ends of [lo, hi]
OCTVR_HD void guard_range(LutGuard* g, double v, double lo, double hi, double tol = kLutGuardTol) {
    guard_near(g, v, lo, tol);
    guard_near(g, v, hi, tol);
}
// (int)(v) of a mask pixel index: fragile next to an integer (tolerance scaled by the image size)
OCTVR_HD void guard_index(LutGuard* g, double v, double scale) {
    if (g && fabs(v - rint(v)) <= kLutGuardTol * (scale > 1 ? scale : 1)) g->hit = true;
}
// (float)v: fragile within tol of a rounding boundary (the midpoints between neighbouring floats), and
// next to 0 (the sign decides the x < 0 test)
OCTVR_HD bool f32_fragile(double v, double tol = kLutGuardTol) {
    if (v != v) return false;
    if (fabs(v) <= tol) return true;
    const float f = (float)v;
    if (fabs((double)f) > 3.0e38) return false;  // |v| beyond any image: invalid on both sides
    const double lo = ((double)f + (double)nextafterf(f, -INFINITY)) * 0.5;
    const double hi = ((double)f + (double)nextafterf(f, INFINITY)) * 0.5;
    return v - lo <= tol || hi - v <= tol;
}

OCTVR_HD void lonlat_to_xyz(double lon, double lat, double* p) {
    double slon, clon, slat, clat;
    sin_cos(lon, &slon, &clon);
    sin_cos(lat, &slat, &clat);
    p[0] = clon * clat;
    p[1] = slat;
    p[2] = -slon * clat;
}

// rotated = m * r.t() evaluated by cv::gemm's A*B^T loop: s = ((0 + a0 b0) + a1 b1) + a2 b2.
OCTVR_HD void rotate_rows(const double* r, const double* p, double* q) {
    for (int k = 0; k < 3; k++) {
        double s0 = 0;
        s0 += p[0] * r[k * 3 + 0];
        s0 += p[1] * r[k * 3 + 1];
        s0 += p[2] * r[k * 3 + 2];
        double z = 0;
        q[k] = (((s0 + z) + z) + z) * 1.0;
    }
}

// sphere_xyz_to_lonlat: p = xyz * (1 / norm(xyz)) (camera.cpp:189-192)
// Guard: next to a pole (|py| ~ 1) the longitude is ill-conditioned and asin's domain edge is near;
// atan2's branch cut (pz ~ 0 with px < 0) flips lon between -pi and pi.
OCTVR_HD void xyz_to_lonlat(const double* xyz, double* lon, double* lat, LutGuard* g = nullptr) {
    double n = sqrt(xyz[0] * xyz[0] + xyz[1] * xyz[1] + xyz[2] * xyz[2]);
    double inv = 1.0 / n;
    double px = xyz[0] * inv, py = xyz[1] * inv, pz = xyz[2] * inv;
    if (g) {
        guard_near(g, fabs(py), 1.0, 0x1p-20);
        if (px < 0) guard_near(g, pz, 0.0);
    }
    *lon = atan2(-pz, px);
    *lat = asin(py);
}
OCTVR_HD void xyz3_to_lonlat(double x, double y, double z, double* lon, double* lat, LutGuard* g = nullptr) {
    const double p[3] = {x, y, z};
    xyz_to_lonlat(p, lon, lat, g);
}

OCTVR_HD bool valid_longitude(const CameraParams& c, double l, LutGuard* g = nullptr) {
    // the default selection [-pi, pi] (camera.cpp:125-135) holds every atan2 result: no threshold to guard
    const bool custom = c.min_lon > -kPi || c.max_lon < kPi;
    auto between = [&](double x) {
        if (custom) guard_range(g, x, c.min_lon, c.max_lon);
        return x >= c.min_lon && x <= c.max_lon;
    };
    return between(l) || between(l + 2 * kPi) || between(l - 2 * kPi) || between(l + 4 * kPi) ||
           between(l - 4 * kPi);
}

// ---- image_to_obj_single (output cameras) -------------------------------------------------------
OCTVR_HD void equirect_image_to_obj(const CameraParams& c, double x, double y, double* lon, double* lat) {
    *lon = (x - 0.5) * kPi * 2.0;
    *lat = (c.min_lat - c.max_lat) * y + c.max_lat;
}

// cam2world (ocam_fisheye.cpp:135-166); point2D = (row, col)
OCTVR_HD void ocam_cam2world(const CameraParams& c, const double* p2, double* p3) {
    double invdet = 1 / (c.oc - c.od * c.oe);
    double xp = invdet * ((p2[0] - c.xc) - c.od * (p2[1] - c.yc));
    double yp = invdet * (-c.oe * (p2[0] - c.xc) + c.oc * (p2[1] - c.yc));
    double r = sqrt(xp * xp + yp * yp);
    double zp = c.pol[0];
    double r_i = 1;
    for (int i = 1; i < c.len_pol; i++) {
        r_i *= r;
        zp += r_i * c.pol[i];
    }
    double invnorm = 1 / sqrt(xp * xp + yp * yp + zp * zp);
    p3[0] = invnorm * xp;
    p3[1] = invnorm * yp;
    p3[2] = invnorm * zp;
}

// world2cam (ocam_fisheye.cpp:183-225)
OCTVR_HD void ocam_world2cam(const CameraParams& c, const double* p3, double* p2) {
    double norm = sqrt(p3[0] * p3[0] + p3[1] * p3[1]);
    double theta = atan(p3[2] / norm);
    if (norm != 0) {
        double invnorm = 1 / norm;
        double t = theta;
        double rho = c.invpol[0];
        double t_i = 1;
        for (int i = 1; i < c.len_invpol; i++) {
            t_i *= t;
            rho += t_i * c.invpol[i];
        }
        double x = p3[0] * invnorm * rho;
        double y = p3[1] * invnorm * rho;
        p2[0] = x * c.oc + y * c.od + c.xc;
        p2[1] = x * c.oe + y + c.yc;
    } else {
        p2[0] = c.xc;
        p2[1] = c.yc;
    }
}

// Output camera: (x, y) in [0,1)^2 -> lonlat before the output rotation; NaN when undefined.
// cv::solvePoly (core/src/mathfuncs.cpp:2063-2182, maxIters 300) on a real polynomial a[0] + a[1] x +
// ... + a[n0] x^n0: trailing zero coefficients trimmed, Durand-Kerner (Weierstrass) iteration from the
// powers of (1 + i), each root updated in place, until no update moves.  Complex ops as cv::Complex
// (core/types.hpp:960-1029).  Returns the trimmed degree n; only re/im[0..n) are defined (the reference
// fills rows n..n0-1 from uninitialised memory).  The coincident-iterate branch (num_same_root > 1,
// :2119-2157) needs two iterates to be bit-identical and is not taken by this restatement.
OCTVR_HD int solve_poly_real(const double* a, int n0, double* re, double* im) {
    int n = n0;
    for (; n > 1; n--)
        if (fabs(a[n]) + 0.0 > 2.220446049250313e-16) break;
    double pr = 1, pi = 0;
    for (int i = 0; i < n; i++) {
        re[i] = pr;
        im[i] = pi;
        const double tr = pr * 1.0 - pi * 1.0, ti = pr * 1.0 + pi * 1.0;
        pr = tr;
        pi = ti;
    }
    for (int iter = 0; iter < 300; iter++) {
        double max_diff = 0;
        for (int i = 0; i < n; i++) {
            const double xr = re[i], xi = im[i];
            double nr = a[n], ni = 0, dr = a[n], di = 0;
            for (int j = 0; j < n; j++) {
                double tr = nr * xr - ni * xi, ti = nr * xi + ni * xr;
                nr = tr + a[n - j - 1];
                ni = ti + 0.0;
                if (j != i) {
                    const double er = xr - re[j], ei = xi - im[j];
                    if (er != 0 || ei != 0) {
                        tr = dr * er - di * ei;
                        ti = dr * ei + di * er;
                        dr = tr;
                        di = ti;
                    }
                }
            }
            const double t = 1. / (dr * dr + di * di);
            const double qr = (nr * dr + ni * di) * t, qi = (-nr * di + ni * dr) * t;
            re[i] = xr - qr;
            im[i] = xi - qi;
            max_diff = fmax(max_diff, sqrt(qr * qr + qi * qi));
        }
        if (max_diff <= 0) break;
    }
    for (int i = 0; i < n; i++)
        if (fabs(im[i]) < 1e-100) im[i] = 0;
    return n;
}

// FullFrameFisheyeCamera::image_to_obj_single (fullframe_fisheye_cam.cpp:223-253) with
// do_reverse_radial_distort (:160-185); the crop must be the whole image (checked at rig creation).
OCTVR_HD void fullframe_fisheye_image_to_obj(const CameraParams& c, double x, double y, double* lon, double* lat,
                                             LutGuard* g = nullptr) {
    x -= 0.5;
    y -= 0.5;
    x *= (double)c.crop_w;
    y *= (double)c.crop_h;
    x -= c.center_dx;
    y -= c.center_dy;
    if (fabs(x) < 1e-5 && fabs(y) < 1e-5) {
        *lon = 0;
        *lat = 0;
        return;
    }
    const double s = sqrt(x * x + y * y);
    const double coeffs[5] = {-s / c.rad[4], c.rad[0], c.rad[1], c.rad[2], c.rad[3]};
    double rre[4], rim[4], r = -1;
    const int n = solve_poly_real(coeffs, 4, rre, rim);
    for (int i = 0; i < n; i++)
        if (fabs(rim[i]) < 1e-3 && rre[i] > 0 && (rre[i] < r || r < 0)) r = rre[i];
    const double scale = (r < c.rad[5] && r > 0) ? s / c.rad[4] / r : 1000.0;
    x = x / scale;
    y = y / scale;
    const double distance = double(c.crop_w) / c.hfov;
    const double alpha = atan2(-y, x);
    double sa, ca;
    sin_cos(alpha, &sa, &ca);
    double theta = -y / distance / sa;
    guard_near(g, fabs(sa), 1e-3);
    if (fabs(sa) < 1e-3) theta = -x / distance / ca;
    double st, ct;
    sin_cos(theta, &st, &ct);
    *lon = atan2(st * ca, ct);
    guard_near(g, fabs(ca), 0.0, 0x1p-20);  // tan(alpha) changes sign through +-infinity
    if (g && ct < 0) guard_near(g, st * ca, 0.0);  // atan2's branch cut
    *lat = atan(tan(alpha) * sin(*lon));
}

OCTVR_HD void image_to_obj_single(const CameraParams& c, double x, double y, double* lon, double* lat,
                                  LutGuard* g = nullptr) {
    switch (c.type) {
        case CAM_FULLFRAME_FISHEYE:
            fullframe_fisheye_image_to_obj(c, x, y, lon, lat, g);
            return;
        case CAM_NORMAL: {
            double xx = c.cam_x;
            double yy = c.cam_y - y * 2.0 * c.cam_y;
            double zz = c.cam_z - x * 2.0 * c.cam_z;
            xyz3_to_lonlat(xx, yy, zz, lon, lat, g);
            return;
        }
        case CAM_PERSPECTIVE: {
            double z = (0.5 - x) * c.aspect;
            double yy = 0.5 - y;
            double xx = 1.0 / c.sf;
            xyz3_to_lonlat(xx, yy, z, lon, lat, g);
            return;
        }
        case CAM_OCAM: {
            double p2[2] = {y * c.height, x * c.width}, p3[3];
            ocam_cam2world(c, p2, p3);
            xyz3_to_lonlat(-p3[2], -p3[0], -p3[1], lon, lat, g);
            return;
        }
        case CAM_STUPIDOVAL: {
            double la = (0.5 - y) * kPi;
            double lo = (x - 0.5) * kPi * 2.0 / cos(la);
            guard_range(g, lo, -kPi, kPi);
            if (lo < -kPi || lo > kPi) {
                *lon = *lat = NAN;
                return;
            }
            *lon = lo;
            *lat = la;
            return;
        }
        case CAM_CUBIC: {
            int ix = 0, iy = 0;
            if (y >= 0.5) iy = 1;
            if (x >= 2.0 / 3.0)
                ix = 2;
            else if (x >= 1.0 / 3.0)
                ix = 1;
            double px = (x - ix * 1.0 / 3.0) * 3.0 * 2.0 - 1.0;
            double py = (y - iy * 1.0 / 2.0) * 2.0 * 2.0 - 1.0;
            switch (iy * 3 + ix) {
                case 0: xyz3_to_lonlat(1.0, py, px, lon, lat, g); return;
                case 1: xyz3_to_lonlat(-1., py, -px, lon, lat, g); return;
                case 2: xyz3_to_lonlat(px, -1., -py, lon, lat, g); return;
                case 3: xyz3_to_lonlat(px, 1.0, py, lon, lat, g); return;
                case 4: xyz3_to_lonlat(px, py, -1.0, lon, lat, g); return;
                default: xyz3_to_lonlat(-px, py, 1.0, lon, lat, g); return;
            }
        }
        case CAM_EQAREA_NORTH: {
            double dx = x - 0.5, dy = y - 0.5;
            double rho = sqrt(dx * dx + dy * dy) * 2;
            *lat = kPi / 2 - (kPi / 2 - c.circle) * rho;
            *lon = atan2(-dx, -dy);  // exact arguments: no device / host difference to guard
            return;
        }
        case CAM_EQAREA_SOUTH: {
            double dx = x - 0.5, dy = y - 0.5;
            double rho = sqrt(dx * dx + dy * dy) * 2;
            *lat = -kPi / 2 + (c.circle + kPi / 2) * rho;
            *lon = atan2(dx, -dy);
            return;
        }
        default:
            equirect_image_to_obj(c, x, y, lon, lat);
            return;
    }
}

// ---- obj_to_image_single (input cameras) --------------------------------------------------------
OCTVR_HD void equirect_obj_to_image(const CameraParams& c, double lon, double lat, double* x, double* y) {
    *x = lon / (kPi * 2.0) + 0.5;
    *y = (lat - c.max_lat) / (c.min_lat - c.max_lat);
}

OCTVR_HD void fullframe_fisheye_obj_to_image(const CameraParams& c, double lon, double lat, double* ox, double* oy,
                                             LutGuard* g = nullptr) {
    double slat, clat, slon, clon;
    sin_cos(lat, &slat, &clat);
    sin_cos(lon, &slon, &clon);
    double s = clat * clon;
    double v1 = slat;
    double v0 = -clat * slon;
    double r = sqrt(v0 * v0 + v1 * v1);
    double theta = atan2(r, s);
    double distance = double(c.crop_w) / (c.hfov);
    double x = -(theta * v0 / r) * distance;
    double y = -(theta * v1 / r) * distance;
    if (g) {
        if (fabs(lat) <= 1e-5 + kLutGuardTol) guard_near(g, fabs(lon), 1e-5);
        if (fabs(lon) <= 1e-5 + kLutGuardTol) guard_near(g, fabs(lat), 1e-5);
    }
    if (fabs(lon) < 1e-5 && fabs(lat) < 1e-5) x = y = 0;
    double rr = (sqrt(x * x + y * y)) / c.rad[4];
    if (g) guard_near(g, rr, c.rad[5], kLutGuardTol * fmax(1.0, fabs(c.rad[5])));
    double scale = (rr < c.rad[5]) ? ((c.rad[3] * rr + c.rad[2]) * rr + c.rad[1]) * rr + c.rad[0] : 1000.0;
    double rx = x * scale, ry = y * scale;
    rx += c.center_dx;
    ry += c.center_dy;
    rx /= double(c.crop_w);
    ry /= double(c.crop_h);
    rx += 0.5;
    ry += 0.5;
    if (c.crop_circular) guard_near(g, (rx - 0.5) * (rx - 0.5) + (ry - 0.5) * (ry - 0.5), 0.25);
    if (c.crop_circular && (rx - 0.5) * (rx - 0.5) + (ry - 0.5) * (ry - 0.5) > 0.25) {
        *ox = NAN;
        *oy = NAN;
        return;
    }
    rx = (rx * c.crop_w) + c.crop_x;
    ry = (ry * c.crop_h) + c.crop_y;
    rx /= double(c.width);
    ry /= double(c.height);
    *ox = rx;
    *oy = ry;
}

OCTVR_HD void cubic_face_to_img(int index, double x, double y, double* ox, double* oy) {
    double rx = (index % 3) * 1.0 / 3.0, ry = (index / 3) * 1.0 / 2.0;
    rx += (x + 1.0) / 2.0 / 3.0;
    ry += (y + 1.0) / 2.0 / 2.0;
    *ox = rx;
    *oy = ry;
}

OCTVR_HD void obj_to_image_single(const CameraParams& c, double lon, double lat, double* ox, double* oy,
                                  LutGuard* g = nullptr) {
    switch (c.type) {
        case CAM_FULLFRAME_FISHEYE:
            fullframe_fisheye_obj_to_image(c, lon, lat, ox, oy, g);
            return;
        case CAM_NORMAL: {
            double p[3];
            lonlat_to_xyz(lon, lat, p);
            guard_near(g, p[0], 0.0);
            if (p[0] < 0) {
                *ox = *oy = NAN;
                return;
            }
            const double t = p[0] / c.cam_x;  // xxyyzz /= (xxyyzz.x / cam_x)
            p[0] /= t;
            p[1] /= t;
            p[2] /= t;
            *ox = (c.cam_z - p[2]) / 2.0 / c.cam_z;
            *oy = (c.cam_y - p[1]) / 2.0 / c.cam_y;
            return;
        }
        case CAM_PERSPECTIVE: {
            double p[3];
            lonlat_to_xyz(lon, lat, p);
            guard_near(g, p[0], 0.0);  // the projection changes sign through infinity
            double y_ = p[1] * (1.0 / c.sf / p[0]);
            double z_ = p[2] * (1.0 / c.sf / p[0]);
            *ox = 0.5 - z_ / c.aspect;
            *oy = 0.5 - y_;
            return;
        }
        case CAM_OCAM: {
            double p[3];
            lonlat_to_xyz(lon, lat, p);
            const double q[3] = {-p[1], -p[2], -p[0]};
            double p2[2];
            ocam_world2cam(c, q, p2);
            *ox = p2[1] / c.width;
            *oy = p2[0] / c.height;
            return;
        }
        case CAM_STUPIDOVAL:
            *ox = cos(lat) * lon / (kPi * 2.0) + 0.5;
            *oy = -lat / kPi + 0.5;
            return;
        case CAM_CUBIC: {
            double p[3], s[3];
            lonlat_to_xyz(lon, lat, p);
            auto within = [g](double a, double b) {
                guard_range(g, a, -1.0, 1.0);
                guard_range(g, b, -1.0, 1.0);
                return a >= -1.0 && a <= 1.0 && b >= -1.0 && b <= 1.0;
            };
            for (int k = 0; k < 3; k++) guard_near(g, fabs(p[k]), 1e-2);
            if (fabs(p[0]) > 1e-2) {  // intersect with x = 1 / x = -1
                const double f = fabs(p[0]);
                s[0] = p[0] / f;
                s[1] = p[1] / f;
                s[2] = p[2] / f;
                if (within(s[1], s[2])) {
                    if (s[0] < 0)
                        cubic_face_to_img(1, -s[2], s[1], ox, oy);
                    else
                        cubic_face_to_img(0, s[2], s[1], ox, oy);
                    return;
                }
            }
            if (fabs(p[2]) > 1e-2) {
                const double f = fabs(p[2]);
                s[0] = p[0] / f;
                s[1] = p[1] / f;
                s[2] = p[2] / f;
                if (within(s[0], s[1])) {
                    if (s[2] < 0)
                        cubic_face_to_img(4, s[0], s[1], ox, oy);
                    else
                        cubic_face_to_img(5, -s[0], s[1], ox, oy);
                    return;
                }
            }
            if (fabs(p[1]) > 1e-2) {
                const double f = fabs(p[1]);
                s[0] = p[0] / f;
                s[1] = p[1] / f;
                s[2] = p[2] / f;
                if (within(s[0], s[2])) {
                    if (s[1] < 0)
                        cubic_face_to_img(2, s[0], -s[2], ox, oy);
                    else
                        cubic_face_to_img(3, s[0], s[2], ox, oy);
                    return;
                }
            }
            *ox = *oy = NAN;
            return;
        }
        case CAM_EQAREA_NORTH: {
            guard_near(g, lat, c.circle);
            if (lat < c.circle) {
                *ox = *oy = NAN;
                return;
            }
            double rho = (kPi / 2 - lat) / (kPi / 2 - c.circle);
            double sl, cl;
            sin_cos(lon, &sl, &cl);
            *ox = -rho * sl / 2 + 0.5;
            *oy = -rho * cl / 2 + 0.5;
            return;
        }
        case CAM_EQAREA_SOUTH: {
            guard_near(g, lat, c.circle);
            if (lat > c.circle) {
                *ox = *oy = NAN;
                return;
            }
            double rho = (lat + kPi / 2) / (c.circle + kPi / 2);
            double sl, cl;
            sin_cos(lon, &sl, &cl);
            *ox = rho * sl / 2 + 0.5;
            *oy = -rho * cl / 2 + 0.5;
            return;
        }
        default:
            equirect_obj_to_image(c, lon, lat, ox, oy);
            return;
    }
}

// Y is the rotated sphere point; Kannala-Brandt projection with zero rvec/tvec and alpha = 0.
OCTVR_HD void fisheye_project(const CameraParams& c, const double* Y, double* ox, double* oy, LutGuard* g = nullptr) {
    guard_near(g, Y[2], 0.0);
    if (Y[2] <= 0) {
        *ox = NAN;
        *oy = NAN;
        return;
    }
    double x0 = Y[0] / Y[2], x1 = Y[1] / Y[2];
    double r2 = x0 * x0 + x1 * x1;
    double r = sqrt(r2);
    double theta = atan(r);
    double theta2 = theta * theta, theta3 = theta2 * theta, theta4 = theta2 * theta2, theta5 = theta4 * theta,
           theta6 = theta3 * theta3, theta7 = theta6 * theta, theta8 = theta4 * theta4, theta9 = theta8 * theta;
    double theta_d = theta + c.k[0] * theta3 + c.k[1] * theta5 + c.k[2] * theta7 + c.k[3] * theta9;
    double inv_r = r > 1e-8 ? 1.0 / r : 1;
    double cdist = r > 1e-8 ? theta_d * inv_r : 1;
    double xd0 = x0 * cdist, xd1 = x1 * cdist;
    double alpha = 0;
    double u = (xd0 + alpha * xd1) * c.fx + c.cx, v = xd1 * c.fy + c.cy;
    *ox = u / c.width;
    *oy = 1.0 - v / c.height;
}

// cvProjectPoints2 for one point with rvec = tvec = 0 (R = I, t = 0) (calibration.cpp:759-793).
// Y is the rotated sphere point (z <= 0 was mapped to NaN by PinholeCamera::obj_to_image).
OCTVR_HD void pinhole_project(const CameraParams& c, const double* Y, double* ox, double* oy, LutGuard* g = nullptr) {
    guard_near(g, Y[2], 0.0);
    double X = Y[0], Yy = Y[1], Z = Y[2];
    if (Z <= 0) X = Yy = Z = NAN;
    const double* k = c.dist;
    double x = 1.0 * X + 0.0 * Yy + 0.0 * Z + 0.0;
    double y = 0.0 * X + 1.0 * Yy + 0.0 * Z + 0.0;
    double z = 0.0 * X + 0.0 * Yy + 1.0 * Z + 0.0;
    z = z ? 1. / z : 1;
    x *= z;
    y *= z;
    double r2 = x * x + y * y;
    double r4 = r2 * r2;
    double r6 = r4 * r2;
    double a1 = 2 * x * y;
    double a2 = r2 + 2 * x * x;
    double a3 = r2 + 2 * y * y;
    double cdist = 1 + k[0] * r2 + k[1] * r4 + k[4] * r6;
    double icdist2 = 1. / (1 + k[5] * r2 + k[6] * r4 + k[7] * r6);
    double xd0 = x * cdist * icdist2 + k[2] * a1 + k[3] * a2 + k[8] * r2 + k[9] * r4;
    double yd0 = y * cdist * icdist2 + k[2] * a3 + k[3] * a1 + k[10] * r2 + k[11] * r4;
    // vecTilt = matTilt * Vec3d(xd0, yd0, 1) (Matx product: s = 0; s += a(i,k) * b(k))
    double v[3];
    for (int i = 0; i < 3; i++) {
        double s = 0;
        s += c.tilt[i * 3 + 0] * xd0;
        s += c.tilt[i * 3 + 1] * yd0;
        s += c.tilt[i * 3 + 2] * 1.0;
        v[i] = s;
    }
    double invProj = v[2] ? 1. / v[2] : 1;
    double xd = invProj * v[0];
    double yd = invProj * v[1];
    double u = xd * c.fx + c.cx, vv = yd * c.fy + c.cy;
    *ox = u / c.width;
    *oy = 1.0 - vv / c.height;
}

// Camera::obj_to_image exclude-mask test for a `selection` rectangle (camera.cpp:96-112, 239-246):
// the mask is 255 outside the filled rectangle [l, r-1] x [t, b-1] of the width x height image.
OCTVR_HD bool selection_excludes(const CameraParams& c, double x, double y) {
    if (!c.sel) return false;
    const int W = (int)(x * c.width), H = (int)(y * c.height);
    return !(W >= c.sel_l && W <= c.sel_r - 1 && H >= c.sel_t && H <= c.sel_b - 1);
}

// Output pixel (u, v) in [0,1)^2 -> input camera normalized image point (x, y) or NaN.  With `vis`,
// also Camera::get_include_mask's verdict for the pixel (camera.cpp:255-294: the same projection
// without the longitude and exclude tests, then include_mask.at(int(y*rows), int(x*cols))).
// g (device LUT build): marks the pixel fragile (see LutGuard); the host evaluation passes none.
OCTVR_HD void project_output_to_input(const CameraParams& out, const CameraParams& in, double u, double v,
                                      double* x, double* y, bool* vis = nullptr, LutGuard* g = nullptr) {
    double lon, lat, p[3], q[3];
    if (vis) *vis = false;
    // out->image_to_obj (camera.cpp:296-315)
    image_to_obj_single(out, u, v, &lon, &lat, g);
    lonlat_to_xyz(lon, lat, p);
    rotate_rows(out.Rinv, p, q);
    xyz_to_lonlat(q, &lon, &lat, g);
    // in->obj_to_image (camera.cpp:212-253; PinholeCamera overrides it, pinhole_cam.cpp:32-50)
    lonlat_to_xyz(lon, lat, p);
    bool lon_ok = valid_longitude(in, lon, g);
    rotate_rows(in.R, p, q);
    if (in.type == CAM_FISHEYE) {
        fisheye_project(in, q, x, y, g);
        return;
    }
    if (in.type == CAM_PINHOLE) {
        pinhole_project(in, q, x, y, g);
        return;
    }
    double ll, la;
    xyz_to_lonlat(q, &ll, &la, g);
    double px = NAN, py = NAN;
    if (lon_ok || (vis && in.incl)) obj_to_image_single(in, ll, la, &px, &py, g);
    const bool inside = px >= 0 && px < 1 && py >= 0 && py < 1;
    const bool masked = in.sel || in.excl || (vis && in.incl);
    if (g && masked) {  // the mask lookups: the [0, 1) test and the pixel indices
        guard_range(g, px, 0.0, 1.0);
        guard_range(g, py, 0.0, 1.0);
        if (inside) {
            guard_index(g, px * in.width, in.width);
            guard_index(g, py * in.height, in.height);
        }
    }
    const size_t at = inside ? (size_t)(int)(py * in.height) * in.width + (int)(px * in.width) : 0;
    if (vis && in.incl && inside) *vis = in.incl[at] != 0;
    if (!lon_ok) px = py = NAN;
    else if (inside && (selection_excludes(in, px, py) || (in.excl && in.excl[at]))) px = py = NAN;
    *x = px;
    *y = py;
}

}  // namespace octvr
