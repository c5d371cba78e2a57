// camera_math.hpp — camera projection models for the LUT build, evaluated per output pixel in FP64.
//
// __host__ __device__ so the same arithmetic runs in the gfx950 LUT kernel and in host-side setup.
// The order of every floating-point operation follows the reference so results agree bit-for-bit
// with it wherever the libm calls agree (the translation unit is built with -ffp-contract=off):
//   sphere helpers          modules/octvr/src/camera.cpp:189-210
//   obj_to_image/image_to_obj camera.cpp:212-253, 296-315
//   equirectangular         modules/octvr/src/cameras/equirectangular.cpp:25-35
//   fullframe_fisheye       modules/octvr/src/cameras/fullframe_fisheye_cam.cpp:146-221
//   fisheye (OpenCV KB)     modules/octvr/src/cameras/pinhole_cam.cpp:32-50 + calib3d/src/fisheye.cpp:95-146
#pragma once

#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdint>

namespace octvr {

enum CameraType : int32_t { CAM_EQUIRECT = 0, CAM_FULLFRAME_FISHEYE = 1, CAM_FISHEYE = 2 };

// Plain-old-data camera description, copied to the device by value as a kernel argument.
struct CameraParams {
    int32_t type;
    int32_t width, height;                      // input image size (fisheye models)
    int32_t crop_x, crop_y, crop_w, crop_h;     // fullframe_fisheye crop rect
    int32_t crop_circular;
    int32_t pad_;
    double R[9];                                // rotate_matrix (camera.cpp:57-70)
    double Rinv[9];                             // rotate_matrix.inv() (camera.cpp:205)
    double min_lon, max_lon;                    // longitude_selection (camera.cpp:125-135)
    double min_lat, max_lat, scale_lon;         // equirectangular.hpp:61-62
    double hfov, center_dx, center_dy;          // fullframe_fisheye_cam.cpp:128-130
    double rad[6];                              // radial_distortion[0..5] (fullframe_fisheye_cam.cpp:133-138)
    double fx, fy, cx, cy, k[4];                // pinhole_cam.cpp:13-30
};

#define OCTVR_HD __host__ __device__ inline
constexpr double kPi = 3.14159265358979323846;

OCTVR_HD void lonlat_to_xyz(double lon, double lat, double* p) {
    p[0] = cos(lon) * cos(lat);
    p[1] = sin(lat);
    p[2] = -sin(lon) * cos(lat);
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

OCTVR_HD void xyz_to_lonlat(const double* xyz, double* lon, double* lat) {
    double n = sqrt(xyz[0] * xyz[0] + xyz[1] * xyz[1] + xyz[2] * xyz[2]);
    double inv = 1.0 / n;
    double px = xyz[0] * inv, py = xyz[1] * inv, pz = xyz[2] * inv;
    *lon = atan2(-pz, px);
    *lat = asin(py);
}

OCTVR_HD bool valid_longitude(const CameraParams& c, double l) {
    auto between = [&](double x) { return x >= c.min_lon && x <= c.max_lon; };
    return between(l) || between(l + 2 * kPi) || between(l - 2 * kPi) || between(l + 4 * kPi) ||
           between(l - 4 * kPi);
}

OCTVR_HD void equirect_image_to_obj(const CameraParams& c, double x, double y, double* lon, double* lat) {
    *lon = (x - 0.5) * kPi * 2.0;
    *lat = (c.min_lat - c.max_lat) * y + c.max_lat;
}

OCTVR_HD void equirect_obj_to_image(const CameraParams& c, double lon, double lat, double* x, double* y) {
    *x = lon / (kPi * 2.0) + 0.5;
    *y = (lat - c.max_lat) / (c.min_lat - c.max_lat);
}

OCTVR_HD void fullframe_fisheye_obj_to_image(const CameraParams& c, double lon, double lat, double* ox, double* oy) {
    double s = cos(lat) * cos(lon);
    double v1 = sin(lat);
    double v0 = -cos(lat) * sin(lon);
    double r = sqrt(v0 * v0 + v1 * v1);
    double theta = atan2(r, s);
    double distance = double(c.crop_w) / (c.hfov);
    double x = -(theta * v0 / r) * distance;
    double y = -(theta * v1 / r) * distance;
    if (fabs(lon) < 1e-5 && fabs(lat) < 1e-5) x = y = 0;
    double rr = (sqrt(x * x + y * y)) / c.rad[4];
    double scale = (rr < c.rad[5]) ? ((c.rad[3] * rr + c.rad[2]) * rr + c.rad[1]) * rr + c.rad[0] : 1000.0;
    double rx = x * scale, ry = y * scale;
    rx += c.center_dx;
    ry += c.center_dy;
    rx /= double(c.crop_w);
    ry /= double(c.crop_h);
    rx += 0.5;
    ry += 0.5;
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

// Y is the rotated sphere point; Kannala-Brandt projection with zero rvec/tvec and alpha = 0.
OCTVR_HD void fisheye_project(const CameraParams& c, const double* Y, double* ox, double* oy) {
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

// Output pixel (u, v) in [0,1)^2 -> input camera normalized image point (x, y) or NaN.
OCTVR_HD void project_output_to_input(const CameraParams& out, const CameraParams& in, double u, double v,
                                      double* x, double* y) {
    double lon, lat, p[3], q[3];
    equirect_image_to_obj(out, u, v, &lon, &lat);
    lonlat_to_xyz(lon, lat, p);
    rotate_rows(out.Rinv, p, q);
    xyz_to_lonlat(q, &lon, &lat);
    lonlat_to_xyz(lon, lat, p);
    bool lon_ok = valid_longitude(in, lon);
    rotate_rows(in.R, p, q);
    if (in.type == CAM_FISHEYE) {
        fisheye_project(in, q, x, y);
        return;
    }
    double ll, la;
    xyz_to_lonlat(q, &ll, &la);
    double px = NAN, py = NAN;
    if (lon_ok) {
        if (in.type == CAM_FULLFRAME_FISHEYE)
            fullframe_fisheye_obj_to_image(in, ll, la, &px, &py);
        else
            equirect_obj_to_image(in, ll, la, &px, &py);
    }
    *x = px;
    *y = py;
}

}  // namespace octvr
