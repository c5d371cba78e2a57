// octvr_hip.cpp — C ABI (include/octvr_hip.h): rig (vr::MapperTemplate) and mapper (vr::Mapper).
//
// Host orchestration only; all per-pixel work runs in kernels.hip.  Exceptions never cross the
// boundary: every entry point converts them into a status code + octvr_last_error().
#include "octvr_hip.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <cfloat>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <memory>
#include <sstream>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "camera_math.hpp"
#include "host_common.hpp"
#include "json_lite.hpp"
#include "kernels.hpp"
#include "masks.hpp"

using namespace octvr;

namespace {

thread_local std::string g_last_error;

template <class F>
int guarded(F&& f) {
    try {
        f();
        return OCTVR_OK;
    } catch (const OctvrError& e) {
        g_last_error = e.what();
        return e.code;
    } catch (const std::bad_alloc&) {
        g_last_error = "out of host memory";
        return OCTVR_E_INVALID;
    } catch (const std::exception& e) {
        g_last_error = e.what();
        return OCTVR_E_PARSE;
    }
}

}  // namespace

void octvr::set_last_error(const std::string& msg) { g_last_error = msg; }

namespace {

// ---- camera setup from JSON (camera.cpp:49-136 and the per-type constructors) ------------------
void rodrigues(double rx, double ry, double rz, double R[9]) {
    // cvRodrigues2 (calib3d/src/calibration.cpp:300-345)
    double theta = sqrt(rx * rx + ry * ry + rz * rz);
    if (theta < DBL_EPSILON) {
        for (int k = 0; k < 9; k++) R[k] = (k % 4 == 0) ? 1.0 : 0.0;
        return;
    }
    static const double I[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
    double c, s;
    sin_cos(theta, &s, &c);  // gcc builds cvRodrigues2's cos / sin pair as one sincos (camera_math.hpp)
    const double c1 = 1. - c;
    double itheta = theta ? 1. / theta : 0.;
    rx *= itheta;
    ry *= itheta;
    rz *= itheta;
    double rrt[9] = {rx * rx, rx * ry, rx * rz, rx * ry, ry * ry, ry * rz, rx * rz, ry * rz, rz * rz};
    double rx_[9] = {0, -rz, ry, rz, 0, -rx, -ry, rx, 0};
    for (int k = 0; k < 9; k++) R[k] = c * I[k] + c1 * rrt[k] + s * rx_[k];
}

void mul33(const double* a, const double* b, double* d) {
    // cv::gemm len==3 path (core/src/matmul.cpp:934-1000): t*1 + 0*0
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
            double t = a[i * 3 + 0] * b[0 * 3 + j] + a[i * 3 + 1] * b[1 * 3 + j] + a[i * 3 + 2] * b[2 * 3 + j];
            d[i * 3 + j] = t * 1.0 + 0.0 * 0.0;
        }
}

void invert33(const double* S, double* D) {
    // cv::invert 3x3 closed form (core/src/lapack.cpp:709-712, 970-990)
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

// CalcCorrectionRadius_copy (fullframe_fisheye_cam.cpp:20-103)
double cube_root(double x) { return x == 0.0 ? 0.0 : x > 0.0 ? pow(x, 1.0 / 3.0) : -pow(-x, 1.0 / 3.0); }
void square_zero(const double* a, int* n, double* root) {
    if (a[2] == 0.0) {
        if (a[1] == 0.0) {
            if (a[0] == 0.0) {
                *n = 1;
                root[0] = 0.0;
            } else {
                *n = 0;
            }
        } else {
            *n = 1;
            root[0] = -a[0] / a[1];
        }
    } else if (4.0 * a[2] * a[0] > a[1] * a[1]) {
        *n = 0;
    } else {
        *n = 2;
        root[0] = (-a[1] + sqrt(a[1] * a[1] - 4.0 * a[2] * a[0])) / (2.0 * a[2]);
        root[1] = (-a[1] - sqrt(a[1] * a[1] - 4.0 * a[2] * a[0])) / (2.0 * a[2]);
    }
}
void cube_zero(const double* a, int* n, double* root) {
    if (a[3] == 0.0) {
        square_zero(a, n, root);
        return;
    }
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
        root[1] = -2.0 * sqrt(-p) * cos(phi / 3.0 + kPi / 3.0) - a[2] / (3.0 * a[3]);
        root[2] = -2.0 * sqrt(-p) * cos(phi / 3.0 - kPi / 3.0) - a[2] / (3.0 * a[3]);
    }
}
double correction_radius(const double* coeff) {
    double a[4];
    for (int k = 0; k < 4; k++) a[k] = coeff[k] != 0.0 ? (k + 1) * coeff[k] : 0.0;
    int n = 0;
    double root[3], sroot = 1000.0;
    cube_zero(a, &n, root);
    for (int i = 0; i < n; i++)
        if (root[i] > 0.0 && root[i] < sroot) sroot = root[i];
    return sroot;
}

void reject_unsupported_options(const JsonValue& o, const std::string& type) {
    // PinholeCamera overrides obj_to_image and never consults the masks (pinhole_cam.cpp:32-50), and its
    // get_include_mask would call the base obj_to_image_single, which throws (camera.hpp:92-94)
    if ((type == "fisheye" || type == "pinhole") && (o.has("include_masks") || o.has("exclude_masks")))
        throw OctvrError(OCTVR_E_UNSUPPORTED, "camera type '" + type + "' does not support include/exclude masks");
}

// The Camera constructor's mask part (camera.cpp:72-123) and draw_mask (camera.cpp:146-187): `selection`
// fills the exclude mask with 255 and clears the rectangle; `exclude_masks` areas set exclude (polygons,
// PNG red) and include (PNG green) bits; `include_masks` areas set include bits.  Empty vector = no mask.
void build_camera_masks(const JsonValue& o, std::vector<uint8_t>& excl, std::vector<uint8_t>& incl) {
    const bool any = o.has("selection") || o.has("exclude_masks") || o.has("include_masks");
    if (!any) return;
    REQUIRE(o.has("width") && o.has("height"), "camera masks need the camera's width and height");
    const int w = o["width"].as_int(), h = o["height"].as_int();
    REQUIRE(w > 0 && h > 0, "camera width/height must be positive");
    const size_t n = (size_t)w * h;
    auto prepare = [&](std::vector<uint8_t>& m, uint8_t init) {
        if (m.empty()) m.assign(n, init);
    };
    auto draw = [&](const JsonValue& areas, bool include) {
        for (size_t a = 0; a < areas.size(); a++) {
            const JsonValue& area = areas[a];
            const std::string& t = area["type"].as_string();
            const JsonValue& args = area["args"];
            if (t == "polygonal") {
                std::vector<int> pts;
                for (size_t k = 0; k + 1 < args.size(); k += 2) {
                    pts.push_back((int)args[k].as_double());
                    pts.push_back((int)args[k + 1].as_double());
                }
                fill_poly_u8(include ? incl.data() : excl.data(), w, h, pts.data(), (int)pts.size() / 2, 255);
            } else if (t == "png") {
                std::vector<uint8_t> bytes(args.size());
                for (size_t k = 0; k < args.size(); k++) bytes[k] = (uint8_t)args[k].as_int();
                int pw = 0, ph = 0;
                // CV_Assert(mask_img.size() == exclude_mask.size()) (camera.cpp:170), checked on the IHDR
                REQUIRE(!excl.empty() && w > 0 && h > 0, "png mask without a camera size");
                std::vector<uint8_t> rgb = png_decode_rgb(bytes.data(), bytes.size(), &pw, &ph, w, h);
                for (size_t k = 0; k < n; k++) {
                    if (rgb[3 * k]) excl[k] = 255;      // RED channel
                    if (rgb[3 * k + 1]) incl[k] = 255;  // GREEN channel
                }
            } else {
                throw OctvrError(OCTVR_E_INVALID, "unknown mask area type '" + t + "'");
            }
        }
    };
    if (o.has("selection")) {
        prepare(excl, 255);
        const JsonValue& sel = o["selection"];
        const int l = sel[0].as_int(), r = sel[1].as_int(), t = sel[2].as_int(), b = sel[3].as_int();
        const int rect[8] = {l, t, l, b - 1, r - 1, b - 1, r - 1, t};
        fill_poly_u8(excl.data(), w, h, rect, 4, 0);
    }
    if (o.has("exclude_masks")) {
        prepare(excl, 0);
        prepare(incl, 0);
        draw(o["exclude_masks"], false);
    }
    if (o.has("include_masks")) {
        prepare(incl, 0);
        draw(o["include_masks"], true);
    }
}

// computeTiltProjectionMatrix (imgproc/detail/distortion_model.hpp:74-94), Matx products s += a*b.
void tilt_matrix(double tauX, double tauY, double* T) {
    auto mul = [](const double* a, const double* b, double* d) {
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) {
                double v = 0;
                for (int k = 0; k < 3; k++) v += a[i * 3 + k] * b[k * 3 + j];
                d[i * 3 + j] = v;
            }
    };
    const double cX = cos(tauX), sX = sin(tauX), cY = cos(tauY), sY = sin(tauY);
    const double rx[9] = {1, 0, 0, 0, cX, sX, 0, -sX, cX};
    const double ry[9] = {cY, 0, -sY, 0, 1, 0, sY, 0, cY};
    double rxy[9];
    mul(ry, rx, rxy);
    const double pz[9] = {rxy[8], 0, -rxy[2], 0, rxy[8], -rxy[5], 0, 0, 1};
    mul(pz, rxy, T);
}

// get_ocam_model (ocam_fisheye.cpp:19-80): the calibration TXT file of the OCamCalib toolbox.
void read_ocam_file(const std::string& path, CameraParams& c) {
    FILE* f = fopen(path.c_str(), "r");
    if (!f) throw OctvrError(OCTVR_E_IO, "ocam_fisheye: cannot open " + path);
    char buf[1024];
    int ok = 1;
    auto line = [&] { ok &= fgets(buf, sizeof buf, f) != nullptr; };
    line();
    ok &= fscanf(f, "\n") >= 0;
    ok &= fscanf(f, "%d", &c.len_pol) == 1;
    ok &= c.len_pol > 0 && c.len_pol <= kOcamMaxPol;
    for (int i = 0; ok && i < c.len_pol; i++) ok &= fscanf(f, " %lf", &c.pol[i]) == 1;
    ok &= fscanf(f, "\n") >= 0;
    line();
    ok &= fscanf(f, "\n") >= 0;
    ok &= fscanf(f, "%d", &c.len_invpol) == 1;
    ok &= c.len_invpol > 0 && c.len_invpol <= kOcamMaxPol;
    for (int i = 0; ok && i < c.len_invpol; i++) ok &= fscanf(f, " %lf", &c.invpol[i]) == 1;
    ok &= fscanf(f, "\n") >= 0;
    line();
    ok &= fscanf(f, "\n") >= 0;
    ok &= fscanf(f, "%lf %lf\n", &c.xc, &c.yc) == 2;
    line();
    ok &= fscanf(f, "\n") >= 0;
    ok &= fscanf(f, "%lf %lf %lf\n", &c.oc, &c.od, &c.oe) == 3;
    line();
    ok &= fscanf(f, "\n") >= 0;
    ok &= fscanf(f, "%d %d", &c.height, &c.width) == 2;
    fclose(f);
    if (!ok) throw OctvrError(OCTVR_E_PARSE, "ocam_fisheye: malformed calibration file " + path);
}

CameraParams camera_from_json(const JsonValue& cam) {
    CameraParams c;
    memset(&c, 0, sizeof c);
    const std::string& type = cam["type"].as_string();
    static const JsonValue empty_obj = [] {
        JsonValue v;
        v.kind = JsonValue::Object;
        return v;
    }();
    const JsonValue& o = cam.has("options") ? cam["options"] : empty_obj;
    reject_unsupported_options(o, type);
    // rotation (camera.cpp:50-70)
    double rv[3] = {0, 0, 0};
    if (o.has("rotation")) {
        rv[0] = o["rotation"]["roll"].as_double();
        rv[1] = -o["rotation"]["yaw"].as_double();
        rv[2] = -o["rotation"]["pitch"].as_double();
    }
    double Rx[9], Ry[9], Rz[9], T[9];
    rodrigues(rv[0], 0, 0, Rx);
    rodrigues(0, rv[1], 0, Ry);
    rodrigues(0, 0, rv[2], Rz);
    mul33(Rx, Rz, T);
    mul33(T, Ry, c.R);
    if (o.has("rotation_matrix"))
        for (int k = 0; k < 9; k++) c.R[k] = o["rotation_matrix"][k].as_double();
    invert33(c.R, c.Rinv);
    if (o.has("longitude_selection")) {
        c.min_lon = o["longitude_selection"][0].as_double();
        c.max_lon = o["longitude_selection"][1].as_double();
        REQUIRE(c.max_lon > c.min_lon, "longitude_selection: max must exceed min");
    } else {
        c.min_lon = -kPi;
        c.max_lon = kPi;
    }
    if (type == "equirectangular") {
        c.type = CAM_EQUIRECT;
        c.min_lat = o.get("min_lat", -kPi / 2);
        c.max_lat = o.get("max_lat", kPi / 2);
        c.scale_lon = o.get("scale_lon", 1.0);
    } else if (type == "fullframe_fisheye") {
        c.type = CAM_FULLFRAME_FISHEYE;
        c.width = o["width"].as_int();
        c.height = o["height"].as_int();
        if (o.has("crop")) {
            const JsonValue& r = o["crop"]["rect"];
            c.crop_x = r[0].as_int();
            c.crop_y = r[2].as_int();
            c.crop_w = r[1].as_int() - r[0].as_int();
            c.crop_h = r[3].as_int() - r[2].as_int();
            c.crop_circular = o["crop"]["is_circular"].as_bool() ? 1 : 0;
        }
        if (c.crop_w * c.crop_h == 0) {
            c.crop_x = c.crop_y = 0;
            c.crop_w = c.width;
            c.crop_h = c.height;
            c.crop_circular = 0;
        }
        c.hfov = o["hfov"].as_double();
        c.center_dx = o["center_dx"].as_double();
        c.center_dy = o["center_dy"].as_double();
        const JsonValue& r = o["radial"];
        c.rad[3] = r[0].as_double();
        c.rad[2] = r[1].as_double();
        c.rad[1] = r[2].as_double();
        c.rad[0] = 1.0 - r[0].as_double() - r[1].as_double() - r[2].as_double();
        c.rad[4] = (c.crop_w < c.crop_h ? c.crop_w : c.crop_h) / 2.0;
        c.rad[5] = correction_radius(c.rad);
    } else if (type == "fisheye") {
        c.type = CAM_FISHEYE;
        c.fx = o["fx"].as_double();
        c.fy = o["fy"].as_double();
        c.cx = o["cx"].as_double();
        c.cy = o["cy"].as_double();
        REQUIRE(o["dist_coeffs"].size() == 4, "fisheye: dist_coeffs must have 4 entries (calib3d/src/fisheye.cpp:90)");
        for (int k = 0; k < 4; k++) c.k[k] = o["dist_coeffs"][k].as_double();
        c.width = o["width"].as_int();
        c.height = o["height"].as_int();
    } else if (type == "pinhole") {  // PinholeCamera (pinhole_cam.cpp:13-30) + cv::projectPoints
        c.type = CAM_PINHOLE;
        c.fx = o["fx"].as_double();
        c.fy = o["fy"].as_double();
        c.cx = o["cx"].as_double();
        c.cy = o["cy"].as_double();
        const size_t nd = o.has("dist_coeffs") ? o["dist_coeffs"].size() : 0;
        REQUIRE(nd == 0 || nd == 4 || nd == 5 || nd == 8 || nd == 12 || nd == 14,
                "pinhole: dist_coeffs must have 4, 5, 8, 12 or 14 entries (calibration.cpp:644-655)");
        for (size_t k = 0; k < nd; k++) c.dist[k] = o["dist_coeffs"][k].as_double();
        for (int k = 0; k < 9; k++) c.tilt[k] = (k % 4 == 0) ? 1.0 : 0.0;
        if (c.dist[12] != 0 || c.dist[13] != 0) tilt_matrix(c.dist[12], c.dist[13], c.tilt);
        c.width = o["width"].as_int();
        c.height = o["height"].as_int();
    } else if (type == "normal") {  // normal.cpp:13-22
        c.type = CAM_NORMAL;
        c.aspect = o["aspect_ratio"].as_double();
        c.cam_x = o["cam_opt"].as_double();
        c.cam_z = sqrt((1.0 - c.cam_x * c.cam_x) / (1.0 + 1.0 / c.aspect / c.aspect));
        c.cam_y = c.cam_z / c.aspect;
    } else if (type == "perspective") {  // perspective.cpp:14-19
        c.type = CAM_PERSPECTIVE;
        c.aspect = o["aspect_ratio"].as_double();
        c.sf = o["sf"].as_double();
    } else if (type == "ocam_fisheye") {  // ocam_fisheye.cpp:82-110
        c.type = CAM_OCAM;
        if (o.has("file")) {
            read_ocam_file(o["file"].as_string(), c);
        } else {
            const JsonValue& pol = o["pol"];
            const JsonValue& inv = o["invpol"];
            c.len_pol = (int)pol.size();
            c.len_invpol = (int)inv.size();
            REQUIRE(c.len_pol > 0 && c.len_pol <= kOcamMaxPol && c.len_invpol > 0 && c.len_invpol <= kOcamMaxPol,
                    "ocam_fisheye: pol / invpol must have 1..64 entries");
            for (int i = 0; i < c.len_pol; i++) c.pol[i] = pol[i].as_double();
            for (int i = 0; i < c.len_invpol; i++) c.invpol[i] = inv[i].as_double();
            c.xc = o["xc"].as_double();
            c.yc = o["yc"].as_double();
            c.oc = o["c"].as_double();
            c.od = o["d"].as_double();
            c.oe = o["e"].as_double();
            c.width = o["width"].as_int();
            c.height = o["height"].as_int();
        }
    } else if (type == "stupidoval") {
        c.type = CAM_STUPIDOVAL;
    } else if (type == "cubic") {
        c.type = CAM_CUBIC;
    } else if (type == "eqareanorthpole") {  // eqareanorthpole.hpp:11-18
        c.type = CAM_EQAREA_NORTH;
        c.circle = o.get("arctic_circle", kPi / 3);
    } else if (type == "eqareasouthpole") {  // eqareasouthpole.hpp:10-17
        c.type = CAM_EQAREA_SOUTH;
        c.circle = o.get("antarctic_circle", -kPi / 3);
    } else {
        throw OctvrError(OCTVR_E_UNSUPPORTED, "camera type '" + type + "' is not implemented in this ABI version");
    }
    if (o.has("selection")) {  // exclude everything outside the rectangle (camera.cpp:96-112)
        REQUIRE(o.has("width") && o.has("height"), "selection needs the camera's width and height");
        c.sel = 1;
        c.width = o["width"].as_int();
        c.height = o["height"].as_int();
        c.sel_l = o["selection"][0].as_int();
        c.sel_r = o["selection"][1].as_int();
        c.sel_t = o["selection"][2].as_int();
        c.sel_b = o["selection"][3].as_int();
    }
    return c;
}

double aspect_ratio(const JsonValue& cam) {
    // Camera::get_aspect_ratio overrides (equirectangular.hpp:32-34, fullframe_fisheye_cam.cpp:142-144,
    // pinhole_cam.hpp:32-34, normal.hpp:26-28, perspective.hpp:24-26, ocam_fisheye.cpp:112-114,
    // stupidoval.hpp:21-23, cubic.hpp:43-45, eqarea*.hpp: 1)
    const CameraParams c = camera_from_json(cam);
    switch (c.type) {
        case CAM_EQUIRECT:
            return (2.0f * c.scale_lon) / ((c.max_lat - c.min_lat) / kPi);
        case CAM_FULLFRAME_FISHEYE:
        case CAM_FISHEYE:
        case CAM_PINHOLE:
        case CAM_OCAM:
            return double(c.width) / c.height;
        case CAM_NORMAL:
        case CAM_PERSPECTIVE:
            return c.aspect;
        case CAM_STUPIDOVAL:
            return 2.0;
        case CAM_CUBIC:
            return 3.0 / 2.0;
        default:
            return 1.0;
    }
}

// Vignette::getMap (vignette.cpp:18-54) at 512x512.
std::vector<float> vignette_map(const JsonValue& o, int width, int height) {
    if (!o.has("vignette")) return {};
    double a = o["vignette"][0].as_double(), b = o["vignette"][1].as_double(), c = o["vignette"][2].as_double(),
           d = o["vignette"][3].as_double();
    if (o.has("exposure")) {
        float ev = (float)std::pow(2.0, o["exposure"].as_double());
        a /= ev;
        b /= ev;
        c /= ev;
        d /= ev;
    }
    std::vector<float> m((size_t)width * height);
    for (int j = 0; j < height; j++)
        for (int i = 0; i < width; i++) {
#define P(X) (float(X) * float(X))
            float r = std::sqrt(P(i - width / 2) + P(j - height / 2)) / std::sqrt(P(width / 2) + P(height / 2));
#undef P
            m[(size_t)j * width + i] = (float)(1.0 / (a + r * r * (b + r * r * (c + d * r * r))));
        }
    return m;
}

// MapperTemplate::add_input (template.cpp:46-153).  `visible` (W x H device bytes, 1 = claimed by an
// include mask) is allocated by the caller once some camera has include masks; `priors` are the inputs
// added before this one, whose masks lose the pixels this camera's include mask claims (:102-116).
void build_input(const CameraParams& out_cam, const JsonValue& cam, int W, int H, bool use_roi, int device,
                 RigInput& in, DevBuf<uint8_t>* visible = nullptr, std::vector<RigInput>* priors = nullptr) {
    CameraParams c = camera_from_json(cam);
    DeviceGuard dg(device);
    std::vector<uint8_t> excl, incl;
    if (cam.has("options")) build_camera_masks(cam["options"], excl, incl);
    DevBuf<uint8_t> excl_d, incl_d;
    if (!excl.empty() || !incl.empty()) {
        c.sel = 0;  // the selection rectangle is rasterised into the exclude mask
        c.width = cam["options"]["width"].as_int();
        c.height = cam["options"]["height"].as_int();
    }
    if (!excl.empty()) {
        excl_d.upload(excl.data(), excl.size());
        c.excl = excl_d.p;
        if (!incl.empty()) {
            incl_d.upload(incl.data(), incl.size());
            c.incl = incl_d.p;
        }
    }
    const size_t total_px = (size_t)W * H;
    if (visible && c.incl && !visible->p) {
        visible->alloc(total_px);
        HIP_CHECK(hipMemset(visible->p, 0, total_px));
    }
    uint8_t* vis_p = visible ? visible->p : nullptr;
    const size_t total = (size_t)W * H;
    REQUIRE(total < ((size_t)1 << 32), "output frame must have fewer than 2^32 pixels");
    DevBuf<float> m1, m2;
    DevBuf<uint8_t> mk;
    DevBuf<int32_t> bb;
    m1.alloc(total);
    m2.alloc(total);
    mk.alloc(total);
    bb.alloc(4);
    const CameraParams both[2] = {out_cam, c};
    DevBuf<CameraParams> cams;
    cams.upload(both, 2);
    // fragile pixels (LutGuard, camera_math.hpp): a list of at most `cap` indices, grown and the kernel
    // re-run if it overflows (the build is idempotent: it writes visible_mask only with 2)
    uint32_t cap = (uint32_t)std::min<size_t>(total, std::max<size_t>(1 << 16, total / 256));
    std::vector<uint32_t> frag;
    int32_t b[4];
    for (;;) {
        DevBuf<uint32_t> fr;
        fr.alloc((size_t)cap + 1);
        HIP_CHECK(hipMemset(fr.p, 0, sizeof(uint32_t)));
        const int32_t init[4] = {INT32_MAX, INT32_MAX, -1, -1};
        HIP_CHECK(hipMemcpy(bb.p, init, sizeof init, hipMemcpyHostToDevice));
        HIP_CHECK(launch_lut_build(cams.p, W, H, m1.p, m2.p, mk.p, bb.p, vis_p, fr.p, cap, nullptr));
        HIP_CHECK(hipDeviceSynchronize());
        uint32_t count = 0;
        HIP_CHECK(hipMemcpy(&count, fr.p, sizeof count, hipMemcpyDeviceToHost));
        if (count > cap) {
            cap = count;
            continue;
        }
        frag.resize(count);
        if (count) HIP_CHECK(hipMemcpy(frag.data(), fr.p + 1, sizeof(uint32_t) * count, hipMemcpyDeviceToHost));
        HIP_CHECK(hipMemcpy(b, bb.p, sizeof b, hipMemcpyDeviceToHost));
        break;
    }
    // the fragile pixels with glibc: the reference's arithmetic exactly (camera_math.hpp on the host)
    std::sort(frag.begin(), frag.end());
    CameraParams ch = c;
    ch.excl = excl.empty() ? nullptr : excl.data();
    ch.incl = (excl.empty() || incl.empty()) ? nullptr : incl.data();
    struct Fix {
        float x, y;
        bool vis;
    };
    std::vector<Fix> fix(frag.size());
    {
        const bool want_vis = vis_p != nullptr;
        std::vector<double> fx(frag.size()), fy(frag.size());
        std::vector<uint8_t> fv(frag.size());
        parallel_for(frag.size(), [&](size_t k) {
            const uint32_t idx = frag[k];
            const int h = (int)(idx / (uint32_t)W), w = (int)(idx - (uint32_t)h * (uint32_t)W);
            bool v = false;
            project_output_to_input(out_cam, ch, (double)w / W, (double)h / H, &fx[k], &fy[k], want_vis ? &v : nullptr);
            fv[k] = v ? 1 : 0;
        });
        for (size_t k = 0; k < frag.size(); k++) fix[k] = Fix{(float)fx[k], (float)fy[k], fv[k] != 0};
    }
    std::vector<uint8_t> vh;  // visible_mask on the host, when this camera reads or writes it
    if (vis_p && (!frag.empty() || c.incl)) {
        vh.resize(total);
        HIP_CHECK(hipMemcpy(vh.data(), vis_p, total, hipMemcpyDeviceToHost));
    }
    std::vector<uint8_t> fvalid(frag.size());
    for (size_t k = 0; k < frag.size(); k++) {  // lut_build_kernel's per-pixel tail, in index order
        const uint32_t idx = frag[k];
        const bool claimed = !vh.empty() && vh[idx] == 1;
        if (!vh.empty() && fix[k].vis && !claimed) vh[idx] = 2;
        const float x = fix[k].x, y = fix[k].y;
        const bool valid = !(std::isnan(x) || std::isnan(y) || x < 0 || x >= 1.0f || y < 0 || y >= 1.0f || claimed);
        fvalid[k] = valid;
        if (valid) {
            const int h = (int)(idx / (uint32_t)W), w = (int)(idx - (uint32_t)h * (uint32_t)W);
            b[0] = std::min(b[0], w);
            b[1] = std::min(b[1], h);
            b[2] = std::max(b[2], w);
            b[3] = std::max(b[3], h);
        }
    }
    in.n_fragile = frag.size();
    // CV_Assert(min_h <= max_h && min_w <= max_w) (template.cpp:124)
    if (!(b[1] <= b[3] && b[0] <= b[2])) throw OctvrError(OCTVR_E_INVALID, "input camera covers no output pixel");
    int min_w = std::max(0, b[0] - 8), min_h = std::max(0, b[1] - 8);
    int max_w = std::min(W - 1, b[2] + 8), max_h = std::min(H - 1, b[3] + 8);
    int roi[4] = {min_w, min_h, max_w + 1 - min_w, max_h + 1 - min_h};
    if (!use_roi) {
        roi[0] = roi[1] = 0;
        roi[2] = W;
        roi[3] = H;
    }
    memcpy(in.roi, roi, sizeof roi);
    const size_t rn = (size_t)roi[2] * roi[3];
    in.map1.resize(rn);
    in.map2.resize(rn);
    in.mask.resize(rn);
    const size_t off = (size_t)roi[1] * W + roi[0];
    HIP_CHECK(hipMemcpy2D(in.map1.data(), roi[2] * sizeof(float), m1.p + off, W * sizeof(float), roi[2] * sizeof(float),
                          roi[3], hipMemcpyDeviceToHost));
    HIP_CHECK(hipMemcpy2D(in.map2.data(), roi[2] * sizeof(float), m2.p + off, W * sizeof(float), roi[2] * sizeof(float),
                          roi[3], hipMemcpyDeviceToHost));
    HIP_CHECK(hipMemcpy2D(in.mask.data(), roi[2], mk.p + off, W, roi[2], roi[3], hipMemcpyDeviceToHost));
    for (size_t k = 0; k < frag.size(); k++) {  // patch the recomputed pixels (every valid one is in the ROI)
        const uint32_t idx = frag[k];
        const int h = (int)(idx / (uint32_t)W), w = (int)(idx - (uint32_t)h * (uint32_t)W);
        const int rx = w - roi[0], ry = h - roi[1];
        if (rx < 0 || ry < 0 || rx >= roi[2] || ry >= roi[3]) continue;
        const size_t j = (size_t)ry * roi[2] + rx;
        in.mask[j] = fvalid[k] ? 255 : 0;
        in.map1[j] = fvalid[k] ? fix[k].x : -1.0f;
        in.map2[j] = fvalid[k] ? fix[k].y : -1.0f;
    }
    if (c.incl && priors) {  // pixels this camera claimed first (2) leave the earlier cameras' masks
        for (RigInput& p : *priors) {
            if (&p == &in) break;
            for (int y = 0; y < p.roi[3]; y++)
                for (int x = 0; x < p.roi[2]; x++)
                    if (vh[(size_t)(y + p.roi[1]) * W + x + p.roi[0]] == 2) p.mask[(size_t)y * p.roi[2] + x] = 0;
        }
    }
    if (c.incl) {
        for (uint8_t& v : vh) v = v ? 1 : 0;
        HIP_CHECK(hipMemcpy(vis_p, vh.data(), total, hipMemcpyHostToDevice));
    }
    const JsonValue& o = cam["options"];
    in.in_w = o.has("width") ? o["width"].as_int() : 0;
    in.in_h = o.has("height") ? o["height"].as_int() : 0;
    in.vignette = vignette_map(o, 512, 512);
    if (!in.vignette.empty()) in.vig_w = in.vig_h = 512;
}

// ---- VRv11 .dat (template.cpp:206-314) -----------------------------------------------------------
constexpr const char* kDatMagic = "VRv11";
constexpr int CV_8UC1 = 0, CV_32FC1 = 5;

struct DatWriter {
    std::ostream& f;
    void i64(int64_t v) { f.write(reinterpret_cast<const char*>(&v), 8); }
    void mat(int type, int rows, int cols, const void* data, size_t elem) {
        i64(type);
        i64(rows);
        i64(cols);
        if (rows * cols == 0 || !data) return;
        f.write(reinterpret_cast<const char*>(data), (std::streamsize)((size_t)rows * cols * elem));
    }
    void input(const RigInput& in) {
        for (int k = 0; k < 4; k++) i64(in.roi[k]);
        mat(CV_32FC1, in.roi[3], in.roi[2], in.map1.data(), 4);
        mat(CV_32FC1, in.roi[3], in.roi[2], in.map2.data(), 4);
        mat(CV_8UC1, in.roi[3], in.roi[2], in.mask.data(), 1);
        if (in.vignette.empty())
            mat(0, 0, 0, nullptr, 1);  // empty cv::Mat: type 0, 0x0 (Mat() header)
        else
            mat(CV_32FC1, in.vig_h, in.vig_w, in.vignette.data(), 4);
    }
};

struct DatReader {
    std::istream& f;
    int64_t i64() {
        int64_t v = 0;
        f.read(reinterpret_cast<char*>(&v), 8);
        if (!f) throw OctvrError(OCTVR_E_PARSE, "truncated .dat file");
        return v;
    }
    // Rmat: returns rows, cols, type; data appended to `out` (bytes)
    void mat(int want_type, int& rows, int& cols, std::vector<uint8_t>& out) {
        const int64_t type = i64(), r64 = i64(), c64 = i64();
        out.clear();
        // cv::Mat dimensions are non-negative ints; bound the element count before allocating
        if (r64 < 0 || c64 < 0 || r64 > INT32_MAX || c64 > INT32_MAX)
            throw OctvrError(OCTVR_E_PARSE, ".dat: bad Mat dimensions");
        rows = (int)r64;
        cols = (int)c64;
        if ((int64_t)rows * cols == 0) {
            rows = cols = 0;
            return;
        }
        if ((uint64_t)rows * (uint64_t)cols > ((uint64_t)1 << 34))
            throw OctvrError(OCTVR_E_PARSE, ".dat: Mat too large");
        if (want_type >= 0 && type != want_type) throw OctvrError(OCTVR_E_PARSE, "unexpected Mat type in .dat");
        size_t elem = type == CV_32FC1 ? 4 : type == CV_8UC1 ? 1 : 0;
        if (!elem) throw OctvrError(OCTVR_E_PARSE, "unsupported Mat type in .dat");
        out.resize((size_t)rows * cols * elem);
        f.read(reinterpret_cast<char*>(out.data()), (std::streamsize)out.size());
        if (!f) throw OctvrError(OCTVR_E_PARSE, "truncated .dat file");
    }
    // ROI x, y >= 0, w, h > 0 and inside the out_w x out_h frame (as octvr_rig_create_from_arrays)
    void input(RigInput& in, int out_w, int out_h) {
        int64_t roi[4];
        for (int k = 0; k < 4; k++) roi[k] = i64();
        // no sums of untrusted int64 fields: each bound is checked against the frame before the next
        // one is derived from it (roi[0] = INT64_MAX, w = 1 must not wrap into range)
        if (roi[0] < 0 || roi[1] < 0 || roi[0] > out_w || roi[1] > out_h || roi[2] <= 0 || roi[3] <= 0 ||
            roi[2] > out_w - roi[0] || roi[3] > out_h - roi[1])
            throw OctvrError(OCTVR_E_PARSE, ".dat: ROI outside the output frame");
        for (int k = 0; k < 4; k++) in.roi[k] = (int)roi[k];
        std::vector<uint8_t> b;
        int r, c;
        mat(CV_32FC1, r, c, b);
        in.map1.resize((size_t)r * c);
        memcpy(in.map1.data(), b.data(), b.size());
        mat(CV_32FC1, r, c, b);
        in.map2.resize((size_t)r * c);
        memcpy(in.map2.data(), b.data(), b.size());
        mat(CV_8UC1, r, c, b);
        in.mask = b;
        const size_t roi_px = (size_t)in.roi[2] * (size_t)in.roi[3];
        if (in.map1.size() != roi_px || in.map2.size() != roi_px || in.mask.size() != roi_px)
            throw OctvrError(OCTVR_E_PARSE, ".dat: map / mask size does not match ROI");
        mat(-1, r, c, b);
        in.vignette.resize(b.size() / 4);
        if (!b.empty()) memcpy(in.vignette.data(), b.data(), b.size());
        in.vig_w = c;
        in.vig_h = r;
    }
};

// std::streambuf over the C ABI's read / write callbacks (octvr_rig_load_stream / dump_stream).
struct CbOutBuf : std::streambuf {
    octvr_write_fn fn;
    void* ctx;
    char buf[1 << 16];
    CbOutBuf(octvr_write_fn f, void* c) : fn(f), ctx(c) { setp(buf, buf + sizeof buf); }
    bool flush_buf() {
        const size_t n = (size_t)(pptr() - pbase());
        if (n && fn(ctx, pbase(), n) != n) return false;
        setp(buf, buf + sizeof buf);
        return true;
    }
    int overflow(int c) override {
        if (!flush_buf()) return traits_type::eof();
        if (c != traits_type::eof()) {
            *pptr() = (char)c;
            pbump(1);
        }
        return traits_type::not_eof(c);
    }
    int sync() override { return flush_buf() ? 0 : -1; }
};
struct CbInBuf : std::streambuf {
    octvr_read_fn fn;
    void* ctx;
    char buf[1 << 16];
    CbInBuf(octvr_read_fn f, void* c) : fn(f), ctx(c) { setg(buf, buf, buf); }
    int underflow() override {
        const size_t n = fn(ctx, buf, sizeof buf);
        if (n == 0) return traits_type::eof();
        setg(buf, buf, buf + n);
        return traits_type::to_int_type(buf[0]);
    }
};

// MapperTemplate::dump body (template.cpp:206-256)
void dat_write(octvr_rig& rig, std::ostream& os) {
    if (rig.seam_masks.empty()) rig_create_masks(rig);  // MapperTemplate::dump (template.cpp:209-210)
    REQUIRE(rig.seam_masks.size() == rig.inputs.size(), "seam mask count does not match the inputs");
    DatWriter w{os};
    w.f.write(kDatMagic, 5);
    w.i64(rig.out_w);
    w.i64(rig.out_h);
    w.i64((int64_t)rig.inputs.size());
    for (auto& in : rig.inputs) w.input(in);
    for (size_t i = 0; i < rig.seam_masks.size(); i++) {
        const RigInput& in = rig.inputs[i];
        w.mat(CV_8UC1, in.roi[3], in.roi[2], rig.seam_masks[i].data(), 1);
    }
    w.i64((int64_t)rig.overlays.size());
    for (auto& in : rig.overlays) w.input(in);
    w.f.flush();
    if (!w.f) throw OctvrError(OCTVR_E_IO, "write failed");
}

// MapperTemplate(std::ifstream&) body (template.cpp:258-314)
std::unique_ptr<octvr_rig> dat_read(std::istream& is) {
    DatReader r{is};
    char magic[5];
    r.f.read(magic, 5);
    if (!r.f || strncmp(magic, kDatMagic, 5) != 0)
        throw OctvrError(OCTVR_E_PARSE, "Invalid data file (version does not match)");
    auto rig = std::make_unique<octvr_rig>();
    const int64_t ow = r.i64(), oh = r.i64();
    if (ow <= 0 || oh <= 0 || ow > 65535 || oh > 65535) throw OctvrError(OCTVR_E_PARSE, ".dat: bad output size");
    rig->out_w = (int)ow;
    rig->out_h = (int)oh;
    int64_t n = r.i64();
    if (n < 0 || n > kMaxCams) throw OctvrError(OCTVR_E_PARSE, ".dat: bad input count");
    rig->inputs.resize(n);
    for (auto& in : rig->inputs) r.input(in, rig->out_w, rig->out_h);
    rig->seam_masks.resize(n);
    for (int64_t i = 0; i < n; i++) {
        int rr, cc;
        r.mat(CV_8UC1, rr, cc, rig->seam_masks[i]);
        // MapperTemplate::dump writes one ROI-sized seam mask per input (template.cpp:245-246)
        if (rig->seam_masks[i].size() != (size_t)rig->inputs[i].roi[2] * (size_t)rig->inputs[i].roi[3])
            throw OctvrError(OCTVR_E_PARSE, ".dat: seam mask size does not match ROI");
    }
    int64_t no = r.i64();
    if (no < 0 || no > kMaxCams) throw OctvrError(OCTVR_E_PARSE, ".dat: bad overlay count");
    rig->overlays.resize(no);
    for (auto& in : rig->overlays) r.input(in, rig->out_w, rig->out_h);
    return rig;
}

// MapperTemplate(to, to_opts, w, h) (template.cpp:23-44): the output camera and size
std::unique_ptr<octvr_rig> rig_new(const JsonValue& oc, int out_w, int out_h, int device) {
    CameraParams out_cam = camera_from_json(oc);
    REQUIRE(!(out_h <= 0 && out_w <= 0), "Output width/height invalid");  // template.cpp:32-33
    double ar = aspect_ratio(oc);
    if (out_h <= 0) out_h = int(double(out_w) / ar);
    if (out_w <= 0) out_w = int(double(out_h) * ar);
    // the output camera needs image_to_obj_single: fisheye / pinhole throw NotImplemented (camera.hpp:101-103)
    if (out_cam.type == CAM_FISHEYE || out_cam.type == CAM_PINHOLE)
        throw OctvrError(OCTVR_E_UNSUPPORTED, "output camera type '" + oc["type"].as_string() + "' is not supported");
    // CV_Assert(crop.size() == size && crop.tl() == Point(0, 0)) (fullframe_fisheye_cam.cpp:224)
    if (out_cam.type == CAM_FULLFRAME_FISHEYE)
        REQUIRE(out_cam.crop_x == 0 && out_cam.crop_y == 0 && out_cam.crop_w == out_cam.width &&
                    out_cam.crop_h == out_cam.height,
                "fullframe_fisheye output camera: crop must cover the whole image");
    auto rig = std::make_unique<octvr_rig>();
    rig->out_w = out_w;
    rig->out_h = out_h;
    rig->device = device;
    // the camera models stay with the rig for add_input / morph_controlpoints
    rig->has_cameras = true;
    rig->out_cam = out_cam;
    rig->out_cam_masks = oc.has("options") && (oc["options"].has("exclude_masks") || oc["options"].has("include_masks"));
    return rig;
}

// MapperTemplate::add_input(from, from_opts, overlay, use_roi) (template.cpp:46-153)
void rig_add(octvr_rig& rig, const JsonValue& cam, bool overlay, bool use_roi) {
    REQUIRE(rig.has_cameras, "add_input needs a template built from camera models (not a .dat)");
    REQUIRE(rig.inputs.size() + rig.overlays.size() < (size_t)kMaxCams, "too many inputs");
    std::vector<RigInput>& dst = overlay ? rig.overlays : rig.inputs;
    RigInput in;
    // overlays go through the same add_input: they share visible_mask and their include masks clear
    // the (non-overlay) inputs' masks (template.cpp:102-116, 147-150)
    build_input(rig.out_cam, cam, rig.out_w, rig.out_h, use_roi, rig.device, in, &rig.visible, &rig.inputs);
    dst.push_back(std::move(in));
    if (!overlay) rig.cams.push_back(camera_from_json(cam));
    rig.seam_masks.clear();  // one seam mask per input: create_masks again (dump does)
}

}  // namespace

// =================================================================================================
// Mapper (vr::Mapper)
// =================================================================================================
struct octvr_mapper {
    int device = 0;
    int n = 0;
    int W = 0, H = 0;
    int use_gain = 0;
    std::vector<int> in_w, in_h;
    // tiled composite LUT (kernels.hpp), blend = 0
    TiledLutDev tiles;
    int n_tiles = 0;
    // multi-band blend state, blend > 0 (multiband_host.cpp)
    std::unique_ptr<MultiBand, MultiBandDeleter> mb;
    int blend = 0;
    DevBuf<double> gains;
    // gain feed
    DevBuf<CompositeEntry> samples;  // working-scale samples that lie in some pair intersection
    DevBuf<uint16_t> partners;       // per sample: bit j = the sample is in the (camera, j) intersection
    DevBuf<unsigned long long> totals;  // [kGainMaxCams][kGainMaxCams] exact pair sums, units of 2^-23
    DevBuf<int32_t> N;
    DevBuf<uint32_t> tickets;        // 8 per-XCD + 1 global last-workgroup-done counters
    int n_chunks = 0, n_samples = 0;
    size_t n_entries = 0;
    std::vector<double> last_gains;
    std::vector<DevBuf<float>> vig;  // per camera: vignette map resized to the input size, or empty
    SourceFootprint foot;            // the input bytes this mapper's kernels read (host_common.hpp)
    int tex = 0;                     // OCTVR_REMAP_TEXTURE: texture-convention entries (make_entry_tex)
    // scaled output (scaled_output_size != stitch size, mapper.cpp:69,153-155,290-306): the RGB result
    // as an RGBA frame, resized + converted to YUV420P by a second kernel
    int SW = 0, SH = 0;
    bool scaled = false;
    DevBuf<uint8_t> result;
    DevBuf<MbCamLevel> result_view;  // the result frame as a one-entry RGBA sink of the composite
    // Per-frame device state that consecutive stitches would otherwise share: the gains, the feed's
    // pair totals and tickets, the composite's work queue.  Slot 0 is the buffers above;
    // octvr_mapper_set_frames_in_flight adds slots so that stitches issued on different streams overlap
    // (frame k+1's gain feed runs under frame k's composite).  A stitch takes the next slot in turn and
    // waits only for that slot's previous stitch when it was issued on another stream.
    struct FrameSlot {
        double* gains = nullptr;
        unsigned long long* totals = nullptr;
        uint32_t* tickets = nullptr;
        uint32_t* queue = nullptr;
        hipEvent_t done = nullptr;  // recorded after the slot's last stitch (its stream may since be gone)
    };
    struct SlotBufs {
        DevBuf<double> gains;
        DevBuf<unsigned long long> totals;
        DevBuf<uint32_t> tickets, queue;
    };
    std::vector<FrameSlot> slots;
    std::vector<std::unique_ptr<SlotBufs>> slot_bufs;  // owners of slots 1..k-1
    int cur_slot = 0;                                  // slot of the last stitch
    int timing = 0;             // event-timing period in stitches (0 = off)
    uint64_t timed_calls = 0;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> events, free_events;  // recorded / reusable
    ~octvr_mapper() {
        for (auto& sl : slots)
            if (sl.done) (void)hipEventDestroy(sl.done);
        for (auto* v : {&events, &free_events})
            for (auto& e : *v) {
                (void)hipEventDestroy(e.first);
                (void)hipEventDestroy(e.second);
            }
    }
};

namespace {

float resize_inv_scale(int d, int s) {
    // cudawarping/src/resize.cpp:82-83,105
    double f = (double)d / s;
    return (float)(1.0 / f);
}

// cuda::resize INTER_LINEAR on u8 (glob path, resize.cu:71-103); nvcc's default FMA contraction of
// `out + src * w` is reproduced with explicit fmaf.
std::vector<uint8_t> resize_linear_u8(const uint8_t* src, int sw, int sh, int dw, int dh) {
    std::vector<uint8_t> dst((size_t)dw * dh);
    float fx = resize_inv_scale(dw, sw), fy = resize_inv_scale(dh, sh);
    for (int y = 0; y < dh; y++)
        for (int x = 0; x < dw; x++) {
            float src_x = x * fx, src_y = y * fy;
            int x1 = (int)floorf(src_x), y1 = (int)floorf(src_y);
            int x2 = x1 + 1, y2 = y1 + 1;
            int x2r = std::min(x2, sw - 1), y2r = std::min(y2, sh - 1);
            float out = 0.f;
            out = fmaf((float)src[(size_t)y1 * sw + x1], (x2 - src_x) * (y2 - src_y), out);
            out = fmaf((float)src[(size_t)y1 * sw + x2r], (src_x - x1) * (y2 - src_y), out);
            out = fmaf((float)src[(size_t)y2r * sw + x1], (x2 - src_x) * (src_y - y1), out);
            out = fmaf((float)src[(size_t)y2r * sw + x2r], (src_x - x1) * (src_y - y1), out);
            int v = !(out > 0.f) ? 0 : out >= 255.f ? 255 : (int)rintf(out);
            dst[(size_t)y * dw + x] = (uint8_t)v;
        }
    return dst;
}

// cuda::resize INTER_LINEAR on f32 (the texture LinearFilter path, filters.hpp:79-117, taken for an
// upscale without a stream): same taps and weights as resize_linear with clamped borders; nvcc's FMA
// contraction of `out + src * w` reproduced with explicit fmaf.
std::vector<float> resize_linear_f32(const float* src, int sw, int sh, int dw, int dh) {
    std::vector<float> dst((size_t)dw * dh);
    float fx = resize_inv_scale(dw, sw), fy = resize_inv_scale(dh, sh);
    for (int y = 0; y < dh; y++)
        for (int x = 0; x < dw; x++) {
            float src_x = x * fx, src_y = y * fy;
            int x1 = (int)floorf(src_x), y1 = (int)floorf(src_y);
            int x2 = x1 + 1, y2 = y1 + 1;
            int x2r = std::min(x2, sw - 1), y2r = std::min(y2, sh - 1);
            float out = 0.f;
            out = fmaf(src[(size_t)y1 * sw + x1], (x2 - src_x) * (y2 - src_y), out);
            out = fmaf(src[(size_t)y1 * sw + x2r], (src_x - x1) * (y2 - src_y), out);
            out = fmaf(src[(size_t)y2r * sw + x1], (x2 - src_x) * (src_y - y1), out);
            out = fmaf(src[(size_t)y2r * sw + x2r], (src_x - x1) * (src_y - y1), out);
            dst[(size_t)y * dw + x] = out;
        }
    return dst;
}

// Working-scale gain setup: Mapper ctor (mapper.cpp:94-114,140-142) + GainCompensatorGPU ctor
// (exposure_compensate.cpp:174-221).  Produces per-pair sample entries of both cameras for every
// pixel of the bitwise-AND intersection of the resized masks, N(i,j), and chunking — on the host only
// (plan_gain), then uploaded (setup_gain).
struct GainPlan {
    std::vector<CompositeEntry> samples;
    std::vector<uint16_t> partners;
    std::vector<int32_t> N;
    int n_chunks = 0;
    size_t pairs_px = 0;
};

GainPlan plan_gain(const octvr_rig& rig, int n, const std::vector<int>& in_w, const std::vector<int>& in_h, int tex) {
    double ws = std::min(1.0, std::sqrt(0.1 * 1e6 / ((double)rig.out_w * rig.out_h)));
    std::vector<std::array<int, 4>> wr(n);
    std::vector<std::vector<uint8_t>> smask(n);
    std::vector<std::vector<CompositeEntry>> samp(n);
    std::vector<int32_t> N((size_t)n * n, 0);
    for (int i = 0; i < n; i++) {
        const RigInput& in = rig.inputs[i];
        wr[i] = {(int)(in.roi[0] * ws), (int)(in.roi[1] * ws), (int)(in.roi[2] * ws), (int)(in.roi[3] * ws)};
        const int ww = wr[i][2], wh = wr[i][3];
        REQUIRE(ww > 0 && wh > 0, "working-scale ROI is empty");
        smask[i] = resize_linear_u8(in.mask.data(), in.roi[2], in.roi[3], ww, wh);
        // warped -> working scale: resize_nearest (resize.cu:57-69), src index = trunc(dst * (float)(1/f))
        float fx = resize_inv_scale(ww, in.roi[2]), fy = resize_inv_scale(wh, in.roi[3]);
        samp[i].resize((size_t)ww * wh);
        for (int y = 0; y < wh; y++)
            for (int x = 0; x < ww; x++) {
                int sx = (int)(x * fx), sy = (int)(y * fy);
                size_t k = (size_t)sy * in.roi[2] + sx;
                CompositeEntry e{0, 0};
                if (in.mask[k])
                    e = tex ? make_entry_tex(in.map1[k], in.map2[k], (float)in_w[i], (float)in_h[i], i)
                            : make_entry(in.map1[k], in.map2[k], (float)in_w[i], (float)in_h[i], i);
                samp[i][(size_t)y * ww + x] = e;
            }
        int nz = 0;
        for (uint8_t v : smask[i]) nz += v != 0;
        N[(size_t)i * n + i] = std::max(1, nz);
    }
    // samples: working pixel k of camera i joins I(i,j) (exposure_compensate.cpp:262-277) for every
    // camera j whose resized-mask intersection holds it -> one entry plus a partner bit per pixel
    std::vector<std::vector<uint16_t>> partner(n);
    for (int i = 0; i < n; i++) partner[i].assign(samp[i].size(), 0);
    for (int i = 0; i < n; i++)
        for (int j = i + 1; j < n; j++) {
            const auto &a = wr[i], &b = wr[j];
            int x0 = std::max(a[0], b[0]), y0 = std::max(a[1], b[1]);
            int x1 = std::min(a[0] + a[2], b[0] + b[2]), y1 = std::min(a[1] + a[3], b[1] + b[3]);
            if (x1 <= x0 || y1 <= y0) {  // overlap_roi.area() == 0
                N[(size_t)i * n + j] = N[(size_t)j * n + i] = 1;
                continue;
            }
            int nz = 0;
            for (int y = y0; y < y1; y++)
                for (int x = x0; x < x1; x++) {
                    size_t ka = (size_t)(y - a[1]) * a[2] + (x - a[0]);
                    size_t kb = (size_t)(y - b[1]) * b[2] + (x - b[0]);
                    if ((smask[i][ka] & smask[j][kb]) == 0) continue;
                    nz++;
                    partner[i][ka] |= (uint16_t)(1u << j);
                    partner[j][kb] |= (uint16_t)(1u << i);
                }
            N[(size_t)i * n + j] = N[(size_t)j * n + i] = std::max(1, nz);
        }
    // per camera: the samples with a partner, ordered by (source row, source column) so the lanes of
    // a wave gather from a few neighbouring source lines; invalid (mask 0) samples read as 0 and go last
    std::vector<CompositeEntry> uniq;
    std::vector<uint16_t> pmask;
    int n_chunks = 0;  // workgroups of kGainChunk samples (4 single-camera wave runs each)
    for (int i = 0; i < n; i++) {
        std::vector<uint32_t> ks;
        for (size_t k = 0; k < samp[i].size(); k++)
            if (partner[i][k]) ks.push_back((uint32_t)k);
        auto key = [&](uint32_t k) {
            const CompositeEntry& e = samp[i][k];
            const uint64_t valid = (e.code & 0x8000u) ? 0 : 1;
            return (valid << 60) | ((uint64_t)(e.xy >> 16) << 24) | (uint64_t)(e.xy & 0xFFFFu);
        };
        std::stable_sort(ks.begin(), ks.end(), [&](uint32_t a, uint32_t b) { return key(a) < key(b); });
        const int begin = (int)uniq.size();
        for (uint32_t k : ks) {
            CompositeEntry e = samp[i][k];
            if (!(e.code & 0x8000u)) e.code = (uint16_t)(i << 10);  // a zero sample of camera i
            uniq.push_back(e);
            pmask.push_back(partner[i][k]);
        }
        while ((uniq.size() - begin) % kGainWaveRun) {  // pad: invalid samples of camera i, no partners
            uniq.push_back(CompositeEntry{0u, (uint32_t)(i << 10)});
            pmask.push_back(0);
        }
    }
    while (uniq.size() % kGainChunk) {  // whole workgroups
        uniq.push_back(CompositeEntry{0u, 0u});
        pmask.push_back(0);
    }
    n_chunks = (int)(uniq.size() / kGainChunk);
    // exactness bound of the fixed-point totals (kernels.hip, gain feed): < 2^21 samples per camera
    for (int i = 0; i < n; i++) REQUIRE(samp[i].size() < (1u << 21), "working-scale ROI too large for exact gain sums");
    GainPlan g;
    g.samples = std::move(uniq);
    g.partners = std::move(pmask);
    g.N = std::move(N);
    g.n_chunks = n_chunks;
    for (uint16_t pm : g.partners) g.pairs_px += (size_t)__builtin_popcount(pm);
    return g;
}

void setup_gain(octvr_mapper& m, const octvr_rig& rig) {
    const GainPlan g = plan_gain(rig, m.n, m.in_w, m.in_h, m.tex);
    for (const CompositeEntry& e : g.samples) m.foot.mark_taps(e);
    m.samples.upload(g.samples.data(), g.samples.size());
    m.partners.upload(g.partners.data(), g.partners.size());
    m.totals.alloc((size_t)kGainMaxCams * kGainMaxCams * kGainTotalStride);
    HIP_CHECK(hipMemset(m.totals.p, 0, sizeof(unsigned long long) * kGainMaxCams * kGainMaxCams * kGainTotalStride));
    m.N.upload(g.N.data(), g.N.size());
    m.tickets.alloc(9);
    HIP_CHECK(hipMemset(m.tickets.p, 0, sizeof(uint32_t) * 9));
    m.n_chunks = g.n_chunks;
    m.n_samples = (int)g.samples.size();
    m.n_entries = g.pairs_px;
}

}  // namespace

// =================================================================================================
// extern "C" entry points
// =================================================================================================
namespace octvr {

// The RGB(A) result frame of the scaled-output and preview paths (allocated on first use).
void ensure_result(octvr_mapper& m) {
    if (m.result.p) return;
    REQUIRE((uint64_t)m.W * m.H * 4 < 0x7FFFFF80ull, "stitch frame larger than 2 GiB as RGBA");
    DeviceGuard dg(m.device);
    // result = 0 (mapper.cpp:156): pixels no camera writes stay black in every frame
    m.result.alloc((size_t)m.W * m.H * 4);
    HIP_CHECK(hipMemset(m.result.p, 0, m.result.n));
    MbCamLevel v{};
    v.g_off = 0;
    v.g_pitch = (uint32_t)m.W * 4;
    v.w = m.W;
    v.h = m.H;
    m.result_view.upload(&v, 1);
}

namespace {

void check_out_pitch(const octvr_mapper* m, size_t out_pitch) {
    REQUIRE(out_pitch >= (size_t)m->SW, "output pitch smaller than width");
    // the stitch kernel addresses the output through a buffer resource with 32-bit offsets
    REQUIRE((uint64_t)out_pitch * (m->SH + m->SH / 2) < 0x7FFFFF80ull, "output frame larger than 2 GiB");
}

// The kernels' view of one frame's inputs, with the limits of their address arithmetic checked.
FrameSet frame_set(const octvr_mapper* m, const uint8_t* const* in_dev, const size_t* in_pitch) {
    FrameSet fs;
    memset(&fs, 0, sizeof fs);
    for (int i = 0; i < m->n; i++) {
        REQUIRE(in_dev[i] && in_pitch[i] >= (size_t)m->in_w[i], "bad input frame");
        // the staging loads form row offsets with 24-bit multiplies (kernels.hip stage_load)
        REQUIRE(in_pitch[i] < ((size_t)1 << 24), "input pitch must be below 16 MiB");
        // the gain feed reads frames through 32-bit buffer resources
        REQUIRE((uint64_t)in_pitch[i] * (uint64_t)(m->in_h[i] + m->in_h[i] / 2) < 0x7FFFFFFFull,
                "input frame larger than 2 GiB");
        // ... in 8-byte segments (kernels.hip feed_rows)
        REQUIRE((uint64_t)in_pitch[i] * (uint64_t)(m->in_h[i] + m->in_h[i] / 2) >= 8, "input frame below 8 bytes");
        fs.f[i] = SourceFrame{in_dev[i], m->in_w[i], m->in_h[i], (int64_t)in_pitch[i], m->vig[i].p};
    }
    return fs;
}

// The frame's gains into its slot: copied from another mapper (gains_dev), set (gains), or estimated by the
// gain feed (GainCompensatorGPU::feed, exposure_compensate.cpp:223-297).
void stitch_gains(octvr_mapper* m, octvr_mapper::FrameSlot& sl, const FrameSet& fs, const double* gains, int n_gains,
                  const double* gains_dev, hipStream_t s) {
    if (!m->use_gain) return;
    if (gains_dev) {
        HIP_CHECK(hipMemcpyAsync(sl.gains, gains_dev, sizeof(double) * m->n, hipMemcpyDeviceToDevice, s));
    } else if (gains) {
        REQUIRE(n_gains == m->n, "gains must have one entry per input");
        HIP_CHECK(launch_set_gains(gains, m->n, sl.gains, s));
    } else if (m->n_chunks == 0) {  // no intersections: A = diag(b), every gain is 1
        const std::vector<double> ones(m->n, 1.0);
        HIP_CHECK(launch_set_gains(ones.data(), m->n, sl.gains, s));
    } else {
        // with frames in flight the feed runs beside the previous frame's composite: the lean
        // variant fits next to it (the wide-prefetch one waits for its workgroups to drain)
        const bool lean = m->slots.size() > 1;
        HIP_CHECK(launch_gain_feed(fs, m->samples.p, m->partners.p, m->tex, m->n_chunks, m->N.p, m->n, sl.totals,
                                   sl.tickets, sl.gains, s, lean));
    }
}

// The timing events of this stitch, or none (octvr_mapper_set_timing: every `timing`-th stitch)
std::pair<hipEvent_t, hipEvent_t> stitch_events(octvr_mapper* m) {
    hipEvent_t e0 = nullptr, e1 = nullptr;
    const bool timed = m->timing > 0 && (m->timed_calls++ % (uint64_t)m->timing) == 0;
    if (!timed) return {e0, e1};
    if (m->free_events.empty()) {
        HIP_CHECK(hipEventCreate(&e0));
        HIP_CHECK(hipEventCreate(&e1));
    } else {
        e0 = m->free_events.back().first;
        e1 = m->free_events.back().second;
        m->free_events.pop_back();
    }
    return {e0, e1};
}

}  // namespace

// Mapper::stitch (mapper.cpp:193-323).  gains_dev (device, n doubles): gains of another mapper of the
// same inputs, copied stream-ordered (AsyncMultiMapper's gain_modes chaining, async.cpp:78-86).
void mapper_stitch(octvr_mapper* m, const uint8_t* const* in_dev, const size_t* in_pitch, uint8_t* out_dev,
                   size_t out_pitch, const double* gains, int n_gains, const double* gains_dev, hipStream_t s,
                   const PreviewOut* preview) {
    {
        REQUIRE(m && in_dev && in_pitch && out_dev, "NULL argument");
        if (preview) {
            REQUIRE(preview->dev && preview->w > 0 && preview->h > 0 && preview->pitch >= (size_t)preview->w * 3,
                    "bad preview output");
            // the preview resizes the whole-frame RGB result, which one frame slot owns
            REQUIRE(m->slots.size() == 1, "preview output needs one frame in flight");
            ensure_result(*m);
        }
        check_out_pitch(m, out_pitch);
        DeviceGuard dg(m->device);
        const FrameSet fs = frame_set(m, in_dev, in_pitch);
        // stitches sharing a frame slot (gains, feed totals, work counters) are ordered: each waits for
        // the slot's previous stitch (with one slot: for the previous stitch, as vr::Mapper is not
        // re-entrant either).  Always through the event, never by comparing stream handles: a destroyed
        // stream's handle value can come back as a new stream that is not ordered after the old one.
        const int k = (m->cur_slot + 1) % (int)m->slots.size();
        octvr_mapper::FrameSlot& sl = m->slots[k];
        if (sl.done) HIP_CHECK(hipStreamWaitEvent(s, sl.done, 0));
        stitch_gains(m, sl, fs, gains, n_gains, gains_dev, s);
        const auto ev = stitch_events(m);
        hipEvent_t e0 = ev.first, e1 = ev.second;
        const bool timed = e0 != nullptr;
        if (timed && (m->scaled || m->mb || preview)) HIP_CHECK(hipEventRecord(e0, s));  // else the composite records its own
        if (m->scaled || preview) {
            // stitch at template size into the RGB(A) result, then resize + RGB -> YUV420P (mapper.cpp:290-306)
            // (one frame slot only: the result frame is shared); without scaling the resize is the identity
            if (m->mb)
                multiband_run(*m->mb, 0, fs, sl.gains, m->use_gain, nullptr, 0, s, m->result.p, (int64_t)m->W * 4);
            else
                HIP_CHECK(launch_mb_remap(fs, m->tiles.view, sl.gains, m->use_gain,
                                          RgbaOut{m->result.p, (uint32_t)m->result.n, m->result_view.p}, s));
            HIP_CHECK(launch_resize_rgba_yuv420(m->result.p, m->W, m->H, (int64_t)m->W * 4, out_dev, m->SW, m->SH,
                                                (int64_t)out_pitch, s));
            if (preview)  // cuda::resize(result, preview_output, ...) (mapper.cpp:308-312)
                HIP_CHECK(launch_resize_rgba_rgb(m->result.p, m->W, m->H, (int64_t)m->W * 4, preview->dev, preview->w,
                                                 preview->h, (int64_t)preview->pitch, s));
        } else if (m->mb) {
            multiband_run(*m->mb, k, fs, sl.gains, m->use_gain, out_dev, (int64_t)out_pitch, s);
        } else {
            TiledLut view = m->tiles.view;
            view.queue = sl.queue;
            HIP_CHECK(launch_stitch(fs, view, m->W, m->H, sl.gains, m->use_gain, out_dev, (int64_t)out_pitch, s, e0, e1));
        }
        if (timed) {
            if (m->scaled || m->mb || preview) HIP_CHECK(hipEventRecord(e1, s));
            m->events.emplace_back(e0, e1);
        }
        if (!sl.done) HIP_CHECK(hipEventCreateWithFlags(&sl.done, hipEventDisableTiming));
        HIP_CHECK(hipEventRecord(sl.done, s));
        m->cur_slot = k;
    }
}

// nb frames (1, 2 or 4) of the same rig in one composite launch (FrameBatch, kernels.hpp): each frame's
// gains into its own frame slot (nb consecutive slots, each waited for as mapper_stitch waits for one),
// then one pass over the tiled LUT for all of them.  Scaled-output and multi-band / feather mappers have no
// batched kernel: their frames are stitched one by one.
void mapper_stitch_batch(octvr_mapper* m, int nb, const uint8_t* const* in_dev, const size_t* in_pitch,
                         uint8_t* const* out_dev, size_t out_pitch, const double* gains, hipStream_t s) {
    REQUIRE(m && in_dev && in_pitch && out_dev, "NULL argument");
    REQUIRE(nb == 1 || nb == 2 || nb == 4, "a batch holds 1, 2 or 4 frames");
    for (int f = 0; f < nb; f++) REQUIRE(out_dev[f], "NULL output");
    if (nb == 1 || m->scaled || m->mb) {
        for (int f = 0; f < nb; f++)
            mapper_stitch(m, in_dev + (size_t)f * m->n, in_pitch + (size_t)f * m->n, out_dev[f], out_pitch,
                          gains ? gains + (size_t)f * m->n : nullptr, gains ? m->n : 0, nullptr, s);
        return;
    }
    REQUIRE((int)m->slots.size() >= nb, "a batch of n frames needs n frames in flight (octvr_mapper_set_frames_in_flight)");
    REQUIRE(nb <= 2 || m->n <= 16, "a batch of 4 frames holds 16 cameras per frame");
    check_out_pitch(m, out_pitch);
    DeviceGuard dg(m->device);
    FrameSet fs[kMaxBatch];
    const double* g[kMaxBatch];
    int ks[kMaxBatch];
    int k = m->cur_slot;
    const bool feed = m->use_gain && !gains && m->n_chunks > 0;  // every frame's gains estimated: one feed launch
    unsigned long long* tot[kMaxBatch];
    uint32_t* tick[kMaxBatch];
    double* gd[kMaxBatch];
    for (int f = 0; f < nb; f++) {
        k = (k + 1) % (int)m->slots.size();
        ks[f] = k;
        octvr_mapper::FrameSlot& sl = m->slots[k];
        fs[f] = frame_set(m, in_dev + (size_t)f * m->n, in_pitch + (size_t)f * m->n);
        if (sl.done) HIP_CHECK(hipStreamWaitEvent(s, sl.done, 0));
        if (!feed) stitch_gains(m, sl, fs[f], gains ? gains + (size_t)f * m->n : nullptr, gains ? m->n : 0, nullptr, s);
        g[f] = sl.gains;
        tot[f] = sl.totals;
        tick[f] = sl.tickets;
        gd[f] = sl.gains;
    }
    if (feed)  // GainCompensatorGPU::feed of each frame (exposure_compensate.cpp:223-297), all in one launch
        HIP_CHECK(launch_gain_feed_batch(fs, nb, m->samples.p, m->partners.p, m->tex, m->n_chunks, m->N.p, m->n, tot, tick,
                                         gd, s, true));
    const auto ev = stitch_events(m);
    TiledLut view = m->tiles.view;
    view.queue = m->slots[ks[0]].queue;  // this launch's work counters (the first frame's slot)
    HIP_CHECK(launch_stitch_batch(fs, nb, view, m->W, m->H, g, m->use_gain, out_dev, (int64_t)out_pitch, s, ev.first,
                                  ev.second));
    if (ev.first) m->events.emplace_back(ev.first, ev.second);
    for (int f = 0; f < nb; f++) {
        octvr_mapper::FrameSlot& sl = m->slots[ks[f]];
        if (!sl.done) HIP_CHECK(hipEventCreateWithFlags(&sl.done, hipEventDisableTiming));
        HIP_CHECK(hipEventRecord(sl.done, s));
    }
    m->cur_slot = ks[nb - 1];
}

int mapper_num_inputs(const octvr_mapper* m) { return m->n; }
bool mapper_has_gain(const octvr_mapper* m) { return m->use_gain != 0; }
const double* mapper_gains_dev(const octvr_mapper* m) { return m->slots[m->cur_slot].gains; }
const SourceFootprint& mapper_footprint(const octvr_mapper* m) { return m->foot; }
void mapper_out_size(const octvr_mapper* m, int* w, int* h) {
    *w = m->SW;
    *h = m->SH;
}


}  // namespace octvr

extern "C" {

int octvr_abi_version(void) { return OCTVR_HIP_ABI_VERSION; }

const char* octvr_last_error(void) { return g_last_error.c_str(); }

int octvr_device_count(int* count) {
    return guarded([&] {
        REQUIRE(count, "count is NULL");
        HIP_CHECK(hipGetDeviceCount(count));
    });
}

int octvr_dev_malloc(int device, size_t bytes, void** ptr) {
    return guarded([&] {
        REQUIRE(ptr, "ptr is NULL");
        DeviceGuard dg(device);
        HIP_CHECK(hipMalloc(ptr, bytes));
    });
}

int octvr_dev_free(void* ptr) {
    return guarded([&] { HIP_CHECK(hipFree(ptr)); });
}

int octvr_memcpy_h2d(void* dst, const void* src, size_t bytes) {
    return guarded([&] { HIP_CHECK(hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice)); });
}

int octvr_fill_poly_u8(uint8_t* img, int w, int h, const int* pts, int npts, uint8_t color) {
    return guarded([&] {
        REQUIRE(img && w > 0 && h > 0 && (pts || npts == 0) && npts >= 0, "bad arguments");
        fill_poly_u8(img, w, h, pts, npts, color);
    });
}

int octvr_png_decode_rgb(const uint8_t* png, size_t n, uint8_t* rgb, size_t rgb_cap, int* w, int* h) {
    return guarded([&] {
        REQUIRE(png && w && h, "bad arguments");
        std::vector<uint8_t> v = png_decode_rgb(png, n, w, h);
        if (rgb) {
            REQUIRE(rgb_cap >= v.size(), "rgb buffer too small");
            memcpy(rgb, v.data(), v.size());
        }
    });
}

int octvr_memcpy_d2h(void* dst, const void* src, size_t bytes) {
    return guarded([&] { HIP_CHECK(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost)); });
}

int octvr_stream_sync(void* stream) {
    return guarded([&] { HIP_CHECK(hipStreamSynchronize((hipStream_t)stream)); });
}

int octvr_rig_create_json(const char* json, int out_w, int out_h, int use_roi, int device, octvr_rig** out) {
    return guarded([&] {
        REQUIRE(json && out, "json/out is NULL");
        JsonValue doc = json_parse(json);
        auto rig = rig_new(doc["output"], out_w, out_h, device);
        // apps/octvr/dump.cpp:84-93: every input, then every overlay, through add_input
        const JsonValue& ins = doc["inputs"];
        for (size_t i = 0; i < ins.size(); i++) rig_add(*rig, ins[i], false, use_roi != 0);
        if (doc.has("overlays")) {
            const JsonValue& ov = doc["overlays"];
            for (size_t i = 0; i < ov.size(); i++) rig_add(*rig, ov[i], true, use_roi != 0);
        }
        *out = rig.release();
    });
}

// camera {"type": type, "options": opts} from the C++ API's separate type / options arguments
static JsonValue camera_json(const char* type, const char* opts_json, int flags) {
    REQUIRE(type && *type, "camera type is empty");
    for (const char* c = type; *c; c++)
        REQUIRE((*c >= 'a' && *c <= 'z') || (*c >= '0' && *c <= '9') || *c == '_', "bad camera type");
    const std::string text = std::string("{\"type\":\"") + type + "\",\"options\":" +
                             (opts_json && *opts_json ? opts_json : "{}") + "}";
    return json_parse(text, (flags & OCTVR_JSON_EXACT) != 0);
}

int octvr_rig_create(const char* out_type, const char* out_opts_json, int out_w, int out_h, int device, int flags,
                     octvr_rig** out) {
    return guarded([&] {
        REQUIRE(out, "out is NULL");
        auto rig = rig_new(camera_json(out_type, out_opts_json, flags), out_w, out_h, device);
        *out = rig.release();
    });
}

int octvr_rig_add_input(octvr_rig* rig, const char* type, const char* opts_json, int overlay, int use_roi, int flags) {
    return guarded([&] {
        REQUIRE(rig, "rig is NULL");
        rig_add(*rig, camera_json(type, opts_json, flags), overlay != 0, use_roi != 0);
    });
}

int octvr_rig_create_from_arrays(int out_w, int out_h, int n, const int* rois, const float* const* map1,
                                 const float* const* map2, const uint8_t* const* masks,
                                 const uint8_t* const* seams, octvr_rig** out) {
    return guarded([&] {
        REQUIRE(out && rois && map1 && map2 && masks && n > 0 && out_w > 0 && out_h > 0, "bad arguments");
        auto rig = std::make_unique<octvr_rig>();
        rig->out_w = out_w;
        rig->out_h = out_h;
        rig->inputs.resize(n);
        for (int i = 0; i < n; i++) {
            RigInput& in = rig->inputs[i];
            memcpy(in.roi, rois + 4 * i, 4 * sizeof(int));
            REQUIRE(in.roi[0] >= 0 && in.roi[1] >= 0 && in.roi[2] > 0 && in.roi[3] > 0 &&
                        in.roi[0] <= out_w - in.roi[2] && in.roi[1] <= out_h - in.roi[3],  // no int overflow
                    "ROI outside the output frame");
            size_t k = (size_t)in.roi[2] * in.roi[3];
            in.map1.assign(map1[i], map1[i] + k);
            in.map2.assign(map2[i], map2[i] + k);
            in.mask.assign(masks[i], masks[i] + k);
        }
        if (seams) {
            rig->seam_masks.resize(n);
            for (int i = 0; i < n; i++) {
                size_t k = (size_t)rig->inputs[i].roi[2] * rig->inputs[i].roi[3];
                rig->seam_masks[i].assign(seams[i], seams[i] + k);
            }
        }
        *out = rig.release();
    });
}

int octvr_rig_load_dat(const char* path, octvr_rig** out) {
    return guarded([&] {
        REQUIRE(path && out, "path/out is NULL");
        std::ifstream f(path, std::ios::binary);
        if (!f) throw OctvrError(OCTVR_E_IO, std::string("cannot open ") + path);
        *out = dat_read(f).release();
    });
}

int octvr_rig_load_stream(octvr_read_fn read, void* ctx, octvr_rig** out) {
    return guarded([&] {
        REQUIRE(read && out, "read/out is NULL");
        CbInBuf buf(read, ctx);
        std::istream is(&buf);
        *out = dat_read(is).release();
    });
}

int octvr_rig_create_masks(octvr_rig* rig, int device) {
    return guarded([&] {
        REQUIRE(rig, "rig is NULL");
        rig->device = device;
        rig_create_masks(*rig);
    });
}

int octvr_rig_dump_dat(octvr_rig* rig, const char* path) {
    return guarded([&] {
        REQUIRE(rig && path, "rig/path is NULL");
        if (rig->seam_masks.empty()) rig_create_masks(*rig);  // before opening: no half-written file on error
        std::ofstream f(path, std::ios::binary);
        if (!f) throw OctvrError(OCTVR_E_IO, std::string("cannot open ") + path);
        dat_write(*rig, f);
    });
}

int octvr_rig_dump_stream(octvr_rig* rig, octvr_write_fn write, void* ctx) {
    return guarded([&] {
        REQUIRE(rig && write, "rig/write is NULL");
        CbOutBuf buf(write, ctx);
        std::ostream os(&buf);
        dat_write(*rig, os);
    });
}

int octvr_rig_set_vignette(octvr_rig* rig, int i, int overlay, const float* map, int w, int h) {
    return guarded([&] {
        REQUIRE(rig && i >= 0, "bad arguments");
        std::vector<RigInput>& v = overlay ? rig->overlays : rig->inputs;
        REQUIRE(i < (int)v.size(), "bad input index");
        REQUIRE(map ? (w > 0 && h > 0) : (w == 0 && h == 0), "bad vignette size");
        v[i].vignette.assign(map, map + (size_t)w * h);
        v[i].vig_w = w;
        v[i].vig_h = h;
    });
}

int octvr_rig_add_overlay_arrays(octvr_rig* rig, const int* roi, const float* map1, const float* map2,
                                 const uint8_t* mask) {
    return guarded([&] {
        REQUIRE(rig && roi && map1 && map2 && mask, "bad arguments");
        REQUIRE(rig->inputs.size() + rig->overlays.size() < (size_t)kMaxCams, "too many inputs");
        REQUIRE(roi[0] >= 0 && roi[1] >= 0 && roi[2] > 0 && roi[3] > 0 && roi[0] <= rig->out_w - roi[2] &&
                    roi[1] <= rig->out_h - roi[3],
                "ROI outside the output frame");
        RigInput in;
        memcpy(in.roi, roi, sizeof in.roi);
        const size_t k = (size_t)roi[2] * roi[3];
        in.map1.assign(map1, map1 + k);
        in.map2.assign(map2, map2 + k);
        in.mask.assign(mask, mask + k);
        rig->overlays.push_back(std::move(in));
    });
}

int octvr_rig_num_inputs(const octvr_rig* rig, int* n) {
    return guarded([&] {
        REQUIRE(rig && n, "NULL argument");
        *n = (int)rig->inputs.size();
    });
}

int octvr_rig_out_size(const octvr_rig* rig, int* w, int* h) {
    return guarded([&] {
        REQUIRE(rig && w && h, "NULL argument");
        *w = rig->out_w;
        *h = rig->out_h;
    });
}

int octvr_rig_get_input(const octvr_rig* rig, int i, octvr_input_view* v) {
    return guarded([&] {
        REQUIRE(rig && v && i >= 0 && i < (int)rig->inputs.size(), "bad input index");
        const RigInput& in = rig->inputs[i];
        v->roi_x = in.roi[0];
        v->roi_y = in.roi[1];
        v->roi_w = in.roi[2];
        v->roi_h = in.roi[3];
        v->map1 = in.map1.data();
        v->map2 = in.map2.data();
        v->mask = in.mask.data();
        v->seam_mask = i < (int)rig->seam_masks.size() ? rig->seam_masks[i].data() : nullptr;
        v->vignette = in.vignette.empty() ? nullptr : in.vignette.data();
        v->vignette_w = in.vig_w;
        v->vignette_h = in.vig_h;
    });
}

int octvr_rig_num_overlays(const octvr_rig* rig, int* n) {
    return guarded([&] {
        REQUIRE(rig && n, "NULL argument");
        *n = (int)rig->overlays.size();
    });
}

int octvr_rig_get_overlay(const octvr_rig* rig, int i, octvr_input_view* v) {
    return guarded([&] {
        REQUIRE(rig && v && i >= 0 && i < (int)rig->overlays.size(), "bad overlay index");
        const RigInput& in = rig->overlays[i];
        v->roi_x = in.roi[0];
        v->roi_y = in.roi[1];
        v->roi_w = in.roi[2];
        v->roi_h = in.roi[3];
        v->map1 = in.map1.data();
        v->map2 = in.map2.data();
        v->mask = in.mask.data();
        v->seam_mask = nullptr;
        v->vignette = in.vignette.empty() ? nullptr : in.vignette.data();
        v->vignette_w = in.vig_w;
        v->vignette_h = in.vig_h;
    });
}

int octvr_rig_morph_controlpoints(octvr_rig* rig, const char* control_points_json, int* n_used) {
    return guarded([&] {
        REQUIRE(rig && control_points_json, "NULL argument");
        if (rig->has_cameras && rig->out_cam_masks)
            throw OctvrError(OCTVR_E_UNSUPPORTED, "morph_controlpoints with output-camera masks is not implemented");
        const JsonValue cps = json_parse(control_points_json);
        const int k = rig_morph_controlpoints(*rig, cps);
        if (n_used) *n_used = k;
    });
}

int octvr_rig_get_triangles(const octvr_rig* rig, int i, float* src, float* dst, int cap, int* n) {
    return guarded([&] {
        REQUIRE(rig && n && i >= 0 && i < (int)rig->inputs.size(), "bad input index");
        const RigInput& in = rig->inputs[i];
        const int nt = (int)in.src_tris.size() / 6;
        *n = nt;
        if (src && dst) {
            REQUIRE(cap >= nt, "triangle buffer too small");
            std::copy(in.src_tris.begin(), in.src_tris.end(), src);
            std::copy(in.dst_tris.begin(), in.dst_tris.end(), dst);
        }
    });
}

void octvr_rig_destroy(octvr_rig* rig) { delete rig; }

int octvr_rig_clone(const octvr_rig* src, octvr_rig** out) {
    return guarded([&] {
        REQUIRE(src && out, "NULL argument");
        auto r = std::make_unique<octvr_rig>();
        r->out_w = src->out_w;
        r->out_h = src->out_h;
        r->device = src->device;
        r->inputs = src->inputs;
        r->overlays = src->overlays;
        r->seam_masks = src->seam_masks;
        r->has_cameras = src->has_cameras;
        r->out_cam_masks = src->out_cam_masks;
        r->out_cam = src->out_cam;
        r->cams = src->cams;
        if (src->visible.p) {  // the include-mask visibility state (template.cpp:86-116) travels with the copy
            DeviceGuard dg(src->device);
            r->visible.alloc(src->visible.n);
            HIP_CHECK(hipMemcpy(r->visible.p, src->visible.p, src->visible.n, hipMemcpyDeviceToDevice));
        }
        *out = r.release();
    });
}

int octvr_mapper_create(const octvr_rig* rig, int device, int n_inputs, const int* in_w, const int* in_h, int blend,
                        int enable_gain, int scale_w, int scale_h, octvr_mapper** out) {
    return octvr_mapper_create_ex(rig, device, n_inputs, in_w, in_h, blend, enable_gain, scale_w, scale_h, 0, out);
}

int octvr_mapper_create_ex(const octvr_rig* rig, int device, int n_inputs, const int* in_w, const int* in_h, int blend,
                           int enable_gain, int scale_w, int scale_h, int flags, octvr_mapper** out) {
    return guarded([&] {
        REQUIRE(rig && out && in_w && in_h, "NULL argument");
        REQUIRE((flags & ~OCTVR_REMAP_TEXTURE) == 0, "unknown mapper flags");
        if (!rig->overlays.empty())  // checked first: the real reason, whatever n_inputs says
            throw OctvrError(OCTVR_E_UNSUPPORTED, "overlay inputs are not implemented in this ABI version");
        REQUIRE(n_inputs == (int)rig->inputs.size(), "in_sizes must cover every input");
        REQUIRE((int)rig->inputs.size() <= kMaxCams, "too many inputs");
        REQUIRE(scale_w >= 0 && scale_h >= 0 && (scale_w == 0) == (scale_h == 0), "bad scaled output size");
        REQUIRE(rig->out_w % 2 == 0 && rig->out_h % 2 == 0, "YUV420 output needs even width/height");
        auto m = std::make_unique<octvr_mapper>();
        m->device = device;
        m->tex = (flags & OCTVR_REMAP_TEXTURE) ? 1 : 0;
        m->n = (int)rig->inputs.size();
        m->W = rig->out_w;
        m->H = rig->out_h;
        // scaled_output_size = scale_output.area() == 0 ? mt.out_size : scale_output (mapper.cpp:69)
        m->SW = scale_w ? scale_w : m->W;
        m->SH = scale_h ? scale_h : m->H;
        REQUIRE(m->SW % 2 == 0 && m->SH % 2 == 0, "YUV420 output needs even width/height");
        m->scaled = m->SW != m->W || m->SH != m->H;
        REQUIRE(!m->scaled || (uint64_t)m->W * m->H * 4 < 0x7FFFFF80ull, "stitch frame larger than 2 GiB as RGBA");
        m->in_w.assign(in_w, in_w + n_inputs);
        m->in_h.assign(in_h, in_h + n_inputs);
        for (int i = 0; i < m->n; i++)
            REQUIRE(m->in_w[i] > 0 && m->in_h[i] > 0 && m->in_w[i] % 2 == 0 && m->in_h[i] % 2 == 0 &&
                        m->in_w[i] <= 65535 && m->in_h[i] <= 65535,
                    "input sizes must be even and < 65536");
        // mapper.cpp:78-82: a single input disables gain (and blend)
        m->use_gain = (enable_gain && m->n > 1) ? 1 : 0;
        m->blend = m->n > 1 ? blend : 0;
        REQUIRE(!m->use_gain || m->n <= 16, "gain estimation supports at most 16 inputs");
        DeviceGuard dg(device);
        // vignette: cv::cuda::resize(vignette, vignette_maps[i], in_size) (mapper.cpp:108-112), applied to
        // every source pixel before the remap (mapper.cpp:230-231)
        m->vig.resize(m->n);
        for (int i = 0; i < m->n; i++) {
            const RigInput& in = rig->inputs[i];
            if (in.vignette.empty()) continue;
            const std::vector<float> v = resize_linear_f32(in.vignette.data(), in.vig_w, in.vig_h, m->in_w[i], m->in_h[i]);
            m->vig[i].upload(v.data(), v.size());
        }
        m->foot.init(m->in_w, m->in_h);
        if (m->blend > 0) {
            // MultiBandGPUBlender(seam_masks, rois, bands), bands = ceil(log2(blend)) - 1 (mapper.cpp:171-176)
            const int bands = (int)(std::ceil(std::log((double)m->blend) / std::log(2.)) - 1.);
            m->mb.reset(multiband_create(*rig, device, bands, m->in_w, m->in_h, 0, &m->foot, m->tex));
        } else if (m->blend < 0) {
            // FeatherGPUBlender(masks, rois, border = -blend) (mapper.cpp:177-182)
            m->mb.reset(multiband_create(*rig, device, 0, m->in_w, m->in_h, -m->blend, &m->foot, m->tex));
        } else {
            // per-camera templates -> device, composite LUT, then drop the per-camera maps
            std::vector<DevBuf<float>> m1(m->n), m2(m->n);
            std::vector<DevBuf<uint8_t>> mk(m->n);
            std::vector<CamTemplate> ct(m->n);
            for (int i = 0; i < m->n; i++) {
                const RigInput& in = rig->inputs[i];
                m1[i].upload(in.map1.data(), in.map1.size());
                m2[i].upload(in.map2.data(), in.map2.size());
                mk[i].upload(in.mask.data(), in.mask.size());
                ct[i] = CamTemplate{m1[i].p, m2[i].p, mk[i].p, in.roi[0], in.roi[1], in.roi[2], in.roi[3],
                                    m->in_w[i], m->in_h[i]};
            }
            DevBuf<CamTemplate> ctd;
            ctd.upload(ct.data(), ct.size());
            DevBuf<CompositeEntry> lut;
            lut.alloc((size_t)m->W * m->H);
            HIP_CHECK(launch_composite_lut(ctd.p, m->n, m->W, m->H, lut.p, nullptr, m->tex));
            HIP_CHECK(hipDeviceSynchronize());
            std::vector<CompositeEntry> lut8((size_t)m->W * m->H);
            HIP_CHECK(hipMemcpy(lut8.data(), lut.p, lut8.size() * sizeof(CompositeEntry), hipMemcpyDeviceToHost));
            lut.reset();
            for (int i = 0; i < m->n; i++) {
                m1[i].reset();
                m2[i].reset();
                mk[i].reset();
            }
            // items of 128 x 16 (two quads per lane, OCTVR_QPL) for the per-frame composite
            const int qpl = composite_qpl();
            const int tx_n = (m->W + kTileW - 1) / kTileW, ty_n = (m->H + kTileH * qpl - 1) / (kTileH * qpl);
            std::vector<TileJob> jobs;
            jobs.reserve((size_t)tx_n * ty_n);
            for (int ty = 0; ty < ty_n; ty++)
                for (int tx = 0; tx < tx_n; tx++) jobs.push_back(TileJob{tx, ty, 0});
            const int W = m->W, H = m->H;
            const TiledLutBuild tb = build_tiled_lut(jobs, [&](int, int x, int y) {
                return (x < W && y < H) ? lut8[(size_t)y * W + x] : CompositeEntry{0u, 0u};
            }, m->in_w, m->in_h, qpl);
            footprint_add_tiles(m->foot, tb);
            m->tiles.upload(tb);
            m->n_tiles = tx_n * ty_n;
        }
        if (m->scaled) ensure_result(*m);
        m->gains.alloc(kMaxCams);
        std::vector<double> ones(kMaxCams, 1.0);
        HIP_CHECK(hipMemcpy(m->gains.p, ones.data(), kMaxCams * sizeof(double), hipMemcpyHostToDevice));
        m->last_gains.assign(m->n, 1.0);
        if (m->use_gain) setup_gain(*m, *rig);
        octvr_mapper::FrameSlot s0;
        s0.gains = m->gains.p;
        s0.totals = m->totals.p;
        s0.tickets = m->tickets.p;
        s0.queue = m->tiles.view.queue;
        m->slots.push_back(s0);
        *out = m.release();
    });
}

int octvr_mapper_stitch_yuv420p(octvr_mapper* m, const uint8_t* const* in_dev, const size_t* in_pitch,
                                uint8_t* out_dev, size_t out_pitch, const double* gains, int n_gains, void* stream) {
    return guarded([&] {
        mapper_stitch(m, in_dev, in_pitch, out_dev, out_pitch, gains, n_gains, nullptr, (hipStream_t)stream);
    });
}

int octvr_mapper_stitch_batch(octvr_mapper* m, int n_frames, const uint8_t* const* in_dev, const size_t* in_pitch,
                              uint8_t* const* out_dev, size_t out_pitch, const double* gains, void* stream) {
    return guarded([&] {
        mapper_stitch_batch(m, n_frames, in_dev, in_pitch, out_dev, out_pitch, gains, (hipStream_t)stream);
    });
}

int octvr_mapper_stitch_preview(octvr_mapper* m, const uint8_t* const* in_dev, const size_t* in_pitch,
                                uint8_t* out_dev, size_t out_pitch, uint8_t* preview_dev, int preview_w, int preview_h,
                                size_t preview_pitch, const double* gains, int n_gains, void* stream) {
    return guarded([&] {
        const PreviewOut pv{preview_dev, preview_w, preview_h, preview_pitch};
        mapper_stitch(m, in_dev, in_pitch, out_dev, out_pitch, gains, n_gains, nullptr, (hipStream_t)stream,
                      preview_dev ? &pv : nullptr);
    });
}

int octvr_mapper_gains(octvr_mapper* m, double* g, int n) {
    return guarded([&] {
        REQUIRE(m && g && n >= m->n, "bad arguments");
        DeviceGuard dg(m->device);
        if (!m->use_gain) {
            for (int i = 0; i < n; i++) g[i] = 1.0;
            return;
        }
        const octvr_mapper::FrameSlot& sl = m->slots[m->cur_slot];
        if (sl.done) HIP_CHECK(hipEventSynchronize(sl.done));
        HIP_CHECK(hipMemcpy(g, sl.gains, m->n * sizeof(double), hipMemcpyDeviceToHost));
    });
}

int octvr_mapper_set_frames_in_flight(octvr_mapper* m, int k) {
    return guarded([&] {
        REQUIRE(m && k >= 1 && k <= OCTVR_MAX_FRAMES_IN_FLIGHT, "frames in flight must be 1..OCTVR_MAX_FRAMES_IN_FLIGHT");
        if (k > 1 && m->scaled)
            throw OctvrError(OCTVR_E_UNSUPPORTED, "frames in flight > 1 need the output at template size (no scaled output)");
        DeviceGuard dg(m->device);
        for (auto& sl : m->slots)
            if (sl.done) HIP_CHECK(hipEventSynchronize(sl.done));
        if (m->cur_slot != 0) {  // keep the last frame's gains for gains() / chaining
            HIP_CHECK(hipMemcpy(m->slots[0].gains, m->slots[m->cur_slot].gains, sizeof(double) * m->n,
                                hipMemcpyDeviceToDevice));
            m->cur_slot = 0;
        }
        for (size_t i = 1; i < m->slots.size(); i++)
            if (m->slots[i].done) (void)hipEventDestroy(m->slots[i].done);
        m->slots.resize(1);
        m->slot_bufs.clear();
        std::vector<double> ones(kMaxCams, 1.0);
        for (int i = 1; i < k; i++) {
            auto b = std::make_unique<octvr_mapper::SlotBufs>();
            b->gains.upload(ones.data(), ones.size());
            if (m->totals.p) {
                b->totals.alloc(m->totals.n);
                HIP_CHECK(hipMemset(b->totals.p, 0, b->totals.n * sizeof(unsigned long long)));
            }
            if (m->tickets.p) {
                b->tickets.alloc(m->tickets.n);
                HIP_CHECK(hipMemset(b->tickets.p, 0, b->tickets.n * sizeof(uint32_t)));
            }
            if (m->tiles.queue.n) {
                b->queue.alloc(m->tiles.queue.n);
                HIP_CHECK(hipMemset(b->queue.p, 0, b->queue.n * sizeof(uint32_t)));
            }
            octvr_mapper::FrameSlot sl;
            sl.gains = b->gains.p;
            sl.totals = b->totals.p;
            sl.tickets = b->tickets.p;
            sl.queue = b->queue.p;
            m->slots.push_back(sl);
            m->slot_bufs.push_back(std::move(b));
        }
        if (m->mb) multiband_set_slots(*m->mb, k);
        HIP_CHECK(hipDeviceSynchronize());  // the memsets complete before any stream uses the slots
    });
}

int octvr_mapper_traffic(const octvr_mapper* m, double* bytes) {
    return guarded([&] {
        REQUIRE(m && bytes, "NULL argument");
        // composite kernel: 4 B tiled-LUT entry (8 B in wide tiles) + 1.5 B YUV420 output per output
        // pixel, the unique source bytes its staged boxes cover (YUV420P, 1.5 B per luma pixel: the
        // circular crops leave the rest of each frame unread), tile headers / slots.  Multi-band: the
        // sum over the sequence's launches (multiband_traffic_parts).
        if (m->mb) {
            *bytes = multiband_traffic(*m->mb);
            return;
        }
        const TiledLut& t = m->tiles.view;
        *bytes = (t.e24 ? 3.0 : 4.0) * t.n_items * kTilePx * t.qpl + 8.0 * t.n_wide * kTilePx + 1.5 * m->W * m->H +
                 (double)t.n_items * (sizeof(TileHdr) + kTileSlots * sizeof(TileSlot)) + 4.0 * t.n_wide +
                 m->tiles.source_bytes;
    });
}

int octvr_mapper_traffic_parts(const octvr_mapper* m, double* lut_bytes, double* frame_bytes) {
    return guarded([&] {
        REQUIRE(m && lut_bytes && frame_bytes, "NULL argument");
        double total = 0;
        REQUIRE(octvr_mapper_traffic(m, &total) == OCTVR_OK, "traffic");
        if (m->mb) {  // no batched kernels: everything is per frame
            *lut_bytes = 0;
            *frame_bytes = total;
            return;
        }
        const TiledLut& t = m->tiles.view;
        *lut_bytes = (t.e24 ? 3.0 : 4.0) * t.n_items * kTilePx * t.qpl + 8.0 * t.n_wide * kTilePx +
                     (double)t.n_items * (sizeof(TileHdr) + kTileSlots * sizeof(TileSlot)) + 4.0 * t.n_wide;
        *frame_bytes = total - *lut_bytes;
    });
}

int octvr_mapper_set_timing(octvr_mapper* m, int enable) {
    return guarded([&] {
        REQUIRE(m && enable >= 0, "bad arguments");
        m->timing = enable;
        m->timed_calls = 0;
        if (enable) {
            // the event pairs of the next timed stitches created now, not inside the caller's timed region
            // (hipEventCreate there cost the 20-step bench region ~20 us of host time per step)
            DeviceGuard dg(m->device);
            constexpr size_t kEventReserve = 1024;
            while (m->free_events.size() + m->events.size() < kEventReserve) {
                hipEvent_t e0 = nullptr, e1 = nullptr;
                HIP_CHECK(hipEventCreate(&e0));
                const hipError_t e = hipEventCreate(&e1);
                if (e != hipSuccess) (void)hipEventDestroy(e0);
                HIP_CHECK(e);
                m->free_events.emplace_back(e0, e1);
            }
        }
    });
}

int octvr_interval_union(const double* start, const double* end, int n, double* span, double* busy) {
    return guarded([&] {
        REQUIRE(n >= 0 && span && busy && (n == 0 || (start && end)), "bad arguments");
        std::vector<std::pair<double, double>> iv;
        double sp = 0;
        for (int k = 0; k < n; k++) {
            REQUIRE(end[k] >= start[k], "interval ends before it starts");
            iv.emplace_back(start[k], end[k]);
            sp += end[k] - start[k];
        }
        // sweep in start order: an interval that starts inside the current run extends it, one that
        // starts after it closes the run
        std::sort(iv.begin(), iv.end());
        double bz = 0;
        bool open = false;
        double ra = 0, rb = 0;
        for (const auto& x : iv) {
            if (open && x.first <= rb) {
                rb = std::max(rb, x.second);
            } else {
                if (open) bz += rb - ra;
                ra = x.first;
                rb = x.second;
                open = true;
            }
        }
        if (open) bz += rb - ra;
        *span = sp;
        *busy = bz;
    });
}

int octvr_mapper_kernel_time(octvr_mapper* m, double* total_ms, int* launches) {
    return guarded([&] {
        REQUIRE(m && total_ms && launches, "NULL argument");
        DeviceGuard dg(m->device);
        double t = 0;
        for (auto& e : m->events) {
            HIP_CHECK(hipEventSynchronize(e.second));
            float ms = 0;
            HIP_CHECK(hipEventElapsedTime(&ms, e.first, e.second));
            t += ms;
            m->free_events.push_back(e);
        }
        *launches = (int)m->events.size();
        *total_ms = t;
        m->events.clear();
    });
}

int octvr_mapper_kernel_busy(octvr_mapper* m, double* span_ms, double* busy_ms, int* launches) {
    return guarded([&] {
        REQUIRE(m && span_ms && busy_ms && launches, "NULL argument");
        DeviceGuard dg(m->device);
        // [start, end] of every recorded launch relative to the first one's start (launches on several
        // streams may overlap): summed spans and the length of their union
        std::vector<double> st, en;
        for (auto& e : m->events) {
            HIP_CHECK(hipEventSynchronize(e.second));
            float a = 0, b = 0;
            HIP_CHECK(hipEventElapsedTime(&a, m->events[0].first, e.first));
            HIP_CHECK(hipEventElapsedTime(&b, m->events[0].first, e.second));
            st.push_back((double)a);
            en.push_back((double)b);
        }
        double busy = 0, span = 0;
        if (octvr_interval_union(st.data(), en.data(), (int)st.size(), &span, &busy) != OCTVR_OK)
            throw OctvrError(OCTVR_E_HIP, "kernel_busy: inconsistent event timestamps");
        for (auto& e : m->events) m->free_events.push_back(e);
        *launches = (int)m->events.size();
        *span_ms = span;
        *busy_ms = busy;
        m->events.clear();
    });
}

int octvr_mapper_kernel_intervals(octvr_mapper* m, double* start_ms, double* end_ms, int cap, int* n) {
    return guarded([&] {
        REQUIRE(m && n && cap >= 0 && (cap == 0 || (start_ms && end_ms)), "bad arguments");
        DeviceGuard dg(m->device);
        int k = 0;
        for (auto& e : m->events) {
            HIP_CHECK(hipEventSynchronize(e.second));
            if (k < cap) {
                float a = 0, b = 0;
                HIP_CHECK(hipEventElapsedTime(&a, m->events[0].first, e.first));
                HIP_CHECK(hipEventElapsedTime(&b, m->events[0].first, e.second));
                start_ms[k] = a;
                end_ms[k] = b;
            }
            k++;
        }
        for (auto& e : m->events) m->free_events.push_back(e);
        *n = k;
        m->events.clear();
    });
}

int octvr_mapper_info(const octvr_mapper* m, char* buf, size_t len) {
    return guarded([&] {
        REQUIRE(m && buf && len > 0, "bad arguments");
        char tmp[512];
        snprintf(tmp, sizeof tmp,
                 "{\"inputs\": %d, \"out\": [%d, %d], \"blend\": %d, \"tiles\": %d, \"wide_tiles\": %d, "
                 "\"staged_bytes\": %.0f, \"source_bytes\": %.0f, \"gain\": %d, \"gain_samples\": %d, \"gain_pairs_px\": %zu, "
                 "\"gain_chunks\": %d, \"scaled_out\": [%d, %d], \"footprint_bytes\": %.0f",
                 m->n, m->W, m->H, m->blend, m->n_tiles, m->tiles.view.n_wide,
                 m->mb ? 0.0 : m->tiles.staged_bytes, m->mb ? 0.0 : m->tiles.source_bytes, m->use_gain, m->n_samples, m->n_entries, m->n_chunks, m->SW, m->SH,
                 m->foot.bytes());
        std::string js = tmp;
        if (m->mb) js += ", " + multiband_info(*m->mb);
        else if (!m->tiles.stats.empty()) js += ", " + m->tiles.stats;
        js += "}";
        REQUIRE(js.size() < len, "buffer too small");
        memcpy(buf, js.c_str(), js.size() + 1);
    });
}

void octvr_mapper_destroy(octvr_mapper* m) {
    if (!m) return;
    int prev = -1;
    if (hipGetDevice(&prev) == hipSuccess && prev != m->device) (void)hipSetDevice(m->device);
    delete m;
    if (prev >= 0) (void)hipSetDevice(prev);
}

int octvr_remap_u8(const uint8_t* src, int sw, int sh, size_t spitch, int cn, const float* map1, const float* map2,
                   int mw, int mh, size_t mpitch, float scale_x, float scale_y, uint8_t* dst, size_t dpitch,
                   void* stream) {
    return guarded([&] {
        REQUIRE(src && map1 && map2 && dst && sw > 0 && sh > 0 && mw >= 0 && mh >= 0, "bad arguments");
        REQUIRE(cn == 1 || cn == 3 || cn == 4, "cn must be 1, 3 or 4");
        if (mw == 0 || mh == 0) return;
        HIP_CHECK(launch_remap_u8(src, sw, sh, (int64_t)spitch, cn, map1, map2, mw, mh, (int64_t)mpitch, scale_x,
                                  scale_y, dst, (int64_t)dpitch, (hipStream_t)stream));
    });
}

int octvr_debug_gain_plan(const octvr_rig* rig, int n_inputs, const int* in_w, const int* in_h, int flags,
                          uint32_t* samples, uint16_t* partners, size_t cap, size_t* count) {
    return guarded([&] {
        REQUIRE(rig && in_w && in_h && count, "bad arguments");
        REQUIRE((flags & ~OCTVR_REMAP_TEXTURE) == 0, "unknown mapper flags");
        const int n = (int)rig->inputs.size();
        REQUIRE(n_inputs == n && n > 0 && n <= kGainMaxCams, "in_sizes must cover the inputs");
        const GainPlan g = plan_gain(*rig, n, std::vector<int>(in_w, in_w + n), std::vector<int>(in_h, in_h + n),
                                     (flags & OCTVR_REMAP_TEXTURE) ? 1 : 0);
        *count = g.samples.size();
        if (!samples || !partners) return;
        REQUIRE(cap >= g.samples.size(), "buffer too small");
        for (size_t k = 0; k < g.samples.size(); k++) {
            samples[2 * k] = g.samples[k].xy;
            samples[2 * k + 1] = g.samples[k].code;
            partners[k] = g.partners[k];
        }
    });
}

int octvr_debug_tiled_lut_info(const octvr_rig* rig, int n_inputs, const int* in_w, const int* in_h, int flags,
                               char* json, size_t len) {
    return guarded([&] {
        REQUIRE(rig && in_w && in_h && json && len > 0, "bad arguments");
        REQUIRE((flags & ~OCTVR_REMAP_TEXTURE) == 0, "unknown mapper flags");
        const bool tex = (flags & OCTVR_REMAP_TEXTURE) != 0;
        const int n = (int)rig->inputs.size();
        REQUIRE(n_inputs == n && n > 0 && n <= kMaxCams, "in_sizes must cover the inputs");
        const int W = rig->out_w, H = rig->out_h;
        // the copy chain's winner per pixel (composite_lut_kernel on the host): the last camera whose ROI
        // holds the pixel and whose LUT mask is set
        std::vector<CompositeEntry> lut((size_t)W * H, CompositeEntry{0u, 0u});
        parallel_for((size_t)H, [&](size_t y) {
            for (int i = 0; i < n; i++) {
                const RigInput& in = rig->inputs[i];
                const int ry = (int)y - in.roi[1];
                if (ry < 0 || ry >= in.roi[3]) continue;
                for (int rx = 0; rx < in.roi[2]; rx++) {
                    const size_t k = (size_t)ry * in.roi[2] + rx;
                    if (!in.mask[k]) continue;
                    lut[y * W + (size_t)(rx + in.roi[0])] =
                        tex ? make_entry_tex(in.map1[k], in.map2[k], (float)in_w[i], (float)in_h[i], i)
                            : make_entry(in.map1[k], in.map2[k], (float)in_w[i], (float)in_h[i], i);
                }
            }
        });
        const int qpl = composite_qpl();
        const int tx_n = (W + kTileW - 1) / kTileW, ty_n = (H + kTileH * qpl - 1) / (kTileH * qpl);
        std::vector<TileJob> jobs;
        for (int ty = 0; ty < ty_n; ty++)
            for (int tx = 0; tx < tx_n; tx++) jobs.push_back(TileJob{tx, ty, 0});
        // build_tiled_lut checks that every tap of every pixel lies in a staged group of its slot
        const TiledLutBuild b = build_tiled_lut(jobs, [&](int, int x, int y) {
            return (x < W && y < H) ? lut[(size_t)y * W + x] : CompositeEntry{0u, 0u};
        }, std::vector<int>(in_w, in_w + n), std::vector<int>(in_h, in_h + n), qpl);
        double box_px = 0;
        for (int t = 0; t < b.n_items; t++)
            for (int j = 0; j < (int)(b.hdr[t].nslots & 0xFFu); j++)
                box_px += (double)b.slots[(size_t)t * kTileSlots + j].bw * b.slots[(size_t)t * kTileSlots + j].bh;
        // LDS bank model of the composite's reads and staging stores (MI355X_MICROARCH.md §LDS): per
        // wave-instruction and lane group, the busiest bank's distinct dword addresses; "extra" = the cycles
        // above one per group, as SQ_LDS_BANK_CONFLICT counts them.  Taps: two ds_read2_b32 per pixel (each
        // dword as a ds_read_b32: 2 x 32 lanes, bank (a/4) mod 32); weights: ds_read_b64 (2 x 32, mod 64);
        // staging: two ds_write_b128 per group (8 x 8 lanes, mod 32).
        double tap_cyc = 0, tap_extra = 0, wt_cyc = 0, wt_extra = 0, st_cyc = 0, st_extra = 0;
        {
            const int item_px = kTilePx * qpl;
            auto group_cost = [](const uint32_t* a, int n, int lanes, int banks, double& cyc, double& extra) {
                // a: n dword addresses per lane, lanes lanes in the group
                uint32_t seen[64][16];
                int cnt[64] = {};
                int mx = 0;
                for (int l = 0; l < lanes; l++)
                    for (int i = 0; i < n; i++) {
                        const uint32_t d = a[l * n + i], bk = d % (uint32_t)banks;
                        bool dup = false;
                        for (int k = 0; k < cnt[bk]; k++) dup |= seen[bk][k] == d;
                        if (!dup && cnt[bk] < 16) seen[bk][cnt[bk]++] = d;
                        mx = std::max(mx, cnt[bk]);
                    }
                cyc += std::max(mx, 1);
                extra += std::max(mx, 1) - 1;
            };
            uint32_t a[64 * 4];
            for (int t = 0; t < b.n_items; t++) {
                const TileHdr& hd = b.hdr[t];
                const uint32_t S = hd.stride & ((1u << kStrideBits) - 1u);
                const uint32_t* E = b.entries.data() + (size_t)t * item_px;
                for (int h = 0; h < qpl; h++)
                    for (int w = 0; w < 4; w++)
                        for (int p = 0; p < 4; p++) {
                            for (int half = 0; half < 2; half++) {
                                const uint32_t* e = E + (size_t)h * kTilePx + (size_t)(w * 64 + half * 32) * 4 + p;
                                for (int r = 0; r < 2; r++)
                                    for (int c = 0; c < 2; c++) {
                                        for (int l = 0; l < 32; l++)
                                            a[l] = (b.tex ? (e[l * 4] >> 17) & 0xFFFu : ((e[l * 4] >> 13) & 0x3FFFu) / 4u) + r * S + c;
                                        group_cost(a, 1, 32, 32, tap_cyc, tap_extra);
                                    }
                                if (b.tex) continue;  // the texture filter reads no weight table
                                for (int l = 0; l < 32; l++) {
                                    const uint32_t d = (0x4000u | (e[l * 4] & 0x1FF8u)) / 4u;
                                    a[2 * l] = d;
                                    a[2 * l + 1] = d + 1;
                                }
                                group_cost(a, 2, 32, 64, wt_cyc, wt_extra);
                            }
                        }
                const int ns = (int)(hd.nslots & 0xFFu), nch = (int)((hd.nslots >> 8) & 0xFFu);
                const TileSlot* ts = b.slots.data() + (size_t)t * kTileSlots;
                for (int c = 0; c < nch; c++) {
                    int j = 0;
                    for (int k = 1; k < ns; k++)
                        if (c >= (int)ts[k].chunk0) j = k;
                    const uint16_t* G = c < kGroupFirst ? b.grp0.data() + ((size_t)t * kGroupFirst + c) * 64
                                                        : b.grp1.data() + ((size_t)(hd.stride >> kStrideBits) + c - kGroupFirst) * 64;
                    for (int sgi = 0; sgi < 2; sgi++)  // the two 16-byte stores of a group
                        for (int grp = 0; grp < 8; grp++) {
                            int n = 0;
                            for (int l = grp * 8; l < grp * 8 + 8; l++) {
                                if (!(G[l] & kGroupValid)) continue;
                                const uint32_t d = ts[j].lds + (G[l] & 255u) * S + ((G[l] >> 8) & 31u) * 8u + 4u * sgi;
                                for (int i = 0; i < 4; i++) a[n * 4 + i] = d + i;
                                n++;
                            }
                            if (n) group_cost(a, 4, n, 32, st_cyc, st_extra);
                        }
                }
            }
        }
        // the composite's source footprint (what the AsyncMultiMapper uploads, gain samples aside)
        SourceFootprint fp;
        fp.init(std::vector<int>(in_w, in_w + n), std::vector<int>(in_h, in_h + n));
        footprint_add_tiles(fp, b);
        const double foot = fp.bytes();
        double frame_bytes = 0;
        for (int i = 0; i < n; i++) frame_bytes += 1.5 * in_w[i] * in_h[i];
        char tmp[1024];
        snprintf(tmp, sizeof tmp,
                 "{\"tex\": %d, \"footprint_bytes\": %.0f, \"frame_bytes\": %.0f, \"lds_model\": {\"tap_cycles\": %.0f, \"tap_extra\": %.0f, \"wtab_cycles\": %.0f, "
                 "\"wtab_extra\": %.0f, \"stage_cycles\": %.0f, \"stage_extra\": %.0f}, "
                 "\"items\": %d, \"wide_tiles\": %d, \"staged_px\": %.0f, \"box_px\": %.0f, \"staged_bytes\": %.0f, "
                 "\"source_bytes\": %.0f, \"grp1_entries\": %zu, ",
                 b.tex, foot, frame_bytes, tap_cyc, tap_extra, wt_cyc, wt_extra, st_cyc, st_extra, b.n_items, b.n_wide, b.staged_bytes / 2.0, box_px, b.staged_bytes, b.source_bytes,
                 b.grp1.size());
        std::string js = std::string(tmp) + b.stats + "}";
        REQUIRE(js.size() < len, "buffer too small");
        memcpy(json, js.c_str(), js.size() + 1);
    });
}

int octvr_debug_json_number(const char* json, int flags, double* value) {
    return guarded([&] {
        REQUIRE(json && value, "NULL argument");
        const JsonValue v = json_parse(json, (flags & OCTVR_JSON_EXACT) != 0);
        const JsonValue& n = v.kind == JsonValue::Array ? v[0] : v;
        *value = n.as_double();
    });
}

int octvr_debug_worker_failure(int n_threads, int failing) {
    return guarded([&] {
        REQUIRE(n_threads > 0 && n_threads <= 64, "bad arguments");
        run_threads((size_t)n_threads, [&](size_t t) {
            REQUIRE((int)t != failing, "worker " + std::to_string(t) + " failed (test hook)");
        });
    });
}

int octvr_rig_lut_recomputed(const octvr_rig* rig, int i, uint64_t* n) {
    return guarded([&] {
        REQUIRE(rig && n && i >= 0 && i < (int)rig->inputs.size(), "bad arguments");
        *n = rig->inputs[i].n_fragile;
    });
}

int octvr_debug_project_f64(const char* json, int out_w, int out_h, int input, int device, int where, double* x,
                            double* y, uint8_t* fragile) {
    return guarded([&] {
        REQUIRE(json && x && y && out_w > 0 && out_h > 0 && (where == 0 || where == 1), "bad arguments");
        JsonValue doc = json_parse(json);
        const CameraParams out_cam = camera_from_json(doc["output"]);
        const JsonValue& ins = doc["inputs"];
        REQUIRE(input >= 0 && input < (int)ins.size(), "bad input index");
        const JsonValue& cam = ins[(size_t)input];
        CameraParams c = camera_from_json(cam);
        std::vector<uint8_t> excl, incl;
        if (cam.has("options")) build_camera_masks(cam["options"], excl, incl);
        if (!excl.empty() || !incl.empty()) {
            c.sel = 0;
            c.width = cam["options"]["width"].as_int();
            c.height = cam["options"]["height"].as_int();
        }
        const size_t total = (size_t)out_w * out_h;
        if (where == 1) {  // host, glibc: the evaluation build_input uses for the fragile pixels
            c.excl = excl.empty() ? nullptr : excl.data();
            c.incl = nullptr;
            parallel_for((size_t)out_h, [&](size_t h) {
                for (int w = 0; w < out_w; w++)
                    project_output_to_input(out_cam, c, (double)w / out_w, (double)h / out_h, &x[h * out_w + w],
                                            &y[h * out_w + w]);
            });
            return;
        }
        REQUIRE(fragile, "fragile is NULL");
        DeviceGuard dg(device);
        DevBuf<uint8_t> excl_d;
        if (!excl.empty()) {
            excl_d.upload(excl.data(), excl.size());
            c.excl = excl_d.p;
        }
        c.incl = nullptr;
        const CameraParams both[2] = {out_cam, c};
        DevBuf<CameraParams> cams;
        cams.upload(both, 2);
        DevBuf<double> xd, yd;
        DevBuf<uint8_t> fd;
        xd.alloc(total);
        yd.alloc(total);
        fd.alloc(total);
        HIP_CHECK(launch_project_f64(cams.p, out_w, out_h, xd.p, yd.p, fd.p, nullptr));
        HIP_CHECK(hipDeviceSynchronize());
        HIP_CHECK(hipMemcpy(x, xd.p, total * sizeof(double), hipMemcpyDeviceToHost));
        HIP_CHECK(hipMemcpy(y, yd.p, total * sizeof(double), hipMemcpyDeviceToHost));
        HIP_CHECK(hipMemcpy(fragile, fd.p, total, hipMemcpyDeviceToHost));
    });
}

int octvr_selftest_sat_u8(const float* in, uint8_t* out, int n, int method, void* stream) {
    return guarded([&] {
        REQUIRE(in && out && n >= 0 && (method == 0 || method == 1), "bad arguments");
        HIP_CHECK(launch_selftest_sat(in, out, n, method, (hipStream_t)stream));
    });
}

}  // extern "C"
