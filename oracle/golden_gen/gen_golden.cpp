// Golden-fixture generator: TEST INFRASTRUCTURE ONLY.
//
// Calls the REFERENCE implementation (blahgeek/OpenCV-octVR, CPU build made during the survey,
// SURVEY.md §8c) on small synthetic rigs and writes raw little-endian outputs that
// pack_golden.py turns into tests/golden/*.npz.  Nothing here ships; the GPU box never runs it.
//
// Reference entry points exercised (file:line in /root/reference):
//   vr::MapperTemplate(type, opts, W, H)       modules/octvr/src/template.cpp:23-44
//   MapperTemplate::add_input                   modules/octvr/src/template.cpp:46-153
//   MapperTemplate::create_masks                modules/octvr/src/template.cpp:155-204
//   MapperTemplate::dump                        modules/octvr/src/template.cpp:208-256
//   cv::remap INTER_LINEAR (fixed point)        modules/imgproc/src/imgwarp.cpp:4689-4828
//   cv::detail::GainCompensator::feed           modules/stitching/src/exposure_compensate.cpp:82-156
//   cv::solve (DECOMP_LU, 2x2/3x3 closed form)  modules/core/src/lapack.cpp:1050-1275
//   cv::Rodrigues                               modules/calib3d/src/calibration.cpp:252-345
//   cv::distanceTransform (DIST_L2, 3)          modules/imgproc/src/distransform.cpp:402-420
//   cv::resize INTER_LINEAR u8                  modules/imgproc/src/imgwarp.cpp (resize)
#include "octvr.hpp"
#include "rapidjson/document.h"
#include "opencv2/core.hpp"
#include "opencv2/imgproc.hpp"
#include "opencv2/calib3d.hpp"
#include "opencv2/stitching/detail/exposure_compensate.hpp"
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <fstream>
#include <string>
#include <vector>

static std::string g_out;

static void write_raw(const std::string& name, const void* p, size_t n) {
    std::string path = g_out + "/" + name;
    FILE* f = fopen(path.c_str(), "wb");
    if (!f) { perror(path.c_str()); exit(1); }
    fwrite(p, 1, n, f);
    fclose(f);
}

static void write_mat(const std::string& name, const cv::Mat& m) {
    cv::Mat c = m.isContinuous() ? m : m.clone();
    write_raw(name, c.data, c.total() * c.elemSize());
    std::string path = g_out + "/" + name + ".meta";
    FILE* f = fopen(path.c_str(), "w");
    fprintf(f, "%d %d %d\n", c.type(), c.rows, c.cols);
    fclose(f);
}

// splitmix64: byte k of an image seeded with `seed` is the low 8 bits of the k-th output.
static uint64_t splitmix64_at(uint64_t seed, uint64_t k) {
    uint64_t z = seed + (k + 1) * 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

static cv::Mat rand_img(int w, int h, int cn, uint64_t seed) {
    cv::Mat m(h, w, CV_8UC(cn));
    size_t n = (size_t)w * h * cn;
    for (size_t k = 0; k < n; k++) m.data[k] = (uint8_t)(splitmix64_at(seed, k) & 0xFF);
    return m;
}

struct Rig {
    const char* name;
    const char* json;
    int out_w, out_h;
    bool use_roi;
};

static void run_rig(const Rig& rig) {
    rapidjson::Document doc;
    doc.Parse(rig.json);
    if (doc.HasParseError()) { fprintf(stderr, "bad json for %s\n", rig.name); exit(1); }
    {
        std::string path = g_out + "/" + rig.name + ".json";
        FILE* f = fopen(path.c_str(), "w");
        fputs(rig.json, f);
        fclose(f);
    }
    vr::MapperTemplate mt(doc["output"]["type"].GetString(), doc["output"]["options"], rig.out_w, rig.out_h);
    std::vector<cv::Size> in_sizes;
    for (auto it = doc["inputs"].Begin(); it != doc["inputs"].End(); ++it) {
        mt.add_input((*it)["type"].GetString(), (*it)["options"], false, rig.use_roi);
        in_sizes.emplace_back((*it)["options"]["width"].GetInt(), (*it)["options"]["height"].GetInt());
    }
    mt.create_masks();
    int n = (int)mt.inputs.size();
    std::string p = std::string(rig.name) + "_";
    {
        std::vector<int64_t> hdr = {mt.out_size.width, mt.out_size.height, n};
        for (auto& in : mt.inputs) { hdr.push_back(in.roi.x); hdr.push_back(in.roi.y); hdr.push_back(in.roi.width); hdr.push_back(in.roi.height); }
        write_raw(p + "rois.i64", hdr.data(), hdr.size() * 8);
    }
    std::vector<cv::Mat> warped3, masks;
    std::vector<cv::Point> corners;
    for (int i = 0; i < n; i++) {
        auto& in = mt.inputs[i];
        std::string q = p + std::to_string(i) + "_";
        write_mat(q + "map1", in.map1);
        write_mat(q + "map2", in.map2);
        write_mat(q + "mask", in.mask);
        write_mat(q + "seam", mt.seam_masks[i]);
        int W = in_sizes[i].width, H = in_sizes[i].height;
        // cv::remap exactly as the reference tooling calls it (template.cpp:174-176, dump.cpp:138-141)
        cv::Mat img1 = rand_img(W, H, 1, 1000ULL * (uint64_t)rig.name[3] + i);
        cv::Mat out1;
        cv::remap(img1, out1, in.map1 * W, in.map2 * H, cv::INTER_LINEAR);
        write_mat(q + "remap_c1", out1);
        cv::Mat img3 = rand_img(W, H, 3, 5000ULL + 31ULL * (uint64_t)rig.name[3] + i);
        cv::Mat out3;
        cv::remap(img3, out3, in.map1 * W, in.map2 * H, cv::INTER_LINEAR);
        write_mat(q + "remap_c3", out3);
        if (i == 0) {
            cv::Mat img4 = rand_img(W, H, 4, 9000ULL + 17ULL * (uint64_t)rig.name[3]);
            cv::Mat out4;
            cv::remap(img4, out4, in.map1 * W, in.map2 * H, cv::INTER_LINEAR);
            write_mat(q + "remap_c4", out4);
        }
        warped3.push_back(out3);
        masks.push_back(in.mask.clone());
        corners.push_back(in.roi.tl());
    }
    // CPU GainCompensator on (warped u8x3, binary LUT mask) — pins the A/b assembly + LU solve.
    {
        std::vector<cv::UMat> uimgs(n), umasks(n);
        for (int i = 0; i < n; i++) { warped3[i].copyTo(uimgs[i]); masks[i].copyTo(umasks[i]); }
        cv::detail::GainCompensator gc;
        std::vector<std::pair<cv::UMat, uchar> > lm;
        for (int i = 0; i < n; i++) lm.push_back(std::make_pair(umasks[i], (uchar)255));
        gc.feed(corners, uimgs, lm);
        std::vector<double> g = gc.gains();
        write_raw(p + "gains.f64", g.data(), g.size() * 8);
    }
    // Byte-exact VRv11 dump of this template (reader/writer parity is checked by hash).
    {
        std::ofstream of(g_out + "/" + rig.name + ".dat", std::ios::binary);
        mt.dump(of);
    }
}

// All 32x32 fractional codes of the 15-bit bilinear table (initInterTab2D, imgwarp.cpp:211-280,
// including its sum-fixup) exercised through cv::remap on 8U data: 256 random integer positions per
// code on a 64x64 random image.  A wrong table entry flips some of these outputs.
static void remap_code_kat() {
    cv::Mat src = rand_img(64, 64, 1, 31337);
    const int per = 256;
    cv::Mat m1(1, 1024 * per, CV_32F), m2(1, 1024 * per, CV_32F);
    for (int code = 0; code < 1024; code++)
        for (int r = 0; r < per; r++) {
            int k = code * per + r;
            uint64_t h = splitmix64_at(2718, k);
            int sx = (int)(h % 63), sy = (int)((h >> 16) % 63);
            m1.at<float>(0, k) = (float)sx + (float)(code & 31) / 32.0f;
            m2.at<float>(0, k) = (float)sy + (float)(code >> 5) / 32.0f;
        }
    cv::Mat out;
    cv::remap(src, out, m1, m2, cv::INTER_LINEAR);
    write_mat("remap_kat_src", src);
    write_mat("remap_kat_out", out);
}

// Rotation matrices exactly as Camera::Camera builds them (camera.cpp:49-64).
static void rotation_kat() {
    const double triples[][3] = {{0, 0, 0}, {0, 1.0471975511965976, 0}, {0.1, 0.2, -0.15},
                                 {-0.3, 3.141592653589793, 0.61}, {0.05, -2.0943951023931953, -0.6108652381980153},
                                 {1e-17, 0, 0}};
    std::vector<double> out;
    for (auto& tr : triples) {
        std::vector<double> rv = {tr[0], -tr[1], -tr[2]};
        cv::Mat rx, ry, rz;
        std::vector<double> v;
        v = rv; v[1] = v[2] = 0; cv::Rodrigues(v, rx);
        v = rv; v[0] = v[2] = 0; cv::Rodrigues(v, ry);
        v = rv; v[0] = v[1] = 0; cv::Rodrigues(v, rz);
        cv::Mat R = (rx * rz) * ry;
        cv::Mat Ri = R.inv();
        for (int k = 0; k < 3; k++) out.push_back(tr[k]);
        for (int r = 0; r < 3; r++) for (int c = 0; c < 3; c++) out.push_back(R.at<double>(r, c));
        for (int r = 0; r < 3; r++) for (int c = 0; c < 3; c++) out.push_back(Ri.at<double>(r, c));
    }
    write_raw("rotation_kat.f64", out.data(), out.size() * 8);
}

// cv::solve KATs: LU path (n>=4) and the closed forms for n = 1, 2, 3 (lapack.cpp:1064-1185).
static void solve_kat() {
    std::vector<double> out;
    for (int n = 1; n <= 12; n++) {
        cv::Mat A(n, n, CV_64F), b(n, 1, CV_64F), x;
        for (int r = 0; r < n; r++) {
            double rs = 0;
            for (int c = 0; c < n; c++) {
                double v = (double)(splitmix64_at(77 + n, r * n + c) % 100000) / 997.0 - 50.0;
                A.at<double>(r, c) = v;
                rs += std::fabs(v);
            }
            if (n % 2 == 0) A.at<double>(r, r) = rs + 1.0;  // mix dominant and general matrices
            b.at<double>(r, 0) = (double)(splitmix64_at(99 + n, r) % 100000) / 331.0;
        }
        cv::solve(A, b, x, cv::DECOMP_LU);
        out.push_back(n);
        for (int k = 0; k < n * n; k++) out.push_back(((double*)A.data)[k]);
        for (int k = 0; k < n; k++) out.push_back(b.at<double>(k, 0));
        for (int k = 0; k < n; k++) out.push_back(x.at<double>(k, 0));
    }
    write_raw("solve_kat.f64", out.data(), out.size() * 8);
}

// distanceTransform(L2, 3x3) and INTER_LINEAR u8 resize KATs (seam-mask building blocks, A9).
static void seam_kats() {
    cv::Mat m(37, 53, CV_8U, cv::Scalar(0));
    cv::circle(m, cv::Point(20, 18), 14, cv::Scalar(255), -1);
    cv::rectangle(m, cv::Point(30, 3), cv::Point(50, 30), cv::Scalar(255), -1);
    m.at<uint8_t>(5, 5) = 255;
    cv::Mat d;
    cv::distanceTransform(m, d, cv::DIST_L2, 3);
    write_mat("dt_src", m);
    write_mat("dt_out", d);
    cv::Mat r = rand_img(61, 29, 1, 4242), up, down;
    cv::resize(r, up, cv::Size(150, 71));
    cv::resize(r, down, cv::Size(23, 11));
    write_mat("rs_src", r);
    write_mat("rs_up", up);
    write_mat("rs_down", down);
}

int main(int argc, char** argv) {
    if (argc < 2) { fprintf(stderr, "usage: %s OUTDIR\n", argv[0]); return 1; }
    g_out = argv[1];
    cv::setNumThreads(1);
    // rigA: config-1 geometry scaled 1/7.5 (2x fullframe_fisheye 200deg, yaw 0/pi).
    static const char* rigA =
        "{\"output\":{\"type\":\"equirectangular\",\"options\":{}},\"inputs\":["
        "{\"type\":\"fullframe_fisheye\",\"options\":{\"width\":256,\"height\":144,\"crop\":{\"rect\":[56,200,0,144],\"is_circular\":true},"
        "\"hfov\":3.490658503988659,\"center_dx\":0.0,\"center_dy\":0.0,\"radial\":[0.0,0.0,0.0],\"rotation\":{\"roll\":0.0,\"yaw\":0.0,\"pitch\":0.0}}},"
        "{\"type\":\"fullframe_fisheye\",\"options\":{\"width\":256,\"height\":144,\"crop\":{\"rect\":[56,200,0,144],\"is_circular\":true},"
        "\"hfov\":3.490658503988659,\"center_dx\":0.0,\"center_dy\":0.0,\"radial\":[0.0,0.0,0.0],\"rotation\":{\"roll\":0.0,\"yaw\":3.141592653589793,\"pitch\":0.0}}}]}";
    // rigB: config-2 geometry scaled 1/20 (6x fullframe_fisheye, yaw k*60deg).
    std::string b = "{\"output\":{\"type\":\"equirectangular\",\"options\":{}},\"inputs\":[";
    for (int k = 0; k < 6; k++) {
        char buf[512];
        snprintf(buf, sizeof buf,
                 "%s{\"type\":\"fullframe_fisheye\",\"options\":{\"width\":192,\"height\":108,\"crop\":{\"rect\":[42,150,0,108],\"is_circular\":true},"
                 "\"hfov\":3.490658503988659,\"center_dx\":0.0,\"center_dy\":0.0,\"radial\":[0.0,0.0,0.0],\"rotation\":{\"roll\":0.0,\"yaw\":%.17g,\"pitch\":0.0}}}",
                 k ? "," : "", k * 3.141592653589793 / 3.0);
        b += buf;
    }
    b += "]}";
    // rigC: distortion, centre shift, non-circular crop, output rotation, partial ROIs.
    static const char* rigC =
        "{\"output\":{\"type\":\"equirectangular\",\"options\":{\"rotation\":{\"roll\":0.1,\"yaw\":0.2,\"pitch\":-0.15}}},\"inputs\":["
        "{\"type\":\"fullframe_fisheye\",\"options\":{\"width\":200,\"height\":150,\"crop\":{\"rect\":[10,190,0,150],\"is_circular\":false},"
        "\"hfov\":3.141592653589793,\"center_dx\":3.5,\"center_dy\":-2.0,\"radial\":[0.02,-0.05,0.01],\"rotation\":{\"roll\":0.05,\"yaw\":0.0,\"pitch\":0.3}}},"
        "{\"type\":\"fullframe_fisheye\",\"options\":{\"width\":200,\"height\":150,\"crop\":{\"rect\":[25,175,0,150],\"is_circular\":true},"
        "\"hfov\":3.3161255787892263,\"center_dx\":-1.25,\"center_dy\":0.75,\"radial\":[-0.01,0.03,-0.02],\"rotation\":{\"roll\":-0.3,\"yaw\":2.0943951023931953,\"pitch\":-0.2}}},"
        "{\"type\":\"fullframe_fisheye\",\"options\":{\"width\":200,\"height\":150,"
        "\"hfov\":2.6179938779914944,\"center_dx\":0.0,\"center_dy\":0.0,\"radial\":[0.0,0.0,0.0],\"rotation\":{\"roll\":0.0,\"yaw\":-2.0943951023931953,\"pitch\":0.1}}}]}";
    // rigD: OpenCV fisheye (Kannala-Brandt) model, front/back.
    static const char* rigD =
        "{\"output\":{\"type\":\"equirectangular\",\"options\":{}},\"inputs\":["
        "{\"type\":\"fisheye\",\"options\":{\"fx\":90.0,\"fy\":91.5,\"cx\":160.0,\"cy\":121.0,\"dist_coeffs\":[0.01,-0.002,0.0005,0.0],\"width\":320,\"height\":240,"
        "\"rotation\":{\"roll\":0.0,\"yaw\":0.0,\"pitch\":0.0}}},"
        "{\"type\":\"fisheye\",\"options\":{\"fx\":90.0,\"fy\":91.5,\"cx\":158.5,\"cy\":119.0,\"dist_coeffs\":[0.02,0.001,0.0,-0.0003],\"width\":320,\"height\":240,"
        "\"rotation\":{\"roll\":0.0,\"yaw\":3.141592653589793,\"pitch\":0.0}}}]}";
    Rig rigs[] = {{"rigA", rigA, 512, 256, true},
                  {"rigB", b.c_str(), 384, 192, true},
                  {"rigC", rigC, 256, 128, true},
                  {"rigD", rigD, 256, 128, false}};
    for (auto& r : rigs) run_rig(r);
    remap_code_kat();
    rotation_kat();
    solve_kat();
    seam_kats();
    return 0;
}
