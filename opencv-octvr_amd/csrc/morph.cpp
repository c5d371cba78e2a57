// morph.cpp — MapperTemplate::morph_controlpoints (modules/octvr/src/template_morph.cpp:69-237).
//
// Control points pair a pixel of camera n0 with a pixel of camera n1 that should coincide in the
// output.  Both are projected to the output (input image_to_obj, output obj_to_image), pulled to a
// distance-weighted midpoint, and every camera's LUT (map1, map2, mask) is warped piecewise-affinely
// over a Delaunay triangulation of its control points plus a 40-point frame around them.
//
// Host side (this file): control-point projection, chamfer distances, the Delaunay triangulation
// (cv::Subdiv2D restated), per-triangle affine matrices (cv::getAffineTransform + cv::solve LU) and
// the fillPoly'd triangle ownership of every ROI pixel.  Device side (kernels.hip,
// morph_warp_kernel): the cv::warpAffine bilinear resampling of the three LUT planes, one pass over
// the ROI instead of the reference's three full-ROI warps per triangle.
#include <algorithm>
#include <array>
#include <cfloat>
#include <cmath>
#include <cstring>
#include <thread>

#include "host_common.hpp"
#include "json_lite.hpp"
#include "masks.hpp"

namespace octvr {
namespace {

// ---- cv::Subdiv2D (imgproc/src/subdivision2d.cpp), Delaunay by incremental insertion on a
// quad-edge structure.  Restated with the same edge / vertex numbering, free lists and walk order,
// because getTriangleList enumerates edges by index (including freed ones, whose stale links it
// follows) — the triangle list, its order and its corner order all depend on them.
class Subdivision {
public:
    // Subdiv2D(Rect(0, 0, 1, 1)) -> initDelaunay (:560-600)
    Subdivision() {
        const float big = 3.f;  // 3 * max(width, height)
        tl_x_ = tl_y_ = 0.f;
        br_x_ = br_y_ = 1.f;
        vtx_.push_back(Vertex());
        qe_.push_back(QuadEdge());
        free_qe_ = free_pt_ = 0;
        const int a = new_point(big, 0.f, false), b = new_point(0.f, big, false), c = new_point(-big, -big, false);
        const int ab = new_edge(), bc = new_edge(), ca = new_edge();
        set_points(ab, a, b);
        set_points(bc, b, c);
        set_points(ca, c, a);
        splice(ab, sym(ca));
        splice(bc, sym(ab));
        splice(ca, sym(bc));
        recent_ = ab;
    }

    // Subdiv2D::insert (:405-480)
    void insert(float x, float y) {
        int edge = 0, vertex = 0;
        const int loc = locate(x, y, edge, vertex);
        if (loc == kLocError) throw OctvrError(OCTVR_E_INVALID, "Subdiv2D: point location failed");
        if (loc == kLocVertex) return;
        if (loc == kLocOnEdge) {
            const int deleted = edge;
            recent_ = edge = get_edge(edge, kPrevAroundOrg);
            delete_edge(deleted);
        }
        const int pt = new_point(x, y, false);
        int base = new_edge();
        const int first = org(edge);
        set_points(base, first, pt);
        splice(base, edge);
        do {
            base = connect(edge, sym(base));
            edge = get_edge(base, kPrevAroundOrg);
        } while (dst(edge) != first);
        edge = get_edge(base, kPrevAroundOrg);
        const int max_edges = (int)qe_.size() * 4;
        for (int i = 0; i < max_edges; i++) {
            const int t = get_edge(edge, kPrevAroundOrg);
            const int t_dst = dst(t), e_org = org(edge), e_dst = dst(edge);
            if (right_of(vtx_[t_dst].x, vtx_[t_dst].y, edge) > 0 &&
                in_circle(vtx_[e_org], vtx_[t_dst], vtx_[e_dst], vtx_[pt]) < 0) {
                swap_edge(edge);
                edge = get_edge(edge, kPrevAroundOrg);
            } else if (e_org == first) {
                break;
            } else {
                edge = get_edge(next(edge), kPrevAroundLeft);
            }
        }
    }

    // Subdiv2D::getTriangleList (:735-760): every even edge not yet visited starts a left-face walk
    std::vector<std::array<float, 6>> triangles() const {
        std::vector<std::array<float, 6>> out;
        const int total = (int)qe_.size() * 4;
        std::vector<char> seen(total, 0);
        auto mark = [&](int e) {
            if (e < 0 || e >= total) throw OctvrError(OCTVR_E_INVALID, "Subdiv2D: corrupt edge list");
            seen[e] = 1;
        };
        for (int i = 4; i < total; i += 2) {
            if (seen[i]) continue;
            std::array<float, 6> t;
            int e = i;
            const Vertex& a = vtx_.at(org(e));
            mark(e);
            e = get_edge(e, kNextAroundLeft);
            const Vertex& b = vtx_.at(org(e));
            mark(e);
            e = get_edge(e, kNextAroundLeft);
            const Vertex& c = vtx_.at(org(e));
            mark(e);
            t = {a.x, a.y, b.x, b.y, c.x, c.y};
            out.push_back(t);
        }
        return out;
    }

private:
    enum { kLocError = -2, kLocInside = 0, kLocVertex = 1, kLocOnEdge = 2 };
    enum { kNextAroundLeft = 0x13, kPrevAroundOrg = 0x11, kPrevAroundDst = 0x33, kPrevAroundLeft = 0x20 };
    struct QuadEdge {
        int next[4] = {0, 0, 0, 0};
        int pt[4] = {0, 0, 0, 0};
    };
    struct Vertex {
        float x = 0.f, y = 0.f;
        int first = 0;
        int type = -1;
    };
    std::vector<QuadEdge> qe_;
    std::vector<Vertex> vtx_;
    int free_qe_ = 0, free_pt_ = 0, recent_ = 0;
    float tl_x_, tl_y_, br_x_, br_y_;

    QuadEdge& q(int e) { return qe_.at((size_t)(e >> 2)); }
    const QuadEdge& q(int e) const { return qe_.at((size_t)(e >> 2)); }
    int next(int e) const { return q(e).next[e & 3]; }
    static int rot(int e, int r) { return (e & ~3) + ((e + r) & 3); }
    static int sym(int e) { return e ^ 2; }
    int get_edge(int e, int type) const {  // :63-68
        e = q(e).next[(e + type) & 3];
        return (e & ~3) + ((e + (type >> 4)) & 3);
    }
    int org(int e) const { return q(e).pt[e & 3]; }
    int dst(int e) const { return q(e).pt[(e + 2) & 3]; }

    void splice(int a, int b) {  // :160-170
        int& an = q(a).next[a & 3];
        int& bn = q(b).next[b & 3];
        const int ar = rot(an, 1), br = rot(bn, 1);
        int& arn = q(ar).next[ar & 3];
        int& brn = q(br).next[br & 3];
        std::swap(an, bn);
        std::swap(arn, brn);
    }
    void set_points(int e, int o, int d) {  // :172-178
        q(e).pt[e & 3] = o;
        q(e).pt[(e + 2) & 3] = d;
        vtx_.at(o).first = e;
        vtx_.at(d).first = e ^ 2;
    }
    int connect(int a, int b) {  // :180-189
        const int e = new_edge();
        splice(e, get_edge(a, kNextAroundLeft));
        splice(sym(e), b);
        set_points(e, dst(a), org(b));
        return e;
    }
    void swap_edge(int e) {  // :191-204
        const int s = sym(e);
        const int a = get_edge(e, kPrevAroundOrg), b = get_edge(s, kPrevAroundOrg);
        splice(e, a);
        splice(s, b);
        set_points(e, dst(a), dst(b));
        splice(e, get_edge(a, kNextAroundLeft));
        splice(s, get_edge(b, kNextAroundLeft));
    }
    // triangleArea (:206-209), in double from the float coordinates
    static double area(double ax, double ay, double bx, double by, double cx, double cy) {
        return (bx - ax) * (cy - ay) - (by - ay) * (cx - ax);
    }
    int right_of(float px, float py, int e) const {  // isRightOf (:211-219)
        const Vertex& o = vtx_.at(org(e));
        const Vertex& d = vtx_.at(dst(e));
        const double a = area(px, py, d.x, d.y, o.x, o.y);
        return (a > 0) - (a < 0);
    }
    int new_edge() {  // :221-233
        if (free_qe_ <= 0) {
            qe_.push_back(QuadEdge());
            free_qe_ = (int)qe_.size() - 1;
        }
        const int e = free_qe_ * 4;
        free_qe_ = q(e).next[1];
        QuadEdge& n = q(e);
        n.next[0] = e;
        n.next[1] = e + 3;
        n.next[2] = e + 2;
        n.next[3] = e + 1;
        n.pt[0] = n.pt[1] = n.pt[2] = n.pt[3] = 0;
        return e;
    }
    void delete_edge(int e) {  // :235-247
        splice(e, get_edge(e, kPrevAroundOrg));
        const int s = sym(e);
        splice(s, get_edge(s, kPrevAroundOrg));
        QuadEdge& d = q(e);
        d.next[0] = 0;
        d.next[1] = free_qe_;
        free_qe_ = e >> 2;
    }
    int new_point(float x, float y, bool is_virtual) {  // :249-262
        if (free_pt_ == 0) {
            vtx_.push_back(Vertex());
            free_pt_ = (int)vtx_.size() - 1;
        }
        const int v = free_pt_;
        free_pt_ = vtx_[v].first;
        vtx_[v] = Vertex{x, y, 0, is_virtual ? 1 : 0};
        return v;
    }

    // Subdiv2D::locate (:272-383)
    int locate(float px, float py, int& out_edge, int& out_vertex) {
        if (qe_.size() < 4) throw OctvrError(OCTVR_E_INVALID, "Subdiv2D: subdivision is empty");
        if (px < tl_x_ || py < tl_y_ || px >= br_x_ || py >= br_y_)
            throw OctvrError(OCTVR_E_INVALID, "Subdiv2D: point outside [0,1) x [0,1)");
        int e = recent_;
        if (e <= 0) throw OctvrError(OCTVR_E_INVALID, "Subdiv2D: no current edge");
        int loc = kLocError, vertex = 0;
        int r_cur = right_of(px, py, e);
        if (r_cur > 0) {
            e = sym(e);
            r_cur = -r_cur;
        }
        const int max_edges = (int)qe_.size() * 4;
        for (int i = 0; i < max_edges; i++) {
            const int onext = next(e), dprev = get_edge(e, kPrevAroundDst);
            const int r_onext = right_of(px, py, onext), r_dprev = right_of(px, py, dprev);
            if (r_dprev > 0) {
                if (r_onext > 0 || (r_onext == 0 && r_cur == 0)) {
                    loc = kLocInside;
                    break;
                }
                r_cur = r_onext;
                e = onext;
            } else if (r_onext > 0) {
                if (r_dprev == 0 && r_cur == 0) {
                    loc = kLocInside;
                    break;
                }
                r_cur = r_dprev;
                e = dprev;
            } else if (r_cur == 0 && right_of(vtx_.at(dst(onext)).x, vtx_.at(dst(onext)).y, e) >= 0) {
                e = sym(e);
            } else {
                r_cur = r_onext;
                e = onext;
            }
        }
        recent_ = e;
        if (loc == kLocInside) {
            const Vertex& o = vtx_.at(org(e));
            const Vertex& d = vtx_.at(dst(e));
            // differences in float (Point2f arithmetic), sums in double
            double t1 = std::fabs(px - o.x);
            t1 += std::fabs(py - o.y);
            double t2 = std::fabs(px - d.x);
            t2 += std::fabs(py - d.y);
            double t3 = std::fabs(o.x - d.x);
            t3 += std::fabs(o.y - d.y);
            if (t1 < FLT_EPSILON) {
                loc = kLocVertex;
                vertex = org(e);
                e = 0;
            } else if (t2 < FLT_EPSILON) {
                loc = kLocVertex;
                vertex = dst(e);
                e = 0;
            } else if ((t1 < t3 || t2 < t3) && std::fabs(area(px, py, o.x, o.y, d.x, d.y)) < FLT_EPSILON) {
                loc = kLocOnEdge;
                vertex = 0;
            }
        }
        if (loc == kLocError) e = vertex = 0;
        out_edge = e;
        out_vertex = vertex;
        return loc;
    }

    // isPtInCircle3 (:386-397)
    static int in_circle(const Vertex& pt, const Vertex& a, const Vertex& b, const Vertex& c) {
        const double eps = FLT_EPSILON * 0.125;
        double v = ((double)a.x * a.x + (double)a.y * a.y) * area(b.x, b.y, c.x, c.y, pt.x, pt.y);
        v -= ((double)b.x * b.x + (double)b.y * b.y) * area(a.x, a.y, c.x, c.y, pt.x, pt.y);
        v += ((double)c.x * c.x + (double)c.y * c.y) * area(a.x, a.y, b.x, b.y, pt.x, pt.y);
        v -= ((double)pt.x * pt.x + (double)pt.y * pt.y) * area(a.x, a.y, b.x, b.y, c.x, c.y);
        return v > eps ? 1 : v < -eps ? -1 : 0;
    }
};

// LUImpl (core/src/matrix_decomp.cpp:50-110) as cv::solve(DECOMP_LU) runs it for n > 3; a
// singular system leaves the solution zero (lapack.cpp:1317-1318).
void solve_lu(double* A, double* b, int n) {
    const double eps = DBL_EPSILON * 100;
    for (int i = 0; i < n; i++) {
        int k = i;
        for (int j = i + 1; j < n; j++)
            if (std::fabs(A[j * n + i]) > std::fabs(A[k * n + i])) k = j;
        if (std::fabs(A[k * n + i]) < eps) {
            std::fill(b, b + n, 0.0);
            return;
        }
        if (k != i) {
            for (int j = i; j < n; j++) std::swap(A[i * n + j], A[k * n + j]);
            std::swap(b[i], b[k]);
        }
        const double d = -1 / A[i * n + i];
        for (int j = i + 1; j < n; j++) {
            const double alpha = A[j * n + i] * d;
            for (int c = i + 1; c < n; c++) A[j * n + c] += alpha * A[i * n + c];
            b[j] += alpha * b[i];
        }
        A[i * n + i] = -d;
    }
    for (int i = n - 1; i >= 0; i--) {
        double s = b[i];
        for (int c = i + 1; c < n; c++) s -= A[i * n + c] * b[c];
        b[i] = s * A[i * n + i];
    }
}

// cv::getAffineTransform(src, dst) (imgproc/src/imgwarp.cpp:6340-6361), then the inversion
// warpAffine applies without WARP_INVERSE_MAP (:5655-5666): the result maps destination pixels to
// source positions.
void warp_matrix(const float* s, const float* d, double* M) {
    double a[36], b[6];
    for (int i = 0; i < 3; i++) {
        const int j = i * 12, k = i * 12 + 6;
        a[j] = a[k + 3] = s[2 * i];
        a[j + 1] = a[k + 4] = s[2 * i + 1];
        a[j + 2] = a[k + 5] = 1;
        a[j + 3] = a[j + 4] = a[j + 5] = 0;
        a[k] = a[k + 1] = a[k + 2] = 0;
        b[i * 2] = d[2 * i];
        b[i * 2 + 1] = d[2 * i + 1];
    }
    solve_lu(a, b, 6);
    for (int k = 0; k < 6; k++) M[k] = b[k];
    double D = M[0] * M[4] - M[1] * M[3];
    D = D != 0 ? 1. / D : 0;
    const double A11 = M[4] * D, A22 = M[0] * D;
    M[0] = A11;
    M[1] *= -D;
    M[3] *= -D;
    M[4] = A22;
    const double b1 = -M[0] * M[2] - M[1] * M[5];
    const double b2 = -M[3] * M[2] - M[4] * M[5];
    M[2] = b1;
    M[5] = b2;
}

struct Pt {
    float x, y;
};
struct ControlPoint {  // template_morph.cpp:15-20
    int n0, n1;
    Pt src0, src1, dst0, dst1, mid;
};

// distanceTransform(DIST_L2, 3) of one camera's ROI mask, three side-by-side copies when the camera
// starts at column 0 and spans the union ROI (DistanceSeamFinder::find, seam_finders.cpp:97-110)
std::vector<float> camera_distance(const RigInput& in, bool wrapped) {
    const int w = in.roi[2], h = in.roi[3];
    std::vector<float> d((size_t)w * h);
    if (!wrapped) {
        chamfer_l2_3x3(in.mask.data(), w, h, d.data());
        return d;
    }
    std::vector<uint8_t> tri((size_t)3 * w * h);
    for (int y = 0; y < h; y++)
        for (int c = 0; c < 3; c++) memcpy(&tri[((size_t)y * 3 + c) * w], &in.mask[(size_t)y * w], w);
    std::vector<float> d3(tri.size());
    chamfer_l2_3x3(tri.data(), 3 * w, h, d3.data());
    for (int y = 0; y < h; y++) memcpy(&d[(size_t)y * w], &d3[((size_t)y * 3 + 1) * w], sizeof(float) * w);
    return d;
}

}  // namespace

int rig_morph_controlpoints(octvr_rig& rig, const JsonValue& cps_json) {
    const int n = (int)rig.inputs.size();
    if (!rig.has_cameras)
        throw OctvrError(OCTVR_E_UNSUPPORTED, "morph_controlpoints needs the camera models (a rig built from JSON, "
                                              "not one loaded from .dat)");
    REQUIRE(cps_json.kind == JsonValue::Array, "control_points must be an array");
    const int W = rig.out_w, H = rig.out_h;

    // _translate (template_morph.cpp:86-90): input image_to_obj, then output obj_to_image
    auto translate = [&](Pt p, int cam) {
        const CameraParams& c = rig.cams[cam];
        if (c.type == CAM_FISHEYE || c.type == CAM_PINHOLE)  // camera.hpp:101-103
            throw OctvrError(OCTVR_E_UNSUPPORTED, "control point camera has no image_to_obj (fisheye / pinhole)");
        if (c.type == CAM_FULLFRAME_FISHEYE)  // fullframe_fisheye_cam.cpp:224
            REQUIRE(c.crop_x == 0 && c.crop_y == 0 && c.crop_w == c.width && c.crop_h == c.height,
                    "control point camera: fullframe_fisheye image_to_obj needs a crop covering the image");
        double x, y;
        project_output_to_input(c, rig.out_cam, p.x, p.y, &x, &y);
        return Pt{(float)x, (float)y};
    };

    // control points (:92-136); the distances are evaluated only for the points kept
    std::vector<ControlPoint> cps;
    struct Local {
        int x0, y0, x1, y1;
    };
    std::vector<Local> local;
    for (size_t k = 0; k < cps_json.size(); k++) {
        const JsonValue& a = cps_json[k];
        REQUIRE(a.kind == JsonValue::Array && a.size() >= 6, "control point must be [n0, n1, x0, y0, x1, y1]");
        ControlPoint cp;
        cp.n0 = a[0].as_int();
        cp.n1 = a[1].as_int();
        cp.src0 = Pt{(float)a[2].as_double(), (float)a[3].as_double()};
        cp.src1 = Pt{(float)a[4].as_double(), (float)a[5].as_double()};
        REQUIRE(cp.n0 < cp.n1, "control point: n0 < n1 required");  // :102
        REQUIRE(cp.n0 >= 0 && cp.n1 < n, "control point camera index out of range");
        cp.dst0 = translate(cp.src0, cp.n0);
        cp.dst1 = translate(cp.src1, cp.n1);
        // |dst0 - dst1|_1 > 0.1 in float, compared in double (:123-124); NaN passes this test in the
        // reference and then indexes the distance maps out of bounds, so it is rejected here
        const float l1 = std::fabs(cp.dst0.x - cp.dst1.x) + std::fabs(cp.dst0.y - cp.dst1.y);
        if ((double)l1 > 0.1) continue;
        REQUIRE(!std::isnan(cp.dst0.x) && !std::isnan(cp.dst0.y) && !std::isnan(cp.dst1.x) && !std::isnan(cp.dst1.y),
                "control point does not project into the output");
        const RigInput& i0 = rig.inputs[cp.n0];
        const RigInput& i1 = rig.inputs[cp.n1];
        Local l;  // :107-110, float arithmetic truncated to int
        l.x0 = (int)(cp.dst0.x * (float)W - (float)i0.roi[0]);
        l.y0 = (int)(cp.dst0.y * (float)H - (float)i0.roi[1]);
        l.x1 = (int)(cp.dst1.x * (float)W - (float)i1.roi[0]);
        l.y1 = (int)(cp.dst1.y * (float)H - (float)i1.roi[1]);
        REQUIRE(l.x0 >= 0 && l.x0 < i0.roi[2] && l.y0 >= 0 && l.y0 < i0.roi[3] && l.x1 >= 0 && l.x1 < i1.roi[2] &&
                    l.y1 >= 0 && l.y1 < i1.roi[3],
                "control point lies outside its camera's ROI");
        cps.push_back(cp);
        local.push_back(l);
    }

    // DistanceSeamFinder(2)::find's distances (:70-79; only getDistances() is used)
    int ux0 = 0, ux1 = 0;
    for (int i = 0; i < n; i++) {
        const RigInput& in = rig.inputs[i];
        ux0 = i ? std::min(ux0, in.roi[0]) : in.roi[0];
        ux1 = i ? std::max(ux1, in.roi[0] + in.roi[2]) : in.roi[0] + in.roi[2];
    }
    std::vector<char> need(n, 0);
    for (const ControlPoint& cp : cps) need[cp.n0] = need[cp.n1] = 1;
    std::vector<std::vector<float>> dist(n);
    {
        run_threads((size_t)n, [&](size_t i) {
            if (!need[i]) return;
            const RigInput& in = rig.inputs[i];
            dist[i] = camera_distance(in, in.roi[0] == 0 && in.roi[2] == ux1 - ux0);
        });
    }
    for (size_t k = 0; k < cps.size(); k++) {  // :126-133, all float
        ControlPoint& cp = cps[k];
        const Local& l = local[k];
        float w0 = dist[cp.n0][(size_t)l.y0 * rig.inputs[cp.n0].roi[2] + l.x0];
        float w1 = dist[cp.n1][(size_t)l.y1 * rig.inputs[cp.n1].roi[2] + l.x1];
        if ((double)(w0 + w1) < 1e-3) w0 = w1 = 1.0f;
        cp.mid.x = (cp.dst0.x * w0 + cp.dst1.x * w1) / (w0 + w1);
        cp.mid.y = (cp.dst0.y * w0 + cp.dst1.y * w1) / (w0 + w1);
    }

    DeviceGuard dg(rig.device);
    for (int i = 0; i < n; i++) {
        RigInput& in = rig.inputs[i];
        std::vector<Pt> sv, dv;  // :140-151
        for (const ControlPoint& cp : cps) {
            if (cp.n0 == i) {
                sv.push_back(cp.dst0);
                dv.push_back(cp.mid);
            }
            if (cp.n1 == i) {
                sv.push_back(cp.dst1);
                dv.push_back(cp.mid);
            }
        }
        // bounding box of both vertex sets, widened by 0.05 and kept inside (0, 1) (:153-169)
        float L = 1.f, R = 0.f, T = 1.f, B = 0.f;
        for (const std::vector<Pt>* vs : {&sv, &dv})
            for (const Pt& v : *vs) {
                L = std::min(L, v.x);
                R = std::max(R, v.x);
                T = std::min(T, v.y);
                B = std::max(B, v.y);
            }
        L = (float)std::max(1e-3, (double)L - 0.05);
        T = (float)std::max(1e-3, (double)T - 0.05);
        R = (float)std::min(1 - 1e-3, (double)R + 0.05);
        B = (float)std::min(1 - 1e-3, (double)B + 0.05);
        // the fixed frame: 11 columns along the top and bottom edges, 9 rows along the sides (:171-182)
        int guard = 0;
        for (float x = L; (double)x < (double)R + 1e-3; x += (R - L) / 10) {
            REQUIRE(++guard < 100000, "morph frame does not advance");
            sv.push_back(Pt{x, T});
            sv.push_back(Pt{x, B});
            dv.push_back(Pt{x, T});
            dv.push_back(Pt{x, B});
        }
        for (float y = T + (B - T) / 10; (double)(B - (B - T) / 10) + 1e-3 > (double)y; y += (B - T) / 10) {
            REQUIRE(++guard < 100000, "morph frame does not advance");
            sv.push_back(Pt{L, y});
            sv.push_back(Pt{R, y});
            dv.push_back(Pt{L, y});
            dv.push_back(Pt{R, y});
        }

        // getTriangleList (:22-41): Delaunay of the source vertices, triangles with a corner outside
        // [0, 1]^2 (those touching the three far initial vertices) dropped
        Subdivision sub;
        for (const Pt& p : sv) sub.insert(p.x, p.y);
        in.src_tris.clear();
        in.dst_tris.clear();
        for (const auto& t : sub.triangles()) {
            bool inside = true;
            for (float c : t) inside = inside && c >= 0.0 && c <= 1.0;
            if (!inside) continue;
            // getTriangleListIndexes / FromIndexes (:43-67): corners by exact equality, first match
            for (int c = 0; c < 6; c++) in.src_tris.push_back(t[c]);
            for (int c = 0; c < 3; c++) {
                size_t j = 0;
                while (j < sv.size() && !(sv[j].x == t[2 * c] && sv[j].y == t[2 * c + 1])) j++;
                REQUIRE(j < sv.size(), "triangle corner is not a morph vertex");
                in.dst_tris.push_back(dv[j].x);
                in.dst_tris.push_back(dv[j].y);
            }
        }
        const int nt = (int)in.src_tris.size() / 6;
        if (nt == 0) continue;  // nothing to warp: the LUT is copied unchanged
        REQUIRE(nt < 32767, "too many morph triangles");

        // per triangle: warp matrix and fillPoly'd ownership (:202-231): later triangles overwrite
        const int rw = in.roi[2], rh = in.roi[3];
        auto Tx = [&](float x) { return x * (float)W - (float)in.roi[0]; };
        auto Ty = [&](float y) { return y * (float)H - (float)in.roi[1]; };
        std::vector<double> M((size_t)nt * 6);
        std::vector<int16_t> owner((size_t)rw * rh, (int16_t)-1);
        std::vector<uint8_t> scratch((size_t)rw * rh, 0);
        for (int k = 0; k < nt; k++) {
            float s[6], d[6];
            for (int c = 0; c < 3; c++) {
                s[2 * c] = Tx(in.src_tris[6 * k + 2 * c]);
                s[2 * c + 1] = Ty(in.src_tris[6 * k + 2 * c + 1]);
                d[2 * c] = Tx(in.dst_tris[6 * k + 2 * c]);
                d[2 * c + 1] = Ty(in.dst_tris[6 * k + 2 * c + 1]);
            }
            warp_matrix(s, d, &M[(size_t)6 * k]);
            int pts[6];
            for (int c = 0; c < 6; c++) pts[c] = (int)std::round(d[c]);
            fill_poly_u8(scratch.data(), rw, rh, pts, 3, 255);
            const int x0 = std::max(0, std::min({pts[0], pts[2], pts[4]})), x1 = std::min(rw - 1, std::max({pts[0], pts[2], pts[4]}));
            const int y0 = std::max(0, std::min({pts[1], pts[3], pts[5]})), y1 = std::min(rh - 1, std::max({pts[1], pts[3], pts[5]}));
            for (int y = y0; y <= y1; y++)
                for (int x = x0; x <= x1; x++) {
                    uint8_t& m = scratch[(size_t)y * rw + x];
                    if (m) {
                        owner[(size_t)y * rw + x] = (int16_t)k;
                        m = 0;
                    }
                }
        }

        const size_t px = (size_t)rw * rh;
        DevBuf<float> m1, m2, o1, o2;
        DevBuf<uint8_t> mk, om;
        DevBuf<int16_t> own;
        DevBuf<double> Md;
        m1.upload(in.map1.data(), px);
        m2.upload(in.map2.data(), px);
        mk.upload(in.mask.data(), px);
        own.upload(owner.data(), px);
        Md.upload(M.data(), M.size());
        o1.alloc(px);
        o2.alloc(px);
        om.alloc(px);
        HIP_CHECK(launch_morph_warp(m1.p, m2.p, mk.p, rw, rh, own.p, Md.p, o1.p, o2.p, om.p, nullptr));
        HIP_CHECK(hipMemcpy(in.map1.data(), o1.p, px * sizeof(float), hipMemcpyDeviceToHost));
        HIP_CHECK(hipMemcpy(in.map2.data(), o2.p, px * sizeof(float), hipMemcpyDeviceToHost));
        HIP_CHECK(hipMemcpy(in.mask.data(), om.p, px, hipMemcpyDeviceToHost));
    }
    return (int)cps.size();
}

}  // namespace octvr
