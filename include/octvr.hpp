/*
 * octvr.hpp — the reference's octvr C++ API on the MI355X path: a header-only layer over the C ABI of
 * include/octvr_hip.h, so that the reference's callers (apps/octvr/dump.cpp, apps/octvr/map.cpp, the
 * AsyncMultiMapper caller) recompile against it unchanged.
 *
 *   vr::CameraInterface, vr::MapperTemplate, vr::PreviewDataHeader, vr::AsyncMultiMapper,
 *   vr::FastMapper, vr::Timer, vr::Queue<T>   <- modules/octvr/include/octvr.hpp:38-184
 *   vr::Mapper (the reference's internal per-frame class)  <- modules/octvr/src/mapper.hpp:29-95
 *
 * OpenCV types: the real ones when <opencv2/core.hpp> is available (define OCTVR_NO_OPENCV to opt
 * out), else the subset in octvr_cv_lite.hpp.  cv::cuda::GpuMat data must be HIP device memory (the
 * lite GpuMat allocates it; with real OpenCV wrap memory from octvr_dev_malloc / hipMalloc with the
 * GpuMat(rows, cols, type, data, step) constructor).  rapidjson::Value overloads exist when
 * "rapidjson/document.h" is available (the reference vendors rapidjson 1.0.2 in
 * modules/octvr/include/rapidjson); the JSON-text overloads always do.
 *
 * Errors: bad JSON / .dat throw std::string as the reference's template code does (template.cpp:30,33,
 * 53,262); everything else throws cv::Exception (the reference's CV_Assert).  Differences from the
 * reference, all deliberate:
 *   - MapperTemplate copies are independent deep copies (octvr_rig_clone; the reference double-deletes
 *     its camera pointers); output_cam / input_cams stay null (camera models live behind the C ABI).
 *   - create_masks(imgs) with images needs GraphCutSeamFinder: not on the path, throws.
 *   - AsyncMultiMapper's preview_size enables the preview in every build (the reference only under
 *     HAVE_QT5, async.cpp:218-221); with HAVE_QT5 it is written into the reference's two Qt shared-memory
 *     zones exactly as async.cpp:149-171 does, and AsyncMultiMapper::preview() reads the latest one in any
 *     build (an addition).  Its worker threads are joined on destruction instead of running forever
 *     (async.cpp:337-349).
 *   - Mapper::override_logo_option is a no-op (trial-mode logo, licensing code not reproduced).
 */
#ifndef OCTVR_HPP
#define OCTVR_HPP

// std::to_chars(double) for the rapidjson overloads where the standard library has it (C++17 and
// libstdc++ 11+ / libc++ 14+); without it write_double falls back to a locale-safe snprintf
#if defined(OCTVR_HAVE_RAPIDJSON) && defined(__has_include) && __cplusplus >= 201703L
#if __has_include(<charconv>)
#include <charconv>
#endif
#endif
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <deque>
#include <fstream>
#include <iostream>
#include <memory>
#include <mutex>
#include <queue>
#include <sstream>
#include <string>
#include <tuple>
#include <utility>
#include <vector>

#include "octvr_hip.h"

#if !defined(OCTVR_NO_OPENCV) && defined(__has_include)
#if __has_include(<opencv2/core.hpp>)
#define OCTVR_HAVE_OPENCV 1
#endif
#endif
#ifdef OCTVR_HAVE_OPENCV
#include <opencv2/core.hpp>
#include <opencv2/core/cuda.hpp>
#else
#include "octvr_cv_lite.hpp"
#endif

#if !defined(OCTVR_NO_RAPIDJSON) && defined(__has_include)
#if __has_include("rapidjson/document.h")
#define OCTVR_HAVE_RAPIDJSON 1
#include "rapidjson/document.h"
#include "rapidjson/stringbuffer.h"
#include "rapidjson/writer.h"
#endif
#endif

#ifdef HAVE_QT5
#include <QSharedMemory>
#endif

#define OCTVR_PREVIEW_DATA0_MEMORY_KEY "opencv_octvr_preview_0"
#define OCTVR_PREVIEW_DATA1_MEMORY_KEY "opencv_octvr_preview_1"
#define OCTVR_PREVIEW_DATA_META_MEMORY_KEY "opencv_octvr_preview_meta"

namespace vr {

namespace detail {

// device for template-side GPU work (LUT build, seam resizes) and mappers: the reference uses the
// current CUDA device; set it here before building templates / mappers on another one
inline int& device() {
    static int d = 0;
    return d;
}

[[noreturn]] inline void fail(int code) {
    const std::string msg = octvr_last_error();
    if (code == OCTVR_E_PARSE) throw std::string(msg);  // template.cpp:30,33,53,262
#ifdef OCTVR_HAVE_OPENCV
    throw cv::Exception(cv::Error::StsAssert, msg, "octvr", __FILE__, __LINE__);
#else
    throw cv::Exception(code, msg);
#endif
}
inline void check(int rc) {
    if (rc != OCTVR_OK) fail(rc);
}

struct RigDeleter {
    void operator()(octvr_rig* r) const { octvr_rig_destroy(r); }
};
typedef std::shared_ptr<octvr_rig> RigPtr;
inline RigPtr own(octvr_rig* r) { return RigPtr(r, RigDeleter()); }
inline RigPtr clone(const RigPtr& r) {
    if (!r) return RigPtr();
    octvr_rig* c = nullptr;
    check(octvr_rig_clone(r.get(), &c));
    return own(c);
}

// The camera-model rig behind a MapperTemplate: copying a template copies it (the reference copies its
// Input vectors by value, so add_input / morph_controlpoints on one copy never reach another).
struct OwnedRig {
    RigPtr p;
    OwnedRig() = default;
    OwnedRig(const OwnedRig& o) : p(clone(o.p)) {}
    OwnedRig& operator=(const OwnedRig& o) {
        if (this != &o) p = clone(o.p);
        return *this;
    }
    OwnedRig(OwnedRig&&) = default;
    OwnedRig& operator=(OwnedRig&&) = default;
};

// a tightly packed copy of `n` elements of T from a caller array into a new Mat
template <typename T>
inline cv::Mat mat_copy(const T* src, int rows, int cols, int type) {
    cv::Mat m(rows, cols, type);
    if (src && rows > 0 && cols > 0)
        for (int r = 0; r < rows; r++) memcpy(m.ptr(r), src + (size_t)r * cols, (size_t)cols * sizeof(T));
    return m;
}
// a Mat's pixels as a packed array (a continuous Mat is used in place)
inline cv::Mat packed(const cv::Mat& m) { return m.isContinuous() ? m : m.clone(); }

#ifdef OCTVR_HAVE_RAPIDJSON
// one double as JSON text that reads back as the same double, whatever the C library's LC_NUMERIC: the
// shortest round-trip form with std::to_chars where the standard library has the floating-point overload
// (C++17, libstdc++ 11+), else 17 significant digits with the locale's radix character put back to '.'
inline void write_double(double d, std::string& out) {
    char buf[64];
#if defined(__cpp_lib_to_chars) && __cpp_lib_to_chars >= 201611L
    const std::to_chars_result r = std::to_chars(buf, buf + sizeof buf, d);
    out.append(buf, r.ptr);
#else
    const int k = snprintf(buf, sizeof buf, "%.17g", d);
    for (int i = 0; i < k; i++)
        if (!((buf[i] >= '0' && buf[i] <= '9') || buf[i] == '-' || buf[i] == '+' || buf[i] == 'e' || buf[i] == 'E' ||
              buf[i] == 'i' || buf[i] == 'n' || buf[i] == 'f' || buf[i] == 'a'))
            buf[i] = '.';
    out.append(buf, buf + k);
#endif
}
// a rapidjson value as JSON text with every number in a round-trip form (write_double), parsed back with
// correct rounding (OCTVR_JSON_EXACT, std::from_chars): the doubles the caller's rapidjson holds,
// unchanged.  Both conversions are locale-independent (a Qt caller has called setlocale(LC_ALL, "");
// printf / strtod would write and read "1,5" under a comma locale).
inline void write_exact(const rapidjson::Value& v, std::string& out) {
    char buf[64];
    if (v.IsObject()) {
        out += '{';
        bool first = true;
        for (auto it = v.MemberBegin(); it != v.MemberEnd(); ++it) {
            if (!first) out += ',';
            first = false;
            write_exact(it->name, out);
            out += ':';
            write_exact(it->value, out);
        }
        out += '}';
    } else if (v.IsArray()) {
        out += '[';
        for (rapidjson::SizeType i = 0; i < v.Size(); i++) {
            if (i) out += ',';
            write_exact(v[i], out);
        }
        out += ']';
    } else if (v.IsString()) {
        rapidjson::StringBuffer sb;
        rapidjson::Writer<rapidjson::StringBuffer> w(sb);
        v.Accept(w);
        out += sb.GetString();
    } else if (v.IsBool()) {
        out += v.GetBool() ? "true" : "false";
    } else if (v.IsNull()) {
        out += "null";
    } else if (v.IsInt64()) {
        snprintf(buf, sizeof buf, "%lld", (long long)v.GetInt64());
        out += buf;
    } else if (v.IsUint64()) {
        snprintf(buf, sizeof buf, "%llu", (unsigned long long)v.GetUint64());
        out += buf;
    } else {
        write_double(v.GetDouble(), out);
    }
}
inline std::string json_exact(const rapidjson::Value& v) {
    std::string s;
    write_exact(v, s);
    return s;
}
#endif

}  // namespace detail

class CameraInterface {
public:
    virtual std::vector<cv::Point2d> obj_to_image(const std::vector<cv::Point2d>& lonlats) = 0;
    virtual std::vector<cv::Point2d> image_to_obj(const std::vector<cv::Point2d>& xys) = 0;
    virtual ~CameraInterface() {}
};

// Multiple input -> single output (octvr.hpp:47-91)
class MapperTemplate {
public:
    std::string out_type;
#ifdef OCTVR_HAVE_RAPIDJSON
    const rapidjson::Value* out_opts = nullptr;
#else
    const void* out_opts = nullptr;
#endif
    cv::Size out_size;

    typedef struct {
        cv::Rect roi;  // related to out_size
        cv::Mat map1, map2;
        cv::Mat mask;
        cv::Mat vignette;
        std::vector<cv::Vec6f> src_triangles, dst_triangles;
    } Input;

    std::vector<Input> inputs;
    std::vector<Input> overlay_inputs;

    std::vector<cv::Mat> seam_masks;  // only for inputs (not overlay_inputs)
    std::vector<bool> visible_mask;   // only used in dumper (for green mask of PTGui)

    CameraInterface* output_cam = nullptr;
    std::vector<CameraInterface*> input_cams;

public:
    // Create new template; width/height must be suitable to the output model
    // (template.cpp:23-44; <= 0 derives one from the other through the output's aspect ratio)
    MapperTemplate(const std::string& to, const std::string& to_opts_json, int width, int height) {
        create(to, to_opts_json, width, height, 0);
    }
#ifdef OCTVR_HAVE_RAPIDJSON
    MapperTemplate(const std::string& to, const rapidjson::Value& to_opts, int width, int height) {
        out_opts = &to_opts;
        create(to, detail::json_exact(to_opts), width, height, OCTVR_JSON_EXACT);
    }
    void add_input(const std::string& from, const rapidjson::Value& from_opts, bool overlay = false,
                   bool use_roi = true) {
        add(from, detail::json_exact(from_opts), overlay, use_roi, OCTVR_JSON_EXACT);
    }
    void morph_controlpoints(const rapidjson::Value& control_points) {
        morph(detail::json_exact(control_points));
    }
#endif
    // add_input (template.cpp:46-153) with the options object as JSON text (parsed as rapidjson does)
    void add_input(const std::string& from, const std::string& from_opts_json, bool overlay = false,
                   bool use_roi = true) {
        add(from, from_opts_json, overlay, use_roi, 0);
    }
    void add_input(const std::string& from, const char* from_opts_json, bool overlay = false, bool use_roi = true) {
        add(from, std::string(from_opts_json), overlay, use_roi, 0);
    }
    // Prepare seam masks (template.cpp:155-204): the L2 distance seam finder without images
    void create_masks(const std::vector<cv::Mat>& imgs = std::vector<cv::Mat>()) {
        if (!imgs.empty())
            throw cv::Exception(OCTVR_E_UNSUPPORTED,
                                "create_masks with images (GraphCutSeamFinder) is not supported; pass no images");
        detail::RigPtr r = from_fields(false);
        detail::check(octvr_rig_create_masks(r.get(), detail::device()));
        pull_seams(r.get());
    }
    // morph_controlpoints (template_morph.cpp:69-237): JSON text of the control-point array
    void morph_controlpoints(const std::string& control_points_json) { morph(control_points_json); }
    void morph_controlpoints(const char* control_points_json) { morph(control_points_json); }

    // VRv11 writer (template.cpp:206-256); creates the seam masks first when there are none
    void dump(std::ofstream& f) {
        detail::RigPtr r = from_fields(true);
        detail::check(octvr_rig_dump_stream(r.get(), &MapperTemplate::write_cb, static_cast<std::ostream*>(&f)));
        if (seam_masks.empty()) pull_seams(r.get());  // dump created them (template.cpp:209-210)
    }

    // Load existing template (template.cpp:258-314)
    explicit MapperTemplate(std::ifstream& f) {
        octvr_rig* r = nullptr;
        detail::check(octvr_rig_load_stream(&MapperTemplate::read_cb, static_cast<std::istream*>(&f), &r));
        detail::RigPtr rp = detail::own(r);
        pull(rp.get());
    }
    ~MapperTemplate() {}

    // the C ABI rig equivalent to the current public fields (for mappers built from this template)
    detail::RigPtr rig() const { return from_fields(true); }

private:
    detail::OwnedRig cams_;  // the rig with the camera models (JSON-built templates), for add_input / morph

    void create(const std::string& to, const std::string& opts, int w, int h, int flags) {
        octvr_rig* r = nullptr;
        detail::check(octvr_rig_create(to.c_str(), opts.c_str(), w, h, detail::device(), flags, &r));
        cams_.p = detail::own(r);
        out_type = to;
        int ow = 0, oh = 0;
        detail::check(octvr_rig_out_size(r, &ow, &oh));
        out_size = cv::Size(ow, oh);
    }
    void add(const std::string& from, const std::string& opts, bool overlay, bool use_roi, int flags) {
        if (!cams_.p) throw cv::Exception(OCTVR_E_UNSUPPORTED, "add_input needs a template created from an output camera");
        detail::check(octvr_rig_add_input(cams_.p.get(), from.c_str(), opts.c_str(), overlay ? 1 : 0, use_roi ? 1 : 0,
                                          flags));
        pull(cams_.p.get());
    }
    void morph(const std::string& cps) {
        if (!cams_.p) throw cv::Exception(OCTVR_E_UNSUPPORTED, "morph_controlpoints needs the camera models (a JSON-built template)");
        int kept = 0;
        detail::check(octvr_rig_morph_controlpoints(cams_.p.get(), cps.c_str(), &kept));
        pull(cams_.p.get());
    }

    static Input input_of(const octvr_rig* r, int i, bool overlay, const uint8_t** seam) {
        octvr_input_view v;
        detail::check(overlay ? octvr_rig_get_overlay(r, i, &v) : octvr_rig_get_input(r, i, &v));
        Input in;
        in.roi = cv::Rect(v.roi_x, v.roi_y, v.roi_w, v.roi_h);
        in.map1 = detail::mat_copy(v.map1, v.roi_h, v.roi_w, CV_32FC1);
        in.map2 = detail::mat_copy(v.map2, v.roi_h, v.roi_w, CV_32FC1);
        in.mask = detail::mat_copy(v.mask, v.roi_h, v.roi_w, CV_8UC1);
        if (v.vignette && v.vignette_w > 0 && v.vignette_h > 0)
            in.vignette = detail::mat_copy(v.vignette, v.vignette_h, v.vignette_w, CV_32FC1);
        if (!overlay) {
            int nt = 0;
            detail::check(octvr_rig_get_triangles(r, i, nullptr, nullptr, 0, &nt));
            if (nt > 0) {
                std::vector<float> s(6 * (size_t)nt), d(6 * (size_t)nt);
                detail::check(octvr_rig_get_triangles(r, i, s.data(), d.data(), nt, &nt));
                in.src_triangles.resize(nt);
                in.dst_triangles.resize(nt);
                for (int t = 0; t < nt; t++)
                    for (int k = 0; k < 6; k++) {
                        in.src_triangles[t][k] = s[6 * t + k];
                        in.dst_triangles[t][k] = d[6 * t + k];
                    }
            }
        }
        if (seam) *seam = v.seam_mask;
        return in;
    }
    void pull(const octvr_rig* r) {
        int ow = 0, oh = 0, n = 0, no = 0;
        detail::check(octvr_rig_out_size(r, &ow, &oh));
        out_size = cv::Size(ow, oh);
        detail::check(octvr_rig_num_inputs(r, &n));
        detail::check(octvr_rig_num_overlays(r, &no));
        inputs.clear();
        overlay_inputs.clear();
        seam_masks.clear();
        std::vector<cv::Mat> seams;
        for (int i = 0; i < n; i++) {
            const uint8_t* s = nullptr;
            inputs.push_back(input_of(r, i, false, &s));
            if (s) seams.push_back(detail::mat_copy(s, inputs.back().roi.height, inputs.back().roi.width, CV_8UC1));
        }
        if ((int)seams.size() == n && n > 0) seam_masks = seams;
        for (int i = 0; i < no; i++) overlay_inputs.push_back(input_of(r, i, true, nullptr));
    }
    void pull_seams(const octvr_rig* r) {
        int n = 0;
        detail::check(octvr_rig_num_inputs(r, &n));
        seam_masks.clear();
        for (int i = 0; i < n; i++) {
            octvr_input_view v;
            detail::check(octvr_rig_get_input(r, i, &v));
            seam_masks.push_back(detail::mat_copy(v.seam_mask, v.roi_h, v.roi_w, CV_8UC1));
        }
    }
    detail::RigPtr from_fields(bool with_seams) const {
        const int n = (int)inputs.size();
        if (n == 0) throw cv::Exception(OCTVR_E_INVALID, "template has no inputs");
        std::vector<int> rois;
        std::vector<cv::Mat> keep;
        std::vector<const float*> m1, m2;
        std::vector<const uint8_t*> mk, sm;
        for (const Input& in : inputs) {
            const cv::Mat a = detail::packed(in.map1), b = detail::packed(in.map2), c = detail::packed(in.mask);
            if (a.type() != CV_32FC1 || b.type() != CV_32FC1 || c.type() != CV_8UC1 || a.size() != in.roi.size() ||
                b.size() != in.roi.size() || c.size() != in.roi.size())
                throw cv::Exception(OCTVR_E_INVALID, "input maps / mask do not match the ROI");
            keep.push_back(a);
            keep.push_back(b);
            keep.push_back(c);
            rois.insert(rois.end(), {in.roi.x, in.roi.y, in.roi.width, in.roi.height});
            m1.push_back(reinterpret_cast<const float*>(a.data));
            m2.push_back(reinterpret_cast<const float*>(b.data));
            mk.push_back(c.data);
        }
        const bool seams = with_seams && !seam_masks.empty();
        if (seams) {
            if ((int)seam_masks.size() != n) throw cv::Exception(OCTVR_E_INVALID, "one seam mask per input");
            for (int i = 0; i < n; i++) {
                const cv::Mat s = detail::packed(seam_masks[i]);
                if (s.type() != CV_8UC1 || s.size() != inputs[i].roi.size())
                    throw cv::Exception(OCTVR_E_INVALID, "seam mask does not match the ROI");
                keep.push_back(s);
                sm.push_back(s.data);
            }
        }
        octvr_rig* r = nullptr;
        detail::check(octvr_rig_create_from_arrays(out_size.width, out_size.height, n, rois.data(), m1.data(), m2.data(),
                                                   mk.data(), seams ? sm.data() : nullptr, &r));
        detail::RigPtr rp = detail::own(r);
        for (int i = 0; i < n; i++) set_vignette(r, i, 0, inputs[i].vignette);
        for (size_t i = 0; i < overlay_inputs.size(); i++) {
            const Input& in = overlay_inputs[i];
            const cv::Mat a = detail::packed(in.map1), b = detail::packed(in.map2), c = detail::packed(in.mask);
            const int roi[4] = {in.roi.x, in.roi.y, in.roi.width, in.roi.height};
            detail::check(octvr_rig_add_overlay_arrays(r, roi, reinterpret_cast<const float*>(a.data),
                                                       reinterpret_cast<const float*>(b.data), c.data));
            set_vignette(r, (int)i, 1, in.vignette);
        }
        return rp;
    }
    static void set_vignette(octvr_rig* r, int i, int overlay, const cv::Mat& v) {
        if (v.empty()) return;
        const cv::Mat p = detail::packed(v);
        if (p.type() != CV_32FC1) throw cv::Exception(OCTVR_E_INVALID, "vignette must be CV_32FC1");
        detail::check(octvr_rig_set_vignette(r, i, overlay, reinterpret_cast<const float*>(p.data), p.cols, p.rows));
    }
    static size_t write_cb(void* ctx, const void* data, size_t n) {
        std::ostream* os = static_cast<std::ostream*>(ctx);
        os->write(static_cast<const char*>(data), (std::streamsize)n);
        return *os ? n : 0;
    }
    static size_t read_cb(void* ctx, void* buf, size_t n) {
        std::istream* is = static_cast<std::istream*>(ctx);
        is->read(static_cast<char*>(buf), (std::streamsize)n);
        return (size_t)is->gcount();
    }
};

// vr::Mapper (modules/octvr/src/mapper.hpp:29-95): one rig's per-frame stitch on the GPU.
class Mapper {
public:
    // blend: 0 = do not blend, > 0 = multi-band blend width, < 0 = feather blend width.
    // flags (not in the reference): OCTVR_REMAP_TEXTURE samples as the reference's CUDA fastRemap does
    // (octvr_hip.h octvr_mapper_create_ex); 0 = cv::remap's fixed point.
    Mapper(const MapperTemplate& mt, std::vector<cv::Size> in_sizes, int blend = 128,
           bool enable_gain_compensator = true, cv::Size scale_output = cv::Size(0, 0), int flags = 0) {
        rig_ = mt.rig();
        std::vector<int> w, h;
        for (const cv::Size& s : in_sizes) {
            w.push_back(s.width);
            h.push_back(s.height);
        }
        n_ = (int)in_sizes.size();
        octvr_mapper* m = nullptr;
        detail::check(octvr_mapper_create_ex(rig_.get(), detail::device(), n_, w.data(), h.data(), blend,
                                             enable_gain_compensator ? 1 : 0, scale_output.width, scale_output.height,
                                             flags, &m));
        m_ = std::shared_ptr<octvr_mapper>(m, [](octvr_mapper* p) { octvr_mapper_destroy(p); });
        out_ = scale_output.width > 0 ? scale_output : mt.out_size;
        sizes_ = in_sizes;
    }
    // inputs and output are YUV420P GpuMats (CV_8U, 3H/2 rows) in the layout of mapper.hpp:75-83;
    // preview_output (CV_8UC3, optional) receives the RGB result resized (mapper.cpp:308-312).
    // Returns after the stitch has completed, as the reference's (stream_final.waitForCompletion()).
    void stitch(std::vector<cv::cuda::GpuMat>& inputs, cv::cuda::GpuMat& output, cv::cuda::GpuMat& preview_output,
                std::vector<double> gains = std::vector<double>()) {
        if ((int)inputs.size() != n_) throw cv::Exception(OCTVR_E_INVALID, "input count does not match the mapper");
        std::vector<const uint8_t*> p;
        std::vector<size_t> pitch;
        for (int i = 0; i < n_; i++) {  // mapper.cpp:208-217
            if (inputs[i].type() != CV_8UC1 || inputs[i].cols != sizes_[i].width ||
                inputs[i].rows / 3 * 2 != sizes_[i].height)
                throw cv::Exception(OCTVR_E_INVALID, "input frame is not a YUV420P image of the mapper's input size");
            p.push_back(inputs[i].data);
            pitch.push_back(inputs[i].step);
        }
        if (output.empty()) output.create(out_.height * 3 / 2, out_.width, CV_8UC1);
        if (output.type() != CV_8UC1 || output.cols != out_.width || output.rows / 3 * 2 != out_.height)
            throw cv::Exception(OCTVR_E_INVALID, "output is not a YUV420P image of the output size");
        const double* g = gains.empty() ? nullptr : gains.data();
        if (!preview_output.empty()) {
            if (preview_output.type() != CV_8UC3) throw cv::Exception(OCTVR_E_INVALID, "preview_output must be CV_8UC3");
            detail::check(octvr_mapper_stitch_preview(m_.get(), p.data(), pitch.data(), output.data, output.step,
                                                      preview_output.data, preview_output.cols, preview_output.rows,
                                                      preview_output.step, g, (int)gains.size(), nullptr));
        } else {
            detail::check(octvr_mapper_stitch_yuv420p(m_.get(), p.data(), pitch.data(), output.data, output.step, g,
                                                      (int)gains.size(), nullptr));
        }
        detail::check(octvr_stream_sync(nullptr));
    }
    std::vector<double> gains() const {
        std::vector<double> g(n_);
        detail::check(octvr_mapper_gains(m_.get(), g.data(), n_));
        return g;
    }
    void override_logo_option(bool option = true) { (void)option; }
    octvr_mapper* handle() const { return m_.get(); }

private:
    detail::RigPtr rig_;
    std::shared_ptr<octvr_mapper> m_;
    int n_ = 0;
    cv::Size out_;
    std::vector<cv::Size> sizes_;
};

struct PreviewDataHeader {
    int width, height;
    int step;
    double fps;
};
static_assert(sizeof(PreviewDataHeader) == sizeof(octvr_preview_header), "PreviewDataHeader = octvr_preview_header");

// AsyncMultiMapper (octvr.hpp:103-121, async.cpp:195-350): several mappers over the same frames, each
// writing its region of one merged output, behind a 3-deep H2D / stitch / D2H pipeline.
class AsyncMultiMapper {
public:
    static AsyncMultiMapper* New(const std::vector<MapperTemplate>& mts, std::vector<cv::Size> in_sizes,
                                 cv::Size out_size, std::vector<int> blend_modes, std::vector<int> gain_modes,
                                 std::vector<cv::Rect_<double>> output_regions, cv::Size preview_size,
                                 int flags = 0);  // flags (not in the reference): octvr_async_create_ex
    // Push one frame, in YUV420P format: per input (Y, U, V) host planes; the output's (Y, U, V) planes
    virtual void push(std::vector<std::tuple<cv::Mat, cv::Mat, cv::Mat>>& inputs,
                      std::tuple<cv::Mat, cv::Mat, cv::Mat>& output) = 0;
    virtual void pop() = 0;
    // Not in the reference: the latest published preview (CV_8UC3, preview_size) and its header; false
    // before the first frame completes.  Throws without a preview.
    virtual bool preview(cv::Mat& rgb, PreviewDataHeader& hdr) = 0;
    virtual ~AsyncMultiMapper() {}
};

namespace detail {
class AsyncMultiMapperImpl : public AsyncMultiMapper {
public:
    AsyncMultiMapperImpl(const std::vector<MapperTemplate>& mts, std::vector<cv::Size> in_sizes, cv::Size out_size,
                         std::vector<int> blend_modes, std::vector<int> gain_modes,
                         std::vector<cv::Rect_<double>> output_regions, cv::Size preview_size, int flags = 0)
        : preview_size_(preview_size.area() > 0 ? preview_size : cv::Size(0, 0)) {
        const size_t k = mts.size();
        if (blend_modes.size() != k || gain_modes.size() != k || output_regions.size() != k)
            throw cv::Exception(OCTVR_E_INVALID, "one blend mode, gain mode and output region per template");
        std::vector<RigPtr> rigs;
        std::vector<const octvr_rig*> rp;
        for (const MapperTemplate& mt : mts) {
            rigs.push_back(mt.rig());
            rp.push_back(rigs.back().get());
        }
        std::vector<int> w, h;
        for (const cv::Size& s : in_sizes) {
            w.push_back(s.width);
            h.push_back(s.height);
        }
        std::vector<double> reg;
        for (const cv::Rect_<double>& r : output_regions) reg.insert(reg.end(), {r.x, r.y, r.width, r.height});
        n_ = (int)in_sizes.size();
        octvr_async* a = nullptr;
        check(octvr_async_create_preview(rp.data(), (int)k, device(), n_, w.data(), h.data(), out_size.width,
                                         out_size.height, blend_modes.data(), gain_modes.data(), reg.data(), flags,
                                         preview_size_.width, preview_size_.height, &a));
        a_ = a;
#ifdef HAVE_QT5
        if (preview_size_.area() > 0) {  // async.cpp:307-334: attach the zones the preview widget created
            qt_.reset(new QtZones());
            attach(qt_->d0, OCTVR_PREVIEW_DATA0_MEMORY_KEY);
            attach(qt_->d1, OCTVR_PREVIEW_DATA1_MEMORY_KEY);
            attach(qt_->meta, OCTVR_PREVIEW_DATA_META_MEMORY_KEY);
            check(octvr_async_set_preview_sink(a_, &AsyncMultiMapperImpl::qt_sink, qt_.get()));
        }
#endif
    }
    ~AsyncMultiMapperImpl() override { octvr_async_destroy(a_); }
    void push(std::vector<std::tuple<cv::Mat, cv::Mat, cv::Mat>>& inputs,
              std::tuple<cv::Mat, cv::Mat, cv::Mat>& output) override {
        if ((int)inputs.size() != n_) throw cv::Exception(OCTVR_E_INVALID, "input count does not match");
        std::vector<const uint8_t*> in;
        std::vector<size_t> ip;
        Held hold;
        for (auto& t : inputs) {
            for (const cv::Mat* m : {&std::get<0>(t), &std::get<1>(t), &std::get<2>(t)}) {
                in.push_back(m->data);
                ip.push_back(m->step);
                hold.push_back(*m);  // the caller's buffers must stay alive until pop (refcounted headers)
            }
        }
        uint8_t* out[3] = {std::get<0>(output).data, std::get<1>(output).data, std::get<2>(output).data};
        size_t op[3] = {std::get<0>(output).step, std::get<1>(output).step, std::get<2>(output).step};
        hold.push_back(std::get<0>(output));
        hold.push_back(std::get<1>(output));
        hold.push_back(std::get<2>(output));
        check(octvr_async_push(a_, in.data(), ip.data(), out, op));
        held_.push_back(std::move(hold));
    }
    void pop() override {
        const int rc = octvr_async_pop(a_);
        if (!held_.empty()) held_.pop_front();
        check(rc);
    }
    bool preview(cv::Mat& rgb, PreviewDataHeader& hdr) override {
        if (preview_size_.area() == 0) throw cv::Exception(OCTVR_E_INVALID, "no preview (preview_size 0)");
        if (rgb.rows != preview_size_.height || rgb.cols != preview_size_.width || rgb.type() != CV_8UC3)
            rgb.create(preview_size_.height, preview_size_.width, CV_8UC3);
        octvr_preview_header h{};
        check(octvr_async_pop_preview(a_, rgb.data, rgb.step, &h));
        hdr.width = h.width;
        hdr.height = h.height;
        hdr.step = h.step;
        hdr.fps = h.fps;
        return h.width != 0;
    }

private:
#ifdef HAVE_QT5
    struct QtZones {
        QSharedMemory d0, d1, meta;
    };
    static void attach(QSharedMemory& x, const char* key) {
        x.setKey(key);
        if (!x.attach()) throw cv::Exception(OCTVR_E_INVALID, "preview shared memory: " + x.errorString().toStdString());
    }
    // run_copy_outputs_hostmem_to_mat's preview write (async.cpp:149-171): the zone the widget is not
    // reading (meta byte), locked, RGB bytes after the header, then the header
    static void qt_sink(void* user, const uint8_t* rgb, size_t pitch, const octvr_preview_header* h) {
        QtZones* z = static_cast<QtZones*>(user);
        const char zone = *static_cast<const char*>(z->meta.data());
        QSharedMemory& target = zone == 0 ? z->d0 : z->d1;
        target.lock();
        char* base = static_cast<char*>(target.data());
        for (int y = 0; y < h->height; y++)
            memcpy(base + sizeof(PreviewDataHeader) + (size_t)y * h->width * 3, rgb + (size_t)y * pitch, (size_t)h->width * 3);
        PreviewDataHeader* hdr = reinterpret_cast<PreviewDataHeader*>(base);
        hdr->width = h->width;
        hdr->height = h->height;
        hdr->step = 0;
        hdr->fps = h->fps;
        target.unlock();
    }
    std::unique_ptr<QtZones> qt_;
#endif
    typedef std::vector<cv::Mat> Held;
    cv::Size preview_size_;
    octvr_async* a_ = nullptr;
    int n_ = 0;
    std::deque<Held> held_;
};
}  // namespace detail

inline AsyncMultiMapper* AsyncMultiMapper::New(const std::vector<MapperTemplate>& mts, std::vector<cv::Size> in_sizes,
                                               cv::Size out_size, std::vector<int> blend_modes,
                                               std::vector<int> gain_modes,
                                               std::vector<cv::Rect_<double>> output_regions, cv::Size preview_size,
                                               int flags) {
    return new detail::AsyncMultiMapperImpl(mts, in_sizes, out_size, blend_modes, gain_modes, output_regions,
                                            preview_size, flags);
}

// FastMapper (octvr.hpp:123-144, mapper_fast.cpp:27-195): the feather-blended NV12 stitch.
class FastMapper {
public:
    FastMapper(const MapperTemplate& mt, std::vector<cv::Size> in_sizes) : in_sizes_(in_sizes), out_size_(mt.out_size) {
        rig_ = mt.rig();
        std::vector<int> w, h;
        for (const cv::Size& s : in_sizes) {
            w.push_back(s.width);
            h.push_back(s.height);
        }
        octvr_fastmapper* f = nullptr;
        detail::check(octvr_fastmapper_create(rig_.get(), detail::device(), (int)in_sizes.size(), w.data(), h.data(), &f));
        f_ = std::shared_ptr<octvr_fastmapper>(f, [](octvr_fastmapper* p) { octvr_fastmapper_destroy(p); });
    }
    // mapper_fast.cpp:111-151 throws: only the NV12 path is implemented in the reference
    void stitch(const std::vector<cv::UMat>& inputs, cv::UMat& output) {
        (void)inputs;
        (void)output;
        throw cv::Exception(OCTVR_E_UNSUPPORTED, "FastMapper::stitch is not implemented (use stitch_nv12)");
    }
    // inputs: NV12 images (3H/2 x W, CV_8U); output: 3H/2 x W NV12 with the reference's swapped chroma
    // order (mapper_fast.cpp:175-193).  Host UMats are uploaded and the result downloaded (the
    // reference's UMat moves through OpenCL buffers the same way).
    void stitch_nv12(const std::vector<cv::UMat>& inputs, cv::UMat& output) {
        const size_t n = inputs.size();
        if (n != in_sizes_.size()) throw cv::Exception(OCTVR_E_INVALID, "input count does not match");
        std::vector<cv::cuda::GpuMat> dev(n);
        std::vector<const uint8_t*> p;
        std::vector<size_t> pitch;
        for (size_t i = 0; i < n; i++) {
            const cv::UMat& u = inputs[i];
            if (u.type() != CV_8UC1 || u.cols != in_sizes_[i].width || u.rows != in_sizes_[i].height * 3 / 2)
                throw cv::Exception(OCTVR_E_INVALID, "input is not an NV12 image of the input size");
            dev[i].upload(u);
            p.push_back(dev[i].data);
            pitch.push_back(dev[i].step);
        }
        if (out_dev_.rows != out_size_.height * 3 / 2 || out_dev_.cols != out_size_.width)
            out_dev_.create(out_size_.height * 3 / 2, out_size_.width, CV_8UC1);
        detail::check(octvr_fastmapper_stitch_nv12(f_.get(), p.data(), pitch.data(), out_dev_.data, out_dev_.step,
                                                   nullptr));
        detail::check(octvr_stream_sync(nullptr));
        cv::Mat host;
        out_dev_.download(host);
        output = cv::UMat(host);
    }

private:
    std::vector<cv::Size> in_sizes_;
    cv::Size out_size_;
    detail::RigPtr rig_;
    std::shared_ptr<octvr_fastmapper> f_;
    cv::cuda::GpuMat out_dev_;
};

// Timer (timer.cpp:20-70): wall-clock milliseconds since the last tick, logged to stderr
class Timer {
protected:
    int64_t t;
    std::string name;

public:
    explicit Timer(std::string n) : t(now_us()), name(std::move(n)) {}
    Timer() : Timer("") {}
    double tick(std::string msg) {
        const int64_t n = now_us();
        const double ms = (double)(n - t) / 1000.0;
        t = n;
        std::cerr << "[ Timer " << name << "] " << msg << ": " << ms << "ms" << std::endl;
        return ms;
    }

private:
    static int64_t now_us() {
        return std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now().time_since_epoch())
            .count();
    }
};

// Queue (octvr.hpp:161-182): a blocking FIFO (empty() takes the lock here; the reference's does not)
template <class T>
class Queue {
private:
    std::queue<T> q;
    std::mutex mtx;
    std::condition_variable cond_empty;

public:
    bool empty() {
        std::lock_guard<std::mutex> guard(mtx);
        return q.empty();
    }
    void push(T&& val) {
        std::lock_guard<std::mutex> guard(mtx);
        q.push(std::forward<T>(val));
        cond_empty.notify_one();
    }
    void push(const T& val) { this->push(T(val)); }
    T pop() {
        std::unique_lock<std::mutex> lock(mtx);
        cond_empty.wait(lock, [this]() { return !q.empty(); });
        T ret = q.front();
        q.pop();
        return ret;
    }
};

}  // namespace vr

#endif
