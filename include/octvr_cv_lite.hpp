/*
 * octvr_cv_lite.hpp — the small part of OpenCV's core types that the octvr C++ API (include/octvr.hpp)
 * exposes, for builds without OpenCV.  With OpenCV present, octvr.hpp uses the real types instead; this
 * header only defines what the reference's API signatures and its callers (apps/octvr/dump.cpp,
 * map.cpp, the AsyncMultiMapper caller) touch:
 *   cv::Size, cv::Point / Point2d, cv::Rect / Rect_<double>, cv::Vec6f, cv::Mat, cv::UMat (host
 *   memory here: the reference's OpenCL UMat path is replaced by HIP behind the C ABI),
 *   cv::cuda::GpuMat (HIP device memory), cv::Exception, CV_8UC1 / CV_8UC3 / CV_8UC4 / CV_32FC1.
 * Mats are reference counted and share data on copy, as OpenCV's do (opencv2/core/mat.hpp).
 */
#ifndef OCTVR_CV_LITE_HPP
#define OCTVR_CV_LITE_HPP

#include <cstddef>
#include <cstdint>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>

#include "octvr_hip.h"

#ifndef CV_8U
#define CV_CN_SHIFT 3
#define CV_MAKETYPE(depth, cn) ((depth) + (((cn)-1) << CV_CN_SHIFT))
#define CV_8U 0
#define CV_8S 1
#define CV_16U 2
#define CV_16S 3
#define CV_32S 4
#define CV_32F 5
#define CV_64F 6
#define CV_8UC1 CV_MAKETYPE(CV_8U, 1)
#define CV_8UC3 CV_MAKETYPE(CV_8U, 3)
#define CV_8UC4 CV_MAKETYPE(CV_8U, 4)
#define CV_32FC1 CV_MAKETYPE(CV_32F, 1)
#define CV_32FC3 CV_MAKETYPE(CV_32F, 3)
#endif

namespace cv {

typedef unsigned char uchar;

class Exception : public std::runtime_error {
public:
    int code;
    explicit Exception(int c, const std::string& msg) : std::runtime_error(msg), code(c) {}
};

template <typename T>
struct Size_ {
    T width = 0, height = 0;
    Size_() = default;
    Size_(T w, T h) : width(w), height(h) {}
    T area() const { return width * height; }
    bool empty() const { return width <= 0 || height <= 0; }
    bool operator==(const Size_& o) const { return width == o.width && height == o.height; }
    bool operator!=(const Size_& o) const { return !(*this == o); }
};
typedef Size_<int> Size;

template <typename T>
struct Point_ {
    T x = 0, y = 0;
    Point_() = default;
    Point_(T x_, T y_) : x(x_), y(y_) {}
};
typedef Point_<int> Point;
typedef Point_<double> Point2d;

template <typename T>
struct Rect_ {
    T x = 0, y = 0, width = 0, height = 0;
    Rect_() = default;
    Rect_(T x_, T y_, T w, T h) : x(x_), y(y_), width(w), height(h) {}
    Size_<T> size() const { return Size_<T>(width, height); }
    Point_<T> tl() const { return Point_<T>(x, y); }
    T area() const { return width * height; }
    bool operator==(const Rect_& o) const { return x == o.x && y == o.y && width == o.width && height == o.height; }
};
typedef Rect_<int> Rect;

template <typename T, int n>
struct Vec {
    T val[n] = {};
    T& operator[](int i) { return val[i]; }
    const T& operator[](int i) const { return val[i]; }
};
typedef Vec<float, 6> Vec6f;

inline int cv_depth(int type) { return type & 7; }
inline int cv_channels(int type) { return (type >> CV_CN_SHIFT) + 1; }
inline size_t cv_elem_size1(int depth) {
    static const size_t s[8] = {1, 1, 2, 2, 4, 4, 8, 2};
    return s[depth & 7];
}

// Host image, reference counted (a copy shares the data; clone() copies it).
class Mat {
public:
    int rows = 0, cols = 0;
    uchar* data = nullptr;
    size_t step = 0;  // bytes per row

    Mat() = default;
    Mat(int r, int c, int type) { create(r, c, type); }
    Mat(Size s, int type) { create(s.height, s.width, type); }
    // wrap caller memory (not owned), as cv::Mat(rows, cols, type, data, step)
    Mat(int r, int c, int type, void* d, size_t st = 0) : rows(r), cols(c), data((uchar*)d), type_(type) {
        step = st ? st : (size_t)c * elemSize();
    }
    void create(int r, int c, int type) {
        if (rows == r && cols == c && type_ == type && data) return;
        type_ = type;
        rows = r;
        cols = c;
        step = (size_t)c * elemSize();
        holder_.reset();
        data = nullptr;
        if (r > 0 && c > 0) {
            holder_ = std::shared_ptr<uchar>(new uchar[step * (size_t)r](), std::default_delete<uchar[]>());
            data = holder_.get();
        }
    }
    void create(Size s, int type) { create(s.height, s.width, type); }
    void release() { *this = Mat(); }
    int type() const { return type_; }
    int depth() const { return cv_depth(type_); }
    int channels() const { return cv_channels(type_); }
    size_t elemSize() const { return cv_elem_size1(depth()) * (size_t)channels(); }
    bool empty() const { return data == nullptr || rows == 0 || cols == 0; }
    Size size() const { return Size(cols, rows); }
    size_t total() const { return (size_t)rows * cols; }
    bool isContinuous() const { return rows <= 1 || step == (size_t)cols * elemSize(); }
    template <typename T>
    T* ptr(int r = 0) { return reinterpret_cast<T*>(data + (size_t)r * step); }
    template <typename T>
    const T* ptr(int r = 0) const { return reinterpret_cast<const T*>(data + (size_t)r * step); }
    uchar* ptr(int r = 0) { return data + (size_t)r * step; }
    const uchar* ptr(int r = 0) const { return data + (size_t)r * step; }
    template <typename T>
    T& at(int r, int c) { return ptr<T>(r)[c]; }
    template <typename T>
    const T& at(int r, int c) const { return ptr<T>(r)[c]; }
    // ROI view sharing the data (cv::Mat::operator()(Rect))
    Mat operator()(const Rect& roi) const {
        Mat m(*this);
        m.data = data + (size_t)roi.y * step + (size_t)roi.x * elemSize();
        m.rows = roi.height;
        m.cols = roi.width;
        return m;
    }
    Mat clone() const {
        Mat m(rows, cols, type_);
        for (int r = 0; r < rows; r++) memcpy(m.ptr(r), ptr(r), (size_t)cols * elemSize());
        return m;
    }
    void copyTo(Mat& dst) const {
        if (dst.data == data && dst.step == step) return;
        dst.create(rows, cols, type_);
        for (int r = 0; r < rows; r++) memcpy(dst.ptr(r), ptr(r), (size_t)cols * elemSize());
    }

private:
    int type_ = CV_8UC1;
    std::shared_ptr<uchar> holder_;
};

// The reference's OpenCL-backed UMat; here a host image like Mat (the FastMapper drop-in uploads it).
class UMat : public Mat {
public:
    using Mat::Mat;
    UMat() = default;
    UMat(const Mat& m) : Mat(m) {}
};

namespace cuda {

// Device image in HIP memory (cv::cuda::GpuMat): create() allocates on the current device through
// the C ABI (octvr_dev_malloc); a wrapped pointer is not owned.
class GpuMat {
public:
    int rows = 0, cols = 0;
    uchar* data = nullptr;
    size_t step = 0;

    GpuMat() = default;
    GpuMat(int r, int c, int type) { create(r, c, type); }
    GpuMat(Size s, int type) { create(s.height, s.width, type); }
    GpuMat(int r, int c, int type, void* d, size_t st) : rows(r), cols(c), data((uchar*)d), step(st), type_(type) {}
    void create(int r, int c, int type) {
        if (rows == r && cols == c && type_ == type && data) return;
        release();
        type_ = type;
        rows = r;
        cols = c;
        step = (size_t)c * cv_elem_size1(cv_depth(type)) * (size_t)cv_channels(type);
        if (r > 0 && c > 0) {
            int dev = 0;
            void* p = nullptr;
            if (octvr_dev_malloc(dev, step * (size_t)r, &p) != OCTVR_OK)
                throw Exception(-4, std::string("GpuMat: device allocation failed: ") + octvr_last_error());
            holder_ = std::shared_ptr<uchar>((uchar*)p, [](uchar* q) { octvr_dev_free(q); });
            data = holder_.get();
        }
    }
    void create(Size s, int type) { create(s.height, s.width, type); }
    void release() {
        holder_.reset();
        data = nullptr;
        rows = cols = 0;
        step = 0;
    }
    int type() const { return type_; }
    bool empty() const { return data == nullptr || rows == 0 || cols == 0; }
    Size size() const { return Size(cols, rows); }
    size_t elemSize() const { return cv_elem_size1(cv_depth(type_)) * (size_t)cv_channels(type_); }
    GpuMat operator()(const Rect& roi) const {
        GpuMat m(*this);
        m.data = data + (size_t)roi.y * step + (size_t)roi.x * elemSize();
        m.rows = roi.height;
        m.cols = roi.width;
        return m;
    }
    void upload(const Mat& src) {
        create(src.rows, src.cols, src.type());
        for (int r = 0; r < rows; r++)
            if (octvr_memcpy_h2d(data + (size_t)r * step, src.ptr(r), (size_t)cols * elemSize()) != OCTVR_OK)
                throw Exception(-3, octvr_last_error());
    }
    void download(Mat& dst) const {
        dst.create(rows, cols, type_);
        for (int r = 0; r < rows; r++)
            if (octvr_memcpy_d2h(dst.ptr(r), data + (size_t)r * step, (size_t)cols * elemSize()) != OCTVR_OK)
                throw Exception(-3, octvr_last_error());
    }

private:
    int type_ = CV_8UC1;
    std::shared_ptr<uchar> holder_;
};

}  // namespace cuda
}  // namespace cv

#endif
