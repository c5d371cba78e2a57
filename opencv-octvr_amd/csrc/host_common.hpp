// host_common.hpp — host-side helpers shared by the library's translation units (internal):
// error model of the C ABI (status codes, never exceptions across the boundary), device buffers,
// and the rig (vr::MapperTemplate) representation.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

#include "octvr_hip.h"

namespace octvr {

struct OctvrError : std::runtime_error {
    int code;
    OctvrError(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

#define HIP_CHECK(expr)                                                                                \
    do {                                                                                               \
        hipError_t e_ = (expr);                                                                        \
        if (e_ != hipSuccess)                                                                          \
            throw ::octvr::OctvrError(OCTVR_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

#define REQUIRE(cond, msg)                                                  \
    do {                                                                    \
        if (!(cond)) throw ::octvr::OctvrError(OCTVR_E_INVALID, (msg));     \
    } while (0)

// Scoped device selection: restores the caller's current device.
struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        HIP_CHECK(hipGetDevice(&prev));
        if (dev != prev) HIP_CHECK(hipSetDevice(dev));
    }
    ~DeviceGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

template <class T>
struct DevBuf {
    T* p = nullptr;
    size_t n = 0;
    DevBuf() = default;
    DevBuf(const DevBuf&) = delete;
    DevBuf& operator=(const DevBuf&) = delete;
    DevBuf(DevBuf&& o) noexcept : p(o.p), n(o.n) { o.p = nullptr; o.n = 0; }
    ~DevBuf() { reset(); }
    void alloc(size_t count) {
        reset();
        if (count == 0) return;
        HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&p), count * sizeof(T)));
        n = count;
    }
    void upload(const T* h, size_t count) {
        alloc(count);
        if (count) HIP_CHECK(hipMemcpy(p, h, count * sizeof(T), hipMemcpyHostToDevice));
    }
    void reset() {
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
    }
};

}  // namespace octvr

// =================================================================================================
// Rig (vr::MapperTemplate, octvr.hpp:47-91): host-resident, like the reference's cv::Mat members.
// =================================================================================================
struct RigInput {
    int roi[4] = {0, 0, 0, 0};
    int in_w = 0, in_h = 0;  // input image size when known (JSON rigs)
    std::vector<float> map1, map2;
    std::vector<uint8_t> mask;
    std::vector<float> vignette;
    int vig_w = 0, vig_h = 0;
};

struct octvr_rig {
    int out_w = 0, out_h = 0;
    int device = 0;  // device used for GPU-side template work (LUT build, seam resizes)
    std::vector<RigInput> inputs;
    std::vector<RigInput> overlays;
    std::vector<std::vector<uint8_t>> seam_masks;
};

namespace octvr {
// MapperTemplate::create_masks() (template.cpp:155-204) — seams.cpp
void rig_create_masks(octvr_rig& rig);
}  // namespace octvr
