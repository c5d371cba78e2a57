// kernels.hip — gfx950 kernels of the octVR remap + gain + composite path.
//
// Built with -ffp-contract=off: every f32/f64 expression rounds exactly as written, matching the
// reference's non-FMA x86 arithmetic (the oracle, oracle/octvr_oracle.c, is compiled the same way).
// No MFMA anywhere: this is a gather + per-pixel fixed-point blend.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstring>

#include "device_common.hpp"
#include "kernels.hpp"

namespace octvr {

constexpr int kLuBlockMin = 9;  // smallest n solved by the workgroup-parallel LU (below: one lane, registers)

// ---------------------------------------------------------------------------------------------
// LUT build: MapperTemplate::add_input (template.cpp:46-133), one thread per output pixel, FP64.
// bbox = {min_w, min_h, max_w, max_h} of valid pixels (int atomics, initialised by the host).
// fragile (optional): pixels whose outcome a last-ulp libm difference could change (LutGuard,
// camera_math.hpp) are appended as indices (fragile[0] = count, entries from fragile[1], at most
// cap kept) and left out of bbox and of the visible_mask update: the host recomputes them with glibc.
// ---------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) lut_build_kernel(const CameraParams* __restrict__ cams, int W, int H,
                                                        float* map1, float* map2, uint8_t* mask, int32_t* bbox,
                                                        uint8_t* visible, uint32_t* fragile, uint32_t cap) {
    const CameraParams& out = cams[0];
    const CameraParams& in = cams[1];
    __shared__ int s_bb[4];
    if (threadIdx.x < 4) s_bb[threadIdx.x] = (threadIdx.x < 2) ? INT32_MAX : -1;
    __syncthreads();
    const int64_t total = (int64_t)W * H;
    int lminw = INT32_MAX, lminh = INT32_MAX, lmaxw = -1, lmaxh = -1;
    for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
         idx += (int64_t)gridDim.x * blockDim.x) {
        const int h = (int)(idx / W), w = (int)(idx - (int64_t)h * W);
        double dx, dy;
        bool vis = false;
        LutGuard g{false};
        project_output_to_input(out, in, (double)w / W, (double)h / H, &dx, &dy, visible ? &vis : nullptr,
                                fragile ? &g : nullptr);
        const bool frag = fragile && (g.hit || f32_fragile(dx) || f32_fragile(dy));
        if (frag) {
            const uint32_t k = atomicAdd(fragile, 1u);
            if (k < cap) fragile[1 + k] = (uint32_t)idx;
        }
        const float x = (float)dx, y = (float)dy;
        // visible_mask arbitration (template.cpp:86-116): a pixel an earlier camera's include mask
        // claimed (1) is rejected; one this camera's include mask claims first is marked 2 so the host
        // clears it from the earlier cameras' masks.
        const bool claimed = visible && visible[idx] == 1;
        if (visible && vis && !claimed && !frag) visible[idx] = 2;
        if (isnan(x) || isnan(y) || x < 0 || x >= 1.0f || y < 0 || y >= 1.0f || claimed) {
            mask[idx] = 0;
            map1[idx] = -1.0f;
            map2[idx] = -1.0f;
        } else {
            mask[idx] = 255;
            map1[idx] = x;
            map2[idx] = y;
            if (!frag) {
                lminw = min(lminw, w);
                lmaxw = max(lmaxw, w);
                lminh = min(lminh, h);
                lmaxh = max(lmaxh, h);
            }
        }
    }
    if (lmaxw >= 0) {
        atomicMin(&s_bb[0], lminw);
        atomicMin(&s_bb[1], lminh);
        atomicMax(&s_bb[2], lmaxw);
        atomicMax(&s_bb[3], lmaxh);
    }
    __syncthreads();
    if (threadIdx.x == 0 && s_bb[2] >= 0) {
        atomicMin(&bbox[0], s_bb[0]);
        atomicMin(&bbox[1], s_bb[1]);
        atomicMax(&bbox[2], s_bb[2]);
        atomicMax(&bbox[3], s_bb[3]);
    }
}

hipError_t launch_lut_build(const CameraParams* cams_dev, int W, int H, float* map1, float* map2, uint8_t* mask,
                            int32_t* bbox, uint8_t* visible, uint32_t* fragile, uint32_t cap, hipStream_t s) {
    const int64_t total = (int64_t)W * H;
    int blocks = (int)std::min<int64_t>((total + 255) / 256, 256 * 16);
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(lut_build_kernel, dim3(blocks), dim3(256), 0, s, cams_dev, W, H, map1, map2, mask, bbox, visible,
                       fragile, cap);
    return hipGetLastError();
}

// Diagnostics (octvr_debug_project_f64): the FP64 projection of every output pixel before the f32
// rounding, with the guard's verdict (1 = fragile), for measuring device-vs-glibc deviations.
__global__ void __launch_bounds__(256) project_f64_kernel(const CameraParams* __restrict__ cams, int W, int H,
                                                          double* xs, double* ys, uint8_t* fragile) {
    const int64_t total = (int64_t)W * H;
    for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
         idx += (int64_t)gridDim.x * blockDim.x) {
        const int h = (int)(idx / W), w = (int)(idx - (int64_t)h * W);
        double dx, dy;
        LutGuard g{false};
        project_output_to_input(cams[0], cams[1], (double)w / W, (double)h / H, &dx, &dy, nullptr, &g);
        xs[idx] = dx;
        ys[idx] = dy;
        fragile[idx] = (g.hit || f32_fragile(dx) || f32_fragile(dy)) ? 1 : 0;
    }
}

hipError_t launch_project_f64(const CameraParams* cams_dev, int W, int H, double* x, double* y, uint8_t* fragile,
                              hipStream_t s) {
    const int64_t total = (int64_t)W * H;
    int blocks = (int)std::min<int64_t>((total + 255) / 256, 256 * 16);
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(project_f64_kernel, dim3(blocks), dim3(256), 0, s, cams_dev, W, H, x, y, fragile);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// Composite LUT: the no-blend copy chain `warped_i.copyTo(result(roi_i), mask_i)` in camera order
// (mapper.cpp:268-277) resolved once per rig: the LAST camera whose ROI contains the pixel and whose
// LUT mask is non-zero wins; its map value is quantized exactly as RemapInvoker does.
// ---------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) composite_lut_kernel(const CamTemplate* cams, int n, int W, int H,
                                                            CompositeEntry* lut, int tex) {
    const int64_t total = (int64_t)W * H;
    for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
         idx += (int64_t)gridDim.x * blockDim.x) {
        const int y = (int)(idx / W), x = (int)(idx - (int64_t)y * W);
        CompositeEntry e;
        e.xy = 0;
        e.code = 0;
        for (int i = 0; i < n; i++) {
            const CamTemplate& c = cams[i];
            const int rx = x - c.roi_x, ry = y - c.roi_y;
            if (rx < 0 || ry < 0 || rx >= c.roi_w || ry >= c.roi_h) continue;
            const int64_t k = (int64_t)ry * c.roi_w + rx;
            if (c.mask[k] == 0) continue;
            e = tex ? make_entry_tex(c.map1[k], c.map2[k], (float)c.in_w, (float)c.in_h, i)
                    : make_entry(c.map1[k], c.map2[k], (float)c.in_w, (float)c.in_h, i);
        }
        lut[idx] = e;
    }
}

hipError_t launch_composite_lut(const CamTemplate* cams_dev, int n, int W, int H, CompositeEntry* lut,
                                hipStream_t s, int tex) {
    const int64_t total = (int64_t)W * H;
    int blocks = (int)std::min<int64_t>((total + 255) / 256, 256 * 16);
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(composite_lut_kernel, dim3(blocks), dim3(256), 0, s, cams_dev, n, W, H, lut, tex);
    return hipGetLastError();
}

// cv::solve (lapack.cpp:1050-1275) with the matrix in registers: closed forms for n <= 3, LUImpl
// (matrix_decomp.cpp:50-110) above, instantiated per n so every index is static.
template <int N>
__device__ bool lu_solve(double (&A)[N * N], double (&b)[N]) {
    const double eps = DBL_EPSILON * 100;
#pragma unroll
    for (int i = 0; i < N; i++) {
        int k = i;
        double best = fabs(A[i * N + i]);
#pragma unroll
        for (int j = i + 1; j < N; j++) {
            const double v = fabs(A[j * N + i]);
            if (v > best) {
                best = v;
                k = j;
            }
        }
        if (best < eps) return false;
        if (k != i) {  // rare (A is diagonally dominant here): the select-based swap only when needed
#pragma unroll
            for (int j = i + 1; j < N; j++) {  // row swap i <-> k as selects (static indices only)
                const bool sw = (j == k);
#pragma unroll
                for (int c = i; c < N; c++) {
                    const double ai = A[i * N + c], aj = A[j * N + c];
                    A[i * N + c] = sw ? aj : ai;
                    A[j * N + c] = sw ? ai : aj;
                }
                const double bi = b[i], bj = b[j];
                b[i] = sw ? bj : bi;
                b[j] = sw ? bi : bj;
            }
        }
        const double d = -1 / A[i * N + i];
#pragma unroll
        for (int j = i + 1; j < N; j++) {
            const double alpha = A[j * N + i] * d;
#pragma unroll
            for (int c = i + 1; c < N; c++) A[j * N + c] += alpha * A[i * N + c];
            b[j] += alpha * b[i];
        }
        A[i * N + i] = -d;
    }
#pragma unroll
    for (int i = N - 1; i >= 0; i--) {
        double s = b[i];
#pragma unroll
        for (int c = i + 1; c < N; c++) s -= A[i * N + c] * b[c];
        b[i] = s * A[i * N + i];
    }
    return true;
}

template <int N>
__device__ bool solve_fixed(const double* Ain, const double* bin, double* x) {
    double A[N * N], b[N];
#pragma unroll
    for (int k = 0; k < N * N; k++) A[k] = Ain[k];
#pragma unroll
    for (int k = 0; k < N; k++) b[k] = bin[k];
#define Sd(y, xx) A[(y) * N + (xx)]
    if constexpr (N == 1) {
        const double d = Sd(0, 0);
        if (d == 0.) return false;
        x[0] = b[0] / d;
        return true;
    } else if constexpr (N == 2) {
        double d = (double)Sd(0, 0) * Sd(1, 1) - (double)Sd(0, 1) * Sd(1, 0);
        if (d == 0.) return false;
        d = 1. / d;
        const double t = (b[0] * Sd(1, 1) - b[1] * Sd(0, 1)) * d;
        x[1] = (b[1] * Sd(0, 0) - b[0] * Sd(1, 0)) * d;
        x[0] = t;
        return true;
    } else if constexpr (N == 3) {
        double d = Sd(0, 0) * ((double)Sd(1, 1) * Sd(2, 2) - (double)Sd(1, 2) * Sd(2, 1)) -
                   Sd(0, 1) * ((double)Sd(1, 0) * Sd(2, 2) - (double)Sd(1, 2) * Sd(2, 0)) +
                   Sd(0, 2) * ((double)Sd(1, 0) * Sd(2, 1) - (double)Sd(1, 1) * Sd(2, 0));
        if (d == 0.) return false;
        d = 1. / d;
        x[0] = ((Sd(1, 1) * Sd(2, 2) - Sd(1, 2) * Sd(2, 1)) * b[0] + (Sd(0, 2) * Sd(2, 1) - Sd(0, 1) * Sd(2, 2)) * b[1] +
                (Sd(0, 1) * Sd(1, 2) - Sd(0, 2) * Sd(1, 1)) * b[2]) * d;
        x[1] = ((Sd(1, 2) * Sd(2, 0) - Sd(1, 0) * Sd(2, 2)) * b[0] + (Sd(0, 0) * Sd(2, 2) - Sd(0, 2) * Sd(2, 0)) * b[1] +
                (Sd(0, 2) * Sd(1, 0) - Sd(0, 0) * Sd(1, 2)) * b[2]) * d;
        x[2] = ((Sd(1, 0) * Sd(2, 1) - Sd(1, 1) * Sd(2, 0)) * b[0] + (Sd(0, 1) * Sd(2, 0) - Sd(0, 0) * Sd(2, 1)) * b[1] +
                (Sd(0, 0) * Sd(1, 1) - Sd(0, 1) * Sd(1, 0)) * b[2]) * d;
        return true;
    } else {
        if (!lu_solve<N>(A, b)) return false;
#pragma unroll
        for (int k = 0; k < N; k++) x[k] = b[k];
        return true;
    }
#undef Sd
}


// The same LUImpl with the whole workgroup: per pivot every thread finds the pivot row (same scan
// order), one thread per column swaps, one thread per (row, column) eliminates; every element sees
// exactly the serial operation sequence of LUImpl (matrix_decomp.cpp:50-110), so the result is
// bit-identical to lu_solve<N>.  Used for n = 9..16 (too large for one lane's registers).
// Call with all threads of the workgroup; returns the same flag everywhere.
__device__ bool lu_solve_block(double* A, double* b, int n, double* x) {
    const double eps = DBL_EPSILON * 100;
    const int tid = threadIdx.x, nt = blockDim.x;
    for (int i = 0; i < n; i++) {
        int k = i;
        for (int j = i + 1; j < n; j++)
            if (fabs(A[j * n + i]) > fabs(A[k * n + i])) k = j;
        if (fabs(A[k * n + i]) < eps) return false;  // uniform: every thread read the same values
        __syncthreads();
        if (k != i) {
            for (int c = i + tid; c <= n; c += nt) {  // column n is b
                double* ri = (c < n) ? &A[i * n + c] : &b[i];
                double* rk = (c < n) ? &A[k * n + c] : &b[k];
                const double t = *ri;
                *ri = *rk;
                *rk = t;
            }
            __syncthreads();
        }
        const double d = -1 / A[i * n + i];
        const int w = n - i;  // columns i+1 .. n (n = b)
        for (int q = tid; q < (n - 1 - i) * w; q += nt) {
            const int j = i + 1 + q / w, c = i + 1 + q % w;
            const double alpha = A[j * n + i] * d;
            if (c < n)
                A[j * n + c] += alpha * A[i * n + c];
            else
                b[j] += alpha * b[i];
        }
        __syncthreads();
        if (tid == 0) A[i * n + i] = -d;
        __syncthreads();
    }
    if (tid == 0) {
        for (int i = n - 1; i >= 0; i--) {
            double s = b[i];
            for (int c = i + 1; c < n; c++) s -= A[i * n + c] * b[c];
            b[i] = s * A[i * n + i];
        }
        for (int i = 0; i < n; i++) x[i] = b[i];
    }
    __syncthreads();
    return true;
}

// inlined into its one call site per feed instance (as a called function — the three frame-count instances
// made the inliner stop — the one-in-flight C2 feed's serial tail grew from 16.4 to 20.0 us)
__device__ __forceinline__ bool solve_dispatch(double* A, double* b, int n, double* x) {
    switch (n) {
#define CASE(K) \
    case K:     \
        return solve_fixed<K>(A, b, x);
        CASE(1) CASE(2) CASE(3) CASE(4) CASE(5) CASE(6) CASE(7) CASE(8)
#undef CASE
        default:
            return false;
    }
}

// n <= 3 only: the closed forms (few registers)
__device__ bool solve_small(double* A, double* b, int n, double* x) {
    switch (n) {
        case 1: return solve_fixed<1>(A, b, x);
        case 2: return solve_fixed<2>(A, b, x);
        case 3: return solve_fixed<3>(A, b, x);
        default: return false;
    }
}

// ---------------------------------------------------------------------------------------------
// Gain feed (GainCompensatorGPU::feed, exposure_compensate.cpp:223-297) — one launch.
// Sample s of camera i (a working-scale pixel, nearest resize of the warped ROI, mapper.cpp:234-237)
// contributes its f32 norm (core/src/cuda/gpu_mat.cu:443-449) to the masked sum of every pair
// (i, j) whose intersection contains it: I(i,j) = sum / N(i,j).
//
// Exact, order-free sums: a norm is sqrtf of an integer, so it is 0 or lies in [1, 442] and is a
// whole multiple of 2^-23; a pair sum of fewer than 2^21 of them (the working scale holds ~1e5
// pixels, checked on the host) is an integer below 2^53 in units of 2^-23.  Every partial sum is
// therefore exact in f64, and the per-pair totals are kept as u64 fixed point (units of 2^-23)
// added with device-scope integer atomics: the result equals the sequential f64 sum bit for bit,
// whatever order the workgroups finish in.
//
// Completion: per-XCD tickets (blockIdx % 8), then one global ticket; the last workgroup reads the
// totals with returning atomics (executed at the memory side, so no L2 staleness across XCDs),
// resets them, assembles A, b and solves.
// ---------------------------------------------------------------------------------------------
// Wave sum of an f64 through DPP moves (quad perms, row rotations, row broadcasts 15 / 31; the
// total lands in lane 63) instead of LDS-routed shuffles.  The gain-feed sums are exact (see below),
// so the summation order does not change the result.
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
    const int lo = __double2loint(v), hi = __double2hiint(v);
    return __hiloint2double(__builtin_amdgcn_update_dpp(0, hi, CTRL, 0xf, 0xf, false),
                            __builtin_amdgcn_update_dpp(0, lo, CTRL, 0xf, 0xf, false));
}
__device__ __forceinline__ double wave_sum(double v) {
    v += dpp_f64<0xb1>(v);   // quad_perm [1,0,3,2]
    v += dpp_f64<0x4e>(v);   // quad_perm [2,3,0,1]
    v += dpp_f64<0x124>(v);  // row_ror 4
    v += dpp_f64<0x128>(v);  // row_ror 8
    v += dpp_f64<0x142>(v);  // row_bcast 15
    v += dpp_f64<0x143>(v);  // row_bcast 31
    return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), 63),
                            __builtin_amdgcn_readlane(__double2loint(v), 63));
}

// Row i of GainCompensatorGPU::feed's system (exposure_compensate.cpp:279-296) from I(i,j) and
// N(i,j) (both n x n), in the reference's j order: A(i,i) = sum_j beta N + (j != i) 2 alpha I^2 N,
// A(i,j) = -2 alpha I(i,j) I(j,i) N, b(i) = sum_j beta N.  A has row stride n.
__device__ __forceinline__ void gain_system_row(const double* I, const int32_t* Nm, int n, int i, double* A, double* b) {
    const double alpha = 0.01, beta = 100;
    double bi = 0.0, aii = 0.0;
    for (int j = 0; j < n; j++) {
        const int Nij = Nm[i * n + j];
        bi += beta * Nij;
        aii += beta * Nij;
        if (j == i) continue;
        aii += 2 * alpha * I[i * n + j] * I[i * n + j] * Nij;
        A[i * n + j] = 0.0 - 2 * alpha * I[i * n + j] * I[j * n + i] * Nij;
    }
    A[i * n + i] = aii;
    b[i] = bi;
}

// Gain-feed gathers: per sample the 2 luma, 2 U and 2 V row segments of its 2x2 taps as 8-byte buffer
// loads from 4-byte aligned starts (6 loads instead of 12 byte loads).  The frame-sized buffer resource
// range-checks whole dwords, so a load may not reach past the frame's last byte: only a V row segment of
// the last chroma row can (Y rows are followed by the chroma rows, U halves by V halves), and its start
// is clamped to size - 8, the bytes taken relative to the clamped start.  Everything the extraction
// needs — the tap bytes' positions in the 8 loaded bytes as v_perm selectors, the taps' in-image flags,
// the fractions — is derived once at issue and carried to feed_taps_finish, after every sample's loads
// are in flight.
struct FeedRaw {
    uint2 y0, y1, u0, u1, v0, v1;
    uint32_t sel;   // bytes of taps x0, x1: luma (bits 0-15), chroma (16-31), as v_perm selectors
    uint32_t meta;  // code bits 0-15 (fx, fy, valid), in-image ix0 ix1 iy0 iy1 at 16-19, V row shifts at 20-22 / 23-25
};

__device__ __forceinline__ void feed_taps_issue(__amdgpu_buffer_rsrc_t rs, const SourceFrame& f, uint32_t xy,
                                                uint32_t code, FeedRaw& r) {
    const TapCell tc = tap_cell(xy, f.w, f.h);
    const uint32_t p = (uint32_t)f.pitch;
    const uint32_t lim = (uint32_t)f.pitch * (uint32_t)(f.h + f.h / 2) - 8u;  // frames >= 8 B (host check)
    const uint32_t uo = (uint32_t)f.h * p, vo = uo + (uint32_t)(f.w >> 1);
    const uint32_t x0 = (uint32_t)tc.x0, x1 = (uint32_t)tc.x1, c0 = x0 >> 1, c1 = x1 >> 1;
    const uint32_t xa = x0 & ~3u, ca = c0 & ~3u;
    const uint32_t ry0 = (uint32_t)tc.y0 * p, ry1 = (uint32_t)tc.y1 * p;
    const uint32_t rc0 = (uint32_t)(tc.y0 >> 1) * p, rc1 = (uint32_t)(tc.y1 >> 1) * p;
    const uint32_t sv0 = vo + rc0 + ca, sv1 = vo + rc1 + ca;
    const uint32_t lv0 = min(sv0, lim), lv1 = min(sv1, lim);
    typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
    u32x2 t;
    t = __builtin_amdgcn_raw_buffer_load_b64(rs, ry0 + xa, 0, 0);
    r.y0 = make_uint2(t.x, t.y);
    t = __builtin_amdgcn_raw_buffer_load_b64(rs, ry1 + xa, 0, 0);
    r.y1 = make_uint2(t.x, t.y);
    t = __builtin_amdgcn_raw_buffer_load_b64(rs, uo + rc0 + ca, 0, 0);
    r.u0 = make_uint2(t.x, t.y);
    t = __builtin_amdgcn_raw_buffer_load_b64(rs, uo + rc1 + ca, 0, 0);
    r.u1 = make_uint2(t.x, t.y);
    t = __builtin_amdgcn_raw_buffer_load_b64(rs, lv0, 0, 0);
    r.v0 = make_uint2(t.x, t.y);
    t = __builtin_amdgcn_raw_buffer_load_b64(rs, lv1, 0, 0);
    r.v1 = make_uint2(t.x, t.y);
    const uint32_t iy = x0 & 3u, ic = c0 & 3u;  // x1 - x0, c1 - c0 in {0, 1}
    r.sel = iy | (iy + (x1 - x0)) << 8 | ic << 16 | (ic + (c1 - c0)) << 24;
    r.meta = (code & 0xFFFFu) | (tc.ix0 ? 1u << 16 : 0u) | (tc.ix1 ? 1u << 17 : 0u) | (tc.iy0 ? 1u << 18 : 0u) |
             (tc.iy1 ? 1u << 19 : 0u) | (sv0 - lv0) << 20 | (sv1 - lv1) << 23;
}

// Same taps, validity and conversions as gather_taps_frame (device_common.hpp), without vignette.
__device__ __forceinline__ void feed_taps_finish(const FeedRaw& r, Taps& t) {
    const uint32_t m = r.meta;
    const uint32_t sy = (r.sel & 0xFFFFu) | 0x0C0C0000u, sc = (r.sel >> 16) | 0x0C0C0000u;
    const uint32_t sv0 = sc + ((m >> 20) & 7u) * 0x0101u, sv1 = sc + ((m >> 23) & 7u) * 0x0101u;
    // two tap bytes of each row segment in bytes 0, 1
    const uint32_t Y0 = __builtin_amdgcn_perm(r.y0.y, r.y0.x, sy), Y1 = __builtin_amdgcn_perm(r.y1.y, r.y1.x, sy);
    const uint32_t U0 = __builtin_amdgcn_perm(r.u0.y, r.u0.x, sc), U1 = __builtin_amdgcn_perm(r.u1.y, r.u1.x, sc);
    const uint32_t V0 = __builtin_amdgcn_perm(r.v0.y, r.v0.x, sv0), V1 = __builtin_amdgcn_perm(r.v1.y, r.v1.x, sv1);
    uint32_t ca, cb, cc, cd;
    yuv_pair_to_rgba(Y0, U0, V0, ca, cb);
    yuv_pair_to_rgba(Y1, U1, V1, cc, cd);
    const bool valid = (m & 0x8000u) != 0;
    const bool ix0 = (m >> 16) & 1u, ix1 = (m >> 17) & 1u, iy0 = (m >> 18) & 1u, iy1 = (m >> 19) & 1u;
    t.c[0] = (valid && ix0 && iy0) ? ca : 0u;
    t.c[1] = (valid && ix1 && iy0) ? cb : 0u;
    t.c[2] = (valid && ix0 && iy1) ? cc : 0u;
    t.c[3] = (valid && ix1 && iy1) ? cd : 0u;
    t.fx = m & 31u;
    t.fy = (m >> 5) & 31u;
}

// LEAN = false: every sample's gathers in flight at once (kGainPer samples per lane) and the register
// LU (163 VGPRs: the shortest feed on an idle GPU).  LEAN = true: kLeanBatch samples per lane per
// round, partner sums in LDS, the workgroup LU above n = 3 (<= 80 VGPRs), so the feed of frame k+1
// fits beside frame k's composite (6 workgroups per CU at 72 VGPRs / 96 SGPRs / 20.7 KiB LDS) and runs
// under it.  Both sum the same exact values: identical gains.
constexpr int kLeanBatch = 3;  // lean feed: samples per lane in flight per round
// The sample's warped pixel (RGB) from its taps: cv::remap's fixed-point bilinear, or the texture filter of
// the texture-convention mode (tex, uniform)
__device__ __forceinline__ void sample_rgb(const Taps& t, int tex, uint32_t (&rgb)[3]) {
    if (tex)
        tex_bilerp(t.c[0], t.c[1], t.c[2], t.c[3], t.fx, t.fy, rgb);
    else
        bilerp_rgba(t.c[0], t.c[1], t.c[2], t.c[3], t.fx, t.fy, rgb);
}

// The feed's FIRST argument (FeedBatch): camera c of frame f read from the kernarg segment (scalar loads)
typedef __attribute__((address_space(4))) const SourceFrame kSourceFrame;
static_assert(offsetof(FeedBatch<1>, src) == 0 && offsetof(FeedBatch<4>, src) == 0, "FeedBatch layout");

template <bool LEAN, int NF>
__device__ __forceinline__ void gain_feed_body(const CompositeEntry* samples, const uint16_t* partners, int tex,
                                               int n_chunks, const int32_t* N, int n) {
    typedef __attribute__((address_space(4))) const FeedBatch<NF> kFeedBatch;
    __shared__ int s_last;
    __shared__ double s_I[kGainMaxCams * kGainMaxCams];
    __shared__ double s_A[kGainMaxCams * kGainMaxCams];
    __shared__ double s_b[kGainMaxCams];
    __shared__ double s_x[kGainMaxCams];
    const int tid = threadIdx.x, lane = tid & 63;
    // Wave w of workgroup b takes the kGainWaveRun contiguous samples from (4 b + w) kGainWaveRun: one
    // camera's (runs padded on the host with invalid samples, partner mask 0), named in every entry's
    // code.  Every norm is 0 or a multiple of 2^-23 in [1, 2^9), so the f64 sums below are exact in any order.
    constexpr int kPer = kGainPer;
    const int wave = tid >> 6;
    __shared__ double s_wsum[4][kGainMaxCams];
    __shared__ int s_wcam[4];
    // workgroup b: frame b / n_chunks of the batch (FeedBatch), chunk cb of it
    const kFeedBatch* kb = (const kFeedBatch*)__builtin_amdgcn_kernarg_segment_ptr();
    const int frame = uniform((int)(blockIdx.x / (uint32_t)n_chunks)), cb = (int)blockIdx.x - frame * n_chunks;
    unsigned long long* const totals = kb->totals[frame];
    uint32_t* const tickets = kb->tickets[frame];
    double* const gains = kb->gains[frame];
    const int k0 = (cb * 4 + wave) * kGainWaveRun + lane;
    const int cam = uniform((int)((samples[(cb * 4 + wave) * kGainWaveRun].code >> 10) & 15u));
    SourceFrame fr;  // one camera per wave: uniform frame
    {
        const kSourceFrame& kf = kb->src[frame * kGainMaxCams + cam];
        fr.yuv = kf.yuv;
        fr.w = kf.w;
        fr.h = kf.h;
        fr.pitch = kf.pitch;
        fr.vig = kf.vig;
    }
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint8_t*>(fr.yuv), 0, (int)((uint32_t)fr.pitch * (uint32_t)(fr.h + fr.h / 2)), 0x00020000);
    if constexpr (LEAN) {
        // one sample per lane at a time; per partner a wave sum added into the wave's LDS row
        // (kLeanBatch samples per lane in flight per round)
        if (lane < kGainMaxCams) s_wsum[wave][lane] = 0.0;
        static_assert(kPer % kLeanBatch == 0, "lean feed batches");
#pragma unroll 1
        for (int u0 = 0; u0 < kPer; u0 += kLeanBatch) {
            CompositeEntry e[kLeanBatch];
            uint32_t pm[kLeanBatch];
#pragma unroll
            for (int u = 0; u < kLeanBatch; u++) {
                e[u] = samples[k0 + (u0 + u) * 64];
                pm[u] = partners[k0 + (u0 + u) * 64];
            }
            Taps t[kLeanBatch];
            if (fr.vig || tex) {  // vignette / clamped texture taps: per-tap byte gathers
#pragma unroll
                for (int u = 0; u < kLeanBatch; u++) gather_taps_frame(fr, e[u].xy, e[u].code, t[u]);
            } else {
                FeedRaw raw[kLeanBatch];
#pragma unroll
                for (int u = 0; u < kLeanBatch; u++) feed_taps_issue(rs, fr, e[u].xy, e[u].code, raw[u]);
#pragma unroll
                for (int u = 0; u < kLeanBatch; u++) feed_taps_finish(raw[u], t[u]);
            }
            double nv[kLeanBatch];
            uint32_t pm_any = 0u;
#pragma unroll
            for (int u = 0; u < kLeanBatch; u++) {
                uint32_t rgb[3];
                sample_rgb(t[u], tex, rgb);
                nv[u] = (double)sqrtf((float)(rgb[0] * rgb[0] + rgb[1] * rgb[1] + rgb[2] * rgb[2]));
                pm_any |= pm[u];
            }
            // partners present in this wave's batch (wave-uniform): one wave sum each
            uint32_t jm = 0u;
            for (int j = 0; j < n; j++) jm |= __ballot((pm_any >> j) & 1u) ? 1u << j : 0u;
#pragma unroll 1
            while (jm) {
                const int j = __builtin_ctz(jm);
                jm &= jm - 1;
                double v = 0.0;
#pragma unroll
                for (int u = 0; u < kLeanBatch; u++) v += ((pm[u] >> j) & 1u) ? nv[u] : 0.0;
                v = wave_sum(v);
                if (lane == 0) s_wsum[wave][j] += v;
            }
        }
    } else {
        // kGainPer samples per lane, all gathers issued before any arithmetic
        double acc[kGainMaxCams];
#pragma unroll
        for (int j = 0; j < kGainMaxCams; j++) acc[j] = 0.0;
        uint32_t pm[kPer];
        Taps t[kPer];
        CompositeEntry es[kPer];
#pragma unroll
        for (int u = 0; u < kPer; u++) {
            es[u] = samples[k0 + u * 64];
            pm[u] = partners[k0 + u * 64];
        }
        if (fr.vig || tex) {  // vignette / clamped texture taps: per-tap byte gathers
#pragma unroll
            for (int u = 0; u < kPer; u++) gather_taps_frame(fr, es[u].xy, es[u].code, t[u]);
        } else {
            FeedRaw raw[kPer];
#pragma unroll
            for (int u = 0; u < kPer; u++) feed_taps_issue(rs, fr, es[u].xy, es[u].code, raw[u]);
#pragma unroll
            for (int u = 0; u < kPer; u++) feed_taps_finish(raw[u], t[u]);
        }
#pragma unroll
        for (int u = 0; u < kPer; u++) {
            uint32_t rgb[3];
            sample_rgb(t[u], tex, rgb);
            const double nv = (double)sqrtf((float)(rgb[0] * rgb[0] + rgb[1] * rgb[1] + rgb[2] * rgb[2]));
#pragma unroll
            for (int j = 0; j < kGainMaxCams; j++)
                if (pm[u] & (1u << j)) acc[j] += nv;
        }
        // exact sums: per wave (DPP)
#pragma unroll
        for (int j = 0; j < kGainMaxCams; j++) {  // unrolled: the n reductions' DPP chains interleave
            if (j < n) {
                const double v = wave_sum(acc[j]);
                if (lane == 0) s_wsum[wave][j] = v;
            }
        }
    }
    // then per (camera, partner) over the workgroup's waves, then one u64 atomic per pair
    if (lane == 0) s_wcam[wave] = cam;
    __syncthreads();
    if (tid < 4 * n) {  // (wave w, partner j); the first wave of each camera adds for all its waves
        const int w = tid / n, j = tid - w * n, c = s_wcam[w];
        bool first = true;
        for (int x = 0; x < w; x++) first &= s_wcam[x] != c;
        if (first) {
            double v = 0.0;
            for (int x = w; x < 4; x++)
                if (s_wcam[x] == c) v += s_wsum[x][j];
            if (v != 0.0)
                __hip_atomic_fetch_add(&totals[(c * kGainMaxCams + j) * kGainTotalStride],
                                       (unsigned long long)(v * 8388608.0), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    // every wave's adds have completed before the workgroup takes its ticket
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
        // the frame's tickets sharded by chunk (cb & 7: mostly one shard per XCD under round-robin dispatch)
        const int xcd = cb & 7;
        const uint32_t in_xcd = (uint32_t)((n_chunks - xcd + 7) >> 3);
        int last = 0;
        if (__hip_atomic_fetch_add(&tickets[xcd], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == in_xcd - 1) {
            const uint32_t groups = (uint32_t)min(n_chunks, 8);
            last = __hip_atomic_fetch_add(&tickets[8], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == groups - 1;
        }
        s_last = last;
    }
    __syncthreads();
    if (!s_last) return;
    // ---- the last workgroup ------------------------------------------------------------------
    __shared__ int32_t s_N[kGainMaxCams * kGainMaxCams];
    if (tid < n * n) {
        const int i = tid / n, j = tid - i * n;
        const int32_t Nij = N[tid];
        s_N[tid] = Nij;
        const unsigned long long raw =
            __hip_atomic_exchange(&totals[(i * kGainMaxCams + j) * kGainTotalStride], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_I[tid] = (i != j) ? ((double)raw * 0x1p-23) / Nij : 0.0;
    }
    if (tid < 9) __hip_atomic_exchange(&tickets[tid], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    if (tid < n) gain_system_row(s_I, s_N, n, tid, s_A, s_b);
    __syncthreads();
    // cv::solve (lapack.cpp:1050-1275): one lane with the matrix in registers for n <= 8 (closed forms
    // n <= 3); the LU across the workgroup for 9..16
    bool ok;
    if (LEAN && n > 3) {  // the register LU would set the lean kernel's VGPR budget
        ok = lu_solve_block(s_A, s_b, n, s_x);
    } else if (LEAN || n < kLuBlockMin || n <= 3) {
        if (tid == 0) s_last = (LEAN ? solve_small(s_A, s_b, n, s_x) : solve_dispatch(s_A, s_b, n, s_x)) ? 1 : 0;
        __syncthreads();
        ok = s_last != 0;
    } else {
        ok = lu_solve_block(s_A, s_b, n, s_x);
    }
    if (tid < n) gains[tid] = ok ? s_x[tid] : 1.0;  // cv::solve failure leaves gains_ unspecified; 1 as the oracle
}

template <int NF>
__global__ void __launch_bounds__(256) gain_feed_kernel(FeedBatch<NF> batch, const CompositeEntry* samples,
                                                        const uint16_t* partners, int tex, int n_chunks, const int32_t* N,
                                                        int n) {
    (void)batch;  // read through the kernarg segment (kFeedBatch)
    gain_feed_body<false, NF>(samples, partners, tex, n_chunks, N, n);
}
template <int NF>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_num_vgpr(80)))
gain_feed_lean_kernel(FeedBatch<NF> batch, const CompositeEntry* samples, const uint16_t* partners, int tex, int n_chunks,
                      const int32_t* N, int n) {
    (void)batch;
    gain_feed_body<true, NF>(samples, partners, tex, n_chunks, N, n);
}

template <int NF>
static void launch_feed_nf(const FrameSet* frames, const CompositeEntry* samples, const uint16_t* partners, int tex,
                           int n_chunks, const int32_t* N, int n, unsigned long long* const* totals,
                           uint32_t* const* tickets, double* const* gains, hipStream_t s, bool lean) {
    FeedBatch<NF> fb;
    memset(&fb, 0, sizeof fb);
    for (int f = 0; f < NF; f++) {
        for (int i = 0; i < kGainMaxCams; i++) fb.src[f * kGainMaxCams + i] = frames[f].f[i];
        fb.totals[f] = totals[f];
        fb.tickets[f] = tickets[f];
        fb.gains[f] = gains[f];
    }
    if (lean)
        hipLaunchKernelGGL(gain_feed_lean_kernel<NF>, dim3(n_chunks * NF), dim3(256), 0, s, fb, samples, partners, tex,
                           n_chunks, N, n);
    else
        hipLaunchKernelGGL(gain_feed_kernel<NF>, dim3(n_chunks * NF), dim3(256), 0, s, fb, samples, partners, tex,
                           n_chunks, N, n);
}

hipError_t launch_gain_feed_batch(const FrameSet* frames, int nf, const CompositeEntry* samples, const uint16_t* partners,
                                  int tex, int n_chunks, const int32_t* N, int n, unsigned long long* const* totals,
                                  uint32_t* const* tickets, double* const* gains, hipStream_t s, bool lean) {
    if (n_chunks <= 0 || n > kGainMaxCams) return hipErrorInvalidValue;
    if (nf == 1)
        launch_feed_nf<1>(frames, samples, partners, tex, n_chunks, N, n, totals, tickets, gains, s, lean);
    else if (nf == 2)
        launch_feed_nf<2>(frames, samples, partners, tex, n_chunks, N, n, totals, tickets, gains, s, lean);
    else if (nf == 4)
        launch_feed_nf<4>(frames, samples, partners, tex, n_chunks, N, n, totals, tickets, gains, s, lean);
    else
        return hipErrorInvalidValue;
    return hipGetLastError();
}

hipError_t launch_gain_feed(const FrameSet& frames, const CompositeEntry* samples, const uint16_t* partners, int tex,
                            int n_chunks, const int32_t* N, int n,
                            unsigned long long* totals, uint32_t* tickets, double* gains, hipStream_t s, bool lean) {
    return launch_gain_feed_batch(&frames, 1, samples, partners, tex, n_chunks, N, n, &totals, &tickets, &gains, s, lean);
}

struct GainArgs {
    double g[kMaxCams];
};
__global__ void set_gains_kernel(GainArgs a, int n, double* gains) {
    if ((int)threadIdx.x < n) gains[threadIdx.x] = a.g[threadIdx.x];
}

hipError_t launch_set_gains(const double* host_gains, int n, double* gains_dev, hipStream_t s) {
    GainArgs a;
    for (int i = 0; i < kMaxCams; i++) a.g[i] = i < n ? host_gains[i] : 1.0;
    hipLaunchKernelGGL(set_gains_kernel, dim3(1), dim3(64), 0, s, a, n, gains_dev);
    return hipGetLastError();
}

// One workgroup per footprint run: its packed bytes into the camera's frame (byte stores of consecutive
// lanes: whole-line writes per wave).
__global__ void __launch_bounds__(256) unpack_runs_kernel(const uint8_t* packed, const FootRun* runs, FootFrames fr) {
    const FootRun r = runs[blockIdx.x];
    const int cam = (int)(r.cam & 31u), rp = (int)(r.cam >> 8);
    const int w = fr.w[cam], h = fr.h[cam];
    const int x0 = 8 * (int)r.g0, yb = min(8 * (int)(r.g0 + r.ng), w) - x0;
    const int c0 = 4 * (int)r.g0, cb = max(0, min(4 * (int)(r.g0 + r.ng), w / 2) - c0);
    const uint8_t* src = packed + r.off;
    uint8_t* const f = fr.f[cam];
    uint8_t* const d0 = f + (size_t)(2 * rp) * (size_t)w + x0;
    uint8_t* const d1 = d0 + w;
    uint8_t* const du = f + (size_t)(h + rp) * (size_t)w + c0;
    uint8_t* const dv = du + w / 2;
    const int tot = 2 * yb + 2 * cb;
    for (int k = threadIdx.x; k < tot; k += 256) {
        uint8_t* d = k < yb ? d0 + k : k < 2 * yb ? d1 + (k - yb) : k < 2 * yb + cb ? du + (k - 2 * yb) : dv + (k - 2 * yb - cb);
        *d = src[k];
    }
}

hipError_t launch_unpack_runs(const uint8_t* packed, const FootRun* runs, int n_runs, const FootFrames& frames,
                              hipStream_t s) {
    if (n_runs <= 0) return hipSuccess;
    hipLaunchKernelGGL(unpack_runs_kernel, dim3(n_runs), dim3(256), 0, s, packed, runs, frames);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// Per-frame stitch, blend = 0 (mapper.cpp:219-306 with the copy chain resolved into the tiled LUT):
// for every 2x2 output quad the winning camera of each pixel is sampled (15-bit bilinear on the
// RGBA the source converts to), gain-scaled (mul_scalar_with_mask, exposure_compensate.cu:15-30:
// saturate_cast<uchar>(px * (float)g)) and written as YUV420P (the library's own BT.601 in place of
// NPP RGBToYUV420, same sequence as oracle rgb_quad_to_yuv).
// One workgroup per 128x8 tile; staged tiles read every tap from LDS (see kernels.hpp).  Tiles are
// walked grid-stride; blocks b, b+8, ... (one XCD under round-robin dispatch) take a contiguous
// band of tiles so their source boxes share that XCD's L2.
// ---------------------------------------------------------------------------------------------
static_assert(sizeof(TileSlot) == 16, "TileSlot layout");

// The per-call FrameBatch is the FIRST argument of the stitch kernels: index it in the kernarg
// segment directly (a wave-uniform index gives scalar loads; indexing the by-value parameter would
// copy it to scratch).  idx = (frame << cam_log2) + camera (kernels.hpp FrameBatch).
typedef __attribute__((address_space(4))) const SourceFrame kSourceFrame;
static_assert(offsetof(FrameBatch<1>, src) == 0 && offsetof(FrameBatch<4>, src) == 0, "FrameBatch layout");
__device__ __forceinline__ SourceFrame kernarg_frame(uint32_t idx) {
    const kSourceFrame* kf = (const kSourceFrame*)__builtin_amdgcn_kernarg_segment_ptr();
    SourceFrame s;
    s.yuv = kf[idx].yuv;
    s.w = kf[idx].w;
    s.h = kf[idx].h;
    s.pitch = kf[idx].pitch;
    s.vig = kf[idx].vig;
    return s;
}
template <int NF>
__device__ __forceinline__ uint8_t* kernarg_out(uint32_t f) {
    typedef __attribute__((address_space(4))) const FrameBatch<NF> kFrameBatch;
    return ((const kFrameBatch*)__builtin_amdgcn_kernarg_segment_ptr())->out[f];
}
template <int NF>
__device__ __forceinline__ const double* kernarg_gains(uint32_t f) {
    typedef __attribute__((address_space(4))) const FrameBatch<NF> kFrameBatch;
    return ((const kFrameBatch*)__builtin_amdgcn_kernarg_segment_ptr())->gains[f];
}

// One 8-pixel staging group of a tile: the YUV bytes it needs and its LDS destination.
struct StageGroup {
    uint32_t y0, y1;  // 8 Y bytes
    uint32_t uq, vq;  // 4 U bytes, 4 V bytes
    int32_t dst;      // dword index of the group's first RGBA pixel; -1 = none
    uint32_t flags;   // kStageBlack: box group outside the image; kStageNoVig: camera without vignette
    float4 g0, g1;    // VIG: vignette gains of the 8 pixels
};
// The loaded bytes are only touched in stage_store (an iteration later): a select on them right
// after the load would make the compiler wait for the load in the iteration that issues it.
constexpr uint32_t kStageBlack = 1u, kStageNoVig = 2u;

// Metadata of a staged item as the waves hold it: one 16-byte load by 5 lanes (lane 0 the TileHdr,
// lane 1 + q slot q's TileSlot), decoded with v_readlane on demand (a uniform lane index), so the
// slot descriptors never occupy scalar registers.
// Slot q, component j of lane 1 + q: 0 = cam | bw << 16, 1 = bh | lds << 16, 2 = bx0 | by0 << 16,
// 3 = chunk0.
struct TileMeta {
    int t;         // the work unit: item t >> nf_log2, frame t & (nf - 1) (FrameBatch)
    uint4 v;
    uint32_t tile, nslots, stride;
    uint32_t map;  // slot of staging chunk c < 4 in bits 2c, 2c + 1 (TiledLutDev::upload)
    uint32_t frame, fbase;  // the unit's frame and its first camera's FrameBatch index (frame << cam_log2)
};

// dword j (0-3) of slot q (wave-uniform)
__device__ __forceinline__ uint32_t slot_word(const TileMeta& m, int q, int j) {
    const uint32_t c = j == 0 ? m.v.x : j == 1 ? m.v.y : j == 2 ? m.v.z : m.v.w;
    return (uint32_t)__builtin_amdgcn_readlane((int)c, 1 + q);
}

// The slot of staging chunk c (wave-uniform) and the frame it reads, resolved with scalar work and
// scalar kernarg loads; done one phase before the vector loads that use it, so their latency hides.
struct StageSlot {
    uint32_t live;             // c is a chunk of a live item
    uint32_t cam, bw, bh, lds, bx0, by0, chunk0;
    SourceFrame f;
};

// FIRST: c < 4 (a wave's first chunk), whose slot the host stored in m.map; else searched.
template <bool FIRST = false>
__device__ __forceinline__ StageSlot stage_slot(const TileMeta& m, int t_end, int c) {
    StageSlot s;
    const uint32_t nchunks = m.t < t_end ? ((m.nslots >> 8) & 0xFFu) : 0u;
    s.live = (uint32_t)c < nchunks ? 1u : 0u;
    int q = 0;
    if constexpr (FIRST) {
        q = (int)((m.map >> (2 * c)) & 3u);
    } else {
        const int nslots = (int)(m.nslots & 0xFFu);
#pragma unroll
        for (int j = 1; j < kTileSlots; j++) q += (j < nslots && c >= (int)(slot_word(m, j, 3) & 0xFFFFu)) ? 1 : 0;
    }
    const uint32_t d0 = slot_word(m, q, 0), d1 = slot_word(m, q, 1);
    const uint32_t d2 = slot_word(m, q, 2), d3 = slot_word(m, q, 3);
    s.cam = s.live ? (d0 & 31u) : 0u;
    s.bw = d0 >> 16;
    s.bh = d1 & 0xFFFFu;
    s.lds = d1 >> 16;
    s.bx0 = d2 & 0xFFFFu;
    s.by0 = d2 >> 16;
    s.chunk0 = d3 & 0xFFFFu;
    s.f = kernarg_frame(m.fbase + s.cam);
    return s;
}

// Loads of one staging group of 8 luma pixels of a slot: g is the lane's u16 group (kernels.hpp: valid,
// column and row in the slot's box, from the item's group table), so a chunk of 64 lanes covers only the
// box rows' tap spans.  Invalid groups (a slot's last chunk, chunks past the item's) read the box origin
// and are marked dst = -1.  With box columns 8-aligned, the Y load is 8-byte and the U / V loads 4-byte
// aligned (DWORD_STAGE).  Offsets use 24-bit multiplies: rows < 256, pitch < 2^24 (checked on the host).
template <bool DWORD_STAGE, bool VIG>
__device__ __forceinline__ void stage_load(const StageSlot& s, uint32_t stride, uint32_t g, StageGroup& sg) {
    const bool ok = s.live && (g & kGroupValid) != 0u;
    const uint32_t row_k = ok ? (g & 255u) : 0u, col_k = ok ? (g >> 8) & 31u : 0u;
    const SourceFrame& f = s.f;
    // box groups past the image's right / bottom edge (w % 8 == 0: whole groups) stage RGBA 0:
    // they load from the box origin and are replaced by Y = 0, U = V = 128 (-> R = G = B = 0)
    const bool img = s.bx0 + col_k * 8u < (uint32_t)f.w && s.by0 + row_k < (uint32_t)f.h;
    const uint32_t row = img ? row_k : 0u, col = img ? col_k : 0u;
    const uint32_t p32 = (uint32_t)f.pitch;
    const gu8* base = (const gu8*)f.yuv;
    const gu8* Yb = base + (int64_t)s.by0 * f.pitch + s.bx0;  // by0, bx0 even: chroma rows / columns exact
    const gu8* Ub = base + (int64_t)(f.h + (int)(s.by0 >> 1)) * f.pitch + (s.bx0 >> 1);
    const gu8* Vb = Ub + (f.w >> 1);
    const uint32_t oy = __umul24(row, p32) + col * 8u, oc = __umul24(row >> 1, p32) + col * 4u;
    if (DWORD_STAGE) {
        const uint64_t yy = *(const gu64*)(Yb + oy);
        sg.y0 = (uint32_t)yy;
        sg.y1 = (uint32_t)(yy >> 32);
        sg.uq = *(const gu32*)(Ub + oc);
        sg.vq = *(const gu32*)(Vb + oc);
    } else {
        const gu8* Yp = Yb + oy;
        const gu8* Up = Ub + oc;
        const gu8* Vp = Vb + oc;
        sg.y0 = (uint32_t)Yp[0] | ((uint32_t)Yp[1] << 8) | ((uint32_t)Yp[2] << 16) | ((uint32_t)Yp[3] << 24);
        sg.y1 = (uint32_t)Yp[4] | ((uint32_t)Yp[5] << 8) | ((uint32_t)Yp[6] << 16) | ((uint32_t)Yp[7] << 24);
        sg.uq = (uint32_t)Up[0] | ((uint32_t)Up[1] << 8) | ((uint32_t)Up[2] << 16) | ((uint32_t)Up[3] << 24);
        sg.vq = (uint32_t)Vp[0] | ((uint32_t)Vp[1] << 8) | ((uint32_t)Vp[2] << 16) | ((uint32_t)Vp[3] << 24);
    }
    sg.flags = img ? 0u : kStageBlack;
    sg.dst = ok ? (int32_t)(s.lds + __umul24(row_k, stride) + col_k * 8u) : -1;
    if (VIG) {  // 8 gains (32-byte aligned: w % 8 == 0); a camera without vignette uses 1.0 gains
        const float* gv = f.vig ? f.vig + (int64_t)(s.by0 + row) * f.w + s.bx0 + col * 8u
                                : reinterpret_cast<const float*>(f.yuv);  // any readable 32 B, unused
        sg.g0 = *reinterpret_cast<const float4*>(gv);
        sg.g1 = *reinterpret_cast<const float4*>(gv + 4);
        if (!f.vig) sg.flags |= kStageNoVig;
    }
}

// The lane's group of an item's chunk c < kGroupFirst (c = the wave: each wave's first chunk), addressed
// by the item index alone (loop-invariant voffset, scalar soffset), so it is loaded one iteration ahead
// with the item's metadata.  Carried across the loop as the u16 the load returns: as a u32 the compiler
// zero-extended it right after the load, into the loop-carried register, and that copy waited on every
// load of the iteration (vmcnt(0) before the compute); widened at the use, an iteration later, it waits
// on nothing (one frame in flight: C2 composite -1 %, C3 +1 %, `u16`).
__device__ __forceinline__ uint16_t group_issue(const __amdgpu_buffer_rsrc_t& gr, int t, int t_end, int lg) {
    const int tt = (t < t_end ? t : 0) >> lg;
    return __builtin_amdgcn_raw_buffer_load_b16(gr, (uint32_t)threadIdx.x * 2u,
                                                (uint32_t)uniform(tt) * (uint32_t)(kGroupFirst * 64 * 2), 0);
}

template <bool VIG>
__device__ __forceinline__ void stage_store(const StageGroup& sg, uint32_t* s_rgb) {
    if (sg.dst < 0) return;
    const bool black = (sg.flags & kStageBlack) != 0;  // Y = 0, U = V = 128 -> RGBA 0
    const uint32_t y0 = black ? 0u : sg.y0, y1 = black ? 0u : sg.y1;
    // chroma bytes xor 0x80 read as signed bytes are u - 128: one v_cvt_f32_i32_sdwa (sext) each
    const uint32_t uq = black ? 0u : sg.uq ^ 0x80808080u, vq = black ? 0u : sg.vq ^ 0x80808080u;
    auto ch = [](uint32_t w, int k) { return (float)(signed char)((w >> (8 * k)) & 255u); };
    uint4 a, b;
    yuv2_to_rgba_c(y0 & 255u, (y0 >> 8) & 255u, ch(uq, 0), ch(vq, 0), a.x, a.y);
    yuv2_to_rgba_c((y0 >> 16) & 255u, y0 >> 24, ch(uq, 1), ch(vq, 1), a.z, a.w);
    yuv2_to_rgba_c(y1 & 255u, (y1 >> 8) & 255u, ch(uq, 2), ch(vq, 2), b.x, b.y);
    yuv2_to_rgba_c((y1 >> 16) & 255u, y1 >> 24, ch(uq, 3), ch(vq, 3), b.z, b.w);
    if (VIG && !(sg.flags & kStageNoVig)) {
        a.x = vig_mul(a.x, sg.g0.x);
        a.y = vig_mul(a.y, sg.g0.y);
        a.z = vig_mul(a.z, sg.g0.z);
        a.w = vig_mul(a.w, sg.g0.w);
        b.x = vig_mul(b.x, sg.g1.x);
        b.y = vig_mul(b.y, sg.g1.y);
        b.z = vig_mul(b.z, sg.g1.z);
        b.w = vig_mul(b.w, sg.g1.w);
    }
    *reinterpret_cast<uint4*>(s_rgb + sg.dst) = a;
    *reinterpret_cast<uint4*>(s_rgb + sg.dst + 4) = b;
}

// Residency and register budget of the composite: 6 workgroups per CU (the grid is one resident wave
// of them), compiled with the registers of 7 (72 VGPRs, 96 SGPRs; residency of 256-thread workgroups is
// also capped by scalar registers, min(8, 800 / (sgpr16 + 16)), MI355X_MICROARCH.md, Residency), so each
// SIMD keeps 80 VGPRs / 96 SGPRs and a wave slot for one wave of the lean gain feed beside 6 composite
// waves: the next frame's feed runs under this frame's composite (frames in flight).  Set explicitly:
// with the weight table the compiler's LDS occupancy model (24 KiB per workgroup) would otherwise relax
// the budget to 5 waves' 102 VGPRs.
constexpr int kStitchBlocksPerCU = 6;
constexpr int kStitchRegBlocks = kStitchBlocksPerCU + 1;
constexpr int kStitchSgprs = 96, kStitchVgprs = 72;
// The texture-convention instance (its f32 filter holds ~20 more values per pixel): the registers of 5
// workgroups per CU instead of spilling at 72 (the composite's time does not depend on 4, 5 or 6
// workgroups per CU, §4 Round 5)
constexpr int kStitchTexRegBlocks = 5, kStitchTexVgprs = 96;

// Software pipeline over a workgroup's items (t, then the items it claims):
//   iteration of item t:  stage item t's YUV (loaded during the previous iteration) into LDS,
//                         read the next item's metadata (loaded one iteration earlier),
//                         store the previous item's output, issue the next item's entries + YUV loads and
//                         the metadata load of the item after it,
//                         then compute item t from LDS while all of those are in flight.
// No global load is waited on in the iteration that issues it, and every iteration issues the
// same vector-memory operations in the same order (clamped addresses instead of branches), so the
// compiler's wait counts stay exact across the loop.
//
// One buffer load by lanes 0..kMetaWords-1: the voffset (lane * 16) is loop-invariant, the item's
// record offset a scalar, so no per-lane 64-bit address is held across the loop.
__device__ __forceinline__ uint4 meta_issue(const __amdgpu_buffer_rsrc_t& mr, int t, int t_end, int lg) {  // t: unit
    const int lane = threadIdx.x & 63;
    const int tt = (t < t_end ? t : 0) >> lg;  // t >= 0: every item index derives from bounded claims
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    uint4 v;
    if (lane < kMetaWords) {  // exec-masked: the instruction (and its vmcnt) is the same for every wave
        const u32x4 r = __builtin_amdgcn_raw_buffer_load_b128(mr, (uint32_t)lane * 16u,
                                                              (uint32_t)uniform(tt) * (uint32_t)(kMetaWords * 16), 0);
        v = uint4{r.x, r.y, r.z, r.w};
    }
    return v;
}

__device__ __forceinline__ TileMeta meta_read(const uint4& v, int t, int lg, int cam_lg) {
    TileMeta m;
    m.t = t;
    m.frame = (uint32_t)t & ((1u << lg) - 1u);
    m.fbase = m.frame << cam_lg;
    m.v = v;
    m.tile = (uint32_t)__builtin_amdgcn_readlane((int)v.x, 0);
    m.nslots = (uint32_t)__builtin_amdgcn_readlane((int)v.y, 0);
    m.stride = (uint32_t)__builtin_amdgcn_readlane((int)v.w, 0);
    m.map = (uint32_t)__builtin_amdgcn_readlane((int)v.z, 0);
    return m;
}

// An item's in-flight loads: its entries (one uint4 = one quad per lane and half) and the staging
// group of the wave's first chunk.
struct TileData {
    uint4 e4[kItemHalves];
    StageGroup sg;
};

// Issue an item's entry loads and the staging loads of its first chunk per wave (sl: the slot of
// chunk `wave`, from stage_slot<true>; g: the lane's group of that chunk, from group_issue).
// er: the entries as a buffer resource — voffset = lane * 16 (loop-invariant), soffset = the item's
// scalar byte offset, so no per-lane 64-bit address is formed per item (TiledLutDev::upload checks
// that the entries fit 32-bit offsets)
// E24: the lane's four 24-bit entries of each half (tiled_entry24) as three dwords (d.e4[h].w unused)
template <bool DWORD_STAGE, bool VIG, bool E24>
__device__ __forceinline__ void data_issue(const __amdgpu_buffer_rsrc_t& er, const TileMeta& m, int t_end, int lg,
                                           const StageSlot& sl, uint32_t g, TileData& d) {
    const bool live = m.t < t_end;
    const int tid = threadIdx.x;
#pragma unroll
    for (int h = 0; h < kItemHalves; h++) {
        const uint32_t so =
            (uint32_t)uniform(((live ? m.t : 0) >> lg) * kItemHalves + h) * (uint32_t)(kTilePx * (E24 ? 3 : 4));
        if constexpr (E24) {
            typedef unsigned int u32x3e __attribute__((ext_vector_type(3)));
            const u32x3e v = __builtin_amdgcn_raw_buffer_load_b96(er, (uint32_t)tid * 12u, so, 0);
            d.e4[h] = uint4{v.x, v.y, v.z, 0u};
        } else {
            typedef unsigned int u32x4e __attribute__((ext_vector_type(4)));
            const u32x4e v = __builtin_amdgcn_raw_buffer_load_b128(er, (uint32_t)tid * 16u, so, 0);
            d.e4[h] = uint4{v.x, v.y, v.z, v.w};
        }
    }
    if (!sl.live) {  // wave-uniform: no loads for a chunk the item lacks
        d.sg.dst = -1;
        return;
    }
    stage_load<DWORD_STAGE, VIG>(sl, m.stride & ((1u << kStrideBits) - 1u), g, d.sg);
}

// The composite's two sinks.  MODE 0: gain + RGB -> YUV420P into the output frame (blend = 0).
// MODE 1: gain-applied RGBA into the camera's level-0 pyramid image (blend > 0; the warped image
// Mapper::stitch hands to the blender, mapper.cpp:233-262); pixels outside the camera's aligned ROI
// are dropped.  Either way a quad's result is 4 dwords.
template <int MODE>
__device__ __forceinline__ QuadOut finish_any(const float (&rgb)[4][3], const f32x2_t (&gain)[4]) {
    if constexpr (MODE == 0) {
        return finish_quad2f(rgb, gain);
    } else {
        uint32_t px[4];
#pragma unroll
        for (int p = 0; p < 4; p++) {
            uint32_t v = pack_u8(rgb[p][0] * gain[p].x, 0, 0u);
            v = pack_u8(rgb[p][1] * gain[p].x, 1, v);
            px[p] = pack_u8(rgb[p][2] * gain[p].x, 2, v);
        }
        return QuadOut{px[0], px[1], px[2], px[3]};
    }
}

struct RgbaSink {
    __amdgpu_buffer_rsrc_t rsrc;
    const MbCamLevel* cams;
};

// MODE 1: the deep tiles' result frame as an OutFrame from the level-0 grid origin (RgbaOut::res), in
// the registers MODE 0's output frame takes
__device__ __forceinline__ OutFrame make_result_frame(const RgbaOut& r) {
    OutFrame o;
    o.rsrc = __builtin_amdgcn_make_buffer_rsrc(r.res, 0, (int)r.res_bytes, 0x00020000);
    o.pitch = r.res_pitch;
    o.u_off = r.res_u_off;
    o.v_off = r.res_v_off;
    return o;
}

// A deep level-0 quad's final result straight from the remap (mb_blend level 0 for owned = 4: R = G0,
// convertTo(CV_8UC3) into result(align_result_roi) and RGB -> YUV420P, or the RGBA result image of a
// scaled output).  q holds the quad's four packed RGB pixels; (x, y): the quad on the level-0 grid.
__device__ __forceinline__ void store_result(const OutFrame& o, bool rgba, const QuadOut& q, int x, int y, bool in) {
    if (rgba) {
        typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
        const uint32_t off = in ? (uint32_t)y * o.pitch + (uint32_t)x * 4u : kDropOffset;
        __builtin_amdgcn_raw_buffer_store_b64(u32x2{q.y01, q.y23}, o.rsrc, off, 0, 0);
        __builtin_amdgcn_raw_buffer_store_b64(u32x2{q.u, q.v}, o.rsrc, in ? off + o.pitch : kDropOffset, 0, 0);
        return;
    }
    const uint32_t px[4] = {q.y01, q.y23, q.u, q.v};
    store_quad(o, quad_yuv(px), x, y, in);
}

__device__ __forceinline__ void store_rgba(const RgbaSink& o, const QuadOut& q, uint32_t cam, int x, int y, bool in) {
    // the camera descriptor through the constant address space: scalar loads.  (As a plain global
    // pointer the compiler cannot rule out the kernel's own stores aliasing it and emitted per-lane
    // loads, each followed by a vmcnt(0) that drained the next item's prefetches: 34 us of C3's 94 us
    // remap.)  cam is uniform (the item's camera).
    typedef __attribute__((address_space(4))) const MbCamLevel kMbCamLevel;
    const kMbCamLevel* c = (const kMbCamLevel*)o.cams + uniform((int)cam);
    const int ox = c->ox, oy = c->oy, cw = c->w, chh = c->h;
    const uint32_t goff = c->g_off, gp = c->g_pitch;
    const int xl = x - ox, yl = y - oy;
    const bool ok = in && xl >= 0 && yl >= 0 && xl < cw && yl < chh;  // w, h even: whole quads
    const uint32_t off = ok ? goff + (uint32_t)yl * gp + (uint32_t)xl * 4u : kDropOffset;
    typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
    const u32x2 r0 = {q.y01, q.y23}, r1 = {q.u, q.v};
    __builtin_amdgcn_raw_buffer_store_b64(r0, o.rsrc, off, 0, 0);
    __builtin_amdgcn_raw_buffer_store_b64(r1, o.rsrc, ok ? off + gp : kDropOffset, 0, 0);
}

// One half of an item: MODE 0 the YUV quad into `of`; MODE 1 the G0 quad where the item's flags say some
// pyrDown or blend reads the lane's sub-tile (item_g0_bit), and the final result into `of` (the result frame)
// where they say the sub-tile is deep (item_result_bit).  The lane's sub-tile: quarter (lane & 63) >> 4.
template <int MODE>
__device__ __forceinline__ void store_half(const OutFrame& of, const RgbaSink& ro, bool res_rgba, const QuadOut& q,
                                           uint32_t cam, uint32_t flags, int h, int x, int y, bool in) {
    if constexpr (MODE == 0) {
        store_quad(of, q, x, y, in);
    } else {
        const int q4 = (int)((threadIdx.x & 63u) >> 4);
        if (flags & item_g0_bit(h, q4)) store_rgba(ro, q, cam, x, y, in);
        if (flags & item_result_bit(h, q4)) store_result(of, res_rgba, q, x, y, in);
    }
}

// The composite's static LDS, one variable (so its size, exactly 16 KiB, is where the dynamic region
// starts).  The weight table is the dynamic region (kWtabBytes at launch): kept out of the static size,
// the compiler's LDS occupancy model still allows 7 workgroups per CU and keeps the 7-wave register
// budget (72 VGPRs: the lean feed's wave fits beside 6 composite waves per SIMD); the table's base is
// then the constant 0x4000 (wtab_read).
struct alignas(16) StitchLds {
    uint32_t rgb[kTileLdsBytes / 4];  // the item's staged RGBA boxes (LDS address 0)
    uint32_t spare[kMaxCams];         // (the frames' camera gains live after the weight table)
    f32x2_t slot_gain[kTileSlots];
    uint32_t claim[2];
    uint32_t pad[2];
};
static_assert(sizeof(StitchLds) == 0x4000, "the weight table at LDS 0x4000 (wtab_read)");

// LDS byte address of a tiled entry's weight pairs: the table sits at 0x4000 (the kernel's static LDS
// is exactly 16 KiB: launch_composite checks the compiled size), so one v_and_or_b32 forms it; an
// address built from an integer, so the compiler does not split off a base it cannot fold into the offset.
__device__ __forceinline__ uint2 wtab_read(uint32_t e) {
    typedef __attribute__((address_space(3))) const uint64_t lds_u64;
    const uint64_t w = *(const lds_u64*)(uintptr_t)((e & 0x1FF8u) | 0x4000u);
    return uint2{(uint32_t)w, (uint32_t)(w >> 32)};
}

// LDS byte offset of a tiled entry's tap (x, y) (kernels.hpp, entry layout): one v_bfe_u32
__device__ __forceinline__ uint32_t tap_off(uint32_t e) { return (e >> 13) & 0x3FFFu; }

// Staged items.  The staged items are split into 8 contiguous bands, one per XCD under round-robin
// dispatch (blocks b, b+8, ...), so neighbouring items' source boxes share that XCD's L2.
// TEX: texture-convention entries (tiled_entry_tex): the taps as usual, the texture filter model instead of
// the weight table.
// LG: 1 << LG frames per launch (FrameBatch; MODE 0 only)
template <bool DWORD_STAGE, int MODE, bool VIG, bool TEX, int LG, bool E24>
__device__ __forceinline__ void stitch_tiled_body(const FrameBatch<1 << LG>& frames, TiledLut lut, int W, int H, int use_gain,
                                                  int64_t out_pitch, RgbaOut rgba) {
    __shared__ StitchLds L;
    extern __shared__ __attribute__((aligned(16))) uint2 s_wtab[];  // 1,024 weight pairs at LDS 0x4000
    uint32_t* const s_rgb = L.rgb;
    // per frame and camera, (frame << cam_log2) + camera: in the dynamic region after the weight table
    float* const s_gain = reinterpret_cast<float*>(s_wtab + 1024);
    constexpr int lg = LG, cam_lg = LG <= 1 ? 5 : 4;  // frames per launch 1 << lg (FrameBatch)
    static_assert(MODE == 0 || LG == 0, "frame batches: MODE 0 only");
    // {g, g} per slot (finish_quad2f).  Written after an item's first barrier and read after its
    // second; the next write comes after the next item's first barrier, i.e. after every wave's last
    // read, so one table suffices.
    f32x2_t* const s_slot_gain = L.slot_gain;
    // per iteration parity: written before an item's staging barrier, read after it (the next write
    // to the same entry is two items later, behind the next barrier)
    uint32_t* const s_claim = L.claim;
    constexpr int kItemH = kTileH * kItemHalves;

    const int groups = kStitchBands;
    const int g = blockIdx.x % groups;
    const int step = (gridDim.x - g + groups - 1) / groups;
    const int t_begin = lut.bands[g] << lg;  // work units: (item, frame) pairs
    const int t_end = lut.bands[g + 1] << lg;
    const __amdgpu_buffer_rsrc_t ersrc = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint32_t*>(lut.entries), 0,
        (int)((uint32_t)max(lut.n_items, 1) * (uint32_t)(kItemHalves * kTilePx * (E24 ? 3 : 4))), 0x00020000);
    const __amdgpu_buffer_rsrc_t mrsrc = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<TileHdr*>(lut.meta), 0, (int)((uint32_t)max(lut.n_items, 1) * (uint32_t)(kMetaWords * 16)), 0x00020000);
    const __amdgpu_buffer_rsrc_t grsrc = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint16_t*>(lut.grp0), 0, (int)((uint32_t)max(lut.n_items, 1) * (uint32_t)(kGroupFirst * 64 * 2)), 0x00020000);
    const __amdgpu_buffer_rsrc_t g1rsrc =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(lut.grp1), 0, (int)(lut.n_grp1 * 2u), 0x00020000);
    OutFrame of{};
    RgbaSink ro{};
    bool res_rgba = false;
    const int out_bytes = (int)((uint32_t)out_pitch * (uint32_t)(H + H / 2));
    if constexpr (MODE == 0) {
        of = make_out_frame(kernarg_out<1 << LG>(0), W, H, out_pitch);
    } else {
        ro = RgbaSink{__builtin_amdgcn_make_buffer_rsrc(rgba.base, 0, (int)rgba.bytes, 0x00020000), rgba.cams};
        of = make_result_frame(rgba);
        res_rgba = rgba.res_rgba != 0;
    }
    const int tid = threadIdx.x;
    const int qx = tid & 63, qy = tid >> 6;

    if (tid < (1 << (lg + cam_lg))) {
        const double* gf = kernarg_gains<1 << LG>((uint32_t)tid >> cam_lg);
        s_gain[tid] = use_gain ? (float)gf[tid & ((1 << cam_lg) - 1)] : 1.0f;
    }
    if (tid < kTileZeroDwords) s_rgb[tid] = 0u;
#pragma unroll
    for (int k = 0; k < 4; k++) s_wtab[tid + 256 * k] = bilerp_weights((uint32_t)(tid + 256 * k));
    // Item sequence of this workgroup: its first three items are static (t0, t0 + step, t0 + 2 step,
    // i.e. the band's first 3 * step items dealt round-robin), every later one is claimed from the
    // band's work counter (one returning atomic per item, issued one iteration before the item's
    // metadata load and handed to the other waves through LDS), so workgroups that drew cheap items
    // keep pulling work while expensive ones finish (static dealing left the band's workgroups
    // finishing between 31 and 80 us on C2).
    const int t0 = t_begin + (int)(blockIdx.x / groups);
    const int dyn0 = t_begin + 3 * step;  // item of claim value 0
    uint32_t* const q = lut.queue + g * kQueueStride;
    const int wave = uniform(tid >> 6);
    TileMeta cur = meta_read(meta_issue(mrsrc, t0, t_end, lg), t0, lg, cam_lg);
    const uint32_t g0 = group_issue(grsrc, t0, t_end, lg);
    __syncthreads();
    TileData d;
    data_issue<DWORD_STAGE, VIG, E24>(ersrc, cur, t_end, lg, stage_slot<true>(cur, t_end, wave), g0, d);
    int t_mv = t0 + step < t_end ? t0 + step : t_end;  // item of the metadata in flight (mv)
    int t_n2 = t_mv < t_end && t0 + 2 * step < t_end ? t0 + 2 * step : t_end;  // item after it
    uint4 mv = meta_issue(mrsrc, t_mv, t_end, lg);
    uint16_t mg = group_issue(grsrc, t_mv, t_end, lg);  // the lane's first staging group of item t_mv
    uint32_t claim = 0u;  // lane 0 of wave 0: returned value of the claim in flight
    bool claimed = false; // a claim for the item after t_n2 is in flight (uniform)
    bool first = true;
    // opaque copies of the prologue loads: the loop-header phis then merge a load with a non-load,
    // so the compiler cannot fold them into one load at the header (waited on right there)
    asm volatile("" : "+v"(mv.x), "+v"(mv.y), "+v"(mv.z), "+v"(mv.w), "+v"(mg));
#pragma unroll
    for (int h = 0; h < kItemHalves; h++) {
        asm volatile("" : "+v"(d.e4[h].x), "+v"(d.e4[h].y), "+v"(d.e4[h].z));
        if constexpr (!E24) asm volatile("" : "+v"(d.e4[h].w));
    }
    asm volatile("" : "+v"(d.sg.y0), "+v"(d.sg.y1), "+v"(d.sg.uq), "+v"(d.sg.vq));

    // the previous item's output, stored in the next iteration: every store is then older than the
    // loads it shares the iteration with (vmcnt waits on a load that is older than a store must drain
    // everything, as loads and stores complete out of order)
    QuadOut prev[kItemHalves];
#pragma unroll
    for (int h = 0; h < kItemHalves; h++) prev[h] = QuadOut{0u, 0u, 0u, 0u};
    int px = 0, py = 0;  // the previous item's quad of this lane in its first half
    // MODE 0 stores of items wholly inside the frame: the lane's part of the byte offsets is
    // loop-invariant (voffset), the item's part a scalar (soffset) — no per-lane address arithmetic
    const uint32_t lane_y = (uint32_t)(2 * qy) * of.pitch + (uint32_t)(2 * qx), lane_c = (uint32_t)qy * of.pitch + (uint32_t)qx;
    int pox = 0, poy = 0;  // the previous item's origin (uniform)
    bool pfull = false;    // the previous item lies wholly inside W x H (uniform)
    uint32_t pcam = 0, pfl = 0;  // the previous item's RGBA-mode camera and flags (item_result_bit / item_g0_bit)
    uint32_t pfr = 0;            // the previous unit's frame (MODE 0 output)
    bool pin = false;
    uint32_t par = 0;  // iteration parity
    while (cur.t < t_end) {
        const int x = (int)(cur.tile & 0xFFFFu) * kTileW + qx * 2, y = (int)(cur.tile >> 16) * kItemH + qy * 2;
        const uint32_t S = cur.stride & ((1u << kStrideBits) - 1u);
        uint4 e4[kItemHalves];
#pragma unroll
        for (int h = 0; h < kItemHalves; h++) e4[h] = d.e4[h];
        // every wave has read the previous item's staging area
        __syncthreads();
        if (tid < kTileZeroDwords) s_rgb[tid] = 0u;  // black pixels read offset 0 of the region
        const TileMeta nxt = meta_read(mv, t_mv, lg, cam_lg);
        {  // slot q's camera word sits in lane 1 + q of the metadata's first component
            const uint32_t cw = (uint32_t)__shfl((int)cur.v.x, 1 + (tid & 3), 64);
            // clamped to [0, FLT_MAX] (NaN -> 0) in MODE 0; no result depends on it (finish_quad2f
            // saturates with v_cvt_pk_u8_f32, which maps negative and NaN products to 0 either way)
            const float gs = s_gain[cur.fbase + (cw & 31u)];
            const float gc = MODE == 0 ? __builtin_fminf(__builtin_fmaxf(gs, 0.f), FLT_MAX) : gs;
            if (tid < kTileSlots) s_slot_gain[tid] = f32x2_t{gc, gc};
        }
        if (claimed && tid == 0) s_claim[par] = claim;  // issued one iteration ago
        stage_store<VIG>(d.sg, s_rgb);
        const uint32_t nch = (cur.nslots >> 8) & 0xFFu;
        if (nch > (uint32_t)kGroupFirst) {  // large items only: the other chunks now, groups from grp1
            const uint32_t ovf = cur.stride >> kStrideBits;
            for (int c = kGroupFirst + wave; c < (int)nch; c += 4) {
                const uint32_t gk = __builtin_amdgcn_raw_buffer_load_b16(
                    g1rsrc, (uint32_t)(tid & 63) * 2u, (ovf + (uint32_t)(c - kGroupFirst)) * 128u, 0);
                StageGroup sg;
                stage_load<DWORD_STAGE, VIG>(stage_slot(cur, t_end, c), S, gk, sg);
                stage_store<VIG>(sg, s_rgb);
            }
        }
        __syncthreads();
        // the item two ahead: static on the first iteration, else the claim handed over above.
        if (!first) {
            // Global addresses derive from this LDS-handed claim (the item's header, slots and entries,
            // and through its slots the camera frames), so it is range-checked as unsigned: a value that
            // is not a claim of this band (the r02 barrier-free ablation read s_claim before wave 0 wrote
            // it, i.e. uninitialised LDS -> negative item index -> out-of-range header and entry loads and
            // a null frame pointer, hipErrorIllegalAddress) ends the sequence instead.
            // (one scalar min: dyn0 + cv then cannot wrap negative, and t_n2 below stays in [0, t_end])
            const uint32_t cv = min((uint32_t)uniform((int)s_claim[par]), 0x3FFFFFFFu);
            const int v = claimed ? dyn0 + (int)cv : t_end;
            t_n2 = v < t_end ? v : t_end;
        }
        first = false;
        if (MODE == 0 && lg) of.rsrc = __builtin_amdgcn_make_buffer_rsrc(kernarg_out<1 << LG>(pfr), 0, out_bytes, 0x00020000);
        if (MODE == 0 && pfull) {
#pragma unroll
            for (int h = 0; h < kItemHalves; h++) {
                const uint32_t sy = (uint32_t)uniform((poy + h * kTileH) * (int)of.pitch + pox);
                const uint32_t sc = (uint32_t)uniform(((poy + h * kTileH) >> 1) * (int)of.pitch + (pox >> 1));
                __builtin_amdgcn_raw_buffer_store_b16((uint16_t)prev[h].y01, of.rsrc, lane_y, sy, kOutPolicy);
                __builtin_amdgcn_raw_buffer_store_b16((uint16_t)prev[h].y23, of.rsrc, lane_y, sy + of.pitch, kOutPolicy);
                __builtin_amdgcn_raw_buffer_store_b8((uint8_t)prev[h].u, of.rsrc, lane_c, sc + of.u_off, kOutPolicy);
                __builtin_amdgcn_raw_buffer_store_b8((uint8_t)prev[h].v, of.rsrc, lane_c, sc + of.v_off, kOutPolicy);
            }
        } else {
#pragma unroll
            for (int h = 0; h < kItemHalves; h++)
                store_half<MODE>(of, ro, res_rgba, prev[h], pcam, pfl, h, px, py + h * kTileH, pin && py + h * kTileH < H);
        }
        // the next item's first staging slot resolved only now (short scalar live ranges), then its loads
        data_issue<DWORD_STAGE, VIG, E24>(ersrc, nxt, t_end, lg, stage_slot<true>(nxt, t_end, wave), mg, d);
        mv = meta_issue(mrsrc, t_n2, t_end, lg);
        mg = group_issue(grsrc, t_n2, t_end, lg);
        t_mv = t_n2;
        claimed = t_n2 < t_end;  // claim the item after it (only while the sequence is live)
        if (claimed && tid == 0) {
            // an opaque (per-lane looking) address: the atomic optimizer would otherwise rewrite the
            // single-lane claim into a wave-level one whose result it broadcasts (and waits for) at once
            int zero = tid;
            asm volatile("" : "+v"(zero));
            claim = __hip_atomic_fetch_add(q + zero, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
#pragma unroll
        for (int h = 0; h < kItemHalves; h++) {
            // E24: the four 24-bit entries from the three dwords (two v_alignbit_b32, one shift)
            const uint32_t ent[4] = {e4[h].x, E24 ? __builtin_amdgcn_alignbit(e4[h].y, e4[h].x, 24u) : e4[h].y,
                                     E24 ? __builtin_amdgcn_alignbit(e4[h].z, e4[h].y, 16u) : e4[h].z,
                                     E24 ? e4[h].z >> 8 : e4[h].w};
            float rgb[4][3];
            f32x2_t gain[4];
#pragma unroll
            for (int p = 0; p < 4; p++) {
                const uint32_t e = ent[p];
                // taps (x, y), (x+1, y) and (x, y+1), (x+1, y+1): two ds_read2_b32, no per-tap masking
                const uint8_t* r0 = reinterpret_cast<const uint8_t*>(s_rgb) +
                                    (TEX ? (e >> 15) & 0x3FFCu : E24 ? (e >> 10) & 0x3FFCu : tap_off(e));
                const uint8_t* r1 = r0 + 4u * S;
                const uint32_t c00 = reinterpret_cast<const uint32_t*>(r0)[0];
                const uint32_t c01 = reinterpret_cast<const uint32_t*>(r0)[1];
                const uint32_t c10 = reinterpret_cast<const uint32_t*>(r1)[0];
                const uint32_t c11 = reinterpret_cast<const uint32_t*>(r1)[1];
                if constexpr (TEX) {
                    tex_bilerp_f(c00, c01, c10, c11, (e >> 1) & 255u, (e >> 9) & 255u, rgb[p]);
                    gain[p] = *reinterpret_cast<const f32x2_t*>(reinterpret_cast<const uint8_t*>(s_slot_gain) + ((e >> 30) << 3));
                } else {
                    // E24: fxy at bits 2-11, so e << 1 holds it where wtab_read masks (bits 3-12)
                    bilerp_rgba_w(c00, c01, c10, c11, wtab_read(E24 ? e << 1 : e), rgb[p]);
                    // slot << 3 = e >> 27 (bits 27-29 of a tiled entry are zero; kernels.hpp); E24: bits 0-1
                    const uint32_t go = E24 ? (e << 3) & 0x18u : e >> 27;
                    gain[p] = *reinterpret_cast<const f32x2_t*>(reinterpret_cast<const uint8_t*>(s_slot_gain) + go);
                }
                if (MODE == 1 && !E24 && (e & kEntryNoGain)) gain[p] = f32x2_t{1.0f, 1.0f};
            }
            prev[h] = finish_any<MODE>(rgb, gain);
        }
        px = x;
        py = y;
        pox = (int)(cur.tile & 0xFFFFu) * kTileW;
        poy = (int)(cur.tile >> 16) * kItemH;
        pfull = pox + kTileW <= W && poy + kItemH <= H;
        pcam = (cur.nslots >> 16) & 31u;
        pfr = cur.frame;
        pfl = MODE == 1 ? (cur.map >> 8) & 0xFFFFu : 0u;
        pin = x < W && y < H;
        par ^= 1u;
        cur = nxt;
    }
    // the last workgroup to finish resets the work counters for the next launch (stream order makes
    // the reset visible to it); every claim of this workgroup has returned before its ticket
    if (tid == 0) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        (void)claim;
        if (__hip_atomic_fetch_add(lut.queue + kStitchBands * kQueueStride, 1u, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1) {
            for (int k = 0; k <= kStitchBands; k++)
                __hip_atomic_exchange(lut.queue + k * kQueueStride, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    if (MODE == 0 && lg) of.rsrc = __builtin_amdgcn_make_buffer_rsrc(kernarg_out<1 << LG>(pfr), 0, out_bytes, 0x00020000);
#pragma unroll
    for (int h = 0; h < kItemHalves; h++)
        store_half<MODE>(of, ro, res_rgba, prev[h], pcam, pfl, h, px, py + h * kTileH, pin && py + h * kTileH < H);
}

template <bool DWORD_STAGE, int MODE, bool VIG, int LG, bool E24>
__global__ void __launch_bounds__(256, kStitchRegBlocks) __attribute__((amdgpu_num_sgpr(kStitchSgprs)))
__attribute__((amdgpu_num_vgpr(kStitchVgprs))) stitch_tiled_kernel(FrameBatch<1 << LG> frames, TiledLut lut, int W, int H,
                                                                   int use_gain, int64_t out_pitch, RgbaOut rgba) {
    stitch_tiled_body<DWORD_STAGE, MODE, VIG, false, LG, E24>(frames, lut, W, H, use_gain, out_pitch, rgba);
}
template <bool DWORD_STAGE, int MODE, bool VIG, int LG>
__global__ void __launch_bounds__(256, kStitchTexRegBlocks) __attribute__((amdgpu_num_sgpr(kStitchSgprs)))
__attribute__((amdgpu_num_vgpr(kStitchTexVgprs))) stitch_tiled_tex_kernel(FrameBatch<1 << LG> frames, TiledLut lut, int W,
                                                                          int H, int use_gain, int64_t out_pitch,
                                                                          RgbaOut rgba) {
    stitch_tiled_body<DWORD_STAGE, MODE, VIG, true, LG, false>(frames, lut, W, H, use_gain, out_pitch, rgba);
}

// Wide tiles: one workgroup per tile, 8-byte absolute entries, direct global gathers.
template <int MODE>
__global__ void __launch_bounds__(256) stitch_wide_kernel(FrameSet frames, TiledLut lut, int W, int H,
                                                          const double* gains, int use_gain, uint8_t* out,
                                                          int64_t out_pitch, RgbaOut rgba) {
    __shared__ float s_gain[kMaxCams];
    const int tid = threadIdx.x;
    if (tid < kMaxCams) s_gain[tid] = use_gain ? (float)gains[tid] : 1.0f;
    __syncthreads();
    OutFrame of{};
    RgbaSink ro{};
    if constexpr (MODE == 0) {
        of = make_out_frame(out, W, H, out_pitch);
    } else {
        ro = RgbaSink{__builtin_amdgcn_make_buffer_rsrc(rgba.base, 0, (int)rgba.bytes, 0x00020000), rgba.cams};
        of = make_result_frame(rgba);
    }
    const uint32_t tile = (uint32_t)uniform((int)lut.wide_tiles[blockIdx.x]);
    const int x = (int)(tile & 0xFFFFu) * kTileW + (tid & 63) * 2, y = (int)(tile >> 16) * kTileH + (tid >> 6) * 2;
    const uint4* wp = reinterpret_cast<const uint4*>(lut.wide + (int64_t)blockIdx.x * kTilePx) + tid * 2;
    const uint4 e0 = wp[0], e1 = wp[1];
    const uint32_t xy[4] = {e0.x, e0.z, e1.x, e1.z};
    const uint32_t cd[4] = {e0.y, e0.w, e1.y, e1.w};
    Taps tp[4];
#pragma unroll
    for (int p = 0; p < 4; p++) gather_taps(frames, xy[p], cd[p], tp[p]);
    uint32_t rgb[4][3];
    f32x2_t gain[4];
#pragma unroll
    for (int p = 0; p < 4; p++) {
        if (cd[p] & kCodeTex)  // texture-convention entries (make_entry_tex)
            tex_bilerp(tp[p].c[0], tp[p].c[1], tp[p].c[2], tp[p].c[3], tp[p].fx, tp[p].fy, rgb[p]);
        else
            bilerp_rgba(tp[p].c[0], tp[p].c[1], tp[p].c[2], tp[p].c[3], tp[p].fx, tp[p].fy, rgb[p]);
        float gp = (MODE == 1 && (cd[p] & kCodeNoGain)) ? 1.0f : s_gain[(cd[p] >> 10) & 31u];
        gain[p] = f32x2_t{gp, gp};
    }
    const uint32_t camb = MODE == 1 ? (uint32_t)uniform((int)lut.wide_cams[blockIdx.x]) : 0u;
    float rgbf[4][3];
#pragma unroll
    for (int p = 0; p < 4; p++)
#pragma unroll
        for (int ch = 0; ch < 3; ch++) rgbf[p][ch] = (float)rgb[p][ch];
    // camera word: camera | the half's quarters' result bits << 8 | G0 bits << 12 (tiling.cpp), i.e. the
    // item flags of a half 0
    const uint32_t fl = ((camb >> 8) & 15u) | ((camb >> 12) & 15u) << 8;
    store_half<MODE>(of, ro, rgba.res_rgba != 0, finish_any<MODE>(rgbf, gain), camb & 31u, fl, 0, x, y, x < W && y < H);
}

// The weight table's address (wtab_read) assumes the dynamic LDS starts right after StitchLds: checked
// once per kernel instance against the compiled static LDS size.
template <bool DW, int MODE, bool V, bool TEX, int LG, bool E24>
static hipError_t stitch_lds_check() {
    hipFuncAttributes a;
    const void* k = TEX ? reinterpret_cast<const void*>(stitch_tiled_tex_kernel<DW, MODE, V, LG>)
                        : reinterpret_cast<const void*>(stitch_tiled_kernel<DW, MODE, V, LG, E24>);
    const hipError_t e = hipFuncGetAttributes(&a, k);
    if (e != hipSuccess) return e;
    return a.sharedSizeBytes == sizeof(StitchLds) ? hipSuccess : hipErrorInvalidKernelFile;
}

// dynamic LDS of the composite: the weight table, then the frames' camera gains (FrameBatch order)
constexpr uint32_t kStitchDynLds = kWtabBytes + 4u * 2u * kMaxCams;

template <bool DW, int MODE, bool V, bool TEX, int LG, bool E24>
static hipError_t launch_tiled(int blocks, const FrameBatch<1 << LG>& frames, const TiledLut& lut, int W, int H, int use_gain,
                               int64_t out_pitch, const RgbaOut& rgba, hipStream_t s, hipEvent_t ev0, hipEvent_t ev1) {
    static const hipError_t lds_ok = stitch_lds_check<DW, MODE, V, TEX, LG, E24>();
    if (lds_ok != hipSuccess) return lds_ok;
    if constexpr (TEX) {
        // (no packet-carried timing events: the texture convention is not a bench line's timed kernel)
        hipLaunchKernelGGL((stitch_tiled_tex_kernel<DW, MODE, V, LG>), dim3(blocks), dim3(256), kStitchDynLds, s,
                           frames, lut, W, H, use_gain, out_pitch, rgba);
        if (ev0) (void)hipEventRecord(ev1, s);
    } else if (ev0) {  // the timing events carried by the dispatch packet itself
        hipExtLaunchKernelGGL((stitch_tiled_kernel<DW, MODE, V, LG, E24>), dim3(blocks), dim3(256), kStitchDynLds, s, ev0,
                              ev1, 0, frames, lut, W, H, use_gain, out_pitch, rgba);
    } else {
        hipLaunchKernelGGL((stitch_tiled_kernel<DW, MODE, V, LG, E24>), dim3(blocks), dim3(256), kStitchDynLds, s, frames,
                           lut, W, H, use_gain, out_pitch, rgba);
    }
    return hipGetLastError();
}

// the frame sets as the kernel's kernarg table for 1 << LG frames
template <int LG>
static void frame_batch(const FrameSet* frames, const double* const* gains, uint8_t* const* out,
                        FrameBatch<1 << LG>& fb) {
    constexpr int cam_lg = FrameBatch<1 << LG>::kCamLog2;
    memset(&fb, 0, sizeof fb);
    for (int f = 0; f < (1 << LG); f++) {
        for (int i = 0; i < (1 << cam_lg); i++) fb.src[(f << cam_lg) + i] = frames[f].f[i];
        fb.out[f] = out ? out[f] : nullptr;
        fb.gains[f] = gains[f];
    }
}

template <bool DW, int MODE, bool V, bool TEX, bool E24>
static hipError_t launch_tiled_lg(int lg, int blocks, const FrameSet* frames, const double* const* gains,
                                  uint8_t* const* out, const TiledLut& lut, int W, int H, int use_gain,
                                  int64_t out_pitch, const RgbaOut& rgba, hipStream_t s, hipEvent_t ev0,
                                  hipEvent_t ev1) {
    if constexpr (MODE == 0) {
        if (lg == 1) {
            FrameBatch<2> fb;
            frame_batch<1>(frames, gains, out, fb);
            return launch_tiled<DW, MODE, V, TEX, 1, E24>(blocks, fb, lut, W, H, use_gain, out_pitch, rgba, s, ev0, ev1);
        }
        if (lg == 2) {
            FrameBatch<4> fb;
            frame_batch<2>(frames, gains, out, fb);
            return launch_tiled<DW, MODE, V, TEX, 2, E24>(blocks, fb, lut, W, H, use_gain, out_pitch, rgba, s, ev0, ev1);
        }
    }
    if (lg != 0) return hipErrorInvalidValue;
    FrameBatch<1> fb;
    frame_batch<0>(frames, gains, out, fb);
    return launch_tiled<DW, MODE, V, TEX, 0, E24>(blocks, fb, lut, W, H, use_gain, out_pitch, rgba, s, ev0, ev1);
}

// the instance for the frames' staging (dword loads, vignette) and the entries' convention
template <int MODE, bool TEX, bool E24>
static hipError_t launch_tiled_vd(bool dw, bool vig, int lg, int blocks, const FrameSet* fr, const double* const* g,
                                  uint8_t* const* o, const TiledLut& lut, int W, int H, int use_gain, int64_t out_pitch,
                                  const RgbaOut& rgba, hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
    if (dw && !vig)
        return launch_tiled_lg<true, MODE, false, TEX, E24>(lg, blocks, fr, g, o, lut, W, H, use_gain, out_pitch, rgba, s, e0, e1);
    if (dw)
        return launch_tiled_lg<true, MODE, true, TEX, E24>(lg, blocks, fr, g, o, lut, W, H, use_gain, out_pitch, rgba, s, e0, e1);
    if (!vig)
        return launch_tiled_lg<false, MODE, false, TEX, E24>(lg, blocks, fr, g, o, lut, W, H, use_gain, out_pitch, rgba, s, e0, e1);
    return launch_tiled_lg<false, MODE, true, TEX, E24>(lg, blocks, fr, g, o, lut, W, H, use_gain, out_pitch, rgba, s, e0, e1);
}

// the entries' width: 24-bit (TiledLut::e24, default sampling only) or 32-bit
template <int MODE, bool TEX>
static hipError_t launch_tiled_for(bool dw, bool vig, int lg, int blocks, const FrameSet* fr, const double* const* g,
                                   uint8_t* const* o, const TiledLut& lut, int W, int H, int use_gain, int64_t out_pitch,
                                   const RgbaOut& rgba, hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
    if constexpr (!TEX) {
        if (lut.e24)
            return launch_tiled_vd<MODE, TEX, true>(dw, vig, lg, blocks, fr, g, o, lut, W, H, use_gain, out_pitch, rgba, s, e0, e1);
    } else {
        if (lut.e24) return hipErrorInvalidValue;  // texture-convention entries are never packed
    }
    return launch_tiled_vd<MODE, TEX, false>(dw, vig, lg, blocks, fr, g, o, lut, W, H, use_gain, out_pitch, rgba, s, e0, e1);
}

// nf frame sets (1, 2 or 4) in one launch of the tiled kernel (FrameBatch); wide tiles one launch per frame
template <int MODE>
static hipError_t launch_composite(const FrameSet* frames, int nf, const TiledLut& lut, int W, int H,
                                   const double* const* gains, int use_gain, uint8_t* const* out, int64_t out_pitch,
                                   const RgbaOut& rgba, hipStream_t s, hipEvent_t ev0 = nullptr,
                                   hipEvent_t ev1 = nullptr) {
    if (lut.n_items > 0 && lut.qpl != kItemHalves) return hipErrorInvalidValue;
    const int lg = nf == 1 ? 0 : nf == 2 ? 1 : nf == 4 ? 2 : -1;
    if (lg < 0 || (MODE == 1 && nf != 1)) return hipErrorInvalidValue;
    const int cam_lg = nf <= 2 ? 5 : 4;
    for (int f = 0; f < nf; f++)
        for (int i = 1 << cam_lg; i < kMaxCams; i++)
            if (frames[f].f[i].yuv) return hipErrorInvalidValue;  // more cameras than a 4-frame batch holds
    // timing events: carried by the dispatch packet when the tiled kernel is the only launch (no marker
    // packets between the launches of the timed loop), else recorded around the launches
    const bool ext_ev = ev0 && lut.n_items > 0 && lut.n_wide == 0;
    if (ev0 && !ext_ev) {
        const hipError_t e = hipEventRecord(ev0, s);
        if (e != hipSuccess) return e;
    }
    if (lut.n_items > 0) {
        // one resident wave of workgroups (256 CUs x kStitchBlocksPerCU), each walking its XCD band's units;
        // fewer than 3 units per workgroup (C1's 4,096 items) get a third as many workgroups as units, so
        // that every workgroup has its three statically dealt units (the first 2.7 rounds of 1,536 left the
        // last round a third empty: C1 17.4 -> 15.6 us, interleaved)
        const int units = lut.n_items * nf;
        int blocks = std::min(units, 256 * kStitchBlocksPerCU);
        if (units < 3 * 256 * kStitchBlocksPerCU) blocks = (units + 2) / 3;
        blocks = std::max(8, (blocks + 7) / 8 * 8);
        // wide staging loads need 8-byte aligned Y rows (then U / V rows are 4-byte aligned)
        bool dw = true, vig = false;
        for (int f = 0; f < nf; f++)
            for (int i = 0; i < kMaxCams; i++) {
                const SourceFrame& sf = frames[f].f[i];
                if (!sf.yuv) continue;
                if ((reinterpret_cast<uintptr_t>(sf.yuv) & 7u) || (sf.pitch & 7) || (sf.w & 7)) dw = false;
                vig |= sf.vig != nullptr;
            }
        hipEvent_t e0 = ext_ev ? ev0 : nullptr, e1 = ext_ev ? ev1 : nullptr;
        const hipError_t e =
            lut.tex ? launch_tiled_for<MODE, true>(dw, vig, lg, blocks, frames, gains, out, lut, W, H, use_gain, out_pitch,
                                                   rgba, s, e0, e1)
                    : launch_tiled_for<MODE, false>(dw, vig, lg, blocks, frames, gains, out, lut, W, H, use_gain, out_pitch,
                                                    rgba, s, e0, e1);
        if (e != hipSuccess) return e;
    }
    if (lut.n_wide > 0)
        for (int f = 0; f < nf; f++)
            hipLaunchKernelGGL(stitch_wide_kernel<MODE>, dim3(lut.n_wide), dim3(256), 0, s, frames[f], lut, W, H,
                               gains[f], use_gain, out ? out[f] : nullptr, out_pitch, rgba);
    if (ev0 && !ext_ev) {
        const hipError_t e = hipEventRecord(ev1, s);
        if (e != hipSuccess) return e;
    }
    return hipGetLastError();
}

int composite_qpl() { return kItemHalves; }

hipError_t launch_stitch_batch(const FrameSet* frames, int nf, const TiledLut& lut, int W, int H,
                               const double* const* gains, int use_gain, uint8_t* const* out, int64_t out_pitch,
                               hipStream_t s, hipEvent_t ev0, hipEvent_t ev1) {
    if (nf < 1 || nf > kMaxBatch) return hipErrorInvalidValue;
    return launch_composite<0>(frames, nf, lut, W, H, gains, use_gain, out, out_pitch, RgbaOut{}, s, ev0, ev1);
}

hipError_t launch_stitch(const FrameSet& frames, const TiledLut& lut, int W, int H, const double* gains,
                         int use_gain, uint8_t* out, int64_t out_pitch, hipStream_t s, hipEvent_t ev0, hipEvent_t ev1) {
    return launch_composite<0>(&frames, 1, lut, W, H, &gains, use_gain, &out, out_pitch, RgbaOut{}, s, ev0, ev1);
}

hipError_t launch_mb_remap(const FrameSet& frames, const TiledLut& lut, const double* gains, int use_gain,
                           const RgbaOut& out, hipStream_t s) {
    // W, H: no level-grid bound of its own (the per-camera ROI check drops what lies outside)
    return launch_composite<1>(&frames, 1, lut, 1 << 16, 1 << 16, &gains, use_gain, nullptr, 0, out, s);
}

// ---------------------------------------------------------------------------------------------
// Standalone cv::remap INTER_LINEAR u8 (cn = 1, 3, 4), BORDER_CONSTANT 0 — one output pixel per lane.
// ---------------------------------------------------------------------------------------------
template <int CN>
__global__ void __launch_bounds__(256) remap_u8_kernel(const uint8_t* src, int sw, int sh, int64_t spitch,
                                                       const float* map1, const float* map2, int mw, int mh,
                                                       int64_t mpitch, float scale_x, float scale_y, uint8_t* dst,
                                                       int64_t dpitch) {
    const int64_t total = (int64_t)mw * mh;
    for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
         idx += (int64_t)gridDim.x * blockDim.x) {
        const int y = (int)(idx / mw), x = (int)(idx - (int64_t)y * mw);
        const float X = map1[(int64_t)y * mpitch + x] * scale_x;
        const float Yv = map2[(int64_t)y * mpitch + x] * scale_y;
        const float fx32 = X * 32.0f, fy32 = Yv * 32.0f;
        // _mm_cvtps_epi32: NaN / out of int range -> INT_MIN
        const int ix = (fx32 != fx32 || fabsf(fx32) >= 2147483648.f) ? INT32_MIN : (int)__builtin_rintf(fx32);
        const int iy = (fy32 != fy32 || fabsf(fy32) >= 2147483648.f) ? INT32_MIN : (int)__builtin_rintf(fy32);
        const int sx = min(max(ix >> 5, -32768), 32767), sy = min(max(iy >> 5, -32768), 32767);
        const uint32_t fx = (uint32_t)(ix & 31), fy = (uint32_t)(iy & 31);
        uint32_t v[4][CN];
#pragma unroll
        for (int t = 0; t < 4; t++) {
            const int tx = sx + (t & 1), ty = sy + (t >> 1);
            const bool in = tx >= 0 && tx < sw && ty >= 0 && ty < sh;
            const uint8_t* p = src + (int64_t)min(max(ty, 0), sh - 1) * spitch + (int64_t)min(max(tx, 0), sw - 1) * CN;
#pragma unroll
            for (int k = 0; k < CN; k++) v[t][k] = in ? p[k] : 0u;
        }
        uint8_t* d = dst + (int64_t)y * dpitch + (int64_t)x * CN;
#pragma unroll
        for (int k = 0; k < CN; k++) d[k] = (uint8_t)bilerp_ch(v[0][k], v[1][k], v[2][k], v[3][k], fx, fy);
    }
}

// ---------------------------------------------------------------------------------------------
// morph_controlpoints' piecewise-affine LUT warp (template_morph.cpp:207-231).  The reference warps
// the whole ROI three times per triangle and copies the triangle's fillPoly'd pixels; here each
// pixel is computed once, by the last triangle that covers it (owner, rasterised on the host).
// cv::warpAffine (imgwarp.cpp:5627-5745, WarpAffineInvoker :5282-5470): AB_BITS = 10 fixed-point
// source coordinates, X = (round((M1 y + M2) 1024) + 16 + round(M0 x 1024)) >> 5, then remap's
// INTER_LINEAR (remapBilinear :3812-4030): f32 planes with the float table ((1-fy)(1-fx), (1-fy)fx,
// fy(1-fx), fy fx in 1/32 steps, exact), u8 with the 15-bit table; taps outside the ROI read 0.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ int cv_round_sse2(double v) {  // _mm_cvtsd_si32: ties to even, out of range -> INT_MIN
    const double r = __builtin_rint(v);
    return (r >= -2147483648.0 && r <= 2147483647.0) ? (int)r : INT32_MIN;
}

__global__ void __launch_bounds__(256) morph_warp_kernel(const float* __restrict__ map1, const float* __restrict__ map2,
                                                         const uint8_t* __restrict__ mask, int w, int h,
                                                         const int16_t* __restrict__ owner, const double* __restrict__ M,
                                                         float* out1, float* out2, uint8_t* out_mask) {
    const int64_t total = (int64_t)w * h;
    for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
         idx += (int64_t)gridDim.x * blockDim.x) {
        const int k = owner[idx];
        if (k < 0) {
            out1[idx] = map1[idx];
            out2[idx] = map2[idx];
            out_mask[idx] = mask[idx];
            continue;
        }
        const int y = (int)(idx / w), x = (int)(idx - (int64_t)y * w);
        const double* m = M + 6 * k;
        const int X0 = cv_round_sse2((m[1] * (double)y + m[2]) * 1024.0) + 16;  // round_delta = 1024 / 32 / 2
        const int Y0 = cv_round_sse2((m[4] * (double)y + m[5]) * 1024.0) + 16;
        const int ad = cv_round_sse2(m[0] * (double)x * 1024.0), bd = cv_round_sse2(m[3] * (double)x * 1024.0);
        const int X = (int)((uint32_t)X0 + (uint32_t)ad) >> 5, Y = (int)((uint32_t)Y0 + (uint32_t)bd) >> 5;
        const int sx = min(max(X >> 5, -32768), 32767), sy = min(max(Y >> 5, -32768), 32767);
        const uint32_t fx = (uint32_t)(X & 31), fy = (uint32_t)(Y & 31);
        float a1[4], a2[4];
        uint32_t am[4];
#pragma unroll
        for (int t = 0; t < 4; t++) {
            const int tx = sx + (t & 1), ty = sy + (t >> 1);
            const bool in = tx >= 0 && tx < w && ty >= 0 && ty < h;
            const int64_t o = in ? (int64_t)ty * w + tx : 0;
            a1[t] = in ? map1[o] : 0.f;
            a2[t] = in ? map2[o] : 0.f;
            am[t] = in ? mask[o] : 0u;
        }
        const float vy1 = (float)fy * (1.f / 32), vy0 = 1.f - vy1, vx1 = (float)fx * (1.f / 32), vx0 = 1.f - vx1;
        const float w0 = vy0 * vx0, w1 = vy0 * vx1, w2 = vy1 * vx0, w3 = vy1 * vx1;
        out1[idx] = a1[0] * w0 + a1[1] * w1 + a1[2] * w2 + a1[3] * w3;
        out2[idx] = a2[0] * w0 + a2[1] * w1 + a2[2] * w2 + a2[3] * w3;
        out_mask[idx] = (uint8_t)bilerp_ch(am[0], am[1], am[2], am[3], fx, fy);
    }
}

hipError_t launch_morph_warp(const float* map1, const float* map2, const uint8_t* mask, int w, int h,
                             const int16_t* owner, const double* M, float* out1, float* out2, uint8_t* out_mask,
                             hipStream_t s) {
    const int64_t total = (int64_t)w * h;
    const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>((total + 255) / 256, 256 * 16));
    hipLaunchKernelGGL(morph_warp_kernel, dim3(blocks), dim3(256), 0, s, map1, map2, mask, w, h, owner, M, out1, out2,
                       out_mask);
    return hipGetLastError();
}

hipError_t launch_remap_u8(const uint8_t* src, int sw, int sh, int64_t spitch, int cn,
                           const float* map1, const float* map2, int mw, int mh, int64_t mpitch, float scale_x,
                           float scale_y, uint8_t* dst, int64_t dpitch, hipStream_t s) {
    const int64_t total = (int64_t)mw * mh;
    int blocks = (int)std::min<int64_t>((total + 255) / 256, 256 * 8);
    if (blocks < 1) blocks = 1;
    switch (cn) {
        case 1:
            hipLaunchKernelGGL(remap_u8_kernel<1>, dim3(blocks), dim3(256), 0, s, src, sw, sh, spitch, map1, map2,
                               mw, mh, mpitch, scale_x, scale_y, dst, dpitch);
            break;
        case 3:
            hipLaunchKernelGGL(remap_u8_kernel<3>, dim3(blocks), dim3(256), 0, s, src, sw, sh, spitch, map1, map2,
                               mw, mh, mpitch, scale_x, scale_y, dst, dpitch);
            break;
        case 4:
            hipLaunchKernelGGL(remap_u8_kernel<4>, dim3(blocks), dim3(256), 0, s, src, sw, sh, spitch, map1, map2,
                               mw, mh, mpitch, scale_x, scale_y, dst, dpitch);
            break;
        default:
            return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// cv::resize INTER_LINEAR u8 (CPU fixed-point rule, tables from the host) — seam-mask build.
// ---------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) resize_u8_kernel(const uint8_t* __restrict__ src, int sw, int sh, int64_t spitch,
                                                        uint8_t* __restrict__ dst, int dw, int dh, int64_t dpitch,
                                                        ResizeTables t) {
    const int64_t total = (int64_t)dw * dh;
    for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
         idx += (int64_t)gridDim.x * blockDim.x) {
        const int y = (int)(idx / dw), x = (int)(idx - (int64_t)y * dw);
        uint32_t v;
        if (t.area2) {
            const uint8_t* s0 = src + (int64_t)(2 * y) * spitch + 2 * x;
            v = ((uint32_t)s0[0] + s0[1] + s0[spitch] + s0[spitch + 1] + 2u) >> 2;
        } else {
            const uint8_t* r0 = src + (int64_t)t.rows[2 * y] * spitch;
            const uint8_t* r1 = src + (int64_t)t.rows[2 * y + 1] * spitch;
            const int sx = t.xofs[x];
            int h0, h1;
            if (x < t.xmax) {
                const int a0 = t.ax[2 * x], a1 = t.ax[2 * x + 1];
                h0 = r0[sx] * a0 + r0[sx + 1] * a1;
                h1 = r1[sx] * a0 + r1[sx + 1] * a1;
            } else {
                h0 = r0[sx] * 2048;
                h1 = r1[sx] * 2048;
            }
            const int b0 = t.by[2 * y], b1 = t.by[2 * y + 1];
            v = (uint32_t)((((b0 * (h0 >> 4)) >> 16) + ((b1 * (h1 >> 4)) >> 16) + 2) >> 2);
        }
        dst[(int64_t)y * dpitch + x] = (uint8_t)v;
    }
}

hipError_t launch_resize_u8(const uint8_t* src, int sw, int sh, int64_t spitch, uint8_t* dst, int dw, int dh,
                            int64_t dpitch, const ResizeTables& t, hipStream_t s) {
    const int64_t total = (int64_t)dw * dh;
    if (total <= 0) return hipSuccess;
    const int blocks = (int)std::min<int64_t>((total + 255) / 256, 256 * 8);
    hipLaunchKernelGGL(resize_u8_kernel, dim3(blocks), dim3(256), 0, s, src, sw, sh, spitch, dst, dw, dh, dpitch, t);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// Scaled output (Mapper with scale_output != template size, mapper.cpp:290-306): the stitched RGB
// result is resized with cuda::resize INTER_LINEAR (the glob kernel, resize.cu:71-103, which a
// 3-channel image always takes) and converted to YUV420P.  Source: the composite's RGBA frame
// (alpha ignored).  One lane per 2x2 output quad: 4 bilinear samples, then the same RGB -> YUV420P
// quad conversion as the fused path.  nvcc contracts `out + src * w` into an FMA: explicit fmaf.
// ---------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) resize_rgba_yuv420_kernel(const uint8_t* __restrict__ rgba, int sw, int sh,
                                                                 int64_t spitch, float fx, float fy, uint8_t* out,
                                                                 int dw, int dh, int64_t out_pitch) {
    const OutFrame of = make_out_frame(out, dw, dh, out_pitch);
    const int qw = dw >> 1, qh = dh >> 1;
    const int64_t total = (int64_t)qw * qh;
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < total; q += (int64_t)gridDim.x * blockDim.x) {
        const int qy = (int)(q / qw), qx = (int)(q - (int64_t)qy * qw);
        uint32_t rgb[4][3];
#pragma unroll
        for (int p = 0; p < 4; p++) {
            const int x = 2 * qx + (p & 1), y = 2 * qy + (p >> 1);
            const float src_x = (float)x * fx, src_y = (float)y * fy;
            const int x1 = (int)floorf(src_x), y1 = (int)floorf(src_y);
            const int x2 = x1 + 1, y2 = y1 + 1;
            const int x2r = min(x2, sw - 1), y2r = min(y2, sh - 1);
            const uint32_t* r1 = reinterpret_cast<const uint32_t*>(rgba + (int64_t)y1 * spitch);
            const uint32_t* r2 = reinterpret_cast<const uint32_t*>(rgba + (int64_t)y2r * spitch);
            const uint32_t c00 = r1[x1], c01 = r1[x2r], c10 = r2[x1], c11 = r2[x2r];
            const float w00 = ((float)x2 - src_x) * ((float)y2 - src_y);
            const float w01 = (src_x - (float)x1) * ((float)y2 - src_y);
            const float w10 = ((float)x2 - src_x) * (src_y - (float)y1);
            const float w11 = (src_x - (float)x1) * (src_y - (float)y1);
#pragma unroll
            for (int ch = 0; ch < 3; ch++) {
                const uint32_t sh8 = 8u * ch;
                float o = 0.f;
                o = __builtin_fmaf((float)((c00 >> sh8) & 255u), w00, o);
                o = __builtin_fmaf((float)((c01 >> sh8) & 255u), w01, o);
                o = __builtin_fmaf((float)((c10 >> sh8) & 255u), w10, o);
                o = __builtin_fmaf((float)((c11 >> sh8) & 255u), w11, o);
                rgb[p][ch] = (uint32_t)sat_u8_rne(o);
            }
        }
        store_quad(of, finish_quad_u8(rgb), 2 * qx, 2 * qy, true);  // rgb already 0..255
    }
}

hipError_t launch_resize_rgba_yuv420(const uint8_t* rgba, int sw, int sh, int64_t spitch, uint8_t* out, int dw, int dh,
                                     int64_t out_pitch, hipStream_t s) {
    if (dw <= 0 || dh <= 0 || (dw & 1) || (dh & 1)) return hipErrorInvalidValue;
    // resize.cpp:82-83,105: the kernel gets (float)(1.0 / (double(dsize) / src))
    const float fx = (float)(1.0 / ((double)dw / sw)), fy = (float)(1.0 / ((double)dh / sh));
    const int64_t total = (int64_t)(dw / 2) * (dh / 2);
    const int blocks = (int)std::min<int64_t>((total + 255) / 256, 256 * 16);
    hipLaunchKernelGGL(resize_rgba_yuv420_kernel, dim3(blocks), dim3(256), 0, s, rgba, sw, sh, spitch, fx, fy, out, dw,
                       dh, out_pitch);
    return hipGetLastError();
}

// Preview output (mapper.cpp:308-312): cv::cuda::resize(result, preview_output, preview_size,
// INTER_LINEAR) of the RGB result into a CV_8UC3 image — the same glob-kernel arithmetic as above,
// one lane per preview pixel, 3 bytes out.
__global__ void __launch_bounds__(256) resize_rgba_rgb_kernel(const uint8_t* __restrict__ rgba, int sw, int sh,
                                                              int64_t spitch, float fx, float fy, uint8_t* out, int dw,
                                                              int dh, int64_t out_pitch) {
    const int64_t total = (int64_t)dw * dh;
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < total; k += (int64_t)gridDim.x * blockDim.x) {
        const int y = (int)(k / dw), x = (int)(k - (int64_t)y * dw);
        const float src_x = (float)x * fx, src_y = (float)y * fy;
        const int x1 = (int)floorf(src_x), y1 = (int)floorf(src_y);
        const int x2 = x1 + 1, y2 = y1 + 1;
        const int x2r = min(x2, sw - 1), y2r = min(y2, sh - 1);
        const uint32_t* r1 = reinterpret_cast<const uint32_t*>(rgba + (int64_t)y1 * spitch);
        const uint32_t* r2 = reinterpret_cast<const uint32_t*>(rgba + (int64_t)y2r * spitch);
        const uint32_t c00 = r1[x1], c01 = r1[x2r], c10 = r2[x1], c11 = r2[x2r];
        const float w00 = ((float)x2 - src_x) * ((float)y2 - src_y);
        const float w01 = (src_x - (float)x1) * ((float)y2 - src_y);
        const float w10 = ((float)x2 - src_x) * (src_y - (float)y1);
        const float w11 = (src_x - (float)x1) * (src_y - (float)y1);
        uint8_t* o3 = out + (int64_t)y * out_pitch + 3 * (int64_t)x;
#pragma unroll
        for (int ch = 0; ch < 3; ch++) {
            const uint32_t sh8 = 8u * ch;
            float o = 0.f;
            o = __builtin_fmaf((float)((c00 >> sh8) & 255u), w00, o);
            o = __builtin_fmaf((float)((c01 >> sh8) & 255u), w01, o);
            o = __builtin_fmaf((float)((c10 >> sh8) & 255u), w10, o);
            o = __builtin_fmaf((float)((c11 >> sh8) & 255u), w11, o);
            o3[ch] = (uint8_t)sat_u8_rne(o);
        }
    }
}

hipError_t launch_resize_rgba_rgb(const uint8_t* rgba, int sw, int sh, int64_t spitch, uint8_t* out, int dw, int dh,
                                  int64_t out_pitch, hipStream_t s) {
    if (dw <= 0 || dh <= 0) return hipErrorInvalidValue;
    const float fx = (float)(1.0 / ((double)dw / sw)), fy = (float)(1.0 / ((double)dh / sh));
    const int64_t total = (int64_t)dw * dh;
    const int blocks = (int)std::min<int64_t>((total + 255) / 256, 256 * 16);
    hipLaunchKernelGGL(resize_rgba_rgb_kernel, dim3(blocks), dim3(256), 0, s, rgba, sw, sh, spitch, fx, fy, out, dw, dh,
                       out_pitch);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// Self-test: device saturating conversions (rint + clamp vs v_cvt_pk_u8_f32).
// ---------------------------------------------------------------------------------------------
__global__ void selftest_sat_kernel(const float* in, uint8_t* out, int n, int method) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float v = in[i];
    out[i] = method == 0 ? (uint8_t)sat_u8_rne(v) : (uint8_t)(__builtin_amdgcn_cvt_pk_u8_f32(v, 0, 0u) & 255u);
}

hipError_t launch_selftest_sat(const float* in, uint8_t* out, int n, int method, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(selftest_sat_kernel, dim3((n + 255) / 256), dim3(256), 0, s, in, out, n, method);
    return hipGetLastError();
}

}  // namespace octvr
