// kernels.hip — gfx950 kernels of the octVR remap + gain + composite path.
//
// Built with -ffp-contract=off: every f32/f64 expression rounds exactly as written, matching the
// reference's non-FMA x86 arithmetic (the oracle, oracle/octvr_oracle.c, is compiled the same way).
// No MFMA anywhere: this is a gather + per-pixel fixed-point blend.
#include <hip/hip_runtime.h>

#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstring>

#include "device_common.hpp"
#include "kernels.hpp"
#ifndef OCTVR_LU_BLOCK_MIN  // smallest n solved by the workgroup-parallel LU (below: one lane, registers)
#define OCTVR_LU_BLOCK_MIN 9
#endif
#ifndef OCTVR_FEED_VARIANT
#define OCTVR_FEED_VARIANT 0
#endif

namespace octvr {

// ---------------------------------------------------------------------------------------------
// LUT build: MapperTemplate::add_input (template.cpp:46-133), one thread per output pixel, FP64.
// bbox = {min_w, min_h, max_w, max_h} of valid pixels (int atomics, initialised by the host).
// ---------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) lut_build_kernel(const CameraParams* __restrict__ cams, int W, int H,
                                                        float* map1, float* map2, uint8_t* mask, int32_t* bbox,
                                                        uint8_t* visible) {
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
        project_output_to_input(out, in, (double)w / W, (double)h / H, &dx, &dy, visible ? &vis : nullptr);
        const float x = (float)dx, y = (float)dy;
        // visible_mask arbitration (template.cpp:86-116): a pixel an earlier camera's include mask
        // claimed (1) is rejected; one this camera's include mask claims first is marked 2 so the host
        // clears it from the earlier cameras' masks.
        const bool claimed = visible && visible[idx] == 1;
        if (visible && vis && !claimed) visible[idx] = 2;
        if (isnan(x) || isnan(y) || x < 0 || x >= 1.0f || y < 0 || y >= 1.0f || claimed) {
            mask[idx] = 0;
            map1[idx] = -1.0f;
            map2[idx] = -1.0f;
        } else {
            mask[idx] = 255;
            map1[idx] = x;
            map2[idx] = y;
            lminw = min(lminw, w);
            lmaxw = max(lmaxw, w);
            lminh = min(lminh, h);
            lmaxh = max(lmaxh, h);
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
                            int32_t* bbox, uint8_t* visible, hipStream_t s) {
    const int64_t total = (int64_t)W * H;
    int blocks = (int)std::min<int64_t>((total + 255) / 256, 256 * 16);
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(lut_build_kernel, dim3(blocks), dim3(256), 0, s, cams_dev, W, H, map1, map2, mask, bbox, visible);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// Composite LUT: the no-blend copy chain `warped_i.copyTo(result(roi_i), mask_i)` in camera order
// (mapper.cpp:268-277) resolved once per rig: the LAST camera whose ROI contains the pixel and whose
// LUT mask is non-zero wins; its map value is quantized exactly as RemapInvoker does.
// ---------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) composite_lut_kernel(const CamTemplate* cams, int n, int W, int H,
                                                            CompositeEntry* lut) {
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
            e = make_entry(c.map1[k], c.map2[k], (float)c.in_w, (float)c.in_h, i);
        }
        lut[idx] = e;
    }
}

hipError_t launch_composite_lut(const CamTemplate* cams_dev, int n, int W, int H, CompositeEntry* lut,
                                hipStream_t s) {
    const int64_t total = (int64_t)W * H;
    int blocks = (int)std::min<int64_t>((total + 255) / 256, 256 * 16);
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(composite_lut_kernel, dim3(blocks), dim3(256), 0, s, cams_dev, n, W, H, lut);
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

__device__ bool solve_dispatch(double* A, double* b, int n, double* x) {
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
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

__global__ void __launch_bounds__(256) gain_feed_kernel(FrameSet frames, const CompositeEntry* samples,
                                                        const uint16_t* partners, const GainChunk* chunks,
                                                        int n_chunks, const int32_t* N, int n,
                                                        unsigned long long* totals, uint32_t* tickets,
                                                        double* gains) {
    __shared__ int s_last;
    __shared__ double s_I[kGainMaxCams * kGainMaxCams];
    __shared__ double s_A[kGainMaxCams * kGainMaxCams];
    __shared__ double s_b[kGainMaxCams];
    __shared__ double s_x[kGainMaxCams];
    const int tid = threadIdx.x, lane = tid & 63;
    const GainChunk ch = chunks[blockIdx.x];
    double acc[kGainMaxCams];
#pragma unroll
    for (int j = 0; j < kGainMaxCams; j++) acc[j] = 0.0;
    // kGainChunk / 256 samples per thread, all gathers issued before any arithmetic
    constexpr int kPer = kGainChunk / 256;
    uint32_t pm[kPer];
    Taps t[kPer];
    const int cam = uniform(ch.cam);  // a chunk holds one camera's samples: its frame is wave-uniform
    const SourceFrame fr = frames.f[cam];
#pragma unroll
    for (int u = 0; u < kPer; u++) {
        const int k = ch.begin + u * 256 + tid;
        const bool in = k < ch.end;
        const CompositeEntry e = in ? samples[k] : CompositeEntry{0u, 0u};
        pm[u] = in ? partners[k] : 0u;
        gather_taps_frame(fr, e.xy, e.code, t[u]);
    }
#pragma unroll
    for (int u = 0; u < kPer; u++) {
        uint32_t rgb[3];
        bilerp_rgba(t[u].c[0], t[u].c[1], t[u].c[2], t[u].c[3], t[u].fx, t[u].fy, rgb);
        const double nv = (double)sqrtf((float)(rgb[0] * rgb[0] + rgb[1] * rgb[1] + rgb[2] * rgb[2]));
#pragma unroll
        for (int j = 0; j < kGainMaxCams; j++)
            if (pm[u] & (1u << j)) acc[j] += nv;
    }
    // exact sums: per wave, then per workgroup, then one u64 atomic per partner
    __shared__ double s_wsum[4][kGainMaxCams];
    for (int j = 0; j < n; j++) {
        double v = 0.0;
#pragma unroll
        for (int q = 0; q < kGainMaxCams; q++)
            if (q == j) v = acc[q];
        v = wave_sum(v);
        if (lane == 0) s_wsum[tid >> 6][j] = v;
    }
    __syncthreads();
    if (tid < n) {
        const double v = (s_wsum[0][tid] + s_wsum[1][tid]) + (s_wsum[2][tid] + s_wsum[3][tid]);
        if (v != 0.0)
            __hip_atomic_fetch_add(&totals[(cam * kGainMaxCams + tid) * kGainTotalStride],
                                   (unsigned long long)(v * 8388608.0), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // every wave's adds have completed before the workgroup takes its ticket
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
        const int xcd = blockIdx.x & 7;
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
#if OCTVR_FEED_VARIANT == 1
    if (tid < n) gains[tid] = s_I[tid];
    return;
#endif
    const double alpha = 0.01, beta = 100;
    if (tid < n) {  // row i of A and b, in the reference's j order (exposure_compensate.cpp:282-294)
        const int i = tid;
        double bi = 0.0, aii = 0.0;
        for (int j = 0; j < n; j++) {
            const int Nij = s_N[i * n + j];
            bi += beta * Nij;
            aii += beta * Nij;
            if (j == i) continue;
            aii += 2 * alpha * s_I[i * n + j] * s_I[i * n + j] * Nij;
            s_A[i * n + j] = 0.0 - 2 * alpha * s_I[i * n + j] * s_I[j * n + i] * Nij;
        }
        s_A[i * n + i] = aii;
        s_b[i] = bi;
    }
    __syncthreads();
    // cv::solve (lapack.cpp:1050-1275): one lane with the matrix in registers for n <= 8 (closed forms
    // n <= 3); the LU across the workgroup for 9..16
    bool ok;
    if (n < OCTVR_LU_BLOCK_MIN || n <= 3) {
        if (tid == 0) s_last = solve_dispatch(s_A, s_b, n, s_x) ? 1 : 0;
        __syncthreads();
        ok = s_last != 0;
    } else {
        ok = lu_solve_block(s_A, s_b, n, s_x);
    }
    if (tid < n) gains[tid] = ok ? s_x[tid] : 1.0;  // cv::solve failure leaves gains_ unspecified; 1 as the oracle
}

hipError_t launch_gain_feed(const FrameSet& frames, const CompositeEntry* samples, const uint16_t* partners,
                            const GainChunk* chunks, int n_chunks, const int32_t* N, int n,
                            unsigned long long* totals, uint32_t* tickets, double* gains, hipStream_t s) {
    if (n_chunks <= 0 || n > kGainMaxCams) return hipErrorInvalidValue;
    hipLaunchKernelGGL(gain_feed_kernel, dim3(n_chunks), dim3(256), 0, s, frames, samples, partners, chunks, n_chunks,
                       N, n, totals, tickets, gains);
    return hipGetLastError();
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
// The tile's slot descriptors as 16 raw dwords in scalar registers (the tile index is wave-uniform).
// Slot q: dword 4q = cam | bw << 16, 4q+1 = bh | lds << 16, 4q+2 = bx0 | by0 << 16, 4q+3 = chunk0.
// Only static indices and explicit selects touch it, so it never lands in scratch memory.
struct SlotSet {
    uint32_t w[4 * kTileSlots];
};
static_assert(sizeof(TileSlot) == 16, "TileSlot layout");

__device__ __forceinline__ uint32_t sel4(int q, uint32_t a0, uint32_t a1, uint32_t a2, uint32_t a3) {
    return q == 0 ? a0 : q == 1 ? a1 : q == 2 ? a2 : a3;
}

// The per-call FrameSet is the FIRST argument of the stitch kernels: index it in the kernarg
// segment directly (a wave-uniform index gives scalar loads; indexing the by-value parameter would
// copy it to scratch).
typedef __attribute__((address_space(4))) const SourceFrame kSourceFrame;
static_assert(offsetof(FrameSet, f) == 0, "FrameSet layout");
__device__ __forceinline__ SourceFrame kernarg_frame(uint32_t cam) {
    const kSourceFrame* kf = (const kSourceFrame*)__builtin_amdgcn_kernarg_segment_ptr();
    SourceFrame s;
    s.yuv = kf[cam].yuv;
    s.w = kf[cam].w;
    s.h = kf[cam].h;
    s.pitch = kf[cam].pitch;
    s.vig = kf[cam].vig;
    return s;
}

// One 8-pixel staging group of a tile: the YUV bytes it needs and its LDS destination.
struct StageGroup {
    uint32_t y0, y1;  // 8 Y bytes
    uint32_t uq, vq;  // 4 U bytes, 4 V bytes
    int32_t dst;      // dword index of the group's first RGBA pixel; -1 = none
    float4 g0, g1;    // VIG: vignette gains of the 8 pixels
};

// Loads of staging chunk c (wave-uniform) of a tile: 64 groups of 8 luma pixels inside one slot.
// The slot is found with scalar compares on the slots' first chunks; a lane's group k within the
// slot is row k / (bw/8), column k % (bw/8) of the slot's box.  Lanes past the slot's groups (and
// chunks past the tile's) read the box origin / frame start and are marked dst = -1.  With box
// columns 8-aligned, the Y load is 8-byte and the U / V loads 4-byte aligned (DWORD_STAGE).
template <bool DWORD_STAGE, bool VIG>
__device__ __forceinline__ void stage_load(const SlotSet& ss, int nslots, uint32_t nchunks, uint32_t stride, int c,
                                           StageGroup& sg) {
    const int lane = threadIdx.x & 63;
    const bool live_chunk = (uint32_t)c < nchunks;
    int q = 0;
#pragma unroll
    for (int j = 1; j < kTileSlots; j++) q += (j < nslots && c >= (int)(ss.w[4 * j + 3] & 0xFFFFu)) ? 1 : 0;
    const uint32_t d0 = sel4(q, ss.w[0], ss.w[4], ss.w[8], ss.w[12]);
    const uint32_t d1 = sel4(q, ss.w[1], ss.w[5], ss.w[9], ss.w[13]);
    const uint32_t d2 = sel4(q, ss.w[2], ss.w[6], ss.w[10], ss.w[14]);
    const uint32_t d3 = sel4(q, ss.w[3], ss.w[7], ss.w[11], ss.w[15]);
    const uint32_t cam = d0 & 31u, bw = d0 >> 16, bh = d1 & 0xFFFFu, lds = d1 >> 16;
    const uint32_t bx0 = d2 & 0xFFFFu, by0 = d2 >> 16, chunk0 = d3 & 0xFFFFu;
    const uint32_t rowg = max(1u, bw >> 3);
    const uint32_t groups = bw * bh >> 3;
    const uint32_t k = (uint32_t)(c - (int)chunk0) * 64u + (uint32_t)lane;
    const bool ok = live_chunk && k < groups;
    // k < 2^14, rowg <= 32: (k + 0.5) / rowg is >= 1/64 away from an integer, far above f32 error
    const float inv = __builtin_amdgcn_rcpf((float)rowg);
    const uint32_t row_f = (uint32_t)(((float)k + 0.5f) * inv);
    const uint32_t row_k = ok ? row_f : 0u, col_k = ok ? k - row_f * rowg : 0u;
    const SourceFrame f = kernarg_frame(live_chunk ? cam : 0u);
    // box groups past the image's right / bottom edge (w % 8 == 0: whole groups) stage RGBA 0:
    // they load from the box origin and are replaced by Y = 0, U = V = 128 (-> R = G = B = 0)
    const bool img = bx0 + col_k * 8u < (uint32_t)f.w && by0 + row_k < (uint32_t)f.h;
    const uint32_t row = img ? row_k : 0u, col = img ? col_k : 0u;
    const uint32_t p32 = (uint32_t)f.pitch;
    const gu8* base = (const gu8*)f.yuv;
    const gu8* Yb = base + (int64_t)by0 * f.pitch + bx0;  // by0, bx0 even: chroma rows / columns exact
    const gu8* Ub = base + (int64_t)(f.h + (int)(by0 >> 1)) * f.pitch + (bx0 >> 1);
    const gu8* Vb = Ub + (f.w >> 1);
    const uint32_t oy = row * p32 + col * 8u, oc = (row >> 1) * p32 + col * 4u;
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
    if (!img) {
        sg.y0 = sg.y1 = 0u;
        sg.uq = sg.vq = 0x80808080u;
    }
    sg.dst = ok ? (int32_t)(lds + row_k * stride + col_k * 8u) : -1;
    if (VIG) {  // 8 gains (32-byte aligned: w % 8 == 0); a camera without vignette reads 1.0 gains
        const float* gv = f.vig ? f.vig + (int64_t)(by0 + row) * f.w + bx0 + col * 8u : nullptr;
        sg.g0 = gv ? *reinterpret_cast<const float4*>(gv) : make_float4(1.f, 1.f, 1.f, 1.f);
        sg.g1 = gv ? *reinterpret_cast<const float4*>(gv + 4) : make_float4(1.f, 1.f, 1.f, 1.f);
    }
}

template <bool VIG>
__device__ __forceinline__ void stage_store(const StageGroup& sg, uint32_t* s_rgb) {
    if (sg.dst < 0) return;
    uint4 a, b;
    yuv2_to_rgba(sg.y0 & 255u, (sg.y0 >> 8) & 255u, sg.uq & 255u, sg.vq & 255u, a.x, a.y);
    yuv2_to_rgba((sg.y0 >> 16) & 255u, sg.y0 >> 24, (sg.uq >> 8) & 255u, (sg.vq >> 8) & 255u, a.z, a.w);
    yuv2_to_rgba(sg.y1 & 255u, (sg.y1 >> 8) & 255u, (sg.uq >> 16) & 255u, (sg.vq >> 16) & 255u, b.x, b.y);
    yuv2_to_rgba((sg.y1 >> 16) & 255u, sg.y1 >> 24, sg.uq >> 24, sg.vq >> 24, b.z, b.w);
    if (VIG) {
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

#ifndef OCTVR_STITCH_BLOCKS_PER_CU
#define OCTVR_STITCH_BLOCKS_PER_CU 6
#endif
constexpr int kStitchBlocksPerCU = OCTVR_STITCH_BLOCKS_PER_CU;
#ifndef OCTVR_STAGE_REGS
#define OCTVR_STAGE_REGS 1
#endif
#ifndef OCTVR_STAGE_SKIP
#define OCTVR_STAGE_SKIP 1
#endif
#ifndef OCTVR_INNER_PAIR
#define OCTVR_INNER_PAIR 0
#endif
constexpr int kStageRegs = OCTVR_STAGE_REGS;  // staging groups per lane loaded one tile ahead (256 per reg)

// Software pipeline over a block's tiles (t, t + step, ...):
//   iteration of tile t:  stage tile t's YUV (loaded during the previous iteration) into LDS,
//                         read tile t+step's metadata (loaded one iteration earlier) into SGPRs,
//                         issue tile t+step's entries + YUV loads and tile t+2*step's metadata load,
//                         then compute tile t from LDS while all of those are in flight.
// No global load is waited on in the iteration that issues it, and every iteration issues the
// same vector-memory operations in the same order (clamped addresses instead of branches), so the
// compiler's wait counts stay exact across the loop.
//
// Metadata in flight is one VGPR: lanes 0-3 hold the header's dwords, lanes 4-19 the 4 slots'.
struct TileMeta {
    int t;
    TileHdr hd;
    SlotSet ss;
};

__device__ __forceinline__ uint32_t meta_issue(const TiledLut& lut, int t, int t_end) {  // t: staged item
    const int lane = threadIdx.x & 63;
    const int tt = t < t_end ? t : 0;
    const uint32_t* p = lane < 4 ? reinterpret_cast<const uint32_t*>(lut.hdr + tt) + lane
                                 : reinterpret_cast<const uint32_t*>(lut.slots + (int64_t)tt * kTileSlots) +
                                       (lane < 20 ? lane - 4 : 0);
    return *p;
}

__device__ __forceinline__ TileMeta meta_read(uint32_t v, int t) {
    TileMeta m;
    m.t = t;
    m.hd.tile = (uint32_t)__builtin_amdgcn_readlane((int)v, 0);
    m.hd.nslots = (uint32_t)__builtin_amdgcn_readlane((int)v, 1);
    m.hd.stage_groups = (uint32_t)__builtin_amdgcn_readlane((int)v, 2);
    m.hd.stride = (uint32_t)__builtin_amdgcn_readlane((int)v, 3);
    uint32_t w[4 * kTileSlots];
#pragma unroll
    for (int q = 0; q < 4 * kTileSlots; q++) w[q] = (uint32_t)__builtin_amdgcn_readlane((int)v, 4 + q);
#pragma unroll
    for (int q = 0; q < 4 * kTileSlots; q++) m.ss.w[q] = w[q];
    return m;
}

struct TileData {
    uint4 e4;
    StageGroup sg[kStageRegs];
};

template <bool DWORD_STAGE, bool VIG>
__device__ __forceinline__ void data_issue(const FrameSet& frames, const TiledLut& lut, const TileMeta& m, int t_end,
                                           TileData& d) {
    const bool live = m.t < t_end;
    const int tid = threadIdx.x;
    const int wave = uniform(tid >> 6);
    d.e4 = reinterpret_cast<const uint4*>(lut.entries + (int64_t)(live ? m.t : 0) * kTilePx)[tid];
    const uint32_t nchunks = live ? ((m.hd.nslots >> 8) & 0xFFu) : 0u;
#pragma unroll
    for (int r = 0; r < kStageRegs; r++) {
#if OCTVR_STAGE_SKIP
        if ((uint32_t)(r * 4 + wave) >= nchunks) {  // wave-uniform: no loads for a chunk the tile lacks
            d.sg[r].dst = -1;
            continue;
        }
#endif
        stage_load<DWORD_STAGE, VIG>(m.ss, (int)(m.hd.nslots & 0xFFu), nchunks, m.hd.stride, r * 4 + wave, d.sg[r]);
    }
}

// The composite's two sinks.  MODE 0: gain + RGB -> YUV420P into the output frame (blend = 0).
// MODE 1: gain-applied RGBA into the camera's level-0 pyramid image (blend > 0; the warped image
// Mapper::stitch hands to the blender, mapper.cpp:233-262); pixels outside the camera's aligned ROI
// are dropped.  Either way a quad's result is 4 dwords.
template <int MODE>
__device__ __forceinline__ QuadOut finish_any(const uint32_t (&rgb)[4][3], const float (&gain)[4]) {
    if constexpr (MODE == 0) {
        return finish_quad(rgb, gain);
    } else {
        uint32_t px[4];
#pragma unroll
        for (int p = 0; p < 4; p++) {
            uint32_t v = pack_u8((float)rgb[p][0] * gain[p], 0, 0u);
            v = pack_u8((float)rgb[p][1] * gain[p], 1, v);
            px[p] = pack_u8((float)rgb[p][2] * gain[p], 2, v);
        }
        return QuadOut{px[0], px[1], px[2], px[3]};
    }
}

struct RgbaSink {
    __amdgpu_buffer_rsrc_t rsrc;
    const MbCamLevel* cams;
};

__device__ __forceinline__ void store_rgba(const RgbaSink& o, const QuadOut& q, uint32_t cam, int x, int y, bool in) {
    const MbCamLevel* c = o.cams + cam;
    const int xl = x - c->ox, yl = y - c->oy;
    const bool ok = in && xl >= 0 && yl >= 0 && xl < c->w && yl < c->h;  // w, h even: whole quads
    const uint32_t off = ok ? c->g_off + (uint32_t)yl * c->g_pitch + (uint32_t)xl * 4u : kDropOffset;
    typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
    const u32x2 r0 = {q.y01, q.y23}, r1 = {q.u, q.v};
    __builtin_amdgcn_raw_buffer_store_b64(r0, o.rsrc, off, 0, 0);
    __builtin_amdgcn_raw_buffer_store_b64(r1, o.rsrc, ok ? off + c->g_pitch : kDropOffset, 0, 0);
}

template <int MODE>
__device__ __forceinline__ void store_any(const OutFrame& of, const RgbaSink& ro, const QuadOut& q, uint32_t cam,
                                          int x, int y, bool in) {
    if constexpr (MODE == 0)
        store_quad(of, q, x, y, in);
    else
        store_rgba(ro, q, cam, x, y, in);
}

// Staged tiles.  The staged items are split into 8 contiguous bands, one per XCD under round-robin
// dispatch (blocks b, b+8, ...), so neighbouring tiles' source boxes share that XCD's L2.
template <bool DWORD_STAGE, int MODE, bool VIG>
__global__ void __launch_bounds__(256, kStitchBlocksPerCU) stitch_tiled_kernel(FrameSet frames, TiledLut lut, int W, int H,
                                                              const double* gains, int use_gain, uint8_t* out,
                                                              int64_t out_pitch, RgbaOut rgba) {
    __shared__ __attribute__((aligned(16))) uint32_t s_rgb[kTileLdsBytes / 4];
    __shared__ float s_gain[kMaxCams];
    __shared__ float s_slot_gain[kTileSlots];

    const int groups = kStitchBands;
    const int g = blockIdx.x % groups;
    const int step = (gridDim.x - g + groups - 1) / groups;
    const int t_begin = lut.bands[g];
    const int t_end = lut.bands[g + 1];
    OutFrame of{};
    RgbaSink ro{};
    if constexpr (MODE == 0)
        of = make_out_frame(out, W, H, out_pitch);
    else
        ro = RgbaSink{__builtin_amdgcn_make_buffer_rsrc(rgba.base, 0, (int)rgba.bytes, 0x00020000), rgba.cams};
    const int tid = threadIdx.x;
    const int qx = tid & 63, qy = tid >> 6;

    if (tid < kMaxCams) s_gain[tid] = use_gain ? (float)gains[tid] : 1.0f;
    if (tid < kTileZeroDwords) s_rgb[tid] = 0u;
    const int t0 = t_begin + (int)(blockIdx.x / groups);
    TileMeta cur = meta_read(meta_issue(lut, t0, t_end), t0);
    __syncthreads();
    TileData d;
    data_issue<DWORD_STAGE, VIG>(frames, lut, cur, t_end, d);
    uint32_t mv = meta_issue(lut, t0 + step, t_end);
    // opaque copies of the prologue loads: the loop-header phis then merge a load with a non-load,
    // so the compiler cannot fold them into one load at the header (waited on right there)
    asm volatile("" : "+v"(mv));
    asm volatile("" : "+v"(d.e4.x), "+v"(d.e4.y), "+v"(d.e4.z), "+v"(d.e4.w));
#pragma unroll
    for (int r = 0; r < kStageRegs; r++)
        asm volatile("" : "+v"(d.sg[r].y0), "+v"(d.sg[r].y1), "+v"(d.sg[r].uq), "+v"(d.sg[r].vq));

    // the previous tile's output, stored at the top of the next iteration: every store is then
    // older than the loads it shares the iteration with (vmcnt waits on a load that is older than
    // a store must drain everything, as loads and stores complete out of order)
    QuadOut prev{0u, 0u, 0u, 0u};
    int px = 0, py = 0;
    uint32_t pcam = 0;
    bool pin = false;
    while (cur.t < t_end) {
        const int x = (int)(cur.hd.tile & 0xFFFFu) * kTileW + qx * 2, y = (int)(cur.hd.tile >> 16) * kTileH + qy * 2;
        const uint32_t S = cur.hd.stride;
        const uint4 e4 = d.e4;
        __syncthreads();  // the previous tile's LDS readers are done
        const TileMeta nxt = meta_read(mv, cur.t + step);
        if (tid < kTileSlots) {
            const uint32_t cam = sel4(tid, cur.ss.w[0], cur.ss.w[4], cur.ss.w[8], cur.ss.w[12]) & 31u;
            s_slot_gain[tid] = s_gain[cam];
        }
#pragma unroll
        for (int r = 0; r < kStageRegs; r++) stage_store<VIG>(d.sg[r], s_rgb);
        const uint32_t nch = (cur.hd.nslots >> 8) & 0xFFu;
        if (nch > (uint32_t)(kStageRegs * 4)) {  // large boxes only: the other chunks now
            const int wave = uniform(tid >> 6);
            int c = kStageRegs * 4 + wave;
#if OCTVR_INNER_PAIR
            for (; c + 4 < (int)nch; c += 8) {  // two chunks' loads in flight before their stores
                StageGroup sa, sb;
                stage_load<DWORD_STAGE, VIG>(cur.ss, (int)(cur.hd.nslots & 0xFFu), nch, S, c, sa);
                stage_load<DWORD_STAGE, VIG>(cur.ss, (int)(cur.hd.nslots & 0xFFu), nch, S, c + 4, sb);
                stage_store<VIG>(sa, s_rgb);
                stage_store<VIG>(sb, s_rgb);
            }
#endif
            for (; c < (int)nch; c += 4) {
                StageGroup sg;
                stage_load<DWORD_STAGE, VIG>(cur.ss, (int)(cur.hd.nslots & 0xFFu), nch, S, c, sg);
                stage_store<VIG>(sg, s_rgb);
            }
        }
        __syncthreads();
        store_any<MODE>(of, ro, prev, pcam, px, py, pin);
        data_issue<DWORD_STAGE, VIG>(frames, lut, nxt, t_end, d);
        mv = meta_issue(lut, cur.t + 2 * step, t_end);
        const uint32_t ent[4] = {e4.x, e4.y, e4.z, e4.w};
        uint32_t rgb[4][3];
        float gain[4];
#pragma unroll
        for (int p = 0; p < 4; p++) {
            const uint32_t e = ent[p];
            // taps (x, y), (x+1, y) and (x, y+1), (x+1, y+1): two ds_read2_b32, no per-tap masking
            const uint8_t* r0 = reinterpret_cast<const uint8_t*>(s_rgb) + (e & 0x7FFFu);
            const uint8_t* r1 = r0 + 4u * S;
            const uint32_t c00 = reinterpret_cast<const uint32_t*>(r0)[0];
            const uint32_t c01 = reinterpret_cast<const uint32_t*>(r0)[1];
            const uint32_t c10 = reinterpret_cast<const uint32_t*>(r1)[0];
            const uint32_t c11 = reinterpret_cast<const uint32_t*>(r1)[1];
            bilerp_rgba(c00, c01, c10, c11, (e >> 15) & 31u, (e >> 20) & 31u, rgb[p]);
            gain[p] = s_slot_gain[(e >> 25) & 3u];
            if (MODE == 1 && (e & kEntryNoGain)) gain[p] = 1.0f;
        }
        prev = finish_any<MODE>(rgb, gain);
        px = x;
        py = y;
        pcam = (cur.hd.nslots >> 16) & 31u;
        pin = x < W && y < H;
        cur = nxt;
    }
    store_any<MODE>(of, ro, prev, pcam, px, py, pin);
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
    if constexpr (MODE == 0)
        of = make_out_frame(out, W, H, out_pitch);
    else
        ro = RgbaSink{__builtin_amdgcn_make_buffer_rsrc(rgba.base, 0, (int)rgba.bytes, 0x00020000), rgba.cams};
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
    float gain[4];
#pragma unroll
    for (int p = 0; p < 4; p++) {
        bilerp_rgba(tp[p].c[0], tp[p].c[1], tp[p].c[2], tp[p].c[3], tp[p].fx, tp[p].fy, rgb[p]);
        gain[p] = (MODE == 1 && (cd[p] & kCodeNoGain)) ? 1.0f : s_gain[(cd[p] >> 10) & 31u];
    }
    const uint32_t cam = MODE == 1 ? (uint32_t)uniform((int)lut.wide_cams[blockIdx.x]) : 0u;
    store_any<MODE>(of, ro, finish_any<MODE>(rgb, gain), cam, x, y, x < W && y < H);
}

template <int MODE>
static hipError_t launch_composite(const FrameSet& frames, const TiledLut& lut, int W, int H, const double* gains,
                                   int use_gain, uint8_t* out, int64_t out_pitch, const RgbaOut& rgba, hipStream_t s) {
    if (lut.n_items > 0) {
        // one resident wave of workgroups (256 CUs x kStitchBlocksPerCU: 25 KiB LDS each), each
        // walking its XCD band's items
        int blocks = std::min(lut.n_items, 256 * kStitchBlocksPerCU);
        blocks = std::max(8, (blocks + 7) / 8 * 8);
        // wide staging loads need 8-byte aligned Y rows (then U / V rows are 4-byte aligned)
        bool dw = true, vig = false;
        for (int i = 0; i < kMaxCams; i++) {
            const SourceFrame& f = frames.f[i];
            if (!f.yuv) continue;
            if ((reinterpret_cast<uintptr_t>(f.yuv) & 7u) || (f.pitch & 7) || (f.w & 7)) dw = false;
            vig |= f.vig != nullptr;
        }
#define OCTVR_LAUNCH_TILED(DW, V)                                                                          \
    hipLaunchKernelGGL((stitch_tiled_kernel<DW, MODE, V>), dim3(blocks), dim3(256), 0, s, frames, lut, W, H, \
                       gains, use_gain, out, out_pitch, rgba)
        if (dw && !vig)
            OCTVR_LAUNCH_TILED(true, false);
        else if (dw)
            OCTVR_LAUNCH_TILED(true, true);
        else if (!vig)
            OCTVR_LAUNCH_TILED(false, false);
        else
            OCTVR_LAUNCH_TILED(false, true);
#undef OCTVR_LAUNCH_TILED
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    if (lut.n_wide > 0)
        hipLaunchKernelGGL(stitch_wide_kernel<MODE>, dim3(lut.n_wide), dim3(256), 0, s, frames, lut, W, H, gains,
                           use_gain, out, out_pitch, rgba);
    return hipGetLastError();
}

hipError_t launch_stitch(const FrameSet& frames, const TiledLut& lut, int W, int H, const double* gains,
                         int use_gain, uint8_t* out, int64_t out_pitch, hipStream_t s) {
    return launch_composite<0>(frames, lut, W, H, gains, use_gain, out, out_pitch, RgbaOut{}, s);
}

hipError_t launch_mb_remap(const FrameSet& frames, const TiledLut& lut, const double* gains, int use_gain,
                           const RgbaOut& out, hipStream_t s) {
    // W, H: no level-grid bound of its own (the per-camera ROI check drops what lies outside)
    return launch_composite<1>(frames, lut, 1 << 16, 1 << 16, gains, use_gain, nullptr, 0, out, s);
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
    const float one[4] = {1.f, 1.f, 1.f, 1.f};
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
        store_quad(of, finish_quad(rgb, one), 2 * qx, 2 * qy, true);
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
