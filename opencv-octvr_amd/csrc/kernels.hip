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

#include "kernels.hpp"

namespace octvr {

// ---------------------------------------------------------------------------------------------
// Bilinear 15-bit weight table: initInterTab2D(INTER_LINEAR, true) (imgwarp.cpp:146-150,211-280),
// including the sum fix-up whose min/max search walks flat indices 3..6, i.e. into the NEXT cell
// (a positive excess can be "corrected" there and later overwritten): reproduced on a flat array.
// ---------------------------------------------------------------------------------------------
static short sat_s16(float v) {
    int iv = (int)rintf(v);
    return (short)(iv < -32768 ? -32768 : iv > 32767 ? 32767 : iv);
}

void bilinear_table(int16_t out[1024 * 4]) {
    float tab1[64];
    const float scale = 1.f / 32;
    for (int i = 0; i < 32; i++) {
        tab1[i * 2] = 1.f - i * scale;
        tab1[i * 2 + 1] = i * scale;
    }
    static short flat[1024 * 4 + 8];
    memset(flat, 0, sizeof flat);
    short* itab = flat;
    for (int i = 0; i < 32; i++)
        for (int j = 0; j < 32; j++, itab += 4) {
            int isum = 0;
            for (int k1 = 0; k1 < 2; k1++) {
                float vy = tab1[i * 2 + k1];
                for (int k2 = 0; k2 < 2; k2++) {
                    float v = vy * tab1[j * 2 + k2];
                    isum += itab[k1 * 2 + k2] = sat_s16(v * 32768);
                }
            }
            if (isum != 32768) {
                int diff = isum - 32768, Mk1 = 1, Mk2 = 1, mk1 = 1, mk2 = 1;
                for (int k1 = 1; k1 < 3; k1++)
                    for (int k2 = 1; k2 < 3; k2++) {
                        if (itab[k1 * 2 + k2] < itab[mk1 * 2 + mk2]) mk1 = k1, mk2 = k2;
                        else if (itab[k1 * 2 + k2] > itab[Mk1 * 2 + Mk2]) Mk1 = k1, Mk2 = k2;
                    }
                if (diff < 0) itab[Mk1 * 2 + Mk2] = (short)(itab[Mk1 * 2 + Mk2] - diff);
                else itab[mk1 * 2 + mk2] = (short)(itab[mk1 * 2 + mk2] - diff);
            }
        }
    memcpy(out, flat, 1024 * 4 * sizeof(short));
}

// ---------------------------------------------------------------------------------------------
// Pixel arithmetic shared by the kernels
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ int sat_u8_rne(float v) {
    // saturate_cast<uchar>(float): round half to even, clamp (NaN -> 0)
    if (!(v > 0.f)) return 0;
    if (v >= 255.f) return 255;
    return (int)__builtin_rintf(v);
}

// Own BT.601 YUV -> RGB (stands in for NPP nppiYUV420ToRGB_8u_P3AC4R, cudaimgproc/src/color.cpp:2269;
// NPP's arithmetic is closed, so this definition is pinned by the oracle only).
__device__ __forceinline__ void yuv_to_rgb(int y, int u, int v, int& r, int& g, int& b) {
    float Yf = (float)y, Uf = (float)u - 128.f, Vf = (float)v - 128.f;
    r = sat_u8_rne(Yf + 1.140f * Vf);
    g = sat_u8_rne(Yf - 0.394f * Uf - 0.581f * Vf);
    b = sat_u8_rne(Yf + 2.032f * Uf);
}

// Bilinear fixed-point sample of one camera at a composite entry: the cv::remap INTER_LINEAR /
// BORDER_CONSTANT rule (imgwarp.cpp:3812-4030) on the RGBA image NPP would have produced.
// Out-of-image taps contribute 0 (cval); result per channel = sat_u8((sum + 2^14) >> 15).
// Branch-free: out-of-image taps read a clamped (in-bounds) address with weight 0, and an invalid
// entry (no camera) gets all-zero weights, so every load of every pixel can be issued up front.
struct Taps {
    uint8_t y[4], u[4], v[4];
    int w[4];
};

__device__ __forceinline__ void gather_taps(const FrameSet& fs, uint32_t xy, uint32_t code, const short* tab,
                                            Taps& t) {
    const bool valid = (code & 0x8000u) != 0;
    const SourceFrame& f = fs.f[(code >> 10) & 31u];
    const int sx = (int)(xy & 0xFFFFu), sy = (int)(xy >> 16);
    const short* w = tab + (code & 1023u) * 4;
    const bool inx = sx + 1 < f.w, iny = sy + 1 < f.h;
    const int x0 = min(sx, f.w - 1), y0 = min(sy, f.h - 1);  // sx <= W_in (X may round up to W)
    const int x1 = inx ? sx + 1 : x0, y1 = iny ? sy + 1 : y0;
    const bool in0 = valid && sx < f.w && sy < f.h;
    t.w[0] = in0 ? w[0] : 0;
    t.w[1] = (valid && inx && sy < f.h) ? w[1] : 0;
    t.w[2] = (valid && iny && sx < f.w) ? w[2] : 0;
    t.w[3] = (valid && inx && iny) ? w[3] : 0;
    const int64_t p = f.pitch;
    const uint8_t* Y = f.yuv;
    const uint8_t* U = Y + (int64_t)f.h * p;
    const uint8_t* V = U + (f.w >> 1);
    const int64_t r0 = (int64_t)y0 * p, r1 = (int64_t)y1 * p;
    const int64_t c0 = (int64_t)(y0 >> 1) * p, c1 = (int64_t)(y1 >> 1) * p;
    t.y[0] = Y[r0 + x0];
    t.y[1] = Y[r0 + x1];
    t.y[2] = Y[r1 + x0];
    t.y[3] = Y[r1 + x1];
    t.u[0] = U[c0 + (x0 >> 1)];
    t.u[1] = U[c0 + (x1 >> 1)];
    t.u[2] = U[c1 + (x0 >> 1)];
    t.u[3] = U[c1 + (x1 >> 1)];
    t.v[0] = V[c0 + (x0 >> 1)];
    t.v[1] = V[c0 + (x1 >> 1)];
    t.v[2] = V[c1 + (x0 >> 1)];
    t.v[3] = V[c1 + (x1 >> 1)];
}

__device__ __forceinline__ void blend_taps(const Taps& t, int& r, int& g, int& b) {
    int ar = 0, ag = 0, ab = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        int cr, cg, cb;
        yuv_to_rgb(t.y[k], t.u[k], t.v[k], cr, cg, cb);
        ar += cr * t.w[k];
        ag += cg * t.w[k];
        ab += cb * t.w[k];
    }
    r = min(max((ar + (1 << 14)) >> 15, 0), 255);
    g = min(max((ag + (1 << 14)) >> 15, 0), 255);
    b = min(max((ab + (1 << 14)) >> 15, 0), 255);
}

__device__ __forceinline__ void load_table_lds(const int16_t* tab, short* lds) {
    // 8 KiB table -> LDS, 16 B per lane
    const int4* src = reinterpret_cast<const int4*>(tab);
    int4* dst = reinterpret_cast<int4*>(lds);
    for (int i = threadIdx.x; i < 1024 * 4 * 2 / 16; i += blockDim.x) dst[i] = src[i];
    __syncthreads();
}

// ---------------------------------------------------------------------------------------------
// LUT build: MapperTemplate::add_input (template.cpp:46-133), one thread per output pixel, FP64.
// bbox = {min_w, min_h, max_w, max_h} of valid pixels (int atomics, initialised by the host).
// ---------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) lut_build_kernel(CameraParams out, CameraParams in, int W, int H, float* map1,
                                                        float* map2, uint8_t* mask, int32_t* bbox) {
    __shared__ int s_bb[4];
    if (threadIdx.x < 4) s_bb[threadIdx.x] = (threadIdx.x < 2) ? INT32_MAX : -1;
    __syncthreads();
    const int64_t total = (int64_t)W * H;
    int lminw = INT32_MAX, lminh = INT32_MAX, lmaxw = -1, lmaxh = -1;
    for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
         idx += (int64_t)gridDim.x * blockDim.x) {
        const int h = (int)(idx / W), w = (int)(idx - (int64_t)h * W);
        double dx, dy;
        project_output_to_input(out, in, (double)w / W, (double)h / H, &dx, &dy);
        const float x = (float)dx, y = (float)dy;
        if (isnan(x) || isnan(y) || x < 0 || x >= 1.0f || y < 0 || y >= 1.0f) {
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

hipError_t launch_lut_build(const CameraParams& out, const CameraParams& in, int W, int H, float* map1, float* map2,
                            uint8_t* mask, int32_t* bbox, hipStream_t s) {
    const int64_t total = (int64_t)W * H;
    int blocks = (int)std::min<int64_t>((total + 255) / 256, 256 * 16);
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(lut_build_kernel, dim3(blocks), dim3(256), 0, s, out, in, W, H, map1, map2, mask, bbox);
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

// ---------------------------------------------------------------------------------------------
// Gain feed (GainCompensatorGPU::feed, exposure_compensate.cpp:223-263).  The working-scale images
// are nearest resizes of the warped ROIs (mapper.cpp:234-237); the host pre-resolves every working
// pixel that lies in some pair intersection into a sample entry of its camera, so one thread per
// sample computes the warped pixel's f32 norm (elementNorm, core/src/cuda/gpu_mat.cu:443-449).
// ---------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) gain_norm_kernel(FrameSet frames, const int16_t* tab,
                                                        const CompositeEntry* samples, int n, float* norms) {
    __shared__ short s_tab[1024 * 4];
    load_table_lds(tab, s_tab);
    for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < n; k += gridDim.x * blockDim.x) {
        const CompositeEntry e = samples[k];
        Taps t;
        gather_taps(frames, e.xy, e.code, s_tab, t);
        int r, g, b;
        blend_taps(t, r, g, b);
        norms[k] = sqrtf((float)(r * r + g * g + b * b));
    }
}

hipError_t launch_gain_norm(const FrameSet& frames, const int16_t* tab, const CompositeEntry* samples, int n_samples,
                            float* norms, hipStream_t s) {
    if (n_samples <= 0) return hipSuccess;
    const int blocks = std::min((n_samples + 255) / 256, 256 * 8);
    hipLaunchKernelGGL(gain_norm_kernel, dim3(blocks), dim3(256), 0, s, frames, tab, samples, n_samples, norms);
    return hipGetLastError();
}

// calcSum over the intersection mask (cudaarithm calcSum, f32 -> f64): one chunk per block, fixed
// reduction order, partial sums stored in chunk order (deterministic, no atomics).
__global__ void __launch_bounds__(256) gain_pairs_kernel(const float* norms, const uint2* idx, const GainChunk* chunks,
                                                         double* partials) {
    __shared__ double s_red[2][256];
    const GainChunk ch = chunks[blockIdx.x];
    double s1 = 0.0, s2 = 0.0;
    for (int e = ch.begin + (int)threadIdx.x; e < ch.end; e += blockDim.x) {
        const uint2 p = idx[e];
        s1 += (double)norms[p.x];
        s2 += (double)norms[p.y];
    }
    s_red[0][threadIdx.x] = s1;
    s_red[1][threadIdx.x] = s2;
    __syncthreads();
    for (int off = 128; off > 0; off >>= 1) {
        if ((int)threadIdx.x < off) {
            s_red[0][threadIdx.x] += s_red[0][threadIdx.x + off];
            s_red[1][threadIdx.x] += s_red[1][threadIdx.x + off];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        partials[2 * blockIdx.x] = s_red[0][0];
        partials[2 * blockIdx.x + 1] = s_red[1][0];
    }
}

hipError_t launch_gain_pairs(const float* norms, const uint2* pair_idx, const GainChunk* chunks, int n_chunks,
                             double* partials, hipStream_t s) {
    if (n_chunks <= 0) return hipSuccess;
    hipLaunchKernelGGL(gain_pairs_kernel, dim3(n_chunks), dim3(256), 0, s, norms, pair_idx, chunks, partials);
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

// Same LUImpl on a matrix held in LDS (n = 9..16: too large to keep in registers).
__device__ bool lu_solve_lds(double* A, double* b, int n, double* x) {
    const double eps = DBL_EPSILON * 100;
    for (int i = 0; i < n; i++) {
        int k = i;
        for (int j = i + 1; j < n; j++)
            if (fabs(A[j * n + i]) > fabs(A[k * n + i])) k = j;
        if (fabs(A[k * n + i]) < eps) return false;
        if (k != i) {
            for (int j = i; j < n; j++) {
                const double t = A[i * n + j];
                A[i * n + j] = A[k * n + j];
                A[k * n + j] = t;
            }
            const double t = b[i];
            b[i] = b[k];
            b[k] = t;
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
    for (int i = 0; i < n; i++) x[i] = b[i];
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
            return n <= 16 ? lu_solve_lds(A, b, n, x) : false;
    }
}

// One workgroup: the chunk partials, their pair ids and N are first staged into LDS by all lanes
// (parallel loads instead of a dependent chain on one lane), lane p then sums pair p's partials in
// chunk order, and lane 0 assembles I, A, b (exposure_compensate.cpp:265-296) and solves.
constexpr int kSolveMaxChunks = 4096;
__global__ void __launch_bounds__(256) gain_solve_kernel(const double* partials, const GainChunk* chunks, int n_chunks,
                                                         const int32_t* N, int n, double* gains) {
    __shared__ double s_part[2 * kSolveMaxChunks];
    __shared__ int s_pair[kSolveMaxChunks];
    __shared__ int s_N[16 * 16];
    __shared__ double s_I[16 * 16];
    __shared__ double s_A[16 * 16];
    __shared__ double s_b[16];
    __shared__ double s_x[16];
    const int tid = threadIdx.x;
    const int n_pairs = n * (n - 1) / 2;
    const int nc = min(n_chunks, kSolveMaxChunks);
    for (int c = tid; c < nc; c += blockDim.x) {
        s_part[2 * c] = partials[2 * c];
        s_part[2 * c + 1] = partials[2 * c + 1];
        s_pair[c] = chunks[c].pair;
    }
    for (int k = tid; k < n * n; k += blockDim.x) {
        s_N[k] = N[k];
        s_I[k] = 0.0;
    }
    __syncthreads();
    for (int p = tid; p < n_pairs; p += blockDim.x) {
        int i = 0, rem = p;  // pair p = (i, j), i < j, in the constructor's loop order
        while (rem >= n - 1 - i) {
            rem -= n - 1 - i;
            i++;
        }
        const int j = i + 1 + rem;
        // chunks are grouped by pair in pair order: binary search for the first chunk of p
        int lo = 0, hi = nc;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (s_pair[mid] < p) lo = mid + 1;
            else hi = mid;
        }
        double s1 = 0.0, s2 = 0.0;
        bool any = false;
        for (int c = lo; c < nc && s_pair[c] == p; c++) {
            s1 += s_part[2 * c];
            s2 += s_part[2 * c + 1];
            any = true;
        }
        if (any) {
            const int nij = s_N[i * n + j];
            s_I[i * n + j] = s1 / nij;
            s_I[j * n + i] = s2 / nij;
        }
    }
    __syncthreads();
    if (tid != 0) return;
    const double alpha = 0.01, beta = 100;
    for (int k = 0; k < n * n; k++) s_A[k] = 0.0;
    for (int i = 0; i < n; i++) s_b[i] = 0.0;
    for (int i = 0; i < n; i++)
        for (int j = 0; j < n; j++) {
            const int Nij = s_N[i * n + j];
            s_b[i] += beta * Nij;
            s_A[i * n + i] += beta * Nij;
            if (j == i) continue;
            s_A[i * n + i] += 2 * alpha * s_I[i * n + j] * s_I[i * n + j] * Nij;
            s_A[i * n + j] -= 2 * alpha * s_I[i * n + j] * s_I[j * n + i] * Nij;
        }
    if (!solve_dispatch(s_A, s_b, n, s_x))
        for (int i = 0; i < n; i++) s_x[i] = 1.0;
    for (int i = 0; i < n; i++) gains[i] = s_x[i];
}

hipError_t launch_gain_solve(const double* partials, const GainChunk* chunks, int n_chunks, const int32_t* N, int n,
                             double* gains, hipStream_t s) {
    if (n_chunks > kSolveMaxChunks) return hipErrorInvalidValue;
    hipLaunchKernelGGL(gain_solve_kernel, dim3(1), dim3(256), 0, s, partials, chunks, n_chunks, N, n, gains);
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
// for every 2x2 output quad the winning camera of each pixel is sampled from its YUV420P source
// (YUV->RGB per tap, 15-bit bilinear), gain-scaled (mul_scalar_with_mask, exposure_compensate.cu:
// 15-30: sat_u8(px * (float)g)) and written as YUV420P (own BT.601 in place of NPP RGBToYUV420).
// One workgroup per 128x8 tile; staged tiles read every tap from LDS (see kernels.hpp).  Tiles are
// walked grid-stride; blocks b, b+8, ... (one XCD under round-robin dispatch) take a contiguous
// band of tiles so their source boxes share that XCD's L2.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ void finish_quad(const int (&rgb)[4][3], const uint32_t (&cam)[4], const float* s_gain,
                                            uint8_t* out, uint8_t* outU, uint8_t* outV, int64_t out_pitch, int x,
                                            int y, int qxg, int qyg) {
    int Yo[4];
    float us = 0.f, vs = 0.f;
#pragma unroll
    for (int p = 0; p < 4; p++) {
        const float gf = s_gain[cam[p]];  // a black pixel stays black under any gain
        const int r = sat_u8_rne((float)rgb[p][0] * gf);
        const int g = sat_u8_rne((float)rgb[p][1] * gf);
        const int b = sat_u8_rne((float)rgb[p][2] * gf);
        const float R = (float)r, G = (float)g, B = (float)b;
        const float Yf = 0.299f * R + 0.587f * G + 0.114f * B;
        Yo[p] = sat_u8_rne(Yf);
        us = us + (0.492f * (B - Yf) + 128.f);
        vs = vs + (0.877f * (R - Yf) + 128.f);
    }
    *reinterpret_cast<uint16_t*>(out + (int64_t)y * out_pitch + x) = (uint16_t)(Yo[0] | (Yo[1] << 8));
    *reinterpret_cast<uint16_t*>(out + (int64_t)(y + 1) * out_pitch + x) = (uint16_t)(Yo[2] | (Yo[3] << 8));
    outU[(int64_t)qyg * out_pitch + qxg] = (uint8_t)sat_u8_rne(us * 0.25f);
    outV[(int64_t)qyg * out_pitch + qxg] = (uint8_t)sat_u8_rne(vs * 0.25f);
}

__device__ __forceinline__ uint32_t rgba_of(int y, int u, int v) {
    int r, g, b;
    yuv_to_rgb(y, u, v, r, g, b);
    return (uint32_t)r | ((uint32_t)g << 8) | ((uint32_t)b << 16);
}

template <bool DWORD_STAGE>
__global__ void __launch_bounds__(256) stitch_tiled_kernel(FrameSet frames, const int16_t* tab, TiledLut lut, int W,
                                                           int H, const double* gains, int use_gain, uint8_t* out,
                                                           int64_t out_pitch) {
    __shared__ __attribute__((aligned(16))) uint32_t s_rgb[kTileLdsBytes / 4];
    __shared__ short s_tab[1024 * 4];
    __shared__ float s_gain[kMaxCams];
    __shared__ TileSlot s_slot[kTileSlots];
    load_table_lds(tab, s_tab);
    if (threadIdx.x < kMaxCams) s_gain[threadIdx.x] = use_gain ? (float)gains[threadIdx.x] : 1.0f;
    __syncthreads();

    const int n_tiles = lut.tiles_x * lut.tiles_y;
    const int groups = 8;
    const int g = blockIdx.x % groups;
    const int blocks_in_g = (gridDim.x - g + groups - 1) / groups;
    const int t_begin = (int)((int64_t)n_tiles * g / groups);
    const int t_end = (int)((int64_t)n_tiles * (g + 1) / groups);
    uint8_t* outU = out + (int64_t)H * out_pitch;
    uint8_t* outV = outU + (W >> 1);
    const int tid = threadIdx.x;
    const int qx = tid & 63, qy = tid >> 6;

    for (int t = t_begin + (int)(blockIdx.x / groups); t < t_end; t += blocks_in_g) {
        const TileHdr hd = lut.hdr[t];
        const int tyi = t / lut.tiles_x, txi = t - tyi * lut.tiles_x;
        const int x = txi * kTileW + qx * 2, y = tyi * kTileH + qy * 2;
        const bool wide = (hd.nslots_flags & 0x100u) != 0;
        const int nslots = (int)(hd.nslots_flags & 7u);
        int rgb[4][3];
        uint32_t cam[4];
        if (wide) {
            const uint4* wp = reinterpret_cast<const uint4*>(lut.wide + hd.wide_off) + tid * 2;
            const uint4 e0 = wp[0], e1 = wp[1];
            const uint32_t xy[4] = {e0.x, e0.z, e1.x, e1.z};
            const uint32_t cd[4] = {e0.y, e0.w, e1.y, e1.w};
            Taps tp[4];
#pragma unroll
            for (int p = 0; p < 4; p++) gather_taps(frames, xy[p], cd[p], s_tab, tp[p]);
#pragma unroll
            for (int p = 0; p < 4; p++) {
                blend_taps(tp[p], rgb[p][0], rgb[p][1], rgb[p][2]);
                cam[p] = (cd[p] >> 10) & 31u;
            }
            if (x < W && y < H) finish_quad(rgb, cam, s_gain, out, outU, outV, out_pitch, x, y, x >> 1, y >> 1);
            continue;  // no LDS touched: no barrier needed
        }
        const uint4 e4 = reinterpret_cast<const uint4*>(lut.entries + (int64_t)t * kTilePx)[tid];
        __syncthreads();  // previous staged tile's LDS readers are done
        if (tid < kTileSlots) s_slot[tid] = lut.slots[(int64_t)t * kTileSlots + tid];
        // ---- convert every slot's box to RGBA in LDS, 4 horizontally adjacent pixels per step ----
        for (uint32_t k = tid; k < hd.stage_groups; k += 256) {
            uint32_t kk = k;
            TileSlot sl = lut.slots[(int64_t)t * kTileSlots];
#pragma unroll
            for (int q = 0; q < kTileSlots; q++) {
                if (q >= nslots) break;
                const TileSlot c = lut.slots[(int64_t)t * kTileSlots + q];
                const uint32_t n = (uint32_t)c.bw * c.bh / 4u;
                if (kk < n) {
                    sl = c;
                    break;
                }
                kk -= n;
            }
            const SourceFrame& f = frames.f[sl.cam];
            const uint32_t rowg = sl.bw / 4u;
            const uint32_t row = kk / rowg, col = kk - row * rowg;
            const int sx = sl.bx0 + (int)col * 4, sy = sl.by0 + (int)row;
            const uint8_t* Yp = f.yuv + (int64_t)sy * f.pitch + sx;
            const uint8_t* Up = f.yuv + (int64_t)(f.h + (sy >> 1)) * f.pitch + (sx >> 1);
            const uint8_t* Vp = Up + (f.w >> 1);
            uint32_t yq, uq, vq;
            if (DWORD_STAGE) {
                yq = *reinterpret_cast<const uint32_t*>(Yp);
                uq = *reinterpret_cast<const uint16_t*>(Up);
                vq = *reinterpret_cast<const uint16_t*>(Vp);
            } else {
                yq = (uint32_t)Yp[0] | ((uint32_t)Yp[1] << 8) | ((uint32_t)Yp[2] << 16) | ((uint32_t)Yp[3] << 24);
                uq = (uint32_t)Up[0] | ((uint32_t)Up[1] << 8);
                vq = (uint32_t)Vp[0] | ((uint32_t)Vp[1] << 8);
            }
            uint4 px;
            px.x = rgba_of(yq & 255u, uq & 255u, vq & 255u);
            px.y = rgba_of((yq >> 8) & 255u, uq & 255u, vq & 255u);
            px.z = rgba_of((yq >> 16) & 255u, (uq >> 8) & 255u, (vq >> 8) & 255u);
            px.w = rgba_of(yq >> 24, (uq >> 8) & 255u, (vq >> 8) & 255u);
            *reinterpret_cast<uint4*>(s_rgb + sl.lds / 4u + row * sl.bw + col * 4u) = px;
        }
        __syncthreads();
        const uint32_t ent[4] = {e4.x, e4.y, e4.z, e4.w};
#pragma unroll
        for (int p = 0; p < 4; p++) {
            const uint32_t e = ent[p];
            const uint32_t m = e >> 28;
            const TileSlot sl = s_slot[(e >> 26) & 3u];
            const int rx = (int)(e & 255u), ry = (int)((e >> 8) & 255u);
            const int dx = (int)(((m >> 1) | (m >> 3)) & 1u), dy = (int)(((m >> 2) | (m >> 3)) & 1u);
            const short* w = s_tab + ((e >> 16) & 1023u) * 4;
            const uint32_t* box = s_rgb + sl.lds / 4u;
            const int r0 = ry * sl.bw + rx, r1 = (ry + dy) * sl.bw + rx;
            const uint32_t c00 = box[r0], c01 = box[r0 + dx], c10 = box[r1], c11 = box[r1 + dx];
            const int w0 = (m & 1u) ? w[0] : 0, w1 = (m & 2u) ? w[1] : 0, w2 = (m & 4u) ? w[2] : 0,
                      w3 = (m & 8u) ? w[3] : 0;
#pragma unroll
            for (int ch = 0; ch < 3; ch++) {
                const int sh = ch * 8;
                const int acc = (int)((c00 >> sh) & 255u) * w0 + (int)((c01 >> sh) & 255u) * w1 +
                                (int)((c10 >> sh) & 255u) * w2 + (int)((c11 >> sh) & 255u) * w3;
                rgb[p][ch] = min(max((acc + (1 << 14)) >> 15, 0), 255);
            }
            cam[p] = sl.cam;
        }
        if (x < W && y < H) finish_quad(rgb, cam, s_gain, out, outU, outV, out_pitch, x, y, x >> 1, y >> 1);
    }
}

hipError_t launch_stitch(const FrameSet& frames, const int16_t* tab, const TiledLut& lut, int W, int H,
                         const double* gains, int use_gain, uint8_t* out, int64_t out_pitch, hipStream_t s) {
    const int tiles = lut.tiles_x * lut.tiles_y;
    int blocks = std::min(tiles, 256 * 8);
    blocks = std::max(8, (blocks + 7) / 8 * 8);
    // dword staging needs 4-byte aligned Y rows and 2-byte aligned chroma rows
    bool dw = true;
    for (int i = 0; i < kMaxCams; i++) {
        const SourceFrame& f = frames.f[i];
        if (!f.yuv) continue;
        if ((reinterpret_cast<uintptr_t>(f.yuv) & 3u) || (f.pitch & 3) || (f.w & 7)) dw = false;
    }
    if (dw)
        hipLaunchKernelGGL(stitch_tiled_kernel<true>, dim3(blocks), dim3(256), 0, s, frames, tab, lut, W, H, gains,
                           use_gain, out, out_pitch);
    else
        hipLaunchKernelGGL(stitch_tiled_kernel<false>, dim3(blocks), dim3(256), 0, s, frames, tab, lut, W, H, gains,
                           use_gain, out, out_pitch);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// Standalone cv::remap INTER_LINEAR u8 (cn = 1, 3, 4), BORDER_CONSTANT 0 — one output pixel per lane.
// ---------------------------------------------------------------------------------------------
template <int CN>
__global__ void __launch_bounds__(256) remap_u8_kernel(const int16_t* tab, const uint8_t* src, int sw, int sh,
                                                       int64_t spitch, const float* map1, const float* map2, int mw,
                                                       int mh, int64_t mpitch, float scale_x, float scale_y,
                                                       uint8_t* dst, int64_t dpitch) {
    __shared__ short s_tab[1024 * 4];
    load_table_lds(tab, s_tab);
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
        const short* w = s_tab + (((iy & 31) << 5) | (ix & 31)) * 4;
        int acc[CN];
#pragma unroll
        for (int k = 0; k < CN; k++) acc[k] = 0;
#pragma unroll
        for (int t = 0; t < 4; t++) {
            const int tx = sx + (t & 1), ty = sy + (t >> 1);
            if (tx >= 0 && tx < sw && ty >= 0 && ty < sh) {
                const uint8_t* p = src + (int64_t)ty * spitch + (int64_t)tx * CN;
#pragma unroll
                for (int k = 0; k < CN; k++) acc[k] += (int)p[k] * w[t];
            }
        }
        uint8_t* d = dst + (int64_t)y * dpitch + (int64_t)x * CN;
#pragma unroll
        for (int k = 0; k < CN; k++) d[k] = (uint8_t)min(max((acc[k] + (1 << 14)) >> 15, 0), 255);
    }
}

hipError_t launch_remap_u8(const int16_t* tab, const uint8_t* src, int sw, int sh, int64_t spitch, int cn,
                           const float* map1, const float* map2, int mw, int mh, int64_t mpitch, float scale_x,
                           float scale_y, uint8_t* dst, int64_t dpitch, hipStream_t s) {
    const int64_t total = (int64_t)mw * mh;
    int blocks = (int)std::min<int64_t>((total + 255) / 256, 256 * 8);
    if (blocks < 1) blocks = 1;
    switch (cn) {
        case 1:
            hipLaunchKernelGGL(remap_u8_kernel<1>, dim3(blocks), dim3(256), 0, s, tab, src, sw, sh, spitch, map1, map2,
                               mw, mh, mpitch, scale_x, scale_y, dst, dpitch);
            break;
        case 3:
            hipLaunchKernelGGL(remap_u8_kernel<3>, dim3(blocks), dim3(256), 0, s, tab, src, sw, sh, spitch, map1, map2,
                               mw, mh, mpitch, scale_x, scale_y, dst, dpitch);
            break;
        case 4:
            hipLaunchKernelGGL(remap_u8_kernel<4>, dim3(blocks), dim3(256), 0, s, tab, src, sw, sh, spitch, map1, map2,
                               mw, mh, mpitch, scale_x, scale_y, dst, dpitch);
            break;
        default:
            return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace octvr
