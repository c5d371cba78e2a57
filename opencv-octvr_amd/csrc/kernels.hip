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
__device__ __forceinline__ void sample_rgb(const SourceFrame& f, uint32_t xy, uint32_t code, const short* tab,
                                           int& r, int& g, int& b) {
    const int sx = (int)(xy & 0xFFFFu), sy = (int)(xy >> 16);
    const int a = (int)(code & 1023u);
    const short* w = tab + a * 4;
    const int64_t pitch = f.pitch;
    const uint8_t* Y = f.yuv;
    const uint8_t* U = f.yuv + (int64_t)f.h * pitch;
    const uint8_t* V = U + (f.w >> 1);
    int ar = 0, ag = 0, ab = 0;
#pragma unroll
    for (int t = 0; t < 4; t++) {
        const int tx = sx + (t & 1), ty = sy + (t >> 1);
        if (tx < f.w && ty < f.h) {  // sx, sy >= 0 for every valid entry
            int yy = Y[(int64_t)ty * pitch + tx];
            int uu = U[(int64_t)(ty >> 1) * pitch + (tx >> 1)];
            int vv = V[(int64_t)(ty >> 1) * pitch + (tx >> 1)];
            int cr, cg, cb;
            yuv_to_rgb(yy, uu, vv, cr, cg, cb);
            const int wt = w[t];
            ar += cr * wt;
            ag += cg * wt;
            ab += cb * wt;
        }
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
// Gain feed (GainCompensatorGPU::feed, exposure_compensate.cpp:223-263): for every overlap pixel of
// every camera pair (i<j), the warped working-scale pixel of both cameras (nearest resize of the
// warped ROI, mapper.cpp:234-237, pre-resolved on the host into sample entries), its f32 RGB norm
// (elementNorm, core/src/cuda/gpu_mat.cu:443-449) and the masked f64 sums (calcSum).  One chunk per
// block; partial sums go to `partials` in chunk order (deterministic, no atomics).
// ---------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) gain_feed_kernel(FrameSet frames, const int16_t* tab,
                                                        const CompositeEntry* sa, const CompositeEntry* sb,
                                                        const GainChunk* chunks, double* partials) {
    __shared__ short s_tab[1024 * 4];
    __shared__ double s_red[2][256];
    load_table_lds(tab, s_tab);
    const GainChunk ch = chunks[blockIdx.x];
    double s1 = 0.0, s2 = 0.0;
    for (int e = ch.begin + (int)threadIdx.x; e < ch.end; e += blockDim.x) {
        const CompositeEntry a = sa[e], b = sb[e];
        int r, g, bl;
        float na = 0.f, nb = 0.f;
        if (a.code & 0x8000u) {
            sample_rgb(frames.f[(a.code >> 10) & 31u], a.xy, a.code, s_tab, r, g, bl);
            na = sqrtf((float)(r * r + g * g + bl * bl));
        }
        if (b.code & 0x8000u) {
            sample_rgb(frames.f[(b.code >> 10) & 31u], b.xy, b.code, s_tab, r, g, bl);
            nb = sqrtf((float)(r * r + g * g + bl * bl));
        }
        s1 += (double)na;
        s2 += (double)nb;
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

hipError_t launch_gain_feed(const FrameSet& frames_dev, const int16_t* tab, const CompositeEntry* samples_a,
                            const CompositeEntry* samples_b, const GainChunk* chunks, int n_chunks,
                            double* partials, hipStream_t s) {
    if (n_chunks <= 0) return hipSuccess;
    hipLaunchKernelGGL(gain_feed_kernel, dim3(n_chunks), dim3(256), 0, s, frames_dev, tab, samples_a, samples_b,
                       chunks, partials);
    return hipGetLastError();
}

// cv::solve (lapack.cpp:1050-1275): closed forms for n <= 3, LUImpl (matrix_decomp.cpp:50-110) above.
__device__ bool solve_small(double* A, double* b, int n, double* x) {
#define Sd(y, xx) A[(y) * n + (xx)]
    if (n == 1) {
        double d = Sd(0, 0);
        if (d == 0.) return false;
        x[0] = b[0] / d;
        return true;
    }
    if (n == 2) {
        double d = (double)Sd(0, 0) * Sd(1, 1) - (double)Sd(0, 1) * Sd(1, 0);
        if (d == 0.) return false;
        d = 1. / d;
        double t = (b[0] * Sd(1, 1) - b[1] * Sd(0, 1)) * d;
        x[1] = (b[1] * Sd(0, 0) - b[0] * Sd(1, 0)) * d;
        x[0] = t;
        return true;
    }
    if (n == 3) {
        double d = Sd(0, 0) * ((double)Sd(1, 1) * Sd(2, 2) - (double)Sd(1, 2) * Sd(2, 1)) -
                   Sd(0, 1) * ((double)Sd(1, 0) * Sd(2, 2) - (double)Sd(1, 2) * Sd(2, 0)) +
                   Sd(0, 2) * ((double)Sd(1, 0) * Sd(2, 1) - (double)Sd(1, 1) * Sd(2, 0));
        if (d == 0.) return false;
        d = 1. / d;
        double t0 = ((Sd(1, 1) * Sd(2, 2) - Sd(1, 2) * Sd(2, 1)) * b[0] + (Sd(0, 2) * Sd(2, 1) - Sd(0, 1) * Sd(2, 2)) * b[1] +
                     (Sd(0, 1) * Sd(1, 2) - Sd(0, 2) * Sd(1, 1)) * b[2]) * d;
        double t1 = ((Sd(1, 2) * Sd(2, 0) - Sd(1, 0) * Sd(2, 2)) * b[0] + (Sd(0, 0) * Sd(2, 2) - Sd(0, 2) * Sd(2, 0)) * b[1] +
                     (Sd(0, 2) * Sd(1, 0) - Sd(0, 0) * Sd(1, 2)) * b[2]) * d;
        double t2 = ((Sd(1, 0) * Sd(2, 1) - Sd(1, 1) * Sd(2, 0)) * b[0] + (Sd(0, 1) * Sd(2, 0) - Sd(0, 0) * Sd(2, 1)) * b[1] +
                     (Sd(0, 0) * Sd(1, 1) - Sd(0, 1) * Sd(1, 0)) * b[2]) * d;
        x[0] = t0;
        x[1] = t1;
        x[2] = t2;
        return true;
    }
#undef Sd
    const double eps = DBL_EPSILON * 100;
    for (int i = 0; i < n; i++) {
        int k = i;
        for (int j = i + 1; j < n; j++)
            if (fabs(A[j * n + i]) > fabs(A[k * n + i])) k = j;
        if (fabs(A[k * n + i]) < eps) return false;
        if (k != i) {
            for (int j = i; j < n; j++) {
                double t = A[i * n + j];
                A[i * n + j] = A[k * n + j];
                A[k * n + j] = t;
            }
            double t = b[i];
            b[i] = b[k];
            b[k] = t;
        }
        double d = -1 / A[i * n + i];
        for (int j = i + 1; j < n; j++) {
            double alpha = A[j * n + i] * d;
            for (int kk = i + 1; kk < n; kk++) A[j * n + kk] += alpha * A[i * n + kk];
            b[j] += alpha * b[i];
        }
        A[i * n + i] = -d;
    }
    for (int i = n - 1; i >= 0; i--) {
        double s = b[i];
        for (int kk = i + 1; kk < n; kk++) s -= A[i * n + kk] * b[kk];
        b[i] = s * A[i * n + i];
    }
    for (int i = 0; i < n; i++) x[i] = b[i];
    return true;
}

// I(i,j), A, b assembly (exposure_compensate.cpp:265-296) and the solve, on one lane.
__global__ void gain_solve_kernel(const double* partials, const GainChunk* chunks, int n_chunks,
                                  const int32_t* pair_ij, const int32_t* N, int n, double* gains) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    double I[kMaxCams * kMaxCams];
    double A[kMaxCams * kMaxCams];
    double b[kMaxCams], x[kMaxCams];
    for (int k = 0; k < n * n; k++) I[k] = 0.0;
    // chunks of one pair are contiguous and in order
    int c = 0;
    const int n_pairs = n * (n - 1) / 2;
    for (int p = 0; p < n_pairs; p++) {
        const int i = pair_ij[2 * p], j = pair_ij[2 * p + 1];
        double s1 = 0.0, s2 = 0.0;
        bool any = false;
        while (c < n_chunks && chunks[c].pair == p) {
            s1 += partials[2 * c];
            s2 += partials[2 * c + 1];
            any = true;
            c++;
        }
        const int nij = N[i * n + j];
        if (nij > 0 && any) {
            I[i * n + j] = s1 / nij;
            I[j * n + i] = s2 / nij;
        }
    }
    const double alpha = 0.01, beta = 100;
    for (int k = 0; k < n * n; k++) A[k] = 0.0;
    for (int i = 0; i < n; i++) b[i] = 0.0;
    for (int i = 0; i < n; i++)
        for (int j = 0; j < n; j++) {
            const int Nij = N[i * n + j];
            b[i] += beta * Nij;
            A[i * n + i] += beta * Nij;
            if (j == i) continue;
            A[i * n + i] += 2 * alpha * I[i * n + j] * I[i * n + j] * Nij;
            A[i * n + j] -= 2 * alpha * I[i * n + j] * I[j * n + i] * Nij;
        }
    if (!solve_small(A, b, n, x))
        for (int i = 0; i < n; i++) x[i] = 1.0;
    for (int i = 0; i < n; i++) gains[i] = x[i];
}

hipError_t launch_gain_solve(const double* partials, const GainChunk* chunks, int n_chunks, const int32_t* pair_ij,
                             const int32_t* N, int n, double* gains, hipStream_t s) {
    hipLaunchKernelGGL(gain_solve_kernel, dim3(1), dim3(64), 0, s, partials, chunks, n_chunks, pair_ij, N, n, gains);
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
// Per-frame stitch, blend = 0: for every 2x2 output quad, the winning camera of each pixel is
// sampled from its YUV420P source (YUV->RGB per tap, 15-bit bilinear), gain-scaled
// (mul_scalar_with_mask, exposure_compensate.cu:15-30: sat_u8(px * (float)g)), and the quad is
// written as YUV420P (own BT.601, stands in for NPP nppiRGBToYUV420_8u_C3P3R).
// Grid-stride over quads; each XCD (blockIdx % 8) takes a contiguous band of output rows so the
// source footprint of its tiles stays in that XCD's L2.
// ---------------------------------------------------------------------------------------------
constexpr int kQuadsX = 64;   // quads per tile row (128 output pixels)
constexpr int kQuadsY = 4;    // quad rows per tile (8 output rows)

__global__ void __launch_bounds__(256) stitch_kernel(FrameSet frames, const int16_t* tab,
                                                     const CompositeEntry* lut, int W, int H, const double* gains,
                                                     int use_gain, uint8_t* out, int64_t out_pitch) {
    __shared__ short s_tab[1024 * 4];
    __shared__ float s_gain[kMaxCams];
    load_table_lds(tab, s_tab);
    if (threadIdx.x < kMaxCams) s_gain[threadIdx.x] = use_gain ? (float)gains[threadIdx.x] : 1.0f;
    __syncthreads();

    const int tiles_x = (W / 2 + kQuadsX - 1) / kQuadsX;
    const int tiles_y = (H / 2 + kQuadsY - 1) / kQuadsY;
    const int n_tiles = tiles_x * tiles_y;
    // XCD-aware split: blocks b, b+8, ... share an XCD; give that group a contiguous tile range.
    const int groups = 8;
    const int g = blockIdx.x % groups;
    const int blocks_in_g = (gridDim.x - g + groups - 1) / groups;
    const int local = blockIdx.x / groups;
    const int t_begin = (int)((int64_t)n_tiles * g / groups);
    const int t_end = (int)((int64_t)n_tiles * (g + 1) / groups);

    uint8_t* outU = out + (int64_t)H * out_pitch;
    uint8_t* outV = outU + (W >> 1);
    const int lx = threadIdx.x % kQuadsX, ly = threadIdx.x / kQuadsX;

    for (int t = t_begin + local; t < t_end; t += blocks_in_g) {
        const int tyi = t / tiles_x, txi = t - tyi * tiles_x;
        const int qx = txi * kQuadsX + lx, qy = tyi * kQuadsY + ly;
        if (qx >= (W >> 1) || qy >= (H >> 1)) continue;
        const int x = qx * 2, y = qy * 2;
        const uint4 e0 = *reinterpret_cast<const uint4*>(lut + (int64_t)y * W + x);
        const uint4 e1 = *reinterpret_cast<const uint4*>(lut + (int64_t)(y + 1) * W + x);
        const uint32_t xy[4] = {e0.x, e0.z, e1.x, e1.z};
        const uint32_t cd[4] = {e0.y, e0.w, e1.y, e1.w};
        int Yo[4];
        float us = 0.f, vs = 0.f;
#pragma unroll
        for (int p = 0; p < 4; p++) {
            int r = 0, gg = 0, b = 0;
            if (cd[p] & 0x8000u) {
                const int cam = (int)((cd[p] >> 10) & 31u);
                sample_rgb(frames.f[cam], xy[p], cd[p], s_tab, r, gg, b);
                const float gf = s_gain[cam];
                r = sat_u8_rne((float)r * gf);
                gg = sat_u8_rne((float)gg * gf);
                b = sat_u8_rne((float)b * gf);
            }
            const float R = (float)r, G = (float)gg, B = (float)b;
            const float Yf = 0.299f * R + 0.587f * G + 0.114f * B;
            Yo[p] = sat_u8_rne(Yf);
            us = us + (0.492f * (B - Yf) + 128.f);
            vs = vs + (0.877f * (R - Yf) + 128.f);
        }
        *reinterpret_cast<uint16_t*>(out + (int64_t)y * out_pitch + x) = (uint16_t)(Yo[0] | (Yo[1] << 8));
        *reinterpret_cast<uint16_t*>(out + (int64_t)(y + 1) * out_pitch + x) = (uint16_t)(Yo[2] | (Yo[3] << 8));
        outU[(int64_t)qy * out_pitch + qx] = (uint8_t)sat_u8_rne(us * 0.25f);
        outV[(int64_t)qy * out_pitch + qx] = (uint8_t)sat_u8_rne(vs * 0.25f);
    }
}

hipError_t launch_stitch(const FrameSet& frames_dev, const int16_t* tab, const CompositeEntry* lut, int W, int H,
                         const double* gains, int use_gain, uint8_t* out, int64_t out_pitch, hipStream_t s) {
    const int tiles = ((W / 2 + kQuadsX - 1) / kQuadsX) * ((H / 2 + kQuadsY - 1) / kQuadsY);
    int blocks = std::min(tiles, 256 * 8);
    blocks = std::max(8, (blocks + 7) / 8 * 8);
    hipLaunchKernelGGL(stitch_kernel, dim3(blocks), dim3(256), 0, s, frames_dev, tab, lut, W, H, gains, use_gain, out,
                       out_pitch);
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
