// multiband.hip — gfx950 kernels of the multi-band blend (blend > 0): MultiBandGPUBlender
// (stitching/src/blenders.cpp:589-735) re-laid out for the level grids and per-camera tile lists
// of kernels.hpp.  Per frame: mb_down (Gaussian levels 1..B of every camera, only the tiles some
// later step reads) and mb_blend (per level, coarsest first: Laplacian accumulate over the tile's
// cameras + weight normalisation + collapse with the coarser level, fused; level 0 writes YUV420P).
//
// All pyramid arithmetic is integer and exact (see oracle/octvr_oracle_blend.c for why the CUDA
// f32 code is):  fastPyrDown = sat(rne(S / 256)), pyrUp = sat(rne(S / 64)) with S the integer
// weighted tap sum.  The weight pyramid (build time) is f32 with nvcc's FMA contraction.
// Built with -ffp-contract=off: every other f32 expression rounds as written.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "device_common.hpp"
#include "kernels.hpp"

namespace octvr {

// round half to even of S / 2^sh (S of any sign): floor((S + half - 1 + bit_sh(S)) / 2^sh) — below
// the half the sum stays under the next multiple, at the half it reaches it only for an odd quotient
template <int SH>
__device__ __forceinline__ int rne_shr(int S) {
    constexpr int half = 1 << (SH - 1);
    return (S + (half - 1) + (int)(((uint32_t)S >> SH) & 1u)) >> SH;
}

__device__ __forceinline__ uint32_t ch_of(uint32_t v, int c) { return (v >> (8 * c)) & 255u; }

// ---------------------------------------------------------------------------------------------
// fastPyrDown<uchar4> (fast_pyr_down.cu:17-76): out = sat(rne(sum_{j,k} w_j w_k src / 256)),
// w = [1 4 6 4 1], texture clamp border (camera-local).  One workgroup per (camera, 128x8 tile of
// level l): each lane loads one column of the 20 x 260 source patch of level l-1 into registers and
// sums it vertically into 8 rows of u16 channel sums in LDS; then the horizontal pass per 2x2 quad.
// ---------------------------------------------------------------------------------------------
constexpr int kDnRows = 2 * kTileH + 4, kDnCols = 2 * kTileW + 4;

__global__ void __launch_bounds__(256) mb_down_kernel(const uint2* __restrict__ items, const MbCamLevel* cams_l,
                                                      const MbCamLevel* cams_prev, const uint8_t* __restrict__ g_prev,
                                                      uint8_t* __restrict__ g_l) {
    __shared__ uint2 s_v[kTileH * kDnCols];             // 16.3 KiB: (R | B << 16, G | A << 16) column sums
    const uint2 it = items[blockIdx.x];
    const int cam = uniform((int)it.x);
    const int tx = uniform((int)(it.y & 0xFFFFu)), ty = uniform((int)(it.y >> 16));
    const MbCamLevel c = cams_l[cam];
    const MbCamLevel p = cams_prev[cam];
    const int tid = threadIdx.x;
    // tile origin in camera-local coordinates of level l, and its source window in level l-1
    const int xo = tx * kTileW - c.ox, yo = ty * kTileH - c.oy;
    const int sx0 = 2 * xo - 2, sy0 = 2 * yo - 2;
    const uint8_t* src = g_prev + p.g_off;
    // Channel sums in packed 16-bit halves: R and B of a pixel as (v & 0x00FF00FF), G and A as
    // (v >> 8) & 0x00FF00FF, so one packed multiply-add serves two channels.  Every sum stays exact in
    // 16 bits: a 5-tap column sum <= 16 * 255 = 4,080, the 5 x 5 sum <= 256 * 255 = 65,280.
    typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
    constexpr unsigned short kW5[5] = {1, 4, 6, 4, 1};
    auto colsum = [&](const uint32_t (&col)[kDnRows], int tgt) {
        u16x2 rb[kDnRows], ga[kDnRows];
#pragma unroll
        for (int k = 0; k < kDnRows; k++) {
            rb[k] = __builtin_bit_cast(u16x2, col[k] & 0x00FF00FFu);
            ga[k] = __builtin_bit_cast(u16x2, (col[k] >> 8) & 0x00FF00FFu);
        }
#pragma unroll
        for (int r = 0; r < kTileH; r++) {
            u16x2 srb = rb[2 * r] * kW5[0], sga = ga[2 * r] * kW5[0];
#pragma unroll
            for (int j = 1; j < 5; j++) {
                srb += rb[2 * r + j] * kW5[j];
                sga += ga[2 * r + j] * kW5[j];
            }
            s_v[r * kDnCols + tgt] = make_uint2(__builtin_bit_cast(uint32_t, srb), __builtin_bit_cast(uint32_t, sga));
        }
    };
    // lane t holds column t of the 20 source rows in registers (lanes 0-3 of wave 0 also columns
    // 256-259), all loads in flight before the first use; the vertical pass runs on them directly
    {
        const int sxa = min(max(sx0 + tid, 0), p.w - 1);
        uint32_t va[kDnRows];
#pragma unroll
        for (int r = 0; r < kDnRows; r++)
            va[r] = *reinterpret_cast<const uint32_t*>(src + (int64_t)min(max(sy0 + r, 0), p.h - 1) * p.g_pitch + (int64_t)sxa * 4);
        if (tid < 4) {
            const int sxb = min(max(sx0 + kDnCols - 4 + tid, 0), p.w - 1);
            uint32_t vb[kDnRows];
#pragma unroll
            for (int r = 0; r < kDnRows; r++)
                vb[r] = *reinterpret_cast<const uint32_t*>(src + (int64_t)min(max(sy0 + r, 0), p.h - 1) * p.g_pitch + (int64_t)sxb * 4);
            colsum(vb, kDnCols - 4 + tid);
        }
        colsum(va, tid);
    }
    __syncthreads();
    const int qx = tid & 63, qy = tid >> 6;
    const int xl = xo + 2 * qx, yl = yo + 2 * qy;  // quad origin, camera-local (any parity at the top level)
    if (xl + 1 < 0 || yl + 1 < 0 || xl >= c.w || yl >= c.h) return;
    uint32_t px[4];
#pragma unroll
    for (int p4 = 0; p4 < 4; p4++) {
        const int r = 2 * qy + (p4 >> 1), cx = 2 * (2 * qx + (p4 & 1));  // source column 2x-2 -> index 2x
        const uint2* v = s_v + r * kDnCols + cx;
        u16x2 hrb = __builtin_bit_cast(u16x2, v[0].x) * kW5[0], hga = __builtin_bit_cast(u16x2, v[0].y) * kW5[0];
#pragma unroll
        for (int k = 1; k < 5; k++) {
            hrb += __builtin_bit_cast(u16x2, v[k].x) * kW5[k];
            hga += __builtin_bit_cast(u16x2, v[k].y) * kW5[k];
        }
        // sat(rne(S / 256)) per channel: (S + 127 + bit8(S)) >> 8 <= 255 (S <= 65,280: no carry, no clamp)
        const u16x2 one = {1, 1}, c127 = {127, 127};
        const u16x2 orb = (hrb + c127 + ((hrb >> 8) & one)) >> 8, oga = (hga + c127 + ((hga >> 8) & one)) >> 8;
        // R | G << 8 | B << 16 (A = 0): bytes 0 and 2 of orb, byte 0 of oga
        px[p4] = __builtin_amdgcn_perm(__builtin_bit_cast(uint32_t, oga), __builtin_bit_cast(uint32_t, orb), 0x0C020400u);
    }
#pragma unroll
    for (int p4 = 0; p4 < 4; p4++) {  // per pixel: odd-sized top levels end mid-quad
        const int px_ = xl + (p4 & 1), py_ = yl + (p4 >> 1);
        if (px_ < 0 || py_ < 0 || px_ >= c.w || py_ >= c.h) continue;
        *reinterpret_cast<uint32_t*>(g_l + c.g_off + (int64_t)py_ * c.g_pitch + (int64_t)px_ * 4) = px[p4];
    }
}

hipError_t launch_mb_down(const uint2* items, int n_items, const MbCamLevel* cams_l, const MbCamLevel* cams_prev,
                          const uint8_t* g_prev, uint8_t* g_l, hipStream_t s) {
    if (n_items <= 0) return hipSuccess;
    hipLaunchKernelGGL(mb_down_kernel, dim3(n_items), dim3(256), 0, s, items, cams_l, cams_prev, g_prev, g_l);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// Blend of one level (blenders.cpp:686-735 for one i, fused with the collapse step of i):
//   D    = sum over the tile's cameras (ascending) of (short)((G_n - pyrUp(G_n,next)) * w_n)   [K5]
//          (at the top level: (short)(G_n * w_n), K6), short adds wrapping; only where w_n != 0
//   L    = sat_s16(rne(D * (1.0f / (1e-5f + sum_n w_n))))                                     [K11]
//   R    = top ? L : sat_s16(L + pyrUp(R_next))                                                [add]
//   level 0: out = sat_u8(R) as RGB -> YUV420P; otherwise R is stored (s16x4) for the next level.
// Multi-band: one wave per 32x8 sub-tile of a per-level work list (feather: one workgroup per 128x8 tile),
// one 2x2 quad per lane.  pyrUp taps are computed in registers (up_arith, kernels.hpp; the host proves
// per rig that they weigh exactly the UpQuad tables' sources, check_up_arith): 3 rows x 3 columns of
// source per quad, per-pixel integer weights over them, read straight from global memory.
// ---------------------------------------------------------------------------------------------
struct Up9 {
    int s[4][3];  // per quad pixel, per channel: the integer tap sum (scale 1/64)
};

// pyrUp sums of a quad from its 3 x 3 union taps and per-pixel integer weights over them (UpArith).
// The 1-D weights of a quad row /
// column sum to 8 (1 6 1 or 4 4), so with s16 sources every product and partial sum fits 24 bits:
// 24-bit multiplies (full rate; a 32-bit v_mul_lo is quarter rate).
template <class QR, class QC>
__device__ __forceinline__ void up_weigh(const QR& ur, const QC& uc, const int (&v)[3][3][3], Up9& o) {
#pragma unroll
    for (int pc = 0; pc < 2; pc++) {
        const auto& wx = pc ? uc.w1 : uc.w0;
        int h[3][3];  // [row][ch]
#pragma unroll
        for (int j = 0; j < 3; j++)
#pragma unroll
            for (int ch = 0; ch < 3; ch++)
                h[j][ch] = __mul24((int)wx[0], v[j][0][ch]) + __mul24((int)wx[1], v[j][1][ch]) +
                           __mul24((int)wx[2], v[j][2][ch]);
#pragma unroll
        for (int pr = 0; pr < 2; pr++) {
            const auto& wy = pr ? ur.w1 : ur.w0;
#pragma unroll
            for (int ch = 0; ch < 3; ch++)
                o.s[pr * 2 + pc][ch] = __mul24((int)wy[0], h[0][ch]) + __mul24((int)wy[1], h[1][ch]) +
                                       __mul24((int)wy[2], h[2][ch]);
        }
    }
}

// The 3 x 3 taps of a quad straight from global memory (indices clamped into the source; neighbouring
// lanes share the lines, so these are mostly L1 / L2 hits): no LDS staging and no barriers.
template <class T>
struct Taps9 {
    T t[3][3];
};
template <class T, class QR, class QC>
__device__ __forceinline__ void up_taps_issue(const QR& ur, const QC& uc, const uint8_t* base, int64_t pitch,
                                              Taps9<T>& o) {
#pragma unroll
    for (int j = 0; j < 3; j++) {
        const uint8_t* row = base + (int64_t)ur.idx[j] * pitch;
#pragma unroll
        for (int k = 0; k < 3; k++) o.t[j][k] = *reinterpret_cast<const T*>(row + (int64_t)uc.idx[k] * sizeof(T));
    }
}
template <class T, class UNPACK, class QR, class QC>
__device__ __forceinline__ void up_quad_taps(const QR& ur, const QC& uc, const Taps9<T>& tp, UNPACK unpack,
                                             Up9& o) {
    int v[3][3][3];
#pragma unroll
    for (int j = 0; j < 3; j++)
#pragma unroll
        for (int k = 0; k < 3; k++) unpack(tp.t[j][k], v[j][k]);
    up_weigh(ur, uc, v, o);
}

// pyrUp of a quad of u8x4 taps (the Gaussian level), rounded: R and B ride as the two 16-bit halves of
// one word, G alone.  Column sums first with the row weights (wave-uniform), then the per-lane column
// weights; every partial sum is <= 64 * 255 per half, so the 32-bit adds never carry across halves,
// the 24-bit multiplies see operands < 2^24, and the round (S + 31 + bit6) / 64 stays inside its half.
// Out: per pixel (R | B << 16) and G of sat_u8(rne(S / 64)) (the clamp is a no-op: S <= 64 * 255).
__device__ __forceinline__ void up_g_packed(const UpArith& ur, const UpArith& uc, const Taps9<uint32_t>& tp,
                                            uint32_t (&rb)[4], uint32_t (&gg)[4]) {
    uint32_t vrb[2][3], vg[2][3];
#pragma unroll
    for (int k = 0; k < 3; k++) {
        uint32_t RB[3], G[3];
#pragma unroll
        for (int j = 0; j < 3; j++) {
            RB[j] = tp.t[j][k] & 0x00FF00FFu;
            G[j] = (tp.t[j][k] >> 8) & 255u;
        }
#pragma unroll
        for (int pr = 0; pr < 2; pr++) {
            const auto& wy = pr ? ur.w1 : ur.w0;
            vrb[pr][k] = __umul24((uint32_t)wy[0], RB[0]) + __umul24((uint32_t)wy[1], RB[1]) +
                         __umul24((uint32_t)wy[2], RB[2]);  // halves <= 8 * 255
            vg[pr][k] = __umul24((uint32_t)wy[0], G[0]) + __umul24((uint32_t)wy[1], G[1]) +
                        __umul24((uint32_t)wy[2], G[2]);
        }
    }
    typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
#pragma unroll
    for (int pc = 0; pc < 2; pc++) {
        const auto& wx = pc ? uc.w1 : uc.w0;
        const u16x2 w0 = {(unsigned short)wx[0], (unsigned short)wx[0]}, w1 = {(unsigned short)wx[1], (unsigned short)wx[1]},
                    w2 = {(unsigned short)wx[2], (unsigned short)wx[2]};
#pragma unroll
        for (int pr = 0; pr < 2; pr++) {
            // halves <= 8 * 2040: 16-bit packed multiply-adds (v_pk_mad_u16)
            const u16x2 s = __builtin_bit_cast(u16x2, vrb[pr][0]) * w0 + __builtin_bit_cast(u16x2, vrb[pr][1]) * w1 +
                            __builtin_bit_cast(u16x2, vrb[pr][2]) * w2;
            const uint32_t S = __builtin_bit_cast(uint32_t, s);
            const uint32_t S2 = S + 0x001F001Fu + ((S >> 6) & 0x00010001u);
            rb[pr * 2 + pc] = (S2 >> 6) & 0x00FF00FFu;
            const uint32_t Sg = __umul24((uint32_t)wx[0], vg[pr][0]) + __umul24((uint32_t)wx[1], vg[pr][1]) +
                                __umul24((uint32_t)wx[2], vg[pr][2]);
            gg[pr * 2 + pc] = (Sg + 31u + ((Sg >> 6) & 1u)) >> 6;
        }
    }
}

constexpr int kBlendWaves = 7;  // waves per SIMD the blend is compiled for (register budget)
// 1e-5f + 1.0f (one weight-1 camera: (float)(1. / 255) * 255.0f rounds to exactly 1.0f) and the
// correctly rounded reciprocals of the two common weight sums (constant-folded)
constexpr float kWsumOwned = 1e-5f + 1.0f, kRcpOwned = 1.0f / kWsumOwned, kRcpNone = 1.0f / 1e-5f;
static_assert((float)(1. / 255) * 255.0f == 1.0f, "seam weight 255 / 255");

__global__ void __launch_bounds__(256, kBlendWaves) mb_blend_kernel(MbBlendArgs a) {
    const int tid = threadIdx.x;
    const int wv = uniform(tid >> 6), lane = tid & 63;
    // Multi-band: wave w of block b blends sub-tile work[4 b + w] (32 x 8: lane = quad, 16 per quad row;
    // a scalar load through the constant address space): tile | quarter << 24 | kind << 27, its cameras.
    // Waves share nothing (no LDS, no barriers: every pyrUp tap is read straight from global memory), so
    // a workgroup's four sub-tiles may lie anywhere.  Feather (no list): one tile per workgroup, wave =
    // quad row, lane = quad.
    typedef __attribute__((address_space(4))) const uint64_t kU64;
    const uint64_t wk64 = a.work ? ((const kU64*)a.work)[blockIdx.x * 4 + wv] : 0ull;
    const uint2 wk = make_uint2((uint32_t)wk64, (uint32_t)(wk64 >> 32));
    const int tile = a.work ? (int)(wk.x & 0xFFFFFFu) : (int)blockIdx.x;
    const int ty = tile / a.tiles_x, tx = tile - ty * a.tiles_x;
    const int x = a.work ? tx * kTileW + (int)((wk.x >> 24) & 3u) * kSubW + 2 * (lane & 15) : tx * kTileW + 2 * lane;
    const int y = a.work ? ty * kTileH + 2 * (lane >> 4) : ty * kTileH + 2 * wv;  // quad origin (even)
    const bool top = a.level == a.bands;
    bool valid[4];
#pragma unroll
    for (int p = 0; p < 4; p++) valid[p] = (x + (p & 1)) < a.W && (y + (p >> 1)) < a.H;
    int R[4][3];
    uint32_t m = a.work ? (uint32_t)uniform((int)wk.y) : (uint32_t)uniform((int)a.tile_cams[tile]);
    // Tiles owned by one camera (its weight is exactly 1.0f on every tile pixel: seam 255 at level 0,
    // the f32 pyramid's 1.0f above; tile_owned): D = G - pyrUp(G_next) (G at the top level) exactly,
    // the weight sum is kWsumOwned and rint(D * kRcpOwned) = D (|D| <= 255), so the Laplacian is taken
    // as is, with no weight loads or sums.
    // Deep tiles (owned = 2, multiband_host.cpp): R = G on every pixel, by induction over the levels
    // above (one camera of weight 1 on all the pyrUp taps, with the camera's and the collapse's taps
    // identical), so neither pyrUp is taken.
    const int own = a.work ? (int)(wk.x >> 27) : a.owned != nullptr ? uniform((int)a.owned[tile]) : 0;
    if (own == 3) return;  // no collapse reads this tile (levels >= 1)
    const bool deep = own == 2;
    if (own == 4) return;  // level 0: a deep tile whose result the remap wrote (kItemResult)
    if (own != 0) {
        const int n = __builtin_ctz(m);
        const MbCamLevel c = a.cams[n];
        const int xl = x - c.ox, yl = y - c.oy;  // inside the camera (seam pixels), even
        const int x0 = min(max(xl, 0), c.w - 2);
        const int cy0 = min(max(yl, 0), c.h - 1), cy1 = min(max(yl + 1, 0), c.h - 1);
        const uint2 gp0 = *reinterpret_cast<const uint2*>(a.g + c.g_off + (int64_t)cy0 * c.g_pitch + x0 * 4);
        const uint2 gp1 = *reinterpret_cast<const uint2*>(a.g + c.g_off + (int64_t)cy1 * c.g_pitch + x0 * 4);
        if (deep) {
#pragma unroll
            for (int p = 0; p < 4; p++) {
                const uint2 gp = (p >> 1) ? gp1 : gp0;
                const uint32_t gv = ((xl + (p & 1) - x0) & 1) ? gp.y : gp.x;
#pragma unroll
                for (int ch = 0; ch < 3; ch++) R[p][ch] = (int)ch_of(gv, ch);
            }
        } else {
        // (the top level reads its own G as a stand-in for the unused taps, as the general path)
        const MbCamLevel cn = *(top ? a.cams + n : a.cams_next + n);
        const UpArith ur = up_arith(y, c.oy, c.h, cn.h, true), uc = up_arith(x, c.ox, c.w, cn.w, false);
        Taps9<uint32_t> tp;
        up_taps_issue<uint32_t>(ur, uc, (top ? a.g : a.g_next) + cn.g_off, cn.g_pitch, tp);
        uint32_t urb[4], ug[4];
        up_g_packed(ur, uc, tp, urb, ug);
#pragma unroll
        for (int p = 0; p < 4; p++) {
            const uint2 gp = (p >> 1) ? gp1 : gp0;
            const uint32_t gv = ((xl + (p & 1) - x0) & 1) ? gp.y : gp.x;
            const uint32_t u0 = top ? 0u : urb[p] & 255u, u1 = top ? 0u : ug[p], u2 = top ? 0u : urb[p] >> 16;
            R[p][0] = (int)ch_of(gv, 0) - (int)u0;
            R[p][1] = (int)ch_of(gv, 1) - (int)u1;
            R[p][2] = (int)ch_of(gv, 2) - (int)u2;
        }
        }
    } else {
    float D[4][3];  // the Laplacian accumulator (a CV_16S sum in the reference; exact here, see below)
    float wsum[4];
#pragma unroll
    for (int p = 0; p < 4; p++) {
        wsum[p] = 1e-5f;
#pragma unroll
        for (int ch = 0; ch < 3; ch++) D[p][ch] = 0.f;
    }
    while (m) {
        const int n = __builtin_ctz(m);
        m &= m - 1;
        const MbCamLevel c = a.cams[n];
        const int xl = x - c.ox, yl = y - c.oy;  // camera-local quad origin (any parity)
        float w[4];
        float g[4][3];  // G - pyrUp(G_next) (G at the top level): small exact integers
        if (c.w >= 2) {
            // Every load of this camera is issued before any of them is used — the G pairs and weight
            // pairs of both quad rows and the 9 pyrUp taps — so a camera costs one memory round trip.
            // Per quad row one 8-byte load of G and of the weights at the clamped pair start x0: pixel
            // px is element px - x0 (0 or 1 whenever it lies inside the camera).  One buffer resource
            // serves both weight kinds: the u8 level-0 seam from the dword at or below the pair (dword
            // loads ignore the low address bits; reads past the end return 0), or the f32 level.
            const int x0 = min(max(xl, 0), c.w - 2);
            const uint32_t dlt = a.w_u8 ? (uint32_t)(reinterpret_cast<uintptr_t>(c.weight) & 3u) : 0u;
            const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(
                const_cast<uint8_t*>(static_cast<const uint8_t*>(c.weight) - dlt), 0,
                (int)(a.w_u8 ? (uint32_t)(c.w * c.h) + dlt : (uint32_t)(c.w * c.h) * 4u), 0x00020000);
            typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
            // (plain scalars, no arrays: a private array here is promoted to LDS and waited on)
            const int cy0 = min(max(yl, 0), c.h - 1), cy1 = min(max(yl + 1, 0), c.h - 1);
            const uint2 gp0 = *reinterpret_cast<const uint2*>(a.g + c.g_off + (int64_t)cy0 * c.g_pitch + x0 * 4);
            const uint2 gp1 = *reinterpret_cast<const uint2*>(a.g + c.g_off + (int64_t)cy1 * c.g_pitch + x0 * 4);
            const uint32_t at0 = dlt + (uint32_t)(cy0 * c.w + x0), at1 = dlt + (uint32_t)(cy1 * c.w + x0);
            const u32x2 wq0 = __builtin_amdgcn_raw_buffer_load_b64(wr, a.w_u8 ? at0 & ~3u : at0 * 4u, 0, 0);
            const u32x2 wq1 = __builtin_amdgcn_raw_buffer_load_b64(wr, a.w_u8 ? at1 & ~3u : at1 * 4u, 0, 0);
            // unconditionally (the top level reads its own G as a stand-in, unused): a branch here would
            // let the compiler merge it with the one below, after the weight decode's waits
            const MbCamLevel cn = *(top ? a.cams + n : a.cams_next + n);
            const UpArith ur = up_arith(y, c.oy, c.h, cn.h, true), uc = up_arith(x, c.ox, c.w, cn.w, false);
            Taps9<uint32_t> tp;
            up_taps_issue<uint32_t>(ur, uc, (top ? a.g : a.g_next) + cn.g_off, cn.g_pitch, tp);
            uint32_t gv[4];
#pragma unroll
            for (int r = 0; r < 2; r++) {
                const int py = yl + r;
                const u32x2 wq = r ? wq1 : wq0;
                const uint2 gp = r ? gp1 : gp0;
                const uint32_t at = r ? at1 : at0;
                float wp[2];
                if (a.w_u8) {
                    const uint64_t q = ((uint64_t)wq.y << 32) | wq.x;
                    const uint32_t sh = 8u * (at & 3u);
                    // level 0: convertTo(CV_32F, 1/255.) of the seam mask (gpu_mat.cu:458-480): alpha * v + 0
                    wp[0] = (float)(1. / 255) * (float)(uint32_t)((q >> sh) & 255u);
                    wp[1] = (float)(1. / 255) * (float)(uint32_t)((q >> (sh + 8u)) & 255u);
                } else {
                    // (__uint_as_float of a copied scalar: __builtin_bit_cast of an ext-vector component
                    // reads the vector's first element with this compiler)
                    const uint32_t lo = wq.x, hi = wq.y;
                    wp[0] = __uint_as_float(lo);
                    wp[1] = __uint_as_float(hi);
                }
#pragma unroll
                for (int pc = 0; pc < 2; pc++) {
                    const int p = 2 * r + pc, px = xl + pc;
                    const bool in = valid[p] && px >= 0 && py >= 0 && px < c.w && py < c.h;
                    const bool hi = ((px - x0) & 1) != 0;
                    w[p] = in ? (hi ? wp[1] : wp[0]) : 0.f;
                    gv[p] = hi ? gp.y : gp.x;
                }
            }
            if (!top) {
                uint32_t urb[4], ug[4];
                up_g_packed(ur, uc, tp, urb, ug);
#pragma unroll
                for (int p = 0; p < 4; p++) {
                    g[p][0] = (float)ch_of(gv[p], 0) - (float)(urb[p] & 255u);
                    g[p][1] = (float)ch_of(gv[p], 1) - (float)ug[p];
                    g[p][2] = (float)ch_of(gv[p], 2) - (float)(urb[p] >> 16);
                }
            } else {
#pragma unroll
                for (int p = 0; p < 4; p++)
#pragma unroll
                    for (int ch = 0; ch < 3; ch++) g[p][ch] = (float)ch_of(gv[p], ch);
            }
        } else {
            // (cameras 1 pixel wide at this level): per-pixel loads
            uint32_t gv[4];
#pragma unroll
            for (int p = 0; p < 4; p++) {
                const int px = xl + (p & 1), py = yl + (p >> 1);
                const bool in = valid[p] && px >= 0 && py >= 0 && px < c.w && py < c.h;
                const int cx = min(max(px, 0), c.w - 1), cy = min(max(py, 0), c.h - 1);
                const int64_t k = (int64_t)cy * c.w + cx;
                // level 0: convertTo(CV_32F, 1/255.) of the seam mask (gpu_mat.cu:458-480): alpha * v + 0
                const float wv_ = a.w_u8 ? (float)(1. / 255) * (float)static_cast<const uint8_t*>(c.weight)[k]
                                         : static_cast<const float*>(c.weight)[k];
                w[p] = in ? wv_ : 0.f;
                gv[p] = *reinterpret_cast<const uint32_t*>(a.g + c.g_off + (int64_t)cy * c.g_pitch + cx * 4);
            }
            if (!top) {
                const MbCamLevel cn = a.cams_next[n];
                const UpArith ur = up_arith(y, c.oy, c.h, cn.h, true), uc = up_arith(x, c.ox, c.w, cn.w, false);
                Taps9<uint32_t> tp;
                up_taps_issue<uint32_t>(ur, uc, a.g_next + cn.g_off, cn.g_pitch, tp);
                uint32_t urb[4], ug[4];
                up_g_packed(ur, uc, tp, urb, ug);
#pragma unroll
                for (int p = 0; p < 4; p++) {
                    g[p][0] = (float)ch_of(gv[p], 0) - (float)(urb[p] & 255u);
                    g[p][1] = (float)ch_of(gv[p], 1) - (float)ug[p];
                    g[p][2] = (float)ch_of(gv[p], 2) - (float)(urb[p] >> 16);
                }
            } else {
#pragma unroll
                for (int p = 0; p < 4; p++)
#pragma unroll
                    for (int ch = 0; ch < 3; ch++) g[p][ch] = (float)ch_of(gv[p], ch);
            }
        }
        // only where w != 0 in the reference; a zero weight adds +-0 to D and 0 to the weight sum, so the
        // sums are the same without a per-pixel branch
#pragma unroll
        for (int p = 0; p < 4; p++) {
#pragma unroll
            for (int ch = 0; ch < 3; ch++) {
                // (short)(g * w), then short += short.  |g * w| <= 255 * w and the weights of a pixel sum
                // to <= 1 (multi-band) or <= n (feather, n <= 32): |D| <= 8160 at every step, so the
                // short adds never wrap and the sum is exact in f32
                D[p][ch] = D[p][ch] + __builtin_truncf(g[p][ch] * w[p]);
            }
            wsum[p] = wsum[p] + w[p];
        }
    }
#pragma unroll
    for (int p = 0; p < 4; p++) {
        // feather: convertTo(CV_8UC3, 1/n) = sat_u8(alpha * D) (clamped to u8 below); multi-band:
        // DivOpSpecial<short3> with the correctly rounded reciprocal (hipcc default, as CUDA's 1.0f / b)
        float rcp = a.feather ? a.out_scale : kRcpOwned;
        // level 0 with 0 / 255 seams: one camera of weight 1 (or none) per pixel, i.e. the two sums below;
        // any other sum takes the division (a branch only the lanes that need it execute)
        if (!a.feather && wsum[p] != kWsumOwned) rcp = wsum[p] == 1e-5f ? kRcpNone : 1.0f / wsum[p];
#pragma unroll
        for (int ch = 0; ch < 3; ch++)
            R[p][ch] = (int)__builtin_amdgcn_fmed3f(__builtin_rintf(D[p][ch] * rcp), -32768.f, 32767.f);
    }
    }
    if (!top && !deep) {
        Up9 u;
        auto unpack = [](uint2 v, int (&o)[3]) {
            o[0] = (int)(int16_t)(v.x & 0xFFFFu);
            o[1] = (int)(int16_t)(v.x >> 16);
            o[2] = (int)(int16_t)(v.y & 0xFFFFu);
        };
        // x and y are even on the level grid: every quad has the even tap pattern (1 6 1 | 0 4 4) as
        // constants; the zero weights up_arith gives pixels outside the level only matter for pixels
        // that are never stored (W, H even at level 0; level > 0 stores valid pixels only)
        UpArith ur = up_arith(y, 0, a.H, a.H_next, true), uc = up_arith(x, 0, a.W, a.W_next, false);
#pragma unroll
        for (int j = 0; j < 3; j++) {
            ur.w0[j] = uc.w0[j] = j == 1 ? 6 : 1;
            ur.w1[j] = uc.w1[j] = j == 0 ? 0 : 4;
        }
        Taps9<uint2> tp;
        up_taps_issue<uint2>(ur, uc, reinterpret_cast<const uint8_t*>(a.r_next), (int64_t)a.W_next * 8, tp);
        up_quad_taps(ur, uc, tp, unpack, u);
#pragma unroll
        for (int p = 0; p < 4; p++)
#pragma unroll
            for (int ch = 0; ch < 3; ch++) {
                const int up = min(max(rne_shr<6>(u.s[p][ch]), -32768), 32767);
                R[p][ch] = min(max(R[p][ch] + up, -32768), 32767);
            }
    }
    if (a.level > 0) {
#pragma unroll
        for (int p = 0; p < 4; p++) {
            if (!valid[p]) continue;
            const uint2 v = make_uint2(((uint32_t)R[p][0] & 0xFFFFu) | ((uint32_t)R[p][1] << 16), (uint32_t)R[p][2] & 0xFFFFu);
            *reinterpret_cast<uint2*>(a.r_out + ((int64_t)(y + (p >> 1)) * a.W + x + (p & 1)) * 4) = v;
        }
        return;
    }
    // level 0: convertTo(CV_8UC3) into result(align_result_roi.tl, crop) and RGB -> YUV420P
    uint32_t rgb[4][3];
#pragma unroll
    for (int p = 0; p < 4; p++)
#pragma unroll
        for (int ch = 0; ch < 3; ch++) rgb[p][ch] = (uint32_t)min(max(R[p][ch], 0), 255);
    const int ox = a.ax + x, oy = a.ay + y;
    const bool in = x < a.crop_w && y < a.crop_h && ox < a.out_w && oy < a.out_h;
    if (a.rgba) {  // scaled output: the result image itself (resized + converted afterwards)
        if (!in) return;
#pragma unroll
        for (int r = 0; r < 2; r++) {
            uint2 v;
            v.x = rgb[2 * r][0] | (rgb[2 * r][1] << 8) | (rgb[2 * r][2] << 16);
            v.y = rgb[2 * r + 1][0] | (rgb[2 * r + 1][1] << 8) | (rgb[2 * r + 1][2] << 16);
            *reinterpret_cast<uint2*>(a.rgba + (int64_t)(oy + r) * a.rgba_pitch + (int64_t)ox * 4) = v;
        }
        return;
    }
    const OutFrame of = make_out_frame(a.out, a.out_w, a.out_h, a.out_pitch);
    store_quad(of, finish_quad_u8(rgb), ox, oy, in);  // rgb already 0..255
}

hipError_t launch_mb_blend(const MbBlendArgs& a, hipStream_t s) {
    const int tiles_y = (a.H + kTileH - 1) / kTileH;
    const int n = a.work ? a.n_work / 4 : a.tiles_x * tiles_y;  // (the list: 4 sub-tiles per workgroup)
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(mb_blend_kernel, dim3(n), dim3(256), 0, s, a);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// Build time: K4 pyrDown<float, BrdReflect101> (pyr_down.cu:55-192).  Column sums first (5 rows,
// reflect-101), then the row sum of 5 column sums; nvcc contracts `sum + w * v` into fmaf.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ int refl101(int v, int last) {
    v = abs(last - abs(last - v)) % (last + 1);
    return abs(v) % (last + 1);
}
__device__ __forceinline__ float sum5(float a, float b, float c, float d, float e) {
    float s = 0.0625f * a;
    s = __builtin_fmaf(0.25f, b, s);
    s = __builtin_fmaf(0.375f, c, s);
    s = __builtin_fmaf(0.25f, d, s);
    return __builtin_fmaf(0.0625f, e, s);
}

__global__ void __launch_bounds__(256) pyr_down_f32_kernel(const float* __restrict__ src, int sw, int sh,
                                                           float* __restrict__ dst, int dw, int dh) {
    const int64_t total = (int64_t)dw * dh;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int y = (int)(i / dw), x = (int)(i - (int64_t)y * dw);
        const float* r[5];
#pragma unroll
        for (int j = 0; j < 5; j++) r[j] = src + (int64_t)refl101(2 * y + j - 2, sh - 1) * sw;
        float cs[5];
#pragma unroll
        for (int k = 0; k < 5; k++) {
            const int cx = refl101(2 * x + k - 2, sw - 1);
            cs[k] = sum5(r[0][cx], r[1][cx], r[2][cx], r[3][cx], r[4][cx]);
        }
        dst[i] = sum5(cs[0], cs[1], cs[2], cs[3], cs[4]);
    }
}

hipError_t launch_pyr_down_f32(const float* src, int sw, int sh, float* dst, int dw, int dh, hipStream_t s) {
    const int64_t total = (int64_t)dw * dh;
    if (total <= 0) return hipSuccess;
    const int blocks = (int)std::min<int64_t>((total + 255) / 256, 256 * 8);
    hipLaunchKernelGGL(pyr_down_f32_kernel, dim3(blocks), dim3(256), 0, s, src, sw, sh, dst, dw, dh);
    return hipGetLastError();
}

// Build time: which 8x8 blocks of the level grid hold a non-zero weight of one camera.  A lane
// scans the 8 pixels of one block row and marks the block (benign duplicate stores of 1).
__global__ void __launch_bounds__(256) block_activity_kernel(const void* weight, int is_u8, int w, int h, int ox,
                                                             int oy, int bx_n, uint8_t* blocks) {
    const int gx_n = (w + 7 + (ox & 7)) / 8 + 1;  // 8-pixel groups per row on the level grid
    const int64_t total = (int64_t)gx_n * h;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int yl = (int)(i / gx_n), gi = (int)(i - (int64_t)yl * gx_n);
        const int gx0 = ((ox >> 3) + gi) * 8;  // level-grid x of the group
        bool nz = false;
        for (int q = 0; q < 8; q++) {
            const int xl = gx0 + q - ox;
            if (xl < 0 || xl >= w) continue;
            const int64_t k = (int64_t)yl * w + xl;
            nz |= is_u8 ? static_cast<const uint8_t*>(weight)[k] != 0 : static_cast<const float*>(weight)[k] != 0.f;
        }
        if (nz) blocks[(int64_t)((yl + oy) >> 3) * bx_n + (gx0 >> 3)] = 1;
    }
}

hipError_t launch_block_activity(const void* weight, int is_u8, int w, int h, int ox, int oy, int bx_n, uint8_t* blocks,
                                 hipStream_t s) {
    if (w <= 0 || h <= 0) return hipSuccess;
    const int64_t total = (int64_t)((w + 7 + (ox & 7)) / 8 + 1) * h;
    const int blocks_n = (int)std::min<int64_t>((total + 255) / 256, 256 * 8);
    hipLaunchKernelGGL(block_activity_kernel, dim3(blocks_n), dim3(256), 0, s, weight, is_u8, w, h, ox, oy, bx_n, blocks);
    return hipGetLastError();
}

}  // namespace octvr
