// device_common.hpp — device-side pixel arithmetic and I/O helpers shared by the gfx950 kernels
// (kernels.hip: remap / gain / composite; multiband.hip: pyramid blend).  Internal header.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "kernels.hpp"

namespace octvr {

// ---------------------------------------------------------------------------------------------
// Pixel arithmetic shared by the kernels
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ int sat_u8_rne(float v) {
    // saturate_cast<uchar>(float): round half to even, clamp (NaN -> 0)
    if (!(v > 0.f)) return 0;
    if (v >= 255.f) return 255;
    return (int)__builtin_rintf(v);
}

// The same conversion in one instruction, written into byte `sel` of `old`: v_cvt_pk_u8_f32 rounds
// half to even and saturates (NaN -> 0); tests/test_gpu_parity.py::test_gpu_saturating_conversion_kat.
__device__ __forceinline__ uint32_t pack_u8(float v, uint32_t sel, uint32_t old) {
    return __builtin_amdgcn_cvt_pk_u8_f32(v, sel, old);
}

// The library's own BT.601 YUV -> RGB (stands in for NPP nppiYUV420ToRGB_8u_P3AC4R,
// cudaimgproc/src/color.cpp:2269, whose arithmetic is closed: pinned by the oracle only).  Same
// operation sequence as oracle/octvr_oracle.c yuv_px_to_rgb.  Returns packed R | G << 8 | B << 16.
// R and B come from one packed fma (v_pk_fma_f32), each element rounded as the scalar fma.
__device__ __forceinline__ uint32_t yuv_to_rgba(uint32_t y, uint32_t u, uint32_t v) {
    typedef float f2 __attribute__((ext_vector_type(2)));
    const float Yf = (float)y, Uf = (float)u - 128.f, Vf = (float)v - 128.f;
    const f2 rb = __builtin_elementwise_fma(f2{1.140f, 2.032f}, f2{Vf, Uf}, f2{Yf, Yf});
    uint32_t p = pack_u8(rb.x, 0, 0u);
    p = pack_u8(__builtin_fmaf(-0.581f, Vf, __builtin_fmaf(-0.394f, Uf, Yf)), 1, p);
    return pack_u8(rb.y, 2, p);
}

// Two horizontally adjacent pixels sharing one (U, V) sample: the same per-element operations as
// yuv_to_rgba, with each fma issued for both pixels as one v_pk_fma_f32.
__device__ __forceinline__ void yuv2_to_rgba(uint32_t y0, uint32_t y1, uint32_t u, uint32_t v, uint32_t& p0,
                                             uint32_t& p1) {
    typedef float f2 __attribute__((ext_vector_type(2)));
    const f2 Y = {(float)y0, (float)y1};
    const float Uf = (float)u - 128.f, Vf = (float)v - 128.f;
    const f2 R = __builtin_elementwise_fma(f2{1.140f, 1.140f}, f2{Vf, Vf}, Y);
    const f2 G = __builtin_elementwise_fma(f2{-0.581f, -0.581f}, f2{Vf, Vf},
                                           __builtin_elementwise_fma(f2{-0.394f, -0.394f}, f2{Uf, Uf}, Y));
    const f2 B = __builtin_elementwise_fma(f2{2.032f, 2.032f}, f2{Uf, Uf}, Y);
    p0 = pack_u8(B.x, 2, pack_u8(G.x, 1, pack_u8(R.x, 0, 0u)));
    p1 = pack_u8(B.y, 2, pack_u8(G.y, 1, pack_u8(R.y, 0, 0u)));
}

// yuv_to_rgba of two pixels with their own chroma: bytes 0 and 1 of y, u, v; each fma issued for both
// as one v_pk_fma_f32 (every element rounded as yuv_to_rgba's)
__device__ __forceinline__ void yuv_pair_to_rgba(uint32_t y, uint32_t u, uint32_t v, uint32_t& p0, uint32_t& p1) {
    typedef float f2 __attribute__((ext_vector_type(2)));
    const f2 Y = {(float)(y & 255u), (float)((y >> 8) & 255u)};
    const f2 U = f2{(float)(u & 255u), (float)((u >> 8) & 255u)} - f2{128.f, 128.f};
    const f2 V = f2{(float)(v & 255u), (float)((v >> 8) & 255u)} - f2{128.f, 128.f};
    const f2 R = __builtin_elementwise_fma(f2{1.140f, 1.140f}, V, Y);
    const f2 G = __builtin_elementwise_fma(f2{-0.581f, -0.581f}, V, __builtin_elementwise_fma(f2{-0.394f, -0.394f}, U, Y));
    const f2 B = __builtin_elementwise_fma(f2{2.032f, 2.032f}, U, Y);
    p0 = pack_u8(B.x, 2, pack_u8(G.x, 1, pack_u8(R.x, 0, 0u)));
    p1 = pack_u8(B.y, 2, pack_u8(G.y, 1, pack_u8(R.y, 0, 0u)));
}

// yuv2_to_rgba with the chroma already as the floats u - 128, v - 128
__device__ __forceinline__ void yuv2_to_rgba_c(uint32_t y0, uint32_t y1, float Uf, float Vf, uint32_t& p0,
                                               uint32_t& p1) {
    typedef float f2 __attribute__((ext_vector_type(2)));
    const f2 Y = {(float)y0, (float)y1};
    const f2 R = __builtin_elementwise_fma(f2{1.140f, 1.140f}, f2{Vf, Vf}, Y);
    const f2 G = __builtin_elementwise_fma(f2{-0.581f, -0.581f}, f2{Vf, Vf},
                                           __builtin_elementwise_fma(f2{-0.394f, -0.394f}, f2{Uf, Uf}, Y));
    const f2 B = __builtin_elementwise_fma(f2{2.032f, 2.032f}, f2{Uf, Uf}, Y);
    p0 = pack_u8(B.x, 2, pack_u8(G.x, 1, pack_u8(R.x, 0, 0u)));
    p1 = pack_u8(B.y, 2, pack_u8(G.y, 1, pack_u8(R.y, 0, 0u)));
}

// Vignette correction of a source pixel: multiply(rgba, vignette_map) = MulOpSpecial_c4
// (cudaarithm/src/cuda/mul_mat.cu:198-214): saturate_cast<uchar>(c * g) per channel.
__device__ __forceinline__ uint32_t vig_mul(uint32_t rgba, float g) {
    uint32_t v = pack_u8((float)(rgba & 255u) * g, 0, 0u);
    v = pack_u8((float)((rgba >> 8) & 255u) * g, 1, v);
    v = pack_u8((float)((rgba >> 16) & 255u) * g, 2, v);
    return pack_u8((float)(rgba >> 24) * g, 3, v);
}

// 15-bit bilinear weights.  initInterTab2D's table (imgwarp.cpp:211-280) holds
// w = {(32-fx)(32-fy), fx(32-fy), (32-fx)fy, fx fy} * 32 exactly (every product is exact in f32),
// except code 0 whose 32768 saturates to 32767 and the fix-up adds the missing unit to the
// bottom-right tap: {32767, 0, 0, 1}.  For u8 taps that cell rounds to c00 exactly like
// {32768, 0, 0, 0} would ((32767 c00 + c11 + 2^14) >> 15 == c00 for c00, c11 <= 255), so the
// separable form below is bit-identical to the table — pinned by the all-codes remap KAT.
// Out-of-image taps are passed as 0 (BORDER_CONSTANT).  Returns (sum + 2^14) >> 15 per channel.
__device__ __forceinline__ uint32_t bilerp_ch(uint32_t a, uint32_t b, uint32_t c, uint32_t d, uint32_t fx,
                                              uint32_t fy) {
    const uint32_t h0 = (32u - fx) * a + fx * b;  // <= 8160
    const uint32_t h1 = (32u - fx) * c + fx * d;
    return ((32u - fy) * h0 + fy * h1 + 512u) >> 10;
}

// The same sum as one 2-D weighted sum, (w00 a + w01 b + w10 c + w11 d + 2^9) >> 10 with
// w = {(32-fx)(32-fy), fx(32-fy), (32-fx)fy, fx fy} (<= 1024 each, exact in u32): per channel two
// v_perm_b32 pair the taps as u16 halves and two v_dot2_u32_u16 accumulate them.
typedef unsigned short u16x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void bilerp_rgba(uint32_t c00, uint32_t c01, uint32_t c10, uint32_t c11, uint32_t fx,
                                            uint32_t fy, uint32_t (&rgb)[3]) {
    const uint32_t X = fx * 0xFFFFu + 32u;  // (32 - fx) | fx << 16
    const u16x2_t w0 = __builtin_bit_cast(u16x2_t, X * (32u - fy)), w1 = __builtin_bit_cast(u16x2_t, X * fy);
#pragma unroll
    for (int ch = 0; ch < 3; ch++) {
        const uint32_t sel = 0x0C000C00u | ((4u + ch) << 16) | (uint32_t)ch;  // {lo.ch, 0, hi.ch, 0}
        const u16x2_t top = __builtin_bit_cast(u16x2_t, __builtin_amdgcn_perm(c01, c00, sel));
        const u16x2_t bot = __builtin_bit_cast(u16x2_t, __builtin_amdgcn_perm(c11, c10, sel));
        rgb[ch] = __builtin_amdgcn_udot2(bot, w1, __builtin_amdgcn_udot2(top, w0, 512u, false), false) >> 10;
    }
}

// bilerp_rgba's weights at scale 2^16 for fraction code fxy = fx | fy << 5, as two packed 16-bit pairs
// w.x = {W00, W01}, w.y = {W10, W11}: X = {64 (32 - fx), 64 fx} (one 24-bit multiply-add), W0 = X (32 - fy)
// and W1 = X fy per half, so (sum + 2^15) >> 16 is bilerp_rgba's (sum' + 2^9) >> 10 exactly (w = 64 w').
// Every half stays <= 63,488 except code 0's (fx = fy = 0) 65,536: w0 is formed as X (31 - fy) + X with
// a saturating packed add (gfx950 ignores the clamp bit of v_pk_mul_lo_u16, scripts/clamp_probe.hip), so
// that half becomes 65,535 and (65535 c00 + 2^15) >> 16 = c00 for c00 <= 255 — the 15-bit table's own
// {32767, 0, 0, 1} result.  The composite keeps all 1,024 in an LDS table.
__device__ __forceinline__ uint2 bilerp_weights(uint32_t fxy) {
    const uint32_t fx = fxy & 31u, fy = fxy >> 5;
    const uint32_t X = __umul24(fx, 0x3FFFC0u) + 2048u;
    const u16x2_t Xv = __builtin_bit_cast(u16x2_t, X);
    const unsigned short gy = (unsigned short)(31u - fy);
    const u16x2_t w0 = __builtin_elementwise_add_sat(Xv * u16x2_t{gy, gy}, Xv);
    const u16x2_t w1 = Xv * u16x2_t{(unsigned short)fy, (unsigned short)fy};
    return uint2{__builtin_bit_cast(uint32_t, w0), __builtin_bit_cast(uint32_t, w1)};
}

// The bilinear sum with the weight pairs given (from the LDS table): the sum stays below 2^24, so the
// channel is byte 2 of it — perm, perm, dot2, dot2, v_cvt_f32_ubyte2 per channel, values as floats
__device__ __forceinline__ void bilerp_rgba_w(uint32_t c00, uint32_t c01, uint32_t c10, uint32_t c11, uint2 w,
                                              float (&rgb)[3]) {
#pragma unroll
    for (int ch = 0; ch < 3; ch++) {
        const uint32_t sel = 0x0C000C00u | ((4u + ch) << 16) | (uint32_t)ch;  // {lo.ch, 0, hi.ch, 0}
        const u16x2_t top = __builtin_bit_cast(u16x2_t, __builtin_amdgcn_perm(c01, c00, sel));
        const u16x2_t bot = __builtin_bit_cast(u16x2_t, __builtin_amdgcn_perm(c11, c10, sel));
        const uint32_t S = __builtin_amdgcn_udot2(
            bot, __builtin_bit_cast(u16x2_t, w.y),
            __builtin_amdgcn_udot2(top, __builtin_bit_cast(u16x2_t, w.x), 32768u, false), false);
        rgb[ch] = (float)((S >> 16) & 255u);
    }
}

// Direct (global-memory) bilinear sample of one camera at an 8-byte composite entry — the gain feed
// samples and "wide" tiles.  Every load is issued unconditionally from a clamped in-image address;
// taps outside the image and invalid entries are zeroed afterwards.
// global-address-space views (loads through pointers held in LDS / structs would otherwise be flat)
typedef __attribute__((address_space(1))) uint8_t gu8;
typedef __attribute__((address_space(1))) uint16_t gu16;
typedef __attribute__((address_space(1))) uint32_t gu32;
typedef __attribute__((address_space(1))) uint64_t gu64;

// wave-uniform value -> SGPR (scalar loads / branches downstream)
__device__ __forceinline__ int uniform(int v) { return __builtin_amdgcn_readfirstlane(v); }

struct Taps {
    uint32_t c[4];  // packed RGBA of the 4 taps (0 when outside / invalid)
    uint32_t fx, fy;
};

__device__ __forceinline__ void gather_taps_frame(const SourceFrame& f, uint32_t xy, uint32_t code, Taps& t) {
    const bool valid = (code & 0x8000u) != 0;
    const TapCell tc = tap_cell(xy, f.w, f.h);
    const int x0 = tc.x0, x1 = tc.x1, y0 = tc.y0, y1 = tc.y1;
    const int64_t p = f.pitch;
    const uint8_t* Y = f.yuv;
    const uint8_t* U = Y + (int64_t)f.h * p;
    const uint8_t* V = U + (f.w >> 1);
    const int64_t r0 = (int64_t)y0 * p, r1 = (int64_t)y1 * p;
    const int64_t q0 = (int64_t)(y0 >> 1) * p, q1 = (int64_t)(y1 >> 1) * p;
    const uint32_t ya = Y[r0 + x0], yb = Y[r0 + x1], yc = Y[r1 + x0], yd = Y[r1 + x1];
    const uint32_t ua = U[q0 + (x0 >> 1)], ub = U[q0 + (x1 >> 1)], uc = U[q1 + (x0 >> 1)], ud = U[q1 + (x1 >> 1)];
    const uint32_t va = V[q0 + (x0 >> 1)], vb = V[q0 + (x1 >> 1)], vc = V[q1 + (x0 >> 1)], vd = V[q1 + (x1 >> 1)];
    uint32_t ca = yuv_to_rgba(ya, ua, va), cb = yuv_to_rgba(yb, ub, vb);
    uint32_t cc = yuv_to_rgba(yc, uc, vc), cd = yuv_to_rgba(yd, ud, vd);
    if (f.vig) {
        const float* g0 = f.vig + (int64_t)y0 * f.w;
        const float* g1 = f.vig + (int64_t)y1 * f.w;
        ca = vig_mul(ca, g0[x0]);
        cb = vig_mul(cb, g0[x1]);
        cc = vig_mul(cc, g1[x0]);
        cd = vig_mul(cd, g1[x1]);
    }
    // texture-convention entries (make_entry_tex): clamp addressing, every (clamped) tap is used
    const bool all = (code & kCodeTex) != 0;
    t.c[0] = (valid && (all || (tc.ix0 && tc.iy0))) ? ca : 0u;
    t.c[1] = (valid && (all || (tc.ix1 && tc.iy0))) ? cb : 0u;
    t.c[2] = (valid && (all || (tc.ix0 && tc.iy1))) ? cc : 0u;
    t.c[3] = (valid && (all || (tc.ix1 && tc.iy1))) ? cd : 0u;
    t.fx = all ? (code & 255u) : (code & 31u);
    t.fy = all ? ((code >> 17) & 255u) : ((code >> 5) & 31u);
}

// fl32(t / 255) for a byte t: the product with the rounded reciprocal, corrected by one residual step
// (two FMAs) — equal to the correctly rounded quotient for every t in 0..255
// (tests/test_tex_division.py), at 3 instead of ~10 instructions.
__device__ __forceinline__ float div255(uint32_t t) {
    const float x = (float)t, r = 1.f / 255.f;
    const float q = x * r;
    return __builtin_fmaf(__builtin_fmaf(-q, 255.f, x), r, q);
}

// The texture unit's linear filter as oracle/octvr_oracle.c orc_fast_remap_tex_rgba models it (the
// texture-convention mode, make_entry_tex): per channel the f32 sum of the four normalized texels with
// weights from the 8-bit fractions, in the oracle's order, then saturate_cast<uchar>(v * 255) (round half
// to even).  Exact f32 operations (no contraction; div255 = the correctly rounded t / 255), so bit-equal to
// it.  (c00, c10, c01, c11): taps (x0, y0), (x1, y0), (x0, y1), (x1, y1); the result as floats of bytes.
__device__ __forceinline__ void tex_bilerp_f(uint32_t c00, uint32_t c10, uint32_t c01, uint32_t c11, uint32_t a8,
                                             uint32_t b8, float (&rgb)[3]) {
    const float a = (float)a8 / 256.f, b = (float)b8 / 256.f;  // exact: 8-bit fractions
    const float w00 = (1.f - a) * (1.f - b), w10 = a * (1.f - b), w01 = (1.f - a) * b, w11 = a * b;
#pragma unroll
    for (int ch = 0; ch < 3; ch++) {
        const uint32_t sh = 8u * ch;
        const float t00 = div255((c00 >> sh) & 255u), t10 = div255((c10 >> sh) & 255u);
        const float t01 = div255((c01 >> sh) & 255u), t11 = div255((c11 >> sh) & 255u);
        const float v = (w00 * t00 + w10 * t10 + w01 * t01 + w11 * t11) * 255.f;
        rgb[ch] = !(v > 0.f) ? 0.f : v >= 255.f ? 255.f : __builtin_rintf(v);
    }
}
__device__ __forceinline__ void tex_bilerp(uint32_t c00, uint32_t c10, uint32_t c01, uint32_t c11, uint32_t a8,
                                           uint32_t b8, uint32_t (&rgb)[3]) {
    float f[3];
    tex_bilerp_f(c00, c10, c01, c11, a8, b8, f);
#pragma unroll
    for (int ch = 0; ch < 3; ch++) rgb[ch] = (uint32_t)f[ch];
}

__device__ __forceinline__ void gather_taps(const FrameSet& fs, uint32_t xy, uint32_t code, Taps& t) {
    gather_taps_frame(fs.f[(code >> 10) & 31u], xy, code, t);
}


struct QuadOut {
    uint32_t y01, y23;  // two Y bytes of each row
    uint32_t u, v;
};

typedef float f32x2_t __attribute__((ext_vector_type(2)));

// The library's own RGB -> YUV420P (it stands in for NPP's closed nppiRGBToYUV420; oracle/octvr_oracle.c
// rgb_quad_to_yuv is the same definition).  NPP documents (and its YUV -> RGB, yuv_to_rgba above,
// inverts) Y = 0.299 R + 0.587 G + 0.114 B, U = 0.492 (B - Y) + 128, V = 0.877 (R - Y) + 128, i.e.
// U' = -0.147 R - 0.289 G + 0.436 B, V' = 0.615 R - 0.515 G - 0.100 B.  In fixed point, chroma as the
// quad's mean (4:2:0):
//   Y = (77 R + 150 G + 29 B + 128) >> 8                                  (0..255, no clamp needed)
//   U = (sum over the quad of -38 R' - 74 G' + 112 B' + 131584) >> 10     (scale 256; 16..240)
//   V = clamp((sum over the quad of 79 R' - 66 G' - 13 B' + 65792) >> 9, 0, 255)   (scale 128)
// with R' = R - 128 etc. (each chroma vector sums to 0, so grey is exact; V's scale-128 vector fits
// i8).  Every coefficient is within 0.002 of NPP's; a YUV -> RGB -> YUV round trip through the
// staging conversion keeps U and V within +-1 (tests/test_oracle_color.py).  Per pixel one
// v_dot4_u32_u8 (Y lands in byte 1) and two v_dot4c_i32_i8 on the pixel xor 0x808080.
// px[p]: R | G << 8 | B << 16 (byte 3 is ignored: every coefficient vector has byte 3 = 0).
__device__ __forceinline__ QuadOut quad_yuv(const uint32_t (&px)[4]) {
    uint32_t yr[4];
    int au = 0, av = 0;
#pragma unroll
    for (int p = 0; p < 4; p++) {
        const uint32_t c = px[p];  // byte 3 meets coefficient 0 in all three products
        yr[p] = __builtin_amdgcn_udot4(c, 0x001D964Du, 128u, false);  // {77, 150, 29, 0}
        const int s = (int)(c ^ 0x00808080u);
        au = __builtin_amdgcn_sdot4(s, 0x0070B6DA, au, false);  // {-38, -74, 112, 0}
        av = __builtin_amdgcn_sdot4(s, 0x00F3BE4F, av, false);  // {79, -66, -13, 0}
    }
    QuadOut q;
    q.y01 = __builtin_amdgcn_perm(yr[1], yr[0], 0x0C0C0501u);  // byte 1 of each
    q.y23 = __builtin_amdgcn_perm(yr[3], yr[2], 0x0C0C0501u);
    q.u = (uint32_t)(au + 131584) >> 10;
    q.v = (uint32_t)min(max((av + 65792) >> 9, 0), 255);
    return q;
}

// gain + pack: sat_u8(rne(c * g)) per channel with v_cvt_pk_u8_f32 (round half to even, saturating,
// NaN -> 0), then quad_yuv.  gain2[p] = {g, g}: (B, R) go through one v_pk_mul_f32.
__device__ __forceinline__ QuadOut finish_quad2f(const float (&rgb)[4][3], const f32x2_t (&gain2)[4]) {
    uint32_t px[4];
#pragma unroll
    for (int p = 0; p < 4; p++) {
        const f32x2_t br = f32x2_t{rgb[p][2], rgb[p][0]} * gain2[p];
        const float G = rgb[p][1] * gain2[p].x;
        px[p] = pack_u8(br.x, 2, pack_u8(G, 1, pack_u8(br.y, 0, 0u)));
    }
    return quad_yuv(px);
}

__device__ __forceinline__ QuadOut finish_quad2(const uint32_t (&rgb)[4][3], const f32x2_t (&gain2)[4]) {
    float f[4][3];
#pragma unroll
    for (int p = 0; p < 4; p++)
#pragma unroll
        for (int ch = 0; ch < 3; ch++) f[p][ch] = (float)rgb[p][ch];
    return finish_quad2f(f, gain2);
}

// quad_yuv of channel values already in 0..255 (no gain): packed directly
__device__ __forceinline__ QuadOut finish_quad_u8(const uint32_t (&rgb)[4][3]) {
    uint32_t px[4];
#pragma unroll
    for (int p = 0; p < 4; p++) px[p] = rgb[p][0] | (rgb[p][1] << 8) | (rgb[p][2] << 16);
    return quad_yuv(px);
}

__device__ __forceinline__ QuadOut finish_quad(const uint32_t (&rgb)[4][3], const float (&gain)[4]) {
    const f32x2_t g2[4] = {{gain[0], gain[0]}, {gain[1], gain[1]}, {gain[2], gain[2]}, {gain[3], gain[3]}};
    return finish_quad2(rgb, g2);
}

// The output frame as a buffer resource: stores of a quad outside W x H get an offset past the
// range and are dropped by the hardware, so every lane issues the same stores (no branch) and the
// per-iteration count of outstanding vector-memory operations is fixed.
struct OutFrame {
    __amdgpu_buffer_rsrc_t rsrc;
    uint32_t pitch;
    uint32_t u_off, v_off;  // byte offsets of the U and V planes
};
constexpr uint32_t kDropOffset = 0x7FFFFFC0u;  // > any valid output byte (host: frame < 2^31 - 64 B)
// Cache-policy bits of the output-frame stores (gfx950: 1 sc0, 2 nt, 16 sc1).  nt: streaming stores (no
// launch reads the frame back): C2 composite 46.1-47.6 against 47.4-51.6 us with sc1 (six interleaved
// pairs, round 5; sc1 had been 1.5 % faster than the default policy), C4 unchanged; nt | sc1 and sc0 | nt
// were no better.
constexpr int kOutPolicy = 2;

__device__ __forceinline__ void store_quad(const OutFrame& o, const QuadOut& q, int x, int y, bool in) {
    const uint32_t oy = in ? (uint32_t)y * o.pitch + (uint32_t)x : kDropOffset;
    const uint32_t oc = in ? (uint32_t)(y >> 1) * o.pitch + (uint32_t)(x >> 1) : kDropOffset;
    __builtin_amdgcn_raw_buffer_store_b16((uint16_t)q.y01, o.rsrc, oy, 0, kOutPolicy);
    __builtin_amdgcn_raw_buffer_store_b16((uint16_t)q.y23, o.rsrc, in ? oy + o.pitch : kDropOffset, 0, kOutPolicy);
    __builtin_amdgcn_raw_buffer_store_b8((uint8_t)q.u, o.rsrc, in ? oc + o.u_off : kDropOffset, 0, kOutPolicy);
    __builtin_amdgcn_raw_buffer_store_b8((uint8_t)q.v, o.rsrc, in ? oc + o.v_off : kDropOffset, 0, kOutPolicy);
}


__device__ __forceinline__ OutFrame make_out_frame(uint8_t* out, int W, int H, int64_t out_pitch) {
    OutFrame of;
    of.pitch = (uint32_t)out_pitch;
    of.u_off = (uint32_t)H * (uint32_t)out_pitch;
    of.v_off = of.u_off + (uint32_t)(W >> 1);
    of.rsrc = __builtin_amdgcn_make_buffer_rsrc(out, 0, (int)((uint32_t)out_pitch * (uint32_t)(H + H / 2)), 0x00020000);
    return of;
}


}  // namespace octvr
