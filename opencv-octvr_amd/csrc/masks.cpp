// masks.cpp — per-camera exclude / include masks of `vr::Camera` (camera.cpp:72-123, 146-187), built
// once per rig on the host (the reference builds them on the CPU in the Camera constructor) and
// uploaded for lut_build_kernel's per-pixel lookups.
//
//  * polygonal areas: cv::fillPoly(mask, {points}, 255) with lineType 8, shift 0
//    (imgproc/src/drawing.cpp:1894-1917 -> CollectPolyEdges :1196-1248 -> FillEdgeCollection
//    :1262-1405; every polygon edge is also drawn by Line :239-265 / LineIterator :153-236 with
//    clipLine :80-137);
//  * png areas: cv::imdecode(bytes, IMREAD_COLOR) (imgcodecs/src/grfmt_png.cpp:240-286: strip_16,
//    strip_alpha, palette_to_rgb, gray 1/2/4 -> 8 expansion, gray_to_rgb, interlace handling), red
//    channel -> exclude, green -> include (camera.cpp:174-178).
#include <zlib.h>

#include <algorithm>
#include <climits>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "host_common.hpp"
#include "masks.hpp"

namespace octvr {

namespace {

constexpr int kXYShift = 16, kXYOne = 1 << kXYShift;  // drawing.cpp:46

// clipLine(Size, pt1, pt2) (drawing.cpp:80-137): Cohen-Sutherland against [0,w-1]x[0,h-1] in int64.
bool clip_segment(int w, int h, int& ax, int& ay, int& bx, int& by) {
    if (w <= 0 || h <= 0) return false;
    int64_t x1 = ax, y1 = ay, x2 = bx, y2 = by;
    const int64_t right = w - 1, bottom = h - 1;
    auto code = [&](int64_t x, int64_t y) { return (x < 0) + (x > right) * 2 + (y < 0) * 4 + (y > bottom) * 8; };
    int c1 = code(x1, y1), c2 = code(x2, y2);
    if ((c1 & c2) == 0 && (c1 | c2) != 0) {
        if (c1 & 12) {
            const int64_t a = c1 < 8 ? 0 : bottom;
            x1 += (a - y1) * (x2 - x1) / (y2 - y1);
            y1 = a;
            c1 = (x1 < 0) + (x1 > right) * 2;
        }
        if (c2 & 12) {
            const int64_t a = c2 < 8 ? 0 : bottom;
            x2 += (a - y2) * (x2 - x1) / (y2 - y1);
            y2 = a;
            c2 = (x2 < 0) + (x2 > right) * 2;
        }
        if ((c1 & c2) == 0 && (c1 | c2) != 0) {
            if (c1) {
                const int64_t a = c1 == 1 ? 0 : right;
                y1 += (a - x1) * (y2 - y1) / (x2 - x1);
                x1 = a;
                c1 = 0;
            }
            if (c2) {
                const int64_t a = c2 == 1 ? 0 : right;
                y2 += (a - x2) * (y2 - y1) / (x2 - x1);
                x2 = a;
                c2 = 0;
            }
        }
        ax = (int)x1;
        ay = (int)y1;
        bx = (int)x2;
        by = (int)y2;
    }
    return (c1 | c2) == 0;
}

// Line(img, pt1, pt2, color, 8) through LineIterator(connectivity 8, left_to_right): Bresenham with
// a major step every pixel and the minor step added while err < 0.
void draw_segment(uint8_t* img, int w, int h, int ax, int ay, int bx, int by, uint8_t color) {
    if ((unsigned)ax >= (unsigned)w || (unsigned)bx >= (unsigned)w || (unsigned)ay >= (unsigned)h ||
        (unsigned)by >= (unsigned)h)
        if (!clip_segment(w, h, ax, ay, bx, by)) return;
    int dx = bx - ax, dy = by - ay;
    if (dx < 0) {  // left_to_right: start from pt2, flip both deltas
        dx = -dx;
        dy = -dy;
        ax = bx;
        ay = by;
    }
    const int ystep = dy < 0 ? -1 : 1;
    dy = dy < 0 ? -dy : dy;
    int major_x = 1, major_y = 0, minor_x = 0, minor_y = ystep;  // minusStep / plusStep
    if (dy > dx) {
        std::swap(dx, dy);
        major_x = 0;
        major_y = ystep;
        minor_x = 1;
        minor_y = 0;
    }
    int err = dx - (dy + dy);
    const int plus_delta = dx + dx, minus_delta = -(dy + dy);
    int x = ax, y = ay;
    for (int i = 0; i <= dx; i++) {
        img[(size_t)y * w + x] = color;
        const bool m = err < 0;
        err += minus_delta + (m ? plus_delta : 0);
        x += major_x + (m ? minor_x : 0);
        y += major_y + (m ? minor_y : 0);
    }
}

struct Edge {
    int y0, y1, x, dx;
    int next;  // index into the edge table, -1 = end of the active list
};

}  // namespace

void fill_poly_u8(uint8_t* img, int w, int h, const int* pts, int npts, uint8_t color) {
    if (npts <= 0) return;
    // CollectPolyEdges (shift 0, no offset): x in 16.16 fixed point, every edge also drawn as a line
    std::vector<Edge> edges;
    edges.reserve(npts + 2);
    int px0 = pts[2 * (npts - 1)] << kXYShift, py0 = pts[2 * (npts - 1) + 1];
    for (int i = 0; i < npts; i++) {
        const int px1 = pts[2 * i] << kXYShift, py1 = pts[2 * i + 1];
        draw_segment(img, w, h, (px0 + (kXYOne >> 1)) >> kXYShift, py0, (px1 + (kXYOne >> 1)) >> kXYShift, py1, color);
        if (py0 != py1) {
            Edge e;
            if (py0 < py1) {
                e.y0 = py0;
                e.y1 = py1;
                e.x = px0;
            } else {
                e.y0 = py1;
                e.y1 = py0;
                e.x = px1;
            }
            e.dx = (px1 - px0) / (py1 - py0);
            e.next = -1;
            edges.push_back(e);
        }
        px0 = px1;
        py0 = py1;
    }
    // FillEdgeCollection
    const int total = (int)edges.size();
    if (total < 2) return;
    int y_max = INT_MIN, x_max = INT_MIN, y_min = INT_MAX, x_min = INT_MAX;
    for (const Edge& e : edges) {
        const int x1 = e.x + (e.y1 - e.y0) * e.dx;
        y_min = std::min(y_min, e.y0);
        y_max = std::max(y_max, e.y1);
        x_min = std::min({x_min, e.x, x1});
        x_max = std::max({x_max, e.x, x1});
    }
    if (y_max < 0 || y_min >= h || x_max < 0 || x_min >= (w << kXYShift)) return;
    std::sort(edges.begin(), edges.end(), [](const Edge& a, const Edge& b) {
        return a.y0 - b.y0 ? a.y0 < b.y0 : a.x - b.x ? a.x < b.x : a.dx < b.dx;
    });
    Edge sentinel{INT_MAX, 0, 0, 0, -1};
    edges.push_back(sentinel);   // [total]: stops the insertion scan
    edges.push_back(sentinel);   // [total+1]: head of the active list
    const int head = total + 1;
    edges[head].next = -1;
    int i = 0, cur = 0;
    y_max = std::min(y_max, h);
    for (int y = edges[cur].y0; y < y_max; y++) {
        int prelast = head, last = edges[head].next, keep;
        int sort_flag = 0, draw = 0;
        const bool clipline = y < 0;
        while (last >= 0 || edges[cur].y0 == y) {
            if (last >= 0 && edges[last].y1 == y) {  // edge ends on this row: unlink it
                edges[prelast].next = edges[last].next;
                last = edges[last].next;
                continue;
            }
            keep = prelast;
            if (last >= 0 && (edges[cur].y0 > y || edges[last].x < edges[cur].x)) {
                prelast = last;
                last = edges[last].next;
            } else if (i < total) {  // edge starts on this row: link it before `last`
                edges[prelast].next = cur;
                edges[cur].next = last;
                prelast = cur;
                cur = ++i;
            } else {
                break;
            }
            if (draw) {
                if (!clipline) {
                    int x1 = edges[keep].x, x2 = edges[prelast].x;
                    if (x1 > x2) std::swap(x1, x2);
                    x1 = (x1 + kXYOne - 1) >> kXYShift;
                    x2 = x2 >> kXYShift;
                    if (x1 < w && x2 >= 0) {
                        x1 = std::max(x1, 0);
                        x2 = std::min(x2, w - 1);
                        memset(img + (size_t)y * w + x1, color, (size_t)(x2 - x1 + 1));
                    }
                }
                edges[keep].x += edges[keep].dx;
                edges[prelast].x += edges[prelast].dx;
            }
            draw ^= 1;
        }
        // bubble-sort the active list by x
        keep = -1;
        do {
            prelast = head;
            last = edges[head].next;
            while (last != keep && edges[last].next >= 0) {
                const int te = edges[last].next;
                if (edges[last].x > edges[te].x) {
                    edges[prelast].next = te;
                    edges[last].next = edges[te].next;
                    edges[te].next = last;
                    prelast = te;
                    sort_flag = 1;
                } else {
                    prelast = last;
                    last = te;
                }
            }
            keep = prelast;
        } while (sort_flag && keep != edges[head].next && keep != head);
    }
}

// ---------------------------------------------------------------------------------------------
// PNG -> 8-bit RGB, as libpng delivers it to OpenCV's PngDecoder for IMREAD_COLOR.
// ---------------------------------------------------------------------------------------------
namespace {

uint32_t be32(const uint8_t* p) { return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]; }

int paeth(int a, int b, int c) {
    const int p = a + b - c, pa = std::abs(p - a), pb = std::abs(p - b), pc = std::abs(p - c);
    return (pa <= pb && pa <= pc) ? a : (pb <= pc ? b : c);
}

// Undo the per-row filters of one (sub-)image in place; returns the offset past it.
size_t unfilter(uint8_t* d, size_t avail, int w, int h, int bits_pp, std::vector<uint8_t>& rows) {
    const size_t stride = ((size_t)w * bits_pp + 7) / 8;
    const int bpp = std::max(1, bits_pp / 8);
    if (w == 0 || h == 0) return 0;
    REQUIRE(avail >= (stride + 1) * h, "png: truncated image data");
    std::vector<uint8_t> prev(stride, 0);
    rows.resize(stride * h);
    for (int y = 0; y < h; y++) {
        const uint8_t f = d[(stride + 1) * y];
        uint8_t* r = d + (stride + 1) * y + 1;
        for (size_t x = 0; x < stride; x++) {
            const int a = x >= (size_t)bpp ? r[x - bpp] : 0, b = prev[x], c = x >= (size_t)bpp ? prev[x - bpp] : 0;
            int v = r[x];
            switch (f) {
                case 0: break;
                case 1: v += a; break;
                case 2: v += b; break;
                case 3: v += (a + b) >> 1; break;
                case 4: v += paeth(a, b, c); break;
                default: throw OctvrError(OCTVR_E_INVALID, "png: bad filter type");
            }
            r[x] = (uint8_t)v;
        }
        memcpy(prev.data(), r, stride);
        memcpy(rows.data() + stride * y, r, stride);
    }
    return (stride + 1) * h;
}

}  // namespace

std::vector<uint8_t> png_decode_rgb(const uint8_t* buf, size_t n, int* out_w, int* out_h, int expect_w, int expect_h) {
    static const uint8_t sig[8] = {137, 80, 78, 71, 13, 10, 26, 10};
    REQUIRE(n >= 8 && memcmp(buf, sig, 8) == 0, "png: bad signature (only PNG masks are supported)");
    int w = 0, h = 0, depth = 0, ctype = 0, interlace = 0;
    std::vector<uint8_t> idat, plte;
    for (size_t p = 8; p + 12 <= n;) {
        const uint32_t len = be32(buf + p);
        REQUIRE(p + 12 + (size_t)len <= n, "png: truncated chunk");
        const uint8_t* t = buf + p + 4;
        const uint8_t* d = buf + p + 8;
        if (!memcmp(t, "IHDR", 4)) {
            REQUIRE(len >= 13, "png: bad IHDR");
            w = (int)be32(d);
            h = (int)be32(d + 4);
            depth = d[8];
            ctype = d[9];
            interlace = d[12];
        } else if (!memcmp(t, "PLTE", 4)) {
            plte.assign(d, d + len);
        } else if (!memcmp(t, "IDAT", 4)) {
            idat.insert(idat.end(), d, d + len);
        } else if (!memcmp(t, "IEND", 4)) {
            break;
        }
        p += 12 + (size_t)len;
    }
    REQUIRE(w > 0 && h > 0, "png: missing IHDR");
    const int chans = ctype == 0 ? 1 : ctype == 2 ? 3 : ctype == 3 ? 1 : ctype == 4 ? 2 : ctype == 6 ? 4 : 0;
    REQUIRE(chans > 0, "png: bad colour type");
    // the colour type / bit depth pairs the PNG spec allows (libpng rejects the others, so
    // cv::imdecode fails and camera.cpp:175-176 asserts): gray 1/2/4/8/16, palette 1/2/4/8,
    // RGB / gray+alpha / RGBA 8/16
    const bool legal = ctype == 0   ? (depth == 1 || depth == 2 || depth == 4 || depth == 8 || depth == 16)
                       : ctype == 3 ? (depth == 1 || depth == 2 || depth == 4 || depth == 8)
                                    : (depth == 8 || depth == 16);
    REQUIRE(legal, "png: bit depth not allowed for this colour type");
    // size check against the camera before anything is inflated or allocated
    if (expect_w > 0) REQUIRE(w == expect_w && h == expect_h, "png mask size differs from the camera's exclude mask");
    REQUIRE((uint64_t)w * (uint64_t)h <= ((uint64_t)1 << 28), "png: image too large for a mask");
    REQUIRE(ctype != 3 || !plte.empty(), "png: palette image without PLTE");
    const int bits_pp = chans * depth;
    // inflate the whole stream (its size is bounded by the passes' (stride + 1) * rows)
    size_t raw_n = 0;
    static const int ax0[7] = {0, 4, 0, 2, 0, 1, 0}, ay0[7] = {0, 0, 4, 0, 2, 0, 1};
    static const int adx[7] = {8, 8, 4, 4, 2, 2, 1}, ady[7] = {8, 8, 8, 4, 4, 2, 2};
    auto pass_dim = [&](int k, int* pw, int* ph) {
        *pw = interlace ? (w - ax0[k] + adx[k] - 1) / adx[k] : w;
        *ph = interlace ? (h - ay0[k] + ady[k] - 1) / ady[k] : h;
        if (*pw <= 0 || *ph <= 0) *pw = *ph = 0;
    };
    const int passes = interlace ? 7 : 1;
    for (int k = 0; k < passes; k++) {
        int pw, ph;
        pass_dim(k, &pw, &ph);
        if (pw) raw_n += (((size_t)pw * bits_pp + 7) / 8 + 1) * ph;
    }
    std::vector<uint8_t> raw(raw_n);
    uLongf got = (uLongf)raw_n;
    REQUIRE(uncompress(raw.data(), &got, idat.data(), (uLong)idat.size()) == Z_OK && got == raw_n,
            "png: corrupt image data");
    std::vector<uint8_t> rgb((size_t)w * h * 3), rows;
    size_t off = 0;
    for (int k = 0; k < passes; k++) {
        int pw, ph;
        pass_dim(k, &pw, &ph);
        if (!pw) continue;
        off += unfilter(raw.data() + off, raw_n - off, pw, ph, bits_pp, rows);
        const size_t stride = ((size_t)pw * bits_pp + 7) / 8;
        for (int y = 0; y < ph; y++) {
            const uint8_t* r = rows.data() + stride * y;
            for (int x = 0; x < pw; x++) {
                auto sample = [&](int c) -> int {  // channel c of pixel x, 8-bit (strip_16 keeps the high byte)
                    if (depth == 16) return r[((size_t)x * chans + c) * 2];
                    if (depth == 8) return r[(size_t)x * chans + c];
                    const int per = 8 / depth, sh = 8 - depth * (x % per + 1);
                    return (r[x / per] >> sh) & ((1 << depth) - 1);
                };
                uint8_t R, G, B;
                if (ctype == 3) {
                    const int idx = sample(0);
                    REQUIRE((size_t)idx * 3 + 2 < plte.size(), "png: palette index out of range");
                    R = plte[idx * 3];
                    G = plte[idx * 3 + 1];
                    B = plte[idx * 3 + 2];
                } else if (ctype == 0 || ctype == 4) {
                    int g = sample(0);
                    if (depth < 8) g = g * 255 / ((1 << depth) - 1);  // expand_gray_1_2_4_to_8
                    R = G = B = (uint8_t)g;
                } else {
                    R = (uint8_t)sample(0);
                    G = (uint8_t)sample(1);
                    B = (uint8_t)sample(2);
                }
                const int X = interlace ? ax0[k] + x * adx[k] : x, Y = interlace ? ay0[k] + y * ady[k] : y;
                uint8_t* o = rgb.data() + ((size_t)Y * w + X) * 3;
                o[0] = R;
                o[1] = G;
                o[2] = B;
            }
        }
    }
    *out_w = w;
    *out_h = h;
    return rgb;
}

}  // namespace octvr
