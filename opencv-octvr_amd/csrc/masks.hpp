// masks.hpp — host-side camera mask rasterisation (camera.cpp:72-123, 146-187); see masks.cpp.
#pragma once
#include <cstddef>
#include <cstdint>
#include <vector>

namespace octvr {

// cv::fillPoly(img, {pts}, color) on a w x h CV_8U image, lineType 8, shift 0; pts = x0,y0,x1,y1,...
void fill_poly_u8(uint8_t* img, int w, int h, const int* pts, int npts, uint8_t color);

// cv::imdecode(png, IMREAD_COLOR) restricted to PNG; returns w*h*3 bytes in R,G,B order.
// expect_w > 0: the image must be expect_w x expect_h (checked on the IHDR, before inflating)
std::vector<uint8_t> png_decode_rgb(const uint8_t* buf, size_t n, int* w, int* h, int expect_w = 0, int expect_h = 0);

}  // namespace octvr
