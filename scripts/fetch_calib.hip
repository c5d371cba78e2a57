// FETCH_SIZE calibration for the access widths this library uses (MI355X_MICROARCH.md, HBM: "on gfx950
// FETCH_SIZE reports exactly half of the bytes of a wide coalesced streaming read ... other access widths
// are uncalibrated").  Each kernel reads a known number of bytes once from a 1 GiB buffer (4x the
// Infinity Cache, so nothing is re-read on die) and sums them into one word per workgroup:
//   w16   16 B per lane, consecutive lanes consecutive (the composite's entry loads)
//   w8    8 B per lane, consecutive (the staging loads' luma rows)
//   w4    4 B per lane, consecutive (chroma staging loads)
//   seg8  16 lanes x 8 B = one 128-B segment per row, rows 4 KiB apart (a blend wave's 32-pixel row of G0)
//   seg4  16 lanes x 4 B = one 64-B segment per row (a blend wave's u8 weight row pair start, widened)
// Run under `rocprofv3 --pmc FETCH_SIZE` (scripts/fetch_calib.sh); the kernel names carry the byte counts.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

constexpr size_t kBuf = size_t(1) << 30;

template <int W>
__global__ void __launch_bounds__(256) stream_read(const uint8_t* __restrict__ src, size_t bytes, uint32_t* out) {
    uint32_t acc = 0;
    const size_t step = (size_t)gridDim.x * 256 * W;
    for (size_t o = ((size_t)blockIdx.x * 256 + threadIdx.x) * W; o + W <= bytes; o += step) {
        if constexpr (W == 16) {
            const uint4 v = *reinterpret_cast<const uint4*>(src + o);
            acc += v.x ^ v.y ^ v.z ^ v.w;
        } else if constexpr (W == 8) {
            const uint2 v = *reinterpret_cast<const uint2*>(src + o);
            acc += v.x ^ v.y;
        } else {
            acc += *reinterpret_cast<const uint32_t*>(src + o);
        }
    }
    if (acc == 0x12345678u) out[blockIdx.x] = acc;  // keeps the loads
}

// one W-byte word per lane, 16 lanes per row segment, row segments 4 KiB apart
template <int W>
__global__ void __launch_bounds__(256) segment_read(const uint8_t* __restrict__ src, size_t rows, uint32_t* out) {
    uint32_t acc = 0;
    const size_t seg = ((size_t)blockIdx.x * 256 + threadIdx.x) / 16, lane = threadIdx.x & 15;
    const size_t nseg = (size_t)gridDim.x * 16;
    for (size_t r = seg; r < rows; r += nseg) {
        const uint8_t* p = src + r * 4096 + lane * W;
        if constexpr (W == 8) {
            const uint2 v = *reinterpret_cast<const uint2*>(p);
            acc += v.x ^ v.y;
        } else {
            acc += *reinterpret_cast<const uint32_t*>(p);
        }
    }
    if (acc == 0x12345678u) out[blockIdx.x] = acc;
}

int main() {
    uint8_t* buf = nullptr;
    uint32_t* out = nullptr;
    if (hipMalloc(&buf, kBuf) != hipSuccess || hipMalloc(&out, 1 << 20) != hipSuccess) return 1;
    if (hipMemset(buf, 1, kBuf) != hipSuccess) return 1;
    const int blocks = 256 * 8;
    const size_t rows = kBuf / 4096;
    for (int rep = 0; rep < 3; rep++) {
        hipLaunchKernelGGL(stream_read<16>, dim3(blocks), dim3(256), 0, 0, buf, kBuf, out);
        hipLaunchKernelGGL(stream_read<8>, dim3(blocks), dim3(256), 0, 0, buf, kBuf, out);
        hipLaunchKernelGGL(stream_read<4>, dim3(blocks), dim3(256), 0, 0, buf, kBuf, out);
        hipLaunchKernelGGL(segment_read<8>, dim3(blocks), dim3(256), 0, 0, buf, rows, out);
        hipLaunchKernelGGL(segment_read<4>, dim3(blocks), dim3(256), 0, 0, buf, rows, out);
    }
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    printf("bytes: stream %zu each; segments %zu rows x {128, 64} B = %zu / %zu\n", kBuf, rows, rows * 128, rows * 64);
    (void)hipFree(buf);
    (void)hipFree(out);
    return 0;
}
