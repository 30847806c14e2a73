// FETCH_SIZE / WRITE_SIZE calibration for the access widths the extractor kernels use
// (MI355X_MICROARCH.md §HBM: "other access widths are uncalibrated: calibrate on a known byte
// count in your own access pattern").  Each kernel streams a known number of bytes of a 1 GiB
// buffer (past the 256 MiB Infinity Cache) with one access width; run it under
//   rocprofv3 --pmc FETCH_SIZE --kernel-trace -- ./fetch_cal      (then WRITE_SIZE separately)
// and divide the counter by the byte count printed here.
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr size_t kBytes = size_t(1) << 30;

__global__ void read16(const uint4* p, size_t n, uint32_t* out) {  // 16 B per lane, coalesced
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        const uint4 v = p[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}
__global__ void read4(const uint32_t* p, size_t n, uint32_t* out) {  // 4 B per lane, coalesced
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) acc ^= p[i];
    if (acc == 0x12345678u) out[0] = acc;
}
__global__ void write16(uint4* p, size_t n) {
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
        p[i] = make_uint4((uint32_t)i, 1u, 2u, 3u);
}
__global__ void write4(uint32_t* p, size_t n) {
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) p[i] = (uint32_t)i;
}

// The describe kernel's window loads: a wave reads a 43-row x 48-byte window (lane (m, g):
// row 16 t + m, bytes 16 g .. 16 g + 15, g < 3, as load_frag) at a 4-byte-aligned column.
// Windows tile the buffer without sharing a 128-byte line (row pitch 2048: 16 windows per row
// band, one per 128-byte slot, 48 rows per band), the column offset inside the slot cycling
// through 0 .. 80, so every needed byte is read once and the 32 / 64 / 128-byte units touched
// are known exactly (printed) — no unit is shared by two windows (or two XCDs' L2s).
constexpr int kWinPitch = 2048, kWinRows = 43, kWinBand = 48, kWinPerRow = 16;
__device__ __host__ inline int win_off(int i, int j) { return 4 * ((i + 3 * j) % 21); }
__global__ void window48(const uint8_t* p, int nwin, uint32_t* out) {
    const int w = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (w >= nwin) return;
    const int i = w % kWinPerRow, j = w / kWinPerRow;
    const uint8_t* base = p + (size_t)j * kWinBand * kWinPitch + 128 * i + win_off(i, j);
    const int m = lane & 15, g = lane >> 4;
    uint32_t acc = 0;
#pragma unroll
    for (int t = 0; t < 3; ++t) {
        const int r = 16 * t + m;
        if (g < 3 && r < kWinRows) {
            uint4 v;
            __builtin_memcpy(&v, __builtin_assume_aligned(base + (size_t)r * kWinPitch + 16 * g, 4), 16);
            acc ^= v.x ^ v.y ^ v.z ^ v.w;
        }
    }
    if (acc == 0x12345678u) out[0] = acc;
}

int main() {
    void* buf = nullptr;
    uint32_t* out = nullptr;
    if (hipMalloc(&buf, kBytes) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
    if (hipMemset(buf, 1, kBytes) != hipSuccess) return 1;
    const dim3 g(8192), b(256);
    hipLaunchKernelGGL(read16, g, b, 0, nullptr, (const uint4*)buf, kBytes / 16, out);
    hipLaunchKernelGGL(read4, g, b, 0, nullptr, (const uint32_t*)buf, kBytes / 4, out);
    hipLaunchKernelGGL(write16, g, b, 0, nullptr, (uint4*)buf, kBytes / 16);
    hipLaunchKernelGGL(write4, g, b, 0, nullptr, (uint32_t*)buf, kBytes / 4);
    const int bands = (int)(kBytes / ((size_t)kWinBand * kWinPitch)), nwin = bands * kWinPerRow;
    hipLaunchKernelGGL(window48, dim3((nwin + 3) / 4), dim3(256), 0, nullptr, (const uint8_t*)buf, nwin, out);
    size_t need = 0, s32 = 0, s64 = 0, s128 = 0;
    for (int w = 0; w < nwin; ++w) {
        const int i = w % kWinPerRow, j = w / kWinPerRow;
        const size_t x0 = 128 * (size_t)i + win_off(i, j), x1 = x0 + 48;  // [x0, x1) of each row
        need += (size_t)kWinRows * 48;
        s32 += (size_t)kWinRows * 32 * ((x1 + 31) / 32 - x0 / 32);
        s64 += (size_t)kWinRows * 64 * ((x1 + 63) / 64 - x0 / 64);
        s128 += (size_t)kWinRows * 128 * ((x1 + 127) / 128 - x0 / 128);
    }
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    printf("{\"bytes_per_kernel\": %zu, \"window48\": {\"windows\": %d, \"needed\": %zu, "
           "\"sectors32\": %zu, \"sectors64\": %zu, \"lines128\": %zu}}\n",
           kBytes, nwin, need, s32, s64, s128);
    hipFree(buf);
    hipFree(out);
    return 0;
}
