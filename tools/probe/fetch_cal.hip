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
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    printf("{\"bytes_per_kernel\": %zu}\n", kBytes);
    hipFree(buf);
    hipFree(out);
    return 0;
}
