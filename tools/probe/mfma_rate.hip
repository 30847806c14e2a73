// Issue rate of the i8 / bf16 MFMA shapes on one SIMD (one wave per SIMD, 4 independent
// accumulators, back-to-back), in shader cycles per instruction (s_memtime).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x16 __attribute__((ext_vector_type(16)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int N = 256;

__global__ void k_i8_32(const i32x4* in, i32x16* out, long long* cyc) {
    i32x4 a = in[threadIdx.x], b = in[threadIdx.x + 64];
    i32x16 c0 = {}, c1 = {}, c2 = {}, c3 = {};
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < N; ++i) {
        c0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c3, 0, 0, 0);
    }
    out[threadIdx.x] = c0 + c1 + c2 + c3;
    long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}
__global__ void k_i8_16(const i32x4* in, i32x4* out, long long* cyc) {
    i32x4 a = in[threadIdx.x], b = in[threadIdx.x + 64];
    i32x4 c0 = {}, c1 = {}, c2 = {}, c3 = {};
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < N; ++i) {
        c0 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c3, 0, 0, 0);
    }
    out[threadIdx.x] = c0 + c1 + c2 + c3;
    long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}
__global__ void k_bf16_32(const bf16x8* in, f32x16* out, long long* cyc) {
    bf16x8 a = in[threadIdx.x], b = in[threadIdx.x + 64];
    f32x16 c0 = {}, c1 = {}, c2 = {}, c3 = {};
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < N; ++i) {
        c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c3, 0, 0, 0);
    }
    out[threadIdx.x] = c0 + c1 + c2 + c3;
    long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

__global__ void k_i8_32_dep(const i32x4* in, i32x16* out, long long* cyc) {
    i32x4 a = in[threadIdx.x], b = in[threadIdx.x + 64];
    i32x16 c0 = {};
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < 4 * N; ++i) c0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c0, 0, 0, 0);
    out[threadIdx.x] = c0;
    long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}
// A operand from LDS: one ds_read_b128 per MFMA (two contiguous 512-B runs per wave), 4 chains
__global__ void k_i8_32_lds(const i32x4* in, i32x16* out, long long* cyc) {
    __shared__ i32x4 t[16][64];
    for (int i = threadIdx.x; i < 16 * 64; i += 64) t[i >> 6][i & 63] = in[i & 127];
    __syncthreads();
    const int col = threadIdx.x & 31, h = threadIdx.x >> 5;
    i32x4 b = in[threadIdx.x + 64];
    i32x16 c0 = {}, c1 = {}, c2 = {}, c3 = {};
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < N; ++i) {
        const int r = 2 * (i & 7) + h;
        c0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(t[r][col], b, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(t[r][32 + col], b, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_i32_32x32x32_i8(t[r ^ 2][col], b, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_i32_32x32x32_i8(t[r ^ 2][32 + col], b, c3, 0, 0, 0);
    }
    out[threadIdx.x] = c0 + c1 + c2 + c3;
    long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
    void *in, *out;
    long long* cyc;
    hipMalloc(&in, 1 << 16);
    hipMemset(in, 1, 1 << 16);
    hipMalloc(&out, 1 << 20);
    hipMalloc(&cyc, 8 * 1024);
    long long h[1024];
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    float ms = 0;
#define RUN(name, kern, IT, OT)                                                              \
    hipLaunchKernelGGL(kern, dim3(1024), dim3(64), 0, 0, (const IT*)in, (OT*)out, cyc);     \
    hipEventRecord(e0, 0);                                                                    \
    hipLaunchKernelGGL(kern, dim3(1024), dim3(64), 0, 0, (const IT*)in, (OT*)out, cyc);     \
    hipEventRecord(e1, 0);                                                                    \
    hipDeviceSynchronize();                                                                   \
    hipEventElapsedTime(&ms, e0, e1);                                                         \
    printf("  kernel %.1f us (%.2f ns per MFMA per SIMD)\n", ms * 1e3, ms * 1e6 / (4.0 * N)); \
    hipMemcpy(h, cyc, 8 * 1024, hipMemcpyDeviceToHost);                                       \
    {                                                                                         \
        double s = 0;                                                                         \
        for (int i = 0; i < 1024; ++i) s += h[i];                                             \
        printf("%-24s %.1f memtime ticks per MFMA (1 wave/SIMD)\n", name, s / 1024 / (4.0 * N)); \
    }
    RUN("i32_32x32x32_i8", k_i8_32, i32x4, i32x16)
    RUN("i32_16x16x64_i8", k_i8_16, i32x4, i32x4)
    RUN("f32_32x32x16_bf16", k_bf16_32, bf16x8, f32x16)
    RUN("i8_32 dependent chain", k_i8_32_dep, i32x4, i32x16)
    RUN("i8_32 A from LDS", k_i8_32_lds, i32x4, i32x16)
    return 0;
}
