// Issue rate of a few VALU integer instructions on gfx950: 8 independent chains per lane of
// one instruction (inline asm, so the compiler keeps it), 2,048 x 256 threads, timed with HIP
// events.  Prints ns per wave-instruction per SIMD-equivalent and the ratio to v_add_u32.
//   hipcc --offload-arch=gfx950 -O3 -o tools/probe/build/valu_rate tools/probe/valu_rate.hip
#include <hip/hip_runtime.h>
#include <cstdio>

#define CHAIN(OP)                                                                          \
    template <int N>                                                                       \
    __global__ __launch_bounds__(256) void k_##OP(unsigned* out, unsigned b) {             \
        unsigned x[8];                                                                     \
        for (int i = 0; i < 8; ++i) x[i] = threadIdx.x * 7u + i;                           \
        for (int it = 0; it < N; ++it) {                                                   \
            _Pragma("unroll") for (int i = 0; i < 8; ++i)                                   \
                asm volatile(#OP " %0, %0, %1" : "+v"(x[i]) : "v"(b));                     \
        }                                                                                  \
        unsigned s = 0;                                                                    \
        for (int i = 0; i < 8; ++i) s ^= x[i];                                             \
        out[blockIdx.x * 256 + threadIdx.x] = s;                                           \
    }
CHAIN(v_add_u32)
CHAIN(v_mul_u32_u24)
CHAIN(v_mul_hi_u32_u24)
CHAIN(v_mul_lo_u32)
CHAIN(v_mul_hi_u32)

int main() {
    unsigned* out;
    hipMalloc(&out, 2048 * 256 * 4);
    hipEvent_t a, z;
    hipEventCreate(&a);
    hipEventCreate(&z);
    constexpr int N = 4096;
    auto run = [&](const char* name, void (*k)(unsigned*, unsigned)) {
        k<<<2048, 256>>>(out, 12345u);
        hipDeviceSynchronize();
        hipEventRecord(a);
        for (int r = 0; r < 5; ++r) k<<<2048, 256>>>(out, 12345u);
        hipEventRecord(z);
        hipEventSynchronize(z);
        float ms = 0;
        hipEventElapsedTime(&ms, a, z);
        const double winstr = 5.0 * 2048 * 4 * (double)N * 8;  // wave-instructions
        printf("{\"op\": \"%s\", \"ms\": %.3f, \"Twave_instr_per_s\": %.4f}\n", name, ms, winstr / (ms * 1e-3) / 1e12);
        return ms;
    };
    run("v_add_u32", k_v_add_u32<N>);
    run("v_mul_u32_u24", k_v_mul_u32_u24<N>);
    run("v_mul_hi_u32_u24", k_v_mul_hi_u32_u24<N>);
    run("v_mul_lo_u32", k_v_mul_lo_u32<N>);
    run("v_mul_hi_u32", k_v_mul_hi_u32<N>);
    return 0;
}
