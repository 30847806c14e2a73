// Probe: operand lane maps of v_mfma_scale_f32_32x32x64_f8f6f4 with FP4 (e2m1) A and B, unit
// scales.  One wave: lane l holds a[l][0..3] / b[l][0..3] (32 nibbles each, 4 dwords); writes
// the 16 f32 accumulators per lane.  tools/probe/fp4_map.py tests lane-map hypotheses on them.
#include <hip/hip_runtime.h>
typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));
__global__ void fp4_probe_kernel(const int* a, const int* b, float* d) {
    const int l = threadIdx.x;
    v8i av = {a[4 * l], a[4 * l + 1], a[4 * l + 2], a[4 * l + 3], 0, 0, 0, 0};
    v8i bv = {b[4 * l], b[4 * l + 1], b[4 * l + 2], b[4 * l + 3], 0, 0, 0, 0};
    v16f acc = {};
    acc = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(av, bv, acc, 4, 4, 0, 127, 0, 127);
    for (int e = 0; e < 16; ++e) d[16 * l + e] = acc[e];
}
extern "C" int fp4_probe(const int* a, const int* b, float* d) {
    hipLaunchKernelGGL(fp4_probe_kernel, dim3(1), dim3(64), 0, 0, a, b, d);
    return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
