// orbfe_device.hpp — gfx950 device helpers shared by the extractor and matcher kernels.
// Built with -ffp-contract=off: every float expression below is evaluated operation by
// operation exactly as the reference writes it (H3/H4 in DESIGN.md).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define ORBFE_WAVE 64

namespace orbfe {

// The reference's compile-time constants, as every kernel and host plan here uses them:
// PATCH_SIZE / HALF_PATCH_SIZE / EDGE_THRESHOLD (ORBextractor.cc:71-73) and ORBmatcher::TH_HIGH /
// TH_LOW / HISTO_LENGTH (ORBmatcher.cc:37-39).  Exported by orbfe_get_reference_constants and
// pinned against the reference text (tests/golden/constants_fixture.json).
constexpr int kPatchSize = 31;
constexpr int kHalfPatchSize = 15;
constexpr int kEdgeThreshold = 19;
constexpr int kThHigh = 100;
constexpr int kThLow = 50;
constexpr int kHistoLength = 30;

// XCD-aware block remap (cdna_hip_programming.md T1): blocks are dealt round-robin over the 8
// XCDs (blocks b and b + 8 share one), so give each XCD a contiguous range of the linear
// (x fastest, then y) grid: the tiles, cells and keypoints of one frame then share one XCD's
// L2 instead of pulling the frame's lines into all eight.  Bijective for any grid size; speed
// only, never correctness.
__device__ __forceinline__ void xcd_block(int& bx, int& by) {
    const unsigned nx = gridDim.x, n = nx * gridDim.y;
    const unsigned id = blockIdx.y * nx + blockIdx.x;
    const unsigned q = n >> 3, r = n & 7, x = id & 7;
    const unsigned l = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (id >> 3);
    by = (int)(l / nx);
    bx = (int)(l - (unsigned)by * nx);
}

// cvRound(float): round half to even (v_rndne_f32), App. A.5.
__device__ __forceinline__ int rne(float v) { return (int)__builtin_rintf(v); }

// cv::fastAtan2 (App. A.4; reference call ORBextractor.cc:102), degrees in [0, 360).
__device__ __forceinline__ float fast_atan2(float y, float x) {
    const float k180pi = (float)(180.0 / 3.14159265358979323846);
    const float p1 = 0.9997878412794807f * k180pi;
    const float p3 = -0.3258083974640975f * k180pi;
    const float p5 = 0.1555786518463281f * k180pi;
    const float p7 = -0.04432655554792128f * k180pi;
    const float eps = (float)2.220446049250313e-16;  // (float)DBL_EPSILON
    const float ax = fabsf(x), ay = fabsf(y);
    float a, c, c2;
    if (ax >= ay) {
        c = ay / (ax + eps);
        c2 = c * c;
        a = (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    } else {
        c = ax / (ay + eps);
        c2 = c * c;
        a = 90.f - (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    }
    if (x < 0) a = 180.f - a;
    if (y < 0) a = 360.f - a;
    return a;
}

// ORBmatcher::DescriptorDistance (ORBmatcher.cc:1650-1666): popcount of XOR over 8 words.
// v_bcnt_u32_b32 adds its second operand, so the 8 counts chain into one accumulator: a
// 256-bit distance is 8 v_xor + 8 v_bcnt (the compiler otherwise sums the counts with add3).
__device__ __forceinline__ uint32_t bcnt_acc(uint32_t x, uint32_t acc) {
    uint32_t r;
    asm("v_bcnt_u32_b32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(acc));
    return r;
}
__device__ __forceinline__ int hamming256(const uint4 a0, const uint4 a1, const uint4 b0,
                                          const uint4 b1) {
    uint32_t d = bcnt_acc(a0.x ^ b0.x, 0u);
    d = bcnt_acc(a0.y ^ b0.y, d);
    d = bcnt_acc(a0.z ^ b0.z, d);
    d = bcnt_acc(a0.w ^ b0.w, d);
    d = bcnt_acc(a1.x ^ b1.x, d);
    d = bcnt_acc(a1.y ^ b1.y, d);
    d = bcnt_acc(a1.z ^ b1.z, d);
    d = bcnt_acc(a1.w ^ b1.w, d);
    return (int)d;
}

// Inclusive sum over a 64-lane wave: the OCKL wavefront scan, six DPP adds (row_shr 1/2/4/8,
// row_bcast 15/31) instead of six ds_bpermute shuffles.  Every lane of the wave must be active.
extern "C" __device__ int __ockl_wfscan_add_i32(int, bool);
extern "C" __device__ int __ockl_wfred_add_i32(int);
extern "C" __device__ uint32_t __ockl_wfred_min_u32(uint32_t);
extern "C" __device__ int __ockl_wfred_min_i32(int);
__device__ __forceinline__ int wave_inclusive_sum(int x) { return __ockl_wfscan_add_i32(x, true); }

// Slot of this lane's item in a block-shared list: one LDS atomic per wave (called by every
// lane of the wave); -1 for lanes without an item.  Order among waves is unspecified.
__device__ __forceinline__ int wave_append(bool pred, int* counter) {
    const unsigned long long m = __ballot(pred);
    if (!m) return -1;
    const int lane = threadIdx.x & 63;
    const int leader = __ffsll((long long)m) - 1;
    int base = 0;
    if (lane == leader) base = atomicAdd(counter, __popcll(m));
    base = __shfl(base, leader, 64);
    return pred ? base + __popcll(m & ((1ull << lane) - 1)) : -1;
}

// Sum over a 64-lane wave (DPP reduction, result in every lane); every lane must be active.
__device__ __forceinline__ int wave_sum(int x) { return __ockl_wfred_add_i32(x); }

// Block-wide exclusive scan of one int per thread.  `tmp` holds >= BLOCK/64 ints of LDS.
// Returns the exclusive prefix; `total` receives the block sum.  Contains barriers: every
// thread of the block must call it.
template <int BLOCK>
__device__ __forceinline__ int block_exclusive_scan(int v, int* tmp, int& total) {
    constexpr int NW = BLOCK / 64;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int inc = wave_inclusive_sum(v);
    if (lane == 63) tmp[wid] = inc;
    __syncthreads();
    if (threadIdx.x < 64) {
        int w = threadIdx.x < NW ? tmp[threadIdx.x] : 0;
        w = wave_inclusive_sum(w);
        if (threadIdx.x < NW) tmp[threadIdx.x] = w;
    }
    __syncthreads();
    const int before = wid ? tmp[wid - 1] : 0;
    total = tmp[NW - 1];
    __syncthreads();
    return before + inc - v;
}

template <int BLOCK>
__device__ __forceinline__ int block_sum(int v, int* tmp) {
    int total;
    block_exclusive_scan<BLOCK>(v, tmp, total);
    return total;
}

}  // namespace orbfe
