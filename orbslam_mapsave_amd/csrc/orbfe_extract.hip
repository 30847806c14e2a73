// orbfe_extract.hip — MI355X (gfx950) ORB extractor: the HIP replacement for ORB-SLAM2's
// ORBextractor::operator() (skaegy/ORBSLAM_MapSave src/ORBextractor.cc:1042-1108).
//
// Pipeline for a batch of B same-size frames (one launch per stage, every launch covers the
// whole batch; DESIGN.md "Kernels" has the roofline and bytes of each):
//   K0 level0_kernel    cvtColor(*2GRAY) (Tracking.cc:409-422) + Mat::copyTo(dst, mask) (1053)
//                       [only for colour input or a mask]
//   K1 resize_kernel    cascaded cv::resize INTER_LINEAR 8U, levels 1..L-1 (1123)
//   K2 fast_kernel      per-cell FAST-9 score + cell-local 3x3 NMS + iniTh->minTh fallback
//                       (764-831); one workgroup per (frame, cell)
//   K3 octree_kernel    DistributeOctTree (538-762) as a data-parallel list emulation; one
//                       workgroup per (frame, level)
//   K4 blur_mfma_kernel GaussianBlur 7x7 sigma 2 REFLECT_101 (1088-1089), integer path
//   K5 describe_kernel  IC_Angle (76-103) + rBRIEF (107-146) + level scaling (1098-1104);
//                       one wave per keypoint, 256 tests packed with 4 ballots
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <memory>
#include <mutex>
#include <new>
#include <type_traits>
#include <array>
#include <vector>

#include "../../include/orbfe.h"
#include "orbfe_device.hpp"
#include "orbfe_internal.hpp"

namespace orbfe {

// ---------------------------------------------------------------------------------------------
// constant tables
__constant__ int8_t c_pattern[1024] = {
#include "../../include/orbfe_pattern.inc"
};
__constant__ int c_umax[16];

constexpr int kEdge = kEdgeThreshold;   // EDGE_THRESHOLD (ORBextractor.cc:73)
constexpr int kMinBorder = kEdge - 3;    // EDGE_THRESHOLD - 3 (772)
constexpr int kCellW = 30;      // W (768)
// 16-byte global loads from addresses aligned to 4 bytes (FAST ROI rows) or to 1 byte (the
// describe kernel's disc rows); memcpy lets the compiler pick dwordx4 with that alignment.
__device__ __forceinline__ uint4 load16_a4(const uint8_t* p) {
    uint4 v;
    __builtin_memcpy(&v, __builtin_assume_aligned(p, 4), 16);
    return v;
}
__device__ __forceinline__ uint4 load16_a1(const uint8_t* p) {
    uint4 v;
    __builtin_memcpy(&v, p, 16);
    return v;
}

// Stages `total` 16-byte chunks of image rows into LDS: chunk i is image row y0 + i / cpr at
// columns x0 + 16 (i % cpr) (x0 4-aligned), stored at dst + (i / cpr) P + 16 (i % cpr).  NT
// threads, four chunks each per round, every 16-byte load issued before any is used: the loads
// are unconditional (an index past the end re-reads the last chunk; a chunk reaching past the
// row end loads a clamped in-row address, or a zero word for rows narrower than 16 bytes, and
// is then rebuilt from dwords / bytes that never leave the row: level 0 may be the caller's
// buffer), since a load under a branch made the compiler wait for it before issuing the next.
__device__ uint4 g_zero16;
template <int NT>
__device__ __forceinline__ void stage_rows16(const uint8_t* src, long long pitch, int y0, int x0,
                                             int sw, int cpr, int total, unsigned char* dst,
                                             int P, int tid) {
    const bool wide = sw >= 16;
    const int xmax = (sw - 16) & ~3;
    for (int base = 0; base < total; base += 4 * NT) {
        uint4 v[4];
        int ro[4], xo[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int i = min(base + NT * u + tid, total - 1);
            const int r = i / cpr, c = i - r * cpr;
            ro[u] = r;
            xo[u] = x0 + 16 * c;
            const uint8_t* p = wide ? src + (long long)(y0 + r) * pitch + min(xo[u], xmax)
                                    : reinterpret_cast<const uint8_t*>(&g_zero16);
            v[u] = load16_a4(p);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int x = xo[u];
            if (x + 16 <= sw) continue;
            const uint8_t* row = src + (long long)(y0 + ro[u]) * pitch;
            uint32_t w[4];
#pragma unroll
            for (int d = 0; d < 4; ++d) {
                const int xd = x + 4 * d;
                w[d] = 0;
                if (xd + 4 <= sw) w[d] = *reinterpret_cast<const uint32_t*>(row + xd);
                else
                    for (int q = 0; q < 4 && xd + q < sw; ++q) w[d] |= (uint32_t)row[xd + q] << (8 * q);
            }
            v[u] = make_uint4(w[0], w[1], w[2], w[3]);
        }
        // (the stores unconditional too, an index past the end rewriting the last chunk with
        // its own bytes: a conditional store let the compiler sink the load into its branch)
#pragma unroll
        for (int u = 0; u < 4; ++u) *reinterpret_cast<uint4*>(dst + ro[u] * P + (xo[u] - x0)) = v[u];
    }
}

// ---------------------------------------------------------------------------------------------
// K0 — pyramid level 0 from the caller's frame: cvtColor(CV_{RGB,BGR,RGBA,BGRA}2GRAY) of
// Tracking::GrabImage* (Tracking.cc:286-310, 350-363, 409-422), then Mat::copyTo(image, mask)
// (ORBextractor.cc:1053, App. A.7) with the mask given as a full u8 plane and/or the zeroed
// rectangle of OpDetector::SkeletonSquareMask (DetectHumanPose.cpp:484-489).  Gray is
// OpenCV's 8U integer path RGB2Gray<uchar>: (c0*s0 + 9617*s1 + c2*s2 + 2^13) >> 14 with
// {c0, c2} = {B2Y 1868, R2Y 4899} for BGR order and swapped for RGB.  Each thread makes 4
// pixels and stores one dword (level-0 rows are padded to 64 B; pixels >= w are written 0).
// Sources whose rows are 4-byte aligned are read with dword / 3-dword / uint4 loads.
template <int CN>
__device__ __forceinline__ void load4(const uint8_t* row, int x, int w, bool aligned, uint8_t (&px)[4][4]) {
    if (aligned && x + 4 <= w) {
        if constexpr (CN == 1) {
            const uint32_t v = *reinterpret_cast<const uint32_t*>(row + x);
#pragma unroll
            for (int i = 0; i < 4; ++i) px[i][0] = (uint8_t)(v >> (8 * i));
        } else if constexpr (CN == 3) {
            const uint32_t* q = reinterpret_cast<const uint32_t*>(row + 3 * x);
            const uint32_t v0 = q[0], v1 = q[1], v2 = q[2];
            const uint8_t b[12] = {(uint8_t)v0, (uint8_t)(v0 >> 8), (uint8_t)(v0 >> 16), (uint8_t)(v0 >> 24),
                                   (uint8_t)v1, (uint8_t)(v1 >> 8), (uint8_t)(v1 >> 16), (uint8_t)(v1 >> 24),
                                   (uint8_t)v2, (uint8_t)(v2 >> 8), (uint8_t)(v2 >> 16), (uint8_t)(v2 >> 24)};
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int c = 0; c < 3; ++c) px[i][c] = b[3 * i + c];
        } else {
            const uint4 v = *reinterpret_cast<const uint4*>(row + 4 * x);
            const uint32_t vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int c = 0; c < 4; ++c) px[i][c] = (uint8_t)(vv[i] >> (8 * c));
        }
        return;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int c = 0; c < CN; ++c) px[i][c] = (x + i < w) ? row[CN * (x + i) + c] : 0;
}

template <int CN>
__device__ __forceinline__ void level0_row(const Level0Args& a, int f, int y, int x) {
    const uint8_t* row = a.src + f * a.src_fpitch + (long long)y * a.src_pitch;
    uint8_t px[4][4];
    load4<CN>(row, x, a.w, a.aligned, px);
    bool keep[4] = {true, true, true, true};
    if (a.mask) {
        const uint8_t* m = a.mask + f * a.mask_fpitch + (long long)y * a.mask_pitch;
#pragma unroll
        for (int i = 0; i < 4; ++i) keep[i] = (x + i < a.w) && m[x + i] != 0;
    }
    if (a.rects) {
        const int4 r = a.rects[f];
        if (y >= r.y && y < r.w) {
#pragma unroll
            for (int i = 0; i < 4; ++i)
                if (x + i >= r.x && x + i < r.z) keep[i] = false;
        }
    }
    uint32_t out = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        int g;
        if constexpr (CN == 1) {
            g = px[i][0];
        } else {
            g = (a.c0 * px[i][0] + 9617 * px[i][1] + a.c2 * px[i][2] + (1 << 13)) >> 14;
        }
        if (!keep[i] || x + i >= a.w) g = 0;
        out |= (uint32_t)g << (8 * i);
    }
    *reinterpret_cast<uint32_t*>(a.dst + f * a.dst_fpitch + (long long)y * a.dst_pitch + x) = out;
}

__global__ __launch_bounds__(256) void level0_kernel(Level0Args a) {
    const int f = blockIdx.z, y = blockIdx.y;
    const int x = 4 * (blockIdx.x * blockDim.x + threadIdx.x);
    if (x >= a.w) return;
    switch (a.cn) {
        case 1: level0_row<1>(a, f, y, x); break;
        case 3: level0_row<3>(a, f, y, x); break;
        default: level0_row<4>(a, f, y, x); break;
    }
}

// ---------------------------------------------------------------------------------------------
// K1 — one pyramid level from the previous one (App. A.1, scalar FixedPtCast<int,uchar,22>),
// one launch per level covering every frame.  A workgroup makes a 128 x 32 output tile: the
// source rows/cols the tile touches are staged in LDS with dword loads, then each thread makes
// 4 x 4 pixels from host-built tables xt[3*dx] = {sx, min(sx+1,sw-1), a0 | a1<<16} and
// yt[3*dy] = {sy0, sy1 clipped, b0 | b1<<16}.
// One output pixel of the vertical pass from the two horizontal sums t0, t1 (< 2^19) and the
// row coefficients b0 + b1 = 2048.  Scalar FixedPtCast<int, uchar, 22>: the sum is never
// negative, so only the upper clamp remains (the signed min(max(x >> 22, 0), 255) form can be
// matched to gfx950's v_ashr_pk_u8_i32 for two of four bytes, and that packing was seen to
// corrupt the upper two).  With `sse2` the x86 body of VResizeLinearVec_32s8u (H5):
// ((((t0 >> 4) * b0) >> 16) + (((t1 >> 4) * b1) >> 16) + 2) >> 2, every operand < 2^24 (no
// 16-bit saturation is reachable).  All products are full-rate v_mul_u32_u24.
template <bool kX86>
__device__ __forceinline__ uint32_t resize_px(uint32_t t0, uint32_t t1, uint32_t b0, uint32_t b1,
                                              bool sse2) {
    const uint32_t sc = (__umul24(t0, b0) + __umul24(t1, b1) + (1u << 21)) >> 22;
    if constexpr (!kX86) return min(sc, 255u);
    const uint32_t sv = ((__umul24(t0 >> 4, b0) >> 16) + (__umul24(t1 >> 4, b1) >> 16) + 2) >> 2;
    return min(sse2 ? sv : sc, 255u);
}

// ORBFE_RS_X86 — the x86 (H5) body formula ((t0 >> 4) * b0 >> 16) + ((t1 >> 4) * b1 >> 16) + 2
// >> 2 (build-time A/B): 0 = shifts, multiplies, shifts and a clamp per pixel; 1 = the
// horizontal sums scaled by 16 (hcoef) so each term is one AND + v_mul_hi_u32_u24; 2 = the +2
// folded into the first product (v_mad_u32_u24) and both >> 16 into one SDWA add.
#ifndef ORBFE_RS_X86
#define ORBFE_RS_X86 2
#endif
constexpr int kRsX86 = ORBFE_RS_X86;

// Horizontal coefficient pairs (a0 | a1 << 16) as the horizontal passes feeding resize4 use
// them: in mode 1 x86 scales both by 16 (a0, a1 <= 2049: each half stays below 2^16), so the
// sums arrive as h = 16 t (< 2^23).
template <bool kX86>
__device__ __forceinline__ uint32_t hcoef(uint32_t a01) { return kX86 && kRsX86 == 1 ? a01 << 4 : a01; }

// (P0 >> 16) + (P1 >> 16) in one VOP2 SDWA add (word 1 of each operand)
__device__ __forceinline__ uint32_t add_hi16(uint32_t p0, uint32_t p1) {
    uint32_t r;
    asm("v_add_u32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:WORD_1"
        : "=v"(r) : "v"(p0), "v"(p1));
    return r;
}

// Four pixels of a row (columns x .. x + 3) from their horizontal sums (16 t in x86 mode 1,
// else t).  x86: a group entirely inside the SSE2 body (x + 3 < xb, nearly every group) takes
// the body formula alone; t >> 4 <= 32,655 and b0 + b1 <= 2049 keep the body's sum <= 1,022,
// so it needs no clamp.  Groups reaching the scalar tail select per pixel.
template <bool kX86>
__device__ __forceinline__ uint32_t resize4(const uint32_t (&h0)[4], const uint32_t (&h1)[4],
                                            uint32_t b0, uint32_t b1, int x, int xb) {
    constexpr int kS = kX86 && kRsX86 == 1 ? 4 : 0;  // h >> kS = t
    uint32_t packed = 0;
    if (kX86 && x + 3 < xb) {
        if constexpr (kRsX86 == 1) {
            const uint32_t c0 = (b0 & 0xffffu) << 8, c1 = (b1 & 0xffffu) << 8;  // < 2^24
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint32_t p0 = (uint32_t)(((unsigned long long)(h0[k] & 0x7fff00u) * c0) >> 32);
                const uint32_t p1 = (uint32_t)(((unsigned long long)(h1[k] & 0x7fff00u) * c1) >> 32);
                packed |= ((p0 + p1 + 2u) >> 2) << (8 * k);
            }
        } else if constexpr (kRsX86 == 2) {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                // (t0 >> 4) b0 + 2^17 < 2^27: its word 1 is ((t0 >> 4) b0 >> 16) + 2
                const uint32_t p0 = __umul24(h0[k] >> 4, b0) + (2u << 16);
                const uint32_t p1 = __umul24(h1[k] >> 4, b1);
                packed |= (add_hi16(p0, p1) >> 2) << (8 * k);
            }
        } else {
#pragma unroll
            for (int k = 0; k < 4; ++k)
                packed |= min((((uint32_t)__umul24(h0[k] >> 4, b0) >> 16) +
                               ((uint32_t)__umul24(h1[k] >> 4, b1) >> 16) + 2u) >> 2, 255u) << (8 * k);
        }
    } else {
#pragma unroll
        for (int k = 0; k < 4; ++k)
            packed |= resize_px<kX86>(h0[k] >> kS, h1[k] >> kS, b0, b1, x + k < xb) << (8 * k);
    }
    return packed;
}

#ifndef ORBFE_RS_TH
#define ORBFE_RS_TH 32
#endif
constexpr int kRsTW = 128, kRsTH = ORBFE_RS_TH;  // output tile; 8 thread rows of kRsTH / 8
constexpr int kRsRPT = kRsTH / 8;
constexpr int kR2Rows = 96;  // resize2_kernel: level-l region rows per tile (host-checked)
template <bool kX86>
__global__ __launch_bounds__(256) void resize_kernel(ResizeArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char rs_lds[];
    int bx, f;
    xcd_block(bx, f);
    const int ox = (bx % a.tiles_x) * kRsTW, oy = (bx / a.tiles_x) * kRsTH;
    const int ex = min(ox + kRsTW, a.dw) - 1, ey = min(oy + kRsTH, a.dh) - 1;
    const int sy0 = a.yt[3 * oy], sy1 = a.yt[3 * ey + 1];
    const int sx0 = a.xt[3 * ox] & ~3, sx1 = a.xt[3 * ex + 1];
    const int nrow = sy1 - sy0 + 1, P = a.lds_pitch;  // P % 16 == 0
    const int cpr = ((sx1 - sx0) >> 4) + 1;                 // 16-byte chunks per source row
    const uint8_t* src = a.src.base + f * a.src.fpitch;
    // this thread's output rows' table entries, loaded with the staging (clamped rows,
    // unconditional): read inside the row loop they cost one round trip per row
    int ytr[kRsRPT][3];
#pragma unroll
    for (int j = 0; j < kRsRPT; ++j) {
        const int yc = min(oy + kRsRPT * (int)(threadIdx.x >> 5) + j, a.dh - 1);
#pragma unroll
        for (int k = 0; k < 3; ++k) ytr[j][k] = a.yt[3 * yc + k];
    }
    // source rows -> LDS in 16-byte chunks (global dwordx4 needs 4-byte alignment: sx0 % 4 ==
    // 0, pitch % 4 == 0); four chunks per thread in flight before any LDS store.  A chunk
    // reaching past the row end is assembled from dwords / bytes (level 0 may be the caller's
    // buffer: nothing past its last row is read).
    const int total = nrow * cpr;
    stage_rows16<256>(src, a.src.pitch, sy0, sx0, a.sw, cpr, total, rs_lds, P, (int)threadIdx.x);
    __syncthreads();
    const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
    const int x = ox + 4 * tx;
    if (x >= a.dw) return;
    const int n = min(4, a.dw - x);
    uint8_t* dst = const_cast<uint8_t*>(a.dst.base) + f * a.dst.fpitch;
    if (a.gtab) {
        // pyramid_kernel's horizontal pass (the level's column-group table): 3 dword LDS reads
        // per source row, an 8-byte window by v_alignbyte, v_perm + v_dot2 per pixel, instead of
        // 4 byte gathers, 4 multiplies and 2 adds per pixel
        typedef unsigned short us2 __attribute__((ext_vector_type(2)));
        const uint4* gp = a.gtab + 3 * (x >> 2);
        const uint4 g0 = gp[0], g1 = gp[1], g2 = gp[2];
        const int base = (int)g0.x - sx0, wofs = base & ~3, sh = base & 3;
        const uint32_t sel[4] = {g0.y, g0.z, g0.w, g1.x};
        const us2 cf[4] = {__builtin_bit_cast(us2, hcoef<kX86>(g1.y)), __builtin_bit_cast(us2, hcoef<kX86>(g1.z)),
                           __builtin_bit_cast(us2, hcoef<kX86>(g1.w)), __builtin_bit_cast(us2, hcoef<kX86>(g2.x))};
        auto hsum = [&](int r, uint32_t (&t)[4]) {
            const uint32_t* row = reinterpret_cast<const uint32_t*>(rs_lds + r * P + wofs);
            const uint32_t w0 = row[0], w1 = row[1], w2 = row[2];
            const uint32_t lo = __builtin_amdgcn_alignbyte(w1, w0, sh), hi = __builtin_amdgcn_alignbyte(w2, w1, sh);
#pragma unroll
            for (int k = 0; k < 4; ++k)
                t[k] = __builtin_amdgcn_udot2(__builtin_bit_cast(us2, __builtin_amdgcn_perm(hi, lo, sel[k])), cf[k], 0u, false);
        };
#pragma unroll
        for (int j = 0; j < kRsRPT; ++j) {
            const int y = oy + kRsRPT * ty + j;
            if (y >= a.dh) break;
            const int ry0 = ytr[j][0] - sy0, ry1 = ytr[j][1] - sy0, bb = ytr[j][2];
            const uint32_t b0 = (uint32_t)bb & 0xffffu, b1 = (uint32_t)bb >> 16;
            uint32_t t0[4], t1[4];
            hsum(ry0, t0);
            hsum(ry1, t1);
            const uint32_t packed = resize4<kX86>(t0, t1, b0, b1, x, a.simd_xb);
            uint8_t* d = dst + (long long)y * a.dst.pitch + x;
            if (n == 4) {
                *reinterpret_cast<uint32_t*>(d) = packed;
            } else {
                for (int k = 0; k < n; ++k) d[k] = (uint8_t)(packed >> (8 * k));
            }
        }
        return;
    }
    int x0[4], x1[4], a0[4], a1[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int dx = min(x + k, a.dw - 1);
        x0[k] = a.xt[3 * dx] - sx0;
        x1[k] = a.xt[3 * dx + 1] - sx0;
        const int aa = a.xt[3 * dx + 2];
        a0[k] = (int)(hcoef<kX86>((uint32_t)aa) & 0xffffu);  // x86: 16 a0, 16 a1 (hcoef)
        a1[k] = (int)(hcoef<kX86>((uint32_t)aa) >> 16);
    }
#pragma unroll
    for (int j = 0; j < kRsRPT; ++j) {
        const int y = oy + kRsRPT * ty + j;
        if (y >= a.dh) break;
        const int ry0 = ytr[j][0] - sy0, ry1 = ytr[j][1] - sy0, bb = ytr[j][2];
        const int b0 = bb & 0xffff, b1 = (int)((unsigned)bb >> 16);
        const uint8_t* s0 = rs_lds + ry0 * P;
        const uint8_t* s1 = rs_lds + ry1 * P;
        uint32_t t0[4], t1[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            // coefficients sum to 2048 (INTER_RESIZE_COEF_SCALE): t < 2^19, t * b < 2^30, so
            // every product is a full-rate v_mul_u32_u24 (not the quarter-rate v_mul_lo_u32)
            t0[k] = __umul24(s0[x0[k]], a0[k]) + __umul24(s0[x1[k]], a1[k]);
            t1[k] = __umul24(s1[x0[k]], a0[k]) + __umul24(s1[x1[k]], a1[k]);
        }
        const uint32_t packed = resize4<kX86>(t0, t1, b0, b1, x, a.simd_xb);
        uint8_t* d = dst + (long long)y * a.dst.pitch + x;
        if (n == 4) {
            *reinterpret_cast<uint32_t*>(d) = packed;
        } else {
            for (int k = 0; k < n; ++k) d[k] = (uint8_t)(packed >> (8 * k));
        }
    }
}

// K1, two levels per launch (1920 x 1080 and other sizes the band kernel leaves to the
// per-level kernels): a workgroup owns a 128 x 32 tile of level l + 1.  It stages the level
// l - 1 rows and columns its level-l region reads (16-byte chunks, as resize_kernel), makes that
// level-l region in LDS (its own part of level l also to the pyramid: the host partitions level
// l among the tiles by the first source row / column of each tile), then the level l + 1 tile
// from LDS.  Level l never makes a round trip through HBM between the two launches it used to
// take (1080p: level 1 is 369 MB per 256 frames written and read back).  The host table gives
// each tile its computed and own level-l rectangles; both passes are resize_kernel's
// column-group horizontal pass and resize4.
template <bool kX86>
__global__ __launch_bounds__(256) void resize2_kernel(Resize2Args a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char r2_lds[];
    int bx, f;
    xcd_block(bx, f);
    const int4 c = a.tiles[2 * bx], own = a.tiles[2 * bx + 1];
    const int tid = threadIdx.x;
    const int oy = (bx / a.tiles_x) * kRsTH;
    // The row tables both passes walk (level l's rows c.x .. c.y, the tile's level l + 1 rows),
    // staged in LDS beside the image rows: read from global inside the row loops they cost one
    // round trip per row.  Loads and stores unconditional at clamped indices.
    __shared__ int ytm_s[3 * kR2Rows];  // c.y - c.x < kR2Rows (host plan)
    __shared__ int ytd_s[3 * kRsTH];
    static_assert(3 * kRsTH <= 256, "ytd_s is filled with one entry per thread (ORBFE_RS_TH <= 85)");
    {
        const int n3 = 3 * (c.y - c.x + 1);
        const int i0 = min(tid, n3 - 1), i1 = min(tid + 256, n3 - 1), i2 = min(tid, 3 * kRsTH - 1);
        const int yd = min(oy + i2 / 3, a.dh - 1);
        const int v0 = a.yt_m[3 * c.x + i0], v1 = a.yt_m[3 * c.x + i1], v2 = a.yt_d[3 * yd + i2 % 3];
        ytm_s[i0] = v0;
        ytm_s[i1] = v1;
        ytd_s[i2] = v2;
    }
    // level l - 1 rectangle the level-l region reads
    const int ay0 = a.yt_m[3 * c.x], ay1 = a.yt_m[3 * c.y + 1];
    const int ax0 = a.xt_m[3 * c.z] & ~3, ax1 = a.xt_m[3 * c.w + 1];
    {
        const int nrow = ay1 - ay0 + 1, cpr = ((ax1 - ax0) >> 4) + 1, total = nrow * cpr;
        const uint8_t* src = a.src.base + f * a.src.fpitch;
        stage_rows16<256>(src, a.src.pitch, ay0, ax0, a.sw, cpr, total, r2_lds, a.pa, tid);
    }
    __syncthreads();
    typedef unsigned short us2 __attribute__((ext_vector_type(2)));
    // one thread per (column group, row phase): the group's table entry loaded once
    auto hsum = [&](const unsigned char* base, int pitch, int r, int wofs, int sh, const uint32_t (&sel)[4],
                    const us2 (&cf)[4], uint32_t (&t)[4]) {
        const uint32_t* row = reinterpret_cast<const uint32_t*>(base + r * pitch + wofs);
        const uint32_t w0 = row[0], w1 = row[1], w2 = row[2];
        const uint32_t lo = __builtin_amdgcn_alignbyte(w1, w0, sh), hi = __builtin_amdgcn_alignbyte(w2, w1, sh);
#pragma unroll
        for (int k = 0; k < 4; ++k)
            t[k] = __builtin_amdgcn_udot2(__builtin_bit_cast(us2, __builtin_amdgcn_perm(hi, lo, sel[k])), cf[k], 0u, false);
    };
    unsigned char* B = r2_lds + a.bofs;
    {   // level l region: rows c.x .. c.y, column groups c.z / 4 .. c.w / 4
        const int gpr = ((c.w - c.z) >> 2) + 1, rps = 256 / gpr;
        const int gx = tid % gpr, ry = tid / gpr;
        if (ry < rps) {
            const int x = c.z + 4 * gx;
            const uint4* gp = a.gtab_m + 3 * (x >> 2);
            const uint4 g0 = gp[0], g1 = gp[1], g2 = gp[2];
            const int xrel = (int)g0.x - ax0, wofs = (xrel >> 2) << 2, sh = xrel & 3;
            const uint32_t sel[4] = {g0.y, g0.z, g0.w, g1.x};
            const us2 cf[4] = {__builtin_bit_cast(us2, hcoef<kX86>(g1.y)), __builtin_bit_cast(us2, hcoef<kX86>(g1.z)),
                               __builtin_bit_cast(us2, hcoef<kX86>(g1.w)), __builtin_bit_cast(us2, hcoef<kX86>(g2.x))};
            const int n = min(4, a.mw - x);
            const bool own_x = x >= own.z && x < own.w;  // own column bounds are multiples of 4
            uint8_t* mid = const_cast<uint8_t*>(a.mid.base) + f * a.mid.fpitch;
            for (int r = c.x + ry; r <= c.y; r += rps) {
                const int* yy = ytm_s + 3 * (r - c.x);
                const uint32_t b0 = (uint32_t)yy[2] & 0xffffu, b1 = (uint32_t)yy[2] >> 16;
                uint32_t t0[4], t1[4];
                hsum(r2_lds, a.pa, yy[0] - ay0, wofs, sh, sel, cf, t0);
                hsum(r2_lds, a.pa, yy[1] - ay0, wofs, sh, sel, cf, t1);
                const uint32_t packed = resize4<kX86>(t0, t1, b0, b1, x, a.xb_m);
                *reinterpret_cast<uint32_t*>(B + (r - c.x) * a.pb + (x - c.z)) = packed;
                if (own_x && r >= own.x && r < own.y) {
                    uint8_t* o = mid + (long long)r * a.mid.pitch + x;
                    if (n == 4) {
                        *reinterpret_cast<uint32_t*>(o) = packed;
                    } else {
                        for (int k = 0; k < n; ++k) o[k] = (uint8_t)(packed >> (8 * k));
                    }
                }
            }
        }
    }
    __syncthreads();
    {   // level l + 1 tile from the level-l region (resize_kernel's thread layout)
        const int tiles_x = a.tiles_x;
        const int ox = (bx % tiles_x) * kRsTW;
        const int tx = tid & 31, ty = tid >> 5;
        const int x = ox + 4 * tx;
        if (x >= a.dw) return;
        const int n = min(4, a.dw - x);
        const uint4* gp = a.gtab_d + 3 * (x >> 2);
        const uint4 g0 = gp[0], g1 = gp[1], g2 = gp[2];
        const int xrel = (int)g0.x - c.z, wofs = (xrel >> 2) << 2, sh = xrel & 3;
        const uint32_t sel[4] = {g0.y, g0.z, g0.w, g1.x};
        const us2 cf[4] = {__builtin_bit_cast(us2, hcoef<kX86>(g1.y)), __builtin_bit_cast(us2, hcoef<kX86>(g1.z)),
                           __builtin_bit_cast(us2, hcoef<kX86>(g1.w)), __builtin_bit_cast(us2, hcoef<kX86>(g2.x))};
        uint8_t* dst = const_cast<uint8_t*>(a.dst.base) + f * a.dst.fpitch;
#pragma unroll
        for (int j = 0; j < kRsRPT; ++j) {
            const int y = oy + kRsRPT * ty + j;
            if (y >= a.dh) break;
            const int* yy = ytd_s + 3 * (y - oy);
            const uint32_t b0 = (uint32_t)yy[2] & 0xffffu, b1 = (uint32_t)yy[2] >> 16;
            uint32_t t0[4], t1[4];
            hsum(B, a.pb, yy[0] - c.x, wofs, sh, sel, cf, t0);
            hsum(B, a.pb, yy[1] - c.x, wofs, sh, sel, cf, t1);
            const uint32_t packed = resize4<kX86>(t0, t1, b0, b1, x, a.xb_d);
            uint8_t* o = dst + (long long)y * a.dst.pitch + x;
            if (n == 4) {
                *reinterpret_cast<uint32_t*>(o) = packed;
            } else {
                for (int k = 0; k < n; ++k) o[k] = (uint8_t)(packed >> (8 * k));
            }
        }
    }
}


// Column-pass rounding.  The sums carry 0x7fff; the scalar FixedPtCastEx (sum + 2^15) >> 16
// adds one more, the x86 SIMD body (H6: float sum, exact below 2^24, _mm_cvtps_epi32) rounds
// half to even: (sum + 0x7fff + bit 16 of sum) >> 16.  v = sum + 0x7fff.
// Lanes whose 32-bit blur sum (+ 0x7fff) has the low half 0xffff — a tie of the x86 body's
// round half to even — as a lane mask: one v_cmp_eq_u16 (the inline constant -1 is 0xffff at
// 16 bits).
__device__ __forceinline__ unsigned long long tie_lanes(uint32_t v) {
    unsigned long long m;
    asm("v_cmp_eq_u16_e64 %0, -1, %1" : "=s"(m) : "v"(v));
    return m;
}
__device__ __forceinline__ uint32_t blur_round_bit(uint32_t v, bool even) {
    return even ? ((v - 0x7fffu) >> 16) & 1u : 1u;
}

// cv::borderInterpolate(p, len, BORDER_REFLECT_101) (App. A.2), any distance from the edge.
__device__ __forceinline__ int reflect101(int p, int len) {
    if (len == 1) return 0;
    while (p < 0 || p >= len) p = p < 0 ? -p : 2 * len - p - 2;
    return p;
}
__device__ __forceinline__ int reflect101_1(int p, int len) {  // |overshoot| < len - 1
    return p < 0 ? -p : (p >= len ? 2 * len - 2 - p : p);
}

// K1 as one launch — the whole pyramid of a horizontal band of every frame per workgroup.
// The host partitions every level's rows into nbands bands (proportionally) and derives, top
// level down, the rows each band must COMPUTE at each level: its own rows plus the source rows
// its rows of the level above read (a few rows of halo, recomputed by the neighbouring band).
// The workgroup stages its level-0 rows in LDS, then makes level 1 .. L-1 one after the other,
// each from the previous one held in LDS (two buffers, ping-pong; every level's y-table rows
// staged beside them), writing only its own rows of each level to the pyramid.  So the levels
// never make a round trip through HBM between launches and one launch replaces nlevels - 1.
// Horizontal pass (App. A.1): a thread makes 4 output pixels of a row, whose source columns
// x0[k], x1[k] lie in 8 bytes from x0[0] (checked on the host for the plan's scale factor): 3
// dword LDS reads per source row, two v_alignbyte make the 8-byte window, one v_perm per pixel
// pairs its two source bytes as u16 and v_dot2 applies (a0, a1) — instead of 4 byte gathers,
// 2 multiplies and an add per pixel.  Vertical pass and rounding: resize_px, as resize_kernel.
constexpr int kPyrBlock = kPyrBlockSize;
#ifndef ORBFE_PYR_ROWS
#define ORBFE_PYR_ROWS 1  // 2 and 4 measured no faster (profiles/r03/experiments/pyramid.json)
#endif
constexpr int kPyrRows = ORBFE_PYR_ROWS;
template <bool kX86>
__global__ __launch_bounds__(kPyrBlock) void pyramid_kernel(PyrArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char py_lds[];
    const int band = blockIdx.x, f = blockIdx.y, tid = threadIdx.x;
    const int L = a.nlevels;
    const int4* bt = a.bands + band * L;
    // (LDS addresses by offset arithmetic from py_lds: a pointer picked from an array would be
    // a generic pointer, and every access a flat instruction)
    {   // level 0 rows c0 .. c1 -> buf[0] (16-byte chunks; a chunk past the row end is assembled
        // from dwords / bytes: level 0 may be the caller's buffer)
        const int4 b0 = bt[0];
        const int w = a.w[0], P = a.lp[0];
        const uint8_t* src = a.src.base + f * a.src.fpitch;
        const int cpr = (w + 15) >> 4, total = (b0.y - b0.x + 1) * cpr;
        for (int base = 0; base < total; base += 4 * kPyrBlock) {
            uint4 v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int i = base + kPyrBlock * u + tid;
                if (i >= total) continue;
                const int r = i / cpr, c = i - r * cpr;
                const uint8_t* row = src + (long long)(b0.x + r) * a.src.pitch;
                const int x = 16 * c;
                if (x + 16 <= w) {
                    v[u] = load16_a4(row + x);
                } else {
                    uint32_t wd[4];
#pragma unroll
                    for (int d = 0; d < 4; ++d) {
                        const int xd = x + 4 * d;
                        wd[d] = 0;
                        if (xd + 4 <= w) wd[d] = *reinterpret_cast<const uint32_t*>(row + xd);
                        else
                            for (int q = 0; q < 4 && xd + q < w; ++q) wd[d] |= (uint32_t)row[xd + q] << (8 * q);
                    }
                    v[u] = make_uint4(wd[0], wd[1], wd[2], wd[3]);
                }
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int i = base + kPyrBlock * u + tid;
                if (i >= total) continue;
                const int r = i / cpr, c = i - r * cpr;
                *reinterpret_cast<uint4*>(py_lds + r * P + 16 * c) = v[u];
                // the band's own level-0 rows to the slab (the 16-byte chunk stays inside the
                // slab's 64-byte row pitch)
                if (a.l0_copy.base && b0.x + r >= b0.z && b0.x + r < b0.w)
                    *reinterpret_cast<uint4*>(const_cast<uint8_t*>(a.l0_copy.base) + f * a.l0_copy.fpitch +
                                              (long long)(b0.x + r) * a.l0_copy.pitch + 16 * c) = v[u];
            }
        }
    }
    for (int l = 1; l < L; ++l) {
        const int4 bs = bt[l - 1], bl = bt[l];
        const int nrows = bl.y - bl.x + 1;  // may be 0 for a thin band of a small level
        const int w = a.w[l], gpr = (w + 3) >> 2, rps = kPyrBlock / gpr;
        const int gx = tid % gpr, ry = tid / gpr;
        // this level's y-table rows, and the thread's column group (issued before the barrier)
        int* yb = reinterpret_cast<int*>(py_lds + a.ybuf) + ((l & 1) ? 3 * a.ymax : 0);
        for (int i = tid; i < 3 * nrows; i += kPyrBlock) yb[i] = a.yt[l][3 * bl.x + i];
        uint4 g0 = make_uint4(0u, 0u, 0u, 0u), g1 = g0, g2 = g0;
        if (ry < rps && nrows > 0) {
            const uint4* gp = a.gtab[l] + 3 * gx;
            g0 = gp[0];
            g1 = gp[1];
            g2 = gp[2];
        }
        __syncthreads();
        if (ry >= rps || nrows <= 0) continue;
        const uint8_t* s = py_lds + (((l - 1) & 1) ? a.buf_b : 0);
        uint8_t* d = py_lds + ((l & 1) ? a.buf_b : 0);
        const int sp = a.lp[l - 1], dpitch = a.lp[l];
        const int xbase = (int)g0.x, wofs = (xbase >> 2) << 2, sh = xbase & 3;
        const uint32_t sel[4] = {g0.y, g0.z, g0.w, g1.x};
        typedef unsigned short us2 __attribute__((ext_vector_type(2)));
        const us2 cf[4] = {__builtin_bit_cast(us2, hcoef<kX86>(g1.y)), __builtin_bit_cast(us2, hcoef<kX86>(g1.z)),
                           __builtin_bit_cast(us2, hcoef<kX86>(g1.w)), __builtin_bit_cast(us2, hcoef<kX86>(g2.x))};
        const int x = 4 * gx, n = min(4, w - x);
        const int xb = a.simd_xb[l];
        const LevelPtr dp = a.dst[l];
        uint8_t* dst = const_cast<uint8_t*>(dp.base) + f * dp.fpitch;
        auto hsum = [&](int r, uint32_t (&t)[4]) {  // horizontal sums of source row r (LDS row)
            const uint32_t* row = reinterpret_cast<const uint32_t*>(s + r * sp + wofs);
            const uint32_t w0 = row[0], w1 = row[1], w2 = row[2];
            const uint32_t lo = __builtin_amdgcn_alignbyte(w1, w0, sh), hi = __builtin_amdgcn_alignbyte(w2, w1, sh);
#pragma unroll
            for (int k = 0; k < 4; ++k)
                t[k] = __builtin_amdgcn_udot2(__builtin_bit_cast(us2, __builtin_amdgcn_perm(hi, lo, sel[k])), cf[k], 0u, false);
        };
        auto row_out = [&](int r) {
            const int* yy = yb + 3 * (r - bl.x);
            const int bb = yy[2];
            const uint32_t b0 = (uint32_t)bb & 0xffffu, b1 = (uint32_t)bb >> 16;
            uint32_t t0[4], t1[4];
            hsum(yy[0] - bs.x, t0);
            hsum(yy[1] - bs.x, t1);
            const uint32_t packed = resize4<kX86>(t0, t1, b0, b1, x, xb);
            *reinterpret_cast<uint32_t*>(d + (r - bl.x) * dpitch + x) = packed;
            if (r >= bl.z && r < bl.w) {
                uint8_t* o = dst + (long long)r * dp.pitch + x;
                if (n == 4) {
                    *reinterpret_cast<uint32_t*>(o) = packed;
                } else {
                    for (int k = 0; k < n; ++k) o[k] = (uint8_t)(packed >> (8 * k));
                }
            }
        };
        // kPyrRows rows per iteration: their LDS reads are issued together.  (Runs of
        // consecutive rows per thread, summing a source row shared with the previous row once
        // — 1.2 instead of 2 sums per row — measured slower: 0.307 -> 0.334 ms)
        int r = bl.x + ry;
        for (; r + (kPyrRows - 1) * rps <= bl.y; r += kPyrRows * rps) {
#pragma unroll
            for (int j = 0; j < kPyrRows; ++j) row_out(r + j * rps);
        }
        for (; r <= bl.y; r += rps) row_out(r);
    }
}
template __global__ void pyramid_kernel<false>(PyrArgs);
template __global__ void pyramid_kernel<true>(PyrArgs);


// Host: pyramid_kernel's per-level column-group tables (3 uint4 per group of 4 output columns:
// x0[0], the 4 perm selectors pairing bytes x0[k] - x0[0], x1[k] - x0[0] as u16 (0x0c = zero),
// the 4 (a0 | a1 << 16) coefficient pairs).  False when a group's source bytes do not fit 8
// bytes from x0[0] (scale factors well above 1.2): the per-level kernels are used instead.
static bool pyramid_group_table(const std::vector<int>& xtab, int xoff, int dw, std::vector<uint32_t>& out) {
    for (int gx = 0; gx < (dw + 3) / 4; ++gx) {
        uint32_t e[12] = {};
        int x0[4], x1[4], c[4];
        for (int k = 0; k < 4; ++k) {
            const int dx = std::min(4 * gx + k, dw - 1);
            x0[k] = xtab[xoff + 3 * dx];
            x1[k] = xtab[xoff + 3 * dx + 1];
            c[k] = xtab[xoff + 3 * dx + 2];
        }
        e[0] = (uint32_t)x0[0];
        for (int k = 0; k < 4; ++k) {
            const int o0 = x0[k] - x0[0], o1 = x1[k] - x0[0];
            if (o0 < 0 || o1 < 0 || o0 > 7 || o1 > 7) return false;
            const uint32_t sv = (uint32_t)o0 | (0x0cu << 8) | ((uint32_t)o1 << 16) | (0x0cu << 24);
            e[1 + k] = sv;        // sel[0..3] = g0.y, g0.z, g0.w, g1.x
            e[5 + k] = (uint32_t)c[k];  // coefficient pairs: g1.y .. g2.x
        }
        out.insert(out.end(), e, e + 12);
    }
    return true;
}

// K1b — the small top levels in one launch: one 1024-thread workgroup per frame copies level
// ts-1 into LDS, then makes levels ts .. L-1 one after the other, each from the previous one
// held in LDS (two buffers, ping-pong), writing every level to the pyramid as well.  Same
// host tables and integer arithmetic as resize_kernel.  Used when the two largest levels of
// the tail fit the workgroup's LDS (levels 5-7 at 640 x 480).
constexpr int kTailBlock = 1024;
constexpr int kTailLds = 144 * 1024;
constexpr int kTailRows = 512;  // rows of a tail level whose y table is staged in LDS
template <bool kX86>
__global__ __launch_bounds__(kTailBlock) void resize_tail_kernel(ResizeTailArgs a) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[kTailLds];
    const int f = blockIdx.x;
    const int tid = threadIdx.x;
    // The tables of each level (its y table for LDS, this thread's four x entries) are loaded
    // one level ahead, so they arrive while the level before is made: loaded at the top of
    // their own level, each level began with two global round trips.  Loads unconditional at
    // clamped indices (3 dh <= 3 kTailRows: entries tid and tid + kTailBlock).
    static_assert(3 * kTailRows <= 2 * kTailBlock, "two y-table entries per thread");
    int yn[2], xn[4][3];
    auto fetch_tables = [&](int k) __attribute__((always_inline)) {
        const int n3 = 3 * a.dh[k], dw = a.dw[k];
        const int* yt = a.yt[k];
        const int* xt = a.xt[k];
        yn[0] = yt[min(tid, n3 - 1)];
        yn[1] = yt[min(tid + kTailBlock, n3 - 1)];
        const int x = 4 * (tid % ((dw + 3) >> 2));
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int dx = min(x + q, dw - 1);
#pragma unroll
            for (int e = 0; e < 3; ++e) xn[q][e] = xt[3 * dx + e];
        }
    };
    fetch_tables(0);
    {   // level ts-1 from the pyramid in 16-byte chunks (LDS pitch lp[0] % 16 == 0, inside the
        // slab's 64-byte row pitch), four per thread in flight before the LDS stores
        const LevelPtr sp = a.src;
        const uint8_t* src = sp.base + f * sp.fpitch;
        const int cpr = a.lp[0] >> 4, total = a.sh * cpr;
        for (int base = 0; base < total; base += 4 * kTailBlock) {
            uint4 v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {  // (unconditional: an index past the end re-reads the last)
                const int i = min(base + kTailBlock * u + tid, total - 1);
                const int r = i / cpr, c = i - r * cpr;
                v[u] = *reinterpret_cast<const uint4*>(src + (long long)r * sp.pitch + 16 * c);
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {  // (unconditional: see stage_rows16)
                const int i = min(base + kTailBlock * u + tid, total - 1);
                const int r = i / cpr, c = i - r * cpr;
                *reinterpret_cast<uint4*>(lds + r * a.lp[0] + 16 * c) = v[u];
            }
        }
    }
    __syncthreads();
    // the row tables of the level being made, staged in LDS: the row loop below would
    // otherwise wait on three dependent global loads per iteration
    __shared__ int yts[3 * kTailRows];
    for (int k = 0; k < a.nt; ++k) {
        // (offsets from lds, not a pointer array: that would make every access a flat one)
        const uint8_t* s = lds + ((k & 1) ? a.buf_b : 0);
        uint8_t* d = lds + (((k + 1) & 1) ? a.buf_b : 0);
        const int sp_l = a.lp[k], dp_l = a.lp[k + 1];
        const int dw = a.dw[k], dh = a.dh[k], xb = a.simd_xb[k];
        const int* yt = yts;
        const int ycur[2] = {yn[0], yn[1]};
        int xc[4][3];
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int e = 0; e < 3; ++e) xc[q][e] = xn[q][e];
        if (k + 1 < a.nt) fetch_tables(k + 1);
        yts[min(tid, 3 * dh - 1)] = ycur[0];
        yts[min(tid + kTailBlock, 3 * dh - 1)] = ycur[1];
        __syncthreads();
        const int gpr = (dw + 3) >> 2;           // 4-pixel groups per row
        const int rps = kTailBlock / gpr;        // rows per sweep
        const int gx = tid % gpr, ry = tid / gpr;
        const LevelPtr dp = a.dst[k];
        uint8_t* dst = const_cast<uint8_t*>(dp.base) + f * dp.fpitch;
        if (ry < rps) {
            const int x = 4 * gx;
            const int n = min(4, dw - x);
            int x0[4], x1[4], a0[4], a1[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                x0[q] = xc[q][0];
                x1[q] = xc[q][1];
                const int aa = xc[q][2];
                a0[q] = (int)(hcoef<kX86>((uint32_t)aa) & 0xffffu);  // x86: 16 a0, 16 a1 (hcoef)
                a1[q] = (int)(hcoef<kX86>((uint32_t)aa) >> 16);
            }
            for (int y = ry; y < dh; y += rps) {
                const int bb = yt[3 * y + 2];
                const int b0 = bb & 0xffff, b1 = (int)((unsigned)bb >> 16);
                const uint8_t* s0 = s + yt[3 * y] * sp_l;
                const uint8_t* s1 = s + yt[3 * y + 1] * sp_l;
                uint32_t t0[4], t1[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    t0[q] = __umul24(s0[x0[q]], a0[q]) + __umul24(s0[x1[q]], a1[q]);
                    t1[q] = __umul24(s1[x0[q]], a0[q]) + __umul24(s1[x1[q]], a1[q]);
                }
                const uint32_t packed = resize4<kX86>(t0, t1, b0, b1, x, xb);
                *reinterpret_cast<uint32_t*>(d + y * dp_l + x) = packed;  // LDS pitch % 4 == 0
                uint8_t* o = dst + (long long)y * dp.pitch + x;
                if (n == 4) {
                    *reinterpret_cast<uint32_t*>(o) = packed;
                } else {
                    for (int q = 0; q < n; ++q) o[q] = (uint8_t)(packed >> (8 * q));
                }
            }
        }
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------------------------
// K2 — FAST per cell.  S(p) = max(q0, -q1) - 1 where q0 (q1) is the max (min) over the 16
// nine-pixel arcs of the min (max) of d = v - circle: p is a cv::FAST corner at threshold t iff
// S(p) >= t, and cornerScore<16> returns exactly S(p) for such p (DESIGN.md "FAST").  So S is
// computed once per pixel and both thresholds of the fallback reuse it.  S ranges over
// [-256, 254]; only S >= 0 can be a corner, so LDS keeps max(S, -1) + 1 as a byte.
constexpr int kFastBlock = 64;   // one wave per cell: ballot compaction keeps row-major order
// The workgroup is one wave, whose LDS operations complete in order: its barriers only keep the
// compiler from moving LDS accesses across them (__syncthreads() would also drain the wave's
// outstanding global stores at each one; measured level: fast 0.2429 vs 0.2440 ms).
__device__ __forceinline__ void fast_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
constexpr int kRoiMax = 72;      // cell ROI <= (59+6) x (59+6): wCell < 2*W for every level size

typedef short short2v __attribute__((ext_vector_type(2)));

// S for the pixel at p (ROI row stride st).  Both arc polarities run in one packed f16 pair
// e = (d, -d), d = v - circle: a byte b enters as the exact f16 1024 + b (bits 0x6400 + b, one
// v_mad_u32_u24 for both halves), so every d in [-255, 255] and every min / max of them is an
// exact f16 integer.  9-arcs come from 3-arcs with v_pk_minimum3_f16:
// lo = max_k min(d[k..k+8]) = q0, hi = max_k min(-d[k..k+8]) = -q1.
typedef _Float16 half2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ half2v fast_h2(uint32_t b) {
    return __builtin_bit_cast(half2v, b * 0x10001u + 0x64006400u);
}
#ifndef ORBFE_FAST_DENORM
#define ORBFE_FAST_DENORM 1
#endif
#if ORBFE_FAST_DENORM
// The same S with every byte taken as the f16 DENORMAL of its bit pattern, b * 2^-24: the
// zero-extended ds_read_u8 result is the operand as loaded (op_sel_hi = 0 puts its low half in
// both halves, neg_lo negates one), so the 17 per-byte conversions vanish.  f16 denormals are
// not flushed (the kernel's f16/f64 denormal mode is IEEE), minimum / maximum order them as the
// integers they encode, and every sum below stays under 1024 units (|q| + |v| <= 510), so each
// value is exact; the result's sign-magnitude bits are S + 1 directly.
__device__ __forceinline__ _Float16 fast_dn(uint32_t b) {
    return __builtin_bit_cast(_Float16, (unsigned short)b);
}
__device__ __forceinline__ int fast_S(const uint8_t* p, int st) {
    const _Float16 V = fast_dn(p[0]);
    const uint32_t x[16] = {p[3 * st],      p[3 * st + 1],  p[2 * st + 2],  p[st + 3],
                            p[3],           p[-st + 3],     p[-2 * st + 2], p[-3 * st + 1],
                            p[-3 * st],     p[-3 * st - 1], p[-2 * st - 2], p[-st - 3],
                            p[-3],          p[st - 3],      p[2 * st - 2],  p[3 * st - 1]};
    half2v e[16], m3[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const _Float16 X = fast_dn(x[k] & 0xffffu);
        e[k] = half2v{-X, X};
    }
#pragma unroll
    for (int k = 0; k < 16; ++k)
        m3[k] = __builtin_elementwise_minimum(__builtin_elementwise_minimum(e[k], e[(k + 1) & 15]),
                                              e[(k + 2) & 15]);
    half2v q = __builtin_elementwise_minimum(__builtin_elementwise_minimum(m3[0], m3[3]), m3[6]);
#pragma unroll
    for (int k = 1; k < 16; ++k) {
        const half2v m9 = __builtin_elementwise_minimum(
            __builtin_elementwise_minimum(m3[k], m3[(k + 3) & 15]), m3[(k + 6) & 15]);
        q = __builtin_elementwise_maximum(q, m9);
    }
    q = q + half2v{V, -V};
    const uint32_t bits = __builtin_bit_cast(unsigned short, __builtin_elementwise_maximum(q.x, q.y));
    const int mag = (int)(bits & 0x3ffu);
    return ((bits & 0x8000u) ? -mag : mag) - 1;
}
#else
__device__ __forceinline__ int fast_S(const uint8_t* p, int st) {
    const half2v V = fast_h2(p[0]);
    const uint32_t x[16] = {p[3 * st],      p[3 * st + 1],  p[2 * st + 2],  p[st + 3],
                            p[3],           p[-st + 3],     p[-2 * st + 2], p[-3 * st + 1],
                            p[-3 * st],     p[-3 * st - 1], p[-2 * st - 2], p[-st - 3],
                            p[-3],          p[st - 3],      p[2 * st - 2],  p[3 * st - 1]};
    // The centre is subtracted once at the end: min over an arc of (x - v) = (min x) - v and of
    // (v - x) = v - (max x), so the arcs run on e = (-X, X) (the sign is a source modifier of
    // v_pk_minimum3_f16) and q + (V, -V) restores (q0, -q1).
    half2v e[16], m3[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const half2v X = fast_h2(x[k]);
        e[k] = half2v{-X.x, X.y};
    }
#pragma unroll
    for (int k = 0; k < 16; ++k)
        m3[k] = __builtin_elementwise_minimum(__builtin_elementwise_minimum(e[k], e[(k + 1) & 15]),
                                              e[(k + 2) & 15]);
    half2v q = __builtin_elementwise_minimum(__builtin_elementwise_minimum(m3[0], m3[3]), m3[6]);
#pragma unroll
    for (int k = 1; k < 16; ++k) {
        const half2v m9 = __builtin_elementwise_minimum(
            __builtin_elementwise_minimum(m3[k], m3[(k + 3) & 15]), m3[(k + 6) & 15]);
        q = __builtin_elementwise_maximum(q, m9);
    }
    q = q + half2v{V.x, -V.y};
    return (int)(float)__builtin_elementwise_maximum(q.x, q.y) - 1;
}
#endif

// Necessary condition for a corner at t (the pre-test): a 9-arc always holds two consecutive
// cardinal points (0/4/8/12), so both must be brighter than v + t or both darker than v - t.

__device__ __forceinline__ int lane_prefix(unsigned long long mask) {
    return __popcll(mask & ((1ull << (threadIdx.x & 63)) - 1));
}

// The pre-test's per-byte flags (bit 7 of each byte of fl) as lane masks: one SDWA compare of
// the sign-extended byte each (the compiler's form is a v_bfe and a v_cmp per byte).  The
// compare honours exec like any VOPC: inactive lanes read 0.
template <int kB>
__device__ __forceinline__ unsigned long long byte_ballot(uint32_t fl) {
    unsigned long long m;
    if constexpr (kB == 0)
        asm("v_cmp_lt_i32_sdwa %0, sext(%1), 0 src0_sel:BYTE_0 src1_sel:DWORD" : "=s"(m) : "v"(fl));
    else if constexpr (kB == 1)
        asm("v_cmp_lt_i32_sdwa %0, sext(%1), 0 src0_sel:BYTE_1 src1_sel:DWORD" : "=s"(m) : "v"(fl));
    else if constexpr (kB == 2)
        asm("v_cmp_lt_i32_sdwa %0, sext(%1), 0 src0_sel:BYTE_2 src1_sel:DWORD" : "=s"(m) : "v"(fl));
    else
        m = __ballot((int)fl < 0);
    return m;
}
// b where this lane's bit of m is set, else a: one v_cndmask on the lane mask itself (a
// ballot's SGPR pair), no per-lane compare to rebuild the condition.
__device__ __forceinline__ int lane_select(unsigned long long m, int a, int b) {
    int r;
    asm("v_cndmask_b32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "s"(m));
    return r;
}

// Ordered emission of the NMS survivors at threshold t among the compacted candidates.
//
// Candidates are ROI offsets o = r * P + c of their window's top-left (row-major order), and
// the score plane S shares the ROI pitch with a zero border, so candidate (r, c) scores at
// S[o + P + 1] and its 8 neighbours sit at fixed offsets.  S holds max(S, -1) + 1, 0 where the
// pre-test ruled a corner out.  cv::FAST's strict 3x3 NMS (H1) keeps s when s >= t and
// s > nv for every neighbour, nv = (ns >= t ? ns : 0): for s >= max(t, 1) that is exactly
// max(ns) < s, and for s = t = 0 it never holds — so one byte compare against the neighbour
// maximum decides it.  ORBFE_FAST_EMIT2 (default): the entries whose own score reaches the
// threshold (about a quarter of the pre-test survivors) are first compacted in order to the
// front of the list, so the eight neighbour reads run over full waves of corners only.
#ifndef ORBFE_FAST_EMIT2
#define ORBFE_FAST_EMIT2 1
#endif
__device__ __forceinline__ int fast_emit(const uint8_t* S, uint16_t* list, int cnt, int P,
                                         unsigned inv_p, int t, const CellDesc& cell,
                                         uint32_t* out, int cap) {
    const int tb = max(t, 1) + 1;
    if (ORBFE_FAST_EMIT2) {
        int nc = 0;  // in place: chunk k's writes land below its own (already read) entries
        for (int base = 0; base < cnt; base += 64) {
            const int i = base + (int)threadIdx.x;
            int off = 0, sb = 0;
            if (i < cnt) {
                off = list[i];
                sb = S[off + P + 1];
            }
            const unsigned long long m = __ballot(sb >= tb);
            if (sb >= tb) list[nc + lane_prefix(m)] = (uint16_t)off;
            nc += __popcll(m);
        }
        fast_sync();
        cnt = nc;
    }
    int o = 0;
    for (int base = 0; base < cnt; base += 64) {
        const int i = base + (int)threadIdx.x;
        bool keep = false;
        int off = 0, sb = 0;
        if (i < cnt) {
            off = list[i];
            const uint8_t* q = S + off + P + 1;
            sb = q[0];
            const int nb = max(max(max(q[-P - 1], q[-P]), max(q[-P + 1], q[-1])),
                               max(max(q[1], q[P - 1]), max(q[P], q[P + 1])));
            keep = sb >= tb && nb < sb;
        }
        const unsigned long long m = __ballot(keep);
        if (keep) {
            const int slot = o + lane_prefix(m);
            const int r = (int)__umulhi((unsigned)off, inv_p), cc = off - r * P;
            // key relative to (minBorderX, minBorderY): pt + (j*wCell, i*hCell) (819-824)
            if (slot < cap)
                out[slot] = pack_key(cell.x0 + 3 + cc - kMinBorder, cell.y0 + 3 + r - kMinBorder, sb - 1);
        }
        o += __popcll(m);
    }
    return o;
}

// ORBFE_FAST_TIMING (attribution builds only, tools/probe/fast_phases.py): lane 0 of each wave
// records per-phase shader-clock totals of cells < kFtCells of frames < kFtFrames into
// g_fast_t[frame][cell][16]: 0 staging (ROI loads + score-plane zeroing), 1 pre-test sweeps,
// 2 list writes, 3 scoring, 4 emission (NMS + key stores), 5 overflow flushes, 6 the minThFAST
// rerun pass (all of it), 7 total, then counts: 8 sweeps, 9 survivors scored, 10 corners
// emitted, 11 flushes, 12 rerun (0 / 1).  Every mark waits for the wave's outstanding memory
// operations first (s_waitcnt 0), so a phase owns the latency of its own loads.
#ifdef ORBFE_FAST_TIMING
constexpr int kFtFrames = 8, kFtCells = 8192;
__device__ long long g_fast_t[kFtFrames * kFtCells * 16];
#define FT_NOW() (__builtin_amdgcn_s_waitcnt(0), (long long)clock64())
#define FT_ADD(k, t0) do { const long long t1_ = FT_NOW(); ft[k] += t1_ - (t0); (t0) = t1_; } while (0)
#define FT_CNT(k, v) do { ft[k] += (v); } while (0)
#else
#define FT_NOW() 0ll
#define FT_ADD(k, t0) do { (void)(t0); } while (0)
#define FT_CNT(k, v) do { } while (0)
#endif

// kP: the ROI pitch as a compile-time constant (48 for every cell width up to 45 px, i.e. the
// common frame sizes), so the 16 circle offsets of fast_S become LDS immediates; 0 = runtime.
// Measured and dropped (profiles/r02/experiments/fast_variants.json): several cells per wave
// with the next ROI prefetched into registers, and 4-pixel groups scored from aligned dwords
// (conflict-free LDS reads, but 1.6x the VALU per survivor: 0.29 -> 0.35 ms).
template <int kP>
__global__ __launch_bounds__(kFastBlock) void fast_kernel(FastArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char fast_lds[];
    int c, f;
    xcd_block(c, f);
    const int lane = threadIdx.x;
#ifdef ORBFE_FAST_TIMING
    long long ft[16] = {};
    const long long ft_start = FT_NOW();
    long long ftc = ft_start;
#endif
    const CellDesc cell = a.cells[c];
    const LevelPtr lp = a.pyr[cell.level];
    const int rows = cell.y1 - cell.y0, cols = cell.x1 - cell.x0;
    const int P = kP ? kP : a.roi_pitch;
    uint8_t* roi_base = fast_lds;
    uint8_t* S = fast_lds + a.roi_rows * P;
    uint16_t* list = reinterpret_cast<uint16_t*>(S + (((a.roi_rows - 4) * P + 15) & ~15));
    // Each lane copies whole ROI rows with 16-byte loads from the dword-aligned x0a (global
    // dwordx4 needs only 4-byte alignment; LDS rows are 16-byte aligned, P % 16 == 0).  A row
    // spans <= 5 chunks; the bytes past x1 (< 16) stay inside the level row or the next one,
    // and ROI rows never reach the level's last row.
    const int x0a = cell.x0 & ~3, shift = cell.x0 - x0a;
    const int nq = (shift + cols + 15) >> 4;
    const uint8_t* img = lp.base + f * lp.fpitch + (long long)cell.y0 * lp.pitch + x0a;
    for (int r0 = 0; r0 < rows; r0 += 64) {
        const int r = r0 + lane;
        if (r < rows) {
            const uint8_t* src = img + (long long)r * lp.pitch;
            uint4 v[5];
#pragma unroll
            for (int q = 0; q < 5; ++q)
                if (q < nq) v[q] = load16_a4(src + 16 * q);
#pragma unroll
            for (int q = 0; q < 5; ++q)
                if (q < nq) *reinterpret_cast<uint4*>(roi_base + r * P + 16 * q) = v[q];
        }
    }
    const uint8_t* roi = roi_base + shift;
    const int nr = rows - 6, nc = cols - 6;  // candidates: ROI rows/cols 3 .. n-4
    const int ncand = (nr > 0 && nc > 0) ? nr * nc : 0;
    // score plane: ROI pitch, rows -1 .. nr of the candidates, zero border
    // (16-byte stores: S is 16-byte aligned and (nr + 2) * P a multiple of 16)
    for (int i = lane; i < (ncand ? ((nr + 2) * P) >> 4 : 0); i += 64) reinterpret_cast<uint4*>(S)[i] = make_uint4(0u, 0u, 0u, 0u);
    const unsigned inv_p = 0xffffffffu / (unsigned)P + 1u;  // r = umulhi(o, inv_p) for o < 2^16
    // Pre-test lanes: (candidate row lr, 4-pixel group lg).  Group g holds ROI-row bytes
    // [4g, 4g + 4) of roi_base (dword aligned, P % 16 == 0); candidate columns are
    // X0 .. X0 + nc - 1 (X0 = shift + 3), so a row spans gpr <= 18 groups (nc <= 66).
    const int X0 = shift + 3, g0 = X0 >> 2;
    const int gpr = ncand ? ((X0 + nc - 1) >> 2) - g0 + 1 : 1;
    const int rps = 64 / gpr;  // candidate rows per sweep
    // lane / gpr through the float reciprocal of the (wave-uniform) gpr <= 18: floor((lane +
    // 0.5) / gpr) is at least 0.5 / gpr from an integer, far above rcp's error (the integer
    // division cost ~20 VALU per cell)
    const int lr = (int)(((float)lane + 0.5f) * __builtin_amdgcn_rcpf((float)gpr)), lg = lane - lr * gpr;
    const int gx = 4 * (g0 + lg);  // roi_base column of the group's byte 0
    // 0x80 in every byte whose pixel is a candidate column: only the row's first group (bytes
    // before X0) and last group (bytes from X0 + nc) are partial
    uint32_t vmask = lr < rps && ncand ? 0x80808080u : 0u;
    if (lg == 0) vmask &= 0x80808080u << (8 * (X0 - gx));
    if (lg == gpr - 1) vmask &= 0x80808080u >> (8 * (4 - min(X0 + nc - gx, 4)));
    const uint32_t* lds32 = reinterpret_cast<const uint32_t*>(roi_base);
    const int P4 = P >> 2;
    fast_sync();
#ifdef ORBFE_FAST_TIMING
    FT_ADD(0, ftc);
#endif
    // Pass at iniThFAST: only pixels passing the pre-test at that threshold can have S >= t,
    // and every other pixel counts as 0 in the NMS, so S is computed for those alone.
    uint32_t* out = a.cell_keys + f * a.cell_cap_total + cell.slot;
    // S for list entries [from, to)
    auto score = [&](int from, int to) {
// S loop unroll: 1 measured 0.2367-0.2394 ms vs 0.2423-0.2451 at 2 and 0.2437 at 4 (fast_pipe.json)
#ifndef ORBFE_FAST_SU
#define ORBFE_FAST_SU 1
#endif
#pragma unroll ORBFE_FAST_SU
        for (int i = from + lane; i < to; i += 64) {
            const int o = list[i];
            // S < 0 is never a corner for t >= 0: clamp to -1 so S + 1 fits a byte
            S[o + P + 1] = (uint8_t)(max(fast_S(roi + o + 3 * P + 3, P), -1) + 1);
        }
    };
    // The list holds cand_max entries (not one per candidate pixel: ~22 % pass the pre-test on
    // textured frames, and the LDS it would take bounds the kernel's occupancy).  Before a
    // sweep that could overflow it, the entries so far are scored and those of rows up to
    // r0 - 2 — whose 3 x 3 neighbourhoods are complete — are emitted; the last pre-tested row's
    // entries move to the front (<= nc <= 66 of them; a sweep adds <= rps * nc <= 256, so
    // cand_max >= 322 always makes progress).
    const int sweep_max = rps * nc;
    int total = 0;
    for (int pass = 0; pass < 2 && total == 0; ++pass) {
        const int t = pass ? a.min_th : a.ini_th;  // rerun at minThFAST when empty (811-815)
#ifdef ORBFE_FAST_TIMING
        const long long ft_pass = ftc;
        FT_CNT(12, pass);
#endif
        // Byte-parallel pre-test (4 pixels per lane): with v_lerp_u8,
        // lerp(c, ~v, R1) = floor((c - v + 255 + (t & 1)) / 2) per byte, and the high bit of
        // lerp(that, M, 0) with M = 128 - ceil(t / 2) is exactly c - v > t (c > v + t); with
        // the roles swapped, v - c > t (c < v - t) — checked for every c, v, t in
        // tests/test_oracle_cpu.py.  A 9-arc holds two consecutive cardinal points, so a
        // corner needs (b0 | b8) & (b4 | b12) of one polarity.
        const uint32_t R1 = (t & 1) ? 0x01010101u : 0u, R0 = R1 ^ 0x01010101u;
        const uint32_t M = (uint32_t)(128 - ((t + 1) >> 1)) * 0x01010101u;
        // dark test without a per-byte NOT (fast_strip_sweep; tests/test_oracle_cpu.py): at
        // t = 255 the byte 256 - M wraps to 0 and every pixel passes, but no score reaches 255
        const uint32_t M2 = (uint32_t)(128 + ((t + 1) >> 1)) * 0x01010101u;
        int cnt = 0, scored = 0, emitted = 0;
        for (int r0 = 0; r0 < nr; r0 += rps) {
            if (cnt + sweep_max > a.cand_max) {  // wave-uniform
#ifdef ORBFE_FAST_TIMING
                FT_CNT(11, 1);
                FT_CNT(9, cnt - scored);
#endif
                fast_sync();
                score(scored, cnt);
                fast_sync();
                const int lim = (r0 - 1) * P;  // entries of rows <= r0 - 2 lie below
                int k = 0;
                for (int i0 = 0; i0 < cnt; i0 += 64)
                    k += __popcll(__ballot(i0 + lane < cnt && list[i0 + lane] < lim));
                emitted += fast_emit(S, list, k, P, inv_p, t, cell, out + emitted, cell.cap - emitted);
                const int n1 = cnt - k;
                const int e0 = lane < n1 ? list[k + lane] : 0, e1 = lane + 64 < n1 ? list[k + 64 + lane] : 0;
                fast_sync();
                if (lane < n1) list[lane] = (uint16_t)e0;
                if (lane + 64 < n1) list[lane + 64] = (uint16_t)e1;
                cnt = scored = n1;
#ifdef ORBFE_FAST_TIMING
                FT_ADD(5, ftc);
#endif
            }
            const int cr = r0 + lr;
            uint32_t fl = 0;
            if (vmask && cr < nr) {
                const int w = (cr + 3) * P4 + (gx >> 2);  // dword of the group's centres
                const uint32_t cur = lds32[w], prv = lds32[w - 1], nxt = lds32[w + 1];
                const uint32_t up = lds32[w - 3 * P4], dn = lds32[w + 3 * P4];
                const uint32_t c4 = __builtin_amdgcn_alignbyte(nxt, cur, 3);   // column + 3
                const uint32_t c12 = __builtin_amdgcn_alignbyte(cur, prv, 1);  // column - 3
                const uint32_t ncur = ~cur;
                auto hb = [&](uint32_t c) {
                    return __builtin_amdgcn_lerp(__builtin_amdgcn_lerp(c, ncur, R1), M, 0u);
                };
                auto xd = [&](uint32_t c) {  // NOT (c < v - t) in the high bits
                    return __builtin_amdgcn_lerp(__builtin_amdgcn_lerp(c, ncur, R0), M2, 0u);
                };
                const uint32_t br = (hb(dn) | hb(up)) & (hb(c4) | hb(c12));
                const uint32_t xk = (xd(dn) & xd(up)) | (xd(c4) & xd(c12));
                fl = (br | ~xk) & vmask;
            }
            const unsigned long long b0 = byte_ballot<0>(fl), b1 = byte_ballot<1>(fl),
                                     b2 = byte_ballot<2>(fl), b3 = byte_ballot<3>(fl);
#ifdef ORBFE_FAST_TIMING
            FT_ADD(1, ftc);
            FT_CNT(8, 1);
#endif
            if (fl) {  // row-major: earlier lanes, then this lane's lower bytes
                auto below = [](unsigned long long b, uint32_t acc) {  // popc(b & lanes below)
                    return __builtin_amdgcn_mbcnt_hi((uint32_t)(b >> 32),
                                                     __builtin_amdgcn_mbcnt_lo((uint32_t)b, acc));
                };
                int pos = (int)below(b3, below(b2, below(b1, below(b0, (uint32_t)cnt))));
                const int ob = cr * P + gx - X0;  // ROI offset of byte 0's window
                // unconditional stores (no exec-mask branch per byte): a byte that is not a
                // survivor writes the lane's trash slot past the list; the slot is chosen by the
                // byte's ballot mask directly
                const int tr = a.cand_max + lane;
                const int f0 = (fl >> 7) & 1, f1 = (fl >> 15) & 1, f2 = (fl >> 23) & 1;
                list[lane_select(b0, tr, pos)] = (uint16_t)ob;
                pos += f0;
                list[lane_select(b1, tr, pos)] = (uint16_t)(ob + 1);
                pos += f1;
                list[lane_select(b2, tr, pos)] = (uint16_t)(ob + 2);
                pos += f2;
                list[lane_select(b3, tr, pos)] = (uint16_t)(ob + 3);
            }
            cnt += __popcll(b0) + __popcll(b1) + __popcll(b2) + __popcll(b3);
#ifdef ORBFE_FAST_TIMING
            FT_ADD(2, ftc);
#endif
        }
        fast_sync();
        score(scored, cnt);
        fast_sync();
#ifdef ORBFE_FAST_TIMING
        FT_ADD(3, ftc);
        FT_CNT(9, cnt - scored);
#endif
        total = emitted + fast_emit(S, list, cnt, P, inv_p, t, cell, out + emitted, cell.cap - emitted);
        fast_sync();
#ifdef ORBFE_FAST_TIMING
        FT_ADD(4, ftc);
        if (pass) ft[6] += ftc - ft_pass;
#endif
    }
    if (lane == 0) {
        const int n = min(total, cell.cap);
        a.cell_cnt[f * a.ncells + c] = n;
        // the level's key total for the oct-tree (which reads it and resets it to 0)
        if (n) atomicAdd(&a.level_keys[f * kMaxLevels + cell.level], n);
    }
#ifdef ORBFE_FAST_TIMING
    ft[7] = FT_NOW() - ft_start;
    ft[10] = total;
    if (lane == 0 && f < kFtFrames && c < kFtCells)
        for (int k = 0; k < 16; ++k) g_fast_t[((long long)f * kFtCells + c) * 16 + k] = ft[k];
#endif
}

template __global__ void fast_kernel<0>(FastArgs);
template __global__ void fast_kernel<kFastPitch>(FastArgs);

// ---------------------------------------------------------------------------------------------
// K3 — DistributeOctTree as a data-parallel emulation of the reference's std::list.
//
// The list is an array in list order, rebuilt every pass into the other buffer:
//   phase-1 pass: new list = reverse(children of the divided nodes, in list order, each
//                 n1..n4) ++ (single-key nodes, in order)              (push_front, 605-663)
//   phase-2 round: the expandable nodes sorted by (size desc, creation seq desc) [H2] are
//                 divided in that order until size >= N: new list = reverse(children in
//                 processing order) ++ (untouched nodes, in order)     (675-736)
// Keys stay in original order (cell-row-major, FAST emission order) in K; NODE[k] is the list
// position of key k's node, or -1 once that node holds this key alone (it then remembers the
// key itself).  Both live in LDS (kOctLdsKeys keys: every level of the bench configs, whose
// FAST lists stay below ~3,300 keys), so every pass is a sweep of LDS reads and LDS atomics;
// a level with more keys runs the same code on global arrays.  Final: per node the max
// response, first (lowest original index) on ties (741-759).
constexpr int kOctBlock = kOctBlockSize;
// small batches (the single-frame call): one tree per CU at most, so the level-0 tree's sweeps
// spread over 16 waves instead of 4
constexpr int kOctBlockSmall = 1024;

// Carve of the dynamic LDS region (sizes in elements).  IT is the type of the per-node key
// counts, single-key indices and quadrant keys / child positions: u16 when the level's keys
// sit in LDS (<= kOctLdsKeys keys, < 2^16 nodes), int on the global-array path (any count).
// With u16 the four quadrant counters of a node are two packed u32 LDS atomics.  The narrow
// form is what lets six trees share a CU (DESIGN.md "oct-tree").
template <class IT>
struct OctLds {
    // two node lists (b = 0 / 1): box x0 | x1 << 16, boy y0 | y1 << 16, creation seq (int);
    // key count, key of a single-key node (IT); addressed by arithmetic, since a
    // runtime-indexed pointer array would live in scratch
    int* lists;
    IT* ilists;
    int nc;
    __device__ __forceinline__ int* box(int b) const { return lists + (b * 3 + 0) * nc; }
    __device__ __forceinline__ int* boy(int b) const { return lists + (b * 3 + 1) * nc; }
    __device__ __forceinline__ int* seq(int b) const { return lists + (b * 3 + 2) * nc; }
    __device__ __forceinline__ IT* cnt(int b) const { return ilists + (b * 2 + 0) * nc; }
    __device__ __forceinline__ IT* key(int b) const { return ilists + (b * 2 + 1) * nc; }
    static constexpr bool kPacked = sizeof(IT) == 2;
    static constexpr int kQcWords = kPacked ? 2 : 4;  // u32 words of quadrant counters per node
    // keys per quadrant of list b's nodes (kPacked: quadrants 2w, 2w + 1 in the halves of word
    // w), kQcWords * nc words per list
    uint32_t* qc;
    IT* qk;         // 4 per node: the child's new list position (initial nodes: a key)
    // per node: scan offsets / kept position / processed flag (16-bit in the LDS form: node
    // positions < nc < 2^15, the kept encoding -(1 + position))
    using AT = std::conditional_t<sizeof(IT) == 2, int16_t, int>;
    AT* aux;
    AT* aux2;
    unsigned long long* s64;  // sort keys (phase 2) / best response (final)
    int* tmp;
    int* scal;      // scalars
    __device__ __forceinline__ uint32_t* qcb(int b) const { return qc + b * kQcWords * nc; }
    __device__ __forceinline__ int qcount(int b, int node, int q) const {
        const uint32_t* c = qcb(b);
        if constexpr (kPacked) return (int)((c[node * 2 + (q >> 1)] >> (16 * (q & 1))) & 0xffffu);
        else return (int)c[node * 4 + q];
    }
    __device__ __forceinline__ void qinc(int b, int node, int q) const {
        uint32_t* c = qcb(b);
        if constexpr (kPacked) atomicAdd(&c[node * 2 + (q >> 1)], 1u << (16 * (q & 1)));
        else atomicAdd(&c[node * 4 + q], 1u);
    }
};

// describe's processing order: 32-row bands per level (the last takes every row below), counted
// in the node lists' first words (24 * nc bytes, nc >= 20)
constexpr int kOctBands = 120;

// Bytes of the carve: the LDS form (keys and node positions in LDS, u16 node fields) and the
// global-array form (wider node fields in place of the keys); the launch takes the larger.
constexpr size_t oct_lds_bytes(bool in_lds, int ncap, int sort_cap, int lds_keys) {
    const size_t it = in_lds ? 2 : 4;
    return (size_t)sort_cap * 8 + (in_lds ? (size_t)lds_keys * 6 : 0) +
           (size_t)ncap * (6 * 4 + 4 * it + 2 * (in_lds ? 8 : 16) + 4 * it + 2 * it) + (16 + 16) * 4 + 16;
}

__device__ __forceinline__ int quadrant(int box, int boy, int x, int y) {
    const int x0 = box & 0xffff, x1 = box >> 16, y0 = boy & 0xffff, y1 = boy >> 16;
    const int hx = (x1 - x0 + 1) >> 1, hy = (y1 - y0 + 1) >> 1;  // ceil((UR.x-UL.x)/2.f)
    const bool left = x < x0 + hx, top = y < y0 + hy;
    return left ? (top ? 0 : 2) : (top ? 1 : 3);
}

__device__ __forceinline__ void child_box(int box, int boy, int q, int& cbx, int& cby) {
    const int x0 = box & 0xffff, x1 = box >> 16, y0 = boy & 0xffff, y1 = boy >> 16;
    const int xm = x0 + ((x1 - x0 + 1) >> 1), ym = y0 + ((y1 - y0 + 1) >> 1);
    const int cx0 = (q & 1) ? xm : x0, cx1 = (q & 1) ? x1 : xm;
    const int cy0 = (q & 2) ? ym : y0, cy1 = (q & 2) ? y1 : ym;
    cbx = cx0 | (cx1 << 16);
    cby = cy0 | (cy1 << 16);
}

// ORBFE_OCT_TIMING builds (tools/probe/oct_timing.py) record per-phase shader-clock stamps of
// every (frame, level) tree: [0] start, [1] counted, [2] compacted, [3] initial nodes,
// [4 + p] phase-1 pass p, [12 + r] phase-2 round r, [30] passes | rounds << 8, [31] end.
#ifdef ORBFE_OCT_TIMING
__device__ long long g_oct_t[256 * 16 * 64];
#define OCT_MARK(tm, i) do { if (threadIdx.x == 0 && (tm)) (tm)[(i)] = clock64(); } while (0)
#else
#define OCT_MARK(tm, i) do { } while (0)
#endif

// Sweep over the live keys (NODE >= 0): body(k, packed key, node) for each.  A thread loads
// kOctU keys and their nodes before using any, so their LDS round trips overlap.
#ifndef ORBFE_OCT_U
#define ORBFE_OCT_U 4
#endif
constexpr int kOctU = ORBFE_OCT_U;
template <int BLK, class KT, class NT, class F>
__device__ __forceinline__ void oct_sweep(const KT* K, const NT* NODE, int nkeys, F&& body) {
    for (int k0 = threadIdx.x; k0 < nkeys; k0 += kOctU * BLK) {
        int node[kOctU];
        uint32_t kk[kOctU];
#pragma unroll
        for (int u = 0; u < kOctU; ++u) {
            const int k = k0 + u * BLK;
            node[u] = k < nkeys ? (int)NODE[k] : -1;
            kk[u] = k < nkeys ? K[k] : 0u;
        }
#pragma unroll
        for (int u = 0; u < kOctU; ++u)
            if (node[u] >= 0) body(k0 + u * BLK, kk[u], node[u]);
    }
}
// The same sweep in stages, each stage's LDS lookups for all kOctU keys issued together (a
// body per key under its own exec mask would wait on each key's lookups in turn): the keys'
// quadrants in their nodes' boxes, then body(k[], node[], q[]) for the kOctU keys at once
// (node < 0: not a live key; its lookups read node 0 and are discarded).
template <int BLK, class KT, class NT, class F>
__device__ __forceinline__ void oct_sweep_q(const KT* K, const NT* NODE, int nkeys, const int* bx,
                                            const int* by, F&& body) {
    for (int k0 = threadIdx.x; k0 < nkeys; k0 += kOctU * BLK) {
        int node[kOctU], q[kOctU], kx[kOctU];
        uint32_t kk[kOctU];
#pragma unroll
        for (int u = 0; u < kOctU; ++u) {
            const int k = k0 + u * BLK;
            kx[u] = k;
            node[u] = k < nkeys ? (int)NODE[k] : -1;
            kk[u] = k < nkeys ? K[k] : 0u;
        }
        int bxv[kOctU], byv[kOctU];
#pragma unroll
        for (int u = 0; u < kOctU; ++u) {
            const int nd = max(node[u], 0);
            bxv[u] = bx[nd];
            byv[u] = by[nd];
        }
#pragma unroll
        for (int u = 0; u < kOctU; ++u) q[u] = quadrant(bxv[u], byv[u], key_x(kk[u]), key_y(kk[u]));
        body(kx, node, q, kk);
    }
}

// The tree of one (frame, level) after its keys are in K (nkeys, original order).
//
// Quadrant counts are double-buffered with the node lists (qcb(b) belongs to list b), so each
// pass / round needs a single sweep over the keys: a key moves to its node's child (or keeps
// its node) in the list being built and at once counts its quadrant in that node for the next
// pass; a key left alone in its node records itself as the node's key.  Per pass: the node
// scan, the node rewrite (which also clears the next list's counters) and the fused sweep.
template <int BLK, class IT, class KT, class NT>
__device__ __forceinline__ void octree_level(const OctArgs& a, const OctLds<IT>& s, const LevelGeo& L, KT* K,
                             NT* NODE, int nkeys, uint32_t* out, int* out_cnt,
                                              long long* tm) {
    const int tid = threadIdx.x;
    const int ncap = L.ncap;
    const int N = L.nfeat;
    int* flag_sh = s.scal + 2;    // scal[2]: counters
    int* rmin_sh = s.scal + 3;    // scal[3]: phase-2 cut index
    int* nexp_sh = s.scal + 4;    // scal[4]: phase-1 expandable children
    constexpr int QW = OctLds<IT>::kQcWords;

    // ---- initial nodes (542-584): per-node key counts in list 1's quadrant buffer (free now),
    // list 0's quadrant counters cleared for the first pass
    const int nini = L.nini;
    const float hX = L.hx;
    const int H = L.bh;
    uint32_t* icnt = s.qcb(1);  // nini <= NC / 4 entries
    for (int i = tid; i < nini; i += BLK) {
        icnt[i] = 0u;
        s.qk[i] = (IT)-1;
    }
    for (int i = tid; i < QW * nini; i += BLK) s.qcb(0)[i] = 0u;
    __syncthreads();
    OCT_MARK(tm, 56);
    if (nini == 1) {  // every key in node 0: its count, and any key (read only if it is alone)
        if (tid == 0) {
            icnt[0] = (uint32_t)nkeys;
            s.qk[0] = (IT)(nkeys - 1);
        }
    } else {
        for (int k = tid; k < nkeys; k += BLK) {
            const int node = min((int)((float)key_x(K[k]) / hX), nini - 1);  // vpIniNodes[kp.pt.x/hX] (568)
            atomicAdd(&icnt[node], 1u);
            s.qk[node] = (IT)k;
        }
    }
    __syncthreads();
    OCT_MARK(tm, 57);
    int size;
    {   // list = non-empty initial nodes in index order; single-key nodes are closed
        int total = 0;
        for (int base = 0; base < nini; base += BLK) {
            const int i = base + tid;
            const int ne = i < nini && icnt[i] > 0u;
            int chunk_total;
            const int off = block_exclusive_scan<BLK>(ne, s.tmp, chunk_total);
            if (ne) {
                const int pos = total + off;
                const int x0 = (int)(hX * (float)i), x1 = (int)(hX * (float)(i + 1));
                s.box(0)[pos] = x0 | (x1 << 16);
                s.boy(0)[pos] = 0 | (H << 16);
                s.cnt(0)[pos] = (IT)icnt[i];
                s.seq(0)[pos] = i;
                s.key(0)[pos] = icnt[i] == 1u ? s.qk[i] : (IT)-1;
                s.aux[i] = pos;
            }
            total += chunk_total;
        }
        size = total;
    }
    __syncthreads();
    OCT_MARK(tm, 58);
    // keys -> list-0 nodes, each live key's quadrant counted for the first pass
    if (nini == 1) {
        const bool live = (int)s.cnt(0)[0] >= 2;
        const int bx0 = s.box(0)[0], by0 = s.boy(0)[0];
        uint32_t w01 = 0u, w23 = 0u;  // this thread's quadrant counts, one atomic pair per wave
        for (int k = tid; k < nkeys; k += BLK) {
            NODE[k] = live ? 0 : -1;
            if (live) {
                const uint32_t kk = K[k];
                const int q = quadrant(bx0, by0, key_x(kk), key_y(kk));
                const uint32_t inc = 1u << (16 * (q & 1));
                if (q < 2) w01 += inc; else w23 += inc;
            }
        }
        if (live) {
            uint32_t c[4] = {w01 & 0xffffu, w01 >> 16, w23 & 0xffffu, w23 >> 16};
#pragma unroll
            for (int q = 0; q < 4; ++q) c[q] = (uint32_t)wave_sum((int)c[q]);
            if ((tid & 63) == 0) {
                if constexpr (OctLds<IT>::kPacked) {
                    atomicAdd(&s.qcb(0)[0], c[0] | (c[1] << 16));
                    atomicAdd(&s.qcb(0)[1], c[2] | (c[3] << 16));
                } else {
#pragma unroll
                    for (int q = 0; q < 4; ++q) atomicAdd(&s.qcb(0)[q], c[q]);
                }
            }
        }
    } else {
        for (int k = tid; k < nkeys; k += BLK) {
            const uint32_t kk = K[k];
            const int node = s.aux[min((int)((float)key_x(kk) / hX), nini - 1)];
            const bool live = (int)s.cnt(0)[node] >= 2;
            NODE[k] = live ? node : -1;
            if (live) s.qinc(0, node, quadrant(s.box(0)[node], s.boy(0)[node], key_x(kk), key_y(kk)));
        }
    }
    __syncthreads();
    OCT_MARK(tm, 3);
    int cur = 0;
    int seq_base = nini;
    bool finished = false;
    bool phase2 = false;
    [[maybe_unused]] int npass = 0, nround = 0;  // read by the ORBFE_OCT_TIMING build

    // ---- phase 1: split every open node per pass (593-671); the current nodes' quadrant
    // counts are in qcb(cur)
    for (int pass = 0; pass < 64 && !finished && !phase2; ++pass) {
        const int prev = size;
        const int nxt = cur ^ 1;
        if (pass == 1) OCT_MARK(tm, 33);
        // per node: children (divided) or kept (single); aux = child offset, aux2 = kept offset
        // (nexp_sh: zeroed here, after the previous barrier; summed after the first scan barrier)
        if (tid == 0) *nexp_sh = 0;
        int csize = 0, ksize = 0;
        for (int base = 0; base < size; base += BLK) {
            const int i = base + tid;
            int nch = 0, keep = 0, ne = 0;
            if (i < size) {
                if ((int)s.cnt(cur)[i] >= 2) {
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const int qn = s.qcount(cur, i, q);
                        nch += qn > 0;
                        ne += qn > 1;
                    }
                } else {
                    keep = 1;
                }
            }
            // one scan for both: children (bits 0-12), kept (13-23); a chunk of BLK <= 1024
            // nodes sums to <= 4096 / 1024, so no field carries into the next.  The expandable
            // count needs only its total: a wave sum and one LDS atomic per wave
            static_assert(BLK <= 1024, "scan packing assumes <= 1024 threads");
            int t;
            const int o = block_exclusive_scan<BLK>(nch | (keep << 13), s.tmp, t);
            if (i < size) {
                s.aux[i] = csize + (o & 0x1fff);
                s.aux2[i] = ksize + ((o >> 13) & 0x7ff);
            }
            const int wne = wave_sum(ne);
            if ((tid & 63) == 0 && wne) atomicAdd(nexp_sh, wne);
            csize += t & 0x1fff;
            ksize += (t >> 13) & 0x7ff;
        }
        const int nsize = csize + ksize;
        if (pass == 1) OCT_MARK(tm, 34);
        if (nsize > ncap) {  // cannot happen for ncap >= max(N + 3, 4 * nIni)
            if (tid == 0) *out_cnt = -1;
            return;
        }
        __syncthreads();
        const int nexp = *nexp_sh;
        for (int i = tid; i < size; i += BLK) {
            if ((int)s.cnt(cur)[i] >= 2) {
                int cp = s.aux[i];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int qn = s.qcount(cur, i, q);
                    if (!qn) continue;
                    const int np = csize - 1 - cp;
                    int cbx, cby;
                    child_box(s.box(cur)[i], s.boy(cur)[i], q, cbx, cby);
                    s.box(nxt)[np] = cbx;
                    s.boy(nxt)[np] = cby;
                    s.cnt(nxt)[np] = (IT)qn;
                    s.seq(nxt)[np] = seq_base + cp;
                    s.key(nxt)[np] = (IT)-1;  // a single-key child's key: set by that key below
                    s.qk[i * 4 + q] = (IT)np;
                    ++cp;
                }
            } else {
                const int np = csize + s.aux2[i];
                s.box(nxt)[np] = s.box(cur)[i];
                s.boy(nxt)[np] = s.boy(cur)[i];
                s.cnt(nxt)[np] = s.cnt(cur)[i];
                s.seq(nxt)[np] = s.seq(cur)[i];
                s.key(nxt)[np] = s.key(cur)[i];
            }
        }
        for (int i = tid; i < QW * nsize; i += BLK) s.qcb(nxt)[i] = 0u;
        __syncthreads();
        if (pass == 1) OCT_MARK(tm, 35);
        {
            const OctLds<IT> ss = s;
            oct_sweep_q<BLK>(K, NODE, nkeys, s.box(cur), s.boy(cur), [=](const int* k, const int* node, const int* q, const uint32_t* kk) {
                int np[kOctU], c[kOctU], nbx[kOctU], nby[kOctU];
#pragma unroll
                for (int u = 0; u < kOctU; ++u) np[u] = node[u] >= 0 ? (int)ss.qk[max(node[u], 0) * 4 + q[u]] : 0;
#pragma unroll
                for (int u = 0; u < kOctU; ++u) {
                    c[u] = (int)ss.cnt(nxt)[np[u]];
                    nbx[u] = ss.box(nxt)[np[u]];
                    nby[u] = ss.boy(nxt)[np[u]];
                }
#pragma unroll
                for (int u = 0; u < kOctU; ++u) {
                    if (node[u] < 0) continue;
                    if (c[u] >= 2) {
                        NODE[k[u]] = np[u];
                        ss.qinc(nxt, np[u], quadrant(nbx[u], nby[u], key_x(kk[u]), key_y(kk[u])));
                    } else {
                        NODE[k[u]] = -1;
                        ss.key(nxt)[np[u]] = (IT)k[u];
                    }
                }
            });
        }
        __syncthreads();
        cur = nxt;
        size = nsize;
        seq_base += csize;
        if (size >= N || size == prev) finished = true;
        else if (size + nexp * 3 > N) phase2 = true;
        OCT_MARK(tm, 4 + min(pass, 7));
        ++npass;
    }

    // ---- phase 2: divide the biggest nodes first until the budget is reached (675-736)
    for (int round = 0; round < 64 && !finished; ++round) {
        const int prev = size;
        const int nxt = cur ^ 1;
        // expandable nodes -> sort keys (size desc, seq desc); carries the list position
        if (tid == 0) { flag_sh[0] = 0; *rmin_sh = 0x7fffffff; }
        __syncthreads();
        if (round == 0) OCT_MARK(tm, 40);
        for (int i = tid; i < size; i += BLK)
            if ((int)s.cnt(cur)[i] >= 2) {
                const int slot = atomicAdd(&flag_sh[0], 1);
                s.s64[slot] = ((unsigned long long)(unsigned)s.cnt(cur)[i] << 40) |
                              ((unsigned long long)(unsigned)s.seq(cur)[i] << 14) | (unsigned)i;
            }
        __syncthreads();
        if (round == 0) OCT_MARK(tm, 41);
        const int m = flag_sh[0];
        int P = 1;
        while (P < m) P <<= 1;
        if (P <= 64) {  // one wave sorts in registers: no barrier per step
            // (measured against one-wave rank sorts over v_readlane broadcasts or LDS broadcast
            // reads: 5.0 K vs 5.9 K / 7.2 K shader cycles at the level-0 tree's ~60 nodes)
            if (tid < 64) {
                unsigned long long v = tid < m ? s.s64[tid] : 0ull;
                for (int k = 2; k <= P; k <<= 1)  // bitonic sort, descending
                    for (int j = k >> 1; j > 0; j >>= 1) {
                        const unsigned lo = __shfl_xor((unsigned)v, j, 64);
                        const unsigned hi = __shfl_xor((unsigned)(v >> 32), j, 64);
                        const unsigned long long y = ((unsigned long long)hi << 32) | lo;
                        // the lower index of a pair keeps the larger key on descending runs
                        const bool keep_max = ((tid & j) == 0) == ((tid & k) == 0);
                        v = keep_max ? (v > y ? v : y) : (v < y ? v : y);
                    }
                if (tid < P) s.s64[tid] = v;
            }
            __syncthreads();
        } else {
            // rank sort (the keys are distinct: seq is unique): an entry's rank is the number of
            // larger keys; every thread scans all m keys (LDS broadcast reads), two barriers
            // instead of a bitonic network's log2(P)(log2(P)+1)/2.  The next list's quadrant
            // buffer (>= 8 NC bytes, 8-byte aligned, cleared below) holds the sorted copy.
            // (8 broadcast reads in flight per step, two keys per ds_read_b128: the rolled loop
            // waited on each read — 13.5 K cycles at the 1080p level-0 tree's ~300 nodes)
            unsigned long long* srt = reinterpret_cast<unsigned long long*>(s.qcb(nxt));
            const ulonglong2* s2 = reinterpret_cast<const ulonglong2*>(s.s64);
            const int m8 = m & ~7;
            for (int j = tid; j < m; j += BLK) {
                const unsigned long long v = s.s64[j];
                int rank = 0;
                for (int i = 0; i < m8; i += 8) {
                    ulonglong2 w[4];
#pragma unroll
                    for (int u = 0; u < 4; ++u) w[u] = s2[(i >> 1) + u];
#pragma unroll
                    for (int u = 0; u < 4; ++u) rank += (w[u].x > v) + (w[u].y > v);
                }
                for (int i = m8; i < m; ++i) rank += s.s64[i] > v;
                srt[rank] = v;
            }
            __syncthreads();
            for (int j = tid; j < m; j += BLK) s.s64[j] = srt[j];
            __syncthreads();
        }
        if (round == 0) OCT_MARK(tm, 44);
        // cut: first j in sorted order with size + sum_{<=j}(nch-1) >= N (else all m)
        {
            int run = 0;
            for (int base = 0; base < m; base += BLK) {
                const int j = base + tid;
                int delta = 0;
                if (j < m) {
                    const int i = (int)(s.s64[j] & 0x3fff);
                    for (int q = 0; q < 4; ++q) delta += s.qcount(cur, i, q) > 0;
                    delta -= 1;
                }
                int t;
                const int ex = block_exclusive_scan<BLK>(delta, s.tmp, t);
                if (j < m && size + run + ex + delta >= N) atomicMin(rmin_sh, j);
                run += t;
            }
            __syncthreads();
        }
        const int r = min(*rmin_sh, m - 1);
        if (round == 0) OCT_MARK(tm, 45);
        // processed flags + children offsets (processing order), kept offsets (list order)
        for (int i = tid; i < size; i += BLK) s.aux2[i] = 0;
        __syncthreads();
        if (round == 0) OCT_MARK(tm, 46);
        int csize = 0;
        for (int base = 0; base <= r; base += BLK) {
            const int j = base + tid;
            int nch = 0, i = -1;
            if (j <= r) {
                i = (int)(s.s64[j] & 0x3fff);
                for (int q = 0; q < 4; ++q) nch += s.qcount(cur, i, q) > 0;
            }
            int t;
            const int o = block_exclusive_scan<BLK>(nch, s.tmp, t);
            if (j <= r) {
                s.aux[i] = csize + o;
                s.aux2[i] = 1;
            }
            csize += t;
        }
        __syncthreads();
        if (round == 0) OCT_MARK(tm, 47);
        int ksize = 0;
        for (int base = 0; base < size; base += BLK) {
            const int i = base + tid;
            const int keep = i < size && !s.aux2[i];
            int t;
            const int o = block_exclusive_scan<BLK>(keep, s.tmp, t);
            if (keep) s.aux2[i] = -(1 + ksize + o);  // kept: encoded new offset
            ksize += t;
        }
        const int nsize = csize + ksize;
        if (round == 0) OCT_MARK(tm, 48);
        if (nsize > ncap) {
            if (tid == 0) *out_cnt = -1;
            return;
        }
        __syncthreads();
        for (int i = tid; i < size; i += BLK) {
            if (s.aux2[i] > 0) {  // processed: children
                int cp = s.aux[i];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int qn = s.qcount(cur, i, q);
                    if (!qn) continue;
                    const int np = csize - 1 - cp;
                    int cbx, cby;
                    child_box(s.box(cur)[i], s.boy(cur)[i], q, cbx, cby);
                    s.box(nxt)[np] = cbx;
                    s.boy(nxt)[np] = cby;
                    s.cnt(nxt)[np] = (IT)qn;
                    s.seq(nxt)[np] = seq_base + cp;
                    s.key(nxt)[np] = (IT)-1;  // a single-key child's key: set by that key below
                    s.qk[i * 4 + q] = (IT)np;
                    ++cp;
                }
            } else {
                const int np = csize + (-s.aux2[i] - 1);
                s.box(nxt)[np] = s.box(cur)[i];
                s.boy(nxt)[np] = s.boy(cur)[i];
                s.cnt(nxt)[np] = s.cnt(cur)[i];
                s.seq(nxt)[np] = s.seq(cur)[i];
                s.key(nxt)[np] = s.key(cur)[i];
                s.aux[i] = np;
            }
        }
        for (int i = tid; i < QW * nsize; i += BLK) s.qcb(nxt)[i] = 0u;
        __syncthreads();
        if (round == 0) OCT_MARK(tm, 49);
        {
            const OctLds<IT> ss = s;
            oct_sweep_q<BLK>(K, NODE, nkeys, s.box(cur), s.boy(cur), [=](const int* k, const int* node, const int* q, const uint32_t* kk) {
                int a2[kOctU], ca[kOctU], cq[kOctU], np[kOctU], c[kOctU], nbx[kOctU], nby[kOctU];
#pragma unroll
                for (int u = 0; u < kOctU; ++u) {
                    const int nd = max(node[u], 0);
                    a2[u] = ss.aux2[nd];
                    ca[u] = ss.aux[nd];
                    cq[u] = (int)ss.qk[nd * 4 + q[u]];
                }
#pragma unroll
                for (int u = 0; u < kOctU; ++u) np[u] = node[u] < 0 ? 0 : a2[u] > 0 ? cq[u] : ca[u];
#pragma unroll
                for (int u = 0; u < kOctU; ++u) {
                    c[u] = (int)ss.cnt(nxt)[np[u]];
                    nbx[u] = ss.box(nxt)[np[u]];
                    nby[u] = ss.boy(nxt)[np[u]];
                }
#pragma unroll
                for (int u = 0; u < kOctU; ++u) {
                    if (node[u] < 0) continue;
                    if (c[u] >= 2) {
                        NODE[k[u]] = np[u];
                        ss.qinc(nxt, np[u], quadrant(nbx[u], nby[u], key_x(kk[u]), key_y(kk[u])));
                    } else {  // alone in a new child (kept nodes hold >= 2 live keys)
                        NODE[k[u]] = -1;
                        ss.key(nxt)[np[u]] = (IT)k[u];
                    }
                }
            });
        }
        __syncthreads();
        cur = nxt;
        size = nsize;
        seq_base += csize;
        if (size >= N || size == prev) finished = true;
        OCT_MARK(tm, 12 + min(round, 17));
        ++nround;
    }

    // ---- retain the best key per node (740-759), emit in list order
    for (int i = tid; i < size; i += BLK) s.s64[i] = 0ull;
    // describe's processing order (a.oct_ord): the level's keypoints by 32-row band, counted in
    // the node boxes' words (dead from here on; >= 24 * nc >= 480 bytes)
    uint16_t* ord = a.oct_ord ? a.oct_ord + (out - a.oct_out) : nullptr;
    int* ybin = s.lists;
    if (ord)
        for (int i = tid; i < kOctBands; i += BLK) ybin[i] = 0;
    __syncthreads();
    OCT_MARK(tm, 52);
    {
        unsigned long long* best = s.s64;
        oct_sweep<BLK>(K, NODE, nkeys, [=](int k, uint32_t kk, int node) {
            atomicMax(&best[node], ((unsigned long long)key_score(kk) << 32) | (0xffffffffu - (unsigned)k));
        });
    }
    __syncthreads();
    OCT_MARK(tm, 53);
    for (int i = tid; i < size; i += BLK) {
        const int k = (int)s.cnt(cur)[i] == 1 ? (int)s.key(cur)[i]
                                          : (int)(0xffffffffu - (unsigned)(s.s64[i] & 0xffffffffu));
        const uint32_t kk = K[k];
        out[i] = pack_key(key_x(kk) + kMinBorder, key_y(kk) + kMinBorder, key_score(kk));
        if (ord) {  // band and rank in it (any order inside a band: only the sweep order changes)
            const int yb = min((int)key_y(kk) >> 5, kOctBands - 1);
            s.s64[i] = ((unsigned long long)yb << 16) | (unsigned)atomicAdd(&ybin[yb], 1);
        }
    }
    if (ord) {
        __syncthreads();
        int t;
        const int ex = block_exclusive_scan<BLK>(tid < kOctBands ? ybin[tid] : 0, s.tmp, t);
        if (tid < kOctBands) ybin[tid] = ex;
        __syncthreads();
        for (int i = tid; i < size; i += BLK) {
            const unsigned long long v = s.s64[i];
            ord[ybin[(int)(v >> 16)] + (int)(v & 0xffffu)] = (uint16_t)i;
        }
    }
    if (tid == 0) *out_cnt = size;
#ifdef ORBFE_OCT_TIMING
    if (tid == 0 && tm) tm[30] = npass | (nround << 8) | ((long long)nkeys << 16);
#endif
    OCT_MARK(tm, 31);
}

template <int BLK>
__global__ __launch_bounds__(BLK) void octree_kernel(OctArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds_raw[];
    // level-major block order: every frame's level-0 tree (the longest) is dispatched first,
    // the small levels fill the remaining slots
    const int level = blockIdx.y, f = blockIdx.x;
    const LevelGeo& L = a.geo.lv[level];
    const int NC = a.ncap_max;
    const int tid = threadIdx.x;
    // carve: sort keys | tmp | scalars | the path's region (oct_lds_bytes)
    unsigned long long* s64 = reinterpret_cast<unsigned long long*>(lds_raw);
    int* tmp = reinterpret_cast<int*>(s64 + a.sort_cap);
    int* scal = tmp + 16;  // block scans: <= 16 waves
    unsigned char* region = reinterpret_cast<unsigned char*>(scal + 16);
    auto carve = [&](auto& s, unsigned char* p) {
        using IT = std::remove_pointer_t<decltype(s.qk)>;
        s.s64 = s64;
        s.tmp = tmp;
        s.scal = scal;
        s.nc = NC;
        s.lists = reinterpret_cast<int*>(p);
        p += 6 * 4 * (size_t)NC;
        s.qc = reinterpret_cast<uint32_t*>(p);  // 8-byte aligned: the rank sort's u64 copy
        p += 2 * (size_t)std::remove_reference_t<decltype(s)>::kQcWords * 4 * NC;
        s.ilists = reinterpret_cast<IT*>(p);
        p += 4 * sizeof(IT) * (size_t)NC;
        s.qk = reinterpret_cast<IT*>(p);
        p += 4 * sizeof(IT) * (size_t)NC;
        using AT = typename std::remove_reference_t<decltype(s)>::AT;
        s.aux = reinterpret_cast<AT*>(p);
        s.aux2 = s.aux + NC;
    };
    uint32_t* out = a.oct_out + f * a.geo.out_total + L.out_off;
    int* out_cnt = a.oct_cnt + f * a.geo.nlevels + level;
    long long* tm = nullptr;
#ifdef ORBFE_OCT_TIMING
    if (f < 256) tm = g_oct_t + (f * 16 + level) * 64;
#endif
    OCT_MARK(tm, 0);

    // ---- 1. this level's key count (summed by the FAST kernel; reset for the next call)
    if (tid == 0) scal[0] = a.level_keys[f * kMaxLevels + level];
    __syncthreads();
    const int total = scal[0];
    if (tid == 0) a.level_keys[f * kMaxLevels + level] = 0;
    if (total == 0 || L.nini < 1) {
        if (tid == 0) *out_cnt = 0;
        OCT_MARK(tm, 31);
        return;
    }
    OCT_MARK(tm, 1);
    // ---- 2. compact the cell outputs into original key order (LDS when they fit).  A thread
    // takes a cell of each of two 256-cell chunks: their counts and slots in one global round
    // trip, the first 8 keys of both cells in a second (their addresses do not depend on the
    // scans, which run meanwhile), then the stores at the scanned offsets; cells with more than
    // 8 keys copy the rest in a loop.
    const bool in_lds = total <= a.lds_keys;
    uint32_t* lkeys = reinterpret_cast<uint32_t*>(region);  // LDS form: keys, node positions
    short* lnode = reinterpret_cast<short*>(lkeys + a.lds_keys);
    uint32_t* K = in_lds ? lkeys : a.keys + f * a.geo.key_total + L.key_off;
    const uint32_t* src = a.cell_keys + f * a.cell_cap_total;
    int nkeys = 0;
    for (int base = L.cell_begin; base < L.cell_end; base += 2 * BLK) {
        int n[2];
        long long slot[2];
        // (every load unconditional, at clamped indices inside the cell's own keys: a load under
        // a branch made the compiler wait for each one before the next, 10 round trips)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int c = base + j * BLK + tid;
            const int cc = min(c, L.cell_end - 1);
            const int nn = a.cell_cnt[f * a.ncells + cc];
            slot[j] = a.cells[cc].slot;
            n[j] = c < L.cell_end ? nn : 0;
        }
        uint32_t v[2][8];
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int i = 0; i < 8; ++i) v[j][i] = src[slot[j] + min(i, max(n[j] - 1, 0))];
        int t0, t1;
        const int o0 = nkeys + block_exclusive_scan<BLK>(n[0], tmp, t0);
        const int o1 = nkeys + t0 + block_exclusive_scan<BLK>(n[1], tmp, t1);
        const int off[2] = {o0, o1};
        // (uniform branch: a store through the selected pointer would be a flat store)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            if (in_lds) {
#pragma unroll
                for (int i = 0; i < 8; ++i)
                    if (i < n[j]) lkeys[off[j] + i] = v[j][i];
            } else {
#pragma unroll
                for (int i = 0; i < 8; ++i)
                    if (i < n[j]) K[off[j] + i] = v[j][i];
            }
            for (int i0 = 8; i0 < n[j]; i0 += 8) {
                uint32_t w[8];
#pragma unroll
                for (int i = 0; i < 8; ++i)
                    if (i0 + i < n[j]) w[i] = src[slot[j] + i0 + i];
                if (in_lds) {
#pragma unroll
                    for (int i = 0; i < 8; ++i)
                        if (i0 + i < n[j]) lkeys[off[j] + i0 + i] = w[i];
                } else {
#pragma unroll
                    for (int i = 0; i < 8; ++i)
                        if (i0 + i < n[j]) K[off[j] + i0 + i] = w[i];
                }
            }
        }
        nkeys += t0 + t1;
    }
    __syncthreads();
    OCT_MARK(tm, 2);
    if (in_lds) {
        OctLds<uint16_t> s;
        carve(s, reinterpret_cast<unsigned char*>(lnode + a.lds_keys));
        octree_level<BLK>(a, s, L, lkeys, lnode, nkeys, out, out_cnt, tm);
    } else {  // more keys than LDS holds: the same passes over global arrays
        OctLds<int> s;
        carve(s, region);
        int* node = reinterpret_cast<int*>(a.act) + (f * a.geo.key_total + L.key_off);
        octree_level<BLK>(a, s, L, K, node, nkeys, out, out_cnt, tm);
    }
}

// ---------------------------------------------------------------------------------------------
template __global__ void octree_kernel<kOctBlock>(OctArgs);
template __global__ void octree_kernel<kOctBlockSmall>(OctArgs);

// ---------------------------------------------------------------------------------------------
// K4 — GaussianBlur(7x7, sigma 2, REFLECT_101), integer path (App. A.2): row pass R = sum k_i I
// (<= 65535, exact in u16), column pass (sum k_j R + 2^15) >> 16 saturated; x86 mode rounds the
// SIMD body half to even (H6).  Both passes are banded integer GEMMs on the i8 matrix cores:
//   row pass     R (32 rows x 32 cols)  = (I - 128) . T + 128 * 257     (v_mfma_i32_32x32x32_i8)
//   column pass  O^T (32 x 32) = (R^T split into hi / lo bytes, each - 128) . V^T, two MFMAs,
//                the hi result shifted by 8 into the lo MFMA's C input, + 0x8000 rounding,
// where T[k][x] = tap(k - 3 - x) and V[y][r] = tap(r - 3 - y) are constant fragments (taps as
// i8, |tap| <= 55), and every sum is exact in i32.  A wave's tile is 26 output rows x 24 output
// columns: its 32 R rows (y - 3 .. y + 28) are one M-tile, its 30 input columns fit one K
// block.  The row pass's accumulator tile has its column on the lane and its rows in the
// registers, so it is the column pass's A operand (R^T: rows = columns x) after a byte split,
// with no lane movement — the column pass's K order is the accumulator's register order, and
// V's fragment follows it.  Memory stays row-contiguous: a workgroup (4 waves, 4 tiles side by
// side: 96 output columns) stages each 32-row input band in LDS with 112-byte row loads (all
// bands' loads issued up front), and writes its 26 x 96 output
// band to LDS and then to the level with 16-byte row stores — per-lane row-strided accesses
// (one row per lane) would make the texture addresser the bound.  A chunk that leaves the
// level loads the row's first / last 16 bytes and v_perm rebuilds the reflected bytes; levels
// narrower than 16 px gather them one by one.
constexpr int kBlurTileW = 24, kBlurTileH = 26, kBlurChunk = 8;
constexpr int kBlurGroupW = 4 * kBlurTileW;   // output columns per workgroup
constexpr int kBlurInQ = 7;                   // 16-byte input chunks per row: X0 - 3 .. X0 + 108
constexpr int kBlurInP = 104;                 // LDS input row (columns X0 - 3 .. X0 + 100 are
                                              // read; 26 dwords: 2-way bank aliasing at most)
constexpr int kBlurOutP = 100;                // LDS output row (25 dwords: conflict-free)
typedef int i32x4b __attribute__((ext_vector_type(4)));
typedef int i32x16b __attribute__((ext_vector_type(16)));
template <bool kX86>
__global__ __launch_bounds__(256) void blur_mfma_kernel(BlurArgs a) {
    __shared__ __attribute__((aligned(16))) uint8_t in_lds[2][32 * kBlurInP];
    __shared__ __attribute__((aligned(16))) uint8_t out_lds[kBlurTileH * kBlurOutP];
    int it, f;
    xcd_block(it, f);
    const uint32_t item = a.items[it];
    const int lv = (int)(item & 15u), gx = (int)((item >> 4) & 0x1ffu), ty0 = (int)((item >> 13) & 0x1ffu),
              nt = (int)(item >> 22);
    const LevelPtr sp = a.src[lv], dp = a.dst[lv];
    const int w = a.w[lv], h = a.h[lv], xb = a.simd_xb[lv];
    const uint8_t* src = sp.base + f * sp.fpitch;
    uint8_t* dst = const_cast<uint8_t*>(dp.base) + f * dp.fpitch;
    const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63, col = lane & 31, hh = lane >> 5;
    const int X0 = gx * kBlurGroupW;
    // constant B fragments (blur_frags, built on the host): T (row pass, K = input column
    // X - 3 + k) and V^T (column pass, K = the row pass's accumulator order)
    const uint4 tq = a.frags[lane], vq = a.frags[64 + lane];
    const i32x4b Tf = i32x4b{(int)tq.x, (int)tq.y, (int)tq.z, (int)tq.w};
    const i32x4b Vf = i32x4b{(int)vq.x, (int)vq.y, (int)vq.z, (int)vq.w};
    // Rows and columns past h + 2 / w + 2 feed only outputs outside the level: clamped there,
    // one reflection suffices (levels of >= 5 px; smaller ones take the general loop)
    auto refl = [](int p, int len) {
        p = min(p, len + 2);
        return len >= 5 ? reflect101_1(p, len) : reflect101(p, len);
    };
    // band loader: thread -> (input row lr, 16-byte chunk lc) of the band's 32 x 112 bytes
    const int lr = tid / kBlurInQ, lc = tid - lr * kBlurInQ;
    const int lx = X0 - 3 + 16 * lc;
    const bool ledge = lx < 0 || lx + 15 >= w;
    // a chunk that leaves the row (level >= 16 px wide) loads the row's first or last 16 bytes
    // instead: every reflected column it needs lies there, and v_perm pairs with per-lane
    // selectors rebuild it (chunk byte k <- loaded byte of column refl(lx + k))
    const bool tiny = w < 16;
    const int ls = lx < 0 ? 0 : (lx + 15 >= w ? w - 16 : lx);
    uint32_t selA[4] = {0u, 0u, 0u, 0u}, selB[4] = {0u, 0u, 0u, 0u};
    if (ledge && !tiny) {
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const int b = refl(lx + k, w) - ls;  // in [0, 16)
            selA[k >> 2] |= (uint32_t)(b < 8 ? b : 0x0c) << (8 * (k & 3));
            selB[k >> 2] |= (uint32_t)(b >= 8 ? b - 8 : 0x0c) << (8 * (k & 3));
        }
    }
    auto load_band = [&](int t) -> uint4 {
        if (lr >= 32) return make_uint4(0u, 0u, 0u, 0u);
        const uint8_t* row = src + (long long)refl((ty0 + t) * kBlurTileH - 3 + lr, h) * sp.pitch;
        if (tiny) {  // levels narrower than 16 px: byte by byte
            uint32_t bb[4] = {0u, 0u, 0u, 0u};
#pragma unroll
            for (int k = 0; k < 16; ++k)
                bb[k >> 2] |= (uint32_t)row[refl(lx + k, w)] << (8 * (k & 3));
            return make_uint4(bb[0], bb[1], bb[2], bb[3]);
        }
        uint4 v = load16_a1(row + ls);
        if (ledge) {
            uint32_t e[4];
#pragma unroll
            for (int k = 0; k < 4; ++k)
                e[k] = __builtin_amdgcn_perm(v.y, v.x, selA[k]) | __builtin_amdgcn_perm(v.w, v.z, selB[k]);
            v = make_uint4(e[0], e[1], e[2], e[3]);
        }
        return v;
    };
    const i32x16b zero = {};
    constexpr uint32_t kRound = kX86 ? 0x7fffu : 0x8000u;
    // hi pass: sum V (Rh - 128) = Dh - 128 * 257; the lo pass's C input restores both offsets
    constexpr uint32_t kC2 = 128u * 257u * 256u + 128u * 257u + kRound;
    // every band's loads are issued up front: a band's compute is far shorter than a global
    // round trip, so one band of prefetch leaves the workgroup waiting on each load
    uint4 pre[kBlurChunk];
#pragma unroll
    for (int t = 0; t < kBlurChunk; ++t)
        if (t < nt) pre[t] = load_band(t);
#pragma unroll
    for (int t = 0; t < kBlurChunk; ++t) {
        if (t >= nt) break;
        uint8_t* inb = in_lds[t & 1];
        if (lr < 32) {  // two 8-byte writes (rows are 8-byte aligned); chunk 6 keeps its first half
            uint2* q = reinterpret_cast<uint2*>(inb + lr * kBlurInP + 16 * lc);
            q[0] = make_uint2(pre[t].x, pre[t].y);
            if (lc < kBlurInQ - 1) q[1] = make_uint2(pre[t].z, pre[t].w);
        }
        __syncthreads();
        // A fragment: R row `col`, input columns X - 3 + 16 hh .. + 15, X = X0 + 24 wv
        const uint8_t* ap = inb + col * kBlurInP + kBlurTileW * wv + 16 * hh;  // 8-byte aligned
        const uint2 a0 = *reinterpret_cast<const uint2*>(ap), a1 = *reinterpret_cast<const uint2*>(ap + 8);
        const i32x4b av = i32x4b{(int)(a0.x ^ 0x80808080u), (int)(a0.y ^ 0x80808080u),
                                 (int)(a1.x ^ 0x80808080u), (int)(a1.y ^ 0x80808080u)};
        // R - 128 * 257 (the sum of T's column is 257 for the 24 output columns)
        const i32x16b R0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(av, Tf, zero, 0, 0, 0);
        i32x4b rlo, rhi;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint32_t e0 = (uint32_t)R0[4 * q] + 128u * 257u, e1 = (uint32_t)R0[4 * q + 1] + 128u * 257u,
                           e2 = (uint32_t)R0[4 * q + 2] + 128u * 257u, e3 = (uint32_t)R0[4 * q + 3] + 128u * 257u;
            rlo[q] = (int)((__builtin_amdgcn_perm(e1, e0, 0x0c0c0400u) |
                            __builtin_amdgcn_perm(e3, e2, 0x04000c0cu)) ^ 0x80808080u);
            rhi[q] = (int)((__builtin_amdgcn_perm(e1, e0, 0x0c0c0501u) |
                            __builtin_amdgcn_perm(e3, e2, 0x05010c0cu)) ^ 0x80808080u);
        }
        const i32x16b Dh = __builtin_amdgcn_mfma_i32_32x32x32_i8(rhi, Vf, zero, 0, 0, 0);
        i32x16b c2;
#pragma unroll
        for (int e = 0; e < 16; ++e) c2[e] = (int)(((uint32_t)Dh[e] << 8) + kC2);
        const i32x16b O = __builtin_amdgcn_mfma_i32_32x32x32_i8(rlo, Vf, c2, 0, 0, 0);
        // O^T: output row `col` of the band, columns 24 wv + 8 g + 4 hh + i in registers 4 g + i
        if (col < kBlurTileH) {
#pragma unroll
            for (int g = 0; g < 3; ++g) {
                const int xo = kBlurTileW * wv + 8 * g + 4 * hh;
                uint32_t s4[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    uint32_t sm = (uint32_t)O[4 * g + i];
                    if constexpr (kX86) sm += blur_round_bit(sm, X0 + xo + i < xb);
                    s4[i] = min(sm, 0xffffffu);  // byte 2 = min(sum >> 16, 255)
                }
                *reinterpret_cast<uint32_t*>(out_lds + col * kBlurOutP + xo) =
                    __builtin_amdgcn_perm(s4[1], s4[0], 0x0c0c0602u) | __builtin_amdgcn_perm(s4[3], s4[2], 0x06020c0cu);
            }
        }
        __syncthreads();
        // the band's 26 output rows x 96 columns, 16 bytes per thread
        if (tid < kBlurTileH * (kBlurGroupW / 16)) {
            const int r = tid / (kBlurGroupW / 16), c = tid - r * (kBlurGroupW / 16);
            const int yo = (ty0 + t) * kBlurTileH + r, xo = X0 + 16 * c;
            if (yo < h && xo < w) {
                const uint32_t* op = reinterpret_cast<const uint32_t*>(out_lds + r * kBlurOutP + 16 * c);
                const uint4 o = make_uint4(op[0], op[1], op[2], op[3]);
                uint8_t* d = dst + (long long)yo * dp.pitch + xo;
                if (xo + 16 <= w) {
                    *reinterpret_cast<uint4*>(d) = o;  // blurred slab rows: 64-B aligned, X0 % 16 == 0
                } else {
                    const uint32_t ow[4] = {o.x, o.y, o.z, o.w};
                    for (int i = 0; i < 16 && xo + i < w; ++i) d[i] = (uint8_t)(ow[i >> 2] >> (8 * (i & 3)));
                }
            }
        }
    }
}
template __global__ void blur_mfma_kernel<false>(BlurArgs);
template __global__ void blur_mfma_kernel<true>(BlurArgs);

// Host: blur_mfma_kernel's work list — per level, per 96-column group of four 24-px tiles,
// runs of up to kBlurChunk 26-row bands.  Item bits: 0-3 level, 4-12 column group, 13-21 first
// band, 22-31 band count.
void blur_items(const Geo& geo, std::vector<uint32_t>& s) {
    s.clear();
    for (int l = 0; l < geo.nlevels; ++l) {
        const int ntx = (geo.lv[l].w + kBlurGroupW - 1) / kBlurGroupW;
        const int nty = (geo.lv[l].h + kBlurTileH - 1) / kBlurTileH;
        for (int tx = 0; tx < ntx; ++tx)
            for (int ty = 0; ty < nty; ty += kBlurChunk)
                s.push_back((uint32_t)l | ((uint32_t)tx << 4) | ((uint32_t)ty << 13) |
                            ((uint32_t)std::min(kBlurChunk, nty - ty) << 22));
    }
}

// Host: blur_mfma_kernel's constant B fragments, lane l = col + 32 hh, byte j of its 16:
// [0, 64)  T[k = 16 hh + j][x = col]  = tap(k - 3 - x)          (row pass)
// [64,128) V^T[slot 16 hh + j][y = col] = tap(rho - 3 - y), rho = (j & 3) + 8 (j >> 2) + 4 hh
//          (the row pass's accumulator row held in register j of lane half hh)
// [128, 512): describe's window blur (v_mfma_i32_16x16x64_i8), lane l = n + 16 g, byte j:
// [128 + 64 s, ...) s < 3: H_s[k = raw column 16 g + j][window column 16 s + n]
//                          = tap(16 g + j - 16 s - n - 4)   (raw column = window column + 4)
// [320 + 64 u, ...) u < 3: V_u[window row 16 u + n][k = R row 16 t + 4 g + i], j = 4 t + i
//                          = tap(16 t + 4 g + i - 16 u - n - 3) for t < 3, 0 for j >= 12
//                          (R row = window row + 3; the R rows are the row pass's accumulator
//                          rows held in register i of tile t, in that K order)
void blur_frags(const int taps[4], uint8_t out[512 * 16]) {
    auto tap = [&](int d) { return d < -3 || d > 3 ? 0 : taps[3 - (d < 0 ? -d : d)]; };
    for (int l = 0; l < 64; ++l) {
        const int col = l & 31, hh = l >> 5;
        for (int j = 0; j < 16; ++j) {
            out[16 * l + j] = (uint8_t)tap(16 * hh + j - 3 - col);
            const int rho = (j & 3) + 8 * (j >> 2) + 4 * hh;
            out[16 * (64 + l) + j] = (uint8_t)tap(rho - 3 - col);
        }
    }
    for (int l = 0; l < 64; ++l) {
        const int n = l & 15, g = l >> 4;
        for (int q = 0; q < 3; ++q)
            for (int j = 0; j < 16; ++j) {
                const int t = j >> 2, i = j & 3;
                out[16 * (kDescFragOff + 64 * q + l) + j] = (uint8_t)tap(16 * g + j - 16 * q - n - 4);
                out[16 * (kDescFragOff + 192 + 64 * q + l) + j] =
                    (uint8_t)(t < 3 ? tap(16 * t + 4 * g + i - 16 * q - n - 3) : 0);
            }
    }
}

// ---------------------------------------------------------------------------------------------
// K5 — IC angle (76-103) on the unblurred level, rBRIEF (107-146) on the blurred level and
// the keypoint scaled to level 0 (1098-1104).  A wave owns kDescGroup consecutive oct-tree
// output slots of one frame:
//   1. per keypoint, the whole wave sums the 31 x 31 disc: lane = (row v, half) loads 16
//      pixels with one 16-byte load and weighs them with v_dot4_u32_u8 against per-lane
//      constant byte masks: m10 = sum (u + 16) I - 16 sum I, m01 = v sum I (integers, exact);
//   2. lane j computes keypoint j's fastAtan2 and its double-precision cos / sin once, so the
//      trig costs one wave instruction stream per group instead of one per keypoint;
//   3. per keypoint, lane k evaluates the rotated pattern pairs k + 64 r (pattern held packed
//      in 4 registers across the group) and 4 ballots make the 256-bit descriptor.
constexpr int kDescBlock = kDescBlockSize;
#ifndef ORBFE_DESC_SKIP
#define ORBFE_DESC_SKIP 0  // attribution experiments only (wrong descriptors): 1 blur passes,
#endif                     // 2 IC, 4 samples, 8 window loads, 16 trig
constexpr int kDescSkip = ORBFE_DESC_SKIP;
// ORBFE_DESC_PIPE: the blur passes' LDS reads issued ahead of their arithmetic (1 row pass,
// 2 column pass).  Measured no faster: 72 -> 85-93 VGPRs, 7 -> 5 waves per SIMD, describe
// 0.2813 (off) / 0.2878 / 0.2915 / 0.283 ms (profiles/r03/experiments/describe_pipe.json)
#ifndef ORBFE_DESC_PIPE
#define ORBFE_DESC_PIPE 0
#endif
constexpr bool kDescPipe = (ORBFE_DESC_PIPE & 1) != 0;
constexpr bool kDescPipeCol = (ORBFE_DESC_PIPE & 2) != 0;
// ORBFE_DESC_FRAG_LDS: the matrix-core blur's constant fragments read from LDS at each use
// instead of held in registers (1 H, 2 V at each use, 4 V once per N-tile).  With
// ORBFE_DESC_WAVES (the register budget: waves per SIMD) the default pair measured best:
// describe 0.2572 ms (in registers, 90 VGPRs, 5 waves) -> 0.2446 (both from LDS, 72 VGPRs,
// 7 waves); 8 waves spill (profiles/r03/experiments/describe_mfma.json)
#ifndef ORBFE_DESC_FRAG_OPAQUE
#define ORBFE_DESC_FRAG_OPAQUE 2
#endif
#ifndef ORBFE_DESC_FRAG_LDS
#define ORBFE_DESC_FRAG_LDS 3
#endif
constexpr int kFragLds = ORBFE_DESC_FRAG_LDS;
#ifndef ORBFE_DESC_LATE_STORE
#define ORBFE_DESC_LATE_STORE 1  // descriptor words stored once per wave, after the keypoint loop
#endif
constexpr bool kDescLateStore = ORBFE_DESC_LATE_STORE != 0;
#ifndef ORBFE_DESC_WAVES
#define ORBFE_DESC_WAVES 6
#endif
#ifndef ORBFE_DESC_WAVES_B
#define ORBFE_DESC_WAVES_B 5  // the small-batch groups (spill at 6)
#endif
#ifndef ORBFE_DESC_WAVES_X86
#define ORBFE_DESC_WAVES_X86 6  // the x86 reading (4 dwords of scratch at 6)
#endif
// ORBFE_DESC_PAT_LDS: the pattern pairs read as floats from LDS per keypoint (one b128 per 64
// pairs) instead of widened from packed bytes held in registers (four v_cvt per 64 pairs)
// ORBFE_DESC_IC_T: the IC moments of 4 keypoints reduced together (10 lane exchanges) instead
// of 8 separate wave reductions
#ifndef ORBFE_DESC_IC_T
#define ORBFE_DESC_IC_T 1
#endif
constexpr bool kIcT = ORBFE_DESC_IC_T != 0;
#ifndef ORBFE_DESC_PAT_LDS
#define ORBFE_DESC_PAT_LDS 1
#endif
constexpr bool kPatLds = ORBFE_DESC_PAT_LDS != 0;
constexpr int kDescGroupSmall = 2;  // small batches (single-frame latency): 4x the waves
// the group's slot -> level lookup assumes a group spans at most two levels, which holds while
// a group is no larger than the smallest per-level slot capacity (ncap >= 20)
static_assert(kDescGroupSize <= 20 && kDescGroupSmall <= 20,
              "describe groups larger than the minimum per-level ncap (20) can span 3 levels");
constexpr int kDescWinR = 18;                        // rotated pattern radius bound (< 18.5)
constexpr int kDescWinRows = 2 * kDescWinR + 1;      // 37
constexpr int kDescWinP = 48;                        // bytes per window row (3 x 16)
constexpr int kDescWinBytes = kDescWinRows * kDescWinP;
constexpr int kMwP = 40;            // kWinMfma window: bytes per column (window rows 0..39)
typedef float float2v __attribute__((ext_vector_type(2)));
// kWin (window source): kWinPre — the levels were blurred by K4 (a.blur); the wave copies each
// keypoint's 37-row blurred window straight into LDS instead of blurring a raw window.
// kWinValu — the raw window is staged in LDS and blurred by v_dot4 / v_dot2 passes (levels in
// pre_mask read blurred windows).  kWinMfma — the raw window goes from its global loads
// straight into i8 MFMA A fragments and both passes run on the matrix cores (below).
template <int kDescGroup, bool kX86, int kWin>
__global__ __launch_bounds__(kDescBlock, kWin == kWinMfma ? (kDescGroup < 8 ? ORBFE_DESC_WAVES_B : kX86 ? ORBFE_DESC_WAVES_X86 : ORBFE_DESC_WAVES) : 1) void describe_kernel(DescArgs a) {
    constexpr bool kPre = kWin == kWinPre, kMfma = kWin == kWinMfma;
    constexpr bool kLate = kDescLateStore && kMfma;
    int bx, f;
    xcd_block(bx, f);
    const int lane = threadIdx.x & 63;
    const int* cnt = a.oct_cnt + f * a.nlevels;
    // The wave's start is a chain of dependent loads (level key counts -> slot order -> key);
    // the counts, the blur fragments and the pattern pairs for LDS are all loaded first, and the
    // LDS stores and the barrier wait until the slot mapping below has issued its loads.
    // (loads without branches, so that no wait lands inside a branch right behind them)
    const int cq_ld = cnt[min(lane, a.nlevels - 1)];
    static_assert(kDescBlock == 256, "one fragment / pattern entry per thread (+128)");
    uint4 fr0 = make_uint4(0u, 0u, 0u, 0u), fr1 = fr0;
    int patw_lds = 0;
    if constexpr (kMfma && kFragLds != 0) {
        fr0 = a.frags[threadIdx.x];
        fr1 = a.frags[256 + (threadIdx.x & 127)];
    }
    if constexpr (kPatLds) patw_lds = reinterpret_cast<const int*>(c_pattern)[threadIdx.x];
    const int cq_raw = lane < a.nlevels ? cq_ld : 0;
    if (bx == 0 && threadIdx.x < 64) {
        const int n = wave_sum(max(cq_raw, 0));
        if (threadIdx.x == 0)
            a.n_out[f] = n;  // the true count: entries past kps_cap are not written (truncation
                             // is visible to the caller as n_out > kps_cap)
    }
    typedef int i32x4m __attribute__((ext_vector_type(4)));
    __shared__ uint4 frag_lds[kMfma && kFragLds ? 384 : 1];
    // kPatLds: the pattern pairs as floats, pat_lds[q][lane] = pair lane + 64 q (x1, y1, x2, y2)
    __shared__ float4 pat_lds[kPatLds ? 256 : 1];
    // the frame's waves: wave wv takes slots wv * G .. wv * G + G - 1 (grouped), or with
    // a.wave_stride = W (the waves of a frame) slots wv, wv + W, wv + 2 W, ... (strided): then at
    // any moment the frame's waves work on one run of W consecutive oct-tree slots — one level,
    // clustered by the node list's quadrant order — so the 128-byte lines their windows share
    // are fetched while they are still in the XCD's L2 (1080p: the frames in flight per XCD
    // overflow it otherwise)
    const int wv = bx * (kDescBlock / 64) + (threadIdx.x >> 6);
    const int stride = a.wave_stride;
    const int s0 = stride ? wv : wv * kDescGroup;

    // lane j < kDescGroup: slot s0 + j (grouped) or s0 + j W (strided) -> level, key, output
    // index.  The level key counts are one load (lane q holds level q's) and their exclusive
    // prefix a wave scan, so a wave's start is one global round trip, not a chain of dependent
    // loads.  Grouped, the group's slots lie in the level of s0 or the next one (every level
    // has >= 20 slots); strided, each lane finds its level.
    const int cq = max(cq_raw, 0);
    const int pre = wave_inclusive_sum(cq) - cq;
    int my_l = 0, my_key = 0, my_o = 0;
    bool valid = false;
    if (stride) {
        const int slot = min(s0 + min(lane, kDescGroup - 1) * stride, a.out_total - 1);
        int lv = 0, off = 0;
        for (int k = 1; k < a.nlevels; ++k) {
            const bool ge = slot >= a.out_off[k];
            lv = ge ? k : lv;
            off = ge ? a.out_off[k] : off;
        }
        const int c = __shfl(cq, lv, 64), pr = __shfl(pre, lv, 64);  // every lane active
        int idx = slot - off;
        if (lane < kDescGroup && s0 + lane * stride < a.out_total && idx < c) {
            // the oct-tree's band order: the frame's waves sweep each level top to bottom, so
            // the windows of one run share their lines (output order unchanged: my_o)
            if (a.oct_ord) idx = a.oct_ord[f * a.out_total + slot];
            if (idx + pr < a.kps_cap) {
                valid = true;
                my_l = lv;
                my_o = idx + pr;
                my_key = (int)a.oct_out[f * a.out_total + off + idx];
            }
        }
    }
    int l0 = 0;
    while (!stride && l0 + 1 < a.nlevels && s0 >= a.out_off[l0 + 1]) ++l0;  // uniform: scalar loads
    const int l1 = min(l0 + 1, a.nlevels - 1);
    const int off0 = a.out_off[l0], off1 = l1 > l0 ? a.out_off[l1] : a.out_total;
    const int c0 = __builtin_amdgcn_readlane(cq, l0), c1 = __builtin_amdgcn_readlane(cq, l1);
    const int p0 = __builtin_amdgcn_readlane(pre, l0), p1 = __builtin_amdgcn_readlane(pre, l1);
    if (!stride && lane < kDescGroup && s0 + lane < a.out_total) {
        const int slot = s0 + lane;
        const bool nx = slot >= off1;
        const int idx = slot - (nx ? off1 : off0);
        if (idx < (nx ? c1 : c0)) {
            const int o = idx + (nx ? p1 : p0);
            if (o < a.kps_cap) {
                valid = true;
                my_l = nx ? l1 : l0;
                my_o = o;
                my_key = (int)a.oct_out[f * a.out_total + slot];
            }
        }
    }
    if constexpr ((kMfma && kFragLds != 0) || kPatLds) {  // before any wave leaves
        if constexpr (kMfma && kFragLds != 0) {
            frag_lds[threadIdx.x] = fr0;
            frag_lds[256 + (threadIdx.x & 127)] = fr1;  // (threads 128.. rewrite 0..'s entries)
        }
        if constexpr (kPatLds) {
            const uint32_t w = (uint32_t)patw_lds;
            pat_lds[threadIdx.x] = make_float4((float)(int8_t)(w & 0xffu), (float)(int8_t)((w >> 8) & 0xffu),
                                               (float)(int8_t)((w >> 16) & 0xffu), (float)(int8_t)(w >> 24));
        }
        __syncthreads();
    }
    if (s0 >= a.out_total) return;
    const unsigned long long vmask = __ballot(valid);
    if (!vmask) return;

    // 3. rBRIEF: lane handles pairs lane + 64 q; bit k of byte i = pair 8 i + k (122-143).
    // Rotated pattern points stay within 13 sqrt 2 < 18.5 px of the keypoint, so keypoint j's
    // 37-row window of the blurred level (48 bytes per row from x0 = (x - 18) & ~3) is copied
    // into LDS with coalesced 16-byte loads (111 chunks, lanes c and c + 64), and the 512
    // scattered byte reads become ds_read_u8.  Windows are double-buffered per wave: the
    // loads of keypoint j + 1 are in flight while keypoint j is sampled.
    //
    // A rotated point is (py, px) = (px sin + py cos, px cos - py sin), each product and the
    // sum rounded separately as the reference writes it (v_pk_mul_f32 / v_pk_add_f32 do both
    // coordinates with the same IEEE roundings; px * -sin == -(px * sin)).  cvRound is the
    // magic-number add (|v| < 2^22, round-to-nearest-even): bits(v + 1.5 * 2^23) =
    // 0x4b400000 + rne(v); v_mul_u32_u24 takes its low 24 bits, 0x400000 + rne(v), so one
    // per-keypoint constant turns the pair into the window index (18 + ry) * 48 + cx + rx.
    //
    // The window is blurred here (GaussianBlur 7x7 sigma 2 REFLECT_101, ORBextractor.cc:1088-1089;
    // K4 does not run on the extraction path): window rows y-18..y+18 x cols x0..x0+47 need raw
    // rows y-21..y+21 and cols x0-3..x0+42 (samples reach window cols 0..39).  The wave copies 43
    // raw rows x 3 chunks of 16 bytes from x0-4 into LDS (loads of the next keypoint in flight
    // during the current one) and blurs window cols 0..39 of all 37 rows; when a
    // sampled pixel's 7x7 support leaves the level, or a chunk would leave the row, the raw
    // window is assembled byte by byte with reflect101 indices instead.  Then K4's
    // integer passes: rows by v_dot4 into u16 row pairs, columns by v_dot2 + 2^15 >> 16.
    uint32_t my_kc = 0;
    int my_x0 = 0;
    if (valid) {
        const int x = key_x((uint32_t)my_key);
        const int x0 = (x - kDescWinR) & ~3;
        my_x0 = x0;
        // (kMfma: the window is stored column-major, column (x - x0) + rx at byte 40 (x - x0 + rx))
        my_kc = kMfma ? (uint32_t)(kDescWinR + (x - x0) * kMwP) - 0x400000u * kMwP - 0x4b400000u
                      : (uint32_t)(kDescWinR * kDescWinP + (x - x0)) - 0x400000u * kDescWinP - 0x4b400000u;
    }
    // Pattern pairs lane + 64 q as 4 packed int8 (x1, y1, x2, y2), widened to float per
    // keypoint: 4 VGPRs held across the loop instead of 16 (and the compiler's hoisted products
    // with them: 98 -> 70 VGPRs, 4 -> 7 waves per SIMD).
    int patw[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) patw[q] = reinterpret_cast<const int*>(c_pattern)[lane + 64 * q];
    const float2v MG = float2v{12582912.f, 12582912.f};
    constexpr int kRawRows = 2 * (kDescWinR + 3) + 2;  // 44 (43 used, one pad row for pairs)
    constexpr int kRawP = 48;                          // raw row: image cols [x0-4, x0+44)
    constexpr int kRawQ = kRawP / 16;                  // 16-byte chunks per raw row
    constexpr int kPairs = kRawRows / 2;               // 22 u16 row pairs
    // samples reach window cols (x - x0) +- 18 with x - x0 in [18, 21]: cols 0..39, 10 quads
    constexpr int kBlurQ = 10;
    // The raw window is dead once the row pass has read it and the blurred window is written
    // after that (same wave, LDS ops in order), so the two share one buffer.
    // kMfma: the blurred window's columns 0..39, rows 0..39 column-major (the tiles' rows 40..
    // and columns 40.. are not stored)
    constexpr int kRawWinBytes = kMfma ? kMwP * kMwP
                                : kPre ? kDescWinBytes
                                       : kRawRows * kRawP > kDescWinBytes ? kRawRows * kRawP : kDescWinBytes;
    __shared__ __attribute__((aligned(16))) uint8_t raw_all[kDescBlock / 64][kRawWinBytes];
    constexpr int kRowpP = 4 * kBlurQ;                 // u16 row-pair pitch: window cols 0..39
    __shared__ __attribute__((aligned(16))) uint32_t rowp_all[kDescBlock / 64][kPre || kMfma ? 4 : kPairs * kRowpP];
    uint8_t* raw = raw_all[threadIdx.x >> 6];
    uint32_t* rowp = rowp_all[threadIdx.x >> 6];
    uint8_t* wb = raw;
    const uint32_t KLO = (uint32_t)(a.taps[0] | (a.taps[1] << 8) | (a.taps[2] << 16) | (a.taps[3] << 24));
    const uint32_t KHI = (uint32_t)(a.taps[2] | (a.taps[1] << 8) | (a.taps[0] << 16));
    typedef unsigned short us2 __attribute__((ext_vector_type(2)));
    const unsigned short k0 = (unsigned short)a.taps[0], k1 = (unsigned short)a.taps[1],
                         k2 = (unsigned short)a.taps[2], k3 = (unsigned short)a.taps[3];
    const us2 T01 = us2{k0, k1}, T23 = us2{k2, k3}, T21 = us2{k2, k1}, T0L = us2{k0, 0},
              T0H = us2{0, k0}, T12 = us2{k1, k2}, T32 = us2{k3, k2}, T10 = us2{k1, k0};
    // raw chunk c = lane + 64 i (i < 3, c < 43 * 3): row c / 3, 16-byte part c % 3
    uint4 rv[3];
    auto load_raw = [&](int j) __attribute__((always_inline)) {
        const int kl = __builtin_amdgcn_readlane(my_l, j);
        const uint32_t kk = (uint32_t)__builtin_amdgcn_readlane(my_key, j);
        const int x = key_x(kk), y = key_y(kk), x0 = (x - kDescWinR) & ~3;
        const LevelPtr pp = a.pyr[kl];
        const int lw = a.w[kl], lh = a.h[kl];
        const uint8_t* fb = pp.base + f * pp.fpitch;
        const bool fast = x0 - 4 >= 0 && x0 + 44 <= pp.pitch && x - 21 >= 0 && x + 21 < lw &&
                          y - 21 >= 0 && y + 21 < lh;
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            const int c = lane + 64 * i, r = c / kRawQ, part = c - kRawQ * r;
            rv[i] = make_uint4(0u, 0u, 0u, 0u);
            if (r >= kRawRows - 1 || (kDescSkip & 8)) continue;
            if (fast) {
                rv[i] = load16_a4(fb + (long long)(y - 21 + r) * pp.pitch + x0 - 4 + 16 * part);
            } else {
                const uint8_t* row = fb + (long long)reflect101(y - 21 + r, lh) * pp.pitch;
                uint32_t bb[4] = {0u, 0u, 0u, 0u};
#pragma unroll
                for (int k = 0; k < 16; ++k)
                    bb[k >> 2] |= (uint32_t)row[reflect101(x0 - 4 + 16 * part + k, lw)] << (8 * (k & 3));
                rv[i] = make_uint4(bb[0], bb[1], bb[2], bb[3]);
            }
        }
    };
    // kPre: blurred window chunk c = lane + 64 i (i < 2, c < 37 * 3): window row c / 3, 16-byte
    // part c % 3, at LDS byte 16 c.  Keypoints lie >= 19 px inside their level, so rows
    // y - 18 .. y + 18 are level rows; the bytes of a row past the level width (< 16, never
    // sampled) stay inside the slab (the last row read is h - 2).
    auto load_win = [&](int j) __attribute__((always_inline)) {
        const int kl = __builtin_amdgcn_readlane(my_l, j);
        const uint32_t kk = (uint32_t)__builtin_amdgcn_readlane(my_key, j);
        const int x = key_x(kk), y = key_y(kk), x0 = (x - kDescWinR) & ~3;
        const LevelPtr bp = a.blur[kl];
        const uint8_t* fb = bp.base + f * bp.fpitch + (long long)(y - kDescWinR) * bp.pitch + x0;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int c = lane + 64 * i, r = c / 3, part = c - 3 * r;
            rv[i] = make_uint4(0u, 0u, 0u, 0u);
            if (r < kDescWinRows) rv[i] = load16_a4(fb + (long long)r * bp.pitch + 16 * part);
        }
    };
    // a keypoint of a level whose bit is set in pre_mask reads its blurred window (the level
    // was blurred by the pyramid kernels); the others blur a raw window here.  The choice is
    // wave-uniform per keypoint.
    // kMfma: A fragment t of the row pass = raw row 16 t + (lane & 15), raw columns 16 g .. 16 g
    // + 15 (g = lane >> 4 < 3; the g = 3 K slots meet zero weights for every sampled column,
    // rows 43.. feed only window rows >= 37): one 16-byte load per tile straight into registers
    // (staging them in LDS with global_load_lds instead measured no faster: describe 0.2488 vs
    // 0.2467 ms, profiles/r03/experiments/describe_mfma.json)
    auto load_frag_to = [&](int j, uint4 (&dst)[3]) __attribute__((always_inline)) {
        const int kl = __builtin_amdgcn_readlane(my_l, j);
        const uint32_t kk = (uint32_t)__builtin_amdgcn_readlane(my_key, j);
        const int x = key_x(kk), y = key_y(kk), x0 = (x - kDescWinR) & ~3;
        const LevelPtr pp = a.pyr[kl];
        const int lw = a.w[kl], lh = a.h[kl];
        const uint8_t* fb = pp.base + f * pp.fpitch;
        const bool fast = x0 - 4 >= 0 && x0 + 44 <= pp.pitch && x - 21 >= 0 && x + 21 < lw &&
                          y - 21 >= 0 && y + 21 < lh;
        const int g = lane >> 4;
#pragma unroll
        for (int t = 0; t < 3; ++t) {
            const int r = 16 * t + (lane & 15);
            dst[t] = make_uint4(0u, 0u, 0u, 0u);
            if (r >= kRawRows - 1 || g == 3 || (kDescSkip & 8)) continue;
            if (fast) {
                dst[t] = load16_a4(fb + (long long)(y - 21 + r) * pp.pitch + x0 - 4 + 16 * g);
            } else {
                // keypoints lie >= 19 px inside their level (>= 39 px wide and high), so the
                // window overshoots an edge by at most 2 rows / 6 columns: one reflection
                const uint8_t* row = fb + (long long)reflect101_1(y - 21 + r, lh) * pp.pitch;
                uint32_t bb[4] = {0u, 0u, 0u, 0u};
#pragma unroll
                for (int k = 0; k < 16; ++k)
                    bb[k >> 2] |= (uint32_t)row[reflect101_1(x0 - 4 + 16 * g + k, lw)] << (8 * (k & 3));
                dst[t] = make_uint4(bb[0], bb[1], bb[2], bb[3]);
            }
        }
    };
    auto load_frag = [&](int j) __attribute__((always_inline)) { load_frag_to(j, rv); };
    auto is_pre = [&](int j) __attribute__((always_inline)) {
        return kPre || (!kMfma && ((a.pre_mask >> __builtin_amdgcn_readlane(my_l, j)) & 1u) != 0u);
    };
    auto load_kp = [&](int j) __attribute__((always_inline)) {
        if constexpr (kMfma) {
            load_frag(j);
        } else if (is_pre(j)) {
            load_win(j);
            rv[2] = make_uint4(0u, 0u, 0u, 0u);
        } else {
            load_raw(j);
        }
    };
    // kMfma constants: the row pass's B fragments H_s (window columns 16 s ..) and the column
    // pass's A fragments V_u (window rows 16 u ..), built on the host (blur_frags)
    i32x4m Hf[3], Vf[3];
    if constexpr (kMfma) {
#pragma unroll
        for (int q = 0; q < 3; ++q) {
            const uint4 h = a.frags[64 * q + lane], v = a.frags[192 + 64 * q + lane];
            Hf[q] = i32x4m{(int)h.x, (int)h.y, (int)h.z, (int)h.w};
            Vf[q] = i32x4m{(int)v.x, (int)v.y, (int)v.z, (int)v.w};
        }
    }
    // (the LDS offset made opaque per use, so the reads are not hoisted back into registers)
    // ORBFE_DESC_FRAG_OPAQUE 2: one opaque base per keypoint (the reads free to move within it)
    int fbase = lane;
    auto frag = [&](int q, const i32x4m& held, bool from_lds) __attribute__((always_inline)) {
        if (!from_lds) return held;
        int o = 64 * q + fbase;
        if (ORBFE_DESC_FRAG_OPAQUE == 1) asm volatile("" : "+v"(o));
        const uint4 h = frag_lds[o];
        return i32x4m{(int)h.x, (int)h.y, (int)h.z, (int)h.w};
    };
    unsigned long long dacc = 0;
    load_kp(__ffsll((long long)vmask) - 1);
    // (the first window's loads are in flight during the IC moments and the trig)
    // 1. IC moments.  Lane (r = lane >> 1, hh = lane & 1): row v = r - 15, columns
    //    u = -15 + 16 hh .. +15 (u = 16 never lies in the disc).
    const int r = lane >> 1, hh = lane & 1, v = r - 15;
    const int av = v < 0 ? -v : v;
    const int ulim = r < 31 ? c_umax[min(av, 15)] : -1;
    uint32_t wu[4], w1[4];
#pragma unroll
    for (int d = 0; d < 4; ++d) {
        uint32_t x = 0, y = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const int u = -15 + 16 * hh + 4 * d + b;
            const bool in = (u < 0 ? -u : u) <= ulim;
            x |= (in ? (uint32_t)(u + 16) : 0u) << (8 * b);
            y |= (in ? 1u : 0u) << (8 * b);
        }
        wu[d] = x;
        w1[d] = y;
    }
    // the 16-byte row loads of kIcBatch keypoints are issued before their first reduction
    // (4 at a time: 16 VGPRs of loads in flight, not 32)
    constexpr int kIcBatch = kDescGroup < 4 ? kDescGroup : 4;
    int M10 = 0, M01 = 0;
    // the rows of up to 8 keypoints in flight before the first reduction, every load
    // unconditional (an empty slot re-reads the first keypoint's rows, lanes past row 30 row
    // 15; both zeroed): a load under a branch made the compiler wait for it on the spot
    constexpr int kIcAhead = kDescGroup < 8 ? kDescGroup : 8;
    const int j_first = __ffsll((long long)vmask) - 1;
#pragma unroll
    for (int ja = 0; ja < kDescGroup; ja += kIcAhead) {
    uint4 pxa[kIcAhead];
#pragma unroll
    for (int jb = 0; jb < kIcAhead; ++jb) {
        const int j = ja + jb;
        const bool use = !(kDescSkip & 2) && ((vmask >> j) & 1);
        const int js = use ? j : j_first;
        const int kl = __builtin_amdgcn_readlane(my_l, js);
        const uint32_t kk = (uint32_t)__builtin_amdgcn_readlane(my_key, js);
        const LevelPtr pp = a.pyr[kl];
        const uint8_t* row = pp.base + f * pp.fpitch + (long long)(key_y(kk) + (r < 31 ? v : 0)) * pp.pitch +
                             key_x(kk) - 15 + 16 * hh;
        const uint4 q = load16_a1(row);
        pxa[jb] = use && r < 31 ? q : make_uint4(0u, 0u, 0u, 0u);
    }
#pragma unroll
    for (int j0 = ja; j0 < ja + kIcAhead; j0 += kIcBatch) {
        uint4 px[kIcBatch];
#pragma unroll
        for (int jb = 0; jb < kIcBatch; ++jb) px[jb] = pxa[j0 - ja + jb];
        int part[2 * kIcBatch];  // lane's partial (m10, m01) of each keypoint of the batch
#pragma unroll
        for (int jb = 0; jb < kIcBatch; ++jb) {
            const uint4 p4 = px[jb];
            const int su = (int)__builtin_amdgcn_udot4(p4.x, wu[0], __builtin_amdgcn_udot4(p4.y, wu[1],
                           __builtin_amdgcn_udot4(p4.z, wu[2], __builtin_amdgcn_udot4(p4.w, wu[3], 0u, false), false), false), false);
            const int s = (int)__builtin_amdgcn_udot4(p4.x, w1[0], __builtin_amdgcn_udot4(p4.y, w1[1],
                          __builtin_amdgcn_udot4(p4.z, w1[2], __builtin_amdgcn_udot4(p4.w, w1[3], 0u, false), false), false), false);
            part[2 * jb] = su - 16 * s;
            part[2 * jb + 1] = v * s;
        }
        if constexpr (kIcBatch == 4 && kIcT) {
            // the batch's 8 sums reduced together, halving the values at each exchange (xor 32,
            // 16, 8) and then summing the last one over 8 lanes: lane L ends with the total of
            // value 4 b5 + 2 b4 + b3 (bits of L), i.e. keypoint 2 b5 + b4, m01 if b3
            const bool h32 = (lane & 32) != 0, h16 = (lane & 16) != 0, h8 = (lane & 8) != 0;
            int a4[4], a2[2];
#pragma unroll
            for (int k = 0; k < 4; ++k)
                a4[k] = (h32 ? part[4 + k] : part[k]) + __shfl_xor(h32 ? part[k] : part[4 + k], 32);
#pragma unroll
            for (int k = 0; k < 2; ++k)
                a2[k] = (h16 ? a4[2 + k] : a4[k]) + __shfl_xor(h16 ? a4[k] : a4[2 + k], 16);
            int a1 = (h8 ? a2[1] : a2[0]) + __shfl_xor(h8 ? a2[0] : a2[1], 8);
            a1 += __shfl_xor(a1, 4);
            a1 += __shfl_xor(a1, 2);
            a1 += __shfl_xor(a1, 1);
            const int jb = (lane - j0) & 3;
            const int src = ((jb >> 1) << 5) | ((jb & 1) << 4);
            const int m10 = __shfl(a1, src), m01 = __shfl(a1, src + 8);
            if (lane >= j0 && lane < j0 + kIcBatch) {
                M10 = m10;
                M01 = m01;
            }
        } else {
#pragma unroll
            for (int jb = 0; jb < kIcBatch; ++jb) {
                const int m10 = wave_sum(part[2 * jb]), m01 = wave_sum(part[2 * jb + 1]);
                if (lane == j0 + jb) {
                    M10 = m10;
                    M01 = m01;
                }
            }
        }
    }
    }

    // 2. angle and its rotation, one keypoint per lane
    const float angle = fast_atan2((float)M01, (float)M10);
    const float ang = angle * (float)(3.14159265358979323846 / 180.f);
    float ca = 1.f, sa = 0.f;
    if (valid && !(kDescSkip & 16)) {
        // one shared argument reduction (OCML's sin and cos are the two halves of its sincos)
        double sd, cd;
        sincos((double)ang, &sd, &cd);
        ca = (float)cd;
        sa = (float)sd;
    }

    for (unsigned long long m = vmask; m; m &= m - 1) {
        const int j = __ffsll((long long)m) - 1;
        const bool pre_j = is_pre(j);
        if constexpr (kMfma) {
            // Both passes as banded i8 GEMMs (v_mfma_i32_16x16x64_i8), every sum exact in i32
            // (K4's integer passes, App. A.2; S = the taps' sum):
            //   row pass     R_t,s = (raw - 128) . H_s + 128 S + 2^15     (M = raw rows 16 t ..)
            //   column pass  O_u,s = (V_u . (lo - 128) + 128 * 257 S + rnd) + ((V_u . (hi - 128)) << 8)
            // where lo / hi are the bytes of R (<= 255 S < 2^16) and the + 2^15 makes byte 1 of
            // the accumulator hi ^ 0x80 already.  R_t,s has window column 16 s + (lane & 15) on
            // the lane and raw rows 16 t + 4 g + i in its registers, so packing its low / high
            // bytes gives the column pass's B operand with no lane movement (the K order V_u
            // follows).  O_u,s has the same shape: its 4 window rows of one column are one
            // dword of the column-major window.
            if (ORBFE_DESC_FRAG_OPAQUE == 2) {
                fbase = lane;
                asm volatile("" : "+v"(fbase));
            }
            const int S = 2 * (a.taps[0] + a.taps[1] + a.taps[2]) + a.taps[3];
            constexpr uint32_t kRndM = kX86 ? 0x7fffu : 0x8000u;
            const int ci = 128 * S + 0x8000;
            const uint32_t kC2 = 128u * 257u * (uint32_t)S + kRndM;
            const i32x4m Ci = i32x4m{ci, ci, ci, ci}, Z = i32x4m{0, 0, 0, 0};
            const i32x4m Kc = i32x4m{(int)kC2, (int)kC2, (int)kC2, (int)kC2};
            i32x4m A[3];
            const int n = lane & 15, g = lane >> 4;
#pragma unroll
            for (int t = 0; t < 3; ++t)
                A[t] = i32x4m{(int)(rv[t].x ^ 0x80808080u), (int)(rv[t].y ^ 0x80808080u),
                              (int)(rv[t].z ^ 0x80808080u), (int)(rv[t].w ^ 0x80808080u)};
            const unsigned long long rest = m & (m - 1);
            if (rest) load_kp(__ffsll((long long)rest) - 1);  // next keypoint's window in flight
            const int xs = kX86 ? (int)__builtin_amdgcn_readlane(my_x0, j) + (lane & 15) -
                                      a.simd_xb[(int)__builtin_amdgcn_readlane(my_l, j)]
                                : 0;
#pragma unroll
            for (int s = 0; s < 3; ++s) {
                i32x4m Blo, Bhi;
                const i32x4m Hs = frag(s, Hf[s], (kFragLds & 1) != 0);
#pragma unroll
                for (int t = 0; t < 3; ++t) {
                    const i32x4m R = __builtin_amdgcn_mfma_i32_16x16x64_i8(A[t], Hs, Ci, 0, 0, 0);
                    const uint32_t x01 = __builtin_amdgcn_perm((uint32_t)R[1], (uint32_t)R[0], 0x05010400u);
                    const uint32_t x23 = __builtin_amdgcn_perm((uint32_t)R[3], (uint32_t)R[2], 0x05010400u);
                    Blo[t] = (int)(__builtin_amdgcn_perm(x23, x01, 0x05040100u) ^ 0x80808080u);
                    Bhi[t] = (int)__builtin_amdgcn_perm(x23, x01, 0x07060302u);
                }
                Blo[3] = 0;
                Bhi[3] = 0;
                // x86: 1 where the column is in the SIMD body (round half to even), else 0
                const uint32_t em = xs + 16 * s < 0 ? 1u : 0u, nem = 1u - em;
                // the tile's columns all in the SIMD body (wave-uniform): then only a tie needs
                // the fix-up below
                const bool body = !kX86 || __ballot(em == 0u) == 0ull;
                i32x4m Vs[3];  // (kFragLds & 4: the three V fragments read once per N-tile)
                if constexpr ((kFragLds & 4) != 0) {
#pragma unroll
                    for (int u = 0; u < 3; ++u) Vs[u] = frag(3 + u, Vf[u], true);
                }
#pragma unroll
                for (int u = 0; u < 3; ++u) {
                    const i32x4m Vu = (kFragLds & 4) ? Vs[u] : frag(3 + u, Vf[u], (kFragLds & 2) != 0);
                    // the two planes' products are independent; the hi one shifted in after
                    const i32x4m Dh = __builtin_amdgcn_mfma_i32_16x16x64_i8(Vu, Bhi, Z, 0, 0, 0);
                    const i32x4m Dl = __builtin_amdgcn_mfma_i32_16x16x64_i8(Vu, Blo, Kc, 0, 0, 0);
                    uint32_t s4[4];
#pragma unroll
                    for (int i = 0; i < 4; ++i) s4[i] = ((uint32_t)Dh[i] << 8) + (uint32_t)Dl[i];
                    if constexpr (kX86) {
                        // x86 (kRndM = 0x7fff): + bit 16 of the sum in the SIMD body, + 1 past
                        // it.  The bit of sum + 0x7fff equals the true sum's bit 16 in the only
                        // case it matters (a tie, low half 0x8000 -> 0xffff), and adding it
                        // elsewhere changes no carry: v_bfe with width em (0 or 1), then one
                        // v_add3 — run only when some lane's sum is a tie or the tile reaches
                        // the scalar tail (one v_cmp_eq_u16 per sum instead of the two VALU of
                        // the fix-up; ties are ~1 in 65,536 sums)
                        if (!body || (tie_lanes(s4[0]) | tie_lanes(s4[1]) | tie_lanes(s4[2]) | tie_lanes(s4[3]))) {
#pragma unroll
                            for (int i = 0; i < 4; ++i) s4[i] = s4[i] + __builtin_amdgcn_ubfe(s4[i], 16u, em) + nem;
                        }
                    }
                    // min(sum >> 16, 255) of two sums at once (sum >> 16 <= 257 < 2^16)
                    const us2 sat = us2{255, 255};
                    const us2 h01 = __builtin_elementwise_min(__builtin_bit_cast(us2, __builtin_amdgcn_perm(s4[1], s4[0], 0x07060302u)), sat);
                    const us2 h23 = __builtin_elementwise_min(__builtin_bit_cast(us2, __builtin_amdgcn_perm(s4[3], s4[2], 0x07060302u)), sat);
                    if ((s < 2 || n < 8) && (u < 2 || g < 2))  // window columns / rows < 40
                        *reinterpret_cast<uint32_t*>(wb + (16 * s + n) * kMwP + 16 * u + 4 * g) =
                            __builtin_amdgcn_perm(__builtin_bit_cast(uint32_t, h23), __builtin_bit_cast(uint32_t, h01), 0x06040200u);
                }
            }
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        } else {
        if (pre_j) {
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const int c = lane + 64 * i;
                if (c < 3 * kDescWinRows) *reinterpret_cast<uint4*>(wb + 16 * c) = rv[i];
            }
        } else {
#pragma unroll
            for (int i = 0; i < 3; ++i) {
                const int c = lane + 64 * i;
                if (c / kRawQ < kRawRows - 1) *reinterpret_cast<uint4*>(raw + 16 * c) = rv[i];
            }
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        const unsigned long long rest = m & (m - 1);
        if (rest) load_kp(__ffsll((long long)rest) - 1);  // next keypoint's window in flight
        if (!kPre && !(kDescSkip & 1) && !pre_j) {
        // row pass: item (pair pr, quad q) -> window cols 4q..4q+3 of raw rows 2pr, 2pr+1.
        // Items it = lane + 64 i: (pr, q) advance by (6, 4) or, when q wraps, (7, -6), and the
        // raw offset with them (no division or multiply in the loop); (pr, q) sits at dword
        // 4 it of rowp (kRowpP = 4 kBlurQ).
        static_assert(64 % kBlurQ == 4 && 64 / kBlurQ == 6 && kRowpP == 4 * kBlurQ,
                      "blur stepping assumes 10 quads");
        {
            const int pr0 = lane / kBlurQ, q0 = lane - pr0 * kBlurQ;
            int q = q0;
            int ro = 2 * pr0 * kRawP + 4 * q0;  // byte offset of (row 2pr, quad q) in raw
            auto row_item = [&](const uint32_t (&w)[2][3], int it) {
                uint32_t hh[2][4];
#pragma unroll
                for (int e = 0; e < 2; ++e) {
#pragma unroll
                    for (int jj = 0; jj < 4; ++jj) {
                        const uint32_t lo = jj < 3 ? __builtin_amdgcn_alignbyte(w[e][1], w[e][0], jj + 1) : w[e][1];
                        const uint32_t hi = jj < 3 ? __builtin_amdgcn_alignbyte(w[e][2], w[e][1], jj + 1) : w[e][2];
                        hh[e][jj] = __builtin_amdgcn_udot4(hi, KHI, __builtin_amdgcn_udot4(lo, KLO, 0u, false), false);
                    }
                }
                // row 2pr in the low half, 2pr+1 in the high half (both < 2^16): one v_perm each
                *reinterpret_cast<uint4*>(rowp + 4 * it) =
                    make_uint4(__builtin_amdgcn_perm(hh[1][0], hh[0][0], 0x05040100u),
                               __builtin_amdgcn_perm(hh[1][1], hh[0][1], 0x05040100u),
                               __builtin_amdgcn_perm(hh[1][2], hh[0][2], 0x05040100u),
                               __builtin_amdgcn_perm(hh[1][3], hh[0][3], 0x05040100u));
            };
            if constexpr (kDescPipe) {
                // every item's six raw dwords are read before the first is used: one LDS round
                // trip for the pass instead of one per 64 items
                constexpr int kRowIt = (kPairs * kBlurQ + 63) / 64;  // 4
                uint32_t w[kRowIt][2][3];
#pragma unroll
                for (int u = 0; u < kRowIt; ++u) {
                    if (lane + 64 * u < kPairs * kBlurQ) {
#pragma unroll
                        for (int e = 0; e < 2; ++e) {
                            const uint32_t* row = reinterpret_cast<const uint32_t*>(raw + ro + e * kRawP);
                            w[u][e][0] = row[0];
                            w[u][e][1] = row[1];
                            w[u][e][2] = row[2];
                        }
                    }
                    const bool wrap = q >= kBlurQ - 4;
                    q += wrap ? 4 - kBlurQ : 4;
                    ro += wrap ? 7 * 2 * kRawP + 4 * (4 - kBlurQ) : 6 * 2 * kRawP + 16;
                }
#pragma unroll
                for (int u = 0; u < kRowIt; ++u)
                    if (lane + 64 * u < kPairs * kBlurQ) row_item(w[u], lane + 64 * u);
            } else {
                for (int it = lane; it < kPairs * kBlurQ; it += 64) {
                    uint32_t w[2][3];
#pragma unroll
                    for (int e = 0; e < 2; ++e) {
                        const uint32_t* row = reinterpret_cast<const uint32_t*>(raw + ro + e * kRawP);
                        w[e][0] = row[0];
                        w[e][1] = row[1];
                        w[e][2] = row[2];
                    }
                    row_item(w, it);
                    const bool wrap = q >= kBlurQ - 4;
                    q += wrap ? 4 - kBlurQ : 4;
                    ro += wrap ? 7 * 2 * kRawP + 4 * (4 - kBlurQ) : 6 * 2 * kRawP + 16;
                }
            }
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        // column pass: item (output rows 2jp, 2jp+1; quad q) from pairs jp..jp+3, stepped as
        // the row pass
        int cq = lane % kBlurQ;
        int wq = 2 * (lane / kBlurQ) * kDescWinP + 4 * cq;  // byte offset of (row 2jp, quad q)
        // x86 arithmetic: window quad cq is level columns x0 + 4 cq ..; x0 and simd_xb are
        // multiples of 4, so a quad is wholly SIMD body or tail
        const int xq = kX86 ? (int)__builtin_amdgcn_readlane(my_x0, j) - a.simd_xb[(int)__builtin_amdgcn_readlane(my_l, j)] : 0;
        // the sums carry 0x7fff (x86: + the half-to-even bit on the SIMD body) or 2^15
        constexpr uint32_t kRnd = kX86 ? 0x7fffu : 0x8000u;
        auto col_item = [&](const uint4 (&P4)[4], int cq_, int wq_) {
            const bool even = xq + 4 * cq_ < 0;
            uint32_t ev[4], od[4];
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const uint32_t p0 = (&P4[0].x)[c], p1 = (&P4[1].x)[c], p2 = (&P4[2].x)[c], p3 = (&P4[3].x)[c];
                uint32_t v = __builtin_amdgcn_udot2(__builtin_bit_cast(us2, p0), T01, kRnd, false);
                v = __builtin_amdgcn_udot2(__builtin_bit_cast(us2, p1), T23, v, false);
                v = __builtin_amdgcn_udot2(__builtin_bit_cast(us2, p2), T21, v, false);
                v = __builtin_amdgcn_udot2(__builtin_bit_cast(us2, p3), T0L, v, false);
                if constexpr (kX86) v += blur_round_bit(v, even);
                ev[c] = min(v, 0xffffffu);  // byte 2 = min(acc >> 16, 255)
                uint32_t u = __builtin_amdgcn_udot2(__builtin_bit_cast(us2, p0), T0H, kRnd, false);
                u = __builtin_amdgcn_udot2(__builtin_bit_cast(us2, p1), T12, u, false);
                u = __builtin_amdgcn_udot2(__builtin_bit_cast(us2, p2), T32, u, false);
                u = __builtin_amdgcn_udot2(__builtin_bit_cast(us2, p3), T10, u, false);
                if constexpr (kX86) u += blur_round_bit(u, even);
                od[c] = min(u, 0xffffffu);
            }
            *reinterpret_cast<uint32_t*>(wb + wq_) =
                __builtin_amdgcn_perm(ev[1], ev[0], 0x0c0c0602u) | __builtin_amdgcn_perm(ev[3], ev[2], 0x06020c0cu);
            if (wq_ < (kDescWinRows - 1) * kDescWinP)  // row 2jp + 1 exists: jp < 18
                *reinterpret_cast<uint32_t*>(wb + wq_ + kDescWinP) =
                    __builtin_amdgcn_perm(od[1], od[0], 0x0c0c0602u) | __builtin_amdgcn_perm(od[3], od[2], 0x06020c0cu);
        };
        constexpr int kColItems = ((kDescWinRows + 1) / 2) * kBlurQ;  // 190
        if constexpr (kDescPipeCol) {
            // two items' row pairs in flight: the next item's four b128 reads are issued before
            // the current item's arithmetic
            constexpr int kColIt = (kColItems + 63) / 64;  // 3
            int cqs[kColIt], wqs[kColIt];
#pragma unroll
            for (int u = 0; u < kColIt; ++u) {
                cqs[u] = cq;
                wqs[u] = wq;
                const bool wrap = cq >= kBlurQ - 4;
                cq += wrap ? 4 - kBlurQ : 4;
                wq += wrap ? 7 * 2 * kDescWinP + 4 * (4 - kBlurQ) : 6 * 2 * kDescWinP + 16;
            }
            uint4 Pc[4], Pn[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) Pc[i] = *reinterpret_cast<const uint4*>(rowp + 4 * lane + i * kRowpP);
#pragma unroll
            for (int u = 0; u < kColIt; ++u) {
                const int itn = lane + 64 * (u + 1);
                if (u + 1 < kColIt && itn < kColItems) {
#pragma unroll
                    for (int i = 0; i < 4; ++i) Pn[i] = *reinterpret_cast<const uint4*>(rowp + 4 * itn + i * kRowpP);
                }
                if (lane + 64 * u < kColItems) col_item(Pc, cqs[u], wqs[u]);
#pragma unroll
                for (int i = 0; i < 4; ++i) Pc[i] = Pn[i];
            }
        } else {
            for (int it = lane; it < kColItems; it += 64) {
                uint4 P4[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) P4[i] = *reinterpret_cast<const uint4*>(rowp + 4 * it + i * kRowpP);
                col_item(P4, cq, wq);
                const bool wrap = cq >= kBlurQ - 4;
                cq += wrap ? 4 - kBlurQ : 4;
                wq += wrap ? 7 * 2 * kDescWinP + 4 * (4 - kBlurQ) : 6 * 2 * kDescWinP + 16;
            }
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        }  // !kPre
        }  // !kMfma
        const float cj = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, ca), j));
        const float sj = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, sa), j));
        const uint32_t kc = (uint32_t)__builtin_amdgcn_readlane((int)my_kc, j);
        const float2v SC = float2v{sj, cj}, CSn = float2v{cj, -sj};
        int i0[4], i1[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            float pat[16];
            if constexpr (kPatLds) {
                const float4 p4 = pat_lds[64 * q + lane];
                pat[4 * q] = p4.x;
                pat[4 * q + 1] = p4.y;
                pat[4 * q + 2] = p4.z;
                pat[4 * q + 3] = p4.w;
            } else {
                asm volatile("" : "+v"(patw[q]));  // keeps the widening inside the loop
#pragma unroll
                for (int c = 0; c < 4; ++c)
                    pat[4 * q + c] = (float)(int)(int8_t)(uint8_t)((uint32_t)patw[q] >> (8 * c));
            }
            // x86 arithmetic (H4): x*b + y*a as a GCC -O3 build on an FMA host contracts
            // it, fma(x, b, y*a) and fma(x, a, -(y*b)) (oracle/variant_rot.cpp)
            float2v r0, r1;
            if constexpr (kX86) {
                r0 = __builtin_elementwise_fma(float2v{pat[4 * q], pat[4 * q]}, SC, pat[4 * q + 1] * CSn) + MG;
                r1 = __builtin_elementwise_fma(float2v{pat[4 * q + 2], pat[4 * q + 2]}, SC, pat[4 * q + 3] * CSn) + MG;
            } else {
                r0 = (pat[4 * q] * SC + pat[4 * q + 1] * CSn) + MG;
                r1 = (pat[4 * q + 2] * SC + pat[4 * q + 3] * CSn) + MG;
            }
            // (__builtin_bit_cast of an ext-vector element reads element 0 in this clang:
            // go through __float_as_uint on copied scalars)
            const float r0y = r0.x, r0x = r0.y, r1y = r1.x, r1x = r1.y;
            if constexpr (kDescSkip & 4) {
                i0[q] = (int)(__float_as_uint(r0y) ^ __float_as_uint(r1x));
                i1[q] = (int)(__float_as_uint(r1y) + kc);
            } else {
            if constexpr (kMfma) {  // column-major window
            i0[q] = wb[__umul24(__float_as_uint(r0x), (uint32_t)kMwP) + __float_as_uint(r0y) + kc];
            i1[q] = wb[__umul24(__float_as_uint(r1x), (uint32_t)kMwP) + __float_as_uint(r1y) + kc];
            } else {
            i0[q] = wb[__umul24(__float_as_uint(r0y), (uint32_t)kDescWinP) + __float_as_uint(r0x) + kc];
            i1[q] = wb[__umul24(__float_as_uint(r1y), (uint32_t)kDescWinP) + __float_as_uint(r1x) + kc];
            }
            }
        }
        unsigned long long words[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) words[q] = __ballot(i0[q] < i1[q]);
        if constexpr (kLate) {
            // lanes 4 j .. 4 j + 3 keep keypoint j's four words for one store after the loop
            // (no store in flight when the next window's loads are waited for)
            if ((lane >> 2) == j)
                dacc = (lane & 3) == 0 ? words[0] : (lane & 3) == 1 ? words[1] : (lane & 3) == 2 ? words[2] : words[3];
        } else {
            const long long outi = (long long)f * a.kps_cap + __builtin_amdgcn_readlane(my_o, j);
            if (lane < 4) {
                const unsigned long long wv = lane == 0 ? words[0] : lane == 1 ? words[1] : lane == 2 ? words[2] : words[3];
                reinterpret_cast<unsigned long long*>(a.desc + outi * 32)[lane] = wv;
            }
        }
        __builtin_amdgcn_wave_barrier();  // the window is rewritten for the next keypoint
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    }
    if constexpr (kLate) {
        const int kj = lane >> 2;
        const int o = __builtin_amdgcn_ds_bpermute(kj << 2, my_o);  // keypoint kj's output index
        if (kj < kDescGroup && ((vmask >> kj) & 1))
            reinterpret_cast<unsigned long long*>(a.desc + ((long long)f * a.kps_cap + o) * 32)[lane & 3] = dacc;
    }
    if (valid) {
        const uint32_t kk = (uint32_t)my_key;
        const int kl = my_l, x = key_x(kk), y = key_y(kk);
        orbfe_keypoint kp;
        const float sc = a.scale[kl];
        kp.x = kl ? (float)x * sc : (float)x;
        kp.y = kl ? (float)y * sc : (float)y;
        kp.size = a.size[kl];
        kp.angle = angle;
        kp.response = (float)key_score(kk);
        kp.octave = kl;
        kp.class_id = -1;
        a.kps[(long long)f * a.kps_cap + my_o] = kp;
    }
}

// =============================================================================================
// host side

namespace {
inline int cv_round_f(float v) { return (int)std::lrintf(v); }
inline short sat_short(float v) {
    int iv = cv_round_f(v);
    return (short)std::min(std::max(iv, -32768), 32767);
}
}  // namespace

int make_tables(const orbfe_params& p, HostTables& t) {
    if (p.nlevels < 1 || p.nlevels > kMaxLevels || p.nfeatures < 0 || !(p.scale_factor > 1.0f))
        return ORBFE_ERR_ARG;
    t.p = p;
    const double sd = (double)p.scale_factor;
    t.scale[0] = 1.0f;
    t.sigma2[0] = 1.0f;
    for (int i = 1; i < p.nlevels; ++i) {  // ORBextractor.cc:414-430
        t.scale[i] = (float)((double)t.scale[i - 1] * sd);
        t.sigma2[i] = t.scale[i] * t.scale[i];
    }
    for (int i = 0; i < p.nlevels; ++i) {
        t.inv[i] = 1.0f / t.scale[i];
        t.inv_sigma2[i] = 1.0f / t.sigma2[i];
    }
    const float factor = (float)(1.0 / sd);  // 434-445
    float per = (float)p.nfeatures * (1 - factor) / (1 - (float)std::pow((double)factor, (double)p.nlevels));
    int sum = 0;
    for (int l = 0; l < p.nlevels - 1; ++l) {
        t.nfeat[l] = cv_round_f(per);
        sum += t.nfeat[l];
        per *= factor;
    }
    t.nfeat[p.nlevels - 1] = std::max(p.nfeatures - sum, 0);
    const int vmax = (int)std::floor(kHalfPatchSize * std::sqrt(2.f) / 2 + 1);  // 453-468
    const int vmin = (int)std::ceil(kHalfPatchSize * std::sqrt(2.f) / 2);
    for (int v = 0; v <= vmax; ++v)
        t.umax[v] = (int)std::lrint(std::sqrt((double)kHalfPatchSize * kHalfPatchSize - v * v));
    for (int v = kHalfPatchSize, v0 = 0; v >= vmin; --v) {
        while (t.umax[v0] == t.umax[v0 + 1]) ++v0;
        t.umax[v] = v0;
        ++v0;
    }
    // getGaussianKernel(7, 2, CV_32F) * 256 rounded (App. A.2)
    float g[7];
    double gs = 0;
    for (int i = 0; i < 7; ++i) {
        const double x = i - 3.0;
        g[i] = (float)std::exp(-0.125 * x * x);
        gs += g[i];
    }
    gs = 1. / gs;
    for (int i = 0; i < 7; ++i) g[i] = (float)(g[i] * gs);
    for (int i = 0; i < 7; ++i) t.taps[i] = cv_round_f(g[i] * 256.f + 0.f);
    return ORBFE_OK;
}

// Plans every size-dependent table for a w x h input (cached per extractor).
int plan_geometry(const HostTables& t, int w, int h, Plan& g) {
    const int L = t.p.nlevels;
    g.w = w;
    g.h = h;
    g.geo.nlevels = L;
    long long slab = 0, keys = 0;
    int out = 0, ncap_max = 0;
    g.cells.clear();
    g.xtab.clear();
    g.ytab.clear();
    for (int l = 0; l < L; ++l) {
        LevelGeo& lv = g.geo.lv[l];
        lv.w = cv_round_f((float)w * t.inv[l]);
        lv.h = cv_round_f((float)h * t.inv[l]);
        if (lv.w < 4 || lv.h < 4) return ORBFE_ERR_UNSUPPORTED;
        lv.pitch = (lv.w + 63) & ~63;
        lv.off = slab;
        slab += (long long)lv.pitch * lv.h;
        slab = (slab + 255) & ~255ll;
        lv.scale = t.scale[l];
        lv.size = (float)(int)(31 * t.scale[l]);  // scaledPatchSize (836)
        lv.nfeat = t.nfeat[l];
        // FAST cells (772-806)
        const int maxbx = lv.w - kEdge + 3, maxby = lv.h - kEdge + 3;
        const float width = (float)(maxbx - kMinBorder), height = (float)(maxby - kMinBorder);
        const int ncols = (int)(width / kCellW), nrows = (int)(height / kCellW);
        lv.cell_begin = (int)g.cells.size();
        lv.key_off = keys;
        long long kcap = 0;
        if (ncols > 0 && nrows > 0) {
            const int wc = (int)std::ceil(width / ncols), hc = (int)std::ceil(height / nrows);
            for (int i = 0; i < nrows; ++i) {
                const int y0 = kMinBorder + i * hc;
                int y1 = y0 + hc + 6;
                if (y0 >= maxby - 3) continue;
                if (y1 > maxby) y1 = maxby;
                for (int j = 0; j < ncols; ++j) {
                    const int x0 = kMinBorder + j * wc;
                    int x1 = x0 + wc + 6;
                    if (x0 >= maxbx - 6) continue;
                    if (x1 > maxbx) x1 = maxbx;
                    CellDesc c;
                    c.level = l;
                    c.y0 = y0; c.y1 = y1; c.x0 = x0; c.x1 = x1;
                    if (y1 - y0 > kRoiMax || x1 - x0 > kRoiMax) return ORBFE_ERR_UNSUPPORTED;
                    const int dh = std::max(y1 - y0 - 6, 0), dw = std::max(x1 - x0 - 6, 0);
                    c.cap = ((dh + 1) / 2) * ((dw + 1) / 2);  // strict NMS: <= 1 per 2x2
                    c.slot = g.cell_cap_total;
                    g.cell_cap_total += c.cap;
                    kcap += c.cap;
                    g.cells.push_back(c);
                }
            }
        }
        lv.cell_end = (int)g.cells.size();
        lv.key_cap = (int)kcap;
        keys += kcap;
        // oct-tree (538-584)
        lv.bw = maxbx - kMinBorder;
        lv.bh = maxby - kMinBorder;
        if (kcap > 0) {
            lv.nini = (int)std::round((float)lv.bw / lv.bh);
            if (lv.nini < 1) return ORBFE_ERR_UNSUPPORTED;  // reference UB
            lv.hx = (float)lv.bw / lv.nini;
        } else {
            lv.nini = 0;
            lv.hx = 1.f;
        }
        // list bound: the first pass <= 4 nIni, later phase-1 passes <= N, phase 2 <= N + 2
        // (DESIGN.md "oct-tree"); the initial nodes index arrays of the same capacity
        lv.ncap = std::max({lv.nfeat + 4, 4 * lv.nini, 20});
        lv.out_off = out;
        out += lv.ncap;
        ncap_max = std::max(ncap_max, lv.ncap);
        // resize tables for level l from level l-1 (App. A.1)
        if (l > 0) {
            const LevelGeo& sv = g.geo.lv[l - 1];
            const int sw = sv.w, sh = sv.h, dw = lv.w, dh = lv.h;
            const double scale_x = 1. / ((double)dw / sw), scale_y = 1. / ((double)dh / sh);
            g.xoff[l] = (int)g.xtab.size();
            for (int dx = 0; dx < dw; ++dx) {
                float fx = (float)((dx + 0.5) * scale_x - 0.5);
                int sx = (int)std::floor(fx);
                fx -= sx;
                if (sx < 0) { fx = 0; sx = 0; }
                if (sx >= sw - 1) { fx = 0; sx = sw - 1; }
                const int a0 = sat_short((1.f - fx) * 2048), a1 = sat_short(fx * 2048);
                g.xtab.push_back(sx);
                g.xtab.push_back(std::min(sx + 1, sw - 1));
                g.xtab.push_back((a0 & 0xffff) | (a1 << 16));
            }
            {   // LDS footprint of a 128 x 32 resize tile of this level
                int need_rows = 0, need_w = 0;
                for (int oy = 0; oy < dh; oy += kRsTH) {
                    const int ey = std::min(oy + kRsTH, dh) - 1;
                    auto sy = [&](int dy) { return (int)std::floor((float)((dy + 0.5) * scale_y - 0.5)); };
                    const int r0 = std::min(std::max(sy(oy), 0), sh - 1), r1 = std::min(std::max(sy(ey) + 1, 0), sh - 1);
                    need_rows = std::max(need_rows, r1 - r0 + 1);
                }
                const size_t xb = g.xtab.size() - 3 * (size_t)dw;
                for (int ox = 0; ox < dw; ox += kRsTW) {
                    const int ex = std::min(ox + kRsTW, dw) - 1;
                    const int a0 = g.xtab[xb + 3 * ox] & ~3, a1 = g.xtab[xb + 3 * ex + 1];
                    // + 2 dwords: the table path reads 3 dwords from a group's first source dword
                    need_w = std::max(need_w, ((a1 - a0) >> 2) + 1 + 2);
                }
                g.rs_tiles_x[l] = (dw + kRsTW - 1) / kRsTW;
                g.rs_tiles[l] = g.rs_tiles_x[l] * ((dh + kRsTH - 1) / kRsTH);
                // 16-byte chunks: the widest tile's dwords rounded up to whole chunks
                g.rs_pitch[l] = 16 * ((need_w + 3) / 4);
                g.rs_lds[l] = (size_t)need_rows * g.rs_pitch[l];
                if (g.rs_lds[l] > 64 * 1024) return ORBFE_ERR_UNSUPPORTED;  // scale factors > ~3
            }
            g.yoff[l] = (int)g.ytab.size();
            for (int dy = 0; dy < dh; ++dy) {
                float fy = (float)((dy + 0.5) * scale_y - 0.5);
                int sy = (int)std::floor(fy);
                fy -= sy;
                const int b0 = sat_short((1.f - fy) * 2048), b1 = sat_short(fy * 2048);
                g.ytab.push_back(std::min(std::max(sy, 0), sh - 1));
                g.ytab.push_back(std::min(std::max(sy + 1, 0), sh - 1));
                g.ytab.push_back((b0 & 0xffff) | (b1 << 16));
            }
        }
    }
    if (w > 4096 || h > 4096) return ORBFE_ERR_UNSUPPORTED;
    {   // K1b: the longest run of top levels ts..L-1 (ts >= 2) whose two largest LDS images,
        // levels ts-1 and ts (rows padded to dwords), fit the tail kernel's LDS
        const int L = g.geo.nlevels;
        auto bytes = [&](int l) { return (size_t)g.geo.lv[l].h * (((size_t)g.geo.lv[l].w + 15) & ~(size_t)15); };
        g.tail_start = L;
        for (int ts = L - 1; ts >= 2; --ts) {
            if (bytes(ts - 1) + bytes(ts) > (size_t)kTailLds || g.geo.lv[ts].h > kTailRows) break;
            g.tail_start = ts;
        }
        if (L - g.tail_start < 2) g.tail_start = L;  // a single level gains nothing
    }
    {   // pyramid_kernel: column-group tables, then two band plans (batches >= kTailMinFrames:
        // the fewest bands whose LDS fits kPyrLdsCap; single frames / small batches: bands of
        // ~kPyrSmallRows level-0 rows, for more workgroups)
        const int L = g.geo.nlevels;
        g.ptab.clear();
        g.pyr_ok = L >= 2;
        for (int l = 1; l < L && g.pyr_ok; ++l) {
            g.gtab_off[l] = (int)(g.ptab.size() / 4);
            g.pyr_ok = pyramid_group_table(g.xtab, g.xoff[l], g.geo.lv[l].w, g.ptab);
        }
        for (int l = 0; l < L; ++l) g.pyr_lp[l] = ((g.geo.lv[l].w + 15) & ~15) + 16;
        double work = 0, own = 0;  // pixels computed by the bands vs the pyramid's
        for (int l = 1; l < L; ++l) own += (double)g.geo.lv[l].w * g.geo.lv[l].h;
        auto plan_bands = [&](int nb, std::vector<int>& bt, size_t& lds, int& bufb, int& ybuf, int& ymax) {
            bt.assign((size_t)nb * L * 4, 0);
            size_t A = 0, B = 0;
            work = 0;
            ymax = 1;
            for (int b = 0; b < nb; ++b) {
                auto R = [&](int l, int bb) { return (int)((long long)bb * g.geo.lv[l].h / nb); };
                int c0[kMaxLevels], c1[kMaxLevels];
                c0[L - 1] = R(L - 1, b);
                c1[L - 1] = R(L - 1, b + 1) - 1;
                for (int l = L - 1; l >= 1; --l) {
                    const int o0 = R(l - 1, b), o1 = R(l - 1, b + 1) - 1;
                    if (c1[l] >= c0[l]) {  // y tables are monotone: the sources of rows c0 .. c1
                        const int s0 = g.ytab[g.yoff[l] + 3 * c0[l]], s1 = g.ytab[g.yoff[l] + 3 * c1[l] + 1];
                        c0[l - 1] = o1 >= o0 ? std::min(o0, s0) : s0;
                        c1[l - 1] = o1 >= o0 ? std::max(o1, s1) : s1;
                    } else {
                        c0[l - 1] = o0;
                        c1[l - 1] = o1;
                    }
                }
                for (int l = 0; l < L; ++l) {
                    int* e = &bt[((size_t)b * L + l) * 4];
                    e[0] = c0[l];
                    e[1] = c1[l];
                    e[2] = R(l, b);
                    e[3] = R(l, b + 1);
                    const size_t n = (size_t)std::max(0, c1[l] - c0[l] + 1);
                    (l & 1 ? B : A) = std::max(l & 1 ? B : A, n * g.pyr_lp[l]);
                    if (l) ymax = std::max(ymax, (int)n);
                    if (l) work += (double)n * g.geo.lv[l].w;
                }
            }
            bufb = (int)((A + 15) & ~(size_t)15);
            ybuf = bufb + (int)((B + 15) & ~(size_t)15);
            lds = (size_t)ybuf + 2 * 3 * (size_t)ymax * sizeof(int);
        };
        const char* cap_env = std::getenv("ORBFE_PYR_LDS_KB");
        const size_t cap = (cap_env ? (size_t)std::atoi(cap_env) : (size_t)kPyrLdsCapKB) * 1024;
        std::vector<int> bt[2];
        const int h0 = g.geo.lv[0].h, htop = g.geo.lv[L - 1].h;
        int nb = 1;
        for (int which = 0; which < 2 && g.pyr_ok; ++which) {
            nb = which == 0 ? 1 : std::max(1, std::min(std::min(64, htop), h0 / kPyrSmallRows));
            for (;; ++nb) {
                plan_bands(nb, bt[which], g.pyr_lds[which], g.pyr_bufb[which], g.pyr_ybuf[which], g.pyr_ymax[which]);
                if (g.pyr_lds[which] <= cap) break;
                if (nb >= htop) { g.pyr_ok = false; break; }  // no band fits: per-level kernels
            }
            g.nbands[which] = nb;
            // thin bands recompute too many seam rows: at 1920x1080 the per-level kernels win
            // (c4: 1.11 vs 1.25-1.45 ms per step), at 640x480 the band kernel (0.135 vs 0.17)
            g.pyr_use[which] = g.pyr_ok && work <= own * (which == 0 ? kPyrMaxWork : kPyrMaxWorkSmall);
        }
        if (g.pyr_ok) {
            for (int which = 0; which < 2; ++which) {
                while (g.ptab.size() % 4) g.ptab.push_back(0u);
                g.band_off[which] = (int)(g.ptab.size() / 4);  // int4 units
                for (int v : bt[which]) g.ptab.push_back((uint32_t)v);
            }
        }
        // resize2_kernel plans: levels (l, l + 1) per launch, tiles of level l + 1.  Level l is
        // partitioned among the tiles by each tile's first source row / column (columns rounded
        // down to whole 4-column groups); a tile computes its own part plus what its level l + 1
        // rows and columns read.
        for (int l = 1; l + 1 < L && g.pyr_ok; ++l) {
            const int mw = g.geo.lv[l].w, mh = g.geo.lv[l].h;
            const int dw = g.geo.lv[l + 1].w, dh = g.geo.lv[l + 1].h;
            const int* xm = &g.xtab[g.xoff[l]];
            const int* ym = &g.ytab[g.yoff[l]];
            const int* xd = &g.xtab[g.xoff[l + 1]];
            const int* yd = &g.ytab[g.yoff[l + 1]];
            const int ntx = (dw + kRsTW - 1) / kRsTW, nty = (dh + kRsTH - 1) / kRsTH;
            std::vector<int> tt;
            tt.reserve((size_t)ntx * nty * 8);
            int arows = 0, awid = 0, brows = 0, bwid = 0, gmax = 0;
            for (int ty = 0; ty < nty; ++ty)
                for (int tx = 0; tx < ntx; ++tx) {
                    const int ox = tx * kRsTW, oy = ty * kRsTH;
                    const int ex = std::min(ox + kRsTW, dw) - 1, ey = std::min(oy + kRsTH, dh) - 1;
                    const int oy0 = ty ? yd[3 * oy] : 0, oy1 = ty + 1 < nty ? yd[3 * (oy + kRsTH)] : mh;
                    const int ox0 = tx ? (xd[3 * ox] & ~3) : 0;
                    const int ox1 = tx + 1 < ntx ? (xd[3 * (ox + kRsTW)] & ~3) : mw;
                    const int cy0 = std::min(yd[3 * oy], oy0), cy1 = std::max(yd[3 * ey + 1], oy1 - 1);
                    const int cx0 = std::min(xd[3 * ox] & ~3, ox0);
                    const int cx1 = std::min(mw - 1, std::max(xd[3 * std::min(ex | 3, dw - 1) + 1], ox1 - 1) | 3);
                    tt.insert(tt.end(), {cy0, cy1, cx0, cx1, oy0, oy1, ox0, ox1});
                    const int ay0 = ym[3 * cy0], ay1 = ym[3 * cy1 + 1];
                    const int ax0 = xm[3 * cx0] & ~3, ax1 = xm[3 * cx1 + 1];
                    arows = std::max(arows, ay1 - ay0 + 1);
                    awid = std::max(awid, ax1 - ax0 + 1);
                    brows = std::max(brows, cy1 - cy0 + 1);
                    bwid = std::max(bwid, cx1 - cx0 + 1);
                    gmax = std::max(gmax, ((cx1 - cx0) >> 2) + 1);
                }
            const int pa = ((awid + 15) & ~15) + 16, pb = ((bwid + 15) & ~15) + 16;
            const size_t bofs = ((size_t)arows * pa + 15) & ~(size_t)15;
            const size_t lds = bofs + (size_t)brows * pb;
            g.rs2_ok[l] = lds <= 64 * 1024 && gmax <= 256 && brows <= kR2Rows;
            if (!g.rs2_ok[l]) continue;
            g.rs2_tiles_x[l] = ntx;
            g.rs2_tiles[l] = ntx * nty;
            g.rs2_pa[l] = pa;
            g.rs2_pb[l] = pb;
            g.rs2_bofs[l] = (int)bofs;
            g.rs2_lds[l] = lds;
            while (g.ptab.size() % 4) g.ptab.push_back(0u);
            g.rs2_off[l] = (int)(g.ptab.size() / 4);
            for (int v : tt) g.ptab.push_back((uint32_t)v);
        }
    }
    int rmax = 7, cmax = 7;
    for (const CellDesc& c : g.cells) {
        rmax = std::max(rmax, c.y1 - c.y0);
        cmax = std::max(cmax, c.x1 - c.x0);
    }
    g.roi_rows = rmax;
    g.roi_pitch = (cmax + 3 + 15) & ~15;  // + alignment shift, 16-byte rows for b128 LDS writes
    // FAST survivor list: every candidate pixel up to kFastListCap, else flushed (fast_kernel)
    g.cand_max = std::min((rmax - 6) * (cmax - 6), kFastListCap);
    // ROI + zero-bordered score plane at the ROI pitch + candidate list of u16 ROI offsets
    if ((long long)rmax * g.roi_pitch >= 65536) return ORBFE_ERR_UNSUPPORTED;
    g.fast_lds = (size_t)rmax * g.roi_pitch + (((rmax - 4) * g.roi_pitch + 15) & ~15) +
                 2 * (size_t)g.cand_max + 16 + 128;  // + a trash slot per lane
    g.geo.key_total = keys;
    blur_items(g.geo, g.bitems);
    g.geo.out_total = out;
    g.slab = slab;
    g.ncap_max = ncap_max;
    // phase-2 sort keys: <= one per node (rank sort), 64 for the one-wave bitonic sort
    g.sort_cap = std::max(ncap_max, 64);
    // LDS-resident keys per level: ~9x the largest level budget covers the FAST lists of
    // textured frames (640x480 @1000: <= 1,900 keys per level of 2,048; 1080p @2000: <= 3,300
    // of 4,096), at most kOctLdsKeys; a level with more runs on global arrays.  At 640x480
    // @1000 the carve is 26.8 KB (six trees per CU; 33.9 KB and four before the u16 node
    // fields and the 10x key capacity)
    int nf_max = 0;
    for (int l = 0; l < L; ++l) nf_max = std::max(nf_max, g.geo.lv[l].nfeat);
    g.oct_keys = std::min(kOctLdsKeys, std::max(1024, (9 * nf_max + 63) & ~63));
    g.oct_lds = std::max(oct_lds_bytes(true, ncap_max, g.sort_cap, g.oct_keys),
                         oct_lds_bytes(false, ncap_max, g.sort_cap, g.oct_keys));
    return ORBFE_OK;
}

}  // namespace orbfe

#ifdef ORBFE_FAST_TIMING
extern "C" int orbfe_debug_fast_timing_reset() {  // device globals start uninitialised
    void* p = nullptr;
    if (hipGetSymbolAddress(&p, HIP_SYMBOL(orbfe::g_fast_t)) != hipSuccess) return -3;
    return hipMemset(p, 0, sizeof(orbfe::g_fast_t)) == hipSuccess ? 0 : -3;
}
extern "C" int orbfe_debug_fast_timing(long long* out, int n) {
    n = n < orbfe::kFtFrames * orbfe::kFtCells * 16 ? n : orbfe::kFtFrames * orbfe::kFtCells * 16;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(orbfe::g_fast_t), (size_t)n * sizeof(long long)) == hipSuccess ? 0 : -3;
}
#endif

#ifdef ORBFE_OCT_TIMING
extern "C" int orbfe_debug_oct_timing(long long* out, int n) {
    n = n < 256 * 16 * 64 ? n : 256 * 16 * 64;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(orbfe::g_oct_t), (size_t)n * sizeof(long long)) == hipSuccess ? 0 : -3;
}
#endif
