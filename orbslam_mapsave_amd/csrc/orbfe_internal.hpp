// orbfe_internal.hpp — structs shared by the extractor kernels and their host orchestration.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <vector>

#include "../../include/orbfe.h"

namespace orbfe {

constexpr int kMaxLevels = 16;

// FAST candidate / oct-tree key: x, y (12 bits each; level coords or coords relative to
// (16,16)) and the FAST score (8 bits).  Images are limited to 4096 x 4096.
__host__ __device__ __forceinline__ uint32_t pack_key(int x, int y, int s) {
    return ((uint32_t)y << 20) | ((uint32_t)x << 8) | (uint32_t)s;
}
__host__ __device__ __forceinline__ int key_x(uint32_t k) { return (int)((k >> 8) & 0xfff); }
__host__ __device__ __forceinline__ int key_y(uint32_t k) { return (int)(k >> 20); }
__host__ __device__ __forceinline__ int key_score(uint32_t k) { return (int)(k & 0xff); }

struct LevelGeo {
    int w, h, pitch;       // level size; row pitch inside the pyramid / blur slabs
    long long off;         // byte offset of the level inside a frame's slab
    int cell_begin, cell_end;
    int key_cap;           // sum of the level's cell capacities
    long long key_off;     // offset (keys) of the level inside a frame's key region
    int nfeat;             // mnFeaturesPerLevel[level]
    int nini;              // initial oct-tree nodes round(bw / bh) (542)
    float hx;              // (maxX - minX) / nIni (544)
    int bw, bh;            // maxBorderX - minBorderX, maxBorderY - minBorderY
    int ncap;              // oct-tree list capacity max(N + 4, 4 nIni + 4)
    int out_off;           // offset of the level inside a frame's oct-tree output
    float scale, size;     // mvScaleFactor[level], (int)(31 * scale)
};

struct Geo {
    int nlevels;
    long long key_total;   // keys per frame (all levels)
    int out_total;         // oct-tree output slots per frame (all levels)
    LevelGeo lv[kMaxLevels];
};

struct CellDesc {
    int level;
    int y0, y1, x0, x1;    // FAST ROI rows [y0,y1) cols [x0,x1) in level coords
    int cap;               // max keys the cell can emit
    long long slot;        // offset of the cell's keys inside a frame's cell-key region
};

struct LevelPtr {
    const uint8_t* base;   // frame 0, level origin
    long long fpitch;      // bytes between frames
    int pitch;             // bytes between rows
};

struct Level0Args {
    const uint8_t* src;    // caller frames (cn bytes per pixel)
    long long src_fpitch;
    int src_pitch, cn, c0, c2;   // channels; gray weights of channel 0 and 2 (RGB2Gray<uchar>)
    bool aligned;          // src rows 4-byte aligned: vector loads
    const uint8_t* mask;   // NULL or u8 plane per frame
    long long mask_fpitch;
    int mask_pitch;
    const int4* rects;     // NULL or per frame (x0, y0, x1, y1) zeroed rectangle
    uint8_t* dst;          // pyramid level 0
    long long dst_fpitch;
    int dst_pitch, w, h;
};

struct ResizeArgs {
    LevelPtr src, dst;
    int sw, sh, dw, dh;
    int tiles_x, lds_pitch;
    const int* xt;
    const int* yt;
    int simd_xb;           // x86 arithmetic: columns [0, simd_xb) use the SSE2 rounding (H5)
    const uint4* gtab;     // resize_kernel: the level's pyramid_kernel column-group table, or null
};

// resize2_kernel: levels l and l + 1 in one launch, tiles of level l + 1 (see the kernel)
struct Resize2Args {
    LevelPtr src, mid, dst;             // levels l - 1, l, l + 1
    int sw, mw, dw, dh;                 // widths of l - 1, l, l + 1; rows of l + 1
    int tiles_x;
    // per tile: {computed rows first, last, computed columns first, last (4-aligned start)} and
    // {own rows [y0, y1), own columns [x0, x1)} of level l
    const int4* tiles;
    const int* yt_m;                    // level l's y / x tables (rows / columns of l - 1)
    const int* xt_m;
    const int* yt_d;                    // level l + 1's (of level l)
    const int* xt_d;
    const uint4* gtab_m;                // column-group tables of levels l, l + 1
    const uint4* gtab_d;
    int pa, pb, bofs;                   // LDS: level l - 1 rows at 0 (pitch pa), level l at bofs (pb)
    int xb_m, xb_d;                     // x86 SIMD-body bounds of levels l, l + 1
};

struct PyrArgs {
    LevelPtr src;                  // level 0
    LevelPtr l0_copy;              // base != null: each band also writes its level-0 rows here
                                   // (src is then the caller's staging copy of the frame)
    LevelPtr dst[kMaxLevels];      // pyramid levels (index = level; 0 unused)
    int nlevels;
    int w[kMaxLevels];             // level widths
    int lp[kMaxLevels];            // LDS row pitch per level
    int buf_b, ybuf, ymax;         // LDS offsets: second level buffer, y-table rows (2 x ymax)
    const int4* bands;             // [band][level] {c0, c1, w0, w1}: rows computed / written
    const uint4* gtab[kMaxLevels]; // per level >= 1: 3 uint4 per column group
    const int* yt[kMaxLevels];     // per level >= 1: the resize y table
    int simd_xb[kMaxLevels];
};

struct ResizeTailArgs {
    LevelPtr src;                 // level ts-1
    int sh;                       // its rows
    int nt;                       // tail levels ts .. ts+nt-1
    int buf_b;                    // LDS offset of the second buffer
    int lp[kMaxLevels + 1];       // LDS row pitch of level ts-1+k (k = 0 .. nt)
    int dw[kMaxLevels], dh[kMaxLevels];
    const int* xt[kMaxLevels];
    const int* yt[kMaxLevels];
    LevelPtr dst[kMaxLevels];
    int simd_xb[kMaxLevels];      // per tail level, as ResizeArgs::simd_xb
};

struct FastArgs {
    const CellDesc* cells;
    int ncells;
    long long cell_cap_total;
    int ini_th, min_th;
    int roi_pitch, roi_rows, cand_max;  // dynamic-LDS carve of fast_kernel
    int* cell_cnt;         // [frame][cell]
    uint32_t* cell_keys;   // [frame][cell_cap_total]
    int* level_keys;       // [frame][kMaxLevels] keys per level (atomic sums; 0 on entry)
    LevelPtr pyr[kMaxLevels];
};

struct OctArgs {
    Geo geo;
    const CellDesc* cells;
    int ncells;
    long long cell_cap_total;
    const int* cell_cnt;
    const uint32_t* cell_keys;
    int* level_keys;       // [frame][kMaxLevels] from fast_kernel; reset to 0 after reading
    uint32_t* keys;        // [frame][key_total] compacted per level
    int4* act;             // [frame][2 * key_total]: node positions of levels whose keys
                           // exceed kOctLdsKeys (int per key)
    uint32_t* oct_out;     // [frame][out_total]
    int* oct_cnt;          // [frame][nlevels]
    uint16_t* oct_ord;     // [frame][out_total] or null: each level's keypoints in 32-row bands
                           // (level-local indices; describe's processing order, not the output's)
    int ncap_max, sort_cap;
    int lds_keys;          // keys of a level held in LDS (Plan::oct_keys)
};

struct BlurArgs {
    int nlevels;
    int w[kMaxLevels], h[kMaxLevels];
    int taps[4];
    LevelPtr src[kMaxLevels];
    LevelPtr dst[kMaxLevels];
    int simd_xb[kMaxLevels];  // x86 arithmetic: columns [0, simd_xb) round half to even (H6)
    const uint32_t* items;     // blur_mfma_kernel: the plan's work list (blur_items)
    int nitems;
    const uint4* frags;        // blur_mfma_kernel: constant B fragments (blur_frags)
};

struct DescArgs {
    int nlevels, out_total, kps_cap;
    int wave_stride;  // 0: a wave takes G consecutive slots; W > 0: slots wv, wv + W, ... (W = waves per frame)
    int out_off[kMaxLevels];
    float scale[kMaxLevels], size[kMaxLevels];
    int w[kMaxLevels], h[kMaxLevels];
    int taps[4];
    LevelPtr pyr[kMaxLevels];
    const uint32_t* oct_out;
    const int* oct_cnt;
    const uint16_t* oct_ord;  // strided waves: slot -> level-local keypoint (OctArgs::oct_ord), or null
    orbfe_keypoint* kps;
    uint8_t* desc;
    int32_t* n_out;
    int simd_xb[kMaxLevels];  // as BlurArgs::simd_xb, for the fused per-keypoint blur
    LevelPtr blur[kMaxLevels];  // blurred levels (K4 output), read by the pre-blurred variant
    uint32_t pre_mask;          // levels whose blurred plane exists (bit l): windows read from it
    const uint4* frags;         // the matrix-core window blur: H / V fragments (blur_frags, 128..)
};

// Pixels [0, n) of a w-pixel row that OpenCV 3.3's x86 SSE2 vertical kernels produce (the rest
// is the scalar tail): VResizeLinearVec_32s8u steps 16 while x <= w - 16, then 4 while
// x < w - 4; SymmColumnVec_32s8u steps 16 while i <= w - 16, then 4 while i <= w - 4.  Both
// are multiples of 4.
inline int sse2_body_resize(int w) {
    int x = 0;
    while (x <= w - 16) x += 16;
    while (x < w - 4) x += 4;
    return x;
}
inline int sse2_body_blur(int w) {
    int i = 0;
    while (i <= w - 16) i += 16;
    while (i <= w - 4) i += 4;
    return i;
}

// Host-side ctor tables (ORBextractor.cc:409-469) + blur taps.
struct HostTables {
    orbfe_params p;
    float scale[kMaxLevels], inv[kMaxLevels], sigma2[kMaxLevels], inv_sigma2[kMaxLevels];
    int nfeat[kMaxLevels];
    int umax[16];
    int taps[7];
};

// Everything that depends on the input size.
struct Plan {
    int w = 0, h = 0;
    Geo geo{};
    std::vector<CellDesc> cells;
    long long cell_cap_total = 0;
    std::vector<int> xtab, ytab;
    int xoff[kMaxLevels] = {}, yoff[kMaxLevels] = {};
    long long slab = 0;
    int ncap_max = 0, sort_cap = 0;
    std::vector<uint32_t> bitems;  // blur_mfma_kernel work items (blur_items)
    size_t oct_lds = 0;
    int oct_keys = 0;      // LDS key capacity of the oct-tree kernel
    int roi_pitch = 0, roi_rows = 0, cand_max = 0;
    size_t fast_lds = 0;
    int rs_tiles_x[kMaxLevels] = {}, rs_tiles[kMaxLevels] = {}, rs_pitch[kMaxLevels] = {};
    size_t rs_lds[kMaxLevels] = {};
    // resize2_kernel plans for the level pairs (l, l + 1): tile table offset (int4 units in ptab)
    bool rs2_ok[kMaxLevels] = {};
    int rs2_tiles_x[kMaxLevels] = {}, rs2_tiles[kMaxLevels] = {}, rs2_off[kMaxLevels] = {};
    int rs2_pa[kMaxLevels] = {}, rs2_pb[kMaxLevels] = {}, rs2_bofs[kMaxLevels] = {};
    size_t rs2_lds[kMaxLevels] = {};
    int tail_start = kMaxLevels;  // levels >= tail_start come from resize_tail_kernel
    // pyramid_kernel: column-group tables (all levels) then the band tables of the two band
    // plans (batches >= kTailMinFrames / smaller), in one device table of u32
    bool pyr_ok = false;
    bool pyr_use[2] = {false, false};  // per band plan: the band kernel is the faster path
    std::vector<uint32_t> ptab;
    int gtab_off[kMaxLevels] = {};  // in uint4 units
    int band_off[2] = {}, nbands[2] = {}, pyr_bufb[2] = {}, pyr_ybuf[2] = {}, pyr_ymax[2] = {};
    int pyr_lp[kMaxLevels] = {};
    size_t pyr_lds[2] = {};
};

int make_tables(const orbfe_params& p, HostTables& t);
int plan_geometry(const HostTables& t, int w, int h, Plan& g);

// kernels (orbfe_extract.hip)
__global__ void level0_kernel(Level0Args);
template <bool kX86> __global__ void resize_kernel(ResizeArgs);
template <bool kX86> __global__ void resize_tail_kernel(ResizeTailArgs);
template <bool kX86> __global__ void pyramid_kernel(PyrArgs);
template <bool kX86> __global__ void resize2_kernel(Resize2Args);
template <int kP> __global__ void fast_kernel(FastArgs);
constexpr int kFastPitch = 48;  // fast_kernel<kFastPitch>: ROI pitch known at compile time
template <int BLK> __global__ void octree_kernel(OctArgs);
template <bool kX86> __global__ void blur_mfma_kernel(BlurArgs);
void blur_items(const Geo& geo, std::vector<uint32_t>& s);
// constant MFMA fragments: [0, 128) blur_mfma_kernel's, [128, 512) describe's window blur
void blur_frags(const int taps[4], uint8_t out[512 * 16]);
constexpr size_t kBlurFragBytes = 512 * 16;
constexpr int kDescFragOff = 128;  // uint4 index of describe's fragments
// describe window source: raw window blurred on the VALU (pre_mask levels read blurred
// windows), every level pre-blurred, or the raw window blurred on the matrix cores
enum { kWinValu = 0, kWinPre = 1, kWinMfma = 2 };
template <int kDescGroup, bool kX86, int kWin> __global__ void describe_kernel(DescArgs);
extern __constant__ int c_umax[16];

// pyramid_kernel band plans: LDS per workgroup for large batches (80 KB: two 1024-thread
// workgroups per CU; ORBFE_PYR_LDS_KB overrides), level-0 rows per band for small ones
constexpr int kPyrLdsCapKB = 80;
constexpr int kPyrBlockSize = 1024;
constexpr int kPyrSmallRows = 12;
// band plans whose rows computed exceed the pyramid's by more than this use the per-level
// kernels instead (large batches: throughput; small ones: latency)
constexpr double kPyrMaxWork = 1.25, kPyrMaxWorkSmall = 3.0;
constexpr int kFastBlockSize = 64;
// FAST survivor-list entries per cell (>= 322: a pre-test sweep adds <= 256 entries and a
// flush keeps <= 66).  512 covers the ~22 % pre-test pass rate of textured cells without a
// flush and brings the kernel's LDS to ~4.8 KB per wave (32 waves per CU, from ~25)
#ifndef ORBFE_FAST_LIST
#define ORBFE_FAST_LIST 512
#endif
constexpr int kFastListCap = ORBFE_FAST_LIST;
static_assert(kFastListCap >= 322, "a FAST list flush must make progress");
#ifndef ORBFE_OCT_BLOCK
#define ORBFE_OCT_BLOCK 256  // 128: 248K, 256: 254K, 512: 243K, 1024: 220K frames/s (c3)
#endif
constexpr int kOctBlockSize = ORBFE_OCT_BLOCK;
constexpr int kOctLdsKeys = 4096;  // max oct-tree keys of one level held in LDS (else global)
#ifndef ORBFE_DESC_BLOCK
#define ORBFE_DESC_BLOCK 256
#endif
// 4 keypoints per describe wave: a frame spreads over twice the waves, so ~3.5 frames are in
// flight per XCD instead of ~7 and each frame's level windows stay in that XCD's 4 MB L2 —
// describe traffic 1.70x -> 0.69x of its algorithmic bytes for +2 % kernel time
// (profiles/r02/experiments/describe_group.json).  With the matrix-core window blur the
// per-wave setup (slot lookup, IC batches, trig, fragment loads) weighs more: 8 per wave measured
// best (describe 0.2408 / 0.2357 / 0.246 / 0.253 ms at 4 / 8 / 10 / 12-16;
// profiles/r03/experiments/describe_mfma.json)
#ifndef ORBFE_DESC_GROUP
#define ORBFE_DESC_GROUP 8
#endif
constexpr int kDescBlockSize = ORBFE_DESC_BLOCK;
constexpr int kDescSmallBatch = 8;  // batches below this use kDescGroupSmall keypoints per wave
constexpr int kTailMinFrames = 8;   // batches below this skip the one-workgroup-per-frame tail
constexpr int kDescGroupSize = ORBFE_DESC_GROUP;  // oct-tree output slots per describe wave

}  // namespace orbfe
