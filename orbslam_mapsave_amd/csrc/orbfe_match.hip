// orbfe_match.hip — MI355X (gfx950) replacement for the hot subset of ORB-SLAM2's ORBmatcher
// (skaegy/ORBSLAM_MapSave src/ORBmatcher.cc) and the Frame grid it queries (src/Frame.cc).
//
//   hamming_kernel       DescriptorDistance (1650-1666), one row pair per lane
//   bf_match_kernel      brute-force best/second (config 3) on the i8 matrix cores: Hamming
//                        as popc(r) - 2 r.q + popc(q), references streamed through LDS
//   grid_kernel          Frame::AssignFeaturesToGrid (Frame.cc:341-356) as a CSR
//   *_cand_kernel        GetFeaturesInArea (Frame.cc:445-498) + distances for every query in
//                        parallel (counts, scan, fill)
//   sfi_round_kernel     SearchForInitialization's sequential greedy-with-steals semantics (H7)
//                        as Jacobi rounds to the unique fixed point of the in-order loop (a
//                        wave per query, lanes over candidates); sfi_final_kernel applies the
//                        steals, the rotation filter and the vbPrevMatched update
//   (the SearchByProjection overloads resolve in orbfe_greedy.hip: parallel Jacobi rounds
//    to the unique fixed point of the in-order loop)
//   frustum_kernel       Frame::isInFrustum (387-443) + MapPoint::PredictScale (MapPoint.cc:633)
#include <hip/hip_runtime.h>

#include <climits>
#include <type_traits>

#include "../../include/orbfe.h"
#include "orbfe_device.hpp"

namespace orbfe {

constexpr int kGridCols = 64, kGridRows = 48;  // FRAME_GRID_COLS/ROWS (Frame.h:37-38)
constexpr int kGridCells = kGridCols * kGridRows;
constexpr int kHistLen = kHistoLength;  // ORBmatcher.cc:39 (kThHigh / kThLow: orbfe_device.hpp)

struct DevFrame {
    const orbfe_keypoint* k;
    const uint4* desc;  // 2 x uint4 per keypoint
    const float* ur;    // NULL: monocular
    int n;
    float minx, maxx, miny, maxy, gwi, ghi;
    const int* cstart;  // kGridCells + 1
    const int* citems;
};

__device__ __forceinline__ int hamming_rows(const uint4* a, const uint4* b) {
    return hamming256(a[0], a[1], b[0], b[1]);
}

// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void hamming_kernel(const uint4* a, const uint4* b, int n,
                                                      int* dist) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < n) dist[i] = hamming_rows(a + 2 * i, b + 2 * i);
}

// Brute force on the matrix cores.  Over the 256 descriptor bits,
//   hamming(r, q) = popc(r) + popc(q) - 2 r.q = X + popc(q),   X = sum_k r_k (1 - 2 q_k),
// so with references as 0/1 bytes (A operand, rows) and queries as -+64 bytes (B operand,
// columns), one chain of 8 v_mfma_i32_32x32x32_i8 (one per 32-bit chunk) gives 64 X exactly,
// and popc(q) is a per-query -- per-lane, the C/D column is the lane -- constant, so each lane
// ranks its references by X alone.  The chain's C input is the row's position p in the 64-row
// reference tile, so every accumulator is already a tile-local key 64 X + p: the lane's two
// smallest keys of a tile take one v_min_i32 + one v_med3_i32 per accumulator
// (s' = med3(b, s, k), b' = min(b, k) for b <= s).  Per tile and query they become 32-bit keys
// (X << 16) + index and merge into the lane's running pair: the first-wins rule of
// ORBmatcher.cc:102-114 (strict <, start at 256) makes the best key the minimum (lowest index
// among equal distances) and the second distance the second-smallest key's; a start key of
// (256 - popc(q)) << 16 keeps distance-256 references out as the strict compare does.
//
// A block = 4 waves x 64 queries (two 32-column N-tiles per wave, their fragments resident in
// VGPRs); references stream through LDS in tiles of 64 (two 32-row M-tiles), expanded once per
// block from packed bits into fragment order [chunk][lane half][row] (16 B per entry, so a
// wave's fragment read is two contiguous 512-B runs), double-buffered, one barrier per tile.
// A tile is 4 chains (m-tile, n-tile); the ranking of each chain's 16 accumulators runs in the
// MFMA gaps of the next chain, beside a slice of the next tile's expansion (about 5 single-issue
// instructions per gap, pinned with sched_group_barrier).  Lane half h holds rows 4h.. of each
// C/D row group; its keys carry the position without the +4, added when the halves merge.
// nr < 65536 (kBfMaxRefs).
constexpr int kBfMaxRefs = 65535;
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x16 __attribute__((ext_vector_type(16)));
constexpr int kBfBlock = 256;               // 4 waves x 64 queries
constexpr int kBfWords = 512 / kBfBlock;    // raw 32-bit words a thread expands per tile
constexpr int kBfRefs = 64;                    // references per LDS tile
constexpr int kBfNone = 0x7fff;                // tile key that never wins (> 64 * 256 + 63)

// bits s .. s+3 of w as four 0/1 bytes (the multiplier spreads bit i to bit 8i, collision-free)
__device__ __forceinline__ uint32_t nibble01(uint32_t w, int s) {
    return ((w >> s) & 15u) * 0x204081u & 0x01010101u;
}
__device__ __forceinline__ i32x4 half01(uint32_t w, int h) {  // bits 16h .. 16h+15 of a chunk
    return i32x4{(int)nibble01(w, 16 * h), (int)nibble01(w, 16 * h + 4),
                 (int)nibble01(w, 16 * h + 8), (int)nibble01(w, 16 * h + 12)};
}
__device__ __forceinline__ int kmin(int a, int b) { return a < b ? a : b; }
__device__ __forceinline__ int kmax(int a, int b) { return a > b ? a : b; }
__device__ __forceinline__ int med3(int a, int b, int c) {
    int r;
    asm("v_med3_i32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
__device__ __forceinline__ constexpr int bf_pos(int mt, int e) {  // C/D row of register e
    return 32 * mt + (e & 3) + 8 * (e >> 2);
}

struct BfLane {  // one N-tile's ranking state in a lane
    int tb, ts;       // the tile's two smallest tile-local keys
    int best, second; // running 32-bit keys
    __device__ __forceinline__ void push(int k) {
        ts = med3(tb, ts, k);
        tb = kmin(tb, k);
    }
    __device__ __forceinline__ void close(int base) {  // the tile's pair into the running pair
        const int kb = ((tb >> 6) << 16) + base + (tb & 63), ks = (ts >> 6) << 16;
        second = kmin(kmin(second, ks), kmax(best, kb));
        best = kmin(best, kb);
        tb = ts = kBfNone;
    }
};

__global__ __launch_bounds__(kBfBlock) void bf_match_kernel(
    const uint8_t* q, long long q_pitch, const int* nq_arr, int nq_cap, const uint8_t* r,
    long long r_pitch, const int* nr_arr, int* out) {
    __shared__ i32x4 tile[2][16][kBfRefs];  // [buffer][2 * chunk + half][row]
    const int b = blockIdx.y;
    // counts above the slab capacities (an extraction reports its true count when it holds
    // more keypoints than kps_cap) are clamped to the rows the slabs hold
    const int nq = min(nq_arr[b], nq_cap);
    // and to kBfMaxRefs: a row index must fit the keys' 16-bit field (past it the index would
    // carry into the distance bits); the ABI documents that rows past it are not searched
    const int nr = (int)min((long long)kBfMaxRefs,
                            r_pitch >= 32 ? min((long long)nr_arr[b], r_pitch / 32) : (long long)nr_arr[b]);
    if ((int)blockIdx.x * kBfBlock >= nq) return;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int col = lane & 31, h = lane >> 5;
    const int q0 = blockIdx.x * kBfBlock + w * 64;
    const uint8_t* R = r + b * r_pitch;

    // query fragments: N-tile nt holds queries q0 + 32 nt + col
    i32x4 bq[2][8];
    int popc[2];
    BfLane st[2];
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
        const int qi = q0 + 32 * nt + col;
        uint4 d0 = make_uint4(0, 0, 0, 0), d1 = d0;
        if (qi < nq) {
            const uint4* Q = reinterpret_cast<const uint4*>(q + b * q_pitch) + 2 * qi;
            d0 = Q[0];
            d1 = Q[1];
        }
        const uint32_t dw[8] = {d0.x, d0.y, d0.z, d0.w, d1.x, d1.y, d1.z, d1.w};
        int pc = 0;
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            pc += __popc(dw[c]);
            const i32x4 v = half01(dw[c], h);  // 64 (1 - 2 bit) as bytes: 0 -> 0x40, 1 -> 0xc0
            bq[nt][c] = i32x4{(int)((uint32_t)v.x << 7 ^ 0x40404040u),
                              (int)((uint32_t)v.y << 7 ^ 0x40404040u),
                              (int)((uint32_t)v.z << 7 ^ 0x40404040u),
                              (int)((uint32_t)v.w << 7 ^ 0x40404040u)};
        }
        popc[nt] = pc;
        st[nt].best = st[nt].second = (256 - pc) << 16;
        st[nt].tb = st[nt].ts = kBfNone;
    }
    i32x16 pos[2];  // C input: the row's position in the tile, without the 4h
#pragma unroll
    for (int e = 0; e < 16; ++e) {
        pos[0][e] = bf_pos(0, e);
        pos[1][e] = bf_pos(1, e);
    }

    // tile loader: thread -> row lrow, raw words kBfWords lcp .. (+kBfWords); rows past nr load
    // zeros, branch-free so that the loop body stays one basic block for the scheduler
    const int lrow = tid & 63, lcp = tid >> 6;
    struct Raw { uint32_t w[kBfWords]; };
    auto fetch = [&](int t) {
        const int j = t * kBfRefs + lrow;
        const uint32_t* src = reinterpret_cast<const uint32_t*>(
            R + (long long)min(j, max(nr - 1, 0)) * 32 + 4 * kBfWords * lcp);
        Raw v;
        if constexpr (kBfWords == 2) {
            const uint2 u = *reinterpret_cast<const uint2*>(src);
            v.w[0] = j < nr ? u.x : 0u;
            v.w[1] = j < nr ? u.y : 0u;
        } else {
            v.w[0] = j < nr ? src[0] : 0u;
        }
        return v;
    };
    const int nfull = nr / kBfRefs, ntiles = (nr + kBfRefs - 1) / kBfRefs;
    if (nr) {
        const Raw v = fetch(0);
#pragma unroll
        for (int j = 0; j < kBfWords; ++j) {
            tile[0][2 * (kBfWords * lcp + j) + 0][lrow] = half01(v.w[j], 0);
            tile[0][2 * (kBfWords * lcp + j) + 1][lrow] = half01(v.w[j], 1);
        }
    }
    __syncthreads();

    // One tile = chains p = 0..3 (m-tile p & 1, n-tile p >> 1), each 8 MFMAs.  In the gaps of
    // chain p: the ranking of chain p - 1 (chain 3 of the previous tile for p = 0) and 1/32 of
    // the next tile's expansion per MFMA.  Raw bits run two tiles ahead.
    Raw raw = fetch(1);
    i32x16 accp;  // the previous chain's keys
#pragma unroll
    for (int e = 0; e < 16; ++e) accp[e] = kBfNone;
    auto step = [&](int t, auto partial_tag) {
        constexpr bool partial = decltype(partial_tag)::value;
        const int cur = t & 1;
        const Raw raw2 = fetch(t + 2);
        const int valid = nr - t * kBfRefs - 4 * h;  // positions >= valid lie past nr
        uint32_t ex[4];
        // fragment ring, two reads ahead: fragment f = 8 p + c is chunk c of m-tile p & 1
        auto frag = [&](int f) { return tile[cur][2 * (f & 7) + h][32 * ((f >> 3) & 1) + col]; };
        i32x4 a = frag(0), a1 = frag(1);
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            const int mt = p & 1, nt = p >> 1;
            const int pmt = (p + 3) & 1, pnt = ((p + 3) & 3) >> 1;  // previous chain
            i32x16 acc;
#pragma unroll
            for (int c = 0; c < 8; ++c) {
                const int f = 8 * p + c;
                i32x4 a2 = a1;
                if (f + 2 < 32) a2 = frag(f + 2);
                acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, bq[nt][c], c ? acc : pos[mt], 0, 0, 0);
#pragma unroll
                for (int u = 0; u < 2; ++u) {
                    const int e = 2 * c + u;
                    int k = accp[e];
                    // chain p - 1 of this tile may be partial; chain 3 of the previous tile not
                    if (partial && p > 0 && bf_pos(pmt, e) >= valid) k = kBfNone;
                    st[pnt].push(k);
                }
                const int n = f * kBfWords / 4;  // nibble slot of this MFMA
                if ((f * kBfWords) % 4 == 0 && n < 8 * kBfWords) {
                    ex[n & 3] = nibble01(raw.w[n >> 3], 16 * ((n >> 2) & 1) + 4 * (n & 3));
                    if ((n & 3) == 3)
                        tile[cur ^ 1][2 * kBfWords * lcp + (n >> 2)][lrow] =
                            i32x4{(int)ex[0], (int)ex[1], (int)ex[2], (int)ex[3]};
                }
                a = a1;
                a1 = a2;
                __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // fragment read, 2 ahead
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
                __builtin_amdgcn_sched_group_barrier(0x002, 5, 0);  // fillers
                __builtin_amdgcn_sched_barrier(0);
            }
            // tile t - 1's n-tile 1 (for t = 0 a no-op merge of "never wins" keys)
            if (p == 0) st[1].close((t - 1) * kBfRefs);
            if (p == 2) st[0].close(t * kBfRefs);  // this tile, n-tile 0
            accp = acc;
        }
        raw = raw2;
        __syncthreads();
    };
    for (int t = 0; t < nfull; ++t) step(t, std::false_type{});
    if (nfull < ntiles) step(nfull, std::true_type{});
    if (ntiles) {  // chain 3 of the last tile
        const int valid = nr - (ntiles - 1) * kBfRefs - 4 * h;
#pragma unroll
        for (int e = 0; e < 16; ++e) st[1].push(bf_pos(1, e) < valid ? accp[e] : kBfNone);
        st[1].close((ntiles - 1) * kBfRefs);
    }
    int best[2] = {st[0].best, st[1].best}, second[2] = {st[0].second, st[1].second};
    // merge the lane halves (the same queries, rows 4h..), then half h reports N-tile h
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
        const int kb = best[nt] + 4 * h, ks = second[nt];
        const int ob = __shfl_xor(kb, 32), os = __shfl_xor(ks, 32);
        second[nt] = kmin(kmin(ks, os), kmax(kb, ob));
        best[nt] = kmin(kb, ob);
    }
    const int qi = q0 + 32 * h + col;
    if (qi < nq) {
        const int kb = h ? best[1] : best[0], ks = h ? second[1] : second[0];
        const int pc = h ? popc[1] : popc[0];
        const int db = (kb >> 16) + pc;
        int* o = out + ((long long)b * nq_cap + qi) * 3;
        o[0] = db >= 256 ? -1 : (kb & 0xffff);
        o[1] = db;
        o[2] = (ks >> 16) + pc;
    }
}

// The same brute force on the FP4 matrix cores (v_mfma_scale_f32_32x32x64_f8f6f4, e2m1 A and B):
// a reference bit is the FP4 value 0 or 1 (nibble 0x0 / 0x2), a query bit +1 or -1 (0x2 /
// 0xA) and the B block scale 2^6 makes it +-64, so each accumulator is again 64 X + p exactly
// (f32 holds every integer below 2^24).  One instruction covers 64 descriptor bits at the
// cycles the i8 form spends on 32, so a 32 x 32 tile is a chain of 4 MFMAs instead of 8.
// Lane half h of chunk c (bits 64 c .. 64 c + 63) holds descriptor dword 2 c + h as 32 nibbles;
// the nibble order inside the lane is the same permutation for references and queries (a K
// permutation common to A and B leaves the product unchanged): bit 8 q + b -> dword q, byte b,
// low nibble; bit 8 q + 4 + b -> the high nibble.  Ranking as above, on f32 keys (min / med3 of
// exact integers), converted to the 32-bit keys when a tile closes.
// ORBFE_BF_WAVES: minimum waves per SIMD the FP4 kernel is compiled for.  At 3 it takes 135
// VGPRs; 4 (<= 128 VGPRs, 3 spilled, all 1,024 blocks of a 256-frame step resident at once
// instead of in 1.33 rounds) measured the same 103.2-103.9 us per launch
// (profiles/r03/experiments/bf_waves.json)
#ifndef ORBFE_BF_WAVES
#define ORBFE_BF_WAVES 3
#endif
typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
constexpr float kBfNoneF = 32767.f;
// 8 bits (s .. s+7 of w) as 8 nibbles of one dword, each 0 or 1 (bit s+b -> byte b low nibble,
// bit s+4+b -> byte b high nibble)
__device__ __forceinline__ uint32_t bits8_nib(uint32_t w, int s) {
    return nibble01(w, s) | (nibble01(w, s + 4) << 4);
}
__device__ __forceinline__ i32x4 ref_fp4(uint32_t w) {  // 0 -> 0.0, 1 -> 1.0 (0x2)
    return i32x4{(int)(bits8_nib(w, 0) << 1), (int)(bits8_nib(w, 8) << 1),
                 (int)(bits8_nib(w, 16) << 1), (int)(bits8_nib(w, 24) << 1)};
}
__device__ __forceinline__ i32x4 qry_fp4(uint32_t w) {  // 0 -> +1.0 (0x2), 1 -> -1.0 (0xA)
    return i32x4{(int)((bits8_nib(w, 0) << 3) | 0x22222222u), (int)((bits8_nib(w, 8) << 3) | 0x22222222u),
                 (int)((bits8_nib(w, 16) << 3) | 0x22222222u), (int)((bits8_nib(w, 24) << 3) | 0x22222222u)};
}
struct BfLaneF {
    float tb, ts;
    int best, second;
    __device__ __forceinline__ void push(float k) {
        // exact integers, never NaN: plain v_min_f32 (fminf would canonicalize its operands)
        ts = __builtin_amdgcn_fmed3f(tb, ts, k);
        float m;
        asm("v_min_f32 %0, %1, %2" : "=v"(m) : "v"(tb), "v"(k));
        tb = m;
    }
    __device__ __forceinline__ void close(int base) {
        const int ib = (int)tb, is = (int)ts;
        const int kb = ((ib >> 6) << 16) + base + (ib & 63), ks = (is >> 6) << 16;
        second = kmin(kmin(second, ks), kmax(best, kb));
        best = kmin(best, kb);
        tb = ts = kBfNoneF;
    }
};
// A reference set shared by every batch entry (r_pitch 0: config 3's one reference frame) is
// expanded to FP4 fragments once per call by bf_expand_kernel, in the LDS tile layout
// E[tile][descriptor dword][row]; the brute force (kPre) then copies each tile with 16-byte loads
// instead of every workgroup expanding the same bits (a third of its VALU in the MFMA gaps).
// Rows at or past nr are zero, as the in-kernel expansion pads them.
constexpr int kBfMaxTiles = (kBfMaxRefs + kBfRefs) / kBfRefs;
constexpr int kBfExpandBlocks = 64;
// kBfExpandBlocks workgroups stride over the tiles (the largest count in nr_arr is read once per
// workgroup, not once per possible tile).
__global__ __launch_bounds__(512) void bf_expand_kernel(const uint8_t* r, const int* nr_arr, int nb,
                                                        i32x4* E) {
    __shared__ int s_nr;
    if (threadIdx.x == 0) s_nr = 0;
    __syncthreads();
    int m = 0;
    for (int b = threadIdx.x; b < nb; b += 512) m = max(m, nr_arr[b]);
    if (m) atomicMax(&s_nr, m);
    __syncthreads();
    const int nr = min(s_nr, kBfMaxRefs);
    const int row = threadIdx.x & 63, dw = threadIdx.x >> 6;  // 8 dwords x 64 rows
    for (int t = blockIdx.x; t * kBfRefs < nr; t += gridDim.x) {
        const int j = t * kBfRefs + row;
        const uint32_t w = j < nr ? reinterpret_cast<const uint32_t*>(r + (long long)j * 32)[dw] : 0u;
        E[((size_t)t * 8 + dw) * kBfRefs + row] = ref_fp4(w);
    }
}

template <bool kPre>
__device__ __forceinline__ void bf_fp4_body(
    const uint8_t* q, long long q_pitch, const int* nq_arr, int nq_cap, const uint8_t* r,
    long long r_pitch, const int* nr_arr, int* out, const i32x4* E) {
    __shared__ i32x4 tile[2][8][kBfRefs];  // [buffer][descriptor dword][row]
    const int b = blockIdx.y;
    const int nq = min(nq_arr[b], nq_cap);
    // and to kBfMaxRefs: a row index must fit the keys' 16-bit field (past it the index would
    // carry into the distance bits); the ABI documents that rows past it are not searched
    const int nr = (int)min((long long)kBfMaxRefs,
                            r_pitch >= 32 ? min((long long)nr_arr[b], r_pitch / 32) : (long long)nr_arr[b]);
    if ((int)blockIdx.x * kBfBlock >= nq) return;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int col = lane & 31, h = lane >> 5;
    const int q0 = blockIdx.x * kBfBlock + w * 64;
    const uint8_t* R = r + b * r_pitch;
    i32x4 bq[2][4];
    int popc[2];
    BfLaneF st[2];
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
        const int qi = q0 + 32 * nt + col;
        uint4 d0 = make_uint4(0, 0, 0, 0), d1 = d0;
        if (qi < nq) {
            const uint4* Q = reinterpret_cast<const uint4*>(q + b * q_pitch) + 2 * qi;
            d0 = Q[0];
            d1 = Q[1];
        }
        const uint32_t dw[8] = {d0.x, d0.y, d0.z, d0.w, d1.x, d1.y, d1.z, d1.w};
        int pc = 0;
#pragma unroll
        for (int c = 0; c < 8; ++c) pc += __popc(dw[c]);
#pragma unroll
        for (int c = 0; c < 4; ++c) bq[nt][c] = qry_fp4(dw[2 * c + h]);
        popc[nt] = pc;
        st[nt].best = st[nt].second = (256 - pc) << 16;
        st[nt].tb = st[nt].ts = kBfNoneF;
    }
    f32x16 pos[2];
#pragma unroll
    for (int e = 0; e < 16; ++e) {
        pos[0][e] = (float)bf_pos(0, e);
        pos[1][e] = (float)bf_pos(1, e);
    }
    const int lrow = tid & 63, lcp = tid >> 6;
    struct Raw { uint32_t w[kBfWords]; };
    struct RawE { i32x4 v[kBfWords]; };
    auto fetch_e = [&](int t) {  // kPre: this thread's kBfWords expanded entries of tile t
        RawE v;
#pragma unroll
        for (int j = 0; j < kBfWords; ++j) v.v[j] = E[((size_t)t * 8 + kBfWords * lcp + j) * kBfRefs + lrow];
        return v;
    };
    auto fetch = [&](int t) {
        const int j = t * kBfRefs + lrow;
        const uint32_t* src = reinterpret_cast<const uint32_t*>(
            R + (long long)min(j, max(nr - 1, 0)) * 32 + 4 * kBfWords * lcp);
        Raw v;
        if constexpr (kBfWords == 2) {
            const uint2 u = *reinterpret_cast<const uint2*>(src);
            v.w[0] = j < nr ? u.x : 0u;
            v.w[1] = j < nr ? u.y : 0u;
        } else {
            v.w[0] = j < nr ? src[0] : 0u;
        }
        return v;
    };
    const int nfull = nr / kBfRefs, ntiles = (nr + kBfRefs - 1) / kBfRefs;
    if (nr) {
        if constexpr (kPre) {
            const RawE v = fetch_e(0);
#pragma unroll
            for (int j = 0; j < kBfWords; ++j) tile[0][kBfWords * lcp + j][lrow] = v.v[j];
        } else {
            const Raw v = fetch(0);
#pragma unroll
            for (int j = 0; j < kBfWords; ++j) tile[0][kBfWords * lcp + j][lrow] = ref_fp4(v.w[j]);
        }
    }
    __syncthreads();
    using RawT = std::conditional_t<kPre, RawE, Raw>;
    auto fetch_any = [&](int t) -> RawT {
        if constexpr (kPre) {
            // tiles past the last are stored to the ring but never read: fetch tile 0 for them
            return fetch_e(t * kBfRefs < nr ? t : 0);
        } else {
            return fetch(t);
        }
    };
    RawT raw = fetch_any(1);
    f32x16 accp;
#pragma unroll
    for (int e = 0; e < 16; ++e) accp[e] = kBfNoneF;
    const int scale_a = 127, scale_b = 127 + 6;  // e8m0: 1 and 2^6
    auto step = [&](int t, auto partial_tag) {
        constexpr bool partial = decltype(partial_tag)::value;
        const int cur = t & 1;
        const RawT raw2 = fetch_any(t + 2);
        const int valid = nr - t * kBfRefs - 4 * h;
        // fragment ring, two reads ahead: fragment f = 4 p + c is chunk c of m-tile p & 1
        auto frag = [&](int f) { return tile[cur][2 * (f & 3) + h][32 * ((f >> 2) & 1) + col]; };
        i32x4 a = frag(0), a1 = frag(1);
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            const int mt = p & 1, nt = p >> 1;
            const int pmt = (p + 3) & 1, pnt = ((p + 3) & 3) >> 1;
            f32x16 acc;
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const int f = 4 * p + c;
                i32x4 a2 = a1;
                if (f + 2 < 16) a2 = frag(f + 2);
                const i32x8 av = i32x8{a[0], a[1], a[2], a[3], 0, 0, 0, 0};
                const i32x8 bv = i32x8{bq[nt][c][0], bq[nt][c][1], bq[nt][c][2], bq[nt][c][3], 0, 0, 0, 0};
                acc = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(av, bv, c ? acc : pos[mt], 4, 4, 0,
                                                                       scale_a, 0, scale_b);
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int e = 4 * c + u;
                    float k = accp[e];
                    if (partial && p > 0 && bf_pos(pmt, e) >= valid) k = kBfNoneF;
                    st[pnt].push(k);
                }
                // next tile's expansion: word f / 8 of this thread's kBfWords at gap f % 8 == 7
                if (f % 8 == 7 && (f >> 3) < kBfWords) {
                    if constexpr (kPre)
                        tile[cur ^ 1][kBfWords * lcp + (f >> 3)][lrow] = raw.v[f >> 3];
                    else
                        tile[cur ^ 1][kBfWords * lcp + (f >> 3)][lrow] = ref_fp4(raw.w[f >> 3]);
                }
                a = a1;
                a1 = a2;
                __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // fragment read, 2 ahead
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
                __builtin_amdgcn_sched_group_barrier(0x002, 10, 0);  // fillers
                __builtin_amdgcn_sched_barrier(0);
            }
            if (p == 0) st[1].close((t - 1) * kBfRefs);
            if (p == 2) st[0].close(t * kBfRefs);
            accp = acc;
        }
        raw = raw2;
        __syncthreads();
    };
    for (int t = 0; t < nfull; ++t) step(t, std::false_type{});
    if (nfull < ntiles) step(nfull, std::true_type{});
    if (ntiles) {
        const int valid = nr - (ntiles - 1) * kBfRefs - 4 * h;
#pragma unroll
        for (int e = 0; e < 16; ++e) st[1].push(bf_pos(1, e) < valid ? accp[e] : kBfNoneF);
        st[1].close((ntiles - 1) * kBfRefs);
    }
    int best[2] = {st[0].best, st[1].best}, second[2] = {st[0].second, st[1].second};
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
        const int kb = best[nt] + 4 * h, ks = second[nt];
        const int ob = __shfl_xor(kb, 32), os = __shfl_xor(ks, 32);
        second[nt] = kmin(kmin(ks, os), kmax(kb, ob));
        best[nt] = kmin(kb, ob);
    }
    const int qi = q0 + 32 * h + col;
    if (qi < nq) {
        const int kb = h ? best[1] : best[0], ks = h ? second[1] : second[0];
        const int pc = h ? popc[1] : popc[0];
        const int db = (kb >> 16) + pc;
        int* o = out + ((long long)b * nq_cap + qi) * 3;
        o[0] = db >= 256 ? -1 : (kb & 0xffff);
        o[1] = db;
        o[2] = (ks >> 16) + pc;
    }
}

__global__ __launch_bounds__(kBfBlock, ORBFE_BF_WAVES) void bf_match_fp4_kernel(
    const uint8_t* q, long long q_pitch, const int* nq_arr, int nq_cap, const uint8_t* r,
    long long r_pitch, const int* nr_arr, int* out) {
    bf_fp4_body<false>(q, q_pitch, nq_arr, nq_cap, r, r_pitch, nr_arr, out, nullptr);
}
// the same with the shared reference set pre-expanded (bf_expand_kernel)
__global__ __launch_bounds__(kBfBlock, ORBFE_BF_WAVES) void bf_match_fp4e_kernel(
    const uint8_t* q, long long q_pitch, const int* nq_arr, int nq_cap, const uint8_t* r,
    long long r_pitch, const int* nr_arr, int* out, const i32x4* E) {
    bf_fp4_body<true>(q, q_pitch, nq_arr, nq_cap, r, r_pitch, nr_arr, out, E);
}

// The brute-force kernel the ABI launches: the FP4 form, or the i8 form (the measured
// alternative) for a matcher created with ORBFE_BF_I8=1 in the environment (the
// GPU suite runs the brute-force parity tests on both).
using BfKernel = void (*)(const uint8_t*, long long, const int*, int, const uint8_t*, long long,
                          const int*, int*);

// ---------------------------------------------------------------------------------------------
// Grid as CSR.  cellof[i] = -1 for keypoints outside the 64 x 48 grid (PosInGrid, 500-510).
constexpr int kGridBlock = 1024;
__global__ __launch_bounds__(kGridBlock) void grid_kernel(const orbfe_keypoint* k, int n,
                                                          float minx, float miny, float gwi,
                                                          float ghi, int* cellof, int* cstart,
                                                          int* citems) {
    __shared__ int cnt[kGridCells];
    __shared__ int tmp[kGridBlock / 64 + 1];
    for (int c = threadIdx.x; c < kGridCells; c += kGridBlock) cnt[c] = 0;
    __syncthreads();
    for (int i = threadIdx.x; i < n; i += kGridBlock) {
        const int gx = (int)roundf((k[i].x - minx) * gwi);
        const int gy = (int)roundf((k[i].y - miny) * ghi);
        int c = -1;
        if (gx >= 0 && gx < kGridCols && gy >= 0 && gy < kGridRows) {
            c = gx * kGridRows + gy;  // mGrid[ix][iy]
            atomicAdd(&cnt[c], 1);
        }
        cellof[i] = c;
    }
    __syncthreads();
    constexpr int PER = (kGridCells + kGridBlock - 1) / kGridBlock;
    int local[PER], sum = 0;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        const int c = threadIdx.x * PER + j;
        local[j] = c < kGridCells ? cnt[c] : 0;
        sum += local[j];
    }
    int total;
    int off = block_exclusive_scan<kGridBlock>(sum, tmp, total);
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        const int c = threadIdx.x * PER + j;
        if (c < kGridCells) {
            cstart[c] = off;
            cnt[c] = off;  // cursor
        }
        off += local[j];
    }
    if (threadIdx.x == 0) cstart[kGridCells] = total;
    __syncthreads();
    for (int i = threadIdx.x; i < n; i += kGridBlock) {
        const int c = cellof[i];
        if (c >= 0) citems[atomicAdd(&cnt[c], 1)] = i;
    }
    __syncthreads();
    for (int c = threadIdx.x; c < kGridCells; c += kGridBlock) {  // insertion order = index order
        const int s = cstart[c], e = cstart[c + 1];
        for (int a = s + 1; a < e; ++a) {
            const int v = citems[a];
            int b = a - 1;
            while (b >= s && citems[b] > v) {
                citems[b + 1] = citems[b];
                --b;
            }
            citems[b + 1] = v;
        }
    }
}

constexpr int kGridPer = 8;                           // keypoints per thread held in registers
constexpr int kGridLdsMax = kGridBlock * kGridPer;    // 8192: the items list fits LDS (32 KB)
// grid_kernel for n <= kGridLdsMax: the cell of every keypoint stays in registers and the items
// list is filled, ordered and only then copied out of LDS, so no step waits on a chain of
// dependent global loads (grid_kernel's insertion sort walks global memory).
__global__ __launch_bounds__(kGridBlock) void grid_lds_kernel(const orbfe_keypoint* k, int n,
                                                              float minx, float miny, float gwi,
                                                              float ghi, int* cstart,
                                                              int* citems) {
    __shared__ int cnt[kGridCells];
    __shared__ int items[kGridLdsMax];
    __shared__ int tmp[kGridBlock / 64 + 1];
    for (int c = threadIdx.x; c < kGridCells; c += kGridBlock) cnt[c] = 0;
    __syncthreads();
    int mine[kGridPer];  // cells of keypoints threadIdx.x + j * kGridBlock
#pragma unroll
    for (int j = 0; j < kGridPer; ++j) {
        const int i = threadIdx.x + j * kGridBlock;
        mine[j] = -1;
        if (i < n) {
            const int gx = (int)roundf((k[i].x - minx) * gwi);
            const int gy = (int)roundf((k[i].y - miny) * ghi);
            if (gx >= 0 && gx < kGridCols && gy >= 0 && gy < kGridRows) {
                mine[j] = gx * kGridRows + gy;  // mGrid[ix][iy]
                atomicAdd(&cnt[mine[j]], 1);
            }
        }
    }
    __syncthreads();
    constexpr int PER = (kGridCells + kGridBlock - 1) / kGridBlock;
    int local[PER], sum = 0;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        const int c = threadIdx.x * PER + j;
        local[j] = c < kGridCells ? cnt[c] : 0;
        sum += local[j];
    }
    int total;
    int off = block_exclusive_scan<kGridBlock>(sum, tmp, total);
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        const int c = threadIdx.x * PER + j;
        if (c < kGridCells) {
            cstart[c] = off;
            cnt[c] = off;  // cursor
        }
        off += local[j];
    }
    if (threadIdx.x == 0) cstart[kGridCells] = total;
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kGridPer; ++j)
        if (mine[j] >= 0) items[atomicAdd(&cnt[mine[j]], 1)] = threadIdx.x + j * kGridBlock;
    __syncthreads();
    // insertion order = index order: sort each cell's items; cnt[c] is now the end of cell c
    // and cnt[c - 1] its start
    for (int c = threadIdx.x; c < kGridCells; c += kGridBlock) {
        const int e = cnt[c], s0 = c ? cnt[c - 1] : 0;
        for (int q = s0 + 1; q < e; ++q) {
            const int v = items[q];
            int b = q - 1;
            while (b >= s0 && items[b] > v) {
                items[b + 1] = items[b];
                --b;
            }
            items[b + 1] = v;
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < total; i += kGridBlock) citems[i] = items[i];
}

// Frame::GetFeaturesInArea (Frame.cc:445-498): visits candidates in ix-major, iy, insertion
// order and calls fn(idx) for each.
template <class Fn>
__device__ __forceinline__ void features_in_area(const DevFrame& F, float x, float y, float r,
                                                 int min_level, int max_level, Fn fn) {
    const int cx0 = max(0, (int)floorf((x - F.minx - r) * F.gwi));
    if (cx0 >= kGridCols) return;
    const int cx1 = min(kGridCols - 1, (int)ceilf((x - F.minx + r) * F.gwi));
    if (cx1 < 0) return;
    const int cy0 = max(0, (int)floorf((y - F.miny - r) * F.ghi));
    if (cy0 >= kGridRows) return;
    const int cy1 = min(kGridRows - 1, (int)ceilf((y - F.miny + r) * F.ghi));
    if (cy1 < 0) return;
    const bool check = min_level > 0 || max_level >= 0;
    for (int ix = cx0; ix <= cx1; ++ix)
        for (int iy = cy0; iy <= cy1; ++iy) {
            const int c = ix * kGridRows + iy;
            for (int e = F.cstart[c]; e < F.cstart[c + 1]; ++e) {
                const int idx = F.citems[e];
                const orbfe_keypoint kp = F.k[idx];
                if (check) {
                    if (kp.octave < min_level) continue;
                    if (max_level >= 0 && kp.octave > max_level) continue;
                }
                if (fabsf(kp.x - x) < r && fabsf(kp.y - y) < r) fn(idx);
            }
        }
}

// Wave-cooperative GetFeaturesInArea for one query per wave (every lane passes the same query):
// lane t takes cell t of the window in the reference's ix-major, iy order (64 cells per
// step), counts its passing items, and an exclusive wave scan of the counts places every
// candidate at its reference rank; emit(idx, rank) runs on the lane owning the candidate.
// Returns the candidate count (wave-uniform).  keep(idx) is an extra per-candidate filter.
template <class Keep, class Emit>
__device__ __forceinline__ int features_in_area_wave(const DevFrame& F, float x, float y, float r,
                                                     int min_level, int max_level, Keep keep,
                                                     Emit emit) {
    const int lane = threadIdx.x & 63;
    const int cx0 = max(0, (int)floorf((x - F.minx - r) * F.gwi));
    if (cx0 >= kGridCols) return 0;
    const int cx1 = min(kGridCols - 1, (int)ceilf((x - F.minx + r) * F.gwi));
    if (cx1 < 0) return 0;
    const int cy0 = max(0, (int)floorf((y - F.miny - r) * F.ghi));
    if (cy0 >= kGridRows) return 0;
    const int cy1 = min(kGridRows - 1, (int)ceilf((y - F.miny + r) * F.ghi));
    if (cy1 < 0) return 0;
    const bool check = min_level > 0 || max_level >= 0;
    const int ny = cy1 - cy0 + 1, ncell = (cx1 - cx0 + 1) * ny;
    auto pass = [&](int idx) {
        const orbfe_keypoint kp = F.k[idx];
        if (check) {
            if (kp.octave < min_level) return false;
            if (max_level >= 0 && kp.octave > max_level) return false;
        }
        return fabsf(kp.x - x) < r && fabsf(kp.y - y) < r && keep(idx);
    };
    int total = 0;
    for (int c0 = 0; c0 < ncell; c0 += 64) {
        const int t = c0 + lane;
        int e0 = 0, e1 = 0, n = 0;
        if (t < ncell) {
            const int c = (cx0 + t / ny) * kGridRows + cy0 + t % ny;
            e0 = F.cstart[c];
            e1 = F.cstart[c + 1];
            for (int e = e0; e < e1; ++e) n += pass(F.citems[e]);
        }
        const int inc = wave_inclusive_sum(n);
        int rank = total + inc - n;
        if (n)
            for (int e = e0; e < e1; ++e) {
                const int idx = F.citems[e];
                if (pass(idx)) emit(idx, rank++);
            }
        total += __shfl(inc, 63, 64);
    }
    return total;
}

// Exclusive scan of counts[0..n) into off[0..n], single workgroup.
__global__ __launch_bounds__(1024) void scan_kernel(const int* counts, int n, int* off) {
    __shared__ int tmp[1024 / 64 + 1];
    int run = 0;
    for (int base = 0; base < n; base += 1024) {
        const int i = base + threadIdx.x;
        const int v = i < n ? counts[i] : 0;
        int t;
        const int ex = block_exclusive_scan<1024>(v, tmp, t);
        if (i < n) off[i] = run + ex;
        run += t;
    }
    if (threadIdx.x == 0) off[n] = run;
}

// ---------------------------------------------------------------------------------------------
// Frame::GetFeaturesInArea (Frame.cc:445-498) as a batch of queries — the parity probe of the
// grid (orbfe_features_in_area): thread-per-query (features_in_area) and wave-per-query
// (features_in_area_wave, which the matchers use: SearchForInitialization, SearchByProjection's
// local-map / last-frame / keyframe forms) write each query's candidates in the reference's
// order to items[off[q] ..).
struct FiaArgs {
    DevFrame f;
    int nq;
    const float* x;
    const float* y;
    const float* r;
    const int* lo;
    const int* hi;
    int* cnt;
    const int* off;
    int* items;
};
template <bool FILL>
__global__ __launch_bounds__(256) void fia_thread_kernel(FiaArgs a) {
    const int q = blockIdx.x * 256 + threadIdx.x;
    if (q >= a.nq) return;
    const int o = FILL ? a.off[q] : 0;
    int n = 0;
    features_in_area(a.f, a.x[q], a.y[q], a.r[q], a.lo[q], a.hi[q], [&](int idx) {
        if (FILL) a.items[o + n] = idx;
        ++n;
    });
    if (!FILL) a.cnt[q] = n;
}
template <bool FILL>
__global__ __launch_bounds__(256) void fia_wave_kernel(FiaArgs a) {
    const int q = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (q >= a.nq) return;
    const int o = FILL ? a.off[q] : 0;
    const int n = features_in_area_wave(
        a.f, a.x[q], a.y[q], a.r[q], a.lo[q], a.hi[q], [](int) { return true; },
        [&](int idx, int rank) {
            if (FILL) a.items[o + rank] = idx;
        });
    if (!FILL && (threadIdx.x & 63) == 0) a.cnt[q] = n;
}

// ---------------------------------------------------------------------------------------------
// SearchForInitialization (ORBmatcher.cc:408-523)
struct SfiArgs {
    DevFrame f1, f2;
    const float* prev;  // 2 per F1 keypoint
    float window;
    long long cand_cap;  // fill writes only lists that end within the capacity
    int* cnt;           // per F1 keypoint
    const int* off;     // n1 + 1
    int2* cand;         // (i2, dist)
};

template <bool FILL>
__global__ __launch_bounds__(256) void sfi_cand_kernel(SfiArgs a) {
    const int i1 = blockIdx.x * 4 + (threadIdx.x >> 6);  // one wave per F1 keypoint
    if (i1 >= a.f1.n) return;
    if (FILL && a.off[i1 + 1] > a.cand_cap) return;
    const orbfe_keypoint k1 = a.f1.k[i1];
    if (k1.octave > 0) {
        if (!FILL && (threadIdx.x & 63) == 0) a.cnt[i1] = 0;
        return;
    }
    const uint4* d1 = a.f1.desc + 2 * i1;
    const uint4 q0 = d1[0], q1 = d1[1];
    int2* out = FILL ? a.cand + a.off[i1] : nullptr;
    const int n = features_in_area_wave(
        a.f2, a.prev[2 * i1], a.prev[2 * i1 + 1], a.window, k1.octave, k1.octave,
        [](int) { return true; },
        [&](int i2, int rank) {
            if (FILL) {
                const uint4* d2 = a.f2.desc + 2 * i2;
                out[rank] = make_int2(i2, hamming256(q0, q1, d2[0], d2[1]));
            }
        });
    if (!FILL && (threadIdx.x & 63) == 0) a.cnt[i1] = n;
}

__device__ __forceinline__ int rot_bin(float a1, float a2) {  // ORBmatcher.cc:478-483
    float rot = a1 - a2;
    if (rot < 0.0) rot += 360.0f;
    int bin = (int)roundf(rot * (1.0f / kHistLen));
    if (bin == kHistLen) bin = 0;
    return bin;
}

// ComputeThreeMaxima (ORBmatcher.cc:1604-1645) over 30 bin counts.
__host__ __device__ __forceinline__ void three_maxima(const int* h, int& i1, int& i2, int& i3) {
    int m1 = 0, m2 = 0, m3 = 0;
    i1 = i2 = i3 = -1;
    for (int i = 0; i < kHistLen; ++i) {
        const int s = h[i];
        if (s > m1) { m3 = m2; m2 = m1; m1 = s; i3 = i2; i2 = i1; i1 = i; }
        else if (s > m2) { m3 = m2; m2 = s; i3 = i2; i2 = i; }
        else if (s > m3) { m3 = s; i3 = i; }
    }
    if (m2 < 0.1f * (float)m1) { i2 = -1; i3 = -1; }
    else if (m3 < 0.1f * (float)m1) { i3 = -1; }
}

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

// Lowest lane of the wave with `pred` set, 64 if none.
__device__ __forceinline__ int first_lane(bool pred) {
    const unsigned long long b = __ballot(pred);
    return b ? __builtin_ctzll(b) : 64;
}

// SearchForInitialization's greedy loop as a fixed point.  Query i (an F1 keypoint, in index
// order) skips candidate s when vMatchedDistance[s] <= dist (447-448); vMatchedDistance only
// decreases, and at query i it is min{d_j : j < i accepted s with distance d_j}.  So query i's
// decision depends only on the decisions of j < i: the system D = decide(D) has one fixed point,
// the in-order loop's result, and Jacobi rounds reach it (after a round the lowest wrong
// decision depends only on correct ones, so the correct prefix grows).  A round is one launch:
// a wave per query, lanes over its candidates, best = min (dist << 16 | rank) (the first minimum
// in GetFeaturesInArea order) and second = the minimum of the other distances, as the
// sequential best / second update yields.  Each accepting query appends (i, dist) to its slot's
// list for the next round (k entries per slot: 64 first, and if a round overflows that, the
// rounds are rerun with room for every query).  Three list buffers rotate (read / write /
// cleared), two decision buffers ping-pong.  After convergence a slot belongs to its last acceptor (steals, 466-470) and the
// rotation histogram counts every acceptance, stolen or not (rotHist is filled at accept time).
constexpr int kSfiSlotK = 64;
struct SfiRoundArgs {
    int n1, n2, k;          // k: list entries per slot
    const int* off;
    const int2* cand;       // (i2, dist) in GetFeaturesInArea order
    long long cand_cap;     // a list ending past it was not filled: read as empty (the host
                            // sees the total exceed the capacity and reruns the call)
    float nnratio;
    int* dec[2];            // round r reads dec[r & 1] (-2 before round 0), writes dec[~r & 1]
    int2* list[3];          // per slot kSfiSlotK acceptors (query, dist)
    int* lcnt[3];           // per slot acceptor count
    int* chg;               // per round: 1 if a decision changed
    int* overflow;          // a slot had more than k acceptors in a round
    int* status;            // a query with 65536+ candidates (ranks do not fit the key)
};

// The rounds' starting state in one launch (three hipMemsetAsync calls before): decisions
// 0xfefefefe (< -1: no decision yet, what round 0 compares against), the first two slot-list
// counts 0, the overflow word and the per-round change flags 0.
__global__ __launch_bounds__(256) void sfi_init_kernel(int* dec0, int nd, int* lcnt, int nl, int* chg, int nc) {
    for (int i = blockIdx.x * 256 + threadIdx.x; i < max(nd, max(nl, nc)); i += gridDim.x * 256) {
        if (i < nd) dec0[i] = (int)0xfefefefe;
        if (i < nl) lcnt[i] = 0;
        if (i < nc) chg[i] = 0;
    }
}

__global__ __launch_bounds__(256) void sfi_round_kernel(SfiRoundArgs a, int r) {
    // A round after a change-free one (the host launches rounds in batches, past convergence)
    // exits before touching anything: it would repeat the converged round's decisions, but it
    // would also clear the list buffer the converged round filled two rounds earlier in the
    // rotation, which the final kernel reads (found by tests/cpp/threads_test.cpp: a problem
    // converging at round 3 of a 6-round batch returned no matches)
    if (r > 0 && a.chg[r - 1] == 0) return;
    const int gid = blockIdx.x * 256 + threadIdx.x;
    if (gid < a.n2) a.lcnt[(r + 2) % 3][gid] = 0;  // the list round r + 1 fills
    const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (i >= a.n1) return;
    const int lane = threadIdx.x & 63;
    const int e0 = a.off[i];
    const int e1 = a.off[i + 1] > a.cand_cap ? e0 : a.off[i + 1];
    if (e1 - e0 >= 65536) {
        if (lane == 0) atomicExch(a.status, ORBFE_ERR_UNSUPPORTED);
        return;
    }
    const int2* Lr = a.list[r % 3];
    const int* Cr = a.lcnt[r % 3];
    uint32_t k1 = 0xffffffffu, k2 = 0xffffffffu;  // this lane's two smallest keys
    for (int e = e0 + lane; e < e1; e += 64) {
        const int2 c = a.cand[e];
        const int n = min(Cr[c.x], a.k);
        int md = INT_MAX;  // vMatchedDistance[i2] as query i sees it
        for (int k = 0; k < n; ++k) {
            const int2 q = Lr[(size_t)c.x * a.k + k];
            if (q.x < i) md = min(md, q.y);
        }
        if (md <= c.y) continue;
        const uint32_t key = ((uint32_t)c.y << 16) | (uint32_t)(e - e0);
        if (key < k1) { k2 = k1; k1 = key; }
        else if (key < k2) { k2 = key; }
    }
    const uint32_t best = __ockl_wfred_min_u32(k1);
    const uint32_t sec = __ockl_wfred_min_u32(k1 == best ? k2 : k1);
    const int bd = best == 0xffffffffu ? INT_MAX : (int)(best >> 16);
    const int sd = sec == 0xffffffffu ? INT_MAX : (int)(sec >> 16);
    const bool acc = bd <= kThLow && (float)bd < (float)sd * a.nnratio;  // 455-456
    if (lane != 0) return;
    const int d = acc ? a.cand[e0 + (int)(best & 0xffff)].x : -1;
    if (d != a.dec[r & 1][i]) a.chg[r] = 1;
    a.dec[~r & 1][i] = d;
    if (d >= 0) {
        const int p = atomicAdd(&a.lcnt[(r + 1) % 3][d], 1);
        if (p < a.k) a.list[(r + 1) % 3][(size_t)d * a.k + p] = make_int2(i, bd);
        else *a.overflow = 1;
    }
}

// The converged state: owners (last acceptor per slot), rotation consistency (492-515),
// nmatches and the vbPrevMatched update (518-520).  One workgroup.
struct SfiFinalArgs {
    int n1, k;
    const orbfe_keypoint* k1;
    const orbfe_keypoint* k2;
    const int* dec;
    const int2* list;
    const int* lcnt;
    int check_ori;
    int* m12;
    int* rotbin;
    float* prev;
    int* nmatches;
};
__global__ __launch_bounds__(1024) void sfi_final_kernel(SfiFinalArgs a) {
    __shared__ int hist[kHistLen];
    __shared__ int top[3];
    __shared__ int nm;
    if (threadIdx.x < kHistLen) hist[threadIdx.x] = 0;
    if (threadIdx.x == 0) nm = 0;
    __syncthreads();
    for (int i = threadIdx.x; i < a.n1; i += 1024) {
        const int d = a.dec[i];
        int own = -1, bin = -1;
        if (d >= 0) {
            int last = -1;
            const int n = min(a.lcnt[d], a.k);
            for (int k = 0; k < n; ++k) last = max(last, a.list[(size_t)d * a.k + k].x);
            if (last == i) own = d;
            if (a.check_ori) {
                bin = rot_bin(a.k1[i].angle, a.k2[d].angle);
                atomicAdd(&hist[bin], 1);
            }
        }
        a.m12[i] = own;
        a.rotbin[i] = bin;
    }
    __syncthreads();
    if (a.check_ori && threadIdx.x == 0) three_maxima(hist, top[0], top[1], top[2]);
    __syncthreads();
    int cnt = 0;
    for (int i = threadIdx.x; i < a.n1; i += 1024) {
        int j = a.m12[i];
        const int b = a.rotbin[i];
        if (j >= 0 && a.check_ori && b != top[0] && b != top[1] && b != top[2]) {
            j = -1;
            a.m12[i] = -1;
        }
        if (j >= 0) {
            ++cnt;
            a.prev[2 * i] = a.k2[j].x;
            a.prev[2 * i + 1] = a.k2[j].y;
        }
    }
    cnt = wave_sum(cnt);
    if ((threadIdx.x & 63) == 0 && cnt) atomicAdd(&nm, cnt);
    __syncthreads();
    if (threadIdx.x == 0) *a.nmatches = nm;
}

// ---------------------------------------------------------------------------------------------
// SearchByProjection(Frame&, const vector<MapPoint*>&, th) (ORBmatcher.cc:45-129)
struct SbpMps {
    int m;
    const uint8_t* in_view;
    const uint8_t* bad;
    const float* px;
    const float* py;
    const float* pxr;
    const int* lvl;
    const float* vcos;
    const uint4* desc;
    const int* nobs;
};

struct SbpLocalArgs {
    DevFrame f;
    SbpMps mp;
    const float* scale;  // per level
    float th;
    int nlevels;         // levels of `scale`; a predicted level outside is UB in the reference
    int* status;         // NULL, or set to ORBFE_ERR_UNSUPPORTED for such a point
    long long cand_cap;  // fill writes only lists that end within the capacity
    int* cnt;
    const int* off;
    int2* cand;          // (idx, dist | octave << 16)
    int kfix;            // kMode 2: candidate slots per point
    int* ovf;            // kMode 2: points with more candidates than kfix
};

// kMode 0: count, 1: fill the CSR lists, 2: fixed slots in one pass (the first kfix candidates at
// i * kfix, min(n, kfix) in cnt[i]; a point with more raises *ovf).  One wave per map point
// (features_in_area_wave): one thread per point (features_in_area, round 5) left a 2,000-point
// map 8 workgroups walking their windows serially (0.17 ms of kernel; the host call 0.252 ->
// 0.097 ms) and was slower at 50,000 points too (the host call 0.41 -> 0.32 ms).
template <int kMode>
__global__ __launch_bounds__(256) void sbp_local_cand_kernel(SbpLocalArgs a) {
    constexpr bool FILL = kMode == 1;
    const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (i >= a.mp.m) return;
    const bool lead = (threadIdx.x & 63) == 0;  // the lane that writes the point's words
    if (!a.mp.in_view[i] || a.mp.bad[i]) {
        if (!FILL && lead) a.cnt[i] = 0;
        return;
    }
    const int pl = a.mp.lvl[i];
    if (pl < 0 || pl >= a.nlevels) {  // F.mvScaleFactors[nPredictedLevel] out of range
        if (a.status && lead) atomicExch(a.status, ORBFE_ERR_UNSUPPORTED);
        if (!FILL && lead) a.cnt[i] = 0;
        return;
    }
    float r = a.mp.vcos[i] > 0.998 ? 2.5f : 4.0f;  // RadiusByViewingCos (131-137)
    if (a.th != 1.0) r *= a.th;
    const float rs = r * a.scale[pl];
    const float pxr = a.mp.pxr[i];
    if (FILL && a.off[i + 1] > a.cand_cap) return;
    const uint4 q0 = a.mp.desc[2 * i], q1 = a.mp.desc[2 * i + 1];
    int n = 0;
    int2* out = FILL ? a.cand + a.off[i] : kMode == 2 ? a.cand + (size_t)i * a.kfix : nullptr;
    n = features_in_area_wave(
        a.f, a.mp.px[i], a.mp.py[i], rs, pl - 1, pl,
        [&](int idx) {  // stereo consistency (91-96)
            return !(a.f.ur && a.f.ur[idx] > 0 && fabsf(pxr - a.f.ur[idx]) > r * a.scale[pl]);
        },
        [&](int idx, int rank) {
            if (FILL || (kMode == 2 && rank < a.kfix)) {
                const uint4* d = a.f.desc + 2 * idx;
                out[rank] = make_int2(idx, hamming256(q0, q1, d[0], d[1]) | (a.f.k[idx].octave << 16));
            }
        });
    if (kMode == 0 && lead) a.cnt[i] = n;
    if (kMode == 2 && lead) {
        a.cnt[i] = min(n, a.kfix);
        if (n > a.kfix) atomicAdd(a.ovf, 1);
    }
}

// ---------------------------------------------------------------------------------------------
// SearchByProjection(Frame& Cur, const Frame& Last, th, bMono) (ORBmatcher.cc:1331-1473)
struct SbpLastArgs {
    DevFrame cur;
    int n_last;
    const orbfe_keypoint* lk;
    const uint8_t* valid;
    const uint8_t* outlier;
    const float* xyz;
    const uint4* desc;
    float T[12];           // current pose [R|t]
    float fx, fy, cx, cy, bf;
    float minx, maxx, miny, maxy;
    const float* scale;
    float th;
    int mode;              // 0: [o-1, o+1], 1: forward [o, -], 2: backward [0, o]
    long long cand_cap;
    int* cnt;
    const int* off;
    int2* cand;
    int kfix;                 // kMode 2: candidate slots per point
    int* ovf;                 // kMode 2: points with more candidates than kfix
};

// kMode as sbp_kf_cand_kernel's: 0 count, 1 fill the CSR lists, 2 fixed slots in one pass
template <int kMode>
__global__ __launch_bounds__(256) void sbp_last_cand_kernel(SbpLastArgs a) {
    constexpr bool FILL = kMode == 1;
    const int i = blockIdx.x * 4 + (threadIdx.x >> 6);  // one wave per last-frame point
    if (i >= a.n_last) return;
    // Inputs read up front, as in sbp_kf_cand_kernel.
    const bool room = !FILL || a.off[i + 1] <= a.cand_cap;
    const bool live = a.valid[i] && !a.outlier[i];
    const float P[3] = {a.xyz[3 * i], a.xyz[3 * i + 1], a.xyz[3 * i + 2]};
    const int o = a.lk[i].octave;
    if (!room) return;
    int n = 0;
    {
        float pc[3];
#pragma unroll
        for (int r = 0; r < 3; ++r)
            pc[r] = ((a.T[4 * r] * P[0] + a.T[4 * r + 1] * P[1]) + a.T[4 * r + 2] * P[2]) + a.T[4 * r + 3];
        const float invz = (float)(1.0 / (double)pc[2]);
        const float u = a.fx * pc[0] * invz + a.cx;
        const float v = a.fy * pc[1] * invz + a.cy;
        if (live && !(invz < 0) && !(u < a.minx || u > a.maxx) && !(v < a.miny || v > a.maxy)) {
            const float radius = a.th * a.scale[o];
            const int lo = a.mode == 0 ? o - 1 : a.mode == 1 ? o : 0;
            const int hi = a.mode == 0 ? o + 1 : a.mode == 1 ? -1 : o;
            const uint4 q0 = a.desc[2 * i], q1 = a.desc[2 * i + 1];
            int2* out = FILL ? a.cand + a.off[i] : kMode == 2 ? a.cand + (size_t)i * a.kfix : nullptr;
            const float ur = u - a.bf * invz;
            n = features_in_area_wave(
                a.cur, u, v, radius, lo, hi,
                [&](int i2) { return !(a.cur.ur && a.cur.ur[i2] > 0 && fabsf(ur - a.cur.ur[i2]) > radius); },
                [&](int i2, int rank) {
                    if (FILL || (kMode == 2 && rank < a.kfix)) {
                        const uint4* d = a.cur.desc + 2 * i2;
                        out[rank] = make_int2(i2, hamming256(q0, q1, d[0], d[1]));
                    }
                });
        }
    }
    if (kMode == 0 && (threadIdx.x & 63) == 0) a.cnt[i] = n;
    if (kMode == 2 && (threadIdx.x & 63) == 0) {
        a.cnt[i] = min(n, a.kfix);
        if (n > a.kfix) atomicAdd(a.ovf, 1);
    }
}

// ---------------------------------------------------------------------------------------------
// Relocalisation SearchByProjection(Frame&, KeyFrame*, sAlreadyFound, th, ORBdist)
// (ORBmatcher.cc:1475-1602): candidates of every keyframe map point in parallel; the greedy
// assignment (a slot taken by an earlier map point blocks later ones, 1529-1530) is resolved
// by orbfe_greedy.hip with every held point blocking and max_dist = ORBdist.
struct SbpKfArgs {
    DevFrame cur;
    int n;
    const uint8_t* valid;     // GetMapPointMatches()[i] != NULL
    const uint8_t* bad;       // isBad()
    const uint8_t* found;     // sAlreadyFound.count()
    const float* xyz;
    const float* mind;        // mfMinDistance
    const float* maxd;        // mfMaxDistance
    const uint4* desc;
    float T[12];
    float ow[3];              // -Rcw^T tcw (host, double accumulation)
    float fx, fy, cx, cy;
    float minx, maxx, miny, maxy;
    const float* scale;
    int nlevels;
    float log_scale, th;
    int* status;
    long long cand_cap;
    int* cnt;
    const int* off;
    int2* cand;
    int kfix;                 // kMode 2: candidate slots per point
    int* ovf;                 // kMode 2: points with more candidates than kfix
};

// kMode 0: count the candidates, 1: fill the CSR lists (after the scan), 2: the fixed-slot form
// in one pass — the first kfix candidates of point i at i * kfix, min(n, kfix) in cnt[i], and a
// point with more raises *ovf (the host then reruns the call on the CSR path).
template <int kMode>
__global__ __launch_bounds__(256) void sbp_kf_cand_kernel(SbpKfArgs a) {
    constexpr bool FILL = kMode == 1;
    const int i = blockIdx.x * 4 + (threadIdx.x >> 6);  // one wave per keyframe map point
    if (i >= a.n) return;
    // Every per-point input is read up front and feeds the unconditional arithmetic below, so
    // the loads issue together instead of one flag test (and one memory round trip) at a time.
    const bool room = !FILL || a.off[i + 1] <= a.cand_cap;
    const bool live = a.valid[i] && !a.bad[i] && !a.found[i];
    const float P[3] = {a.xyz[3 * i], a.xyz[3 * i + 1], a.xyz[3 * i + 2]};
    const float maxd = a.maxd[i], mind = a.mind[i];
    if (!room) return;
    int n = 0;
    {
        float pc[3];
#pragma unroll
        for (int r = 0; r < 3; ++r)
            pc[r] = ((a.T[4 * r] * P[0] + a.T[4 * r + 1] * P[1]) + a.T[4 * r + 2] * P[2]) + a.T[4 * r + 3];
        const float invz = (float)(1.0 / (double)pc[2]);  // 1.0/x3Dc.at<float>(2): double divide
        const float u = a.fx * pc[0] * invz + a.cx;
        const float v = a.fy * pc[1] * invz + a.cy;
        const float po0 = P[0] - a.ow[0], po1 = P[1] - a.ow[1], po2 = P[2] - a.ow[2];
        const float dist = (float)sqrt((double)po0 * po0 + (double)po1 * po1 + (double)po2 * po2);
        const float dmax = 1.2f * maxd, dmin = 0.8f * mind;  // MapPoint.cc:621-631
        const bool ok = live && !(u < a.minx || u > a.maxx) && !(v < a.miny || v > a.maxy) &&
                        !(dist < dmin || dist > dmax);
        if (ok) {
            const float ratio = maxd / dist;
            const int lvl = (int)ceilf((float)log((double)ratio) / a.log_scale);
            if (lvl < 0 || lvl >= a.nlevels) {
                if ((threadIdx.x & 63) == 0) atomicExch(a.status, ORBFE_ERR_UNSUPPORTED);  // mvScaleFactors[lvl]
            } else {
                const float radius = a.th * a.scale[lvl];
                const uint4 q0 = a.desc[2 * i], q1 = a.desc[2 * i + 1];
                int2* out = FILL ? a.cand + a.off[i] : kMode == 2 ? a.cand + (size_t)i * a.kfix : nullptr;
                n = features_in_area_wave(
                    a.cur, u, v, radius, lvl - 1, lvl + 1, [](int) { return true; },
                    [&](int i2, int rank) {
                        if (FILL || (kMode == 2 && rank < a.kfix)) {
                            const uint4* d = a.cur.desc + 2 * i2;
                            out[rank] = make_int2(i2, hamming256(q0, q1, d[0], d[1]));
                        }
                    });
            }
        }
    }
    if (kMode == 0 && (threadIdx.x & 63) == 0) a.cnt[i] = n;
    if (kMode == 2 && (threadIdx.x & 63) == 0) {
        a.cnt[i] = min(n, a.kfix);
        if (n > a.kfix) atomicAdd(a.ovf, 1);
    }
}

// ---------------------------------------------------------------------------------------------
// MapPoint::ComputeDistinctiveDescriptors (MapPoint.cc:483-548): one wave per map point.  Lane
// i owns observation i (i = lane, lane + 64, ...); the median of its distance row
// (sorted row[(size_t)(0.5 (N-1))], self distance 0 included) is the smallest v with
// #{j : d(i, j) <= v} > (N-1)/2, found by bisection over v in [0, 256] with the row recomputed
// from the descriptors (staged in LDS when N <= kDdStage).  The winner is the first i with the
// smallest median: min over (median << 16 | i).
constexpr int kDdBlock = 256;
constexpr int kDdStage = 64;  // descriptors per wave staged in LDS
__global__ __launch_bounds__(kDdBlock) void distinctive_kernel(int n_mp, const int* off,
                                                               const uint4* desc, int* best,
                                                               uint4* desc_out) {
    __shared__ uint4 s_d[kDdBlock / 64][2 * kDdStage];
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int mp = blockIdx.x * (kDdBlock / 64) + wid;
    if (mp >= n_mp) return;
    const int o = off[mp], N = off[mp + 1] - o;
    if (N <= 0) {
        if (lane == 0) best[mp] = -1;
        return;
    }
    const uint4* d = desc + 2 * (size_t)o;
    const bool staged = N <= kDdStage;
    if (staged) {
        for (int k = lane; k < 2 * N; k += 64) s_d[wid][k] = d[k];
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    }
    const uint4* src = staged ? s_d[wid] : d;
    const int k = (int)(0.5 * (double)(N - 1));  // vDists[0.5*(N-1)]
    uint32_t key = 0xffffffffu;
    for (int i = lane; i < N; i += 64) {
        const uint4 a0 = src[2 * i], a1 = src[2 * i + 1];
        int lo = 0, hi = 256;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            int c = 0;
            for (int j = 0; j < N; ++j) c += hamming256(a0, a1, src[2 * j], src[2 * j + 1]) <= mid;
            if (c > k) hi = mid; else lo = mid + 1;
        }
        key = min(key, ((uint32_t)lo << 16) | (uint32_t)i);
    }
#pragma unroll
    for (int s = 32; s > 0; s >>= 1) key = min(key, (uint32_t)__shfl_xor((int)key, s, 64));
    const int bi = (int)(key & 0xffff);
    if (lane == 0) best[mp] = bi;
    if (desc_out && lane < 2) desc_out[2 * (size_t)mp + lane] = d[2 * bi + lane];
}

// ---------------------------------------------------------------------------------------------
// Frame::isInFrustum (Frame.cc:387-443) with MapPoint::PredictScale (MapPoint.cc:633-642).
struct FrustumArgs {
    int n;
    const float* xyz;
    const float* normal;
    const float* mind;
    const float* maxd;
    float T[12];
    float ow[3];   // camera centre -R^T t (computed on the host, double accumulation)
    float fx, fy, cx, cy, bf;
    float minx, maxx, miny, maxy, log_scale, cos_limit;
    uint8_t* in_view;
    float* px;
    float* py;
    float* pxr;
    int* lvl;
    float* vcos;
    // Tracking::SearchLocalPoints (Tracking.cc:1403-1438): points already matched in the frame
    // (skip) get mbTrackInView = false, bad points are not projected; in-view points are
    // counted (nToMatch).  All NULL for the plain isInFrustum entry point.
    const uint8_t* skip;
    const uint8_t* bad;
    int* n_in_view;
};

struct FrustumOut {
    float u, ur, v, vc;
    int lvl;
};
// Frame::isInFrustum (Frame.cc:387-443) + MapPoint::PredictScale (MapPoint.cc:633-642) of point
// i into registers; false when not in view.  Writes nothing.  Every input of the point (the skip
// and bad flags, position, distances, normal) is loaded at once and the tests are evaluated
// together: the reference's early returns had put five dependent global round trips in front of
// the answer.  The tests and their order of evaluation are the reference's; a point failing one
// computes the others for nothing (about 10 % of a local map).
__device__ uint8_t g_zero_u8;
__device__ __forceinline__ bool frustum_eval(const FrustumArgs& a, int i, FrustumOut& o) {
    const uint8_t sk = *(a.skip ? a.skip + i : &g_zero_u8);
    const uint8_t bd = *(a.bad ? a.bad + i : &g_zero_u8);
    const float* P = a.xyz + 3 * i;
    const float* nv = a.normal + 3 * i;
    const float P0 = P[0], P1 = P[1], P2 = P[2];
    const float n0 = nv[0], n1 = nv[1], n2 = nv[2];
    const float maxd = a.maxd[i], mind = a.mind[i];
    const float Pv[3] = {P0, P1, P2};
    float pc[3];
#pragma unroll
    for (int r = 0; r < 3; ++r)
        pc[r] = ((a.T[4 * r] * Pv[0] + a.T[4 * r + 1] * Pv[1]) + a.T[4 * r + 2] * Pv[2]) + a.T[4 * r + 3];
    const float invz = 1.0f / pc[2];
    const float u = a.fx * pc[0] * invz + a.cx;
    const float v = a.fy * pc[1] * invz + a.cy;
    const float dmax = 1.2f * maxd, dmin = 0.8f * mind;
    const float po0 = P0 - a.ow[0], po1 = P1 - a.ow[1], po2 = P2 - a.ow[2];
    const float dist = (float)sqrt((double)po0 * po0 + (double)po1 * po1 + (double)po2 * po2);
    const double dot = (double)po0 * n0 + (double)po1 * n1 + (double)po2 * n2;
    const float vc = (float)(dot / dist);
    const bool in = !sk && !bd && !(pc[2] < 0.0f) && !(u < a.minx || u > a.maxx) &&
                    !(v < a.miny || v > a.maxy) && !(dist < dmin || dist > dmax) && !(vc < a.cos_limit);
    if (!in) return false;
    const float ratio = maxd / dist;
    o.lvl = (int)ceilf((float)log((double)ratio) / a.log_scale);
    o.u = u;
    o.ur = u - a.bf * invz;
    o.v = v;
    o.vc = vc;
    return true;
}

__device__ __forceinline__ bool frustum_point(const FrustumArgs& a, int i) {
    FrustumOut o;
    const bool in = frustum_eval(a, i, o);
    a.in_view[i] = in ? 1 : 0;  // isInFrustum starts with mbTrackInView = false (Frame.cc:389)
    if (!in) return false;
    a.px[i] = o.u;
    a.pxr[i] = o.ur;
    a.py[i] = o.v;
    a.lvl[i] = o.lvl;
    a.vcos[i] = o.vc;
    return true;
}

__global__ __launch_bounds__(256) void frustum_kernel(FrustumArgs a) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    bool in = false;
    if (i < a.n) in = frustum_point(a, i);
    if (a.n_in_view) {
        const unsigned long long b = __ballot(in);
        if ((threadIdx.x & 63) == 0 && b) atomicAdd(a.n_in_view, __popcll(b));
    }
}

}  // namespace orbfe
