// orbfe_stereo.hip — MI355X (gfx950) replacement for Frame::ComputeStereoMatches
// (skaegy/ORBSLAM_MapSave src/Frame.cc:584-756): the rectified-stereo matcher that runs on
// every stereo frame right after the two extractors (Frame.cc:78-81 -> 103).
//
//   S1 stereo_rows_kernel    the row table vRowIndices (591-606) as a per-frame CSR built in
//                            LDS (count, scan, fill); one workgroup per frame
//   S2 stereo_match_kernel   one wave per left keypoint: the band candidates in lanes with
//                            Hamming distances (617-660), lexicographic (distance, iR) minimum
//                            = the reference's first-wins strict '<' over ascending iR; then
//                            the 11 x 11 SAD sliding window over +-5 px on the keypoint's
//                            pyramid level (663-706), parabola fit and depth (708-735)
//   S3 stereo_filter_kernel  the median rule over accepted SADs (738-755): a two-pass byte
//                            histogram select of the (n/2)-th smallest SAD, then every
//                            match with SAD >= 1.5f*1.4f*median is dropped
//
// All window arithmetic is integer-valued (|diffs| <= 510, sums < 2^24), so the float SADs of
// the reference are exact; the parabola fit, disparity and depth follow its float expression
// order operation by operation (-ffp-contract=off).
#include <hip/hip_runtime.h>

#include <climits>

#include "../../include/orbfe.h"
#include "orbfe_device.hpp"
#include "orbfe_internal.hpp"

namespace orbfe {

constexpr int kStereoThHigh = kThHigh;  // ORBmatcher::TH_HIGH (ORBmatcher.cc:37)
constexpr int kStereoW = 5;         // window half size w (Frame.cc:672)
constexpr int kStereoL = 5;         // search half range L (Frame.cc:680)
constexpr int kStereoRowsBlock = 1024;
constexpr int kStereoMaxRows = 4096;  // images are limited to 4096 rows

struct StereoArgs {
    int nrows, row_cap, kps_cap, nlevels;
    const orbfe_keypoint* kl;
    const uint4* dl;
    const int* nl;
    const orbfe_keypoint* kr;
    const uint4* dr;
    const int* nr;
    float scale[kMaxLevels], inv[kMaxLevels];
    LevelPtr pl[kMaxLevels], pr[kMaxLevels];
    int lw[kMaxLevels], lh[kMaxLevels];
    float bf, b;
    int* row_off;    // [frame][nrows + 1]
    int* row_items;  // [frame][kps_cap * row_cap]
    float* u_right;  // [frame][kps_cap]
    float* depth;    // [frame][kps_cap]
    int* sad;        // [frame][kps_cap]: SAD of an accepted match, else -1
    int* status;     // ORBFE_ERR_UNSUPPORTED when an input hits the reference's UB / asserts
};

// Rows of right keypoint k: floor(y - r) .. ceil(y + r), r = 2 * mvScaleFactors[octave]
// (Frame.cc:600-605).
__device__ __forceinline__ void stereo_rows_of(const StereoArgs& a, const orbfe_keypoint& k,
                                               int& r0, int& r1) {
    const int oct = min(max(k.octave, 0), a.nlevels - 1);
    const float r = 2.0f * a.scale[oct];
    r1 = (int)ceilf(k.y + r);
    r0 = (int)floorf(k.y - r);
}

__global__ __launch_bounds__(kStereoRowsBlock) void stereo_rows_kernel(StereoArgs a) {
    __shared__ int cnt[kStereoMaxRows + 1];
    __shared__ int tmp[kStereoRowsBlock / 64];
    const int f = blockIdx.x;
    const int nr = min(a.nr[f], a.kps_cap);
    const orbfe_keypoint* kr = a.kr + (size_t)f * a.kps_cap;
    const int R = a.nrows;
    for (int y = threadIdx.x; y <= R; y += kStereoRowsBlock) cnt[y] = 0;
    __syncthreads();
    for (int i = threadIdx.x; i < nr; i += kStereoRowsBlock) {
        int r0, r1;
        stereo_rows_of(a, kr[i], r0, r1);
        if (r0 < 0 || r1 >= R || kr[i].octave < 0 || kr[i].octave >= a.nlevels) {
            atomicExch(a.status, ORBFE_ERR_UNSUPPORTED);  // vRowIndices[yi] out of range
            continue;
        }
        for (int y = r0; y <= r1; ++y) atomicAdd(&cnt[y], 1);
    }
    __syncthreads();
    // exclusive scan: each thread owns a run of consecutive rows
    const int per = (R + kStereoRowsBlock - 1) / kStereoRowsBlock;
    const int y0 = threadIdx.x * per, y1 = min(R, y0 + per);
    int run = 0;
    for (int y = y0; y < y1; ++y) run += cnt[y];
    int total;
    int pre = block_exclusive_scan<kStereoRowsBlock>(run, tmp, total);
    int* off = a.row_off + (size_t)f * (R + 1);
    for (int y = y0; y < y1; ++y) {
        const int c = cnt[y];
        off[y] = pre;
        cnt[y] = pre;  // becomes the row's fill cursor
        pre += c;
    }
    if (threadIdx.x == 0) off[R] = total;
    __syncthreads();
    int* items = a.row_items + (size_t)f * a.kps_cap * a.row_cap;
    for (int i = threadIdx.x; i < nr; i += kStereoRowsBlock) {
        int r0, r1;
        stereo_rows_of(a, kr[i], r0, r1);
        if (r0 < 0 || r1 >= R || kr[i].octave < 0 || kr[i].octave >= a.nlevels) continue;
        for (int y = r0; y <= r1; ++y) items[atomicAdd(&cnt[y], 1)] = i;
    }
}

constexpr int kStereoBlock = 256;  // 4 waves, one left keypoint per wave

__global__ __launch_bounds__(kStereoBlock) void stereo_match_kernel(StereoArgs a) {
    __shared__ uint8_t s_il[kStereoBlock / 64][121];
    __shared__ uint8_t s_ir[kStereoBlock / 64][11 * 21];
    __shared__ int s_part[kStereoBlock / 64][11 * 11];
    const int f = blockIdx.y;
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int il = blockIdx.x * (kStereoBlock / 64) + wid;
    const int nl = min(a.nl[f], a.kps_cap);
    if (il >= nl) return;
    const size_t fo = (size_t)f * a.kps_cap;
    float* ur_out = a.u_right + fo;
    float* dp_out = a.depth + fo;
    int* sad_out = a.sad + fo;
    const orbfe_keypoint kpl = a.kl[fo + il];
    const int level_l = kpl.octave;
    const float vl = kpl.y, ul = kpl.x;
    // defaults of 586-587; a rejected keypoint keeps them
    if (lane == 0) {
        ur_out[il] = -1.0f;
        dp_out[il] = -1.0f;
        sad_out[il] = -1;
    }
    const int R = a.nrows;
    if (!(vl >= 0.f) || (int)vl >= R || level_l < 0 || level_l >= a.nlevels) {
        if (lane == 0) atomicExch(a.status, ORBFE_ERR_UNSUPPORTED);
        return;
    }
    const int row = (int)vl;  // vRowIndices[vL]: float -> size_t truncation
    const int* off = a.row_off + (size_t)f * (R + 1);
    const int c0 = off[row], c1 = off[row + 1];
    if (c0 == c1) return;
    const float min_z = a.b, min_d = -3.f, max_d = a.bf / min_z;  // 609-611
    const float min_u = ul - max_d, max_u = ul - min_d;
    if (max_u < 0) return;
    // candidates (641-660): key = dist << 16 | iR, min over the band == first-wins over ascending iR
    const uint4* dl = a.dl + 2 * (fo + il);
    const uint4 q0 = dl[0], q1 = dl[1];
    const int* items = a.row_items + fo * a.row_cap;
    const orbfe_keypoint* kr = a.kr + fo;
    const uint4* dr = a.dr + 2 * fo;
    uint32_t best = (uint32_t)kStereoThHigh << 16;
    for (int c = c0 + lane; c < c1; c += 64) {
        const int ir = items[c];
        const orbfe_keypoint kpr = kr[ir];
        if (kpr.octave < level_l - 1 || kpr.octave > level_l + 1) continue;
        const float ur = kpr.x;
        if (ur >= min_u && ur <= max_u) {
            const int d = hamming256(q0, q1, dr[2 * ir], dr[2 * ir + 1]);
            best = min(best, ((uint32_t)d << 16) | (uint32_t)ir);
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) best = min(best, (uint32_t)__shfl_xor((int)best, o, 64));
    if ((best >> 16) >= (uint32_t)kStereoThHigh) return;
    const int best_ir = (int)(best & 0xffff);
    // sub-pixel match by correlation (663-706)
    const float ur0 = kr[best_ir].x;
    const float sf = a.inv[level_l];
    const float sul = roundf(kpl.x * sf), svl = roundf(kpl.y * sf);
    const float sur0 = roundf(ur0 * sf);
    const int W5 = kStereoW, L5 = kStereoL;
    const int lw = a.lw[level_l], lh = a.lh[level_l];
    const int r0 = (int)(svl - W5), cl0 = (int)(sul - W5);
    if (r0 < 0 || r0 + 2 * W5 + 1 > lh || cl0 < 0 || cl0 + 2 * W5 + 1 > lw) {
        if (lane == 0) atomicExch(a.status, ORBFE_ERR_UNSUPPORTED);  // rowRange/colRange assert
        return;
    }
    const float iniu = sur0 + L5 - W5, endu = sur0 + L5 + W5 + 1;  // 684-687
    if (iniu < 0 || endu >= lw) return;
    const int cr0 = (int)(sur0 - L5 - W5);
    if (cr0 < 0 || cr0 + 2 * (L5 + W5) + 1 > lw) {
        if (lane == 0) atomicExch(a.status, ORBFE_ERR_UNSUPPORTED);
        return;
    }
    const LevelPtr PL = a.pl[level_l], PR = a.pr[level_l];
    const uint8_t* bl = PL.base + f * PL.fpitch + (long long)r0 * PL.pitch + cl0;
    const uint8_t* br = PR.base + f * PR.fpitch + (long long)r0 * PR.pitch + cr0;
    uint8_t* sil = s_il[wid];
    uint8_t* sir = s_ir[wid];
    int* part = s_part[wid];
    for (int i = lane; i < 121; i += 64) sil[i] = bl[(i / 11) * PL.pitch + i % 11];
    for (int i = lane; i < 231; i += 64) sir[i] = br[(i / 21) * PR.pitch + i % 21];
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    const int ilc = sil[5 * 11 + 5];
    for (int qd = lane; qd < 121; qd += 64) {
        const int inc = qd / 11, y = qd % 11;  // inc 0..10 <-> incR -5..5
        const int irc = sir[5 * 21 + 5 + inc];
        int s = 0;
#pragma unroll
        for (int x = 0; x < 11; ++x) s += abs((sil[y * 11 + x] - ilc) - (sir[y * 21 + x + inc] - irc));
        part[qd] = s;
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    if (lane != 0) return;
    float dists[2 * kStereoL + 1];
    int best_sad = INT_MAX, best_inc = 0;
    for (int k = 0; k <= 2 * L5; ++k) {
        int s = 0;
        for (int y = 0; y < 11; ++y) s += part[k * 11 + y];
        const float dist = (float)s;
        if (dist < best_sad) {
            best_sad = (int)dist;
            best_inc = k - L5;
        }
        dists[k] = dist;
    }
    if (best_inc == -L5 || best_inc == L5) return;
    // parabola fitting (708-716)
    const float d1 = dists[L5 + best_inc - 1], d2 = dists[L5 + best_inc], d3 = dists[L5 + best_inc + 1];
    const float delta = (d1 - d3) / (2.0f * (d1 + d3 - 2.0f * d2));
    if (delta < -1 || delta > 1) return;
    float best_ur = a.scale[level_l] * ((float)sur0 + (float)best_inc + delta);
    float disparity = (ul - best_ur);
    if (disparity >= 0 && disparity < max_d) {
        if (disparity <= 0) {
            disparity = 0.01;            // double literal -> float
            best_ur = (float)((double)ul - 0.01);  // uL - 0.01 evaluated in double
        }
        dp_out[il] = a.bf / disparity;
        ur_out[il] = best_ur;
        sad_out[il] = best_sad;
    }
}

// S3 — median filter (738-755).  SADs are < 2^16 (121 * 510), so the (n/2)-th smallest is
// found with a high-byte then a low-byte histogram.
constexpr int kStereoFilterBlock = 1024;
__global__ __launch_bounds__(kStereoFilterBlock) void stereo_filter_kernel(StereoArgs a) {
    __shared__ int hist[256];
    __shared__ int s_sel[2];
    const int f = blockIdx.x;
    const int nl = min(a.nl[f], a.kps_cap);
    const size_t fo = (size_t)f * a.kps_cap;
    const int* sad = a.sad + fo;
    if (threadIdx.x < 256) hist[threadIdx.x] = 0;
    __syncthreads();
    for (int i = threadIdx.x; i < nl; i += kStereoFilterBlock) {
        const int s = sad[i];
        if (s >= 0) atomicAdd(&hist[s >> 8], 1);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        int n = 0;
        for (int b = 0; b < 256; ++b) n += hist[b];
        int k = n / 2, bin = -1;
        if (n > 0) {
            for (bin = 0; bin < 256; ++bin) {
                if (k < hist[bin]) break;
                k -= hist[bin];
            }
        }
        s_sel[0] = bin;
        s_sel[1] = k;
    }
    __syncthreads();
    const int bin = s_sel[0];
    if (bin < 0) return;  // no accepted match: nothing to filter (vDistIdx empty)
    if (threadIdx.x < 256) hist[threadIdx.x] = 0;
    __syncthreads();
    for (int i = threadIdx.x; i < nl; i += kStereoFilterBlock) {
        const int s = sad[i];
        if (s >= 0 && (s >> 8) == bin) atomicAdd(&hist[s & 255], 1);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        int k = s_sel[1], lo = 0;
        for (lo = 0; lo < 256; ++lo) {
            if (k < hist[lo]) break;
            k -= hist[lo];
        }
        s_sel[0] = (bin << 8) | lo;
    }
    __syncthreads();
    const float median = (float)s_sel[0];
    const float th_dist = 1.5f * 1.4f * median;
    for (int i = threadIdx.x; i < nl; i += kStereoFilterBlock) {
        const int s = sad[i];
        if (s >= 0 && !((float)s < th_dist)) {
            a.u_right[fo + i] = -1.0f;
            a.depth[fo + i] = -1.0f;
        }
    }
}

}  // namespace orbfe
