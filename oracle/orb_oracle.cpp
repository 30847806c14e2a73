// orb_oracle.cpp — TEST INFRASTRUCTURE ONLY: the CPU parity oracle and the timed CPU baseline.
//
// A from-scratch C++17 restatement of the reference hot path:
//   * ORBextractor (skaegy/ORBSLAM_MapSave src/ORBextractor.cc) — pyramid, per-cell FAST with
//     threshold fallback, oct-tree distribution, IC angle, Gaussian blur, rBRIEF;
//   * the OpenCV 3.3.1 primitives it calls (cv::resize INTER_LINEAR 8U, cv::FAST TYPE_9_16,
//     cv::GaussianBlur 7x7 sigma 2 REFLECT_101, cv::fastAtan2, cvRound) — SURVEY.md App. A;
//   * ORBmatcher::DescriptorDistance / SearchForInitialization / SearchByProjection x2 and the
//     Frame grid (src/ORBmatcher.cc, src/Frame.cc), Frame::isInFrustum + PredictScale.
// Each function cites the reference lines it follows.  Loaded only by tests/, by
// __graft_entry__.smoke() and by bench.py's cpu_baseline leg — never by the product library.
//
// PARITY UNPINNED (no reference build and no reference fixtures exist; DESIGN.md "Oracle").
// Semantic choices where upstream behaviour is build-dependent:
//   H2  oct-tree phase-2 ties between equal-size nodes: higher creation sequence first
//       (stands in for the heap address in pair<int, ExtractorNode*>);
//   H3  fastAtan2: float polynomial, no FMA contraction (built with -ffp-contract=off);
//   H4  descriptor rotation: a=(float)cos((double)ang), b=(float)sin((double)ang), no FMA;
//   H5  resize: scalar FixedPtCast<int,uchar,22> vertical pass everywhere;
//   H6  blur: integer 8U smooth path ((sum + 2^15) >> 16) everywhere (no IPP, no float SIMD);
//   H8  PredictScale log: (float)log((double)ratio), i.e. correctly rounded logf.
// oracle_set_variant switches to the other build-dependent readings (H2 heap-address order,
// H4 glibc cosf/sinf and FMA contraction, H5 SSE2 resize rounding, H6 SIMD blur rounding) for
// the residual study only (oracle/residuals.py); the GPU is checked against variant 0.
#include "orb_oracle.h"

#include <algorithm>
#include <cfloat>
#include <climits>
#include <cmath>
#include <cstring>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <string>
#include <list>
#include <thread>
#include <vector>

namespace {

// ---------------------------------------------------------------------------------------------
// OpenCV scalar helpers (App. A.5): cvRound = round half to even under the default MXCSR.
inline int cv_round(float v) { return (int)std::lrintf(v); }
inline int cv_round(double v) { return (int)std::lrint(v); }
inline int cv_floor(float v) { return (int)std::floor(v); }
inline short sat_short(float v) {
    int iv = cv_round(v);
    return (short)std::min(std::max(iv, (int)SHRT_MIN), (int)SHRT_MAX);
}
inline uint8_t sat_u8(int v) { return (uint8_t)std::min(std::max(v, 0), 255); }

// Build-dependent readings for the residual study; 0 = the pinned oracle.
enum {
    kVarH2Addr = 1,   // oct-tree phase-2 ties by real heap address (ORBextractor.cc:680-683)
    kVarH4Cosf = 2,   // rBRIEF rotation with glibc cosf / sinf (std::cos(float), 111-112)
    kVarH4Fma = 4,    // ... and x*b + y*a contracted as GCC -O3 -march=<FMA host> does (117-119)
    kVarH5Sse2 = 8,   // resize vertical pass: OpenCV's SSE2 VResizeLinearVec_32s8u body
    kVarH6Simd = 16,  // blur column pass: OpenCV's SSE2 SymmColumnVec_32s8u (float) body
};
// The default reading is the reference's x86-64 build: SSE2 resize / blur bodies
// and the FMA-contracted rotation; 0 is OpenCV's portable scalar reading.
int g_variant = kVarH4Fma | kVarH5Sse2 | kVarH6Simd;

// Pixels [0, n) of a row that OpenCV 3.3's SSE2 vertical kernels produce (the rest goes to
// the scalar tail): VResizeLinearVec_32s8u runs 16-pixel steps while x <= w - 16, then 4-pixel
// steps while x < w - 4; SymmColumnVec_32s8u runs 16-pixel steps while i <= w - 16, then
// 4-pixel steps while i <= w - 4.
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
inline int sat_s16(int v) { return std::min(std::max(v, -32768), 32767); }

const int kPatchSize = 31;      // PATCH_SIZE      (ORBextractor.cc:71)
const int kHalfPatch = 15;      // HALF_PATCH_SIZE (ORBextractor.cc:72)
const int kEdge = 19;           // EDGE_THRESHOLD  (ORBextractor.cc:73)
const int kMaxLevels = 32;

const int kPattern[1024] = {
#include "../include/orbfe_pattern.inc"
};

// ---------------------------------------------------------------------------------------------
// A1 — ORBextractor ctor tables (ORBextractor.cc:409-469).
struct Tables {
    int nfeatures = 0, nlevels = 0, ini_th = 0, min_th = 0;
    double scale_d = 1.0;  // the `double scaleFactor` member (ORBextractor.h:103)
    float scale[kMaxLevels], inv[kMaxLevels], sigma2[kMaxLevels], inv_sigma2[kMaxLevels];
    int nfeat[kMaxLevels];
    int umax[kHalfPatch + 1];
};

bool make_tables(const orbfe_params* p, Tables& t) {
    if (!p || p->nlevels < 1 || p->nlevels > kMaxLevels || p->nfeatures < 0 ||
        !(p->scale_factor > 1.0f))
        return false;
    t.nfeatures = p->nfeatures;
    t.nlevels = p->nlevels;
    t.ini_th = p->ini_th_fast;
    t.min_th = p->min_th_fast;
    t.scale_d = (double)p->scale_factor;
    t.scale[0] = 1.0f;
    t.sigma2[0] = 1.0f;
    for (int i = 1; i < t.nlevels; ++i) {  // float * double member, rounded back to float (418-422)
        t.scale[i] = (float)((double)t.scale[i - 1] * t.scale_d);
        t.sigma2[i] = t.scale[i] * t.scale[i];
    }
    for (int i = 0; i < t.nlevels; ++i) {  // 426-430
        t.inv[i] = 1.0f / t.scale[i];
        t.inv_sigma2[i] = 1.0f / t.sigma2[i];
    }
    // Feature budget per level (434-445): geometric series, cvRound per level, rest to the top.
    const float factor = (float)(1.0 / t.scale_d);
    float per_scale = (float)t.nfeatures * (1 - factor) /
                      (1 - (float)std::pow((double)factor, (double)t.nlevels));
    int total = 0;
    for (int l = 0; l < t.nlevels - 1; ++l) {
        t.nfeat[l] = cv_round(per_scale);
        total += t.nfeat[l];
        per_scale *= factor;
    }
    t.nfeat[t.nlevels - 1] = std::max(t.nfeatures - total, 0);
    // umax: half-widths of the radius-15 circular patch, made symmetric (453-468).
    const int vmax = cv_floor(kHalfPatch * std::sqrt(2.f) / 2 + 1);
    const int vmin = (int)std::ceil(kHalfPatch * std::sqrt(2.f) / 2);
    const double r2 = (double)kHalfPatch * kHalfPatch;
    for (int v = 0; v <= vmax; ++v) t.umax[v] = cv_round(std::sqrt(r2 - v * v));
    for (int v = kHalfPatch, v0 = 0; v >= vmin; --v) {
        while (t.umax[v0] == t.umax[v0 + 1]) ++v0;
        t.umax[v] = v0;
        ++v0;
    }
    return true;
}

// ---------------------------------------------------------------------------------------------
// Images: dense u8 planes (stride == width).
struct Plane {
    int w = 0, h = 0;
    std::vector<uint8_t> px;
    uint8_t at(int y, int x) const { return px[(size_t)y * w + x]; }
    const uint8_t* row(int y) const { return px.data() + (size_t)y * w; }
};

// cv::resize(src, dst, dsize, 0, 0, INTER_LINEAR) for 8UC1 (App. A.1; call ORBextractor.cc:1123).
void resize_linear(const uint8_t* src, int sw, int sh, size_t sstride, uint8_t* dst, int dw,
                   int dh, size_t dstride) {
    const double scale_x = 1. / ((double)dw / sw), scale_y = 1. / ((double)dh / sh);
    const int kOne = 2048;  // INTER_RESIZE_COEF_SCALE
    std::vector<int> xofs(dw), xofs1(dw);
    std::vector<int> ax0(dw), ax1(dw);
    for (int dx = 0; dx < dw; ++dx) {
        float fx = (float)((dx + 0.5) * scale_x - 0.5);
        int sx = cv_floor(fx);
        fx -= sx;
        if (sx < 0) { fx = 0; sx = 0; }
        if (sx + 1 >= sw && sx >= sw - 1) { fx = 0; sx = sw - 1; }
        xofs[dx] = sx;
        xofs1[dx] = std::min(sx + 1, sw - 1);
        ax0[dx] = sat_short((1.f - fx) * kOne);
        ax1[dx] = sat_short(fx * kOne);
    }
    std::vector<int> t0(dw), t1(dw);
    auto hpass = [&](int sy, std::vector<int>& t) {
        const uint8_t* s = src + (size_t)sy * sstride;
        for (int dx = 0; dx < dw; ++dx) t[dx] = s[xofs[dx]] * ax0[dx] + s[xofs1[dx]] * ax1[dx];
    };
    for (int dy = 0; dy < dh; ++dy) {
        float fy = (float)((dy + 0.5) * scale_y - 0.5);
        int sy = cv_floor(fy);
        fy -= sy;
        const int b0 = sat_short((1.f - fy) * kOne), b1 = sat_short(fy * kOne);
        const int r0 = std::min(std::max(sy, 0), sh - 1), r1 = std::min(std::max(sy + 1, 0), sh - 1);
        hpass(r0, t0);
        hpass(r1, t1);
        uint8_t* d = dst + (size_t)dy * dstride;
        int dx = 0;
        if (g_variant & kVarH5Sse2) {  // H5: ((((T0>>4)*b0)>>16) + (((T1>>4)*b1)>>16) + 2) >> 2
            const int xb = sse2_body_resize(dw);
            for (; dx < xb; ++dx) {
                const int x0 = sat_s16(t0[dx] >> 4), y0 = sat_s16(t1[dx] >> 4);
                const int m = sat_s16(((x0 * (int)(short)b0) >> 16) + ((y0 * (int)(short)b1) >> 16));
                d[dx] = sat_u8(sat_s16(m + 2) >> 2);
            }
        }
        for (; dx < dw; ++dx)  // FixedPtCast<int, uchar, 22>
            d[dx] = sat_u8((t0[dx] * b0 + t1[dx] * b1 + (1 << 21)) >> 22);
    }
}

// Integer 7-tap Gaussian (getGaussianKernel(7, 2, CV_32F) converted with scale 256).
void gaussian_taps(int k[7]) {
    float g[7];
    double sum = 0;
    const double s2 = -0.5 / (2.0 * 2.0);
    for (int i = 0; i < 7; ++i) {
        double x = i - 3.0;
        g[i] = (float)std::exp(s2 * x * x);
        sum += g[i];
    }
    sum = 1. / sum;
    for (int i = 0; i < 7; ++i) g[i] = (float)(g[i] * sum);
    for (int i = 0; i < 7; ++i) k[i] = cv_round(g[i] * 256.f + 0.f);
}

inline int reflect101(int p, int n) {
    if (n == 1) return 0;
    while (p < 0 || p >= n) p = p < 0 ? -p : 2 * n - p - 2;
    return p;
}

// cv::GaussianBlur(img, img, Size(7,7), 2, 2, BORDER_REFLECT_101) on a level clone
// (ORBextractor.cc:1088-1089; App. A.2, integer path).
void gaussian_blur(const uint8_t* src, int w, int h, size_t stride, uint8_t* dst, size_t dstride) {
    int k[7];
    gaussian_taps(k);
    std::vector<int> rows((size_t)w * h);
    for (int y = 0; y < h; ++y) {
        const uint8_t* s = src + (size_t)y * stride;
        for (int x = 0; x < w; ++x) {
            int acc = 0;
            for (int i = 0; i < 7; ++i) acc += k[i] * s[reflect101(x + i - 3, w)];
            rows[(size_t)y * w + x] = acc;
        }
    }
    // H6: the SSE2 body sums k_j / 2^16 * R in float (every partial sum exact below 2^24) and
    // converts with _mm_cvtps_epi32, i.e. rounds the same value half to EVEN; the scalar
    // FixedPtCastEx rounds half up.  They differ only when acc % 2^16 == 2^15.
    const int xb = (g_variant & kVarH6Simd) ? sse2_body_blur(w) : 0;
    for (int y = 0; y < h; ++y) {
        uint8_t* d = dst + (size_t)y * dstride;
        for (int x = 0; x < w; ++x) {
            int acc = 0;
            for (int j = 0; j < 7; ++j) acc += k[j] * rows[(size_t)reflect101(y + j - 3, h) * w + x];
            if (x < xb) {
                int q = acc >> 16;
                const int rem = acc & 0xffff;
                if (rem > 0x8000 || (rem == 0x8000 && (q & 1))) ++q;
                d[x] = acc >= (1 << 24) ? 255 : sat_u8(q);
            } else {
                d[x] = sat_u8((acc + (1 << 15)) >> 16);
            }
        }
    }
}

// ---------------------------------------------------------------------------------------------
// cv::FAST(roi, kps, threshold, nonmax=true), TYPE_9_16 (App. A.3; calls ORBextractor.cc:808,813).
const int kCircle[16][2] = {{0, 3},  {1, 3},   {2, 2},   {3, 1},   {3, 0},   {3, -1},
                            {2, -2}, {1, -3},  {0, -3},  {-1, -3}, {-2, -2}, {-3, -1},
                            {-3, 0}, {-3, 1},  {-2, 2},  {-1, 3}};

struct Key {  // the cv::KeyPoint fields the extractor uses
    float x, y, response, angle = -1.f;
    int octave = 0;
};

// cornerScore<16>: largest threshold at which the pixel is still a 9-of-16 corner.
int corner_score(const uint8_t* p, const int* ring, int threshold) {
    short d[25];
    const int v = p[0];
    for (int k = 0; k < 25; ++k) d[k] = (short)(v - p[ring[k]]);
    int a0 = threshold;
    for (int k = 0; k < 16; k += 2) {  // darker arcs: max over arcs of min(d)
        int a = std::min(std::min((int)d[k + 1], (int)d[k + 2]), (int)d[k + 3]);
        if (a <= a0) continue;
        for (int m = 4; m <= 8; ++m) a = std::min(a, (int)d[k + m]);
        a0 = std::max(a0, std::min(a, (int)d[k]));
        a0 = std::max(a0, std::min(a, (int)d[k + 9]));
    }
    int b0 = -a0;
    for (int k = 0; k < 16; k += 2) {  // brighter arcs: min over arcs of max(d)
        int b = std::max(std::max((int)d[k + 1], (int)d[k + 2]), (int)d[k + 3]);
        b = std::max(b, (int)d[k + 4]);
        b = std::max(b, (int)d[k + 5]);
        if (b >= b0) continue;
        for (int m = 6; m <= 8; ++m) b = std::max(b, (int)d[k + m]);
        b0 = std::min(b0, std::max(b, (int)d[k]));
        b0 = std::min(b0, std::max(b, (int)d[k + 9]));
    }
    return -b0 - 1;
}

void fast_detect(const uint8_t* img, int rows, int cols, size_t step, int threshold,
                 std::vector<Key>& out) {
    out.clear();
    if (rows < 7 || cols < 7) return;
    int ring[25];
    for (int k = 0; k < 16; ++k) ring[k] = kCircle[k][0] + kCircle[k][1] * (int)step;
    for (int k = 16; k < 25; ++k) ring[k] = ring[k - 16];
    threshold = std::min(std::max(threshold, 0), 255);
    uint8_t cls[512];  // 1: darker than v - t, 2: brighter than v + t
    for (int i = -255; i <= 255; ++i) cls[i + 255] = (uint8_t)(i < -threshold ? 1 : i > threshold ? 2 : 0);

    std::vector<uint8_t> score[3];
    std::vector<int> pos[3];
    for (int r = 0; r < 3; ++r) score[r].assign(cols, 0);
    for (int i = 3; i < rows - 2; ++i) {
        std::vector<uint8_t>& cur = score[(i - 3) % 3];
        std::vector<int>& cpos = pos[(i - 3) % 3];
        std::fill(cur.begin(), cur.end(), 0);
        cpos.clear();
        if (i < rows - 3) {
            const uint8_t* p = img + (size_t)i * step + 3;
            for (int j = 3; j < cols - 3; ++j, ++p) {
                const int v = p[0];
                const uint8_t* c = cls + 255 - v;
                int d = c[p[ring[0]]] | c[p[ring[8]]];
                if (!d) continue;
                d &= c[p[ring[2]]] | c[p[ring[10]]];
                d &= c[p[ring[4]]] | c[p[ring[12]]];
                d &= c[p[ring[6]]] | c[p[ring[14]]];
                if (!d) continue;
                for (int q = 1; q < 8; q += 2) d &= c[p[ring[q]]] | c[p[ring[q + 8]]];
                for (int pass = 0; pass < 2; ++pass) {  // pass 0: darker arc, pass 1: brighter
                    if (!(d & (1 << pass))) continue;
                    const int vt = pass == 0 ? v - threshold : v + threshold;
                    int run = 0;
                    for (int k = 0; k < 25; ++k) {
                        const int x = p[ring[k]];
                        const bool in = pass == 0 ? x < vt : x > vt;
                        if (!in) { run = 0; continue; }
                        if (++run > 8) {
                            cpos.push_back(j);
                            cur[j] = (uint8_t)corner_score(p, ring, threshold);
                            break;
                        }
                    }
                }
            }
        }
        if (i == 3) continue;
        const std::vector<uint8_t>& prev = score[(i - 4 + 3) % 3];
        const std::vector<uint8_t>& pprev = score[(i - 5 + 3) % 3];
        for (int j : pos[(i - 4 + 3) % 3]) {  // strict 3x3 non-maximum suppression, row i-1
            const int s = prev[j];
            if (s > prev[j + 1] && s > prev[j - 1] && s > pprev[j - 1] && s > pprev[j] &&
                s > pprev[j + 1] && s > cur[j - 1] && s > cur[j] && s > cur[j + 1])
                out.push_back(Key{(float)j, (float)(i - 1), (float)s});
        }
    }
}

// ---------------------------------------------------------------------------------------------
// A4 — per-cell FAST with the minThFAST fallback (ComputeKeyPointsOctTree, 764-831).
void level_fast_keys(const Tables& t, const Plane& lev, std::vector<Key>& keys,
                     std::vector<int>* cell_counts = nullptr) {
    keys.clear();
    if (cell_counts) cell_counts->clear();
    const float kW = 30;
    const int min_bx = kEdge - 3, min_by = min_bx;
    const int max_bx = lev.w - kEdge + 3, max_by = lev.h - kEdge + 3;
    const float width = (float)(max_bx - min_bx), height = (float)(max_by - min_by);
    const int ncols = (int)(width / kW), nrows = (int)(height / kW);
    if (ncols <= 0 || nrows <= 0) return;  // reference: no cell loop iterations
    const int wcell = (int)std::ceil(width / ncols), hcell = (int)std::ceil(height / nrows);
    std::vector<Key> cell;
    for (int i = 0; i < nrows; ++i) {
        const float ini_y = (float)(min_by + i * hcell);
        float max_y = ini_y + hcell + 6;
        if (ini_y >= max_by - 3) continue;
        if (max_y > max_by) max_y = (float)max_by;
        for (int j = 0; j < ncols; ++j) {
            const float ini_x = (float)(min_bx + j * wcell);
            float max_x = ini_x + wcell + 6;
            if (ini_x >= max_bx - 6) continue;
            if (max_x > max_bx) max_x = (float)max_bx;
            const int y0 = (int)ini_y, x0 = (int)ini_x;
            const uint8_t* roi = lev.px.data() + (size_t)y0 * lev.w + x0;
            fast_detect(roi, (int)max_y - y0, (int)max_x - x0, lev.w, t.ini_th, cell);
            if (cell.empty()) fast_detect(roi, (int)max_y - y0, (int)max_x - x0, lev.w, t.min_th, cell);
            for (Key& k : cell) {  // relative to (minBorderX, minBorderY) (819-824)
                k.x += (float)(j * wcell);
                k.y += (float)(i * hcell);
                keys.push_back(k);
            }
            if (cell_counts) cell_counts->push_back((int)cell.size());
        }
    }
}

// ---------------------------------------------------------------------------------------------
// A6 — DistributeOctTree (538-762) + ExtractorNode::DivideNode (480-536), list semantics kept.
struct OctNode {
    std::vector<Key> keys;
    int ulx, uly, urx, ury, blx, bly, brx, bry;  // UL, UR, BL, BR corners
    bool no_more = false;
    long seq = 0;  // creation order: the H2 stand-in for the node's heap address
    std::list<OctNode>::iterator self;
};

void split_node(const OctNode& p, OctNode c[4]) {
    const int hx = (int)std::ceil((float)(p.urx - p.ulx) / 2);
    const int hy = (int)std::ceil((float)(p.bry - p.uly) / 2);
    // children: 0 upper-left, 1 upper-right, 2 lower-left, 3 lower-right (n1..n4)
    c[0].ulx = p.ulx;      c[0].uly = p.uly;      c[0].urx = p.ulx + hx; c[0].ury = p.uly;
    c[0].blx = p.ulx;      c[0].bly = p.uly + hy; c[0].brx = p.ulx + hx; c[0].bry = p.uly + hy;
    c[1].ulx = c[0].urx;   c[1].uly = c[0].ury;   c[1].urx = p.urx;      c[1].ury = p.ury;
    c[1].blx = c[0].brx;   c[1].bly = c[0].bry;   c[1].brx = p.urx;      c[1].bry = p.uly + hy;
    c[2].ulx = c[0].blx;   c[2].uly = c[0].bly;   c[2].urx = c[0].brx;   c[2].ury = c[0].bry;
    c[2].blx = p.blx;      c[2].bly = p.bly;      c[2].brx = c[0].brx;   c[2].bry = p.bly;
    c[3].ulx = c[2].urx;   c[3].uly = c[2].ury;   c[3].urx = c[1].brx;   c[3].ury = c[1].bry;
    c[3].blx = c[2].brx;   c[3].bly = c[2].bry;   c[3].brx = p.brx;      c[3].bry = p.bry;
    for (int q = 0; q < 4; ++q) c[q].keys.reserve(p.keys.size());
    for (const Key& k : p.keys) {
        const bool left = k.x < c[0].urx, top = k.y < c[0].bry;
        c[left ? (top ? 0 : 2) : (top ? 1 : 3)].keys.push_back(k);
    }
    for (int q = 0; q < 4; ++q)
        if (c[q].keys.size() == 1) c[q].no_more = true;
}

std::vector<Key> distribute(const std::vector<Key>& in, int min_x, int max_x, int min_y,
                            int max_y, int n_target) {
    std::vector<Key> result;
    if (in.empty()) return result;
    const int n_ini = (int)std::round((float)(max_x - min_x) / (max_y - min_y));
    const float hx = (float)(max_x - min_x) / n_ini;
    long seq = 0;
    std::list<OctNode> nodes;
    std::vector<OctNode*> ini(n_ini);
    for (int i = 0; i < n_ini; ++i) {
        OctNode n;
        n.ulx = (int)(hx * (float)i);       n.uly = 0;
        n.urx = (int)(hx * (float)(i + 1)); n.ury = 0;
        n.blx = n.ulx;                      n.bly = max_y - min_y;
        n.brx = n.urx;                      n.bry = max_y - min_y;
        n.seq = seq++;
        nodes.push_back(n);
        ini[i] = &nodes.back();
    }
    for (const Key& k : in)  // initial node by float division (568); the clamp only guards UB
        ini[std::min((size_t)(k.x / hx), (size_t)n_ini - 1)]->keys.push_back(k);
    for (auto it = nodes.begin(); it != nodes.end();) {
        if (it->keys.size() == 1) { it->no_more = true; ++it; }
        else if (it->keys.empty()) it = nodes.erase(it);
        else ++it;
    }
    // Push the non-empty children of `parent` to the list front; expandable ones are recorded.
    auto spawn = [&](const OctNode& parent, std::vector<std::pair<int, OctNode*>>& expand) {
        OctNode c[4];
        split_node(parent, c);
        int added = 0;
        for (int q = 0; q < 4; ++q) {
            if (c[q].keys.empty()) continue;
            c[q].seq = seq++;
            nodes.push_front(std::move(c[q]));
            ++added;
            if (nodes.front().keys.size() > 1) {
                expand.emplace_back((int)nodes.front().keys.size(), &nodes.front());
                nodes.front().self = nodes.begin();
            }
        }
        return added;
    };
    std::vector<std::pair<int, OctNode*>> expand;
    bool done = false;
    while (!done) {
        const int prev = (int)nodes.size();
        expand.clear();
        int n_expand = 0;
        for (auto it = nodes.begin(); it != nodes.end();) {  // phase 1: split every open node
            if (it->no_more) { ++it; continue; }
            const size_t before = expand.size();
            spawn(*it, expand);
            n_expand += (int)(expand.size() - before);
            it = nodes.erase(it);
        }
        if ((int)nodes.size() >= n_target || (int)nodes.size() == prev) {
            done = true;
        } else if ((int)nodes.size() + n_expand * 3 > n_target) {
            while (!done) {  // phase 2: split the largest nodes first until the budget is met
                const int prev2 = (int)nodes.size();
                std::vector<std::pair<int, OctNode*>> order = expand;
                expand.clear();
                std::sort(order.begin(), order.end(), [](const std::pair<int, OctNode*>& a,
                                                         const std::pair<int, OctNode*>& b) {
                    return a.first != b.first ? a.first < b.first : a.second->seq < b.second->seq;
                });
                for (int j = (int)order.size() - 1; j >= 0; --j) {
                    spawn(*order[j].second, expand);
                    nodes.erase(order[j].second->self);
                    if ((int)nodes.size() >= n_target) break;
                }
                if ((int)nodes.size() >= n_target || (int)nodes.size() == prev2) done = true;
            }
        }
    }
    // keep the strongest response per node, first one on ties (740-759)
    result.reserve(nodes.size());
    for (const OctNode& n : nodes) {
        const Key* best = &n.keys[0];
        for (size_t k = 1; k < n.keys.size(); ++k)
            if (n.keys[k].response > best->response) best = &n.keys[k];
        result.push_back(*best);
    }
    return result;
}

// H2 variant — the oct-tree with the reference's own heap objects, so that phase 2's
// sort(pair<int, ExtractorNode*>) (680-683) orders equal sizes by real glibc addresses instead
// of creation sequence.  RefNode has ExtractorNode's layout (ORBextractor.h:37-48: a vector of
// 28-byte cv::KeyPoints, four cv::Point2i, a list iterator, a bool: 72 bytes, list node 88),
// and the function performs the reference's allocations in the reference's order: the initial
// nodes' reserve + push_back copies and the vKeys growth of the assignment loop (548-568); per
// division four children reserving the parent's size (DivideNode 486-507), the push_front copy
// of each non-empty child (list node first, then its exact-size vector), the parent's erase,
// then the children's destruction in reverse declaration order (605-663, 694-736); the
// size/pointer vectors (reserve 4 x nodes, the phase-2 copy); the result reserve.
struct KP28 {  // cv::KeyPoint
    float x, y, size, angle, response;
    int octave, class_id;
};
struct RefNode {
    std::vector<KP28> vKeys;
    int UL[2], UR[2], BL[2], BR[2];
    std::list<RefNode>::iterator lit;
    bool bNoMore = false;

    void divide(RefNode& n1, RefNode& n2, RefNode& n3, RefNode& n4) const {
        const int hx = (int)std::ceil((float)(UR[0] - UL[0]) / 2);
        const int hy = (int)std::ceil((float)(BR[1] - UL[1]) / 2);
        auto set = [](int* p, int x, int y) { p[0] = x; p[1] = y; };
        set(n1.UL, UL[0], UL[1]);          set(n1.UR, UL[0] + hx, UL[1]);
        set(n1.BL, UL[0], UL[1] + hy);     set(n1.BR, UL[0] + hx, UL[1] + hy);
        n1.vKeys.reserve(vKeys.size());
        set(n2.UL, n1.UR[0], n1.UR[1]);    set(n2.UR, UR[0], UR[1]);
        set(n2.BL, n1.BR[0], n1.BR[1]);    set(n2.BR, UR[0], UL[1] + hy);
        n2.vKeys.reserve(vKeys.size());
        set(n3.UL, n1.BL[0], n1.BL[1]);    set(n3.UR, n1.BR[0], n1.BR[1]);
        set(n3.BL, BL[0], BL[1]);          set(n3.BR, n1.BR[0], BL[1]);
        n3.vKeys.reserve(vKeys.size());
        set(n4.UL, n3.UR[0], n3.UR[1]);    set(n4.UR, n2.BR[0], n2.BR[1]);
        set(n4.BL, n3.BR[0], n3.BR[1]);    set(n4.BR, BR[0], BR[1]);
        n4.vKeys.reserve(vKeys.size());
        for (const KP28& k : vKeys) {
            if (k.x < n1.UR[0]) (k.y < n1.BR[1] ? n1 : n3).vKeys.push_back(k);
            else (k.y < n1.BR[1] ? n2 : n4).vKeys.push_back(k);
        }
        for (RefNode* c : {&n1, &n2, &n3, &n4})
            if (c->vKeys.size() == 1) c->bNoMore = true;
    }
};

std::vector<KP28> distribute_heap(const std::vector<KP28>& in, int min_x, int max_x, int min_y,
                                  int max_y, int n_target, int nfeatures) {
    const int n_ini = (int)std::round((float)(max_x - min_x) / (max_y - min_y));
    const float hx = (float)(max_x - min_x) / n_ini;
    std::list<RefNode> nodes;
    std::vector<RefNode*> ini;
    ini.resize(n_ini);
    for (int i = 0; i < n_ini; ++i) {
        RefNode ni;
        ni.UL[0] = (int)(hx * (float)i);        ni.UL[1] = 0;
        ni.UR[0] = (int)(hx * (float)(i + 1));  ni.UR[1] = 0;
        ni.BL[0] = ni.UL[0];                    ni.BL[1] = max_y - min_y;
        ni.BR[0] = ni.UR[0];                    ni.BR[1] = max_y - min_y;
        ni.vKeys.reserve(in.size());
        nodes.push_back(ni);
        ini[i] = &nodes.back();
    }
    for (const KP28& k : in) ini[std::min((size_t)(k.x / hx), (size_t)n_ini - 1)]->vKeys.push_back(k);
    for (auto it = nodes.begin(); it != nodes.end();) {
        if (it->vKeys.size() == 1) { it->bNoMore = true; ++it; }
        else if (it->vKeys.empty()) it = nodes.erase(it);
        else ++it;
    }
    bool finish = false;
    std::vector<std::pair<int, RefNode*>> size_ptr;
    size_ptr.reserve(nodes.size() * 4);
    // the non-empty children of a division, pushed to the front; expandable ones recorded
    auto push_children = [&](RefNode& n1, RefNode& n2, RefNode& n3, RefNode& n4, int* n_expand) {
        for (RefNode* c : {&n1, &n2, &n3, &n4}) {
            if (c->vKeys.empty()) continue;
            nodes.push_front(*c);
            if (c->vKeys.size() > 1) {
                if (n_expand) ++*n_expand;
                size_ptr.push_back(std::make_pair((int)c->vKeys.size(), &nodes.front()));
                nodes.front().lit = nodes.begin();
            }
        }
    };
    while (!finish) {
        int prev = (int)nodes.size();
        int n_expand = 0;
        size_ptr.clear();
        for (auto it = nodes.begin(); it != nodes.end();) {
            if (it->bNoMore) { ++it; continue; }
            RefNode n1, n2, n3, n4;
            it->divide(n1, n2, n3, n4);
            push_children(n1, n2, n3, n4, &n_expand);
            it = nodes.erase(it);
        }
        if ((int)nodes.size() >= n_target || (int)nodes.size() == prev) {
            finish = true;
        } else if ((int)nodes.size() + n_expand * 3 > n_target) {
            while (!finish) {
                prev = (int)nodes.size();
                std::vector<std::pair<int, RefNode*>> order = size_ptr;
                size_ptr.clear();
                std::sort(order.begin(), order.end());  // equal sizes: by address
                for (int j = (int)order.size() - 1; j >= 0; --j) {
                    RefNode n1, n2, n3, n4;
                    order[j].second->divide(n1, n2, n3, n4);
                    push_children(n1, n2, n3, n4, nullptr);
                    nodes.erase(order[j].second->lit);
                    if ((int)nodes.size() >= n_target) break;
                }
                if ((int)nodes.size() >= n_target || (int)nodes.size() == prev) finish = true;
            }
        }
    }
    std::vector<KP28> result;
    result.reserve(nfeatures);
    for (RefNode& n : nodes) {  // max response per node, first on ties (741-759)
        const KP28* best = &n.vKeys[0];
        for (size_t k = 1; k < n.vKeys.size(); ++k)
            if (n.vKeys[k].response > best->response) best = &n.vKeys[k];
        result.push_back(*best);
    }
    return result;
}

// ---------------------------------------------------------------------------------------------
// A8 — IC_Angle (76-103) with cv::fastAtan2 (App. A.4).
const float kAtanP1 = 0.9997878412794807f * (float)(180 / M_PI);
const float kAtanP3 = -0.3258083974640975f * (float)(180 / M_PI);
const float kAtanP5 = 0.1555786518463281f * (float)(180 / M_PI);
const float kAtanP7 = -0.04432655554792128f * (float)(180 / M_PI);

float fast_atan2(float y, float x) {
    const float ax = std::fabs(x), ay = std::fabs(y);
    float a, c, c2;
    if (ax >= ay) {
        c = ay / (ax + (float)DBL_EPSILON);
        c2 = c * c;
        a = (((kAtanP7 * c2 + kAtanP5) * c2 + kAtanP3) * c2 + kAtanP1) * c;
    } else {
        c = ax / (ay + (float)DBL_EPSILON);
        c2 = c * c;
        a = 90.f - (((kAtanP7 * c2 + kAtanP5) * c2 + kAtanP3) * c2 + kAtanP1) * c;
    }
    if (x < 0) a = 180.f - a;
    if (y < 0) a = 360.f - a;
    return a;
}

float ic_angle(const uint8_t* img, size_t step, float px, float py, const int* umax) {
    const uint8_t* c = img + (size_t)cv_round(py) * step + cv_round(px);
    int m01 = 0, m10 = 0;
    for (int u = -kHalfPatch; u <= kHalfPatch; ++u) m10 += u * c[u];
    const long s = (long)step;
    for (int v = 1; v <= kHalfPatch; ++v) {
        int vsum = 0;
        for (int u = -umax[v]; u <= umax[v]; ++u) {
            const int up = c[u + v * s], dn = c[u - v * s];
            vsum += up - dn;
            m10 += u * (up + dn);
        }
        m01 += v * vsum;
    }
    return fast_atan2((float)m01, (float)m10);
}

// A10 — computeOrbDescriptor (107-146): 256 intensity tests on the blurred level.
const float kDegToRad = (float)(M_PI / 180.f);
}  // namespace
extern "C" void oracle_rot_fma(float, int, const int*, int, int*, int*);
extern "C" void oracle_rot_plain(float, int, const int*, int, int*, int*);
namespace {

void orb_descriptor(const uint8_t* img, size_t step, const Key& k, uint8_t* desc) {
    const float ang = k.angle * kDegToRad;
    const float a = (float)std::cos((double)ang), b = (float)std::sin((double)ang);
    const uint8_t* c = img + (size_t)cv_round(k.y) * step + cv_round(k.x);
    const long s = (long)step;
    int vy[512], vx[512];  // H4 variants: offsets from oracle/variant_rot.cpp
    const bool h4 = (g_variant & (kVarH4Cosf | kVarH4Fma)) != 0;
    if (h4)
        ((g_variant & kVarH4Fma) ? oracle_rot_fma : oracle_rot_plain)(
            k.angle, (g_variant & kVarH4Cosf) != 0, kPattern, 512, vy, vx);
    auto sample = [&](int idx) {
        if (h4) return (int)c[vy[idx] * s + vx[idx]];
        const float px = (float)kPattern[2 * idx], py = (float)kPattern[2 * idx + 1];
        return (int)c[cv_round(px * b + py * a) * s + cv_round(px * a - py * b)];
    };
    for (int i = 0; i < 32; ++i) {
        int byte = 0;
        for (int bit = 0; bit < 8; ++bit) {
            const int p = 16 * i + 2 * bit;
            byte |= (sample(p) < sample(p + 1)) << bit;
        }
        desc[i] = (uint8_t)byte;
    }
}

// ---------------------------------------------------------------------------------------------
// A2/A3 — operator() (1042-1108) and ComputePyramid (1110-1135).
void level_sizes(const Tables& t, int w, int h, int* lw, int* lh) {
    for (int l = 0; l < t.nlevels; ++l) {
        lw[l] = cv_round((float)w * t.inv[l]);
        lh[l] = cv_round((float)h * t.inv[l]);
    }
}

void build_pyramid(const Tables& t, const uint8_t* img, int w, int h, size_t stride,
                   const uint8_t* mask, size_t mstride, std::vector<Plane>& pyr) {
    int lw[kMaxLevels], lh[kMaxLevels];
    level_sizes(t, w, h, lw, lh);
    pyr.resize(t.nlevels);
    pyr[0].w = w;
    pyr[0].h = h;
    pyr[0].px.assign((size_t)w * h, 0);
    for (int y = 0; y < h; ++y)  // imageIn.copyTo(image, Mask) (1053; App. A.7)
        for (int x = 0; x < w; ++x)
            if (!mask || mask[(size_t)y * mstride + x]) pyr[0].px[(size_t)y * w + x] = img[(size_t)y * stride + x];
    for (int l = 1; l < t.nlevels; ++l) {  // cascaded: level l from level l-1 (1123)
        pyr[l].w = lw[l];
        pyr[l].h = lh[l];
        pyr[l].px.assign((size_t)lw[l] * lh[l], 0);
        resize_linear(pyr[l - 1].px.data(), pyr[l - 1].w, pyr[l - 1].h, pyr[l - 1].w,
                      pyr[l].px.data(), lw[l], lh[l], lw[l]);
    }
}

// Oct-tree keypoints of one level, with the post-distribution fix-up (833-846) and angle.
void level_keypoints(const Tables& t, int level, const Plane& lev, std::vector<Key>& out) {
    std::vector<Key> cand;
    level_fast_keys(t, lev, cand);
    const int min_b = kEdge - 3;
    out = distribute(cand, min_b, lev.w - kEdge + 3, min_b, lev.h - kEdge + 3, t.nfeat[level]);
    for (Key& k : out) {
        k.x += min_b;
        k.y += min_b;
        k.octave = level;
    }
    for (Key& k : out) k.angle = ic_angle(lev.px.data(), lev.w, k.x, k.y, t.umax);
}

// H2 variant of level_keypoints: ComputeKeyPointsOctTree's per-level allocations (the
// vToDistributeKeys reserve, one growing vKeysCell per cell, 777-828; allKeypoints[level]
// reserve + copy-assignment of the result, 830-833) around distribute_heap.
void level_keypoints_heap(const Tables& t, int level, const Plane& lev,
                          std::vector<KP28>& all_level, std::vector<Key>& out) {
    std::vector<Key> cand;
    std::vector<int> counts;
    level_fast_keys(t, lev, cand, &counts);
    std::vector<KP28> to_distribute;
    to_distribute.reserve((size_t)t.nfeatures * 10);
    size_t k0 = 0;
    for (int c : counts) {
        std::vector<KP28> cell;
        for (int i = 0; i < c; ++i) {
            const Key& k = cand[k0 + i];
            cell.push_back(KP28{k.x, k.y, 7.f, -1.f, k.response, 0, -1});
        }
        for (const KP28& k : cell) to_distribute.push_back(k);
        k0 += c;
    }
    all_level.reserve(t.nfeatures);
    const int min_b = kEdge - 3;
    if (!to_distribute.empty())
        all_level = distribute_heap(to_distribute, min_b, lev.w - kEdge + 3, min_b,
                                    lev.h - kEdge + 3, t.nfeat[level], t.nfeatures);
    out.clear();
    for (const KP28& k : all_level) {
        Key o{k.x + min_b, k.y + min_b, k.response};
        o.octave = level;
        out.push_back(o);
    }
    for (Key& k : out) k.angle = ic_angle(lev.px.data(), lev.w, k.x, k.y, t.umax);
}

int extract(const Tables& t, const uint8_t* img, int w, int h, size_t stride,
            const uint8_t* mask, size_t mstride, orbfe_keypoint* kps, int cap, uint8_t* desc,
            int* n_out) {
    if (!img || w <= 0 || h <= 0) return ORBFE_OK;  // empty image: outputs untouched (1045-1046)
    std::vector<Plane> pyr;
    build_pyramid(t, img, w, h, stride, mask, mstride, pyr);
    std::vector<std::vector<Key>> all(t.nlevels);
    std::vector<std::vector<KP28>> all_heap;  // H2: allKeypoints.resize(nlevels) (766)
    if (g_variant & kVarH2Addr) all_heap.resize(t.nlevels);
    int total = 0;
    for (int l = 0; l < t.nlevels; ++l) {
        if (g_variant & kVarH2Addr) level_keypoints_heap(t, l, pyr[l], all_heap[l], all[l]);
        else level_keypoints(t, l, pyr[l], all[l]);
        total += (int)all[l].size();
    }
    if (n_out) *n_out = total;
    if (total > cap) return ORBFE_ERR_CAPACITY;
    int off = 0;
    Plane blurred;
    for (int l = 0; l < t.nlevels; ++l) {
        if (all[l].empty()) continue;
        blurred.w = pyr[l].w;
        blurred.h = pyr[l].h;
        blurred.px.resize(pyr[l].px.size());
        gaussian_blur(pyr[l].px.data(), pyr[l].w, pyr[l].h, pyr[l].w, blurred.px.data(), blurred.w);
        const int patch = (int)(kPatchSize * t.scale[l]);
        for (const Key& k : all[l]) {
            if (desc) orb_descriptor(blurred.px.data(), blurred.w, k, desc + (size_t)off * 32);
            orbfe_keypoint& o = kps[off];
            o.x = l ? k.x * t.scale[l] : k.x;
            o.y = l ? k.y * t.scale[l] : k.y;
            o.size = (float)patch;
            o.angle = k.angle;
            o.response = k.response;
            o.octave = l;
            o.class_id = -1;
            ++off;
        }
    }
    return ORBFE_OK;
}

bool extract_supported(const Tables& t, int w, int h) {
    // DistributeOctTree divides by round(width/height) (542): a level tall enough to hold FAST
    // cells but with round(w/h) == 0 indexes an empty node vector in the reference (UB).
    int lw[kMaxLevels], lh[kMaxLevels];
    level_sizes(t, w, h, lw, lh);
    for (int l = 0; l < t.nlevels; ++l) {
        const int bw = lw[l] - 2 * (kEdge - 3), bh = lh[l] - 2 * (kEdge - 3);
        if (bw >= 30 && bh >= 30 && std::round((float)bw / bh) < 1) return false;
    }
    return w <= 4096 && h <= 4096;
}

// ---------------------------------------------------------------------------------------------
// A12 — DescriptorDistance (ORBmatcher.cc:1650-1666): SWAR popcount over 8 int32 words.
int descriptor_distance(const uint8_t* a, const uint8_t* b) {
    int dist = 0;
    for (int i = 0; i < 8; ++i) {
        uint32_t wa, wb;
        std::memcpy(&wa, a + 4 * i, 4);
        std::memcpy(&wb, b + 4 * i, 4);
        uint32_t v = wa ^ wb;
        v = v - ((v >> 1) & 0x55555555u);
        v = (v & 0x33333333u) + ((v >> 2) & 0x33333333u);
        dist += (int)((((v + (v >> 4)) & 0xF0F0F0Fu) * 0x1010101u) >> 24);
    }
    return dist;
}

// A16 — Frame grid (Frame.cc:341-356, 445-510).
const int kGridCols = 64, kGridRows = 48;  // FRAME_GRID_COLS / FRAME_GRID_ROWS (Frame.h:37-38)
struct Grid {
    std::vector<int> cell[kGridCols][kGridRows];
};

void build_grid(const orbfe_frame_view* f, Grid& g) {
    for (int i = 0; i < f->n; ++i) {
        const orbfe_keypoint& k = f->keys_un[i];
        const int gx = (int)std::round((k.x - f->min_x) * f->grid_w_inv);
        const int gy = (int)std::round((k.y - f->min_y) * f->grid_h_inv);
        if (gx < 0 || gx >= kGridCols || gy < 0 || gy >= kGridRows) continue;
        g.cell[gx][gy].push_back(i);
    }
}

void features_in_area(const orbfe_frame_view* f, const Grid& g, float x, float y, float r,
                      int min_level, int max_level, std::vector<int>& out) {
    out.clear();
    const int cx0 = std::max(0, (int)std::floor((x - f->min_x - r) * f->grid_w_inv));
    if (cx0 >= kGridCols) return;
    const int cx1 = std::min(kGridCols - 1, (int)std::ceil((x - f->min_x + r) * f->grid_w_inv));
    if (cx1 < 0) return;
    const int cy0 = std::max(0, (int)std::floor((y - f->min_y - r) * f->grid_h_inv));
    if (cy0 >= kGridRows) return;
    const int cy1 = std::min(kGridRows - 1, (int)std::ceil((y - f->min_y + r) * f->grid_h_inv));
    if (cy1 < 0) return;
    const bool check_levels = min_level > 0 || max_level >= 0;
    for (int ix = cx0; ix <= cx1; ++ix)
        for (int iy = cy0; iy <= cy1; ++iy)
            for (int idx : g.cell[ix][iy]) {
                const orbfe_keypoint& k = f->keys_un[idx];
                if (check_levels) {
                    if (k.octave < min_level) continue;
                    if (max_level >= 0 && k.octave > max_level) continue;
                }
                if (std::fabs(k.x - x) < r && std::fabs(k.y - y) < r) out.push_back(idx);
            }
}

const int kThHigh = 100, kThLow = 50, kHistLen = 30;  // ORBmatcher.cc:37-39

// ComputeThreeMaxima (ORBmatcher.cc:1604-1645).
void three_maxima(const std::vector<int>* hist, int& i1, int& i2, int& i3) {
    int m1 = 0, m2 = 0, m3 = 0;
    i1 = i2 = i3 = -1;
    for (int i = 0; i < kHistLen; ++i) {
        const int s = (int)hist[i].size();
        if (s > m1) { m3 = m2; m2 = m1; m1 = s; i3 = i2; i2 = i1; i1 = i; }
        else if (s > m2) { m3 = m2; m2 = s; i3 = i2; i2 = i; }
        else if (s > m3) { m3 = s; i3 = i; }
    }
    if (m2 < 0.1f * (float)m1) { i2 = -1; i3 = -1; }
    else if (m3 < 0.1f * (float)m1) { i3 = -1; }
}

int rot_bin(float a1, float a2) {  // ORBmatcher.cc:478-483
    float rot = a1 - a2;
    if (rot < 0.0) rot += 360.0f;
    int bin = (int)std::round(rot * (1.0f / kHistLen));
    if (bin == kHistLen) bin = 0;
    return bin;
}

// 3x4 row-major [R|t] helpers with the float evaluation order of cv::Mat small products.
void rigid(const float* T, const float* p, float* out) {
    for (int r = 0; r < 3; ++r)
        out[r] = ((T[4 * r] * p[0] + T[4 * r + 1] * p[1]) + T[4 * r + 2] * p[2]) + T[4 * r + 3];
}
void camera_center(const float* T, float* c) {  // -R^T t, accumulated in double (GEMM_1_T path)
    for (int i = 0; i < 3; ++i)
        c[i] = (float)-((double)T[i] * T[3] + (double)T[4 + i] * T[7] + (double)T[8 + i] * T[11]);
}

}  // namespace

// =============================================================================================
// C ABI
extern "C" {

int oracle_tables(const orbfe_params* p, float* scale, float* inv, float* sigma2,
                  float* inv_sigma2, int32_t* nfeat, int32_t* umax) {
    Tables t;
    if (!make_tables(p, t)) return ORBFE_ERR_ARG;
    for (int l = 0; l < t.nlevels; ++l) {
        if (scale) scale[l] = t.scale[l];
        if (inv) inv[l] = t.inv[l];
        if (sigma2) sigma2[l] = t.sigma2[l];
        if (inv_sigma2) inv_sigma2[l] = t.inv_sigma2[l];
        if (nfeat) nfeat[l] = t.nfeat[l];
    }
    if (umax)
        for (int v = 0; v <= kHalfPatch; ++v) umax[v] = t.umax[v];
    return ORBFE_OK;
}

int oracle_set_variant(int flags) {
    if (flags < 0 || flags > 31) return ORBFE_ERR_ARG;
    g_variant = flags;
    return ORBFE_OK;
}
int oracle_get_variant(void) { return g_variant; }

int oracle_level_sizes(const orbfe_params* p, int w, int h, int32_t* lw, int32_t* lh) {
    Tables t;
    if (!make_tables(p, t)) return ORBFE_ERR_ARG;
    int a[kMaxLevels], b[kMaxLevels];
    level_sizes(t, w, h, a, b);
    for (int l = 0; l < t.nlevels; ++l) { lw[l] = a[l]; lh[l] = b[l]; }
    return ORBFE_OK;
}

int oracle_extract(const orbfe_params* p, const uint8_t* img, int w, int h, size_t stride,
                   const uint8_t* mask, size_t mask_stride, orbfe_keypoint* kps, int kps_cap,
                   uint8_t* desc, int* n_out) {
    Tables t;
    if (!make_tables(p, t)) return ORBFE_ERR_ARG;
    if (!img || w <= 0 || h <= 0) return ORBFE_OK;
    if (!extract_supported(t, w, h)) return ORBFE_ERR_UNSUPPORTED;
    if (!kps || kps_cap < 0) return ORBFE_ERR_ARG;
    return extract(t, img, w, h, stride, mask, mask_stride, kps, kps_cap, desc, n_out);
}

int oracle_extract_batch(const orbfe_params* p, const uint8_t* imgs, int n, int w, int h,
                         size_t frame_pitch, orbfe_keypoint* kps, int kps_cap, uint8_t* desc,
                         int32_t* n_out, int nthreads) {
    Tables t;
    if (!make_tables(p, t) || n < 0) return ORBFE_ERR_ARG;
    if (!extract_supported(t, w, h)) return ORBFE_ERR_UNSUPPORTED;
    nthreads = std::max(1, std::min(nthreads, n));
    std::vector<int> status(n, ORBFE_OK);
    auto work = [&](int tid) {
        for (int f = tid; f < n; f += nthreads) {
            int cnt = 0;
            status[f] = extract(t, imgs + (size_t)f * frame_pitch, w, h, w, nullptr, 0,
                                kps + (size_t)f * kps_cap, kps_cap,
                                desc ? desc + (size_t)f * kps_cap * 32 : nullptr, &cnt);
            n_out[f] = cnt;
        }
    };
    if (nthreads == 1) {
        work(0);
    } else {
        std::vector<std::thread> pool;
        for (int i = 0; i < nthreads; ++i) pool.emplace_back(work, i);
        for (auto& th : pool) th.join();
    }
    for (int s : status)
        if (s != ORBFE_OK) return s;
    return ORBFE_OK;
}

// cvtColor(src, dst, CV_{RGB,BGR,RGBA,BGRA}2GRAY) for 8U, as called by Tracking::GrabImage*
// (Tracking.cc:286-310, 350-363, 409-422).  OpenCV 3.3.1 RGB2Gray<uchar> (App. A, DESIGN H9):
// three 256-entry tables built by repeated addition, coefficients R2Y 4899, G2Y 9617, B2Y 1868
// (yuv_shift 14), the rounding constant folded into the table of source channel 2;
// blueIdx = 0 for BGR(A), 2 for RGB(A) picks which weight goes to channel 0.
int oracle_cvt_gray(const uint8_t* src, int pix, int w, int h, size_t stride, uint8_t* dst) {
    int scn, blue_idx;
    switch (pix) {
        case ORBFE_PIX_RGB: scn = 3; blue_idx = 2; break;
        case ORBFE_PIX_BGR: scn = 3; blue_idx = 0; break;
        case ORBFE_PIX_RGBA: scn = 4; blue_idx = 2; break;
        case ORBFE_PIX_BGRA: scn = 4; blue_idx = 0; break;
        default: return ORBFE_ERR_ARG;
    }
    if (!src || !dst || w <= 0 || h <= 0) return ORBFE_ERR_ARG;
    const int coeffs[3] = {4899, 9617, 1868};  // R2Y, G2Y, B2Y
    int tab[256 * 3];
    int b = 0, g = 0, r = 1 << 13;
    const int db = coeffs[blue_idx ^ 2], dg = coeffs[1], dr = coeffs[blue_idx];
    for (int i = 0; i < 256; ++i, b += db, g += dg, r += dr) {
        tab[i] = b;
        tab[i + 256] = g;
        tab[i + 512] = r;
    }
    for (int y = 0; y < h; ++y) {
        const uint8_t* s = src + (size_t)y * stride;
        for (int x = 0; x < w; ++x, s += scn)
            dst[(size_t)y * w + x] = (uint8_t)((tab[s[0]] + tab[s[1] + 256] + tab[s[2] + 512]) >> 14);
    }
    return ORBFE_OK;
}

// Frame::ComputeStereoMatches (Frame.cc:584-756) on the two pyramids of imL / imR (built as
// ORBextractor::ComputePyramid does).  kl/kr are mvKeys / mvKeysRight (distorted, as extracted).
int oracle_compute_stereo_matches(const orbfe_params* p, const uint8_t* imL, const uint8_t* imR,
                                  int w, int h, const orbfe_keypoint* kl, const uint8_t* dl,
                                  int nl, const orbfe_keypoint* kr, const uint8_t* dr, int nr,
                                  float bf, float b, float* u_right, float* depth) {
    Tables t;
    if (!make_tables(p, t) || !imL || !imR || w <= 0 || h <= 0 || nl < 0 || nr < 0 ||
        (nl && (!kl || !dl || !u_right || !depth)) || (nr && (!kr || !dr)))
        return ORBFE_ERR_ARG;
    std::vector<Plane> pl, pr;
    build_pyramid(t, imL, w, h, w, nullptr, 0, pl);
    build_pyramid(t, imR, w, h, w, nullptr, 0, pr);
    for (int i = 0; i < nl; ++i) u_right[i] = depth[i] = -1.0f;  // 586-587
    const int n_rows = pl[0].h;                                   // 589
    // row table (591-606): right keypoint iR is listed in rows floor(y-r) .. ceil(y+r)
    std::vector<std::vector<int>> rows(n_rows);
    for (int ir = 0; ir < nr; ++ir) {
        const float ky = kr[ir].y;
        const float r = 2.0f * t.scale[kr[ir].octave];
        const int maxr = (int)std::ceil(ky + r);
        const int minr = (int)std::floor(ky - r);
        for (int yi = minr; yi <= maxr; ++yi) {
            if (yi < 0 || yi >= n_rows) return ORBFE_ERR_UNSUPPORTED;  // out-of-range vector index
            rows[yi].push_back(ir);
        }
    }
    const float min_z = b, min_d = -3, max_d = bf / min_z;  // 609-611
    std::vector<std::pair<int, int>> dist_idx;              // vDistIdx
    for (int il = 0; il < nl; ++il) {
        const orbfe_keypoint& kpl = kl[il];
        const int level_l = kpl.octave;
        const float vl = kpl.y, ul = kpl.x;
        const size_t row = (size_t)vl;  // vRowIndices[vL]: float -> size_t
        if (row >= (size_t)n_rows) return ORBFE_ERR_UNSUPPORTED;
        const std::vector<int>& cand = rows[row];
        if (cand.empty()) continue;
        const float min_u = ul - max_d, max_u = ul - min_d;
        if (max_u < 0) continue;
        int best_dist = kThHigh;
        int best_ir = 0;
        for (int ir : cand) {  // 641-660
            const orbfe_keypoint& kpr = kr[ir];
            if (kpr.octave < level_l - 1 || kpr.octave > level_l + 1) continue;
            const float ur = kpr.x;
            if (ur >= min_u && ur <= max_u) {
                const int d = descriptor_distance(dl + 32 * (size_t)il, dr + 32 * (size_t)ir);
                if (d < best_dist) { best_dist = d; best_ir = ir; }
            }
        }
        if (best_dist >= kThHigh) continue;
        // sub-pixel match by correlation (663-735)
        const float ur0 = kr[best_ir].x;
        const float sf = t.inv[level_l];
        const float sul = std::round(kpl.x * sf), svl = std::round(kpl.y * sf);
        const float sur0 = std::round(ur0 * sf);
        const int W5 = 5, L5 = 5;
        const Plane& PL = pl[level_l];
        const Plane& PR = pr[level_l];
        const int r0 = (int)(svl - W5), c0 = (int)(sul - W5);
        if (r0 < 0 || r0 + 2 * W5 + 1 > PL.h || c0 < 0 || c0 + 2 * W5 + 1 > PL.w)
            return ORBFE_ERR_UNSUPPORTED;  // rowRange / colRange assert (CV_Assert)
        const float iniu = sur0 + L5 - W5, endu = sur0 + L5 + W5 + 1;  // 684-685
        if (iniu < 0 || endu >= PR.w) continue;
        const int rc0 = (int)(sur0 - L5 - W5);
        if (rc0 < 0 || (int)(sur0 + L5 + W5 + 1) > PR.w) return ORBFE_ERR_UNSUPPORTED;
        float il_win[11][11];
        for (int y = 0; y < 11; ++y)
            for (int x = 0; x < 11; ++x) il_win[y][x] = (float)PL.at(r0 + y, c0 + x);
        const float ilc = il_win[W5][W5];
        for (int y = 0; y < 11; ++y)
            for (int x = 0; x < 11; ++x) il_win[y][x] = il_win[y][x] - ilc;
        int best_sad = INT_MAX, best_inc = 0;
        float dists[2 * L5 + 1];
        for (int inc = -L5; inc <= L5; ++inc) {
            const int cc0 = (int)(sur0 + inc - W5);
            const float irc = (float)PR.at(r0 + W5, cc0 + W5);
            double acc = 0.0;  // cv::norm(NORM_L1) of two CV_32F Mats accumulates in double
            for (int y = 0; y < 11; ++y)
                for (int x = 0; x < 11; ++x)
                    acc += std::fabs(il_win[y][x] - ((float)PR.at(r0 + y, cc0 + x) - irc));
            const float dist = (float)acc;
            if (dist < best_sad) { best_sad = (int)dist; best_inc = inc; }
            dists[L5 + inc] = dist;
        }
        if (best_inc == -L5 || best_inc == L5) continue;
        const float d1 = dists[L5 + best_inc - 1], d2 = dists[L5 + best_inc], d3 = dists[L5 + best_inc + 1];
        const float delta = (d1 - d3) / (2.0f * (d1 + d3 - 2.0f * d2));
        if (delta < -1 || delta > 1) continue;
        float best_ur = t.scale[level_l] * ((float)sur0 + (float)best_inc + delta);
        float disparity = (ul - best_ur);
        if (disparity >= 0 && disparity < max_d) {
            if (disparity <= 0) {
                disparity = 0.01;
                best_ur = ul - 0.01;
            }
            depth[il] = bf / disparity;
            u_right[il] = best_ur;
            dist_idx.push_back(std::make_pair(best_sad, il));
        }
    }
    if (dist_idx.empty()) return ORBFE_OK;  // the reference reads vDistIdx[0] of an empty vector
    std::sort(dist_idx.begin(), dist_idx.end());
    const float median = dist_idx[dist_idx.size() / 2].first;
    const float th_dist = 1.5f * 1.4f * median;
    for (int i = (int)dist_idx.size() - 1; i >= 0; --i) {
        if (dist_idx[i].first < th_dist) break;
        u_right[dist_idx[i].second] = -1;
        depth[dist_idx[i].second] = -1;
    }
    return ORBFE_OK;
}

int oracle_pyramid(const orbfe_params* p, const uint8_t* img, int w, int h, size_t stride,
                   const uint8_t* mask, size_t mask_stride, uint8_t* out) {
    Tables t;
    if (!make_tables(p, t) || !img || !out) return ORBFE_ERR_ARG;
    std::vector<Plane> pyr;
    build_pyramid(t, img, w, h, stride, mask, mask_stride, pyr);
    for (const Plane& l : pyr) {
        std::memcpy(out, l.px.data(), l.px.size());
        out += l.px.size();
    }
    return ORBFE_OK;
}

int oracle_resize_linear(const uint8_t* src, int sw, int sh, size_t sstride, uint8_t* dst,
                         int dw, int dh, size_t dstride) {
    if (!src || !dst || sw <= 0 || sh <= 0 || dw <= 0 || dh <= 0) return ORBFE_ERR_ARG;
    resize_linear(src, sw, sh, sstride, dst, dw, dh, dstride);
    return ORBFE_OK;
}

int oracle_gaussian_blur(const uint8_t* src, int w, int h, size_t stride, uint8_t* dst) {
    if (!src || !dst || w <= 0 || h <= 0) return ORBFE_ERR_ARG;
    gaussian_blur(src, w, h, stride, dst, w);
    return ORBFE_OK;
}

static int emit_keys(const std::vector<Key>& v, orbfe_keypoint* out, int cap, int* n_out) {
    if (n_out) *n_out = (int)v.size();
    if ((int)v.size() > cap) return ORBFE_ERR_CAPACITY;
    for (size_t i = 0; i < v.size(); ++i)
        out[i] = orbfe_keypoint{v[i].x, v[i].y, 7.f, v[i].angle, v[i].response, v[i].octave, -1};
    return ORBFE_OK;
}

int oracle_fast(const uint8_t* roi, int rows, int cols, size_t stride, int threshold,
                orbfe_keypoint* out, int cap, int* n_out) {
    if (!roi || rows < 0 || cols < 0) return ORBFE_ERR_ARG;
    std::vector<Key> v;
    fast_detect(roi, rows, cols, stride, threshold, v);
    return emit_keys(v, out, cap, n_out);
}

int oracle_fast_keys(const orbfe_params* p, const uint8_t* level, int lw, int lh,
                     size_t stride, orbfe_keypoint* out, int cap, int* n_out) {
    Tables t;
    if (!make_tables(p, t) || !level) return ORBFE_ERR_ARG;
    Plane pl;
    pl.w = lw;
    pl.h = lh;
    pl.px.resize((size_t)lw * lh);
    for (int y = 0; y < lh; ++y) std::memcpy(&pl.px[(size_t)y * lw], level + (size_t)y * stride, lw);
    std::vector<Key> v;
    level_fast_keys(t, pl, v);
    return emit_keys(v, out, cap, n_out);
}

int oracle_distribute(const orbfe_params* p, int level, int lw, int lh,
                      const orbfe_keypoint* keys, int n, orbfe_keypoint* out, int cap,
                      int* n_out) {
    Tables t;
    if (!make_tables(p, t) || level < 0 || level >= t.nlevels) return ORBFE_ERR_ARG;
    std::vector<Key> in(n);
    for (int i = 0; i < n; ++i) in[i] = Key{keys[i].x, keys[i].y, keys[i].response};
    const int min_b = kEdge - 3;
    std::vector<Key> v = distribute(in, min_b, lw - kEdge + 3, min_b, lh - kEdge + 3, t.nfeat[level]);
    for (Key& k : v) { k.x += min_b; k.y += min_b; k.octave = level; }
    return emit_keys(v, out, cap, n_out);
}

int oracle_fast_atan2(const float* y, const float* x, int n, float* out) {
    for (int i = 0; i < n; ++i) out[i] = fast_atan2(y[i], x[i]);
    return ORBFE_OK;
}

int oracle_ic_angle(const uint8_t* level, int lw, int lh, size_t stride,
                    const orbfe_keypoint* kps, int n, float* angle) {
    Tables t;
    orbfe_params p{1000, 1.2f, 8, 20, 7};
    make_tables(&p, t);
    (void)lw; (void)lh;
    for (int i = 0; i < n; ++i) angle[i] = ic_angle(level, stride, kps[i].x, kps[i].y, t.umax);
    return ORBFE_OK;
}

int oracle_describe(const uint8_t* blurred, int lw, int lh, size_t stride,
                    const orbfe_keypoint* kps, int n, uint8_t* desc) {
    (void)lw; (void)lh;
    for (int i = 0; i < n; ++i) {
        Key k{kps[i].x, kps[i].y, kps[i].response, kps[i].angle};
        orb_descriptor(blurred, stride, k, desc + (size_t)i * 32);
    }
    return ORBFE_OK;
}

int oracle_hamming(const uint8_t* a, const uint8_t* b, int n, int32_t* dist) {
    if (n < 0 || (n && (!a || !b || !dist))) return ORBFE_ERR_ARG;
    for (int i = 0; i < n; ++i) dist[i] = descriptor_distance(a + 32 * (size_t)i, b + 32 * (size_t)i);
    return ORBFE_OK;
}

int oracle_bf_match(const uint8_t* q, int nq, const uint8_t* r, int nr, int32_t* best_idx,
                    int32_t* best_dist, int32_t* second_dist) {
    if (nq < 0 || nr < 0) return ORBFE_ERR_ARG;
    for (int i = 0; i < nq; ++i) {
        int best = 256, second = 256, bi = -1;
        for (int j = 0; j < nr; ++j) {
            const int d = descriptor_distance(q + 32 * (size_t)i, r + 32 * (size_t)j);
            if (d < best) { second = best; best = d; bi = j; }
            else if (d < second) { second = d; }
        }
        best_idx[i] = bi;
        best_dist[i] = best;
        second_dist[i] = second;
    }
    return ORBFE_OK;
}

int oracle_features_in_area(const orbfe_frame_view* f, float x, float y, float r,
                            int min_level, int max_level, int32_t* out, int cap, int* n_out) {
    Grid g;
    build_grid(f, g);
    std::vector<int> v;
    features_in_area(f, g, x, y, r, min_level, max_level, v);
    *n_out = (int)v.size();
    if ((int)v.size() > cap) return ORBFE_ERR_CAPACITY;
    for (size_t i = 0; i < v.size(); ++i) out[i] = v[i];
    return ORBFE_OK;
}

// A13 — SearchForInitialization (ORBmatcher.cc:408-523).
int oracle_search_for_initialization(float nnratio, int check_ori, const orbfe_frame_view* f1,
                                     const orbfe_frame_view* f2, float* prev_matched,
                                     int window, int32_t* matches12, int32_t* nmatches) {
    Grid g2;
    build_grid(f2, g2);
    int nm = 0;
    std::vector<int> hist[kHistLen];
    std::vector<int> matched_dist(f2->n, INT_MAX), matches21(f2->n, -1);
    for (int i = 0; i < f1->n; ++i) matches12[i] = -1;
    std::vector<int> cand;
    for (int i1 = 0; i1 < f1->n; ++i1) {
        const orbfe_keypoint& k1 = f1->keys_un[i1];
        if (k1.octave > 0) continue;
        features_in_area(f2, g2, prev_matched[2 * i1], prev_matched[2 * i1 + 1], (float)window,
                         k1.octave, k1.octave, cand);
        if (cand.empty()) continue;
        int best = INT_MAX, second = INT_MAX, bi = -1;
        for (int i2 : cand) {
            const int d = descriptor_distance(f1->desc + 32 * (size_t)i1, f2->desc + 32 * (size_t)i2);
            if (matched_dist[i2] <= d) continue;
            if (d < best) { second = best; best = d; bi = i2; }
            else if (d < second) { second = d; }
        }
        if (best <= kThLow && best < (float)second * nnratio) {
            if (matches21[bi] >= 0) {  // steal from the earlier query
                matches12[matches21[bi]] = -1;
                --nm;
            }
            matches12[i1] = bi;
            matches21[bi] = i1;
            matched_dist[bi] = best;
            ++nm;
            if (check_ori) hist[rot_bin(f1->keys_un[i1].angle, f2->keys_un[bi].angle)].push_back(i1);
        }
    }
    if (check_ori) {
        int a, b, c;
        three_maxima(hist, a, b, c);
        for (int i = 0; i < kHistLen; ++i) {
            if (i == a || i == b || i == c) continue;
            for (int i1 : hist[i])
                if (matches12[i1] >= 0) { matches12[i1] = -1; --nm; }
        }
    }
    for (int i1 = 0; i1 < f1->n; ++i1)
        if (matches12[i1] >= 0) {
            prev_matched[2 * i1] = f2->keys_un[matches12[i1]].x;
            prev_matched[2 * i1 + 1] = f2->keys_un[matches12[i1]].y;
        }
    *nmatches = nm;
    return ORBFE_OK;
}

// A14 — SearchByProjection(Frame&, vector<MapPoint*>, th) (ORBmatcher.cc:45-137).
int oracle_search_by_projection_local(float nnratio, const orbfe_frame_view* f,
                                      int32_t* frame_mp, int32_t* frame_mp_obs,
                                      const orbfe_mappoint_view* mps, const int32_t* mp_ids,
                                      float th, int32_t* nmatches) {
    for (int i = 0; i < mps->m; ++i)
        if (mps->track_in_view[i] && !mps->is_bad[i] &&
            (mps->pred_level[i] < 0 || mps->pred_level[i] >= f->nlevels))
            return ORBFE_ERR_UNSUPPORTED;
    Grid g;
    build_grid(f, g);
    const bool factor = th != 1.0;
    int nm = 0;
    std::vector<int> cand;
    for (int i = 0; i < mps->m; ++i) {
        if (!mps->track_in_view[i] || mps->is_bad[i]) continue;
        const int pl = mps->pred_level[i];
        float r = mps->view_cos[i] > 0.998 ? 2.5f : 4.0f;  // RadiusByViewingCos (131-137)
        if (factor) r *= th;
        const float rs = r * f->scale_factors[pl];
        features_in_area(f, g, mps->proj_x[i], mps->proj_y[i], rs, pl - 1, pl, cand);
        if (cand.empty()) continue;
        int best = 256, best_lvl = -1, second = 256, second_lvl = -1, bi = -1;
        for (int idx : cand) {
            if (frame_mp[idx] >= 0 && frame_mp_obs[idx] > 0) continue;
            if (f->u_right && f->u_right[idx] > 0) {
                const float er = std::fabs(mps->proj_xr[i] - f->u_right[idx]);
                if (er > r * f->scale_factors[pl]) continue;
            }
            const int d = descriptor_distance(mps->desc + 32 * (size_t)i, f->desc + 32 * (size_t)idx);
            if (d < best) {
                second = best; best = d; second_lvl = best_lvl;
                best_lvl = f->keys_un[idx].octave; bi = idx;
            } else if (d < second) {
                second_lvl = f->keys_un[idx].octave; second = d;
            }
        }
        if (best <= kThHigh) {
            if (best_lvl == second_lvl && best > nnratio * second) continue;
            frame_mp[bi] = mp_ids ? mp_ids[i] : i;
            frame_mp_obs[bi] = mps->n_obs[i];
            ++nm;
        }
    }
    *nmatches = nm;
    return ORBFE_OK;
}

// A15 — SearchByProjection(Frame& Cur, const Frame& Last, th, bMono) (ORBmatcher.cc:1331-1473).
int oracle_search_by_projection_last(int check_ori, const orbfe_frame_view* cur,
                                     const float* tcw_cur, const orbfe_camera* cam,
                                     int32_t* frame_mp, int32_t* frame_mp_obs, int n_last,
                                     const orbfe_keypoint* last_keys,
                                     const uint8_t* last_mp_valid, const uint8_t* last_outlier,
                                     const float* last_mp_xyz, const uint8_t* last_mp_desc,
                                     const int32_t* last_mp_nobs, const int32_t* last_mp_ids,
                                     const float* tcw_last, float th, int mono,
                                     int32_t* nmatches) {
    for (int i = 0; i < n_last; ++i)
        if (last_mp_valid[i] && (last_keys[i].octave < 0 || last_keys[i].octave >= cur->nlevels))
            return ORBFE_ERR_UNSUPPORTED;
    Grid g;
    build_grid(cur, g);
    float twc[3], tlc[3];
    camera_center(tcw_cur, twc);
    rigid(tcw_last, twc, tlc);
    const bool fwd = tlc[2] > cam->b && !mono;
    const bool bwd = -tlc[2] > cam->b && !mono;
    int nm = 0;
    std::vector<int> hist[kHistLen];
    std::vector<int> cand;
    for (int i = 0; i < n_last; ++i) {
        if (!last_mp_valid[i] || last_outlier[i]) continue;
        float pc[3];
        rigid(tcw_cur, last_mp_xyz + 3 * (size_t)i, pc);
        const float invz = (float)(1.0 / pc[2]);
        if (invz < 0) continue;
        const float u = cam->fx * pc[0] * invz + cam->cx;
        const float v = cam->fy * pc[1] * invz + cam->cy;
        if (u < cur->min_x || u > cur->max_x) continue;
        if (v < cur->min_y || v > cur->max_y) continue;
        const int oct = last_keys[i].octave;
        const float radius = th * cur->scale_factors[oct];
        if (fwd) features_in_area(cur, g, u, v, radius, oct, -1, cand);
        else if (bwd) features_in_area(cur, g, u, v, radius, 0, oct, cand);
        else features_in_area(cur, g, u, v, radius, oct - 1, oct + 1, cand);
        if (cand.empty()) continue;
        int best = 256, bi = -1;
        for (int i2 : cand) {
            if (frame_mp[i2] >= 0 && frame_mp_obs[i2] > 0) continue;
            if (cur->u_right && cur->u_right[i2] > 0) {
                const float ur = u - cam->bf * invz;
                if (std::fabs(ur - cur->u_right[i2]) > radius) continue;
            }
            const int d = descriptor_distance(last_mp_desc + 32 * (size_t)i, cur->desc + 32 * (size_t)i2);
            if (d < best) { best = d; bi = i2; }
        }
        if (best <= kThHigh) {
            frame_mp[bi] = last_mp_ids ? last_mp_ids[i] : i;
            frame_mp_obs[bi] = last_mp_nobs[i];
            ++nm;
            if (check_ori) hist[rot_bin(last_keys[i].angle, cur->keys_un[bi].angle)].push_back(bi);
        }
    }
    if (check_ori) {
        int a, b, c;
        three_maxima(hist, a, b, c);
        for (int i = 0; i < kHistLen; ++i) {
            if (i == a || i == b || i == c) continue;
            for (int i2 : hist[i]) { frame_mp[i2] = -1; frame_mp_obs[i2] = 0; --nm; }
        }
    }
    *nmatches = nm;
    return ORBFE_OK;
}

// Relocalisation SearchByProjection(Frame&, KeyFrame*, sAlreadyFound, th, ORBdist)
// (ORBmatcher.cc:1475-1602).  The keyframe is its n_kf map-point slots (GetMapPointMatches).
int oracle_search_by_projection_keyframe(int check_ori, const orbfe_frame_view* cur,
                                         const float* tcw_cur, const orbfe_camera* cam,
                                         float log_scale_factor, int32_t* frame_mp, int n_kf,
                                         const float* kf_key_angle, const uint8_t* kf_mp_valid,
                                         const uint8_t* kf_mp_bad, const uint8_t* already_found,
                                         const float* kf_mp_xyz, const uint8_t* kf_mp_desc,
                                         const float* kf_mp_min_dist,
                                         const float* kf_mp_max_dist, const int32_t* kf_mp_ids,
                                         float th, int orb_dist, int32_t* nmatches) {
    Grid g;
    build_grid(cur, g);
    float ow[3];
    camera_center(tcw_cur, ow);  // Ow = -Rcw^T tcw (1479-1481)
    int nm = 0;
    std::vector<int> hist[kHistLen];
    std::vector<int> cand;
    for (int i = 0; i < n_kf; ++i) {
        if (!kf_mp_valid[i] || kf_mp_bad[i] || already_found[i]) continue;
        const float* P = kf_mp_xyz + 3 * (size_t)i;
        float pc[3];
        rigid(tcw_cur, P, pc);
        const float invz = (float)(1.0 / pc[2]);
        const float u = cam->fx * pc[0] * invz + cam->cx;
        const float v = cam->fy * pc[1] * invz + cam->cy;
        if (u < cur->min_x || u > cur->max_x) continue;
        if (v < cur->min_y || v > cur->max_y) continue;
        const float po[3] = {P[0] - ow[0], P[1] - ow[1], P[2] - ow[2]};
        const float dist3d = (float)std::sqrt((double)po[0] * po[0] + (double)po[1] * po[1] +
                                              (double)po[2] * po[2]);  // cv::norm (double)
        const float max_d = 1.2f * kf_mp_max_dist[i], min_d = 0.8f * kf_mp_min_dist[i];
        if (dist3d < min_d || dist3d > max_d) continue;
        const float ratio = kf_mp_max_dist[i] / dist3d;  // PredictScale (MapPoint.cc:633-642)
        const int lvl = (int)std::ceil((float)std::log((double)ratio) / log_scale_factor);
        if (lvl < 0 || lvl >= cur->nlevels) return ORBFE_ERR_UNSUPPORTED;  // mvScaleFactors[lvl]
        const float radius = th * cur->scale_factors[lvl];
        features_in_area(cur, g, u, v, radius, lvl - 1, lvl + 1, cand);
        if (cand.empty()) continue;
        int best = 256, bi = -1;
        for (int i2 : cand) {
            if (frame_mp[i2] >= 0) continue;
            const int d = descriptor_distance(kf_mp_desc + 32 * (size_t)i, cur->desc + 32 * (size_t)i2);
            if (d < best) { best = d; bi = i2; }
        }
        if (best <= orb_dist) {
            frame_mp[bi] = kf_mp_ids ? kf_mp_ids[i] : i;
            ++nm;
            if (check_ori) hist[rot_bin(kf_key_angle[i], cur->keys_un[bi].angle)].push_back(bi);
        }
    }
    if (check_ori) {
        int a, b, c;
        three_maxima(hist, a, b, c);
        for (int i = 0; i < kHistLen; ++i) {
            if (i == a || i == b || i == c) continue;
            for (int i2 : hist[i]) { frame_mp[i2] = -1; --nm; }
        }
    }
    *nmatches = nm;
    return ORBFE_OK;
}

// MapPoint::ComputeDistinctiveDescriptors (MapPoint.cc:483-548) for n_mp map points; the
// observation descriptors of point i are rows obs_off[i] .. obs_off[i+1]-1.
int oracle_distinctive_descriptors(int n_mp, const int32_t* obs_off, const uint8_t* obs_desc,
                                   int32_t* best, uint8_t* desc_out) {
    if (n_mp < 0 || (n_mp && (!obs_off || !best))) return ORBFE_ERR_ARG;
    for (int i = 0; i < n_mp; ++i) {
        const int o = obs_off[i];
        const size_t N = (size_t)(obs_off[i + 1] - o);
        best[i] = -1;
        if (N == 0) continue;  // no observation: mDescriptor untouched (498-499, 510-511)
        std::vector<float> dmat(N * N);
        for (size_t a = 0; a < N; ++a) {
            dmat[a * N + a] = 0;
            for (size_t b = a + 1; b < N; ++b) {
                const int d = descriptor_distance(obs_desc + 32 * (size_t)(o + a), obs_desc + 32 * (size_t)(o + b));
                dmat[a * N + b] = (float)d;
                dmat[b * N + a] = (float)d;
            }
        }
        int best_median = INT_MAX, best_idx = 0;
        std::vector<int> row(N);
        for (size_t a = 0; a < N; ++a) {
            for (size_t b = 0; b < N; ++b) row[b] = (int)dmat[a * N + b];
            std::sort(row.begin(), row.end());
            const int median = row[(size_t)(0.5 * (N - 1))];
            if (median < best_median) { best_median = median; best_idx = (int)a; }
        }
        best[i] = best_idx;
        if (desc_out) std::memcpy(desc_out + 32 * (size_t)i, obs_desc + 32 * (size_t)(o + best_idx), 32);
    }
    return ORBFE_OK;
}

// ---------------------------------------------------------------------------------------------
// DBoW2 (vendored in the reference: Thirdparty/DBoW2) — TemplatedVocabulary<FORB> text format,
// transform, BowVector / FeatureVector, and ORBmatcher::SearchByBoW(KeyFrame*, Frame&, ...).
}  // extern "C"

struct oracle_vocab {
    int k = 0, L = 0, scoring = 0, weighting = 0;
    struct Node {
        int parent = 0;
        std::vector<int> children;
        uint8_t desc[32] = {};
        double weight = 0;
        int word_id = 0;  // Node() default (TemplatedVocabulary.h:329)
    };
    std::vector<Node> nodes;
    int nwords = 0;
};

namespace {
// loadFromTextFile (TemplatedVocabulary.h:1351-1436): header "k L scoring weighting", then one
// line per node "parent isLeaf d0 .. d31 weight", node ids in file order from 1.  Blank lines
// are skipped (the reference turns a trailing blank line into a phantom child
// of the root with an uninitialised descriptor).
bool vocab_parse(const char* path, oracle_vocab& v) {
    FILE* f = std::fopen(path, "r");
    if (!f) return false;
    std::string line;
    auto getline = [&](std::string& out) -> bool {
        out.clear();
        int c;
        bool any = false;
        while ((c = std::fgetc(f)) != EOF) {
            any = true;
            if (c == '\n') break;
            out.push_back((char)c);
        }
        return any;
    };
    if (!getline(line)) { std::fclose(f); return false; }
    int n1 = -1, n2 = -1;
    if (std::sscanf(line.c_str(), "%d %d %d %d", &v.k, &v.L, &n1, &n2) != 4 || v.k < 0 ||
        v.k > 20 || v.L < 1 || v.L > 10 || n1 < 0 || n1 > 5 || n2 < 0 || n2 > 3) {
        std::fclose(f);
        return false;
    }
    v.scoring = n1;
    v.weighting = n2;
    v.nodes.assign(1, oracle_vocab::Node());
    while (getline(line)) {
        const char* p = line.c_str();
        char* e;
        while (*p == ' ' || *p == '\t' || *p == '\r') ++p;
        if (!*p) continue;
        oracle_vocab::Node nd;
        nd.parent = (int)std::strtol(p, &e, 10); p = e;
        const int leaf = (int)std::strtol(p, &e, 10); p = e;
        for (int i = 0; i < 32; ++i) { nd.desc[i] = (uint8_t)std::strtol(p, &e, 10); p = e; }
        nd.weight = std::strtod(p, &e);
        const int id = (int)v.nodes.size();
        if (nd.parent < 0 || nd.parent >= id) { std::fclose(f); return false; }
        if (leaf > 0) nd.word_id = v.nwords++;
        v.nodes.push_back(nd);
        v.nodes[nd.parent].children.push_back(id);
    }
    std::fclose(f);
    return true;
}

// transform(feature, word_id, weight, &nid, levelsup) (TemplatedVocabulary.h:1233-1270)
void vocab_descend(const oracle_vocab& v, const uint8_t* d, int levelsup, int& word, double& w,
                   int& nid) {
    const int nid_level = v.L - levelsup;
    if (nid_level <= 0) nid = 0;
    int final_id = 0, level = 0;
    do {
        ++level;
        const std::vector<int>& ch = v.nodes[final_id].children;
        final_id = ch[0];
        int best = descriptor_distance(d, v.nodes[final_id].desc);
        for (size_t c = 1; c < ch.size(); ++c) {
            const int dd = descriptor_distance(d, v.nodes[ch[c]].desc);
            if (dd < best) { best = dd; final_id = ch[c]; }
        }
        if (level == nid_level) nid = final_id;
    } while (!v.nodes[final_id].children.empty());
    word = v.nodes[final_id].word_id;
    w = v.nodes[final_id].weight;
}
}  // namespace

extern "C" {
oracle_vocab* oracle_vocab_load_text(const char* path, int* status) {
    oracle_vocab* v = new oracle_vocab();
    const bool ok = path && vocab_parse(path, *v);
    if (status) *status = ok ? ORBFE_OK : ORBFE_ERR_ARG;
    if (!ok) { delete v; return nullptr; }
    return v;
}
void oracle_vocab_free(oracle_vocab* v) { delete v; }
int oracle_vocab_info(const oracle_vocab* v, int32_t* info /* k, L, scoring, weighting, nodes, words */) {
    if (!v || !info) return ORBFE_ERR_ARG;
    info[0] = v->k; info[1] = v->L; info[2] = v->scoring; info[3] = v->weighting;
    info[4] = (int32_t)v->nodes.size(); info[5] = v->nwords;
    return ORBFE_OK;
}

// TemplatedVocabulary::transform(features, BowVector, FeatureVector, levelsup)
// (TemplatedVocabulary.h:1140-1196) as called by Frame::ComputeBoW (Frame.cc:513-520).
int oracle_bow_transform(const oracle_vocab* v, const uint8_t* desc, int n, int levelsup,
                         int32_t* word_ids, double* values, int32_t* nw, int32_t* node_ids,
                         int32_t* node_off, int32_t* feat, int32_t* nn) {
    if (!v || n < 0 || (n && !desc) || !nw || !nn) return ORBFE_ERR_ARG;
    std::map<int, double> bow;
    std::map<int, std::vector<int>> fv;
    if (v->nwords > 0) {
        const bool must = v->scoring != 5;  // DotProductScoring only skips normalisation
        for (int i = 0; i < n; ++i) {
            int word = 0, nid = 0;
            double w = 0;
            vocab_descend(*v, desc + 32 * (size_t)i, levelsup, word, w, nid);
            if (w > 0) {
                if (v->weighting == 0 || v->weighting == 1) {  // TF_IDF, TF: addWeight
                    auto it = bow.find(word);
                    if (it != bow.end()) it->second += w; else bow[word] = w;
                } else {                                         // IDF, BINARY: addIfNotExist
                    bow.emplace(word, w);
                }
                fv[nid].push_back(i);
            }
        }
        if ((v->weighting == 0 || v->weighting == 1) && !bow.empty() && !must) {
            const double nd = (double)bow.size();
            for (auto& kv : bow) kv.second /= nd;
        }
        if (must) {  // BowVector::normalize: L2 for L2Scoring, L1 otherwise
            double norm = 0.0;
            if (v->scoring == 1) {
                for (auto& kv : bow) norm += kv.second * kv.second;
                norm = std::sqrt(norm);
            } else {
                for (auto& kv : bow) norm += std::fabs(kv.second);
            }
            if (norm > 0.0)
                for (auto& kv : bow) kv.second /= norm;
        }
    }
    *nw = (int32_t)bow.size();
    *nn = (int32_t)fv.size();
    int i = 0;
    for (auto& kv : bow) {
        if (word_ids) word_ids[i] = kv.first;
        if (values) values[i] = kv.second;
        ++i;
    }
    int j = 0, o = 0;
    for (auto& kv : fv) {
        if (node_ids) node_ids[j] = kv.first;
        if (node_off) node_off[j] = o;
        for (int f : kv.second) {
            if (feat) feat[o] = f;
            ++o;
        }
        ++j;
    }
    if (node_off) node_off[j] = o;
    return ORBFE_OK;
}

// ORBmatcher::SearchByBoW(KeyFrame* pKF, Frame& F, vector<MapPoint*>& vpMapPointMatches)
// (ORBmatcher.cc:159-291).  kf_mp_ok[i] = (GetMapPointMatches()[i] != NULL && !isBad());
// matches[f] = the keyframe feature matched to frame feature f, or -1.
int oracle_search_by_bow(float nnratio, int check_ori, const uint8_t* kf_desc,
                         const float* kf_angle, const uint8_t* kf_mp_ok,
                         const int32_t* kf_node_ids, const int32_t* kf_node_off,
                         const int32_t* kf_feat, int kf_nn, int n_f, const uint8_t* f_desc,
                         const float* f_angle, const int32_t* f_node_ids,
                         const int32_t* f_node_off, const int32_t* f_feat, int f_nn,
                         int32_t* matches, int32_t* nmatches) {
    if (kf_nn < 0 || f_nn < 0 || n_f < 0 || !nmatches || (n_f && !matches)) return ORBFE_ERR_ARG;
    for (int i = 0; i < n_f; ++i) matches[i] = -1;
    int nm = 0;
    std::vector<int> hist[kHistLen];
    int a = 0, b = 0;
    while (a < kf_nn && b < f_nn) {
        if (kf_node_ids[a] == f_node_ids[b]) {
            for (int x = kf_node_off[a]; x < kf_node_off[a + 1]; ++x) {
                const int ikf = kf_feat[x];
                if (!kf_mp_ok[ikf]) continue;
                const uint8_t* dkf = kf_desc + 32 * (size_t)ikf;
                int best1 = 256, bidx = -1, best2 = 256;
                for (int y = f_node_off[b]; y < f_node_off[b + 1]; ++y) {
                    const int jf = f_feat[y];
                    if (matches[jf] >= 0) continue;
                    const int d = descriptor_distance(dkf, f_desc + 32 * (size_t)jf);
                    if (d < best1) { best2 = best1; best1 = d; bidx = jf; }
                    else if (d < best2) { best2 = d; }
                }
                if (best1 <= kThLow && (float)best1 < nnratio * (float)best2) {
                    matches[bidx] = ikf;
                    if (check_ori) hist[rot_bin(kf_angle[ikf], f_angle[bidx])].push_back(bidx);
                    ++nm;
                }
            }
            ++a;
            ++b;
        } else if (kf_node_ids[a] < f_node_ids[b]) {
            while (a < kf_nn && kf_node_ids[a] < f_node_ids[b]) ++a;  // lower_bound
        } else {
            while (b < f_nn && f_node_ids[b] < kf_node_ids[a]) ++b;
        }
    }
    if (check_ori) {
        int i1, i2, i3;
        three_maxima(hist, i1, i2, i3);
        for (int i = 0; i < kHistLen; ++i) {
            if (i == i1 || i == i2 || i == i3) continue;
            for (int jf : hist[i]) { matches[jf] = -1; --nm; }
        }
    }
    *nmatches = nm;
    return ORBFE_OK;
}

// A17 — Frame::isInFrustum (Frame.cc:387-443) + MapPoint::PredictScale (MapPoint.cc:633-642).
int oracle_is_in_frustum(int n, const float* xyz, const float* normal, const float* min_dist,
                         const float* max_dist, const float* tcw, const orbfe_camera* cam,
                         float min_x, float max_x, float min_y, float max_y,
                         float log_scale_factor, float viewing_cos_limit, uint8_t* in_view,
                         float* proj_x, float* proj_y, float* proj_xr, int32_t* pred_level,
                         float* view_cos) {
    float ow[3];
    camera_center(tcw, ow);
    for (int i = 0; i < n; ++i) {
        in_view[i] = 0;
        const float* P = xyz + 3 * (size_t)i;
        float pc[3];
        rigid(tcw, P, pc);
        if (pc[2] < 0.0f) continue;
        const float invz = 1.0f / pc[2];
        const float u = cam->fx * pc[0] * invz + cam->cx;
        const float v = cam->fy * pc[1] * invz + cam->cy;
        if (u < min_x || u > max_x) continue;
        if (v < min_y || v > max_y) continue;
        const float dmax = 1.2f * max_dist[i], dmin = 0.8f * min_dist[i];
        const float po[3] = {P[0] - ow[0], P[1] - ow[1], P[2] - ow[2]};
        const float dist = (float)std::sqrt((double)po[0] * po[0] + (double)po[1] * po[1] +
                                            (double)po[2] * po[2]);
        if (dist < dmin || dist > dmax) continue;
        const float* nv = normal + 3 * (size_t)i;
        const double dot = (double)po[0] * nv[0] + (double)po[1] * nv[1] + (double)po[2] * nv[2];
        const float vc = (float)(dot / dist);
        if (vc < viewing_cos_limit) continue;
        const float ratio = max_dist[i] / dist;
        const int lvl = (int)std::ceil((float)std::log((double)ratio) / log_scale_factor);
        in_view[i] = 1;
        proj_x[i] = u;
        proj_xr[i] = u - cam->bf * invz;
        proj_y[i] = v;
        pred_level[i] = lvl;
        view_cos[i] = vc;
    }
    return ORBFE_OK;
}

}  // extern "C"

extern "C" int oracle_reference_constants(int32_t out[6]) {
    if (!out) return -1;
    const int32_t v[6] = {kPatchSize, kHalfPatch, kEdge, kThHigh, kThLow, kHistLen};
    for (int i = 0; i < 6; ++i) out[i] = v[i];
    return 0;
}
