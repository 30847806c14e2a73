// orbfe_greedy.hip — exact parallel resolution of the matchers' greedy, order-dependent
// assignment (SearchByProjection local map / last frame / keyframe; H7 in DESIGN.md).
//
// The reference visits map points i = 0, 1, ... and lets point i take its best unblocked
// candidate keypoint; a keypoint ("slot") becomes blocked for every later point once a point
// with Observations() > 0 is put there (ORBmatcher.cc:87-89, 1406-1408, 1529-1530) or if it
// already held one.  With T(s) = the index of the first such acceptor of slot s (-1 when
// blocked beforehand, +inf when never), point i sees slot s blocked iff T(s) < i, and
// T(s) = min{ i : D_i = s, nobs_i > 0 } where D_i is point i's decision.  By induction on i the
// fixed point of { D = decide(T), T = first_blocking(D) } is unique and equals the in-order
// loop, and Jacobi iteration reaches it: after a round, the lowest-index wrong decision only
// depends on correct decisions, so the correct prefix grows every round.  Each round is one
// fully parallel pass (a thread per point over its candidate list, atomicMin into the next T);
// rounds stop when no decision changed.  Three T buffers rotate (read, write, reset), so a
// round is a single launch.
//
// Final state (G2-G4): a slot ends with its LAST acceptor (points after T(s) cannot take it,
// points before it with nobs = 0 are overwritten), nmatches counts every acceptance, and the
// orientation filter (ComputeThreeMaxima, 1451-1470 / 1570-1599) clears the slot of every
// acceptance whose rotation bin is not among the three largest.
#include <hip/hip_runtime.h>

#include <climits>

#include "orbfe_device.hpp"

namespace orbfe {

constexpr int kGreedyBlock = 256;
constexpr int kGreedyLocal = 0;  // SBP local map: TH_HIGH + same-level ratio test (110-119)
constexpr int kGreedyMaxD = 1;   // best <= max_dist (last frame 1411, keyframe 1545)

struct GreedyArgs {
    int m, nkp, mode, max_dist;
    float nnratio;
    const int* off;       // m + 1
    const int2* cand;     // (slot, dist | octave << 16)
    long long cand_cap;   // entries the fill could write: a list ending past it was not
                          // filled (the host then retries with the exact total), so it is
                          // read as empty and never indexes past the buffer
    int kfix;             // > 0: fixed-slot layout, point i's candidates at i * kfix ..
    const int* fcnt;      //      with fcnt[i] of them (off unused)
    int* save_fmp;        // fused path: fmp0 / fobs0 saved here (restore point of a
    int* save_fobs;       //   speculative call)
    int* done;            // fused path (non-NULL): greedy_accept_kernel's finished-workgroup
                          //   counter (0 between calls); its last workgroup finalises
    const int* blk;       //   per-workgroup tallies of sbp_local_fused_kernel (3 each, nblk)
    int nblk;
    int* stats;           //   [1] nToMatch [2] status [3] overflow [4] chg[conv_round] [5] rounds
    int conv_round;
    const int* nobs;      // per point; NULL: every point blocks (keyframe overload)
    const int* fmp0;      // slot contents before the call (-1 = NULL)
    const int* fobs0;     // their Observations(); NULL: any held point blocks
    int* T[3];
    int* dec;             // decision per point (-2 before round 0, -1 = none)
    int* chg;             // changed decisions per round
    int* last;            // per slot: last acceptor
    int* nm;
    // orientation filter
    int check_ori;
    const float* q_angle; // per point (last-frame keypoint / keyframe keypoint angle)
    const orbfe_keypoint* k;
    int* hist;            // 30
    int* bins;            // per point
    const int* ids;       // NULL: index
    int* fmp;             // out
    int* fobs;            // out (may be NULL)
};

__device__ __forceinline__ bool greedy_preblocked(const GreedyArgs& a, int s) {
    return a.fmp0[s] >= 0 && (!a.fobs0 || a.fobs0[s] > 0);
}

__global__ __launch_bounds__(kGreedyBlock) void greedy_init_kernel(GreedyArgs a) {
    const int t = blockIdx.x * kGreedyBlock + threadIdx.x;
    if (t < a.nkp) {
        const int v = greedy_preblocked(a, t) ? -1 : INT_MAX;
        a.T[0][t] = v;
        a.T[1][t] = v;
        a.last[t] = -1;
    }
    if (t < a.m) a.dec[t] = -2;
    if (t < 30 && a.hist) a.hist[t] = 0;
    if (t == 0) *a.nm = 0;
}

// Point i's decision given T: its best candidate among the slots not blocked for it.
struct GreedyAcc {
    int best = 256, bl = -1, second = 256, sl = -1, bi = -1;
    __device__ __forceinline__ void add(const GreedyArgs& a, const int* Tc, int i, int2 c) {
        if (Tc[c.x] < i) return;
        const int d = c.y & 0xffff;
        if (a.mode == kGreedyLocal) {
            const int lv = c.y >> 16;
            if (d < best) { second = best; best = d; sl = bl; bl = lv; bi = c.x; }
            else if (d < second) { sl = lv; second = d; }
        } else if (d < best) {
            best = d;
            bi = c.x;
        }
    }
    __device__ __forceinline__ int result(const GreedyArgs& a) const {
        if (a.mode == kGreedyLocal) {
            if (best > 100) return -1;  // TH_HIGH
            if (bl == sl && best > a.nnratio * second) return -1;
            return bi;
        }
        return best <= a.max_dist ? bi : -1;
    }
};

// [e0, e1) of point i's candidates, empty when the list was not filled (past cand_cap).
__device__ __forceinline__ void greedy_range(const GreedyArgs& a, int i, int& e0, int& e1) {
    if (a.kfix) {
        e0 = i * a.kfix;
        e1 = e0 + a.fcnt[i];
        return;
    }
    e0 = a.off[i];
    e1 = a.off[i + 1];
    if (e1 > a.cand_cap) e1 = e0;
}

__device__ __forceinline__ int greedy_decide(const GreedyArgs& a, const int* Tc, int i) {
    GreedyAcc acc;
    int e0, e1;
    greedy_range(a, i, e0, e1);
    for (int e = e0; e < e1; ++e) acc.add(a, Tc, i, a.cand[e]);
    return acc.result(a);
}

// The first kCandCache candidates of a point held in registers across the rounds of the
// single-workgroup resolver (a round then costs LDS lookups only, no global load chain).
constexpr int kCandCache = 8;
struct CandCache {
    int e0, e1;
    int2 c[kCandCache];
};
__device__ __forceinline__ void cand_cache_load(const GreedyArgs& a, int i, CandCache& cc) {
    greedy_range(a, i, cc.e0, cc.e1);
#pragma unroll
    for (int k = 0; k < kCandCache; ++k) cc.c[k] = cc.e0 + k < cc.e1 ? a.cand[cc.e0 + k] : make_int2(0, 0);
}
__device__ __forceinline__ int greedy_decide_cached(const GreedyArgs& a, const int* Tc, int i,
                                                    const CandCache& cc) {
    GreedyAcc acc;
#pragma unroll
    for (int k = 0; k < kCandCache; ++k)
        if (cc.e0 + k < cc.e1) acc.add(a, Tc, i, cc.c[k]);
    for (int e = cc.e0 + kCandCache; e < cc.e1; ++e) acc.add(a, Tc, i, a.cand[e]);
    return acc.result(a);
}

// Round r: decisions from T[r % 3], first blocking acceptors into T[(r + 1) % 3] (holding the
// pre-blocked state), T[(r + 2) % 3] reset for round r + 1.  A round after a round without
// changes is a no-op (the fixed point is reached).
__global__ __launch_bounds__(kGreedyBlock) void greedy_round_kernel(GreedyArgs a, int r) {
    if (r > 0 && a.chg[r - 1] == 0) return;
    const int t = blockIdx.x * kGreedyBlock + threadIdx.x;
    const int* Tc = a.T[r % 3];
    int* Tn = a.T[(r + 1) % 3];
    int* Tz = a.T[(r + 2) % 3];
    if (t < a.nkp) Tz[t] = greedy_preblocked(a, t) ? -1 : INT_MAX;
    bool changed = false;
    if (t < a.m) {
        const int d = greedy_decide(a, Tc, t);
        if (d >= 0 && (!a.nobs || a.nobs[t] > 0)) atomicMin(&Tn[d], t);
        changed = d != a.dec[t];
        if (changed) a.dec[t] = d;
    }
    const unsigned long long b = __ballot(changed);
    if ((threadIdx.x & 63) == 0 && b) atomicAdd(&a.chg[r], __popcll(b));
}

// G2: acceptances -> last acceptor per slot, nmatches, rotation bins.
__global__ __launch_bounds__(kGreedyBlock) void greedy_accept_kernel(GreedyArgs a) {
    const int i = blockIdx.x * kGreedyBlock + threadIdx.x;
    bool acc = false;
    if (i < a.m) {
        const int s = a.dec[i];
        acc = s >= 0;
        if (acc) {
            atomicMax(&a.last[s], i);
            if (a.check_ori) {
                const int bin = rot_bin(a.q_angle[i], a.k[s].angle);
                a.bins[i] = bin;
                atomicAdd(&a.hist[bin], 1);
            }
        }
    }
    const unsigned long long b = __ballot(acc);
    if ((threadIdx.x & 63) == 0 && b) atomicAdd(a.nm, __popcll(b));
    if (!a.done) return;
    // fused path: the last workgroup to finish writes the slots (greedy_slots_kernel's work),
    // sums the candidate kernel's per-workgroup tallies and reports convergence; it resets
    // the counter for the next call
    __shared__ int is_last;
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence();
        is_last = atomicAdd(a.done, 1) == (int)gridDim.x - 1;
    }
    __syncthreads();
    if (!is_last) return;
    __threadfence();
    for (int s = threadIdx.x; s < a.nkp; s += kGreedyBlock) {
        const int j = __hip_atomic_load(&a.last[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (j < 0) continue;
        a.fmp[s] = a.ids ? a.ids[j] : j;
        if (a.fobs) a.fobs[s] = a.nobs ? a.nobs[j] : 1;
    }
    if (threadIdx.x < 64) {
        int in = 0, ovf = 0, bad = 0;
        for (int k = threadIdx.x; k < a.nblk; k += 64) {
            in += a.blk[3 * k];
            ovf += a.blk[3 * k + 1];
            bad += a.blk[3 * k + 2];
        }
        in = wave_sum(in);
        ovf = wave_sum(ovf);
        bad = wave_sum(bad);
        if (threadIdx.x == 0) {
            a.stats[1] = in;                               // nToMatch
            a.stats[2] = bad ? ORBFE_ERR_UNSUPPORTED : 0;  // a predicted level outside the pyramid
            a.stats[3] = ovf;                              // points past kSbpFix candidates
            a.stats[4] = a.chg[a.conv_round];              // 0: converged
            int r = 0;
            while (r < a.conv_round && a.chg[r] != 0) ++r;
            a.stats[5] = r + 1;                            // rounds to the fixed point
            *a.done = 0;
        }
    }
}

// G3: slot contents = last acceptor.
__global__ __launch_bounds__(kGreedyBlock) void greedy_slots_kernel(GreedyArgs a) {
    const int s = blockIdx.x * kGreedyBlock + threadIdx.x;
    if (s >= a.nkp) return;
    const int i = a.last[s];
    if (i < 0) return;
    a.fmp[s] = a.ids ? a.ids[i] : i;
    if (a.fobs) a.fobs[s] = a.nobs ? a.nobs[i] : 1;
}

// G4: orientation filter over the acceptances (every block recomputes the three maxima).
__global__ __launch_bounds__(kGreedyBlock) void greedy_ori_kernel(GreedyArgs a) {
    __shared__ int h[30];
    __shared__ int top[3];
    if (threadIdx.x < 30) h[threadIdx.x] = a.hist[threadIdx.x];
    __syncthreads();
    if (threadIdx.x == 0) three_maxima(h, top[0], top[1], top[2]);
    __syncthreads();
    const int i = blockIdx.x * kGreedyBlock + threadIdx.x;
    bool removed = false;
    if (i < a.m && a.dec[i] >= 0) {
        const int bin = a.bins[i];
        if (bin != top[0] && bin != top[1] && bin != top[2]) {
            const int s = a.dec[i];
            a.fmp[s] = -1;
            if (a.fobs) a.fobs[s] = 0;
            removed = true;
        }
    }
    const unsigned long long b = __ballot(removed);
    if ((threadIdx.x & 63) == 0 && b) atomicSub(a.nm, __popcll(b));
}

// Small problems (tracking one frame: ~1-2k points) in ONE workgroup: the same rounds, separated
// by barriers instead of launches, then G2-G4; no host round trip.  T ping-pongs between
// T[0] and T[1]: a round reads one and writes the other (pre-filled with the blocked-before
// state), then the buffer it read is reset for the next round.  The converged round count is
// left in chg[0].  T, the last-acceptor table and the blocked-before state live in LDS (4 x nkp ints), so every
// cross-thread exchange is an LDS atomic or an LDS read after a barrier.
constexpr int kGreedySmallBlock = 1024;
constexpr int kGreedySmallMax = 16384;     // points handled by the single-workgroup form
constexpr int kGreedySmallSlots = 5000;    // slots (keypoints): 4 x 4 B each within 80 KB of LDS
__global__ __launch_bounds__(kGreedySmallBlock) void greedy_small_kernel(GreedyArgs a) {
    extern __shared__ int lds[];
    __shared__ int changed, nm;
    __shared__ int h[30];
    __shared__ int top[3];
    const int tid = threadIdx.x;
    int* T[2] = {lds, lds + a.nkp};
    int* last = lds + 2 * a.nkp;
    int* pre = lds + 3 * a.nkp;  // blocked-before state per slot
    for (int s = tid; s < a.nkp; s += kGreedySmallBlock) {
        const int v = greedy_preblocked(a, s) ? -1 : INT_MAX;
        pre[s] = v;  // the per-round reset reads LDS, not the slot arrays
        T[0][s] = v;
        T[1][s] = v;
        last[s] = -1;
    }
    for (int i = tid; i < a.m; i += kGreedySmallBlock) a.dec[i] = -2;
    CandCache cc;  // the candidates of point tid (most calls have <= one point per thread)
    if (tid < a.m) cand_cache_load(a, tid, cc);
    else cc.e0 = cc.e1 = 0;
    if (tid < 30) h[tid] = 0;
    if (tid == 0) nm = 0;
    __syncthreads();
    int cur = 0, r = 0;
    while (true) {
        if (tid == 0) changed = 0;
        __syncthreads();
        const int* Tc = T[cur];
        int* Tn = T[cur ^ 1];
        bool ch = false;
        for (int i = tid; i < a.m; i += kGreedySmallBlock) {
            const int d = i == tid ? greedy_decide_cached(a, Tc, i, cc) : greedy_decide(a, Tc, i);
            if (d >= 0 && (!a.nobs || a.nobs[i] > 0)) atomicMin(&Tn[d], i);
            if (d != a.dec[i]) {
                a.dec[i] = d;
                ch = true;
            }
        }
        if (ch) changed = 1;
        __syncthreads();
        ++r;
        if (!changed) break;
        for (int s = tid; s < a.nkp; s += kGreedySmallBlock)
            T[cur][s] = pre[s];
        cur ^= 1;
        __syncthreads();
    }
    // G2: last acceptor per slot, nmatches, rotation bins
    for (int i = tid; i < a.m; i += kGreedySmallBlock) {
        const int s = a.dec[i];
        if (s < 0) continue;
        atomicMax(&last[s], i);
        atomicAdd(&nm, 1);
        if (a.check_ori) {
            const int bin = rot_bin(a.q_angle[i], a.k[s].angle);
            a.bins[i] = bin;
            atomicAdd(&h[bin], 1);
        }
    }
    __syncthreads();
    // G3: slot contents
    for (int s = tid; s < a.nkp; s += kGreedySmallBlock) {
        const int i = last[s];
        if (i < 0) continue;
        a.fmp[s] = a.ids ? a.ids[i] : i;
        if (a.fobs) a.fobs[s] = a.nobs ? a.nobs[i] : 1;
    }
    __syncthreads();
    // G4: orientation filter
    if (a.check_ori) {
        if (tid == 0) three_maxima(h, top[0], top[1], top[2]);
        __syncthreads();
        for (int i = tid; i < a.m; i += kGreedySmallBlock) {
            const int s = a.dec[i];
            if (s < 0) continue;
            const int bin = a.bins[i];
            if (bin != top[0] && bin != top[1] && bin != top[2]) {
                a.fmp[s] = -1;
                if (a.fobs) a.fobs[s] = 0;
                atomicSub(&nm, 1);
            }
        }
        __syncthreads();
    }
    if (tid == 0) {
        *a.nm = nm;
        a.chg[0] = r;
    }
}

// Single-pass form of the tracking call (Tracking::SearchLocalPoints, config 5): isInFrustum and
// the candidate search of SearchByProjection in ONE kernel, which also does greedy_init_kernel's
// work.  Every workgroup stages the frame's grid (cstart, citems) and its keypoints' x, y,
// octave in LDS, so the per-point GetFeaturesInArea walk reads LDS instead of chains of
// dependent global loads; each point writes its candidates straight to kSbpFix fixed slots
// (i * kSbpFix ..) with the count in cnt[i] (no count / scan / fill passes).  Per-workgroup
// tallies (points in view, points with more than kSbpFix candidates, predicted levels outside
// the pyramid) go to blk[3 * block ..] and greedy_accept_kernel's last workgroup sums them, so
// nothing needs clearing before the launch.  Frames of up to kSbpFixKp keypoints; an overflow
// makes the host rerun the call through the CSR path.
constexpr int kSbpFix = 16;
constexpr int kSbpFixKp = 2048;
struct SbpFusedArgs {
    FrustumArgs fr;        // in_view is written; px / py / pxr / lvl / vcos are not
    SbpLocalArgs s;        // f, mp.m, mp.desc, th, nlevels, cnt, cand
    float scalev[kMaxLevels];  // mvScaleFactors
    int* blk;              // 3 per workgroup: in view, overflow, bad level
    GreedyArgs g;          // initialised here (greedy_init_kernel's work)
    int rounds;            // g.chg[0 .. rounds] cleared
};
__global__ __launch_bounds__(256) void sbp_local_fused_kernel(SbpFusedArgs fa) {
    const SbpLocalArgs& a = fa.s;
    __shared__ int cs[kGridCells + 1];
    __shared__ int ci[kSbpFixKp];
    __shared__ float2 kxy[kSbpFixKp];
    __shared__ int8_t koct[kSbpFixKp];
    __shared__ int tally[3];
    const DevFrame& F = a.f;
    const int tid = threadIdx.x;
    const int i = blockIdx.x * 256 + tid;
    {   // greedy_init_kernel's work, spread over the grid (which covers max(m, nkp) threads)
        const GreedyArgs& g = fa.g;
        if (i < g.nkp) {
            const int v = greedy_preblocked(g, i) ? -1 : INT_MAX;
            g.T[0][i] = v;
            g.T[1][i] = v;
            g.last[i] = -1;
            g.save_fmp[i] = g.fmp0[i];
            g.save_fobs[i] = g.fobs0[i];
        }
        if (i < g.m) g.dec[i] = -2;
        if (i <= fa.rounds) g.chg[i] = 0;
        if (i == 0) *g.nm = 0;
    }
    if (tid < 3) tally[tid] = 0;
    for (int c = tid; c <= kGridCells; c += 256) cs[c] = F.cstart[c];
    for (int k = tid; k < F.n; k += 256) {
        const orbfe_keypoint kp = F.k[k];
        kxy[k] = make_float2(kp.x, kp.y);
        koct[k] = (int8_t)min(max(kp.octave, -128), 127);
    }
    __syncthreads();
    const int total = cs[kGridCells];
    for (int e = tid; e < total; e += 256) ci[e] = F.citems[e];
    __syncthreads();
    int in = 0, ovf = 0, bad_level = 0;
    if (i < a.mp.m) {
        fa.fr.in_view[i] = 0;  // isInFrustum starts with mbTrackInView = false (Frame.cc:389)
        FrustumOut o;
        int n = 0;
        if (frustum_eval(fa.fr, i, o)) {
            fa.fr.in_view[i] = 1;
            in = 1;
            const int pl = o.lvl;
            if (pl < 0 || pl >= a.nlevels) {  // F.mvScaleFactors[nPredictedLevel] out of range
                bad_level = 1;
            } else {
                float r = o.vc > 0.998 ? 2.5f : 4.0f;  // RadiusByViewingCos (131-137)
                if (a.th != 1.0) r *= a.th;
                const float rs = r * fa.scalev[pl];
                const float x = o.u, y = o.v;
                int2* out = a.cand + (size_t)i * kSbpFix;
                // GetFeaturesInArea(x, y, rs, pl - 1, pl) (Frame.cc:445-498) on the LDS copy, in
                // features_in_area's order (ix-major, iy, insertion); the level check is on
                // (maxLevel = pl >= 0)
                const int cx0 = max(0, (int)floorf((x - F.minx - rs) * F.gwi));
                const int cx1 = min(kGridCols - 1, (int)ceilf((x - F.minx + rs) * F.gwi));
                const int cy0 = max(0, (int)floorf((y - F.miny - rs) * F.ghi));
                const int cy1 = min(kGridRows - 1, (int)ceilf((y - F.miny + rs) * F.ghi));
                if (cx0 < kGridCols && cx1 >= 0 && cy0 < kGridRows && cy1 >= 0) {
                    uint4 q0 = make_uint4(0, 0, 0, 0), q1 = q0;
                    bool qd = false;
                    for (int ix = cx0; ix <= cx1; ++ix)
                        for (int iy = cy0; iy <= cy1; ++iy) {
                            const int c = ix * kGridRows + iy;
                            for (int e = cs[c], e1 = cs[c + 1]; e < e1; ++e) {
                                const int idx = ci[e];
                                const int oct = koct[idx];
                                if (oct < pl - 1 || oct > pl) continue;
                                const float2 kp = kxy[idx];
                                if (!(fabsf(kp.x - x) < rs && fabsf(kp.y - y) < rs)) continue;
                                if (F.ur && F.ur[idx] > 0) {  // stereo consistency (91-96)
                                    const float er = fabsf(o.ur - F.ur[idx]);
                                    if (er > r * fa.scalev[pl]) continue;
                                }
                                if (n < kSbpFix) {
                                    if (!qd) {
                                        q0 = a.mp.desc[2 * i];
                                        q1 = a.mp.desc[2 * i + 1];
                                        qd = true;
                                    }
                                    const uint4* d = F.desc + 2 * idx;
                                    out[n] = make_int2(idx, hamming256(q0, q1, d[0], d[1]) | (oct << 16));
                                }
                                ++n;
                            }
                        }
                }
                ovf = n > kSbpFix;
            }
        }
        a.cnt[i] = min(n, kSbpFix);
    }
    const int w_in = wave_sum(in), w_ovf = wave_sum(ovf), w_bad = wave_sum(bad_level);
    if ((tid & 63) == 0) {
        if (w_in) atomicAdd(&tally[0], w_in);
        if (w_ovf) atomicAdd(&tally[1], w_ovf);
        if (w_bad) atomicAdd(&tally[2], w_bad);
    }
    __syncthreads();
    if (tid < 3) fa.blk[3 * blockIdx.x + tid] = tally[tid];
}

}  // namespace orbfe
