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
constexpr int kGreedyBow = 2;    // SearchByBoW: best <= TH_LOW && best < nnratio * second (236-238)

struct GreedyArgs {
    int m, nkp, mode, max_dist;
    float nnratio;
    const int* off;       // m + 1
    const int2* cand;     // (slot, dist | octave << 16)
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

__device__ __forceinline__ int greedy_decide(const GreedyArgs& a, const int* Tc, int i) {
    const int e0 = a.off[i], e1 = a.off[i + 1];
    if (a.mode == kGreedyLocal) {
        int best = 256, bl = -1, second = 256, sl = -1, bi = -1;
        for (int e = e0; e < e1; ++e) {
            const int2 c = a.cand[e];
            if (Tc[c.x] < i) continue;
            const int d = c.y & 0xffff, lv = c.y >> 16;
            if (d < best) { second = best; best = d; sl = bl; bl = lv; bi = c.x; }
            else if (d < second) { sl = lv; second = d; }
        }
        if (best > 100) return -1;  // TH_HIGH
        if (bl == sl && best > a.nnratio * second) return -1;
        return bi;
    }
    if (a.mode == kGreedyBow) {
        int best = 256, second = 256, bi = -1;
        for (int e = e0; e < e1; ++e) {
            const int2 c = a.cand[e];
            if (Tc[c.x] < i) continue;
            const int d = c.y & 0xffff;
            if (d < best) { second = best; best = d; bi = c.x; }
            else if (d < second) { second = d; }
        }
        if (best > 50) return -1;  // TH_LOW
        return (float)best < a.nnratio * (float)second ? bi : -1;
    }
    int best = 256, bi = -1;
    for (int e = e0; e < e1; ++e) {
        const int2 c = a.cand[e];
        if (Tc[c.x] < i) continue;
        const int d = c.y & 0xffff;
        if (d < best) { best = d; bi = c.x; }
    }
    return best <= a.max_dist ? bi : -1;
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

}  // namespace orbfe
