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

}  // namespace orbfe
