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
    int* hstats;          //   non-NULL: [0..5] also written here (device-mapped pinned host
                          //   memory: the host reads them after the synchronisation, no D2H copy)
    int conv_round;
    const int* nobs;      // per point; NULL: every point blocks (keyframe overload)
    const int* fmp0;      // slot contents before the call (-1 = NULL)
    const int* fobs0;     // their Observations(); NULL: any held point blocks
    int* T[3];
    int* dec;             // decision per point (-2 before round 0, -1 = none)
    int* chg;             // per round: nonzero iff a decision changed
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
    if (t < a.m + 2) a.chg[t] = 0;
    if (t < kHistoLength && a.hist) a.hist[t] = 0;
    if (t == 0) *a.nm = 0;
}

// Point i's decision given T: its best candidate among the slots not blocked for it.
struct GreedyAcc {
    int best = 256, bl = -1, second = 256, sl = -1, bi = -1;
    __device__ __forceinline__ void add(const GreedyArgs& a, const int* Tc, int i, int2 c) {
        if (Tc[c.x] < i) return;
        add_unblocked(a, c);
    }
    __device__ __forceinline__ void add_unblocked(const GreedyArgs& a, int2 c) {
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
            if (best > kThHigh) return -1;  // TH_HIGH
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
    // 4 candidates and their 4 T lookups in flight at a time (the lookups depend on the
    // candidates, the accumulation on both; acc.add keeps the reference's order)
    int e = e0;
    for (; e + 4 <= e1; e += 4) {
        int2 c[4];
        int tv[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) c[k] = a.cand[e + k];
#pragma unroll
        for (int k = 0; k < 4; ++k) tv[k] = Tc[c[k].x];
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (tv[k] >= i) acc.add_unblocked(a, c[k]);
    }
    for (; e < e1; ++e) acc.add(a, Tc, i, a.cand[e]);
    return acc.result(a);
}

// The first kCandCache candidates of a point held in registers across the rounds of the
// single-workgroup resolver (a round then costs LDS lookups only, no global load chain).
constexpr int kCandCache = 16;
struct CandCache {
    int e0, e1;
    int2 c[kCandCache];
};
// (the 16 loads unconditional, at indices clamped into the point's own list — a point without
// candidates reads a zero word — so they are in flight together: loaded under the per-candidate
// condition, each was waited for before the next was issued)
__device__ int2 g_zero_int2;
__device__ __forceinline__ void cand_cache_load(const GreedyArgs& a, int i, CandCache& cc) {
    greedy_range(a, i, cc.e0, cc.e1);
    const bool any = cc.e1 > cc.e0;
#pragma unroll
    for (int k = 0; k < kCandCache; ++k) {
        // (no select on the value: the compiler turned it into a branch around the load;
        // greedy_decide_cached reads only entries below e1)
        cc.c[k] = *(any ? a.cand + min(cc.e0 + k, cc.e1 - 1) : &g_zero_int2);
    }
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
// Fixed-slot layout (kfix): the count, the first 4 candidates (one 32-byte load, read before
// the count is known: their slot indices are clamped, entries past the count ignored) and the
// point's own state are in flight together, then the 4 T lookups: two dependent global
// latencies per point instead of four.
__device__ __forceinline__ int greedy_decide_fix(const GreedyArgs& a, const int* Tc, int i) {
    const int n = a.fcnt[i];
    const int2* cp = a.cand + (size_t)i * a.kfix;
    const uint4 p0 = reinterpret_cast<const uint4*>(cp)[0], p1 = reinterpret_cast<const uint4*>(cp)[1];
    const int2 c[4] = {make_int2((int)p0.x, (int)p0.y), make_int2((int)p0.z, (int)p0.w),
                       make_int2((int)p1.x, (int)p1.y), make_int2((int)p1.z, (int)p1.w)};
    int tv[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) tv[k] = Tc[min(max(c[k].x, 0), max(a.nkp - 1, 0))];  // T holds >= 1 entry
    GreedyAcc acc;
#pragma unroll
    for (int k = 0; k < 4; ++k)
        if (k < n && tv[k] >= i) acc.add_unblocked(a, c[k]);
    for (int e = 4; e < n; ++e) acc.add(a, Tc, i, cp[e]);
    return acc.result(a);
}

// The fixed-slot round's per-point state, loaded in one round trip: the previous decision, the
// Observations() count, the candidate count and the first 4 candidates, and for the T reset the
// slot's pre-blocked state.  Every load is unconditional at a clamped index (a load under a
// branch made the compiler wait for it before issuing the next: four round trips per round).
struct FixPoint {
    int prev, nb, n, f0, o0;
    uint4 p0, p1;
};
__device__ __forceinline__ FixPoint fix_point_loads(const GreedyArgs& a, int t) {  // a.m >= 1
    const int tm = min(t, max(a.m - 1, 0)), tk = min(t, max(a.nkp - 1, 0));
    FixPoint q;
    q.prev = a.dec[tm];
    q.nb = (a.nobs ? a.nobs : a.dec)[tm];
    q.n = a.fcnt[tm];
    const uint4* cp = reinterpret_cast<const uint4*>(a.cand + (size_t)tm * a.kfix);
    q.p0 = cp[0];
    q.p1 = cp[1];
    // (a frame without keypoints may pass NULL slot arrays: then the point's own state stands in)
    const int* f0p = a.nkp > 0 ? a.fmp0 : a.dec;
    q.f0 = f0p[tk];
    q.o0 = (a.nkp > 0 && a.fobs0 ? a.fobs0 : f0p)[tk];
    return q;
}
// greedy_decide_fix on loaded state
__device__ __forceinline__ int greedy_decide_fixq(const GreedyArgs& a, const int* Tc, int i, const FixPoint& q) {
    const int2 c[4] = {make_int2((int)q.p0.x, (int)q.p0.y), make_int2((int)q.p0.z, (int)q.p0.w),
                       make_int2((int)q.p1.x, (int)q.p1.y), make_int2((int)q.p1.z, (int)q.p1.w)};
    int tv[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) tv[k] = Tc[min(max(c[k].x, 0), max(a.nkp - 1, 0))];  // T holds >= 1 entry
    GreedyAcc acc;
#pragma unroll
    for (int k = 0; k < 4; ++k)
        if (k < q.n && tv[k] >= i) acc.add_unblocked(a, c[k]);
    const int2* cp = a.cand + (size_t)i * a.kfix;
    for (int e = 4; e < q.n; ++e) acc.add(a, Tc, i, cp[e]);
    return acc.result(a);
}

// kFix: the fixed-slot layout (a.kfix > 0, the fused SearchLocalPoints path), its per-point
// loads issued before the round's no-op check; otherwise the CSR layout.
template <bool kFix>
__global__ __launch_bounds__(kGreedyBlock) void greedy_round_kernel(GreedyArgs a, int r) {
    const int t = blockIdx.x * kGreedyBlock + threadIdx.x;
    FixPoint q{};
    if constexpr (kFix) q = fix_point_loads(a, t);
    if (r > 0 && a.chg[r - 1] == 0) return;
    const int* Tc = a.T[r % 3];
    int* Tn = a.T[(r + 1) % 3];
    int* Tz = a.T[(r + 2) % 3];
    if (t < a.nkp) {
        const bool pre = kFix ? q.f0 >= 0 && (!a.fobs0 || q.o0 > 0) : greedy_preblocked(a, t);
        Tz[t] = pre ? -1 : INT_MAX;
    }
    bool changed = false;
    if (t < a.m) {
        const int prev = kFix ? q.prev : a.dec[t];
        const bool blocks = !a.nobs || (kFix ? q.nb : a.nobs[t]) > 0;
        const int d = kFix ? greedy_decide_fixq(a, Tc, t, q) : a.kfix ? greedy_decide_fix(a, Tc, t) : greedy_decide(a, Tc, t);
        // contended slots: an acceptor whose index cannot lower the slot's minimum (as read
        // now; a stale read only costs the atomic) skips the atomic
        if (d >= 0 && blocks && __hip_atomic_load(&Tn[d], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) > t)
            atomicMin(&Tn[d], t);
        changed = d != prev;
        if (changed) a.dec[t] = d;
    }
    // chg[r] only needs to be nonzero when something changed: one atomic per wave until a
    // wave sees it set (one counter hit by every wave serialised the first rounds)
    const unsigned long long b = __ballot(changed);
    if ((threadIdx.x & 63) == 0 && b &&
        __hip_atomic_load(&a.chg[r], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0)
        atomicOr(&a.chg[r], 1);
}

// G2: acceptances -> last acceptor per slot, nmatches, rotation bins.  kRound: the launch is
// also round r of the resolver (the fused path's last blind round): when round r - 1 changed
// nothing the round is a no-op and the decisions are final; otherwise this round's decisions
// are accepted and chg[r] != 0 reports that they may not be (the host then reruns the call).
// Either way a point's acceptance needs only its own decision, so no second launch.
// (kRound is the fused path's, whose layout is the fixed-slot one: its per-point loads go first)
template <bool kRound>
__global__ __launch_bounds__(kGreedyBlock) void greedy_accept_kernel(GreedyArgs a, int r) {
    const int i = blockIdx.x * kGreedyBlock + threadIdx.x;
    bool acc = false;
    FixPoint q{};
    if constexpr (kRound) q = fix_point_loads(a, i);
    if (kRound && !(r > 0 && a.chg[r - 1] == 0)) {
        const int* Tc = a.T[r % 3];
        int* Tn = a.T[(r + 1) % 3];
        bool changed = false;
        if (i < a.m) {
            const int prev = q.prev;
            const bool blocks = !a.nobs || q.nb > 0;
            const int d = greedy_decide_fixq(a, Tc, i, q);
            if (d >= 0 && blocks && __hip_atomic_load(&Tn[d], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) > i)
                atomicMin(&Tn[d], i);
            changed = d != prev;
            if (changed) a.dec[i] = d;
        }
        const unsigned long long b = __ballot(changed);
        if ((threadIdx.x & 63) == 0 && b &&
            __hip_atomic_load(&a.chg[r], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0)
            atomicOr(&a.chg[r], 1);
    }
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
    // the slots and the tallies in batches whose loads are all issued before any is used (one
    // workgroup does this work alone: a dependent load chain per element would be serial)
    for (int s0 = 0; s0 < a.nkp; s0 += 4 * kGreedyBlock) {
        int j[4], id[4], ob[4];
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const int s = s0 + threadIdx.x + kGreedyBlock * b;
            j[b] = s < a.nkp ? __hip_atomic_load(&a.last[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : -1;
        }
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            id[b] = j[b] >= 0 ? (a.ids ? a.ids[j[b]] : j[b]) : 0;
            ob[b] = j[b] >= 0 && a.fobs ? (a.nobs ? a.nobs[j[b]] : 1) : 0;
        }
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const int s = s0 + threadIdx.x + kGreedyBlock * b;
            if (j[b] < 0) continue;
            a.fmp[s] = id[b];
            if (a.fobs) a.fobs[s] = ob[b];
        }
    }
    if (threadIdx.x < 64) {
        int in = 0, ovf = 0, bad = 0;
        for (int k0 = 0; k0 < a.nblk; k0 += 4 * 64) {
            int v[4][3];
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                const int k = k0 + threadIdx.x + 64 * b;
#pragma unroll
                for (int q = 0; q < 3; ++q) v[b][q] = k < a.nblk ? a.blk[3 * k + q] : 0;
            }
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                in += v[b][0];
                ovf += v[b][1];
                bad += v[b][2];
            }
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
            if (a.hstats) {
                a.hstats[0] = __hip_atomic_load(a.nm, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                a.hstats[1] = in;
                a.hstats[2] = a.stats[2];
                a.hstats[3] = ovf;
                a.hstats[5] = r + 1;
            }
        }
    }
    // hstats[4] last, released to system scope after every thread's slot writes: the host waits
    // on it (it holds -1 until then) instead of synchronising the stream
    if (a.hstats) {
        __syncthreads();
        if (threadIdx.x == 0)
            __hip_atomic_store(&a.hstats[4], a.stats[4], __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
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
    __shared__ int h[kHistoLength];
    __shared__ int top[3];
    if (threadIdx.x < kHistoLength) h[threadIdx.x] = a.hist[threadIdx.x];
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
    __shared__ int h[kHistoLength];
    __shared__ int top[3];
    const int tid = threadIdx.x;
    int* T[2] = {lds, lds + a.nkp};
    int* last = lds + 2 * a.nkp;
    int* pre = lds + 3 * a.nkp;  // blocked-before state per slot
    for (int s = tid; s < a.nkp; s += kGreedySmallBlock) {
        // (both words loaded together: greedy_preblocked's short circuit chained them)
        const int f0 = a.fmp0[s], o0 = a.fobs0 ? a.fobs0[s] : 1;
        const int v = f0 >= 0 && o0 > 0 ? -1 : INT_MAX;
        pre[s] = v;  // the per-round reset reads LDS, not the slot arrays
        T[0][s] = v;
        T[1][s] = v;
        last[s] = -1;
    }
    for (int i = tid + kGreedySmallBlock; i < a.m; i += kGreedySmallBlock) a.dec[i] = -2;
    // point tid (most calls have <= one point per thread): its candidates, its decision and
    // whether it blocks held in registers across the rounds; further points go through memory
    CandCache cc;
    if (tid < a.m) cand_cache_load(a, tid, cc);
    else cc.e0 = cc.e1 = 0;
    int my_dec = -2;
    const int my_nobs = a.nobs ? a.nobs[min(tid, max(a.m - 1, 0))] : 1;  // (unconditional)
    const bool my_blocks = tid < a.m && my_nobs > 0;
    if (tid < kHistoLength) h[tid] = 0;
    if (tid == 0) nm = 0;
    __syncthreads();
    int cur = 0, r = 0;
    while (true) {
        if (tid == 0) changed = 0;
        __syncthreads();
        const int* Tc = T[cur];
        int* Tn = T[cur ^ 1];
        bool ch = false;
        if (tid < a.m) {
            const int d = greedy_decide_cached(a, Tc, tid, cc);
            if (d >= 0 && my_blocks) atomicMin(&Tn[d], tid);
            if (d != my_dec) {
                my_dec = d;
                ch = true;
            }
        }
        for (int i = tid + kGreedySmallBlock; i < a.m; i += kGreedySmallBlock) {
            const int d = greedy_decide(a, Tc, i);
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
    if (tid < a.m) a.dec[tid] = my_dec;  // read back by the host path's ori / slot passes
    for (int i = tid; i < a.m; i += kGreedySmallBlock) {
        const int s = i == tid ? my_dec : a.dec[i];
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
            const int s = i == tid ? my_dec : a.dec[i];
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
// kSbpLpp lanes per map point: the point's window cells are dealt round-robin over them in the
// reference's (ix-major, iy) order, so 256 points make a 1024-thread workgroup (16 waves per
// CU instead of 4: the per-point walk is LDS-latency bound).
#ifndef ORBFE_SBP_LPP
#define ORBFE_SBP_LPP 4
#endif
constexpr int kSbpLpp = ORBFE_SBP_LPP;
constexpr int kSbpPts = 1024 / kSbpLpp;  // map points per workgroup
struct SbpFusedArgs {
    FrustumArgs fr;        // in_view is written; px / py / pxr / lvl / vcos are not
    SbpLocalArgs s;        // f, mp.m, mp.desc, th, nlevels, cnt, cand
    float scalev[kMaxLevels];  // mvScaleFactors
    int* blk;              // 3 per workgroup: in view, overflow, bad level
    GreedyArgs g;          // initialised here (greedy_init_kernel's work)
    int rounds;            // g.chg[0 .. rounds] cleared
};
// exclusive / total sum over the kSbpLpp lanes of a point (aligned sub-groups of the wave)
__device__ __forceinline__ int sub_scan(int x, int& total) {
    int inc = x;
#pragma unroll
    for (int d = 1; d < kSbpLpp; d <<= 1) {
        const int y = __shfl_up(inc, d, kSbpLpp);
        if ((threadIdx.x & (kSbpLpp - 1)) >= d) inc += y;
    }
    total = __shfl(inc, kSbpLpp - 1, kSbpLpp);
    return inc - x;
}
// kPre: the isInFrustum outputs are already resident (orbfe_search_by_projection_local_device:
// a.mp's track_in_view / is_bad / projection / level / viewing cosine), so the point reads them
// instead of evaluating the frustum test and fa.fr is unused.
__device__ orbfe_keypoint g_dummy_kp;  // sbp_local_fused_kernel: a frame without keypoints
template <bool kPre>
__global__ __launch_bounds__(1024) void sbp_local_fused_kernel(SbpFusedArgs fa) {
    const SbpLocalArgs& a = fa.s;
    __shared__ int cs[kGridCells + 1];
    __shared__ int ci[kSbpFixKp];
    __shared__ float2 kxy[kSbpFixKp];
    __shared__ int8_t koct[kSbpFixKp];
    __shared__ int tally[3];
    __shared__ int scan_tmp[1024 / 64 + 1];
    // the frame's descriptors (2 x uint4 per keypoint, F.n of them: dynamic LDS sized by the
    // host), so a candidate's Hamming distance reads LDS instead of waiting on a global load
    extern __shared__ uint4 fdesc[];
    const DevFrame& F = a.f;
    const int tid = threadIdx.x;
    const int sub = tid & (kSbpLpp - 1);
    const int i = blockIdx.x * kSbpPts + tid / kSbpLpp;
    if (sub == 0) {  // greedy_init_kernel's work, spread over the grid (max(m, nkp) points)
        const GreedyArgs& g = fa.g;
        if (i < g.nkp) {  // (both words loaded together, each once)
            const int f0 = g.fmp0[i], o0 = g.fobs0[i];
            const int v = f0 >= 0 && o0 > 0 ? -1 : INT_MAX;  // greedy_preblocked (fobs0 set here)
            g.T[0][i] = v;
            g.T[1][i] = v;
            g.last[i] = -1;
            g.save_fmp[i] = f0;
            g.save_fobs[i] = o0;
        }
        if (i < g.m) g.dec[i] = -2;
        if (i <= fa.rounds) g.chg[i] = 0;
        if (i == 0) {
            *g.nm = 0;
            // the accept kernel's last-workgroup counter starts every call at 0, and its
            // convergence word reads "not converged" until that last workgroup overwrites it:
            // an accept launch that never completes sends the host to the CSR fallback instead
            // of returning a previous call's tallies
            *g.done = 0;
            g.stats[4] = -1;
        }
    }
    if (tid < 3) tally[tid] = 0;
    // Staging: every load of a batch is issued before its LDS stores (one global latency per
    // batch, not one per element).
    for (int c = tid; c <= kGridCells; c += 1024) cs[c] = 0;
    static_assert(kSbpFixKp == 2 * 1024, "two keypoints per thread");
    int mine[2] = {-1, -1};  // AssignFeaturesToGrid's cell of keypoints tid, tid + 1024
    {
        // (unconditional loads at clamped indices: a load under a branch was waited for on the
        // spot; a frame without keypoints reads a dummy record)
        float kx[2], ky[2];
        int ko[2];
        const orbfe_keypoint* kp = F.n > 0 ? F.k : &g_dummy_kp;
#pragma unroll
        for (int b = 0; b < 2; ++b) {
            const int k = min(tid + 1024 * b, max(F.n - 1, 0));
            kx[b] = kp[k].x;
            ky[b] = kp[k].y;
            ko[b] = kp[k].octave;
        }
        __syncthreads();  // cs cleared
#pragma unroll
        for (int b = 0; b < 2; ++b) {
            const int k = tid + 1024 * b;
            if (k < F.n) {
                kxy[k] = make_float2(kx[b], ky[b]);
                koct[k] = (int8_t)min(max(ko[b], -128), 127);
                // PosInGrid (Frame.cc:500-510), as grid_lds_kernel
                const int gx = (int)roundf((kx[b] - F.minx) * F.gwi);
                const int gy = (int)roundf((ky[b] - F.miny) * F.ghi);
                if (gx >= 0 && gx < kGridCols && gy >= 0 && gy < kGridRows) {
                    mine[b] = gx * kGridRows + gy;
                    atomicAdd(&cs[mine[b]], 1);
                }
            }
        }
    }
    for (int q0 = 0; q0 < 2 * F.n; q0 += 4 * 1024) {
        uint4 d[4];
#pragma unroll
        for (int b = 0; b < 4; ++b) d[b] = F.desc[min(q0 + tid + 1024 * b, 2 * F.n - 1)];
        // (stores at the same clamped indices, unconditional too: a conditional store let the
        // compiler sink each load into its branch, one global latency per load again)
#pragma unroll
        for (int b = 0; b < 4; ++b) fdesc[min(q0 + tid + 1024 * b, 2 * F.n - 1)] = d[b];
    }
    // The frame's grid built in this workgroup's LDS (grid_lds_kernel's counting sort): cs[c]
    // the start of cell c, ci its keypoints in index (insertion) order.
    __syncthreads();
    {
        constexpr int PER = (kGridCells + 1023) / 1024;
        int local[PER], sum = 0;
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            const int c = tid * PER + j;
            local[j] = c < kGridCells ? cs[c] : 0;
            sum += local[j];
        }
        int total;
        int off = block_exclusive_scan<1024>(sum, scan_tmp, total);
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            const int c = tid * PER + j;
            if (c < kGridCells) cs[c] = off;  // cursor
            off += local[j];
        }
        __syncthreads();
#pragma unroll
        for (int b = 0; b < 2; ++b)
            if (mine[b] >= 0) ci[atomicAdd(&cs[mine[b]], 1)] = tid + 1024 * b;
        __syncthreads();
        // cs[c] is now the end of cell c: sort each cell (index order), then shift to starts
        int endp[PER];
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            const int c = tid * PER + j;
            endp[j] = 0;
            if (c < kGridCells) {
                const int e = cs[c], s0 = c ? cs[c - 1] : 0;
                for (int q = s0 + 1; q < e; ++q) {
                    const int v = ci[q];
                    int b = q - 1;
                    while (b >= s0 && ci[b] > v) {
                        ci[b + 1] = ci[b];
                        --b;
                    }
                    ci[b + 1] = v;
                }
                endp[j] = c ? cs[c - 1] : 0;
            }
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            const int c = tid * PER + j;
            if (c < kGridCells) cs[c] = endp[j];
        }
        if (tid == 0) cs[kGridCells] = total;
    }
    __syncthreads();
    int in = 0, ovf = 0, bad_level = 0;
    if (i < a.mp.m) {  // every lane of the point evaluates the (cheap, uniform) frustum test
        if (!kPre && sub == 0) fa.fr.in_view[i] = 0;  // isInFrustum starts with mbTrackInView = false (Frame.cc:389)
        FrustumOut o;
        int n = 0;
        bool ok;
        if constexpr (kPre) {  // SearchByProjection's mbTrackInView / isBad skips (ORBmatcher.cc:56-60)
            ok = a.mp.in_view[i] && !a.mp.bad[i];
            if (ok) {
                o.u = a.mp.px[i];
                o.v = a.mp.py[i];
                o.ur = a.mp.pxr[i];
                o.lvl = a.mp.lvl[i];
                o.vc = a.mp.vcos[i];
            }
        } else {
            ok = frustum_eval(fa.fr, i, o);
        }
        if (ok) {
            if (sub == 0) {
                if (!kPre) fa.fr.in_view[i] = 1;
                in = 1;
            }
            const int pl = o.lvl;
            if (pl < 0 || pl >= a.nlevels) {  // F.mvScaleFactors[nPredictedLevel] out of range
                bad_level = sub == 0;
            } else {
                float r = o.vc > 0.998 ? 2.5f : 4.0f;  // RadiusByViewingCos (131-137)
                if (a.th != 1.0) r *= a.th;
                const float rs = r * fa.scalev[pl];
                const float x = o.u, y = o.v;
                int2* out = a.cand + (size_t)i * kSbpFix;
                // GetFeaturesInArea(x, y, rs, pl - 1, pl) (Frame.cc:445-498) on the LDS copy, in
                // features_in_area's order (ix-major, iy, insertion); the level check is on
                // (maxLevel = pl >= 0).  Lane sub takes window cells sub, sub + kSbpLpp, ..;
                // a sub-group scan of the per-cell counts gives each candidate its rank.
                const int cx0 = max(0, (int)floorf((x - F.minx - rs) * F.gwi));
                const int cx1 = min(kGridCols - 1, (int)ceilf((x - F.minx + rs) * F.gwi));
                const int cy0 = max(0, (int)floorf((y - F.miny - rs) * F.ghi));
                const int cy1 = min(kGridRows - 1, (int)ceilf((y - F.miny + rs) * F.ghi));
                if (cx0 < kGridCols && cx1 >= 0 && cy0 < kGridRows && cy1 >= 0) {
                    const uint4 q0 = a.mp.desc[2 * i], q1 = a.mp.desc[2 * i + 1];
                    const int ny = cy1 - cy0 + 1, ncell = (cx1 - cx0 + 1) * ny;
                    auto pass = [&](int idx) {
                        const int oct = koct[idx];
                        if (oct < pl - 1 || oct > pl) return false;
                        const float2 kp = kxy[idx];
                        if (!(fabsf(kp.x - x) < rs && fabsf(kp.y - y) < rs)) return false;
                        if (F.ur && F.ur[idx] > 0) {  // stereo consistency (91-96)
                            const float er = fabsf(o.ur - F.ur[idx]);
                            if (er > r * fa.scalev[pl]) return false;
                        }
                        return true;
                    };
                    for (int t0 = 0; t0 < ncell; t0 += kSbpLpp) {
                        const int t = t0 + sub;
                        int e0 = 0, e1 = 0, cnt = 0;
                        if (t < ncell) {
                            const int c = (cx0 + t / ny) * kGridRows + cy0 + t % ny;
                            e0 = cs[c];
                            e1 = cs[c + 1];
                            for (int e = e0; e < e1; ++e) cnt += pass(ci[e]);
                        }
                        int tot;
                        int rank = n + sub_scan(cnt, tot);
                        if (cnt)
                            for (int e = e0; e < e1; ++e) {
                                const int idx = ci[e];
                                if (!pass(idx)) continue;
                                if (rank < kSbpFix) {
                                    const uint4* d = fdesc + 2 * idx;
                                    out[rank] = make_int2(idx, hamming256(q0, q1, d[0], d[1]) | ((int)koct[idx] << 16));
                                }
                                ++rank;
                            }
                        n += tot;
                    }
                }
                ovf = sub == 0 && n > kSbpFix;
            }
        }
        if (sub == 0) a.cnt[i] = min(n, kSbpFix);
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
template __global__ void sbp_local_fused_kernel<false>(SbpFusedArgs);
template __global__ void sbp_local_fused_kernel<true>(SbpFusedArgs);

}  // namespace orbfe
