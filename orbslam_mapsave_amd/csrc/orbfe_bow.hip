// orbfe_bow.hip — DBoW2 on the GPU: the vocabulary tree of TemplatedVocabulary<FORB>
// (reference Thirdparty/DBoW2, loaded from the ORBvoc.txt text format) and
// Frame::ComputeBoW -> transform(features, BowVector, FeatureVector, levelsup)
// (Frame.cc:513-520, TemplatedVocabulary.h:1140-1270).
//
//   bow_descend_kernel   one thread per descriptor walks the tree: at each level the children
//                        in insertion order, FORB::distance (Hamming), strict '<' so the first
//                        closest child wins; records the node at level L - levelsup and the
//                        leaf's word id / weight (weight 0 = stopped word, dropped)
//   bow_assemble_kernel  one workgroup per frame: LDS bitonic sorts of (word, feature) and
//                        (node, feature) give the BowVector (ascending words; TF / TF-IDF
//                        weights summed by repeated addition in feature order, IDF / BINARY
//                        first value) and the FeatureVector (ascending nodes, features in
//                        order); normalisation (L1, or L2 for L2 scoring; / nd for dot product
//                        scoring) in double with the norm accumulated in word order, as
//                        BowVector::normalize does
//
// The vocabulary lives in HBM as a CSR of children (child_off / child_ids in insertion order),
// 32-byte node descriptors, word ids and double weights (≈ 40 B per node: ~45 MB for the
// 1.1M-node ORBvoc).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <climits>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/orbfe.h"
#include "orbfe_device.hpp"

namespace orbfe {

constexpr int kBowMaxFeatures = 4096;  // features per frame the assembly sorts in LDS
constexpr int kBowBlock = 1024;

struct VocabDev {
    int L, nodes, nwords, scoring, weighting;
    const int* child_off;  // nodes + 1
    const int* child_ids;
    const uint4* desc;     // 2 per node
    const int* word;       // word id (0 for nodes that are not words, as Node())
    const double* weight;
};

struct BowArgs {
    VocabDev v;
    int levelsup, cap;          // cap: features per frame slot (descriptor / output stride)
    const uint4* desc;          // [frame][cap] x 2
    const int* n;               // [frame] features
    int* f_word;                // [frame][cap] scratch: word, node, weight per feature
    int* f_node;
    double* f_w;
    int* word_ids;              // [frame][cap]
    double* values;             // [frame][cap]
    int* nw;                    // [frame]
    int* node_ids;              // [frame][cap]
    int* node_off;              // [frame][cap + 1]
    int* feat;                  // [frame][cap]
    int* nn;                    // [frame]
};

__global__ __launch_bounds__(256) void bow_descend_kernel(BowArgs a) {
    const int f = blockIdx.y;
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= a.n[f]) return;
    const size_t o = (size_t)f * a.cap + i;
    const uint4 q0 = a.desc[2 * o], q1 = a.desc[2 * o + 1];
    const VocabDev& v = a.v;
    const int nid_level = v.L - a.levelsup;
    int nid = 0, node = 0, level = 0;
    do {
        ++level;
        const int c0 = v.child_off[node], c1 = v.child_off[node + 1];
        node = v.child_ids[c0];
        int best = hamming256(q0, q1, v.desc[2 * node], v.desc[2 * node + 1]);
        for (int c = c0 + 1; c < c1; ++c) {
            const int id = v.child_ids[c];
            const int d = hamming256(q0, q1, v.desc[2 * id], v.desc[2 * id + 1]);
            if (d < best) {
                best = d;
                node = id;
            }
        }
        if (level == nid_level) nid = node;
    } while (v.child_off[node + 1] > v.child_off[node]);
    a.f_word[o] = v.word[node];
    a.f_node[o] = nid;
    a.f_w[o] = v.weight[node];
}

// LDS bitonic sort of n_pad 64-bit keys by all threads of the block.
__device__ __forceinline__ void bitonic_sort_u64(unsigned long long* k, int n_pad) {
    for (int size = 2; size <= n_pad; size <<= 1) {
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            for (int t = threadIdx.x; t < n_pad / 2; t += blockDim.x) {
                const int lo = 2 * t - (t & (stride - 1));
                const int hi = lo + stride;
                const bool up = ((lo & size) == 0);
                const unsigned long long x = k[lo], y = k[hi];
                if ((x > y) == up) {
                    k[lo] = y;
                    k[hi] = x;
                }
            }
            __syncthreads();
        }
    }
}

__global__ __launch_bounds__(kBowBlock) void bow_assemble_kernel(BowArgs a) {
    __shared__ unsigned long long keys[kBowMaxFeatures];
    __shared__ double vals[kBowMaxFeatures];
    __shared__ int pos[kBowMaxFeatures];
    __shared__ int tmp[kBowBlock / 64 + 1];
    __shared__ double s_norm;
    const int f = blockIdx.x;
    const int n = a.n[f];
    const size_t fo = (size_t)f * a.cap;
    int n_pad = 1;
    while (n_pad < n) n_pad <<= 1;
    const VocabDev& v = a.v;
    const bool must = v.scoring != 5;                 // DotProductScoring does not normalise
    const bool tf = v.weighting == 0 || v.weighting == 1;  // addWeight vs addIfNotExist
    // ---- BowVector: sort (word, feature) of the kept features
    for (int t = threadIdx.x; t < n_pad; t += kBowBlock)
        keys[t] = (t < n && a.f_w[fo + t] > 0)
                      ? ((unsigned long long)(unsigned)a.f_word[fo + t] << 32) | (unsigned)t
                      : ~0ull;
    __syncthreads();
    bitonic_sort_u64(keys, n_pad);
    // run heads -> compact index by a block scan over runs of kBowBlock-strided chunks
    int base = 0;
    for (int c = 0; c < n_pad; c += kBowBlock) {
        const int t = c + threadIdx.x;
        bool head = false;
        if (t < n_pad && keys[t] != ~0ull)
            head = t == 0 || (keys[t] >> 32) != (keys[t - 1] >> 32);
        int total;
        const int ex = block_exclusive_scan<kBowBlock>(head ? 1 : 0, tmp, total);
        if (head) pos[t] = base + ex;
        base += total;
        __syncthreads();
    }
    const int nw = base;
    // value of each word: weights summed in feature order (TF / TF-IDF) or the first (IDF /
    // BINARY); a run's features are sorted by index, i.e. in insertion order
    for (int c = 0; c < n_pad; c += kBowBlock) {
        const int t = c + threadIdx.x;
        if (t < n_pad && keys[t] != ~0ull && (t == 0 || (keys[t] >> 32) != (keys[t - 1] >> 32))) {
            const unsigned wd = (unsigned)(keys[t] >> 32);
            const double w = a.f_w[fo + (unsigned)(keys[t] & 0xffffffffu)];
            double s = w;
            if (tf)
                for (int u = t + 1; u < n_pad && keys[u] != ~0ull && (unsigned)(keys[u] >> 32) == wd; ++u) s += w;
            vals[pos[t]] = s;
            a.word_ids[fo + pos[t]] = (int)wd;
        }
    }
    __syncthreads();
    __shared__ int s_div;
    if (threadIdx.x == 0) {
        double norm = 0.0;
        int div = 0;
        if (must) {  // BowVector::normalize, norm accumulated in ascending word order
            if (v.scoring == 1) {
                for (int i = 0; i < nw; ++i) norm += vals[i] * vals[i];
                norm = sqrt(norm);
            } else {
                for (int i = 0; i < nw; ++i) norm += fabs(vals[i]);
            }
            div = norm > 0.0;
        } else if (tf && nw > 0) {
            norm = (double)nw;  // TF / TF-IDF without normalisation: / nd (1174-1180)
            div = 1;
        }
        s_norm = norm;
        s_div = div;
        a.nw[f] = nw;
    }
    __syncthreads();
    const double norm = s_norm;
    const bool div = s_div != 0;
    for (int i = threadIdx.x; i < nw; i += kBowBlock) a.values[fo + i] = div ? vals[i] / norm : vals[i];
    __syncthreads();
    // ---- FeatureVector: sort (node, feature) of the kept features
    for (int t = threadIdx.x; t < n_pad; t += kBowBlock)
        keys[t] = (t < n && a.f_w[fo + t] > 0)
                      ? ((unsigned long long)(unsigned)a.f_node[fo + t] << 32) | (unsigned)t
                      : ~0ull;
    __syncthreads();
    bitonic_sort_u64(keys, n_pad);
    int* noff = a.node_off + (size_t)f * (a.cap + 1);
    base = 0;
    int nvalid = 0;
    for (int c = 0; c < n_pad; c += kBowBlock) {
        const int t = c + threadIdx.x;
        const bool valid = t < n_pad && keys[t] != ~0ull;
        const bool head = valid && (t == 0 || (keys[t] >> 32) != (keys[t - 1] >> 32));
        if (valid) a.feat[fo + t] = (int)(keys[t] & 0xffffffffu);
        int total;
        const int ex = block_exclusive_scan<kBowBlock>(head ? 1 : 0, tmp, total);
        if (head) {
            a.node_ids[fo + base + ex] = (int)(keys[t] >> 32);
            noff[base + ex] = t;  // kept features are sorted first: position = CSR offset
        }
        base += total;
        nvalid += block_sum<kBowBlock>(valid ? 1 : 0, tmp);
    }
    if (threadIdx.x == 0) {
        noff[base] = nvalid;
        a.nn[f] = base;
    }
}

// ---------------------------------------------------------------------------------------------
// ORBmatcher::SearchByBoW(KeyFrame* pKF, Frame& F, vector<MapPoint*>&) (ORBmatcher.cc:159-291),
// over P (keyframe, frame) pairs at once: Tracking::Relocalization matches the current frame
// against every candidate keyframe (Tracking.cc:1636-1656), and the host form is P = 1.
// Keyframes and frames are "slots" in the layout orbfe_bow_transform_batch_device writes:
// per slot s, features at s*cap (descriptors 32 B each, angles, map-point flags, FeatureVector
// node ids and feature indices), node offsets at s*(cap + 1), node counts nn[s].
struct BowMatchArgs {
    int kf_cap, f_cap;
    const int* pair_kf;       // [P] keyframe slot per pair (NULL: slot 0)
    const int* pair_f;        // [P] frame slot per pair (NULL: slot 0)
    const int* kf_nn;         // [slot] FeatureVector nodes
    const int* kf_node_ids;
    const int* kf_node_off;
    const int* kf_feat;
    const uint8_t* kf_ok;     // map point present and not bad
    const uint4* kf_desc;
    const float* kf_angle;    // pKF->mvKeysUn[i].angle
    const int* f_nn;
    const int* f_node_ids;
    const int* f_node_off;
    const int* f_feat;
    const uint4* f_desc;
    const float* f_angle;     // F.mvKeys[i].angle
    int* matches;             // [P][f_cap] keyframe feature per frame feature, -1 = NULL
    int* bins;                // [P][f_cap] scratch: rotation bin of each match
    int* hist;                // [P][32] rotation histogram
    int* nm;                  // [P] nmatches
    int* done;                // [P] workgroups of the pair that finished the node loop
    int* status;              // ORBFE_ERR_UNSUPPORTED / ORBFE_ERR_ARG on bad input
    // host form (one pair): the pair's last workgroup also copies matches[0, out_n) and
    // {nm, status} here — the device-mapped pinned staging buffer — so the call needs no
    // download kernel or copy after the search
    int* out_host;
    int out_n;
};

// One workgroup per pair: vpMapPointMatches = NULL (164), empty histogram, nmatches = 0, the
// pair's finished-workgroup counter; workgroup 0 clears the status.
__global__ __launch_bounds__(256) void bow_init_kernel(BowMatchArgs a) {
    const int p = blockIdx.x;
    int* mt = a.matches + (size_t)p * a.f_cap;
    for (int j = threadIdx.x; j < a.f_cap; j += 256) mt[j] = -1;
    if (threadIdx.x < 32) a.hist[p * 32 + threadIdx.x] = 0;
    if (threadIdx.x == 0) {
        a.nm[p] = 0;
        a.done[p] = 0;
        if (p == 0) *a.status = 0;
    }
}

// The orientation filter (259-281) of pair p over its matched frame features, by one workgroup.
__device__ void bow_ori_filter(const BowMatchArgs& a, int p) {
    __shared__ int top[3];
    if (threadIdx.x == 0) three_maxima(a.hist + p * 32, top[0], top[1], top[2]);
    __syncthreads();
    int* matches = a.matches + (size_t)p * a.f_cap;
    const int* bins = a.bins + (size_t)p * a.f_cap;
    int removed = 0;
    for (int j = threadIdx.x; j < a.f_cap; j += blockDim.x) {
        if (matches[j] < 0) continue;
        const int bin = bins[j];
        if (bin != top[0] && bin != top[1] && bin != top[2]) {
            matches[j] = -1;
            ++removed;
        }
    }
    if (removed) atomicSub(&a.nm[p], removed);
}

// A frame feature belongs to exactly one vocabulary node, so the blocking
// (vpMapPointMatches[realIdxF] != NULL) only couples keyframe features of the same common node:
// each node's loop (198-245) is run by one wave, in the reference's order, and the nodes run in
// parallel (waves stride over the keyframe's nodes; grid.y = pairs).  Lanes hold the node's
// frame features (candidate rank r = lane + 64 j, i.e. vIndicesF order); for each keyframe
// feature the wave computes every unmatched candidate's distance, best = min (distance << 16 |
// rank) -- the first minimum in order -- and second = the smallest distance of the other
// candidates, which is exactly what the sequential best/second update yields.  The rotation
// histogram is accumulated with atomics; bow_ori_kernel then applies ComputeThreeMaxima
// (259-281) and clears the slots of the non-top bins.
constexpr int kBowSearchBlock = 256;   // 4 waves
constexpr int kBowNodeMax = 256;  // frame features per node handled in registers (4 per lane)
__device__ __forceinline__ int bow_pair_of(const int* f_node_ids, int f_nn, int id) {
    int lo = 0, hi = f_nn;  // FeatureVector::lower_bound in the frame's nodes
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (f_node_ids[mid] < id) lo = mid + 1; else hi = mid;
    }
    return (lo < f_nn && f_node_ids[lo] == id) ? lo : -1;
}

__global__ __launch_bounds__(kBowSearchBlock) void bow_search_kernel(BowMatchArgs a, float nnratio,
                                                                     int check_ori) {
    const int lane = threadIdx.x & 63;
    const int p = blockIdx.y;
    const int ks = a.pair_kf ? a.pair_kf[p] : 0, fs = a.pair_f ? a.pair_f[p] : 0;
    const int kf_nn = a.kf_nn[ks], f_nn = a.f_nn[fs];
    const size_t kb = (size_t)ks * a.kf_cap, fbase = (size_t)fs * a.f_cap;
    const int* kf_node_ids = a.kf_node_ids + kb;
    const int* kf_node_off = a.kf_node_off + (size_t)ks * (a.kf_cap + 1);
    const int* kf_feat = a.kf_feat + kb;
    const uint8_t* kf_ok = a.kf_ok + kb;
    const uint4* kf_desc = a.kf_desc + 2 * kb;
    const float* kf_angle = a.kf_angle + kb;
    const int* f_node_ids = a.f_node_ids + fbase;
    const int* f_node_off = a.f_node_off + (size_t)fs * (a.f_cap + 1);
    const int* f_feat = a.f_feat + fbase;
    const uint4* f_desc = a.f_desc + 2 * fbase;
    const float* f_angle = a.f_angle + fbase;
    int* matches = a.matches + (size_t)p * a.f_cap;
    int* bins = a.bins + (size_t)p * a.f_cap;
    int* hist = a.hist + p * 32;
    const bool bad = kf_nn < 0 || kf_nn > a.kf_cap || f_nn < 0 || f_nn > a.f_cap;
    if (bad && threadIdx.x == 0) atomicExch(a.status, ORBFE_ERR_ARG);
    const int nwaves = gridDim.x * (kBowSearchBlock / 64);
    const int n_nodes = bad ? 0 : kf_nn;
    for (int na = blockIdx.x * (kBowSearchBlock / 64) + (threadIdx.x >> 6); na < n_nodes; na += nwaves) {
        const int fb = bow_pair_of(f_node_ids, f_nn, kf_node_ids[na]);
        if (fb < 0) continue;
        const int y0 = f_node_off[fb], ny = f_node_off[fb + 1] - y0;
        const int x0 = kf_node_off[na], nx = kf_node_off[na + 1] - x0;
        if (y0 < 0 || ny < 0 || y0 + ny > a.f_cap || x0 < 0 || nx < 0 || x0 + nx > a.kf_cap) {
            if (lane == 0) atomicExch(a.status, ORBFE_ERR_ARG);
            continue;
        }
        if (ny > kBowNodeMax) {
            if (lane == 0) atomicExch(a.status, ORBFE_ERR_UNSUPPORTED);
            continue;
        }
        int jf[4];
        uint4 d0[4], d1[4];
        bool free_[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int r = lane + 64 * j;
            jf[j] = r < ny ? f_feat[y0 + r] : -1;
            free_[j] = jf[j] >= 0 && jf[j] < a.f_cap;
            d0[j] = free_[j] ? f_desc[2 * jf[j]] : make_uint4(0, 0, 0, 0);
            d1[j] = free_[j] ? f_desc[2 * jf[j] + 1] : make_uint4(0, 0, 0, 0);
        }
        // the node's keyframe features are fetched by the lanes in parallel (64 at a time) and
        // broadcast in order, so the sequential loop carries no memory latency
        for (int xb = 0; xb < nx; xb += 64) {
            const int xl = xb + lane;
            int my_ikf = -1;
            uint4 my0 = make_uint4(0, 0, 0, 0), my1 = my0;
            if (xl < nx) {
                my_ikf = kf_feat[x0 + xl];
                if (my_ikf < 0 || my_ikf >= a.kf_cap || !kf_ok[my_ikf]) {
                    my_ikf = -1;
                } else {
                    my0 = kf_desc[2 * my_ikf];
                    my1 = kf_desc[2 * my_ikf + 1];
                }
            }
            const int cnt = min(64, nx - xb);
            const int nj = (ny + 63) >> 6;  // candidate registers in use (wave-uniform)
            for (int t = 0; t < cnt; ++t) {
                // t is wave-uniform: v_readlane into scalar registers, no LDS round trip
                const int ikf = __builtin_amdgcn_readlane(my_ikf, t);
                if (ikf < 0) continue;
                const uint4 q0 = make_uint4(__builtin_amdgcn_readlane(my0.x, t),
                                            __builtin_amdgcn_readlane(my0.y, t),
                                            __builtin_amdgcn_readlane(my0.z, t),
                                            __builtin_amdgcn_readlane(my0.w, t));
                const uint4 q1 = make_uint4(__builtin_amdgcn_readlane(my1.x, t),
                                            __builtin_amdgcn_readlane(my1.y, t),
                                            __builtin_amdgcn_readlane(my1.z, t),
                                            __builtin_amdgcn_readlane(my1.w, t));
                uint32_t key = 0xffffffffu;
                int dist[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    dist[j] = 256;
                    if (j < nj && free_[j]) {
                        dist[j] = hamming256(q0, q1, d0[j], d1[j]);
                        key = min(key, ((uint32_t)dist[j] << 16) | (uint32_t)(lane + 64 * j));
                    }
                }
                key = __ockl_wfred_min_u32(key);  // DPP wave reduction
                const int b1 = key == 0xffffffffu ? 256 : (int)(key >> 16);
                const int brank = (int)(key & 0xffff);
                int sec = 256;
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    if (j < nj && free_[j] && lane + 64 * j != brank) sec = min(sec, dist[j]);
                sec = __ockl_wfred_min_i32(sec);
                if (b1 <= kThLow && (float)b1 < nnratio * (float)sec) {  // TH_LOW, ratio (233-237)
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        if (lane + 64 * j == brank) {
                            free_[j] = false;
                            matches[jf[j]] = ikf;
                            if (check_ori) {
                                const int bin = rot_bin(kf_angle[ikf], f_angle[jf[j]]);
                                bins[jf[j]] = bin;
                                atomicAdd(&hist[bin], 1);
                            }
                            atomicAdd(&a.nm[p], 1);
                        }
                    }
                }
            }
        }
    }
    if (!check_ori && !a.out_host) return;
    // the pair's last workgroup to finish runs the orientation filter: release this
    // workgroup's matches / bins, count it, and the last one acquires everyone's
    __shared__ int last;
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence();
        last = atomicAdd(&a.done[p], 1) == (int)gridDim.x - 1;
    }
    __syncthreads();
    if (!last) return;
    __threadfence();
    if (check_ori) bow_ori_filter(a, p);
    if (a.out_host) {  // host form: results straight into the pinned staging buffer
        __syncthreads();
        for (int j = threadIdx.x; j < a.out_n; j += blockDim.x) a.out_host[2 + j] = matches[j];
        if (threadIdx.x == 0) {
            a.out_host[0] = atomicAdd(&a.nm[p], 0);
            a.out_host[1] = atomicAdd(a.status, 0);
        }
    }
}

// Host form, one (keyframe, frame) pair with at most kBow1Nodes common nodes: the host walks the
// two FeatureVectors as the reference does (ORBmatcher.cc:195-256: equal node ids are matched,
// otherwise the lagging side jumps to lower_bound of the other's id) and gathers each common
// node's features, in the reference's order, into the device-mapped pinned staging buffer —
// keyframe features without a good map point (202-207) left out — so a node's workgroup reads
// its descriptors, indices and angles in one round of loads with no index chain (the common
// nodes themselves ride in the kernel arguments).  Each frame feature's outcome — its keyframe
// feature and rotation bin, or -1 — is written to its own slot of the pinned output (one slot per
// gathered frame feature: no counter, no atomics); the host waits on the slots and applies the
// orientation filter (259-281, ComputeThreeMaxima over the slots) as the reference does on the
// CPU: one launch per call.
constexpr int kBow1Nodes = 192;
constexpr int kSlotPending = INT_MIN;  // an output slot the kernel has not written yet
constexpr int kSlotWaitUs = 2000;      // slot polling before the stream synchronisation
struct Bow1Args {
    const uint4* kd;  // keyframe features in node order: descriptors (2 x uint4 each),
    const int* ki;    //   keyframe feature indices,
    const float* ka;  //   angles (pKF->mvKeysUn[i].angle)
    const uint4* fd;  // frame features in node order: descriptors,
    const int* fi;    //   frame feature indices,
    const float* fa;  //   angles (F.mvKeys[i].angle)
    int* out;         // pinned, one slot per gathered frame feature: kf << 5 | bin, or -1
    int nodes;
    int4 node[kBow1Nodes];  // (keyframe start, count, frame start, count) per common node
};

// One workgroup per common node.  The node's loop over its keyframe features t is sequential in
// the reference (a frame feature taken by an earlier t is skipped, 212); here it is two parallel
// steps per chunk of up to 256 keyframe features (one per thread):
//   A. every (t, frame feature) distance, on all four waves (lane = t; the chunk's 64-lane blocks
//      times a split of the frame features fill the waves; frame descriptors broadcast from LDS),
//      reduced to each t's kBowK smallest keys dist << 16 | frame rank;
//   B. the greedy order as a fixed point (as the SearchForInitialization rounds, §4): every t
//      decides at once against the claims of the previous round — a frame feature counts as taken
//      for t when an earlier t (this chunk's or a finished chunk's) claimed it — and the rounds
//      repeat until no decision changes.  After round k the decisions of the first k keyframe
//      features are final, so the fixed point is the sequential result; it is reached in 2-4
//      rounds on the adapter's problem.  t's best and second are its first two keys whose frame
//      features are free — exact, since every key not kept is larger; when fewer than two of the
//      kept keys are free (and more frame features exist) the wave recomputes t's two smallest
//      free keys over the node, one such t at a time.
// Ties: keys order equal distances by rank, so the first frame feature wins and counts as the
// second too, as the strict < updates of 226-231 do.
constexpr int kBow1Chunk = 256;  // keyframe features per chunk (one per thread)
constexpr int kBowK = 8;         // smallest keys kept per keyframe feature
__device__ __forceinline__ void topk_insert(uint32_t (&t)[kBowK], uint32_t k) {
#pragma unroll
    for (int i = kBowK - 1; i > 0; --i) t[i] = min(t[i], max(t[i - 1], k));
    t[0] = min(t[0], k);
}

__global__ __launch_bounds__(256) void bow_search1_kernel(Bow1Args a, float nnratio, int check_ori) {
    __shared__ uint4 fdesc[2 * kBowNodeMax];   // the node's frame descriptors
    __shared__ uint4 kdesc[2 * kBow1Chunk];    // the chunk's keyframe descriptors
    __shared__ uint4 part[kBowK / 4 * kBow1Chunk];  // partial smallest keys, [split][t][kBowK / 4]
    __shared__ float fang[kBowNodeMax];
    __shared__ int prior[kBowNodeMax];         // claim of a finished chunk (node-wide t), or INT_MAX
    __shared__ int owner[2][kBowNodeMax];      // claims of a round: smallest claiming t
    __shared__ int res[kBowNodeMax];           // per frame feature: kf << 5 | bin, or -1
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int4 nd = a.node[blockIdx.x];
    const int x0 = nd.x, nx = nd.y, y0 = nd.z, ny = nd.w;  // ny <= kBowNodeMax (host-checked)
    // the frame features and the first chunk's keyframe features in one round of loads (the
    // inputs are in device-mapped host memory: each round is a PCIe round trip)
    uint4 f0 = make_uint4(0, 0, 0, 0), f1 = f0, c0 = f0, c1 = f0;
    float fa = 0.f, ang = 0.f;
    int ikf = -1;
    if (tid < ny) {
        f0 = a.fd[2 * (y0 + tid)];
        f1 = a.fd[2 * (y0 + tid) + 1];
        fa = a.fa[y0 + tid];
    }
    if (tid < min(nx, kBow1Chunk)) {
        c0 = a.kd[2 * (x0 + tid)];
        c1 = a.kd[2 * (x0 + tid) + 1];
        ikf = a.ki[x0 + tid];
        ang = a.ka[x0 + tid];
    }
    if (tid < ny) {
        fdesc[2 * tid] = f0;
        fdesc[2 * tid + 1] = f1;
        fang[tid] = fa;
        prior[tid] = INT_MAX;
        owner[0][tid] = INT_MAX;
        res[tid] = -1;
    }
    for (int xc = 0; xc < nx; xc += kBow1Chunk) {
        const int T = min(kBow1Chunk, nx - xc);
        const bool mine = tid < T;  // thread tid is the chunk's t = tid (node-wide xc + tid)
        if (mine) {
            if (xc) {
                c0 = a.kd[2 * (x0 + xc + tid)];
                c1 = a.kd[2 * (x0 + xc + tid) + 1];
                ikf = a.ki[x0 + xc + tid];
                ang = a.ka[x0 + xc + tid];
            }
            kdesc[2 * tid] = c0;
            kdesc[2 * tid + 1] = c1;
        }
        __syncthreads();
        // A. wave wv: block tb of the chunk's t, frame features sp, sp + S, ...
        const int TB = (T + 63) >> 6, S = TB == 1 ? 4 : TB == 2 ? 2 : 1;
        uint32_t kk[kBowK];
#pragma unroll
        for (int u = 0; u < kBowK; ++u) kk[u] = 0xffffffffu;
        if (wv < TB * S) {
            const int tb = wv / S, sp = wv % S, t = tb * 64 + lane;
            const uint4 q0 = kdesc[2 * t], q1 = kdesc[2 * t + 1];
            for (int r = sp; r < ny; r += S)
                topk_insert(kk, ((uint32_t)hamming256(q0, q1, fdesc[2 * r], fdesc[2 * r + 1]) << 16) | (uint32_t)r);
            uint4* pp = part + (kBowK / 4) * (sp * (TB * 64) + t);
#pragma unroll
            for (int v = 0; v < kBowK / 4; ++v)
                pp[v] = make_uint4(kk[4 * v], kk[4 * v + 1], kk[4 * v + 2], kk[4 * v + 3]);
        }
        __syncthreads();
        if (mine) {
#pragma unroll
            for (int v = 0; v < kBowK / 4; ++v) {
                const uint4 o = part[(kBowK / 4) * tid + v];
                kk[4 * v] = o.x;
                kk[4 * v + 1] = o.y;
                kk[4 * v + 2] = o.z;
                kk[4 * v + 3] = o.w;
            }
            for (int sp = 1; sp < S; ++sp) {
#pragma unroll
                for (int v = 0; v < kBowK / 4; ++v) {
                    const uint4 o = part[(kBowK / 4) * (sp * (TB * 64) + tid) + v];
                    topk_insert(kk, o.x);
                    topk_insert(kk, o.y);
                    topk_insert(kk, o.z);
                    topk_insert(kk, o.w);
                }
            }
        }
        // B. rounds: decide against owner[cur], claim into owner[cur ^ 1]
        const int tg = xc + tid;  // node-wide t
        int dec = -1, cur = 0;
        for (int round = 0; round <= T; ++round) {
            const int* own = owner[cur];
            uint32_t kb = 0xffffffffu, ks = 0xffffffffu;
            bool known = !mine;  // both found among the kept keys, or the candidates ran out
            if (mine) {
                int ow[kBowK];  // every kept key's claim read at once (no chain of LDS reads)
#pragma unroll
                for (int u = 0; u < kBowK; ++u) ow[u] = own[min((int)(kk[u] & 0xffffu), kBowNodeMax - 1)];
#pragma unroll
                for (int u = 0; u < kBowK; ++u) {
                    if (known) break;
                    const uint32_t k = kk[u];
                    if (k == 0xffffffffu) { known = true; break; }  // no further frame features
                    if (ow[u] < tg) continue;  // taken by an earlier t
                    if (kb == 0xffffffffu) kb = k;
                    else { ks = k; known = true; }
                }
            }
            // fewer than two of the kept keys free: the wave recomputes those t one at a time
            for (unsigned long long need = __ballot(!known); need; need &= need - 1) {
                const int l = __builtin_ctzll(need);
                const int tq = (wv << 6) + l;
                const uint4 q0 = kdesc[2 * tq], q1 = kdesc[2 * tq + 1];
                uint32_t kj[4], key = 0xffffffffu;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int r = lane + 64 * j;
                    kj[j] = 0xffffffffu;
                    if (r < ny && own[r] >= xc + tq) {
                        kj[j] = ((uint32_t)hamming256(q0, q1, fdesc[2 * r], fdesc[2 * r + 1]) << 16) | (uint32_t)r;
                        key = min(key, kj[j]);
                    }
                }
                const uint32_t b = __ockl_wfred_min_u32(key);
                uint32_t k2 = 0xffffffffu;
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    if (kj[j] != b) k2 = min(k2, kj[j]);
                const uint32_t sc = __ockl_wfred_min_u32(k2);
                if (lane == l) { kb = b; ks = sc; }
            }
            const int b1 = kb == 0xffffffffu ? 256 : (int)(kb >> 16);
            const int sec = ks == 0xffffffffu ? 256 : (int)(ks >> 16);
            const int d = mine && b1 <= kThLow && (float)b1 < nnratio * (float)sec  // TH_LOW, ratio (233-237)
                              ? (int)(kb & 0xffffu) : -1;
            if (tid < ny) owner[cur ^ 1][tid] = prior[tid];
            __syncthreads();
            if (d >= 0) atomicMin(&owner[cur ^ 1][d], tg);
            const bool changed = __syncthreads_or(d != dec);
            dec = d;
            cur ^= 1;
            if (!changed) break;
        }
        // the fixed point: record the chunk's matches; they are final for the next chunk
        if (dec >= 0) {
            res[dec] = (ikf << 5) | (check_ori ? rot_bin(ang, fang[dec]) : 0);
            prior[dec] = tg;
        }
        __syncthreads();
        if (tid < ny) owner[cur][tid] = prior[tid];  // the next chunk's first round
        __syncthreads();
    }
    // every frame feature's outcome to its slot (the node's frame features are slots y0 ..): a
    // system-scope store, since the host polls the slots
    if (tid < ny) __hip_atomic_store(a.out + y0 + tid, res[tid], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

}  // namespace orbfe

using namespace orbfe;

struct orbfe_vocabulary {
    int device = 0;
    int k = 0, L = 0, scoring = 0, weighting = 0, nodes = 0, nwords = 0;
    DevBuf child_off, child_ids, desc, word, weight;
    // per-call scratch / staging (host forms)
    DevBuf s_desc, s_n, s_word, s_node, s_w, o_wid, o_val, o_nw, o_nid, o_noff, o_feat, o_nn;
    hipStream_t own = nullptr, stream = nullptr;
    // the host transform's staging: descriptors in, results out, in one device-mapped pinned
    // block the kernels read and write directly (no H2D / D2H copies); null: DMA copies
    uint8_t* pin = nullptr;
    uint8_t* pin_dev = nullptr;
    size_t pin_cap = 0;
    uint8_t* stage(size_t bytes) {
        if (bytes <= pin_cap) return pin;
        if (pin) {
            hipStreamSynchronize(stream);
            hipHostFree(pin);
        }
        pin = pin_dev = nullptr;
        pin_cap = 0;
        void* q = nullptr;
        void* dq = nullptr;
        const size_t cap = std::max<size_t>(bytes, (size_t)64 << 10);
        if (hipHostMalloc(&q, cap, hipHostMallocDefault) != hipSuccess) return nullptr;
        if (hipHostGetDevicePointer(&dq, q, 0) != hipSuccess) {
            hipHostFree(q);
            return nullptr;
        }
        pin = static_cast<uint8_t*>(q);
        pin_dev = static_cast<uint8_t*>(dq);
        pin_cap = cap;
        return pin;
    }

    VocabDev dev() const {
        return VocabDev{L, nodes, nwords, scoring, weighting, child_off.as<int>(),
                        child_ids.as<int>(), desc.as<uint4>(), word.as<int>(), weight.as<double>()};
    }
    ~orbfe_vocabulary() {
        for (DevBuf* b : {&child_off, &child_ids, &desc, &word, &weight, &s_desc, &s_n, &s_word,
                          &s_node, &s_w, &o_wid, &o_val, &o_nw, &o_nid, &o_noff, &o_feat, &o_nn})
            b->release();
        if (pin) hipHostFree(pin);
        if (own) hipStreamDestroy(own);
    }
};

namespace {
// Builds the device tree from host node arrays (node 0 = root; parent[i] < i for i >= 1).
int vocab_upload(orbfe_vocabulary* v, const std::vector<int>& parent,
                 const std::vector<uint8_t>& is_word, const std::vector<uint8_t>& desc,
                 const std::vector<double>& weight) {
    const int n = (int)parent.size();
    std::vector<int> cnt(n + 1, 0), off(n + 1, 0), ids(std::max(n - 1, 1)), word(n, 0);
    for (int i = 1; i < n; ++i) {
        if (parent[i] < 0 || parent[i] >= i) return ORBFE_ERR_ARG;
        ++cnt[parent[i]];
    }
    for (int i = 0; i < n; ++i) off[i + 1] = off[i] + cnt[i];
    std::vector<int> cur(off.begin(), off.end() - 1);
    for (int i = 1; i < n; ++i) ids[cur[parent[i]]++] = i;  // insertion (file) order
    int nw = 0;
    for (int i = 1; i < n; ++i)
        if (is_word[i]) word[i] = nw++;
    v->nodes = n;
    v->nwords = nw;
    int st;
    if ((st = v->child_off.ensure((n + 1) * sizeof(int)))) return st;
    if ((st = v->child_ids.ensure(ids.size() * sizeof(int)))) return st;
    if ((st = v->desc.ensure((size_t)n * 32))) return st;
    if ((st = v->word.ensure((size_t)n * sizeof(int)))) return st;
    if ((st = v->weight.ensure((size_t)n * sizeof(double)))) return st;
    ORBFE_HIP(hipMemcpy(v->child_off.p, off.data(), (n + 1) * sizeof(int), hipMemcpyHostToDevice));
    ORBFE_HIP(hipMemcpy(v->child_ids.p, ids.data(), ids.size() * sizeof(int), hipMemcpyHostToDevice));
    ORBFE_HIP(hipMemcpy(v->desc.p, desc.data(), (size_t)n * 32, hipMemcpyHostToDevice));
    ORBFE_HIP(hipMemcpy(v->word.p, word.data(), (size_t)n * sizeof(int), hipMemcpyHostToDevice));
    ORBFE_HIP(hipMemcpy(v->weight.p, weight.data(), (size_t)n * sizeof(double), hipMemcpyHostToDevice));
    return ORBFE_OK;
}

// TemplatedVocabulary::loadFromTextFile (TemplatedVocabulary.h:1351-1436).  Blank lines are
// skipped.
int vocab_parse_text(const char* path, int& k, int& L, int& scoring, int& weighting,
                     std::vector<int>& parent, std::vector<uint8_t>& is_word,
                     std::vector<uint8_t>& desc, std::vector<double>& weight) {
    FILE* fp = std::fopen(path, "rb");
    if (!fp) return ORBFE_ERR_ARG;
    std::vector<char> buf;
    {
        std::fseek(fp, 0, SEEK_END);
        const long sz = std::ftell(fp);
        std::fseek(fp, 0, SEEK_SET);
        if (sz < 0) { std::fclose(fp); return ORBFE_ERR_ARG; }
        buf.resize((size_t)sz + 1);
        const size_t got = std::fread(buf.data(), 1, (size_t)sz, fp);
        buf[got] = 0;
        buf.resize(got + 1);
    }
    std::fclose(fp);
    char* p = buf.data();
    char* end = buf.data() + buf.size() - 1;
    auto line_end = [&](char* s) { char* e = s; while (e < end && *e != '\n') ++e; return e; };
    char* e = line_end(p);
    *e = 0;
    int n1 = -1, n2 = -1;
    if (std::sscanf(p, "%d %d %d %d", &k, &L, &n1, &n2) != 4 || k < 0 || k > 20 || L < 1 ||
        L > 10 || n1 < 0 || n1 > 5 || n2 < 0 || n2 > 3)
        return ORBFE_ERR_ARG;
    scoring = n1;
    weighting = n2;
    parent.assign(1, 0);
    is_word.assign(1, 0);
    desc.assign(32, 0);
    weight.assign(1, 0.0);
    p = e < end ? e + 1 : end;
    while (p < end) {
        e = line_end(p);
        *e = 0;
        char* q = p;
        while (*q == ' ' || *q == '\t' || *q == '\r') ++q;
        if (*q) {
            char* r;
            const int pid = (int)std::strtol(q, &r, 10); q = r;
            const int leaf = (int)std::strtol(q, &r, 10); q = r;
            uint8_t d[32];
            for (int i = 0; i < 32; ++i) { d[i] = (uint8_t)std::strtol(q, &r, 10); q = r; }
            const double w = std::strtod(q, &r);
            if (pid < 0 || pid >= (int)parent.size()) return ORBFE_ERR_ARG;
            parent.push_back(pid);
            is_word.push_back(leaf > 0);
            desc.insert(desc.end(), d, d + 32);
            weight.push_back(w);
        }
        p = e + 1;
    }
    return ORBFE_OK;
}
}  // namespace

extern "C" {

orbfe_vocabulary* orbfe_vocabulary_load_text(const char* path, int device, int* status) {
    int st = check_device(device);
    orbfe_vocabulary* v = nullptr;
    try {
        if (st == ORBFE_OK && !path) st = ORBFE_ERR_ARG;
        if (st == ORBFE_OK) {
            DeviceGuard dg(device);
            v = new orbfe_vocabulary();
            v->device = device;
            std::vector<int> parent;
            std::vector<uint8_t> is_word, desc;
            std::vector<double> weight;
            st = vocab_parse_text(path, v->k, v->L, v->scoring, v->weighting, parent, is_word,
                                  desc, weight);
            if (st == ORBFE_OK) st = vocab_upload(v, parent, is_word, desc, weight);
            if (st == ORBFE_OK && hipStreamCreateWithFlags(&v->own, hipStreamNonBlocking) != hipSuccess)
                st = ORBFE_ERR_HIP;
            v->stream = v->own;
        }
    } catch (const std::bad_alloc&) {
        st = ORBFE_ERR_NOMEM;
    } catch (...) {
        st = ORBFE_ERR_HIP;
    }
    if (st != ORBFE_OK && v) {
        delete v;
        v = nullptr;
    }
    if (status) *status = st;
    return v;
}

orbfe_vocabulary* orbfe_vocabulary_create(int k, int L, int scoring, int weighting, int n_nodes,
                                          const int32_t* parent, const uint8_t* is_word,
                                          const uint8_t* desc, const double* weight, int device,
                                          int* status) {
    int st = check_device(device);
    orbfe_vocabulary* v = nullptr;
    try {
        if (st == ORBFE_OK && (n_nodes < 1 || !parent || !is_word || !desc || !weight || k < 0 ||
                               L < 1 || scoring < 0 || scoring > 5 || weighting < 0 || weighting > 3))
            st = ORBFE_ERR_ARG;
        if (st == ORBFE_OK) {
            DeviceGuard dg(device);
            v = new orbfe_vocabulary();
            v->device = device;
            v->k = k;
            v->L = L;
            v->scoring = scoring;
            v->weighting = weighting;
            st = vocab_upload(v, std::vector<int>(parent, parent + n_nodes),
                              std::vector<uint8_t>(is_word, is_word + n_nodes),
                              std::vector<uint8_t>(desc, desc + (size_t)n_nodes * 32),
                              std::vector<double>(weight, weight + n_nodes));
            if (st == ORBFE_OK && hipStreamCreateWithFlags(&v->own, hipStreamNonBlocking) != hipSuccess)
                st = ORBFE_ERR_HIP;
            v->stream = v->own;
        }
    } catch (const std::bad_alloc&) {
        st = ORBFE_ERR_NOMEM;
    } catch (...) {
        st = ORBFE_ERR_HIP;
    }
    if (st != ORBFE_OK && v) {
        delete v;
        v = nullptr;
    }
    if (status) *status = st;
    return v;
}

void orbfe_vocabulary_destroy(orbfe_vocabulary* v) {
    if (!v) return;
    DeviceGuard dg(v->device);
    if (v->stream) hipStreamSynchronize(v->stream);
    delete v;
}

int orbfe_vocabulary_info(const orbfe_vocabulary* v, int32_t* info) {
    if (!v || !info) return ORBFE_ERR_ARG;
    info[0] = v->k;
    info[1] = v->L;
    info[2] = v->scoring;
    info[3] = v->weighting;
    info[4] = v->nodes;
    info[5] = v->nwords;
    return ORBFE_OK;
}

int orbfe_vocabulary_set_stream(orbfe_vocabulary* v, void* hip_stream) {
    if (!v) return ORBFE_ERR_ARG;
    v->stream = hip_stream ? static_cast<hipStream_t>(hip_stream) : v->own;
    return ORBFE_OK;
}

static int bow_launch(orbfe_vocabulary* v, int nframes, int cap, const uint8_t* d_desc,
                      const int32_t* d_n, int levelsup, int32_t* d_word_ids, double* d_values,
                      int32_t* d_nw, int32_t* d_node_ids, int32_t* d_node_off, int32_t* d_feat,
                      int32_t* d_nn) {
    int st;
    const size_t tot = (size_t)nframes * cap;
    if ((st = v->s_word.ensure(std::max<size_t>(tot, 1) * sizeof(int)))) return st;
    if ((st = v->s_node.ensure(std::max<size_t>(tot, 1) * sizeof(int)))) return st;
    if ((st = v->s_w.ensure(std::max<size_t>(tot, 1) * sizeof(double)))) return st;
    BowArgs a;
    a.v = v->dev();
    a.levelsup = levelsup;
    a.cap = cap;
    a.desc = reinterpret_cast<const uint4*>(d_desc);
    a.n = d_n;
    a.f_word = v->s_word.as<int>();
    a.f_node = v->s_node.as<int>();
    a.f_w = v->s_w.as<double>();
    a.word_ids = d_word_ids;
    a.values = d_values;
    a.nw = d_nw;
    a.node_ids = d_node_ids;
    a.node_off = d_node_off;
    a.feat = d_feat;
    a.nn = d_nn;
    if (v->nwords > 0) {
        hipLaunchKernelGGL(bow_descend_kernel, dim3((cap + 255) / 256, nframes), dim3(256), 0,
                           v->stream, a);
    } else {  // empty() vocabulary: transform returns empty vectors
        ORBFE_HIP(hipMemsetAsync(v->s_w.p, 0, tot * sizeof(double), v->stream));
    }
    hipLaunchKernelGGL(bow_assemble_kernel, dim3(nframes), dim3(kBowBlock), 0, v->stream, a);
    ORBFE_HIP(hipGetLastError());
    return ORBFE_OK;
}

static int bow_search_launch(orbfe_matcher* m, const BowMatchArgs& a, int n_pairs, int gx,
                             float nnratio, int check_ori, bool init = true) {
    if (init) hipLaunchKernelGGL(bow_init_kernel, dim3(n_pairs), dim3(256), 0, m->stream, a);
    hipLaunchKernelGGL(bow_search_kernel, dim3(gx, n_pairs), dim3(kBowSearchBlock), 0, m->stream,
                       a, nnratio, check_ori);
    ORBFE_HIP(hipGetLastError());
    return ORBFE_OK;
}

// A FeatureVector as DBoW2 builds it (FeatureVector::addFeature, FeatureVector.cpp:31-45): node
// offsets ascending from 0, every feature index in [0, n) and listed under at most one node —
// the gathered path blocks a matched frame feature only within its node (the reference's
// vpMapPointMatches check, ORBmatcher.cc:212, spans nodes), so a repeated index is refused.
static bool fv_ok(int nn, const int32_t* off, const int32_t* feat, int n) {
    if (!nn) return true;
    if (off[0] != 0) return false;
    for (int i = 0; i < nn; ++i)
        if (off[i + 1] < off[i]) return false;
    if (off[nn] > n) return false;  // more entries than features: some index repeats
    std::vector<uint8_t> seen((size_t)n, 0);
    for (int i = 0; i < off[nn]; ++i) {
        if (feat[i] < 0 || feat[i] >= n || seen[feat[i]]) return false;
        seen[feat[i]] = 1;
    }
    return true;
}

// ORBFE_ZERO_COPY=0: the vocabulary's host transform copies through device buffers (DMA)
static bool zero_copy_off() {
    const char* e = std::getenv("ORBFE_ZERO_COPY");
    return e && std::strcmp(e, "0") == 0;
}

// ORBFE_BOW1=0: the host form takes the general two-launch path (bow_search_kernel) instead of
// the gathered one
static bool bow1_off() {
    const char* e = std::getenv("ORBFE_BOW1");
    return e && std::strcmp(e, "0") == 0;
}

// The host form's gathered path (bow_search1_kernel, then the orientation filter on the host;
// inputs validated by the caller).  *done = false: the pair does not fit it (more than kBow1Nodes common nodes or a
// node of more than kBowNodeMax frame features) and the caller takes the general path.
static int search_by_bow1(orbfe_matcher* m, float nnratio, int check_ori, const uint8_t* kf_desc,
                          const float* kf_angle, const uint8_t* kf_mp_ok, int kf_nn,
                          const int32_t* kf_node_ids, const int32_t* kf_node_off,
                          const int32_t* kf_feat, const uint8_t* f_desc, const float* f_angle,
                          int f_nn, const int32_t* f_node_ids, const int32_t* f_node_off,
                          const int32_t* f_feat, int32_t* matches, int32_t* nmatches, bool* done) {
    *done = false;
    Bow1Args a{};
    int2 pij[kBow1Nodes];  // (keyframe node, frame node) of each common node kept
    // the reference's walk over the two FeatureVectors (195-256)
    int ktot = 0, ftot = 0, i = 0, j = 0;
    while (i < kf_nn && j < f_nn) {
        if (kf_node_ids[i] == f_node_ids[j]) {
            int nx = 0;
            for (int e = kf_node_off[i]; e < kf_node_off[i + 1]; ++e) nx += kf_mp_ok[kf_feat[e]] != 0;
            const int ny = f_node_off[j + 1] - f_node_off[j];
            if (ny > kBowNodeMax) return ORBFE_OK;
            if (nx && ny) {
                if (a.nodes == kBow1Nodes) return ORBFE_OK;
                pij[a.nodes] = make_int2(i, j);
                a.node[a.nodes++] = make_int4(ktot, nx, ftot, ny);
                ktot += nx;
                ftot += ny;
            }
            ++i;
            ++j;
        } else if (kf_node_ids[i] < f_node_ids[j]) {
            i = (int)(std::lower_bound(kf_node_ids + i, kf_node_ids + kf_nn, f_node_ids[j]) - kf_node_ids);
        } else {
            j = (int)(std::lower_bound(f_node_ids + j, f_node_ids + f_nn, kf_node_ids[i]) - f_node_ids);
        }
    }
    if (!a.nodes) {  // no common node with candidates: no match (the caller set matches to NULL)
        *done = true;
        *nmatches = 0;
        return ORBFE_OK;
    }
    int st;
    // one staging block: kd | fd | ki | ka | fi | fa | out
    const size_t o_fd = (size_t)ktot * 32, o_ki = o_fd + (size_t)ftot * 32, o_ka = o_ki + 4 * (size_t)ktot,
                 o_fi = o_ka + 4 * (size_t)ktot, o_fa = o_fi + 4 * (size_t)ftot, o_out = o_fa + 4 * (size_t)ftot,
                 bytes = o_out + 4 * (size_t)ftot;
    uint8_t* q = m->stage(bytes);
    if (!q) return ORBFE_ERR_NOMEM;
    if (!m->pin_dev) return ORBFE_OK;  // the staging buffer is not device-mapped: general path
    *done = true;
    // each common node's features in FeatureVector order (keyframe features with a good map
    // point only), as the node loop visits them (198-245)
    int* ki = reinterpret_cast<int*>(q + o_ki);
    float* ka = reinterpret_cast<float*>(q + o_ka);
    int* fi = reinterpret_cast<int*>(q + o_fi);
    float* fa = reinterpret_cast<float*>(q + o_fa);
    for (int c = 0, kx = 0, fy = 0; c < a.nodes; ++c) {
        for (int e = kf_node_off[pij[c].x]; e < kf_node_off[pij[c].x + 1]; ++e) {
            const int k = kf_feat[e];
            if (!kf_mp_ok[k]) continue;
            std::memcpy(q + 32 * (size_t)kx, kf_desc + 32 * (size_t)k, 32);
            ki[kx] = k;
            ka[kx] = kf_angle[k];
            ++kx;
        }
        for (int e = f_node_off[pij[c].y]; e < f_node_off[pij[c].y + 1]; ++e) {
            const int k = f_feat[e];
            std::memcpy(q + o_fd + 32 * (size_t)fy, f_desc + 32 * (size_t)k, 32);
            fi[fy] = k;
            fa[fy] = f_angle[k];
            ++fy;
        }
    }
    const uint8_t* d = m->pin_dev + (q - m->pin);
    a.kd = reinterpret_cast<const uint4*>(d);
    a.fd = reinterpret_cast<const uint4*>(d + o_fd);
    a.ki = reinterpret_cast<const int*>(d + o_ki);
    a.ka = reinterpret_cast<const float*>(d + o_ka);
    a.fi = reinterpret_cast<const int*>(d + o_fi);
    a.fa = reinterpret_cast<const float*>(d + o_fa);
    a.out = reinterpret_cast<int*>(const_cast<uint8_t*>(d + o_out));
    volatile int* out = reinterpret_cast<volatile int*>(q + o_out);
    for (int s = 0; s < ftot; ++s) out[s] = kSlotPending;
    if ((st = m->flush())) return st;
    hipLaunchKernelGGL(bow_search1_kernel, dim3(a.nodes), dim3(256), 0, m->stream, a,
                       nnratio, check_ori);
    if (hipGetLastError() != hipSuccess) return ORBFE_ERR_HIP;
    if (!m->pend.empty() || !m->dnq.empty() || m->cand_check) {
        if ((st = m->sync())) return st;
    } else {
        // every slot is written once, after its node's last read of the staging buffer: the host
        // waits on the slots themselves instead of a stream synchronisation; past kSlotWaitUs it
        // synchronises the stream (which reports a failed kernel) and checks the slots again
        const auto t0 = std::chrono::steady_clock::now();
        for (int s = 0; s < ftot; ++s) {
            while (out[s] == kSlotPending) {
                if (std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(kSlotWaitUs)) {
                    ORBFE_HIP(hipStreamSynchronize(m->stream));
                    for (int u = s; u < ftot; ++u)
                        if (out[u] == kSlotPending) return ORBFE_ERR_HIP;
                    s = ftot;
                    break;
                }
                __builtin_ia32_pause();
            }
        }
    }
    // the orientation filter (259-281) on the host, as in the reference: the rotation histogram
    // of every match, ComputeThreeMaxima (1604-1645), matches outside the three bins dropped
    int hist[kHistLen] = {};
    int top[3] = {-1, -1, -1};
    if (check_ori) {
        for (int s = 0; s < ftot; ++s) {
            const int r = out[s];
            if (r >= 0) ++hist[r & 31];
        }
        three_maxima(hist, top[0], top[1], top[2]);
    }
    int kept = 0;
    for (int s = 0; s < ftot; ++s) {
        const int r = out[s];
        if (r < 0) continue;
        const int bin = r & 31;
        if (check_ori && bin != top[0] && bin != top[1] && bin != top[2]) continue;
        matches[fi[s]] = r >> 5;
        ++kept;
    }
    *nmatches = kept;
    return ORBFE_OK;
}

int orbfe_search_by_bow(orbfe_matcher* m, float nnratio, int check_ori, int n_kf,
                        const uint8_t* kf_desc, const float* kf_angle, const uint8_t* kf_mp_ok,
                        int kf_nn, const int32_t* kf_node_ids, const int32_t* kf_node_off,
                        const int32_t* kf_feat, int n_f, const uint8_t* f_desc,
                        const float* f_angle, int f_nn, const int32_t* f_node_ids,
                        const int32_t* f_node_off, const int32_t* f_feat, int32_t* matches,
                        int32_t* nmatches) {
    if (n_kf < 0 || n_f < 0 || kf_nn < 0 || f_nn < 0 || !nmatches || (n_f && !matches) ||
        (n_kf && (!kf_desc || !kf_angle || !kf_mp_ok)) || (n_f && (!f_desc || !f_angle)) ||
        (kf_nn && (!kf_node_ids || !kf_node_off || !kf_feat)) ||
        (f_nn && (!f_node_ids || !f_node_off || !f_feat)))
        return ORBFE_ERR_ARG;
    if (!fv_ok(kf_nn, kf_node_off, kf_feat, n_kf) || !fv_ok(f_nn, f_node_off, f_feat, n_f))
        return ORBFE_ERR_ARG;
    const int kf_tot = kf_nn ? kf_node_off[kf_nn] : 0, f_tot = f_nn ? f_node_off[f_nn] : 0;
    return guarded(m, [&]() {
        int st;
        for (int i = 0; i < n_f; ++i) matches[i] = -1;  // vpMapPointMatches = NULL (164)
        *nmatches = 0;
        if (!kf_nn || !f_nn || !n_f) return ORBFE_OK;
        if (!m->zero_copy_off && !bow1_off()) {
            bool done = false;
            if ((st = search_by_bow1(m, nnratio, check_ori, kf_desc, kf_angle, kf_mp_ok, kf_nn,
                                     kf_node_ids, kf_node_off, kf_feat, f_desc, f_angle, f_nn,
                                     f_node_ids, f_node_off, f_feat, matches, nmatches, &done)))
                return st;
            if (done) return ORBFE_OK;
        }
        // slot 0 of each set; the caps bound every offset and index (validated above)
        const int kf_cap = std::max({n_kf, kf_tot, kf_nn}), f_cap = std::max({n_f, f_tot, f_nn});
        const int nn[2] = {kf_nn, f_nn};
        if ((st = m->up(m->fa_d, kf_desc, (size_t)n_kf * 32))) return st;
        if ((st = m->up(m->fb_d, f_desc, (size_t)n_f * 32))) return st;
        if ((st = m->up(m->m_f0, kf_angle, (size_t)n_kf * 4))) return st;
        if ((st = m->up(m->m_f1, f_angle, (size_t)n_f * 4))) return st;
        if ((st = m->up(m->m_u0, kf_mp_ok, n_kf))) return st;
        if ((st = m->up(m->m_i0, kf_node_ids, (size_t)kf_nn * 4))) return st;
        if ((st = m->up(m->m_i1, kf_node_off, (size_t)(kf_nn + 1) * 4))) return st;
        if ((st = m->up(m->o_i, kf_feat, (size_t)kf_tot * 4))) return st;
        if ((st = m->up(m->fb_cs, f_node_ids, (size_t)f_nn * 4))) return st;
        if ((st = m->up(m->fb_ci, f_node_off, (size_t)(f_nn + 1) * 4))) return st;
        if ((st = m->up(m->fb_co, f_feat, (size_t)f_tot * 4))) return st;
        if ((st = m->up(m->nq, nn, sizeof(nn)))) return st;
        if ((st = m->s1.ensure((size_t)f_cap * 4))) return st;  // bins per frame feature
        // bow_init_kernel's work as uploads (the scatter runs anyway): every match NULL (164),
        // an empty histogram, the finished-workgroup counter, nmatches and status 0
        const bool zc = m->pin_dev != nullptr;
        if (zc) {
            m->init_neg.assign((size_t)f_cap, -1);
            const int zeros[64] = {};
            if ((st = m->up(m->fa_k, m->init_neg.data(), (size_t)f_cap * 4))) return st;
            if ((st = m->up(m->g_hist, zeros, sizeof(zeros)))) return st;
            if ((st = m->up(m->scal, zeros, 16))) return st;
        } else {
            if ((st = m->fa_k.ensure((size_t)f_cap * 4))) return st;
            if ((st = m->scal.ensure(16))) return st;
            if ((st = m->g_hist.ensure(64 * sizeof(int)))) return st;
        }
        // zero-copy results: {nmatches, status, matches[n_f]} written by the search kernel
        int* res = nullptr;
        int* res_dev = nullptr;
        if (zc) {
            uint8_t* q = m->stage((size_t)(n_f + 2) * 4);
            if (!q) return ORBFE_ERR_NOMEM;
            res = reinterpret_cast<int*>(q);
            res_dev = reinterpret_cast<int*>(m->pin_dev + (q - m->pin));
        }
        BowMatchArgs a{};
        a.kf_cap = kf_cap;
        a.f_cap = f_cap;
        a.kf_nn = m->nq.as<int>();
        a.f_nn = m->nq.as<int>() + 1;
        a.kf_node_ids = m->m_i0.as<int>();
        a.kf_node_off = m->m_i1.as<int>();
        a.kf_feat = m->o_i.as<int>();
        a.kf_ok = m->m_u0.as<uint8_t>();
        a.kf_desc = m->fa_d.as<uint4>();
        a.kf_angle = m->m_f0.as<float>();
        a.f_node_ids = m->fb_cs.as<int>();
        a.f_node_off = m->fb_ci.as<int>();
        a.f_feat = m->fb_co.as<int>();
        a.f_desc = m->fb_d.as<uint4>();
        a.f_angle = m->m_f1.as<float>();
        a.matches = m->fa_k.as<int>();
        a.bins = m->s1.as<int>();
        a.hist = m->g_hist.as<int>();
        a.nm = m->scal.as<int>();
        a.status = m->scal.as<int>() + 1;
        a.done = m->g_hist.as<int>() + 32;
        a.out_host = res_dev;
        a.out_n = n_f;
        if ((st = m->flush())) return st;
        if ((st = bow_search_launch(m, a, 1, (kf_nn + 3) / 4, nnratio, check_ori, !zc))) return st;
        int cnt[2] = {0, 0};
        if (zc) {
            if ((st = m->sync())) return st;
            std::memcpy(matches, res + 2, (size_t)n_f * 4);
            cnt[0] = res[0];
            cnt[1] = res[1];
        } else {
            if ((st = m->down(matches, m->fa_k, (size_t)n_f * 4))) return st;
            if ((st = m->down(cnt, m->scal, sizeof(cnt)))) return st;
            if ((st = m->sync())) return st;
        }
        *nmatches = cnt[0];
        return cnt[1];  // ORBFE_ERR_UNSUPPORTED: a node held more than 256 frame features
    });
}

int orbfe_search_by_bow_batch_device(orbfe_matcher* m, float nnratio, int check_ori, int n_pairs,
                                     const int32_t* d_pair_kf, const int32_t* d_pair_f,
                                     int kf_cap, const uint8_t* d_kf_desc,
                                     const float* d_kf_angle, const uint8_t* d_kf_mp_ok,
                                     const int32_t* d_kf_nn, const int32_t* d_kf_node_ids,
                                     const int32_t* d_kf_node_off, const int32_t* d_kf_feat,
                                     int f_cap, const uint8_t* d_f_desc, const float* d_f_angle,
                                     const int32_t* d_f_nn, const int32_t* d_f_node_ids,
                                     const int32_t* d_f_node_off, const int32_t* d_f_feat,
                                     int32_t* d_matches, int32_t* d_nmatches, int32_t* d_status) {
    if (n_pairs < 0 || n_pairs > 65535 || kf_cap < 1 || f_cap < 1 || !d_pair_kf || !d_pair_f ||
        !d_kf_desc || !d_kf_angle || !d_kf_mp_ok || !d_kf_nn || !d_kf_node_ids ||
        !d_kf_node_off || !d_kf_feat || !d_f_desc || !d_f_angle || !d_f_nn || !d_f_node_ids ||
        !d_f_node_off || !d_f_feat || !d_matches || !d_nmatches || !d_status)
        return ORBFE_ERR_ARG;
    return guarded(m, [&]() {
        int st;
        if (n_pairs == 0) {
            ORBFE_HIP(hipMemsetAsync(d_status, 0, sizeof(int32_t), m->stream));
            return ORBFE_OK;
        }
        if ((st = m->s1.ensure((size_t)n_pairs * f_cap * 4))) return st;
        if ((st = m->g_hist.ensure((size_t)n_pairs * 33 * sizeof(int)))) return st;
        BowMatchArgs a{};
        a.kf_cap = kf_cap;
        a.f_cap = f_cap;
        a.pair_kf = d_pair_kf;
        a.pair_f = d_pair_f;
        a.kf_nn = d_kf_nn;
        a.kf_node_ids = d_kf_node_ids;
        a.kf_node_off = d_kf_node_off;
        a.kf_feat = d_kf_feat;
        a.kf_ok = d_kf_mp_ok;
        a.kf_desc = reinterpret_cast<const uint4*>(d_kf_desc);
        a.kf_angle = d_kf_angle;
        a.f_nn = d_f_nn;
        a.f_node_ids = d_f_node_ids;
        a.f_node_off = d_f_node_off;
        a.f_feat = d_f_feat;
        a.f_desc = reinterpret_cast<const uint4*>(d_f_desc);
        a.f_angle = d_f_angle;
        a.matches = d_matches;
        a.bins = m->s1.as<int>();
        a.hist = m->g_hist.as<int>();
        a.nm = d_nmatches;
        a.done = m->g_hist.as<int>() + (size_t)n_pairs * 32;
        a.status = d_status;
        // waves stride over a keyframe's nodes (ORBvoc level 2: ~100 common nodes of ~10
        // features); enough workgroups per pair to fill the chip for a handful of candidates
        const int gx = std::max(1, std::min((kf_cap + 3) / 4, (1024 + n_pairs - 1) / n_pairs));
        return bow_search_launch(m, a, n_pairs, std::min(gx, 32), nnratio, check_ori);
    });
}

int orbfe_bow_transform(orbfe_vocabulary* v, const uint8_t* desc, int n, int levelsup,
                        int32_t* word_ids, double* values, int32_t* nw, int32_t* node_ids,
                        int32_t* node_off, int32_t* feat, int32_t* nn) {
    if (!v || n < 0 || (n && !desc) || !nw || !nn || !word_ids || !values || !node_ids ||
        !node_off || !feat)
        return ORBFE_ERR_ARG;
    if (n > kBowMaxFeatures) return ORBFE_ERR_UNSUPPORTED;
    try {
        DeviceGuard dg(v->device);
        int st;
        const int cap = std::max(n, 1);
        if ((st = v->s_desc.ensure((size_t)cap * 32))) return st;
        if ((st = v->s_n.ensure(16))) return st;
        if ((st = v->o_wid.ensure((size_t)cap * 4))) return st;
        if ((st = v->o_val.ensure((size_t)cap * 8))) return st;
        if ((st = v->o_nid.ensure((size_t)cap * 4))) return st;
        if ((st = v->o_noff.ensure((size_t)(cap + 1) * 4))) return st;
        if ((st = v->o_feat.ensure((size_t)cap * 4))) return st;
        if ((st = v->o_nw.ensure(16))) return st;
        if ((st = v->o_nn.ensure(16))) return st;
        {   // one pinned block: desc | n | word ids | values | node ids | node offsets | feat | nw | nn
            auto al = [](size_t x) { return (x + 15) & ~(size_t)15; };  // every part 16-byte aligned
            const size_t o_n = al((size_t)cap * 32), o_wid = o_n + 16, o_val = al(o_wid + (size_t)cap * 4),
                         o_nid = al(o_val + (size_t)cap * 8), o_noff = al(o_nid + (size_t)cap * 4),
                         o_feat = al(o_noff + (size_t)(cap + 1) * 4), o_nw = al(o_feat + (size_t)cap * 4),
                         o_nn = o_nw + 16, bytes = o_nn + 16;
            uint8_t* q = zero_copy_off() ? nullptr : v->stage(bytes);
            if (q) {
                const uint8_t* d = v->pin_dev;
                if (n) std::memcpy(q, desc, (size_t)n * 32);
                std::memcpy(q + o_n, &n, sizeof(int));
                if ((st = bow_launch(v, 1, cap, d, reinterpret_cast<const int32_t*>(d + o_n), levelsup,
                                     reinterpret_cast<int32_t*>(const_cast<uint8_t*>(d + o_wid)),
                                     reinterpret_cast<double*>(const_cast<uint8_t*>(d + o_val)),
                                     reinterpret_cast<int32_t*>(const_cast<uint8_t*>(d + o_nw)),
                                     reinterpret_cast<int32_t*>(const_cast<uint8_t*>(d + o_nid)),
                                     reinterpret_cast<int32_t*>(const_cast<uint8_t*>(d + o_noff)),
                                     reinterpret_cast<int32_t*>(const_cast<uint8_t*>(d + o_feat)),
                                     reinterpret_cast<int32_t*>(const_cast<uint8_t*>(d + o_nn)))))
                    return st;
                ORBFE_HIP(hipStreamSynchronize(v->stream));
                int cnt[2];
                std::memcpy(&cnt[0], q + o_nw, sizeof(int));
                std::memcpy(&cnt[1], q + o_nn, sizeof(int));
                *nw = cnt[0];
                *nn = cnt[1];
                std::memcpy(word_ids, q + o_wid, (size_t)cnt[0] * 4);
                std::memcpy(values, q + o_val, (size_t)cnt[0] * 8);
                std::memcpy(node_ids, q + o_nid, (size_t)cnt[1] * 4);
                std::memcpy(node_off, q + o_noff, (size_t)(cnt[1] + 1) * 4);
                if (!cnt[1]) node_off[0] = 0;
                const int nfeat = cnt[1] ? node_off[cnt[1]] : 0;
                std::memcpy(feat, q + o_feat, (size_t)nfeat * 4);
                return ORBFE_OK;
            }
        }
        if (n) ORBFE_HIP(hipMemcpyAsync(v->s_desc.p, desc, (size_t)n * 32, hipMemcpyHostToDevice, v->stream));
        ORBFE_HIP(hipMemcpyAsync(v->s_n.p, &n, sizeof(int), hipMemcpyHostToDevice, v->stream));
        if ((st = bow_launch(v, 1, cap, v->s_desc.as<uint8_t>(), v->s_n.as<int32_t>(), levelsup,
                             v->o_wid.as<int32_t>(), v->o_val.as<double>(), v->o_nw.as<int32_t>(),
                             v->o_nid.as<int32_t>(), v->o_noff.as<int32_t>(),
                             v->o_feat.as<int32_t>(), v->o_nn.as<int32_t>())))
            return st;
        int cnt[2] = {0, 0};
        ORBFE_HIP(hipMemcpyAsync(&cnt[0], v->o_nw.p, sizeof(int), hipMemcpyDeviceToHost, v->stream));
        ORBFE_HIP(hipMemcpyAsync(&cnt[1], v->o_nn.p, sizeof(int), hipMemcpyDeviceToHost, v->stream));
        ORBFE_HIP(hipStreamSynchronize(v->stream));
        *nw = cnt[0];
        *nn = cnt[1];
        int nfeat = 0;
        ORBFE_HIP(hipMemcpy(word_ids, v->o_wid.p, (size_t)cnt[0] * 4, hipMemcpyDeviceToHost));
        ORBFE_HIP(hipMemcpy(values, v->o_val.p, (size_t)cnt[0] * 8, hipMemcpyDeviceToHost));
        ORBFE_HIP(hipMemcpy(node_ids, v->o_nid.p, (size_t)cnt[1] * 4, hipMemcpyDeviceToHost));
        ORBFE_HIP(hipMemcpy(node_off, v->o_noff.p, (size_t)(cnt[1] + 1) * 4, hipMemcpyDeviceToHost));
        nfeat = cnt[1] ? node_off[cnt[1]] : 0;
        if (!cnt[1]) node_off[0] = 0;
        ORBFE_HIP(hipMemcpy(feat, v->o_feat.p, (size_t)nfeat * 4, hipMemcpyDeviceToHost));
        return ORBFE_OK;
    } catch (const std::bad_alloc&) {
        return ORBFE_ERR_NOMEM;
    } catch (...) {
        return ORBFE_ERR_HIP;
    }
}

int orbfe_bow_transform_batch_device(orbfe_vocabulary* v, int nframes, const uint8_t* d_desc,
                                     const int32_t* d_n, int cap, int levelsup,
                                     int32_t* d_word_ids, double* d_values, int32_t* d_nw,
                                     int32_t* d_node_ids, int32_t* d_node_off, int32_t* d_feat,
                                     int32_t* d_nn) {
    if (!v || nframes < 0 || cap < 1 || !d_desc || !d_n || !d_word_ids || !d_values || !d_nw ||
        !d_node_ids || !d_node_off || !d_feat || !d_nn)
        return ORBFE_ERR_ARG;
    if (cap > kBowMaxFeatures) return ORBFE_ERR_UNSUPPORTED;
    if (nframes == 0) return ORBFE_OK;
    try {
        DeviceGuard dg(v->device);
        return bow_launch(v, nframes, cap, d_desc, d_n, levelsup, d_word_ids, d_values, d_nw,
                          d_node_ids, d_node_off, d_feat, d_nn);
    } catch (...) {
        return ORBFE_ERR_HIP;
    }
}

}  // extern "C"
