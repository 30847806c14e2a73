// orbfe_match_api.hip — host orchestration and C ABI of the matchers (include/orbfe.h).
// Every call uploads the flat SoA views, runs the kernels of orbfe_match.hip on the matcher's
// stream and downloads the results (synchronous, like the reference's member functions).
#include <hip/hip_runtime.h>
#include <map>

#include <algorithm>
#include <chrono>
#include <climits>
#include <functional>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/orbfe.h"

namespace orbfe {
// Uploads of one host call: a single H2D copy of the pinned staging range into a device
// staging buffer, then this kernel scatters the segments to their buffers (one launch instead
// of one blit per array).  Segments are 256-byte aligned on both sides.
constexpr int kMaxUpSeg = 24;
struct UpScatter {
    int n;
    uint8_t* dst[kMaxUpSeg];
    const uint8_t* src[kMaxUpSeg];
    uint32_t bytes[kMaxUpSeg];
};
// Results of a host-form call go the other way in one launch: each segment copies device
// bytes into the (device-mapped) pinned staging buffer, so a call ends with this kernel instead
// of a DMA per output array.  With a done word (flag, device-mapped pinned memory) the last
// workgroup to finish writes seq to it after every workgroup's copies are released to system
// scope: the host waits on that word instead of synchronising the stream.
struct DnDone {
    int* ctr;   // device counter of finished workgroups (zero between launches)
    int* flag;  // null: no done word
    int seq, blocks;
};
__global__ __launch_bounds__(256) void download_gather_kernel(UpScatter a, DnDone dd) {
    const int s = blockIdx.y;
    if (s < a.n) {
        const uint32_t nb = a.bytes[s];
        const uint8_t* src = a.src[s];
        uint8_t* dst = a.dst[s];
        // dword copies when both ends are 4-byte aligned (device buffers and 256-B staging slots)
        if (((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) & 3) == 0) {
            const uint32_t n4 = nb >> 2;
            const uint32_t* s4 = reinterpret_cast<const uint32_t*>(src);
            uint32_t* d4 = reinterpret_cast<uint32_t*>(dst);
            for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n4; i += gridDim.x * 256) d4[i] = s4[i];
            if (blockIdx.x == 0 && threadIdx.x < (nb & 3)) dst[4 * n4 + threadIdx.x] = src[4 * n4 + threadIdx.x];
        } else {
            for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < nb; i += gridDim.x * 256) dst[i] = src[i];
        }
    }
    if (!dd.flag) return;
    __threadfence_system();  // this thread's copies, to system scope
    __syncthreads();
    if (threadIdx.x == 0 &&
        __hip_atomic_fetch_add(dd.ctr, 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == dd.blocks - 1) {
        __hip_atomic_store(dd.ctr, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(dd.flag, dd.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}
__global__ __launch_bounds__(256) void upload_scatter_kernel(UpScatter a) {
    const int s = blockIdx.y;
    if (s >= a.n) return;
    const uint32_t nb = a.bytes[s], n16 = nb >> 4;
    const uint4* src = reinterpret_cast<const uint4*>(a.src[s]);
    uint4* dst = reinterpret_cast<uint4*>(a.dst[s]);
    for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n16; i += gridDim.x * 256) dst[i] = src[i];
    if (blockIdx.x == 0 && threadIdx.x < (nb & 15)) a.dst[s][16 * n16 + threadIdx.x] = a.src[s][16 * n16 + threadIdx.x];
}
}  // namespace orbfe

using namespace orbfe;

struct orbfe_matcher {
    int device = 0;
    hipStream_t own = nullptr, stream = nullptr;
    DevBuf fa_k, fa_d, fa_ur, fa_cs, fa_ci, fa_co;  // frame A (+ grid)
    DevBuf fb_k, fb_d, fb_ur, fb_cs, fb_ci, fb_co;  // frame B (+ grid)
    DevBuf q, r, nq, nr, out;                       // brute force / hamming
    DevBuf cnt, off, cand;                          // candidate CSR
    DevBuf s1, s2, s3, s4, s5;                      // resolve scratch / outputs
    DevBuf m_f0, m_f1, m_f2, m_f3, m_f4, m_u0, m_u1, m_i0, m_i1, m_d;  // per-map-point inputs
    DevBuf o_u, o_f0, o_f1, o_f2, o_f3, o_i;        // frustum outputs
    DevBuf scal, done_ctr;
    DevBuf g_t0, g_t1, g_t2, g_dec, g_chg, g_last, g_bins, g_hist;  // greedy resolver
    Profiler prof;
    int last_rounds = 0;  // rounds the most recent greedy resolution took (diagnostics)
    int capacity_retries = 0;  // calls rerun because the candidates outgrew the buffer
    bool rounds_on_device = false;  // single-workgroup form: the count sits in g_chg[0]
    // ORBFE_ZERO_COPY=0: uploads and downloads as DMA copies (the staging buffer unmapped)
    bool zero_copy_off = std::getenv("ORBFE_ZERO_COPY") && std::strcmp(std::getenv("ORBFE_ZERO_COPY"), "0") == 0;
    BfKernel bf_kernel = bf_match_fp4_kernel;  // ORBFE_BF_I8=1 at creation: bf_match_kernel
    // a reference set shared by the whole batch is expanded to FP4 fragments once per call
    // (bf_expand_kernel) instead of by every workgroup: c3 bf_match 0.159 -> 0.148 ms per 512
    // frames (profiles/r04/experiments/bf_pre/); ORBFE_BF_PRE=0: every workgroup expands it
    bool bf_pre = !(std::getenv("ORBFE_BF_PRE") && std::strcmp(std::getenv("ORBFE_BF_PRE"), "0") == 0);
    // the shared reference set as FP4 fragments (bf_expand_kernel), one buffer per stream the
    // batch form was called on (calls on different streams may overlap), at most kBfStreams of
    // them.  Each buffer carries an event recorded behind the last launch that reads it; a call
    // on another stream takes the least recently used buffer once that event has completed — a
    // wait on that one buffer's readers, not on the device (a caller creating a stream per call,
    // or a destroyed stream whose handle is reused, cannot grow the set or find a buffer another
    // stream still reads; the event stays valid after its stream is destroyed).
    static constexpr int kBfStreams = 4;
    struct BfSlot {
        DevBuf buf;
        hipEvent_t done = nullptr;  // recorded after the last launch reading buf
        unsigned long long used = 0;
    };
    std::map<hipStream_t, BfSlot> bf_e;
    unsigned long long bf_e_clock = 0;
    BfSlot* bf_buffer(hipStream_t s, int* st) {
        *st = ORBFE_OK;
        auto it = bf_e.find(s);
        if (it == bf_e.end() && (int)bf_e.size() >= kBfStreams) {
            auto lru = bf_e.begin();
            for (auto i = bf_e.begin(); i != bf_e.end(); ++i)
                if (i->second.used < lru->second.used) lru = i;
            if (lru->second.done && hipEventSynchronize(lru->second.done) != hipSuccess) {
                *st = ORBFE_ERR_HIP;
                return nullptr;
            }
            BfSlot moved = lru->second;  // reuse the allocation and the event for the new stream
            bf_e.erase(lru);
            it = bf_e.emplace(s, moved).first;
        }
        BfSlot& e = bf_e[s];
        e.used = ++bf_e_clock;
        if (!e.done && hipEventCreateWithFlags(&e.done, hipEventDisableTiming) != hipSuccess) {
            e.done = nullptr;
            *st = ORBFE_ERR_HIP;
            return nullptr;
        }
        if ((*st = e.buf.ensure((size_t)kBfMaxTiles * 8 * kBfRefs * sizeof(i32x4)))) return nullptr;
        return &e;
    }

    ~orbfe_matcher() {
        for (DevBuf* b : {&fa_k, &fa_d, &fa_ur, &fa_cs, &fa_ci, &fa_co, &fb_k, &fb_d, &fb_ur,
                          &fb_cs, &fb_ci, &fb_co, &q, &r, &nq, &nr, &out, &cnt, &off, &cand, &s1,
                          &s2, &s3, &s4, &s5, &m_f0, &m_f1, &m_f2, &m_f3, &m_f4, &m_u0, &m_u1,
                          &m_i0, &m_i1, &m_d, &o_u, &o_f0, &o_f1, &o_f2, &o_f3, &o_i, &scal,
                          &g_t0, &g_t1, &g_t2, &g_dec, &g_chg, &g_last, &g_bins, &g_hist, &done_ctr})
            b->release();
        for (auto& kv : bf_e) {
            kv.second.buf.release();
            if (kv.second.done) hipEventDestroy(kv.second.done);
        }
        prof.release();
        if (own) hipStreamDestroy(own);
        if (stat_host) hipHostFree(stat_host);
        if (dn_flag_host) hipHostFree(dn_flag_host);
        dn_ctr.release();
    }

    // Host transfers go through a pinned staging buffer: the copy into it is a CPU memcpy and
    // the DMA is asynchronous (pageable hipMemcpyAsync stages and blocks per call).  Every
    // host-form entry point starts with begin() and ends with sync(), which completes the
    // deferred downloads; the staging memory is reused from call to call.
    // SearchLocalPoints' fast-path tallies: 6 ints of device-mapped pinned memory written by the
    // accept kernel's last workgroup (null: read back by a D2H copy)
    int* stat_host = nullptr;
    int* stat_dev = nullptr;
    uint8_t* pin = nullptr;
    uint8_t* pin_dev = nullptr;  // the staging buffer's device-mapped address (null: DMA path)
    size_t pin_cap = 0, pin_used = 0;
    struct DnSeg { const uint8_t* src; uint8_t* dst; size_t bytes; };
    std::vector<DnSeg> dnq;  // downloads not yet gathered (zero-copy path)
    std::vector<int32_t> init_neg;  // host-side -1 fill staged as an upload (SearchByBoW)
    std::vector<uint8_t*> pin_retired;  // outgrown buffers, freed once the stream is idle
    struct Pending { void* dst; const uint8_t* src; size_t bytes; };
    std::vector<Pending> pend;

    struct UpSeg { uint8_t* dst; size_t off; size_t bytes; };
    std::vector<UpSeg> upq;  // staged uploads not yet copied
    DevBuf d_stage;

    void begin() {
        for (uint8_t* q : pin_retired) hipHostFree(q);
        pin_retired.clear();
        pin_used = 0;
        pend.clear();
        upq.clear();
        dnq.clear();
        cand_check = false;
    }
    // Copies the staged uploads to their device buffers (call before any kernel reads them).
    // With a device-mapped staging buffer the scatter kernel reads the pinned bytes itself
    // (zero-copy: no DMA in front of it); otherwise one H2D copy into d_stage first.
    int flush() {
        if (upq.empty()) return ORBFE_OK;
        size_t lo = upq[0].off, hi = 0;
        for (const UpSeg& u : upq) { lo = std::min(lo, u.off); hi = std::max(hi, u.off + u.bytes); }
        int st;
        const uint8_t* sbase = pin_dev;
        if (!sbase) {
            if ((st = d_stage.ensure(pin_cap))) return st;
            ORBFE_HIP(hipMemcpyAsync(d_stage.as<uint8_t>() + lo, pin + lo, hi - lo, hipMemcpyHostToDevice, stream));
            sbase = d_stage.as<uint8_t>();
        }
        for (size_t b = 0; b < upq.size(); b += kMaxUpSeg) {
            UpScatter a;
            a.n = (int)std::min<size_t>(kMaxUpSeg, upq.size() - b);
            size_t mx = 0;
            for (int i = 0; i < a.n; ++i) {
                const UpSeg& u = upq[b + i];
                a.dst[i] = u.dst;
                a.src[i] = sbase + u.off;
                a.bytes[i] = (uint32_t)u.bytes;
                mx = std::max(mx, u.bytes);
            }
            const int gx = (int)std::min<size_t>(64, std::max<size_t>(1, (mx / 16 + 255) / 256));
            hipLaunchKernelGGL(upload_scatter_kernel, dim3(gx, a.n), dim3(256), 0, stream, a);
        }
        upq.clear();
        ORBFE_HIP(hipGetLastError());
        return ORBFE_OK;
    }
    uint8_t* stage(size_t bytes) {
        const size_t off = (pin_used + 255) & ~(size_t)255;
        if (off + bytes > pin_cap) {
            const size_t cap = std::max<size_t>((off + bytes) * 2, (size_t)1 << 20);
            void* q = nullptr;
            if (hipHostMalloc(&q, cap, hipHostMallocDefault) != hipSuccess) return nullptr;
            if (flush() != ORBFE_OK) return nullptr;  // staged uploads reference the old buffer
            if (pin) pin_retired.push_back(pin);  // in-flight copies may still read it
            pin = static_cast<uint8_t*>(q);
            pin_cap = cap;
            void* dq = nullptr;
            pin_dev = (!zero_copy_off && hipHostGetDevicePointer(&dq, q, 0) == hipSuccess) ? static_cast<uint8_t*>(dq) : nullptr;
            pin_used = 0;
            return stage(bytes);
        }
        pin_used = off + bytes;
        return pin + off;
    }
    int up(DevBuf& b, const void* src, size_t bytes) {
        int st = b.ensure(std::max<size_t>(bytes, 16));
        if (st) return st;
        if (!bytes) return ORBFE_OK;
        uint8_t* q = stage(bytes);
        if (!q) return ORBFE_ERR_NOMEM;
        std::memcpy(q, src, bytes);
        upq.push_back(UpSeg{b.as<uint8_t>(), (size_t)(q - pin), bytes});
        return ORBFE_OK;
    }
    int down(void* dst, const DevBuf& b, size_t bytes) { return down_ptr(dst, b.p, bytes); }
    int down_ptr(void* dst, const void* src, size_t bytes) {
        if (!bytes) return ORBFE_OK;
        uint8_t* q = stage(bytes);
        if (!q) return ORBFE_ERR_NOMEM;
        if (pin_dev) {  // gathered at sync() by one kernel
            dnq.push_back(DnSeg{static_cast<const uint8_t*>(src), pin_dev + (q - pin), bytes});
        } else {
            ORBFE_HIP(hipMemcpyAsync(q, src, bytes, hipMemcpyDeviceToHost, stream));
        }
        pend.push_back(Pending{dst, q, bytes});
        return ORBFE_OK;
    }
    // The done word of the download gather (device-mapped pinned memory) and its counter.
    int* dn_flag_host = nullptr;
    int* dn_flag_dev = nullptr;
    int dn_seq = 0;
    DevBuf dn_ctr;
    // *waited = true: the last launch carries the done word and the host waited on it
    int gather(bool* waited = nullptr) {
        if (waited) *waited = false;
        if (waited && !dnq.empty() && !prof.on && !dn_flag_host) {
            void* q = nullptr;
            void* dq = nullptr;
            if (dn_ctr.ensure(64) == ORBFE_OK && hipMemsetAsync(dn_ctr.p, 0, 64, stream) == hipSuccess &&
                hipHostMalloc(&q, 64, hipHostMallocDefault) == hipSuccess) {
                if (hipHostGetDevicePointer(&dq, q, 0) == hipSuccess) {
                    dn_flag_host = static_cast<int*>(q);
                    dn_flag_dev = static_cast<int*>(dq);
                    *dn_flag_host = dn_seq;
                } else {
                    hipHostFree(q);
                }
            }
        }
        const bool flagged = waited && !dnq.empty() && !prof.on && dn_flag_host;
        for (size_t b = 0; b < dnq.size(); b += kMaxUpSeg) {
            UpScatter a;
            a.n = (int)std::min<size_t>(kMaxUpSeg, dnq.size() - b);
            size_t mx = 0;
            for (int i = 0; i < a.n; ++i) {
                a.src[i] = dnq[b + i].src;
                a.dst[i] = dnq[b + i].dst;
                a.bytes[i] = (uint32_t)dnq[b + i].bytes;
                mx = std::max(mx, dnq[b + i].bytes);
            }
            const int gx = (int)std::min<size_t>(64, std::max<size_t>(1, (mx / 4 + 255) / 256));
            DnDone dd{nullptr, nullptr, 0, 0};
            if (flagged && b + kMaxUpSeg >= dnq.size()) dd = DnDone{dn_ctr.as<int>(), dn_flag_dev, ++dn_seq, gx * a.n};
            hipLaunchKernelGGL(download_gather_kernel, dim3(gx, a.n), dim3(256), 0, stream, a, dd);
        }
        dnq.clear();
        ORBFE_HIP(hipGetLastError());
        if (flagged) {
            // the stream's earlier kernels finished before the gather ran; bounded wait, then the
            // stream synchronisation (which also reports a failed kernel)
            const volatile int* fl = dn_flag_host;
            const auto t0 = std::chrono::steady_clock::now();
            while (*fl != dn_seq) {
                if (std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(2000)) {
                    ORBFE_HIP(hipStreamSynchronize(stream));
                    if (*fl != dn_seq) return ORBFE_ERR_HIP;
                    break;
                }
                __builtin_ia32_pause();
            }
            *waited = true;
        }
        return ORBFE_OK;
    }
    int sync() {
        int st;
        if ((st = flush())) return st;
        bool waited = false;
        if ((st = gather(&waited))) return st;
        if (!waited) ORBFE_HIP(hipStreamSynchronize(stream));
        if (cand_check) {  // csr_async: the candidates must have fit before results count
            int total = 0;
            for (const Pending& d : pend)
                if (d.dst == &cand_total) std::memcpy(&total, d.src, sizeof(int));
            cand_check = false;
            if ((size_t)total > cand_cap_used) {
                pend.clear();
                cand_need = (size_t)total;
                return ORBFE_ERR_CAPACITY;
            }
        }
        for (const Pending& d : pend) std::memcpy(d.dst, d.src, d.bytes);
        pend.clear();
        return ORBFE_OK;
    }

    // Frame::AssignFeaturesToGrid: the LDS form up to kGridLdsMax keypoints.
    void launch_grid(const orbfe_keypoint* k, int n, const orbfe_frame_view* v, int* cellof,
                     int* cstart, int* citems) {
        if (n <= kGridLdsMax)
            hipLaunchKernelGGL(grid_lds_kernel, dim3(1), dim3(kGridBlock), 0, stream, k, n,
                               v->min_x, v->min_y, v->grid_w_inv, v->grid_h_inv, cstart, citems);
        else
            hipLaunchKernelGGL(grid_kernel, dim3(1), dim3(kGridBlock), 0, stream, k, n, v->min_x,
                               v->min_y, v->grid_w_inv, v->grid_h_inv, cellof, cstart, citems);
    }

    // Uploads a frame view and builds its 64 x 48 grid (Frame::AssignFeaturesToGrid).
    int frame(const orbfe_frame_view* v, bool second, DevFrame& F) {
        DevBuf& k = second ? fb_k : fa_k;
        DevBuf& d = second ? fb_d : fa_d;
        DevBuf& u = second ? fb_ur : fa_ur;
        DevBuf& cs = second ? fb_cs : fa_cs;
        DevBuf& ci = second ? fb_ci : fa_ci;
        DevBuf& co = second ? fb_co : fa_co;
        const int n = v->n;
        int st;
        if ((st = up(k, v->keys_un, (size_t)n * sizeof(orbfe_keypoint)))) return st;
        if ((st = up(d, v->desc, (size_t)n * 32))) return st;
        if (v->u_right && (st = up(u, v->u_right, (size_t)n * sizeof(float)))) return st;
        if ((st = cs.ensure((kGridCells + 1) * sizeof(int)))) return st;
        if ((st = ci.ensure(std::max(n, 1) * sizeof(int)))) return st;
        if ((st = co.ensure(std::max(n, 1) * sizeof(int)))) return st;
        if ((st = flush())) return st;
        launch_grid(k.as<orbfe_keypoint>(), n, v, co.as<int>(), cs.as<int>(), ci.as<int>());
        F.k = k.as<orbfe_keypoint>();
        F.desc = d.as<uint4>();
        F.ur = v->u_right ? u.as<float>() : nullptr;
        F.n = n;
        F.minx = v->min_x;
        F.maxx = v->max_x;
        F.miny = v->min_y;
        F.maxy = v->max_y;
        F.gwi = v->grid_w_inv;
        F.ghi = v->grid_h_inv;
        F.cstart = cs.as<int>();
        F.citems = ci.as<int>();
        return ORBFE_OK;
    }

    // Device-resident frame view (keys_un / desc / u_right are device pointers): builds the grid.
    // grid = false: F's grid arrays are not built (a kernel that builds the grid itself)
    int frame_device(const orbfe_frame_view* v, DevFrame& F, bool grid = true) {
        const int n = v->n;
        int st;
        if ((st = fa_cs.ensure((kGridCells + 1) * sizeof(int)))) return st;
        if ((st = fa_ci.ensure(std::max(n, 1) * sizeof(int)))) return st;
        if ((st = fa_co.ensure(std::max(n, 1) * sizeof(int)))) return st;
        if (grid) launch_grid(v->keys_un, n, v, fa_co.as<int>(), fa_cs.as<int>(), fa_ci.as<int>());
        F.k = v->keys_un;
        F.desc = reinterpret_cast<const uint4*>(v->desc);
        F.ur = v->u_right;
        F.n = n;
        F.minx = v->min_x;
        F.maxx = v->max_x;
        F.miny = v->min_y;
        F.maxy = v->max_y;
        F.gwi = v->grid_w_inv;
        F.ghi = v->grid_h_inv;
        F.cstart = fa_cs.as<int>();
        F.citems = fa_ci.as<int>();
        return ORBFE_OK;
    }

    // count -> scan -> fill for a candidate kernel family; returns the candidate total.
    // per_block: queries per 256-thread block (256: thread per query, 4: wave per query).
    // Without a host round trip: the fill is bounded by a grow-only capacity and the true total
    // is checked by sync() (ORBFE_ERR_CAPACITY: the caller grows to cand_need and runs again).
    int cand_total = 0;          // written by the deferred download of off[nq]
    size_t cand_cap_used = 0;
    bool cand_check = false;
    size_t cand_need = 0;
    template <class Args, class CountK, class FillK>
    int csr_async(Args& a, int nq, CountK ck, FillK fk, int per_block) {
        int st;
        if ((st = cnt.ensure(std::max(nq, 1) * sizeof(int)))) return st;
        if ((st = off.ensure((nq + 1) * sizeof(int)))) return st;
        const size_t cap = std::max(std::max(cand.bytes / sizeof(int2), (size_t)nq * 64), cand_need);
        if ((st = cand.ensure(std::max<size_t>(cap, 1) * sizeof(int2)))) return st;
        a.cnt = cnt.as<int>();
        a.off = off.as<int>();
        a.cand = cand.as<int2>();
        a.cand_cap = (long long)cap;
        if ((st = flush())) return st;
        const int blocks = std::max(1, (nq + per_block - 1) / per_block);
        hipLaunchKernelGGL(ck, dim3(blocks), dim3(256), 0, stream, a);
        hipLaunchKernelGGL(scan_kernel, dim3(1), dim3(1024), 0, stream, cnt.as<int>(), nq, off.as<int>());
        hipLaunchKernelGGL(fk, dim3(blocks), dim3(256), 0, stream, a);
        ORBFE_HIP(hipGetLastError());
        if ((st = down_ptr(&cand_total, off.as<int>() + nq, sizeof(int)))) return st;
        cand_cap_used = cap;
        cand_check = true;
        return ORBFE_OK;
    }

    template <class Args, class CountK, class FillK>
    int csr(Args& a, int nq, CountK ck, FillK fk, int& total, int per_block = 256) {
        int st;
        if ((st = cnt.ensure(std::max(nq, 1) * sizeof(int)))) return st;
        if ((st = off.ensure((nq + 1) * sizeof(int)))) return st;
        a.cnt = cnt.as<int>();
        a.off = off.as<int>();
        if ((st = flush())) return st;
        const int blocks = std::max(1, (nq + per_block - 1) / per_block);
        hipLaunchKernelGGL(ck, dim3(blocks), dim3(256), 0, stream, a);
        hipLaunchKernelGGL(scan_kernel, dim3(1), dim3(1024), 0, stream, cnt.as<int>(), nq, off.as<int>());
        ORBFE_HIP(hipMemcpyAsync(&total, off.as<int>() + nq, sizeof(int), hipMemcpyDeviceToHost, stream));
        ORBFE_HIP(hipStreamSynchronize(stream));
        if ((st = cand.ensure(std::max(total, 1) * sizeof(int2)))) return st;
        a.cand = cand.as<int2>();
        hipLaunchKernelGGL(fk, dim3(blocks), dim3(256), 0, stream, a);
        ORBFE_HIP(hipGetLastError());
        return ORBFE_OK;
    }

    // Exact parallel resolution of the greedy assignment (orbfe_greedy.hip).  `g` carries the
    // problem (m points, nkp slots, CSR candidates, decision mode, slot arrays fmp/fobs that
    // hold the state before the call and receive the result); the scratch is owned here.
    // `total` / `cap` (optional): a candidate total that is only known on the device; it is
    // checked at the first synchronization, before any slot is written (ORBFE_ERR_CAPACITY).
    int greedy(GreedyArgs& g, int first_batch = 8, const int* total = nullptr, size_t cap = 0) {
        int st;
        const int M = g.m, N = g.nkp;
        if ((st = g_t0.ensure(std::max(N, 1) * sizeof(int)))) return st;
        if ((st = g_t1.ensure(std::max(N, 1) * sizeof(int)))) return st;
        if ((st = g_t2.ensure(std::max(N, 1) * sizeof(int)))) return st;
        if ((st = g_last.ensure(std::max(N, 1) * sizeof(int)))) return st;
        if ((st = g_dec.ensure(std::max(M, 1) * sizeof(int)))) return st;
        if ((st = g_bins.ensure(std::max(M, 1) * sizeof(int)))) return st;
        if ((st = g_chg.ensure((size_t)(M + 2) * sizeof(int)))) return st;
        if ((st = g_hist.ensure(32 * sizeof(int)))) return st;
        if ((st = scal.ensure(16))) return st;
        if ((st = flush())) return st;
        g.T[0] = g_t0.as<int>();
        g.T[1] = g_t1.as<int>();
        g.T[2] = g_t2.as<int>();
        g.dec = g_dec.as<int>();
        g.chg = g_chg.as<int>();
        g.last = g_last.as<int>();
        g.bins = g_bins.as<int>();
        g.hist = g_hist.as<int>();
        g.nm = scal.as<int>();
        // the fill's capacity: csr() sized it to the exact total; csr_async() and a device
        // total (`total`) bound it, and lists past it were not filled
        g.cand_cap = total ? (long long)cap : cand_check ? (long long)cand_cap_used : LLONG_MAX;
        if (M <= kGreedySmallMax && N <= kGreedySmallSlots && !total) {  // one workgroup
            hipLaunchKernelGGL(greedy_small_kernel, dim3(1), dim3(kGreedySmallBlock),
                               (size_t)4 * std::max(N, 1) * sizeof(int), stream, g);
            ORBFE_HIP(hipGetLastError());
            rounds_on_device = true;
            return ORBFE_OK;
        }
        rounds_on_device = false;
        const int blocks = std::max(1, (std::max(std::max(M + 2, N), 32) + kGreedyBlock - 1) / kGreedyBlock);
        const int mblocks = std::max(1, (M + kGreedyBlock - 1) / kGreedyBlock);
        const int nblocks = std::max(1, (N + kGreedyBlock - 1) / kGreedyBlock);
        // (greedy_init_kernel also clears the change flags: blocks cover max(M, N, 32) >= M + 2)
        hipLaunchKernelGGL(greedy_init_kernel, dim3(blocks), dim3(kGreedyBlock), 0, stream, g);
        // rounds in batches; a round after a change-free round exits at once
        int r = 0, batch = first_batch;
        std::vector<int> chg_h;
        while (true) {
            const int r0 = r;
            for (int b = 0; b < batch && r <= M; ++b, ++r)
                hipLaunchKernelGGL(greedy_round_kernel<false>, dim3(blocks), dim3(kGreedyBlock), 0, stream, g, r);
            // the batch's change flags through the staging gather and its done word (sync()
            // also checks an asynchronous candidate fill's capacity first)
            chg_h.assign(r - r0, 0);
            if ((st = down_ptr(chg_h.data(), g.chg + r0, (size_t)(r - r0) * sizeof(int)))) return st;
            if ((st = sync())) return st;
            if (total && (size_t)*total > cap) return ORBFE_ERR_CAPACITY;
            const auto z = std::find(chg_h.begin(), chg_h.end(), 0);
            if (z != chg_h.end()) {
                last_rounds = r0 + (int)(z - chg_h.begin()) + 1;  // the change-free round included
                break;
            }
            if (r > M) return ORBFE_ERR_HIP;  // cannot happen: the correct prefix grows every round
            batch = std::min(batch * 2, 64);
        }
        hipLaunchKernelGGL(greedy_accept_kernel<false>, dim3(mblocks), dim3(kGreedyBlock), 0, stream, g, 0);
        hipLaunchKernelGGL(greedy_slots_kernel, dim3(nblocks), dim3(kGreedyBlock), 0, stream, g);
        if (g.check_ori)
            hipLaunchKernelGGL(greedy_ori_kernel, dim3(mblocks), dim3(kGreedyBlock), 0, stream, g);
        ORBFE_HIP(hipGetLastError());
        return ORBFE_OK;
    }
};

namespace {
int frame_ok(const orbfe_frame_view* f) {
    if (!f || f->n < 0 || (f->n && (!f->keys_un || !f->desc)) || !f->scale_factors ||
        f->nlevels < 1)
        return 0;
    return 1;
}
// 3x4 [R|t]: camera centre -R^T t, accumulated in double like cv::gemm's GEMM_1_T path.
void camera_center(const float* T, float* c) {
    for (int i = 0; i < 3; ++i)
        c[i] = (float)-((double)T[i] * T[3] + (double)T[4 + i] * T[7] + (double)T[8 + i] * T[11]);
}
void rigid(const float* T, const float* p, float* out) {
    for (int r = 0; r < 3; ++r)
        out[r] = ((T[4 * r] * p[0] + T[4 * r + 1] * p[1]) + T[4 * r + 2] * p[2]) + T[4 * r + 3];
}
template <class F>
int guarded(orbfe_matcher* m, F&& f) {
    if (!m) return ORBFE_ERR_ARG;
    try {
        DeviceGuard dg(m->device);
        m->begin();
        const size_t need0 = m->cand_need;
        int st = f();
        if (st == ORBFE_ERR_CAPACITY && m->cand_need > need0) {  // candidates outgrew the bound
            ++m->capacity_retries;
            m->begin();
            st = f();
        }
        return st;
    } catch (const std::bad_alloc&) {
        return ORBFE_ERR_NOMEM;
    } catch (...) {
        return ORBFE_ERR_HIP;
    }
}
// SearchLocalPoints' fast path (frames of <= kSbpFixKp keypoints): the grid, ONE kernel for
// isInFrustum (kPre: its outputs already resident) + candidates (fixed per-point slots) + the
// greedy initialisation, kBlindRounds rounds launched without looking (a round after a change-free
// one is a no-op), the acceptances whose last workgroup writes the slots and the tallies, and ONE
// synchronisation reading host[0..5] = {nmatches, nToMatch, status, overflow, last round's
// changes, rounds}.  A point with more than kSbpFix candidates or a map that needs more rounds
// (rare: host[3] or host[4] set) has the slots saved by the fused kernel restored, and the caller
// reruns the call through the CSR path.
template <bool kPre>
int sbp_local_fast(orbfe_matcher* m, const orbfe_frame_view* frame, const FrustumArgs& fr,
                   const SbpMps& mp, float nnratio, float th, const int32_t* d_nobs,
                   const int32_t* d_mp_ids, int32_t* d_frame_mp, int32_t* d_frame_mp_obs,
                   int host[6]) {
    int st;
    const int M = mp.m, N = frame->n;
    constexpr int kBlindRounds = 6;
    const int fblocks = (std::max(std::max(M, N), kBlindRounds + 1) + kSbpPts - 1) / kSbpPts;
    if ((st = m->cand.ensure((size_t)M * kSbpFix * sizeof(int2)))) return st;
    if ((st = m->cnt.ensure((size_t)M * sizeof(int)))) return st;
    if ((st = m->s1.ensure(std::max(N, 1) * sizeof(int)))) return st;
    if ((st = m->s2.ensure(std::max(N, 1) * sizeof(int)))) return st;
    if ((st = m->s3.ensure((size_t)3 * fblocks * sizeof(int)))) return st;
    if ((st = m->g_t0.ensure(std::max(N, 1) * sizeof(int)))) return st;
    if ((st = m->g_t1.ensure(std::max(N, 1) * sizeof(int)))) return st;
    if ((st = m->g_t2.ensure(std::max(N, 1) * sizeof(int)))) return st;
    if ((st = m->g_last.ensure(std::max(N, 1) * sizeof(int)))) return st;
    if ((st = m->g_dec.ensure((size_t)M * sizeof(int)))) return st;
    if ((st = m->g_chg.ensure((size_t)std::max(M + 2, kBlindRounds + 2) * sizeof(int)))) return st;
    // the accept kernel's counter (zeroed by sbp_local_fused_kernel on every call)
    if ((st = m->done_ctr.ensure(64))) return st;
    SbpFusedArgs fu{};
    fu.fr = fr;
    SbpLocalArgs& a = fu.s;
    // AssignFeaturesToGrid: built by every workgroup of the fused kernel in its LDS
    if ((st = m->frame_device(frame, a.f, false))) return st;
    a.mp = mp;
    a.th = th;
    a.nlevels = frame->nlevels;
    a.cnt = m->cnt.as<int>();
    a.cand = m->cand.as<int2>();
    for (int l = 0; l < frame->nlevels; ++l) fu.scalev[l] = frame->scale_factors[l];
    fu.blk = m->s3.as<int>();
    fu.rounds = kBlindRounds;
    GreedyArgs& g = fu.g;
    g.m = M;
    g.nkp = N;
    g.mode = kGreedyLocal;
    g.nnratio = nnratio;
    g.kfix = kSbpFix;
    g.fcnt = m->cnt.as<int>();
    g.cand = m->cand.as<int2>();
    g.cand_cap = LLONG_MAX;
    g.nobs = d_nobs;
    g.fmp0 = g.fmp = d_frame_mp;
    g.fobs0 = g.fobs = d_frame_mp_obs;
    g.ids = d_mp_ids;
    g.T[0] = m->g_t0.as<int>();
    g.T[1] = m->g_t1.as<int>();
    g.T[2] = m->g_t2.as<int>();
    g.dec = m->g_dec.as<int>();
    g.chg = m->g_chg.as<int>();
    g.last = m->g_last.as<int>();
    g.nm = m->scal.as<int>();
    g.save_fmp = m->s1.as<int>();
    g.save_fobs = m->s2.as<int>();
    g.done = m->done_ctr.as<int>();
    g.blk = m->s3.as<int>();
    g.nblk = fblocks;
    g.stats = m->scal.as<int>();
    g.conv_round = kBlindRounds - 1;
    if (!m->stat_host && !m->zero_copy_off) {
        void* q = nullptr;
        void* dq = nullptr;
        if (hipHostMalloc(&q, 64, hipHostMallocDefault) == hipSuccess) {
            if (hipHostGetDevicePointer(&dq, q, 0) == hipSuccess) {
                m->stat_host = static_cast<int*>(q);
                m->stat_dev = static_cast<int*>(dq);
            } else {
                hipHostFree(q);
            }
        }
    }
    g.hstats = m->stat_dev;
    if (m->stat_host)  // "not converged" until the last workgroup writes it
        for (int k = 0; k < 6; ++k) m->stat_host[k] = k == 4 ? -1 : 0;
    const int rblocks = std::max(1, (std::max(std::max(M, N), 32) + kGreedyBlock - 1) / kGreedyBlock);
    const dim3 grid[3] = {dim3(fblocks), dim3(rblocks), dim3((M + kGreedyBlock - 1) / kGreedyBlock)};
    const size_t shm = (size_t)N * 32;
    hipLaunchKernelGGL(sbp_local_fused_kernel<kPre>, grid[0], dim3(1024), shm, m->stream, fu);
    for (int r = 0; r < kBlindRounds - 1; ++r)
        hipLaunchKernelGGL(greedy_round_kernel<true>, grid[1], dim3(kGreedyBlock), 0, m->stream, g, r);
    // the last blind round and the acceptances in one launch
    hipLaunchKernelGGL(greedy_accept_kernel<true>, grid[2], dim3(kGreedyBlock), 0, m->stream,
                       g, kBlindRounds - 1);
    ORBFE_HIP(hipGetLastError());
    m->rounds_on_device = false;
    for (int k = 0; k < 6; ++k) host[k] = 0;
    if (!m->stat_host)
        ORBFE_HIP(hipMemcpyAsync(host, m->scal.p, 6 * sizeof(int), hipMemcpyDeviceToHost, m->stream));
    if (m->stat_host && !m->prof.on) {
        // the accept kernel's last workgroup releases the slots and then writes stat_host[4]
        // (-1 until then): wait on it; past 2 ms synchronise the stream (reports a failed kernel)
        const auto t0 = std::chrono::steady_clock::now();
        while (__atomic_load_n(&m->stat_host[4], __ATOMIC_ACQUIRE) == -1) {
            if (std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(2000)) {
                ORBFE_HIP(hipStreamSynchronize(m->stream));
                break;
            }
            __builtin_ia32_pause();
        }
    } else {
        ORBFE_HIP(hipStreamSynchronize(m->stream));
    }
    if (m->stat_host)
        for (int k = 0; k < 6; ++k) host[k] = __atomic_load_n(&m->stat_host[k], __ATOMIC_ACQUIRE);
    if (!host[3] && host[4] == 0) {  // no overflow, converged
        m->last_rounds = host[5];
        return ORBFE_OK;
    }
    // restore the frame's slots; the caller takes the CSR path
    ORBFE_HIP(hipMemcpyAsync(d_frame_mp, m->s1.p, (size_t)N * 4, hipMemcpyDeviceToDevice, m->stream));
    ORBFE_HIP(hipMemcpyAsync(d_frame_mp_obs, m->s2.p, (size_t)N * 4, hipMemcpyDeviceToDevice, m->stream));
    ++m->capacity_retries;
    return ORBFE_OK;
}
}  // namespace

extern "C" {

orbfe_matcher* orbfe_matcher_create(int device, int* status) {
    int st = check_device(device);
    orbfe_matcher* m = nullptr;
    if (st == ORBFE_OK) {
        try {
            DeviceGuard dg(device);
            m = new orbfe_matcher();
            m->device = device;
            const char* i8 = std::getenv("ORBFE_BF_I8");
            if (i8 && i8[0] == '1') m->bf_kernel = bf_match_kernel;
            if (hipStreamCreateWithFlags(&m->own, hipStreamNonBlocking) != hipSuccess) st = ORBFE_ERR_HIP;
            m->stream = m->own;
        } catch (...) {
            st = ORBFE_ERR_NOMEM;
        }
    }
    if (st != ORBFE_OK && m) {
        delete m;
        m = nullptr;
    }
    if (status) *status = st;
    return m;
}

void orbfe_matcher_destroy(orbfe_matcher* m) {
    if (!m) return;
    DeviceGuard dg(m->device);
    hipStreamSynchronize(m->stream);
    delete m;
}

int orbfe_matcher_set_stream(orbfe_matcher* m, void* s) {
    if (!m) return ORBFE_ERR_ARG;
    m->stream = s ? static_cast<hipStream_t>(s) : m->own;
    return ORBFE_OK;
}

int orbfe_hamming(orbfe_matcher* m, const uint8_t* a, const uint8_t* b, int n, int32_t* dist) {
    if (n < 0 || (n && (!a || !b || !dist))) return ORBFE_ERR_ARG;
    if (n == 0) return m ? ORBFE_OK : ORBFE_ERR_ARG;
    return guarded(m, [&]() {
        int st;
        if ((st = m->up(m->q, a, (size_t)n * 32))) return st;
        if ((st = m->up(m->r, b, (size_t)n * 32))) return st;
        if ((st = m->out.ensure((size_t)n * sizeof(int)))) return st;
        if ((st = m->flush())) return st;
        hipLaunchKernelGGL(hamming_kernel, dim3((n + 255) / 256), dim3(256), 0, m->stream,
                           m->q.as<uint4>(), m->r.as<uint4>(), n, m->out.as<int>());
        if ((st = m->down(dist, m->out, (size_t)n * sizeof(int)))) return st;
        return m->sync();
    });
}

int orbfe_bf_match(orbfe_matcher* m, const uint8_t* q, int nq, const uint8_t* r, int nr,
                   int32_t* best_idx, int32_t* best_dist, int32_t* second_dist) {
    if (nq < 0 || nr < 0 || (nq && (!q || !best_idx || !best_dist || !second_dist)) || (nr && !r))
        return ORBFE_ERR_ARG;
    if (nq == 0) return m ? ORBFE_OK : ORBFE_ERR_ARG;
    return guarded(m, [&]() {
        int st;
        if ((st = m->up(m->q, q, (size_t)nq * 32))) return st;
        if ((st = m->up(m->r, r, (size_t)std::max(nr, 1) * 32))) return st;
        const int counts[2] = {nq, nr};
        if ((st = m->up(m->nq, counts, sizeof(counts)))) return st;
        if ((st = m->out.ensure((size_t)nq * 3 * sizeof(int)))) return st;
        if (nr >= 65536) return ORBFE_ERR_UNSUPPORTED;
        if ((st = m->flush())) return st;
        hipLaunchKernelGGL(m->bf_kernel, dim3((nq + kBfBlock - 1) / kBfBlock, 1), dim3(kBfBlock),
                           0, m->stream, m->q.as<uint8_t>(), 0ll, m->nq.as<int>(), nq,
                           m->r.as<uint8_t>(), 0ll, m->nq.as<int>() + 1, m->out.as<int>());
        std::vector<int> tri((size_t)nq * 3);
        if ((st = m->down(tri.data(), m->out, tri.size() * sizeof(int)))) return st;
        if ((st = m->sync())) return st;
        for (int i = 0; i < nq; ++i) {
            best_idx[i] = tri[3 * i];
            best_dist[i] = tri[3 * i + 1];
            second_dist[i] = tri[3 * i + 2];
        }
        return ORBFE_OK;
    });
}

int orbfe_bf_match_batch_device(orbfe_matcher* m, const uint8_t* d_q, size_t q_pitch,
                                const int32_t* d_nq, int nq_cap, const uint8_t* d_r,
                                size_t r_pitch, const int32_t* d_nr, int nb, int32_t* d_out) {
    if (!m || nb < 0 || nq_cap < 0 || (nb && (!d_q || !d_nq || !d_r || !d_nr || !d_out)))
        return ORBFE_ERR_ARG;
    if (nb == 0 || nq_cap == 0) return ORBFE_OK;
    if ((q_pitch | r_pitch) & 15) return ORBFE_ERR_ARG;
    return guarded(m, [&]() {
        // one reference set for the whole batch (r_pitch 0) on the FP4 path: expanded to FP4
        // fragments once (ORBFE_BF_PRE=0: every workgroup expands it, as for per-entry sets)
        if (r_pitch == 0 && m->bf_kernel == bf_match_fp4_kernel && m->bf_pre) {
            int st;
            orbfe_matcher::BfSlot* pe = m->bf_buffer(m->stream, &st);
            if (!pe) return st;
            DevBuf& e = pe->buf;
            // its own profiler stage (1): the bench's per-launch figures are the match kernel's
            ORBFE_LAUNCH(m->prof, 1, bf_expand_kernel, dim3(kBfExpandBlocks), dim3(512), 0, m->stream,
                         d_r, d_nr, nb, e.as<i32x4>());
            ORBFE_LAUNCH(m->prof, 0, bf_match_fp4e_kernel, dim3((nq_cap + kBfBlock - 1) / kBfBlock, nb),
                         dim3(kBfBlock), 0, m->stream, d_q, (long long)q_pitch, d_nq, nq_cap, d_r,
                         (long long)r_pitch, d_nr, d_out, (const i32x4*)e.as<i32x4>());
            ORBFE_HIP(hipEventRecord(pe->done, m->stream));
            ORBFE_HIP(hipGetLastError());
            return ORBFE_OK;
        }
        ORBFE_LAUNCH(m->prof, 0, m->bf_kernel, dim3((nq_cap + kBfBlock - 1) / kBfBlock, nb),
                     dim3(kBfBlock), 0, m->stream, d_q, (long long)q_pitch, d_nq, nq_cap, d_r,
                     (long long)r_pitch, d_nr, d_out);
        ORBFE_HIP(hipGetLastError());
        return ORBFE_OK;
    });
}

int orbfe_matcher_profile(orbfe_matcher* m, int enable) {
    if (!m) return ORBFE_ERR_ARG;
    m->prof.on = enable != 0;
    m->prof.used = 0;
    return ORBFE_OK;
}

int orbfe_matcher_profile_read_stages(orbfe_matcher* m, double* total_ms, int32_t* launches) {
    if (!m || !total_ms || !launches) return ORBFE_ERR_ARG;
    DeviceGuard dg(m->device);
    ORBFE_HIP(hipStreamSynchronize(m->stream));
    for (int k = 0; k < ORBFE_MATCHER_STAGES; ++k) {
        total_ms[k] = 0;
        launches[k] = 0;
    }
    for (size_t i = 0; i < m->prof.used; ++i) {
        float ms = 0.f;
        ORBFE_HIP(hipEventElapsedTime(&ms, m->prof.a[i], m->prof.b[i]));
        const int k = m->prof.kind[i];
        if (k < 0 || k >= ORBFE_MATCHER_STAGES) continue;
        total_ms[k] += ms;
        launches[k] += 1;
    }
    m->prof.used = 0;
    return ORBFE_OK;
}

int orbfe_matcher_profile_read(orbfe_matcher* m, double* total_ms, int32_t* launches) {
    if (!m || !total_ms || !launches) return ORBFE_ERR_ARG;
    double ms[ORBFE_MATCHER_STAGES];
    int32_t n[ORBFE_MATCHER_STAGES];
    const int st = orbfe_matcher_profile_read_stages(m, ms, n);
    if (st) return st;
    *total_ms = ms[0];  // the matcher kernels (stage 0); the expansion is stage 1
    *launches = n[0];
    return ORBFE_OK;
}

int orbfe_search_for_initialization(orbfe_matcher* m, float nnratio, int check_ori,
                                    const orbfe_frame_view* f1, const orbfe_frame_view* f2,
                                    float* prev_matched, int window, int32_t* matches12,
                                    int32_t* nmatches) {
    if (!frame_ok(f1) || !frame_ok(f2) || !nmatches || (f1->n && (!prev_matched || !matches12)))
        return ORBFE_ERR_ARG;
    bool retried = false;
    return guarded(m, [&]() {
        std::function<int()> attempt = [&]() -> int {
        int st;
        SfiArgs a;
        if ((st = m->up(m->s5, prev_matched, (size_t)f1->n * 2 * sizeof(float)))) return st;
        const int32_t zero[4] = {0, 0, 0, 0};
        if ((st = m->up(m->scal, zero, sizeof(zero)))) return st;
        if ((st = m->frame(f1, false, a.f1))) return st;
        if ((st = m->frame(f2, true, a.f2))) return st;
        a.prev = m->s5.as<float>();
        a.window = (float)window;
        const int n1 = f1->n, n2 = f2->n;
        // candidates without a host round trip: the fill is bounded by the current capacity,
        // checked at the first synchronisation of the rounds (one retry with the exact total)
        const size_t cap = std::max(m->cand.bytes / sizeof(int2), (size_t)64 * std::max(n1, 1));
        if ((st = m->cand.ensure(cap * sizeof(int2)))) return st;
        if ((st = m->cnt.ensure(std::max(n1, 1) * sizeof(int)))) return st;
        if ((st = m->off.ensure((n1 + 1) * sizeof(int)))) return st;
        a.cnt = m->cnt.as<int>();
        a.off = m->off.as<int>();
        a.cand = m->cand.as<int2>();
        a.cand_cap = (long long)cap;
        const int qb = std::max(1, (n1 + 3) / 4);
        hipLaunchKernelGGL(sfi_cand_kernel<false>, dim3(qb), dim3(256), 0, m->stream, a);
        hipLaunchKernelGGL(scan_kernel, dim3(1), dim3(1024), 0, m->stream, m->cnt.as<int>(), n1, m->off.as<int>());
        hipLaunchKernelGGL(sfi_cand_kernel<true>, dim3(qb), dim3(256), 0, m->stream, a);
        // fixed-point rounds (sfi_round_kernel): decisions, slot lists, change flags
        const int L2 = std::max(n2, 1);
        if ((st = m->g_dec.ensure((size_t)2 * std::max(n1, 1) * sizeof(int)))) return st;
        if ((st = m->g_t1.ensure((size_t)3 * L2 * sizeof(int)))) return st;
        if ((st = m->g_chg.ensure((size_t)(n1 + 4) * sizeof(int)))) return st;  // overflow, -, rounds 0..n1
        if ((st = m->s2.ensure(std::max(n1, 1) * 2 * sizeof(int)))) return st;
        if ((st = m->flush())) return st;
        int total = 0;  // read back with the first batch's change flags
        if ((st = m->down_ptr(&total, m->off.as<int>() + n1, sizeof(int)))) return st;
        SfiRoundArgs r{};
        r.n1 = n1;
        r.n2 = n2;
        r.off = m->off.as<int>();
        r.cand = m->cand.as<int2>();
        r.cand_cap = (long long)cap;
        r.nnratio = nnratio;
        r.dec[0] = m->g_dec.as<int>();
        r.dec[1] = r.dec[0] + std::max(n1, 1);
        r.chg = m->g_chg.as<int>() + 2;
        r.overflow = m->g_chg.as<int>();
        r.status = m->scal.as<int>() + 1;
        const int rb = std::max(1, (std::max(n1 * 64, n2) + 255) / 256);
        // slot lists of 64 acceptors; a slot drawing more in some round (one query per slot is
        // the usual case) reruns the rounds with room for every query
        // conv: the first round without a change; the rounds a batch launches past it exit at
        // once (sfi_round_kernel), so conv's decision and list buffers hold the final state
        int conv = -1;
        for (int k : {kSfiSlotK, std::max(n1, 1)}) {
            r.k = k;
            if ((st = m->g_t0.ensure((size_t)3 * L2 * k * sizeof(int2)))) return st;
            for (int b = 0; b < 3; ++b) {
                r.list[b] = m->g_t0.as<int2>() + (size_t)b * L2 * k;
                r.lcnt[b] = m->g_t1.as<int>() + (size_t)b * L2;
            }
            // round 0 compares against 0xfefefefe (< -1: no decision), reads an empty list 0
            {
                const int nmax = std::max(std::max(std::max(n1, 1), 2 * L2), n1 + 4);
                hipLaunchKernelGGL(sfi_init_kernel, dim3(std::min(64, (nmax + 255) / 256)), dim3(256), 0,
                                   m->stream, r.dec[0], std::max(n1, 1), m->g_t1.as<int>(), 2 * L2,
                                   m->g_chg.as<int>(), n1 + 4);
            }
            int rr = 0, batch = 6, ovf = 0;
            std::vector<int> chg_h;
            while (conv < 0) {
                const int r0 = rr;
                for (int b = 0; b < batch && rr <= n1; ++b, ++rr)
                    hipLaunchKernelGGL(sfi_round_kernel, dim3(rb), dim3(256), 0, m->stream, r, rr);
                ORBFE_HIP(hipGetLastError());
                // the overflow word and the batch's change flags through the staging buffer (the
                // gather kernel and the done word, not two pageable copies and a stream sync)
                chg_h.assign(rr - r0 + 2, 0);
                if ((st = m->down_ptr(chg_h.data(), m->g_chg.as<int>(), sizeof(int)))) return st;
                if ((st = m->down_ptr(chg_h.data() + 2, r.chg + r0, (size_t)(rr - r0) * sizeof(int)))) return st;
                if ((st = m->sync())) return st;
                if ((size_t)total > cap) {
                    if (retried) return ORBFE_ERR_HIP;
                    if ((st = m->cand.ensure((size_t)total * sizeof(int2)))) return st;
                    retried = true;
                    ++m->capacity_retries;
                    m->begin();
                    return attempt();
                }
                ovf = chg_h[0];
                if (ovf) break;
                for (int q = 0; q < rr - r0; ++q)
                    if (!chg_h[2 + q]) { conv = r0 + q; break; }
                if (conv < 0 && rr > n1) return ORBFE_ERR_HIP;  // cannot happen: the prefix grows
                batch = std::min(batch * 2, 64);
            }
            if (conv >= 0) break;
        }
        if (conv < 0) return ORBFE_ERR_HIP;  // lists sized for every query cannot overflow
        m->rounds_on_device = false;
        m->last_rounds = conv + 1;
        SfiFinalArgs fa;
        fa.n1 = n1;
        fa.k = r.k;
        fa.k1 = a.f1.k;
        fa.k2 = a.f2.k;
        fa.dec = r.dec[~conv & 1];
        fa.list = r.list[(conv + 1) % 3];
        fa.lcnt = r.lcnt[(conv + 1) % 3];
        fa.check_ori = check_ori;
        fa.m12 = m->s2.as<int>();
        fa.rotbin = fa.m12 + std::max(n1, 1);
        fa.prev = m->s5.as<float>();
        fa.nmatches = m->scal.as<int>();
        hipLaunchKernelGGL(sfi_final_kernel, dim3(1), dim3(1024), 0, m->stream, fa);
        ORBFE_HIP(hipGetLastError());
        if ((st = m->down(matches12, m->s2, (size_t)n1 * sizeof(int)))) return st;
        if ((st = m->down(prev_matched, m->s5, (size_t)n1 * 2 * sizeof(float)))) return st;
        int res[2] = {0, 0};
        if ((st = m->down(res, m->scal, sizeof(res)))) return st;
        if ((st = m->sync())) return st;
        *nmatches = res[0];
        return res[1];
        };
        return attempt();
    });
}

int orbfe_search_by_projection_local(orbfe_matcher* m, float nnratio,
                                     const orbfe_frame_view* f, int32_t* frame_mp,
                                     int32_t* frame_mp_obs, const orbfe_mappoint_view* mps,
                                     const int32_t* mp_ids, float th, int32_t* nmatches) {
    if (!frame_ok(f) || !mps || mps->m < 0 || !nmatches || (f->n && (!frame_mp || !frame_mp_obs)))
        return ORBFE_ERR_ARG;
    const int M = mps->m;
    if (M && (!mps->track_in_view || !mps->is_bad || !mps->proj_x || !mps->proj_y ||
              !mps->proj_xr || !mps->pred_level || !mps->view_cos || !mps->desc || !mps->n_obs))
        return ORBFE_ERR_ARG;
    for (int i = 0; i < M; ++i)  // mvScaleFactors[nPredictedLevel] outside the table is UB
        if (mps->track_in_view[i] && !mps->is_bad[i] &&
            (mps->pred_level[i] < 0 || mps->pred_level[i] >= f->nlevels))
            return ORBFE_ERR_UNSUPPORTED;
    // fixed-slot candidates (one kernel, no mid-call count read-back) unless a point has more
    // than kSbpFix of them: then the CSR path from the saved slots
    std::vector<int32_t> fmp_in, fobs_in;
    bool fix = f->n > 0 && M > 0;
    if (fix) {
        fmp_in.assign(frame_mp, frame_mp + f->n);
        fobs_in.assign(frame_mp_obs, frame_mp_obs + f->n);
    }
    return guarded(m, [&]() {
      for (;;) {
        int st;
        SbpLocalArgs a;
        const int32_t zero[4] = {0, 0, 0, 0};  // nmatches, -, overflow
        if ((st = m->up(m->scal, zero, sizeof(zero)))) return st;
        if ((st = m->frame(f, false, a.f))) return st;
        if ((st = m->up(m->m_u0, mps->track_in_view, M))) return st;
        if ((st = m->up(m->m_u1, mps->is_bad, M))) return st;
        if ((st = m->up(m->m_f0, mps->proj_x, (size_t)M * 4))) return st;
        if ((st = m->up(m->m_f1, mps->proj_y, (size_t)M * 4))) return st;
        if ((st = m->up(m->m_f2, mps->proj_xr, (size_t)M * 4))) return st;
        if ((st = m->up(m->m_i0, mps->pred_level, (size_t)M * 4))) return st;
        if ((st = m->up(m->m_f3, mps->view_cos, (size_t)M * 4))) return st;
        if ((st = m->up(m->m_d, mps->desc, (size_t)M * 32))) return st;
        if ((st = m->up(m->m_i1, mps->n_obs, (size_t)M * 4))) return st;
        if ((st = m->up(m->m_f4, f->scale_factors, (size_t)f->nlevels * 4))) return st;
        if (mp_ids && (st = m->up(m->o_i, mp_ids, (size_t)M * 4))) return st;
        a.mp = SbpMps{M, m->m_u0.as<uint8_t>(), m->m_u1.as<uint8_t>(), m->m_f0.as<float>(),
                      m->m_f1.as<float>(), m->m_f2.as<float>(), m->m_i0.as<int>(),
                      m->m_f3.as<float>(), m->m_d.as<uint4>(), m->m_i1.as<int>()};
        a.scale = m->m_f4.as<float>();
        a.th = th;
        a.nlevels = f->nlevels;
        a.status = nullptr;  // levels were checked on the host
        a.cand_cap = LLONG_MAX;
        a.kfix = kSbpFix;
        a.ovf = m->scal.as<int>() + 2;
        if (fix) {
            if ((st = m->cnt.ensure((size_t)M * sizeof(int)))) return st;
            if ((st = m->cand.ensure((size_t)M * kSbpFix * sizeof(int2)))) return st;
            a.cnt = m->cnt.as<int>();
            a.cand = m->cand.as<int2>();
            if ((st = m->flush())) return st;
            hipLaunchKernelGGL(sbp_local_cand_kernel<2>, dim3((M + 3) / 4), dim3(256), 0, m->stream, a);
            ORBFE_HIP(hipGetLastError());
        } else {
            int total = 0;
            if ((st = m->csr(a, M, sbp_local_cand_kernel<0>, sbp_local_cand_kernel<1>, total, 4)))
                return st;
        }
        const int N = f->n;
        if ((st = m->up(m->s1, frame_mp, (size_t)N * 4))) return st;
        if ((st = m->up(m->s2, frame_mp_obs, (size_t)N * 4))) return st;
        if ((st = m->s3.ensure(std::max(N, 1) * sizeof(int)))) return st;
        if ((st = m->scal.ensure(16))) return st;
        GreedyArgs g{};
        g.m = M;
        g.nkp = N;
        g.mode = kGreedyLocal;
        g.nnratio = nnratio;
        g.off = m->off.as<int>();
        g.cand = m->cand.as<int2>();
        g.nobs = m->m_i1.as<int>();
        g.fmp0 = g.fmp = m->s1.as<int>();
        g.fobs0 = g.fobs = m->s2.as<int>();
        g.ids = mp_ids ? m->o_i.as<int>() : nullptr;
        if (fix) {
            g.kfix = kSbpFix;
            g.fcnt = m->cnt.as<int>();
        }
        if ((st = m->greedy(g))) return st;
        if ((st = m->down(frame_mp, m->s1, (size_t)N * 4))) return st;
        if ((st = m->down(frame_mp_obs, m->s2, (size_t)N * 4))) return st;
        int res[3] = {0, 0, 0};  // {nmatches, -, overflow}
        if ((st = m->down(res, m->scal, sizeof(res)))) return st;
        if ((st = m->sync())) return st;
        if (fix && res[2] > 0) {  // a point past kSbpFix candidates: the CSR path from the input
            std::memcpy(frame_mp, fmp_in.data(), (size_t)N * 4);
            std::memcpy(frame_mp_obs, fobs_in.data(), (size_t)N * 4);
            fix = false;
            ++m->capacity_retries;
            m->begin();
            continue;
        }
        *nmatches = res[0];
        return ORBFE_OK;
      }
    });
}

constexpr int kSbpLastFix = 64;  // SearchByProjection(last frame): fixed candidate slots per point

int orbfe_search_by_projection_last(orbfe_matcher* m, int check_ori,
                                    const orbfe_frame_view* cur, const float* tcw_cur,
                                    const orbfe_camera* cam, int32_t* frame_mp,
                                    int32_t* frame_mp_obs, int n_last,
                                    const orbfe_keypoint* last_keys,
                                    const uint8_t* last_mp_valid, const uint8_t* last_outlier,
                                    const float* last_mp_xyz, const uint8_t* last_mp_desc,
                                    const int32_t* last_mp_nobs, const int32_t* last_mp_ids,
                                    const float* tcw_last, float th, int mono,
                                    int32_t* nmatches) {
    if (!frame_ok(cur) || !tcw_cur || !tcw_last || !cam || !nmatches || n_last < 0 ||
        (cur->n && (!frame_mp || !frame_mp_obs)) ||
        (n_last && (!last_keys || !last_mp_valid || !last_outlier || !last_mp_xyz ||
                    !last_mp_desc || !last_mp_nobs)))
        return ORBFE_ERR_ARG;
    for (int i = 0; i < n_last; ++i)
        if (last_mp_valid[i] && (last_keys[i].octave < 0 || last_keys[i].octave >= cur->nlevels))
            return ORBFE_ERR_UNSUPPORTED;
    // fixed-slot candidates unless a point has more than kSbpLastFix (then the CSR path from the
    // saved slots), as the keyframe overload below; 64 slots: the mono th = 15 window over three
    // octaves holds more than 16 keypoints for some points of a 1000-keypoint frame
    std::vector<int32_t> fmp_in, fobs_in;
    bool fix = cur->n > 0 && n_last > 0;
    if (fix) {
        fmp_in.assign(frame_mp, frame_mp + cur->n);
        fobs_in.assign(frame_mp_obs, frame_mp_obs + cur->n);
    }
    return guarded(m, [&]() {
      for (;;) {
        int st;
        SbpLastArgs a;
        const int32_t zero[4] = {0, 0, 0, 0};  // nmatches, -, overflow
        if ((st = m->up(m->scal, zero, sizeof(zero)))) return st;
        if ((st = m->frame(cur, false, a.cur))) return st;
        if ((st = m->up(m->fb_k, last_keys, (size_t)n_last * sizeof(orbfe_keypoint)))) return st;
        if ((st = m->up(m->m_u0, last_mp_valid, n_last))) return st;
        if ((st = m->up(m->m_u1, last_outlier, n_last))) return st;
        if ((st = m->up(m->m_f0, last_mp_xyz, (size_t)n_last * 12))) return st;
        if ((st = m->up(m->m_d, last_mp_desc, (size_t)n_last * 32))) return st;
        if ((st = m->up(m->m_i1, last_mp_nobs, (size_t)n_last * 4))) return st;
        if ((st = m->up(m->m_f4, cur->scale_factors, (size_t)cur->nlevels * 4))) return st;
        if (last_mp_ids && (st = m->up(m->o_i, last_mp_ids, (size_t)n_last * 4))) return st;
        a.n_last = n_last;
        a.lk = m->fb_k.as<orbfe_keypoint>();
        a.valid = m->m_u0.as<uint8_t>();
        a.outlier = m->m_u1.as<uint8_t>();
        a.xyz = m->m_f0.as<float>();
        a.desc = m->m_d.as<uint4>();
        std::memcpy(a.T, tcw_cur, sizeof(a.T));
        a.fx = cam->fx;
        a.fy = cam->fy;
        a.cx = cam->cx;
        a.cy = cam->cy;
        a.bf = cam->bf;
        a.minx = cur->min_x;
        a.maxx = cur->max_x;
        a.miny = cur->min_y;
        a.maxy = cur->max_y;
        a.scale = m->m_f4.as<float>();
        a.th = th;
        float twc[3], tlc[3];  // 1341-1352: motion direction for stereo/RGB-D
        camera_center(tcw_cur, twc);
        rigid(tcw_last, twc, tlc);
        const bool fwd = tlc[2] > cam->b && !mono;
        const bool bwd = -tlc[2] > cam->b && !mono;
        a.mode = fwd ? 1 : bwd ? 2 : 0;
        a.kfix = kSbpLastFix;
        a.ovf = m->scal.as<int>() + 2;
        if (fix) {
            if ((st = m->cnt.ensure((size_t)n_last * sizeof(int)))) return st;
            if ((st = m->cand.ensure((size_t)n_last * kSbpLastFix * sizeof(int2)))) return st;
            a.cnt = m->cnt.as<int>();
            a.cand = m->cand.as<int2>();
            if ((st = m->flush())) return st;
            hipLaunchKernelGGL(sbp_last_cand_kernel<2>, dim3((n_last + 3) / 4), dim3(256), 0, m->stream, a);
            ORBFE_HIP(hipGetLastError());
        } else if ((st = m->csr_async(a, n_last, sbp_last_cand_kernel<0>, sbp_last_cand_kernel<1>, 4))) {
            return st;
        }
        const int N = cur->n;
        if ((st = m->up(m->s1, frame_mp, (size_t)N * 4))) return st;
        if ((st = m->up(m->s2, frame_mp_obs, (size_t)N * 4))) return st;
        if ((st = m->s3.ensure(std::max(N, 1) * sizeof(int)))) return st;
        if ((st = m->s4.ensure(std::max(n_last, 1) * sizeof(int2)))) return st;
        if ((st = m->scal.ensure(16))) return st;
        if ((st = m->o_f3.ensure(std::max<size_t>(16, (size_t)n_last * 4)))) return st;
        std::vector<float> qa(n_last);
        for (int i = 0; i < n_last; ++i) qa[i] = last_keys[i].angle;
        if ((st = m->up(m->o_f3, qa.data(), (size_t)n_last * 4))) return st;
        GreedyArgs g{};
        g.m = n_last;
        g.nkp = N;
        g.mode = kGreedyMaxD;
        g.max_dist = kThHigh;
        g.off = m->off.as<int>();
        g.cand = m->cand.as<int2>();
        g.nobs = m->m_i1.as<int>();
        g.fmp0 = g.fmp = m->s1.as<int>();
        g.fobs0 = g.fobs = m->s2.as<int>();
        g.check_ori = check_ori;
        g.q_angle = m->o_f3.as<float>();
        g.k = a.cur.k;
        g.ids = last_mp_ids ? m->o_i.as<int>() : nullptr;
        if (fix) {
            g.kfix = kSbpLastFix;
            g.fcnt = m->cnt.as<int>();
        }
        if ((st = m->greedy(g))) return st;
        if ((st = m->down(frame_mp, m->s1, (size_t)N * 4))) return st;
        if ((st = m->down(frame_mp_obs, m->s2, (size_t)N * 4))) return st;
        int res[3] = {0, 0, 0};  // {nmatches, -, overflow}
        if ((st = m->down(res, m->scal, sizeof(res)))) return st;
        if ((st = m->sync())) return st;
        if (fix && res[2] > 0) {  // a point past kSbpLastFix candidates: the CSR path from the input
            std::memcpy(frame_mp, fmp_in.data(), (size_t)N * 4);
            std::memcpy(frame_mp_obs, fobs_in.data(), (size_t)N * 4);
            fix = false;
            ++m->capacity_retries;
            m->begin();
            continue;
        }
        *nmatches = res[0];
        return ORBFE_OK;
      }
    });
}

int orbfe_search_by_projection_keyframe(orbfe_matcher* m, int check_ori,
                                        const orbfe_frame_view* cur, const float* tcw_cur,
                                        const orbfe_camera* cam, float log_scale_factor,
                                        int32_t* frame_mp, int n_kf, const float* kf_key_angle,
                                        const uint8_t* kf_mp_valid, const uint8_t* kf_mp_bad,
                                        const uint8_t* already_found, const float* kf_mp_xyz,
                                        const uint8_t* kf_mp_desc, const float* kf_mp_min_dist,
                                        const float* kf_mp_max_dist, const int32_t* kf_mp_ids,
                                        float th, int orb_dist, int32_t* nmatches) {
    if (!frame_ok(cur) || !tcw_cur || !cam || !nmatches || n_kf < 0 || (cur->n && !frame_mp) ||
        (n_kf && (!kf_key_angle || !kf_mp_valid || !kf_mp_bad || !already_found || !kf_mp_xyz ||
                  !kf_mp_desc || !kf_mp_min_dist || !kf_mp_max_dist)))
        return ORBFE_ERR_ARG;
    // the fixed-slot candidates (one kernel instead of count / scan / fill) unless a point has
    // more than kSbpFix of them: then the call runs again on the CSR path from the saved slots
    std::vector<int32_t> fmp_in;
    bool fix = cur->n > 0 && n_kf > 0;
    if (fix) fmp_in.assign(frame_mp, frame_mp + cur->n);
    return guarded(m, [&]() {
      for (;;) {
        int st;
        SbpKfArgs a;
        // every upload is staged before the frame's flush: one H2D copy + one scatter launch;
        // the status word is cleared by the same copy
        const int32_t zero[4] = {0, 0, 0, 0};
        if ((st = m->up(m->scal, zero, sizeof(zero)))) return st;
        // a slot already holding a map point blocks (1529-1530), whatever its observations
        if ((st = m->up(m->s1, frame_mp, (size_t)cur->n * 4))) return st;
        if ((st = m->up(m->m_u0, kf_mp_valid, n_kf))) return st;
        if ((st = m->up(m->m_u1, kf_mp_bad, n_kf))) return st;
        if ((st = m->up(m->o_u, already_found, n_kf))) return st;
        if ((st = m->up(m->m_f0, kf_mp_xyz, (size_t)n_kf * 12))) return st;
        if ((st = m->up(m->m_f1, kf_mp_min_dist, (size_t)n_kf * 4))) return st;
        if ((st = m->up(m->m_f2, kf_mp_max_dist, (size_t)n_kf * 4))) return st;
        if ((st = m->up(m->m_f3, kf_key_angle, (size_t)n_kf * 4))) return st;
        if ((st = m->up(m->m_d, kf_mp_desc, (size_t)n_kf * 32))) return st;
        if ((st = m->up(m->m_f4, cur->scale_factors, (size_t)cur->nlevels * 4))) return st;
        if (kf_mp_ids && (st = m->up(m->o_i, kf_mp_ids, (size_t)n_kf * 4))) return st;
        if ((st = m->frame(cur, false, a.cur))) return st;
        a.n = n_kf;
        a.valid = m->m_u0.as<uint8_t>();
        a.bad = m->m_u1.as<uint8_t>();
        a.found = m->o_u.as<uint8_t>();
        a.xyz = m->m_f0.as<float>();
        a.mind = m->m_f1.as<float>();
        a.maxd = m->m_f2.as<float>();
        a.desc = m->m_d.as<uint4>();
        std::memcpy(a.T, tcw_cur, sizeof(a.T));
        camera_center(tcw_cur, a.ow);
        a.fx = cam->fx;
        a.fy = cam->fy;
        a.cx = cam->cx;
        a.cy = cam->cy;
        a.minx = cur->min_x;
        a.maxx = cur->max_x;
        a.miny = cur->min_y;
        a.maxy = cur->max_y;
        a.scale = m->m_f4.as<float>();
        a.nlevels = cur->nlevels;
        a.log_scale = log_scale_factor;
        a.th = th;
        a.status = m->scal.as<int>() + 1;
        a.kfix = kSbpFix;
        a.ovf = m->scal.as<int>() + 2;
        if (fix) {
            if ((st = m->cnt.ensure((size_t)n_kf * sizeof(int)))) return st;
            if ((st = m->cand.ensure((size_t)n_kf * kSbpFix * sizeof(int2)))) return st;
            a.cnt = m->cnt.as<int>();
            a.cand = m->cand.as<int2>();
            if ((st = m->flush())) return st;
            hipLaunchKernelGGL(sbp_kf_cand_kernel<2>, dim3((n_kf + 3) / 4), dim3(256), 0, m->stream, a);
            ORBFE_HIP(hipGetLastError());
        } else if ((st = m->csr_async(a, n_kf, sbp_kf_cand_kernel<0>, sbp_kf_cand_kernel<1>, 4))) {
            return st;
        }
        const int N = cur->n;
        GreedyArgs g{};
        g.m = n_kf;
        g.nkp = N;
        g.mode = kGreedyMaxD;
        g.max_dist = orb_dist;
        g.off = m->off.as<int>();
        g.cand = m->cand.as<int2>();
        g.nobs = nullptr;
        g.fmp0 = g.fmp = m->s1.as<int>();
        g.fobs0 = g.fobs = nullptr;
        g.check_ori = check_ori;
        g.q_angle = m->m_f3.as<float>();  // pKF->mvKeysUn[i].angle (1549)
        g.k = a.cur.k;
        g.ids = kf_mp_ids ? m->o_i.as<int>() : nullptr;
        if (fix) {
            g.kfix = kSbpFix;
            g.fcnt = m->cnt.as<int>();
        }
        if ((st = m->greedy(g))) return st;
        if ((st = m->down(frame_mp, m->s1, (size_t)N * 4))) return st;
        // {nmatches, status, overflow}: status != 0 is a predicted level outside the pyramid
        // (outputs then unspecified)
        int res[3] = {0, 0, 0};
        if ((st = m->down(res, m->scal, sizeof(res)))) return st;
        if ((st = m->sync())) return st;
        if (fix && res[2] > 0) {  // a point past kSbpFix candidates: the CSR path from the input
            std::memcpy(frame_mp, fmp_in.data(), (size_t)N * 4);
            fix = false;
            ++m->capacity_retries;
            m->begin();
            continue;
        }
        *nmatches = res[0];
        return res[1];
      }
    });
}

int orbfe_distinctive_descriptors_device(orbfe_matcher* m, int n_mp, const int32_t* d_obs_off,
                                         const uint8_t* d_obs_desc, int32_t* d_best,
                                         uint8_t* d_desc_out) {
    if (n_mp < 0 || (n_mp && (!d_obs_off || !d_obs_desc || !d_best))) return ORBFE_ERR_ARG;
    return guarded(m, [&]() {
        if (n_mp == 0) return ORBFE_OK;
        hipLaunchKernelGGL(distinctive_kernel, dim3((n_mp + 3) / 4), dim3(kDdBlock), 0, m->stream,
                           n_mp, d_obs_off, reinterpret_cast<const uint4*>(d_obs_desc), d_best,
                           reinterpret_cast<uint4*>(d_desc_out));
        ORBFE_HIP(hipGetLastError());
        return ORBFE_OK;
    });
}

int orbfe_distinctive_descriptors(orbfe_matcher* m, int n_mp, const int32_t* obs_off,
                                  const uint8_t* obs_desc, int32_t* best, uint8_t* desc_out) {
    if (n_mp < 0 || (n_mp && (!obs_off || !best))) return ORBFE_ERR_ARG;
    if (n_mp == 0) return m ? ORBFE_OK : ORBFE_ERR_ARG;
    if (obs_off[0] < 0) return ORBFE_ERR_ARG;
    for (int i = 0; i < n_mp; ++i)
        if (obs_off[i + 1] < obs_off[i] || obs_off[i + 1] - obs_off[i] >= 65536) return ORBFE_ERR_ARG;
    const size_t nobs = (size_t)obs_off[n_mp];
    if (nobs && !obs_desc) return ORBFE_ERR_ARG;
    return guarded(m, [&]() {
        int st;
        if ((st = m->up(m->o_i, obs_off, (size_t)(n_mp + 1) * 4))) return st;
        if ((st = m->up(m->m_d, obs_desc, nobs * 32))) return st;
        if ((st = m->s1.ensure((size_t)n_mp * 4))) return st;
        if ((st = m->q.ensure((size_t)n_mp * 32))) return st;
        if ((st = m->flush())) return st;
        hipLaunchKernelGGL(distinctive_kernel, dim3((n_mp + 3) / 4), dim3(kDdBlock), 0, m->stream,
                           n_mp, m->o_i.as<int>(), m->m_d.as<uint4>(), m->s1.as<int>(),
                           desc_out ? m->q.as<uint4>() : nullptr);
        ORBFE_HIP(hipGetLastError());
        if ((st = m->down(best, m->s1, (size_t)n_mp * 4))) return st;
        if (desc_out && (st = m->down(desc_out, m->q, (size_t)n_mp * 32))) return st;
        return m->sync();
    });
}

int orbfe_search_local_points_device(orbfe_matcher* m, const orbfe_frame_view* frame,
                                     const float* tcw, const orbfe_camera* cam,
                                     float log_scale_factor, float viewing_cos_limit, int n_mp,
                                     const float* d_xyz, const float* d_normal,
                                     const float* d_min_dist, const float* d_max_dist,
                                     const uint8_t* d_desc, const int32_t* d_nobs,
                                     const uint8_t* d_bad, const uint8_t* d_skip,
                                     const int32_t* d_mp_ids, float nnratio, float th,
                                     int32_t* d_frame_mp, int32_t* d_frame_mp_obs,
                                     uint8_t* d_in_view, int32_t* counts) {
    if (!frame_ok(frame) || !tcw || !cam || n_mp < 0 || !counts ||
        (frame->n && (!d_frame_mp || !d_frame_mp_obs)) ||
        (n_mp && (!d_xyz || !d_normal || !d_min_dist || !d_max_dist || !d_desc || !d_nobs ||
                  !d_bad || !d_in_view)))
        return ORBFE_ERR_ARG;
    return guarded(m, [&]() {
        int st;
        const int M = n_mp, N = frame->n;
        if ((st = m->scal.ensure(64))) return st;
        for (DevBuf* b : {&m->o_f0, &m->o_f1, &m->o_f2, &m->o_f3, &m->o_i})
            if ((st = b->ensure(std::max<size_t>(16, (size_t)M * 4)))) return st;
        int* d_cnt = m->scal.as<int>() + 1;     // nToMatch
        int* d_status = m->scal.as<int>() + 2;  // UB level
        // fast path (sbp_local_fast), else / on its fallback the CSR path below
        if (N <= kSbpFixKp && frame->nlevels <= kMaxLevels && M > 0) {
            FrustumArgs fa{};
            fa.n = M;
            fa.xyz = d_xyz;
            fa.normal = d_normal;
            fa.mind = d_min_dist;
            fa.maxd = d_max_dist;
            std::memcpy(fa.T, tcw, sizeof(fa.T));
            camera_center(tcw, fa.ow);
            fa.fx = cam->fx;
            fa.fy = cam->fy;
            fa.cx = cam->cx;
            fa.cy = cam->cy;
            fa.bf = cam->bf;
            fa.minx = frame->min_x;
            fa.maxx = frame->max_x;
            fa.miny = frame->min_y;
            fa.maxy = frame->max_y;
            fa.log_scale = log_scale_factor;
            fa.cos_limit = viewing_cos_limit;
            fa.in_view = d_in_view;
            fa.skip = d_skip;
            fa.bad = d_bad;
            SbpMps mp{};
            mp.m = M;
            mp.desc = reinterpret_cast<const uint4*>(d_desc);
            int host[6];
            if ((st = sbp_local_fast<false>(m, frame, fa, mp, nnratio, th, d_nobs, d_mp_ids, d_frame_mp,
                                            d_frame_mp_obs, host)))
                return st;
            if (!host[3] && host[4] == 0) {  // no overflow, converged
                counts[0] = host[0];
                counts[1] = host[1];
                return host[2] ? host[2] : ORBFE_OK;
            }
        }
        bool retried = false;
        // (the fast path above passes mvScaleFactors in its kernel arguments)
        if ((st = m->m_f4.ensure(std::max<size_t>(16, (size_t)frame->nlevels * 4)))) return st;
        ORBFE_HIP(hipMemcpyAsync(m->m_f4.p, frame->scale_factors, (size_t)frame->nlevels * 4,
                                 hipMemcpyHostToDevice, m->stream));
        std::function<int()> attempt = [&]() -> int {
        ORBFE_HIP(hipMemsetAsync(m->scal.p, 0, 16, m->stream));
        // Tracking::SearchLocalPoints: isInFrustum(pMP, 0.5) over the local map (1425-1438)
        FrustumArgs fa;
        fa.n = M;
        fa.xyz = d_xyz;
        fa.normal = d_normal;
        fa.mind = d_min_dist;
        fa.maxd = d_max_dist;
        std::memcpy(fa.T, tcw, sizeof(fa.T));
        camera_center(tcw, fa.ow);
        fa.fx = cam->fx;
        fa.fy = cam->fy;
        fa.cx = cam->cx;
        fa.cy = cam->cy;
        fa.bf = cam->bf;
        fa.minx = frame->min_x;
        fa.maxx = frame->max_x;
        fa.miny = frame->min_y;
        fa.maxy = frame->max_y;
        fa.log_scale = log_scale_factor;
        fa.cos_limit = viewing_cos_limit;
        fa.in_view = d_in_view;
        fa.px = m->o_f0.as<float>();
        fa.py = m->o_f1.as<float>();
        fa.pxr = m->o_f2.as<float>();
        fa.lvl = m->o_i.as<int>();
        fa.vcos = m->o_f3.as<float>();
        fa.skip = d_skip;
        fa.bad = d_bad;
        fa.n_in_view = d_cnt;
        if (M) hipLaunchKernelGGL(frustum_kernel, dim3((M + 255) / 256), dim3(256), 0, m->stream, fa);
        // SearchByProjection(F, vpLocalMapPoints, th) (1440-1453, ORBmatcher.cc:45-129)
        SbpLocalArgs a;
        if ((st = m->frame_device(frame, a.f))) return st;
        a.mp = SbpMps{M, d_in_view, d_bad, fa.px, fa.py, fa.pxr, fa.lvl, fa.vcos,
                      reinterpret_cast<const uint4*>(d_desc), d_nobs};
        a.scale = m->m_f4.as<float>();
        a.th = th;
        a.nlevels = frame->nlevels;
        a.status = d_status;
        // candidates without a host round trip: the fill is bounded by the current capacity
        // (16 per point to start); the total is checked after the first greedy batch and the
        // call is redone once with the exact capacity if it did not fit
        const size_t cap = std::max(m->cand.bytes / sizeof(int2), (size_t)16 * std::max(M, 1));
        if ((st = m->cand.ensure(cap * sizeof(int2)))) return st;
        if ((st = m->cnt.ensure(std::max(M, 1) * sizeof(int)))) return st;
        if ((st = m->off.ensure((M + 1) * sizeof(int)))) return st;
        a.cnt = m->cnt.as<int>();
        a.off = m->off.as<int>();
        a.cand = m->cand.as<int2>();
        a.cand_cap = (long long)cap;
        const int qb = std::max(1, (M + 3) / 4);  // one wave per map point
        hipLaunchKernelGGL(sbp_local_cand_kernel<0>, dim3(qb), dim3(256), 0, m->stream, a);
        hipLaunchKernelGGL(scan_kernel, dim3(1), dim3(1024), 0, m->stream, m->cnt.as<int>(), M, m->off.as<int>());
        hipLaunchKernelGGL(sbp_local_cand_kernel<1>, dim3(qb), dim3(256), 0, m->stream, a);
        int total = 0;
        ORBFE_HIP(hipMemcpyAsync(&total, m->off.as<int>() + M, sizeof(int), hipMemcpyDeviceToHost, m->stream));
        GreedyArgs g{};
        g.m = M;
        g.nkp = N;
        g.mode = kGreedyLocal;
        g.nnratio = nnratio;
        g.off = m->off.as<int>();
        g.cand = m->cand.as<int2>();
        g.nobs = d_nobs;
        g.fmp0 = g.fmp = d_frame_mp;
        g.fobs0 = g.fobs = d_frame_mp_obs;
        g.ids = d_mp_ids;
        // synchronizes per batch of rounds; ORBFE_ERR_CAPACITY (nothing written yet) when the
        // candidates did not fit: grow to the exact total and run again
        st = m->greedy(g, 8, &total, cap);
        if (st == ORBFE_ERR_CAPACITY && !retried) {
            if ((st = m->cand.ensure((size_t)total * sizeof(int2)))) return st;
            retried = true;
            ++m->capacity_retries;
            return attempt();
        }
        if (st) return st;
        int host[3] = {0, 0, 0};
        ORBFE_HIP(hipMemcpyAsync(host, m->scal.p, sizeof(host), hipMemcpyDeviceToHost, m->stream));
        ORBFE_HIP(hipStreamSynchronize(m->stream));
        counts[0] = host[0];  // nmatches
        counts[1] = host[1];  // nToMatch
        return host[2] ? host[2] : ORBFE_OK;
        };
        return attempt();
    });
}

int orbfe_search_by_projection_local_device(orbfe_matcher* m, float nnratio,
                                            const orbfe_frame_view* frame, int32_t* d_frame_mp,
                                            int32_t* d_frame_mp_obs,
                                            const orbfe_mappoint_view* d_mps,
                                            const int32_t* d_mp_ids, float th, int32_t* nmatches) {
    if (!frame_ok(frame) || !d_mps || d_mps->m < 0 || !nmatches ||
        (frame->n && (!d_frame_mp || !d_frame_mp_obs)))
        return ORBFE_ERR_ARG;
    const int M = d_mps->m;
    if (M && (!d_mps->track_in_view || !d_mps->is_bad || !d_mps->proj_x || !d_mps->proj_y ||
              !d_mps->proj_xr || !d_mps->pred_level || !d_mps->view_cos || !d_mps->desc ||
              !d_mps->n_obs))
        return ORBFE_ERR_ARG;
    return guarded(m, [&]() {
        int st;
        const int N = frame->n;
        if ((st = m->scal.ensure(64))) return st;
        // fast path (sbp_local_fast on the resident isInFrustum outputs; the scale factors go
        // as kernel arguments), else / on its fallback the CSR path below
        if (N <= kSbpFixKp && frame->nlevels <= kMaxLevels && M > 0 &&
            !std::getenv("ORBFE_SBP_DEVICE_CSR")) {
            const SbpMps mp{M, d_mps->track_in_view, d_mps->is_bad, d_mps->proj_x, d_mps->proj_y,
                            d_mps->proj_xr, d_mps->pred_level, d_mps->view_cos,
                            reinterpret_cast<const uint4*>(d_mps->desc), d_mps->n_obs};
            int host[6];
            if ((st = sbp_local_fast<true>(m, frame, FrustumArgs{}, mp, nnratio, th, d_mps->n_obs,
                                           d_mp_ids, d_frame_mp, d_frame_mp_obs, host)))
                return st;
            if (!host[3] && host[4] == 0) {  // no overflow, converged
                *nmatches = host[0];
                return host[2] ? host[2] : ORBFE_OK;
            }
        }
        // the CSR path reads the scale factors from device memory
        if ((st = m->m_f4.ensure(std::max<size_t>(16, (size_t)frame->nlevels * 4)))) return st;
        ORBFE_HIP(hipMemcpyAsync(m->m_f4.p, frame->scale_factors, (size_t)frame->nlevels * 4,
                                 hipMemcpyHostToDevice, m->stream));
        bool retried = false;
        std::function<int()> attempt = [&]() -> int {
            ORBFE_HIP(hipMemsetAsync(m->scal.p, 0, 16, m->stream));
            SbpLocalArgs a;
            if ((st = m->frame_device(frame, a.f))) return st;  // AssignFeaturesToGrid
            a.mp = SbpMps{M, d_mps->track_in_view, d_mps->is_bad, d_mps->proj_x, d_mps->proj_y,
                          d_mps->proj_xr, d_mps->pred_level, d_mps->view_cos,
                          reinterpret_cast<const uint4*>(d_mps->desc), d_mps->n_obs};
            a.scale = m->m_f4.as<float>();
            a.th = th;
            a.nlevels = frame->nlevels;
            a.status = m->scal.as<int>() + 2;  // a predicted level outside the pyramid
            // count -> scan -> fill bounded by the grow-only capacity; checked after the first
            // batch of greedy rounds, redone once with the exact total if it did not fit
            const size_t cap = std::max(m->cand.bytes / sizeof(int2), (size_t)16 * std::max(M, 1));
            if ((st = m->cand.ensure(cap * sizeof(int2)))) return st;
            if ((st = m->cnt.ensure(std::max(M, 1) * sizeof(int)))) return st;
            if ((st = m->off.ensure((M + 1) * sizeof(int)))) return st;
            a.cnt = m->cnt.as<int>();
            a.off = m->off.as<int>();
            a.cand = m->cand.as<int2>();
            a.cand_cap = (long long)cap;
            const int qb = std::max(1, (M + 3) / 4);  // one wave per map point
            hipLaunchKernelGGL(sbp_local_cand_kernel<0>, dim3(qb), dim3(256), 0, m->stream, a);
            hipLaunchKernelGGL(scan_kernel, dim3(1), dim3(1024), 0, m->stream, m->cnt.as<int>(), M, m->off.as<int>());
            hipLaunchKernelGGL(sbp_local_cand_kernel<1>, dim3(qb), dim3(256), 0, m->stream, a);
            int total = 0;
            ORBFE_HIP(hipMemcpyAsync(&total, m->off.as<int>() + M, sizeof(int), hipMemcpyDeviceToHost, m->stream));
            GreedyArgs g{};
            g.m = M;
            g.nkp = N;
            g.mode = kGreedyLocal;
            g.nnratio = nnratio;
            g.off = m->off.as<int>();
            g.cand = m->cand.as<int2>();
            g.nobs = d_mps->n_obs;
            g.fmp0 = g.fmp = d_frame_mp;
            g.fobs0 = g.fobs = d_frame_mp_obs;
            g.ids = d_mp_ids;
            st = m->greedy(g, 8, &total, cap);
            if (st == ORBFE_ERR_CAPACITY && !retried) {
                if ((st = m->cand.ensure((size_t)total * sizeof(int2)))) return st;
                retried = true;
                ++m->capacity_retries;
                return attempt();
            }
            if (st) return st;
            int host[3] = {0, 0, 0};
            ORBFE_HIP(hipMemcpyAsync(host, m->scal.p, sizeof(host), hipMemcpyDeviceToHost, m->stream));
            ORBFE_HIP(hipStreamSynchronize(m->stream));
            *nmatches = host[0];
            return host[2] ? host[2] : ORBFE_OK;
        };
        return attempt();
    });
}

int orbfe_features_in_area(orbfe_matcher* m, const orbfe_frame_view* f, int nq, const float* x,
                           const float* y, const float* r, const int32_t* min_level,
                           const int32_t* max_level, int wave, int32_t* off, int32_t* items,
                           int items_cap) {
    if (!frame_ok(f) || nq < 0 || !off || items_cap < 0 || (items_cap && !items) ||
        (nq && (!x || !y || !r || !min_level || !max_level)))
        return ORBFE_ERR_ARG;
    return guarded(m, [&]() {
        int st;
        FiaArgs a;
        if ((st = m->up(m->m_f0, x, (size_t)nq * 4))) return st;
        if ((st = m->up(m->m_f1, y, (size_t)nq * 4))) return st;
        if ((st = m->up(m->m_f2, r, (size_t)nq * 4))) return st;
        if ((st = m->up(m->m_i0, min_level, (size_t)nq * 4))) return st;
        if ((st = m->up(m->m_i1, max_level, (size_t)nq * 4))) return st;
        if ((st = m->frame(f, false, a.f))) return st;  // AssignFeaturesToGrid (flushes)
        if ((st = m->cnt.ensure(std::max(nq, 1) * sizeof(int)))) return st;
        if ((st = m->off.ensure((size_t)(nq + 1) * sizeof(int)))) return st;
        a.nq = nq;
        a.x = m->m_f0.as<float>();
        a.y = m->m_f1.as<float>();
        a.r = m->m_f2.as<float>();
        a.lo = m->m_i0.as<int>();
        a.hi = m->m_i1.as<int>();
        a.cnt = m->cnt.as<int>();
        a.off = m->off.as<int>();
        const int blocks = std::max(1, wave ? (nq + 3) / 4 : (nq + 255) / 256);
        if (wave) hipLaunchKernelGGL(fia_wave_kernel<false>, dim3(blocks), dim3(256), 0, m->stream, a);
        else hipLaunchKernelGGL(fia_thread_kernel<false>, dim3(blocks), dim3(256), 0, m->stream, a);
        hipLaunchKernelGGL(scan_kernel, dim3(1), dim3(1024), 0, m->stream, m->cnt.as<int>(), nq,
                           m->off.as<int>());
        ORBFE_HIP(hipGetLastError());
        if ((st = m->down(off, m->off, (size_t)(nq + 1) * 4))) return st;
        if ((st = m->sync())) return st;
        const int total = off[nq];
        if (total > items_cap) return ORBFE_ERR_CAPACITY;
        if ((st = m->s1.ensure((size_t)std::max(total, 1) * sizeof(int)))) return st;
        a.items = m->s1.as<int>();
        if (wave) hipLaunchKernelGGL(fia_wave_kernel<true>, dim3(blocks), dim3(256), 0, m->stream, a);
        else hipLaunchKernelGGL(fia_thread_kernel<true>, dim3(blocks), dim3(256), 0, m->stream, a);
        ORBFE_HIP(hipGetLastError());
        m->begin();
        if ((st = m->down(items, m->s1, (size_t)total * 4))) return st;
        return m->sync();
    });
}

int orbfe_matcher_capacity_retries(const orbfe_matcher* m) {
    return m ? m->capacity_retries : ORBFE_ERR_ARG;
}

int orbfe_matcher_last_rounds(const orbfe_matcher* m) {
    if (!m) return ORBFE_ERR_ARG;
    if (!m->rounds_on_device) return m->last_rounds;
    int r = 0;
    DeviceGuard dg(m->device);
    if (hipStreamSynchronize(m->stream) != hipSuccess ||
        hipMemcpy(&r, m->g_chg.p, sizeof(int), hipMemcpyDeviceToHost) != hipSuccess)
        return ORBFE_ERR_HIP;
    return r;
}

int orbfe_is_in_frustum(orbfe_matcher* m, int n, const float* xyz, const float* normal,
                        const float* min_dist, const float* max_dist, const float* tcw,
                        const orbfe_camera* cam, float min_x, float max_x, float min_y,
                        float max_y, float log_scale_factor, float viewing_cos_limit,
                        uint8_t* in_view, float* proj_x, float* proj_y, float* proj_xr,
                        int32_t* pred_level, float* view_cos) {
    if (n < 0 || !tcw || !cam ||
        (n && (!xyz || !normal || !min_dist || !max_dist || !in_view || !proj_x || !proj_y ||
               !proj_xr || !pred_level || !view_cos)))
        return ORBFE_ERR_ARG;
    if (n == 0) return m ? ORBFE_OK : ORBFE_ERR_ARG;
    return guarded(m, [&]() {
        int st;
        if ((st = m->up(m->m_f0, xyz, (size_t)n * 12))) return st;
        if ((st = m->up(m->m_f1, normal, (size_t)n * 12))) return st;
        if ((st = m->up(m->m_f2, min_dist, (size_t)n * 4))) return st;
        if ((st = m->up(m->m_f3, max_dist, (size_t)n * 4))) return st;
        for (DevBuf* b : {&m->o_f0, &m->o_f1, &m->o_f2, &m->o_f3, &m->o_i})
            if ((st = b->ensure((size_t)n * 4))) return st;
        if ((st = m->o_u.ensure(n))) return st;
        // outputs of map points that fail a check keep their previous scratch values
        if ((st = m->up(m->o_f0, proj_x, (size_t)n * 4))) return st;
        if ((st = m->up(m->o_f1, proj_y, (size_t)n * 4))) return st;
        if ((st = m->up(m->o_f2, proj_xr, (size_t)n * 4))) return st;
        if ((st = m->up(m->o_f3, view_cos, (size_t)n * 4))) return st;
        if ((st = m->up(m->o_i, pred_level, (size_t)n * 4))) return st;
        FrustumArgs a;
        a.n = n;
        a.xyz = m->m_f0.as<float>();
        a.normal = m->m_f1.as<float>();
        a.mind = m->m_f2.as<float>();
        a.maxd = m->m_f3.as<float>();
        std::memcpy(a.T, tcw, sizeof(a.T));
        camera_center(tcw, a.ow);
        a.fx = cam->fx;
        a.fy = cam->fy;
        a.cx = cam->cx;
        a.cy = cam->cy;
        a.bf = cam->bf;
        a.minx = min_x;
        a.maxx = max_x;
        a.miny = min_y;
        a.maxy = max_y;
        a.log_scale = log_scale_factor;
        a.cos_limit = viewing_cos_limit;
        a.in_view = m->o_u.as<uint8_t>();
        a.px = m->o_f0.as<float>();
        a.py = m->o_f1.as<float>();
        a.pxr = m->o_f2.as<float>();
        a.lvl = m->o_i.as<int>();
        a.vcos = m->o_f3.as<float>();
        a.skip = a.bad = nullptr;
        a.n_in_view = nullptr;
        if ((st = m->flush())) return st;
        hipLaunchKernelGGL(frustum_kernel, dim3((n + 255) / 256), dim3(256), 0, m->stream, a);
        ORBFE_HIP(hipGetLastError());
        if ((st = m->down(in_view, m->o_u, n))) return st;
        if ((st = m->down(proj_x, m->o_f0, (size_t)n * 4))) return st;
        if ((st = m->down(proj_y, m->o_f1, (size_t)n * 4))) return st;
        if ((st = m->down(proj_xr, m->o_f2, (size_t)n * 4))) return st;
        if ((st = m->down(pred_level, m->o_i, (size_t)n * 4))) return st;
        if ((st = m->down(view_cos, m->o_f3, (size_t)n * 4))) return st;
        return m->sync();
    });
}

}  // extern "C"
