// orbfe_api.hip — host orchestration and the C ABI of the extractor (include/orbfe.h).
// Replaces ORBextractor's public surface (ORBextractor.h:56-90); see the header for the
// per-function citations.  No CPU compute path exists: every result comes from the kernels.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <algorithm>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <new>
#include <vector>

#include "../../include/orbfe.h"
#include "orbfe_internal.hpp"

namespace orbfe {

#define ORBFE_HIP(call)                                                                    \
    do {                                                                                   \
        hipError_t e_ = (call);                                                            \
        if (e_ != hipSuccess) {                                                            \
            fprintf(stderr, "orbfe: %s failed: %s (%s:%d)\n", #call, hipGetErrorString(e_), \
                    __FILE__, __LINE__);                                                   \
            return e_ == hipErrorOutOfMemory ? ORBFE_ERR_NOMEM : ORBFE_ERR_HIP;            \
        }                                                                                  \
    } while (0)

// Device buffer that only grows.
struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    int ensure(size_t n) {
        if (n <= bytes) return ORBFE_OK;
        if (p) hipFree(p);
        p = nullptr;
        bytes = 0;
        if (hipMalloc(&p, n) != hipSuccess) return ORBFE_ERR_NOMEM;
        bytes = n;
        return ORBFE_OK;
    }
    template <class T> T* as() const { return static_cast<T*>(p); }
    void release() {
        if (p) hipFree(p);
        p = nullptr;
        bytes = 0;
    }
};

// Bytes per pixel of an ORBFE_PIX_* format (0 for an unknown format).
int pix_channels(int pix) {
    switch (pix) {
        case ORBFE_PIX_GRAY: return 1;
        case ORBFE_PIX_RGB: case ORBFE_PIX_BGR: return 3;
        case ORBFE_PIX_RGBA: case ORBFE_PIX_BGRA: return 4;
        default: return 0;
    }
}

// Returns ORBFE_OK when `device` is a usable gfx950 agent (the only target this library is
// built for); the library has no CPU fallback.
int check_device(int device) {
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) return ORBFE_ERR_HIP;
    if (device < 0 || device >= count) return ORBFE_ERR_ARG;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) return ORBFE_ERR_HIP;
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
        fprintf(stderr, "orbfe: device %d is %s, this build targets gfx950 only\n", device,
                prop.gcnArchName);
        return ORBFE_ERR_HIP;
    }
    return ORBFE_OK;
}

// Start/stop events bound to kernel dispatches (hipExtLaunchKernel records them from the
// dispatch packet itself, so a pair brackets exactly one kernel), read by orbfe_profile_read.
struct Profiler {
    bool on = false;
    unsigned mask = ~0u;  // stages that get events (orbfe_profile)
    unsigned run_mask = ~0u;  // stages whose launches run (orbfe_debug_replay: one stage alone)
    std::vector<hipEvent_t> a, b;
    std::vector<int> kind;
    size_t used = 0;
    // Returns the event pair for the next launch of stage k (nullptrs when off).
    void slot(int k, hipEvent_t* e0, hipEvent_t* e1) {
        *e0 = *e1 = nullptr;
        if (!on || !((mask >> k) & 1u)) return;
        if (used == a.size()) {
            hipEvent_t x, y;
            if (hipEventCreate(&x) != hipSuccess) return;
            if (hipEventCreate(&y) != hipSuccess) { hipEventDestroy(x); return; }
            a.push_back(x);
            b.push_back(y);
            kind.push_back(k);
        }
        kind[used] = k;
        *e0 = a[used];
        *e1 = b[used];
        ++used;
    }
    void release() {
        for (hipEvent_t e : a) hipEventDestroy(e);
        for (hipEvent_t e : b) hipEventDestroy(e);
        a.clear();
        b.clear();
        kind.clear();
        used = 0;
    }
};

// Kernel launch through hipExtLaunchKernelGGL with the stage's profiling events.
#define ORBFE_LAUNCH(prof, stage, kernel, grid, block, shmem, stream, ...)                 \
    do {                                                                                   \
        if (!(((prof).run_mask >> (stage)) & 1u)) break;                                   \
        hipEvent_t e0_, e1_;                                                               \
        (prof).slot(stage, &e0_, &e1_);                                                    \
        hipExtLaunchKernelGGL(kernel, grid, block, shmem, stream, e0_, e1_, 0, __VA_ARGS__); \
    } while (0)

}  // namespace orbfe

using namespace orbfe;

struct orbfe_extractor {
    int device = 0;
    hipStream_t own = nullptr, stream = nullptr;
    HostTables tab{};
    int arith = ORBFE_ARITH_X86_SIMD;  // orbfe_set_arithmetic (default: the reference's x86-64 build)
    bool x86() const { return arith == ORBFE_ARITH_X86_SIMD; }
    Plan plan;
    bool planned = false;
    int frames_cap = 0;
    DevBuf cells, xtab, ytab, bslot, ptab;
    DevBuf pyr, blur, cell_cnt, cell_keys, keys, act, oct_out, oct_cnt, oct_ord, level_keys;
    DevBuf out_kps, out_desc, out_n;  // staging for the host-pointer entry points
    DevBuf lk_snap;                   // orbfe_debug_replay: one FAST's per-level key totals
    DevBuf stage, rects;              // host colour frames / rectangle masks (level-0 inputs)
    DevBuf st_off, st_items, st_sad, st_status;           // stereo workspaces (left handle)
    DevBuf st_ur;  // stereo host path: u_right | depth | status, copied back in one piece
    std::vector<int4> h_rects;
    // last run, for the probes
    int last_n = 0;
    LevelPtr last_pyr[kMaxLevels] = {};
    Profiler prof;
    std::vector<orbfe_keypoint> h_kps;
    std::vector<uint8_t> h_desc;
    // the last single-frame host call's outputs where the call left them (orbfe_staged_outputs)
    const orbfe_keypoint* staged_kps = nullptr;
    const uint8_t* staged_desc = nullptr;
    int staged_n = 0;
    std::vector<int32_t> h_n;

    // Single-frame host path (Frame::ExtractORB's per-frame call): pinned staging and the whole
    // H2D copy + pipeline + D2H sequence captured once into a HIP graph per frame size and
    // replayed, so a call costs one graph launch instead of ~15 kernel launches and pageable
    // copies.  Rebuilt when the plan or any buffer it captured changes.
    struct Pinned {
        uint8_t* p = nullptr;
        uint8_t* d = nullptr;  // device-mapped address (kernels read / write it over PCIe)
        size_t bytes = 0;
        int ensure(size_t n) {
            if (n <= bytes) return ORBFE_OK;
            if (p) hipHostFree(p);
            p = d = nullptr;
            bytes = 0;
            if (hipHostMalloc(reinterpret_cast<void**>(&p), n, hipHostMallocDefault) != hipSuccess)
                return ORBFE_ERR_NOMEM;
            void* dq = nullptr;
            d = hipHostGetDevicePointer(&dq, p, 0) == hipSuccess ? static_cast<uint8_t*>(dq) : nullptr;
            bytes = n;
            return ORBFE_OK;
        }
        void release() {
            if (p) hipHostFree(p);
            p = d = nullptr;
            bytes = 0;
        }
    };
    // pin_in: the copy staging of orbfe_extract (rewritten by every copying call); pin_user: the
    // buffer orbfe_input_buffer hands out — only orbfe_input_buffer (at a larger size) and
    // orbfe_destroy reallocate it and no copying call writes it, so the caller's pointer and the
    // frame staged in it stay valid across orbfe_extract calls of any size.
    Pinned pin_in, pin_user, pin_kps, pin_desc, pin_n;
    // orbfe_compute_stereo_matches: the pair's keypoints, descriptors and counts in one pinned
    // block (one H2D copy into st_in), the outputs back into it (st_pin)
    Pinned st_pin;
    DevBuf st_in;
    // Every buffer the capture embeds is either in g1_key (outputs, pinned staging) or is a
    // plan / workspace buffer: set_plan and a growing ensure_frames drop the graphs.  One graph
    // per input source ([0] copy staging, [1] the handed-out buffer), so callers alternating the
    // two forms do not recapture.
    hipGraphExec_t g1[2] = {nullptr, nullptr};
    const void* g1_key[2][11] = {};  // the buffers, plan and staging mode each graph was captured with
    // K4 fused into K5 per keypoint window (default), or its own pass over every level with
    // K5 reading the blurred levels (ORBFE_PREBLUR=1: describe 0.30 -> 0.20 ms per 256 frames,
    // but the pass costs 0.19 ms; profiles/r02/experiments/preblur.json)
    bool fused_blur = std::getenv("ORBFE_PREBLUR") == nullptr;
    // ORBFE_PREBLUR with ORBFE_PRE_MASK=<hex>: the describe reads blurred windows only for the
    // levels in the mask and blurs the others per keypoint (experiments)
    uint32_t pre_mask_env = std::getenv("ORBFE_PRE_MASK") ? (uint32_t)std::strtoul(std::getenv("ORBFE_PRE_MASK"), nullptr, 16) : 0xffffffffu;
    // the pyramid in one launch (pyramid_kernel); ORBFE_PYR=0: per-level resize launches + the
    // one-workgroup tail
    bool use_pyr = !(std::getenv("ORBFE_PYR") && std::strcmp(std::getenv("ORBFE_PYR"), "0") == 0);
    // ORBFE_PYR=2: the band kernel even where its plan recomputes many seam rows (tests, A/B)
    bool force_pyr = std::getenv("ORBFE_PYR") && std::strcmp(std::getenv("ORBFE_PYR"), "2") == 0;
    // ORBFE_ZERO_COPY=0: the single-frame host call copies its frame in and its outputs out
    // with DMA copies instead of kernels reading / writing the pinned buffers
    bool zero_copy = !(std::getenv("ORBFE_ZERO_COPY") && std::strcmp(std::getenv("ORBFE_ZERO_COPY"), "0") == 0);
    // run(): the pyramid kernel reads level 0 from l0_stage and writes it to the slab level 0
    LevelPtr l0_stage{};
    bool l0_from_stage = false;
    // ORBFE_PYR_SMALL_BELOW (A/B): batches below it take the small-batch band plans (thin bands)
    int pyr_small_below = std::getenv("ORBFE_PYR_SMALL_BELOW") ? std::atoi(std::getenv("ORBFE_PYR_SMALL_BELOW")) : kTailMinFrames;
    // Batches of >= pyr_small_below frames take the per-level kernels (resize2 pairs + the
    // one-workgroup tail) even where the band plan is the faster path alone: under the bench's
    // two sub-batch streams the band kernel's 1024-thread, 80 KB workgroups find few CUs free
    // beside the other stream's FAST / describe waves (a 256-frame launch stretched to 0.70 ms
    // against 0.154 alone), the per-level kernels' 256-thread workgroups co-reside: c3 365.4 K
    // -> 368.7 K frames/s (profiles/r05/pyramid_overlap/).  ORBFE_PYR_BATCH=band restores it.
    bool pyr_batch_band = std::getenv("ORBFE_PYR_BATCH") && std::strcmp(std::getenv("ORBFE_PYR_BATCH"), "band") == 0;
    bool band_path(int n) const {  // run() makes the pyramid with pyramid_kernel for n frames
        const int which = n >= pyr_small_below ? 0 : 1;
        if (which == 0 && !pyr_batch_band && !force_pyr) return false;
        return plan.pyr_ok && (plan.pyr_use[which] || force_pyr) && use_pyr && plan.geo.nlevels >= 2;
    }
    bool pyr_path(int n) const { return band_path(n); }  // one launch
    // ORBFE_RS2=0: one resize launch per level where resize2_kernel would take two (A/B)
    bool use_rs2 = !(std::getenv("ORBFE_RS2") && std::strcmp(std::getenv("ORBFE_RS2"), "0") == 0);
    // ORBFE_RESIZE_TABLE=0: resize_kernel's horizontal pass by byte gathers (A/B)
    bool table_off = std::getenv("ORBFE_RESIZE_TABLE") && std::strcmp(std::getenv("ORBFE_RESIZE_TABLE"), "0") == 0;
    // ORBFE_DESC_MFMA=0: describe blurs its raw windows on the VALU instead of the matrix cores
    bool desc_mfma = !(std::getenv("ORBFE_DESC_MFMA") && std::strcmp(std::getenv("ORBFE_DESC_MFMA"), "0") == 0);
    // ORBFE_DESC_STRIDE=0: describe waves take consecutive slots in batches too (A/B)
    bool desc_stride = !(std::getenv("ORBFE_DESC_STRIDE") && std::strcmp(std::getenv("ORBFE_DESC_STRIDE"), "0") == 0);
    // ORBFE_DESC_ORDER=0: strided describe waves take the oct-tree output order (A/B); 2: the
    // band order at every frame size
    bool desc_order = !(std::getenv("ORBFE_DESC_ORDER") && std::strcmp(std::getenv("ORBFE_DESC_ORDER"), "0") == 0);
    bool desc_order_all = std::getenv("ORBFE_DESC_ORDER") && std::strcmp(std::getenv("ORBFE_DESC_ORDER"), "2") == 0;
    int num_cus = 256;  // compute units of the device (launch-shape choices)
    // ORBFE_OCT_SMALL=0: small batches keep the 256-thread oct-tree (A/B)
    bool oct_small = !(std::getenv("ORBFE_OCT_SMALL") && std::strcmp(std::getenv("ORBFE_OCT_SMALL"), "0") == 0);
    int desc_g16 = std::getenv("ORBFE_DESC_G16") ? std::atoi(std::getenv("ORBFE_DESC_G16")) : 0;
    bool graph_broken = std::getenv("ORBFE_NO_GRAPH") != nullptr;  // capture failed once (or
                                 // disabled for A/B runs): keep to the launch path

    void drop_graph() {
        for (hipGraphExec_t& g : g1) {
            if (g) hipGraphExecDestroy(g);
            g = nullptr;
        }
    }

    // ORBFE_OK with *done = true when the graph path ran; *done = false to take the plain path.
    int run_single_graph(const uint8_t* img, int w, int h, size_t stride, bool* done) {
        *done = false;
        // (the legacy default stream cannot be captured: plain launches there)
        if (graph_broken || prof.on || stream == hipStreamLegacy || stage_mask != ~0u) return ORBFE_OK;
        int st;
        if ((st = set_plan(w, h))) return st;
        if ((st = ensure_frames(1))) return st;
        const int cap = kp_capacity();
        if ((st = out_kps.ensure((size_t)cap * sizeof(orbfe_keypoint)))) return st;
        if ((st = out_desc.ensure((size_t)cap * 32))) return st;
        if ((st = out_n.ensure(sizeof(int32_t)))) return st;
        const int gi = img == pin_user.p ? 1 : 0;  // staged: the GPU reads the handed-out buffer
        Pinned& src = gi ? pin_user : pin_in;
        if (!gi && (st = pin_in.ensure((size_t)w * h))) return st;
        if ((st = pin_kps.ensure((size_t)cap * sizeof(orbfe_keypoint)))) return st;
        if ((st = pin_desc.ensure((size_t)cap * 32))) return st;
        if ((st = pin_n.ensure(sizeof(int32_t)))) return st;
        // every buffer the capture can embed (the zero-copy outputs write pin_kps / pin_desc /
        // pin_n through their device mappings) and the staging mode
        const void* key[11] = {pyr.p, out_kps.p, out_desc.p, out_n.p, src.p, pin_kps.p,
                               pin_desc.p, pin_n.p,
                               reinterpret_cast<const void*>((uintptr_t)w << 32 | (uint32_t)h),
                               reinterpret_cast<const void*>((uintptr_t)frames_cap),
                               reinterpret_cast<const void*>((uintptr_t)zero_copy)};
        if (g1[gi] && std::memcmp(key, g1_key[gi], sizeof(key)) != 0) {
            hipGraphExecDestroy(g1[gi]);
            g1[gi] = nullptr;
        }
        const Plan& g = plan;
        const LevelGeo& l0 = g.geo.lv[0];
        if (!g1[gi]) {
            hipGraph_t graph = nullptr;
            if (hipStreamBeginCapture(stream, hipStreamCaptureModeThreadLocal) != hipSuccess) {
                graph_broken = true;
                return ORBFE_OK;
            }
            // zero-copy: the pyramid kernel reads the frame from the pinned staging buffer and
            // writes level 0 into the slab as it goes (no H2D copy), describe writes keypoints,
            // descriptors and the count straight into the pinned outputs (no D2H copies)
            const bool zc_out = zero_copy && pin_kps.d && pin_desc.d && pin_n.d;
            const bool zc_in = zero_copy && src.d && pyr_path(1);
            LevelPtr lp0{pyr.as<uint8_t>() + l0.off, g.slab, l0.pitch};
            bool ok = true;
            if (zc_in) {
                l0_stage = LevelPtr{src.d, (long long)w * h, w};
                l0_from_stage = true;
            } else {
                ok = hipMemcpy2DAsync(pyr.as<uint8_t>() + l0.off, l0.pitch, src.p, w, w, h,
                                      hipMemcpyHostToDevice, stream) == hipSuccess;
            }
            if (zc_out) {
                ok = ok && run(1, lp0, reinterpret_cast<orbfe_keypoint*>(pin_kps.d), cap, pin_desc.d,
                               reinterpret_cast<int32_t*>(pin_n.d)) == ORBFE_OK;
            } else {
                ok = ok && run(1, lp0, out_kps.as<orbfe_keypoint>(), cap, out_desc.as<uint8_t>(),
                               out_n.as<int32_t>()) == ORBFE_OK;
                ok = ok && hipMemcpyAsync(pin_n.p, out_n.p, sizeof(int32_t), hipMemcpyDeviceToHost,
                                          stream) == hipSuccess;
                ok = ok && hipMemcpyAsync(pin_kps.p, out_kps.p, (size_t)cap * sizeof(orbfe_keypoint),
                                          hipMemcpyDeviceToHost, stream) == hipSuccess;
                ok = ok && hipMemcpyAsync(pin_desc.p, out_desc.p, (size_t)cap * 32,
                                          hipMemcpyDeviceToHost, stream) == hipSuccess;
            }
            l0_from_stage = false;
            const bool ended = hipStreamEndCapture(stream, &graph) == hipSuccess;
            ok = ok && ended && graph &&
                 hipGraphInstantiate(&g1[gi], graph, nullptr, nullptr, 0) == hipSuccess;
            if (graph) hipGraphDestroy(graph);
            (void)hipGetLastError();
            if (!ok) {
                g1[gi] = nullptr;
                graph_broken = true;
                return ORBFE_OK;
            }
            std::memcpy(g1_key[gi], key, sizeof(key));
        }
        if (gi) {
            // staged (orbfe_input_buffer): the caller wrote the frame into pin_user already
        } else if (stride == (size_t)w) {
            std::memcpy(pin_in.p, img, (size_t)w * h);
        } else {
            for (int r = 0; r < h; ++r) std::memcpy(pin_in.p + (size_t)r * w, img + r * stride, w);
        }
        ORBFE_HIP(hipGraphLaunch(g1[gi], stream));
        ORBFE_HIP(hipStreamSynchronize(stream));
        last_n = 1;
        *done = true;
        return ORBFE_OK;
    }

    int set_plan(int w, int h) {
        if (planned && plan.w == w && plan.h == h) return ORBFE_OK;
        Plan g;
        int st = plan_geometry(tab, w, h, g);
        if (st != ORBFE_OK) return st;
        if ((st = cells.ensure(std::max<size_t>(1, g.cells.size()) * sizeof(CellDesc)))) return st;
        if ((st = xtab.ensure(std::max<size_t>(1, g.xtab.size()) * sizeof(int)))) return st;
        if ((st = ytab.ensure(std::max<size_t>(1, g.ytab.size()) * sizeof(int)))) return st;
        if ((st = bslot.ensure(kBlurFragBytes + g.bitems.size() * sizeof(uint32_t)))) return st;
        if ((st = ptab.ensure(std::max<size_t>(16, g.ptab.size() * sizeof(uint32_t))))) return st;
        if (!g.ptab.empty())
            ORBFE_HIP(hipMemcpyAsync(ptab.p, g.ptab.data(), g.ptab.size() * sizeof(uint32_t),
                                     hipMemcpyHostToDevice, stream));
        if (g.pyr_ok) {  // dynamic LDS above 64 KB must be allowed per kernel
            const int mx = (int)std::max(g.pyr_lds[0], g.pyr_lds[1]);
            hipFuncSetAttribute(reinterpret_cast<const void*>(&pyramid_kernel<false>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, mx);
            hipFuncSetAttribute(reinterpret_cast<const void*>(&pyramid_kernel<true>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, mx);
        }
        ORBFE_HIP(hipMemcpyAsync(cells.p, g.cells.data(), g.cells.size() * sizeof(CellDesc),
                                 hipMemcpyHostToDevice, stream));
        ORBFE_HIP(hipMemcpyAsync(xtab.p, g.xtab.data(), g.xtab.size() * sizeof(int),
                                 hipMemcpyHostToDevice, stream));
        ORBFE_HIP(hipMemcpyAsync(ytab.p, g.ytab.data(), g.ytab.size() * sizeof(int),
                                 hipMemcpyHostToDevice, stream));
        // blur_mfma_kernel: its constant fragments, then its work list
        std::vector<uint8_t> bb(kBlurFragBytes + g.bitems.size() * sizeof(uint32_t));
        blur_frags(tab.taps, bb.data());
        std::memcpy(bb.data() + kBlurFragBytes, g.bitems.data(), g.bitems.size() * sizeof(uint32_t));
        ORBFE_HIP(hipMemcpyAsync(bslot.p, bb.data(), bb.size(), hipMemcpyHostToDevice, stream));
        ORBFE_HIP(hipStreamSynchronize(stream));
        plan = std::move(g);
        planned = true;
        frames_cap = 0;  // workspace sizes depend on the plan
        drop_graph();    // the captured launches embed the old plan's tables and buffers
        return ORBFE_OK;
    }

    int kp_capacity() const { return plan.geo.out_total; }

    int ensure_frames(int n) {
        if (n <= frames_cap) return ORBFE_OK;
        const Plan& g = plan;
        int st;
        const size_t N = (size_t)n;
        if ((st = pyr.ensure(N * g.slab))) return st;
        if ((st = blur.ensure(N * g.slab))) return st;
        if ((st = cell_cnt.ensure(N * std::max<size_t>(1, g.cells.size()) * sizeof(int)))) return st;
        if ((st = cell_keys.ensure(N * std::max<long long>(1, g.cell_cap_total) * sizeof(uint32_t)))) return st;
        if ((st = keys.ensure(N * std::max<long long>(1, g.geo.key_total) * sizeof(uint32_t)))) return st;
        if ((st = act.ensure(N * 2 * std::max<long long>(1, g.geo.key_total) * sizeof(int4)))) return st;
        if ((st = oct_out.ensure(N * g.geo.out_total * sizeof(uint32_t)))) return st;
        if ((st = oct_cnt.ensure(N * g.geo.nlevels * sizeof(int)))) return st;
        if ((st = oct_ord.ensure(N * g.geo.out_total * sizeof(uint16_t)))) return st;
        if ((st = level_keys.ensure(N * kMaxLevels * sizeof(int)))) return st;
        // the FAST kernel adds into these, the oct-tree kernel reads and clears them
        ORBFE_HIP(hipMemsetAsync(level_keys.p, 0, N * kMaxLevels * sizeof(int), stream));
        frames_cap = n;
        drop_graph();  // any workspace above may have moved
        return ORBFE_OK;
    }

    // Runs the whole pipeline on `n` frames whose level 0 is described by `l0`.
    // the last run's arguments (orbfe_debug_replay)
    unsigned stage_mask = ~0u;  // orbfe_set_stage_mask: the stages extraction calls run
    struct LastRun { int n = 0; LevelPtr l0{}; orbfe_keypoint* kps = nullptr; int cap = 0; uint8_t* desc = nullptr; int32_t* nout = nullptr; } last_run;
    int run(int n, LevelPtr l0, orbfe_keypoint* d_kps, int kps_cap, uint8_t* d_desc,
            int32_t* d_n) {
        last_run = LastRun{n, l0, d_kps, kps_cap, d_desc, d_n};
        const Plan& g = plan;
        const int L = g.geo.nlevels;
        LevelPtr lp[kMaxLevels], bp[kMaxLevels];
        for (int l = 0; l < L; ++l) {
            const LevelGeo& lv = g.geo.lv[l];
            lp[l] = LevelPtr{pyr.as<uint8_t>() + lv.off, g.slab, lv.pitch};
            bp[l] = LevelPtr{blur.as<uint8_t>() + lv.off, g.slab, lv.pitch};
        }
        lp[0] = l0;
        // K1 cascaded pyramid: one launch per level, 128 x 32 tiles of every frame; the small
        // top levels (tail_start ..) in one K1b launch, a workgroup per frame
        // (a batch of a few frames would leave most CUs idle in the tail: per-level launches)
        const int ts = n >= kTailMinFrames ? std::min(g.tail_start, L) : L;
        // K1 as one launch (pyramid_kernel): every level of a band of every frame in LDS
        const int which = n >= pyr_small_below ? 0 : 1;
        const bool one_pyr = pyr_path(n);
        if (l0_from_stage && !one_pyr) return ORBFE_ERR_ARG;  // callers check pyr_path first
        if (one_pyr) {
            PyrArgs pa;
            pa.src = l0_from_stage ? l0_stage : lp[0];
            pa.l0_copy = l0_from_stage ? lp[0] : LevelPtr{nullptr, 0, 0};
            pa.nlevels = L;
            for (int l = 0; l < L; ++l) {
                pa.dst[l] = lp[l];
                pa.w[l] = g.geo.lv[l].w;
                pa.lp[l] = g.pyr_lp[l];
                pa.gtab[l] = ptab.as<uint4>() + g.gtab_off[l];
                pa.yt[l] = ytab.as<int>() + g.yoff[l];
                pa.simd_xb[l] = x86() ? sse2_body_resize(pa.w[l]) : 0;
            }
            pa.buf_b = g.pyr_bufb[which];
            pa.ybuf = g.pyr_ybuf[which];
            pa.ymax = g.pyr_ymax[which];
            pa.bands = reinterpret_cast<const int4*>(ptab.as<uint4>() + g.band_off[which]);
            if (x86())
                ORBFE_LAUNCH(prof, ORBFE_STAGE_RESIZE, pyramid_kernel<true>, dim3(g.nbands[which], n),
                             dim3(kPyrBlockSize), g.pyr_lds[which], stream, pa);
            else
                ORBFE_LAUNCH(prof, ORBFE_STAGE_RESIZE, pyramid_kernel<false>, dim3(g.nbands[which], n),
                             dim3(kPyrBlockSize), g.pyr_lds[which], stream, pa);
        }
        for (int l = 1; l < (one_pyr ? 1 : ts); ++l) {
            // levels l and l + 1 in one launch (resize2_kernel) where planned; ORBFE_RS2=0: one
            // launch per level
            if (use_rs2 && l + 1 < ts && g.rs2_ok[l] && !table_off) {
                Resize2Args r2;
                r2.src = lp[l - 1];
                r2.mid = lp[l];
                r2.dst = lp[l + 1];
                r2.sw = g.geo.lv[l - 1].w;
                r2.mw = g.geo.lv[l].w;
                r2.dw = g.geo.lv[l + 1].w;
                r2.dh = g.geo.lv[l + 1].h;
                r2.tiles_x = g.rs2_tiles_x[l];
                r2.tiles = reinterpret_cast<const int4*>(ptab.as<uint4>() + g.rs2_off[l]);
                r2.yt_m = ytab.as<int>() + g.yoff[l];
                r2.xt_m = xtab.as<int>() + g.xoff[l];
                r2.yt_d = ytab.as<int>() + g.yoff[l + 1];
                r2.xt_d = xtab.as<int>() + g.xoff[l + 1];
                r2.gtab_m = ptab.as<uint4>() + g.gtab_off[l];
                r2.gtab_d = ptab.as<uint4>() + g.gtab_off[l + 1];
                r2.pa = g.rs2_pa[l];
                r2.pb = g.rs2_pb[l];
                r2.bofs = g.rs2_bofs[l];
                r2.xb_m = x86() ? sse2_body_resize(r2.mw) : 0;
                r2.xb_d = x86() ? sse2_body_resize(r2.dw) : 0;
                if (x86())
                    ORBFE_LAUNCH(prof, ORBFE_STAGE_RESIZE, resize2_kernel<true>, dim3(g.rs2_tiles[l], n),
                                 dim3(256), g.rs2_lds[l], stream, r2);
                else
                    ORBFE_LAUNCH(prof, ORBFE_STAGE_RESIZE, resize2_kernel<false>, dim3(g.rs2_tiles[l], n),
                                 dim3(256), g.rs2_lds[l], stream, r2);
                ++l;
                continue;
            }
            ResizeArgs ra;
            ra.src = lp[l - 1];
            ra.dst = lp[l];
            ra.sw = g.geo.lv[l - 1].w;
            ra.sh = g.geo.lv[l - 1].h;
            ra.dw = g.geo.lv[l].w;
            ra.dh = g.geo.lv[l].h;
            ra.tiles_x = g.rs_tiles_x[l];
            ra.lds_pitch = g.rs_pitch[l];
            ra.xt = xtab.as<int>() + g.xoff[l];
            ra.yt = ytab.as<int>() + g.yoff[l];
            ra.simd_xb = x86() ? sse2_body_resize(ra.dw) : 0;
            ra.gtab = g.pyr_ok && !table_off ? ptab.as<uint4>() + g.gtab_off[l] : nullptr;
            if (x86()) {
                ORBFE_LAUNCH(prof, ORBFE_STAGE_RESIZE, resize_kernel<true>, dim3(g.rs_tiles[l], n),
                             dim3(256), g.rs_lds[l], stream, ra);
            } else {
                ORBFE_LAUNCH(prof, ORBFE_STAGE_RESIZE, resize_kernel<false>, dim3(g.rs_tiles[l], n),
                             dim3(256), g.rs_lds[l], stream, ra);
            }
        }
        if (!one_pyr && ts < L) {
            ResizeTailArgs ta;
            ta.src = lp[ts - 1];
            ta.sh = g.geo.lv[ts - 1].h;
            ta.nt = L - ts;
            ta.lp[0] = (g.geo.lv[ts - 1].w + 15) & ~15;  // 16-byte chunk staging
            ta.buf_b = ta.lp[0] * ta.sh;
            for (int k = 0; k < ta.nt; ++k) {
                const int l = ts + k;
                ta.lp[k + 1] = (g.geo.lv[l].w + 3) & ~3;
                ta.dw[k] = g.geo.lv[l].w;
                ta.dh[k] = g.geo.lv[l].h;
                ta.xt[k] = xtab.as<int>() + g.xoff[l];
                ta.yt[k] = ytab.as<int>() + g.yoff[l];
                ta.dst[k] = lp[l];
                ta.simd_xb[k] = x86() ? sse2_body_resize(ta.dw[k]) : 0;
            }
            if (x86())
                ORBFE_LAUNCH(prof, ORBFE_STAGE_RESIZE, resize_tail_kernel<true>, dim3(n),
                             dim3(kTailBlock), 0, stream, ta);
            else
                ORBFE_LAUNCH(prof, ORBFE_STAGE_RESIZE, resize_tail_kernel<false>, dim3(n),
                             dim3(kTailBlock), 0, stream, ta);
        }
        // K2 FAST per cell
        const int ncells = (int)g.cells.size();
        if (ncells > 0) {
            FastArgs fa;
            fa.cells = cells.as<CellDesc>();
            fa.ncells = ncells;
            fa.cell_cap_total = g.cell_cap_total;
            fa.ini_th = std::min(std::max(tab.p.ini_th_fast, 0), 255);
            fa.min_th = std::min(std::max(tab.p.min_th_fast, 0), 255);
            fa.roi_pitch = g.roi_pitch;
            fa.roi_rows = g.roi_rows;
            fa.cand_max = g.cand_max;
            fa.cell_cnt = cell_cnt.as<int>();
            fa.cell_keys = cell_keys.as<uint32_t>();
            fa.level_keys = level_keys.as<int>();
            for (int l = 0; l < L; ++l) fa.pyr[l] = lp[l];
            if (g.roi_pitch == kFastPitch)
                ORBFE_LAUNCH(prof, ORBFE_STAGE_FAST, fast_kernel<kFastPitch>, dim3(ncells, n), dim3(kFastBlockSize), g.fast_lds, stream, fa);
            else
                ORBFE_LAUNCH(prof, ORBFE_STAGE_FAST, fast_kernel<0>, dim3(ncells, n), dim3(kFastBlockSize), g.fast_lds, stream, fa);
        }
        // K3 oct-tree per (frame, level)
        OctArgs oa;
        oa.geo = g.geo;
        oa.cells = cells.as<CellDesc>();
        oa.ncells = ncells;
        oa.cell_cap_total = g.cell_cap_total;
        oa.cell_cnt = cell_cnt.as<int>();
        oa.cell_keys = cell_keys.as<uint32_t>();
        oa.level_keys = level_keys.as<int>();
        oa.keys = keys.as<uint32_t>();
        oa.act = act.as<int4>();
        oa.oct_out = oct_out.as<uint32_t>();
        oa.oct_cnt = oct_cnt.as<int>();
        // describe's strided waves (batches) sweep each level in 32-row bands where a frame's
        // pyramid overflows half an XCD's L2 (level 0 >= 1 Mpx; 1080p: describe traffic -13 %,
        // 640 x 480: no traffic to save, oct-tree +2.5 %): the oct-tree writes that order beside
        // its output (ORBFE_DESC_ORDER=0: never, =2: at every size)
        const bool banded = n >= kDescSmallBatch && desc_stride && desc_order &&
                            (desc_order_all || (long long)g.geo.lv[0].w * g.geo.lv[0].h >= (1 << 20));
        oa.oct_ord = banded ? oct_ord.as<uint16_t>() : nullptr;
        oa.ncap_max = g.ncap_max;
        oa.sort_cap = g.sort_cap;
        oa.lds_keys = g.oct_keys;
        // 1024-thread trees while the launch has at most one tree per CU (the single-frame call,
        // config 4 at 32 frames per rank: each level-0 tree is the launch's long pole); 256-thread
        // trees, six per CU, for larger batches (throughput)
        if (n * L <= num_cus && oct_small)
            ORBFE_LAUNCH(prof, ORBFE_STAGE_OCTREE, octree_kernel<1024>, dim3(n, L), dim3(1024), g.oct_lds, stream, oa);
        else
            ORBFE_LAUNCH(prof, ORBFE_STAGE_OCTREE, octree_kernel<kOctBlockSize>, dim3(n, L), dim3(kOctBlockSize), g.oct_lds, stream, oa);
        // K4 blur: fused into K5, where each keypoint's window is blurred in LDS, or (PREBLUR)
        // every level of every frame, read by the pre-blurred describe
        if (!fused_blur) {
            BlurArgs ba;
            ba.nlevels = L;
            for (int l = 0; l < L; ++l) {
                ba.w[l] = g.geo.lv[l].w;
                ba.h[l] = g.geo.lv[l].h;
                ba.src[l] = lp[l];
                ba.dst[l] = bp[l];
                ba.simd_xb[l] = x86() ? sse2_body_blur(g.geo.lv[l].w) : 0;
            }
            ba.frags = bslot.as<uint4>();
            ba.items = reinterpret_cast<const uint32_t*>(bslot.as<uint8_t>() + kBlurFragBytes);
            ba.nitems = (int)g.bitems.size();
            for (int i = 0; i < 4; ++i) ba.taps[i] = tab.taps[i];
            if (x86())
                ORBFE_LAUNCH(prof, ORBFE_STAGE_BLUR, blur_mfma_kernel<true>, dim3(ba.nitems, n), dim3(256), 0, stream, ba);
            else
                ORBFE_LAUNCH(prof, ORBFE_STAGE_BLUR, blur_mfma_kernel<false>, dim3(ba.nitems, n), dim3(256), 0, stream, ba);
        }
        // K5 describe
        DescArgs da;
        da.nlevels = L;
        da.out_total = g.geo.out_total;
        da.kps_cap = kps_cap;
        for (int l = 0; l < L; ++l) {
            da.out_off[l] = g.geo.lv[l].out_off;
            da.scale[l] = g.geo.lv[l].scale;
            da.size[l] = g.geo.lv[l].size;
            da.pyr[l] = lp[l];
            da.blur[l] = bp[l];
            da.w[l] = g.geo.lv[l].w;
            da.h[l] = g.geo.lv[l].h;
            da.simd_xb[l] = x86() ? sse2_body_blur(da.w[l]) : 0;
        }
        for (int i = 0; i < 4; ++i) da.taps[i] = tab.taps[i];
        da.oct_out = oct_out.as<uint32_t>();
        da.oct_cnt = oct_cnt.as<int>();
        da.oct_ord = banded ? oct_ord.as<uint16_t>() : nullptr;
        da.kps = d_kps;
        da.desc = d_desc;
        da.n_out = d_n;
        const bool all_pre = !fused_blur && pre_mask_env == 0xffffffffu;
        da.pre_mask = fused_blur ? 0u : pre_mask_env;
        // a wave takes kDescGroupSize keypoints (the trig and pattern loads amortised over the
        // group); small batches take kDescGroupSmall, for four times the waves in flight
        // (x86 arithmetic: the rotation FMA-contracted, kFma)
        // window source: every level pre-blurred, some levels pre-blurred (VALU blur for the
        // rest), or none (the matrix-core blur unless ORBFE_DESC_MFMA=0)
        const int win = all_pre ? kWinPre : (da.pre_mask == 0u && desc_mfma ? kWinMfma : kWinValu);
        // ORBFE_DESC_G16=1 (opt-in): 16 keypoints per wave in strided x86 matrix-core batches.
        // At 640 x 480 describe runs 2 % faster (c3 +1.3 % frames/s) but moves 1.30 GB per
        // 512-frame launch instead of 0.70 (1.65x its algorithmic bytes: the frames in flight
        // per XCD double); at 1080p it is 9 % slower (profiles/r04/experiments/describe_g16/)
        const bool g16 = desc_g16 == 1 && n >= kDescSmallBatch && desc_stride && x86() && win == kWinMfma;
        const int group = g16 ? 16 : n >= kDescSmallBatch ? kDescGroupSize : kDescGroupSmall;
        const int per_block = (kDescBlockSize / 64) * group;  // slots per workgroup
        const dim3 dgrid((g.geo.out_total + per_block - 1) / per_block, n);
        // batches: strided slots (a frame's waves sweep its oct-tree output in runs of W
        // consecutive slots, sharing window lines in L2); ORBFE_DESC_STRIDE=0: grouped slots
        da.wave_stride = (group == kDescGroupSize || g16) && desc_stride ? (int)dgrid.x * (kDescBlockSize / 64) : 0;
        da.frags = bslot.as<uint4>() + kDescFragOff;
        const int variant = g16 ? 12 : (group == kDescGroupSize ? 6 : 0) + (x86() ? 3 : 0) + win;
        switch (variant) {
#define ORBFE_DESC_CASE(V, G, X, W) \
            case V: ORBFE_LAUNCH(prof, ORBFE_STAGE_DESCRIBE, (describe_kernel<G, X, W>), dgrid, dim3(kDescBlockSize), 0, stream, da); break;
            ORBFE_DESC_CASE(0, kDescGroupSmall, false, kWinValu)
            ORBFE_DESC_CASE(1, kDescGroupSmall, false, kWinPre)
            ORBFE_DESC_CASE(2, kDescGroupSmall, false, kWinMfma)
            ORBFE_DESC_CASE(3, kDescGroupSmall, true, kWinValu)
            ORBFE_DESC_CASE(4, kDescGroupSmall, true, kWinPre)
            ORBFE_DESC_CASE(5, kDescGroupSmall, true, kWinMfma)
            ORBFE_DESC_CASE(6, kDescGroupSize, false, kWinValu)
            ORBFE_DESC_CASE(7, kDescGroupSize, false, kWinPre)
            ORBFE_DESC_CASE(8, kDescGroupSize, false, kWinMfma)
            ORBFE_DESC_CASE(9, kDescGroupSize, true, kWinValu)
            ORBFE_DESC_CASE(10, kDescGroupSize, true, kWinPre)
            ORBFE_DESC_CASE(11, kDescGroupSize, true, kWinMfma)
            ORBFE_DESC_CASE(12, 16, true, kWinMfma)
#undef ORBFE_DESC_CASE
        }
        ORBFE_HIP(hipGetLastError());
        last_n = n;
        for (int l = 0; l < L; ++l) last_pyr[l] = lp[l];
        return ORBFE_OK;
    }

    // K0: level 0 of every frame from the caller's frames (gray or colour), full masks laid out
    // like the frames' rows (mask_fpitch / mask_pitch) and/or per-frame zeroed rectangles.
    int launch_level0(int n, const uint8_t* src, long long src_fpitch, int src_pitch, int pix,
                      const uint8_t* mask, long long mask_fpitch, int mask_pitch,
                      const int4* d_rects) {
        const Plan& g = plan;
        const LevelGeo& l0 = g.geo.lv[0];
        Level0Args a;
        a.src = src;
        a.src_fpitch = src_fpitch;
        a.src_pitch = src_pitch;
        a.cn = pix_channels(pix);
        const bool rgb_first = pix == ORBFE_PIX_RGB || pix == ORBFE_PIX_RGBA;
        a.c0 = rgb_first ? 4899 : 1868;  // R2Y : B2Y (yuv_shift 14)
        a.c2 = rgb_first ? 1868 : 4899;
        a.aligned = ((uintptr_t)src % 4 == 0) && src_pitch % 4 == 0 && src_fpitch % 4 == 0;
        a.mask = mask;
        a.mask_fpitch = mask_fpitch;
        a.mask_pitch = mask_pitch;
        a.rects = d_rects;
        a.dst = pyr.as<uint8_t>() + l0.off;
        a.dst_fpitch = g.slab;
        a.dst_pitch = l0.pitch;
        a.w = g.w;
        a.h = g.h;
        ORBFE_LAUNCH(prof, ORBFE_STAGE_MASK, level0_kernel, dim3((g.w + 1023) / 1024, g.h, n), dim3(256),
                     0, stream, a);
        return ORBFE_OK;
    }

    // Host-pointer path: upload, run into the staging slabs, download.
    int run_host(const uint8_t* const* imgs, int n, int w, int h, size_t stride, int pix,
                 const uint8_t* const* masks, size_t mstride, const orbfe_rect* host_rects) {
        int st;
        if ((st = set_plan(w, h))) return st;
        if ((st = ensure_frames(n))) return st;
        const Plan& g = plan;
        const LevelGeo& l0 = g.geo.lv[0];
        const int cap = kp_capacity();
        if ((st = out_kps.ensure((size_t)n * cap * sizeof(orbfe_keypoint)))) return st;
        if ((st = out_desc.ensure((size_t)n * cap * 32))) return st;
        if ((st = out_n.ensure((size_t)n * sizeof(int32_t)))) return st;
        bool any_mask = false;
        if (masks)
            for (int f = 0; f < n; ++f) any_mask |= masks[f] != nullptr;
        const int cn = pix_channels(pix);
        if (pix == ORBFE_PIX_GRAY && !any_mask && !host_rects) {
            for (int f = 0; f < n; ++f) {
                uint8_t* dst = pyr.as<uint8_t>() + (size_t)f * g.slab + l0.off;
                ORBFE_HIP(hipMemcpy2DAsync(dst, l0.pitch, imgs[f], stride, w, h,
                                           hipMemcpyHostToDevice, stream));
            }
        } else {
            // frames -> `stage` (rows padded to 4 B so K0 reads them with vector loads)
            const size_t spitch = ((size_t)w * cn + 3) & ~(size_t)3;
            const size_t sfp = spitch * h;
            if ((st = stage.ensure(n * sfp))) return st;
            for (int f = 0; f < n; ++f)
                ORBFE_HIP(hipMemcpy2DAsync(stage.as<uint8_t>() + f * sfp, spitch, imgs[f], stride,
                                           (size_t)w * cn, h, hipMemcpyHostToDevice, stream));
            // masks -> the blur slab, which is free until K4
            if (any_mask) {
                for (int f = 0; f < n; ++f) {
                    uint8_t* mdst = blur.as<uint8_t>() + (size_t)f * g.slab + l0.off;
                    if (masks[f]) {
                        ORBFE_HIP(hipMemcpy2DAsync(mdst, l0.pitch, masks[f], mstride, w, h,
                                                   hipMemcpyHostToDevice, stream));
                    } else {
                        ORBFE_HIP(hipMemset2DAsync(mdst, l0.pitch, 1, w, h, stream));
                    }
                }
            }
            const int4* d_rects = nullptr;
            if (host_rects) {
                if ((st = rects.ensure(n * sizeof(int4)))) return st;
                h_rects.resize(n);
                for (int f = 0; f < n; ++f)
                    h_rects[f] = int4{host_rects[f].x0, host_rects[f].y0, host_rects[f].x1,
                                      host_rects[f].y1};
                ORBFE_HIP(hipMemcpyAsync(rects.p, h_rects.data(), n * sizeof(int4),
                                         hipMemcpyHostToDevice, stream));
                d_rects = rects.as<int4>();
            }
            if ((st = launch_level0(n, stage.as<uint8_t>(), (long long)sfp, (int)spitch, pix,
                                    any_mask ? blur.as<uint8_t>() + l0.off : nullptr, g.slab,
                                    l0.pitch, d_rects)))
                return st;
        }
        LevelPtr lp0{pyr.as<uint8_t>() + l0.off, g.slab, l0.pitch};
        if ((st = run(n, lp0, out_kps.as<orbfe_keypoint>(), cap, out_desc.as<uint8_t>(),
                      out_n.as<int32_t>())))
            return st;
        h_n.resize(n);
        h_kps.resize((size_t)n * cap);
        h_desc.resize((size_t)n * cap * 32);
        ORBFE_HIP(hipMemcpyAsync(h_n.data(), out_n.p, n * sizeof(int32_t), hipMemcpyDeviceToHost, stream));
        ORBFE_HIP(hipMemcpyAsync(h_kps.data(), out_kps.p, h_kps.size() * sizeof(orbfe_keypoint),
                                 hipMemcpyDeviceToHost, stream));
        ORBFE_HIP(hipMemcpyAsync(h_desc.data(), out_desc.p, h_desc.size(), hipMemcpyDeviceToHost, stream));
        ORBFE_HIP(hipStreamSynchronize(stream));
        return ORBFE_OK;
    }

    ~orbfe_extractor() {
        for (DevBuf* b : {&cells, &xtab, &ytab, &bslot, &ptab, &pyr, &blur, &cell_cnt, &cell_keys, &keys, &act,
                          &oct_out, &oct_cnt, &oct_ord, &level_keys, &lk_snap, &out_kps, &out_desc, &out_n, &stage, &rects, &st_off, &st_items,
                          &st_sad, &st_status, &st_ur})
            b->release();
        drop_graph();
        for (Pinned* q : {&pin_in, &pin_user, &pin_kps, &pin_desc, &pin_n, &st_pin}) q->release();
        st_in.release();
        prof.release();
        if (own) hipStreamDestroy(own);
    }
};

namespace {
struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int d) {
        hipGetDevice(&prev);
        if (prev != d) hipSetDevice(d);
    }
    ~DeviceGuard() {
        int cur = -1;
        hipGetDevice(&cur);
        if (prev >= 0 && cur != prev) hipSetDevice(prev);
    }
};
}  // namespace

extern "C" {

orbfe_extractor* orbfe_create(const orbfe_params* params, int device, int max_width,
                              int max_height, int max_batch, int* status) {
    int st = ORBFE_OK;
    orbfe_extractor* h = nullptr;
    try {
        if (!params) {
            st = ORBFE_ERR_ARG;
        } else if ((st = check_device(device)) == ORBFE_OK) {
            DeviceGuard dg(device);
            h = new orbfe_extractor();
            h->device = device;
            int cus = 0;
            if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && cus > 0)
                h->num_cus = cus;
            st = make_tables(*params, h->tab);
            if (st == ORBFE_OK && hipStreamCreateWithFlags(&h->own, hipStreamNonBlocking) != hipSuccess)
                st = ORBFE_ERR_HIP;
            h->stream = h->own;
            if (st == ORBFE_OK && hipMemcpyToSymbol(HIP_SYMBOL(c_umax), h->tab.umax, sizeof(h->tab.umax)) != hipSuccess)
                st = ORBFE_ERR_HIP;
            const int w = max_width > 0 ? max_width : 1920, hh = max_height > 0 ? max_height : 1080;
            if (st == ORBFE_OK) st = h->set_plan(w, hh);
            if (st == ORBFE_OK) st = h->ensure_frames(std::max(1, max_batch));
        }
    } catch (const std::bad_alloc&) {
        st = ORBFE_ERR_NOMEM;
    } catch (...) {
        st = ORBFE_ERR_HIP;
    }
    if (st != ORBFE_OK && h) {
        delete h;
        h = nullptr;
    }
    if (status) *status = st;
    return h;
}

void orbfe_destroy(orbfe_extractor* h) {
    if (!h) return;
    DeviceGuard dg(h->device);
    hipStreamSynchronize(h->stream);
    delete h;
}

int orbfe_set_arithmetic(orbfe_extractor* h, int mode) {
    if (!h || (mode != ORBFE_ARITH_SCALAR && mode != ORBFE_ARITH_X86_SIMD)) return ORBFE_ERR_ARG;
    DeviceGuard dg(h->device);
    if (hipStreamSynchronize(h->stream) != hipSuccess) return ORBFE_ERR_HIP;
    if (mode != h->arith) h->drop_graph();  // the captured launches carry the old mode
    h->arith = mode;
    return ORBFE_OK;
}

int orbfe_get_arithmetic(const orbfe_extractor* h) { return h ? h->arith : ORBFE_ERR_ARG; }

int orbfe_get_reference_constants(orbfe_reference_constants* out) {
    if (!out) return ORBFE_ERR_ARG;
    *out = orbfe_reference_constants{kPatchSize, kHalfPatchSize, kEdgeThreshold,
                                     kThHigh, kThLow, kHistoLength};
    return ORBFE_OK;
}

int orbfe_get_levels(const orbfe_extractor* h) { return h ? h->tab.p.nlevels : ORBFE_ERR_ARG; }
float orbfe_get_scale_factor(const orbfe_extractor* h) { return h ? h->tab.p.scale_factor : 0.f; }

int orbfe_get_scale_tables(const orbfe_extractor* h, float* scale, float* inv, float* sigma2,
                           float* inv_sigma2) {
    if (!h) return ORBFE_ERR_ARG;
    for (int l = 0; l < h->tab.p.nlevels; ++l) {
        if (scale) scale[l] = h->tab.scale[l];
        if (inv) inv[l] = h->tab.inv[l];
        if (sigma2) sigma2[l] = h->tab.sigma2[l];
        if (inv_sigma2) inv_sigma2[l] = h->tab.inv_sigma2[l];
    }
    return ORBFE_OK;
}

int orbfe_get_features_per_level(const orbfe_extractor* h, int32_t* out) {
    if (!h || !out) return ORBFE_ERR_ARG;
    for (int l = 0; l < h->tab.p.nlevels; ++l) out[l] = h->tab.nfeat[l];
    return ORBFE_OK;
}

int orbfe_keypoint_capacity(const orbfe_extractor* h) {
    if (!h) return ORBFE_ERR_ARG;
    // Sum over levels of the oct-tree list bound max(N + 4, 4 nIni, 20) (plan_geometry) at the
    // largest nIni any supported input (w, h <= 4096) gives that level: a level with FAST
    // cells has bh = h_l - 32 >= 30, so nIni <= round((round(4096 / s_l) - 32) / 30).
    int c = 0;
    for (int l = 0; l < h->tab.p.nlevels; ++l) {
        const int wl = (int)std::lrintf(4096.f * h->tab.inv[l]);
        const int nini = std::max(1, (int)std::lround((double)(wl - 32) / 30.0));
        c += std::max({h->tab.nfeat[l] + 4, 4 * nini, 20});
    }
    return c;
}

int orbfe_keypoint_capacity_for(const orbfe_extractor* h, int w, int hgt) {
    if (!h || w <= 0 || hgt <= 0) return ORBFE_ERR_ARG;
    if (h->planned && h->plan.w == w && h->plan.h == hgt) return h->plan.geo.out_total;
    try {
        Plan g;
        const int st = plan_geometry(h->tab, w, hgt, g);
        return st != ORBFE_OK ? st : g.geo.out_total;
    } catch (const std::bad_alloc&) {
        return ORBFE_ERR_NOMEM;
    }
}

int orbfe_keypoint_capacity_params(const orbfe_params* p, int w, int hgt) {
    if (!p || w <= 0 || hgt <= 0) return ORBFE_ERR_ARG;
    try {
        HostTables t{};
        int st = make_tables(*p, t);
        if (st != ORBFE_OK) return st;
        Plan g;
        st = plan_geometry(t, w, hgt, g);
        return st != ORBFE_OK ? st : g.geo.out_total;
    } catch (const std::bad_alloc&) {
        return ORBFE_ERR_NOMEM;
    }
}

static int extract_host_common(orbfe_extractor* h, const uint8_t* const* imgs, int n, int w,
                               int hgt, size_t stride, int pix, const uint8_t* const* masks,
                               size_t mask_stride, const orbfe_rect* rects, orbfe_keypoint* kps,
                               int kps_cap, uint8_t* desc, int32_t* n_out) {
    DeviceGuard dg(h->device);
    h->staged_kps = nullptr;
    h->staged_desc = nullptr;
    h->staged_n = 0;
    if (n == 1 && pix == ORBFE_PIX_GRAY && !(masks && masks[0]) && !rects) {
        bool done = false;
        int st = h->run_single_graph(imgs[0], w, hgt, stride, &done);
        if (st != ORBFE_OK) return st;
        if (done) {
            const int cnt = *reinterpret_cast<const int32_t*>(h->pin_n.p);
            n_out[0] = cnt;
            h->staged_kps = reinterpret_cast<const orbfe_keypoint*>(h->pin_kps.p);
            h->staged_desc = h->pin_desc.p;
            h->staged_n = std::min(cnt, h->kp_capacity());
            if (!kps) return ORBFE_OK;  // orbfe_extract_staged: outputs stay in the staging
            if (cnt > kps_cap) return ORBFE_ERR_CAPACITY;
            std::memcpy(kps, h->pin_kps.p, (size_t)cnt * sizeof(orbfe_keypoint));
            if (desc) std::memcpy(desc, h->pin_desc.p, (size_t)cnt * 32);
            return ORBFE_OK;
        }
    }
    int st = h->run_host(imgs, n, w, hgt, stride, pix, masks, mask_stride, rects);
    if (st != ORBFE_OK) return st;
    const int cap = h->kp_capacity();
    if (n == 1) {
        h->staged_kps = h->h_kps.data();
        h->staged_desc = h->h_desc.data();
        h->staged_n = std::min(h->h_n[0], cap);
        if (!kps) {
            n_out[0] = h->h_n[0];
            return ORBFE_OK;
        }
    }
    int worst = ORBFE_OK;
    for (int f = 0; f < n; ++f) {
        const int cnt = h->h_n[f];
        n_out[f] = cnt;
        if (cnt > kps_cap) {
            worst = ORBFE_ERR_CAPACITY;
            continue;
        }
        std::memcpy(kps + (size_t)f * kps_cap, h->h_kps.data() + (size_t)f * cap,
                    (size_t)cnt * sizeof(orbfe_keypoint));
        if (desc)
            std::memcpy(desc + (size_t)f * kps_cap * 32, h->h_desc.data() + (size_t)f * cap * 32,
                        (size_t)cnt * 32);
    }
    return worst;
}

static bool rect_ok(const orbfe_rect* r) { return !r || (r->x0 <= r->x1 && r->y0 <= r->y1); }

int orbfe_extract(orbfe_extractor* h, const uint8_t* img, int w, int hgt, size_t stride,
                  const uint8_t* mask, size_t mask_stride, orbfe_keypoint* kps, int kps_cap,
                  uint8_t* desc, int* n_out) {
    return orbfe_extract_color(h, img, ORBFE_PIX_GRAY, w, hgt, stride, mask, mask_stride, nullptr,
                               kps, kps_cap, desc, n_out);
}

int orbfe_extract_color(orbfe_extractor* h, const uint8_t* img, int pix, int w, int hgt,
                        size_t stride, const uint8_t* mask, size_t mask_stride,
                        const orbfe_rect* rect, orbfe_keypoint* kps, int kps_cap, uint8_t* desc,
                        int* n_out) {
    if (!h) return ORBFE_ERR_ARG;
    if (!img || w <= 0 || hgt <= 0) return ORBFE_OK;  // empty image: no-op (1045-1046)
    const int cn = pix_channels(pix);
    if (!cn || !kps || !n_out || kps_cap < 0 || stride < (size_t)w * cn ||
        (mask && mask_stride < (size_t)w))
        return ORBFE_ERR_ARG;
    if (!rect_ok(rect)) return ORBFE_ERR_UNSUPPORTED;
    try {
        const uint8_t* m[1] = {mask};
        int32_t cnt = 0;
        const int st = extract_host_common(h, &img, 1, w, hgt, stride, pix, mask ? m : nullptr,
                                           mask_stride, rect, kps, kps_cap, desc, &cnt);
        *n_out = cnt;
        return st;
    } catch (const std::bad_alloc&) {
        return ORBFE_ERR_NOMEM;
    } catch (...) {
        return ORBFE_ERR_HIP;
    }
}

int orbfe_input_buffer(orbfe_extractor* h, int w, int hgt, uint8_t** buf, size_t* stride) {
    if (!h || w <= 0 || hgt <= 0 || !buf || !stride) return ORBFE_ERR_ARG;
    try {
        DeviceGuard dg(h->device);
        int st;
        if ((st = h->set_plan(w, hgt))) return st;  // the size must be one the plan supports
        if ((st = h->pin_user.ensure((size_t)w * hgt))) return st;
        *buf = h->pin_user.p;
        *stride = (size_t)w;
        return ORBFE_OK;
    } catch (const std::bad_alloc&) {
        return ORBFE_ERR_NOMEM;
    } catch (...) {
        return ORBFE_ERR_HIP;
    }
}

int orbfe_extract_staged(orbfe_extractor* h, int w, int hgt, orbfe_keypoint* kps, int kps_cap,
                         uint8_t* desc, int* n_out) {
    if (!h || w <= 0 || hgt <= 0 || !n_out || kps_cap < 0 || (kps_cap > 0 && !kps)) return ORBFE_ERR_ARG;
    if (!h->pin_user.p || h->pin_user.bytes < (size_t)w * hgt) return ORBFE_ERR_ARG;  // no buffer handed out
    try {
        const uint8_t* img = h->pin_user.p;
        int32_t cnt = 0;
        const int st = extract_host_common(h, &img, 1, w, hgt, (size_t)w, ORBFE_PIX_GRAY, nullptr, 0,
                                           nullptr, kps_cap ? kps : nullptr, kps_cap, desc, &cnt);
        *n_out = cnt;
        return st;
    } catch (const std::bad_alloc&) {
        return ORBFE_ERR_NOMEM;
    } catch (...) {
        return ORBFE_ERR_HIP;
    }
}

int orbfe_staged_outputs(const orbfe_extractor* h, const orbfe_keypoint** kps, const uint8_t** desc,
                         int* n) {
    if (!h || !kps || !desc || !n) return ORBFE_ERR_ARG;
    *kps = h->staged_kps;
    *desc = h->staged_desc;
    *n = h->staged_kps ? h->staged_n : 0;
    return ORBFE_OK;
}

int orbfe_extract_batch(orbfe_extractor* h, const uint8_t* const* imgs, int n, int w, int hgt,
                        size_t stride, const uint8_t* const* masks, size_t mask_stride,
                        orbfe_keypoint* kps, int kps_cap, uint8_t* desc, int32_t* n_out) {
    if (!h || n < 0 || !imgs || !kps || !n_out || kps_cap < 0) return ORBFE_ERR_ARG;
    if (n == 0 || w <= 0 || hgt <= 0) return ORBFE_OK;
    if (stride < (size_t)w || (masks && mask_stride < (size_t)w)) return ORBFE_ERR_ARG;
    for (int f = 0; f < n; ++f)
        if (!imgs[f]) return ORBFE_ERR_ARG;
    try {
        return extract_host_common(h, imgs, n, w, hgt, stride, ORBFE_PIX_GRAY, masks, mask_stride,
                                   nullptr, kps, kps_cap, desc, n_out);
    } catch (const std::bad_alloc&) {
        return ORBFE_ERR_NOMEM;
    } catch (...) {
        return ORBFE_ERR_HIP;
    }
}

int orbfe_extract_batch_device(orbfe_extractor* h, const uint8_t* d_imgs, int n, int w, int hgt,
                               size_t stride, size_t frame_pitch, const uint8_t* d_masks,
                               orbfe_keypoint* d_kps, int kps_cap, uint8_t* d_desc,
                               int32_t* d_n_out) {
    return orbfe_extract_color_batch_device(h, d_imgs, ORBFE_PIX_GRAY, n, w, hgt, stride,
                                            frame_pitch, d_masks, stride, frame_pitch, nullptr,
                                            d_kps, kps_cap, d_desc, d_n_out);
}

int orbfe_extract_color_batch_device(orbfe_extractor* h, const uint8_t* d_imgs, int pix, int n,
                                     int w, int hgt, size_t stride, size_t frame_pitch,
                                     const uint8_t* d_masks, size_t mask_stride,
                                     size_t mask_frame_pitch, const orbfe_rect* d_rects,
                                     orbfe_keypoint* d_kps, int kps_cap, uint8_t* d_desc,
                                     int32_t* d_n_out) {
    const int cn = pix_channels(pix);
    if (!h || n < 0 || !d_imgs || !d_kps || !d_desc || !d_n_out || !cn) return ORBFE_ERR_ARG;
    if (n == 0 || w <= 0 || hgt <= 0) return ORBFE_OK;
    if (stride < (size_t)w * cn || (n > 1 && frame_pitch < stride * hgt)) return ORBFE_ERR_ARG;
    if (d_masks && (mask_stride < (size_t)w || (n > 1 && mask_frame_pitch < mask_stride * hgt)))
        return ORBFE_ERR_ARG;
    try {
        DeviceGuard dg(h->device);
        int st;
        if ((st = h->set_plan(w, hgt))) return st;
        if (kps_cap < h->kp_capacity()) return ORBFE_ERR_CAPACITY;
        if ((st = h->ensure_frames(n))) return st;
        const Plan& g = h->plan;
        const LevelGeo& l0 = g.geo.lv[0];
        LevelPtr lp0{d_imgs, (long long)frame_pitch, (int)stride};
        const bool aligned = ((uintptr_t)d_imgs % 4 == 0) && stride % 4 == 0 && frame_pitch % 4 == 0;
        if (pix != ORBFE_PIX_GRAY || d_masks || d_rects || !aligned) {
            // K0 writes level 0 into the slab (the kernels read level 0 as dwords)
            if ((st = h->launch_level0(n, d_imgs, (long long)frame_pitch, (int)stride, pix, d_masks,
                                       (long long)mask_frame_pitch, (int)mask_stride,
                                       reinterpret_cast<const int4*>(d_rects))))
                return st;
            lp0 = LevelPtr{h->pyr.as<uint8_t>() + l0.off, g.slab, l0.pitch};
        }
        return h->run(n, lp0, d_kps, kps_cap, d_desc, d_n_out);
    } catch (...) {
        return ORBFE_ERR_HIP;
    }
}

// ---- stereo (Frame::ComputeStereoMatches, Frame.cc:584-756) ----------------------------------
// Launches S1-S3 of orbfe_stereo.hip on the left handle's stream for frames [f0, f0 + n) of
// the two handles' most recent extractions; keypoint slabs are `kps_cap` apart per frame.
static int stereo_launch(orbfe_extractor* L, orbfe_extractor* R, int f0, int n,
                         const orbfe_keypoint* d_kl, const uint8_t* d_dl, const int32_t* d_nl,
                         const orbfe_keypoint* d_kr, const uint8_t* d_dr, const int32_t* d_nr,
                         int kps_cap, float bf, float b, float* d_ur, float* d_dp) {
    const Plan& g = L->plan;
    const int nlev = L->tab.p.nlevels;
    StereoArgs a;
    a.nrows = g.h;
    float smax = 1.f;
    for (int l = 0; l < nlev; ++l) smax = std::max(smax, L->tab.scale[l]);
    a.row_cap = (int)std::ceil(4.0f * smax) + 3;  // rows floor(y-r)..ceil(y+r), r = 2 scale
    a.kps_cap = kps_cap;
    a.nlevels = nlev;
    a.kl = d_kl;
    a.dl = reinterpret_cast<const uint4*>(d_dl);
    a.nl = d_nl;
    a.kr = d_kr;
    a.dr = reinterpret_cast<const uint4*>(d_dr);
    a.nr = d_nr;
    for (int l = 0; l < nlev; ++l) {
        a.scale[l] = L->tab.scale[l];
        a.inv[l] = L->tab.inv[l];
        a.pl[l] = L->last_pyr[l];
        a.pr[l] = R->last_pyr[l];
        a.pl[l].base += f0 * a.pl[l].fpitch;
        a.pr[l].base += f0 * a.pr[l].fpitch;
        a.lw[l] = g.geo.lv[l].w;
        a.lh[l] = g.geo.lv[l].h;
    }
    a.bf = bf;
    a.b = b;
    int st;
    if ((st = L->st_off.ensure((size_t)n * (g.h + 1) * sizeof(int)))) return st;
    if ((st = L->st_items.ensure((size_t)n * kps_cap * a.row_cap * sizeof(int)))) return st;
    if ((st = L->st_sad.ensure((size_t)n * kps_cap * sizeof(int)))) return st;
    if ((st = L->st_status.ensure(sizeof(int)))) return st;
    a.row_off = L->st_off.as<int>();
    a.row_items = L->st_items.as<int>();
    a.u_right = d_ur;
    a.depth = d_dp;
    a.sad = L->st_sad.as<int>();
    a.status = L->st_status.as<int>();
    // the right handle's extraction must be complete on its own stream
    if (R->stream != L->stream) {
        hipEvent_t ev;
        ORBFE_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        ORBFE_HIP(hipEventRecord(ev, R->stream));
        ORBFE_HIP(hipStreamWaitEvent(L->stream, ev, 0));
        ORBFE_HIP(hipEventDestroy(ev));
    }
    ORBFE_HIP(hipMemsetAsync(a.status, 0, sizeof(int), L->stream));
    hipLaunchKernelGGL(stereo_rows_kernel, dim3(n), dim3(kStereoRowsBlock), 0, L->stream, a);
    hipLaunchKernelGGL(stereo_match_kernel, dim3((kps_cap + 3) / 4, n), dim3(kStereoBlock), 0,
                       L->stream, a);
    hipLaunchKernelGGL(stereo_filter_kernel, dim3(n), dim3(kStereoFilterBlock), 0, L->stream, a);
    ORBFE_HIP(hipGetLastError());
    return ORBFE_OK;
}

static int stereo_pair_ok(const orbfe_extractor* L, const orbfe_extractor* R, int f_end) {
    if (!L || !R || !L->planned || !R->planned || L->device != R->device) return ORBFE_ERR_ARG;
    if (L->plan.w != R->plan.w || L->plan.h != R->plan.h ||
        L->tab.p.nlevels != R->tab.p.nlevels || L->tab.p.scale_factor != R->tab.p.scale_factor)
        return ORBFE_ERR_ARG;
    if (f_end > L->last_n || f_end > R->last_n) return ORBFE_ERR_ARG;
    if (L->plan.h > kStereoMaxRows) return ORBFE_ERR_UNSUPPORTED;
    return ORBFE_OK;
}

int orbfe_compute_stereo_matches(orbfe_extractor* left, orbfe_extractor* right, int frame,
                                 const orbfe_keypoint* kl, const uint8_t* dl, int nl,
                                 const orbfe_keypoint* kr, const uint8_t* dr, int nr, float bf,
                                 float b, float* u_right, float* depth) {
    if (frame < 0 || nl < 0 || nr < 0 || (nl && (!kl || !dl || !u_right || !depth)) ||
        (nr && (!kr || !dr)))
        return ORBFE_ERR_ARG;
    int st = stereo_pair_ok(left, right, frame + 1);
    if (st) return st;
    if (nl == 0) return ORBFE_OK;
    if (nr >= 65536) return ORBFE_ERR_UNSUPPORTED;  // candidate keys pack iR in 16 bits
    try {
        DeviceGuard dg(left->device);
        orbfe_extractor* L = left;
        const int cap = std::max(nl, nr);
        hipStream_t s = L->stream;
        const int32_t counts[2] = {nl, nr};
        // inputs kl | dl | kr | dr | counts staged in one pinned block and copied in by one DMA;
        // outputs u_right | depth (one device block) and the status copied back into it
        auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
        const size_t o_dl = al((size_t)nl * sizeof(orbfe_keypoint)), o_kr = o_dl + al((size_t)nl * 32),
                     o_dr = o_kr + al((size_t)nr * sizeof(orbfe_keypoint)), o_n = o_dr + al((size_t)nr * 32),
                     in_bytes = o_n + 256, o_ur = 0, o_dp = al((size_t)nl * 4), o_st = o_dp + al((size_t)nl * 4),
                     out_bytes = o_st + 256;
        if ((st = L->st_pin.ensure(std::max(in_bytes, out_bytes)))) return st;
        if ((st = L->st_in.ensure(in_bytes))) return st;
        uint8_t* q = L->st_pin.p;
        std::memcpy(q, kl, (size_t)nl * sizeof(orbfe_keypoint));
        std::memcpy(q + o_dl, dl, (size_t)nl * 32);
        if (nr) {
            std::memcpy(q + o_kr, kr, (size_t)nr * sizeof(orbfe_keypoint));
            std::memcpy(q + o_dr, dr, (size_t)nr * 32);
        }
        std::memcpy(q + o_n, counts, sizeof(counts));
        ORBFE_HIP(hipMemcpyAsync(L->st_in.p, q, in_bytes, hipMemcpyHostToDevice, s));
        uint8_t* din = L->st_in.as<uint8_t>();
        if ((st = L->st_ur.ensure(out_bytes))) return st;
        uint8_t* dout = L->st_ur.as<uint8_t>();
        if ((st = stereo_launch(L, right, frame, 1, reinterpret_cast<const orbfe_keypoint*>(din), din + o_dl,
                                reinterpret_cast<const int32_t*>(din + o_n),
                                reinterpret_cast<const orbfe_keypoint*>(din + o_kr), din + o_dr,
                                reinterpret_cast<const int32_t*>(din + o_n) + 1, cap, bf, b,
                                reinterpret_cast<float*>(dout + o_ur), reinterpret_cast<float*>(dout + o_dp))))
            return st;
        ORBFE_HIP(hipMemcpyAsync(dout + o_st, L->st_status.p, sizeof(int), hipMemcpyDeviceToDevice, s));
        ORBFE_HIP(hipMemcpyAsync(q, dout, out_bytes, hipMemcpyDeviceToHost, s));
        ORBFE_HIP(hipStreamSynchronize(s));
        std::memcpy(u_right, q + o_ur, (size_t)nl * sizeof(float));
        std::memcpy(depth, q + o_dp, (size_t)nl * sizeof(float));
        int status = 0;
        std::memcpy(&status, q + o_st, sizeof(int));
        return status;
    } catch (const std::bad_alloc&) {
        return ORBFE_ERR_NOMEM;
    } catch (...) {
        return ORBFE_ERR_HIP;
    }
}

int orbfe_compute_stereo_matches_device(orbfe_extractor* left, orbfe_extractor* right, int n,
                                        const orbfe_keypoint* d_kl, const uint8_t* d_dl,
                                        const int32_t* d_nl, const orbfe_keypoint* d_kr,
                                        const uint8_t* d_dr, const int32_t* d_nr, int kps_cap,
                                        float bf, float b, float* d_u_right, float* d_depth) {
    if (n < 0 || kps_cap <= 0 || !d_kl || !d_dl || !d_nl || !d_kr || !d_dr || !d_nr ||
        !d_u_right || !d_depth)
        return ORBFE_ERR_ARG;
    int st = stereo_pair_ok(left, right, n);
    if (st || n == 0) return st;
    if (kps_cap >= 65536) return ORBFE_ERR_UNSUPPORTED;
    try {
        DeviceGuard dg(left->device);
        return stereo_launch(left, right, 0, n, d_kl, d_dl, d_nl, d_kr, d_dr, d_nr, kps_cap, bf,
                             b, d_u_right, d_depth);
    } catch (...) {
        return ORBFE_ERR_HIP;
    }
}

int orbfe_stereo_status(orbfe_extractor* left) {
    if (!left) return ORBFE_ERR_ARG;
    if (!left->st_status.p) return ORBFE_OK;
    DeviceGuard dg(left->device);
    int status = 0;
    ORBFE_HIP(hipMemcpyAsync(&status, left->st_status.p, sizeof(int), hipMemcpyDeviceToHost, left->stream));
    ORBFE_HIP(hipStreamSynchronize(left->stream));
    return status;
}

int orbfe_human_mask_rect(const float* joints, int njoints, int w, int hgt, orbfe_rect* out) {
    if (!joints || njoints < 0 || w <= 0 || hgt <= 0 || !out) return ORBFE_ERR_ARG;
    // OpDetector::SkeletonSquareMask (DetectHumanPose.cpp:453-489): the bounding box of the
    // joints' (x, y) (a float ternary truncated by static_cast<int>), grown by 30 px, clamped.
    int xmin = w - 1, ymin = hgt - 1, xmax = 0, ymax = 0;
    for (int i = 0; i < njoints; ++i) {
        const float x = joints[3 * i], y = joints[3 * i + 1];
        xmin = static_cast<int>(x < xmin ? x : (float)xmin);
        xmax = static_cast<int>(x > xmax ? x : (float)xmax);
        ymin = static_cast<int>(y < ymin ? y : (float)ymin);
        ymax = static_cast<int>(y > ymax ? y : (float)ymax);
    }
    xmin -= 30; xmax += 30;
    ymin -= 30; ymax += 30;
    out->x0 = xmin <= 0 ? 0 : xmin;
    out->y0 = ymin <= 0 ? 0 : ymin;
    out->x1 = xmax >= w - 1 ? w - 1 : xmax;
    out->y1 = ymax >= hgt - 1 ? hgt - 1 : ymax;
    // rowRange(y0, y1).colRange(x0, x1) asserts start <= end (CV_Assert stays in release)
    return rect_ok(out) ? ORBFE_OK : ORBFE_ERR_UNSUPPORTED;
}

int orbfe_profile(orbfe_extractor* h, int enable) {
    if (!h) return ORBFE_ERR_ARG;
    if (enable < 0 || (enable > 1 && (enable & 1))) return ORBFE_ERR_ARG;
    h->prof.on = enable != 0;
    h->prof.mask = enable > 1 ? (unsigned)enable >> 1 : ~0u;
    h->prof.used = 0;
    return ORBFE_OK;
}

int orbfe_profile_read(orbfe_extractor* h, double* total_ms, int32_t* launches) {
    if (!h || !total_ms || !launches) return ORBFE_ERR_ARG;
    DeviceGuard dg(h->device);
    ORBFE_HIP(hipStreamSynchronize(h->stream));
    for (int k = 0; k < ORBFE_STAGE_COUNT; ++k) {
        total_ms[k] = 0;
        launches[k] = 0;
    }
    for (size_t i = 0; i < h->prof.used; ++i) {
        float ms = 0.f;
        ORBFE_HIP(hipEventElapsedTime(&ms, h->prof.a[i], h->prof.b[i]));
        total_ms[h->prof.kind[i]] += ms;
        launches[h->prof.kind[i]] += 1;
    }
    h->prof.used = 0;
    return ORBFE_OK;
}

// Test / measurement hook (no reference counterpart): relaunch the stages in `stage_mask`
// (bit ORBFE_STAGE_*) of the most recent device-batch extraction on the handle's stream, on
// that extraction's buffers, `reps` times, asynchronously.  A stage alone reads what the
// previous stages left (the replayed FAST re-adds its per-level key totals, which only the
// oct-tree reads), so the outputs are only meaningful for a full mask; used to time kernels of
// different stages running concurrently on two handles.
int orbfe_debug_replay(orbfe_extractor* h, unsigned stage_mask, int reps) {
    if (!h || !h->planned || h->last_run.n < 1 || reps < 0 || !h->last_run.kps) return ORBFE_ERR_ARG;
    DeviceGuard dg(h->device);
    const auto r = h->last_run;
    // FAST adds its per-level key totals into level_keys and the oct-tree reads and clears them
    // (0 between calls).  A FAST replay without the oct-tree starts from zero each time; an
    // oct-tree replay without FAST restores one FAST's totals (recomputed once) before each
    // launch; both leave the totals at zero, as a full extraction does.
    const bool fast = (stage_mask >> ORBFE_STAGE_FAST) & 1u, oct = (stage_mask >> ORBFE_STAGE_OCTREE) & 1u;
    const size_t lk = (size_t)r.n * kMaxLevels * sizeof(int);
    int st = ORBFE_OK;
    auto hip = [&](hipError_t e) { if (e != hipSuccess && st == ORBFE_OK) st = ORBFE_ERR_HIP; };
    if (oct && !fast) {
        if ((st = h->lk_snap.ensure(lk))) return st;
        h->prof.run_mask = 1u << ORBFE_STAGE_FAST;
        hip(hipMemsetAsync(h->level_keys.p, 0, lk, h->stream));
        if (st == ORBFE_OK) st = h->run(r.n, r.l0, r.kps, r.cap, r.desc, r.nout);
        hip(hipMemcpyAsync(h->lk_snap.p, h->level_keys.p, lk, hipMemcpyDeviceToDevice, h->stream));
    }
    h->prof.run_mask = stage_mask;
    for (int i = 0; i < reps && st == ORBFE_OK; ++i) {
        if (fast && !oct) hip(hipMemsetAsync(h->level_keys.p, 0, lk, h->stream));
        if (oct && !fast) hip(hipMemcpyAsync(h->level_keys.p, h->lk_snap.p, lk, hipMemcpyDeviceToDevice, h->stream));
        if (st == ORBFE_OK) st = h->run(r.n, r.l0, r.kps, r.cap, r.desc, r.nout);
    }
    if (fast != oct) hip(hipMemsetAsync(h->level_keys.p, 0, lk, h->stream));
    h->prof.run_mask = h->stage_mask;
    return st;
}

int orbfe_set_stage_mask(orbfe_extractor* h, unsigned stage_mask) {
    if (!h) return ORBFE_ERR_ARG;
    h->stage_mask = stage_mask ? stage_mask : ~0u;
    h->prof.run_mask = h->stage_mask;
    return ORBFE_OK;
}

int orbfe_pyramid_path(const orbfe_extractor* h, int nframes) {
    if (!h || !h->planned || nframes < 1) return ORBFE_ERR_ARG;
    return h->band_path(nframes) ? ORBFE_PYR_BANDS : ORBFE_PYR_PER_LEVEL;
}

int orbfe_set_stream(orbfe_extractor* h, void* s) {
    if (!h) return ORBFE_ERR_ARG;
    h->stream = s ? static_cast<hipStream_t>(s) : h->own;
    return ORBFE_OK;
}

int orbfe_synchronize(orbfe_extractor* h) {
    if (!h) return ORBFE_ERR_ARG;
    DeviceGuard dg(h->device);
    return hipStreamSynchronize(h->stream) == hipSuccess ? ORBFE_OK : ORBFE_ERR_HIP;
}

static int copy_level(orbfe_extractor* h, const LevelPtr& lp, int frame, int level, uint8_t* out,
                      int* w, int* hgt) {
    const LevelGeo& lv = h->plan.geo.lv[level];
    if (w) *w = lv.w;
    if (hgt) *hgt = lv.h;
    if (!out) return ORBFE_OK;
    DeviceGuard dg(h->device);
    ORBFE_HIP(hipMemcpy2DAsync(out, lv.w, lp.base + frame * lp.fpitch, lp.pitch, lv.w, lv.h,
                               hipMemcpyDeviceToHost, h->stream));
    ORBFE_HIP(hipStreamSynchronize(h->stream));
    return ORBFE_OK;
}

int orbfe_get_level(orbfe_extractor* h, int frame, int level, uint8_t* out, int* w, int* hgt) {
    if (!h || !h->planned || frame < 0 || frame >= h->last_n || level < 0 ||
        level >= h->tab.p.nlevels)
        return ORBFE_ERR_ARG;
    return copy_level(h, h->last_pyr[level], frame, level, out, w, hgt);
}

int orbfe_get_blurred_level(orbfe_extractor* h, int frame, int level, uint8_t* out, int* w,
                            int* hgt) {
    if (!h || !h->planned || frame < 0 || frame >= h->last_n || level < 0 ||
        level >= h->tab.p.nlevels)
        return ORBFE_ERR_ARG;
    const Plan& g = h->plan;
    const LevelGeo& lv = g.geo.lv[level];
    LevelPtr bp{h->blur.as<uint8_t>() + lv.off, g.slab, lv.pitch};
    // K4 on demand (the default extraction path blurs level 0 and the tail levels inside K5);
    // ORBFE_PROBE_AS_EXTRACTED=1 copies the slab as the extraction left it (the levels
    // ORBFE_PREBLUR's pass made)
    if (out && !std::getenv("ORBFE_PROBE_AS_EXTRACTED")) {
        DeviceGuard dg(h->device);
        BlurArgs ba;
        ba.nlevels = g.geo.nlevels;
        for (int l = 0; l < ba.nlevels; ++l) {
            ba.w[l] = g.geo.lv[l].w;
            ba.h[l] = g.geo.lv[l].h;
            ba.src[l] = h->last_pyr[l];
            ba.dst[l] = LevelPtr{h->blur.as<uint8_t>() + g.geo.lv[l].off, g.slab, g.geo.lv[l].pitch};
            ba.simd_xb[l] = h->x86() ? sse2_body_blur(g.geo.lv[l].w) : 0;
        }
        ba.frags = h->bslot.as<uint4>();
        ba.items = reinterpret_cast<const uint32_t*>(h->bslot.as<uint8_t>() + kBlurFragBytes);
        ba.nitems = (int)g.bitems.size();
        for (int i = 0; i < 4; ++i) ba.taps[i] = h->tab.taps[i];
        if (h->x86())
            hipLaunchKernelGGL(blur_mfma_kernel<true>, dim3(ba.nitems, h->last_n), dim3(256), 0, h->stream, ba);
        else
            hipLaunchKernelGGL(blur_mfma_kernel<false>, dim3(ba.nitems, h->last_n), dim3(256), 0, h->stream, ba);
        ORBFE_HIP(hipGetLastError());
    }
    return copy_level(h, bp, frame, level, out, w, hgt);
}

int orbfe_get_fast_keys(orbfe_extractor* h, int frame, int level, orbfe_keypoint* out, int cap,
                        int* n_out) {
    if (!h || !h->planned || frame < 0 || frame >= h->last_n || level < 0 ||
        level >= h->tab.p.nlevels || !n_out)
        return ORBFE_ERR_ARG;
    DeviceGuard dg(h->device);
    const Plan& g = h->plan;
    const LevelGeo& lv = g.geo.lv[level];
    const int nc = lv.cell_end - lv.cell_begin;
    std::vector<int> cnt(std::max(nc, 1));
    std::vector<uint32_t> keys(std::max<long long>(1, lv.key_cap));
    if (nc > 0) {
        ORBFE_HIP(hipMemcpyAsync(cnt.data(), h->cell_cnt.as<int>() + (size_t)frame * g.cells.size() + lv.cell_begin,
                                 nc * sizeof(int), hipMemcpyDeviceToHost, h->stream));
        ORBFE_HIP(hipMemcpyAsync(keys.data(), h->cell_keys.as<uint32_t>() + (size_t)frame * g.cell_cap_total +
                                     g.cells[lv.cell_begin].slot,
                                 lv.key_cap * sizeof(uint32_t), hipMemcpyDeviceToHost, h->stream));
    }
    ORBFE_HIP(hipStreamSynchronize(h->stream));
    int n = 0;
    for (int c = 0; c < nc; ++c) n += cnt[c];
    *n_out = n;
    if (n > cap) return ORBFE_ERR_CAPACITY;
    int o = 0;
    for (int c = 0; c < nc; ++c) {
        const long long base = g.cells[lv.cell_begin + c].slot - g.cells[lv.cell_begin].slot;
        for (int i = 0; i < cnt[c]; ++i) {
            const uint32_t k = keys[base + i];
            out[o++] = orbfe_keypoint{(float)key_x(k), (float)key_y(k), 7.f, -1.f,
                                      (float)key_score(k), 0, -1};
        }
    }
    return ORBFE_OK;
}

}  // extern "C"
