// orbfe_api.hip — host orchestration and the C ABI of the extractor (include/orbfe.h).
// Replaces ORBextractor's public surface (ORBextractor.h:56-90); see the header for the
// per-function citations.  No CPU compute path exists: every result comes from the kernels.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <algorithm>
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
    std::vector<hipEvent_t> a, b;
    std::vector<int> kind;
    size_t used = 0;
    // Returns the event pair for the next launch of stage k (nullptrs when off).
    void slot(int k, hipEvent_t* e0, hipEvent_t* e1) {
        *e0 = *e1 = nullptr;
        if (!on) return;
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
    Plan plan;
    bool planned = false;
    int frames_cap = 0;
    DevBuf cells, xtab, ytab;
    DevBuf pyr, blur, cell_cnt, cell_keys, keys, act, oct_out, oct_cnt;
    DevBuf out_kps, out_desc, out_n;  // staging for the host-pointer entry points
    // last run, for the probes
    int last_n = 0;
    LevelPtr last_pyr[kMaxLevels] = {};
    Profiler prof;
    std::vector<orbfe_keypoint> h_kps;
    std::vector<uint8_t> h_desc;
    std::vector<int32_t> h_n;

    int set_plan(int w, int h) {
        if (planned && plan.w == w && plan.h == h) return ORBFE_OK;
        Plan g;
        int st = plan_geometry(tab, w, h, g);
        if (st != ORBFE_OK) return st;
        if ((st = cells.ensure(std::max<size_t>(1, g.cells.size()) * sizeof(CellDesc)))) return st;
        if ((st = xtab.ensure(std::max<size_t>(1, g.xtab.size()) * sizeof(int)))) return st;
        if ((st = ytab.ensure(std::max<size_t>(1, g.ytab.size()) * sizeof(int)))) return st;
        ORBFE_HIP(hipMemcpyAsync(cells.p, g.cells.data(), g.cells.size() * sizeof(CellDesc),
                                 hipMemcpyHostToDevice, stream));
        ORBFE_HIP(hipMemcpyAsync(xtab.p, g.xtab.data(), g.xtab.size() * sizeof(int),
                                 hipMemcpyHostToDevice, stream));
        ORBFE_HIP(hipMemcpyAsync(ytab.p, g.ytab.data(), g.ytab.size() * sizeof(int),
                                 hipMemcpyHostToDevice, stream));
        ORBFE_HIP(hipStreamSynchronize(stream));
        plan = std::move(g);
        planned = true;
        frames_cap = 0;  // workspace sizes depend on the plan
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
        frames_cap = n;
        return ORBFE_OK;
    }

    // Runs the whole pipeline on `n` frames whose level 0 is described by `l0`.
    int run(int n, LevelPtr l0, orbfe_keypoint* d_kps, int kps_cap, uint8_t* d_desc,
            int32_t* d_n) {
        const Plan& g = plan;
        const int L = g.geo.nlevels;
        LevelPtr lp[kMaxLevels], bp[kMaxLevels];
        for (int l = 0; l < L; ++l) {
            const LevelGeo& lv = g.geo.lv[l];
            lp[l] = LevelPtr{pyr.as<uint8_t>() + lv.off, g.slab, lv.pitch};
            bp[l] = LevelPtr{blur.as<uint8_t>() + lv.off, g.slab, lv.pitch};
        }
        lp[0] = l0;
        // K1 cascaded pyramid: one launch per level, 128 x 32 tiles of every frame
        for (int l = 1; l < L; ++l) {
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
            ORBFE_LAUNCH(prof, ORBFE_STAGE_RESIZE, resize_kernel, dim3(g.rs_tiles[l], n), dim3(256),
                         g.rs_lds[l], stream, ra);
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
            for (int l = 0; l < L; ++l) fa.pyr[l] = lp[l];
            ORBFE_LAUNCH(prof, ORBFE_STAGE_FAST, fast_kernel, dim3(ncells, n), dim3(kFastBlockSize), g.fast_lds, stream, fa);
        }
        // K3 oct-tree per (frame, level)
        OctArgs oa;
        oa.geo = g.geo;
        oa.cells = cells.as<CellDesc>();
        oa.ncells = ncells;
        oa.cell_cap_total = g.cell_cap_total;
        oa.cell_cnt = cell_cnt.as<int>();
        oa.cell_keys = cell_keys.as<uint32_t>();
        oa.keys = keys.as<uint32_t>();
        oa.act = act.as<int4>();
        oa.oct_out = oct_out.as<uint32_t>();
        oa.oct_cnt = oct_cnt.as<int>();
        oa.ncap_max = g.ncap_max;
        oa.sort_cap = g.sort_cap;
        ORBFE_LAUNCH(prof, ORBFE_STAGE_OCTREE, octree_kernel, dim3(L, n), dim3(kOctBlockSize), g.oct_lds, stream, oa);
        // K4 blur
        BlurArgs ba;
        ba.nlevels = L;
        for (int l = 0; l < L; ++l) {
            ba.tile_begin[l] = g.tile_begin[l];
            ba.w[l] = g.geo.lv[l].w;
            ba.h[l] = g.geo.lv[l].h;
            ba.src[l] = lp[l];
            ba.dst[l] = bp[l];
        }
        for (int i = 0; i < 4; ++i) ba.taps[i] = tab.taps[i];
        ORBFE_LAUNCH(prof, ORBFE_STAGE_BLUR, blur_kernel, dim3(g.tiles_total, n), dim3(256), 0, stream, ba);
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
        }
        da.oct_out = oct_out.as<uint32_t>();
        da.oct_cnt = oct_cnt.as<int>();
        da.kps = d_kps;
        da.desc = d_desc;
        da.n_out = d_n;
        const int per_block = (kDescBlockSize / 64) * kDescGroupSize;  // slots per workgroup
        ORBFE_LAUNCH(prof, ORBFE_STAGE_DESCRIBE, describe_kernel, dim3((g.geo.out_total + per_block - 1) / per_block, n),
                           dim3(kDescBlockSize), 0, stream, da);
        ORBFE_HIP(hipGetLastError());
        last_n = n;
        for (int l = 0; l < L; ++l) last_pyr[l] = lp[l];
        return ORBFE_OK;
    }

    // Host-pointer path: upload, run into the staging slabs, download.
    int run_host(const uint8_t* const* imgs, int n, int w, int h, size_t stride,
                 const uint8_t* const* masks, size_t mstride) {
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
        for (int f = 0; f < n; ++f) {
            uint8_t* dst = pyr.as<uint8_t>() + (size_t)f * g.slab + l0.off;
            ORBFE_HIP(hipMemcpy2DAsync(dst, l0.pitch, imgs[f], stride, w, h,
                                       hipMemcpyHostToDevice, stream));
            if (masks && masks[f]) any_mask = true;
        }
        if (any_mask) {
            // the blur slab is free until K4: stage the masks there, then zero masked pixels
            for (int f = 0; f < n; ++f) {
                uint8_t* mdst = blur.as<uint8_t>() + (size_t)f * g.slab + l0.off;
                if (masks[f]) {
                    ORBFE_HIP(hipMemcpy2DAsync(mdst, l0.pitch, masks[f], mstride, w, h,
                                               hipMemcpyHostToDevice, stream));
                } else {
                    ORBFE_HIP(hipMemset2DAsync(mdst, l0.pitch, 1, w, h, stream));
                }
            }
            uint8_t* p0 = pyr.as<uint8_t>() + l0.off;
            hipLaunchKernelGGL(mask_kernel, dim3((w + 255) / 256, h, n), dim3(256), 0, stream,
                               p0, g.slab, l0.pitch, blur.as<uint8_t>() + l0.off, g.slab,
                               l0.pitch, p0, g.slab, l0.pitch, w, h);
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
        for (DevBuf* b : {&cells, &xtab, &ytab, &pyr, &blur, &cell_cnt, &cell_keys, &keys, &act,
                          &oct_out, &oct_cnt, &out_kps, &out_desc, &out_n})
            b->release();
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
    // per-level list bound max(N + 4, 20) (nIni <= 4 is enforced), summed over levels
    int c = 0;
    for (int l = 0; l < h->tab.p.nlevels; ++l) c += std::max(h->tab.nfeat[l] + 4, 20);
    return c;
}

static int extract_host_common(orbfe_extractor* h, const uint8_t* const* imgs, int n, int w,
                               int hgt, size_t stride, const uint8_t* const* masks,
                               size_t mask_stride, orbfe_keypoint* kps, int kps_cap,
                               uint8_t* desc, int32_t* n_out) {
    DeviceGuard dg(h->device);
    int st = h->run_host(imgs, n, w, hgt, stride, masks, mask_stride);
    if (st != ORBFE_OK) return st;
    const int cap = h->kp_capacity();
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

int orbfe_extract(orbfe_extractor* h, const uint8_t* img, int w, int hgt, size_t stride,
                  const uint8_t* mask, size_t mask_stride, orbfe_keypoint* kps, int kps_cap,
                  uint8_t* desc, int* n_out) {
    if (!h) return ORBFE_ERR_ARG;
    if (!img || w <= 0 || hgt <= 0) return ORBFE_OK;  // empty image: no-op (1045-1046)
    if (!kps || !n_out || kps_cap < 0 || stride < (size_t)w || (mask && mask_stride < (size_t)w))
        return ORBFE_ERR_ARG;
    try {
        const uint8_t* m[1] = {mask};
        int32_t cnt = 0;
        const int st = extract_host_common(h, &img, 1, w, hgt, stride, mask ? m : nullptr,
                                           mask_stride, kps, kps_cap, desc, &cnt);
        *n_out = cnt;
        return st;
    } catch (const std::bad_alloc&) {
        return ORBFE_ERR_NOMEM;
    } catch (...) {
        return ORBFE_ERR_HIP;
    }
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
        return extract_host_common(h, imgs, n, w, hgt, stride, masks, mask_stride, kps, kps_cap,
                                   desc, n_out);
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
    if (!h || n < 0 || !d_imgs || !d_kps || !d_desc || !d_n_out) return ORBFE_ERR_ARG;
    if (n == 0 || w <= 0 || hgt <= 0) return ORBFE_OK;
    if (stride < (size_t)w || (n > 1 && frame_pitch < stride * hgt)) return ORBFE_ERR_ARG;
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
        if (!aligned && !d_masks) {  // kernels read level 0 as dwords: stage it in the slab
            for (int f = 0; f < n; ++f)
                ORBFE_HIP(hipMemcpy2DAsync(h->pyr.as<uint8_t>() + (size_t)f * g.slab + l0.off, l0.pitch,
                                           d_imgs + (size_t)f * frame_pitch, stride, w, hgt,
                                           hipMemcpyDeviceToDevice, h->stream));
            lp0 = LevelPtr{h->pyr.as<uint8_t>() + l0.off, g.slab, l0.pitch};
        }
        if (d_masks) {
            uint8_t* p0 = h->pyr.as<uint8_t>() + l0.off;
            ORBFE_LAUNCH(h->prof, ORBFE_STAGE_MASK, mask_kernel, dim3((w + 255) / 256, hgt, n), dim3(256), 0,
                               h->stream, d_imgs, (long long)frame_pitch, (int)stride, d_masks,
                               (long long)frame_pitch, (int)stride, p0, g.slab, l0.pitch, w, hgt);
            lp0 = LevelPtr{p0, g.slab, l0.pitch};
        }
        return h->run(n, lp0, d_kps, kps_cap, d_desc, d_n_out);
    } catch (...) {
        return ORBFE_ERR_HIP;
    }
}

int orbfe_profile(orbfe_extractor* h, int enable) {
    if (!h) return ORBFE_ERR_ARG;
    h->prof.on = enable != 0;
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
    const LevelGeo& lv = h->plan.geo.lv[level];
    LevelPtr bp{h->blur.as<uint8_t>() + lv.off, h->plan.slab, lv.pitch};
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
