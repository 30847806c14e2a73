// GPU parity check of the C++ adapter (include/orbfe_orbslam.hpp) against the CPU oracle, as
// C++ host code of the reference would use it.  Built by __graft_entry__.build(); run by
// tests/test_gpu_cpp.py on the MI355X.  Prints "ADAPTER PASS" on success.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

#include "../../include/orbfe_orbslam.hpp"
#include "../../oracle/orb_oracle.h"

static std::vector<uint8_t> make_image(int w, int h, unsigned seed) {
    std::vector<uint8_t> img((size_t)w * h);
    unsigned s = seed * 2654435761u + 12345u;
    auto rnd = [&]() { s = s * 1664525u + 1013904223u; return (s >> 8) & 0xffff; };
    for (int y = 0; y < h; ++y)
        for (int x = 0; x < w; ++x)
            img[(size_t)y * w + x] = (uint8_t)(128 + 60 * std::sin(x * 0.05) * std::cos(y * 0.07));
    for (int r = 0; r < 150; ++r) {  // random rectangles: corners for FAST
        const int x0 = rnd() % w, y0 = rnd() % h, rw = 5 + rnd() % 50, rh = 5 + rnd() % 50;
        const uint8_t g = (uint8_t)(rnd() & 255);
        for (int y = y0; y < std::min(h, y0 + rh); ++y)
            for (int x = x0; x < std::min(w, x0 + rw); ++x) img[(size_t)y * w + x] = g;
    }
    return img;
}

int main() {
    const int W = 640, H = 480;
    int fails = 0;
    orbfe::ORBextractor ex(1000, 1.2f, 8, 32, 7);
    orbfe_params p{1000, 1.2f, 8, 32, 7};
    for (unsigned seed = 0; seed < 3; ++seed) {
        std::vector<uint8_t> img = make_image(W, H, seed);
        std::vector<orbfe_keypoint> kps;
        std::vector<uint8_t> desc;
        ex(img.data(), W, H, W, nullptr, 0, kps, desc);
        std::vector<orbfe_keypoint> okps(2000);
        std::vector<uint8_t> odesc(2000 * 32);
        int n = 0;
        if (oracle_extract(&p, img.data(), W, H, W, nullptr, 0, okps.data(), 2000, odesc.data(), &n)) return 2;
        const bool same = (int)kps.size() == n && !std::memcmp(kps.data(), okps.data(), n * sizeof(orbfe_keypoint)) &&
                          !std::memcmp(desc.data(), odesc.data(), (size_t)n * 32);
        std::printf("seed %u: %zu keypoints (oracle %d) %s\n", seed, kps.size(), n, same ? "bit-exact" : "MISMATCH");
        fails += !same;
        // the zero-copy form: the frame written into the staging buffer, outputs read in place
        size_t step = 0;
        uint8_t* buf = ex.InputBuffer(W, H, &step);
        for (int y = 0; y < H; ++y) std::memcpy(buf + (size_t)y * step, img.data() + (size_t)y * W, W);
        std::vector<orbfe_keypoint> skps;
        std::vector<uint8_t> sdesc;
        ex.ExtractStaged(W, H, skps, sdesc);
        const bool same_staged = (int)skps.size() == n && !std::memcmp(skps.data(), okps.data(), n * sizeof(orbfe_keypoint)) &&
                                 !std::memcmp(sdesc.data(), odesc.data(), (size_t)n * 32);
        std::printf("seed %u staged: %zu keypoints %s\n", seed, skps.size(), same_staged ? "bit-exact" : "MISMATCH");
        fails += !same_staged;
    }
    // single-frame latency from a C++ caller (Frame::ExtractORB's position): the host form
    // (frame copied into the staging buffer by the call) and the staged form (frame already in
    // the staging buffer: the caller's cvtColor target; outputs read in place, or copied into
    // the adapter's vectors as Frame keeps them).  Mean over 2,000 calls after 100 warm-up calls.
    {
        std::vector<uint8_t> img = make_image(W, H, 5);
        std::vector<orbfe_keypoint> kps;
        std::vector<uint8_t> desc;
        size_t step = 0;
        uint8_t* buf = ex.InputBuffer(W, H, &step);
        for (int y = 0; y < H; ++y) std::memcpy(buf + (size_t)y * step, img.data() + (size_t)y * W, W);
        auto mean_us = [&](auto&& call) {
            for (int i = 0; i < 100; ++i) call();
            const auto t0 = std::chrono::steady_clock::now();
            for (int i = 0; i < 2000; ++i) call();
            return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / 2000;
        };
        const double host_us = mean_us([&] { ex(img.data(), W, H, W, nullptr, 0, kps, desc); });
        const double staged_copy_us = mean_us([&] { ex.ExtractStaged(W, H, kps, desc); });
        const double staged_us = mean_us([&] {
            int n = 0;
            const orbfe_keypoint* k = nullptr;
            const uint8_t* d = nullptr;
            if (orbfe_extract_staged(ex.handle(), W, H, nullptr, 0, nullptr, &n) ||
                orbfe_staged_outputs(ex.handle(), &k, &d, &n))
                ++fails;
        });
        std::printf("LATENCY host_us=%.2f staged_copy_us=%.2f staged_us=%.2f\n", host_us, staged_copy_us, staged_us);
    }
    // scale tables through the getters
    std::vector<float> sf = ex.GetScaleFactors(), osf(8);
    oracle_tables(&p, osf.data(), nullptr, nullptr, nullptr, nullptr, nullptr);
    fails += std::memcmp(sf.data(), osf.data(), 8 * sizeof(float)) != 0;
    // SearchForInitialization on two extracted frames
    orbfe::ORBextractor ini(2000, 1.2f, 8, 32, 7);
    orbfe::FrameData F1, F2;
    std::vector<uint8_t> i1 = make_image(W, H, 7), i2 = make_image(W, H, 7);
    std::memmove(i2.data() + 3, i2.data(), i2.size() - 3);  // shifted view
    ini(i1.data(), W, H, W, nullptr, 0, F1.keys_un, F1.descriptors);
    ini(i2.data(), W, H, W, nullptr, 0, F2.keys_un, F2.descriptors);
    for (orbfe::FrameData* F : {&F1, &F2}) {
        F->max_x = W;
        F->max_y = H;
        F->scale_factors = sf;
    }
    orbfe::ORBmatcher matcher(0.9f, true);
    std::vector<float> prev, oprev;
    for (const orbfe_keypoint& k : F1.keys_un) { prev.push_back(k.x); prev.push_back(k.y); }
    oprev = prev;
    std::vector<int> m12, om12(F1.keys_un.size());
    const int nm = matcher.SearchForInitialization(F1, F2, prev, m12, 100);
    int onm = 0;
    const orbfe_frame_view v1 = F1.view(), v2 = F2.view();
    oracle_search_for_initialization(0.9f, 1, &v1, &v2, oprev.data(), 100, om12.data(), &onm);
    const bool sfi_same = nm == onm && m12 == om12 && prev == oprev;
    std::printf("SearchForInitialization: %d matches (oracle %d) %s\n", nm, onm, sfi_same ? "exact" : "MISMATCH");
    fails += !sfi_same;
    // SearchByBoW(KeyFrame*, Frame&) on two 1000-keypoint views of one scene: FeatureVectors with
    // a feature's node given by its descriptor's first byte (64 nodes, ~16 features each, ids
    // ascending, features in index order as DBoW2 fills them); every fifth keyframe feature has
    // no good MapPoint.  Parity against the oracle, then the latency of both from C++ (mean over
    // 2,000 calls after 100 warm-up calls; the CPU port single-threaded).
    {
        orbfe::FrameData K, F;
        std::vector<uint8_t> b1 = make_image(W, H, 11), b2 = make_image(W, H, 11);
        std::memmove(b2.data() + 2 * W + 2, b2.data(), b2.size() - 2 * W - 2);  // shifted view
        ex(b1.data(), W, H, W, nullptr, 0, K.keys_un, K.descriptors);
        ex(b2.data(), W, H, W, nullptr, 0, F.keys_un, F.descriptors);
        struct Fv { std::vector<int32_t> ids, off, feat; };
        auto make_fv = [](const std::vector<uint8_t>& d, int n) {
            std::vector<std::vector<int32_t>> nodes(64);
            for (int i = 0; i < n; ++i) nodes[d[32 * (size_t)i] >> 2].push_back(i);
            Fv v;
            v.off.push_back(0);
            for (int k = 0; k < 64; ++k) {
                if (nodes[k].empty()) continue;
                v.ids.push_back(k);
                v.feat.insert(v.feat.end(), nodes[k].begin(), nodes[k].end());
                v.off.push_back((int32_t)v.feat.size());
            }
            return v;
        };
        const int nk = (int)K.keys_un.size(), nf = (int)F.keys_un.size();
        const Fv kfv = make_fv(K.descriptors, nk), ffv = make_fv(F.descriptors, nf);
        const orbfe::FeatureVectorView kv{kfv.ids.data(), kfv.off.data(), kfv.feat.data(), (int)kfv.ids.size()};
        const orbfe::FeatureVectorView fv{ffv.ids.data(), ffv.off.data(), ffv.feat.data(), (int)ffv.ids.size()};
        std::vector<uint8_t> ok(nk);
        for (int i = 0; i < nk; ++i) ok[i] = i % 5 != 0;
        std::vector<float> ka(nk), fa(nf);
        for (int i = 0; i < nk; ++i) ka[i] = K.keys_un[i].angle;
        for (int i = 0; i < nf; ++i) fa[i] = F.keys_un[i].angle;
        orbfe::ORBmatcher bm(0.75f, true);
        std::vector<int> mg;
        const int ng = bm.SearchByBoW(K, ok, kv, F, fv, mg);
        std::vector<int32_t> mo(nf, -1);
        int no = 0;
        auto cpu = [&] {
            return oracle_search_by_bow(0.75f, 1, K.descriptors.data(), ka.data(), ok.data(), kfv.ids.data(),
                                        kfv.off.data(), kfv.feat.data(), kv.nn, nf, F.descriptors.data(),
                                        fa.data(), ffv.ids.data(), ffv.off.data(), ffv.feat.data(), fv.nn,
                                        mo.data(), &no);
        };
        if (cpu()) return 2;
        const bool bow_same = ng == no && std::equal(mg.begin(), mg.end(), mo.begin());
        std::printf("SearchByBoW: %d matches (oracle %d) %s\n", ng, no, bow_same ? "exact" : "MISMATCH");
        fails += !bow_same;
        auto mean_us = [&](auto&& call) {
            for (int i = 0; i < 100; ++i) call();
            const auto t0 = std::chrono::steady_clock::now();
            for (int i = 0; i < 2000; ++i) call();
            return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / 2000;
        };
        const double gpu_us = mean_us([&] { bm.SearchByBoW(K, ok, kv, F, fv, mg); });
        const double cpu_us = mean_us([&] { fails += cpu() != 0; });
        std::printf("BOW_LATENCY gpu_us=%.2f cpu_us=%.2f nodes=%d/%d\n", gpu_us, cpu_us, kv.nn, fv.nn);
    }
    std::printf(fails ? "ADAPTER FAIL\n" : "ADAPTER PASS\n");
    return fails ? 1 : 0;
}
