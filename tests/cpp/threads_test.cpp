// Concurrency of the C ABI's handles (include/orbfe.h: distinct handles may be used from
// different threads at once), in the reference's own pattern:
//   * Tracking owns three extractors — Left and Right at nFeatures, Ini at 2 x nFeatures
//     (Tracking.cc:208-215) — and a stereo Frame extracts left and right on two std::threads
//     that it joins (Frame.cc:78-81);
//   * here, while the stereo pairs run, a third thread drives the Ini extractor (monocular
//     initialisation frames) and a fourth a matcher (SearchForInitialization and brute force,
//     as the LocalMapping / LoopClosing threads call ORBmatcher concurrently with Tracking).
// Every output of every iteration is compared with the oracle's, computed single-threaded
// beforehand.  Built by __graft_entry__.build(); run by tests/test_gpu_threads.py on the
// MI355X.  Prints "THREADS PASS" on success.
#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>

#include "../../include/orbfe_orbslam.hpp"
#include "../../oracle/orb_oracle.h"

namespace {

std::vector<uint8_t> make_image(int w, int h, unsigned seed) {
    std::vector<uint8_t> img((size_t)w * h);
    unsigned s = seed * 2654435761u + 12345u;
    auto rnd = [&]() { s = s * 1664525u + 1013904223u; return (s >> 8) & 0xffff; };
    for (int y = 0; y < h; ++y)
        for (int x = 0; x < w; ++x)
            img[(size_t)y * w + x] = (uint8_t)(128 + 60 * std::sin(x * 0.05 + seed) * std::cos(y * 0.07));
    for (int r = 0; r < 150; ++r) {
        const int x0 = rnd() % w, y0 = rnd() % h, rw = 5 + rnd() % 50, rh = 5 + rnd() % 50;
        const uint8_t g = (uint8_t)(rnd() & 255);
        for (int y = y0; y < std::min(h, y0 + rh); ++y)
            for (int x = x0; x < std::min(w, x0 + rw); ++x) img[(size_t)y * w + x] = g;
    }
    return img;
}

struct Expected {
    std::vector<orbfe_keypoint> kps;
    std::vector<uint8_t> desc;
};

Expected oracle_of(const orbfe_params& p, const std::vector<uint8_t>& img, int w, int h) {
    Expected e;
    const int cap = p.nfeatures + 3 * p.nlevels + 64;
    e.kps.resize(cap);
    e.desc.resize((size_t)cap * 32);
    int n = 0;
    if (oracle_extract(&p, img.data(), w, h, w, nullptr, 0, e.kps.data(), cap, e.desc.data(), &n)) n = -1;
    e.kps.resize(n < 0 ? 0 : n);
    e.desc.resize((size_t)(n < 0 ? 0 : n) * 32);
    return e;
}

bool same(const std::vector<orbfe_keypoint>& k, const std::vector<uint8_t>& d, const Expected& e) {
    return k.size() == e.kps.size() && d.size() == e.desc.size() &&
           !std::memcmp(k.data(), e.kps.data(), k.size() * sizeof(orbfe_keypoint)) &&
           !std::memcmp(d.data(), e.desc.data(), d.size());
}

}  // namespace

int main(int argc, char** argv) {
    const int W = 640, H = 480;
    const int iters = argc > 1 ? std::atoi(argv[1]) : 60;
    const int kImgs = 6;
    const orbfe_params p1{1000, 1.2f, 8, 20, 7}, p2{2000, 1.2f, 8, 20, 7};
    std::vector<std::vector<uint8_t>> left, right;
    std::vector<Expected> eL, eR, eI;
    for (int i = 0; i < kImgs; ++i) {
        left.push_back(make_image(W, H, 100 + i));
        right.push_back(make_image(W, H, 200 + i));
        eL.push_back(oracle_of(p1, left[i], W, H));
        eR.push_back(oracle_of(p1, right[i], W, H));
        eI.push_back(oracle_of(p2, left[i], W, H));
    }
    // the matcher thread's problem: SearchForInitialization between two Ini frames, and brute
    // force of frame 0's descriptors against frame 1's
    orbfe::FrameData F1, F2;
    F1.keys_un = eI[0].kps;
    F1.descriptors = eI[0].desc;
    F2.keys_un = eI[1].kps;
    F2.descriptors = eI[1].desc;
    std::vector<float> sf(8);
    oracle_tables(&p2, sf.data(), nullptr, nullptr, nullptr, nullptr, nullptr);
    for (orbfe::FrameData* F : {&F1, &F2}) {
        F->max_x = W;
        F->max_y = H;
        F->scale_factors = sf;
    }
    std::vector<float> prev0;
    for (const orbfe_keypoint& k : F1.keys_un) { prev0.push_back(k.x); prev0.push_back(k.y); }
    std::vector<float> oprev = prev0;
    std::vector<int> om12(F1.keys_un.size());
    int onm = 0;
    {
        const orbfe_frame_view v1 = F1.view(), v2 = F2.view();
        oracle_search_for_initialization(0.9f, 1, &v1, &v2, oprev.data(), 100, om12.data(), &onm);
    }
    if (const char* dump = std::getenv("THREADS_DUMP")) {  // the matcher problem, for debugging
        if (FILE* fp = std::fopen(dump, "wb")) {
            for (const orbfe::FrameData* F : {&F1, &F2}) {
                const int n = (int)F->keys_un.size();
                std::fwrite(&n, 4, 1, fp);
                std::fwrite(F->keys_un.data(), sizeof(orbfe_keypoint), n, fp);
                std::fwrite(F->descriptors.data(), 32, n, fp);
            }
            std::fclose(fp);
        }
    }
    const int nq = (int)F1.keys_un.size(), nr = (int)F2.keys_un.size();
    std::vector<int32_t> obi(nq), obd(nq), osd(nq);
    oracle_bf_match(F1.descriptors.data(), nq, F2.descriptors.data(), nr, obi.data(), obd.data(), osd.data());

    orbfe::ORBextractor exL(1000, 1.2f, 8, 20, 7), exR(1000, 1.2f, 8, 20, 7), exI(2000, 1.2f, 8, 20, 7);
    orbfe::ORBmatcher matcher(0.9f, true);
    std::atomic<int> fails{0}, done_ini{0}, done_match{0}, stereo_pairs{0};
    {   // the matcher's problem once on this thread before any concurrency
        std::vector<float> prev = prev0;
        std::vector<int> m12;
        const int nm = matcher.SearchForInitialization(F1, F2, prev, m12, 100);
        int diff = 0;
        for (size_t i = 0; i < m12.size(); ++i) diff += m12[i] != om12[i];
        std::printf("single-thread SearchForInitialization: %d matches (oracle %d), %d entries differ, "
                    "%zu / %zu keypoints\n", nm, onm, diff, F1.keys_un.size(), F2.keys_un.size());
        if (nm != onm || m12 != om12 || prev != oprev) ++fails;
    }
    std::atomic<bool> stop{false};
    // Ini extractor: its own thread for the whole run
    std::thread ini([&] {
        std::vector<orbfe_keypoint> k;
        std::vector<uint8_t> d;
        for (int i = 0; i < iters || !stop.load(); ++i) {
            const int f = i % kImgs;
            exI(left[f].data(), W, H, W, nullptr, 0, k, d);
            if (!same(k, d, eI[f])) {
                std::printf("Ini extractor iteration %d frame %d: MISMATCH (%zu vs %zu)\n", i, f, k.size(), eI[f].kps.size());
                ++fails;
            }
            ++done_ini;
        }
    });
    // matcher: its own thread for the whole run
    std::thread mt([&] {
        for (int i = 0; i < iters || !stop.load(); ++i) {
            std::vector<float> prev = prev0;
            std::vector<int> m12;
            const int nm = matcher.SearchForInitialization(F1, F2, prev, m12, 100);
            std::vector<int32_t> bi(nq), bd(nq), sd(nq);
            const int st = orbfe_bf_match(matcher.handle(), F1.descriptors.data(), nq, F2.descriptors.data(), nr,
                                          bi.data(), bd.data(), sd.data());
            if (nm != onm || m12 != om12 || prev != oprev || st || bi != obi || bd != obd || sd != osd) {
                std::printf("matcher iteration %d: MISMATCH (sfi %d vs %d, bf status %d)\n", i, nm, onm, st);
                ++fails;
            }
            ++done_match;
        }
    });
    // stereo frames: each pair on two std::threads joined by the frame (Frame.cc:78-81)
    for (int i = 0; i < iters; ++i) {
        const int f = i % kImgs;
        std::vector<orbfe_keypoint> kl, kr;
        std::vector<uint8_t> dl, dr;
        std::thread tl([&] { exL(left[f].data(), W, H, W, nullptr, 0, kl, dl); });
        std::thread tr([&] { exR(right[f].data(), W, H, W, nullptr, 0, kr, dr); });
        tl.join();
        tr.join();
        if (!same(kl, dl, eL[f]) || !same(kr, dr, eR[f])) {
            std::printf("stereo pair %d frame %d: MISMATCH\n", i, f);
            ++fails;
        }
        ++stereo_pairs;
    }
    stop = true;
    ini.join();
    mt.join();
    std::printf("stereo pairs %d, Ini extractions %d, matcher iterations %d, failures %d\n",
                stereo_pairs.load(), done_ini.load(), done_match.load(), fails.load());
    std::printf(fails ? "THREADS FAIL\n" : "THREADS PASS\n");
    return fails ? 1 : 0;
}
