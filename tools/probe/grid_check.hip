// Standalone check of the Frame grid kernels (Frame::AssignFeaturesToGrid): grid_lds_kernel and
// grid_kernel on random keypoints against a CPU CSR (cell = ix * 48 + iy, items in index order).
// The kernels only write cstart / citems inside their buffers, so a wrong grid is reported here
// instead of surfacing as a wild read in the matchers that consume it.
//   hipcc --offload-arch=gfx950 -O2 -std=c++17 -ffp-contract=off -w \
//       -o /tmp/grid_check tools/probe/grid_check.hip && /tmp/grid_check
#include "../../orbslam_mapsave_amd/csrc/orbfe_lib.hip"

#include <cstdio>
#include <random>

int main() {
    int bad = 0;
    for (int n : {1, 100, 1000, 1023, 1025, 4000, 8192, 9000}) {
        std::mt19937 rng(n);
        std::uniform_real_distribution<float> ux(-5.f, 645.f), uy(-5.f, 485.f);
        std::vector<orbfe_keypoint> k(n);
        for (auto& p : k) p = orbfe_keypoint{ux(rng), uy(rng), 31.f, 0.f, 0.f, 0, -1};
        const float gwi = 64.f / 640.f, ghi = 48.f / 480.f;
        // CPU reference
        std::vector<std::vector<int>> cells(orbfe::kGridCells);
        for (int i = 0; i < n; ++i) {
            const int gx = (int)std::round((k[i].x - 0.f) * gwi), gy = (int)std::round((k[i].y - 0.f) * ghi);
            if (gx >= 0 && gx < orbfe::kGridCols && gy >= 0 && gy < orbfe::kGridRows)
                cells[gx * orbfe::kGridRows + gy].push_back(i);
        }
        std::vector<int> rs(orbfe::kGridCells + 1), ri;
        for (int c = 0; c < orbfe::kGridCells; ++c) {
            rs[c] = (int)ri.size();
            ri.insert(ri.end(), cells[c].begin(), cells[c].end());
        }
        rs[orbfe::kGridCells] = (int)ri.size();
        orbfe_keypoint* dk;
        int *dcs, *dci, *dco;
        if (hipMalloc(&dk, n * sizeof(orbfe_keypoint)) || hipMalloc(&dcs, (orbfe::kGridCells + 1) * 4) ||
            hipMalloc(&dci, n * 4) || hipMalloc(&dco, n * 4))
            return 2;
        if (hipMemcpy(dk, k.data(), n * sizeof(orbfe_keypoint), hipMemcpyHostToDevice)) return 2;
        for (int variant = 0; variant < 2; ++variant) {
            if (variant == 0 && n > orbfe::kGridLdsMax) continue;
            if (hipMemset(dcs, 0xff, (orbfe::kGridCells + 1) * 4) || hipMemset(dci, 0xff, n * 4)) return 2;
            if (variant == 0)
                hipLaunchKernelGGL(orbfe::grid_lds_kernel, dim3(1), dim3(orbfe::kGridBlock), 0, nullptr,
                                   dk, n, 0.f, 0.f, gwi, ghi, dcs, dci);
            else
                hipLaunchKernelGGL(orbfe::grid_kernel, dim3(1), dim3(orbfe::kGridBlock), 0, nullptr,
                                   dk, n, 0.f, 0.f, gwi, ghi, dco, dcs, dci);
            if (hipDeviceSynchronize()) return 3;
            std::vector<int> gs(orbfe::kGridCells + 1), gi(n);
            if (hipMemcpy(gs.data(), dcs, gs.size() * 4, hipMemcpyDeviceToHost) ||
                hipMemcpy(gi.data(), dci, n * 4, hipMemcpyDeviceToHost))
                return 2;
            const bool ok_s = gs == rs;
            bool ok_i = true;
            for (size_t i = 0; i < ri.size(); ++i) ok_i &= gi[i] == ri[i];
            printf("{\"n\": %d, \"kernel\": \"%s\", \"cstart_ok\": %d, \"citems_ok\": %d}\n", n,
                   variant ? "grid_kernel" : "grid_lds_kernel", ok_s, ok_i);
            bad += !(ok_s && ok_i);
        }
        hipFree(dk);
        hipFree(dcs);
        hipFree(dci);
        hipFree(dco);
    }
    return bad ? 1 : 0;
}
