// orbfe_orbslam.hpp — header-only C++ mirror of ORB-SLAM2's ORBextractor / ORBmatcher
// interface over the C ABI (include/orbfe.h), for host code that is compiled C++ like the
// reference.  Names, argument meaning and ordering follow include/ORBextractor.h:50-119 and
// include/ORBmatcher.h:38-110 of skaegy/ORBSLAM_MapSave; OpenCV types are replaced by plain
// buffers (INTEGRATION.md shows the cv::Mat glue).  Errors surface as orbfe::Error exceptions
// on the C++ side only; nothing throws across the C ABI.
#pragma once

#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "orbfe.h"

namespace orbfe {

struct Error : std::runtime_error {
    int status;
    Error(const char* fn, int st)
        : std::runtime_error(std::string(fn) + " failed with status " + std::to_string(st)),
          status(st) {}
};

inline void check(const char* fn, int st) {
    if (st != ORBFE_OK) throw Error(fn, st);
}

// ORB_SLAM2::ORBextractor (ORBextractor.h:50-119) on a gfx950 GPU.
class ORBextractor {
public:
    enum { HARRIS_SCORE = 0, FAST_SCORE = 1 };

    ORBextractor(int nfeatures, float scaleFactor, int nlevels, int iniThFAST, int minThFAST,
                 int device = 0, int max_width = 0, int max_height = 0)
        : nlevels_(nlevels) {
        orbfe_params p{nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST};
        int st = ORBFE_OK;
        h_ = orbfe_create(&p, device, max_width, max_height, 1, &st);
        if (!h_) throw Error("orbfe_create", st);
    }
    ~ORBextractor() { orbfe_destroy(h_); }
    ORBextractor(const ORBextractor&) = delete;
    ORBextractor& operator=(const ORBextractor&) = delete;

    // operator()(image, mask, keypoints, descriptors) (ORBextractor.cc:1042-1108):
    // image = rows x cols u8 with row step `step`; mask NULL or same size.  An empty image
    // leaves the outputs untouched; zero keypoints clears both.
    void operator()(const uint8_t* image, int cols, int rows, size_t step, const uint8_t* mask,
                    size_t mask_step, std::vector<orbfe_keypoint>& keypoints,
                    std::vector<uint8_t>& descriptors) {
        if (!image || cols <= 0 || rows <= 0) return;
        const int cap = orbfe_keypoint_capacity_for(h_, cols, rows);
        if (cap < 0) throw Error("orbfe_keypoint_capacity_for", cap);
        keypoints.resize(cap);
        descriptors.resize((size_t)cap * 32);
        int n = 0;
        check("orbfe_extract", orbfe_extract(h_, image, cols, rows, step, mask, mask_step,
                                             keypoints.data(), cap, descriptors.data(), &n));
        keypoints.resize(n);
        descriptors.resize((size_t)n * 32);
    }

    // Zero-copy form (orbfe_input_buffer / orbfe_extract_staged): the caller writes the gray
    // frame into InputBuffer (GrabImageMonocular's cvtColor target, Tracking.cc:409-422), then
    // ExtractStaged runs operator() on it in place (Frame::ExtractORB, Frame.cc:358-364).
    uint8_t* InputBuffer(int cols, int rows, size_t* step) {
        uint8_t* buf = nullptr;
        check("orbfe_input_buffer", orbfe_input_buffer(h_, cols, rows, &buf, step));
        return buf;
    }
    void ExtractStaged(int cols, int rows, std::vector<orbfe_keypoint>& keypoints,
                       std::vector<uint8_t>& descriptors) {
        int n = 0;
        check("orbfe_extract_staged", orbfe_extract_staged(h_, cols, rows, nullptr, 0, nullptr, &n));
        const orbfe_keypoint* k = nullptr;
        const uint8_t* d = nullptr;
        check("orbfe_staged_outputs", orbfe_staged_outputs(h_, &k, &d, &n));
        keypoints.assign(k, k + n);
        descriptors.assign(d, d + (size_t)n * 32);
    }

    int GetLevels() { return orbfe_get_levels(h_); }
    float GetScaleFactor() { return orbfe_get_scale_factor(h_); }
    std::vector<float> GetScaleFactors() { return table(0); }
    std::vector<float> GetInverseScaleFactors() { return table(1); }
    std::vector<float> GetScaleSigmaSquares() { return table(2); }
    std::vector<float> GetInverseScaleSigmaSquares() { return table(3); }

    // mvImagePyramid[level] of the last call (ORBextractor.h:90): rows x cols, dense.
    std::vector<uint8_t> ImagePyramidLevel(int level, int* cols, int* rows) {
        int w = 0, h = 0;
        check("orbfe_get_level", orbfe_get_level(h_, 0, level, nullptr, &w, &h));
        std::vector<uint8_t> out((size_t)w * h);
        check("orbfe_get_level", orbfe_get_level(h_, 0, level, out.data(), &w, &h));
        if (cols) *cols = w;
        if (rows) *rows = h;
        return out;
    }

    orbfe_extractor* handle() { return h_; }

private:
    std::vector<float> table(int which) {
        std::vector<float> t[4];
        for (auto& v : t) v.resize(nlevels_);
        check("orbfe_get_scale_tables",
              orbfe_get_scale_tables(h_, t[0].data(), t[1].data(), t[2].data(), t[3].data()));
        return t[which];
    }
    orbfe_extractor* h_ = nullptr;
    int nlevels_;
};

// Flat stand-in for the Frame members the matchers read (Frame.h): owns nothing.
// A DBoW2 FeatureVector (node id -> feature indices, ids ascending) as flat arrays: node i's
// features are feat[node_off[i] .. node_off[i + 1]).
struct FeatureVectorView {
    const int32_t* node_ids;
    const int32_t* node_off;  // nn + 1
    const int32_t* feat;
    int nn;
};

struct FrameData {
    std::vector<orbfe_keypoint> keys_un;   // mvKeysUn
    std::vector<uint8_t> descriptors;      // mDescriptors, N x 32
    std::vector<float> u_right;            // mvuRight (empty: monocular)
    float min_x = 0, max_x = 0, min_y = 0, max_y = 0;  // mnMinX ... (Frame.cc:554-582)
    std::vector<float> scale_factors;      // mvScaleFactors
    std::vector<int> map_points;           // mvpMapPoints as MapPoint ids, -1 = NULL
    std::vector<int> map_point_obs;        // Observations() of those MapPoints

    orbfe_frame_view view() const {
        orbfe_frame_view v;
        v.n = (int)keys_un.size();
        v.keys_un = keys_un.data();
        v.desc = descriptors.data();
        v.u_right = u_right.empty() ? nullptr : u_right.data();
        v.min_x = min_x;
        v.max_x = max_x;
        v.min_y = min_y;
        v.max_y = max_y;
        v.grid_w_inv = 64.f / (max_x - min_x);  // FRAME_GRID_COLS / width (Frame.cc:212)
        v.grid_h_inv = 48.f / (max_y - min_y);
        v.scale_factors = scale_factors.data();
        v.nlevels = (int)scale_factors.size();
        return v;
    }
};

// ORB_SLAM2::ORBmatcher hot subset (ORBmatcher.h:38-110) on a gfx950 GPU.
class ORBmatcher {
public:
    static const int TH_HIGH = 100, TH_LOW = 50, HISTO_LENGTH = 30;  // ORBmatcher.cc:37-39

    explicit ORBmatcher(float nnratio = 0.6f, bool checkOri = true, int device = 0)
        : mfNNratio(nnratio), mbCheckOrientation(checkOri) {
        int st = ORBFE_OK;
        m_ = orbfe_matcher_create(device, &st);
        if (!m_) throw Error("orbfe_matcher_create", st);
    }
    ~ORBmatcher() { orbfe_matcher_destroy(m_); }
    ORBmatcher(const ORBmatcher&) = delete;
    ORBmatcher& operator=(const ORBmatcher&) = delete;

    // DescriptorDistance (ORBmatcher.cc:1650-1666), batched: dist[i] = H(a_i, b_i).
    std::vector<int> DescriptorDistance(const uint8_t* a, const uint8_t* b, int n) {
        std::vector<int> d(n);
        check("orbfe_hamming", orbfe_hamming(m_, a, b, n, d.data()));
        return d;
    }

    // SearchForInitialization (ORBmatcher.cc:408-523); vbPrevMatched holds (x, y) pairs.
    int SearchForInitialization(const FrameData& F1, const FrameData& F2,
                                std::vector<float>& vbPrevMatched, std::vector<int>& vnMatches12,
                                int windowSize = 10) {
        vnMatches12.assign(F1.keys_un.size(), -1);
        const orbfe_frame_view v1 = F1.view(), v2 = F2.view();
        int n = 0;
        check("orbfe_search_for_initialization",
              orbfe_search_for_initialization(m_, mfNNratio, mbCheckOrientation, &v1, &v2,
                                              vbPrevMatched.data(), windowSize,
                                              vnMatches12.data(), &n));
        return n;
    }

    // SearchByProjection(Frame& F, const vector<MapPoint*>&, th) (ORBmatcher.cc:45-129).
    int SearchByProjection(FrameData& F, const orbfe_mappoint_view& mps, const int* mp_ids,
                           float th = 3) {
        prepare(F);
        const orbfe_frame_view v = F.view();
        int n = 0;
        check("orbfe_search_by_projection_local",
              orbfe_search_by_projection_local(m_, mfNNratio, &v, F.map_points.data(),
                                               F.map_point_obs.data(), &mps, mp_ids, th, &n));
        return n;
    }

    // SearchByProjection(Frame& Cur, const Frame& Last, th, bMono) (ORBmatcher.cc:1331-1473).
    // last_*: per last-frame keypoint, the MapPoint it holds (valid flag, world position,
    // descriptor, Observations(), id) and mvbOutlier; poses are row-major 3x4 world->camera.
    int SearchByProjection(FrameData& Cur, const float* Tcw, const orbfe_camera& cam,
                           const FrameData& Last, const std::vector<uint8_t>& last_valid,
                           const std::vector<uint8_t>& last_outlier,
                           const std::vector<float>& last_xyz,
                           const std::vector<uint8_t>& last_desc,
                           const std::vector<int>& last_nobs, const std::vector<int>& last_ids,
                           const float* Tlw, float th, bool bMono) {
        prepare(Cur);
        const orbfe_frame_view v = Cur.view();
        int n = 0;
        check("orbfe_search_by_projection_last",
              orbfe_search_by_projection_last(
                  m_, mbCheckOrientation, &v, Tcw, &cam, Cur.map_points.data(),
                  Cur.map_point_obs.data(), (int)Last.keys_un.size(), Last.keys_un.data(),
                  last_valid.data(), last_outlier.data(), last_xyz.data(), last_desc.data(),
                  last_nobs.data(), last_ids.empty() ? nullptr : last_ids.data(), Tlw, th,
                  bMono, &n));
        return n;
    }

    // SearchByBoW(KeyFrame* pKF, Frame& F, vpMapPointMatches) (ORBmatcher.cc:159-291).
    // kf_mp_ok[i]: the keyframe's feature i holds a MapPoint that is not bad (202-207); the two
    // FeatureVectors as their (node id, features) lists; vpMapPointMatches[f] = the keyframe
    // feature matched to frame feature f, or -1.
    int SearchByBoW(const FrameData& KF, const std::vector<uint8_t>& kf_mp_ok,
                    const FeatureVectorView& kf_fv, const FrameData& F,
                    const FeatureVectorView& f_fv, std::vector<int>& vpMapPointMatches) {
        kf_angle_.resize(KF.keys_un.size());
        for (size_t i = 0; i < KF.keys_un.size(); ++i) kf_angle_[i] = KF.keys_un[i].angle;
        f_angle_.resize(F.keys_un.size());
        for (size_t i = 0; i < F.keys_un.size(); ++i) f_angle_[i] = F.keys_un[i].angle;
        vpMapPointMatches.resize(F.keys_un.size());
        int n = 0;
        check("orbfe_search_by_bow",
              orbfe_search_by_bow(m_, mfNNratio, mbCheckOrientation, (int)KF.keys_un.size(),
                                  KF.descriptors.data(), kf_angle_.data(), kf_mp_ok.data(),
                                  kf_fv.nn, kf_fv.node_ids, kf_fv.node_off, kf_fv.feat,
                                  (int)F.keys_un.size(), F.descriptors.data(), f_angle_.data(),
                                  f_fv.nn, f_fv.node_ids, f_fv.node_off, f_fv.feat,
                                  vpMapPointMatches.data(), &n));
        return n;
    }

    orbfe_matcher* handle() { return m_; }

private:
    static void prepare(FrameData& F) {
        F.map_points.resize(F.keys_un.size(), -1);
        F.map_point_obs.resize(F.keys_un.size(), 0);
    }
    orbfe_matcher* m_ = nullptr;
    float mfNNratio;
    bool mbCheckOrientation;
    std::vector<float> kf_angle_, f_angle_;  // SearchByBoW: the keypoints' angles as arrays
};

}  // namespace orbfe
