/*
 * orb_oracle.h — TEST INFRASTRUCTURE ONLY (parity checker + CPU baseline), never shipped.
 *
 * CPU restatement of the reference hot path (skaegy/ORBSLAM_MapSave src/ORBextractor.cc,
 * src/ORBmatcher.cc, src/Frame.cc, src/MapPoint.cc) and of the OpenCV 3.3.1 primitives it
 * calls.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it.  The product library (liborbfe.so) never links or calls it.
 *
 * PARITY UNPINNED: the reference cannot be built here (OpenCV/Boost/Eigen/Pangolin absent)
 * and holds no tests, fixtures or golden vectors for this path.  See
 * DESIGN.md "Oracle" for every semantic choice (H1-H8) this restatement fixes.
 *
 * Signatures mirror include/orbfe.h with an `oracle_` prefix and host pointers only.
 */
#ifndef ORB_ORACLE_H
#define ORB_ORACLE_H
#include "../include/orbfe.h"

#ifdef __cplusplus
extern "C" {
#endif

/* A1 tables: scale, inv_scale, sigma2, inv_sigma2, features per level, umax[16]. */
int oracle_tables(const orbfe_params* p, float* scale, float* inv_scale, float* sigma2,
                  float* inv_sigma2, int32_t* nfeat, int32_t* umax);
/* The constants the restatement uses, in the order PATCH_SIZE, HALF_PATCH_SIZE, EDGE_THRESHOLD
 * (ORBextractor.cc:71-73), TH_HIGH, TH_LOW, HISTO_LENGTH (ORBmatcher.cc:37-39). */
int oracle_reference_constants(int32_t out[6]);
/* Level sizes of the pyramid for a w x h input (ORBextractor.cc:1114-1115). */
int oracle_level_sizes(const orbfe_params* p, int w, int h, int32_t* lw, int32_t* lh);

/* The build-dependent reading of the reference the oracle computes.  Bits: 1 H2 oct-tree ties
 * by real heap address (residual study only), 2 H4 glibc cosf/sinf, 4 H4 FMA contraction, 8 H5
 * SSE2 resize rounding, 16 H6 SIMD blur rounding.  Default 4 | 8 | 16: the reference's x86-64
 * build, which the GPU's default (ORBFE_ARITH_X86_SIMD) is checked against; 0 = OpenCV's
 * portable scalar reading (ORBFE_ARITH_SCALAR).  Process-global, not thread-safe. */
int oracle_set_variant(int flags);
int oracle_get_variant(void);

/* Full operator() (ORBextractor.cc:1042-1108). */
int oracle_extract(const orbfe_params* p, const uint8_t* img, int w, int h, size_t stride,
                   const uint8_t* mask, size_t mask_stride, orbfe_keypoint* kps, int kps_cap,
                   uint8_t* desc, int* n_out);
/* n frames on `nthreads` CPU threads, one extractor state per thread (Frame.cc:78-81). */
int oracle_extract_batch(const orbfe_params* p, const uint8_t* imgs, int n, int w, int h,
                         size_t frame_pitch, orbfe_keypoint* kps, int kps_cap, uint8_t* desc,
                         int32_t* n_out, int nthreads);

/* cvtColor(*2GRAY) 8U of Tracking::GrabImage* (pix = ORBFE_PIX_RGB/BGR/RGBA/BGRA); dst is
 * w x h dense. */
int oracle_cvt_gray(const uint8_t* src, int pix, int w, int h, size_t stride, uint8_t* dst);

/* Frame::ComputeStereoMatches (Frame.cc:584-756) over the pyramids of the two images. */
int oracle_compute_stereo_matches(const orbfe_params* p, const uint8_t* imL, const uint8_t* imR,
                                  int w, int h, const orbfe_keypoint* kl, const uint8_t* dl,
                                  int nl, const orbfe_keypoint* kr, const uint8_t* dr, int nr,
                                  float bf, float b, float* u_right, float* depth);

/* Stage probes. */
int oracle_pyramid(const orbfe_params* p, const uint8_t* img, int w, int h, size_t stride,
                   const uint8_t* mask, size_t mask_stride, uint8_t* out /* levels packed,
                   rows dense */);
int oracle_resize_linear(const uint8_t* src, int sw, int sh, size_t sstride, uint8_t* dst,
                         int dw, int dh, size_t dstride);
int oracle_gaussian_blur(const uint8_t* src, int w, int h, size_t stride, uint8_t* dst);
int oracle_fast(const uint8_t* roi, int rows, int cols, size_t stride, int threshold,
                orbfe_keypoint* out, int cap, int* n_out);
int oracle_fast_keys(const orbfe_params* p, const uint8_t* level, int lw, int lh,
                     size_t stride, orbfe_keypoint* out, int cap, int* n_out);
int oracle_distribute(const orbfe_params* p, int level, int lw, int lh,
                      const orbfe_keypoint* keys, int n, orbfe_keypoint* out, int cap,
                      int* n_out);
int oracle_fast_atan2(const float* y, const float* x, int n, float* out);
int oracle_ic_angle(const uint8_t* level, int lw, int lh, size_t stride,
                    const orbfe_keypoint* kps, int n, float* angle);
int oracle_describe(const uint8_t* blurred, int lw, int lh, size_t stride,
                    const orbfe_keypoint* kps, int n, uint8_t* desc);

/* Matchers. */
int oracle_hamming(const uint8_t* a, const uint8_t* b, int n, int32_t* dist);
int oracle_bf_match(const uint8_t* q, int nq, const uint8_t* r, int nr, int32_t* best_idx,
                    int32_t* best_dist, int32_t* second_dist);
int oracle_features_in_area(const orbfe_frame_view* f, float x, float y, float r,
                            int min_level, int max_level, int32_t* out, int cap, int* n_out);
int oracle_search_for_initialization(float nnratio, int check_ori, const orbfe_frame_view* f1,
                                     const orbfe_frame_view* f2, float* prev_matched,
                                     int window, int32_t* matches12, int32_t* nmatches);
int oracle_search_by_projection_local(float nnratio, const orbfe_frame_view* f,
                                      int32_t* frame_mp, int32_t* frame_mp_obs,
                                      const orbfe_mappoint_view* mps, const int32_t* mp_ids,
                                      float th, int32_t* nmatches);
int oracle_search_by_projection_last(int check_ori, const orbfe_frame_view* cur,
                                     const float* tcw_cur, const orbfe_camera* cam,
                                     int32_t* frame_mp, int32_t* frame_mp_obs, int n_last,
                                     const orbfe_keypoint* last_keys,
                                     const uint8_t* last_mp_valid, const uint8_t* last_outlier,
                                     const float* last_mp_xyz, const uint8_t* last_mp_desc,
                                     const int32_t* last_mp_nobs, const int32_t* last_mp_ids,
                                     const float* tcw_last, float th, int mono,
                                     int32_t* nmatches);
int oracle_search_by_projection_keyframe(int check_ori, const orbfe_frame_view* cur,
                                         const float* tcw_cur, const orbfe_camera* cam,
                                         float log_scale_factor, int32_t* frame_mp, int n_kf,
                                         const float* kf_key_angle, const uint8_t* kf_mp_valid,
                                         const uint8_t* kf_mp_bad, const uint8_t* already_found,
                                         const float* kf_mp_xyz, const uint8_t* kf_mp_desc,
                                         const float* kf_mp_min_dist,
                                         const float* kf_mp_max_dist, const int32_t* kf_mp_ids,
                                         float th, int orb_dist, int32_t* nmatches);
int oracle_distinctive_descriptors(int n_mp, const int32_t* obs_off, const uint8_t* obs_desc,
                                   int32_t* best, uint8_t* desc_out);
/* DBoW2 (Thirdparty/DBoW2 of the reference): text vocabulary, transform, SearchByBoW. */
typedef struct oracle_vocab oracle_vocab;
oracle_vocab* oracle_vocab_load_text(const char* path, int* status);
void oracle_vocab_free(oracle_vocab* v);
int oracle_vocab_info(const oracle_vocab* v, int32_t* info);
int oracle_bow_transform(const oracle_vocab* v, const uint8_t* desc, int n, int levelsup,
                         int32_t* word_ids, double* values, int32_t* nw, int32_t* node_ids,
                         int32_t* node_off, int32_t* feat, int32_t* nn);
int oracle_search_by_bow(float nnratio, int check_ori, const uint8_t* kf_desc,
                         const float* kf_angle, const uint8_t* kf_mp_ok,
                         const int32_t* kf_node_ids, const int32_t* kf_node_off,
                         const int32_t* kf_feat, int kf_nn, int n_f, const uint8_t* f_desc,
                         const float* f_angle, const int32_t* f_node_ids,
                         const int32_t* f_node_off, const int32_t* f_feat, int f_nn,
                         int32_t* matches, int32_t* nmatches);
int oracle_is_in_frustum(int n, const float* xyz, const float* normal, const float* min_dist,
                         const float* max_dist, const float* tcw, const orbfe_camera* cam,
                         float min_x, float max_x, float min_y, float max_y,
                         float log_scale_factor, float viewing_cos_limit, uint8_t* in_view,
                         float* proj_x, float* proj_y, float* proj_xr, int32_t* pred_level,
                         float* view_cos);

#ifdef __cplusplus
}
#endif
#endif
