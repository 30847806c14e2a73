/*
 * orbfe.h — C ABI of the MI355X-native ORB front-end (extractor + matchers).
 *
 * This is the drop-in seam for ORB-SLAM2's hot path as shipped in skaegy/ORBSLAM_MapSave.
 * Every entry point below replaces one reference interface; the replaced interface is cited
 * (file:line under the reference tree).  Plain C: no C++ types, no torch types, no exceptions.
 *
 * Conventions
 *   - Every function returns an int status (ORBFE_OK == 0, negative on error) unless it is a
 *     pure getter.  No function throws or aborts across the ABI.
 *   - "host" pointers are ordinary CPU memory; "_device" entry points take HIP device pointers
 *     and run asynchronously on the handle's stream (orbfe_set_stream); every other entry point
 *     is synchronous on return, matching the blocking semantics of the reference.
 *   - One handle is NOT reentrant (the reference ORBextractor keeps mvImagePyramid as instance
 *     state, ORBextractor.h:90).  Distinct handles are fully independent (own stream, own
 *     device buffers) and may be used from different threads concurrently.
 *   - The library never falls back to a CPU path: if no gfx950 device is usable, orbfe_create /
 *     orbfe_matcher_create fail with ORBFE_ERR_HIP.
 */
#ifndef ORBFE_H
#define ORBFE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes ------------------------------------------------------------------------- */
#define ORBFE_OK               0
#define ORBFE_ERR_ARG         -1   /* bad argument (NULL, negative size, ...)                   */
#define ORBFE_ERR_CAPACITY    -2   /* caller buffer too small; *n_out holds the required count  */
#define ORBFE_ERR_HIP         -3   /* HIP runtime error / no usable device                      */
#define ORBFE_ERR_UNSUPPORTED -4   /* input the reference handles only through UB (see DESIGN) */
#define ORBFE_ERR_NOMEM       -5   /* device allocation failed                                  */

/* ---- plain data types ----------------------------------------------------------------------- */

/* Extractor parameters: the five ctor arguments of ORBextractor (ORBextractor.h:56-57),
 * read from ORBextractor.{nFeatures,scaleFactor,nLevels,iniThFAST,minThFAST} (Tracking.cc:200-204). */
typedef struct orbfe_params {
    int32_t nfeatures;
    float   scale_factor;
    int32_t nlevels;
    int32_t ini_th_fast;
    int32_t min_th_fast;
} orbfe_params;

/* Layout-compatible with cv::KeyPoint (28 bytes): pt.x, pt.y, size, angle, response, octave,
 * class_id.  Extractor output sets class_id = -1 exactly as cv::FAST does. */
typedef struct orbfe_keypoint {
    float   x, y;
    float   size;
    float   angle;
    float   response;
    int32_t octave;
    int32_t class_id;
} orbfe_keypoint;

/* Pixel formats of the frames handed to the colour entry points: the four cvtColor codes of
 * Tracking::GrabImageStereo / GrabImageRGBD / GrabImageMonocular (Tracking.cc:286-310,
 * 350-363, 409-422), chosen there by channels() and mbRGB (Camera.RGB, Tracking.cc:192). */
#define ORBFE_PIX_GRAY 0   /* CV_8UC1, no conversion                                          */
#define ORBFE_PIX_RGB  1   /* CV_8UC3, CV_RGB2GRAY  (mbRGB = 1)                               */
#define ORBFE_PIX_BGR  2   /* CV_8UC3, CV_BGR2GRAY  (mbRGB = 0)                               */
#define ORBFE_PIX_RGBA 3   /* CV_8UC4, CV_RGBA2GRAY                                           */
#define ORBFE_PIX_BGRA 4   /* CV_8UC4, CV_BGRA2GRAY                                           */

/* Zeroed rectangle of the human mask: rows [y0, y1) x cols [x0, x1) of an all-ones mask
 * (OpDetector::SkeletonSquareMask, DetectHumanPose.cpp:484-489). */
typedef struct orbfe_rect {
    int32_t x0, y0, x1, y1;
} orbfe_rect;

typedef struct orbfe_extractor  orbfe_extractor;
typedef struct orbfe_matcher    orbfe_matcher;
typedef struct orbfe_vocabulary orbfe_vocabulary;

/* ---- extractor ---------------------------------------------------------------------------- */

/* Replaces ORBextractor::ORBextractor (ORBextractor.cc:409-469).  `device` is the HIP ordinal;
 * `max_width`/`max_height`/`max_batch` size the device workspace (0 => 1920 x 1080 x 1, grown
 * on demand outside any captured region). */
orbfe_extractor* orbfe_create(const orbfe_params* params, int device, int max_width,
                              int max_height, int max_batch, int* status);
void orbfe_destroy(orbfe_extractor* h);

/* Which build of the reference's OpenCV 3.3 primitives the pixel arithmetic reproduces
 * (tests/golden/README.md).  ORBFE_ARITH_SCALAR: OpenCV's portable scalar
 * paths — resize FixedPtCast<int,uchar,22>, blur FixedPtCastEx, uncontracted rotation products.
 * ORBFE_ARITH_X86_SIMD (the default, what the reference's build.sh Release build computes on
 * x86-64, where SSE2 is always on): the SSE2 bodies of
 * VResizeLinearVec_32s8u (ORBextractor.cc:1123; ~18 % of the pixels of levels >= 1 differ
 * by 1 from the scalar path) and SymmColumnVec_32s8u (1089; ties rounded to even) with the
 * scalar tails past them, and the descriptor rotation FMA-contracted as GCC -O3 on an FMA host
 * builds computeOrbDescriptor (117-119).  The oct-tree's heap-address tie order (H2) cannot
 * be reproduced by any build and stays the documented creation-sequence rule.  Synchronizes
 * the handle's stream; applies to later calls. */
#define ORBFE_ARITH_SCALAR   0
#define ORBFE_ARITH_X86_SIMD 1
int orbfe_set_arithmetic(orbfe_extractor* h, int mode);
int orbfe_get_arithmetic(const orbfe_extractor* h);

/* The reference's compile-time constants as this library's kernels use them: PATCH_SIZE,
 * HALF_PATCH_SIZE, EDGE_THRESHOLD (ORBextractor.cc:71-73) and ORBmatcher::TH_HIGH, TH_LOW,
 * HISTO_LENGTH (ORBmatcher.cc:37-39).  Needs no device; for the known-answer check against the
 * reference text (tests/golden/constants_fixture.json). */
typedef struct orbfe_reference_constants {
    int32_t patch_size, half_patch_size, edge_threshold;
    int32_t th_high, th_low, histo_length;
} orbfe_reference_constants;
int orbfe_get_reference_constants(orbfe_reference_constants* out);

/* Getters — ORBextractor::GetLevels / GetScaleFactor / GetScaleFactors /
 * GetInverseScaleFactors / GetScaleSigmaSquares / GetInverseScaleSigmaSquares
 * (ORBextractor.h:68-88).  Table outputs hold nlevels floats each; any may be NULL. */
int   orbfe_get_levels(const orbfe_extractor* h);
float orbfe_get_scale_factor(const orbfe_extractor* h);
int   orbfe_get_scale_tables(const orbfe_extractor* h, float* scale, float* inv_scale,
                             float* sigma2, float* inv_sigma2);
/* mnFeaturesPerLevel (ORBextractor.cc:434-445). */
int   orbfe_get_features_per_level(const orbfe_extractor* h, int32_t* out);
/* Per-frame keypoint capacity that can never overflow for this handle's params and ANY
 * supported input size (w, h <= 4096): the sum over levels of the oct-tree output bound
 * max(N_l + 4, 4 nIni_l, 20) at the widest aspect ratio (DESIGN.md "capacity"). */
int   orbfe_keypoint_capacity(const orbfe_extractor* h);
/* The same bound for one input size (w x hgt): what DistributeOctTree (ORBextractor.cc:538-762)
 * can return per level at that size, summed.  <= orbfe_keypoint_capacity(h); negative status
 * for an unsupported size. */
int   orbfe_keypoint_capacity_for(const orbfe_extractor* h, int w, int hgt);
/* orbfe_keypoint_capacity_for without a handle (host arithmetic only, no device): the bound
 * for extractor parameters `p` at w x hgt, so a caller can size its output slabs (e.g. config
 * 4's all-gathered descriptor slabs) before any extractor exists.  Negative status for bad
 * parameters or an unsupported size. */
int   orbfe_keypoint_capacity_params(const orbfe_params* p, int w, int hgt);

/* Replaces ORBextractor::operator()(image, mask, keypoints, descriptors)
 * (ORBextractor.h:64-66, ORBextractor.cc:1042-1108), called from Frame::ExtractORB
 * (Frame.cc:358-364, mask empty) and Frame::ExtractORBMask (Frame.cc:366-371).
 *   img   : w x h u8 gray, row stride `stride` bytes (CV_8UC1, asserted at ORBextractor.cc:1051)
 *   mask  : NULL for none, else w x h u8 with row stride `mask_stride`; pixels where mask==0
 *           are zeroed before the pyramid (Mat::copyTo(dst, mask), ORBextractor.cc:1053)
 *   kps   : kps_cap keypoints out, level-major order (ORBextractor.cc:1079-1107)
 *   desc  : kps_cap x 32 bytes out, row i <-> kps[i]
 *   n_out : number of keypoints written.
 * Empty image (img==NULL or w==0 or h==0): returns ORBFE_OK and touches nothing
 * (ORBextractor.cc:1045-1046).  kps_cap too small: ORBFE_ERR_CAPACITY, *n_out = required. */
int orbfe_extract(orbfe_extractor* h, const uint8_t* img, int w, int hgt, size_t stride,
                  const uint8_t* mask, size_t mask_stride, orbfe_keypoint* kps, int kps_cap,
                  uint8_t* desc, int* n_out);

/* Zero-copy form of the same call for the tracking loop.  Frame::ExtractORB
 * (Frame.cc:358-364) hands operator() the cv::Mat that GrabImageMonocular's cvtColor just
 * produced (Tracking.cc:409-422); orbfe_extract copies it into the handle's pinned staging
 * buffer first.  Instead:
 *   orbfe_input_buffer   : the handle's pinned, device-mapped w x h u8 staging buffer (*buf,
 *                          row stride *stride bytes) — wrap it as cv::Mat(h, w, CV_8UC1, buf,
 *                          stride) and let cvtColor write the gray frame straight into it.
 *                          It is separate from the staging orbfe_extract copies into: no
 *                          other call writes or moves it, and it stays valid until an
 *                          orbfe_input_buffer for a larger w x h or orbfe_destroy on h.
 *   orbfe_extract_staged : operator() on that buffer (the GPU reads it in place).  With
 *                          kps_cap == 0 (kps, desc NULL) the outputs stay in the handle's pinned
 *                          output buffers and orbfe_staged_outputs returns them (*n_out is set).
 *   orbfe_staged_outputs : the last single-frame call's keypoints / descriptors (n of them), in
 *                          handle-owned memory valid until the next call on h.
 * Errors and capacity rules as orbfe_extract; orbfe_extract_staged without a buffer handed out
 * for at least w x h returns ORBFE_ERR_ARG. */
int orbfe_input_buffer(orbfe_extractor* h, int w, int hgt, uint8_t** buf, size_t* stride);
int orbfe_extract_staged(orbfe_extractor* h, int w, int hgt, orbfe_keypoint* kps, int kps_cap,
                         uint8_t* desc, int* n_out);
int orbfe_staged_outputs(const orbfe_extractor* h, const orbfe_keypoint** kps,
                         const uint8_t** desc, int* n);

/* Colour front-end: cvtColor(img, gray, CV_*2GRAY) of Tracking::GrabImage* (Tracking.cc:409-422
 * and the stereo / RGB-D twins) fused with Frame::ExtractORBMask -> operator()(gray, mask)
 * (Frame.cc:366-371, ORBextractor.cc:1053).  `pix` is an ORBFE_PIX_* format, `stride` the row
 * stride of img in bytes (>= w * channels).  The mask is given as a u8 plane (`mask`, NULL for
 * none) and/or as the zeroed rectangle `rect` (NULL for none) of OpDetector's square mask;
 * a pixel survives when both keep it.  rect with x1 < x0 or y1 < y0 (where the reference's
 * rowRange/colRange assert) returns ORBFE_ERR_UNSUPPORTED.  Gray values follow OpenCV's 8U
 * integer path.  Otherwise as orbfe_extract. */
int orbfe_extract_color(orbfe_extractor* h, const uint8_t* img, int pix, int w, int hgt,
                        size_t stride, const uint8_t* mask, size_t mask_stride,
                        const orbfe_rect* rect, orbfe_keypoint* kps, int kps_cap, uint8_t* desc,
                        int* n_out);

/* The human-mask rectangle from 25 OpenPose joints (x, y, score) — the bounding box of the
 * joints grown by 30 px and clamped to the image, exactly as OpDetector::SkeletonSquareMask
 * computes it (DetectHumanPose.cpp:453-489).  Host-only helper (no device work). */
int orbfe_human_mask_rect(const float* joints, int njoints, int w, int hgt, orbfe_rect* out);

/* Throughput form of orbfe_extract over n same-size frames (host buffers).  Frame f's
 * keypoints go to kps[f*kps_cap ...], descriptors to desc[f*kps_cap*32 ...], count n_out[f].
 * masks may be NULL (no masks) or an array of n pointers (entries may be NULL). */
int orbfe_extract_batch(orbfe_extractor* h, const uint8_t* const* imgs, int n, int w, int hgt,
                        size_t stride, const uint8_t* const* masks, size_t mask_stride,
                        orbfe_keypoint* kps, int kps_cap, uint8_t* desc, int32_t* n_out);

/* Device-resident throughput form: d_imgs holds n frames, frame f at d_imgs + f*frame_pitch,
 * rows `stride` bytes apart.  d_masks NULL or laid out like d_imgs.  Outputs are device
 * slabs laid out as in orbfe_extract_batch.  Asynchronous on the handle's stream.
 * kps_cap below orbfe_keypoint_capacity_for(h, w, hgt) returns ORBFE_ERR_CAPACITY before any
 * device work, so no frame is ever truncated; d_n_out[f] is frame f's keypoint count. */
int orbfe_extract_batch_device(orbfe_extractor* h, const uint8_t* d_imgs, int n, int w, int hgt,
                               size_t stride, size_t frame_pitch, const uint8_t* d_masks,
                               orbfe_keypoint* d_kps, int kps_cap, uint8_t* d_desc,
                               int32_t* d_n_out);

/* Device-resident colour form: frame f at d_imgs + f*frame_pitch in format `pix`; d_masks NULL
 * or n u8 planes (mask_stride, mask_frame_pitch); d_rects NULL or n device orbfe_rect.  Level 0
 * (the gray, masked image) is made by one fused kernel before the pipeline. */
int orbfe_extract_color_batch_device(orbfe_extractor* h, const uint8_t* d_imgs, int pix, int n,
                                     int w, int hgt, size_t stride, size_t frame_pitch,
                                     const uint8_t* d_masks, size_t mask_stride,
                                     size_t mask_frame_pitch, const orbfe_rect* d_rects,
                                     orbfe_keypoint* d_kps, int kps_cap, uint8_t* d_desc,
                                     int32_t* d_n_out);

/* Stream control: `hip_stream` is a hipStream_t (NULL => the handle's own stream, which is
 * non-blocking: it does not order against the legacy default stream).  To run on the device's
 * legacy default stream (handle 0 in frameworks that expose it, e.g. torch's default stream),
 * pass hipStreamLegacy ((void*)1); the same holds for the matcher and vocabulary handles. */
int orbfe_set_stream(orbfe_extractor* h, void* hip_stream);
int orbfe_synchronize(orbfe_extractor* h);

/* Per-kernel timing of the extraction pipeline: when enabled, a HIP event pair is recorded on
 * the handle's stream around every kernel launch.  orbfe_profile_read synchronizes the stream
 * and returns, per stage (ORBFE_STAGE_*), the summed duration in ms and the launch count since
 * the previous read.  Used by bench.py for the roofline figure; off by default.
 * enable: 0 off, 1 every stage, or ORBFE_PROFILE_STAGE(s) OR-ed together to time only those
 * stages (the other launches carry no events). */
#define ORBFE_PROFILE_STAGE(s) (2 << (s))
#define ORBFE_STAGE_MASK     0   /* K0: colour conversion + mask (level 0) */
#define ORBFE_STAGE_RESIZE   1
#define ORBFE_STAGE_FAST     2
#define ORBFE_STAGE_OCTREE   3
#define ORBFE_STAGE_BLUR     4
#define ORBFE_STAGE_DESCRIBE 5
#define ORBFE_STAGE_COUNT    6
int orbfe_profile(orbfe_extractor* h, int enable);
int orbfe_profile_read(orbfe_extractor* h, double* total_ms, int32_t* launches);

/* Which pyramid path an extraction of `nframes` frames at the extractor's current frame size
 * takes (the last extracted size; a test hook, no reference counterpart): ORBFE_PYR_PER_LEVEL
 * (resize2_kernel pairs / resize_kernel + resize_tail_kernel), ORBFE_PYR_BANDS
 * (pyramid_kernel); ORBFE_ERR_ARG before any extraction.  (Value 2, the rolling-band kernel of
 * rounds 4-5, was removed with that kernel and is never returned.) */
#define ORBFE_PYR_PER_LEVEL 0
#define ORBFE_PYR_BANDS     1
int orbfe_pyramid_path(const orbfe_extractor* h, int nframes);
/* Measurement hook: relaunch the stages in `stage_mask` (bits 1 << ORBFE_STAGE_*) of the most
 * recent extraction on its own buffers, `reps` times, asynchronously on the handle's stream
 * (outputs meaningful only for a full mask). */
int orbfe_debug_replay(orbfe_extractor* h, unsigned stage_mask, int reps);
/* Stage pipelining: later extraction calls on `h` run only the stages in `stage_mask` (bits
 * 1 << ORBFE_STAGE_*; 0 = all, the default).  A batch extracted in two calls on the same handle,
 * buffers and frames — stages up to the oct-tree, then describe — equals one full call; the
 * caller orders the calls (e.g. on two streams, so that one sub-batch's describe runs beside
 * another's FAST). */
int orbfe_set_stage_mask(orbfe_extractor* h, unsigned stage_mask);

/* Pyramid access — replaces the public member mvImagePyramid (ORBextractor.h:90) read by
 * stereo matching (Frame.cc:589, 679, 696).  Copies level `level` of frame `frame` of the
 * most recent extraction (interior pixels only, rows w bytes apart) into `out`
 * (out may be NULL to query w/h). */
int orbfe_get_level(orbfe_extractor* h, int frame, int level, uint8_t* out, int* w, int* hgt);

/* Stage probes of the most recent extraction, for parity tests against the oracle:
 * blurred level (GaussianBlur 7x7 sigma 2 REFLECT_101, ORBextractor.cc:1088-1089) and the
 * per-level FAST output before distribution (vToDistributeKeys, ORBextractor.cc:777-828;
 * coordinates relative to (16,16), response = FAST score). */
int orbfe_get_blurred_level(orbfe_extractor* h, int frame, int level, uint8_t* out, int* w,
                            int* hgt);
int orbfe_get_fast_keys(orbfe_extractor* h, int frame, int level, orbfe_keypoint* out, int cap,
                        int* n_out);

/* ---- stereo ------------------------------------------------------------------------------ */

/* Frame::ComputeStereoMatches (Frame.cc:584-756), called by the stereo Frame ctor right after
 * the two extractions (Frame.cc:78-103).  kl/dl: mvKeys + mDescriptors of the left image (nl,
 * distorted keypoints as extracted); kr/dr: mvKeysRight + mDescriptorsRight (nr).  The pyramids
 * read are mpORBextractorLeft/Right->mvImagePyramid: frame `frame` of the most recent
 * extraction of `left` / `right` (same image size and scale parameters).  bf = mbf, b = mb.
 * Writes mvuRight / mvDepth (nl floats each, -1 = no match).  Inputs on which the reference
 * indexes vRowIndices out of range or trips a rowRange/colRange assert return
 * ORBFE_ERR_UNSUPPORTED.  Synchronous; runs on left's stream after right's stream. */
int orbfe_compute_stereo_matches(orbfe_extractor* left, orbfe_extractor* right, int frame,
                                 const orbfe_keypoint* kl, const uint8_t* dl, int nl,
                                 const orbfe_keypoint* kr, const uint8_t* dr, int nr, float bf,
                                 float b, float* u_right, float* depth);

/* Device-resident batch form over frames 0..n-1 of the two handles' most recent
 * orbfe_extract*_batch_device calls: keypoint / descriptor / count slabs as those calls write
 * them (kps_cap keypoints per frame); u_right / depth are n x kps_cap floats.  The device frames
 * the extractions read must still be valid (level 0 is read in place).  Asynchronous on left's
 * stream (ordered after right's stream); orbfe_stereo_status reports UB inputs afterwards. */
int orbfe_compute_stereo_matches_device(orbfe_extractor* left, orbfe_extractor* right, int n,
                                        const orbfe_keypoint* d_kl, const uint8_t* d_dl,
                                        const int32_t* d_nl, const orbfe_keypoint* d_kr,
                                        const uint8_t* d_dr, const int32_t* d_nr, int kps_cap,
                                        float bf, float b, float* d_u_right, float* d_depth);
/* Synchronizes left's stream; ORBFE_OK or ORBFE_ERR_UNSUPPORTED for the last stereo call. */
int orbfe_stereo_status(orbfe_extractor* left);

/* ---- matchers ------------------------------------------------------------------------------- */

/* Frame data the matchers read.  Mirrors the Frame members the reference matchers touch:
 * mvKeysUn (x, y, octave, angle), mDescriptors, mvuRight, image bounds mnMin/MaxX/Y and
 * mfGridElementWidthInv/HeightInv (Frame.cc:212-213), mvScaleFactors.  The 64 x 48 grid of
 * Frame::AssignFeaturesToGrid (Frame.cc:341-356) is rebuilt from keys_un inside the call. */
typedef struct orbfe_frame_view {
    int32_t               n;
    const orbfe_keypoint* keys_un;        /* n                                                 */
    const uint8_t*        desc;           /* n x 32                                            */
    const float*          u_right;        /* n, or NULL for monocular (all -1)                 */
    float                 min_x, max_x, min_y, max_y;
    float                 grid_w_inv, grid_h_inv;
    const float*          scale_factors;  /* nlevels                                           */
    int32_t               nlevels;
} orbfe_frame_view;

/* Per-MapPoint tracking scratch (MapPoint.h:106-111) + the getters SearchByProjection reads. */
typedef struct orbfe_mappoint_view {
    int32_t        m;
    const uint8_t* track_in_view;  /* mbTrackInView                                         */
    const uint8_t* is_bad;         /* isBad()                                               */
    const float*   proj_x;         /* mTrackProjX                                           */
    const float*   proj_y;         /* mTrackProjY                                           */
    const float*   proj_xr;        /* mTrackProjXR                                          */
    const int32_t* pred_level;     /* mnTrackScaleLevel                                     */
    const float*   view_cos;       /* mTrackViewCos                                         */
    const uint8_t* desc;           /* GetDescriptor(), m x 32                               */
    const int32_t* n_obs;          /* Observations()                                        */
} orbfe_mappoint_view;

/* Camera + pose for the last-frame projection matcher (ORBmatcher.cc:1341-1379). Row-major
 * 3x4 [R|t] world->camera. */
typedef struct orbfe_camera {
    float fx, fy, cx, cy, bf, b;   /* mbf and mb (= mbf/fx, Frame.cc:225)                    */
} orbfe_camera;

orbfe_matcher* orbfe_matcher_create(int device, int* status);
void orbfe_matcher_destroy(orbfe_matcher* m);
int  orbfe_matcher_set_stream(orbfe_matcher* m, void* hip_stream);

/* ORBmatcher::DescriptorDistance (ORBmatcher.cc:1650-1666): dist[i] = Hamming(a_i, b_i). */
int orbfe_hamming(orbfe_matcher* m, const uint8_t* a, const uint8_t* b, int n, int32_t* dist);

/* Brute-force Hamming (config 3, no single reference function): for each query the best and
 * second-best distance over all references with the first-wins update rule of
 * ORBmatcher.cc:102-114 (best/second start at 256).  Host buffers. */
int orbfe_bf_match(orbfe_matcher* m, const uint8_t* q, int nq, const uint8_t* r, int nr,
                   int32_t* best_idx, int32_t* best_dist, int32_t* second_dist);
/* Device-resident batched form: `nb` independent (query-set, reference-set) problems;
 * problem b reads d_q + b*q_pitch (nq_b = d_nq[b] rows) against d_r + b*r_pitch
 * (nr_b = d_nr[b] rows) and writes d_out + b*nq_cap*3 as (best_idx, best, second) triples.
 * Reference sets hold fewer than 65536 rows: the kernels search the first 65,535 rows of a
 * larger set (indices are 16-bit fields of the ranking keys). */
int orbfe_bf_match_batch_device(orbfe_matcher* m, const uint8_t* d_q, size_t q_pitch,
                                const int32_t* d_nq, int nq_cap, const uint8_t* d_r,
                                size_t r_pitch, const int32_t* d_nr, int nb, int32_t* d_out);

/* Timing of orbfe_bf_match_batch_device launches (dispatch-bound HIP events, as
 * orbfe_profile): summed ms and launch count since the previous read.  Stage 0 is the
 * brute-force match kernels, stage 1 the expansion of a batch-shared reference set (r_pitch 0)
 * into matrix-core fragments; orbfe_matcher_profile_read reports stage 0,
 * orbfe_matcher_profile_read_stages fills ORBFE_MATCHER_STAGES entries.  Either read resets. */
#define ORBFE_MATCHER_STAGES 2
int orbfe_matcher_profile(orbfe_matcher* m, int enable);
int orbfe_matcher_profile_read(orbfe_matcher* m, double* total_ms, int32_t* launches);
int orbfe_matcher_profile_read_stages(orbfe_matcher* m, double* total_ms, int32_t* launches);

/* ORBmatcher::SearchForInitialization (ORBmatcher.cc:408-523), matcher built as
 * ORBmatcher(nnratio, check_ori) (Tracking.cc:843).  prev_matched: inout F1.n (x,y) pairs
 * (vbPrevMatched); matches12: out F1.n (vnMatches12). */
int orbfe_search_for_initialization(orbfe_matcher* m, float nnratio, int check_ori,
                                    const orbfe_frame_view* f1, const orbfe_frame_view* f2,
                                    float* prev_matched, int window, int32_t* matches12,
                                    int32_t* nmatches);

/* ORBmatcher::SearchByProjection(Frame&, const vector<MapPoint*>&, th) (ORBmatcher.cc:45-129).
 * frame_mp: inout F.n, id of the MapPoint held by each keypoint or -1 (F.mvpMapPoints);
 * frame_mp_obs: inout F.n, Observations() of that MapPoint.  A match writes
 * mp_ids[i] (or i when mp_ids is NULL) and mps->n_obs[i]. */
int orbfe_search_by_projection_local(orbfe_matcher* m, float nnratio,
                                     const orbfe_frame_view* f, int32_t* frame_mp,
                                     int32_t* frame_mp_obs, const orbfe_mappoint_view* mps,
                                     const int32_t* mp_ids, float th, int32_t* nmatches);

/* ORBmatcher::SearchByProjection(Frame& Cur, const Frame& Last, th, bMono)
 * (ORBmatcher.cc:1331-1473).  The last frame is given as its N_last keypoints (octave, angle
 * from last_keys), the world position/descriptor/Observations() of the MapPoint it holds
 * (last_mp_valid[i] == 0 <=> NULL), and mvbOutlier. Poses are row-major 3x4 world->camera. */
int orbfe_search_by_projection_last(orbfe_matcher* m, int check_ori,
                                    const orbfe_frame_view* cur, const float* tcw_cur,
                                    const orbfe_camera* cam, int32_t* frame_mp,
                                    int32_t* frame_mp_obs, int n_last,
                                    const orbfe_keypoint* last_keys,
                                    const uint8_t* last_mp_valid, const uint8_t* last_outlier,
                                    const float* last_mp_xyz, const uint8_t* last_mp_desc,
                                    const int32_t* last_mp_nobs, const int32_t* last_mp_ids,
                                    const float* tcw_last, float th, int mono,
                                    int32_t* nmatches);

/* Tracking::SearchLocalPoints (Tracking.cc:1403-1455) on device-resident data: for every local
 * map point that is neither bad (d_bad) nor already matched in the frame (d_skip[i] != 0 <=>
 * mnLastFrameSeen == mCurrentFrame.mnId), Frame::isInFrustum(pMP, viewing_cos_limit) with
 * MapPoint::PredictScale (Frame.cc:387-443, MapPoint.cc:633-642), then
 * ORBmatcher(nnratio).SearchByProjection(F, vpLocalMapPoints, th) (ORBmatcher.cc:45-129).
 * `frame` is a view whose keys_un / desc / u_right are DEVICE pointers (scale_factors stays a
 * host table).  Map-point arrays (xyz, normal n x 3; mfMinDistance / mfMaxDistance; descriptor
 * n x 32; Observations(); ids or NULL) are device arrays.  d_in_view receives mbTrackInView
 * (0 for skipped or bad points); d_frame_mp / d_frame_mp_obs are updated in place.
 * counts[0] = nmatches, counts[1] = nToMatch (host).  A predicted level outside the pyramid
 * returns ORBFE_ERR_UNSUPPORTED (such points are not matched).  Synchronous on return. */
int orbfe_search_local_points_device(orbfe_matcher* m, const orbfe_frame_view* frame,
                                     const float* tcw, const orbfe_camera* cam,
                                     float log_scale_factor, float viewing_cos_limit, int n_mp,
                                     const float* d_xyz, const float* d_normal,
                                     const float* d_min_dist, const float* d_max_dist,
                                     const uint8_t* d_desc, const int32_t* d_nobs,
                                     const uint8_t* d_bad, const uint8_t* d_skip,
                                     const int32_t* d_mp_ids, float nnratio, float th,
                                     int32_t* d_frame_mp, int32_t* d_frame_mp_obs,
                                     uint8_t* d_in_view, int32_t* counts);
/* ORBmatcher::SearchByProjection(Frame&, const vector<MapPoint*>&, th) (ORBmatcher.cc:45-129)
 * alone, on device-resident data: the isInFrustum outputs (mbTrackInView, mTrackProjX/Y/XR,
 * mnTrackScaleLevel, mTrackViewCos — Tracking.cc:1425-1438 computed them) are already in HBM.
 * `frame` as for orbfe_search_local_points_device (device keys_un / desc / u_right, host
 * scale_factors); every pointer in `d_mps` and d_mp_ids (or NULL) is a device pointer;
 * d_frame_mp / d_frame_mp_obs are updated in place; *nmatches (host).  A tracked point whose
 * predicted level is outside the pyramid returns ORBFE_ERR_UNSUPPORTED.  Synchronous. */
int orbfe_search_by_projection_local_device(orbfe_matcher* m, float nnratio,
                                            const orbfe_frame_view* frame, int32_t* d_frame_mp,
                                            int32_t* d_frame_mp_obs,
                                            const orbfe_mappoint_view* d_mps,
                                            const int32_t* d_mp_ids, float th, int32_t* nmatches);
/* Jacobi rounds the most recent SearchByProjection / SearchForInitialization resolution took
 * (diagnostics). */
int orbfe_matcher_last_rounds(const orbfe_matcher* m);
/* Calls of this matcher rerun because their candidate lists outgrew the device buffer (the
 * first attempt bounds every fill by the buffer and reads unfilled lists as empty; the rerun
 * uses the exact total) — diagnostics for the capacity tests. */
int orbfe_matcher_capacity_retries(const orbfe_matcher* m);

/* Frame::GetFeaturesInArea (Frame.cc:445-498) over the 64 x 48 grid of
 * Frame::AssignFeaturesToGrid / PosInGrid (Frame.cc:341-356, 500-510), exactly as every matcher
 * above builds and queries it — exported for the grid's parity tests.  Query q is
 * (x[q], y[q], r[q], min_level[q], max_level[q]); its candidates, in the reference's order (cell
 * column ix, then row iy, then insertion order), go to items[off[q] .. off[q + 1]).  off holds
 * nq + 1 entries (off[nq] = total).  wave != 0 runs the wave-per-query form
 * (SearchForInitialization, last-frame and keyframe SearchByProjection), wave == 0 the
 * thread-per-query form (local-map SearchByProjection).  total > items_cap: ORBFE_ERR_CAPACITY
 * with off filled and items untouched.  Synchronous; host buffers. */
int orbfe_features_in_area(orbfe_matcher* m, const orbfe_frame_view* f, int nq, const float* x,
                           const float* y, const float* r, const int32_t* min_level,
                           const int32_t* max_level, int wave, int32_t* off, int32_t* items,
                           int items_cap);

/* Relocalisation ORBmatcher::SearchByProjection(Frame& CurrentFrame, KeyFrame* pKF,
 * const set<MapPoint*>& sAlreadyFound, th, ORBdist) (ORBmatcher.cc:1475-1602), called by
 * Tracking::Relocalization with ORBmatcher(0.9, true), th/ORBdist = 10/100 and 3/64
 * (Tracking.cc:1664, 1723, 1737).  The keyframe is given as its n_kf map-point slots
 * (pKF->GetMapPointMatches(); kf_mp_valid[i] == 0 <=> NULL) with isBad(), sAlreadyFound
 * membership, world position (n_kf x 3), descriptor (n_kf x 32), mfMinDistance /
 * mfMaxDistance and the rotation angle pKF->mvKeysUn[i].angle.  frame_mp: inout cur->n ids
 * (-1 = NULL; a slot holding a point is never re-assigned); a match writes kf_mp_ids[i] (or i).
 * log_scale_factor = mfLogScaleFactor.  A predicted scale level outside the pyramid (where the
 * fork indexes mvScaleFactors out of range; MapPoint::PredictScale has no clamp) returns
 * ORBFE_ERR_UNSUPPORTED. */
int orbfe_search_by_projection_keyframe(orbfe_matcher* m, int check_ori,
                                        const orbfe_frame_view* cur, const float* tcw_cur,
                                        const orbfe_camera* cam, float log_scale_factor,
                                        int32_t* frame_mp, int n_kf, const float* kf_key_angle,
                                        const uint8_t* kf_mp_valid, const uint8_t* kf_mp_bad,
                                        const uint8_t* already_found, const float* kf_mp_xyz,
                                        const uint8_t* kf_mp_desc, const float* kf_mp_min_dist,
                                        const float* kf_mp_max_dist, const int32_t* kf_mp_ids,
                                        float th, int orb_dist, int32_t* nmatches);

/* MapPoint::ComputeDistinctiveDescriptors (MapPoint.cc:483-548) for n_mp map points at once
 * (LocalMapping calls it for every new / fused point, LocalMapping.cc:268, 489).  The
 * descriptors of map point i's observations in non-bad keyframes, in mObservations order, are
 * rows obs_off[i] .. obs_off[i+1]-1 of obs_desc (obs_off has n_mp + 1 entries, < 65536
 * observations per point).  best[i] = the chosen row relative to obs_off[i] (least median
 * distance to the others, first on ties), -1 for a point without observations (mDescriptor
 * untouched); desc_out (n_mp x 32, may be NULL) receives mDescriptor. */
int orbfe_distinctive_descriptors(orbfe_matcher* m, int n_mp, const int32_t* obs_off,
                                  const uint8_t* obs_desc, int32_t* best, uint8_t* desc_out);
/* Device form of the same (asynchronous on the matcher's stream); d_desc_out may be NULL. */
int orbfe_distinctive_descriptors_device(orbfe_matcher* m, int n_mp, const int32_t* d_obs_off,
                                         const uint8_t* d_obs_desc, int32_t* d_best,
                                         uint8_t* d_desc_out);

/* Frame::isInFrustum (Frame.cc:387-443) + MapPoint::PredictScale (MapPoint.cc:633-642) over
 * m MapPoints: world pos (m x 3), normal (m x 3), mfMinDistance/mfMaxDistance.  Writes the
 * tracking scratch fields (mbTrackInView, mTrackProjX/Y/XR, mnTrackScaleLevel,
 * mTrackViewCos). log_scale_factor = mfLogScaleFactor (Frame.cc:185). */
int orbfe_is_in_frustum(orbfe_matcher* m, int n, const float* xyz, const float* normal,
                        const float* min_dist, const float* max_dist, const float* tcw,
                        const orbfe_camera* cam, float min_x, float max_x, float min_y,
                        float max_y, float log_scale_factor, float viewing_cos_limit,
                        uint8_t* in_view, float* proj_x, float* proj_y, float* proj_xr,
                        int32_t* pred_level, float* view_cos);

/* ---- bag of words (DBoW2, vendored in the reference as Thirdparty/DBoW2) ----------------- */

/* ORBVocabulary::loadFromTextFile (TemplatedVocabulary.h:1351-1436), called by System::System
 * on ORBvoc.txt: header "k L scoring weighting", one line per node "parent isLeaf d0..d31
 * weight".  The tree is kept in HBM of `device`.  Blank lines are skipped. */
orbfe_vocabulary* orbfe_vocabulary_load_text(const char* path, int device, int* status);
/* The same from node arrays: node 0 is the root (its entries are ignored); parent[i] < i;
 * is_word flags the leaves that are words (word ids in node order); desc n_nodes x 32. */
orbfe_vocabulary* orbfe_vocabulary_create(int k, int L, int scoring, int weighting, int n_nodes,
                                          const int32_t* parent, const uint8_t* is_word,
                                          const uint8_t* desc, const double* weight, int device,
                                          int* status);
void orbfe_vocabulary_destroy(orbfe_vocabulary* v);
/* info[6] = {k, L, scoring, weighting, nodes, words}. */
int orbfe_vocabulary_info(const orbfe_vocabulary* v, int32_t* info);
int orbfe_vocabulary_set_stream(orbfe_vocabulary* v, void* hip_stream);

/* Frame::ComputeBoW / KeyFrame::ComputeBoW (Frame.cc:513-520) = TemplatedVocabulary::transform(
 * features, BowVector, FeatureVector, levelsup) (TemplatedVocabulary.h:1140-1196) over n
 * descriptors (n <= 4096).  BowVector: nw ascending word ids + values (double, normalised as the
 * vocabulary's scoring requires); FeatureVector: nn ascending node ids (level L - levelsup),
 * CSR offsets node_off[nn + 1] into feat (feature indices, ascending within a node).  Every
 * output array holds at least n entries (node_off n + 1).  Synchronous. */
int orbfe_bow_transform(orbfe_vocabulary* v, const uint8_t* desc, int n, int levelsup,
                        int32_t* word_ids, double* values, int32_t* nw, int32_t* node_ids,
                        int32_t* node_off, int32_t* feat, int32_t* nn);
/* Batched device form: frame f's descriptors at d_desc + f*cap*32 (d_n[f] rows, cap <= 4096);
 * outputs per frame at f*cap (node_off at f*(cap+1)), counts in d_nw[f] / d_nn[f].
 * Asynchronous on the vocabulary's stream (orbfe_vocabulary_set_stream). */
int orbfe_bow_transform_batch_device(orbfe_vocabulary* v, int nframes, const uint8_t* d_desc,
                                     const int32_t* d_n, int cap, int levelsup,
                                     int32_t* d_word_ids, double* d_values, int32_t* d_nw,
                                     int32_t* d_node_ids, int32_t* d_node_off, int32_t* d_feat,
                                     int32_t* d_nn);

/* ORBmatcher::SearchByBoW(KeyFrame* pKF, Frame& F, vector<MapPoint*>& vpMapPointMatches)
 * (ORBmatcher.cc:159-291) with ORBmatcher(nnratio, check_ori) (Tracking.cc:1011 / 1621 use 0.7 /
 * 0.75, checkOri true).  Keyframe: n_kf descriptors, keypoint angles (mvKeysUn), kf_mp_ok[i] =
 * GetMapPointMatches()[i] != NULL && !isBad(), its FeatureVector (kf_nn nodes, CSR).  Frame: n_f
 * descriptors, angles (mvKeys) and FeatureVector.  matches[f] = the keyframe feature whose map
 * point lands in vpMapPointMatches[f], or -1; *nmatches as returned.  A common node holding more
 * than 256 frame features returns ORBFE_ERR_UNSUPPORTED (ORBvoc level-2 nodes hold ~10).  Each
 * FeatureVector must list a feature index under at most one node, as DBoW2 builds it
 * (FeatureVector.cpp:31-45); one that repeats an index returns ORBFE_ERR_ARG.  One kernel
 * launch per call (the common nodes' features gathered into pinned memory); the orientation
 * filter (ORBmatcher.cc:259-281) runs on the host, as in the reference. */
int orbfe_search_by_bow(orbfe_matcher* m, float nnratio, int check_ori, int n_kf,
                        const uint8_t* kf_desc, const float* kf_angle, const uint8_t* kf_mp_ok,
                        int kf_nn, const int32_t* kf_node_ids, const int32_t* kf_node_off,
                        const int32_t* kf_feat, int n_f, const uint8_t* f_desc,
                        const float* f_angle, int f_nn, const int32_t* f_node_ids,
                        const int32_t* f_node_off, const int32_t* f_feat, int32_t* matches,
                        int32_t* nmatches);

/* Batched device form of SearchByBoW for Tracking::Relocalization's candidate loop, which
 * matches the current frame against every relocalisation candidate keyframe with
 * ORBmatcher(0.75, true) (Tracking.cc:1621, 1636-1656): n_pairs (keyframe, frame) problems in
 * one call (n_pairs <= 65535).  Keyframes and frames are slots in the layout
 * orbfe_bow_transform_batch_device writes, with per-slot capacity kf_cap / f_cap: slot s holds
 * descriptors at d_*_desc + s*cap*32, angles (and the keyframe's map-point flags) at s*cap,
 * its FeatureVector's node ids and feature indices at s*cap, node offsets at s*(cap + 1) and
 * node count d_*_nn[s].  Pair p matches keyframe slot d_pair_kf[p] against frame slot
 * d_pair_f[p]; d_matches[p*f_cap + j] = the keyframe feature matched to frame feature j or -1
 * (all f_cap entries written), d_nmatches[p] = the returned count.  *d_status = 0, or
 * ORBFE_ERR_UNSUPPORTED (a common node over 256 frame features) / ORBFE_ERR_ARG (an offset or
 * index outside its slot; that node is skipped).  Asynchronous on the matcher's stream. */
int orbfe_search_by_bow_batch_device(orbfe_matcher* m, float nnratio, int check_ori, int n_pairs,
                                     const int32_t* d_pair_kf, const int32_t* d_pair_f,
                                     int kf_cap, const uint8_t* d_kf_desc,
                                     const float* d_kf_angle, const uint8_t* d_kf_mp_ok,
                                     const int32_t* d_kf_nn, const int32_t* d_kf_node_ids,
                                     const int32_t* d_kf_node_off, const int32_t* d_kf_feat,
                                     int f_cap, const uint8_t* d_f_desc, const float* d_f_angle,
                                     const int32_t* d_f_nn, const int32_t* d_f_node_ids,
                                     const int32_t* d_f_node_off, const int32_t* d_f_feat,
                                     int32_t* d_matches, int32_t* d_nmatches, int32_t* d_status);

/* ---- map-archive records of the extractor outputs (device side) ---------------------------
 * The bodies the reference's Boost map archive stores for the extractor's outputs, written
 * from / read into HBM (MapPoint.h:196-247; KeyFrame::serialize KeyFrame.cc:133-134 / 354-355
 * stores mvKeys, mvKeysUn and mDescriptors, MapPoint::serialize MapPoint.cc:121 / 194 stores
 * mDescriptor).  Keypoint record (serialize(Archive&, cv::KeyPoint&), MapPoint.h:196-209):
 * angle, class_id, octave, response, response, pt.x, pt.y — 28 bytes, size not stored (a
 * loaded keypoint has size 0).  cv::Mat record (save / load, MapPoint.h:215-247): cols i32,
 * rows i32, elemSize u64, type u64, raw bytes; descriptors are rows x 32 CV_8UC1.  Boost's
 * own framing (class-info preamble, collection counts) is the archive writer's.  All entry
 * points are asynchronous on hip_stream (NULL = the null stream) of the current device and take
 * at most 65535 frames / Mats per call. */

/* Bytes of one cv::Mat record: 24 + rows * cols * elem_size (-1 on negative arguments). */
int64_t orbfe_archive_mat_bytes(int rows, int cols, int elem_size);
/* Frame f's min(d_n[f], cap) keypoints (d_keys + f*keys_pitch, orbfe_keypoint units) as
 * consecutive 28-byte records at d_out + f*out_pitch (bytes; a multiple of 4, >= 28*cap). */
int orbfe_archive_write_keypoints_device(int n_frames, const orbfe_keypoint* d_keys,
                                         size_t keys_pitch, const int32_t* d_n, int cap,
                                         uint8_t* d_out, size_t out_pitch, void* hip_stream);
/* The inverse: min(d_n[f], cap) records -> keypoints (size 0, response = the second value). */
int orbfe_archive_read_keypoints_device(int n_frames, const uint8_t* d_in, size_t in_pitch,
                                        const int32_t* d_n, int cap, orbfe_keypoint* d_keys,
                                        size_t keys_pitch, void* hip_stream);
/* Mat k's descriptors (d_desc + k*desc_pitch, rows = d_rows[k], or rows_fixed when d_rows is
 * NULL — 1 for MapPoint::mDescriptor — clipped to cap) as one rows x 32 CV_8UC1 record at
 * d_out + k*out_pitch; d_len[k] (may be NULL) = its bytes.  Pitches are multiples of 8,
 * out_pitch >= orbfe_archive_mat_bytes(cap, 32, 1). */
int orbfe_archive_write_descriptors_device(int n_mats, const uint8_t* d_desc, size_t desc_pitch,
                                           const int32_t* d_rows, int rows_fixed, int cap,
                                           uint8_t* d_out, size_t out_pitch, int64_t* d_len,
                                           void* hip_stream);
/* Reads n_mats descriptor records (d_in + k*in_pitch) into d_desc + k*desc_pitch; d_rows[k]
 * (may be NULL) = rows, or -1 for a record whose header is not (32, rows <= cap, 1, CV_8UC1),
 * which sets *d_status = ORBFE_ERR_ARG (0 otherwise). */
int orbfe_archive_read_descriptors_device(int n_mats, const uint8_t* d_in, size_t in_pitch,
                                          int cap, uint8_t* d_desc, size_t desc_pitch,
                                          int32_t* d_rows, int32_t* d_status, void* hip_stream);

#ifdef __cplusplus
}
#endif
#endif /* ORBFE_H */
