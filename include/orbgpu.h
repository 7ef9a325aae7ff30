/*
 * orbgpu.h -- C ABI of the MI355X-native ORB-SLAM3 front-end / local-BA hot path (liborbgpu.so).
 *
 * Plain pointers, sizes and int status codes only (no OpenCV, Eigen, torch or C++ types), so the
 * reference's C++ (through include/orbgpu_cv.hpp) or any FFI can bind it.
 * Each entry point names the reference interface it replaces (file:line in the reference tree).
 *
 * Threading (reference semantics): calls on DIFFERENT handles may run
 * concurrently from different threads; a single handle is not thread-safe (like one
 * ORB_SLAM3::ORBextractor object, whose mvImagePyramid is per-object state).
 */
#ifndef ORBGPU_H
#define ORBGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes ---------------------------------------------------------------------------- */
#define ORB_OK 0
#define ORB_ERR_EMPTY (-1)     /* empty image: ORBextractor::operator() returns -1 (src/ORBextractor.cc:1561-1562) */
#define ORB_ERR_ARG (-2)       /* invalid argument (null pointer, size beyond the handle's capacity, ...) */
#define ORB_ERR_CAPACITY (-3)  /* caller's output capacity too small; the needed count is still reported */
#define ORB_ERR_DEVICE (-4)    /* HIP runtime error (no GPU, launch failure, out of memory) */
#define ORB_ERR_ABORTED (-5)   /* stopped through the caller's stop flag (LocalBA pbStopFlag) */
#define ORB_ERR_INTERNAL (-6)  /* a device-side capacity guard tripped (should not happen) */

/* cv::KeyPoint memory layout (28 bytes): pt.x, pt.y, size, angle, response, octave, class_id */
typedef struct orb_keypoint {
    float x, y, size, angle, response;
    int32_t octave, class_id;
} orb_keypoint_t;

/* ORBextractor(int nfeatures, float scaleFactor, int nlevels, int iniThFAST, int minThFAST)
 * (include/ORBextractor.h:52-53; values from the YAML keys ORBextractor.* e.g.
 * Examples/Monocular/EuRoC.yaml:50-56) */
typedef struct orb_params {
    int32_t nfeatures;
    float scale_factor;
    int32_t nlevels;
    int32_t ini_th_fast;
    int32_t min_th_fast;
} orb_params_t;

typedef struct orb_extractor_s* orb_extractor_t;

/* Query the library: returns the number of visible HIP devices (0 = none), never fails. */
int orb_device_count(void);
/* Human readable message for the last error on this thread. */
const char* orb_last_error(void);

/* ---- ORBextractor (src/ORBextractor.cc) ------------------------------------------------------ */

/* Create an extractor for frames up to max_width x max_height, batches up to max_batch frames.
 * Replaces ORBextractor::ORBextractor (src/ORBextractor.cc:468-571).  Allocates all device
 * buffers once; no allocation happens per call. */
int orb_extractor_create(const orb_params_t* params, int max_width, int max_height, int max_batch,
                         orb_extractor_t* out);
int orb_extractor_destroy(orb_extractor_t h);

/* GetLevels/GetScaleFactors/GetInverseScaleFactors/GetScaleSigmaSquares/GetInverseScaleSigmaSquares
 * (include/ORBextractor.h:61-83) and the per-level feature budget mnFeaturesPerLevel.
 * Each array receives nlevels values; any pointer may be NULL. */
int orb_extractor_scales(orb_extractor_t h, float* scale, float* inv_scale, float* sigma2,
                         float* inv_sigma2, int32_t* features_per_level);

/* ORBextractor::operator()(image, mask, keypoints, descriptors, vLappingArea)
 * (src/ORBextractor.cc:1557-1682; called from Frame::ExtractORB src/Frame.cc:513-523).
 * Host buffers, synchronous.  image: 8-bit gray, row stride `stride` bytes.  kps/desc hold `cap`
 * entries (desc: cap x 32 bytes).  Keypoints are placed as the reference does: those with
 * lap_x0 <= x <= lap_x1 (level-0 coordinates) from the end backwards, the others from the front.
 * Returns monoIndex (>= 0, the number of front-placed keypoints), ORB_ERR_EMPTY for an empty
 * image, or another negative status.  *n_kps receives the keypoint count (also when the capacity
 * is too small). */
int orb_extract(orb_extractor_t h, const uint8_t* image, int width, int height, int stride,
                int lap_x0, int lap_x1, orb_keypoint_t* kps, uint8_t* desc, int cap, int* n_kps);

/* Batched, device-resident, asynchronous form (the throughput path; no reference counterpart --
 * it runs operator() on n frames at once).  d_images: n frames, frame f at d_images + f*frame_stride,
 * rows `stride` bytes apart.  Frame f writes d_kps[f*cap ...], d_desc[(f*cap ...)*32] and
 * d_counts[2f] = number of keypoints, d_counts[2f+1] = monoIndex (or ORB_ERR_CAPACITY if the frame
 * had more than cap keypoints; then d_counts[2f] still holds the count).  stream: hipStream_t
 * (NULL = default stream).  Returns after enqueueing.  The outputs (and d_images) may also be pinned,
 * device-mapped host memory (hipHostMalloc): the kernels then read / write it over the link, which is
 * how a host-input pipeline skips the download copy. */
int orb_extract_batch_device(orb_extractor_t h, const uint8_t* d_images, int n, int width, int height,
                             int stride, size_t frame_stride, int lap_x0, int lap_x1,
                             orb_keypoint_t* d_kps, uint8_t* d_desc, int cap, int32_t* d_counts,
                             void* stream);

/* Scheduling of a batch on the device path (no reference counterpart).  mode 1 (the default): the
 * early levels' FAST, quad-tree and descriptors run on the handle's side streams beside the small
 * pyramid levels -- the shortest time for one batch alone.  mode 0: a batch runs as one chain on the
 * caller's stream -- the higher throughput when several handles keep batches in flight on their own
 * streams (their side streams would share the process's hardware queues).  Results are identical;
 * takes effect at the next call. */
int orb_extractor_set_overlap(orb_extractor_t h, int mode);

/* mvImagePyramid[level] of frame `frame` of the last call (include/ORBextractor.h:83; read by
 * Frame::ComputeStereoMatches src/Frame.cc:1126,1249).  Gives the device address of the view
 * (first pixel of the level image inside its padded plane), its size and row pitch.  On the device
 * only a 3-pixel REFLECT_101 border around the view is written (all that the stereo matcher's SAD
 * windows and the descriptor's blur reach); the plane extends 19 pixels each way. */
int orb_extractor_level(orb_extractor_t h, int frame, int level, const uint8_t** d_view, int* width,
                        int* height, int* pitch);
/* Copy the padded level plane ((w+38) x (h+38), row-major, tight) to host memory, with its whole
 * 19-pixel border REFLECT_101 as the reference's copyMakeBorder makes it (src/ORBextractor.cc:1712-1716,
 * 1734-1736): the part beyond the device's 3-pixel border is filled on the host. */
int orb_extractor_level_download(orb_extractor_t h, int frame, int level, uint8_t* host_padded);

/* ---- REGISTER_TIMES (include/Settings.h:24, src/Tracking.cc:318-420) ------------------------- */
/* Wall-clock stage timers with the reference's names: "ORB Extraction" (orb_extract; mTimeORB_Ext,
 * src/Frame.cc:132-146), "Stereo Matching" (orb_compute_stereo_matches; src/Frame.cc:158-170), "LBA"
 * (the host side of Optimizer::LocalBundleAdjustment in include/orbgpu_optimizer.hpp, gather to
 * write-back, as vdLBA_ms brackets the whole call, src/LocalMapping.cc:208-219; no sample when the
 * shim returns kFallback).  Off by default.  orb_timers_enable(1) (or ORBGPU_REGISTER_TIMES=1): every
 * orb_extract / orb_compute_stereo_matches call records a sample -- one per image, where the reference
 * records one per Frame (a stereo pair's two extractions, run in parallel, are one sample).
 * orb_timers_enable(2) (or ORBGPU_REGISTER_TIMES=2): no per-call samples; the caller brackets its
 * Frame and records it with orb_timer_add, as Frame.cc does.  orb_timer_stats gives mean and
 * population std (calcAverage / calcDeviation, src/Tracking.cc:189-208); orb_timers_write writes them
 * as ExecMean.txt lines ("ORB Extraction: mean$\pm$std", fixed with 5 decimals: `f << fixed`,
 * src/Tracking.cc:327, then setprecision(5), :335). */
int orb_timers_enable(int on);
/* The timer mode (0 off, 1 per-call brackets, 2 caller brackets only). */
int orb_timers_enabled(void);
int orb_timers_reset(void);
int orb_timer_add(const char* name, double ms);
int orb_timer_stats(const char* name, double* mean_ms, double* std_ms, long long* count);
int orb_timers_write(const char* path);

/* ---- ORBmatcher (src/ORBmatcher.cc) ---------------------------------------------------------- */

/* ORBmatcher::DescriptorDistance (src/ORBmatcher.cc:2384-2404) on host data, for ABI completeness. */
int orb_descriptor_distance(const uint8_t* a, const uint8_t* b);

/* Brute-force Hamming matching on device data: for each query i (n_query x 32 B) find the best and
 * second-best train descriptor (n_train x 32 B).  Writes best_idx[i], best_dist[i], second_dist[i]
 * (256+1 = "none").  The distance is DescriptorDistance.  Device pointers, async on `stream`. */
int orb_hamming_knn2_device(const uint8_t* d_query, int n_query, const uint8_t* d_train, int n_train,
                            int32_t* d_best_idx, int32_t* d_best_dist, int32_t* d_second_dist,
                            void* stream);

/* Cross-frame matching on a batch of device feature blocks (the extractor's [F][cap] layout, e.g. the
 * C4 all-gather's): for each pair p = (query frame pairs[2p], train frame pairs[2p+1]) every query
 * descriptor's best / second-best train descriptor, as orb_hamming_knn2_device (DescriptorDistance,
 * src/ORBmatcher.cc:2384-2404; first index on ties).  Frame f holds counts[f * count_stride] descriptors
 * (read on the device); outputs are [n_pairs][cap], rows beyond the query frame's count get
 * (-1, 257, 257).  cap <= 2048.  One launch, async on `stream`. */
int orb_hamming_knn2_frames_device(const uint8_t* d_desc, const int32_t* d_counts, int count_stride, int cap,
                                   const int32_t* d_pairs, int n_pairs, int32_t* d_best_idx, int32_t* d_best_dist,
                                   int32_t* d_second_dist, void* stream);

/* ---- ORBmatcher::SearchForTriangulation (src/ORBmatcher.cc:1046-1324) ------------------------- */

/* Flat view of the KeyFrame fields SearchForTriangulation reads (host memory).  Pinhole camera,
 * no second camera (mpCamera2 == NULL, NLeft == -1): the configuration LocalMapping runs for
 * monocular / stereo / RGB-D pinhole rigs. */
typedef struct orb_kf_view {
    int32_t n;                     /* KeyFrame::N */
    const orb_keypoint_t* kps_un;  /* mvKeysUn (n) */
    const uint8_t* desc;           /* mDescriptors, n x 32 bytes, row-major */
    const float* u_right;          /* mvuRight (n); NULL = monocular (every entry -1) */
    const uint8_t* has_mappoint;   /* n flags, 1 = GetMapPoint(i) != NULL; NULL = no map points */
    int32_t n_nodes;               /* mFeatVec.size() (DBoW2::FeatureVector, a std::map) */
    const uint32_t* fv_node;       /* node ids, strictly ascending (map order) */
    const int32_t* fv_offset;      /* n_nodes + 1 CSR offsets into fv_index */
    const int32_t* fv_index;       /* feature indices, each node's vector in its order */
    float fx, fy, cx, cy;          /* mpCamera->mvParameters (Pinhole::toK_, src/CameraModels/Pinhole.cpp:168-173) */
    int32_t nlevels;               /* <= 12 */
    const float* scale_factors;    /* mvScaleFactors (nlevels) */
    const float* level_sigma2;     /* mvLevelSigma2 (nlevels) */
} orb_kf_view_t;

/* Per-pair geometry SearchForTriangulation derives from the two poses (src/ORBmatcher.cc:1063-1090):
 * T12 = T1w * Tw2 (R12 row-major, t12) and the epipole ep = pKF2->mpCamera->project(T2w * Cw1).
 * A C++ caller fills it with Sophus exactly as the reference does; orb_kf_pair_geometry computes
 * it from two 3x4 [R|t] poses for callers without Sophus. */
typedef struct orb_kf_pair_geom {
    float R12[9];
    float t12[3];
    float ep[2];
} orb_kf_pair_geom_t;

typedef struct orb_matcher_s* orb_matcher_t;

/* ORBmatcher(float nnratio, bool checkOri) (include/ORBmatcher.h:40).  The handle owns device
 * staging buffers and a stream; one handle per thread (like one ORBmatcher object). */
int orb_matcher_create(float nnratio, int check_orientation, orb_matcher_t* out);
int orb_matcher_destroy(orb_matcher_t m);

/* ---- MapPoint::ComputeDistinctiveDescriptors (src/MapPoint.cc:438-529), batched over map points.
 * Point p's descriptors are rows [offsets[p], offsets[p+1]) of desc (n x 32 bytes): the reference's
 * vDescriptors, i.e. the observations in std::map order, left then right index, bad keyframes
 * skipped.  best[p] receives the row (within the point) whose median distance to the point's rows
 * (index floor(0.5 (N - 1)) of the sorted row, self included) is the smallest, the first one on ties,
 * or -1 for a point without rows; out[32 p ..] receives that descriptor (mDescriptor), untouched for
 * an empty point (the reference returns early).  N < 65536 per point: the host entry rejects a larger
 * point with ORB_ERR_ARG; the device entry cannot see the offsets, so its caller keeps that limit. */
/* Host arrays through the matcher handle's staging buffers, synchronous. */
int orb_compute_distinctive_descriptors(orb_matcher_t m, const uint8_t* desc, const int32_t* offsets, int n_points,
                                        int32_t* best, uint8_t* out);
/* Device arrays (d_offsets: n_points + 1 ints, d_desc / d_out 16-byte aligned), async on `stream`. */
int orb_compute_distinctive_descriptors_device(const uint8_t* d_desc, const int32_t* d_offsets, int n_points,
                                               int32_t* d_best, uint8_t* d_out, void* stream);

/* T1w, T2w: 3x4 row-major [R|t] world->camera poses (float); fx..cy: camera of KF2. */
int orb_kf_pair_geometry(const float T1w[12], const float T2w[12], float fx2, float fy2, float cx2, float cy2,
                         orb_kf_pair_geom_t* out);

/* SearchForTriangulation(pKF1, pKF2[p], vMatchedPairs, bOnlyStereo, bCoarse) for n_pairs
 * neighbours of one keyframe in one launch (LocalMapping::CreateNewMapPoints calls it once per
 * covisible KF, src/LocalMapping.cc:610).  Host memory, synchronous.  Writes
 * matches12[p * kf1->n + i] = matched index in kf2s[p] or -1 (vMatchedPairs is the list of
 * (i, matches12[i]) with matches12[i] >= 0 in increasing i) and n_matches[p] (the return value). */
int orb_search_for_triangulation(orb_matcher_t m, const orb_kf_view_t* kf1, const orb_kf_view_t* kf2s,
                                 const orb_kf_pair_geom_t* geoms, int n_pairs, int only_stereo, int coarse,
                                 int32_t* matches12, int32_t* n_matches);

/* The same search on device-resident keyframes: the features orb_extract_batch_device wrote (d_kps /
 * d_desc at frame f * cap, the count at d_counts[2 f]), the u_right orb_compute_stereo_matches_batch_device
 * wrote and the FeatureVector orb_bow_transform_frames_device wrote, with no host hop for any of them
 * (the chain KeyFrame::ComputeBoW -> LocalMapping::CreateNewMapPoints, src/KeyFrame.cc:109,
 * src/LocalMapping.cc:536-610, after the stereo Frame of src/Frame.cc:136-146).  Counts are read on
 * the device; `cap` bounds them. */
typedef struct orb_kf_device {
    const orb_keypoint_t* kps;     /* device: mvKeysUn, cap entries */
    const uint8_t* desc;           /* device: cap x 32 bytes */
    const int32_t* n;              /* device: KeyFrame::N (e.g. &d_counts[2 f] of orb_extract_batch_device) */
    const float* u_right;          /* device: mvuRight (cap), NULL = monocular */
    const uint8_t* has_mappoint;   /* device: cap flags (GetMapPoint(i) != NULL), NULL = none */
    const int32_t* fv_node;        /* device: FeatureVector node ids, ascending */
    const int32_t* fv_begin;       /* device: n_nodes + 1 offsets into fv_feat */
    const int32_t* fv_feat;        /* device: feature indices, each node's in ascending order */
    const int32_t* n_nodes;        /* device: FeatureVector size (e.g. &d_bow_counts[2 f + 1]) */
    int32_t cap;                   /* upper bound of *n and *n_nodes */
    float fx, fy, cx, cy;          /* host: pinhole parameters */
    int32_t nlevels;               /* <= 12 */
    const float* scale_factors;    /* host: mvScaleFactors */
    const float* level_sigma2;     /* host: mvLevelSigma2 */
} orb_kf_device_t;

/* SearchForTriangulation(kf1s[pair_kf1[p]], kf2s[p]) for p < n_pairs in one launch, device-resident,
 * asynchronous on `stream`: the neighbours of one new keyframe (pair_kf1 = NULL: every pair uses
 * kf1s[0]), or of several queued keyframes.  With C = max over kf1s of cap:
 * d_matches12[p * C + i] = index in kf2s[p] or -1 (i < C); d_n_matches[p] = the count.  The pair
 * geometry and F12 are uploaded from the host (a few hundred bytes per pair).  Counts are clamped to
 * cap; a keyframe whose *n is negative or above cap, or whose *n_nodes is negative (a frame the
 * extractor flagged ORB_ERR_CAPACITY, which the BoW transform passes on), gets no matches and its
 * pairs report d_n_matches[p] = ORB_ERR_CAPACITY. */
int orb_search_for_triangulation_device(orb_matcher_t m, const orb_kf_device_t* kf1s, int n_kf1,
                                        const orb_kf_device_t* kf2s, const int32_t* pair_kf1,
                                        const orb_kf_pair_geom_t* geoms, int n_pairs, int only_stereo, int coarse,
                                        int32_t* d_matches12, int32_t* d_n_matches, void* stream);

/* ---- Frame::UndistortKeyPoints (src/Frame.cc:1003-1051): mvKeysUn from mvKeys by cv::undistortPoints
 * (OpenCV 4.x: five fixed-point iterations of the inverse k1 k2 p1 p2 k3 model in double, P = K, the
 * result rounded to float; parity with a real OpenCV build unpinned), on the extractor's device layout:
 * frame f's keypoints at d_kps[f * cap], its count at d_counts[2 f] (orb_extract_batch_device).
 * d_kps_un receives the same records with pt undistorted (i < count; the rest is not written); a frame
 * flagged ORB_ERR_CAPACITY is skipped.  K = (fx, fy, cx, cy); dist = mDistCoef (n_dist 4 or 5 floats);
 * dist[0] == 0 copies mvKeys, as the reference does.  d_kps_un may equal d_kps.  Async on `stream`. */
int orb_undistort_keypoints_device(const orb_keypoint_t* d_kps, const int32_t* d_counts, int n_frames, int cap,
                                   const float K[4], const float* dist, int n_dist, orb_keypoint_t* d_kps_un,
                                   void* stream);

/* ---- ORBmatcher::SearchByProjection(Frame&, const Frame&, th, bMono) (src/ORBmatcher.cc:1951-2185)
 * Pinhole frames without a second camera (Nleft == -1). */

/* The current frame: keypoints, descriptors, the feature grid bounds (Frame::mnMinX.., the grid
 * element inverse sizes; FRAME_GRID_COLS x ROWS = 64 x 48, include/Frame.h:44-45) and its pose. */
typedef struct orb_frame_view {
    int32_t n;
    const orb_keypoint_t* kps_un;   /* mvKeysUn */
    const uint8_t* desc;            /* mDescriptors, n x 32 */
    const float* u_right;           /* mvuRight (n); NULL = monocular */
    float min_x, max_x, min_y, max_y;       /* mnMinX, mnMaxX, mnMinY, mnMaxY */
    float grid_inv_w, grid_inv_h;           /* mfGridElementWidthInv, mfGridElementHeightInv */
    float fx, fy, cx, cy;                   /* mpCamera parameters */
    float bf, b;                            /* mbf, mb */
    int32_t nlevels;
    const float* scale_factors;             /* mvScaleFactors (nlevels) */
    float Tcw[12];                          /* GetPose(), 3x4 row-major [R|t] */
} orb_frame_view_t;

/* The last frame's tracked map points, indexed like LastFrame's keypoints. */
typedef struct orb_last_points {
    int32_t n;                      /* LastFrame.N */
    const uint8_t* valid;           /* mvpMapPoints[i] != NULL && !mvbOutlier[i] */
    const uint8_t* observed;        /* mvpMapPoints[i]->Observations() > 0 */
    const float* xyz;               /* mvpMapPoints[i]->GetWorldPos(), n x 3 */
    const uint8_t* desc;            /* mvpMapPoints[i]->GetDescriptor(), n x 32 */
    const orb_keypoint_t* kps_un;   /* LastFrame.mvKeysUn (octave and angle) */
    float Tcw[12];                  /* LastFrame.GetPose() */
} orb_last_points_t;

/* match[i2] receives the LastFrame index whose map point was assigned to current keypoint i2 (-1:
 * none).  Like the reference, points are processed in index order and a keypoint already holding
 * a map point with observations is skipped by later points; `check_ori` comes from the matcher
 * handle.  Returns the number of matches in *n_matches.  Host memory, synchronous. */
int orb_search_by_projection_frame(orb_matcher_t m, const orb_frame_view_t* cur, const orb_last_points_t* last,
                                   float th, int mono, int32_t* match, int32_t* n_matches);

/* ---- ORBmatcher::SearchByProjection(Frame&, const vector<MapPoint*>&, th, bFarPoints, thFarPoints)
 * (src/ORBmatcher.cc:46-240, called from Tracking::SearchLocalPoints).  The local map points with the
 * tracking fields Frame::isInFrustum wrote into them (src/Frame.cc:667-773). */
typedef struct orb_local_points {
    int32_t n;                      /* vpMapPoints.size() */
    const uint8_t* track_in_view;   /* mbTrackInView */
    const uint8_t* is_bad;          /* isBad() */
    const uint8_t* observed;        /* Observations() > 0 */
    const float* track_proj;        /* n x 3: mTrackProjX, mTrackProjY, mTrackProjXR */
    const float* track_view_cos;    /* mTrackViewCos */
    const float* track_depth;       /* mTrackDepth */
    const int32_t* track_level;     /* mnTrackScaleLevel */
    const uint8_t* desc;            /* GetDescriptor(), n x 32 */
} orb_local_points_t;

/* frame_taken[i]: F.mvpMapPoints[i] != NULL && ->Observations() > 0 before the call (NULL: none).
 * match[i] receives the index into vpMapPoints of the map point assigned to keypoint i by this
 * call (-1: none); points are processed in order and the ratio test uses the handle's nnratio. */
int orb_search_by_projection_local(orb_matcher_t m, const orb_frame_view_t* frame, const uint8_t* frame_taken,
                                   const orb_local_points_t* pts, float th, int far_points, float th_far_points,
                                   int32_t* match, int32_t* n_matches);

/* ---- The same two searches on device-resident frames (the tracking chain of Tracking::TrackWithMotionModel
 * -> TrackLocalMap, src/Tracking.cc:4112-4217, 4742-4825, without a host hop between the stages).  The
 * current frame's keypoints are the extractor's (or orb_undistort_keypoints_device's) device outputs;
 * counts are read on the device and clamped to `cap`.  Host scalars (pose, bounds, camera) travel in the
 * struct.  Results land in device memory, asynchronously on `stream`: d_match[i] for i < cap (-1 past
 * the frame's count), *d_n_matches.  Every candidate list is sized for the whole frame, so no call is
 * redone; scratch is allocated and freed on `stream`.  The matcher handle contributes only its ratio
 * and orientation flag (calls on different streams may share it). */
typedef struct orb_frame_device {
    const orb_keypoint_t* kps_un;   /* device: mvKeysUn, cap entries */
    const uint8_t* desc;            /* device: cap x 32 */
    const int32_t* n;               /* device: N (e.g. &d_counts[2 f] of orb_extract_batch_device) */
    const float* u_right;           /* device: mvuRight (cap), NULL = monocular */
    int32_t cap;                    /* upper bound of *n, <= 16384 */
    float min_x, max_x, min_y, max_y;       /* mnMinX, mnMaxX, mnMinY, mnMaxY */
    float grid_inv_w, grid_inv_h;           /* mfGridElementWidthInv, mfGridElementHeightInv */
    float fx, fy, cx, cy;                   /* mpCamera parameters */
    float bf, b;                            /* mbf, mb */
    int32_t nlevels;
    const float* scale_factors;             /* host: mvScaleFactors (nlevels) */
    float Tcw[12];                          /* host: GetPose(), 3x4 row-major [R|t] */
} orb_frame_device_t;

/* The last frame's tracked map points, device arrays indexed like its keypoints (cap entries). */
typedef struct orb_last_points_device {
    const int32_t* n;               /* device: LastFrame.N */
    int32_t cap;
    const uint8_t* valid;           /* mvpMapPoints[i] != NULL && !mvbOutlier[i] */
    const uint8_t* observed;        /* mvpMapPoints[i]->Observations() > 0 */
    const float* xyz;               /* mvpMapPoints[i]->GetWorldPos(), cap x 3 */
    const uint8_t* desc;            /* mvpMapPoints[i]->GetDescriptor(), cap x 32 */
    const orb_keypoint_t* kps_un;   /* LastFrame.mvKeysUn (octave and angle) */
    float Tcw[12];                  /* host: LastFrame.GetPose() */
} orb_last_points_device_t;

/* Local map points, device arrays (n on the host: the size of mvpLocalMapPoints), e.g. the outputs of
 * orb_is_in_frustum_device for the tracking fields. */
typedef struct orb_local_points_device {
    int32_t n;
    const uint8_t* track_in_view;
    const uint8_t* is_bad;
    const uint8_t* observed;
    const float* track_proj;        /* n x 3 */
    const float* track_view_cos;
    const float* track_depth;
    const int32_t* track_level;
    const uint8_t* desc;            /* n x 32 */
} orb_local_points_device_t;

int orb_search_by_projection_frame_device(orb_matcher_t m, const orb_frame_device_t* cur,
                                          const orb_last_points_device_t* last, float th, int mono, int32_t* d_match,
                                          int32_t* d_n_matches, void* stream);
/* d_frame_taken: device, cap flags (NULL: none). */
int orb_search_by_projection_local_device(orb_matcher_t m, const orb_frame_device_t* frame, const uint8_t* d_frame_taken,
                                          const orb_local_points_device_t* pts, float th, int far_points,
                                          float th_far_points, int32_t* d_match, int32_t* d_n_matches, void* stream);

/* ---- Frame::isInFrustum (src/Frame.cc:667-773, pinhole, Nleft == -1) + MapPoint::PredictScale
 * (src/MapPoint.cc:715-731): the tracking fields of the local map points that
 * orb_search_by_projection_local reads.  Per point: Pc = Rcw P + tcw, depth > 0, projection inside
 * [mnMinX, mnMaxX] x [mnMinY, mnMaxY], distance to mOw inside [0.8 mfMinDistance, 1.2 mfMaxDistance],
 * viewing cosine against the normal >= viewingCosLimit, predicted level ceil(log(mfMaxDistance /
 * dist) / mfLogScaleFactor) clamped to [0, mnScaleLevels).  Float arithmetic as the reference build
 * contracts it (see oracle/orb_frustum_oracle.cpp). */
typedef struct orb_frustum_frame {
    float Tcw[12];              /* [mRcw | mtcw], row-major 3 x 4 */
    float Ow[3];                /* mOw (camera centre) */
    float fx, fy, cx, cy, bf;   /* pinhole parameters, mbf */
    float min_x, max_x, min_y, max_y;  /* mnMinX, mnMaxX, mnMinY, mnMaxY */
    float log_scale_factor;     /* mfLogScaleFactor */
    int32_t n_levels;           /* mnScaleLevels */
} orb_frustum_frame_t;

/* Host arrays: pos / normal n x 3 (GetWorldPos, GetNormal), min_dist / max_dist (mfMinDistance,
 * mfMaxDistance).  Writes in_view (mbTrackInView), proj n x 3 (mTrackProjX, mTrackProjY -- also set,
 * as in the reference, when only the distance / angle tests fail; -1 before the image test --
 * and mTrackProjXR), depth (mTrackDepth), level (mnTrackScaleLevel), view_cos (mTrackViewCos);
 * fields the reference leaves untouched for rejected points are written as 0.  Synchronous;
 * returns the number of points in view. */
int orb_is_in_frustum(const orb_frustum_frame_t* frame, int n, const float* pos, const float* normal,
                      const float* min_dist, const float* max_dist, float viewing_cos_limit, uint8_t* in_view,
                      float* proj, float* depth, int32_t* level, float* view_cos);
/* The same on device arrays, async on `stream`. */
int orb_is_in_frustum_device(const orb_frustum_frame_t* frame, int n, const float* d_pos, const float* d_normal,
                             const float* d_min_dist, const float* d_max_dist, float viewing_cos_limit,
                             uint8_t* d_in_view, float* d_proj, float* d_depth, int32_t* d_level, float* d_view_cos,
                             void* stream);

/* The same with the frame's pose read on the device: d_pose7 is PoseOptimization's output (the
 * g2o SE3Quat vector tx ty tz qx qy qz qw); the frame's Tcw / Ow follow Frame::SetPose on its float cast
 * (src/Optimizer.cc:390-395, src/Frame.cc:533-599: the quaternion normalised, Eigen's rotation matrix, Ow =
 * q^-1 (-t)); frame->Tcw and frame->Ow are ignored.  The link between PoseOptimization and
 * SearchLocalPoints in the device tracking chain. */
int orb_is_in_frustum_pose_device(const orb_frustum_frame_t* frame, const double* d_pose7, int n, const float* d_pos,
                                  const float* d_normal, const float* d_min_dist, const float* d_max_dist,
                                  float viewing_cos_limit, uint8_t* d_in_view, float* d_proj, float* d_depth,
                                  int32_t* d_level, float* d_view_cos, void* stream);

/* ---- Frame::ComputeStereoMatches (src/Frame.cc:1102-1358) ------------------------------------ */

/* Stereo matching of a rectified pair, on the two extractors' device pyramids (mvImagePyramid of
 * mpORBextractorLeft / mpORBextractorRight, src/Frame.cc:1241,1262) and their keypoints /
 * descriptors: per left keypoint the row-band Hamming search (TH_HIGH start, octave +-1, u range
 * [uL - bf/b, uL], accept < (TH_HIGH+TH_LOW)/2), the 11x11 SAD over +-5 px at the keypoint's
 * level, the parabola sub-pixel fit, the disparity test, then the median cull
 * (SAD >= 1.5*1.4*median dropped).  Writes mvuRight / mvDepth (-1 = no match) for the left
 * keypoints.  `left` and `right` must have extracted frames of the same size with the same
 * parameters; the pyramids of their last extraction are read.
 *
 * Host arrays, frame 0 of each handle (after orb_extract): returns the number of keypoints kept
 * (>= 0) or a negative status.  Synchronous. */
int orb_compute_stereo_matches(orb_extractor_t left, orb_extractor_t right, const orb_keypoint_t* kps_l, int n_l,
                               const uint8_t* desc_l, const orb_keypoint_t* kps_r, int n_r, const uint8_t* desc_r,
                               float bf, float b, float* u_right, float* depth);
/* Device batch: frames 0..n-1 of both handles (after orb_extract_batch_device), keypoints
 * [n][cap] and counts [n][2] (element 0 = keypoint count) exactly as orb_extract_batch_device wrote
 * them.  Writes u_right / depth [n][cap_l] and kept[n].  Async on `stream`. */
int orb_compute_stereo_matches_batch_device(orb_extractor_t left, orb_extractor_t right, int n,
                                            const orb_keypoint_t* d_kps_l, const int32_t* d_counts_l,
                                            const uint8_t* d_desc_l, int cap_l, const orb_keypoint_t* d_kps_r,
                                            const int32_t* d_counts_r, const uint8_t* d_desc_r, int cap_r,
                                            float bf, float b, float* d_u_right, float* d_depth, int32_t* d_kept,
                                            void* stream);

/* ---- DBoW2 TemplatedVocabulary::transform (Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1125-1260)
 * KeyFrame::ComputeBoW / Frame::ComputeBoW (src/KeyFrame.cc:109, src/Frame.cc:1010) call
 * mpORBvocabulary->transform(descriptors, mBowVec, mFeatVec, 4).  Per descriptor: descend the tree
 * from the root taking, at every level, the first child of minimal DescriptorDistance (FORB); the
 * leaf gives the word and its weight; the node passed at level L - levelsup is the FeatureVector
 * node.  TF_IDF / TF weighting: BowVector += weight per word (words with weight 0 are stop words
 * and skipped), then the scoring's normalisation (L1 for ORBvoc's L1_NORM).  The vocabulary is
 * given as flat arrays (ORBvoc.txt itself is not shipped with the reference: .MISSING_LARGE_BLOBS). */

typedef struct orb_vocabulary_view {
    int32_t k, L;                 /* m_k, m_L (the tree may be unbalanced) */
    int32_t weighting;            /* DBoW2 WeightingType: 0 TF_IDF, 1 TF, 2 IDF, 3 BINARY */
    int32_t scoring;              /* DBoW2 ScoringType: 0 L1_NORM, 1 L2_NORM, 2 CHI_SQUARE, 3 KL, 4 BHATTACHARYYA, 5 DOT_PRODUCT */
    int32_t n_nodes;              /* node 0 = root */
    const int32_t* child_begin;   /* n_nodes + 1: children of node i = child_idx[child_begin[i] .. child_begin[i+1]) in Node::children order */
    const int32_t* child_idx;
    const uint8_t* desc;          /* n_nodes x 32 bytes (the root's is unused) */
    const int32_t* word_id;       /* per node: WordId of a leaf, -1 for inner nodes */
    const double* weight;         /* per node: the leaf's WordValue */
} orb_vocabulary_view_t;

typedef struct orb_vocabulary_s* orb_vocabulary_t;

/* Upload a vocabulary (copied; the view may be freed afterwards). */
int orb_vocabulary_create(const orb_vocabulary_view_t* view, orb_vocabulary_t* out);
int orb_vocabulary_destroy(orb_vocabulary_t v);

/* transform() of n descriptors (host, n x 32 bytes).  Outputs, each with capacity n:
 * bow_word / bow_value (BowVector in ascending WordId order, *n_words entries), fv_node (FeatureVector
 * nodes ascending, *n_nodes entries), fv_begin (n_nodes + 1 offsets into fv_feat), fv_feat (feature
 * indices, ascending within a node).  Synchronous.  n <= 8192. */
int orb_bow_transform(orb_vocabulary_t v, const uint8_t* desc, int n, int levelsup, int32_t* bow_word,
                      double* bow_value, int32_t* n_words, int32_t* fv_node, int32_t* fv_begin, int32_t* fv_feat,
                      int32_t* n_nodes);
/* Device batch: frames f = 0..n_frames-1 hold descriptors d_desc[frame_begin[f] .. frame_begin[f+1])
 * (d_frame_begin: n_frames + 1 device ints, each frame <= 8192).  Per frame f the outputs start at
 * frame_begin[f] in every array (capacity = the frame's count; fv_begin: frame_begin[f] + f, with
 * count + 1 entries); d_counts[2 f] = n_words, d_counts[2 f + 1] = n_nodes.  Async on `stream`. */
int orb_bow_transform_batch_device(orb_vocabulary_t v, const uint8_t* d_desc, const int32_t* d_frame_begin,
                                   int n_frames, int n_total, int levelsup, int32_t* d_bow_word,
                                   double* d_bow_value, int32_t* d_fv_node, int32_t* d_fv_begin, int32_t* d_fv_feat,
                                   int32_t* d_counts, void* stream);
/* The same on the frames as orb_extract_batch_device leaves them: frame f's descriptors at
 * d_desc[f * cap * 32 ..], its count at d_kp_counts[2 f] (<= cap, <= 8192).  Per frame f the outputs
 * start at f * cap in every array (fv_begin at f * (cap + 1)); d_counts[2 f] = n_words,
 * d_counts[2 f + 1] = n_nodes.  A frame the extractor flagged (d_kp_counts[2 f + 1] ==
 * ORB_ERR_CAPACITY, or a count outside [0, cap]) is not read: both its counts are ORB_ERR_CAPACITY.
 * Async on `stream`. */
int orb_bow_transform_frames_device(orb_vocabulary_t v, const uint8_t* d_desc, const int32_t* d_kp_counts, int n_frames,
                                    int cap, int levelsup, int32_t* d_bow_word, double* d_bow_value, int32_t* d_fv_node,
                                    int32_t* d_fv_begin, int32_t* d_fv_feat, int32_t* d_counts, void* stream);

/* ---- Optimizer::LocalBundleAdjustment (src/Optimizer.cc:1740-2188) ----------------------------- */
/* The shim keeps the reference's graph gather (B1, src/Optimizer.cc:1744-1855) and the culling /
 * write-back (B10, :2107-2185) on the host and hands the flattened g2o problem across this ABI; the
 * library runs g2o's Levenberg-Marquardt (optimization_algorithm_levenberg.cpp:61-169) with the
 * BlockSolver_6_3 Schur complement (block_solver.hpp:354-486) on the GPU, FP64 throughout. */

typedef struct orb_ba_camera {  /* per keyframe: pKFi->fx, fy, cx, cy, mbf (floats upstream) */
    float fx, fy, cx, cy, bf;
} orb_ba_camera_t;

typedef struct orb_ba_edge {
    int32_t point;      /* index into the point arrays (vertex 0 of the g2o edge) */
    int32_t pose;       /* index into the pose arrays (vertex 1) */
    int32_t stereo;     /* 0: ORB_SLAM3::EdgeSE3ProjectXYZ (u, v), Huber sqrt(5.991);
                           1: g2o::EdgeStereoSE3ProjectXYZ (u, v, u_right), Huber sqrt(7.815) */
    float inv_sigma2;   /* pKFi->mvInvLevelSigma2[kpUn.octave]: information = I * inv_sigma2 */
    double obs[3];      /* measurement (obs[2] unused for mono edges) */
} orb_ba_edge_t;

typedef struct orb_ba_problem {
    int32_t n_poses, n_points, n_edges;
    double* pose;                         /* n_poses x 7, in/out: g2o::SE3Quat::toVector (tx ty tz qx qy qz qw) of Tcw */
    const int64_t* pose_id;               /* vertex ids (KeyFrame::mnId), unique */
    const uint8_t* pose_fixed;            /* 1 = setFixed(true) (the map's init KF and the fixed covisible KFs) */
    const orb_ba_camera_t* pose_camera;   /* n_poses */
    double* point;                        /* n_points x 3, in/out: world position */
    const int64_t* point_id;              /* vertex ids (MapPoint::mnId + maxKFid + 1), above every pose id */
    const orb_ba_edge_t* edges;           /* n_edges, in insertion (edge id) order */
} orb_ba_problem_t;

typedef struct orb_ba_options {
    int32_t iterations;                   /* optimizer.optimize(10) (src/Optimizer.cc:2101) */
    double user_lambda_init;              /* 0: tau * max diag(H) (tau = 1e-5); >0: setUserLambdaInit */
    const volatile int32_t* stop_flag;    /* pbStopFlag (polled between iterations and trials), may be NULL */
    const volatile uint8_t* stop_flag_bool;  /* the same for a C++ `bool* pbStopFlag` (one byte, nonzero = stop),
                                                as LocalMapping passes &mbAbortBA (src/LocalMapping.cc:208); may be NULL */
} orb_ba_options_t;

typedef struct orb_ba_result {
    int32_t iterations;       /* iterations run (SparseOptimizer::optimize's return value) */
    int32_t trials;           /* LM trials (linear solves) over all iterations */
    int32_t terminated;       /* 1 if the algorithm returned Terminate (no progress / 3 bad steps) */
    int32_t stopped;          /* 1 if the stop flag ended the run */
    double initial_chi2;      /* robust chi2 before the first update */
    double final_chi2;        /* robust chi2 of the accepted state */
    double lambda;            /* final LM damping */
} orb_ba_result_t;

typedef struct orb_ba_s* orb_ba_t;

int orb_ba_create(orb_ba_t* out);
int orb_ba_destroy(orb_ba_t h);

/* Optimise `problem` in place (poses and points).  edge_chi2[e] receives e->chi2() as the culling
 * pass reads it after optimize() (the error of the last evaluated state, robust kernel not applied)
 * and edge_depth_ok[e] e->isDepthPositive() for the final estimates (either may be NULL).
 * Returns ORB_OK, ORB_ERR_ABORTED if the stop flag was set before the first iteration, or an error. */
int orb_ba_optimize(orb_ba_t h, orb_ba_problem_t* problem, const orb_ba_options_t* options, double* edge_chi2,
                    uint8_t* edge_depth_ok, orb_ba_result_t* result);

/* ---- Optimizer::PoseOptimization (src/Optimizer.cc:55-415) ------------------------------------ */
/* Motion-only BA of tracking, batched over frames.  Per frame: one g2o::VertexSE3Expmap (Tcw) and a
 * unary edge per matched MapPoint -- ORB_SLAM3::EdgeSE3ProjectXYZOnlyPose (mono, Huber sqrt(5.991))
 * or g2o::EdgeStereoSE3ProjectXYZOnlyPose (mvuRight >= 0, Huber sqrt(7.815)) -- then 4 rounds of
 * optimize(10) with g2o's Levenberg-Marquardt and LinearSolverDense, each round restarting from the
 * frame's pose, re-classifying every edge by chi2 > 5.991 / 7.815 (the error of the last evaluated
 * state for active edges, recomputed for outliers), the robust kernels removed after round 2, and
 * the early exit when the frame has fewer than 10 edges.  Pinhole, single camera (mpCamera2 ==
 * NULL); the fisheye two-camera edge (EdgeSE3ProjectXYZOnlyPoseToBody) is not covered. */

typedef struct orb_pose_edge {
    double xw[3];        /* pMP->GetWorldPos().cast<double>() */
    double obs[3];       /* kpUn.pt.x, kpUn.pt.y, mvuRight[i] (stereo only) */
    float inv_sigma2;    /* mvInvLevelSigma2[kpUn.octave] */
    int32_t stereo;      /* mvuRight[i] >= 0 */
} orb_pose_edge_t;

typedef struct orb_pose_frame {
    double pose[7];          /* Tcw as g2o::SE3Quat::toVector (tx ty tz qx qy qz qw), in */
    orb_ba_camera_t cam;     /* fx, fy, cx, cy, mbf */
    int32_t edge_begin;      /* this frame's edges: edges[edge_begin, edge_begin + n_edges) */
    int32_t n_edges;         /* = nInitialCorrespondences */
} orb_pose_frame_t;

/* Host arrays, synchronous.  pose_out[7 f]: the optimised Tcw (unchanged when the frame has fewer
 * than 3 edges); outlier[e]: mvbOutlier of edge e after the last round; inliers[f]: the return value
 * of PoseOptimization (nInitialCorrespondences - nBad, 0 below 3 correspondences). */
int orb_pose_optimization(int n_frames, const orb_pose_frame_t* frames, int n_edges, const orb_pose_edge_t* edges,
                          double* pose_out, uint8_t* outlier, int32_t* inliers);
/* The same on device arrays, asynchronous on `stream` (one workgroup per frame). */
int orb_pose_optimization_device(int n_frames, const orb_pose_frame_t* d_frames, int n_edges,
                                 const orb_pose_edge_t* d_edges, double* d_pose_out, uint8_t* d_outlier,
                                 int32_t* d_inliers, void* stream);

/* ---- the device tracking chain's glue (Tracking::TrackWithMotionModel / TrackLocalMap,
 * src/Tracking.cc:4112-4217, 4234-4300) between the matchers and PoseOptimization, on device arrays.
 * PoseOptimization's graph for one device frame (src/Optimizer.cc:93-180): an edge per keypoint i < N
 * whose map point is d_match_b[i] (>= 0, a row of d_xyz_b) or else d_match_a[i] (a row of d_xyz_a), in
 * keypoint order; stereo when u_right[i] >= 0; information inv_level_sigma2[octave] (host, nlevels);
 * the camera from the frame view.  The start pose is d_pose (device, 7 doubles: the previous
 * optimisation's result) or else pose (host).  Writes *d_frame (edge_begin 0, n_edges = the count),
 * d_edges (up to cap) and d_edge_kp[e] = the keypoint of edge e.  d_match_b may be NULL. */
int orb_tracking_pose_edges_device(const orb_frame_device_t* frame, const int32_t* d_match_a, const float* d_xyz_a,
                                   const int32_t* d_match_b, const float* d_xyz_b, const float* inv_level_sigma2,
                                   const double* d_pose, const double pose[7], orb_pose_frame_t* d_frame,
                                   orb_pose_edge_t* d_edges, int32_t* d_edge_kp, void* stream);
/* TrackWithMotionModel's outlier discard (src/Tracking.cc:4180-4203): each edge PoseOptimization marked
 * an outlier clears its keypoint's map point in both match arrays; d_n_out[0] = the edges kept,
 * d_n_out[1] = those whose map point has observations (nmatchesMap; d_observed_a / _b per table row,
 * NULL = all observed).  d_match_b may be NULL.  d_taken (optional, cap entries): afterwards, whether
 * keypoint i holds a map point with observations -- SearchByProjection(F, local points)'s skip set. */
int orb_tracking_discard_outliers_device(const orb_pose_frame_t* d_frame, const int32_t* d_edge_kp,
                                         const uint8_t* d_outlier, int32_t* d_match_a, const uint8_t* d_observed_a,
                                         int32_t* d_match_b, const uint8_t* d_observed_b, int32_t* d_n_out, int cap,
                                         uint8_t* d_taken, void* stream);
/* SearchLocalPoints' skip of the map points the frame has seen (src/Tracking.cc:4745-4766, 4778, the
 * mnLastFrameSeen test): local map point j is the last frame's row d_last_row[j] (-1: not tracked by the
 * last frame); when a keypoint's d_match_a (cap entries: SearchByProjection(LastFrame)'s assignments
 * BEFORE the discard, since the discarded outliers are marked seen too, :4195) names that row,
 * d_in_view[j] (orb_is_in_frustum*_device's output) is cleared.  last_cap <= 16384. */
int orb_tracking_local_seen_device(const int32_t* d_match_a, int cap, int last_cap, const int32_t* d_last_row,
                                   int n_local, uint8_t* d_in_view, void* stream);

/* The whole chain in one call (the sequence above): SearchByProjection(F, LastFrame)
 * -> PoseOptimization -> isInFrustum at the new pose + the seen skip -> discard -> SearchByProjection(F,
 * local points) -> PoseOptimization, every stage async on `stream`.  The caller owns the per-frame
 * device buffers (sized for frame->cap; m1 / m2 and the pose outputs are the results) and the local
 * map's tracking-field arrays (local->track_* are written by the frustum stage).
 *
 * With params->motion_gate, TrackWithMotionModel's decisions run on the device with no host sync
 * (src/Tracking.cc:4149-4217): fewer than 20 matches -> the search again with 2 th; still fewer than 20
 * -> TrackWithMotionModel returns false: no PoseOptimization, no local-map stages; after the first
 * PoseOptimization and the discard, nmatchesMap < 10 -> it returns false too and the local-map stages
 * are skipped (the reference's Track() then runs TrackReferenceKeyFrame, the caller's).  The per-frame
 * status word says which (ORB_TRACK_*).  For a frame that fails: m1 holds the last search's matches
 * (status FAIL_SEARCH: not discarded, no graph: n_edges 0, pose1 = the motion model's pose) or the
 * discarded ones (FAIL_MAP); m2 is all -1 and n_match[1] 0; the second graph is empty and pose2 is the
 * pose the Frame keeps after TrackWithMotionModel (pose1 through Frame::SetPose's float round trip);
 * the local map's track_* fields hold the frustum test at pose1 (no reference step reads them before
 * recomputing them). */
#define ORB_TRACK_RETRIED 1      /* the first search found < 20: the 2 th search ran */
#define ORB_TRACK_FAIL_SEARCH 2  /* < 20 matches after the retry: TrackWithMotionModel false */
#define ORB_TRACK_FAIL_MAP 4     /* nmatchesMap < 10 after PoseOptimization: TrackWithMotionModel false */
typedef struct orb_tracking_chain_params {
    float th_motion;            /* TrackWithMotionModel's th: 7 stereo, 15 otherwise (src/Tracking.cc:4141-4146) */
    int32_t mono;               /* bMono of SearchByProjection(F, LastFrame) */
    float th_local;             /* SearchLocalPoints' th (src/Tracking.cc:4801-4823) */
    int32_t far_points;         /* mpLocalMapper->mbFarPoints */
    float th_far_points;        /* mpLocalMapper->mThFarPoints */
    float viewing_cos_limit;    /* isInFrustum's 0.5 */
    int32_t motion_gate;        /* 1: TrackWithMotionModel's retry / failure decisions on the device (above);
                                   0: every stage runs on every frame with th_motion as given */
} orb_tracking_chain_params_t;

typedef struct orb_tracking_chain_buffers {
    int32_t* m1;                /* cap: SearchByProjection(LastFrame)'s last-frame row per keypoint, after the discard */
    int32_t* m2;                /* cap: SearchByProjection(local)'s local point per keypoint */
    int32_t* n_match;           /* 2: the two searches' counts */
    orb_pose_frame_t* frames;   /* 2: the two PoseOptimization graphs' frame records */
    orb_pose_edge_t* edges1;    /* cap */
    orb_pose_edge_t* edges2;    /* cap */
    int32_t* edge_kp1;          /* cap: keypoint of each edge */
    int32_t* edge_kp2;
    uint8_t* outlier1;          /* cap: mvbOutlier per edge */
    uint8_t* outlier2;
    double* poses;              /* 14: the two optimised poses (SE3Quat vectors) */
    int32_t* inliers;           /* 2: the two PoseOptimization returns */
    int32_t* n_out;             /* 2: nmatches after the discard, nmatchesMap */
    uint8_t* taken;             /* cap: SearchLocalPoints' skip set */
    void* scratch;              /* orb_tracking_chain_scratch_bytes(cap, last cap, local points), reused stage
                                   after stage on the stream (required) */
    int32_t* status;            /* 1: ORB_TRACK_* bits (0: tracked by the motion model); NULL: not reported */
} orb_tracking_chain_buffers_t;

/* Scratch bytes of one chain call for frames of `cap` keypoints, a last frame of `last_cap` and `n_local`
 * local map points (the largest of its stages'). */
size_t orb_tracking_chain_scratch_bytes(int cap, int last_cap, int n_local);

/* m_motion: ORBmatcher(0.9, true); m_local: ORBmatcher(0.8) (the handles' ratio / orientation).
 * local: the local map's view (track_* arrays written here); pos / normal / min_dist / max_dist:
 * GetWorldPos / GetNormal / mfMinDistance / mfMaxDistance per local point; last_row: -1 or the last
 * frame's row holding the point (NULL: none holds one).  frustum: the frame's bounds, camera, log scale
 * and levels (its pose fields are ignored).  pose7: the motion model's pose as PoseOptimization reads
 * it (tx ty tz qx qy qz qw of the frame's float pose; frame->Tcw must be the same pose). */
int orb_tracking_chain_device(orb_matcher_t m_motion, orb_matcher_t m_local, const orb_frame_device_t* frame,
                              const orb_last_points_device_t* last, const orb_local_points_device_t* local,
                              const float* d_pos, const float* d_normal, const float* d_min_dist,
                              const float* d_max_dist, const int32_t* d_last_row, const orb_frustum_frame_t* frustum,
                              const float* inv_level_sigma2, const double pose7[7],
                              const orb_tracking_chain_params_t* params, const orb_tracking_chain_buffers_t* bufs,
                              void* stream);

/* The chain over a batch of frames in one call: every stage is one launch for the whole batch (one
 * grid row per frame), so B frames cost one host crossing and ~20 launches instead of B of each, and
 * the frames' single-workgroup stages (the resolve, PoseOptimization) run side by side over the CUs.
 * Frame b's results are the single call's on the same inputs, bit for bit.  All frames share `cap`
 * (their frame views' cap); a last frame and a local map per frame; at most 65535 frames per call. */
typedef struct orb_tracking_chain_frame {
    const orb_frame_device_t* frame;
    const orb_last_points_device_t* last;
    const orb_local_points_device_t* local;   /* its track_* arrays are written */
    const float* pos;                         /* the local map's fields, as orb_tracking_chain_device */
    const float* normal;
    const float* min_dist;
    const float* max_dist;
    const int32_t* last_row;                  /* NULL: no local point is held by the last frame */
    const orb_frustum_frame_t* frustum;
    const float* inv_level_sigma2;            /* host, nlevels floats */
    double pose7[7];                          /* the motion model's pose (tx ty tz qx qy qz qw) */
} orb_tracking_chain_frame_t;

typedef struct orb_tracking_chain_batch_buffers {
    int32_t* m1;                /* B x cap */
    int32_t* m2;                /* B x cap */
    int32_t* n_match;           /* B x 2 */
    orb_pose_frame_t* frames;   /* 2 x B (B = the call's n_frames): the first graphs, then the second ones */
    orb_pose_edge_t* edges1;    /* B x cap (frame b's edges from b cap on) */
    orb_pose_edge_t* edges2;    /* B x cap */
    int32_t* edge_kp1;          /* B x cap */
    int32_t* edge_kp2;          /* B x cap */
    uint8_t* outlier1;          /* B x cap */
    uint8_t* outlier2;          /* B x cap */
    double* poses;              /* 2 x B x 7 (B = the call's n_frames) */
    int32_t* inliers;           /* 2 x B */
    int32_t* n_out;             /* B x 2 */
    uint8_t* taken;             /* B x cap */
    void* scratch;              /* orb_tracking_chain_batch_scratch_bytes(B, cap, max last cap, max local points) */
    int32_t* status;            /* B: ORB_TRACK_* bits per frame; NULL: not reported */
} orb_tracking_chain_batch_buffers_t;

size_t orb_tracking_chain_batch_scratch_bytes(int n_frames, int cap, int last_cap, int n_local);
/* Release the pinned host staging the batch calls keep for `scratch`: waits until the last call made
 * with it has finished on the device (every kernel, not only its argument copies), then frees the
 * staging; call it before the scratch or the call's output buffers are freed or reused for something
 * else.  A NULL or unknown scratch is a no-op.
 * Memory: the scratch holds, per frame, the SearchByProjection candidate lists (8 B per (point,
 * keypoint) pair: cap x max(last cap, local points) x 8 B) -- e.g. cap 2048 and 2048 points: 32 MiB per
 * frame, 16 GiB for 512 frames; orb_tracking_chain_batch_scratch_bytes gives the exact size. */
int orb_tracking_chain_batch_release(void* scratch);
int orb_tracking_chain_batch_device(orb_matcher_t m_motion, orb_matcher_t m_local, int n_frames,
                                    const orb_tracking_chain_frame_t* frames, const orb_tracking_chain_params_t* params,
                                    const orb_tracking_chain_batch_buffers_t* bufs, void* stream);

/* ---- multi-GPU local BA: one process per GPU, every rank passes the same
 * problem; rank r owns a contiguous, edge-balanced range of the landmarks and their edges, and
 * the ranks all-reduce the partial Hpp/b_p, the partial reduced camera system (S, b_S) of each LM
 * trial and the chi2 / scale partials.  Every rank factors S and updates the poses identically,
 * and the results of all ranks are identical. */
#define ORB_BA_SUM 0
#define ORB_BA_MAX 1
/* In-place all-reduce of n doubles in host memory across the ranks; returns 0 on success. */
typedef int (*orb_ba_host_reduce_fn)(void* ctx, double* host_buf, size_t n, int op);

/* ncclGetUniqueId of the RCCL loaded in the process (librccl.so.1); 128 bytes. */
int orb_ba_dist_unique_id(uint8_t id[128]);
/* Attach an RCCL communicator (ncclCommInitRank over `id`) to the handle: device all-reduces. */
int orb_ba_dist_init_rccl(orb_ba_t h, const uint8_t id[128], int world, int rank);
/* Attach a host-memory reducer instead (e.g. an MPI or gloo all-reduce). */
int orb_ba_dist_init_host(orb_ba_t h, orb_ba_host_reduce_fn fn, void* ctx, int world, int rank);

#ifdef __cplusplus
}
#endif

#endif /* ORBGPU_H */
