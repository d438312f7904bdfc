/*
 * orbslam_gpu.h -- C ABI of the MI355X-native ORB-SLAM2 per-frame hot path.
 *
 * Drop-in boundary for junejunejune/c_orb_slam (ORB-SLAM2, C++11).  The
 * reference exposes these operations as C++ class methods taking cv::Mat /
 * std::vector; each entry point below replaces one of them with plain
 * pointers + sizes.  The C++ adapter in
 * c_orb_slam_amd/adapter/ re-exposes the reference class signatures on top
 * of this header; INTEGRATION.md shows the binding a maintainer adds.
 *
 * Conventions
 *   - every call returns int status: ORB_OK (0) or a negative ORB_E_*;
 *   - the caller owns all host buffers (pointer + capacity; counts are
 *     written to *n_out; ORB_E_CAPACITY if a buffer is too small);
 *   - each handle owns its device workspace and one HIP stream; handles are
 *     not shared between threads (the reference calls the extractor from two
 *     threads per stereo frame, Frame.cc:78-81: create one handle per thread);
 *   - there is no CPU fallback: without a usable gfx950 device, create()
 *     returns ORB_E_NODEVICE.
 */
#ifndef ORBSLAM_GPU_H
#define ORBSLAM_GPU_H
#include <stdbool.h>
#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ORB_OK 0
#define ORB_E_INVALID -1
#define ORB_E_HIP -2
#define ORB_E_CAPACITY -3
#define ORB_E_NODEVICE -4

/* cv::KeyPoint memory layout (28 B): pt.x, pt.y, size, angle, response, octave, class_id */
typedef struct orb_kp {
    float x, y, size, angle, response;
    int32_t octave, class_id;
} orb_kp;

/* Library info: 1 if a HIP device is usable, else 0 (never aborts). */
int orbgpu_device_available(void);
const char* orbgpu_version(void);
/* ABI revision of this header.  A caller compiled against revision R checks
 * orbgpu_abi_version() == R at start-up: an entry point whose signature changed bumps it.
 *   1: round 1-3 ABI
 *   2: ORBmatcher_SearchLocalPoints_batch takes the ORBmatcher(nnratio) float before the
 *      outputs (a revision-1 binary would pass its pointers with nnratio undefined) */
#define ORBGPU_ABI_VERSION 2
int orbgpu_abi_version(void);

/* ======================================================================
 * ORBextractor  (reference include/ORBextractor.h:51-113, src/ORBextractor.cc)
 * ====================================================================== */
typedef struct ORBextractor_t* ORBextractor_h;

/* ORBextractor::ORBextractor(int nfeatures, float scaleFactor, int nlevels,
 *                            int iniThFAST, int minThFAST)   ORBextractor.cc:410-470
 * max_width/max_height size the device pyramid (images up to that size). */
int ORBextractor_create(int nfeatures, float scaleFactor, int nlevels, int iniThFAST,
                        int minThFAST, int max_width, int max_height, int max_batch,
                        ORBextractor_h* out);
int ORBextractor_destroy(ORBextractor_h h);

/* ORBextractor::operator()(image, mask(ignored), keypoints, descriptors)
 *                                                          ORBextractor.cc:1043-1105
 * img: u8 grey, row stride `step`.  kps: capacity entries; desc: capacity x 32.
 * Empty image (w or h == 0) returns ORB_OK with *n_out = 0 (1046-1047). */
int ORBextractor_extract(ORBextractor_h h, const uint8_t* img, int width, int height, int step,
                         orb_kp* kps, uint8_t* desc, int capacity, int* n_out);

/* Batched form: `batch` images of equal size; image b at imgs + b*img_stride.
 * imgs_on_device != 0: imgs is a device pointer (HBM-resident input).
 * Outputs for image b at kps + b*cap_per_image, desc + b*cap_per_image*32;
 * outputs_on_device != 0: kps/desc are device pointers.  n_out[b] host. */
int ORBextractor_extract_batch(ORBextractor_h h, const uint8_t* imgs, int batch, int width,
                               int height, int step, size_t img_stride, int imgs_on_device,
                               orb_kp* kps, uint8_t* desc, int cap_per_image,
                               int outputs_on_device, int* n_out);

/* Host images at separate addresses: Frame(imLeft, imRight)'s two cv::Mat (Frame.cc:78-81 runs
 * the left and right extractors on two threads; here both are one call on one stream).  Image b
 * at imgs[b] (host, row stride `step`); the images are staged in one pinned block and copied to
 * HBM with one H2D copy.  Outputs as ORBextractor_extract_batch (image b at kps + b*cap). */
int ORBextractor_extract_images(ORBextractor_h h, const uint8_t* const* imgs, int batch, int width,
                                int height, int step, orb_kp* kps, uint8_t* desc, int cap_per_image,
                                int outputs_on_device, int* n_out);

/* mvImagePyramid[level] (ORBextractor.h:85) of image `index` of the last call,
 * copied to host WITH its 19-px REFLECT_101 border (Frame.cc:573-580 reads it).
 * dst must hold (w+38)*(h+38) bytes at stride dst_step; *w,*h = unpadded dims. */
int ORBextractor_get_level(ORBextractor_h h, int index, int level, uint8_t* dst, int dst_step,
                           int* w, int* h_);
/* Diagnostic: the GaussianBlur(7x7, 2) working image of `level` (ORBextractor.cc:1085-1086,
 * no border) of image `index` of the last call; dst holds w*h bytes at dst_step. */
int ORBextractor_get_blurred_level(ORBextractor_h h, int index, int level, uint8_t* dst,
                                   int dst_step, int* w, int* h_);
/* GetLevels/GetScaleFactor/GetScaleFactors/GetInverseScaleFactors/
 * GetScaleSigmaSquares/GetInverseScaleSigmaSquares   ORBextractor.h:63-85 */
int ORBextractor_get_levels(ORBextractor_h h, int* nlevels, float* scaleFactor);
int ORBextractor_get_scale_tables(ORBextractor_h h, float* scale, float* invScale,
                                  float* sigma2, float* invSigma2, int* nFeaturesPerLevel);
/* HIP stream (hipStream_t) the extractor launches on; for event timing. */
void* ORBextractor_stream(ORBextractor_h h);
/* Per-stage device time of the last call (ms), from HIP events:
 * [0]=pyramid [1]=blur [2]=FAST cells [3]=compaction [4]=octree(host) [5]=orientation+rBRIEF */
int ORBextractor_last_timings(ORBextractor_h h, float* ms6);
/* FAST corners kept by the last call, summed over its images (after the per-cell NMS and cell
 * caps of ORBextractor.cc:776-829, before DistributeOctTree): the k_fast_cells output that the
 * bench's algorithmic-bytes figure counts. */
int ORBextractor_last_corner_count(ORBextractor_h h, long long* total);
/* Scheduling (no reference counterpart): keep one CU in every `one_in_n` of each XCD out of
 * this extractor's launches (its stream is recreated with a CU mask), so the tracking lane's
 * one-workgroup-per-frame kernels (matcher greedy replay, PoseOptimization) find free wave
 * slots while a batch is being extracted.  one_in_n = 0 restores the full device.  Call
 * between extractions; ORBextractor_stream() changes. */
int ORBextractor_reserve_cus(ORBextractor_h h, int one_in_n);
/* Scheduling (no reference counterpart): h launches on `with`'s stream from now on, so the
 * extractions of two extractors queue back to back on the device in call order (a pipeline
 * that enqueues batch k+1 while batch k runs leaves no gap between them).  `with` keeps owning
 * the stream and must outlive h; ORBextractor_reserve_cus is refused on both afterwards. */
int ORBextractor_share_stream(ORBextractor_h h, ORBextractor_h with);

/* ======================================================================
 * ORBmatcher  (reference include/ORBmatcher.h:41-103, src/ORBmatcher.cc)
 * ====================================================================== */
typedef struct ORBmatcher_t* ORBmatcher_h;

/* ORBmatcher::ORBmatcher(float nnratio=0.6, bool checkOri=true)  ORBmatcher.cc:41-43 */
int ORBmatcher_create(float nnratio, int checkOri, ORBmatcher_h* out);
int ORBmatcher_destroy(ORBmatcher_h h);
/* Pointer space of every array argument below (and inside orb_frame /
 * orb_mappoints): 0 = host memory (default, copied per call), 1 = device
 * (HBM-resident, e.g. ORBextractor_extract_batch outputs); counts stay host. */
int ORBmatcher_set_device_pointers(ORBmatcher_h h, int on);
void* ORBmatcher_stream(ORBmatcher_h h);

/* Measurement (no reference counterpart; bench roofline): with timing on, every search,
 * stereo and CSR call on this matcher records HIP events around its kernels on
 * ORBmatcher_stream() and counts its work on the device.  ORBmatcher_last_timings waits for
 * the stream and returns the last call's kernel times (ms, -1 = not run):
 *   ms8[0..6]: k_build_grid, k_candidates, k_select, k_stereo_rows, k_stereo_match,
 *              k_stereo_filter, k_csr_hamming;
 * and work counts:
 *   counts8[0..5]: SearchByProjection (query, candidate) pairs scored, queries with a window,
 *                  ComputeStereoMatches (left, right) pairs scored, left keypoints searched,
 *                  SearchCandidates pairs, SearchCandidates queries;
 *   counts8[7]: ComputeStereoMatches left keypoints whose 11x11 SAD windows were read. */
int ORBmatcher_enable_timing(ORBmatcher_h h, int on);
int ORBmatcher_last_timings(ORBmatcher_h h, float* ms8, long long* counts8);
/* Deferred completion (no reference counterpart; the reference's calls are synchronous).
 * With deferred on (device-pointer matchers only), the device-resident batch calls
 * ORBmatcher_ComputeStereoMatches_batch, MapPoint_CreateStereo_batch_device,
 * ORBmatcher_SearchByProjection_LastFrame_batch, Tracking_PrepareLocalSearch_batch_device,
 * ORBmatcher_SearchLocalPoints_batch and Optimizer_PoseOptimization_frames_device_deferred
 * return as soon as their work is queued on ORBmatcher_stream(h); their per-problem counts
 * (nmatches, nvisible, ninliers) are written when ORBmatcher_finish(h) returns.  A chain of
 * TrackWithMotionModel + TrackLocalMap calls then runs without a host round trip between
 * the calls.  Turning deferred off finishes a pending chain. */
int ORBmatcher_set_deferred(ORBmatcher_h h, int on);
int ORBmatcher_finish(ORBmatcher_h h);
/* Overlapping chains: close the calls queued so far into an epoch (returns at once), queue the
 * next step's calls, and finish the older epoch later.  chain_wait blocks until an epoch's
 * device work is done (no counts written; callable from another host thread, e.g. before
 * reusing that epoch's input buffers); chain_finish(e) waits for every epoch <= e and writes
 * their counts. */
int ORBmatcher_chain_close(ORBmatcher_h h, long long* epoch);
int ORBmatcher_chain_wait(ORBmatcher_h h, long long epoch);
int ORBmatcher_chain_finish(ORBmatcher_h h, long long epoch);

/* static int ORBmatcher::DescriptorDistance(a, b)   ORBmatcher.cc:1647-1663 (host) */
int ORBmatcher_DescriptorDistance(const uint8_t* a, const uint8_t* b);

/* Frame view used for guided search (Frame.h fields the matcher reads).
 * Grid: Frame::mGrid (64 x 48, Frame.h:37-38) is rebuilt on device from
 * kpsUn (AssignFeaturesToGrid, Frame.cc:230-245). */
typedef struct orb_frame {
    int N;
    const orb_kp* keysUn;        /* mvKeysUn (N) */
    const uint8_t* desc;         /* mDescriptors (N x 32) */
    const float* uRight;         /* mvuRight (N) or NULL (monocular) */
    float minX, maxX, minY, maxY;/* mnMinX.. (Frame.cc:442-470) */
    float gridWInv, gridHInv;    /* mfGridElementWidthInv/HeightInv */
    const float* scaleFactors;   /* mvScaleFactors */
    int nlevels;
    float fx, fy, cx, cy, bf, b; /* intrinsics, mbf, mb */
    const float* Tcw;            /* 4x4 row-major float (mTcw) */
} orb_frame;

/* Map point table shared by the search calls (MapPoint fields read by the matcher). */
typedef struct orb_mappoints {
    int n;
    const float* pos;            /* GetWorldPos (n x 3) */
    const uint8_t* desc;         /* GetDescriptor (n x 32) */
    const int* observations;     /* Observations() (n) */
} orb_mappoints;

/* int SearchByProjection(Frame& CurrentFrame, const Frame& LastFrame, float th, bool bMono)
 *                                                          ORBmatcher.cc:1328-1470
 * last_mp[i]: map point index of LastFrame.mvpMapPoints[i] (-1 = NULL);
 * last_outlier[i]: LastFrame.mvbOutlier; last_keys: LastFrame.mvKeys (octave),
 * last_keysUn: LastFrame.mvKeysUn (angle).
 * cur_mp (in/out, N of current): CurrentFrame.mvpMapPoints as indices (-1 = NULL).
 * *nmatches = return value of the reference. */
int ORBmatcher_SearchByProjection_LastFrame(ORBmatcher_h h, const orb_frame* cur, int32_t* cur_mp,
                                            const orb_frame* last, const orb_kp* last_keys,
                                            const int32_t* last_mp, const uint8_t* last_outlier,
                                            const orb_mappoints* mps, float th, int bMono,
                                            int* nmatches);

/* Batched form of the above over `npairs` independent (cur, last) pairs in ONE launch. */
int ORBmatcher_SearchByProjection_LastFrame_batch(ORBmatcher_h h, int npairs, const orb_frame* cur,
                                                  int32_t* const* cur_mp, const orb_frame* last,
                                                  const orb_kp* const* last_keys,
                                                  const int32_t* const* last_mp,
                                                  const uint8_t* const* last_outlier,
                                                  const orb_mappoints* mps, float th, int bMono,
                                                  int* nmatches);

/* int SearchByProjection(Frame& F, const vector<MapPoint*>& vpMapPoints, float th)
 *                                                          ORBmatcher.cc:45-129
 * Per map point j (order = vpMapPoints order): track_in_view (mbTrackInView),
 * proj_x/proj_xr/proj_y (mTrackProjX/XR/Y), level (mnTrackScaleLevel),
 * view_cos (mTrackViewCos), mp_index (index into mps, written to cur_mp). */
int ORBmatcher_SearchByProjection_MapPoints(ORBmatcher_h h, const orb_frame* F, int32_t* cur_mp,
                                            int n, const uint8_t* track_in_view,
                                            const float* proj_x, const float* proj_xr,
                                            const float* proj_y, const int32_t* level,
                                            const float* view_cos, const int32_t* mp_index,
                                            const orb_mappoints* mps, float th, int* nmatches);

/* Tracking::mvpLocalMapPoints with the MapPoint fields isInFrustum and SearchByProjection read. */
typedef struct orb_localmap {
    int n;
    const float* pos;            /* GetWorldPos (n x 3) */
    const uint8_t* desc;         /* GetDescriptor (n x 32) */
    const int* observations;     /* Observations() (n) */
    const float* max_dist;       /* mfMaxDistance (n) */
    const float* min_dist;       /* mfMinDistance (n) */
    const float* normal;         /* GetNormal() (n x 3) */
    const uint8_t* skip;         /* mnLastFrameSeen == CurrentFrame.mnId, or isBad() (n) */
} orb_localmap;

/* bool Frame::isInFrustum(MapPoint* pMP, float viewingCosLimit)      Frame.cc:269-325
 * For every point of maps[p] not skipped: the visibility test against frame F[p] (Tcw, bounds,
 * intrinsics, mbf, nlevels) and the MapPoint tracking fields it fills: in_view (mbTrackInView),
 * proj_x / proj_xr / proj_y (mTrackProjX / XR / Y), level (mnTrackScaleLevel, PredictScale),
 * view_cos (mTrackViewCos); outputs of points not in view are left untouched except in_view = 0.
 * nvisible[p] = points in view.  Device pointers only; desc / observations of maps unused. */
int Frame_isInFrustum_batch(ORBmatcher_h h, int count, const orb_frame* F, const orb_localmap* maps,
                            float viewingCosLimit, float logScaleFactor, uint8_t* const* in_view,
                            float* const* proj_x, float* const* proj_xr, float* const* proj_y,
                            int32_t* const* level, float* const* view_cos, int* nvisible);

/* void Tracking::SearchLocalPoints()                          Tracking.cc:1143-1193
 * For every local map point not skipped: Frame::isInFrustum(pMP, 0.5) (Frame.cc:269-325,
 * MapPoint::PredictScale MapPoint.cc:402-417), then SearchByProjection(F, mvpLocalMapPoints,
 * th) with ratio `nnratio` (the reference constructs ORBmatcher matcher(0.8) for this search,
 * Tracking.cc:1184; ORBmatcher.cc:45-129): pass 0.8 to follow it on any matcher, or <= 0 to
 * use the matcher's own nnratio (so one deferred chain serves every search of a step).
 * cur_mp[p] (in/out, F[p].N): mCurrentFrame.mvpMapPoints as rows of maps[p] (-1 = NULL);
 * the caller clears the outliers of the first PoseOptimization and marks the matched and
 * discarded points in `skip` first (Tracking.cc:893-913, 1146-1161).  logScaleFactor =
 * Frame::mfLogScaleFactor.  nmatches[p] = SearchByProjection's return value, nvisible[p] =
 * nToMatch (points IncreaseVisible() counts).  Device pointers only (ORBmatcher_set_device_
 * pointers(h, 1)); one launch set for all `count` frames. */
int ORBmatcher_SearchLocalPoints_batch(ORBmatcher_h h, int count, const orb_frame* F, int32_t* const* cur_mp,
                                       const orb_localmap* maps, float logScaleFactor, float th,
                                       float nnratio, int* nmatches, int* nvisible);

/* void Frame::ComputeStereoMatches()                            Frame.cc:466-640
 * Rectified stereo matching of the left keypoints of image `index` (0 only for the single
 * form; image p of the batch form) of the last ORBextractor_extract[_batch] call of `left`
 * and `right`: mvImagePyramid (with border) is read from those extractors, the scale
 * tables from `left`.  keysL/descL: mvKeys/mDescriptors (NL), keysR/descR: mvKeysRight /
 * mDescriptorsRight (NR).  mbf, mb: Frame::mbf, mb.  Outputs mvuRight / mvDepth (NL
 * floats, -1 = no stereo) and *nmatches = the stereo matches kept after the median filter.
 * Pointer space per ORBmatcher_set_device_pointers.  NL <= 4096. */
int ORBmatcher_ComputeStereoMatches(ORBmatcher_h h, ORBextractor_h left, ORBextractor_h right, int index,
                                    int NL, const orb_kp* keysL, const uint8_t* descL, int NR,
                                    const orb_kp* keysR, const uint8_t* descR, float mbf, float mb,
                                    float* uRight, float* depth, int* nmatches);
/* `npairs` stereo pairs (images 0..npairs-1 of the last batch calls) in one launch. */
int ORBmatcher_ComputeStereoMatches_batch(ORBmatcher_h h, ORBextractor_h left, ORBextractor_h right,
                                          int npairs, const int* NL, const orb_kp* const* keysL,
                                          const uint8_t* const* descL, const int* NR,
                                          const orb_kp* const* keysR, const uint8_t* const* descR,
                                          float mbf, float mb, float* const* uRight,
                                          float* const* depth, int* nmatches);
/* The same with pair p = (image first_left + p of `left`'s last batch, image first_right + p of
 * `right`'s): both images of every pair may come from ONE extractor's batch call over
 * [lefts..., rights...] (left == right, first_right = npairs), i.e. Frame(imLeft, imRight)'s two
 * extractions (Frame.cc:78-81) as one batch launch set. */
int ORBmatcher_ComputeStereoMatches_batch_at(ORBmatcher_h h, ORBextractor_h left, int first_left,
                                             ORBextractor_h right, int first_right, int npairs,
                                             const int* NL, const orb_kp* const* keysL,
                                             const uint8_t* const* descL, const int* NR,
                                             const orb_kp* const* keysR, const uint8_t* const* descR,
                                             float mbf, float mb, float* const* uRight,
                                             float* const* depth, int* nmatches);

/* cv::Mat Frame::UnprojectStereo(const int& i)                   Frame.cc:666-680
 * x3D = mRwc * ((u-cx)*z*invfx, (v-cy)*z*invfy, z) + mOw for every keypoint with
 * mvDepth[i] = z > 0 (invfx = 1.0f/fx, Frame.cc:108); the callers are Tracking's
 * UpdateLastFrame / CreateNewKeyFrame / StereoInitialization (Tracking.cc:520-840).
 * Twc: 16 floats row-major, [mRwc | mOw] (the inverse pose).  Rows with z <= 0 are not
 * written; mp (optional) gets i for z > 0 and -1 otherwise (the frame's new map-point
 * slots).  Every pointer is device memory; runs asynchronously on the matcher's stream
 * (ORBmatcher_stream), so a following search on `h` sees the points. */
typedef struct orb_unproject {
    int N;
    const orb_kp* keysUn;        /* mvKeysUn (N) */
    const float* depth;          /* mvDepth (N) */
    const float* Twc;            /* 16 floats: [mRwc | mOw] */
    float fx, fy, cx, cy;
    float* x3D;                  /* out: N x 3 */
    int32_t* mp;                 /* out (may be NULL): i if depth > 0, else -1 */
} orb_unproject;
int Frame_UnprojectStereo_batch_device(ORBmatcher_h h, int count, const orb_unproject* U);

/* void Frame::UndistortKeyPoints()                               Frame.cc:404-430
 * mvKeysUn from mvKeys: when mDistCoef.at<float>(0) == 0 a copy; otherwise every keypoint's pt
 * through cv::undistortPoints(pts, pts, mK, mDistCoef, Mat(), mK) (OpenCV 3.2
 * cvUndistortPoints: double arithmetic, 5 fixed-point iterations; "parity unpinned" at that
 * OpenCV call site) and the rest of each KeyPoint copied.  K: mK row-major;
 * dist: mDistCoef (k1 k2 p1 p2 [k3] [k4 k5 k6]), ndist = 4, 5 or 8.  Pointer space per
 * ORBmatcher_set_device_pointers: device arrays are enqueued on ORBmatcher_stream (batch form)
 * and host arrays are copied and waited for. */
typedef struct orb_undistort {
    int N;
    const orb_kp* keys;          /* mvKeys (N) */
    orb_kp* keysUn;              /* out: mvKeysUn (N); may not alias keys */
    float K[9];                  /* mK */
    float dist[8];               /* mDistCoef, ndist used */
    int ndist;
} orb_undistort;
int Frame_UndistortKeyPoints(ORBmatcher_h h, const orb_undistort* U);
int Frame_UndistortKeyPoints_batch(ORBmatcher_h h, int count, const orb_undistort* U);
/* void Frame::ComputeImageBounds(const cv::Mat&)                    Frame.cc:436-464
 * plus the grid factors the Frame constructors derive from it (Frame.cc:155-156):
 * bounds[0..5] = mnMinX, mnMaxX, mnMinY, mnMaxY, mfGridElementWidthInv, mfGridElementHeightInv.
 * With distortion the four image corners go through the UndistortKeyPoints kernel. */
int Frame_ComputeImageBounds(ORBmatcher_h h, int cols, int rows, const float* K, const float* dist, int ndist,
                             float* bounds);

/* New MapPoints from a stereo frame (Tracking::StereoInitialization / CreateNewKeyFrame /
 * UpdateLastFrame, Tracking.cc:520-560, 1025-1080, 837-860): for every keypoint with depth > 0,
 * x3D = UnprojectStereo(i) as above and MapPoint::UpdateNormalAndDepth (MapPoint.cc:331-371)
 * with the frame as the only observation: normal = (x3D - mOw) / |x3D - mOw|, mfMaxDistance =
 * |x3D - mOw| * mvScaleFactors[octave], mfMinDistance = mfMaxDistance / mvScaleFactors[nlevels-1].
 * row[i] = row_base + i (the point's row in the caller's map table) for depth > 0, else -1.
 * Device pointers; enqueued on ORBmatcher_stream. */
typedef struct orb_newpoints {
    int N;
    const orb_kp* keysUn;        /* mvKeysUn (N) */
    const float* depth;          /* mvDepth (N) */
    const float* Twc;            /* 16 floats: [mRwc | mOw] */
    float fx, fy, cx, cy;
    const float* scaleFactors;   /* mvScaleFactors (nlevels) */
    int nlevels;
    int32_t row_base;
    float* x3D;                  /* out: N x 3 */
    int32_t* row;                /* out: N */
    float* normal;               /* out: N x 3 (GetNormal) */
    float* max_dist;             /* out: N (mfMaxDistance) */
    float* min_dist;             /* out: N (mfMinDistance) */
} orb_newpoints;
int MapPoint_CreateStereo_batch_device(ORBmatcher_h h, int count, const orb_newpoints* P);

/* Tracking's bookkeeping between TrackWithMotionModel and SearchLocalPoints: the outliers of
 * the first PoseOptimization are dropped from mvpMapPoints and their points marked seen
 * (Tracking.cc:893-913), the frame's points are skipped by SearchLocalPoints (1146-1161).
 * skip[j] (out, n) = (row[j] < 0: no map point / isBad) or j in cur_mp; then cur_mp[i] = -1
 * where outlier[i].  One launch for all frames; device pointers; synchronous. */
typedef struct orb_localprep {
    int N;
    int32_t* cur_mp;             /* in/out (N): mvpMapPoints as local-map rows */
    const uint8_t* outlier;      /* mvbOutlier (N) after PoseOptimization */
    int n;                       /* local-map rows */
    const int32_t* row;          /* n: < 0 = no map point */
    uint8_t* skip;               /* out: n */
} orb_localprep;
int Tracking_PrepareLocalSearch_batch_device(ORBmatcher_h h, int count, const orb_localprep* P);

/* ======================================================================
 * ORBVocabulary (reference include/ORBVocabulary.h: DBoW2::TemplatedVocabulary<
 * FORB::TDescriptor, FORB>, Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h)
 * ====================================================================== */
typedef struct ORBvocabulary_t* ORBvocabulary_h;
int ORBvocabulary_create(ORBvocabulary_h* out);
int ORBvocabulary_destroy(ORBvocabulary_h h);
/* bool loadFromTextFile(const std::string&)  TemplatedVocabulary.h:1338-1424 (host parse).
 * ORB_E_INVALID where the reference returns false (unreadable file, header out of range) or
 * a node names a parent not yet defined.  The trailing line after saveToTextFile's final endl
 * is the reference's undefined behaviour; DESIGN.md §5 states how it is realised. */
int ORBvocabulary_loadFromTextFile(ORBvocabulary_h h, const char* path);
/* m_k, m_L, m_scoring, m_weighting, size of m_nodes (root included), size of m_words */
int ORBvocabulary_info(ORBvocabulary_h h, int* k, int* L, int* scoring, int* weighting, int* n_nodes,
                       int* n_words);
/* One frame's DBoW2::BowVector (std::map<WordId, WordValue>: ascending words) and
 * DBoW2::FeatureVector (as orb_featvec CSR: fv_node ascending, fv_start[n_nodes + 1],
 * fv_feat in insertion order).  Host buffers of capacity `cap` >= N (fv_start: cap + 1). */
typedef struct orb_bow {
    int cap;
    uint32_t* word;
    double* value;
    int n_words;                 /* out */
    uint32_t* fv_node;
    int32_t* fv_start;
    int32_t* fv_feat;
    int n_nodes;                 /* out */
} orb_bow;
/* void transform(const vector<TDescriptor>& features, BowVector& v, FeatureVector& fv,
 *                int levelsup) const                       TemplatedVocabulary.h:1126-1197
 * = Frame::ComputeBoW / KeyFrame::ComputeBoW with levelsup 4 (Frame.cc:395-402).
 * desc: N x 32 descriptors (host).  N <= 4096 per frame (ORB_E_CAPACITY). */
int ORBvocabulary_transform(ORBvocabulary_h h, const uint8_t* desc, int N, int levelsup, orb_bow* out);
/* `count` frames in one launch (one tree walk per descriptor, one assembly per frame). */
int ORBvocabulary_transform_batch(ORBvocabulary_h h, int count, const uint8_t* const* desc, const int* N,
                                  int levelsup, orb_bow* out);
/* void transform(const TDescriptor& feature, WordId& id, WordValue& weight, NodeId* nid,
 *                int levelsup) const, for each of N descriptors  TemplatedVocabulary.h:1217-1256 */
int ORBvocabulary_transform_features(ORBvocabulary_h h, const uint8_t* desc, int N, int levelsup,
                                     uint32_t* word, double* weight, uint32_t* node);
/* double score(const BowVector& a, const BowVector& b) const  (L1Scoring::score,
 * ScoringObject.cpp:21-66) of one query BowVector against `count` candidates given as CSR
 * (candidate c: words/values [cstart[c], cstart[c+1])), as KeyFrameDatabase scores the
 * keyframes sharing words (KeyFrameDatabase.cc:133, 249).  L1_NORM vocabularies only. */
int ORBvocabulary_score(ORBvocabulary_h h, const uint32_t* qw, const double* qv, int nq, int count,
                        const int32_t* cstart, const uint32_t* cw, const double* cv, double* scores);

/* DBoW2::FeatureVector (std::map<NodeId, std::vector<unsigned>>) as CSR: strictly ascending
 * node ids, the feature indices of node a at feat[start[a] .. start[a+1]) in insertion order.
 * (Computed by the caller's vocabulary; ORBvoc.txt is not shipped with the reference.) */
typedef struct orb_featvec {
    int n_nodes;
    const uint32_t* node_id;
    const int32_t* start;
    const int32_t* feat;
} orb_featvec;

/* The searches below take host arrays only (ORBmatcher_set_device_pointers(h, 0)).  The
 * device enumerates every window / vocabulary-node candidate with its Hamming distance; the
 * order-dependent selection is replayed on the host, in the reference's order. */

/* int SearchByProjection(Frame& CurrentFrame, KeyFrame* pKF, const set<MapPoint*>& sAlreadyFound,
 *                        const float th, const int ORBdist)          ORBmatcher.cc:1472-1599
 * F: CurrentFrame (grid over keysUn, Tcw = mTcw); cur_mp in/out (mvpMapPoints as indices).
 * n = pKF->GetMapPointMatches().size(); kf_mp[i]: map point index or -1; skip[i] = isBad() ||
 * sAlreadyFound.count(pMP); kf_angle[i] = pKF->mvKeysUn[i].angle.  mp_max_dist / mp_min_dist:
 * MapPoint::mfMaxDistance / mfMinDistance; logScaleFactor = CurrentFrame.mfLogScaleFactor. */
int ORBmatcher_SearchByProjection_KeyFrame(ORBmatcher_h h, const orb_frame* F, int32_t* cur_mp, int n,
                                           const int32_t* kf_mp, const uint8_t* skip,
                                           const float* kf_angle, const orb_mappoints* mps,
                                           const float* mp_max_dist, const float* mp_min_dist,
                                           float logScaleFactor, float th, int ORBdist, int* nmatches);

/* int SearchForInitialization(Frame& F1, Frame& F2, vector<cv::Point2f>& vbPrevMatched,
 *                             vector<int>& vnMatches12, int windowSize)  ORBmatcher.cc:405-520
 * prev_matched: F1.N x 2 (in/out); matches12: F1.N (out). */
int ORBmatcher_SearchForInitialization(ORBmatcher_h h, const orb_frame* F1, const orb_frame* F2,
                                       float* prev_matched, int32_t* matches12, int windowSize,
                                       int* nmatches);

/* int SearchByBoW(KeyFrame* pKF, Frame& F, vector<MapPoint*>& vpMapPointMatches)  ORBmatcher.cc:159-288
 * kf_mp[i]: pKF->GetMapPointMatches()[i] index or -1, kf_mp_bad[i]: isBad(); kf_angle =
 * pKF->mvKeysUn angles, f_angle = F.mvKeys angles; matches[NF] (out): vpMapPointMatches. */
int ORBmatcher_SearchByBoW_Frame(ORBmatcher_h h, int nKF, const uint8_t* kf_desc, const float* kf_angle,
                                 const int32_t* kf_mp, const uint8_t* kf_mp_bad, const orb_featvec* fvKF,
                                 int NF, const uint8_t* f_desc, const float* f_angle,
                                 const orb_featvec* fvF, int32_t* matches, int* nmatches);

/* int SearchByBoW(KeyFrame* pKF1, KeyFrame* pKF2, vector<MapPoint*>& vpMatches12)  ORBmatcher.cc:522-655
 * matches12[n1] (out): the map point of KF2 matched to feature i of KF1, or -1. */
int ORBmatcher_SearchByBoW_KeyFrames(ORBmatcher_h h, int n1, const uint8_t* desc1, const float* angle1,
                                     const int32_t* mp1, const uint8_t* bad1, const orb_featvec* fv1,
                                     int n2, const uint8_t* desc2, const float* angle2,
                                     const int32_t* mp2, const uint8_t* bad2, const orb_featvec* fv2,
                                     int32_t* matches12, int* nmatches);

/* int SearchForTriangulation(KeyFrame* pKF1, KeyFrame* pKF2, cv::Mat F12,
 *                            vector<pair<size_t,size_t>>& vMatchedPairs, const bool bOnlyStereo)
 *                                                                    ORBmatcher.cc:657-823
 * KF1/KF2: keysUn, desc, uRight (mvuRight, NULL = all monocular), Tcw, intrinsics, scaleFactors;
 * has_mp[i] = GetMapPoint(i) != NULL; levelSigma2_2 = pKF2->mvLevelSigma2; F12 3x3 row-major.
 * pairs: cap x 2 (idx1, idx2) in idx1 order; *npairs = count (ORB_E_CAPACITY if > cap). */
int ORBmatcher_SearchForTriangulation(ORBmatcher_h h, const orb_frame* KF1, const uint8_t* has_mp1,
                                      const orb_featvec* fv1, const orb_frame* KF2,
                                      const uint8_t* has_mp2, const orb_featvec* fv2,
                                      const float* levelSigma2_2, const float* F12, int bOnlyStereo,
                                      int32_t* pairs, int cap, int* npairs);

/* ---- LocalMapping / LoopClosing projection searches -------------------------------------
 * Map points are the rows of `pts` (GetWorldPos, GetDescriptor) with their
 * orb_mappoint_geo (mfMaxDistance, mfMinDistance, GetNormal).  KeyFrame::GetFeaturesInArea
 * (KeyFrame.cc:569-608, no level filter) and KeyFrame::IsInImage (strict upper bounds)
 * semantics.  Host pointers only (ORB_E_INVALID in device-pointer mode). */
typedef struct orb_mappoint_geo {
    const float* max_dist;     /* MapPoint::mfMaxDistance (n) */
    const float* min_dist;     /* MapPoint::mfMinDistance (n) */
    const float* normal;       /* GetNormal() (n x 3) */
} orb_mappoint_geo;

/* int SearchByProjection(KeyFrame* pKF, cv::Mat Scw, const vector<MapPoint*>& vpPoints,
 *                        vector<MapPoint*>& vpMatched, int th)      ORBmatcher.cc:290-403
 * pts = vpPoints; skip[i] = isBad() || spAlreadyFound.count(pMP); matched (KF->N, in/out):
 * vpMatched as row indices of pts (-1 = NULL).  KF: keysUn, desc, grid bounds, intrinsics,
 * scaleFactors (Tcw unused: the pose is Scw, 4x4 row-major similarity). */
int ORBmatcher_SearchByProjection_Sim3(ORBmatcher_h h, const orb_frame* KF, const float* Scw,
                                       const orb_mappoints* pts, const orb_mappoint_geo* geo,
                                       const uint8_t* skip, float logScaleFactor, int th,
                                       int32_t* matched, int* nmatches);
/* int Fuse(KeyFrame* pKF, const vector<MapPoint*>& vpMapPoints, float th)   825-975
 * skip[i] = !pMP || isBad() || IsInKeyFrame(pKF).  best[i] (out) = keypoint of pKF the
 * reference fuses point i with (bestIdx, 951-971) or -1; *nfused = the return value.  The
 * caller applies 953-969 (Replace / AddObservation) in point order: the selection never
 * depends on those mutations (no occupancy test in Fuse), so the plan is exact. */
int ORBmatcher_Fuse(ORBmatcher_h h, const orb_frame* KF, const orb_mappoints* pts,
                    const orb_mappoint_geo* geo, const uint8_t* skip, float logScaleFactor, float th,
                    int32_t* best, int* nfused);
/* int Fuse(KeyFrame* pKF, cv::Mat Scw, const vector<MapPoint*>& vpPoints, float th,
 *          vector<MapPoint*>& vpReplacePoint)                         977-1100
 * skip[i] = isBad() || pKF->GetMapPoints().count(pMP); best / nfused as Fuse (the caller
 * fills vpReplacePoint[i] from pKF->GetMapPoint(best[i]) or adds the observation). */
int ORBmatcher_Fuse_Sim3(ORBmatcher_h h, const orb_frame* KF, const float* Scw, const orb_mappoints* pts,
                         const orb_mappoint_geo* geo, const uint8_t* skip, float logScaleFactor, float th,
                         int32_t* best, int* nfused);
/* int SearchBySim3(KeyFrame* pKF1, KeyFrame* pKF2, vector<MapPoint*>& vpMatches12,
 *                  const float& s12, const cv::Mat& R12, const cv::Mat& t12, float th)  1102-1326
 * mp1 (KF1->N) / mp2 (KF2->N): GetMapPointMatches() as rows of pts (-1 = NULL); bad[row] =
 * isBad().  matches12 (KF1->N, in/out): -1 = NULL, >= 0 = the KF2 keypoint of the matched
 * point (GetIndexInKeyFrame(pKF2)), -2 = matched to a point not observed in KF2; every new
 * agreement writes the KF2 keypoint (vpMatches12[i1] = vpMapPoints2[idx2]).  R12: 3x3, t12: 3.
 * KF1's intrinsics project into both keyframes, as in the reference. */
int ORBmatcher_SearchBySim3(ORBmatcher_h h, const orb_frame* KF1, const int32_t* mp1, const orb_frame* KF2,
                            const int32_t* mp2, const orb_mappoints* pts, const orb_mappoint_geo* geo,
                            const uint8_t* bad, float s12, const float* R12, const float* t12,
                            float logScaleFactor, float th, int32_t* matches12, int* nfound);

/* Hamming distances for CSR candidate lists (the inner loop of every Search*):
 * query q (descriptor qdesc[q]) against train rows cand[off[q] .. off[q+1]).
 * Writes dist[k] for every candidate k (dist may be NULL: best/second only) and best/second
 * per query (strict '<', earliest candidate wins ties, like the reference loops). */
/* Brute-force matching (SURVEY config 2 (ii): the dense descriptor tile; north star "Hamming
 * brute-force ... over LDS-resident descriptor blocks"): for `count` problems, every query
 * descriptor qdesc[p] (nq[p] x 32) against every train row tdesc[p] (nt[p] x 32); per query the
 * best train index (-1 if none), its distance and the second-best distance (256 if none), by
 * the reference loops' rule (ORBmatcher.cc: DescriptorDistance 1647-1663; best on a strictly
 * smaller distance, so the earliest index wins ties; an equal distance becomes the second).
 * Pointer space per ORBmatcher_set_device_pointers (device mode: enqueued, deferred-chain aware). */
int ORBmatcher_SearchDense_batch(ORBmatcher_h h, int count, const uint8_t* const* qdesc, const int* nq,
                                 const uint8_t* const* tdesc, const int* nt, int32_t* const* best_idx,
                                 int32_t* const* best_dist, int32_t* const* second_dist);
/* Measurement: the last SearchDense_batch's kernel time (ms, HIP events on ORBmatcher_stream,
 * timing on) and its (query, train) pair count. */
int ORBmatcher_last_dense_timing(ORBmatcher_h h, float* ms, long long* pairs);
int ORBmatcher_SearchCandidates(ORBmatcher_h h, const uint8_t* qdesc, int nq,
                                const uint8_t* tdesc, int nt, const int32_t* off,
                                const int32_t* cand, int32_t* dist, int32_t* best_idx,
                                int32_t* best_dist, int32_t* second_dist);

/* ======================================================================
 * RANSAC random stream  (DUtils::Random::RandomInt over glibc rand(),
 * Thirdparty/DBoW2/DUtils/Random.cpp:47-50)
 * The reference draws from the process-global rand() (never seeded on the
 * stereo path => seed 1).  The boundary takes the stream explicitly: an
 * orb_rng is the glibc TYPE_3 additive-feedback state, bit-identical to
 * rand() after srand(seed); the solvers advance it by exactly the draws the
 * reference's loops consume (early returns included).
 * ====================================================================== */
typedef struct orb_rng {
    int32_t tbl[31];
    int32_t f, r;
} orb_rng;
void orb_rng_seed(orb_rng* g, unsigned seed);   /* srand(seed) */
int orb_rng_rand(orb_rng* g);                    /* rand() */

/* ======================================================================
 * PnPsolver  (reference include/PnPsolver.h:59-196, src/PnPsolver.cc)
 * ====================================================================== */
typedef struct PnPsolver_t* PnPsolver_h;

/* PnPsolver(const Frame& F, const vector<MapPoint*>& vpMapPointMatches)  PnPsolver.cc:67-110
 * The adapter packs the N matched, non-bad map points: p3d (N x 3, GetWorldPos),
 * p2d (N x 2, F.mvKeysUn[i].pt), sigma2 (N, F.mvLevelSigma2[octave]),
 * kp_index (N, mvKeyPointIndices) into vpMapPointMatches of size n_matches.
 * SetRansacParameters() defaults are applied as in the reference ctor. */
int PnPsolver_create(int N, const float* p3d, const float* p2d, const float* sigma2,
                     const int32_t* kp_index, int n_matches, float fx, float fy, float cx,
                     float cy, PnPsolver_h* out);
int PnPsolver_destroy(PnPsolver_h h);
/* SetRansacParameters(probability, minInliers, maxIterations, minSet, epsilon, th2)  121-157 */
int PnPsolver_set_ransac(PnPsolver_h h, double probability, int minInliers, int maxIterations,
                         int minSet, float epsilon, float th2);
/* cv::Mat iterate(int nIterations, bool& bNoMore, vector<bool>& vbInliers, int& nInliers) 165-258
 * inliers: n_matches bytes (vbInliers); Tcw: 16 floats (row-major CV_32F 4x4);
 * *has_pose = 0 where the reference returns an empty cv::Mat. */
int PnPsolver_iterate(PnPsolver_h h, int nIterations, orb_rng* rng, int* bNoMore,
                      uint8_t* inliers, int* nInliers, float* Tcw, int* has_pose);
/* `count` independent solvers in one hypothesis launch; solver k draws from rngs[k]
 * (pass the same pointer for all to share one stream in solver order). Per-solver
 * outputs at inliers[k] / Tcw + 16k / bNoMore[k] / nInliers[k] / has_pose[k]. */
int PnPsolver_iterate_batch(int count, PnPsolver_h* hs, int nIterations, orb_rng** rngs,
                            int* bNoMore, uint8_t** inliers, int* nInliers, float* Tcw,
                            int* has_pose);
/* RANSAC bookkeeping (mnIterations, mRansacMaxIts, mRansacMinInliers) */
int PnPsolver_get_state(PnPsolver_h h, int* iterations, int* max_its, int* min_inliers);
/* Measurement (no reference counterpart): HIP-event timing of the calling thread's
 * hypothesis launches.  last_timings: ms2 = {EPnP solve, CheckInliers} of the last timed
 * iterate call, counts2 = {hypotheses, (hypothesis, correspondence) pairs}. */
int PnPsolver_enable_timing(int on);
int PnPsolver_last_timings(float* ms2, long long* counts2);

/* ======================================================================
 * Sim3Solver  (reference include/Sim3Solver.h:39-137, src/Sim3Solver.cc)
 * ====================================================================== */
typedef struct Sim3Solver_t* Sim3Solver_h;

/* Sim3Solver(pKF1, pKF2, vpMatched12, bFixScale)  Sim3Solver.cc:37-112
 * The adapter packs the N valid pairs in vpMatched12 order: X1c/X2c (N x 3,
 * Rcw*Xw+tcw of each keyframe = mvX3Dc1/2), sigma2_1/2 (N, mvLevelSigma2[octave]),
 * idx1 (N, mvnIndices1) into vpMatched12 of size N1; K1/K2 = {fx, fy, cx, cy}.
 * SetRansacParameters() defaults (0.99, 6, 300) are applied as in the reference
 * ctor. N must be >= 3 (the reference's loop-closing caller guarantees >= 20). */
int Sim3Solver_create(int N, const float* X1c, const float* X2c, const float* sigma2_1,
                      const float* sigma2_2, const int32_t* idx1, int N1, const float* K1,
                      const float* K2, int bFixScale, Sim3Solver_h* out);
int Sim3Solver_destroy(Sim3Solver_h h);
/* SetRansacParameters(probability, minInliers, maxIterations)  114-138 */
int Sim3Solver_set_ransac(Sim3Solver_h h, double probability, int minInliers, int maxIterations);
/* cv::Mat iterate(nIterations, bNoMore, vbInliers, nInliers)  140-207
 * inliers: N1 bytes; T12: 16 floats (row-major 4x4 sim3 [sR t; 0 1]);
 * *has_pose = 0 where the reference returns an empty cv::Mat. */
int Sim3Solver_iterate(Sim3Solver_h h, int nIterations, orb_rng* rng, int* bNoMore,
                       uint8_t* inliers, int* nInliers, float* T12, int* has_pose);
/* `count` independent solvers in one hypothesis launch (LoopClosing::ComputeSim3
 * runs one per loop candidate); same conventions as PnPsolver_iterate_batch. */
int Sim3Solver_iterate_batch(int count, Sim3Solver_h* hs, int nIterations, orb_rng** rngs,
                             int* bNoMore, uint8_t** inliers, int* nInliers, float* T12,
                             int* has_pose);
/* GetEstimatedRotation / GetEstimatedTranslation / GetEstimatedScale  366-379:
 * R (9, row-major), t (3), s of the best hypothesis so far. */
int Sim3Solver_get_estimate(Sim3Solver_h h, float* R, float* t, float* s);
/* (mnIterations, mRansacMaxIts, mRansacMinInliers) */
int Sim3Solver_get_state(Sim3Solver_h h, int* iterations, int* max_its, int* min_inliers);
/* Measurement, as PnPsolver_enable_timing / PnPsolver_last_timings: {ComputeSim3, CheckInliers}. */
int Sim3Solver_enable_timing(int on);
int Sim3Solver_last_timings(float* ms2, long long* counts2);

/* ======================================================================
 * Local bundle adjustment  (reference Optimizer::LocalBundleAdjustment,
 * src/Optimizer.cc:453-778; include/Optimizer.h:45)
 * The adapter gathers lLocalKeyFrames / lLocalMapPoints / lFixedCameras
 * (Optimizer.cc:456-504) and the observations in the order the reference
 * creates its g2o edges (map points in list order, then each point's
 * observation map order, 572-653), and applies the results (Converter
 * round trip, EraseMapPointMatch / EraseObservation, 711-777).
 * Requirements: unique kf_id / pt_id; at most one edge per (keyframe, point).
 * ====================================================================== */
typedef struct ba_problem {
    int n_kf;
    const int32_t* kf_id;      /* KeyFrame::mnId (g2o vertex id) */
    const float* kf_Tcw;       /* n_kf x 16 row-major CV_32F pose */
    const uint8_t* kf_local;   /* 1 = local keyframe (written back; fixed iff mnId == 0), 0 = fixed camera */
    const float* kf_cam;       /* n_kf x 5: fx fy cx cy mbf */
    int n_pt;
    const int32_t* pt_id;      /* MapPoint::mnId */
    const float* pt_pos;       /* n_pt x 3 GetWorldPos() */
    int n_edge;
    const int32_t* edge_pt;    /* index into the points */
    const int32_t* edge_kf;    /* index into the keyframes */
    const float* edge_obs;     /* n_edge x 3: kpUn.pt.x, kpUn.pt.y, mvuRight (< 0 = monocular edge) */
    const float* edge_inv_sigma2;  /* mvInvLevelSigma2[kpUn.octave] */
} ba_problem;

typedef struct ba_result {
    float* kf_Tcw;             /* n_kf x 16 (local keyframes updated, fixed cameras copied) */
    float* pt_pos;             /* n_pt x 3 */
    uint8_t* edge_erase;       /* n_edge: 1 = (pKFi, pMP) pushed to vToErase */
    int32_t iterations[2];     /* optimize(5) / optimize(10) return values */
    int32_t n_erased;
    int32_t aborted;           /* *pbStopFlag was set before optimising: nothing written back */
} ba_result;

/* static void Optimizer::LocalBundleAdjustment(KeyFrame*, bool* pbStopFlag, Map*)
 * stop may be NULL; it is read between LM iterations and trials like g2o's
 * force-stop flag. */
int Optimizer_LocalBundleAdjustment(const ba_problem* P, const volatile bool* stop, ba_result* R);
/* static void Optimizer::BundleAdjustment(vpKFs, vpMP, nIterations, pbStopFlag, nLoopKF, bRobust)
 *                                                          Optimizer.cc:49-237
 * (GlobalBundleAdjustemnt, Optimizer.cc:41-47, passes every keyframe and map point.)
 * Every keyframe is a vertex, fixed iff kf_id == 0 (kf_local is ignored); one
 * optimize(nIterations); Huber deltas sqrt(5.99)/sqrt(7.815) when bRobust; no outlier
 * gating.  R->kf_Tcw: every keyframe; R->pt_pos: points with >= 1 edge updated
 * (vbNotIncludedMP points copied); R->iterations[0] = optimize() iterations. */
int Optimizer_BundleAdjustment(const ba_problem* P, int nIterations, int bRobust, const volatile bool* stop,
                               ba_result* R);

/* ======================================================================
 * Sim3 refinement of a loop candidate  (reference Optimizer::OptimizeSim3,
 * src/Optimizer.cc:1046-1241; include/Optimizer.h:56-57; called from
 * LoopClosing::ComputeSim3, LoopClosing.cc:326)
 * One VertexSim3Expmap (numeric Jacobians of EdgeSim3ProjectXYZ and
 * EdgeInverseSim3ProjectXYZ), fixed point vertices, Huber sqrt(th2),
 * optimize(5), chi2 > th2 gating, optimize(10 | 5) on the inliers.
 * ====================================================================== */
typedef struct sim3opt_problem {
    int N;                       /* vpMatches1.size() (= pKF1->N) */
    const uint8_t* valid;        /* N: vpMatches1[i] && pMP1 && !pMP1->isBad() && !pMP2->isBad() && i2 >= 0 */
    const float* X1c;            /* N x 3: R1w*P3D1w + t1w (CV_32F, as Optimizer.cc:1118) */
    const float* X2c;            /* N x 3: R2w*P3D2w + t2w */
    const float* obs1;           /* N x 2: pKF1->mvKeysUn[i].pt */
    const float* obs2;           /* N x 2: pKF2->mvKeysUn[i2].pt */
    const float* inv_sigma2_1;   /* N: pKF1->mvInvLevelSigma2[kpUn1.octave] */
    const float* inv_sigma2_2;   /* N: pKF2->mvInvLevelSigma2[kpUn2.octave] */
    float K1[4], K2[4];          /* fx fy cx cy of pKF1->mK / pKF2->mK */
    float th2;                   /* chi2 threshold (LoopClosing passes 10) */
    int bFixScale;
} sim3opt_problem;

/* static int Optimizer::OptimizeSim3(pKF1, pKF2, vpMatches1, g2oS12, th2, bFixScale).
 * S12: g2o::Sim3 as 8 doubles (quaternion x y z w = Eigen coeffs(), t, s), in/out; left
 * unchanged on the reference's early return (fewer than 10 inliers after gating).
 * erased: N bytes out, 1 where the reference sets vpMatches1[i] = NULL.
 * *nIn = the return value.  At most 2048 valid correspondences (ORB_E_CAPACITY). */
int Optimizer_OptimizeSim3(const sim3opt_problem* P, double* S12, uint8_t* erased, int* nIn);
/* `count` candidates in one launch (one workgroup each): S12 count x 8, erased[c] N_c bytes. */
int Optimizer_OptimizeSim3_batch(int count, const sim3opt_problem* P, double* S12, uint8_t* const* erased,
                                 int* nIn);

/* ======================================================================
 * Motion-only pose optimisation  (reference Optimizer::PoseOptimization,
 * src/Optimizer.cc:239-451; include/Optimizer.h:48)
 * One SE3 vertex, one unary edge per keypoint with a map point
 * (EdgeSE3ProjectXYZOnlyPose if mvuRight[i] < 0, else the stereo edge),
 * Huber sqrt(5.991) / sqrt(7.815), 4 rounds of optimize(10) each restarted
 * from mTcw, chi2 outlier classification after every round, robust kernel
 * dropped after round 3, early exit when fewer than 10 edges.
 * ====================================================================== */
typedef struct pose_problem {
    int N;                     /* keypoints (pFrame->N) */
    const float* Tcw;          /* 16 row-major pFrame->mTcw */
    const uint8_t* has_mp;     /* N: mvpMapPoints[i] != NULL */
    const float* Xw;           /* N x 3: pMP->GetWorldPos() (rows with has_mp) */
    const float* obs;          /* N x 3: mvKeysUn[i].pt.x, .y, mvuRight[i] */
    const float* inv_sigma2;   /* N: mvInvLevelSigma2[mvKeysUn[i].octave] */
    float fx, fy, cx, cy, bf;  /* pFrame->fx ... mbf */
} pose_problem;

/* static int Optimizer::PoseOptimization(Frame* pFrame).
 * Tcw_out: 16 floats (pFrame->SetPose(toCvMat(SE3quat_recov))); unchanged copy of
 * Tcw when fewer than 3 correspondences.  outlier: N bytes, in/out like
 * pFrame->mvbOutlier -- rows with has_mp are written, the others left as they are.
 * *ninliers = the return value (nInitialCorrespondences - nBad).  At most 8192 map
 * points per frame (ORB_E_CAPACITY). */
int Optimizer_PoseOptimization(const pose_problem* P, float* Tcw_out, uint8_t* outlier, int* ninliers);
/* `count` frames in one launch (one workgroup per frame): Tcw_out count x 16,
 * outlier[f] N_f bytes, ninliers[count]. */
int Optimizer_PoseOptimization_batch(int count, const pose_problem* P, float* Tcw_out, uint8_t* const* outlier,
                                     int* ninliers);

/* Device-resident variant: every array of P[f], Tcw_out[f] (16 floats) and outlier[f]
 * are HIP device pointers (e.g. the matcher's device-mode outputs gathered in HBM);
 * the edges are built on the device.  Synchronous; ninliers is host memory.
 * ORB_E_CAPACITY if a frame has more than 8192 map points (its outputs are not written). */
int Optimizer_PoseOptimization_batch_device(int count, const pose_problem* P, float* const* Tcw_out,
                                            uint8_t* const* outlier, int* ninliers);

/* The frame as PoseOptimization(Frame*) reads it (Optimizer.cc:255-347), every array in
 * device memory: mvpMapPoints as indices into a map-point table (mp[i] = -1: NULL),
 * pMP->GetWorldPos() = mp_pos[3*mp[i]..], mvKeysUn, mvuRight (< 0: monocular edge) and
 * the mvInvLevelSigma2 table indexed by kpUn.octave.  The edges are gathered on the
 * device, so no per-frame host or framework-side packing is needed. */
typedef struct pose_frame {
    int N;
    const float* Tcw;            /* 16 row-major pFrame->mTcw */
    const int32_t* mp;           /* N */
    const float* mp_pos;         /* map point rows, 3 floats each */
    const orb_kp* keysUn;        /* N */
    const float* uRight;         /* N */
    const float* invLevelSigma2; /* nlevels */
    int nlevels;
    float fx, fy, cx, cy, bf;
} pose_frame;
/* Measurement: enable >= 0 switches k_pose_opt timing (HIP events around the launch on the calling
 * thread's pose engine) on or off; last_ms (optional) receives the duration of the last timed
 * launch (waits for it).  ORB_E_INVALID when nothing was timed yet.  No reference counterpart. */
int Optimizer_pose_timing(int enable, float* last_ms);

/* Same outputs and capacity rule as Optimizer_PoseOptimization_batch_device. */
int Optimizer_PoseOptimization_frames_device(int count, const pose_frame* F, float* const* Tcw_out,
                                             uint8_t* const* outlier, int* ninliers);
/* The same, queued on the deferred chain of matcher `chain` (ORBmatcher_set_deferred): behind
 * the chain's earlier calls on ORBmatcher_stream(chain); ninliers[f] is written at
 * ORBmatcher_finish(chain), -1 for a frame over the edge capacity. */
int Optimizer_PoseOptimization_frames_device_deferred(ORBmatcher_h chain, int count, const pose_frame* F,
                                                      float* const* Tcw_out, uint8_t* const* outlier,
                                                      int* ninliers);

/* ----------------------------------------------------------------------
 * Keyframe-block sharded BA across GPUs: one process (or
 * thread) per rank, map points partitioned by the block of their reference
 * keyframe, poses replicated.  Per LM trial the ranks all-reduce the partial
 * Schur complement {S, b_s} and the scalars {chi2, scale, stop}; every rank
 * solves the identical reduced system -- or, with the separator-tree partition
 * (Optimizer_partition_points_nd) of a block-sparse system, each rank factors
 * its own subtrees and only the separators' tiles and rows are exchanged.  Pass each rank the SAME keyframes and
 * its own points + all of their edges (edge order preserved); the results are
 * the rank's points / edges and the (identical) poses.
 * ---------------------------------------------------------------------- */
typedef struct orbgpu_comm_t* orbgpu_comm_h;
/* RCCL over xGMI: rank 0 calls orbgpu_comm_unique_id, the caller distributes the
 * 128 bytes (e.g. MPI / torch.distributed), every rank calls init_rccl with the
 * HIP device it runs on already current.  ORB_E_NODEVICE if librccl is absent. */
int orbgpu_comm_unique_id(uint8_t* id128);
int orbgpu_comm_init_rccl(int nranks, int rank, const uint8_t* id128, orbgpu_comm_h* out);
/* `nranks` in-process ranks (one host thread each, one device): out[0..nranks). */
int orbgpu_comm_init_local(int nranks, orbgpu_comm_h* out);
/* One process per rank on one host (e.g. several ranks sharing one GPU, where RCCL cannot place
 * them): every rank calls this with the same fresh POSIX shm name ("/..."), nranks and
 * max_doubles (the largest exchange, in doubles); rank 0 creates the segment, the others attach
 * (bounded wait, ORBGPU_SHM_TIMEOUT s, default 300), and the name is unlinked once all attached.
 * Partials go through host memory and are summed in rank order on every rank (the in-process
 * group's order).  ORB_E_CAPACITY if an exchange exceeds max_doubles. */
int orbgpu_comm_init_shm(const char* name, int nranks, int rank, size_t max_doubles, orbgpu_comm_h* out);
int orbgpu_comm_rank(orbgpu_comm_h h, int* rank, int* size);
int orbgpu_comm_destroy(orbgpu_comm_h h);
/* Keyframe-block partition: pt_rank[p] = rank owning point p.  Reference keyframe
 * of a point = keyframe of its first edge; keyframes in mnId order are cut into
 * nranks contiguous blocks of ~equal edge weight.  Host only (no device needed). */
int Optimizer_partition_points(const ba_problem* P, int nranks, int32_t* pt_rank);
/* Separator-tree partition for the sharded factorisation of a global BA (BundleAdjustment):
 * the nested dissection of the pose graph the engine derives (ordering.hpp), whole subtrees
 * to ranks (nd_assign), each point to the rank of the first subtree pose it observes (a point
 * of separator poses only: round robin).  With it every rank's Schur terms stay inside its own
 * subtrees and the separators, so the ranks factor their subtrees alone and exchange only the
 * separator tiles and rows (Optimizer_BundleAdjustment_sharded checks this and otherwise keeps
 * the replicated factorisation).  Fewer than 24 free poses or one rank: the keyframe-block
 * partition.  kf_owner (optional, n_kf entries): the rank whose subtree holds keyframe k's
 * pose, -1 for a separator pose, -2 for a keyframe that is no free pose; with the
 * keyframe-block fallback, a free pose's owner is its keyframe's block.  Host only. */
int Optimizer_partition_points_nd(const ba_problem* P, int nranks, int32_t* pt_rank, int32_t* kf_owner);
/* The calling thread's last BA run: [sharded factorisation used (0/1), separator tiles and
 * separator rows exchanged per LM trial, Schur-pattern tiles (what the replicated path
 * all-reduces)]. */
int Optimizer_last_sharding(int* info4);
/* The calling thread's last BA run's LM control: info4[0] = steps the device-resident LM queued
 * (k_lm_trial_end decides each trial on the device; a sharded run exchanges between the step's
 * kernels), info4[1] = trials the host loop decided after reading a trial's result back,
 * info4[2] = 1 if the run was sharded over more than one rank, info4[3] = 0. */
int Optimizer_last_lm_path(int* info4);
int Optimizer_LocalBundleAdjustment_sharded(const ba_problem* shard, orbgpu_comm_h comm,
                                            const volatile bool* stop, ba_result* R);
int Optimizer_BundleAdjustment_sharded(const ba_problem* shard, orbgpu_comm_h comm, int nIterations,
                                       int bRobust, const volatile bool* stop, ba_result* R);

/* LM trace of the calling thread's last run (for diagnostics / parity tests):
 * per solve() the initial and final robust chi2, per trial the chi2 and lambda. */
int Optimizer_last_trace(double* solve_ini_chi2, double* solve_chi2, int solve_cap, int* n_solves,
                         double* trial_chi2, double* trial_lambda, int trial_cap, int* n_trials);
/* host milliseconds of the calling thread's last run: [total, structure build] */
int Optimizer_last_timings(double* ms2);

/* Unit entry points of the BA building blocks (parity tests): the dense LDL^T
 * solve of the reduced pose system (variant 0 = register-resident panel kernel,
 * n <= 127; 1 = generic kernel; 2 / 3 = block-sparse tiled, natural / nested-dissection order;
 * 4 = row-owner kernel, n <= 96; 5 / 6 / 7 = column-owner / row-lane / 2-D block-cyclic kernel,
 * n <= 96) and
 * the canonical FP64 sum. */
int orbgpu_unit_ldlt_solve(int n, const double* S, const double* b, double* x, int variant, int* ok);
int orbgpu_unit_csum(const double* v, int n, double* out);
/* tiled LDL^T factorisation only (n x n row-major, upper triangle read): out = d on the
 * diagonal, L in the strict lower triangle, eliminated rows in the strict upper. */
/* PnPsolver batch work-area layout invariant (host only, no device): for n solvers with
 * N[k] correspondences, K[k] hypotheses and minSet[k], out4 = {device bytes allocated, device
 * end touched, host bytes allocated, host end touched}; ORB_OK iff everything touched fits. */
int orbgpu_unit_pnp_layout(int n, const int* N, const int* K, const int* minSet, long long* out4);
int orbgpu_unit_ldlt_factor(int n, const double* S, double* out);
/* Host only (no device): the BA structure of one optimisation level (csrc/ba_struct.cpp,
 * initializeOptimization + buildIndexMapping + BlockSolver::buildStructure) packed into out:
 * [nE nP nL nBlk nPair | poseKf[nP] | landPt[nL] | ePose[nE] | eLand[nE] | lpStart[nL+1] |
 *  lpList | blkI[nBlk] | blkJ[nBlk] | blkStart[nBlk+1] | pairA[nPair] | pairB[nPair]];
 * ORB_E_CAPACITY when cap (int32 entries) is too small, ORB_E_INVALID on a duplicate
 * (pose, landmark) edge. */
int orbgpu_unit_ba_struct(int nkf, int npt, int ne, const int32_t* edge_kf, const int32_t* edge_pt,
                          const uint8_t* edge_level, const uint8_t* kf_fixed, const int32_t* kf_id,
                          const int32_t* pt_id, int level, int32_t* out, long long cap);
/* The same structure from the builders: gpu = 1 the multi-launch device builder (ba_struct_gpu.hip),
 * gpu = 2 the one-workgroup device builder local-BA sizes run (the multi-launch one outside its
 * limits), gpu = 0 the host restatement.  out = [nE nP nL nBlk nPair nPe nLe nLp |
 * aE | ePose | eLand | poseKf | landPt | peStart | peList | leStart | leList | lpStart | lpList |
 * blkI | blkJ | blkStart | pairA | pairB]; *n_out = its length (ORB_E_CAPACITY beyond cap). */
int orbgpu_unit_ba_struct_all(int nkf, int npt, int ne, const int32_t* edge_kf, const int32_t* edge_pt,
                              const uint8_t* edge_level, const uint8_t* kf_fixed, const int32_t* kf_id,
                              const int32_t* pt_id, int level, int gpu, int32_t* out, long long cap,
                              long long* n_out);
/* one wave's canonical 64-tree of v64[0..64) (cross-lane permlane/DPP path) */
int orbgpu_unit_wave_tree(const double* v64, double* out);
/* The BA kernels' shared-denominator division (SharedDiv, ba_math.hpp) against the plain FP64
 * division on n pairs: out[2i] = SharedDiv(b[i]).div(a[i]), out[2i + 1] = a[i] / b[i]. */
int orbgpu_unit_shared_div(const double* a, const double* b, int n, double* out);
/* Test knob: the BA chi2 canonical sum keeps at most m2_max level-2 trees in LDS (default and
 * maximum 1024, i.e. 4.2 M edges) and writes larger sets to its chunk buffer's tail; 0 sends
 * every problem down the tail path.  Process-wide, device-side. */
int orbgpu_unit_set_csum_lds_max(int m2_max);
/* Test knob: computeScale runs in the LM trial's single workgroup for 6 nP + 3 nL <= terms
 * (default and maximum 2048 * 64) and as a chunked two-kernel sum above it; 0 sends every
 * problem down the chunked path.  Process-wide, host-side. */
int orbgpu_unit_set_scale_small_max(int terms);
/* Test knob: BA runs with at least `edges` edges build their structure lists on the device
 * (ba_struct_gpu.hip), smaller ones on the host (default 100000; 0 sends every run to the
 * device builder).  ORBGPU_STRUCT_HOST=1 / 0 in the environment overrides it.  Process-wide. */
int orbgpu_unit_set_struct_gpu_min_edges(int edges);
/* Test knob: an unsharded global BA derives its first pose graph from the caller's edges on the
 * host, beside the device's structure lists; on = 1 also fetches the device's off-diagonal Schur
 * blocks and fails the call (ORB_E_HIP) if the two graphs differ.  Process-wide. */
int orbgpu_unit_set_posegraph_check(int on);
/* The elimination order of the block-sparse pose system (host only, no device): nested
 * dissection of a graph (adjStart[n + 1] / adj: symmetric, sorted lists) with leaves of at
 * most `leaf` nodes; perm[k] = node eliminated k-th; the separator tree's node count and
 * height (0 = a single leaf). */
int orbgpu_unit_nd_order(int n, const int32_t* adjStart, const int32_t* adj, int leaf, int32_t* perm,
                         int32_t* n_nodes, int32_t* height);
/* Instrumented builds only (make prof): read and clear the BA/pose section timers (32 x u64
 * clock64 deltas of workgroup 0); ORB_E_INVALID in normal builds. */
int orbgpu_debug_prof(unsigned long long* out32);
/* Section timers of the matcher's greedy replay kernel (instrumented builds only). */
int orbgpu_debug_prof_match(unsigned long long* out32);
/* Section timers of the FAST cell kernel (instrumented builds only). */
int orbgpu_debug_prof_extract(unsigned long long* out32);

#ifdef __cplusplus
}
#endif
#endif
