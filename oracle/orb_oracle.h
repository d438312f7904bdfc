/*
 * orb_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement (plain C11, built with -ffp-contract=off) of the reference
 * junejunejune/c_orb_slam per-frame hot path.  It is the parity CHECKER for the
 * HIP product in c_orb_slam_amd/: only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load it.  The product never links it.
 *
 * Parity status (see DESIGN.md "Oracle"): the reference cannot be compiled in
 * this image (needs OpenCV/Eigen, absent) and ships no tests or golden
 * vectors, so the OpenCV call sites are restated from OpenCV 3.2's scalar
 * code paths ("parity unpinned" at that boundary).  What IS pinned:
 *   - glibc sinf/cosf restatement: exhaustively equal to the host libm over
 *     every float in [0, 2*pi] (tests/test_oracle_kat.py);
 *   - glibc rand() (TYPE_3 additive feedback) against the host libc;
 *   - the BRIEF pattern table parsed from the reference source.
 * Every function cites the reference file:line it follows.
 */
#ifndef ORB_ORACLE_H
#define ORB_ORACLE_H
#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* cv::KeyPoint layout (28 bytes): pt.x, pt.y, size, angle, response, octave, class_id */
typedef struct {
    float x, y, size, angle, response;
    int32_t octave, class_id;
} ora_kp;

/* ---- OpenCV-semantic primitives (ocv_semantics.c) ---------------------- */
int   ora_cvRound_f(float v);
int   ora_cvRound_d(double v);
float ora_fastAtan2(float y, float x);
float ora_sinf(float x);           /* glibc 2.35 sinf restatement, |x| < 120 */
float ora_cosf(float x);           /* glibc 2.35 cosf restatement, |x| < 120 */
/* FAST-9/16 score S = max(A,B)-1 (A,B = best dark/bright 9-arc contrast). */
int   ora_fast_score(const uint8_t* p, int step);
/* cv::FAST(roi, kps, th, nonmax=true) on a ROI view; returns count (raster order). */
int   ora_fast_roi(const uint8_t* roi, int step, int cols, int rows, int th,
                   int* xs, int* ys, int* scores, int cap);
/* resize(INTER_LINEAR, 8U fixed point) dst (dw x dh) from src (sw x sh) */
void  ora_resize_linear_u8(const uint8_t* src, int sstep, int sw, int sh,
                           uint8_t* dst, int dstep, int dw, int dh);
/* GaussianBlur 7x7 sigma 2, 8U fixed-point separable, REFLECT_101, into contiguous dst */
void  ora_gaussian7_u8(const uint8_t* src, int sstep, int w, int h, uint8_t* dst, int dstep);
void  ora_gaussian7_taps(int taps[7]);

/* ---- ORBextractor (orb_extract.c) ---------------------------------------- */
typedef struct ora_extractor ora_extractor;
ora_extractor* ora_extractor_new(int nfeatures, float scaleFactor, int nlevels,
                                 int iniThFAST, int minThFAST);
void  ora_extractor_free(ora_extractor* e);
/* operator()(image) -> keypoints+descriptors. Returns number of keypoints, or
 * -(needed) if cap is too small (nothing written then). */
int   ora_extract(ora_extractor* e, const uint8_t* img, int w, int h, int step,
                  ora_kp* kps, uint8_t* desc, int cap);
/* Padded pyramid level (after the last ora_extract): returns pointer to the
 * top-left of the 19-px bordered image, its padded dims and step. */
int   ora_extractor_level(const ora_extractor* e, int level, const uint8_t** data,
                          int* pw, int* ph, int* step);
int   ora_extractor_nlevels(const ora_extractor* e);
void  ora_extractor_tables(const ora_extractor* e, float* scale, float* invScale,
                           float* sigma2, float* invSigma2, int* nPerLevel, int* umax16);
/* Debug taps for stage tests: candidates (pre-octree) per level, in reference order */
int   ora_extractor_candidates(const ora_extractor* e, int level, ora_kp* out, int cap);
/* Blurred level (contiguous w x h), valid after ora_extract */
int   ora_extractor_blurred(const ora_extractor* e, int level, const uint8_t** data, int* w, int* h);

/* ---- ORBmatcher (orb_match.c) -------------------------------------------- */
int   ora_descriptor_distance(const uint8_t* a, const uint8_t* b);

/* Frame-side data for guided matching (Frame.h:37-38, Frame.cc:230-392) */
#define ORA_GRID_COLS 64
#define ORA_GRID_ROWS 48
typedef struct {
    int N;
    const ora_kp* kpsUn;       /* undistorted keypoints (mvKeysUn) */
    const uint8_t* desc;       /* N x 32 */
    const float* uRight;       /* mvuRight (N), <0 = none; may be NULL */
    float minX, maxX, minY, maxY;
    float gridWInv, gridHInv;
    const float* scaleFactors; /* per level */
    int nlevels;
    /* grid (built by ora_frame_build_grid): CSR over 64*48 cells, cell = ix*48+iy */
    int* cellStart;            /* 64*48+1 */
    int* cellIdx;              /* N */
} ora_frame;
void  ora_frame_build_grid(ora_frame* f);
/* Frame::GetFeaturesInArea -> writes indices, returns count */
int   ora_frame_features_in_area(const ora_frame* f, float x, float y, float r,
                                 int minLevel, int maxLevel, int* out, int cap);

/* SearchByProjection(Frame& Cur, const Frame& Last, th, bMono), ORBmatcher.cc:1328-1470.
 * Last-frame map points: per last keypoint i, lastMP[i] = map point id or -1,
 * lastOutlier[i], mpPos[id*3] world position, mpDesc[id*32] descriptor.
 * Current frame occupancy: curMP[i2] (in/out) map point id or -1;
 * mpObs[id] = observations of that map point.  Poses: Tcw row-major 4x4 float. */
typedef struct {
    const float* Tcw_cur;    /* 16 */
    const float* Tcw_last;   /* 16 */
    float fx, fy, cx, cy, mbf, mb;
    const ora_kp* lastKeys;  /* mvKeys of last (octave) */
    const ora_kp* lastKeysUn;/* mvKeysUn of last (angle) */
    const int* lastMP;
    const uint8_t* lastOutlier;
    int lastN;
    const float* mpPos;
    const uint8_t* mpDesc;
    const int* mpObs;
} ora_lastframe;
int   ora_search_by_projection_last(const ora_frame* cur, int* curMP,
                                    const ora_lastframe* last, float th, int bMono,
                                    float nnratio, int checkOri);

/* SearchByProjection(Frame& F, const vector<MapPoint*>&, th), ORBmatcher.cc:45-129.
 * Per map point: trackInView, projX, projXR, projY, predictedLevel, viewCos, desc. */
typedef struct {
    int n;
    const uint8_t* inView;
    const float* projX;
    const float* projXR;
    const float* projY;
    const int* level;
    const float* viewCos;
    const uint8_t* desc;   /* n x 32 */
    const int* mpId;       /* id written into curMP */
} ora_localmaps;
int   ora_search_by_projection_local(const ora_frame* f, int* curMP, const int* mpObs,
                                     const ora_localmaps* m, float th, float nnratio);

void  ora_compute_three_maxima(const int* histSizes, int L, int* ind1, int* ind2, int* ind3);

/* ---- glibc rand() restatement (rng.c) ------------------------------------- */
typedef struct { int32_t tbl[31]; int f, r; } ora_rng;
void  ora_rng_seed(ora_rng* g, unsigned int seed);
int   ora_rng_rand(ora_rng* g);
int   ora_rng_random_int(ora_rng* g, int min, int max);  /* DUtils::Random::RandomInt */

/* RANSAC event log (test instrumentation): the events of the last iterate() call as
 * (hypothesis index within the call, kind) pairs; returns the number of events */
#define ORA_EV_CAP 512
static inline void ora_ev_push(int (*ev)[2], int* n, int h, int kind)
{
    if (*n < ORA_EV_CAP) { ev[*n][0] = h; ev[*n][1] = kind; }
    (*n)++;
}

/* ---- OpenCV C-API linear algebra restated (linalg.c) --------------------- */
void  ora_svd(const double* A, int m, int n, double* w, double* Ut, double* Vt);
void  ora_svd_solve(const double* A, int m, int n, const double* b, double* x);
void  ora_svd_invert(const double* A, int n, double* X);
void  ora_mul_transposed_ata(const double* src, int rows, int cols, double* dst);

/* ---- PnPsolver (pnp.c), reference src/PnPsolver.cc ------------------------ */
typedef struct ora_pnp ora_pnp;
double ora_epnp_compute_pose(const double* pws, const double* us, int n, double fu, double fv, double uc,
                             double vc, double R[3][3], double t[3]);
ora_pnp* ora_pnp_new(int N, const float* p3d, const float* p2d, const float* sigma2, const int* kpIdx,
                     int nMatches, float fx, float fy, float cx, float cy);
void  ora_pnp_free(ora_pnp* P);
void  ora_pnp_set_ransac(ora_pnp* P, double probability, int minInliers, int maxIterations, int minSet,
                         float epsilon, float th2);
int   ora_pnp_iterate(ora_pnp* P, int nIterations, ora_rng* rng, int* bNoMore, uint8_t* inliers_out,
                      int* nInliers, float* Tcw);
int   ora_pnp_iterations(const ora_pnp* P);
int   ora_pnp_max_its(const ora_pnp* P);
int   ora_pnp_min_inliers(const ora_pnp* P);
int   ora_pnp_events(const ora_pnp* P, int* out, int cap);   /* kinds: 1 best, 2 Refine failed, 3 Refine ok */


/* ---- Sim3Solver (sim3.c), reference src/Sim3Solver.cc --------------------- */
typedef struct ora_sim3 ora_sim3;
void  ora_det_sincos(double x, double* s, double* c);
double ora_det_atan2(double y, double x);
void  ora_jacobi_eigen_f(float* A, int n, float* W, float* V);
ora_sim3* ora_sim3_new(int N, const float* X1c, const float* X2c, const float* sigma2_1, const float* sigma2_2,
                       const int* idx1, int N1, const float* K1, const float* K2, int bFixScale);
void  ora_sim3_free(ora_sim3* S);
void  ora_sim3_set_ransac(ora_sim3* S, double probability, int minInliers, int maxIterations);
int   ora_sim3_iterate(ora_sim3* S, int nIterations, ora_rng* rng, int* bNoMore, uint8_t* inliers, int* nInliers,
                       float* T12);
void  ora_sim3_estimate(const ora_sim3* S, float* R, float* t, float* s);
int   ora_sim3_iterations(const ora_sim3* S);
int   ora_sim3_events(const ora_sim3* S, int* out, int cap);  /* kinds: 1 best update, 3 returned */


/* ---- remaining ORBmatcher searches (matchers2.c) ------------------------------
 * DBoW2::FeatureVector as CSR: ascending node ids, the feature indices of each node. */
typedef struct {
    int n_nodes;
    const uint32_t* node_id;
    const int32_t* start;      /* n_nodes + 1 */
    const int32_t* feat;
} ora_featvec;
/* SearchByProjection(Frame&, KeyFrame*, sAlreadyFound, th, ORBdist), ORBmatcher.cc:1472-1599.
 * F grid over mvKeysUn (ora_frame_build_grid); Tcw = CurrentFrame.mTcw; K = {fx,fy,cx,cy}; curMP in/out.
 * KF map points i < n: kfMP[i] (-1 = NULL), skip[i] (isBad || in sAlreadyFound), kfAngle[i].
 * mpMaxDist/mpMinDist: mfMaxDistance / mfMinDistance per map point. */
int   ora_search_by_projection_kf(const ora_frame* F, const float* Tcw, const float* K, int* curMP, int n, const int* kfMP,
                                  const uint8_t* skip, const float* kfAngle, const float* mpPos,
                                  const uint8_t* mpDesc, const float* mpMaxDist, const float* mpMinDist,
                                  float logScaleFactor, float th, int ORBdist, int checkOri);
/* SearchByBoW(KeyFrame*, Frame&, vpMapPointMatches), ORBmatcher.cc:159-288: matchesF[i] = map point or -1 */
int   ora_search_by_bow_frame(const ora_featvec* fvKF, const int* kfMP, const uint8_t* kfMPbad,
                              const uint8_t* kfDesc, const float* kfAngle, int nKF, const ora_featvec* fvF,
                              const uint8_t* fDesc, const float* fAngle, int NF, float nnratio, int checkOri,
                              int* matchesF);
/* SearchByBoW(KeyFrame*, KeyFrame*, vpMatches12), ORBmatcher.cc:522-655: matches12[i] = map point or -1 */
int   ora_search_by_bow_kf(const ora_featvec* fv1, const int* mp1, const uint8_t* bad1, const uint8_t* desc1,
                           const float* ang1, int n1, const ora_featvec* fv2, const int* mp2, const uint8_t* bad2,
                           const uint8_t* desc2, const float* ang2, int n2, float nnratio, int checkOri,
                           int* matches12);
/* SearchForInitialization(F1, F2, vbPrevMatched, vnMatches12, windowSize), ORBmatcher.cc:405-520 */
int   ora_search_for_initialization(const ora_frame* F1, const ora_frame* F2, float* prevMatched, int* matches12,
                                    int windowSize, float nnratio, int checkOri);
/* SearchForTriangulation(KF1, KF2, F12, vMatchedPairs, bOnlyStereo), ORBmatcher.cc:657-823.
 * K2 = {fx, fy, cx, cy} of KF2; writes min(cap, n) pairs (idx1, idx2) in idx1 order, returns n. */
int   ora_search_for_triangulation(const ora_featvec* fv1, const ora_kp* k1, const uint8_t* d1, const float* uR1,
                                   const uint8_t* hasMP1, int n1, const float* Tcw1, const ora_featvec* fv2,
                                   const ora_kp* k2, const uint8_t* d2, const float* uR2, const uint8_t* hasMP2,
                                   int n2, const float* Tcw2, const float* K2, const float* scale2,
                                   const float* sigma2_2, const float* F12, int bOnlyStereo, int checkOri,
                                   int* pairs, int cap);

/* ---- DBoW2 vocabulary (dbow2.c), reference Thirdparty/DBoW2 ------------------------ */
typedef struct ora_voc ora_voc;
ora_voc* ora_voc_load_text(const char* path, int* err);   /* loadFromTextFile, TemplatedVocabulary.h:1338 */
void  ora_voc_free(ora_voc* v);
void  ora_voc_info(const ora_voc* v, int* k, int* L, int* scoring, int* weighting, int* nnodes, int* nwords);
void  ora_voc_transform_feature(const ora_voc* v, const uint8_t* f, int levelsup, uint32_t* word, double* weight,
                                uint32_t* nid);
int   ora_voc_transform(const ora_voc* v, const uint8_t* desc, int N, int levelsup, uint32_t* bow_w, double* bow_v,
                        int* n_bow, uint32_t* fv_node, int* fv_start, int* fv_feat, int* n_fv);
double ora_voc_score_l1(const uint32_t* w1, const double* v1, int n1, const uint32_t* w2, const double* v2, int n2);

/* ---- Frame::UnprojectStereo (stereo.c), reference Frame.cc:666-680 ----------------
 * x3D = Rwc * ((u-cx)*z*invfx, (v-cy)*z*invfy, z) + Ow for depth z > 0 (invfx = 1.0f/fx,
 * Frame.cc:108); Twc = [Rwc | Ow] row-major 4x4; rows with z <= 0 untouched, mp[i] = i or -1. */
void  ora_unproject_stereo(const ora_kp* kps, const float* depth, int N, const float* Twc, float fx, float fy,
                           float cx, float cy, float* x3D, int* mp);

/* ---- cv::undistortPoints (ocv_semantics.c), OpenCV 3.2 cvUndistortPoints with R = I, P = K;
 * Frame::UndistortKeyPoints / ComputeImageBounds (stereo.c), Frame.cc:404-464 ------------
 * src/dst: n (x, y) float pairs; k: 8 double coefficients; has_dist = 0 runs one iteration
 * with k = 0 (no distortion).  bounds: minX, maxX, minY, maxY, grid width/height inverses. */
void  ora_undistort_points(const float* src, int n, const float K[9], const double k[8], int has_dist, float* dst);
void  ora_undistort_keypoints(const ora_kp* keys, int N, const float K[9], const float* dist, int ndist,
                              ora_kp* keysUn);
void  ora_compute_image_bounds(int cols, int rows, const float K[9], const float* dist, int ndist, float bounds[6]);

/* ---- Frame::ComputeStereoMatches (stereo.c), reference Frame.cc:466-640 ----------
 * kL/dL: left mvKeys + descriptors (NL), kR/dR: right (NR); exL/exR: the extractors that
 * produced them (their last pyramids); rows0 = level-0 rows.  Writes mvuRight / mvDepth
 * (-1 = none) and returns the number of stereo matches kept after the median filter. */
int   ora_compute_stereo_matches(const ora_kp* kL, const uint8_t* dL, int NL, const ora_kp* kR,
                                 const uint8_t* dR, int NR, const ora_extractor* exL,
                                 const ora_extractor* exR, int rows0, float mbf, float mb,
                                 float* uRight, float* depth);

/* ---- Local bundle adjustment (ba.c), reference Optimizer.cc:453-778 + g2o --- */
typedef struct {
    int n_kf;
    const int32_t* kf_id;      /* KeyFrame::mnId (vertex id) */
    const float* kf_Tcw;       /* n_kf x 16 row-major */
    const uint8_t* kf_local;   /* 1 = lLocalKeyFrames (written back; fixed iff id 0), 0 = lFixedCameras */
    const float* kf_cam;       /* n_kf x 5: fx fy cx cy bf */
    int n_pt;
    const int32_t* pt_id;      /* MapPoint::mnId */
    const float* pt_pos;       /* n_pt x 3 */
    int n_edge;                /* in the reference's creation order (map point, then observation order) */
    const int32_t* edge_pt;
    const int32_t* edge_kf;
    const float* edge_obs;     /* n_edge x 3: u, v, uRight (uRight < 0 = monocular edge) */
    const float* edge_inv_sigma2;
} ora_ba_problem;
typedef struct {
    float* kf_Tcw;             /* n_kf x 16 (local keyframes updated) */
    float* pt_pos;             /* n_pt x 3 */
    uint8_t* edge_erase;       /* n_edge: vToErase membership */
    int iterations[2];         /* optimize(5) / optimize(10) return values */
    int n_erased, aborted;
} ora_ba_result;
#define ORA_BA_TRACE_MAX 256
typedef struct {
    int n_solves, n_trials;
    double solve_ini_chi2[ORA_BA_TRACE_MAX], solve_chi2[ORA_BA_TRACE_MAX];
    double trial_chi2[ORA_BA_TRACE_MAX], trial_lambda[ORA_BA_TRACE_MAX];
} ora_ba_trace;
/* Optimizer::PoseOptimization (Optimizer.cc:239-451).  Per keypoint i < N: has_mp[i]
 * (mvpMapPoints[i] != NULL), Xw (GetWorldPos), obs = (kpUn.x, kpUn.y, mvuRight),
 * inv_sigma2 = mvInvLevelSigma2[kpUn.octave]. */
typedef struct {
    int N;
    const float* Tcw;
    const uint8_t* has_mp;
    const float* Xw;
    const float* obs;
    const float* inv_sigma2;
    float fx, fy, cx, cy, bf;
} ora_pose_problem;
/* ---- LocalMapping / LoopClosing projection searches (matchers3.c) ------- */
/* SearchByProjection(KeyFrame*, Scw, vpPoints, vpMatched, th)  ORBmatcher.cc:290-403.
 * K = fx fy cx cy; skip[i] = isBad || already found; matched: KF->N in/out (point index or -1). */
int   ora_search_by_projection_sim3(const ora_frame* KF, const float* K, const float* Scw, int np, const float* pos,
                                    const uint8_t* desc, const float* maxD, const float* minD, const float* normal,
                                    const uint8_t* skip, float logScaleFactor, int th, int* matched);
/* Fuse(KeyFrame*, vpMapPoints, th) 825-975: best[i] = KF keypoint to fuse with or -1.
 * K5 = fx fy cx cy mbf; skip[i] = !pMP || isBad || IsInKeyFrame(pKF). Returns nFused. */
int   ora_fuse(const ora_frame* KF, const float* Tcw, const float* K5, int np, const float* pos, const uint8_t* desc,
               const float* maxD, const float* minD, const float* normal, const uint8_t* skip, float logScaleFactor,
               float th, int* best);
/* Fuse(KeyFrame*, Scw, vpPoints, th, vpReplacePoint) 977-1100 (skip = isBad || in pKF's map points) */
int   ora_fuse_sim3(const ora_frame* KF, const float* K4, const float* Scw, int np, const float* pos,
                    const uint8_t* desc, const float* maxD, const float* minD, const float* normal,
                    const uint8_t* skip, float logScaleFactor, float th, int* best);
/* SearchBySim3(pKF1, pKF2, vpMatches12, s12, R12, t12, th) 1102-1326. mp1/mp2: map point of
 * each keypoint or -1; K = KF1 fx fy cx cy (used for both projections, as the reference);
 * matches12 (N1 in/out): -1 none, >= 0 KF2 keypoint of the matched point, -2 matched to a
 * point not in KF2.  Returns nFound (new agreements written as KF2 keypoint indices). */
int   ora_search_by_sim3(const ora_frame* KF1, const float* T1w, const int* mp1, const ora_frame* KF2,
                         const float* T2w, const int* mp2, const float* K, const float* pos, const uint8_t* desc,
                         const float* maxD, const float* minD, const uint8_t* bad, int* matches12, float s12,
                         const float* R12, const float* t12, float logScaleFactor, float th);

int   ora_pose_optimization(const ora_pose_problem* P, float* Tcw_out, uint8_t* outlier, ora_ba_trace* trace);
int   ora_ldlt_pivot_solve(double* H, int n, const double* b, double* x);
double ora_csum(double* v, int n);
int   ora_ldlt_solve(double* S, int n, const double* b, double* x);
/* ordering.c: nested-dissection order of a graph (adjacency lists sorted, symmetric) and the
 * block-sparse LDL^T of a grouped system in a given group order (perm: position -> group) */
#define ORA_TILED_MIN_POSES 24   /* the GPU's dense solvers take fewer free poses */
#define ORA_ND_LEAF 32
void  ora_nd_order(int n, const int* adjStart, const int* adj, int leaf, int* perm);
typedef struct ora_sp ora_sp;
ora_sp* ora_sp_create(int n, int g, const int* adjStart, const int* adj, const int* perm);
double* ora_sp_at(ora_sp* s, int r, int c);
int   ora_sp_solve(ora_sp* s, const double* b, double* x);
void  ora_sp_free(ora_sp* s);
int   ora_ldlt_solve_nd(const double* S, int n, const double* b, double* x);
enum { ORA_BA_CANONICAL = 0, ORA_BA_G2O = 1 };
void  ora_ba_set_order(int mode);   /* accumulation order of the BA / pose oracle (ba.c) */
int   ora_ba_get_order(void);
int   ora_local_ba(const ora_ba_problem* P, const volatile int* stop, ora_ba_result* R, ora_ba_trace* trace);
/* Optimizer::BundleAdjustment (Optimizer.cc:49-237): all keyframes vertices (fixed iff id 0),
 * one optimize(nIterations), Huber sqrt(5.99)/sqrt(7.815) iff bRobust, no gating. */
int   ora_global_ba(const ora_ba_problem* P, int nIterations, int bRobust, const volatile int* stop,
                    ora_ba_result* R, ora_ba_trace* trace);
/* Optimizer::OptimizeSim3 (Optimizer.cc:1046-1241).  Per index i < N of vpMatches1:
 * valid[i] (vpMatches1[i] && pMP1 && !isBad both && i2 >= 0), X1c/X2c = R1w*P3D1w+t1w /
 * R2w*P3D2w+t2w (N x 3, CV_32F), obs1 = pKF1->mvKeysUn[i].pt, obs2 = pKF2->mvKeysUn[i2].pt
 * (N x 2), inv_sigma2_1/2 = mvInvLevelSigma2[octave]; K = fx fy cx cy. */
typedef struct {
    int N;
    const uint8_t* valid;
    const float* X1c;
    const float* X2c;
    const float* obs1;
    const float* obs2;
    const float* inv_sigma2_1;
    const float* inv_sigma2_2;
    float K1[4], K2[4];
    float th2;
    int bFixScale;
} ora_sim3opt_problem;
/* S12 (8 doubles: quaternion x y z w, t, s) in/out (written only when the reference
 * reaches its second optimize); erased[i] = 1 where vpMatches1[i] is set to NULL.
 * Returns nIn (0 on the early return). */
int   ora_optimize_sim3(const ora_sim3opt_problem* P, double* S12, uint8_t* erased, ora_ba_trace* trace);
/* g2o::Sim3(Converter::toMatrix3d(R), toVector3d(t), s) */
void  ora_sim3_from_Rts(const float* R, const float* t, float s, double* S12);
double ora_det_exp(double x);
double ora_det_log(double x);
int ora_is_in_frustum(const float* Tcw, float fx, float fy, float cx, float cy, float mbf, float minX, float maxX,
                      float minY, float maxY, int nlevels, float logScaleFactor, int n, const float* pos,
                      const float* maxDist, const float* minDist, const float* normal, const uint8_t* skip,
                      float viewingCosLimit, uint8_t* inView, float* projX, float* projXR, float* projY, int* level,
                      float* viewCos);
long long ora_predict_scale_mismatches(float lo, float hi, float lsf, long long* n_checked, long long* n_logf_diff);

#ifdef __cplusplus
}
#endif
#endif
