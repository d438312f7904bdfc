// ba.hpp -- gfx950 local bundle adjustment (Optimizer::LocalBundleAdjustment,
// reference src/Optimizer.cc:453-778, g2o BlockSolver<6,3> + Levenberg).
#pragma once
#include <functional>
#include <hip/hip_runtime.h>

#include <cstdint>
#include <future>
#include <vector>

#include "../../include/orbslam_gpu.h"
#include "ba_struct.hpp"
#include "ba_struct_gpu.hpp"
#include "ba_types.hpp"
#include "comm.hpp"
#include "ldlt.hpp"
#include "orb_common.hpp"

namespace orbgpu {

// from this many free poses the reduced system is factored block-sparse (ldlt.hip)
constexpr int kBaTiledMinPoses = 24;

struct Se3 {  // g2o::SE3Quat: q = (x, y, z, w) like Eigen coeffs(), t
    double q[4];
    double t[3];
    double pad;
};

struct BaTrace {
    std::vector<double> solve_ini_chi2, solve_chi2, trial_chi2, trial_lambda;
};

// Which reference optimisation a run restates.
struct BaMode {
    bool global = false;   // false: Optimizer::LocalBundleAdjustment (Optimizer.cc:453-778)
                           // true:  Optimizer::BundleAdjustment (Optimizer.cc:49-237)
    int iterations = 10;   // global: optimize(nIterations)
    bool robust = true;    // global: bRobust
};

// device-resident LM state (ba.hip k_lm_begin / k_lm_decide): gates of the next step's kernels
// (ctl: 0 trial, 1 system, 2 lambda init), the Levenberg state and the per-trial trace
constexpr int kLmTrials = 128;   // 10 trials x <= 12 iterations per optimize() call
constexpr int kLmSolves = 16;
struct LmDev {
    int ctl[4];
    int it, iterations, qmax, nBad, haveChi, done, nTrial, nSolve, steps;
    double ni, currentChi, iniChi;
    double trialChi[kLmTrials], trialLam[kLmTrials], solveIni[kLmSolves], solveChi[kLmSolves];
};

class BaEngine {
public:
    ~BaEngine();
    int init();
    // comm == nullptr: the whole problem on this device.  Otherwise P is this rank's
    // shard (every keyframe, the rank's own map points and all of their edges) and
    // every rank of comm calls run() with the same keyframes and mode.
    int run(const ba_problem* P, const volatile bool* stop, ba_result* R, Comm* comm = nullptr,
            const BaMode* mode = nullptr);
    const BaTrace& trace() const { return trace_; }
    double last_ms[4] = {0, 0, 0, 0};  // total, structure (host), solves (device+control), io
    // last run: sharded factorisation used, separator tiles and rows exchanged, Schur-pattern tiles
    int last_dist[4] = {0, 0, 0, 0};
    // the last run's LM control: [0] steps the device-resident LM queued, [1] trials the host loop
    // (lm_solve) decided after a readback, [2] 1 if sharded (Optimizer_last_lm_path)
    int last_lm[4] = {0, 0, 0, 0};
    // set by the C ABI before run(): every map point's edges form one run (validated), so the
    // unsharded global BA may derive the pose graph from the caller's edges on the host while
    // the device builds the lists (early_pose_graph)
    bool edgesGrouped = false;
    // set by the C ABI before run(): one edge per (map point, keyframe) was checked there, so the
    // host structure builder skips its own duplicate check
    bool edgesValidated = false;

private:
    int upload_problem(const ba_problem* P);
    int build_structure(int level);
    int gather_blocks(const std::vector<int64_t>& mine, std::vector<int64_t>* all);
    int optimize(int iterations, const volatile bool* stop, int* its);
    int lm_solve(int iteration, const volatile bool* stop, bool* terminate);
    bool device_lm(int iterations) const;
    int optimize_device(int iterations, const volatile bool* stop, int* its);
    void enqueue_lm_step(bool first);
    // the same step for a rank of a sharded run: lm_solve's kernels and exchanges, gated
    int enqueue_lm_step_comm(bool first);
    // the structure builder of this call: the one-workgroup device builder (local-BA sizes,
    // unsharded), else the host lists below the device builder's edge threshold
    bool small_struct() const;
    bool host_lists() const;
    bool smallUp_ = false;                          // this call's upload staged the builder's inputs
    int32_t *dKp_ = nullptr, *dPtOrd_ = nullptr;    // (keyframe << 13) | point per edge; points by id
    int32_t* dSmKid_ = nullptr;                     // keyframe ids and fixed flags (same block)
    uint8_t* dSmFx_ = nullptr;
    char* dSmallIn_ = nullptr;
    // the problem's H2D copy + unpack, prepared by upload_problem and queued by issue_upload
    // (right away, or behind the level-0 one-workgroup structure kernel)
    bool deferredUpload_ = false;
    std::vector<char> deferArgs_;
    size_t deferBytes_ = 0;
    int issue_upload();
    double* dLmStage_ = nullptr;   // the system's all-reduce staging (Hpp, b_p, chi2) of enqueue_lm_step_comm
    size_t lmStageCap_ = 0;
    int gate_edges(int final_check, uint8_t* erase);
    int carve(bool commit, size_t* total);
    bool stopped(const volatile bool* stop) const { return comm_ ? stopRed_ : (stop && *stop); }
    int reduce_stop(const volatile bool* stop);
    bool sharded() const { return comm_ && comm_->size() > 1; }
    // the single-workgroup dense solvers (register-resident or LDS-resident S) take n
    bool dense_solver(int n) const;

    hipStream_t stream_ = nullptr;
    // problem (device)
    int nkf_ = 0, npt_ = 0, ne_ = 0;
    Se3 *dT_ = nullptr, *dTbak_ = nullptr;
    double *dX_ = nullptr, *dXbak_ = nullptr;
    EdgeDev* dE_ = nullptr;
    uint8_t *dLevel_ = nullptr, *dRobust_ = nullptr;
    double* dErr_ = nullptr;       // ne x 3, last computed _error
    // host mirror of the static problem
    std::vector<int32_t> kfId_, ptId_;
    const int32_t* ePt_ = nullptr;   // the current call's edge arrays (ba_problem, caller-owned)
    const int32_t* eKf_ = nullptr;
    std::vector<uint8_t> kfFixed_, kfLocal_, level_, ptHasEdge_, kfHasEdge_;
    // structure
    BaStructDev st_{};
    BaHostStruct hs_;              // host lists of the current structure (ORBGPU_STRUCT_HOST=1 path)
    GpuStructBuilder gs_;          // the lists built on the device (default)
    uint8_t* dKfFixed_ = nullptr;  // device copies of the static vertex data the builder reads
    int32_t *dKfId_ = nullptr, *dPtId_ = nullptr;
    int32_t* dStruct_ = nullptr;
    size_t dStructCap_ = 0;
    // system / workspace
    double *dTerms_ = nullptr, *dRc_ = nullptr, *dHpp_ = nullptr, *dBp_ = nullptr, *dHll_ = nullptr, *dBl_ = nullptr;
    double *dB_ = nullptr, *dX2_ = nullptr, *dS_ = nullptr, *dBs_ = nullptr, *dDinv_ = nullptr, *dDb_ = nullptr;
    double *dEmat_ = nullptr, *dCb_ = nullptr, *dScal_ = nullptr, *dScratch_ = nullptr, *dHplA_ = nullptr;
    int32_t* dPePos_ = nullptr;   // device-built structures: active edge -> pose-list position
    Se3* dTn_ = nullptr;          // the device LM's trial poses / points (fused update), committed on acceptance
    double* dXn_ = nullptr;
    std::vector<int32_t> hPePos_;   // host-built structures: the same, packed with the lists
    int blkChunks_ = 1;   // chunks (64 terms) of the structure's longest Schur block
    double *tmpA0_ = nullptr, *tmpA1_ = nullptr, *tmpB0_ = nullptr, *tmpB1_ = nullptr;
    unsigned* dCounter_ = nullptr;
    SparseLdlt sp_;                // block-sparse pose system (n > the dense solvers' reach)
    // the early pose graph (host, from the caller's edges) + nested dissection + symbolic
    // factorisation, started before the device lists: its pose count, and its keys when checked
    std::future<int> spEarly_;
    int spEarlyNP_ = -1;
    std::vector<int64_t> spEarlyKeys_;
    int start_early_pose_graph();
    std::future<int> spBuild_;     // sp_.build on a helper thread (unsharded global BA): joined by
                                   // join_sp_build() before the first use of sp_ (lm_solve's Schur)
    int join_sp_build();
    bool tiled_ = false;
    bool distOk_ = false;   // sharded factorisation planned and the ranks' points aligned to it
    void* arena_ = nullptr;
    size_t arenaCap_ = 0;
    double* hScal_ = nullptr;      // pinned
    LmDev* dLm_ = nullptr;         // device LM state (arena)
    int* hLm_ = nullptr;           // pinned coherent: stop mirror, done, steps, iterations
    hipEvent_t lmEv_[2] = {nullptr, nullptr};
    // pinned staging of the setup uploads (problem arrays, structure): several engines set up
    // concurrently from different host threads, so no pageable hipMemcpy staging path is used
    void* hStage_ = nullptr;
    size_t hStageCap_ = 0;
    bool uploadPending_ = false;   // upload_problem's copies may still read hStage_
    // the structure lists' own staging block: packed while the problem upload still reads hStage_,
    // its copy not waited for (the next structure's pack waits if it is still pending)
    void* hStage2_ = nullptr;
    size_t hStage2Cap_ = 0;
    bool stage2Pending_ = false;
    int stage2_reserve(size_t bytes);
    int h2d_sync(void* dst, const void* src, size_t bytes);
    int d2h_sync(void* dst, const void* src, size_t bytes);
    int d2h_poll(void* dst, const void* src, size_t bytes);   // d2h_sync without the blocking wait
    int poll_stream();                                         // drain the stream by polling hLm_[8]
    BaHostStruct hs2_;            // the refined lists of a second pass (swapped into hs_)
    bool hsValid_ = false, refineNext_ = false;
    int signalSeq_ = 0;
    int stage_reserve(size_t bytes);
    size_t scratchN_ = 0;
    size_t ldsMax_ = 0;
    // sharding
    Comm* comm_ = nullptr;
    bool stopRed_ = false;
    int nEglob_ = 0, nLglob_ = 0;
    int nTiles_ = 0;               // union Schur tiles exchanged per trial
    void* dPack_ = nullptr;
    size_t packCap_ = 0;
    int2* dTiles_ = nullptr;
    double* dPackBuf_ = nullptr;
    BaMode mode_{};
    // LM state (g2o OptimizationAlgorithmLevenberg)
    double lambda_ = 0, ni_ = 2;
    int nBad_ = 0;
    BaTrace trace_;
};

struct PoseEdgeDev;
struct PoseProbDev;

// Optimizer::PoseOptimization for a batch of frames: one persistent workgroup per frame.
struct PoseProbDev;
class PoseEngine {
public:
    ~PoseEngine();
    int init();
    int run(int count, const pose_problem* P, float* Tcw_out, uint8_t* const* outlier, int* ninliers);
    // P's arrays, Tcw_out[f] (16 floats) and outlier[f] are device pointers
    int run_device(int count, const pose_problem* P, float* const* Tcw_out, uint8_t* const* outlier, int* ninliers);
    // pose_frame form: the edges are gathered from the frame's own arrays on the device
    // s / chain: enqueue on the caller's stream inside its DeferredChain (results at finish())
    int run_frames_device(int count, const pose_frame* F, float* const* Tcw_out, uint8_t* const* outlier,
                          int* ninliers, hipStream_t s = nullptr, DeferredChain* chain = nullptr);
    hipStream_t stream() const { return stream_; }
    // k_pose_opt duration of the last launch (HIP events on its stream) while timing is on
    void set_timing(bool on) { timing_ = on; }
    int last_timing(float* ms);

private:
    int launch_device(int count, const int* Ns, const std::function<void(int, PoseProbDev&)>& fill,
                      float* const* Tcw_out, uint8_t* const* outlier, int* ninliers, hipStream_t s = nullptr,
                      DeferredChain* chain = nullptr);
    hipStream_t stream_ = nullptr;
    void* dArena_ = nullptr;
    void* hArena_ = nullptr;   // pinned staging: problems + edges in, outliers back
    size_t cap_ = 0;
    // recorded after the last work that reads dArena_ (on whichever stream it was queued):
    // the next user waits on it before overwriting the arena
    hipEvent_t lastUse_ = nullptr;
    bool lastUseSet_ = false;
    bool timing_ = false, timed_ = false;
    hipEvent_t tA_ = nullptr, tB_ = nullptr;
};

int debug_ldlt(int n, const double* S, const double* b, double* x, int variant);
int debug_csum(const double* v, int n, double* out);
int debug_ldlt_factor(int n, const double* S, double* out);
int debug_wave_tree(const double* v64, double* out);
int debug_shared_div(const double* a, const double* b, int n, double* out);
int debug_set_csum_lds_max(int v);
int debug_set_scale_small_max(int v);
int debug_set_struct_gpu_min_edges(int v);
int debug_set_posegraph_check(int on);
int debug_prof(unsigned long long* out32);

}  // namespace orbgpu
