// pnp.hpp -- gfx950 EPnP RANSAC (see pnp.hip).  Reference: src/PnPsolver.cc, include/PnPsolver.h.
#pragma once
#include <cstdint>
#include <vector>

#include "orb_common.hpp"
#include "../../include/orbslam_gpu.h"

namespace orbgpu {

void rng_seed(orb_rng* g, unsigned seed);
int rng_rand(orb_rng* g);

// per solver, persistent across iterate() calls, in the solver's device block: the best-so-far
// hypothesis (mnBestInliers, mBestTcw; its inlier mask follows) and the Refine() of that set
// (PnPsolver.cc:260-305, cached: it depends only on the best set and mvMaxError)
struct PnPStateDev {
    int nBest, refValid, refNin, pad;
    float bestTcw[16];
    double refRt[12];
};
// per solver per call: iterate()'s outputs (the inlier mask, N bits, follows)
struct PnPOutDev {
    int has_pose, bNoMore, nInliers, nIterations, consumed, pad[3];
    float Tcw[16];
    orb_rng rng;   // the stream after the draws the reference loop consumed
    int pad2[3];
};

struct PnPProbDev {
    const float* p3d;
    const float* p2d;
    const float* maxErr;
    int N;
    double fu, fv, uc, vc;
    // hypotheses
    int* hyp_idx;
    uint32_t* raw;   // the stream words behind the draws
    int nhyp, minSet;
    int* counts;
    uint32_t* masks;
    double* rt;
    // replay (PnPsolver::iterate's loop on the device)
    int minInliers, maxIts, nIt0, pad;
    orb_rng rng;     // the caller's stream at the call
    PnPStateDev* state;
    uint32_t* bestMask;
    uint32_t* refMask;
    int* refIdx;
    PnPOutDev* out;
    uint32_t* outMask;
};

struct PnPResult {
    int has_pose, bNoMore, nInliers;
    uint8_t* inliers;  // nMatches, caller-owned
    float Tcw[16];
};

class PnPSolver {
public:
    PnPSolver(int N, const float* p3d, const float* p2d, const float* sigma2, const int* kpIdx, int nMatches, float fx,
              float fy, float cx, float cy);
    ~PnPSolver();
    void set_ransac(double probability, int minInliers, int maxIterations, int minSet, float epsilon, float th2);
    int upload(hipStream_t s);
    int n_matches() const { return nMatches_; }
    int iterations() const { return nIterations_; }
    int max_its() const { return maxIts_; }
    int min_inliers() const { return minInliers_; }

    // data (PnPsolver.h:139-197)
    int N_, nMatches_;
    double fu_, fv_, uc_, vc_;
    std::vector<float> p3d_, p2d_, sigma2_, maxErr_;
    std::vector<int> kpIdx_;
    double prob_ = 0.99;
    int minInliers_ = 8, maxIts_ = 300, minSet_ = 4;
    float epsilon_ = 0.4f;
    // RANSAC state persisting across iterate() calls: the iteration counter here (it sizes a
    // call's hypotheses), the best set and its Refine() in the device block (PnPStateDev)
    int nIterations_ = 0;
    // device block: correspondences | PnPStateDev | best mask | Refine mask | Refine index list
    void* d_pts_ = nullptr;
    size_t d_pts_cap_ = 0;
    bool dev_dirty_ = true;
    bool ref_stale_ = false;   // set_ransac changed mvMaxError: the cached Refine() is void
    size_t state_off() const;
};

class PnPBatch {
public:
    ~PnPBatch();
    int init();
    int iterate(int n, PnPSolver** S, int nIterations, orb_rng** rngs, PnPResult* res);
    hipStream_t stream() const { return stream_; }
    void enable_timing(bool on) { timing_ = on; }
    int last_timings(float* ms2, long long* hyp_pts2);

private:
    bool timing_ = false, timed_ = false;
    hipEvent_t ev_[3] = {};
    long long last_hyp_ = 0, last_pts_ = 0;
    int ensure(size_t dev_bytes, size_t host_bytes, size_t probs);
    hipStream_t stream_ = nullptr;
    void* d_work_ = nullptr;
    void* d_probs_ = nullptr;
    void* h_work_ = nullptr;
    size_t work_cap_ = 0, hwork_cap_ = 0, probs_cap_ = 0;
};

// Layout invariant of PnPBatch::iterate's work area (unit entry): out4 = {device bytes
// allocated, device end touched, host bytes allocated, host end touched}; 0 if both fit.
int pnp_layout_check(int n, const int* N, const int* K, const int* minSet, long long* out4);

}  // namespace orbgpu
