// pnp.hpp -- gfx950 EPnP RANSAC (see pnp.hip).  Reference: src/PnPsolver.cc, include/PnPsolver.h.
#pragma once
#include <cstdint>
#include <vector>

#include "orb_common.hpp"
#include "../../include/orbslam_gpu.h"

namespace orbgpu {

void rng_seed(orb_rng* g, unsigned seed);
int rng_rand(orb_rng* g);

struct PnPProbDev {
    const float* p3d;
    const float* p2d;
    const float* maxErr;
    int N;
    double fu, fv, uc, vc;
    // hypotheses
    const int* hyp_idx;
    int nhyp, minSet;
    int* counts;
    uint32_t* masks;
    double* rt;
    // refine
    const int* ref_idx;
    int ref_n;
    uint32_t* ref_mask;
    double* ref_rt;
    int* ref_out;
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
    // RANSAC state persisting across iterate() calls
    int nIterations_ = 0, nBestInliers_ = 0;
    std::vector<uint8_t> bestInliers_;
    float bestTcw_[16] = {};
    // cached Refine() of the current best set
    bool refine_valid_ = false;
    int refine_pending_ = -1;
    int refNin_ = 0;
    std::vector<uint32_t> refMask_;
    double refRt_[12] = {};
    // device copy of the correspondences
    void* d_pts_ = nullptr;
    size_t d_pts_cap_ = 0;
    bool dev_dirty_ = true;
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
