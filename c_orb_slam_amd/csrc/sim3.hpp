// sim3.hpp -- gfx950 Sim3 RANSAC (see sim3.hip).  Reference: src/Sim3Solver.cc, include/Sim3Solver.h.
#pragma once
#include <cstdint>
#include <vector>

#include "orb_common.hpp"
#include "pnp.hpp"

namespace orbgpu {

// per solver, persistent across iterate() calls, in the solver's device block: the best-so-far
// estimate (mnBestInliers, mBestRotation / mBestTranslation / mBestScale / mBestT12)
struct Sim3StateDev {
    int nBest, pad[3];
    float bestR[9], bestT[3], bestS, bestT12[16], pad2[3];
};
// per solver per call: iterate()'s outputs (the inlier mask, N bits, follows)
struct Sim3OutDev {
    int has_pose, bNoMore, nInliers, nIterations, consumed, nBest, pad[2];
    float T12[16];
    float bestR[9], bestT[3], bestS, pad2[3];
    orb_rng rng;   // the stream after the draws the reference loop consumed
    int pad3[3];
};

struct Sim3ProbDev {
    const float* X1;   // N x 3 camera-frame points of KF1 (mvX3Dc1)
    const float* X2;   // N x 3 (mvX3Dc2)
    const float* p1;   // N x 2 mvP1im1
    const float* p2;   // N x 2 mvP2im2
    const float* maxErr1;  // (float)(size_t)(9.210*sigma2)
    const float* maxErr2;
    int N, bFixScale;
    float K1[4], K2[4];
    int* hyp_idx;  // nhyp x 3
    uint32_t* raw;     // the stream words behind the draws
    int nhyp;
    int* counts;
    uint32_t* masks;
    float* est;          // nhyp x 32: R9 t3 s T12[16]
    // replay (Sim3Solver::iterate's loop on the device)
    int minInliers, maxIts, nIt0, pad;
    orb_rng rng;
    Sim3StateDev* state;
    Sim3OutDev* out;
    uint32_t* outMask;
};

class Sim3Solver {
public:
    Sim3Solver(int N, const float* X1c, const float* X2c, const float* sigma2_1, const float* sigma2_2,
               const int* idx1, int N1, const float* K1, const float* K2, bool bFixScale);
    ~Sim3Solver();
    void set_ransac(double probability, int minInliers, int maxIterations);
    int upload(hipStream_t s);

    int N_, N1_;
    bool bFixScale_;
    std::vector<float> X1_, X2_, p1_, p2_, maxErr1_, maxErr2_;
    std::vector<int> idx1_;
    float K1_[4], K2_[4];
    double prob_ = 0.99;
    int minInliers_ = 6, maxIts_ = 300;
    int nIterations_ = 0, nBestInliers_ = 0;   // mirrors of the device state after each call
    float bestR_[9] = {}, bestT_[3] = {}, bestS_ = 0;
    size_t state_off() const;
    void* d_pts_ = nullptr;
    size_t d_cap_ = 0;
    bool dirty_ = true;
};

struct Sim3Result {
    int has_pose, bNoMore, nInliers;
    uint8_t* inliers;  // N1
    float T12[16];
};

class Sim3Batch {
public:
    ~Sim3Batch();
    int init();
    int iterate(int n, Sim3Solver** S, int nIterations, orb_rng** rngs, Sim3Result* res);
    void enable_timing(bool on) { timing_ = on; }
    int last_timings(float* ms2, long long* hyp_pts2);

private:
    bool timing_ = false, timed_ = false;
    hipEvent_t ev_[3] = {};
    long long last_hyp_ = 0, last_pts_ = 0;
    hipStream_t stream_ = nullptr;
    void *d_work_ = nullptr, *d_probs_ = nullptr, *h_work_ = nullptr;
    size_t work_cap_ = 0, probs_cap_ = 0, hwork_cap_ = 0;
};

}  // namespace orbgpu
