// sim3.hpp -- gfx950 Sim3 RANSAC (see sim3.hip).  Reference: src/Sim3Solver.cc, include/Sim3Solver.h.
#pragma once
#include <cstdint>
#include <vector>

#include "orb_common.hpp"
#include "pnp.hpp"

namespace orbgpu {

struct Sim3ProbDev {
    const float* X1;   // N x 3 camera-frame points of KF1 (mvX3Dc1)
    const float* X2;   // N x 3 (mvX3Dc2)
    const float* p1;   // N x 2 mvP1im1
    const float* p2;   // N x 2 mvP2im2
    const float* maxErr1;  // (float)(size_t)(9.210*sigma2)
    const float* maxErr2;
    int N, bFixScale;
    float K1[4], K2[4];
    const int* hyp_idx;  // nhyp x 3
    int nhyp;
    int* counts;
    uint32_t* masks;
    float* est;          // nhyp x 32: R9 t3 s T12[16]
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
    int nIterations_ = 0, nBestInliers_ = 0;
    std::vector<uint8_t> bestInliers_;
    float bestR_[9] = {}, bestT_[3] = {}, bestS_ = 0, bestT12_[16] = {};
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
