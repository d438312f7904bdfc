// capi_sim3.cpp -- extern "C" Sim3Solver_* (include/orbslam_gpu.h).
// Replaces ORB_SLAM2::Sim3Solver (reference include/Sim3Solver.h:39-137).
#include <cstring>
#include <new>
#include <vector>

#include "sim3.hpp"

struct Sim3Solver_t {
    orbgpu::Sim3Solver* s;
};

namespace {
orbgpu::Sim3Batch* engine(int* rc) {
    thread_local orbgpu::Sim3Batch* e = nullptr;
    thread_local int erc = 0;
    if (!e) {
        e = new orbgpu::Sim3Batch();
        erc = e->init();
    }
    *rc = erc;
    return e;
}
}  // namespace

extern "C" {

int Sim3Solver_create(int N, const float* X1c, const float* X2c, const float* sigma2_1, const float* sigma2_2,
                      const int32_t* idx1, int N1, const float* K1, const float* K2, int bFixScale,
                      Sim3Solver_h* out) {
    if (!out || N < 3 || N1 < N || !X1c || !X2c || !sigma2_1 || !sigma2_2 || !idx1 || !K1 || !K2)
        return ORB_E_INVALID;
    for (int i = 0; i < N; i++)
        if (idx1[i] < 0 || idx1[i] >= N1) return ORB_E_INVALID;
    *out = nullptr;
    int rc = 0;
    engine(&rc);
    if (rc) return rc == -4 ? ORB_E_NODEVICE : ORB_E_HIP;
    auto* s = new (std::nothrow) orbgpu::Sim3Solver(N, X1c, X2c, sigma2_1, sigma2_2, idx1, N1, K1, K2, bFixScale != 0);
    if (!s) return ORB_E_INVALID;
    *out = new Sim3Solver_t{s};
    return ORB_OK;
}

int Sim3Solver_destroy(Sim3Solver_h h) {
    if (!h) return ORB_E_INVALID;
    delete h->s;
    delete h;
    return ORB_OK;
}

int Sim3Solver_set_ransac(Sim3Solver_h h, double probability, int minInliers, int maxIterations) {
    if (!h) return ORB_E_INVALID;
    h->s->set_ransac(probability, minInliers, maxIterations);
    return ORB_OK;
}

int Sim3Solver_get_state(Sim3Solver_h h, int* iterations, int* max_its, int* min_inliers) {
    if (!h) return ORB_E_INVALID;
    if (iterations) *iterations = h->s->nIterations_;
    if (max_its) *max_its = h->s->maxIts_;
    if (min_inliers) *min_inliers = h->s->minInliers_;
    return ORB_OK;
}

int Sim3Solver_get_estimate(Sim3Solver_h h, float* R, float* t, float* s) {
    if (!h) return ORB_E_INVALID;
    if (R) std::memcpy(R, h->s->bestR_, 36);
    if (t) std::memcpy(t, h->s->bestT_, 12);
    if (s) *s = h->s->bestS_;
    return ORB_OK;
}

int Sim3Solver_iterate_batch(int count, Sim3Solver_h* hs, int nIterations, orb_rng** rngs, int* bNoMore,
                             uint8_t** inliers, int* nInliers, float* T12, int* has_pose) {
    if (count < 0 || (count > 0 && (!hs || !rngs || !bNoMore || !inliers || !nInliers || !T12 || !has_pose)))
        return ORB_E_INVALID;
    for (int k = 0; k < count; k++)
        if (!hs[k] || !rngs[k] || !inliers[k]) return ORB_E_INVALID;
    int rc = 0;
    orbgpu::Sim3Batch* e = engine(&rc);
    if (rc) return rc == -4 ? ORB_E_NODEVICE : ORB_E_HIP;
    std::vector<orbgpu::Sim3Solver*> S(count);
    std::vector<orbgpu::Sim3Result> R(count);
    for (int k = 0; k < count; k++) {
        S[k] = hs[k]->s;
        R[k].inliers = inliers[k];
    }
    // a stream shared by several solvers is consumed in solver order, and a handle listed twice
    // carries its state (best set, counter) from one entry to the next: both run sequentially
    // (one replay workgroup per entry would otherwise race on the handle's device state)
    bool shared = false;
    for (int k = 1; k < count && !shared; k++)
        for (int j = 0; j < k; j++)
            if (rngs[j] == rngs[k] || hs[j] == hs[k]) { shared = true; break; }
    int r = 0;
    if (!shared) r = e->iterate(count, S.data(), nIterations, rngs, R.data());
    else
        for (int k = 0; k < count && !r; k++) r = e->iterate(1, &S[k], nIterations, &rngs[k], &R[k]);
    if (r) return r == -2 ? ORB_E_HIP : ORB_E_INVALID;
    for (int k = 0; k < count; k++) {
        bNoMore[k] = R[k].bNoMore;
        nInliers[k] = R[k].nInliers;
        has_pose[k] = R[k].has_pose;
        for (int i = 0; i < 16; i++) T12[16 * k + i] = R[k].has_pose ? R[k].T12[i] : 0.f;
    }
    return ORB_OK;
}

int Sim3Solver_iterate(Sim3Solver_h h, int nIterations, orb_rng* rng, int* bNoMore, uint8_t* inliers, int* nInliers,
                       float* T12, int* has_pose) {
    return Sim3Solver_iterate_batch(1, &h, nIterations, &rng, bNoMore, &inliers, nInliers, T12, has_pose);
}

int Sim3Solver_enable_timing(int on) {
    int rc = 0;
    orbgpu::Sim3Batch* e = engine(&rc);
    if (rc) return rc == -4 ? ORB_E_NODEVICE : ORB_E_HIP;
    e->enable_timing(on != 0);
    return ORB_OK;
}

int Sim3Solver_last_timings(float* ms2, long long* counts2) {
    if (!ms2 || !counts2) return ORB_E_INVALID;
    int rc = 0;
    orbgpu::Sim3Batch* e = engine(&rc);
    if (rc) return rc == -4 ? ORB_E_NODEVICE : ORB_E_HIP;
    return e->last_timings(ms2, counts2) ? ORB_E_INVALID : ORB_OK;
}

}  // extern "C"
