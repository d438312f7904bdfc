// capi_pnp.cpp -- extern "C" PnPsolver_* and orb_rng_* (include/orbslam_gpu.h).
// Replaces ORB_SLAM2::PnPsolver (reference include/PnPsolver.h:59-196).
#include <mutex>
#include <new>
#include <vector>

#include "pnp.hpp"

struct PnPsolver_t {
    orbgpu::PnPSolver* s;
};

namespace {
// one batch engine (stream + workspace) per thread that calls the solvers
orbgpu::PnPBatch* engine(int* rc) {
    thread_local orbgpu::PnPBatch* e = nullptr;
    thread_local int erc = 0;
    if (!e) {
        e = new orbgpu::PnPBatch();
        erc = e->init();
    }
    *rc = erc;
    return e;
}
}  // namespace

extern "C" {

void orb_rng_seed(orb_rng* g, unsigned seed) {
    if (g) orbgpu::rng_seed(g, seed);
}

int orb_rng_rand(orb_rng* g) { return g ? orbgpu::rng_rand(g) : 0; }

int PnPsolver_create(int N, const float* p3d, const float* p2d, const float* sigma2, const int32_t* kp_index,
                     int n_matches, float fx, float fy, float cx, float cy, PnPsolver_h* out) {
    if (!out || N < 0 || n_matches < N || (N > 0 && (!p3d || !p2d || !sigma2 || !kp_index))) return ORB_E_INVALID;
    for (int i = 0; i < N; i++)
        if (kp_index[i] < 0 || kp_index[i] >= n_matches) return ORB_E_INVALID;
    *out = nullptr;
    int rc = 0;
    engine(&rc);
    if (rc) return rc == -4 ? ORB_E_NODEVICE : ORB_E_HIP;
    auto* s = new (std::nothrow) orbgpu::PnPSolver(N, p3d, p2d, sigma2, kp_index, n_matches, fx, fy, cx, cy);
    if (!s) return ORB_E_INVALID;
    *out = new PnPsolver_t{s};
    return ORB_OK;
}

int PnPsolver_destroy(PnPsolver_h h) {
    if (!h) return ORB_E_INVALID;
    delete h->s;
    delete h;
    return ORB_OK;
}

int PnPsolver_set_ransac(PnPsolver_h h, double probability, int minInliers, int maxIterations, int minSet,
                         float epsilon, float th2) {
    if (!h || minSet < 1 || minSet > 64) return ORB_E_INVALID;
    h->s->set_ransac(probability, minInliers, maxIterations, minSet, epsilon, th2);
    return ORB_OK;
}

int PnPsolver_get_state(PnPsolver_h h, int* iterations, int* max_its, int* min_inliers) {
    if (!h) return ORB_E_INVALID;
    if (iterations) *iterations = h->s->iterations();
    if (max_its) *max_its = h->s->max_its();
    if (min_inliers) *min_inliers = h->s->min_inliers();
    return ORB_OK;
}

int PnPsolver_iterate_batch(int count, PnPsolver_h* hs, int nIterations, orb_rng** rngs, int* bNoMore,
                            uint8_t** inliers, int* nInliers, float* Tcw, int* has_pose) {
    if (count < 0 || (count > 0 && (!hs || !rngs || !bNoMore || !inliers || !nInliers || !Tcw || !has_pose)))
        return ORB_E_INVALID;
    for (int k = 0; k < count; k++)
        if (!hs[k] || !rngs[k] || (!inliers[k] && hs[k]->s->n_matches() > 0) || hs[k]->s->minSet_ > hs[k]->s->N_ + 64)
            return ORB_E_INVALID;
    int rc = 0;
    orbgpu::PnPBatch* e = engine(&rc);
    if (rc) return rc == -4 ? ORB_E_NODEVICE : ORB_E_HIP;
    // the same stream object shared by several solvers must be consumed in solver order, and a
    // handle listed twice carries its state (best set, cached Refine, counter) from one entry to
    // the next: run those batches sequentially (one replay workgroup per entry would race on the
    // handle's device state), independent entries together
    std::vector<orbgpu::PnPSolver*> S(count);
    std::vector<orbgpu::PnPResult> R(count);
    for (int k = 0; k < count; k++) {
        S[k] = hs[k]->s;
        R[k].inliers = inliers[k];
        if (S[k]->N_ >= S[k]->minInliers_ && S[k]->minSet_ > S[k]->N_) return ORB_E_INVALID;
    }
    bool shared = false;
    for (int k = 1; k < count && !shared; k++)
        for (int j = 0; j < k; j++)
            if (rngs[j] == rngs[k] || hs[j] == hs[k]) { shared = true; break; }
    int r = 0;
    if (!shared) {
        r = e->iterate(count, S.data(), nIterations, rngs, R.data());
    } else {
        for (int k = 0; k < count && !r; k++) r = e->iterate(1, &S[k], nIterations, &rngs[k], &R[k]);
    }
    if (r) return r == -2 ? ORB_E_HIP : ORB_E_INVALID;
    for (int k = 0; k < count; k++) {
        bNoMore[k] = R[k].bNoMore;
        nInliers[k] = R[k].nInliers;
        has_pose[k] = R[k].has_pose;
        for (int i = 0; i < 16; i++) Tcw[16 * k + i] = R[k].has_pose ? R[k].Tcw[i] : 0.f;
    }
    return ORB_OK;
}

int PnPsolver_iterate(PnPsolver_h h, int nIterations, orb_rng* rng, int* bNoMore, uint8_t* inliers, int* nInliers,
                      float* Tcw, int* has_pose) {
    return PnPsolver_iterate_batch(1, &h, nIterations, &rng, bNoMore, &inliers, nInliers, Tcw, has_pose);
}

int PnPsolver_enable_timing(int on) {
    int rc = 0;
    orbgpu::PnPBatch* e = engine(&rc);
    if (rc) return rc == -4 ? ORB_E_NODEVICE : ORB_E_HIP;
    e->enable_timing(on != 0);
    return ORB_OK;
}

int PnPsolver_last_timings(float* ms2, long long* counts2) {
    if (!ms2 || !counts2) return ORB_E_INVALID;
    int rc = 0;
    orbgpu::PnPBatch* e = engine(&rc);
    if (rc) return rc == -4 ? ORB_E_NODEVICE : ORB_E_HIP;
    return e->last_timings(ms2, counts2) ? ORB_E_INVALID : ORB_OK;
}

int orbgpu_unit_pnp_layout(int n, const int* N, const int* K, const int* minSet, long long* out4) {
    if (n < 0 || (n > 0 && (!N || !K || !minSet)) || !out4) return ORB_E_INVALID;
    return orbgpu::pnp_layout_check(n, N, K, minSet, out4) ? ORB_E_CAPACITY : ORB_OK;
}

}  // extern "C"
