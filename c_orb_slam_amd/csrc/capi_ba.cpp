// capi_ba.cpp -- extern "C" Optimizer_LocalBundleAdjustment (include/orbslam_gpu.h).
// Replaces ORB_SLAM2::Optimizer::LocalBundleAdjustment (reference src/Optimizer.cc:453-778).
#include <algorithm>
#include <cstring>
#include <new>
#include <unordered_set>

#include "ba.hpp"

namespace {
orbgpu::BaEngine* engine(int* rc) {
    thread_local orbgpu::BaEngine* e = nullptr;
    thread_local int erc = 0;
    if (!e) {
        e = new orbgpu::BaEngine();
        erc = e->init();
    }
    *rc = erc;
    return e;
}

int validate(const ba_problem* P, const ba_result* R) {
    if (!P || !R || P->n_kf < 0 || P->n_pt < 0 || P->n_edge < 0) return ORB_E_INVALID;
    if (P->n_kf && (!P->kf_id || !P->kf_Tcw || !P->kf_local || !P->kf_cam || !R->kf_Tcw)) return ORB_E_INVALID;
    if (P->n_pt && (!P->pt_id || !P->pt_pos || !R->pt_pos)) return ORB_E_INVALID;
    if (P->n_edge && (!P->edge_pt || !P->edge_kf || !P->edge_obs || !P->edge_inv_sigma2 || !R->edge_erase))
        return ORB_E_INVALID;
    std::unordered_set<int32_t> ids;
    for (int k = 0; k < P->n_kf; k++)
        if (!ids.insert(P->kf_id[k]).second) return ORB_E_INVALID;
    ids.clear();
    for (int p = 0; p < P->n_pt; p++)
        if (!ids.insert(P->pt_id[p]).second) return ORB_E_INVALID;
    std::unordered_set<int64_t> pairs;
    for (int i = 0; i < P->n_edge; i++) {
        const int32_t pt = P->edge_pt[i], kf = P->edge_kf[i];
        if (pt < 0 || pt >= P->n_pt || kf < 0 || kf >= P->n_kf) return ORB_E_INVALID;
        if (!pairs.insert((int64_t)pt * P->n_kf + kf).second) return ORB_E_INVALID;
    }
    if (6LL * P->n_kf > 6LL * 4096) return ORB_E_CAPACITY;
    return ORB_OK;
}
}  // namespace

extern "C" {

int Optimizer_LocalBundleAdjustment(const ba_problem* P, const volatile bool* stop, ba_result* R) {
    if (int v = validate(P, R)) return v;
    int rc = 0;
    orbgpu::BaEngine* e = engine(&rc);
    if (rc) return rc == -4 ? ORB_E_NODEVICE : ORB_E_HIP;
    const int r = e->run(P, stop, R);
    if (r == -1) return ORB_E_INVALID;
    if (r == -3) return ORB_E_CAPACITY;
    return r ? ORB_E_HIP : ORB_OK;
}

int Optimizer_last_trace(double* solve_ini_chi2, double* solve_chi2, int solve_cap, int* n_solves,
                         double* trial_chi2, double* trial_lambda, int trial_cap, int* n_trials) {
    int rc = 0;
    orbgpu::BaEngine* e = engine(&rc);
    if (rc) return rc == -4 ? ORB_E_NODEVICE : ORB_E_HIP;
    const orbgpu::BaTrace& t = e->trace();
    const int ns = (int)t.solve_chi2.size(), nt = (int)t.trial_chi2.size();
    if (n_solves) *n_solves = ns;
    if (n_trials) *n_trials = nt;
    for (int i = 0; i < std::min(ns, solve_cap); i++) {
        if (solve_ini_chi2) solve_ini_chi2[i] = t.solve_ini_chi2[i];
        if (solve_chi2) solve_chi2[i] = t.solve_chi2[i];
    }
    for (int i = 0; i < std::min(nt, trial_cap); i++) {
        if (trial_chi2) trial_chi2[i] = t.trial_chi2[i];
        if (trial_lambda) trial_lambda[i] = t.trial_lambda[i];
    }
    return ORB_OK;
}

int Optimizer_last_timings(double* ms2) {
    if (!ms2) return ORB_E_INVALID;
    int rc = 0;
    orbgpu::BaEngine* e = engine(&rc);
    if (rc) return rc == -4 ? ORB_E_NODEVICE : ORB_E_HIP;
    ms2[0] = e->last_ms[0];
    ms2[1] = e->last_ms[1];
    return ORB_OK;
}

int orbgpu_unit_ldlt_solve(int n, const double* S, const double* b, double* x, int variant, int* ok) {
    if (n < 0 || (n > 0 && (!S || !b || !x)) || !ok) return ORB_E_INVALID;
    int rc = 0;
    engine(&rc);
    if (rc) return rc == -4 ? ORB_E_NODEVICE : ORB_E_HIP;
    const int r = orbgpu::debug_ldlt(n, S, b, x, variant);
    if (r < 0) return r == -3 ? ORB_E_CAPACITY : ORB_E_HIP;
    *ok = r;
    return ORB_OK;
}

int orbgpu_unit_wave_tree(const double* v64, double* out) {
    if (!v64 || !out) return ORB_E_INVALID;
    int rc = 0;
    engine(&rc);
    if (rc) return rc == -4 ? ORB_E_NODEVICE : ORB_E_HIP;
    return orbgpu::debug_wave_tree(v64, out) ? ORB_E_HIP : ORB_OK;
}

int orbgpu_unit_csum(const double* v, int n, double* out) {
    if (n < 0 || (n > 0 && !v) || !out) return ORB_E_INVALID;
    int rc = 0;
    engine(&rc);
    if (rc) return rc == -4 ? ORB_E_NODEVICE : ORB_E_HIP;
    return orbgpu::debug_csum(v, n, out) ? ORB_E_HIP : ORB_OK;
}

}  // extern "C"
