// pnp.hip -- gfx950 EPnP RANSAC: the device side of PnPsolver::iterate
// (reference src/PnPsolver.cc:165-339).
//
// The reference loop draws a minimal set with the process rand(), solves
// EPnP, scores every correspondence, and returns as soon as Refine() on the
// best-so-far inliers succeeds.  The draws do not depend on the results, so a
// call's hypotheses are generated up front from a snapshot of the caller's
// glibc-rand state and scored in ONE launch for every solver of the batch
// (k_pnp_hypotheses: a thread per hypothesis, EPnP in FP64 + CheckInliers over
// all N correspondences, inlier bitmask out).  The host then replays the
// sequential accept/Refine logic; each Refine it reaches is one more launch
// (k_pnp_refine), and the RNG is re-advanced by exactly the draws the
// reference would have consumed.
#include "pnp.hpp"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "epnp.hpp"

namespace orbgpu {

struct IdxPts {
    const float* p3d;
    const float* p2d;
    const int* idx;
    __device__ __forceinline__ void pw(int k, double out[3]) const {
        const int i = idx[k];
        out[0] = p3d[3 * i];
        out[1] = p3d[3 * i + 1];
        out[2] = p3d[3 * i + 2];
    }
    __device__ __forceinline__ void uv(int k, double& u, double& v) const {
        const int i = idx[k];
        u = p2d[2 * i];
        v = p2d[2 * i + 1];
    }
};

// PnPsolver::CheckInliers (308-339): float/double mix kept expression by expression.
__device__ __forceinline__ int check_inliers(const PnPProbDev& P, const double R[3][3], const double t[3], uint32_t* mask) {
    int n = 0;
    const int words = (P.N + 31) >> 5;
    for (int w = 0; w < words; w++) {
        uint32_t bits = 0;
        for (int b = 0; b < 32; b++) {
            const int i = w * 32 + b;
            if (i >= P.N) break;
            const float X = P.p3d[3 * i], Y = P.p3d[3 * i + 1], Z = P.p3d[3 * i + 2];
            const float Xc = (float)(R[0][0] * X + R[0][1] * Y + R[0][2] * Z + t[0]);
            const float Yc = (float)(R[1][0] * X + R[1][1] * Y + R[1][2] * Z + t[1]);
            const float invZc = (float)(1 / (R[2][0] * X + R[2][1] * Y + R[2][2] * Z + t[2]));
            const double ue = P.uc + P.fu * Xc * invZc;
            const double ve = P.vc + P.fv * Yc * invZc;
            const float distX = (float)(P.p2d[2 * i] - ue);
            const float distY = (float)(P.p2d[2 * i + 1] - ve);
            const float error2 = distX * distX + distY * distY;
            if (error2 < P.maxErr[i]) {
                bits |= 1u << b;
                n++;
            }
        }
        mask[w] = bits;
    }
    return n;
}

__device__ __forceinline__ void store_rt(double* out, const double R[3][3], const double t[3]) {
    for (int i = 0; i < 3; i++) {
        for (int j = 0; j < 3; j++) out[3 * i + j] = R[i][j];
        out[9 + i] = t[i];
    }
}

// Hypothesis solve (PnPsolver.cc:196-210): a thread per hypothesis runs EPnP on its minimal set
// in FP64 and stores (R, t); counts[h] = -1 flags an invalid draw (never expected).
__global__ void __launch_bounds__(64) k_pnp_hypotheses(const PnPProbDev* __restrict__ probs) {
    const PnPProbDev P = probs[blockIdx.y];
    const int h = blockIdx.x * blockDim.x + threadIdx.x;
    if (h >= P.nhyp) return;
    for (int k = 0; k < P.minSet; k++) {
        const int i = P.hyp_idx[(size_t)h * P.minSet + k];
        if (i < 0 || i >= P.N) {  // never expected: host draws from [0, N)
            P.counts[h] = -1;
            return;
        }
    }
    IdxPts pts{P.p3d, P.p2d, P.hyp_idx + (size_t)h * P.minSet};
    epnp::Solver<IdxPts> S(pts, P.minSet, P.fu, P.fv, P.uc, P.vc);
    double R[3][3], t[3];
    S.compute_pose(R, t);
    store_rt(P.rt + (size_t)h * 12, R, t);
    P.counts[h] = 0;
}

// CheckInliers (308-339) of every hypothesis, lane-parallel over correspondences: a workgroup
// per (solver, kPnPCheckHyp hypotheses), the solver's 24-B correspondences staged once in LDS
// (when they fit) and reused by every hypothesis of the block; each wave scores a hypothesis
// 64 points at a time, the inlier bits of a 64-point chunk are one ballot (two mask words) and
// the count a popcount.  Per point the same float/double expression sequence as the reference.
constexpr int kPnPCheckThreads = 256;
constexpr int kPnPCheckHyp = 16;
constexpr int kPnPStageMax = 2048;   // 48 KiB of LDS
__global__ void __launch_bounds__(kPnPCheckThreads) k_pnp_check(const PnPProbDev* __restrict__ probs) {
    const PnPProbDev& P = probs[blockIdx.y];
    const int N = P.N, nhyp = P.nhyp;
    const int h0 = blockIdx.x * kPnPCheckHyp;
    if (h0 >= nhyp) return;
    __shared__ float sX[kPnPStageMax * 3], sU[kPnPStageMax * 2], sE[kPnPStageMax];
    const bool staged = N <= kPnPStageMax;
    if (staged) {
        for (int i = threadIdx.x; i < 3 * N; i += blockDim.x) sX[i] = P.p3d[i];
        for (int i = threadIdx.x; i < 2 * N; i += blockDim.x) sU[i] = P.p2d[i];
        for (int i = threadIdx.x; i < N; i += blockDim.x) sE[i] = P.maxErr[i];
    }
    __syncthreads();
    const float* X3 = staged ? sX : P.p3d;
    const float* U2 = staged ? sU : P.p2d;
    const float* ME = staged ? sE : P.maxErr;
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, nw = blockDim.x >> 6;
    const int words = (N + 31) >> 5;
    const double uc = P.uc, vc = P.vc, fu = P.fu, fv = P.fv;
    for (int h = h0 + w; h < min(h0 + kPnPCheckHyp, nhyp); h += nw) {
        if (P.counts[h] < 0) continue;   // invalid draw
        const double* rt = P.rt + (size_t)h * 12;
        double R[9], t[3];
#pragma unroll
        for (int j = 0; j < 9; j++) R[j] = rt[j];
#pragma unroll
        for (int j = 0; j < 3; j++) t[j] = rt[9 + j];
        uint32_t* mask = P.masks + (size_t)h * words;
        int n = 0;
        for (int c = 0; c * 64 < N; c++) {
            const int i = c * 64 + lane;
            bool in = false;
            if (i < N) {
                const float X = X3[3 * i], Y = X3[3 * i + 1], Z = X3[3 * i + 2];
                const float Xc = (float)(R[0] * X + R[1] * Y + R[2] * Z + t[0]);
                const float Yc = (float)(R[3] * X + R[4] * Y + R[5] * Z + t[1]);
                const float invZc = (float)(1 / (R[6] * X + R[7] * Y + R[8] * Z + t[2]));
                const double ue = uc + fu * Xc * invZc;
                const double ve = vc + fv * Yc * invZc;
                const float distX = (float)(U2[2 * i] - ue);
                const float distY = (float)(U2[2 * i + 1] - ve);
                const float error2 = distX * distX + distY * distY;
                in = error2 < ME[i];
            }
            const unsigned long long b = __ballot(in);
            n += __popcll(b);
            if (lane == 0) {
                mask[2 * c] = (uint32_t)b;
                if (2 * c + 1 < words) mask[2 * c + 1] = (uint32_t)(b >> 32);
            }
        }
        if (lane == 0) P.counts[h] = n;
    }
}

// Refine (260-305): EPnP on the best-so-far inliers, then CheckInliers.
__global__ void __launch_bounds__(64) k_pnp_refine(const PnPProbDev* __restrict__ probs, int nprob) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= nprob) return;
    const PnPProbDev P = probs[p];
    IdxPts pts{P.p3d, P.p2d, P.ref_idx};
    epnp::Solver<IdxPts> S(pts, P.ref_n, P.fu, P.fv, P.uc, P.vc);
    double R[3][3], t[3];
    S.compute_pose(R, t);
    P.ref_out[0] = check_inliers(P, R, t, P.ref_mask);
    store_rt(P.ref_rt, R, t);
}

// ------------------------------------------------------------------- host
// glibc random_r TYPE_3 (degree 31, separation 3, 310 warm-up draws)
void rng_seed(orb_rng* g, unsigned seed) {
    if (seed == 0) seed = 1;
    int32_t word = (int32_t)seed;
    g->tbl[0] = word;
    for (int i = 1; i < 31; i++) {
        const long hi = word / 127773, lo = word % 127773;
        word = (int32_t)(16807 * lo - 2836 * hi);
        if (word < 0) word += 2147483647;
        g->tbl[i] = word;
    }
    g->f = 3;
    g->r = 0;
    for (int i = 0; i < 310; i++) (void)rng_rand(g);
}

int rng_rand(orb_rng* g) {
    const uint32_t val = (uint32_t)g->tbl[g->f] + (uint32_t)g->tbl[g->r];
    g->tbl[g->f] = (int32_t)val;
    const int result = (int)(val >> 1);
    if (++g->f >= 31) {
        g->f = 0;
        ++g->r;
    } else if (++g->r >= 31) {
        g->r = 0;
    }
    return result;
}

// DUtils::Random::RandomInt (Random.cpp:47-50)
static int random_int(orb_rng* g, int min, int max) {
    const int d = max - min + 1;
    return int(((double)rng_rand(g) / ((double)2147483647 + 1.0)) * d) + min;
}

PnPSolver::PnPSolver(int N, const float* p3d, const float* p2d, const float* sigma2, const int* kpIdx, int nMatches,
                     float fx, float fy, float cx, float cy)
    : N_(N), nMatches_(nMatches), fu_(fx), fv_(fy), uc_(cx), vc_(cy) {
    p3d_.assign(p3d, p3d + 3 * (size_t)N);
    p2d_.assign(p2d, p2d + 2 * (size_t)N);
    sigma2_.assign(sigma2, sigma2 + N);
    kpIdx_.assign(kpIdx, kpIdx + N);
    maxErr_.assign(N, 0.f);
    bestInliers_.assign(N, 0);
    set_ransac(0.99, 8, 300, 4, 0.4f, 5.991f);  // PnPsolver.h:67 defaults (ctor calls SetRansacParameters())
}

PnPSolver::~PnPSolver() {
    if (d_pts_) (void)hipFree(d_pts_);
}

// SetRansacParameters, PnPsolver.cc:121-157
void PnPSolver::set_ransac(double probability, int minInliers, int maxIterations, int minSet, float epsilon, float th2) {
    prob_ = probability;
    minInliers_ = minInliers;
    maxIts_ = maxIterations;
    epsilon_ = epsilon;
    minSet_ = minSet;
    int nMinInliers = (int)(N_ * epsilon_);
    if (nMinInliers < minInliers_) nMinInliers = minInliers_;
    if (nMinInliers < minSet) nMinInliers = minSet;
    minInliers_ = nMinInliers;
    if (epsilon_ < (float)minInliers_ / N_) epsilon_ = (float)minInliers_ / N_;
    int nIterations;
    if (minInliers_ == N_) nIterations = 1;
    else nIterations = (int)std::ceil(std::log(1 - prob_) / std::log(1 - std::pow(epsilon_, 3)));
    maxIts_ = std::max(1, std::min(nIterations, maxIts_));
    for (int i = 0; i < N_; i++) maxErr_[i] = sigma2_[i] * th2;
    dev_dirty_ = true;
}

int PnPSolver::upload(hipStream_t s) {
    if (!dev_dirty_) return 0;
    const size_t bytes = (size_t)N_ * (3 + 2 + 1) * 4 + 64;
    if (bytes > d_pts_cap_) {
        if (d_pts_) (void)hipFree(d_pts_);
        ORB_HIP_CHECK(hipMalloc(&d_pts_, bytes));
        d_pts_cap_ = bytes;
    }
    float* d = (float*)d_pts_;
    ORB_HIP_CHECK(hipMemcpyAsync(d, p3d_.data(), (size_t)N_ * 12, hipMemcpyHostToDevice, s));
    ORB_HIP_CHECK(hipMemcpyAsync(d + 3 * N_, p2d_.data(), (size_t)N_ * 8, hipMemcpyHostToDevice, s));
    ORB_HIP_CHECK(hipMemcpyAsync(d + 5 * N_, maxErr_.data(), (size_t)N_ * 4, hipMemcpyHostToDevice, s));
    dev_dirty_ = false;
    return 0;
}

static void rt_to_tcw(const double* rt, float* T) {
    // cv::Mat(3,3,CV_64F,mRi).convertTo(CV_32F) into eye(4) (PnPsolver.cc:217-224)
    for (int i = 0; i < 16; i++) T[i] = 0.f;
    for (int i = 0; i < 3; i++) {
        for (int j = 0; j < 3; j++) T[4 * i + j] = (float)rt[3 * i + j];
        T[4 * i + 3] = (float)rt[9 + i];
    }
    T[15] = 1.f;
}

PnPBatch::~PnPBatch() {
    for (auto& e : ev_)
        if (e) (void)hipEventDestroy(e);
    if (d_work_) (void)hipFree(d_work_);
    if (d_probs_) (void)hipFree(d_probs_);
    if (h_work_) (void)hipHostFree(h_work_);
    if (stream_) (void)hipStreamDestroy(stream_);
}

int PnPBatch::init() {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return -4;
    ORB_HIP_CHECK(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
    for (auto& e : ev_) ORB_HIP_CHECK(hipEventCreate(&e));
    return 0;
}

// ms of the last timed iterate()'s hypothesis launches: {solve, check}; plus the hypotheses
// and (hypothesis, point) pairs they covered
int PnPBatch::last_timings(float* ms2, long long* hyp_pts2) {
    if (!timed_) return -1;
    ORB_HIP_CHECK(hipEventSynchronize(ev_[2]));
    ORB_HIP_CHECK(hipEventElapsedTime(&ms2[0], ev_[0], ev_[1]));
    ORB_HIP_CHECK(hipEventElapsedTime(&ms2[1], ev_[1], ev_[2]));
    hyp_pts2[0] = last_hyp_;
    hyp_pts2[1] = last_pts_;
    return 0;
}

int PnPBatch::ensure(size_t dev_bytes, size_t host_bytes, size_t probs) {
    if (dev_bytes > work_cap_) {
        if (d_work_) (void)hipFree(d_work_);
        ORB_HIP_CHECK(hipMalloc(&d_work_, dev_bytes));
        work_cap_ = dev_bytes;
    }
    if (host_bytes > hwork_cap_) {
        if (h_work_) (void)hipHostFree(h_work_);
        ORB_HIP_CHECK(hipHostMalloc(&h_work_, host_bytes));
        hwork_cap_ = host_bytes;
    }
    if (probs * sizeof(PnPProbDev) > probs_cap_) {
        if (d_probs_) (void)hipFree(d_probs_);
        ORB_HIP_CHECK(hipMalloc(&d_probs_, probs * sizeof(PnPProbDev)));
        probs_cap_ = probs * sizeof(PnPProbDev);
    }
    return 0;
}

// PnPsolver::iterate for `n` solvers; solver k draws from rngs[k] (may alias).
// Byte layout of one iterate() call's device work area and pinned staging.  The accounting
// (how much to allocate) and the carve (where each buffer goes) both come from here, so they
// cannot drift apart: an earlier version summed unaligned sizes for the Refine scratch while
// the carve aligned each sub-buffer, and the last solvers' Refine buffers ran past the work
// area (the PnP fault of 9f527cb; tests/test_pnp_layout.py pins the invariant).
//   device: [draws of every solver | (masks, counts, (R, t)) of every solver | Refine slots]
//   pinned host: a byte-for-byte mirror of the first two regions, so the draws go up in one
//   copy and the results come back in one copy for any number of solvers.
struct PnPLayout {
    static size_t al(size_t v) { return (v + 255) & ~(size_t)255; }
    static int words(int N) { return (N + 31) >> 5; }
    static size_t hyp_bytes(int K, int minSet) { return al((size_t)K * minSet * 4); }
    static size_t mask_bytes(int K, int N) { return al((size_t)K * words(N) * 4); }
    static size_t cnt_bytes(int K) { return al((size_t)K * 4); }
    static size_t rt_bytes(int K) { return al((size_t)K * 12 * 8); }
    static size_t res_bytes(int K, int N) { return mask_bytes(K, N) + cnt_bytes(K) + rt_bytes(K); }
    // Refine slot of a solver: inlier idx list | mask | (R, t) | inlier count
    static size_t ref_mask_off(int N) { return al((size_t)N * 4); }
    static size_t ref_rt_off(int N) { return ref_mask_off(N) + al((size_t)words(N) * 4); }
    static size_t ref_out_off(int N) { return ref_rt_off(N) + 96; }
    static size_t ref_slot(int N) { return al(ref_out_off(N) + 4); }
};

int pnp_layout_check(int n, const int* N, const int* K, const int* minSet, long long* out4) {
    // accounting as iterate() does it
    size_t dev = 0;
    for (int k = 0; k < n; k++) dev += PnPLayout::hyp_bytes(K[k], minSet[k]) + PnPLayout::res_bytes(K[k], N[k]);
    const size_t mirror = dev;
    for (int k = 0; k < n; k++) dev += PnPLayout::ref_slot(N[k]);
    const size_t dev_cap = dev + 256, host_cap = mirror + 256;
    // every byte the carve touches: the draw region, the result region (kernels write masks,
    // counts and K * 96 B of poses), every solver's Refine slot at once; the host mirror
    size_t dend = 0, o = 0;
    for (int k = 0; k < n; k++) {
        dend = std::max(dend, o + (size_t)K[k] * minSet[k] * 4);
        o += PnPLayout::hyp_bytes(K[k], minSet[k]);
    }
    for (int k = 0; k < n; k++) {
        dend = std::max(dend, o + (size_t)K[k] * PnPLayout::words(N[k]) * 4);
        o += PnPLayout::mask_bytes(K[k], N[k]);
        dend = std::max(dend, o + (size_t)K[k] * 4);
        o += PnPLayout::cnt_bytes(K[k]);
        dend = std::max(dend, o + (size_t)K[k] * 96);
        o += PnPLayout::rt_bytes(K[k]);
    }
    const size_t hend = o;
    size_t ro = o;
    for (int k = 0; k < n; k++) {
        dend = std::max(dend, ro + PnPLayout::ref_out_off(N[k]) + 4);
        dend = std::max(dend, ro + (size_t)N[k] * 4);
        ro += PnPLayout::ref_slot(N[k]);
    }
    out4[0] = (long long)dev_cap;
    out4[1] = (long long)dend;
    out4[2] = (long long)host_cap;
    out4[3] = (long long)hend;
    return dend <= dev_cap && hend <= host_cap ? 0 : 1;
}

int PnPBatch::iterate(int n, PnPSolver** S, int nIterations, orb_rng** rngs, PnPResult* res) {
    hipStream_t s = stream_;
    struct Job {
        int K = 0;            // hypotheses generated for this call
        orb_rng snap;         // RNG state before the call
        size_t hyp_off = 0, mask_off = 0, cnt_off = 0, rt_off = 0;
        bool active = false;
        int next = 0;         // next hypothesis to replay
    };
    std::vector<Job> jobs(n);
    size_t dev = 0;
    using LY = PnPLayout;
    for (int k = 0; k < n; k++) {
        PnPSolver& P = *S[k];
        PnPResult& r = res[k];
        r.has_pose = 0;
        r.bNoMore = 0;
        r.nInliers = 0;
        if (r.inliers) std::fill(r.inliers, r.inliers + P.nMatches_, 0);  // vbInliers.clear()
        if (P.N_ < P.minInliers_) {  // 176-180
            r.bNoMore = 1;
            continue;
        }
        Job& J = jobs[k];
        J.K = std::max(P.maxIts_ - P.nIterations_, nIterations);  // `while (it < max || cur < nIt)`
        if (J.K <= 0) J.K = 0;
        J.active = J.K > 0;
        J.snap = *rngs[k];
        J.hyp_off = dev; dev += LY::hyp_bytes(J.K, P.minSet_);
        if (int e = P.upload(s)) return e;
    }
    const size_t res_base = dev;
    for (int k = 0; k < n; k++) {
        Job& J = jobs[k];
        const int N = S[k]->N_;
        J.mask_off = dev; dev += LY::mask_bytes(J.K, N);
        J.cnt_off = dev; dev += LY::cnt_bytes(J.K);
        J.rt_off = dev; dev += LY::rt_bytes(J.K);
    }
    // refine scratch (per solver): idx list N + mask + rt + count
    const size_t ref_base = dev;
    for (int k = 0; k < n; k++) dev += LY::ref_slot(S[k]->N_);
    if (int e = ensure(dev + 256, ref_base + 256, (size_t)n)) return e;
    char* D = (char*)d_work_;
    char* Hh = (char*)h_work_;
    // 1. generate all hypotheses (draws as the reference would make them), straight into the
    //    pinned mirror of the draw region
    std::vector<PnPProbDev> pd(n);
    int maxK = 0;
    for (int k = 0; k < n; k++) {
        Job& J = jobs[k];
        PnPSolver& P = *S[k];
        std::memset(&pd[k], 0, sizeof(PnPProbDev));
        if (!J.active) continue;
        orb_rng g = J.snap;
        int* hyp = (int*)(Hh + J.hyp_off);
        // vAvailableIndices = mvAllIndices per iteration (PnPsolver.cc:196-203): the draw writes
        // minSet slots, undone after each hypothesis instead of re-filling all N
        std::vector<int> avail(P.N_), pos(P.minSet_), old(P.minSet_);
        for (int i = 0; i < P.N_; i++) avail[i] = i;
        for (int h = 0; h < J.K; h++) {
            int navail = P.N_;
            for (int i = 0; i < P.minSet_; ++i) {
                const int randi = random_int(&g, 0, navail - 1);
                hyp[(size_t)h * P.minSet_ + i] = avail[randi];
                pos[i] = randi;
                old[i] = avail[randi];
                avail[randi] = avail[navail - 1];
                navail--;
            }
            for (int i = P.minSet_ - 1; i >= 0; --i) avail[pos[i]] = old[i];
        }
        const float* dp = (const float*)P.d_pts_;
        PnPProbDev& q = pd[k];
        q.p3d = dp;
        q.p2d = dp + 3 * P.N_;
        q.maxErr = dp + 5 * P.N_;
        q.N = P.N_;
        q.fu = P.fu_; q.fv = P.fv_; q.uc = P.uc_; q.vc = P.vc_;
        q.hyp_idx = (const int*)(D + J.hyp_off);
        q.nhyp = J.K;
        q.minSet = P.minSet_;
        q.counts = (int*)(D + J.cnt_off);
        q.masks = (uint32_t*)(D + J.mask_off);
        q.rt = (double*)(D + J.rt_off);
        maxK = std::max(maxK, J.K);
    }
    if (getenv("ORBGPU_CHECK_PTRS")) {
        auto in = [](const void* p, size_t bytes) {
            void* base = nullptr;
            size_t size = 0;
            if (hipMemGetAddressRange((hipDeviceptr_t*)&base, &size, (hipDeviceptr_t)p) != hipSuccess) return false;
            return (const char*)p >= (const char*)base && (const char*)p + bytes <= (const char*)base + size;
        };
        for (int k = 0; k < n; k++) {
            const PnPProbDev& q = pd[k];
            if (!jobs[k].active) continue;
            const int words = (q.N + 31) >> 5;
            const bool ok = in(q.p3d, q.N * 12) && in(q.p2d, q.N * 8) && in(q.maxErr, q.N * 4) &&
                            in(q.hyp_idx, (size_t)q.nhyp * q.minSet * 4) && in(q.counts, (size_t)q.nhyp * 4) &&
                            in(q.masks, (size_t)q.nhyp * words * 4) && in(q.rt, (size_t)q.nhyp * 96) &&
                            in(d_probs_, sizeof(PnPProbDev) * n);
            fprintf(stderr, "[pnp] k=%d N=%d nhyp=%d minSet=%d ptrs %s p3d=%p hyp=%p work=%p cap=%zu\n", k, q.N, q.nhyp,
                    q.minSet, ok ? "ok" : "BAD", (const void*)q.p3d, (const void*)q.hyp_idx, d_work_, work_cap_);
            if (!ok) return -1;
        }
    }
    if (res_base > 0) ORB_HIP_CHECK(hipMemcpyAsync(D, Hh, res_base, hipMemcpyHostToDevice, s));
    ORB_HIP_CHECK(hipMemcpyAsync(d_probs_, pd.data(), sizeof(PnPProbDev) * n, hipMemcpyHostToDevice, s));
    if (maxK > 0) {
        if (timing_) ORB_HIP_CHECK(hipEventRecord(ev_[0], s));
        hipLaunchKernelGGL(k_pnp_hypotheses, dim3((maxK + 63) / 64, n), dim3(64), 0, s, (const PnPProbDev*)d_probs_);
        if (timing_) ORB_HIP_CHECK(hipEventRecord(ev_[1], s));
        hipLaunchKernelGGL(k_pnp_check, dim3((maxK + kPnPCheckHyp - 1) / kPnPCheckHyp, n), dim3(kPnPCheckThreads), 0, s,
                           (const PnPProbDev*)d_probs_);
        if (timing_) ORB_HIP_CHECK(hipEventRecord(ev_[2], s));
        last_hyp_ = 0;
        for (int k = 0; k < n; k++) last_hyp_ += jobs[k].active ? jobs[k].K : 0;
        last_pts_ = 0;
        for (int k = 0; k < n; k++) last_pts_ += jobs[k].active ? (long long)jobs[k].K * S[k]->N_ : 0;
        timed_ = timing_;
    }
    ORB_HIP_CHECK(hipGetLastError());
    // 2. results back (counts, masks, poses of every solver) in one copy
    if (ref_base > res_base)
        ORB_HIP_CHECK(hipMemcpyAsync(Hh + res_base, D + res_base, ref_base - res_base, hipMemcpyDeviceToHost, s));
    ORB_HIP_CHECK(hipStreamSynchronize(s));
    // 3. sequential replay; Refine requests batched across solvers
    std::vector<char> done(n, 0);
    std::vector<int> ref_n(n, 0);
    for (int k = 0; k < n; k++) done[k] = !jobs[k].active;
    for (;;) {
        std::vector<int> need;  // solvers waiting for a Refine
        for (int k = 0; k < n; k++) {
            if (done[k]) continue;
            Job& J = jobs[k];
            PnPSolver& P = *S[k];
            const int words = (P.N_ + 31) >> 5;
            const int* cnt = (const int*)(Hh + J.cnt_off);
            const uint32_t* masks = (const uint32_t*)(Hh + J.mask_off);
            const double* rts = (const double*)(Hh + J.rt_off);
            bool wait = false;
            while (J.next < J.K) {
                const int h = J.next;
                if (P.refine_pending_ < 0) {  // iteration h not yet counted
                    P.nIterations_++;
                    const int c = cnt[h];
                    if (c >= P.minInliers_) {
                        if (c > P.nBestInliers_) {
                            for (int i = 0; i < P.N_; i++)
                                P.bestInliers_[i] = (masks[(size_t)h * words + (i >> 5)] >> (i & 31)) & 1;
                            P.nBestInliers_ = c;
                            rt_to_tcw(rts + (size_t)h * 12, P.bestTcw_);
                            P.refine_valid_ = false;
                        }
                        P.refine_pending_ = h;
                        if (!P.refine_valid_) {  // Refine(best) not computed for this best set yet
                            wait = true;
                            break;
                        }
                    } else {
                        J.next++;
                        continue;
                    }
                }
                // Refine result for the current best set is available
                P.refine_pending_ = -1;
                if (P.refNin_ > P.minInliers_) {
                    PnPResult& r = res[k];
                    r.has_pose = 1;
                    r.nInliers = P.refNin_;
                    std::fill(r.inliers, r.inliers + P.nMatches_, 0);
                    for (int i = 0; i < P.N_; i++)
                        if (P.refMask_[i >> 5] >> (i & 31) & 1) r.inliers[P.kpIdx_[i]] = 1;
                    rt_to_tcw(P.refRt_, r.Tcw);
                    // consumed draws: hypotheses 0..h
                    *rngs[k] = J.snap;
                    for (int d = 0; d < (h + 1) * P.minSet_; d++) (void)rng_rand(rngs[k]);
                    done[k] = 1;
                    break;
                }
                J.next++;
            }
            if (done[k]) continue;
            if (wait) {
                need.push_back(k);
                continue;
            }
            // loop exhausted (PnPsolver.cc:241-257)
            *rngs[k] = J.snap;
            for (int d = 0; d < J.K * P.minSet_; d++) (void)rng_rand(rngs[k]);
            PnPResult& r = res[k];
            if (P.nIterations_ >= P.maxIts_) {
                r.bNoMore = 1;
                if (P.nBestInliers_ >= P.minInliers_) {
                    r.has_pose = 1;
                    r.nInliers = P.nBestInliers_;
                    std::fill(r.inliers, r.inliers + P.nMatches_, 0);
                    for (int i = 0; i < P.N_; i++)
                        if (P.bestInliers_[i]) r.inliers[P.kpIdx_[i]] = 1;
                    std::memcpy(r.Tcw, P.bestTcw_, sizeof(float) * 16);
                }
            }
            done[k] = 1;
        }
        if (need.empty()) break;
        // Refine launch for every waiting solver
        std::vector<PnPProbDev> rq(need.size());
        size_t ro = ref_base;
        std::vector<size_t> roff(need.size());
        for (size_t q = 0; q < need.size(); q++) {
            PnPSolver& P = *S[need[q]];
            std::vector<int> idx;
            for (int i = 0; i < P.N_; i++)
                if (P.bestInliers_[i]) idx.push_back(i);
            roff[q] = ro;
            ORB_HIP_CHECK(hipMemcpyAsync(D + ro, idx.data(), idx.size() * 4, hipMemcpyHostToDevice, s));
            PnPProbDev r = pd[need[q]];
            r.ref_idx = (const int*)(D + ro);
            r.ref_n = (int)idx.size();
            r.ref_mask = (uint32_t*)(D + ro + LY::ref_mask_off(P.N_));
            r.ref_rt = (double*)(D + ro + LY::ref_rt_off(P.N_));
            r.ref_out = (int*)(D + ro + LY::ref_out_off(P.N_));
            rq[q] = r;
            ro += LY::ref_slot(P.N_);
        }
        ORB_HIP_CHECK(hipMemcpyAsync(d_probs_, rq.data(), sizeof(PnPProbDev) * rq.size(), hipMemcpyHostToDevice, s));
        hipLaunchKernelGGL(k_pnp_refine, dim3((unsigned)(need.size() + 63) / 64), dim3(64), 0, s,
                           (const PnPProbDev*)d_probs_, (int)need.size());
        ORB_HIP_CHECK(hipGetLastError());
        for (size_t q = 0; q < need.size(); q++) {
            PnPSolver& P = *S[need[q]];
            const int words = (P.N_ + 31) >> 5;
            P.refMask_.resize(words);
            ORB_HIP_CHECK(hipMemcpyAsync(P.refMask_.data(), rq[q].ref_mask, (size_t)words * 4, hipMemcpyDeviceToHost, s));
            ORB_HIP_CHECK(hipMemcpyAsync(P.refRt_, rq[q].ref_rt, 96, hipMemcpyDeviceToHost, s));
            ORB_HIP_CHECK(hipMemcpyAsync(&P.refNin_, rq[q].ref_out, 4, hipMemcpyDeviceToHost, s));
        }
        ORB_HIP_CHECK(hipStreamSynchronize(s));
        for (int k : need) S[k]->refine_valid_ = true;
    }
    return 0;
}

}  // namespace orbgpu
