// pnp.hip -- gfx950 EPnP RANSAC: PnPsolver::iterate (reference src/PnPsolver.cc:165-339) on the
// device, host only at the call's two ends.
//
// The reference loop draws a minimal set with the process rand(), solves EPnP, scores every
// correspondence and returns as soon as Refine() on the best-so-far inliers succeeds.  The draws
// do not depend on the results, so a call's hypotheses are generated up front from the caller's
// stream (inside k_pnp_hypotheses: each workgroup regenerates the glibc recurrence up to its own
// draws, ransac_dev.hpp draw_range), solved (k_pnp_hypotheses: a thread per hypothesis, EPnP in
// FP64) and scored (k_pnp_check: CheckInliers
// lane-parallel) for every solver of the batch at once.  k_pnp_replay then walks each solver's
// hypotheses in the reference's order -- best on `>`, Refine() of the best set (cached while the
// set stands), early return, the `||` loop's exhaustion branch -- and writes one record per solver
// with the stream advanced by exactly the draws consumed.  One H2D (the problem table), one D2H
// (the records).
#include "pnp.hpp"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "epnp.hpp"
#include "ransac_dev.hpp"

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
    __shared__ uint32_t win[32];
    const PnPProbDev& P = probs[blockIdx.y];
    const int h0 = blockIdx.x * 64;
    if (h0 >= P.nhyp) return;   // workgroup-uniform
    // this workgroup's minimal sets from the caller's stream (PnPsolver.cc:189-201)
    draw_range(P.rng, P.minSet, P.N, P.raw, P.hyp_idx, win, h0, min(P.nhyp, h0 + 64));
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

// The call's minimal sets from the caller's stream, a wave per solver (PnPsolver.cc:189-201).

// CheckInliers of pose (R, t) over all N correspondences by one wave: mask words + count.
__device__ __forceinline__ int check_inliers_wave(const PnPProbDev& P, const double* R, const double* t, uint32_t* mask) {
    const int lane = threadIdx.x & 63, N = P.N, words = (N + 31) >> 5;
    int n = 0;
    for (int c = 0; c * 64 < N; c++) {
        const int i = c * 64 + lane;
        bool in = false;
        if (i < N) {
            const float X = P.p3d[3 * i], Y = P.p3d[3 * i + 1], Z = P.p3d[3 * i + 2];
            const float Xc = (float)(R[0] * X + R[1] * Y + R[2] * Z + t[0]);
            const float Yc = (float)(R[3] * X + R[4] * Y + R[5] * Z + t[1]);
            const float invZc = (float)(1 / (R[6] * X + R[7] * Y + R[8] * Z + t[2]));
            const double ue = P.uc + P.fu * Xc * invZc;
            const double ve = P.vc + P.fv * Yc * invZc;
            const float distX = (float)(P.p2d[2 * i] - ue);
            const float distY = (float)(P.p2d[2 * i + 1] - ve);
            const float error2 = distX * distX + distY * distY;
            in = error2 < P.maxErr[i];
        }
        const unsigned long long b = __ballot(in);
        n += __popcll(b);
        if (lane == 0) {
            mask[2 * c] = (uint32_t)b;
            if (2 * c + 1 < words) mask[2 * c + 1] = (uint32_t)(b >> 32);
        }
    }
    return n;
}

__device__ __forceinline__ void rt_to_tcw_d(const double* rt, float* T) {
    // cv::Mat(3,3,CV_64F,mRi).convertTo(CV_32F) into eye(4) (PnPsolver.cc:217-224)
    for (int i = 0; i < 16; i++) T[i] = 0.f;
    for (int i = 0; i < 3; i++) {
        for (int j = 0; j < 3; j++) T[4 * i + j] = (float)rt[3 * i + j];
        T[4 * i + 3] = (float)rt[9 + i];
    }
    T[15] = 1.f;
}

// PnPsolver::iterate's loop (165-258) over the scored hypotheses, a wave per solver.  The
// control flow is wave-uniform (every lane reads the same counts and state); lane 0 runs the
// serial EPnP of Refine() (260-305) on the best set, the wave its CheckInliers.
__global__ void __launch_bounds__(64) k_pnp_replay(const PnPProbDev* __restrict__ probs) {
    const PnPProbDev& P = probs[blockIdx.x];
    const int lane = threadIdx.x & 63, N = P.N, words = (N + 31) >> 5;
    PnPStateDev* st = P.state;
    int nBest = st->nBest, refValid = st->refValid, refNin = st->refNin;
    int consumed = P.nhyp, success = 0;
    // The reference's loop only acts at an "event": a hypothesis with at least minInliers inliers
    // that beats the best (c > nBest), meets an invalid Refine, or meets a cached Refine that
    // succeeds -- Refine() runs for every hypothesis with >= minInliers, so when the best set of
    // a previous call refined successfully (that call returned it), the first such hypothesis of
    // this call returns it again (PnPsolver.cc:203-235).  Between events the state is constant,
    // so 64 counts at a time are tested lane-parallel and the first event of the chunk (ballot)
    // is replayed; the walk resumes right after it.  Iterations = hypotheses consumed.
    int h0 = 0;
    while (h0 < P.nhyp && !success) {
        const int h = h0 + lane;
        const int c = h < P.nhyp ? P.counts[h] : -1;
        const bool refOk = refValid && refNin > P.minInliers;
        const bool ev = h < P.nhyp && c >= P.minInliers && (c > nBest || !refValid || refOk);
        const unsigned long long evb = __ballot(ev);
        if (!evb) {
            h0 += 64;
            continue;
        }
        const int e = __ffsll((long long)evb) - 1;
        const int he = h0 + e, ce = __shfl(c, e, 64);
        if (ce > nBest) {   // mvbBestInliers = mvbInliersi; mnBestInliers; mBestTcw
            const uint32_t* m = P.masks + (size_t)he * words;
            for (int w = lane; w < words; w += 64) P.bestMask[w] = m[w];
            if (lane == 0) rt_to_tcw_d(P.rt + (size_t)he * 12, st->bestTcw);
            nBest = ce;
            refValid = 0;
        }
        if (!refValid) {   // Refine(): EPnP on the best inliers in index order, then CheckInliers
            __syncthreads();
            int n = 0;
            for (int base = 0; base < N; base += 64) {
                const int i = base + lane;
                const bool in = i < N && ((P.bestMask[i >> 5] >> (i & 31)) & 1);
                const unsigned long long b = __ballot(in);
                if (in) P.refIdx[n + __popcll(b & ((1ull << lane) - 1))] = i;
                n += __popcll(b);
            }
            __syncthreads();
            if (lane == 0) {
                IdxPts pts{P.p3d, P.p2d, P.refIdx};
                epnp::Solver<IdxPts> S(pts, n, P.fu, P.fv, P.uc, P.vc);
                double R[3][3], t[3];
                S.compute_pose(R, t);
                store_rt(st->refRt, R, t);
            }
            __syncthreads();
            double R[9], t[3];
            for (int j = 0; j < 9; j++) R[j] = st->refRt[j];
            for (int j = 0; j < 3; j++) t[j] = st->refRt[9 + j];
            refNin = check_inliers_wave(P, R, t, P.refMask);
            refValid = 1;
        }
        if (refNin > P.minInliers) {   // Refine() succeeded: return the refined pose (228-235)
            success = 1;
            consumed = he + 1;
        }
        h0 = he + 1;
    }
    const int nIt = P.nIt0 + consumed;
    __syncthreads();
    PnPOutDev* o = P.out;
    const uint32_t* src = nullptr;
    if (lane == 0) {
        o->has_pose = 0;
        o->bNoMore = 0;
        o->nInliers = 0;
        o->consumed = consumed;
        o->nIterations = nIt;
        for (int i = 0; i < 16; i++) o->Tcw[i] = 0.f;
    }
    if (success) {
        src = P.refMask;
        if (lane == 0) {
            o->has_pose = 1;
            o->nInliers = refNin;
            rt_to_tcw_d(st->refRt, o->Tcw);
        }
    } else if (nIt >= P.maxIts) {   // 241-257: the loop ran out
        if (lane == 0) o->bNoMore = 1;
        if (nBest >= P.minInliers) {
            src = P.bestMask;
            if (lane == 0) {
                o->has_pose = 1;
                o->nInliers = nBest;
                for (int i = 0; i < 16; i++) o->Tcw[i] = st->bestTcw[i];
            }
        }
    }
    for (int w = lane; w < words; w += 64) P.outMask[w] = src ? src[w] : 0u;
    rng_after(P.rng, P.raw, consumed * P.minSet, &o->rng);
    if (lane == 0) {
        st->nBest = nBest;
        st->refValid = refValid;
        st->refNin = refNin;
    }
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
    ref_stale_ = true;
}

static size_t al256(size_t v) { return (v + 255) & ~(size_t)255; }
static int mask_words(int N) { return (N + 31) >> 5; }

// device block: p3d | p2d | maxErr | PnPStateDev | best mask | Refine mask | Refine index list
size_t PnPSolver::state_off() const { return al256((size_t)N_ * 24 + 64); }

int PnPSolver::upload(hipStream_t s) {
    if (!dev_dirty_) return 0;
    const size_t so = state_off(), W = (size_t)mask_words(N_) * 4;
    const size_t bytes = so + al256(sizeof(PnPStateDev)) + 2 * al256(W) + al256((size_t)N_ * 4 + 4);
    if (bytes > d_pts_cap_) {   // first upload: a fresh state (no best set, no Refine cached)
        if (d_pts_) (void)hipFree(d_pts_);
        ORB_HIP_CHECK(hipMalloc(&d_pts_, bytes));
        d_pts_cap_ = bytes;
        ORB_HIP_CHECK(hipMemsetAsync((char*)d_pts_ + so, 0, bytes - so, s));
    } else if (ref_stale_) {   // PnPStateDev::refValid = 0 (mvMaxError changed)
        ORB_HIP_CHECK(hipMemsetAsync((char*)d_pts_ + so + offsetof(PnPStateDev, refValid), 0, 4, s));
    }
    ref_stale_ = false;
    float* d = (float*)d_pts_;
    ORB_HIP_CHECK(hipMemcpyAsync(d, p3d_.data(), (size_t)N_ * 12, hipMemcpyHostToDevice, s));
    ORB_HIP_CHECK(hipMemcpyAsync(d + 3 * N_, p2d_.data(), (size_t)N_ * 8, hipMemcpyHostToDevice, s));
    ORB_HIP_CHECK(hipMemcpyAsync(d + 5 * N_, maxErr_.data(), (size_t)N_ * 4, hipMemcpyHostToDevice, s));
    dev_dirty_ = false;
    return 0;
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

// Byte layout of one iterate() call's device work area and pinned staging.  The accounting
// (how much to allocate) and the carve (where each buffer goes) both come from here, so they
// cannot drift apart (the PnP fault of 9f527cb: an earlier accounting summed unaligned sizes
// while the carve aligned every sub-buffer; tests/test_pnp_layout.py pins the invariant).
//   device: [per solver: draws | stream words | counts | masks | (R, t)] [per solver: record]
//   pinned host: a byte-for-byte mirror of the record region (ONE copy back per call)
struct PnPLayout {
    static size_t al(size_t v) { return al256(v); }
    static int words(int N) { return mask_words(N); }
    static size_t hyp_bytes(int K, int minSet) { return al((size_t)K * minSet * 4); }
    static size_t raw_bytes(int K, int minSet) { return al((size_t)K * minSet * 4); }
    static size_t cnt_bytes(int K) { return al((size_t)K * 4); }
    static size_t mask_bytes(int K, int N) { return al((size_t)K * words(N) * 4); }
    static size_t rt_bytes(int K) { return al((size_t)K * 12 * 8); }
    static size_t scratch_bytes(int K, int N, int minSet) {
        return hyp_bytes(K, minSet) + raw_bytes(K, minSet) + cnt_bytes(K) + mask_bytes(K, N) + rt_bytes(K);
    }
    static size_t out_bytes(int N) { return al(sizeof(PnPOutDev) + (size_t)words(N) * 4); }
};

int pnp_layout_check(int n, const int* N, const int* K, const int* minSet, long long* out4) {
    using LY = PnPLayout;
    // accounting as iterate() does it
    size_t dev = 0, host = 0;
    for (int k = 0; k < n; k++) dev += LY::scratch_bytes(K[k], N[k], minSet[k]);
    const size_t out_base = dev;
    for (int k = 0; k < n; k++) host += LY::out_bytes(N[k]);
    dev += host;
    const size_t dev_cap = dev + 256, host_cap = host + 256;
    // every byte the kernels touch, carved as iterate() carves it
    size_t dend = 0, o = 0;
    for (int k = 0; k < n; k++) {
        const size_t W = (size_t)LY::words(N[k]) * 4;
        dend = std::max(dend, o + (size_t)K[k] * minSet[k] * 4);   // hyp_idx
        o += LY::hyp_bytes(K[k], minSet[k]);
        dend = std::max(dend, o + (size_t)K[k] * minSet[k] * 4);   // raw
        o += LY::raw_bytes(K[k], minSet[k]);
        dend = std::max(dend, o + (size_t)K[k] * 4);               // counts
        o += LY::cnt_bytes(K[k]);
        dend = std::max(dend, o + (size_t)K[k] * W);               // masks
        o += LY::mask_bytes(K[k], N[k]);
        dend = std::max(dend, o + (size_t)K[k] * 96);              // (R, t)
        o += LY::rt_bytes(K[k]);
    }
    size_t hend = 0, ho = 0;
    for (int k = 0; k < n; k++) {
        const size_t end = ho + sizeof(PnPOutDev) + (size_t)LY::words(N[k]) * 4;
        dend = std::max(dend, out_base + end);
        hend = std::max(hend, end);
        ho += LY::out_bytes(N[k]);
    }
    out4[0] = (long long)dev_cap;
    out4[1] = (long long)dend;
    out4[2] = (long long)host_cap;
    out4[3] = (long long)hend;
    return dend <= dev_cap && hend <= host_cap ? 0 : 1;
}

// PnPsolver::iterate for `n` solvers; solver k draws from rngs[k] (distinct streams: the C
// entry runs solvers that share a stream one after another)
int PnPBatch::iterate(int n, PnPSolver** S, int nIterations, orb_rng** rngs, PnPResult* res) {
    hipStream_t s = stream_;
    using LY = PnPLayout;
    std::vector<int> K(n, 0), act(n, 0);
    size_t dev = 0, host = 0;
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
        act[k] = 1;
        K[k] = std::max(std::max(P.maxIts_ - P.nIterations_, nIterations), 0);   // `while (it < max || cur < nIt)`
        if ((size_t)P.N_ >= (size_t)kRngMaxRange) return -1;
        dev += LY::scratch_bytes(K[k], P.N_, P.minSet_);
        host += LY::out_bytes(P.N_);
        if (int e = P.upload(s)) return e;
    }
    const size_t out_base = dev;
    dev += host;
    // the problem table is staged in the pinned block too (after the records): a pageable
    // source would make its copy a synchronous staging round trip
    const size_t probs_h = al256(host);
    if (int e = ensure(dev + 256, probs_h + sizeof(PnPProbDev) * n + 256, (size_t)n)) return e;
    char* D = (char*)d_work_;
    char* Hh = (char*)h_work_;
    PnPProbDev* pd = (PnPProbDev*)(Hh + probs_h);
    std::vector<size_t> out_off(n, 0);
    size_t o = 0, ho = 0;
    int maxK = 0, nact = 0;
    long long hyp = 0, pts = 0;
    for (int k = 0; k < n; k++) {
        PnPProbDev& q = pd[nact];
        if (!act[k]) continue;
        PnPSolver& P = *S[k];
        std::memset(&q, 0, sizeof(PnPProbDev));
        const size_t W = (size_t)mask_words(P.N_) * 4;
        char* blk = (char*)P.d_pts_;
        const float* dp = (const float*)blk;
        q.p3d = dp;
        q.p2d = dp + 3 * P.N_;
        q.maxErr = dp + 5 * P.N_;
        q.N = P.N_;
        q.fu = P.fu_; q.fv = P.fv_; q.uc = P.uc_; q.vc = P.vc_;
        q.nhyp = K[k];
        q.minSet = P.minSet_;
        q.hyp_idx = (int*)(D + o); o += LY::hyp_bytes(K[k], P.minSet_);
        q.raw = (uint32_t*)(D + o); o += LY::raw_bytes(K[k], P.minSet_);
        q.counts = (int*)(D + o); o += LY::cnt_bytes(K[k]);
        q.masks = (uint32_t*)(D + o); o += LY::mask_bytes(K[k], P.N_);
        q.rt = (double*)(D + o); o += LY::rt_bytes(K[k]);
        q.minInliers = P.minInliers_;
        q.maxIts = P.maxIts_;
        q.nIt0 = P.nIterations_;
        q.rng = *rngs[k];
        const size_t so = P.state_off();
        q.state = (PnPStateDev*)(blk + so);
        q.bestMask = (uint32_t*)(blk + so + al256(sizeof(PnPStateDev)));
        q.refMask = (uint32_t*)((char*)q.bestMask + al256(W));
        q.refIdx = (int*)((char*)q.refMask + al256(W));
        out_off[k] = ho;
        q.out = (PnPOutDev*)(D + out_base + ho);
        q.outMask = (uint32_t*)(D + out_base + ho + sizeof(PnPOutDev));
        ho += LY::out_bytes(P.N_);
        maxK = std::max(maxK, K[k]);
        hyp += K[k];
        pts += (long long)K[k] * P.N_;
        nact++;
    }
    if (nact == 0) return 0;
    ORB_HIP_CHECK(hipMemcpyAsync(d_probs_, pd, sizeof(PnPProbDev) * nact, hipMemcpyHostToDevice, s));
    const PnPProbDev* dprobs = (const PnPProbDev*)d_probs_;
    if (maxK > 0) {
        if (timing_) ORB_HIP_CHECK(hipEventRecord(ev_[0], s));
        hipLaunchKernelGGL(k_pnp_hypotheses, dim3((maxK + 63) / 64, nact), dim3(64), 0, s, dprobs);
        if (timing_) ORB_HIP_CHECK(hipEventRecord(ev_[1], s));
        hipLaunchKernelGGL(k_pnp_check, dim3((maxK + kPnPCheckHyp - 1) / kPnPCheckHyp, nact), dim3(kPnPCheckThreads), 0,
                           s, dprobs);
        if (timing_) ORB_HIP_CHECK(hipEventRecord(ev_[2], s));
        last_hyp_ = hyp;
        last_pts_ = pts;
        timed_ = timing_;
    }
    hipLaunchKernelGGL(k_pnp_replay, dim3(nact), dim3(64), 0, s, dprobs);
    ORB_HIP_CHECK(hipGetLastError());
    ORB_HIP_CHECK(hipMemcpyAsync(Hh, D + out_base, host, hipMemcpyDeviceToHost, s));
    ORB_HIP_CHECK(hipStreamSynchronize(s));
    for (int k = 0; k < n; k++) {
        if (!act[k]) continue;
        PnPSolver& P = *S[k];
        PnPResult& r = res[k];
        const PnPOutDev* od = (const PnPOutDev*)(Hh + out_off[k]);
        const uint32_t* m = (const uint32_t*)(Hh + out_off[k] + sizeof(PnPOutDev));
        P.nIterations_ = od->nIterations;
        *rngs[k] = od->rng;
        r.has_pose = od->has_pose;
        r.bNoMore = od->bNoMore;
        r.nInliers = od->nInliers;
        if (r.has_pose) {
            std::memcpy(r.Tcw, od->Tcw, sizeof(float) * 16);
            for (int i = 0; i < P.N_; i++)
                if ((m[i >> 5] >> (i & 31)) & 1) r.inliers[P.kpIdx_[i]] = 1;
        }
    }
    return 0;
}

}  // namespace orbgpu
