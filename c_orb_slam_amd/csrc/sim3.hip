// sim3.hip -- gfx950 Sim3 RANSAC: the device side of Sim3Solver::iterate
// (reference src/Sim3Solver.cc:140-403).
//
// Each hypothesis (3 pairs drawn with rand(), Sim3Solver.cc:165-177) runs
// Horn's closed form (centroids, M, N, Jacobi eigenvector of the 4x4 N,
// angle-axis, Rodrigues, scale, t, T12/T21) and the bidirectional reprojection
// test over all N pairs in one thread; every hypothesis of every solver of the
// batch is one launch.  The draws do not depend on results, so the host
// replays the `>=` best update and the `> minInliers` early return and
// advances the RNG by exactly 3 draws per consumed iteration.
#include "sim3.hpp"
#include "ransac_dev.hpp"

#include <algorithm>
#include <cmath>
#include <cstring>

#include "detmath.hpp"

namespace orbgpu {

// cv::eigen for a symmetric 4x4 CV_32F matrix: OpenCV 3.2 JacobiImpl_<float> (hypot as sqrtf).
__device__ __forceinline__ void jacobi_eigen4(float* A, float* W, float* V) {
    const int n = 4;
    const float eps = 1.1920928955078125e-07f;
    int i, j, k, m;
    int indR[4], indC[4];
    float mv = 0;
    for (i = 0; i < n; i++) {
        for (j = 0; j < n; j++) V[i * n + j] = 0;
        V[i * n + i] = 1;
    }
    for (k = 0; k < n; k++) {
        W[k] = A[(n + 1) * k];
        if (k < n - 1) {
            for (m = k + 1, mv = fabsf(A[n * k + m]), i = k + 2; i < n; i++) {
                const float val = fabsf(A[n * k + i]);
                if (mv < val) mv = val, m = i;
            }
            indR[k] = m;
        }
        if (k > 0) {
            for (m = 0, mv = fabsf(A[k]), i = 1; i < k; i++) {
                const float val = fabsf(A[n * i + k]);
                if (mv < val) mv = val, m = i;
            }
            indC[k] = m;
        }
    }
    for (int iters = 0; iters < n * n * 30; iters++) {
        for (k = 0, mv = fabsf(A[indR[0]]), i = 1; i < n - 1; i++) {
            const float val = fabsf(A[n * i + indR[i]]);
            if (mv < val) mv = val, k = i;
        }
        int l = indR[k];
        for (i = 1; i < n; i++) {
            const float val = fabsf(A[n * indC[i] + i]);
            if (mv < val) mv = val, k = indC[i], l = i;
        }
        const float p = A[n * k + l];
        if (fabsf(p) <= eps) break;
        const float y = (float)((W[l] - W[k]) * 0.5);
        float t = fabsf(y) + sqrtf(p * p + y * y);
        float s = sqrtf(p * p + t * t);
        const float c = t / s;
        s = p / s;
        t = (p / t) * p;
        if (y < 0) s = -s, t = -t;
        A[n * k + l] = 0;
        W[k] -= t;
        W[l] += t;
        float a0, b0;
#define ROT(v0, v1) a0 = v0, b0 = v1, v0 = a0 * c - b0 * s, v1 = a0 * s + b0 * c
        for (i = 0; i < k; i++) ROT(A[n * i + k], A[n * i + l]);
        for (i = k + 1; i < l; i++) ROT(A[n * k + i], A[n * i + l]);
        for (i = l + 1; i < n; i++) ROT(A[n * k + i], A[n * l + i]);
        for (i = 0; i < n; i++) ROT(V[n * k + i], V[n * l + i]);
#undef ROT
        for (j = 0; j < 2; j++) {
            const int idx = j == 0 ? k : l;
            if (idx < n - 1) {
                for (m = idx + 1, mv = fabsf(A[n * idx + m]), i = idx + 2; i < n; i++) {
                    const float val = fabsf(A[n * idx + i]);
                    if (mv < val) mv = val, m = i;
                }
                indR[idx] = m;
            }
            if (idx > 0) {
                for (m = 0, mv = fabsf(A[idx]), i = 1; i < idx; i++) {
                    const float val = fabsf(A[n * i + idx]);
                    if (mv < val) mv = val, m = i;
                }
                indC[idx] = m;
            }
        }
    }
    for (k = 0; k < n - 1; k++) {
        m = k;
        for (i = k + 1; i < n; i++)
            if (W[m] < W[i]) m = i;
        if (k != m) {
            const float tw = W[m]; W[m] = W[k]; W[k] = tw;
            for (i = 0; i < n; i++) { const float tv = V[n * m + i]; V[n * m + i] = V[n * k + i]; V[n * k + i] = tv; }
        }
    }
}

// mT21i = [sR^-1 | -sR^-1 t] (Sim3Solver.cc:323-335); shared by the solve and the check kernel
__device__ __forceinline__ void sim3_T21(const float* R, const float* t, float s, float* T21) {
    float sRinv[9];
    const double is = 1.0 / s;
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
            sRinv[3 * i + j] = (float)(is * (double)R[3 * j + i]);
            T21[4 * i + j] = sRinv[3 * i + j];
        }
    for (int i = 0; i < 3; i++) {
        const double v = (double)sRinv[3 * i] * t[0] + (double)sRinv[3 * i + 1] * t[1] + (double)sRinv[3 * i + 2] * t[2];
        T21[4 * i + 3] = (float)(-v);
    }
    T21[12] = T21[13] = T21[14] = 0.f;
    T21[15] = 1.f;
}

// ComputeSim3 (226-337); P1/P2 [row][col], column i = point i.  est: R9 t3 s T12[16] T21[16]
__device__ __forceinline__ void compute_sim3(const float P1[3][3], const float P2[3][3], int bFixScale, float* R,
                                             float* t, float* s_out, float* T12, float* T21) {
    float O1[3], O2[3], Pr1[3][3], Pr2[3][3];
    for (int r = 0; r < 3; r++) {
        O1[r] = (P1[r][0] + P1[r][1]) + P1[r][2];
        O2[r] = (P2[r][0] + P2[r][1]) + P2[r][2];
        O1[r] = O1[r] * (float)(1.0 / 3);
        O2[r] = O2[r] * (float)(1.0 / 3);
        for (int c = 0; c < 3; c++) {
            Pr1[r][c] = P1[r][c] - O1[r];
            Pr2[r][c] = P2[r][c] - O2[r];
        }
    }
    float M[3][3];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++)
            M[i][j] = (float)((double)Pr2[i][0] * Pr1[j][0] + (double)Pr2[i][1] * Pr1[j][1] + (double)Pr2[i][2] * Pr1[j][2]);
    const double N11 = M[0][0] + M[1][1] + M[2][2];
    const double N12 = M[1][2] - M[2][1];
    const double N13 = M[2][0] - M[0][2];
    const double N14 = M[0][1] - M[1][0];
    const double N22 = M[0][0] - M[1][1] - M[2][2];
    const double N23 = M[0][1] + M[1][0];
    const double N24 = M[2][0] + M[0][2];
    const double N33 = -M[0][0] + M[1][1] - M[2][2];
    const double N34 = M[1][2] + M[2][1];
    const double N44 = -M[0][0] - M[1][1] + M[2][2];
    float N[16] = {(float)N11, (float)N12, (float)N13, (float)N14, (float)N12, (float)N22, (float)N23, (float)N24,
                   (float)N13, (float)N23, (float)N33, (float)N34, (float)N14, (float)N24, (float)N34, (float)N44};
    float eval[4], evec[16];
    jacobi_eigen4(N, eval, evec);
    float vec[3] = {evec[1], evec[2], evec[3]};
    const double nv = sqrt((double)vec[0] * vec[0] + (double)vec[1] * vec[1] + (double)vec[2] * vec[2]);
    const double ang = detmath::atan2_d(nv, evec[0]);
    const double f = 2 * ang / nv;
    for (int i = 0; i < 3; i++) vec[i] = (float)(vec[i] * f);
    {  // cv::Rodrigues
        double rx = vec[0], ry = vec[1], rz = vec[2];
        const double theta = sqrt(rx * rx + ry * ry + rz * rz);
        if (theta < 2.220446049250313e-16) {
            for (int i = 0; i < 9; i++) R[i] = (i % 4 == 0) ? 1.f : 0.f;
        } else {
            double sn, cs;
            detmath::sincos_d(theta, &sn, &cs);
            const double c1 = 1. - cs;
            const double itheta = theta ? 1. / theta : 0.;
            rx *= itheta; ry *= itheta; rz *= itheta;
            const double rrt[9] = {rx * rx, rx * ry, rx * rz, rx * ry, ry * ry, ry * rz, rx * rz, ry * rz, rz * rz};
            const double r_x[9] = {0, -rz, ry, rz, 0, -rx, -ry, rx, 0};
            for (int i = 0; i < 9; i++) R[i] = (float)(cs * ((i % 4 == 0) ? 1.0 : 0.0) + c1 * rrt[i] + sn * r_x[i]);
        }
    }
    float P3[3][3];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++)
            P3[i][j] = (float)((double)R[3 * i] * Pr2[0][j] + (double)R[3 * i + 1] * Pr2[1][j] + (double)R[3 * i + 2] * Pr2[2][j]);
    float s;
    if (!bFixScale) {
        double nom = 0, den = 0;
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) {
                nom += (double)Pr1[i][j] * P3[i][j];
                den += (float)(P3[i][j] * P3[i][j]);
            }
        s = (float)(nom / den);
    } else {
        s = 1.0f;
    }
    *s_out = s;
    for (int i = 0; i < 3; i++) {
        const double rO2 = (double)R[3 * i] * O2[0] + (double)R[3 * i + 1] * O2[1] + (double)R[3 * i + 2] * O2[2];
        t[i] = O1[i] - (float)(s * rO2);
    }
    for (int i = 0; i < 16; i++) T12[i] = T21[i] = 0.f;
    T12[15] = T21[15] = 1.f;
    for (int i = 0; i < 3; i++) {
        for (int j = 0; j < 3; j++) T12[4 * i + j] = (float)(s * (double)R[3 * i + j]);
        T12[4 * i + 3] = t[i];
    }
    sim3_T21(R, t, s, T21);
}

__device__ __forceinline__ void project(const float* X, const float* T, const float* K, float* uv) {
    float p[3];
    for (int r = 0; r < 3; r++)
        p[r] = (float)((double)T[4 * r] * X[0] + (double)T[4 * r + 1] * X[1] + (double)T[4 * r + 2] * X[2] + (double)T[4 * r + 3]);
    const float invz = 1 / p[2];
    const float x = p[0] * invz, y = p[1] * invz;
    uv[0] = K[0] * x + K[2];
    uv[1] = K[1] * y + K[3];
}

__global__ void __launch_bounds__(64) k_sim3_hypotheses(const Sim3ProbDev* __restrict__ probs) {
    __shared__ uint32_t win[32];
    const Sim3ProbDev& P = probs[blockIdx.y];
    const int h0 = blockIdx.x * 64;
    if (h0 >= P.nhyp) return;   // workgroup-uniform
    // this workgroup's minimal sets from the caller's stream (Sim3Solver.cc:166-178)
    draw_range(P.rng, 3, P.N, P.raw, P.hyp_idx, win, h0, min(P.nhyp, h0 + 64));
    const int h = blockIdx.x * blockDim.x + threadIdx.x;
    if (h >= P.nhyp) return;
    float P1[3][3], P2[3][3];
    for (int i = 0; i < 3; i++) {
        const int idx = P.hyp_idx[3 * h + i];
        for (int r = 0; r < 3; r++) {
            P1[r][i] = P.X1[3 * idx + r];
            P2[r][i] = P.X2[3 * idx + r];
        }
    }
    float R[9], t[3], s, T12[16], T21[16];
    compute_sim3(P1, P2, P.bFixScale, R, t, &s, T12, T21);
    float* e = P.est + (size_t)h * 32;
    for (int i = 0; i < 9; i++) e[i] = R[i];
    for (int i = 0; i < 3; i++) e[9 + i] = t[i];
    e[12] = s;
    for (int i = 0; i < 16; i++) e[16 + i] = T12[i];
}

// CheckInliers (340-364) lane-parallel over the matched pairs: a workgroup per (solver,
// kSim3CheckHyp hypotheses), the solver's 48-B pairs staged once in LDS when they fit, a wave
// per hypothesis, one ballot per 64 pairs.  T21 is re-derived from the stored (R, t, s) by the
// same sim3_T21 the solve used.
constexpr int kSim3CheckThreads = 256;
constexpr int kSim3CheckHyp = 16;
constexpr int kSim3StageMax = 1024;   // 48 KiB of LDS
__global__ void __launch_bounds__(kSim3CheckThreads) k_sim3_check(const Sim3ProbDev* __restrict__ probs) {
    const Sim3ProbDev& P = probs[blockIdx.y];
    const int N = P.N, nhyp = P.nhyp;
    const int h0 = blockIdx.x * kSim3CheckHyp;
    if (h0 >= nhyp) return;
    __shared__ float sX1[kSim3StageMax * 3], sX2[kSim3StageMax * 3], sp1[kSim3StageMax * 2],
        sp2[kSim3StageMax * 2], sE1[kSim3StageMax], sE2[kSim3StageMax];
    const bool staged = N <= kSim3StageMax;
    if (staged) {
        for (int i = threadIdx.x; i < 3 * N; i += blockDim.x) {
            sX1[i] = P.X1[i];
            sX2[i] = P.X2[i];
        }
        for (int i = threadIdx.x; i < 2 * N; i += blockDim.x) {
            sp1[i] = P.p1[i];
            sp2[i] = P.p2[i];
        }
        for (int i = threadIdx.x; i < N; i += blockDim.x) {
            sE1[i] = P.maxErr1[i];
            sE2[i] = P.maxErr2[i];
        }
    }
    __syncthreads();
    const float* X1 = staged ? sX1 : P.X1;
    const float* X2 = staged ? sX2 : P.X2;
    const float* p1 = staged ? sp1 : P.p1;
    const float* p2 = staged ? sp2 : P.p2;
    const float* E1 = staged ? sE1 : P.maxErr1;
    const float* E2 = staged ? sE2 : P.maxErr2;
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, nw = blockDim.x >> 6;
    const int words = (N + 31) >> 5;
    for (int h = h0 + w; h < min(h0 + kSim3CheckHyp, nhyp); h += nw) {
        const float* e = P.est + (size_t)h * 32;
        float R[9], t[3], T12[16], T21[16];
        for (int i = 0; i < 9; i++) R[i] = e[i];
        for (int i = 0; i < 3; i++) t[i] = e[9 + i];
        const float s = e[12];
        for (int i = 0; i < 16; i++) T12[i] = e[16 + i];
        sim3_T21(R, t, s, T21);
        uint32_t* mask = P.masks + (size_t)h * words;
        int n = 0;
        for (int c = 0; c * 64 < N; c++) {
            const int i = c * 64 + lane;
            bool in = false;
            if (i < N) {
                float p2im1[2], p1im2[2];
                project(X2 + 3 * i, T12, P.K1, p2im1);
                project(X1 + 3 * i, T21, P.K2, p1im2);
                const float d1x = p1[2 * i] - p2im1[0], d1y = p1[2 * i + 1] - p2im1[1];
                const float d2x = p1im2[0] - p2[2 * i], d2y = p1im2[1] - p2[2 * i + 1];
                const float err1 = (float)((double)d1x * d1x + (double)d1y * d1y);
                const float err2 = (float)((double)d2x * d2x + (double)d2y * d2y);
                in = err1 < E1[i] && err2 < E2[i];
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


// Sim3Solver::iterate's loop (158-206) over the scored hypotheses, a wave per solver: best on
// `>=`, return the CURRENT hypothesis as soon as it has more than mRansacMinInliers inliers.
// (mvbBestInliers is written by the reference and never read: not kept.)
__global__ void __launch_bounds__(64) k_sim3_replay(const Sim3ProbDev* __restrict__ probs) {
    const Sim3ProbDev& P = probs[blockIdx.x];
    const int lane = threadIdx.x & 63, words = (P.N + 31) >> 5;
    Sim3StateDev* st = P.state;
    int nBest = st->nBest, best = -1, consumed = P.nhyp, success = 0;
    // 64 hypotheses per step: the best before hypothesis h is the running maximum of the counts
    // (nBest takes c whenever c >= nBest), i.e. an exclusive prefix max over the chunk carried
    // across chunks; the walk stops at the first update with more than minInliers (ballot), else
    // the chunk's last update is the best so far.
    for (int base = 0; base < P.nhyp && !success; base += 64) {
        const int h = base + lane;
        const int c = h < P.nhyp ? P.counts[h] : INT_MIN;
        int inc = c;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int t = __shfl_up(inc, o, 64);
            if (lane >= o) inc = max(inc, t);
        }
        int exc = __shfl_up(inc, 1, 64);
        if (lane == 0) exc = INT_MIN;
        const bool upd = h < P.nhyp && c >= max(nBest, exc);
        const unsigned long long ex = __ballot(upd && c > P.minInliers), up = __ballot(upd);
        if (ex) {
            const int e = __ffsll((long long)ex) - 1;
            best = base + e;
            nBest = __shfl(c, e, 64);
            success = 1;
            consumed = best + 1;
        } else {
            if (up) best = base + 63 - __clzll((long long)up);
            nBest = max(nBest, __shfl(inc, 63, 64));
        }
    }
    const int nIt = P.nIt0 + consumed;
    Sim3OutDev* o = P.out;
    if (lane == 0) {
        if (best >= 0) {
            const float* e = P.est + (size_t)best * 32;
            for (int i = 0; i < 9; i++) st->bestR[i] = e[i];
            for (int i = 0; i < 3; i++) st->bestT[i] = e[9 + i];
            st->bestS = e[12];
            for (int i = 0; i < 16; i++) st->bestT12[i] = e[16 + i];
        }
        st->nBest = nBest;
        o->has_pose = success;
        o->nInliers = success ? nBest : 0;
        o->bNoMore = !success && nIt >= P.maxIts;
        o->nIterations = nIt;
        o->consumed = consumed;
        o->nBest = nBest;
        for (int i = 0; i < 16; i++) o->T12[i] = success ? st->bestT12[i] : 0.f;
        for (int i = 0; i < 9; i++) o->bestR[i] = st->bestR[i];
        for (int i = 0; i < 3; i++) o->bestT[i] = st->bestT[i];
        o->bestS = st->bestS;
    }
    const uint32_t* m = P.masks + (size_t)(success ? best : 0) * words;
    for (int w = lane; w < words; w += 64) P.outMask[w] = success ? m[w] : 0u;
    rng_after(P.rng, P.raw, consumed * 3, &o->rng);
}

// ----------------------------------------------------------------------- host

Sim3Solver::Sim3Solver(int N, const float* X1c, const float* X2c, const float* s1, const float* s2, const int* idx1,
                       int N1, const float* K1, const float* K2, bool bFixScale)
    : N_(N), N1_(N1), bFixScale_(bFixScale) {
    X1_.assign(X1c, X1c + 3 * (size_t)N);
    X2_.assign(X2c, X2c + 3 * (size_t)N);
    idx1_.assign(idx1, idx1 + N);
    std::memcpy(K1_, K1, 16);
    std::memcpy(K2_, K2, 16);
    p1_.resize(2 * (size_t)N);
    p2_.resize(2 * (size_t)N);
    maxErr1_.resize(N);
    maxErr2_.resize(N);
    for (int i = 0; i < N; i++) {
        // mvnMaxError are vector<size_t> (Sim3Solver.h:78-79): truncated, compared as float
        maxErr1_[i] = (float)(size_t)(9.210 * s1[i]);
        maxErr2_[i] = (float)(size_t)(9.210 * s2[i]);
        for (int k = 0; k < 2; k++) {  // FromCameraToImage (405-423)
            const float* X = k ? &X2_[3 * i] : &X1_[3 * i];
            const float* K = k ? K2_ : K1_;
            float* out = k ? &p2_[2 * i] : &p1_[2 * i];
            const float invz = 1 / X[2];
            const float x = X[0] * invz, y = X[1] * invz;
            out[0] = K[0] * x + K[2];
            out[1] = K[1] * y + K[3];
        }
    }
    set_ransac(0.99, 6, 300);  // Sim3Solver.h:45 defaults, called by the ctor
}

Sim3Solver::~Sim3Solver() {
    if (d_pts_) (void)hipFree(d_pts_);
}

// SetRansacParameters (114-138)
void Sim3Solver::set_ransac(double probability, int minInliers, int maxIterations) {
    prob_ = probability;
    minInliers_ = minInliers;
    maxIts_ = maxIterations;
    const float epsilon = (float)minInliers_ / N_;
    int nIterations;
    if (minInliers_ == N_) nIterations = 1;
    else nIterations = (int)std::ceil(std::log(1 - prob_) / std::log(1 - std::pow(epsilon, 3)));
    maxIts_ = std::max(1, std::min(nIterations, maxIts_));
    nIterations_ = 0;
}

static size_t al256s(size_t v) { return (v + 255) & ~(size_t)255; }

// device block: X1 | X2 | p1 | p2 | maxErr1 | maxErr2 | Sim3StateDev
size_t Sim3Solver::state_off() const { return al256s((size_t)N_ * 12 * 4 + 64); }

int Sim3Solver::upload(hipStream_t s) {
    if (!dirty_) return 0;
    const size_t so = state_off(), bytes = so + al256s(sizeof(Sim3StateDev));
    if (bytes > d_cap_) {   // first upload: a fresh state (no best estimate yet)
        if (d_pts_) (void)hipFree(d_pts_);
        ORB_HIP_CHECK(hipMalloc(&d_pts_, bytes));
        d_cap_ = bytes;
        ORB_HIP_CHECK(hipMemsetAsync((char*)d_pts_ + so, 0, bytes - so, s));
    }
    float* d = (float*)d_pts_;
    ORB_HIP_CHECK(hipMemcpyAsync(d, X1_.data(), (size_t)N_ * 12, hipMemcpyHostToDevice, s));
    ORB_HIP_CHECK(hipMemcpyAsync(d + 3 * N_, X2_.data(), (size_t)N_ * 12, hipMemcpyHostToDevice, s));
    ORB_HIP_CHECK(hipMemcpyAsync(d + 6 * N_, p1_.data(), (size_t)N_ * 8, hipMemcpyHostToDevice, s));
    ORB_HIP_CHECK(hipMemcpyAsync(d + 8 * N_, p2_.data(), (size_t)N_ * 8, hipMemcpyHostToDevice, s));
    ORB_HIP_CHECK(hipMemcpyAsync(d + 10 * N_, maxErr1_.data(), (size_t)N_ * 4, hipMemcpyHostToDevice, s));
    ORB_HIP_CHECK(hipMemcpyAsync(d + 11 * N_, maxErr2_.data(), (size_t)N_ * 4, hipMemcpyHostToDevice, s));
    dirty_ = false;
    return 0;
}

Sim3Batch::~Sim3Batch() {
    for (auto& e : ev_)
        if (e) (void)hipEventDestroy(e);
    if (d_work_) (void)hipFree(d_work_);
    if (d_probs_) (void)hipFree(d_probs_);
    if (h_work_) (void)hipHostFree(h_work_);
    if (stream_) (void)hipStreamDestroy(stream_);
}

int Sim3Batch::init() {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return -4;
    ORB_HIP_CHECK(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
    for (auto& e : ev_) ORB_HIP_CHECK(hipEventCreate(&e));
    return 0;
}

int Sim3Batch::last_timings(float* ms2, long long* hyp_pts2) {
    if (!timed_) return -1;
    ORB_HIP_CHECK(hipEventSynchronize(ev_[2]));
    ORB_HIP_CHECK(hipEventElapsedTime(&ms2[0], ev_[0], ev_[1]));
    ORB_HIP_CHECK(hipEventElapsedTime(&ms2[1], ev_[1], ev_[2]));
    hyp_pts2[0] = last_hyp_;
    hyp_pts2[1] = last_pts_;
    return 0;
}

// Sim3Solver::iterate for `n` solvers (distinct streams).  Device work area: [per solver: draws |
// stream words | counts | masks | estimates] [per solver: record]; the pinned host buffer
// mirrors the record region (ONE copy back per call).
int Sim3Batch::iterate(int n, Sim3Solver** S, int nIterations, orb_rng** rngs, Sim3Result* res) {
    hipStream_t s = stream_;
    auto al = al256s;
    auto words_of = [](int N) { return (N + 31) >> 5; };
    auto out_bytes = [&](int N) { return al(sizeof(Sim3OutDev) + (size_t)words_of(N) * 4); };
    auto scratch = [&](int K, int N) {
        return 2 * al((size_t)K * 12) + al((size_t)K * 4) + al((size_t)K * words_of(N) * 4) + al((size_t)K * 128);
    };
    std::vector<int> K(n, 0), act(n, 0);
    size_t dev = 0, host = 0;
    for (int k = 0; k < n; k++) {
        Sim3Solver& P = *S[k];
        Sim3Result& r = res[k];
        r.has_pose = 0;
        r.bNoMore = 0;
        r.nInliers = 0;
        if (r.inliers) std::fill(r.inliers, r.inliers + P.N1_, 0);  // vbInliers = vector<bool>(mN1,false)
        if (P.N_ < P.minInliers_) {
            r.bNoMore = 1;
            continue;
        }
        if ((size_t)P.N_ >= (size_t)kRngMaxRange) return -1;
        act[k] = 1;
        // `while (mnIterations < max && nCurrent < nIterations)`
        K[k] = std::max(0, std::min(P.maxIts_ - P.nIterations_, nIterations));
        dev += scratch(K[k], P.N_);
        host += out_bytes(P.N_);
        if (int e = P.upload(s)) return e;
    }
    const size_t out_base = dev;
    dev += host;
    if (dev + 256 > work_cap_) {
        if (d_work_) (void)hipFree(d_work_);
        ORB_HIP_CHECK(hipMalloc(&d_work_, dev + 256));
        work_cap_ = dev + 256;
    }
    // the problem table is staged in the pinned block too (after the records): a pageable
    // source would make its copy a synchronous staging round trip
    const size_t probs_h = al(host), hbytes = probs_h + sizeof(Sim3ProbDev) * n + 256;
    if (hbytes > hwork_cap_) {
        if (h_work_) (void)hipHostFree(h_work_);
        ORB_HIP_CHECK(hipHostMalloc(&h_work_, hbytes));
        hwork_cap_ = hbytes;
    }
    if (sizeof(Sim3ProbDev) * n > probs_cap_) {
        if (d_probs_) (void)hipFree(d_probs_);
        ORB_HIP_CHECK(hipMalloc(&d_probs_, sizeof(Sim3ProbDev) * n + 16));
        probs_cap_ = sizeof(Sim3ProbDev) * n;
    }
    char* D = (char*)d_work_;
    char* Hh = (char*)h_work_;
    Sim3ProbDev* pd = (Sim3ProbDev*)(Hh + probs_h);
    std::vector<size_t> out_off(n, 0);
    size_t o = 0, ho = 0;
    int maxK = 0, nact = 0;
    long long hyp = 0, pts = 0;
    for (int k = 0; k < n; k++) {
        if (!act[k]) continue;
        Sim3Solver& P = *S[k];
        Sim3ProbDev& q = pd[nact++];
        std::memset(&q, 0, sizeof(Sim3ProbDev));
        const float* d = (const float*)P.d_pts_;
        q.X1 = d; q.X2 = d + 3 * P.N_; q.p1 = d + 6 * P.N_; q.p2 = d + 8 * P.N_;
        q.maxErr1 = d + 10 * P.N_; q.maxErr2 = d + 11 * P.N_;
        q.N = P.N_;
        q.bFixScale = P.bFixScale_ ? 1 : 0;
        std::memcpy(q.K1, P.K1_, 16);
        std::memcpy(q.K2, P.K2_, 16);
        q.nhyp = K[k];
        q.hyp_idx = (int*)(D + o); o += al((size_t)K[k] * 12);
        q.raw = (uint32_t*)(D + o); o += al((size_t)K[k] * 12);
        q.counts = (int*)(D + o); o += al((size_t)K[k] * 4);
        q.masks = (uint32_t*)(D + o); o += al((size_t)K[k] * words_of(P.N_) * 4);
        q.est = (float*)(D + o); o += al((size_t)K[k] * 128);
        q.minInliers = P.minInliers_;
        q.maxIts = P.maxIts_;
        q.nIt0 = P.nIterations_;
        q.rng = *rngs[k];
        q.state = (Sim3StateDev*)((char*)P.d_pts_ + P.state_off());
        out_off[k] = ho;
        q.out = (Sim3OutDev*)(D + out_base + ho);
        q.outMask = (uint32_t*)(D + out_base + ho + sizeof(Sim3OutDev));
        ho += out_bytes(P.N_);
        maxK = std::max(maxK, K[k]);
        hyp += K[k];
        pts += (long long)K[k] * P.N_;
    }
    if (nact == 0) return 0;
    ORB_HIP_CHECK(hipMemcpyAsync(d_probs_, pd, sizeof(Sim3ProbDev) * nact, hipMemcpyHostToDevice, s));
    const Sim3ProbDev* dprobs = (const Sim3ProbDev*)d_probs_;
    if (maxK > 0) {
        if (timing_) ORB_HIP_CHECK(hipEventRecord(ev_[0], s));
        hipLaunchKernelGGL(k_sim3_hypotheses, dim3((maxK + 63) / 64, nact), dim3(64), 0, s, dprobs);
        if (timing_) ORB_HIP_CHECK(hipEventRecord(ev_[1], s));
        hipLaunchKernelGGL(k_sim3_check, dim3((maxK + kSim3CheckHyp - 1) / kSim3CheckHyp, nact), dim3(kSim3CheckThreads),
                           0, s, dprobs);
        if (timing_) ORB_HIP_CHECK(hipEventRecord(ev_[2], s));
        last_hyp_ = hyp;
        last_pts_ = pts;
        timed_ = timing_;
    }
    hipLaunchKernelGGL(k_sim3_replay, dim3(nact), dim3(64), 0, s, dprobs);
    ORB_HIP_CHECK(hipGetLastError());
    ORB_HIP_CHECK(hipMemcpyAsync(Hh, D + out_base, host, hipMemcpyDeviceToHost, s));
    ORB_HIP_CHECK(hipStreamSynchronize(s));
    for (int k = 0; k < n; k++) {
        if (!act[k]) continue;
        Sim3Solver& P = *S[k];
        Sim3Result& r = res[k];
        const Sim3OutDev* od = (const Sim3OutDev*)(Hh + out_off[k]);
        const uint32_t* m = (const uint32_t*)(Hh + out_off[k] + sizeof(Sim3OutDev));
        P.nIterations_ = od->nIterations;
        P.nBestInliers_ = od->nBest;
        std::memcpy(P.bestR_, od->bestR, 36);
        std::memcpy(P.bestT_, od->bestT, 12);
        P.bestS_ = od->bestS;
        *rngs[k] = od->rng;
        r.has_pose = od->has_pose;
        r.bNoMore = od->bNoMore;
        r.nInliers = od->nInliers;
        if (r.has_pose) {
            std::memcpy(r.T12, od->T12, 64);
            for (int i = 0; i < P.N_; i++)
                if ((m[i >> 5] >> (i & 31)) & 1) r.inliers[P.idx1_[i]] = 1;
        }
    }
    return 0;
}

}  // namespace orbgpu
