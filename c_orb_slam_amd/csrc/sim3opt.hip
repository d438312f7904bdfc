// sim3opt.hip -- gfx950 Optimizer::OptimizeSim3 (reference src/Optimizer.cc:1046-1241):
// the loop-candidate Sim3 refinement of LoopClosing::ComputeSim3 (LoopClosing.cc:326).
//
// One persistent workgroup per candidate (a batch of candidates is one launch).  The
// problem is a single 7-dof VertexSim3Expmap against fixed points, so per LM iteration:
//   - 15 lanes build the estimate's inverse and the 14 perturbed estimates of g2o's
//     numeric linearizeOplus (base_binary_edge.hpp:131-204: Sim3(+-1e-9 e_d) * T and
//     their inverses) ONCE for all edges, into LDS;
//   - one fused pass over the active edges: error, robust chi2, the 2x7 central-difference
//     Jacobian and the 35 terms of the 7x7 system (28 upper H + 7 b), canonical 64-tree sums
//     (oracle/ba.c ora_csum);
//   - per trial: thread 0 runs the pivoted LDL^T (LinearSolverDense), the in-place
//     fix-scale zeroing of _x and the Sim3 update; one error pass gives the new chi2.
// Every operation sequence equals oracle/ba.c ora_optimize_sim3, so the result is
// bit-identical to it.  Edges are 32 B in HBM (float inputs, as the reference's).
#include "sim3opt.hpp"

#include <algorithm>
#include <cstring>
#include <vector>

#include "ba_math.hpp"
#include "detmath.hpp"
#include "orb_common.hpp"

namespace orbgpu {

struct Sim3d {   // g2o::Sim3: q = (x, y, z, w) like Eigen coeffs(), t, s
    double q[4];
    double t[3];
    double s;
};

// g2o::Sim3(const Vector7d& update)  sim3.h:64-146
__device__ __forceinline__ void sim3_exp(const double* upd, Sim3d& o) {
    const double w0 = upd[0], w1 = upd[1], w2 = upd[2];
    const double sigma = upd[6];
    const double theta = sqrt((w0 * w0 + w1 * w1) + w2 * w2);
    const double Om[9] = {0, -w2, w1, w2, 0, -w0, -w1, w0, 0};
    double Om2[9], R[9];
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
        for (int j = 0; j < 3; j++)
            Om2[i * 3 + j] = (Om[i * 3] * Om[j] + Om[i * 3 + 1] * Om[3 + j]) + Om[i * 3 + 2] * Om[6 + j];
    const double s = detmath::exp_d(sigma);
    const double eps = 0.00001;
    double A, B, C, ra = 1.0, rb = 1.0;
    const bool small = theta < eps;
    if (!small) {
        double sn, cs;
        detmath::sincos_d(theta, &sn, &cs);
        ra = sn / theta;
        rb = (1 - cs) / (theta * theta);
        if (fabs(sigma) < eps) {
            C = 1;
            const double theta2 = theta * theta;
            A = (1 - cs) / theta2;
            B = (theta - sn) / (theta2 * theta);
        } else {
            C = (s - 1) / sigma;
            const double a = s * sn, b = s * cs;
            const double theta2 = theta * theta, sigma2 = sigma * sigma;
            const double c = theta2 + sigma2;
            A = (a * sigma + (1 - b) * theta) / (theta * c);
            B = (C - ((b - 1) * sigma + a * theta) / c) * 1. / theta2;
        }
    } else if (fabs(sigma) < eps) {
        C = 1;
        A = 1. / 2.;
        B = 1. / 6.;
    } else {
        C = (s - 1) / sigma;
        const double sigma2 = sigma * sigma;
        A = ((sigma - 1) * s + 1) / sigma2;
        B = ((0.5 * sigma2 - sigma + 1) * s) / (sigma2 * sigma);
    }
#pragma unroll
    for (int i = 0; i < 9; i++) {
        const double I = (i % 4) == 0 ? 1.0 : 0.0;
        R[i] = small ? (I + Om[i]) + Om2[i] : (I + ra * Om[i]) + rb * Om2[i];
    }
    quat_from_R(R, o.q);
    double W[9];
#pragma unroll
    for (int i = 0; i < 9; i++) W[i] = (A * Om[i] + B * Om2[i]) + C * ((i % 4) == 0 ? 1.0 : 0.0);
#pragma unroll
    for (int i = 0; i < 3; i++) o.t[i] = (W[i * 3] * upd[3] + W[i * 3 + 1] * upd[4]) + W[i * 3 + 2] * upd[5];
    o.s = s;
}

// operator*  sim3.h:264-270
__device__ __forceinline__ void sim3_mul(const Sim3d& a, const Sim3d& b, Sim3d& o) {
    Sim3d r;
    r.q[3] = ((a.q[3] * b.q[3] - a.q[0] * b.q[0]) - a.q[1] * b.q[1]) - a.q[2] * b.q[2];
    r.q[0] = ((a.q[3] * b.q[0] + a.q[0] * b.q[3]) + a.q[1] * b.q[2]) - a.q[2] * b.q[1];
    r.q[1] = ((a.q[3] * b.q[1] + a.q[1] * b.q[3]) + a.q[2] * b.q[0]) - a.q[0] * b.q[2];
    r.q[2] = ((a.q[3] * b.q[2] + a.q[2] * b.q[3]) + a.q[0] * b.q[1]) - a.q[1] * b.q[0];
    double rt[3];
    quat_rotate(a.q, b.t, rt);
#pragma unroll
    for (int i = 0; i < 3; i++) r.t[i] = a.s * rt[i] + a.t[i];
    r.s = a.s * b.s;
    o = r;
}

// inverse  sim3.h:235-238
__device__ __forceinline__ void sim3_inverse(const Sim3d& T, Sim3d& o) {
    Sim3d r;
    r.q[0] = -T.q[0];
    r.q[1] = -T.q[1];
    r.q[2] = -T.q[2];
    r.q[3] = T.q[3];
    const double ms = -1. / T.s;
    const double v[3] = {ms * T.t[0], ms * T.t[1], ms * T.t[2]};
    quat_rotate(r.q, v, r.t);
    r.s = 1. / T.s;
    o = r;
}

// edge in HBM: 32 B
struct S3EdgeDev {
    float X[3];     // the fixed point vertex (X2c for EdgeSim3ProjectXYZ, X1c for the inverse edge)
    float obs[2];   // kpUn.pt
    float info;     // mvInvLevelSigma2[octave]
    int meta;       // bit 31: EdgeInverseSim3ProjectXYZ; bits 0-30: correspondence index
    int pad;
};

struct S3ProbDev {
    int ne, e0;         // edges E[e0 .. e0+ne): pairs (e12, e21) per correspondence
    int nIn, reached;   // out
    int fix;
    float th2f;
    double f1[2], p1[2], f2[2], p2[2];
    Sim3d S;            // in / out
};

constexpr int kS3MaxEdges = 4096;
constexpr int kS3Threads = 256;
constexpr int kS3Per = kS3MaxEdges / kS3Threads;
constexpr int kS3Terms = 36;   // robust chi2 | 28 upper H | 7 b
__constant__ int kDiag28[7] = {0, 7, 13, 18, 22, 25, 27};

struct S3EdgeD {
    double X[3], obs[2], info;
    bool inv;
};

__device__ __forceinline__ S3EdgeD s3_load(const S3EdgeDev* E, int i) {
    const uint4* p = reinterpret_cast<const uint4*>(E + i);
    const uint4 a = p[0], b = p[1];
    S3EdgeD e;
    e.X[0] = (double)__uint_as_float(a.x);
    e.X[1] = (double)__uint_as_float(a.y);
    e.X[2] = (double)__uint_as_float(a.z);
    e.obs[0] = (double)__uint_as_float(a.w);
    e.obs[1] = (double)__uint_as_float(b.x);
    e.info = (double)__uint_as_float(b.y);
    e.inv = (b.z >> 31) != 0;
    return e;
}

// EdgeSim3ProjectXYZ / EdgeInverseSim3ProjectXYZ::computeError (types_seven_dof_expmap.h:138-145,
// 160-167) with the estimate T (direct edge) or its inverse Ti (inverse edge)
__device__ __forceinline__ void s3_err(const S3EdgeD& e, const Sim3d& T, const Sim3d& Ti, const S3ProbDev& P,
                                       double* err) {
    const Sim3d& M = e.inv ? Ti : T;
    double r[3], p[3];
    quat_rotate(M.q, e.X, r);
#pragma unroll
    for (int i = 0; i < 3; i++) p[i] = M.s * r[i] + M.t[i];
    const double px = p[0] / p[2], py = p[1] / p[2];
    const double* f = e.inv ? P.f2 : P.f1;
    const double* c = e.inv ? P.p2 : P.p1;
    err[0] = e.obs[0] - (px * f[0] + c[0]);
    err[1] = e.obs[1] - (py * f[1] + c[1]);
}

__device__ __forceinline__ double s3_chi2(const double* err, double info) {
    return err[0] * (info * err[0]) + err[1] * (info * err[1]);
}

__device__ __forceinline__ double s3_rho0(double c, double delta, double dsqr) {
    if (c <= dsqr) return c;
    const double sq = sqrt(c);
    return (2 * sq) * delta - dsqr;
}

// Block-wide canonical sums of K per-active-edge values (as k_pose_opt's pose_pass)
template <int K, class F>
__device__ __forceinline__ void s3_pass(F f, int nA, const int* aE, const S3EdgeDev* E,
                                        double (*cs)[kS3MaxEdges / 64], double* res) {
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, nw = blockDim.x >> 6;
    const int m = (nA + 63) >> 6;
    for (int c = w; c < m; c += nw) {
        const int a = c * 64 + lane;
        double v[K];
        if (a < nA) {
            const int i = aE[a];
            f(s3_load(E, i), i, v);
        } else {
#pragma unroll
            for (int q = 0; q < K; q++) v[q] = 0.0;
        }
#pragma unroll
        for (int q = 0; q < K; q++) {
            const double t = nA == 1 ? v[q] : wave_tree(v[q]);   // ora_csum keeps a single term untouched
            if (lane == 0) cs[q][c] = t;
        }
    }
    __syncthreads();
    if ((int)threadIdx.x < K) res[threadIdx.x] = nA > 0 ? local_csum_inplace(cs[threadIdx.x], m) : 0.0;
    __syncthreads();
}

__global__ void __launch_bounds__(kS3Threads) k_sim3_opt(S3ProbDev* probs, const S3EdgeDev* __restrict__ Eall,
                                                         double* errAll, uint8_t* eraseAll) {
    S3ProbDev& P = probs[blockIdx.x];
    const int ne = P.ne;
    const S3EdgeDev* E = Eall + P.e0;
    double* err = errAll + 2 * (size_t)P.e0;
    uint8_t* erase = eraseAll + P.e0 / 2;
    __shared__ uint8_t level[kS3MaxEdges];
    __shared__ int aE[kS3MaxEdges];
    __shared__ double cs[kS3Terms][kS3MaxEdges / 64];
    __shared__ double red[kS3Terms];
    __shared__ Sim3d T, Ti, Tbak, Tp[14], Tpi[14];
    __shared__ double xs[7], Hs[28], bs[7];
    __shared__ double lambda, ni, currentChi, iniChi;
    __shared__ int nA, nBadLM, okS, term, nBad, wsum[kS3Threads / 64];
    const int tid = threadIdx.x;
    if (ne < 0) return;   // capacity exceeded (reported by the host)
    const int nc = ne / 2;
    const double delta = (double)sqrtf(P.th2f);   // const float deltaHuber = sqrt(th2)
    const double dsqr = delta * delta;
    const double th2 = (double)P.th2f;
    const double scalar = 1.0 / (2 * 1e-9);
    for (int i = tid; i < ne; i += blockDim.x) level[i] = 0;
    for (int c = tid; c < nc; c += blockDim.x) erase[c] = 0;
    if (tid == 0) {
        T = P.S;
        P.nIn = 0;
        P.reached = 0;
        nBad = 0;
    }
    __syncthreads();
    for (int round = 0; round < 2; round++) {
        const int its = round == 0 ? 5 : (nBad > 0 ? 10 : 5);
        // active edges (level 0) in edge order
        {
            const int base = tid * kS3Per;
            int c = 0;
            for (int j = 0; j < kS3Per; j++) c += (base + j < ne && level[base + j] == 0) ? 1 : 0;
            int incl = c;
            for (int o = 1; o < 64; o <<= 1) {
                const int t = __shfl_up(incl, o, 64);
                if ((tid & 63) >= o) incl += t;
            }
            if ((tid & 63) == 63) wsum[tid >> 6] = incl;
            __syncthreads();
            int off = 0;
            for (int w = 0; w < (tid >> 6); w++) off += wsum[w];
            int pos = off + incl - c;
            for (int j = 0; j < kS3Per; j++)
                if (base + j < ne && level[base + j] == 0) aE[pos++] = base + j;
            if (tid == blockDim.x - 1) nA = off + incl;
            if (tid == 0)
                for (int j = 0; j < 7; j++) xs[j] = 0.0;   // BlockSolver::_x after buildStructure
            __syncthreads();
        }
        const int na = nA;
        if (na > 0) {
            for (int k = 0; k < its; k++) {
                // inverse + the 14 perturbed estimates (push / oplus(+-delta e_d) / pop)
                if (tid < 14) {
                    const int d = tid >> 1;
                    double add[7] = {0, 0, 0, 0, 0, 0, 0};
#pragma unroll
                    for (int j = 0; j < 7; j++)
                        if (j == d) add[j] = (tid & 1) ? -1e-9 : 1e-9;
                    if (P.fix) add[6] = 0;
                    Sim3d U, M;
                    sim3_exp(add, U);
                    sim3_mul(U, T, M);
                    Tp[tid] = M;
                    sim3_inverse(M, Tpi[tid]);
                } else if (tid == 14) {
                    sim3_inverse(T, Ti);
                }
                __syncthreads();
                // computeActiveErrors + activeRobustChi2 (entry 0), buildSystem (1..35)
                s3_pass<kS3Terms>([&](const S3EdgeD& e, int i, double* v) {
                    double e2[2];
                    s3_err(e, T, Ti, P, e2);
                    err[2 * i] = e2[0];
                    err[2 * i + 1] = e2[1];
                    const double c = s3_chi2(e2, e.info);
                    v[0] = s3_rho0(c, delta, dsqr);
                    double J[14];
#pragma unroll
                    for (int d = 0; d < 7; d++) {
                        double ep[2], em[2];
                        s3_err(e, Tp[2 * d], Tpi[2 * d], P, ep);
                        s3_err(e, Tp[2 * d + 1], Tpi[2 * d + 1], P, em);
                        J[d] = scalar * (ep[0] - em[0]);
                        J[7 + d] = scalar * (ep[1] - em[1]);
                    }
                    double r1 = 1.;
                    if (!(c <= dsqr)) r1 = delta / sqrt(c);
                    const double wgt = r1 * e.info;
                    const double om0 = -(e.info * e2[0]) * r1, om1 = -(e.info * e2[1]) * r1;
                    int q = 1;
#pragma unroll
                    for (int r = 0; r < 7; r++) {
                        v[29 + r] = J[r] * om0 + J[7 + r] * om1;
#pragma unroll
                        for (int cc = r; cc < 7; cc++) {
                            v[q] = (J[r] * wgt) * J[cc] + (J[7 + r] * wgt) * J[7 + cc];
                            q++;
                        }
                    }
                }, na, aE, E, cs, red);
                if (tid == 0) {
                    currentChi = iniChi = red[0];
                    for (int j = 0; j < 28; j++) Hs[j] = red[1 + j];
                    for (int j = 0; j < 7; j++) bs[j] = red[29 + j];
                    if (k == 0) {   // computeLambdaInit
                        double mx = 0.;
                        for (int j = 0; j < 7; j++) mx = fmax(fabs(Hs[kDiag28[j]]), mx);
                        lambda = 1e-5 * mx;
                        ni = 2;
                        nBadLM = 0;
                    }
                }
                __syncthreads();
                int qmax = 0;
                double rho = 0;
                do {
                    if (tid == 0) {
                        Tbak = T;
                        double Hd[49], x[7];
                        for (int r = 0, q = 0; r < 7; r++)
                            for (int cc = r; cc < 7; cc++, q++) {
                                double h = Hs[q];
                                if (cc == r) h += lambda;
                                Hd[r * 7 + cc] = h;
                                Hd[cc * 7 + r] = h;
                            }
                        const bool ok2 = ldlt_pivot<7>(Hd, bs, x);
                        okS = ok2 ? 1 : 0;
                        if (ok2)
                            for (int j = 0; j < 7; j++) xs[j] = x[j];
                        if (P.fix) xs[6] = 0;   // oplusImpl writes through the Map of the solver's _x
                        Sim3d U, M;
                        sim3_exp(xs, U);
                        sim3_mul(U, T, M);
                        T = M;
                        sim3_inverse(M, Ti);
                    }
                    __syncthreads();
                    s3_pass<1>([&](const S3EdgeD& e, int i, double* v) {
                        double e2[2];
                        s3_err(e, T, Ti, P, e2);
                        err[2 * i] = e2[0];
                        err[2 * i + 1] = e2[1];
                        v[0] = s3_rho0(s3_chi2(e2, e.info), delta, dsqr);
                    }, na, aE, E, cs, red);
                    if (tid == 0) {
                        double tc = red[0];
                        if (!okS) tc = DBL_MAX;
                        double r = currentChi - tc;
                        double sv[7];
                        for (int j = 0; j < 7; j++) sv[j] = xs[j] * (lambda * xs[j] + bs[j]);
                        double scale = local_csum_inplace(sv, 7);
                        scale += 1e-3;
                        r /= scale;
                        if (r > 0 && isfinite(tc)) {
                            const double a3 = 2 * r - 1;
                            double alpha = 1. - (a3 * a3) * a3;
                            alpha = fmin(alpha, 2. / 3.);
                            const double scaleFactor = fmax(1. / 3., alpha);
                            lambda *= scaleFactor;
                            ni = 2;
                            currentChi = tc;
                        } else {
                            lambda *= ni;
                            ni *= 2;
                            T = Tbak;
                        }
                        red[0] = r;
                    }
                    __syncthreads();
                    rho = red[0];
                    qmax++;
                    __syncthreads();
                } while (rho < 0 && qmax < 10);
                if (tid == 0) {
                    int t = 0;
                    if (qmax == 10 || rho == 0) t = 1;
                    else {
                        if ((iniChi - currentChi) * 1e3 < iniChi) nBadLM++;
                        else nBadLM = 0;
                        t = nBadLM >= 3;
                    }
                    term = t;
                }
                __syncthreads();
                if (term) break;
            }
        }
        // chi2 gating on the last evaluated errors (Optimizer.cc:1185-1209 / 1219-1234)
        int cnt = 0;
        for (int c = tid; c < nc; c += blockDim.x) {
            if (level[2 * c]) continue;
            const double i1 = (double)E[2 * c].info, i2 = (double)E[2 * c + 1].info;
            const double* ea = err + 4 * (size_t)c;
            const bool bad = s3_chi2(ea, i1) > th2 || s3_chi2(ea + 2, i2) > th2;
            if (bad) erase[c] = 1;
            if (round == 0) {
                cnt += bad ? 1 : 0;
                if (bad) {
                    level[2 * c] = 1;
                    level[2 * c + 1] = 1;
                }
            } else {
                cnt += bad ? 0 : 1;
            }
        }
        for (int o = 32; o >= 1; o >>= 1) cnt += __shfl_xor(cnt, o, 64);
        if ((tid & 63) == 0) wsum[tid >> 6] = cnt;
        __syncthreads();
        if (tid == 0) {
            int s = 0;
            for (int w = 0; w < (int)(blockDim.x >> 6); w++) s += wsum[w];
            if (round == 0) nBad = s;
            else {
                P.nIn = s;
                P.reached = 1;
                P.S = T;
            }
        }
        __syncthreads();
        if (round == 0 && nc - nBad < 10) break;   // early return: g2oS12 untouched, nIn = 0
    }
}

// ---------------------------------------------------------------- host
class Sim3OptEngine {
public:
    ~Sim3OptEngine() {
        if (dArena_) (void)hipFree(dArena_);
        if (hArena_) (void)hipHostFree(hArena_);
        if (stream_) (void)hipStreamDestroy(stream_);
    }
    int init() {
        int n = 0;
        if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return -4;
        ORB_HIP_CHECK(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
        return 0;
    }
    int run(int count, const sim3opt_problem* P, double* S12, uint8_t* const* erased, int* nIn);

private:
    hipStream_t stream_ = nullptr;
    void* dArena_ = nullptr;
    void* hArena_ = nullptr;
    size_t cap_ = 0;
};

// Edge creation (Optimizer.cc:1099-1178): for each valid correspondence in index order,
// e12 (point 2 -> camera 1) then e21 (point 1 -> camera 2).
int Sim3OptEngine::run(int count, const sim3opt_problem* P, double* S12, uint8_t* const* erased, int* nIn) {
    std::vector<int> nc(count);
    size_t ne = 0;
    for (int f = 0; f < count; f++) {
        int c = 0;
        for (int i = 0; i < P[f].N; i++) c += P[f].valid[i] ? 1 : 0;
        if (2 * c > kS3MaxEdges) return -3;
        nc[f] = c;
        ne += 2 * (size_t)c;
    }
    const auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
    const size_t bProb = al(sizeof(S3ProbDev) * count), bEdge = al(sizeof(S3EdgeDev) * std::max<size_t>(ne, 1));
    const size_t bErr = al(sizeof(double) * 2 * std::max<size_t>(ne, 1)), bEr = al(std::max<size_t>(ne / 2, 1));
    const size_t need = bProb + bEdge + bErr + bEr;
    if (need > cap_) {
        if (dArena_) (void)hipFree(dArena_);
        if (hArena_) (void)hipHostFree(hArena_);
        dArena_ = hArena_ = nullptr;
        cap_ = 0;
        ORB_HIP_CHECK(hipMalloc(&dArena_, need));
        ORB_HIP_CHECK(hipHostMalloc(&hArena_, need));
        cap_ = need;
    }
    char* h = (char*)hArena_;
    char* d = (char*)dArena_;
    S3ProbDev* hp = (S3ProbDev*)h;
    S3EdgeDev* hE = (S3EdgeDev*)(h + bProb);
    size_t e0 = 0;
    for (int f = 0; f < count; f++) {
        const sim3opt_problem& Q = P[f];
        S3ProbDev& pp = hp[f];
        memset(&pp, 0, sizeof(pp));
        pp.ne = 2 * nc[f];
        pp.e0 = (int)e0;
        pp.fix = Q.bFixScale ? 1 : 0;
        pp.th2f = Q.th2;
        pp.f1[0] = Q.K1[0]; pp.f1[1] = Q.K1[1]; pp.p1[0] = Q.K1[2]; pp.p1[1] = Q.K1[3];
        pp.f2[0] = Q.K2[0]; pp.f2[1] = Q.K2[1]; pp.p2[0] = Q.K2[2]; pp.p2[1] = Q.K2[3];
        memcpy(pp.S.q, S12 + 8 * f, 4 * sizeof(double));
        memcpy(pp.S.t, S12 + 8 * f + 4, 3 * sizeof(double));
        pp.S.s = S12[8 * f + 7];
        S3EdgeDev* e = hE + e0;
        for (int i = 0; i < Q.N; i++) {
            if (!Q.valid[i]) continue;
            S3EdgeDev& a = *e++;
            S3EdgeDev& b = *e++;
            memcpy(a.X, Q.X2c + 3 * (size_t)i, 3 * sizeof(float));
            memcpy(a.obs, Q.obs1 + 2 * (size_t)i, 2 * sizeof(float));
            a.info = Q.inv_sigma2_1[i];
            a.meta = i;
            a.pad = 0;
            memcpy(b.X, Q.X1c + 3 * (size_t)i, 3 * sizeof(float));
            memcpy(b.obs, Q.obs2 + 2 * (size_t)i, 2 * sizeof(float));
            b.info = Q.inv_sigma2_2[i];
            b.meta = (int)(0x80000000u | (unsigned)i);
            b.pad = 0;
        }
        e0 += 2 * (size_t)nc[f];
    }
    uint8_t* hEr = (uint8_t*)(h + bProb + bEdge + bErr);
    ORB_HIP_CHECK(hipMemcpyAsync(d, h, bProb + sizeof(S3EdgeDev) * ne, hipMemcpyHostToDevice, stream_));
    hipLaunchKernelGGL(k_sim3_opt, dim3(count), dim3(kS3Threads), 0, stream_, (S3ProbDev*)d,
                       (const S3EdgeDev*)(d + bProb), (double*)(d + bProb + bEdge),
                       (uint8_t*)(d + bProb + bEdge + bErr));
    ORB_HIP_CHECK(hipGetLastError());
    ORB_HIP_CHECK(hipMemcpyAsync(h, d, bProb, hipMemcpyDeviceToHost, stream_));
    ORB_HIP_CHECK(hipMemcpyAsync(hEr, d + bProb + bEdge + bErr, std::max<size_t>(ne / 2, 1), hipMemcpyDeviceToHost,
                                 stream_));
    ORB_HIP_CHECK(hipStreamSynchronize(stream_));
    for (int f = 0; f < count; f++) {
        const sim3opt_problem& Q = P[f];
        const S3ProbDev& pp = hp[f];
        memset(erased[f], 0, (size_t)Q.N);
        const S3EdgeDev* e = hE + pp.e0;
        for (int c = 0; c < nc[f]; c++)
            if (hEr[pp.e0 / 2 + c]) erased[f][e[2 * c].meta] = 1;
        nIn[f] = pp.reached ? pp.nIn : 0;
        if (pp.reached) {
            memcpy(S12 + 8 * f, pp.S.q, 4 * sizeof(double));
            memcpy(S12 + 8 * f + 4, pp.S.t, 3 * sizeof(double));
            S12[8 * f + 7] = pp.S.s;
        }
    }
    return 0;
}

int sim3opt_run(int count, const sim3opt_problem* P, double* S12, uint8_t* const* erased, int* nIn) {
    thread_local Sim3OptEngine* e = nullptr;
    thread_local int erc = 0;
    if (!e) {
        e = new Sim3OptEngine();
        erc = e->init();
    }
    if (erc) return erc;
    return e->run(count, P, S12, erased, nIn);
}

}  // namespace orbgpu
