// ba.hip -- gfx950 local bundle adjustment: Optimizer::LocalBundleAdjustment
// (reference src/Optimizer.cc:453-778) on g2o's BlockSolver<6,3> +
// OptimizationAlgorithmLevenberg (Thirdparty/g2o/g2o/core/*.cpp|hpp).
//
// Layout in HBM (FP64 inside, FP32 I/O like the reference):
//   poses  Se3[n_kf] (q xyzw, t) + backup; points double[3][n_pt] + backup;
//   edges  EdgeDev[n_edge] (static) + level/robust flags + last _error[3];
//   per active edge: quadratic-form terms SoA (Hpp 21 | bp 6 | Hll 9 | bl 3),
//   Hpl 6x3 AoS, BDinv 6x3 AoS, B*db 6; per pose Hpp/bp; per landmark Hll/bl/Dinv/db;
//   dense Schur system S (6 nP)^2 (upper triangle used).
// Kernels per LM solve():  k_linearize (edge ||) -> k_pose_reduce (workgroup per pose)
//   + k_land_reduce (wave per landmark) -> [k_lambda_init] ; per trial:
//   k_point_prep (thread per landmark) -> k_schur (workgroup per pose block)
//   -> k_ldlt (one workgroup) -> k_update (thread per vertex) -> k_errors (edge ||)
//   -> k_csum2 (canonical chi2 and computeScale) ; host reads 4 scalars, decides.
// Every accumulation uses the canonical 64-wide tree order (oracle/ba.c ora_csum),
// so results are bit-identical to the CPU restatement.
#include "ba.hpp"
#include <atomic>

#include <tuple>
#include <type_traits>

#include <functional>

#include <algorithm>
#include <cfloat>
#include <chrono>
#include <cmath>
#include <cstring>
#include <numeric>
#include <thread>

#include "ba_math.hpp"
#include "ba_struct.hpp"
#include "detmath.hpp"
#include "host_par.hpp"
#include "ldlt.hpp"
#include "orb_common.hpp"

namespace orbgpu {


__device__ __forceinline__ void se3_exp(const double* upd, Se3& out) {
    const double* w = upd;
    const double* u = upd + 3;
    const double theta = sqrt((w[0] * w[0] + w[1] * w[1]) + w[2] * w[2]);
    const double Om[9] = {0, -w[2], w[1], w[2], 0, -w[0], -w[1], w[0], 0};
    double Om2[9], R[9], V[9];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++)
            Om2[i * 3 + j] = (Om[i * 3] * Om[j] + Om[i * 3 + 1] * Om[3 + j]) + Om[i * 3 + 2] * Om[6 + j];
    if (theta < 0.00001) {
        for (int i = 0; i < 9; i++) {
            R[i] = (((i % 4) == 0 ? 1.0 : 0.0) + Om[i]) + Om2[i];
            V[i] = R[i];
        }
    } else {
        double s, c;
        detmath::sincos_d(theta, &s, &c);
        const double a = s / theta, b = (1 - c) / (theta * theta);
        const double cc = (theta - s) / ((theta * theta) * theta);
        for (int i = 0; i < 9; i++) {
            const double I = (i % 4) == 0 ? 1.0 : 0.0;
            R[i] = (I + a * Om[i]) + b * Om2[i];
            V[i] = (I + b * Om[i]) + cc * Om2[i];
        }
    }
    quat_from_R(R, out.q);
    for (int i = 0; i < 3; i++) out.t[i] = (V[i * 3] * u[0] + V[i * 3 + 1] * u[1]) + V[i * 3 + 2] * u[2];
    out.pad = 0;
    se3_normalize(out);
}

// computeError (types_six_dof_expmap.h:94-99, 126-131; .cpp:141-157)
__device__ __forceinline__ void edge_error(const EdgeDev& e, const Se3& T, const double* X, double* err) {
    double p[3];
    se3_map(T, X, p);
    const SharedDiv dz(p[2]);
    if (!e.stereo) {
        const double px = dz.div(p[0]), py = dz.div(p[1]);
        err[0] = e.obs[0] - (px * e.fx + e.cx);
        err[1] = e.obs[1] - (py * e.fy + e.cy);
        err[2] = 0;
    } else {
        const float invz = (float)dz.div(1.0);
        const float bf = (float)e.bf;
        const double u = (p[0] * (double)invz) * e.fx + e.cx;
        const double v = (p[1] * (double)invz) * e.fy + e.cy;
        err[0] = e.obs[0] - u;
        err[1] = e.obs[1] - v;
        err[2] = e.obs[2] - (u - (double)(bf * invz));
    }
}

__device__ __forceinline__ double edge_chi2(const EdgeDev& e, const double* err) {
    double s = 0;
    const int D = e.stereo ? 3 : 2;
    for (int j = 0; j < D; j++) s += err[j] * (e.info * err[j]);
    return s;
}

__device__ __forceinline__ void huber(const EdgeDev& e, double chi, double* rho0, double* rho1) {
    if (chi <= e.dsqr) {
        *rho0 = chi;
        *rho1 = 1.;
    } else {
        const double sq = sqrt(chi);
        *rho0 = (2 * sq) * e.delta - e.dsqr;
        *rho1 = e.delta / sq;
    }
}


// K canonical 64-trees at once: lane holds v[0..K); lane q < K receives the tree of entry q.
// Transpose through this wave's LDS buffer (K x 65 doubles), then per-lane register trees.
template <int K>
__device__ __forceinline__ double wave_trees(const double* v, double* buf) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int q = 0; q < K; q++) buf[q * 65 + lane] = v[q];
    __builtin_amdgcn_wave_barrier();
    double r = 0.0;
    if (lane < K) {
        const double* row = buf + lane * 65;
        r = tree64_local([&](int i) { return row[i]; }, 64);
    }
    __builtin_amdgcn_wave_barrier();
    return r;
}


constexpr int DIAG21[6] = {0, 6, 11, 15, 18, 20};

// Device-resident LM (BaEngine::optimize_device): every kernel of a step takes a gate word that
// k_lm_trial_end set for it; a step the decision made unnecessary runs as empty launches.
// nullptr: always run (the host-driven path).
#define BA_GATE(run)                  \
    do {                              \
        if ((run) && !*(run)) return; \
    } while (0)

// term layout (SoA, stride nE): Hpp 0..20 | bp 21..26 | Hll 27..35 | bl 36..38
constexpr int T_HPP = 0, T_BP = 21, T_HLL = 27, T_BL = 36, T_N = 39;

// ---------------------------------------------------------------- kernels
struct LinArgs {
    BaStructDev s;
    const EdgeDev* E;
    const Se3* T;
    const double* X;
    const uint8_t* robust;
    double* err;      // ne x 3
    double* rc;       // nE robust chi2 terms
    double* terms;    // T_N x nE
    double* Hpl;      // nE x 18
    int linearize;
    double* chunks;   // per-wave chunk trees of rc (ceil(nE/64))
    unsigned* counter;
    double* out;      // canonical sum of rc
    const int* run;   // gate (device LM) or nullptr
    // the device LM's trial pass with the update fused in (fuse = 1): blocks [0, edgeBlocks) take
    // the edges at the trial's poses and points, computed from x on the fly with k_update's
    // operations; the blocks after them write the trial's poses / points to Tn / Xn (committed
    // by k_lm_trial_end on acceptance) and the landmarks' steps into x
    int fuse = 0;
    int edgeBlocks = 0;
    double* x = nullptr;
    const double* Hll = nullptr;
    const double* bl = nullptr;
    const double* scal = nullptr;
    Se3* Tn = nullptr;
    double* Xn = nullptr;
};

// computeActiveErrors + activeRobustChi2 terms (+ linearizeOplus + constructQuadraticForm)
// canonical total of chunk sums c[0..m) with 256 threads, into *out: the level-2 trees go to an
// LDS buffer (m <= 64 * 1024 chunks, 4.2 M edges) or, for larger problems (config 5 at 8-16 k
// keyframes), to the chunk buffer's tail c[m..m + m/64] (carve sizes it); m <= 64 * kCsumLv
constexpr int kCsumLv = 4096;
// level-2 trees up to this many go to LDS (1024 = the LDS buffer); tests lower it through
// orbgpu_unit_set_csum_lds_max to drive the chunk-buffer tail path at small sizes
__device__ int g_csum_lds_max = 1024;
__device__ __forceinline__ void block_finish_csum(double* c, int m, int nterms, const double* single, double* out) {
    __shared__ double lv[1024];
    if (nterms <= 1) {
        if (threadIdx.x == 0) *out = nterms == 1 ? *single : 0.0;
        return;
    }
    if (m == 1) {
        if (threadIdx.x == 0) *out = c[0];
        return;
    }
    int m2 = (m + 63) >> 6;
    double* L = m2 <= min(g_csum_lds_max, 1024) ? lv : c + m;
    for (int t = threadIdx.x; t < m2; t += blockDim.x)
        L[t] = tree64_local([&](int k) { return c[t * 64 + k]; }, min(64, m - t * 64));
    __threadfence_block();   // L may be the chunk buffer's tail: read by thread 0 of this block
    __syncthreads();
    if (threadIdx.x == 0) *out = local_csum_inplace(L, m2);
}

// The chi2 total of k_linearize's chunk trees, one workgroup.  A launch of its own: the kernel
// boundary orders the chunk stores for this reader, where the former last-block-finishes
// pattern needed a device-scope fence in every wave (an L2 writeback + invalidate on gfx950).
// Eigen 3x3 inverse (compute_inverse_size3)
__device__ __forceinline__ void inv3(const double* m, double* r) {
#define M(i, j) m[(i) * 3 + (j)]
#define COF(i, j) (M(((i) + 1) % 3, ((j) + 1) % 3) * M(((i) + 2) % 3, ((j) + 2) % 3) - \
                   M(((i) + 1) % 3, ((j) + 2) % 3) * M(((i) + 2) % 3, ((j) + 1) % 3))
    const double c0 = COF(0, 0), c1 = COF(1, 0), c2 = COF(2, 0);
    const double det = (c0 * M(0, 0) + c1 * M(1, 0)) + c2 * M(2, 0);
    const double invdet = 1.0 / det;
    r[0] = c0 * invdet; r[1] = c1 * invdet; r[2] = c2 * invdet;
    r[3] = COF(0, 1) * invdet; r[4] = COF(1, 1) * invdet; r[5] = COF(2, 1) * invdet;
    r[6] = COF(0, 2) * invdet; r[7] = COF(1, 2) * invdet; r[8] = COF(2, 2) * invdet;
#undef COF
#undef M
}

typedef double bd2 __attribute__((ext_vector_type(2)));   // 16-B loads / stores of aligned FP64 records

// Dinv = (Hll + lambda I)^-1 of landmark l (setLambda + D->inverse(), block_solver.hpp:383-389)
__device__ __forceinline__ void land_dinv(const double* Hll, int l, double lambda, double* Di) {
    double D[9];
    for (int q = 0; q < 9; q++) D[q] = Hll[9 * l + q];
    for (int j = 0; j < 3; j++) D[4 * j] += lambda;
    inv3(D, Di);
}

// k_update's operations, shared with the fused trial pass (k_linearize, fuse = 1) so the two give
// the same values: the pose step T <- exp(x_p) T, and the landmark step xl = Dinv (b_l - sum_i
// B_i^T xp_i) over the landmark's pose edges in pose order (x's own entries when the solve failed)
__device__ __forceinline__ Se3 pose_step(const Se3& t0, const double* xp) {
    double upd[6];
    for (int k = 0; k < 6; k++) upd[k] = xp[k];
    Se3 d, r;
    se3_exp(upd, d);
    se3_mul(d, t0, r);
    return r;
}
__device__ __forceinline__ void land_step(const BaStructDev& s, int l, const double* __restrict__ Hpl, const double* Hll,
                                          const double* bl, const double* x, double lambda, bool solved, double* xl) {
    if (!solved) {
        for (int k = 0; k < 3; k++) xl[k] = x[6 * s.nP + 3 * l + k];
        return;
    }
    double cl[3] = {bl[3 * l], bl[3 * l + 1], bl[3 * l + 2]};
    // the landmark's pose edges four at a time: their list entries, then their positions and
    // poses, then their Hpl blocks and pose steps are loaded before any is used, so the chain of
    // dependent loads is paid once per four edges; the sums keep the list order
    const int j1 = s.lpStart[l + 1];
    for (int j0 = s.lpStart[l]; j0 < j1; j0 += 4) {
        int a[4];
#pragma unroll
        for (int u = 0; u < 4; u++) a[u] = j0 + u < j1 ? s.lpList[j0 + u] : -1;
        int pp[4], pe[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            pp[u] = a[u] >= 0 ? s.pePos[a[u]] : 0;
            pe[u] = a[u] >= 0 ? s.ePose[a[u]] : 0;
        }
        double Bv[4][18], cv[4][6];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const bd2* B = (const bd2*)(Hpl + 18 * (size_t)pp[u]);   // 16-B aligned 144-B records
            const bd2* cp = (const bd2*)(x + 6 * pe[u]);
#pragma unroll
            for (int q = 0; q < 9; q++) {
                const bd2 v = B[q];
                Bv[u][2 * q] = a[u] >= 0 ? v.x : 0.0;
                Bv[u][2 * q + 1] = a[u] >= 0 ? v.y : 0.0;
            }
#pragma unroll
            for (int r = 0; r < 3; r++) {
                const bd2 v = cp[r];
                cv[u][2 * r] = a[u] >= 0 ? v.x : 0.0;
                cv[u][2 * r + 1] = a[u] >= 0 ? v.y : 0.0;
            }
        }
#pragma unroll
        for (int u = 0; u < 4; u++) {
            if (a[u] < 0) break;
#pragma unroll
            for (int k = 0; k < 3; k++) {
                double acc = 0;
#pragma unroll
                for (int r = 0; r < 6; r++) acc += Bv[u][r * 3 + k] * (-cv[u][r]);
                cl[k] += acc;
            }
        }
    }
    double Di[9];
    land_dinv(Hll, l, lambda, Di);
    for (int r = 0; r < 3; r++) xl[r] = (Di[r * 3] * cl[0] + Di[r * 3 + 1] * cl[1]) + Di[r * 3 + 2] * cl[2];
}

__global__ void __launch_bounds__(256) k_chi2_finish(LinArgs a);

template <bool FUSE>
__global__ void __launch_bounds__(256) k_linearize_t(LinArgs a) {
    BA_GATE(a.run);
    if (FUSE && (int)blockIdx.x >= a.edgeBlocks) {   // owners: the trial's poses and points
        const int g = ((int)blockIdx.x - a.edgeBlocks) * (int)blockDim.x + (int)threadIdx.x;
        const int nP = a.s.nP;
        if (g < nP) {
            a.Tn[g] = pose_step(a.T[a.s.poseKf[g]], a.x + 6 * g);
        } else if (g - nP < a.s.nL) {
            const int l = g - nP, pt = a.s.landPt[l];
            const bool solved = a.scal[3] != 0.0;
            double xl[3];
            land_step(a.s, l, a.Hpl, a.Hll, a.bl, a.x, a.scal[5], solved, xl);
            for (int k = 0; k < 3; k++) {
                if (solved) a.x[6 * nP + 3 * l + k] = xl[k];
                a.Xn[3 * l + k] = a.X[3 * pt + k] + xl[k];
            }
        }
        return;
    }
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const bool valid = i < a.s.nE;
    double r0 = 0.0, rho1 = 1.0;
    double err[3] = {0, 0, 0};
    EdgeDev e;
    Se3 T;
    double X[3] = {0, 0, 0};
    int robust = 0;
    if (valid) {
        const int ei = a.s.aE[i];
        e = a.E[ei];
        if (FUSE) {   // the trial's pose and point of this edge (what the owners write)
            const int g = a.s.ePose[i];
            T = g >= 0 ? pose_step(a.T[e.kf], a.x + 6 * g) : a.T[e.kf];
            double xl[3];
            land_step(a.s, a.s.eLand[i], a.Hpl, a.Hll, a.bl, a.x, a.scal[5], a.scal[3] != 0.0, xl);
            for (int k = 0; k < 3; k++) X[k] = a.X[3 * e.pt + k] + xl[k];
        } else {
            T = a.T[e.kf];
            X[0] = a.X[3 * e.pt]; X[1] = a.X[3 * e.pt + 1]; X[2] = a.X[3 * e.pt + 2];
        }
        edge_error(e, T, X, err);
        for (int k = 0; k < 3; k++) a.err[3 * ei + k] = err[k];
        const double chi = edge_chi2(e, err);
        robust = a.robust[ei];
        r0 = chi;
        if (robust) huber(e, chi, &r0, &rho1);
        a.rc[i] = r0;
    }
    // activeRobustChi2: chunk tree per wave (64 consecutive active edges); k_chi2_finish sums
    // the chunks in its own launch
    {
        const double t = wave_tree(r0);
        if ((threadIdx.x & 63) == 0) a.chunks[i >> 6] = t;
    }
    if (!valid || !a.linearize) return;
    {
    // linearizeOplus (.cpp:103-147 mono, 188-234 stereo)
    double p[3], R[9], A[9], B[18];
    se3_map(T, X, p);
    quat_to_R(T.q, R);
    const double x = p[0], y = p[1], z = p[2], z_2 = z * z;
    // every x / z and x / z_2 through one reciprocal each (SharedDiv: the same correctly rounded
    // quotients as the division)
    const SharedDiv dz(z), dz2(z_2);
    const double fx = e.fx, fy = e.fy;
    const int D = e.stereo ? 3 : 2;
    if (!e.stereo) {
        const double tmp[6] = {fx, 0, dz.div(-x) * fx, 0, fy, dz.div(-y) * fy};
        const double s = dz.div(-1.);
        double st[6];
#pragma unroll
        for (int k = 0; k < 6; k++) st[k] = s * tmp[k];
#pragma unroll
        for (int r = 0; r < 2; r++)
#pragma unroll
            for (int c = 0; c < 3; c++) A[r * 3 + c] = (st[r * 3] * R[c] + st[r * 3 + 1] * R[3 + c]) + st[r * 3 + 2] * R[6 + c];
    } else {
        const double bf = e.bf;
#pragma unroll
        for (int c = 0; c < 3; c++) {
            A[0 * 3 + c] = dz.div((-fx) * R[0 * 3 + c]) + dz2.div((fx * x) * R[2 * 3 + c]);
            A[1 * 3 + c] = dz.div((-fy) * R[1 * 3 + c]) + dz2.div((fy * y) * R[2 * 3 + c]);
            A[2 * 3 + c] = A[0 * 3 + c] - dz2.div(bf * R[2 * 3 + c]);
        }
    }
    const double m1z = dz.div(-1.);
    B[0] = dz2.div(x * y) * fx;
    B[1] = (-(1 + dz2.div(x * x))) * fx;
    B[2] = dz.div(y) * fx;
    B[3] = m1z * fx;
    B[4] = 0;
    B[5] = dz2.div(x) * fx;
    B[6] = (1 + dz2.div(y * y)) * fy;
    B[7] = dz2.div((-x) * y) * fy;
    B[8] = dz.div(-x) * fy;
    B[9] = 0;
    B[10] = m1z * fy;
    B[11] = dz2.div(y) * fy;
    if (e.stereo) {
        const double bf = e.bf;
        B[12] = B[0] - dz2.div(bf * y);
        B[13] = B[1] + dz2.div(bf * x);
        B[14] = B[2];
        B[15] = B[3];
        B[16] = 0;
        B[17] = B[5] - dz2.div(bf);
    } else {
#pragma unroll
        for (int k = 12; k < 18; k++) B[k] = 0;
    }
    // constructQuadraticForm (base_binary_edge.hpp:55-120); every loop unrolled with static
    // indices (k < D as a predicate, the same k-ascending sums), so A, B, omr stay in registers
    const double w = robust ? rho1 * e.info : e.info;
    double omr[3] = {0, 0, 0};
#pragma unroll
    for (int k = 0; k < 3; k++) {
        if (k < D) {
            omr[k] = -(e.info * err[k]);
            if (robust) omr[k] *= rho1;
        }
    }
    const int nE = a.s.nE;
    double* t = a.terms;
#pragma unroll
    for (int r = 0; r < 3; r++) {
        double s = 0;
#pragma unroll
        for (int k = 0; k < 3; k++)
            if (k < D) s += A[k * 3 + r] * omr[k];
        t[(T_BL + r) * nE + i] = s;
#pragma unroll
        for (int c = 0; c < 3; c++) {
            double h = 0;
#pragma unroll
            for (int k = 0; k < 3; k++)
                if (k < D) h += (A[k * 3 + r] * w) * A[k * 3 + c];
            t[(T_HLL + r * 3 + c) * nE + i] = h;
        }
    }
    const int pp = a.s.pePos[i];   // the pose terms and Hpl at the edge's pose-list position
    if (pp < 0) return;
    double hpl[18];
#pragma unroll
    for (int r = 0; r < 6; r++) {
        double s = 0;
#pragma unroll
        for (int k = 0; k < 3; k++)
            if (k < D) s += B[k * 6 + r] * omr[k];
        t[(T_BP + r) * nE + pp] = s;
#pragma unroll
        for (int c = r; c < 6; c++) {
            double h = 0;
#pragma unroll
            for (int k = 0; k < 3; k++)
                if (k < D) h += (B[k * 6 + r] * w) * B[k * 6 + c];
            t[(T_HPP + (r * (13 - r)) / 2 + (c - r)) * nE + pp] = h;
        }
#pragma unroll
        for (int c = 0; c < 3; c++) {
            double h = 0;
#pragma unroll
            for (int k = 0; k < 3; k++)
                if (k < D) h += robust ? (B[k * 6 + r] * w) * A[k * 3 + c] : B[k * 6 + r] * (A[k * 3 + c] * e.info);
            hpl[r * 3 + c] = h;
        }
    }
    bd2* hd = (bd2*)(a.Hpl + 18 * (size_t)pp);   // the 144-B record as nine 16-B stores
#pragma unroll
    for (int q = 0; q < 9; q++) hd[q] = bd2{hpl[2 * q], hpl[2 * q + 1]};
    }
}

// the plain pass (system linearisation, host-driven trials) and the device LM's trial pass with
// the update fused in: two instances, so the plain pass keeps its registers (88 VGPRs, not 256)
static constexpr auto k_linearize = k_linearize_t<false>;
static constexpr auto k_linearize_upd = k_linearize_t<true>;

__global__ void __launch_bounds__(256) k_chi2_finish(LinArgs a) {
    BA_GATE(a.run);
    block_finish_csum(a.chunks, (a.s.nE + 63) >> 6, a.s.nE, a.rc, a.out);
}

// Reduce chunk sums arr[0..m) (already level-1 trees) to the canonical total, one wave.
__device__ __forceinline__ double wave_lds_csum(double* arr, int m) {
    const int lane = threadIdx.x & 63;
    while (m > 1) {
        const int m2 = (m + 63) >> 6;
        for (int c = 0; c < m2; c++) {
            double u = (c * 64 + lane < m) ? arr[c * 64 + lane] : 0.0;
            u = wave_tree(u);
            __builtin_amdgcn_wave_barrier();
            if (lane == 0) arr[c] = u;
            __builtin_amdgcn_wave_barrier();
        }
        m = m2;
    }
    __builtin_amdgcn_wave_barrier();
    return arr[0];
}


constexpr int kChunks = 128;  // per-list LDS chunk sums: lists up to 8192 terms
constexpr int kSysThreads = 512;   // 256 VGPRs per lane: the 27 packed chunk trees stay unspilled

// per free pose: Hpp (upper 21) and b_p as canonical sums over its active edges (edge order).
// Each lane loads the 27 terms of one edge; the 27 chunk trees run packed; chunk sums
// reduced per entry by one thread.
__device__ __forceinline__ void pose_reduce_block(const BaStructDev& s, const double* __restrict__ terms, double* Hpp,
                                                  double* bp, int i) {
    __shared__ double cs[27][kChunks];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, nw = blockDim.x >> 6;
    const int s0 = s.peStart[i], n = s.peStart[i + 1] - s0;
    const int m = (n + 63) >> 6;
    const int nE = s.nE;
    for (int c = w; c < m; c += nw) {
        const int j = c * 64 + lane;
        const bool valid = j < n;
        const int a = valid ? s0 + j : 0;   // the pose's edges' terms sit at their list positions
        double v[27];
#pragma unroll
        for (int q = 0; q < 27; q++) {
            const int col = q < 21 ? T_HPP + q : T_BP + (q - 21);
            v[q] = valid ? terms[(size_t)col * nE + a] : 0.0;
        }
        if (n == 1) {   // ora_csum keeps a single term untouched
            if (lane == 0)
#pragma unroll
                for (int q = 0; q < 27; q++) cs[q][c] = v[q];
        } else {   // the 27 canonical chunk trees, packed
            const double t = packed_trees<27>(v);
            const int q = bitrev6(lane);
            if (q < 27) cs[q][c] = t;
        }
    }
    __syncthreads();
    if (threadIdx.x < 27) {
        const int q = threadIdx.x;
        const double v = n > 0 ? local_csum_inplace(cs[q], m) : 0.0;
        if (q < 21) Hpp[21 * i + q] = v;
        else bp[6 * i + (q - 21)] = v;
    }
}

__global__ void __launch_bounds__(kSysThreads) k_pose_reduce(BaStructDev s, const double* __restrict__ terms, double* Hpp,
                                                      double* bp, const int* run) {
    BA_GATE(run);
    pose_reduce_block(s, terms, Hpp, bp, blockIdx.x);
}

// per (landmark, entry): Hll (full 3x3) and b_l over the landmark's active edges (edge order)
__global__ void __launch_bounds__(256) k_land_reduce(BaStructDev s, const double* __restrict__ terms, double* Hll,
                                                     double* bl, const int* run);
__device__ __forceinline__ double land_reduce_value(const BaStructDev& s, const double* __restrict__ terms, int g) {
    const int l = g / 12, q = g % 12;
    const int s0 = s.leStart[l], n = s.leStart[l + 1] - s0;
    const int col = q < 9 ? T_HLL + q : T_BL + (q - 9);
    const double* cp = terms + (size_t)col * s.nE;
    const int* li = s.leList + s0;
    double v;
    if (n == 1) {
        v = cp[li[0]];
    } else if (n <= 64) {
        v = tree64_local([&](int k) { return cp[li[k]]; }, n);
    } else {  // long tracks (<= 4096 edges, validated): chunk trees, then one more level
        // tree64_local over the m chunk trees without an array (scratch): its pairing tree is walked
        // depth-first, leaf t = chunk bitrev6(t), with a binary-counter stack of partial sums
        const int m = (n + 63) >> 6;
        double st[6];
        v = 0.0;
        for (int t = 0; t < 64; t++) {
            const int c = bitrev6(t);
            double u = c < m ? tree64_local([&](int k) { return cp[li[c * 64 + k]]; }, min(64, n - c * 64)) : 0.0;
#pragma unroll
            for (int lvl = 0; lvl < 6; lvl++) {
                if ((t >> lvl) & 1) {
                    u = st[lvl] + u;
                } else {
                    st[lvl] = u;
                    break;
                }
            }
            v = u;
        }
    }
    return v;
}
__device__ __forceinline__ void land_reduce_thread(const BaStructDev& s, const double* __restrict__ terms, double* Hll,
                                                   double* bl, int g) {
    if (g >= 12 * s.nL) return;
    const int l = g / 12, q = g % 12;
    const double v = land_reduce_value(s, terms, g);
    if (q < 9) Hll[9 * l + q] = v;
    else bl[3 * l + (q - 9)] = v;
}

// Threads landmark-major (thread g: entry g mod 12 of landmark g / 12).  Measured against the
// entry-major mapping (one SoA column over neighbouring landmarks per wave load): 178 vs 232 us
// per config-5 launch (gpurun_out r06o2 / r06t), the twelve columns of a landmark's few edges
// share their lines in L2.
__global__ void __launch_bounds__(256) k_land_reduce(BaStructDev s, const double* __restrict__ terms, double* Hll,
                                                     double* bl, const int* run) {
    BA_GATE(run);
    land_reduce_thread(s, terms, Hll, bl, blockIdx.x * blockDim.x + threadIdx.x);
}

// both reductions of buildSystem in one launch: blocks [0, nP) reduce a pose each, the rest
// a (landmark, entry) per thread
__global__ void __launch_bounds__(kSysThreads) k_sys_reduce(BaStructDev s, const double* __restrict__ terms, double* Hpp,
                                                     double* bp, double* Hll, double* bl, const int* run) {
    BA_GATE(run);
    if ((int)blockIdx.x < s.nP) pose_reduce_block(s, terms, Hpp, bp, blockIdx.x);
    else land_reduce_thread(s, terms, Hll, bl, (blockIdx.x - s.nP) * blockDim.x + threadIdx.x);
}

// computeLambdaInit: tau * max |diag| over poses and landmarks (order-free max)
__global__ void __launch_bounds__(1024) k_lambda_init(int nP, int nL, const double* Hpp, const double* Hll,
                                                      double* scal, const int* run) {
    BA_GATE(run);
    __shared__ double red[1024];
    double m = 0.;
    for (int j = threadIdx.x; j < 6 * nP + 3 * nL; j += blockDim.x) {
        const double d = j < 6 * nP ? Hpp[21 * (j / 6) + DIAG21[j % 6]] : Hll[9 * ((j - 6 * nP) / 3) + 4 * ((j - 6 * nP) % 3)];
        m = fmax(fabs(d), m);
    }
    red[threadIdx.x] = m;
    __syncthreads();
    for (int o = 512; o >= 1; o >>= 1) {
        if ((int)threadIdx.x < o) red[threadIdx.x] = fmax(red[threadIdx.x], red[threadIdx.x + o]);
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        scal[4] = red[0];
        scal[5] = 1e-5 * red[0];
    }
}

__device__ __forceinline__ double lam_of(double lam_host, int use_dev, const double* scal) {
    return use_dev ? scal[5] : lam_host;
}

// per active edge with a free pose: BDinv = Hpl Dinv and B (Dinv b_l)  (block_solver.hpp:376-404);
// H9 / b3: the landmark's Hll and b_l, a: the edge's pose-list position
__device__ __forceinline__ void prep_entry(const double* H9, const double* b3, double lambda,
                                           const double* __restrict__ Hpl, int a, double* Emat, double* cb) {
    double Di[9], d[3];
    land_dinv(H9, 0, lambda, Di);
    const double b[3] = {b3[0], b3[1], b3[2]};
    for (int r = 0; r < 3; r++) d[r] = (Di[r * 3] * b[0] + Di[r * 3 + 1] * b[1]) + Di[r * 3 + 2] * b[2];
    // the 144-B Hpl record in, the 144-B E record and 48-B c_b record out as 16-B accesses
    double Bi[18], Eo[18], co[6];
    {
        const bd2* src = (const bd2*)(Hpl + 18 * (size_t)a);
#pragma unroll
        for (int q = 0; q < 9; q++) {
            const bd2 v = src[q];
            Bi[2 * q] = v.x;
            Bi[2 * q + 1] = v.y;
        }
    }
#pragma unroll
    for (int r = 0; r < 6; r++) {
        const double b0 = Bi[r * 3], b1 = Bi[r * 3 + 1], b2 = Bi[r * 3 + 2];
#pragma unroll
        for (int k = 0; k < 3; k++) Eo[r * 3 + k] = (b0 * Di[k] + b1 * Di[3 + k]) + b2 * Di[6 + k];
        co[r] = (b0 * d[0] + b1 * d[1]) + b2 * d[2];
    }
    bd2* Ed = (bd2*)(Emat + 18 * (size_t)a);
    bd2* cd = (bd2*)(cb + 6 * (size_t)a);
#pragma unroll
    for (int q = 0; q < 9; q++) Ed[q] = bd2{Eo[2 * q], Eo[2 * q + 1]};
#pragma unroll
    for (int q = 0; q < 3; q++) cd[q] = bd2{co[2 * q], co[2 * q + 1]};
}

__global__ void __launch_bounds__(256) k_point_prep(BaStructDev s, const double* Hll, const double* bl,
                                                    const double* __restrict__ Hpl, double lam_host, int use_dev,
                                                    const double* scal, double* Emat, double* cb, const int* run) {
    BA_GATE(run);
    const int a = blockIdx.x * blockDim.x + threadIdx.x;   // pose-list position
    if (a >= s.nPe) return;
    const int l = s.eLand[s.peList[a]];
    prep_entry(Hll + 9 * l, bl + 3 * l, lam_of(lam_host, use_dev, scal), Hpl, a, Emat, cb);
}

// The device LM's steps after the first (lambda already on the device): buildSystem's reductions
// and k_point_prep in one launch.  Blocks [0, nP) reduce a pose each (system gate ctl[1]); each
// later block reduces kLandBlk whole landmarks (12 threads per landmark, ctl[1]) and then, under
// the trial gate ctl[0], preps the pose-list entries of those landmarks (their lpList edges) from
// the values it just reduced -- or, on a rejected trial's step (system gated off), from Hll / b_l
// as the last system left them.  Same values as k_sys_reduce + k_point_prep.
constexpr int kLandBlk = kSysThreads / 12;
__global__ void __launch_bounds__(kSysThreads) k_sys_reduce_prep(BaStructDev s, const double* __restrict__ terms,
                                                                 double* Hpp, double* bp, double* Hll, double* bl,
                                                                 const double* __restrict__ Hpl, const double* scal,
                                                                 double* Emat, double* cb, const int* ctl) {
    __shared__ double sH[kLandBlk * 9], sB[kLandBlk * 3];
    const bool sys = ctl[1] != 0, trial = ctl[0] != 0;
    if (!sys && !trial) return;
    if ((int)blockIdx.x < s.nP) {
        if (sys) pose_reduce_block(s, terms, Hpp, bp, blockIdx.x);
        return;
    }
    const int l0 = ((int)blockIdx.x - s.nP) * kLandBlk, l1 = min(s.nL, l0 + kLandBlk);
    const int t = threadIdx.x;
    if (sys && t < 12 * kLandBlk) {
        const int g = 12 * l0 + t;
        if (g < 12 * l1) {
            const int l = g / 12, q = g % 12;
            const double v = land_reduce_value(s, terms, g);
            if (q < 9) {
                Hll[9 * l + q] = v;
                sH[9 * (l - l0) + q] = v;
            } else {
                bl[3 * l + (q - 9)] = v;
                sB[3 * (l - l0) + (q - 9)] = v;
            }
        }
    }
    if (!trial) return;
    __syncthreads();
    const double lambda = scal[5];
    for (int j = s.lpStart[l0] + t; j < s.lpStart[l1]; j += blockDim.x) {
        const int e = s.lpList[j], l = s.eLand[e];
        const double* H9 = sys ? sH + 9 * (l - l0) : Hll + 9 * l;
        const double* b3 = sys ? sB + 3 * (l - l0) : bl + 3 * l;
        prep_entry(H9, b3, lambda, Hpl, s.pePos[e], Emat, cb);
    }
}

// Schur complement block (i1, i2): S = [Hpp + lambda I] - csum_l BDinv_l,i1 B_l,i2^T
// (upper triangle of the diagonal blocks), and b_s = b_p - csum_l B db.
// Each lane loads the two 6x3 blocks of one landmark term once and feeds all entries; a chunk's
// 27 / 36 canonical 64-trees run packed (packed_trees: every value's tree is the canonical one).
// NT = 256 for systems of many blocks (global BA): a workgroup takes one diagonal block with its
// four waves (the blocks of the poses' own edges, the longest), or four off-diagonal blocks, one
// wave each (most hold one or two chunks: a wave per block keeps four times the blocks in
// flight); the chunk sums in dynamic LDS sized by the longest block (ldc chunks).  512 for the
// few long blocks of a local BA (chunk sums in static LDS, ldc = kChunks).
template <int NT>
__global__ void __launch_bounds__(NT) k_schur(BaStructDev s, const double* __restrict__ Emat,
                                              const double* __restrict__ Hpl, const double* __restrict__ cb,
                                              const double* Hpp, const double* bp, double lam_host, int use_dev,
                                              const double* scal, SysAddr S, double* bs, int own,
                                              const uint8_t* poseAdd, const int* run, int ldcDyn) {
    BA_GATE(run);
    ORBGPU_PROF_START;
#ifdef ORBGPU_PROF
    const unsigned long long tBlk0 = clock64();   // (instrumented builds: per-wave block durations)
#endif
    constexpr bool kMixed = NT == 256;
    __shared__ double csS[kMixed ? 1 : 36 * kChunks];
    extern __shared__ double lds[];
    const int ldc = kMixed ? ldcDyn : kChunks;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    // the block's waves: all of the workgroup (group) or this wave alone
    const bool group = !kMixed || (int)blockIdx.x < s.nP;
    const int blk = group ? (int)blockIdx.x : s.nP + ((int)blockIdx.x - s.nP) * 4 + wave;
    if (blk >= s.nBlk) return;   // (wave-uniform: only a per-wave block can be past the end)
    const int w = group ? wave : 0, nw = group ? (int)(blockDim.x >> 6) : 1;
    const int tq = group ? (int)threadIdx.x : lane;   // the thread's index inside the block's waves
    double* cs = !kMixed ? csS : (group ? lds : lds + (size_t)wave * 36 * ldc);   // cs[q * ldc + c]
    const int i1 = s.blkI[blk], i2 = s.blkJ[blk];
    const int s0 = s.blkStart[blk], n = s.blkStart[blk + 1] - s0;
    const int m = (n + 63) >> 6;
    const bool diag = i1 == i2;
    const int nent = diag ? 27 : 36;
    // the next chunk's pair entries are loaded one iteration ahead: a chunk's record loads then
    // wait on one memory round trip, not two
    int a1n = 0, a2n = 0;
    if (w < m && w * 64 + lane < n) {
        a1n = s.pairA[s0 + w * 64 + lane];
        a2n = s.pairB[s0 + w * 64 + lane];
    }
    for (int c = w; c < m; c += nw) {
        const int j = c * 64 + lane;
        const bool valid = j < n;
        const int a1 = valid ? a1n : 0, a2 = valid ? a2n : 0;
        {
            const int jn = j + 64 * nw;
            a1n = jn < n ? s.pairA[s0 + jn] : 0;
            a2n = jn < n ? s.pairB[s0 + jn] : 0;
        }
        // the two 144-B records as nine 16-B loads each (records are 16-B aligned in the arena):
        // half the gather instructions of element-wise 8-B loads
        double E[18], B[18];
        {
            typedef double d2 __attribute__((ext_vector_type(2)));
            const d2* Er = (const d2*)(Emat + 18 * (size_t)a1);
            const d2* Br = (const d2*)(Hpl + 18 * (size_t)a2);
#pragma unroll
            for (int q = 0; q < 9; q++) {
                const d2 e = Er[q], b = Br[q];   // (a1 = a2 = 0 on invalid lanes: in bounds)
                E[2 * q] = valid ? e.x : 0.0;
                E[2 * q + 1] = valid ? e.y : 0.0;
                B[2 * q] = valid ? b.x : 0.0;
                B[2 * q + 1] = valid ? b.y : 0.0;
            }
        }
        auto put = [&](double* v, auto kk) {
            constexpr int K = decltype(kk)::value;
            if (n == 1) {   // ora_csum keeps a single term untouched
                if (lane == 0)
#pragma unroll
                    for (int q = 0; q < K; q++) cs[q * ldc + c] = v[q];
            } else {
                const double t = packed_trees<K>(v);
                const int q = bitrev6(lane);
                if (q < K) cs[q * ldc + c] = t;
            }
        };
        if (diag) {
            double v[27];
            int q = 0;
#pragma unroll
            for (int r = 0; r < 6; r++)
#pragma unroll
                for (int cc = r; cc < 6; cc++, q++)
                    v[q] = valid ? (E[r * 3] * B[cc * 3] + E[r * 3 + 1] * B[cc * 3 + 1]) + E[r * 3 + 2] * B[cc * 3 + 2] : 0.0;
#pragma unroll
            for (int r = 0; r < 6; r++) v[21 + r] = valid ? cb[6 * (size_t)a1 + r] : 0.0;
            put(v, std::integral_constant<int, 27>{});
        } else {
            double v[36];
#pragma unroll
            for (int r = 0; r < 6; r++)
#pragma unroll
                for (int cc = 0; cc < 6; cc++)
                    v[r * 6 + cc] = valid ? (E[r * 3] * B[cc * 3] + E[r * 3 + 1] * B[cc * 3 + 1]) + E[r * 3 + 2] * B[cc * 3 + 2] : 0.0;
            put(v, std::integral_constant<int, 36>{});
        }
    }
    ORBGPU_PROF_MARK(11);   // (instrumented builds: block 0's wave 0 -- chunk terms and trees)
#ifdef ORBGPU_PROF
    if (kMixed && lane == 0) {   // the many-block launch: log2 histogram of the waves' chunk phases
        const unsigned long long dt = clock64() - tBlk0;
        int bkt = 63 - __builtin_clzll(dt | 1ull) - 10;
        bkt = bkt < 0 ? 0 : (bkt > 9 ? 9 : bkt);
        atomicAdd(&g_orbgpu_prof[bkt], 1ull);
        atomicAdd(&g_orbgpu_prof[group ? 10 : 14], dt);
    }
#endif
    if (group) {
        __syncthreads();
    } else {
        __builtin_amdgcn_s_waitcnt(0);
        __builtin_amdgcn_wave_barrier();
    }
    ORBGPU_PROF_MARK(12);
    ORBGPU_PROF_COUNT(15);
    if (tq >= nent) return;
    const int q = tq;
    const double v = local_csum_inplace(cs + q * ldc, m);
    ORBGPU_PROF_MARK(13);
    const double lambda = lam_of(lam_host, use_dev, scal);
    if (poseAdd) own = poseAdd[i1];   // sharded factorisation: the pose's owner adds its terms
    if (diag && q >= 21) {  // a shard that does not own the pose terms contributes -sum only
        bs[6 * i1 + (q - 21)] = (own ? bp[6 * i1 + (q - 21)] : 0.0) - v;
        return;
    }
    int r, c;
    if (diag) {
        r = 0;
        while (r < 5 && q >= DIAG21[r + 1]) r++;
        c = r + (q - DIAG21[r]);
    } else {
        r = q / 6;
        c = q % 6;
    }
    double h = 0;
    if (diag && own) {
        h = Hpp[21 * i1 + q];
        if (c == r) h += lambda;
    }
    *S.at(6 * i1 + r, 6 * i2 + c) = h - v;
}

// ldc: chunks of the longest block (the one-wave kernel's LDS rows)
template <class... A>
static void schur_launch(int nBlk, int ldc, hipStream_t st, A... args) {
    if (nBlk >= 256) {
        const int nP = std::get<0>(std::make_tuple(args...)).nP;   // the leading diagonal blocks
        hipLaunchKernelGGL(k_schur<256>, dim3(nP + (nBlk - nP + 3) / 4), dim3(256),
                           sizeof(double) * 4 * 36 * (size_t)std::max(ldc, 1), st, args..., std::max(ldc, 1));
    }
    else
        hipLaunchKernelGGL(k_schur<512>, dim3(nBlk), dim3(512), 0, st, args..., kChunks);
}

// Dense LDL^T of the upper triangle + solve, one workgroup (256 threads).
// Same per-element operation sequence as oracle ora_ldlt_solve, blocked by 6-column panels:
// wave 0 factorises the panel rows and writes L (lower triangle), then every wave
// applies the panel's rank-1 updates, in k order, to its trailing rows.
__global__ void __launch_bounds__(256) k_ldlt(int n, double* Sg, const double* bs, double* x, double* scal, int in_lds,
                                              const int* run) {
    BA_GATE(run);
    extern __shared__ double lds[];
    double* y = lds;            // n
    double* A = in_lds ? lds + n : Sg;
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    __shared__ int ok;
    if (in_lds)
        for (int q = tid; q < n * n; q += blockDim.x) A[q] = Sg[q];
    for (int q = tid; q < n; q += blockDim.x) y[q] = bs[q];
    if (tid == 0) ok = 1;
    __syncthreads();
    for (int p0 = 0; p0 < n; p0 += 6) {
        const int p1 = min(p0 + 6, n);
        if (w == 0) {
            for (int k = p0; k < p1; k++) {
                const double d = A[(size_t)k * n + k];
                if (d == 0.0) {
                    if (lane == 0) ok = 0;
                    break;
                }
                for (int i = k + 1 + lane; i < n; i += 64) A[(size_t)i * n + k] = A[(size_t)k * n + i] / d;
                __builtin_amdgcn_wave_barrier();
                for (int i = k + 1; i < p1; i++) {
                    const double li = A[(size_t)i * n + k];
                    for (int j = i + lane; j < n; j += 64) A[(size_t)i * n + j] -= li * A[(size_t)k * n + j];
                }
                __builtin_amdgcn_wave_barrier();
            }
        }
        __syncthreads();
        if (!ok) break;
        for (int i = p1 + w; i < n; i += 4) {
            double L[6];
            for (int k = p0; k < p1; k++) L[k - p0] = A[(size_t)i * n + k];
            for (int j = i + lane; j < n; j += 64) {
                double v = A[(size_t)i * n + j];
                for (int k = p0; k < p1; k++) v -= L[k - p0] * A[(size_t)k * n + j];
                A[(size_t)i * n + j] = v;
            }
        }
        __syncthreads();
    }
    if (!ok) {
        if (tid == 0) scal[3] = 0.0;
        return;
    }
    if (w == 0) {
        // L y = b: per row, subtractions in k order (column-sweep order of the oracle)
        for (int r0 = 0; r0 < n; r0 += 64) {
            const int i = r0 + lane;
            double acc = i < n ? y[i] : 0.0;
            for (int k = 0; k < r0; k++)
                if (i < n) acc -= A[(size_t)i * n + k] * y[k];
            for (int k = r0; k < min(r0 + 64, n); k++) {
                const double yk = __shfl(acc, k - r0, 64);
                if (i > k && i < n) acc -= A[(size_t)i * n + k] * yk;
            }
            if (i < n) y[i] = acc;
            __builtin_amdgcn_wave_barrier();
        }
        for (int k = lane; k < n; k += 64) y[k] = y[k] / A[(size_t)k * n + k];
        __builtin_amdgcn_wave_barrier();
        // L^T x = z: per row, subtractions in descending k order
        for (int r1 = n; r1 > 0; r1 -= 64) {
            const int r0 = max(r1 - 64, 0);
            const int i = r0 + lane;
            double acc = i < r1 ? y[i] : 0.0;
            for (int k = n - 1; k >= r1; k--)
                if (i < r1) acc -= A[(size_t)k * n + i] * y[k];
            for (int k = r1 - 1; k >= r0; k--) {
                const double yk = __shfl(acc, k - r0, 64);
                if (i < k) acc -= A[(size_t)k * n + i] * yk;
            }
            if (i < r1) y[i] = acc;
            __builtin_amdgcn_wave_barrier();
        }
        for (int k = lane; k < n; k += 64) x[k] = y[k];
        if (lane == 0) scal[3] = 1.0;
    }
}

__device__ __forceinline__ double readlane_d(double v, int l) {
    const unsigned long long u = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)(u & 0xffffffffu), l);
    const int hi = __builtin_amdgcn_readlane((int)(u >> 32), l);
    return __longlong_as_double(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}

// z = D^-1 y, then L^T x = z (per row, subtractions in descending k order; L[k][i] =
// Lall[i * n + k]) by one wave; y is overwritten.  The oracle's ora_ldlt_solve sequence.
__device__ __forceinline__ void ldlt_backward_wave(int n, const double* Lall, const double* dvec, double* y, double* x,
                                                   double* scal) {
    const int lane = threadIdx.x & 63;
    for (int k = lane; k < n; k += 64) y[k] = y[k] / dvec[k];
    __builtin_amdgcn_wave_barrier();
    for (int r1 = n; r1 > 0; r1 -= 64) {
        const int r0 = max(r1 - 64, 0);
        const int i = r0 + lane;
        const bool on = i < r1;
        const int ic = on ? i : r0;
        double acc = on ? y[i] : 0.0;
        int k = n - 1;
        for (; k - 8 >= r1 - 1; k -= 8) {
            double L8[8], Y8[8];
#pragma unroll
            for (int u = 0; u < 8; u++) {
                L8[u] = Lall[(size_t)ic * n + (k - u)];
                Y8[u] = y[k - u];
            }
#pragma unroll
            for (int u = 0; u < 8; u++) acc -= L8[u] * Y8[u];
        }
        for (; k >= r1; k--) acc -= Lall[(size_t)ic * n + k] * y[k];
        k = r1 - 1;
        for (; k - 8 >= r0 - 1; k -= 8) {
            double L8[8];
#pragma unroll
            for (int u = 0; u < 8; u++) L8[u] = Lall[(size_t)ic * n + (k - u)];
#pragma unroll
            for (int u = 0; u < 8; u++) {
                const double yk = readlane_d(acc, k - u - r0);
                if (i < k - u) acc -= L8[u] * yk;
            }
        }
        for (; k >= r0; k--) {
            const double yk = readlane_d(acc, k - r0);
            if (i < k) acc -= Lall[(size_t)ic * n + k] * yk;
        }
        if (on) y[i] = acc;
        __builtin_amdgcn_wave_barrier();
    }
    for (int k = lane; k < n; k += 64) x[k] = y[k];
    if (lane == 0) scal[3] = 1.0;
}

// Row-owner LDL^T + forward substitution for n <= kLdltRowMax (16 free keyframes: a local BA),
// two waves.  Thread i holds row i of [S | b] (its upper part, j >= i) in registers.  At pivot
// k, row k -- final after its k updates -- sits in LDS (published by its owner at the end of
// pivot k - 1, double-buffered); every row i > k forms l_ik = u_ki / d_k and subtracts
// l_ik * u_kj from each of its entries, k ascending per element: the oracle's ora_ldlt_solve
// sequence (the right-hand side, column n, runs the forward substitution y_i -= l_ik y_k).
// Row k + 1 then publishes itself: one barrier per pivot, no panel round trips.
constexpr int kLdltRowMax = 96;
__global__ void __launch_bounds__(128) k_ldlt_row(int n, const double* __restrict__ Sg, const double* bs, double* x,
                                                  double* scal, const int* run) {
    BA_GATE(run);
    __shared__ double Ur[2][kLdltRowMax + 1];   // published row k: entries j < n, b_k at [kLdltRowMax]
    __shared__ double Lall[kLdltRowMax * kLdltRowMax];   // L[i][k] at Lall[k * n + i]
    __shared__ double dvec[kLdltRowMax], y[kLdltRowMax];
    const int i = threadIdx.x;
    const bool mine = i < n;
    double a[kLdltRowMax];
#pragma unroll
    for (int j = 0; j < kLdltRowMax; j++) a[j] = (mine && j < n && j >= i) ? Sg[(size_t)i * n + j] : 0.0;
    double bi = mine ? bs[i] : 0.0;
    if (i == 0) {
#pragma unroll
        for (int j = 0; j < kLdltRowMax; j++)
            if (j < n) Ur[0][j] = a[j];
        Ur[0][kLdltRowMax] = bi;
    }
    __syncthreads();
    bool ok = true;
    for (int k = 0; k < n; k++) {
        const double* U = Ur[k & 1];
        const double d = U[k];
        if (d == 0.0) {   // uniform: every thread reads the same pivot
            ok = false;
            break;
        }
        if (i == 0) {
            dvec[k] = d;
            y[k] = U[kLdltRowMax];   // b_k after its k updates: forward-substituted y_k
        }
        if (i > k && mine) {
            const double l = U[i] / d;
            Lall[(size_t)k * n + i] = l;
#pragma unroll
            for (int c = 0; c < kLdltRowMax / 8; c++) {
                if (8 * c + 7 < i) continue;
#pragma unroll
                for (int q = 0; q < 8; q++) {
                    const int j = 8 * c + q;
                    if (j >= i && j < n) a[j] -= l * U[j];
                }
            }
            bi -= l * U[kLdltRowMax];
            if (i == k + 1) {   // row k + 1 is final: publish it for the next pivot
                double* V = Ur[(k + 1) & 1];
#pragma unroll
                for (int j = 0; j < kLdltRowMax; j++)
                    if (j >= i && j < n) V[j] = a[j];
                V[kLdltRowMax] = bi;
            }
        }
        __syncthreads();
    }
    if (!ok) {
        if (i == 0) scal[3] = 0.0;
        return;
    }
    if (i >= 64) return;
    ldlt_backward_wave(n, Lall, dvec, y, x, scal);
}

// Column-owner LDL^T + solve for n <= kLdltColMax (16 free keyframes: a local BA), 4 waves.
// Lane c owns columns c and c + 64 of [S | b] (b in column n); wave w owns rows i = 4 r + w,
// so a thread holds A[i][c] for its wave's rows in registers.  Pivot k: the pivot row (final
// after k updates) sits in LDS, published by its owner at the end of pivot k - 1 (double-
// buffered); every thread forms l_ck = u_kc / d_k for its columns (two lane-parallel quotients,
// one reciprocal), the wave reads back the l of its own rows, and subtracts l_ik u_kj from its
// rows, k ascending per element: the oracle's ora_ldlt_solve sequence (column n runs the
// forward substitution y_i -= l_ik y_k).  The owner of row k + 1 updates that row first and
// publishes it, one barrier per pivot.  The pivot loop is rolled: its body (24 rows x 2
// columns) stays in the instruction cache, unlike a fully unrolled 90-pivot chain.
constexpr int kLdltColMax = 96;
constexpr int kLdltColRows = kLdltColMax / 4;
__global__ void __launch_bounds__(256) k_ldlt_col(int n, const double* __restrict__ Sg, const double* bs, double* x,
                                                  double* scal, const int* run) {
    BA_GATE(run);
    __shared__ double Ur[2][128];                        // published row k: columns 0..n (b at n)
    __shared__ double Lall[kLdltColMax * kLdltColMax];   // L[i][k] at Lall[k * n + i]
    __shared__ __attribute__((aligned(16))) double lw[4][kLdltColRows + 8];   // l_ik of wave w's rows (r = i / 4)
    __shared__ double dvec[kLdltColMax], y[kLdltColMax];
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    const int c0 = lane, c1 = lane + 64;
    double A0[kLdltColRows], A1[kLdltColRows];
#pragma unroll
    for (int r = 0; r < kLdltColRows; r++) {
        const int i = 4 * r + w;
        const bool row = i < n;
        A0[r] = (row && c0 < n && c0 >= i) ? Sg[(size_t)i * n + c0] : (row && c0 == n) ? bs[i] : 0.0;
        A1[r] = (row && c1 < n && c1 >= i) ? Sg[(size_t)i * n + c1] : (row && c1 == n) ? bs[i] : 0.0;
    }
    if (w == 0) {
        Ur[0][c0] = A0[0];
        Ur[0][c1] = A1[0];
    }
    __syncthreads();
    bool ok = true;
    for (int k = 0; k < n; k++) {
        const double* U = Ur[k & 1];
        double* V = Ur[(k + 1) & 1];
        const double d = U[k];
        if (d == 0.0) {   // uniform: every thread reads the same pivot
            ok = false;
            break;
        }
        const double u0 = U[c0], u1 = U[c1];
        const int own = (k + 1) & 3;   // the wave of row k + 1
        if (w == own) {
            // row k + 1 first: its l from the broadcast u_{k,k+1} (the same quotient lane k + 1 forms)
            const int r1 = (k + 1) >> 2;
            const double l1 = U[k + 1 < n ? k + 1 : k] / d;
#pragma unroll
            for (int r = 0; r < kLdltColRows; r++)
                if (r == r1 && k + 1 < n) {
                    A0[r] -= l1 * u0;
                    A1[r] -= l1 * u1;
                    V[c0] = A0[r];
                    V[c1] = A1[r];
                }
        }
        // plain divisions: two cost 160 cycles, one reciprocal shared by two 324
        // (tools/micro/ldlt_col.hip)
        const double l0 = u0 / d, l1v = u1 / d;
        if (w == 0) {
            if (c0 > k && c0 < n) Lall[k * n + c0] = l0;
            if (c1 > k && c1 < n) Lall[k * n + c1] = l1v;
            if (lane == 0) {
                dvec[k] = d;
                y[k] = U[n];   // b_k after its k updates: the forward-substituted y_k
            }
        }
        if ((lane & 3) == w) {   // the l of this wave's rows, c = 4 r + w
            lw[w][lane >> 2] = l0;
            lw[w][16 + (lane >> 2)] = l1v;
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0): the wave's own LDS writes are visible
        __builtin_amdgcn_wave_barrier();
        // rows i = 4 r + w > k + 1 (row k + 1 was done above), four at a time: a group with a live
        // row loads its four l together and updates branch-free (a branch per row serialised the
        // LDS latency of every row: 2.1 k cycles per pivot, tools/micro/ldlt_col.hip)
        const int rlive = (k + 5 - w) >> 2;   // first r with 4 r + w >= k + 2
#pragma unroll
        for (int g = 0; g < kLdltColRows / 4; g++) {
            if (4 * g + 3 >= rlive && 16 * g + w < n) {
                const double2 la = *reinterpret_cast<const double2*>(&lw[w][4 * g]);
                const double2 lb = *reinterpret_cast<const double2*>(&lw[w][4 * g + 2]);
                const double lv[4] = {la.x, la.y, lb.x, lb.y};
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const int r = 4 * g + q, i = 4 * r + w;
                    const bool live = i > k + 1 && i < n;
                    const double v0 = A0[r] - lv[q] * u0, v1 = A1[r] - lv[q] * u1;
                    A0[r] = live ? v0 : A0[r];
                    A1[r] = live ? v1 : A1[r];
                }
            }
        }
        __syncthreads();
    }
    if (!ok) {
        if (tid == 0) scal[3] = 0.0;
        return;
    }
    if (w != 0) return;
    ldlt_backward_wave(n, Lall, dvec, y, x, scal);
}

// Row-lane LDL^T + solve for n <= kLdltColMax, 4 waves: lane i owns rows i and i + 64 of
// [S | b] (b in column n), wave w the columns j = 4 r + w (r <= 24).  Pivot k: the published row
// k (final after k updates) sits in LDS, permuted so a wave's columns are contiguous; every lane
// forms its rows' l_ik = u_ki / d_k itself (no l broadcast), reads u_kj of its wave's live
// columns as broadcasts and subtracts l_ik u_kj, k ascending per element: the oracle's
// ora_ldlt_solve sequence (column n runs the forward substitution).  Then lane k + 1 publishes
// its row; one barrier per pivot.  Rows at or above the pivot and lower-triangle entries carry
// values nobody reads, so the updates need no per-row predicate.
constexpr int kLdltTCols = kLdltColMax / 4 + 1;   // 25 columns per wave: j <= 96 covers b at n <= 96
__global__ void __launch_bounds__(256) k_ldlt_t(int n, const double* __restrict__ Sg, const double* bs, double* x,
                                                double* scal, const int* run) {
    BA_GATE(run);
    __shared__ __attribute__((aligned(16))) double Up[2][4][kLdltTCols + 3];   // row k: Up[.][j & 3][j >> 2]
    __shared__ double Lall[kLdltColMax * kLdltColMax];   // S staging, then L[i][k] at Lall[k * n + i]
    __shared__ double dvec[kLdltColMax], y[kLdltColMax];
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    const int i0 = lane, i1 = lane + 64;
    // S through LDS: coalesced global reads, then each lane its rows
    for (int q = tid; q < n * n; q += 256) Lall[q] = Sg[q];
    __syncthreads();
    double A0[kLdltTCols], A1[kLdltTCols];
#pragma unroll
    for (int r = 0; r < kLdltTCols; r++) {
        const int j = 4 * r + w;
        A0[r] = (i0 < n && j < n && j >= i0) ? Lall[i0 * n + j] : (i0 < n && j == n) ? bs[i0] : 0.0;
        A1[r] = (i1 < n && j < n && j >= i1) ? Lall[i1 * n + j] : (i1 < n && j == n) ? bs[i1] : 0.0;
    }
    if (lane == 0) {   // row 0
#pragma unroll
        for (int r = 0; r < kLdltTCols; r++) Up[0][w][r] = A0[r];
    }
    __syncthreads();   // the staging area is free for L from here
    bool ok = true;
    for (int k = 0; k < n; k++) {
        const double(*U)[kLdltTCols + 3] = Up[k & 1];
        const double d = U[k & 3][k >> 2];
        if (d == 0.0) {   // uniform
            ok = false;
            break;
        }
        // this lane's rows: l = u_ki / d_k (rows <= k compute values nobody reads)
        const double l0 = k < 63 ? U[i0 & 3][i0 >> 2] / d : 0.0;
        const double l1 = n > 64 ? U[i1 & 3][i1 >> 2] / d : 0.0;
        if (w == 0) {
            if (i0 > k && i0 < n) Lall[k * n + i0] = l0;
            if (i1 > k && i1 < n) Lall[k * n + i1] = l1;
            if (lane == 0) {
                dvec[k] = d;
                y[k] = U[n & 3][n >> 2];   // b_k after its k updates: the forward-substituted y_k
            }
        }
        // live columns j > k of this wave, four at a time (a uniform skip of dead groups)
        const int rlive = (k + 4 - w) >> 2;   // first r with 4 r + w >= k + 1
#pragma unroll
        for (int g = 0; g < (kLdltTCols + 3) / 4; g++) {
            if (4 * g + 3 >= rlive && 16 * g + w <= n) {
                const double2 ua = *reinterpret_cast<const double2*>(&U[w][4 * g]);
                const double2 ub = *reinterpret_cast<const double2*>(&U[w][4 * g + 2]);
                const double uv[4] = {ua.x, ua.y, ub.x, ub.y};
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const int r = 4 * g + q;
                    if (r < kLdltTCols) {
                        if (k < 63) A0[r] -= l0 * uv[q];
                        if (n > 64) A1[r] -= l1 * uv[q];
                    }
                }
            }
        }
        // row k + 1 is final: its lane publishes this wave's columns
        const int kp = k + 1;
        if (kp < n && (kp < 64 ? lane == kp : lane == kp - 64)) {
            double* V = Up[kp & 1][w];
            if (kp < 64) {   // two loops: a select of the arrays would move them to scratch
#pragma unroll
                for (int r = 0; r < kLdltTCols; r++) V[r] = A0[r];
            } else {
#pragma unroll
                for (int r = 0; r < kLdltTCols; r++) V[r] = A1[r];
            }
        }
        __syncthreads();
    }
    if (!ok) {
        if (tid == 0) scal[3] = 0.0;
        return;
    }
    if (w != 0) return;
    ldlt_backward_wave(n, Lall, dvec, y, x, scal);
}

// 2-D block-cyclic LDL^T + solve for n <= kLdltColMax, 4 waves: thread (a, b) holds A[i][j] for
// i = 16 r + a, j = 16 c + b of [S | b] (b in column n); a wave holds four row classes, so a
// register row or column past the live part of the matrix is skipped by the whole wave.  Per
// panel of 8 pivots: the owners publish the panel rows, wave 0 factors them right-looking
// (lane = column: l_jk = u_kj / d_k lane-parallel, the later panel rows updated with the l read
// back by readlane), writing the final U rows and the L columns to LDS, then every thread
// applies the panel's pivots, ascending, to its live entries.  Per element the oracle's
// ora_ldlt_solve sequence; two barriers per panel.
constexpr int k2dPW = 8, k2dR = 6, k2dC = 7;   // panel width; rows 16 r + a (r < 6), columns 16 c + b (c < 7)
__global__ void __launch_bounds__(256) k_ldlt_2d(int n, const double* __restrict__ Sg, const double* bs, double* x,
                                                 double* scal, const int* run) {
    BA_GATE(run);
    __shared__ double Lall[kLdltColMax * kLdltColMax];   // S staging, then L[i][k] at Lall[k * n + i]
    __shared__ double UP[k2dPW][128];                    // the panel's final U rows, columns 0..n
    __shared__ double Pn[k2dPW][128];                    // the panel rows as published
    __shared__ double dvec[kLdltColMax], y[kLdltColMax];
    __shared__ int ok;
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    const int a = 4 * w + (lane & 3), b = lane >> 2;
    for (int q = tid; q < n * n; q += 256) Lall[q] = Sg[q];
    if (tid == 0) ok = 1;
    __syncthreads();
    double A[k2dR][k2dC];
#pragma unroll
    for (int r = 0; r < k2dR; r++)
#pragma unroll
        for (int c = 0; c < k2dC; c++) {
            const int i = 16 * r + a, j = 16 * c + b;
            A[r][c] = (i < n && j < n && j >= i) ? Lall[i * n + j] : (i < n && j == n) ? bs[i] : 0.0;
        }
    for (int p0 = 0; p0 < n; p0 += k2dPW) {
        const int p1 = min(p0 + k2dPW, n);
        // the panel rows' current values (final: every earlier panel is applied)
#pragma unroll
        for (int r = 0; r < k2dR; r++) {
            const int i = 16 * r + a;
            if (i >= p0 && i < p1)
#pragma unroll
                for (int c = 0; c < k2dC; c++) Pn[i - p0][16 * c + b] = A[r][c];
        }
        __syncthreads();   // also: every thread is done with the previous panel's UP
        if (w == 0) {
            double u0[k2dPW], u1[k2dPW];
#pragma unroll
            for (int t = 0; t < k2dPW; t++) {
                u0[t] = p0 + t < n ? Pn[t][lane] : 0.0;
                u1[t] = p0 + t < n ? Pn[t][lane + 64] : 0.0;
            }
            bool good = true;
#pragma unroll
            for (int t = 0; t < k2dPW; t++) {
                const int k = p0 + t;
                if (k < n && good) {
                    UP[t][lane] = u0[t];   // row k is final
                    UP[t][lane + 64] = u1[t];
                    const double d = k < 64 ? readlane_d(u0[t], k) : readlane_d(u1[t], k - 64);
                    if (d == 0.0) {   // uniform
                        good = false;
                        if (lane == 0) ok = 0;
                    } else {
                        const double l0 = u0[t] / d, l1 = u1[t] / d;   // l_jk, j = lane / lane + 64
                        if (lane > k && lane < n) Lall[k * n + lane] = l0;
                        if (lane + 64 > k && lane + 64 < n) Lall[k * n + lane + 64] = l1;
                        const double yk = n < 64 ? readlane_d(u0[t], n) : readlane_d(u1[t], n - 64);
                        if (lane == 0) {
                            dvec[k] = d;
                            y[k] = yk;   // b_k after its k updates: the forward-substituted y_k
                        }
#pragma unroll
                        for (int t2 = t + 1; t2 < k2dPW; t2++) {
                            const int i = p0 + t2;
                            if (i < n) {
                                const double li = i < 64 ? readlane_d(l0, i) : readlane_d(l1, i - 64);
                                u0[t2] -= li * u0[t];
                                u1[t2] -= li * u1[t];
                            }
                        }
                    }
                }
            }
        }
        __syncthreads();
        if (!ok) break;
        // rows >= p1: the panel's pivots, ascending, on the live register rows / columns
        const int pw = p1 - p0;
#pragma unroll
        for (int r = 0; r < k2dR; r++) {
            if (16 * r + 4 * w + 3 < p1) continue;   // the wave's four rows of register row r are done
            const int i = 16 * r + a;
            double lv[k2dPW];
#pragma unroll
            for (int t = 0; t < k2dPW; t++) lv[t] = t < pw ? Lall[(p0 + t) * n + i] : 0.0;
#pragma unroll
            for (int c = 0; c < k2dC; c++) {
                if (16 * c + 15 < p1) continue;      // every column of register column c is done
                const int j = 16 * c + b;
                double v = A[r][c];
#pragma unroll
                for (int t = 0; t < k2dPW; t++)
                    if (t < pw) v -= lv[t] * UP[t][j];
                A[r][c] = v;
            }
        }
    }
    if (!ok) {
        if (tid == 0) scal[3] = 0.0;
        return;
    }
    __syncthreads();
    if (w != 0) return;
    ldlt_backward_wave(n, Lall, dvec, y, x, scal);
}

// The dense LDL^T of the local BA's reduced system (k_ldlt_reg, below).
#ifdef ORB_LDLT_PROBE
__device__ long long g_ldlt_probe[256];
#define LDLT_PROBE(slot) \
    do {                                                  \
        if (threadIdx.x == 0) g_ldlt_probe[slot] = clock64(); \
    } while (0)
#else
#define LDLT_PROBE(slot) \
    do {                 \
    } while (0)
#endif
constexpr int kLdltMax = 128;
constexpr int kTiledMinPoses = kBaTiledMinPoses;   // 6 x 24 = 144 rows: the first n the LDS-resident dense solver cannot hold
constexpr int kDenseMaxN = 144;   // >= every n the dense single-workgroup solvers take (n^2 doubles in LDS)
constexpr int kLdltWaves = 8;     // 512 threads: 256 VGPRs per lane, the panel registers stay unspilled
constexpr int kLdltThreads = 64 * kLdltWaves;
// LDS of k_ldlt_reg: Lall (n x n), three 6 x kLdltMax panel row buffers, two kLdltMax x 6 panel L
// buffers, d, y
static inline size_t ldlt_reg_shm(int n) { return sizeof(double) * ((size_t)n * n + 1 + 32 * kLdltMax); }

// SharedDiv::div without its branch: the quotient of an in-range numerator, or a * r for a zero
// one (a / b = a signed zero); any other numerator (or an out-of-range divisor) sets `bad` and the
// caller redoes the work with SharedDiv::div.
__device__ __forceinline__ double div_fast(const SharedDiv& d, double a, bool& bad) {
    const double q = a * d.r;
    const double rem = fma(-d.b, q, a);
    const double res = __builtin_amdgcn_div_fixup(fma(rem, d.r, q), d.b, a);
    const double aa = fabs(a);
    const bool inr = aa > 0x1p-300 && aa < 0x1p300;
    bad = bad || !(inr || aa == 0.0);
    return inr ? res : q;
}

// the panel factorisation of k_ldlt_reg for one column thread j, any panel width pw <= 6, with
// SharedDiv::div (the fallback of ldlt_panel6)
__device__ __forceinline__ void ldlt_panel_generic(int n, int p0, int pw, int j, double* U, double* Lall,
                                                   double* Lpan, double* dvec, double* y, int* ok) {
    double Bk[6][6], Lb[6][6], dd[6];
#pragma unroll
    for (int t = 0; t < 6; t++)
#pragma unroll
        for (int c = 0; c < 6; c++) {
            Bk[t][c] = (t < pw && c < pw && c >= t) ? U[t * kLdltMax + p0 + c] : 0.0;
            Lb[t][c] = 0.0;
        }
    bool bad = false;
    SharedDiv sd[6] = {SharedDiv(1.0), SharedDiv(1.0), SharedDiv(1.0), SharedDiv(1.0), SharedDiv(1.0),
                       SharedDiv(1.0)};
#pragma unroll
    for (int t = 0; t < 6; t++) {
        dd[t] = Bk[t][t];
        if (t < pw) {
            bad |= dd[t] == 0.0;
            sd[t] = SharedDiv(dd[t]);
#pragma unroll
            for (int t2 = t + 1; t2 < 6; t2++)
                if (t2 < pw) Lb[t2][t] = sd[t].div(Bk[t][t2]);
#pragma unroll
            for (int t2 = t + 1; t2 < 6; t2++)
#pragma unroll
                for (int c = t2; c < 6; c++)
                    if (c < pw) Bk[t2][c] -= Lb[t2][t] * Bk[t][c];
        }
    }
    double u[6];
#pragma unroll
    for (int t = 0; t < 6; t++) u[t] = t < pw ? U[t * kLdltMax + j] : 0.0;
#pragma unroll
    for (int t = 0; t < 6; t++) {
        if (t < pw) {
            const int k = p0 + t;
            const bool act = j > k && j < n;
            const double l = act ? sd[t].div(u[t]) : 0.0;
#pragma unroll
            for (int t2 = t + 1; t2 < 6; t2++)
                if (t2 < pw && j >= p0 + t2) u[t2] -= Lb[t2][t] * u[t];
            if (act) {
                Lall[(size_t)k * n + j] = l;
                Lpan[j * 6 + t] = l;
            }
            if (j == n) y[k] = u[t];   // row k's right-hand side is final: forward-substituted y_k
        }
    }
#pragma unroll
    for (int t = 0; t < 6; t++)
        if (t < pw) U[t * kLdltMax + j] = u[t];
    if (j == 0) {
#pragma unroll
        for (int t = 0; t < 6; t++)
            if (t < pw) dvec[p0 + t] = dd[t];
        if (bad) *ok = 0;
    }
}

// A full panel (pw = 6) in one basic block: every thread first factorises the 6x6 diagonal block
// from LDS itself (the same operations as the block's own columns perform, so d and the block's L
// agree bit for bit), then its own column: l_jk = u_kj / d_k and u_tj -= L[t][k] u_kj, k
// ascending.  Results stay in registers until the wave knows that every division was a fast one;
// a wave with a zero pivot or an out-of-range operand redoes the panel with ldlt_panel_generic.
__device__ __forceinline__ void ldlt_panel6(int n, int p0, int j, double* U, double* Lall, double* Lpan,
                                            double* dvec, double* y, int* ok) {
    double B[6][6], Lb[6][6], dd[6];
#pragma unroll
    for (int t = 0; t < 6; t++)
#pragma unroll
        for (int c = t; c < 6; c++) B[t][c] = U[t * kLdltMax + p0 + c];
    double u[6];
#pragma unroll
    for (int t = 0; t < 6; t++) u[t] = U[t * kLdltMax + j];
    bool bad = false;
    SharedDiv sd[6] = {SharedDiv(1.0), SharedDiv(1.0), SharedDiv(1.0), SharedDiv(1.0), SharedDiv(1.0),
                       SharedDiv(1.0)};
#pragma unroll
    for (int t = 0; t < 6; t++) {
        dd[t] = B[t][t];
        sd[t] = SharedDiv(dd[t]);
        bad = bad || !sd[t].ok;
#pragma unroll
        for (int t2 = t + 1; t2 < 6; t2++) Lb[t2][t] = div_fast(sd[t], B[t][t2], bad);
#pragma unroll
        for (int t2 = t + 1; t2 < 6; t2++)
#pragma unroll
            for (int c = t2; c < 6; c++) B[t2][c] -= Lb[t2][t] * B[t][c];
    }
    double l[6];
    bool badc = false;
#pragma unroll
    for (int t = 0; t < 6; t++) {
        const bool act = j > p0 + t && j < n;
        bool bt = false;
        const double q = div_fast(sd[t], u[t], bt);
        badc = badc || (act && bt);
        l[t] = act ? q : 0.0;
#pragma unroll
        for (int t2 = t + 1; t2 < 6; t2++) {
            const double v = u[t2] - Lb[t2][t] * u[t];
            u[t2] = j >= p0 + t2 ? v : u[t2];
        }
    }
    if (__ballot(bad || badc)) {
        ldlt_panel_generic(n, p0, 6, j, U, Lall, Lpan, dvec, y, ok);
        return;
    }
#pragma unroll
    for (int t = 0; t < 6; t++) {
        const int k = p0 + t;
        if (j > k && j < n) {
            Lall[(size_t)k * n + j] = l[t];
            Lpan[j * 6 + t] = l[t];
        }
        U[t * kLdltMax + j] = u[t];
    }
    if (j == n)
#pragma unroll
        for (int t = 0; t < 6; t++) y[p0 + t] = u[t];   // forward-substituted y_k
    if (j == 0)
#pragma unroll
        for (int t = 0; t < 6; t++) dvec[p0 + t] = dd[t];
}

// Row waves of k_ldlt_reg (waves 2..7, kRowWaves of them): wave 2 + t owns rows i = 6 r + t
// (slot r < kRowSlots) of columns j = lane, lane + 64, so a 6-row panel p is slot p of every row
// wave.  In phase p a row wave applies panel p - 1's six rank-one updates (its L from Lp, its
// rows u from Up) in k order to its rows i >= 6 (p + 1) -- panel p's own rows were handed to the
// factor waves one phase earlier -- and publishes slot p + 1 (panel p + 1's row, now updated by
// every panel up to p - 1) to Un.  Rows i >= 64 own no column below 64 on or right of the
// diagonal; column registers 64.. matter only for n >= 64 (the right-hand side sits at column n).
constexpr int kRowWaves = 6;
constexpr int kRowSlots = (kLdltMax + kRowWaves - 1) / kRowWaves;
__device__ __forceinline__ void ldlt_rows(double (&R)[2][kRowSlots], const double* Up, const double* Lp, double* Un,
                                          int n, int p1, int t6, int lane) {
    double u0[6], u1[6];
#pragma unroll
    for (int t = 0; t < 6; t++) {
        u0[t] = Up[t * kLdltMax + lane];
        u1[t] = Up[t * kLdltMax + lane + 64];
    }
#pragma unroll
    for (int r = 0; r < kRowSlots; r++) {
        const int i = kRowWaves * r + t6;
        if (i >= p1 && i < n) {
            double L[6];
#pragma unroll
            for (int t = 0; t < 6; t++) L[t] = Lp[i * 6 + t];
            if (i < 64) {
                double v0 = R[0][r];
#pragma unroll
                for (int t = 0; t < 6; t++) v0 -= L[t] * u0[t];
                R[0][r] = lane >= i ? v0 : R[0][r];
            }
            if (n >= 64) {
                double v1 = R[1][r];
#pragma unroll
                for (int t = 0; t < 6; t++) v1 -= L[t] * u1[t];
                R[1][r] = lane + 64 >= i ? v1 : R[1][r];
            }
            if (i < p1 + 6) {   // panel p + 1's row
                Un[(i - p1) * kLdltMax + lane] = R[0][r];
                Un[(i - p1) * kLdltMax + lane + 64] = R[1][r];
            }
        }
    }
}

// Register-resident LDL^T + solve for n < 128 (<= 21 free keyframes), 512 threads, with a
// one-panel lookahead: waves 0-1 factorise 6-column panels (one thread per column j), waves 2-7
// hold the rows.  Phase p: the factor waves factorise panel p from its rows in LDS (every earlier
// panel's updates applied) and signal; the row waves apply panel p - 1 to their rows below panel
// p (the trailing update runs under the factorisation), publish panel p + 1's rows to LDS and,
// once panel p is factored, apply panel p to those rows there (one row per wave, no register
// indexing).  One barrier per phase; panel rows rotate through three buffers, panel L through
// two.  Per-element operation sequence identical to oracle ora_ldlt_solve (every element receives
// the pivots' updates in ascending k).
__global__ void __launch_bounds__(kLdltThreads) k_ldlt_reg(int n, const double* __restrict__ Sg, const double* bs,
                                                           double* x, double* scal, const int* run) {
    BA_GATE(run);
    extern __shared__ double lds[];
    double* Lall = lds;                               // n x n, Lall[k * n + i] = L[i][k]
    double* Ub = Lall + (((size_t)n * n + 1) & ~(size_t)1);   // 3 x (6 x kLdltMax) panel rows (16-B aligned)
    double* Lb = Ub + 18 * kLdltMax;                  // 2 x (kLdltMax x 6) panel L
    double* dvec = Lb + 12 * kLdltMax;                // n
    double* y = dvec + kLdltMax;                      // n
    __shared__ int ok, done;
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform: row branches stay scalar
    const bool factor = w < kLdltMax / 64;
    const int t6 = w - kLdltMax / 64;
    // [S | b] (n <= 126 < kLdltMax): column n carries the right-hand side, so the row updates run
    // the forward substitution L y = b with the oracle's sequence (y_i -= l_ik y_k, k ascending)
    // and y_k is final when row k becomes a pivot row
    double R[2][kRowSlots];
    if (!factor) {
#pragma unroll
        for (int c = 0; c < 2; c++)
#pragma unroll
            for (int r = 0; r < kRowSlots; r++) {
                const int i = kRowWaves * r + t6, j = lane + 64 * c;
                R[c][r] = (i < n && j < n && i <= j) ? Sg[(size_t)i * n + j] : (i < n && j == n) ? bs[i] : 0.0;
            }
        if (t6 < n) {   // panel 0's rows (slot 0)
            Ub[t6 * kLdltMax + lane] = R[0][0];
            Ub[t6 * kLdltMax + lane + 64] = R[1][0];
        }
    }
    LDLT_PROBE(0);
    if (tid == 0) {
        ok = 1;
        done = 0;
    }
    __syncthreads();
    LDLT_PROBE(1);
    int cur = 0;   // panel p's row buffer: p mod 3
    for (int p0 = 0; p0 < n; p0 += 6) {
        const int p1 = min(p0 + 6, n), pw = p1 - p0, pi = p0 / 6;
        const int prv = cur == 0 ? 2 : cur - 1, nxt = cur == 2 ? 0 : cur + 1;
        double* U = Ub + cur * 6 * kLdltMax;
        double* Un = Ub + nxt * 6 * kLdltMax;
        double* Lpan = Lb + (pi & 1) * 6 * kLdltMax;
        LDLT_PROBE(11 + 4 * (pi < 20 ? pi : 20));
        if (factor) {
            if (pw == 6) ldlt_panel6(n, p0, tid, U, Lall, Lpan, dvec, y, &ok);
            else ldlt_panel_generic(n, p0, pw, tid, U, Lall, Lpan, dvec, y, &ok);
            // (also after a zero pivot: the row waves wait for this count)
            if (lane == 0) __hip_atomic_fetch_add(&done, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
#ifdef ORB_LDLT_PROBE
            if (tid == 0 && pi < 20) g_ldlt_probe[220 + pi] = clock64();   // factor done
#endif
        } else {
            // panel p - 1's updates on the rows below panel p, panel p + 1's rows published.  The
            // slot index is re-made opaque per panel: hoisted out of the panel loop, the rows'
            // offsets and tests spill SGPRs into VGPR lanes (a v_readlane each per row)
            int tv = t6;
            asm volatile("" : "+s"(tv));
            if (p0 > 0) {
                ldlt_rows(R, Ub + prv * 6 * kLdltMax, Lb + ((pi & 1) ^ 1) * 6 * kLdltMax, Un, n, p1, tv, lane);
            } else if (6 + t6 < n) {   // phase 0: panel 1's rows (slot 1) as they are
                Un[t6 * kLdltMax + lane] = R[0][1];
                Un[t6 * kLdltMax + lane + 64] = R[1][1];
            }
#ifdef ORB_LDLT_PROBE
            if (lane == 0 && pi < 16) g_ldlt_probe[124 + 6 * pi + t6] = clock64();   // bulk done
#endif
            const int i = p1 + tv;   // this wave's row of panel p + 1 (panel p is full when it exists)
            if (i < n) {
                while (__hip_atomic_load(&done, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < 2 * (pi + 1))
                    __builtin_amdgcn_s_sleep(1);
                double L[6], u0[6], u1[6];
#pragma unroll
                for (int t = 0; t < 6; t++) {
                    L[t] = Lpan[i * 6 + t];
                    u0[t] = U[t * kLdltMax + lane];
                    u1[t] = U[t * kLdltMax + lane + 64];
                }
                double v0 = Un[tv * kLdltMax + lane], v1 = Un[tv * kLdltMax + lane + 64];
                const double o0 = v0, o1 = v1;
#pragma unroll
                for (int t = 0; t < 6; t++) {
                    v0 -= L[t] * u0[t];
                    v1 -= L[t] * u1[t];
                }
                Un[tv * kLdltMax + lane] = lane >= i ? v0 : o0;
                Un[tv * kLdltMax + lane + 64] = lane + 64 >= i ? v1 : o1;
            }
        }
        __syncthreads();
        LDLT_PROBE(12 + 4 * (pi < 20 ? pi : 20));
        if (!ok) break;
        cur = nxt;
    }
    LDLT_PROBE(2);
    if (!ok) {
        if (tid == 0) scal[3] = 0.0;
        return;
    }
    if (w != 0) return;
    LDLT_PROBE(3);
    ldlt_backward_wave(n, Lall, dvec, y, x, scal);
    LDLT_PROBE(4);
}

// push + back-substitution (block_solver.hpp:457-484) + SparseOptimizer::update (oplus)
__global__ void __launch_bounds__(256) k_update(BaStructDev s, Se3* T, Se3* Tbak, double* X, double* Xbak,
                                                double* x, const double* __restrict__ Hpl, const double* Hll,
                                                const double* bl, double lam_host, int use_dev, const double* scal,
                                                const int* run) {
    BA_GATE(run);
    const int g = blockIdx.x * blockDim.x + threadIdx.x;
    const int nP = s.nP;
    if (g < nP) {
        const int kf = s.poseKf[g];
        const Se3 t0 = T[kf];
        Tbak[kf] = t0;
        T[kf] = pose_step(t0, x + 6 * g);
        return;
    }
    const int l = g - nP;
    if (l >= s.nL) return;
    const int pt = s.landPt[l];
    const bool solved = scal[3] != 0.0;
    double xl[3];
    land_step(s, l, Hpl, Hll, bl, x, lam_of(lam_host, use_dev, scal), solved, xl);
    for (int k = 0; k < 3; k++) {
        if (solved) x[6 * nP + 3 * l + k] = xl[k];
        const double v = X[3 * pt + k];
        Xbak[3 * pt + k] = v;
        X[3 * pt + k] = v + xl[k];
    }
}

__global__ void __launch_bounds__(256) k_pop(BaStructDev s, Se3* T, const Se3* Tbak, double* X, const double* Xbak,
                                             const int* run) {
    BA_GATE(run);
    const int g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g < s.nP) {
        const int kf = s.poseKf[g];
        T[kf] = Tbak[kf];
        return;
    }
    const int l = g - s.nP;
    if (l >= s.nL) return;
    const int pt = s.landPt[l];
    for (int k = 0; k < 3; k++) X[3 * pt + k] = Xbak[3 * pt + k];
}

// computeScale: csum_j x_j (lambda x_j + b_j) over poses then landmarks, one workgroup:
// wave trees of 64 consecutive terms (coalesced), chunk sums reduced by one thread.
__global__ void __launch_bounds__(1024) k_scale(int nP, int nL, const double* x, const double* bp, const double* bl,
                                                double lam_host, int use_dev, const double* scal, double* out,
                                                int poses, const int* run) {
    BA_GATE(run);
    __shared__ double lv[2048];
    const int n = 6 * nP + 3 * nL;
    const double lambda = lam_of(lam_host, use_dev, scal);
    auto term = [&](int j) {  // poses == 0: a shard that does not own the (replicated) pose terms
        if (j < 6 * nP && !poses) return 0.0;
        const double b = j < 6 * nP ? bp[j] : bl[j - 6 * nP];
        return x[j] * (lambda * x[j] + b);
    };
    if (n <= 1) {
        if (threadIdx.x == 0) *out = n == 1 ? term(0) : 0.0;
        return;
    }
    const int m = (n + 63) >> 6;   // <= 2048 (validated)
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (int c = w; c < m; c += 16) {
        const int j = c * 64 + lane;
        const double t = wave_tree(j < n ? term(j) : 0.0);
        if (lane == 0) lv[c] = t;
    }
    __syncthreads();
    if (threadIdx.x == 0) *out = local_csum_inplace(lv, m);
}

// computeScale terms for large problems (6 nP + 3 nL > 2048 * 64) fused with the first
// canonical level: wave c writes the 64-tree of
// v[64c .. 64c + 64) (zero past the end) to chunks[c]; k_csum then sums the chunk trees, which
// continues ora_csum at its second level
__global__ void __launch_bounds__(256) k_scale_chunks(int nP, int nL, const double* x, const double* bp,
                                                      const double* bl, double lam_host, int use_dev,
                                                      const double* scal, double* chunks, int poses, const int* run) {
    BA_GATE(run);
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    double v = 0.0;
    if (j < 6 * nP + 3 * nL && (j >= 6 * nP || poses)) {
        const double lambda = lam_of(lam_host, use_dev, scal);
        const double b = j < 6 * nP ? bp[j] : bl[j - 6 * nP];
        v = x[j] * (lambda * x[j] + b);
    }
    const double t = wave_tree(v);
    if ((threadIdx.x & 63) == 0) chunks[j >> 6] = t;
}

// canonical sum of one list per workgroup (blockIdx.x selects the list), 1024 threads,
// level buffers ping-pong in global scratch.
struct CsumList {
    const double* v;
    int n;
    double* tmp0;
    double* tmp1;
    double* out;
};
__global__ void __launch_bounds__(1024) k_csum(CsumList L0, CsumList L1, const int* run) {
    BA_GATE(run);
    const CsumList L = blockIdx.x == 0 ? L0 : L1;
    if (L.n <= 1) {
        if (threadIdx.x == 0) *L.out = L.n == 1 ? L.v[0] : 0.0;
        return;
    }
    const double* src = L.v;
    double* dst = L.tmp0;
    int m = L.n;
    while (true) {
        const int m2 = (m + 63) >> 6;
        for (int c = threadIdx.x; c < m2; c += blockDim.x) {
            const double* p = src + c * 64;
            dst[c] = tree64_local([&](int i) { return p[i]; }, min(64, m - c * 64));
        }
        __threadfence_block();
        __syncthreads();
        if (m2 == 1) break;
        src = dst;
        dst = (dst == L.tmp0) ? L.tmp1 : L.tmp0;
        m = m2;
    }
    if (threadIdx.x == 0) *L.out = dst[0];
}

// ---------------------------------------------------------------- device-resident LM control
// OptimizationAlgorithmLevenberg::solve's trial loop and SparseOptimizer::optimize's iteration
// loop (optimization_algorithm_levenberg.cpp:59-164, sparse_optimizer.cpp:354-418) decided on the
// device, so a run's kernels queue back to back with no host round trip per trial.  The host
// queues whole steps (system kernels gated by ctl[1], trial kernels by ctl[0]) one step ahead of
// the decisions it has seen; k_lm_trial_end sets the gates of the next step.
// Host-pinned coherent words (LmHost): [0] stop flag mirror (host writes), [1] done, [2] steps
// decided, [3] iterations, [4..5] (done, steps) as one 8-byte word the host polls (device writes).
__global__ void __launch_bounds__(64) k_lm_begin(LmDev* L, int iterations) {
    if (threadIdx.x != 0) return;
    L->ctl[0] = 1;
    L->ctl[1] = 1;
    L->ctl[2] = 1;   // computeLambdaInit on the first iteration
    L->it = 0;
    L->iterations = iterations;
    L->qmax = 0;
    L->nBad = 0;
    L->haveChi = 0;
    L->done = 0;
    L->nTrial = 0;
    L->nSolve = 0;
    L->steps = 0;
    L->ni = 2;
    L->currentChi = 0;
    L->iniChi = 0;
}

// one thread: the host code of BaEngine::lm_solve after its readback, verbatim in order;
// returns whether the trial is undone (pop).  The LM state's scalars, the trial's scalars and the
// host's stop flag are read by the caller at the start of k_lm_trial_end (independent loads in
// flight together, behind the workgroup's sums) and written back at the end: through the global
// pointers every access would wait for the one before it.
struct LmHead {
    int ctl[4];
    int it, iterations, qmax, nBad, haveChi, done, nTrial, nSolve, steps;
    double ni, currentChi, iniChi;
};
__device__ __forceinline__ void lm_load(const LmDev* Lg, LmHead& L) {
    L.ctl[0] = Lg->ctl[0];
    L.ctl[1] = Lg->ctl[1];
    L.ctl[2] = Lg->ctl[2];
    L.ctl[3] = Lg->ctl[3];
    L.it = Lg->it;
    L.iterations = Lg->iterations;
    L.qmax = Lg->qmax;
    L.nBad = Lg->nBad;
    L.haveChi = Lg->haveChi;
    L.done = Lg->done;
    L.nTrial = Lg->nTrial;
    L.nSolve = Lg->nSolve;
    L.steps = Lg->steps;
    L.ni = Lg->ni;
    L.currentChi = Lg->currentChi;
    L.iniChi = Lg->iniChi;
}
// L: the state as lm_load read it; stop: the host's flag; s0..s5: the trial's scalars (chi2 of the
// system and the trial, scale, the trial's solve status, -, lambda)
__device__ int lm_decide(LmDev* Lg, LmHead L, double* scal, volatile int* host, bool stop, double s0, double s1,
                         double s2, double s3, double s5) {
    if (!L.haveChi) {
        L.currentChi = L.iniChi = s0;
        L.haveChi = 1;
    }
    const bool ok2 = s3 != 0.0;
    double tempChi = s1;
    if (!ok2) tempChi = DBL_MAX;
    double rho = L.currentChi - tempChi;
    double scale = s2;
    scale += 1e-3;
    rho /= scale;
    double lambda = s5;
    int pop = 0;
    if (rho > 0 && isfinite(tempChi)) {
        const double a3 = 2 * rho - 1;
        double alpha = 1. - (a3 * a3) * a3;
        alpha = fmin(alpha, 2. / 3.);
        const double scaleFactor = fmax(1. / 3., alpha);
        lambda *= scaleFactor;
        L.ni = 2;
        L.currentChi = tempChi;
    } else {
        lambda *= L.ni;
        L.ni *= 2;
        pop = 1;
    }
    scal[5] = lambda;
    L.qmax++;
    if (L.nTrial < kLmTrials) {
        Lg->trialChi[L.nTrial] = tempChi;
        Lg->trialLam[L.nTrial] = lambda;
    }
    L.nTrial++;
    L.ctl[2] = 0;
    if (rho < 0 && L.qmax < 10 && !stop) {   // another trial on the same system
        L.ctl[1] = 0;
    } else {                                  // lm_solve returns
        if (L.nSolve < kLmSolves) {
            Lg->solveIni[L.nSolve] = L.iniChi;
            Lg->solveChi[L.nSolve] = L.currentChi;
        }
        L.nSolve++;
        bool term = false;
        if (L.qmax == 10 || rho == 0) {
            term = true;
        } else {
            if ((L.iniChi - L.currentChi) * 1e3 < L.iniChi) L.nBad++;
            else L.nBad = 0;
            if (L.nBad >= 3) term = true;
        }
        L.it++;
        if (term || L.it >= L.iterations || stop) {
            L.done = 1;
            L.ctl[0] = 0;
            L.ctl[1] = 0;
        } else {
            L.ctl[1] = 1;
            L.haveChi = 0;
            L.qmax = 0;
        }
    }
    L.steps++;
    Lg->ctl[0] = L.ctl[0];
    Lg->ctl[1] = L.ctl[1];
    Lg->ctl[2] = L.ctl[2];
    Lg->it = L.it;
    Lg->qmax = L.qmax;
    Lg->nBad = L.nBad;
    Lg->haveChi = L.haveChi;
    Lg->done = L.done;
    Lg->nTrial = L.nTrial;
    Lg->nSolve = L.nSolve;
    Lg->steps = L.steps;
    Lg->ni = L.ni;
    Lg->currentChi = L.currentChi;
    Lg->iniChi = L.iniChi;
    host[3] = L.it;
    host[2] = L.steps;
    host[1] = L.done;
    // the pair (done, steps) as one aligned 8-byte store: the host's poll sees both or neither
    *(volatile unsigned long long*)(host + 4) = ((unsigned long long)(unsigned)L.steps << 32) | (unsigned)L.done;
    return pop;
}

// End of a trial: the chi2 totals of the step's two linearisations (ChiFuse: k_linearize's chunk
// trees, summed here instead of by two k_chi2_finish launches), computeScale (k_scale's canonical
// sum, problems with 6 nP + 3 nL <= 2048 * 64; larger ones ran k_scale_chunks + k_csum into
// scal[2] and pass scale = 0), the LM decision, and the pop of a rejected trial, in one workgroup.
constexpr int kChiFuseMax = 1024;   // chunk trees per linearisation (nE <= 65536) summed in LDS
constexpr int kTeThreads = 1024;
constexpr int kTePre = 4;      // committed landmarks per thread loaded ahead
constexpr int kScalePre = 8;   // scale chunks per wave loaded ahead of their trees
struct ChiFuse {
    const double* chunksSys;     // the system linearisation's chunk trees (chi2 -> scal[0]), or null
    const double* chunksTrial;   // the trial's (-> scal[1])
    int nE;
};
__global__ void __launch_bounds__(kTeThreads) k_lm_trial_end(LmDev* L, double* scal, volatile int* host, BaStructDev s,
                                                       Se3* T, const Se3* Tbak, double* X, const double* Xbak,
                                                       const double* x, const double* bp, const double* bl, int scale,
                                                       ChiFuse cf, const Se3* Tn, const double* Xn,
                                                       const double* stopDev) {
    __shared__ double lv[2048];
    __shared__ double cA[kChiFuseMax], cB[kChiFuseMax];
    __shared__ double tot[3];   // the fused chi2 totals (system, trial) and the scale sum
    __shared__ int pop, live;
    const int nP = s.nP, nL = s.nL;
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    // Everything this kernel reads is loaded before its first barrier, in flight together: the LM
    // state, the host's stop flag and the trial's scalars (thread 0), the chunk trees, the scale
    // terms and the values an accepted trial commits.  Nothing is written before that barrier, which
    // publishes the run flag: a step queued after the run ended stops there (its loads read
    // allocated buffers).  One read of the flag for the whole workgroup: lm_decide may clear
    // ctl[0] and a wave reading it after that would skip the pop.
    LmHead H;
    bool stop = false;
    double g0 = 0, g1 = 0, g2 = 0, g3 = 0;
    if (threadIdx.x == 0) {
        lm_load(L, H);
        // a sharded run's stop flag is the ranks' all-reduced one (every rank decides alike)
        stop = stopDev ? stopDev[0] != 0.0 : host[0] != 0;
        g0 = scal[0];
        g1 = scal[1];
        g2 = scal[2];
        g3 = scal[3];
    }
    const bool fuse = cf.chunksSys != nullptr;
    const int mc = (cf.nE + 63) >> 6;   // fuse: 2 <= nE, mc <= kChiFuseMax (host)
    if (fuse)
        for (int c = threadIdx.x; c < mc; c += kTeThreads) {
            cA[c] = cf.chunksSys[c];
            cB[c] = cf.chunksTrial[c];
        }
    const int n = 6 * nP + 3 * nL;
    const int m = (n + 63) >> 6;
    const double lambda = scal[5];
    auto term = [&](int j) {
        const double* b = j < 6 * nP ? bp + j : bl + (j - 6 * nP);
        return x[j] * (lambda * x[j] + *b);
    };
    // the scale terms of kScalePre chunks per wave loaded before their trees
    if (scale && n > 1)
        for (int c0 = w; c0 < m; c0 += 16 * kScalePre) {
            double tv[kScalePre];
#pragma unroll
            for (int k = 0; k < kScalePre; k++) {
                const int j = (c0 + 16 * k) * 64 + lane;
                tv[k] = j < n ? term(j) : 0.0;
            }
#pragma unroll
            for (int k = 0; k < kScalePre; k++) {
                const double t = wave_tree(tv[k]);
                if (lane == 0 && c0 + 16 * k < m) lv[c0 + 16 * k] = t;
            }
        }
    // an accepted trial's commit (Tn set): the first kTePre landmarks and the pose of each thread
    double xc[kTePre][3], tc[8];
    int pc[kTePre];
    int kc = -1;
    if (Tn) {
#pragma unroll
        for (int k = 0; k < kTePre; k++) {
            const int l = threadIdx.x + k * kTeThreads;
            pc[k] = -1;
            if (l < nL) {
                pc[k] = s.landPt[l];
                for (int d = 0; d < 3; d++) xc[k][d] = Xn[3 * l + d];
            }
        }
        if ((int)threadIdx.x < nP) {
            kc = s.poseKf[threadIdx.x];
            const double* src = (const double*)(Tn + threadIdx.x);
#pragma unroll
            for (int d = 0; d < 8; d++) tc[d] = src[d];
        }
    }
    if (threadIdx.x == 0) live = H.ctl[0];
    __syncthreads();
    if (!live) return;   // a step queued after the run ended
    // block_finish_csum's totals: wave_tree pairs as tree64_local, so wave_lds_csum is
    // local_csum_inplace's canonical sum
    if (scale && w == 0) {
        const double t = n > 1 ? wave_lds_csum(lv, m) : n == 1 ? term(0) : 0.0;
        if (lane == 0) {
            tot[2] = t;
            scal[2] = t;
        }
    }
    if (fuse && (w == 1 || w == 2)) {
        double* c = w == 1 ? cA : cB;
        const double t = mc == 1 ? c[0] : wave_lds_csum(c, mc);
        if (lane == 0) {
            tot[w - 1] = t;
            scal[w - 1] = t;
        }
    }
    __syncthreads();
    if (threadIdx.x == 0)
        pop = lm_decide(L, H, scal, host, stop, fuse ? tot[0] : g0, fuse ? tot[1] : g1, scale ? tot[2] : g2, g3,
                        lambda);
    __syncthreads();
    if (Tn) {   // the update was fused into the trial pass: an accepted trial commits its poses / points
        if (pop) return;
        if (kc >= 0) {
            double* dst = (double*)(T + kc);
#pragma unroll
            for (int d = 0; d < 8; d++) dst[d] = tc[d];
        }
        for (int g = threadIdx.x + kTeThreads; g < nP; g += kTeThreads) T[s.poseKf[g]] = Tn[g];
#pragma unroll
        for (int k = 0; k < kTePre; k++)
            if (pc[k] >= 0)
                for (int d = 0; d < 3; d++) X[3 * pc[k] + d] = xc[k][d];
        for (int l = threadIdx.x + kTePre * kTeThreads; l < nL; l += kTeThreads) {
            const int pt = s.landPt[l];
            for (int d = 0; d < 3; d++) X[3 * pt + d] = Xn[3 * l + d];
        }
        return;
    }
    if (!pop) return;
    for (int g = threadIdx.x; g < nP + nL; g += kTeThreads) {   // k_pop
        if (g < nP) {
            const int kf = s.poseKf[g];
            T[kf] = Tbak[kf];
        } else {
            const int pt = s.landPt[g - nP];
            for (int k = 0; k < 3; k++) X[3 * pt + k] = Xbak[3 * pt + k];
        }
    }
}

// outlier gating / final check over all edges (Optimizer.cc:674-706, 714-746):
// flag = chi2(last _error) > th || !isDepthPositive()
__global__ void __launch_bounds__(256) k_gate(int ne, const EdgeDev* E, const Se3* T, const double* X,
                                              const double* err, uint8_t* flag, uint8_t* level, uint8_t* robust,
                                              int set_level) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= ne) return;
    const EdgeDev e = E[i];
    const double chi = edge_chi2(e, err + 3 * i);
    double p[3];
    const double Xp[3] = {X[3 * e.pt], X[3 * e.pt + 1], X[3 * e.pt + 2]};
    se3_map(T[e.kf], Xp, p);
    const double th = e.stereo ? 7.815 : 5.991;
    const uint8_t bad = (chi > th || !(p[2] > 0.0)) ? 1 : 0;
    flag[i] = bad;
    if (set_level) {
        if (bad) level[i] = 1;
        robust[i] = 0;
    }
}

// Sharded exchange of S: only the 64x64 tiles of the union Schur pattern travel.
// tiles[t] = (I, J) with I <= J; buf = T * 4096 doubles (row-major tile, zero padded).
__global__ void __launch_bounds__(256) k_tile_pack(int n, const double* __restrict__ S, const int2* tiles,
                                                   double* buf) {
    const int2 tj = tiles[blockIdx.x];
    double* o = buf + (size_t)blockIdx.x * 4096;
    for (int q = threadIdx.x; q < 4096; q += 256) {
        const int r = tj.x * 64 + (q >> 6), c = tj.y * 64 + (q & 63);
        o[q] = (r < n && c < n) ? S[(size_t)r * n + c] : 0.0;
    }
}

__global__ void __launch_bounds__(256) k_tile_unpack(int n, double* __restrict__ S, const int2* tiles,
                                                     const double* buf) {
    const int2 tj = tiles[blockIdx.x];
    const double* o = buf + (size_t)blockIdx.x * 4096;
    for (int q = threadIdx.x; q < 4096; q += 256) {
        const int r = tj.x * 64 + (q >> 6), c = tj.y * 64 + (q & 63);
        if (r < n && c < n) S[(size_t)r * n + c] = o[q];
    }
}

// ---------------------------------------------------------------- PoseOptimization
// Optimizer::PoseOptimization (Optimizer.cc:239-451): one SE3 vertex with unary
// EdgeSE3ProjectXYZOnlyPose / EdgeStereoSE3ProjectXYZOnlyPose edges
// (types_six_dof_expmap.cpp:266-364), solved by LinearSolverDense (Eigen LDLT with diagonal
// pivoting).  The whole call -- 4 rounds of optimize(10), each restarted from mTcw, with the
// outlier classification after every round -- is ONE persistent workgroup per frame (a batch
// of frames is one launch).  Per LM iteration: one fused pass over the active edges (errors,
// robust chi2 and the 27 terms of the 6x6 system, canonical 64-tree sums of oracle/ba.c),
// then per trial the register-resident pivoted LDL^T + SE3 update on thread 0 and one error
// pass.  Edges are 32 B (the reference's float inputs; converted to double on load) and each
// wave prefetches its next chunk's edges while it computes the current one.
struct PoseEdgeDev {
    float Xw[3], obs[3];   // GetWorldPos(); kpUn.pt.x, .y, mvuRight
    float info;            // mvInvLevelSigma2[octave]
    int meta;              // bit 31: stereo edge; bits 0-30: keypoint index
};

struct PoseProbDev {
    int ne, e0;            // edges E[e0 .. e0+ne)
    int nbad, N;           // out: nBad of the last round (-1: < 3 correspondences)
    Se3 T0;                // Converter::toSE3Quat(pFrame->mTcw)
    Se3 T;                 // out
    double fx, fy, cx, cy, bf;
    // device mode: the frame's arrays in HBM (edges are built by k_pose_pack, results
    // written back by k_pose_opt's epilogue); null in host mode
    const float* Tcw;
    const uint8_t* has_mp;
    const float* Xw;
    const float* obs;
    const float* inv_sigma2;
    float* Tcw_out;
    uint8_t* outlier;
    // frame mode (pose_frame): gathered by k_pose_pack instead of the packed arrays above
    const int* mpidx;          // mvpMapPoints as indices (-1 NULL)
    const float* mp_pos;       // map point rows (GetWorldPos)
    const float* keys;         // mvKeysUn, 7 words per cv::KeyPoint (x y size angle response octave class_id)
    const float* uR;           // mvuRight
    const float* isig_tab;     // mvInvLevelSigma2
    int nlev;
    int* ninl;                 // optional device out: inliers (ne - nBad), 0 below 3 edges, -1 over capacity
};

// one edge in double (the g2o edge's _measurement / information / Huber delta)
struct PoseEdgeD {
    double X[3], obs[3], info, delta, dsqr;
    bool stereo;
};

__device__ __forceinline__ PoseEdgeD pose_edge_load(const PoseEdgeDev* E, int i, double dM, double dS) {
    const uint4* p = reinterpret_cast<const uint4*>(E + i);
    const uint4 a = p[0], b = p[1];
    PoseEdgeD e;
    e.X[0] = (double)__uint_as_float(a.x);
    e.X[1] = (double)__uint_as_float(a.y);
    e.X[2] = (double)__uint_as_float(a.z);
    e.obs[0] = (double)__uint_as_float(a.w);
    e.obs[1] = (double)__uint_as_float(b.x);
    e.obs[2] = (double)__uint_as_float(b.y);
    e.info = (double)__uint_as_float(b.z);
    e.stereo = (b.w >> 31) != 0;
    e.delta = e.stereo ? dS : dM;   // RobustKernelHuber delta = sqrt(chi2 threshold) as float
    e.dsqr = e.delta * e.delta;
    return e;
}

// the error at camera point p (dz: the shared divisions by p[2])
__device__ __forceinline__ void pose_err_p(const PoseEdgeD& e, const double* p, const SharedDiv& dz,
                                           const PoseProbDev& P, double* err) {
    if (!e.stereo) {
        const double px = dz.div(p[0]), py = dz.div(p[1]);
        err[0] = e.obs[0] - (px * P.fx + P.cx);
        err[1] = e.obs[1] - (py * P.fy + P.cy);
        err[2] = 0;
    } else {
        const float invz = (float)dz.div(1.0);
        const double u = (p[0] * (double)invz) * P.fx + P.cx;
        const double v = (p[1] * (double)invz) * P.fy + P.cy;
        err[0] = e.obs[0] - u;
        err[1] = e.obs[1] - v;
        err[2] = e.obs[2] - (u - P.bf * (double)invz);
    }
}

__device__ __forceinline__ void pose_err(const PoseEdgeD& e, const Se3& T, const PoseProbDev& P, double* err) {
    double p[3];
    se3_map(T, e.X, p);
    pose_err_p(e, p, SharedDiv(p[2]), P, err);
}

__device__ __forceinline__ double pose_chi2(const PoseEdgeD& e, const double* err) {
    double s = err[0] * (e.info * err[0]);
    s += err[1] * (e.info * err[1]);
    if (e.stereo) s += err[2] * (e.info * err[2]);
    return s;
}

__device__ __forceinline__ double pose_rho0(const PoseEdgeD& e, double c, bool robust) {
    if (!robust || c <= e.dsqr) return c;
    const double sq = sqrt(c);
    return (2 * sq) * e.delta - e.dsqr;
}


constexpr int kPoseMaxEdges = 8192;
// two waves per SIMD (512 threads): half the chunks per wave in every edge pass (the same
// canonical sums: bit-identical).  Measured in the pipeline beside the extraction grids too:
// 28.8 k vs 28.1 k frames/s for the one-wave-per-SIMD instance (256 threads) at B = 64, so
// every batch takes it; ORBGPU_POSE_WIDE_MAX = F keeps it for batches of at most F frames only
constexpr int kPoseThreads = 256, kPoseThreadsWide = 512;
static int pose_wide_max() {
    static const int v = [] {
        const char* e = getenv("ORBGPU_POSE_WIDE_MAX");
        return e ? atoi(e) : (1 << 30);
    }();
    return v;
}

// Opt-in (ORBGPU_POSE_LDS_KB=n): reserve n KiB of LDS per pose workgroup in the chained batch
// launch, so that the extraction grids' LDS-staged kernels cannot share the CUs the pose
// workgroups run on (dynamic bytes added on top of the kernel's static LDS)
static size_t pose_lds_pad(const void* fn) {
    static const int kb = [] {
        const char* e = getenv("ORBGPU_POSE_LDS_KB");
        return e ? atoi(e) : 0;
    }();
    if (kb <= 0) return 0;
    hipFuncAttributes a;
    if (hipFuncGetAttributes(&a, fn) != hipSuccess) return 0;
    const size_t want = (size_t)std::min(kb, 160) * 1024;
    return want > a.sharedSizeBytes ? want - a.sharedSizeBytes : 0;
}

// Canonical totals (ora_csum level 2) of the m chunk trees cs[q][0..m) of K sums, by wave 0:
// lane c holds chunk c and the K trees run packed (the same pairing as local_csum_inplace).
// K = 28 is split over waves 0-3, 7 trees each (every value's packed tree is the canonical one
// whatever the packing width, so the split changes no bit; wave 0 alone was a serial segment of
// every LM trial).
template <int K>
__device__ __forceinline__ void pose_chunk_totals(double (*cs)[kPoseMaxEdges / 64], int m, double* res) {
    constexpr int KW = K == 28 ? 7 : K;
    const int w = threadIdx.x >> 6;
    if (w >= K / KW) return;
    const int lane = threadIdx.x & 63, q0 = w * KW;
    if (m <= 1) {
        if (lane < KW) res[q0 + lane] = m == 1 ? cs[q0 + lane][0] : 0.0;
    } else if (m <= 64) {
        double v[KW];
#pragma unroll
        for (int q = 0; q < KW; q++) v[q] = lane < m ? cs[q0 + q][lane] : 0.0;
        const double t = packed_trees<KW>(v);
        const int q = bitrev6(lane);
        if (q < KW) res[q0 + q] = t;
    } else if (lane < KW) {
        res[q0 + lane] = local_csum_inplace(cs[q0 + lane], m);
    }
}

// Block-wide canonical sums (ora_csum) of K per-active-edge values: wave w owns chunks
// c = w, w + nw, ... of 64 active edges; the edge of chunk c + nw is loaded while chunk c is
// computed.  f(e, i, out[K]) evaluates active edge i (edge e loaded).  Chunk trees go to
// cs[q][c]; thread q < K finishes entry q.
template <int K, class F, class Post>
// post: run by thread 0 right after its own totals (res[0] among them) and before the closing
// barrier, i.e. beside the other waves' totals
__device__ __forceinline__ void pose_pass_post(F f, int nA, const uint16_t* aE, const PoseEdgeDev* E, double dM,
                                               double dS, double (*cs)[kPoseMaxEdges / 64], double* res,
                                               const PoseEdgeD& mine, int mineIdx, Post post) {
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, nw = blockDim.x >> 6;
    const int m = (nA + 63) >> 6;
    // chunk c = w is active edge tid: this thread's for the whole round, kept in registers
    // (loaded once per round); later chunks are loaded one ahead.  One code path for every
    // chunk count keeps a single inlined copy of f per call site (instruction-cache footprint)
    int c = w;
    int a = threadIdx.x;
    int i = mineIdx;
    PoseEdgeD e = mine;
    while (c < m) {
        const int cn = c + nw, an = cn * 64 + lane;
        int in = 0;
        PoseEdgeD en = e;
        if (cn < m) {   // prefetch the next chunk's edge
            in = an < nA ? aE[an] : 0;
            en = pose_edge_load(E, in, dM, dS);
        }
        double v[K];
        if (a < nA) f(e, i, v);
        else
#pragma unroll
            for (int q = 0; q < K; q++) v[q] = 0.0;
        if (nA == 1) {   // ora_csum keeps a single term untouched
            if (lane == 0)
#pragma unroll
                for (int q = 0; q < K; q++) cs[q][0] = v[q];
        } else {
            const double t = packed_trees<K>(v);
            const int q = bitrev6(lane);
            if (q < K) cs[q][c] = t;
        }
        c = cn;
        a = an;
        i = in;
        e = en;
    }
    __syncthreads();
    pose_chunk_totals<K>(cs, nA > 0 ? m : 0, res);
    if (threadIdx.x == 0) post();
    __syncthreads();
}
template <int K, class F>
__device__ __forceinline__ void pose_pass(F f, int nA, const uint16_t* aE, const PoseEdgeDev* E, double dM, double dS,
                                          double (*cs)[kPoseMaxEdges / 64], double* res, const PoseEdgeD& mine,
                                          int mineIdx) {
    pose_pass_post<K>(f, nA, aE, E, dM, dS, cs, res, mine, mineIdx, [] {});
}


// ---- wave-level dense solve of the pose system ---------------------------------------
__device__ __forceinline__ double lane_bcast(double v, int l) {
    const unsigned long long u = __double_as_longlong(v);
    const unsigned lo = __builtin_amdgcn_readlane((unsigned)(u & 0xffffffffu), l);
    const unsigned hi = __builtin_amdgcn_readlane((unsigned)(u >> 32), l);
    return __longlong_as_double(((unsigned long long)hi << 32) | lo);
}
// N independent IEEE divisions num[j] / den[j] as ONE lane-parallel division (lane j), results
// broadcast to every lane.  The whole wave must be active and hold the same operands.
template <int N>
__device__ __forceinline__ void lane_div(const double* num, const double* den, double* out) {
    const int lane = threadIdx.x & 63;
    double a = num[0], b = den[0];
#pragma unroll
    for (int j = 1; j < N; j++) {
        // opaque operands: a select chain over an array indexed by the lane otherwise becomes
        // a scratch-memory lookup
        double nj = num[j], dj = den[j];
        asm volatile("" : "+v"(nj), "+v"(dj));
        a = lane == j ? nj : a;
        b = lane == j ? dj : b;
    }
    const double q = a / b;
#pragma unroll
    for (int j = 0; j < N; j++) out[j] = lane_bcast(q, j);
}

// LinearSolverDense (Eigen LDLT with diagonal pivoting) of (H + lambda I) x = b, H the packed
// upper triangle Hs[21], run redundantly by a whole wave: the same IEEE operations as
// ldlt_pivot6.  Left-looking LDLT never touches a diagonal entry before its own step, so the
// pivot sequence is a function of |diag(H) + lambda| alone: it is fixed first, the
// factorisation then runs unpivoted on P A P^T with static register indices, and the row
// divisions of a step (and the 6 of the solve) are one lane-parallel division each.
__device__ __forceinline__ bool pose_solve_w(const double* Hs, const double* bs, double lambda, double* x) {
    // With distinct |pivots| the sequence is the descending order of |diag| (ties or NaN take
    // the reference routine: its tie-break follows the swap history).  Ranks instead of swaps
    // keep every index static (no scratch).
    double dv[6];
#pragma unroll
    for (int i = 0; i < 6; i++) dv[i] = fabs(Hs[DIAG21[i]] + lambda);
    bool distinct = true;
    int rank[6];
#pragma unroll
    for (int j = 0; j < 6; j++) {
        int r = 0;
        distinct = distinct && dv[j] == dv[j];
#pragma unroll
        for (int i = 0; i < 6; i++)
            if (i != j) {
                r += dv[i] > dv[j] ? 1 : 0;
                distinct = distinct && dv[i] != dv[j];
            }
        rank[j] = r;
    }
    int ord[6];
#pragma unroll
    for (int r = 0; r < 6; r++) {
        int o = 0;
#pragma unroll
        for (int j = 0; j < 6; j++) o = rank[j] == r ? j : o;
        ord[r] = o;
    }
    double A[36];   // lower triangle of P (H + lambda I) P^T
#pragma unroll
    for (int r = 0; r < 6; r++)
#pragma unroll
        for (int c = 0; c <= r; c++) {
            const int a = min(ord[r], ord[c]), b = max(ord[r], ord[c]);
            double h = Hs[a * 6 - (a * (a - 1)) / 2 + (b - a)];
            if (r == c) h += lambda;
            A[r * 6 + c] = h;
        }
    if (!distinct || !(fabs(A[0]) > 0.0)) {   // ties / NaN, or the reference's zero-pivot stop
        double Hd[36], bb[6];
#pragma unroll
        for (int r = 0, q = 0; r < 6; r++)
#pragma unroll
            for (int cc = r; cc < 6; cc++, q++) {
                double h = Hs[q];
                if (cc == r) h += lambda;
                Hd[r * 6 + cc] = h;
                Hd[cc * 6 + r] = h;
            }
#pragma unroll
        for (int j = 0; j < 6; j++) bb[j] = bs[j];
        return ldlt_pivot6(Hd, bb, x);
    }
    int sign = 0;
#pragma unroll
    for (int k = 0; k < 6; k++) {
        if (k > 0) {
            double tmp[6];
#pragma unroll
            for (int j = 0; j < k; j++) tmp[j] = A[j * 6 + j] * A[k * 6 + j];
            double s = 0;
#pragma unroll
            for (int j = 0; j < k; j++) s += A[k * 6 + j] * tmp[j];
            A[k * 6 + k] -= s;
#pragma unroll
            for (int i = k + 1; i < 6; i++) {
                double t = 0;
#pragma unroll
                for (int j = 0; j < k; j++) t += A[i * 6 + j] * tmp[j];
                A[i * 6 + k] -= t;
            }
        }
        const double akk = A[k * 6 + k];
        if (k < 5 && fabs(akk) > 0.0) {
            double num[5], den[5], q[5];
#pragma unroll
            for (int j = 0; j < 5; j++) {
                num[j] = k + 1 + j < 6 ? A[(k + 1 + j) * 6 + k] : 1.0;
                den[j] = akk;
            }
            lane_div<5>(num, den, q);
#pragma unroll
            for (int i = k + 1; i < 6; i++) A[i * 6 + k] = q[i - k - 1];
        }
        if (sign == 1) {
            if (akk < 0) sign = 3;
        } else if (sign == 2) {
            if (akk > 0) sign = 3;
        } else if (sign == 0) {
            if (akk > 0) sign = 1;
            else if (akk < 0) sign = 2;
        }
    }
    if (!(sign == 1 || sign == 0)) return false;
    double y[6];
#pragma unroll
    for (int i = 0; i < 6; i++) y[i] = bs[ord[i]];
#pragma unroll
    for (int i = 0; i < 6; i++)
#pragma unroll
        for (int j = 0; j < i; j++) y[i] -= A[i * 6 + j] * y[j];
    {
        double den[6], q[6];
#pragma unroll
        for (int i = 0; i < 6; i++) den[i] = A[i * 6 + i];
        lane_div<6>(y, den, q);
#pragma unroll
        for (int i = 0; i < 6; i++) y[i] = fabs(A[i * 6 + i]) > DBL_MIN ? q[i] : 0.0;
    }
#pragma unroll
    for (int i = 5; i >= 0; i--)
#pragma unroll
        for (int j = 5; j > i; j--) y[i] -= A[j * 6 + i] * y[j];
#pragma unroll
    for (int j = 0; j < 6; j++) {
        double v = 0.0;
#pragma unroll
        for (int p = 0; p < 6; p++)
            if (ord[p] == j) v = y[p];
        x[j] = v;
    }
    return true;
}

// The same solve with lane r holding row r of P (H + lambda I) P^T (lanes >= 6 shadow row 5):
// every IEEE operation of pose_solve_w, each row's in the lane that owns it, so a step's row
// updates and divisions are one lane-parallel instruction each and only the pivot and the
// finished y_j travel between lanes; the backward sweep reads the columns of L through scr
// (36 doubles of this wave's LDS).  x is returned in every lane.
__device__ __forceinline__ bool pose_solve_l(const double* Hs, const double* bs, double lambda, double* x,
                                             double* scr) {
    double dv[6];
#pragma unroll
    for (int i = 0; i < 6; i++) dv[i] = fabs(Hs[DIAG21[i]] + lambda);
    bool distinct = true;
    int rank[6];
#pragma unroll
    for (int j = 0; j < 6; j++) {
        int r = 0;
        distinct = distinct && dv[j] == dv[j];
#pragma unroll
        for (int i = 0; i < 6; i++)
            if (i != j) {
                r += dv[i] > dv[j] ? 1 : 0;
                distinct = distinct && dv[i] != dv[j];
            }
        rank[j] = r;
    }
    int ord[6];
#pragma unroll
    for (int r = 0; r < 6; r++) {
        int o = 0;
#pragma unroll
        for (int j = 0; j < 6; j++) o = rank[j] == r ? j : o;
        ord[r] = o;
    }
    const double a00 = Hs[DIAG21[ord[0]]] + lambda;
    if (!distinct || !(fabs(a00) > 0.0)) {   // ties / NaN, or the reference's zero-pivot stop
        double Hd[36], bb[6];
#pragma unroll
        for (int r = 0, q = 0; r < 6; r++)
#pragma unroll
            for (int cc = r; cc < 6; cc++, q++) {
                double h = Hs[q];
                if (cc == r) h += lambda;
                Hd[r * 6 + cc] = h;
                Hd[cc * 6 + r] = h;
            }
#pragma unroll
        for (int j = 0; j < 6; j++) bb[j] = bs[j];
        return ldlt_pivot6(Hd, bb, x);
    }
    const int lane = threadIdx.x & 63, row = lane < 6 ? lane : 5;
    int orow = ord[0];
#pragma unroll
    for (int p = 1; p < 6; p++) orow = row == p ? ord[p] : orow;
    double a[6];   // row `row` of P (H + lambda I) P^T, lower part used
#pragma unroll
    for (int c = 0; c < 6; c++) {
        const int i0 = min(orow, ord[c]), i1 = max(orow, ord[c]);
        double h = Hs[i0 * 6 - (i0 * (i0 - 1)) / 2 + (i1 - i0)];
        if (row == c) h += lambda;
        a[c] = h;
    }
    // branch-free: the reference's sign state machine ends in 1 / 2 / 3 / 0 exactly when some /
    // only positive, only negative, both, no nonzero pivots were seen, so two flags replace it
    double d[6];
    bool anyNeg = false;
#pragma unroll
    for (int k = 0; k < 6; k++) {
        if (k > 0) {
            double tmp[6];
#pragma unroll
            for (int j = 0; j < k; j++) tmp[j] = d[j] * lane_bcast(a[j], k);   // A[j][j] * A[k][j]
            double u = 0;
#pragma unroll
            for (int j = 0; j < k; j++) u += a[j] * tmp[j];
            const double ak = a[k] - u;
            a[k] = row >= k ? ak : a[k];
        }
        const double akk = lane_bcast(a[k], k);
        d[k] = akk;
        if (k < 5) {
            const double q = a[k] / akk;
            a[k] = (fabs(akk) > 0.0 && row > k) ? q : a[k];
        }
        anyNeg = anyNeg || akk < 0;
    }
    if (anyNeg) return false;
    double y = bs[orow];
#pragma unroll
    for (int j = 0; j < 5; j++) {
        const double yj = lane_bcast(y, j);
        const double v = y - a[j] * yj;
        y = row > j ? v : y;
    }
    double arr = a[0];
#pragma unroll
    for (int c = 1; c < 6; c++) arr = row == c ? a[c] : arr;   // own diagonal
    {
        const double q = y / arr;
        y = fabs(arr) > DBL_MIN ? q : 0.0;
    }
    // columns of L: lane r needs A[j][r], j > r
    if (lane < 6)
#pragma unroll
        for (int c = 0; c < 6; c++) scr[lane * 6 + c] = a[c];
    __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0)
    __builtin_amdgcn_wave_barrier();
    double col[6];
#pragma unroll
    for (int j = 0; j < 6; j++) col[j] = scr[j * 6 + row];
#pragma unroll
    for (int j = 5; j >= 1; j--) {
        const double xj = lane_bcast(y, j);
        const double v = y - col[j] * xj;
        y = row < j ? v : y;
    }
    double yb[6];
#pragma unroll
    for (int p = 0; p < 6; p++) yb[p] = lane_bcast(y, p);
#pragma unroll
    for (int j = 0; j < 6; j++) {
        double v = 0.0;
#pragma unroll
        for (int p = 0; p < 6; p++)
            if (ord[p] == j) v = yb[p];
        x[j] = v;
    }
    return true;
}

template <int NT>
__global__ void __launch_bounds__(NT) k_pose_opt(PoseProbDev* probs, const PoseEdgeDev* __restrict__ Eall,
                                                 double* errAll, uint8_t* outlAll) {
    ORBGPU_LATENCY_WAVE();
    constexpr int kPosePer = kPoseMaxEdges / NT;
    PoseProbDev& P = probs[blockIdx.x];
    const int ne = P.ne;
    const PoseEdgeDev* E = Eall + P.e0;
    (void)errAll;   // errors are recomputed at classification instead of kept per pass
    uint8_t* outl = outlAll + P.e0;
    // LDS kept near 53 KiB so three workgroups fit a CU next to the extraction kernels: edge
    // flags (bit 0: level 1 = inactive, bit 1: robust kernel set), active-edge list as u16
    __shared__ uint8_t fl[kPoseMaxEdges];
    __shared__ uint16_t aE[kPoseMaxEdges];
    __shared__ double cs[28][kPoseMaxEdges / 64];
    __shared__ double red[32];
    // speculative solves for 1..kPoseSpec consecutive rejections of a trial (waves 1..kPoseSpec)
    constexpr int kPoseSpec = 3;
    __shared__ Se3 T, Terr, Tbase, Tc[kPoseSpec + 1];   // Tc: the candidates of a round of trials
    __shared__ double xc[kPoseSpec + 1][6];
    __shared__ int okc[kPoseSpec + 1];
    __shared__ double scrSolve[kPoseSpec + 1][36];   // pose_solve_l's column exchange, one per solving wave
    __shared__ double xs[6], Hs[21], bs[6], sysN[28];
    __shared__ double lambda, ni, currentChi, iniChi;
    __shared__ int nA, nBadLM, qmax, again, term, nBad, haveSys, specPass, wsum[16];
    const int tid = threadIdx.x;
    const double dM = (double)(float)sqrt(5.991), dS = (double)(float)sqrt(7.815);
    if (ne < 0) {   // device mode: capacity exceeded (reported by the host)
        if (tid == 0 && P.ninl) *P.ninl = -1;
        return;
    }
    if (ne < 3) {
        if (tid == 0) {
            P.T = P.T0;
            P.nbad = -1;
            if (P.ninl) *P.ninl = 0;
        }
        if (P.Tcw_out) {
            if (tid < 16) P.Tcw_out[tid] = P.Tcw[tid];
            for (int i = tid; i < ne; i += blockDim.x) P.outlier[E[i].meta & 0x7fffffff] = 0;
            // Tcw_out may be pinned host memory read by a host that polls a later kernel's signal
            // word: write the pose back at system scope before this workgroup ends
            if (tid < 16) __threadfence_system();
        }
        return;
    }
    for (int i = tid; i < ne; i += blockDim.x) {
        fl[i] = 2;
        outl[i] = 0;
    }
    __syncthreads();
    const float chi2Mono = 5.991f, chi2Stereo = 7.815f;
    for (int it = 0; it < 4; it++) {
        if (tid == 0) {
            T = P.T0;   // vSE3->setEstimate(Converter::toSE3Quat(pFrame->mTcw)) every round
            for (int j = 0; j < 6; j++) xs[j] = 0.0;
        }
        // active edges (level 0) in edge order: block prefix over kPosePer edges per thread
        {
            const int base = tid * kPosePer;
            int c = 0;
            for (int j = 0; j < kPosePer; j++) c += (base + j < ne && (fl[base + j] & 1) == 0) ? 1 : 0;
            int incl = c;   // inclusive scan within the wave
            for (int o = 1; o < 64; o <<= 1) {
                const int t = __shfl_up(incl, o, 64);
                if ((tid & 63) >= o) incl += t;
            }
            if ((tid & 63) == 63) wsum[tid >> 6] = incl;
            __syncthreads();
            int off = 0;
            for (int w = 0; w < (tid >> 6); w++) off += wsum[w];
            int pos = off + incl - c;
            for (int j = 0; j < kPosePer; j++)
                if (base + j < ne && (fl[base + j] & 1) == 0) aE[pos++] = (uint16_t)(base + j);
            if (tid == blockDim.x - 1) nA = off + incl;
            __syncthreads();
        }
        const int na = nA;
        const int myIdx = tid < na ? aE[tid] : 0;
        const PoseEdgeD myE = pose_edge_load(E, myIdx, dM, dS);
        if (na > 0) {   // optimize(10); without active edges the vertex is not optimised at all
            ORBGPU_PROF_START;
            // J, robust weight and the 28 entries (robust chi2, J^T W J upper triangle, -J^T W e)
            // of active edge i at pose X, into v[0..28)
            auto sys_terms = [&](const PoseEdgeD& e, int i, const Se3& X, double* v) {
                double p[3];
                se3_map(X, e.X, p);
                const SharedDiv dz(p[2]);
                double e3[3];
                pose_err_p(e, p, dz, P, e3);
                const double c = pose_chi2(e, e3);
                const bool rb = (fl[i] & 2) != 0;
                v[0] = pose_rho0(e, c, rb);
                const double x = p[0], y = p[1], invz = dz.div(1.0), invz_2 = invz * invz;
                double J[18];
                J[0] = ((x * y) * invz_2) * P.fx;
                J[1] = (-(1 + ((x * x) * invz_2))) * P.fx;
                J[2] = (y * invz) * P.fx;
                J[3] = (-invz) * P.fx;
                J[4] = 0;
                J[5] = (x * invz_2) * P.fx;
                J[6] = (1 + ((y * y) * invz_2)) * P.fy;
                J[7] = (((-x) * y) * invz_2) * P.fy;
                J[8] = ((-x) * invz) * P.fy;
                J[9] = 0;
                J[10] = (-invz) * P.fy;
                J[11] = (y * invz_2) * P.fy;
                J[12] = J[0] - ((P.bf * y) * invz_2);
                J[13] = J[1] + ((P.bf * x) * invz_2);
                J[14] = J[2];
                J[15] = J[3];
                J[16] = 0;
                J[17] = J[5] - (P.bf * invz_2);
                // monocular edges: a zero third Jacobian row (and err[2] = 0) makes every
                // third term +-0, an exact identity on the two-term partial sums (which
                // start from +0 + t0 and so are never -0): the sums run branch-free
#pragma unroll
                for (int j = 12; j < 18; j++) J[j] = e.stereo ? J[j] : 0.0;
                double r1 = 1.;
                if (rb && !(c <= e.dsqr)) r1 = e.delta / sqrt(c);
                const double wgt = rb ? r1 * e.info : e.info;
                double omr[3];
#pragma unroll
                for (int kk = 0; kk < 3; kk++) {
                    omr[kk] = -(e.info * e3[kk]);
                    if (rb) omr[kk] *= r1;
                }
#pragma unroll
                for (int r = 0; r < 6; r++) {
                    double sb = 0;
#pragma unroll
                    for (int kk = 0; kk < 3; kk++) sb += J[kk * 6 + r] * omr[kk];
                    v[22 + r] = sb;
#pragma unroll
                    for (int cc = r; cc < 6; cc++) {
                        double hh = 0;
#pragma unroll
                        for (int kk = 0; kk < 3; kk++) hh += (J[kk * 6 + r] * wgt) * J[kk * 6 + cc];
                        v[1 + r * 6 - (r * (r - 1)) / 2 + (cc - r)] = hh;
                    }
                }
            };
            // One LM iteration is a system pass at T (skipped when the accepted trial of the
            // previous iteration already evaluated it) followed by trials; a trial is the solves
            // (waves 0..kPoseSpec) and ONE pass at candidate 0.  Both passes run through the same
            // call site (sysPhase picks the pose), and the four solves through one: a single
            // inlined copy of the 28-sum edge body keeps the LM loop's code within the
            // instruction cache the workgroup shares with its neighbours.
            if (tid == 0) haveSys = 0;
            __syncthreads();
            int kit = 0;            // LM iteration (uniform: every thread steps it alike)
            bool sysPhase = true;   // the next pass evaluates the system at T
            for (;;) {
                if (!sysPhase) {
                    ORBGPU_PROF_MARK(10);
                    // Trials, up to four per round: candidate 0 solves at the current lambda
                    // (wave 0) while waves 1..kPoseSpec solve the systems of 1..kPoseSpec
                    // consecutive rejections (lambda *= ni; ni *= 2, the same H, b and starting
                    // estimate).  The pass of the first trial computes the whole system at
                    // candidate 0 (its robust chi2 is entry 0), so an accepted first trial hands
                    // the next iteration its system; a rejected one is followed by ONE pass for
                    // the speculative candidates, whose trials are then replayed in the
                    // reference's order.
                    if (tid < 64 * (kPoseSpec + 1)) {
                        const int L = tid >> 6;   // 0: the current trial, L: L rejections ahead
                        double ls = lambda, ns = ni;
                        for (int j = 0; j < L; j++) {
                            ls *= ns;
                            ns *= 2;
                        }
                        double xn[6];
#ifndef ORBGPU_POSE_SOLVE_W
                        const bool ok = pose_solve_l(Hs, bs, ls, xn, scrSolve[L]);
#else
                        const bool ok = pose_solve_w(Hs, bs, ls, xn);
#endif
                        ORBGPU_PROF_MARK(5);
                        ORBGPU_PROF_COUNT(9);
                        // candidate 0 steps from xs when the solve fails (its trial is then
                        // rejected: tempChi = DBL_MAX); a failed speculative solve stays at Tbase
                        double xl[6];
#pragma unroll
                        for (int j = 0; j < 6; j++) xl[j] = (ok || L > 0) ? xn[j] : xs[j];
                        Se3 r = Tbase;
                        if (ok || L == 0) {
                            Se3 d;
                            se3_exp(xl, d);
                            se3_mul(d, Tbase, r);
                        }
                        if ((tid & 63) == 0) {
                            Tc[L] = r;
#pragma unroll
                            for (int j = 0; j < 6; j++) xc[L][j] = xl[j];
                            okc[L] = ok ? 1 : 0;
                        }
                    }
                    __syncthreads();
                    ORBGPU_PROF_MARK(2);
                } else {
                    ORBGPU_PROF_MARK(0);
                    ORBGPU_PROF_COUNT(8);
                }
                // one trial of the reference's loop (optimization_algorithm_levenberg.cpp:100-149)
                // at candidate j with robust chi2 tempChi; tid 0 only
                auto trial = [&](int j, double tempChi) {
                    if (!okc[j]) tempChi = DBL_MAX;
#pragma unroll
                    for (int q = 0; q < 6; q++) xs[q] = xc[j][q];
                    double rho = currentChi - tempChi;
                    double sv[6];
                    for (int q = 0; q < 6; q++) sv[q] = xs[q] * (lambda * xs[q] + bs[q]);
                    double scale = tree64_local([&](int q) { return sv[q]; }, 6);
                    scale += 1e-3;
                    rho /= scale;
                    Terr = Tc[j];   // the pose of the last computeActiveErrors
                    if (rho > 0 && isfinite(tempChi)) {
                        const double a3 = 2 * rho - 1;
                        double alpha = 1. - (a3 * a3) * a3;
                        alpha = fmin(alpha, 2. / 3.);
                        const double scaleFactor = fmax(1. / 3., alpha);
                        lambda *= scaleFactor;
                        ni = 2;
                        currentChi = tempChi;
                        T = Tc[j];
                        if (j == 0) haveSys = 1;   // red[0..28) is the system at the new estimate
                    } else {
                        lambda *= ni;
                        ni *= 2;
                        T = Tbase;
                    }
                    qmax++;
                    again = (rho < 0 && qmax < 10) ? 1 : 0;
                    if (!again) {
                        if (qmax == 10 || rho == 0) {
                            term = 1;
                        } else {
                            if ((iniChi - currentChi) * 1e3 < iniChi) nBadLM++;
                            else nBadLM = 0;
                            term = nBadLM >= 3 ? 1 : 0;
                        }
                    }
                };
                // sysPhase: computeActiveErrors + activeRobustChi2 (entry 0) and buildSystem
                // (entries 1..27) at T; a trial: its robust chi2 at candidate 0 and, with it, the
                // system at that estimate (the next iteration's whenever the trial is accepted).
                // Canonical sums per entry.
                {   // a trial's decision runs on thread 0 as soon as its chi2 total (red[0]) is in,
                    // beside the other waves' totals (the pass reads no state the decision writes)
                    const Se3& X = sysPhase ? T : Tc[0];
                    pose_pass_post<28>([&](const PoseEdgeD& e, int i, double* v) { sys_terms(e, i, X, v); }, na, aE, E,
                                       dM, dS, cs, red, myE, myIdx, [&] {
                                           if (!sysPhase) {
                                               trial(0, red[0]);
                                               specPass = again && okc[1] ? 1 : 0;
                                           }
                                       });
                }
                if (sysPhase) {
                    ORBGPU_PROF_MARK(1);
                    if (tid < 28) {
                        if (tid == 0) currentChi = iniChi = red[0];
                        else if (tid < 22) Hs[tid - 1] = red[tid];
                        else bs[tid - 22] = red[tid];
                    }
                } else {
                    ORBGPU_PROF_MARK(3);
                    if (haveSys && tid < 28) sysN[tid] = red[tid];
                    if (specPass) {
                        // candidate 0 rejected: the speculative candidates' robust chi2 in one pass,
                        // then their trials in order while they are rejected
                        pose_pass<kPoseSpec>([&](const PoseEdgeD& e, int i, double* v) {
#pragma unroll
                            for (int L = 1; L <= kPoseSpec; L++) {
                                double e3[3];
                                pose_err(e, Tc[L], P, e3);
                                v[L - 1] = pose_rho0(e, pose_chi2(e, e3), (fl[i] & 2) != 0);
                            }
                        }, na, aE, E, dM, dS, cs, red, myE, myIdx);
                        if (tid == 0)
                            for (int j = 1; j <= kPoseSpec && again && okc[j]; j++) trial(j, red[j - 1]);
                        __syncthreads();
                    }
                    ORBGPU_PROF_MARK(4);
                    if (again) continue;   // the next trial of this iteration
                    __syncthreads();
                    if (term || ++kit == 10) break;
                    if (!haveSys) {   // the next iteration starts with a system pass at T
                        sysPhase = true;
                        continue;
                    }
                    if (tid < 28) {   // the system at this estimate came with its accepted trial
                        if (tid == 0) currentChi = iniChi = sysN[0];
                        else if (tid < 22) Hs[tid - 1] = sysN[tid];
                        else bs[tid - 22] = sysN[tid];
                    }
                }
                // iteration start (Hs, bs, currentChi = iniChi are the system at T)
                __syncthreads();
                if (tid == 0) {
                    if (kit == 0) {   // computeLambdaInit over the pose diagonal
                        double mx = 0.;
                        for (int j = 0; j < 6; j++) mx = fmax(fabs(Hs[DIAG21[j]]), mx);
                        lambda = 1e-5 * mx;
                        ni = 2;
                        nBadLM = 0;
                    }
                    qmax = 0;
                    haveSys = 0;
                    Tbase = T;   // the estimate every trial of this iteration starts from
                }
                sysPhase = false;
                __syncthreads();
            }
        }
        // classification (Optimizer.cc:376-426): outliers get their error recomputed
        if (tid == 0) nBad = 0;
        __syncthreads();
        int mybad = 0;
        for (int i = tid; i < ne; i += blockDim.x) {
            const PoseEdgeD e = pose_edge_load(E, i, dM, dS);
            // active edges keep the error of the last pass (recomputed: the same operations on
            // the same pose), outliers get computeError() at the final estimate
            double e3[3];
            pose_err(e, outl[i] ? T : Terr, P, e3);
            const float chi2 = (float)pose_chi2(e, e3);
            uint8_t f = fl[i];
            if (chi2 > (e.stereo ? chi2Stereo : chi2Mono)) {
                outl[i] = 1;
                f |= 1;
                mybad++;
            } else {
                outl[i] = 0;
                f &= 2;
            }
            if (it == 2) f &= 1;   // setRobustKernel(0)
            fl[i] = f;
        }
        if (mybad) atomicAdd(&nBad, mybad);
        __syncthreads();
        if (ne < 10) break;   // optimizer.edges().size() < 10
    }
    if (tid == 0) {
        P.T = T;
        P.nbad = nBad;
        if (P.ninl) *P.ninl = ne - nBad;
    }
    if (P.Tcw_out) {   // pFrame->SetPose(Converter::toCvMat(SE3quat_recov)); mvbOutlier
        if (tid == 0) {
            double R[9];
            quat_to_R(T.q, R);
            float* o = P.Tcw_out;
            for (int r = 0; r < 3; r++) {
                for (int c = 0; c < 3; c++) o[r * 4 + c] = (float)R[r * 3 + c];
                o[r * 4 + 3] = (float)T.t[r];
            }
            o[12] = o[13] = o[14] = 0.f;
            o[15] = 1.f;
            __threadfence_system();   // see the ne < 3 exit above: host-visible before the workgroup ends
        }
        for (int i = tid; i < ne; i += blockDim.x) P.outlier[E[i].meta & 0x7fffffff] = outl[i];
    }
}

// Device mode edge creation (Optimizer.cc:268-347): rows with a map point, keypoint order,
// compacted by a block scan; the initial pose from the frame's Tcw.  One workgroup per frame.
// 4 waves: the pack fits in the slot of one retiring extraction workgroup
constexpr int kPackThreads = 256;
__global__ void __launch_bounds__(kPackThreads) k_pose_pack(PoseProbDev* probs, PoseEdgeDev* Eall) {
    ORBGPU_LATENCY_WAVE();
    PoseProbDev& P = probs[blockIdx.x];
    const int N = P.N, tid = threadIdx.x;
    PoseEdgeDev* E = Eall + P.e0;
    __shared__ int wsum[kPackThreads / 64], base;
    if (tid == 0) {
        base = 0;
        double R[9];
        for (int r = 0; r < 3; r++)
            for (int c = 0; c < 3; c++) R[r * 3 + c] = (double)P.Tcw[r * 4 + c];
        quat_from_R(R, P.T0.q);
        for (int r = 0; r < 3; r++) P.T0.t[r] = (double)P.Tcw[r * 4 + 3];
        P.T0.pad = 0;
        se3_normalize(P.T0);
    }
    __syncthreads();
    for (int c0 = 0; c0 < N; c0 += kPackThreads) {
        const int i = c0 + tid;
        const int f = i < N ? (P.mpidx ? (P.mpidx[i] >= 0 ? 1 : 0) : (P.has_mp[i] ? 1 : 0)) : 0;
        int incl = f;
        for (int o = 1; o < 64; o <<= 1) {
            const int t = __shfl_up(incl, o, 64);
            if ((tid & 63) >= o) incl += t;
        }
        if ((tid & 63) == 63) wsum[tid >> 6] = incl;
        __syncthreads();
        int off = base;
        for (int w = 0; w < (tid >> 6); w++) off += wsum[w];
        if (f) {
            const int k = off + incl - 1;
            if (k < kPoseMaxEdges) {
                PoseEdgeDev e;
                if (P.mpidx) {
                    // Optimizer.cc:268-347: pMP->GetWorldPos(), kpUn.pt, mvuRight, mvInvLevelSigma2[kpUn.octave]
                    const size_t m = (size_t)P.mpidx[i];
                    for (int j = 0; j < 3; j++) e.Xw[j] = P.mp_pos[3 * m + j];
                    e.obs[0] = P.keys[7 * (size_t)i];
                    e.obs[1] = P.keys[7 * (size_t)i + 1];
                    e.obs[2] = P.uR[i];
                    const int oct = min(max(__float_as_int(P.keys[7 * (size_t)i + 5]), 0), P.nlev - 1);
                    e.info = P.isig_tab[oct];
                } else {
                    for (int j = 0; j < 3; j++) {
                        e.Xw[j] = P.Xw[3 * i + j];
                        e.obs[j] = P.obs[3 * i + j];
                    }
                    e.info = P.inv_sigma2[i];
                }
                e.meta = i | (!(e.obs[2] < 0) ? (int)0x80000000u : 0);
                E[k] = e;
            }
        }
        __syncthreads();
        if (tid == kPackThreads - 1) base = off + incl;
        __syncthreads();
    }
    if (tid == 0) P.ne = base > kPoseMaxEdges ? -1 : base;
}

// ---------------------------------------------------------------- host
static void host_se3_from_Tcw(const float* T, Se3& o) {
    double R[9];
    for (int r = 0; r < 3; r++)
        for (int c = 0; c < 3; c++) R[r * 3 + c] = (double)T[r * 4 + c];
    quat_from_R(R, o.q);
    for (int r = 0; r < 3; r++) o.t[r] = (double)T[r * 4 + 3];
    o.pad = 0;
    se3_normalize(o);
}

static void host_se3_to_Tcw(const Se3& s, float* T) {
    double R[9];
    quat_to_R(s.q, R);
    for (int r = 0; r < 3; r++) {
        for (int c = 0; c < 3; c++) T[r * 4 + c] = (float)R[r * 3 + c];
        T[r * 4 + 3] = (float)s.t[r];
    }
    T[12] = T[13] = T[14] = 0.f;
    T[15] = 1.f;
}

// ---------------------------------------------------------------- PoseEngine
int PoseEngine::run_device(int count, const pose_problem* P, float* const* Tcw_out, uint8_t* const* outlier,
                           int* ninliers) {
    std::vector<int> Ns(count);
    for (int f = 0; f < count; f++) Ns[f] = P[f].N;
    return launch_device(count, Ns.data(), [&](int f, PoseProbDev& pp) {
        const pose_problem& Q = P[f];
        pp.fx = Q.fx; pp.fy = Q.fy; pp.cx = Q.cx; pp.cy = Q.cy; pp.bf = Q.bf;
        pp.Tcw = Q.Tcw; pp.has_mp = Q.has_mp; pp.Xw = Q.Xw; pp.obs = Q.obs; pp.inv_sigma2 = Q.inv_sigma2;
    }, Tcw_out, outlier, ninliers);
}

int PoseEngine::run_frames_device(int count, const pose_frame* F, float* const* Tcw_out, uint8_t* const* outlier,
                                  int* ninliers, hipStream_t s, DeferredChain* chain) {
    std::vector<int> Ns(count);
    for (int f = 0; f < count; f++) Ns[f] = F[f].N;
    return launch_device(count, Ns.data(), [&](int f, PoseProbDev& pp) {
        const pose_frame& Q = F[f];
        pp.fx = Q.fx; pp.fy = Q.fy; pp.cx = Q.cx; pp.cy = Q.cy; pp.bf = Q.bf;
        pp.Tcw = Q.Tcw;
        pp.mpidx = Q.mp; pp.mp_pos = Q.mp_pos; pp.keys = (const float*)Q.keysUn; pp.uR = Q.uRight;
        pp.isig_tab = Q.invLevelSigma2; pp.nlev = Q.nlevels;
    }, Tcw_out, outlier, ninliers, s, chain);
}

// Device-mode launch.  Default: own stream, results synchronised before return.  With a
// DeferredChain: enqueued on `s` behind the caller's previous work, the problem table staged
// through the chain's pinned blocks and the inlier counts landing in `ninliers` at
// chain.finish() (-1 for a frame over kPoseMaxEdges).
int PoseEngine::launch_device(int count, const int* Ns, const std::function<void(int, PoseProbDev&)>& fill,
                              float* const* Tcw_out, uint8_t* const* outlier, int* ninliers, hipStream_t s,
                              DeferredChain* chain) {
    hipStream_t st = s ? s : stream_;
    size_t nmax = 0;
    for (int f = 0; f < count; f++) nmax += (size_t)std::min(Ns[f], kPoseMaxEdges + 1);
    const auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
    const size_t bProb = al(sizeof(PoseProbDev) * count), bEdge = al(sizeof(PoseEdgeDev) * std::max<size_t>(nmax, 1));
    const size_t bOut = al(std::max<size_t>(nmax, 1)), bNin = al(sizeof(int) * count);
    const size_t need = bProb + bEdge + bOut + bNin;
    if (need > cap_) {
        if (lastUseSet_) ORB_HIP_CHECK(hipEventSynchronize(lastUse_));   // queued kernels may still read it
        if (dArena_) (void)hipFree(dArena_);
        if (hArena_) (void)hipHostFree(hArena_);
        dArena_ = hArena_ = nullptr;
        cap_ = 0;
        ORB_HIP_CHECK(hipMalloc(&dArena_, need));
        ORB_HIP_CHECK(hipHostMalloc(&hArena_, need));
        cap_ = need;
    }
    char* d = (char*)dArena_;
    // inlier counts: the arena, or in a chain its count blocks (copied when the chain closes)
    int* dNin = chain ? (int*)chain->dev_counts(sizeof(int) * count) : (int*)(d + bProb + bEdge + bOut);
    if (!dNin) return -2;
    std::vector<PoseProbDev> tmp;
    PoseProbDev* hp = (PoseProbDev*)hArena_;
    if (chain) {   // hArena_ may still be the source of an earlier queued copy: stage instead
        tmp.resize(count);
        hp = tmp.data();
    }
    size_t e0 = 0;
    for (int f = 0; f < count; f++) {
        PoseProbDev& pp = hp[f];
        memset(&pp, 0, sizeof(pp));
        pp.N = Ns[f];
        pp.e0 = (int)e0;
        e0 += (size_t)std::min(Ns[f], kPoseMaxEdges + 1);
        fill(f, pp);
        pp.Tcw_out = Tcw_out[f];
        pp.outlier = outlier[f];
        pp.ninl = dNin + f;
    }
    PoseProbDev* dp = (PoseProbDev*)d;
    PoseEdgeDev* dE = (PoseEdgeDev*)(d + bProb);
    const void* src = chain ? chain->stage(hp, sizeof(PoseProbDev) * count) : (const void*)hp;
    if (!src) return -2;
    // the arena's previous user may be queued on another stream (a deferred chain of another
    // matcher, or this engine's own stream): overwrite the problem table only after it is done
    if (lastUseSet_) ORB_HIP_CHECK(hipStreamWaitEvent(st, lastUse_, 0));
    ORB_HIP_CHECK(hipMemcpyAsync(d, src, sizeof(PoseProbDev) * count, hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(k_pose_pack, dim3(count), dim3(kPackThreads), 0, st, dp, dE);
    if (timing_) ORB_HIP_CHECK(hipEventRecord(tA_, st));
    if (count <= pose_wide_max())
        hipLaunchKernelGGL(k_pose_opt<kPoseThreadsWide>, dim3(count), dim3(kPoseThreadsWide),
                           pose_lds_pad((const void*)k_pose_opt<kPoseThreadsWide>), st, dp, (const PoseEdgeDev*)dE,
                           nullptr, (uint8_t*)(d + bProb + bEdge));
    else
        hipLaunchKernelGGL(k_pose_opt<kPoseThreads>, dim3(count), dim3(kPoseThreads),
                           pose_lds_pad((const void*)k_pose_opt<kPoseThreads>), st, dp, (const PoseEdgeDev*)dE, nullptr,
                           (uint8_t*)(d + bProb + bEdge));
    ORB_HIP_CHECK(hipGetLastError());
    if (timing_) {
        ORB_HIP_CHECK(hipEventRecord(tB_, st));
        timed_ = true;
    }
    if (chain) {
        chain->land_dev(ninliers, dNin, sizeof(int) * count);
        ORB_HIP_CHECK(hipEventRecord(lastUse_, st));
        lastUseSet_ = true;
        return 0;
    }
    ORB_HIP_CHECK(hipMemcpyAsync(hp, d, bProb, hipMemcpyDeviceToHost, st));
    ORB_HIP_CHECK(hipEventRecord(lastUse_, st));
    lastUseSet_ = true;
    ORB_HIP_CHECK(stream_wait(st));
    int rc = 0;
    for (int f = 0; f < count; f++) {
        const PoseProbDev& pp = hp[f];
        if (pp.ne < 0) rc = -3;
        ninliers[f] = pp.ne < 0 || pp.nbad < 0 ? 0 : pp.ne - pp.nbad;
    }
    return rc;
}

int PoseEngine::last_timing(float* ms) {
    if (!timed_) return -1;
    ORB_HIP_CHECK(hipEventSynchronize(tB_));
    ORB_HIP_CHECK(hipEventElapsedTime(ms, tA_, tB_));
    return 0;
}

PoseEngine::~PoseEngine() {
    if (lastUseSet_) (void)hipEventSynchronize(lastUse_);
    if (lastUse_) (void)hipEventDestroy(lastUse_);
    if (tA_) (void)hipEventDestroy(tA_);
    if (tB_) (void)hipEventDestroy(tB_);
    if (dArena_) (void)hipFree(dArena_);
    if (hArena_) (void)hipHostFree(hArena_);
    if (stream_) (void)hipStreamDestroy(stream_);
}

int PoseEngine::init() {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return -4;
    ORB_HIP_CHECK(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
    ORB_HIP_CHECK(hipEventCreateWithFlags(&lastUse_, hipEventDisableTiming));
    ORB_HIP_CHECK(hipEventCreate(&tA_));
    ORB_HIP_CHECK(hipEventCreate(&tB_));
    return 0;
}

// Edge creation (Optimizer.cc:268-347): rows with a map point in keypoint order.
int PoseEngine::run(int count, const pose_problem* P, float* Tcw_out, uint8_t* const* outlier, int* ninliers) {
    size_t ne = 0;
    std::vector<int> nE(count);
    for (int f = 0; f < count; f++) {
        int c = 0;
        for (int i = 0; i < P[f].N; i++) c += P[f].has_mp[i] ? 1 : 0;
        if (c > kPoseMaxEdges) return -3;
        nE[f] = c;
        ne += c;
    }
    const auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
    const size_t bProb = al(sizeof(PoseProbDev) * count), bEdge = al(sizeof(PoseEdgeDev) * std::max<size_t>(ne, 1));
    const size_t bErr = al(sizeof(double) * 3 * std::max<size_t>(ne, 1)), bOut = al(std::max<size_t>(ne, 1));
    const size_t need = bProb + bEdge + bErr + bOut;
    if (lastUseSet_) ORB_HIP_CHECK(hipEventSynchronize(lastUse_));   // hArena_ / dArena_ free again
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
    PoseProbDev* hp = (PoseProbDev*)h;
    PoseEdgeDev* he = (PoseEdgeDev*)(h + bProb);
    uint8_t* hOut = (uint8_t*)(h + bProb + bEdge + bErr);
    int e0 = 0;
    for (int f = 0; f < count; f++) {
        const pose_problem& Q = P[f];
        PoseProbDev& pp = hp[f];
        memset(&pp, 0, sizeof(pp));
        pp.ne = nE[f];
        pp.e0 = e0;
        host_se3_from_Tcw(Q.Tcw, pp.T0);
        pp.fx = Q.fx; pp.fy = Q.fy; pp.cx = Q.cx; pp.cy = Q.cy; pp.bf = Q.bf;
        for (int i = 0; i < Q.N; i++) {
            if (!Q.has_mp[i]) continue;
            PoseEdgeDev& e = he[e0++];
            for (int j = 0; j < 3; j++) {
                e.Xw[j] = Q.Xw[3 * i + j];
                e.obs[j] = Q.obs[3 * i + j];
            }
            e.info = Q.inv_sigma2[i];
            e.meta = i | (!(Q.obs[3 * i + 2] < 0) ? (int)0x80000000u : 0);
        }
    }
    PoseProbDev* dp = (PoseProbDev*)d;
    ORB_HIP_CHECK(hipMemcpyAsync(d, h, bProb + sizeof(PoseEdgeDev) * ne, hipMemcpyHostToDevice, stream_));
    if (count > 0)
    {
        if (count <= pose_wide_max())
            hipLaunchKernelGGL(k_pose_opt<kPoseThreadsWide>, dim3(count), dim3(kPoseThreadsWide), 0, stream_, dp, (const PoseEdgeDev*)(d + bProb),
                               (double*)(d + bProb + bEdge), (uint8_t*)(d + bProb + bEdge + bErr));
        else
            hipLaunchKernelGGL(k_pose_opt<kPoseThreads>, dim3(count), dim3(kPoseThreads), 0, stream_, dp, (const PoseEdgeDev*)(d + bProb),
                               (double*)(d + bProb + bEdge), (uint8_t*)(d + bProb + bEdge + bErr));
    }
    ORB_HIP_CHECK(hipGetLastError());
    ORB_HIP_CHECK(hipMemcpyAsync(h, d, bProb, hipMemcpyDeviceToHost, stream_));
    if (ne) ORB_HIP_CHECK(hipMemcpyAsync(hOut, d + bProb + bEdge + bErr, ne, hipMemcpyDeviceToHost, stream_));
    ORB_HIP_CHECK(hipEventRecord(lastUse_, stream_));
    lastUseSet_ = true;
    ORB_HIP_CHECK(hipStreamSynchronize(stream_));
    for (int f = 0; f < count; f++) {
        const pose_problem& Q = P[f];
        const PoseProbDev& pp = hp[f];
        const uint8_t* o = hOut + pp.e0;
        for (int i = 0, k = 0; i < Q.N; i++)
            if (Q.has_mp[i]) {
                outlier[f][i] = pp.nbad < 0 ? 0 : o[k];
                k++;
            }
        if (pp.nbad < 0) {   // nInitialCorrespondences < 3: return 0, pose untouched
            memcpy(Tcw_out + 16 * (size_t)f, Q.Tcw, sizeof(float) * 16);
            ninliers[f] = 0;
        } else {
            host_se3_to_Tcw(pp.T, Tcw_out + 16 * (size_t)f);
            ninliers[f] = pp.ne - pp.nbad;
        }
    }
    return 0;
}

BaEngine::~BaEngine() {
    if (stream_) (void)hipStreamSynchronize(stream_);
    if (dPack_) (void)hipFree(dPack_);
    if (arena_) (void)hipFree(arena_);
    if (dStruct_) (void)hipFree(dStruct_);
    if (dLmStage_) (void)hipFree(dLmStage_);
    if (hScal_) (void)hipHostFree(hScal_);
    if (hLm_) (void)hipHostFree(hLm_);
    for (auto ev : lmEv_)
        if (ev) (void)hipEventDestroy(ev);
    if (hStage_) (void)hipHostFree(hStage_);
    if (hStage2_) (void)hipHostFree(hStage2_);
    if (stream_) (void)hipStreamDestroy(stream_);
}

int BaEngine::stage_reserve(size_t bytes) {
    if (uploadPending_) {   // the problem upload may still read the staging block
        uploadPending_ = false;
        if (int e = poll_stream()) return e;
    }
    if (bytes <= hStageCap_) return 0;
    if (hStage_) (void)hipHostFree(hStage_);
    hStage_ = nullptr;
    hStageCap_ = 0;
    ORB_HIP_CHECK(hipHostMalloc(&hStage_, bytes));
    hStageCap_ = bytes;
    return 0;
}

int BaEngine::stage2_reserve(size_t bytes) {
    if (stage2Pending_) {   // the previous structure's copy may still read the block
        stage2Pending_ = false;
        if (int e = poll_stream()) return e;
    }
    if (bytes <= hStage2Cap_) return 0;
    if (hStage2_) (void)hipHostFree(hStage2_);
    hStage2_ = nullptr;
    hStage2Cap_ = 0;
    ORB_HIP_CHECK(hipHostMalloc(&hStage2_, bytes));
    hStage2Cap_ = bytes;
    return 0;
}

// H2D / D2H copies of host bytes through the engine's pinned staging block, complete on return
int BaEngine::h2d_sync(void* dst, const void* src, size_t bytes) {
    if (!bytes) return 0;
    if (int e = stage_reserve(bytes)) return e;
    std::memcpy(hStage_, src, bytes);
    ORB_HIP_CHECK(hipMemcpyAsync(dst, hStage_, bytes, hipMemcpyHostToDevice, stream_));
    ORB_HIP_CHECK(hipStreamSynchronize(stream_));
    return 0;
}

// Stream drain by polling: a one-thread kernel queued behind the stream's work writes a sequence
// number to pinned coherent memory and the host spins on it.  A blocking stream sync sleeps and
// wakes tens of microseconds after the copy it waits for (the gaps before k_gate and after each
// optimize() in profiles/r05d2lba_lba_timeline.txt); past 50 ms the spin hands over to it.
__global__ void k_signal(volatile int* w, int v) {
    if (threadIdx.x == 0) *w = v;
}
int BaEngine::poll_stream() {
    volatile int* w = (volatile int*)hLm_ + 8;
    const int v = ++signalSeq_;
    hipLaunchKernelGGL(k_signal, dim3(1), dim3(64), 0, stream_, w, v);
    ORB_HIP_CHECK(hipGetLastError());
    const auto w0 = std::chrono::steady_clock::now();
    for (unsigned spin = 1; *w != v; spin++) {
        if ((spin & 4095) == 0 && std::chrono::steady_clock::now() - w0 > std::chrono::milliseconds(50)) {
            ORB_HIP_CHECK(hipStreamSynchronize(stream_));
            break;
        }
        __builtin_ia32_pause();
    }
    const hipError_t q = hipStreamQuery(stream_);   // a sticky error of the drained work
    if (q != hipSuccess && q != hipErrorNotReady) {
        fprintf(stderr, "[orbgpu] HIP error %s after the stream drain\n", hipGetErrorString(q));
        return -2;
    }
    return 0;
}
int BaEngine::d2h_poll(void* dst, const void* src, size_t bytes) {
    if (!bytes) return 0;
    if (int e = stage_reserve(bytes)) return e;
    ORB_HIP_CHECK(hipMemcpyAsync(hStage_, src, bytes, hipMemcpyDeviceToHost, stream_));
    if (int e = poll_stream()) return e;
    std::memcpy(dst, hStage_, bytes);
    return 0;
}

int BaEngine::d2h_sync(void* dst, const void* src, size_t bytes) {
    if (!bytes) return 0;
    if (int e = stage_reserve(bytes)) return e;
    ORB_HIP_CHECK(hipMemcpyAsync(hStage_, src, bytes, hipMemcpyDeviceToHost, stream_));
    ORB_HIP_CHECK(hipStreamSynchronize(stream_));
    std::memcpy(dst, hStage_, bytes);
    return 0;
}

int BaEngine::init() {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return -4;
    ORB_HIP_CHECK(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
    ORB_HIP_CHECK(hipHostMalloc((void**)&hScal_, 64 * sizeof(double)));
    ORB_HIP_CHECK(hipHostMalloc((void**)&hLm_, 16 * sizeof(int), hipHostMallocCoherent));
    std::memset((void*)hLm_, 0, 16 * sizeof(int));   // [8]: poll_stream's sequence word
    for (auto& ev : lmEv_) ORB_HIP_CHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    int dev = 0;
    ORB_HIP_CHECK(hipGetDevice(&dev));
    hipDeviceProp_t prop;
    ORB_HIP_CHECK(hipGetDeviceProperties(&prop, dev));
    ldsMax_ = prop.sharedMemPerBlock > 2048 ? prop.sharedMemPerBlock - 1024 : 0;
    return 0;
}

bool BaEngine::dense_solver(int n) const {
    const size_t regShm = ldlt_reg_shm(n);
    const size_t ldsBytes = sizeof(double) * ((size_t)n + (size_t)n * n);
    return n <= kDenseMaxN && ((n < kLdltMax && regShm <= ldsMax_) || ldsBytes <= ldsMax_);
}

// Carve every device buffer of the problem out of one grow-only arena.
struct UploadLayout {   // byte offsets in the staging span (all 8-byte aligned)
    size_t oT, oX, oPt, oKf, oObs, oIs, oCam, oFx, oKid, oPid, total;
};
static UploadLayout upload_layout(size_t ne, size_t nkf, size_t npt) {
    auto al8 = [](size_t b) { return (b + 7) & ~(size_t)7; };
    UploadLayout L;
    L.oT = 0;
    L.oX = L.oT + sizeof(Se3) * nkf;
    L.oPt = L.oX + sizeof(double) * 3 * npt;
    L.oKf = L.oPt + al8(sizeof(int32_t) * ne);
    L.oObs = L.oKf + al8(sizeof(int32_t) * ne);
    L.oIs = L.oObs + al8(sizeof(float) * 3 * ne);
    L.oCam = L.oIs + al8(sizeof(float) * ne);
    L.oFx = L.oCam + al8(sizeof(float) * 5 * nkf);
    L.oKid = L.oFx + al8(nkf);
    L.oPid = L.oKid + al8(sizeof(int32_t) * nkf);
    L.total = L.oPid + al8(sizeof(int32_t) * npt);
    return L;
}
// The one-workgroup structure builder's inputs, staged and copied as one block ahead of the rest
// of the problem: per edge (keyframe << 13) | point, the points by (mnId, index), the keyframe ids
// and fixed flags.
static std::atomic<int> g_ba_runs{0};   // BaEngine::run calls in flight in this process
struct SmallInLayout {
    size_t oKp, oOrd, oKid, oFx, total;
};
static SmallInLayout small_in_layout(size_t ne, size_t nkf, size_t npt) {
    auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
    SmallInLayout S;
    S.oKp = 0;
    S.oOrd = S.oKp + al(sizeof(int32_t) * ne);
    S.oKid = S.oOrd + al(sizeof(int32_t) * npt);
    S.oFx = S.oKid + al(sizeof(int32_t) * nkf);
    S.total = S.oFx + al(nkf);
    return S;
}
int BaEngine::carve(bool commit, size_t* total) {
    const size_t ne = (size_t)std::max(ne_, 1), nkf = (size_t)std::max(nkf_, 1), npt = (size_t)std::max(npt_, 1);
    scratchN_ = 6 * nkf + 3 * npt + ne + 64;
    const size_t tmpN = scratchN_ / 64 + scratchN_ / 4096 + 128;   // chunk trees + their level-2 tail
    size_t off = 0;
    char* base = (char*)arena_;
    auto take = [&](size_t bytes) -> void* {
        void* p = commit ? (void*)(base + off) : nullptr;
        off += (bytes + 255) & ~(size_t)255;
        return p;
    };
    dT_ = (Se3*)take(sizeof(Se3) * nkf);
    dTbak_ = (Se3*)take(sizeof(Se3) * nkf);
    dX_ = (double*)take(sizeof(double) * 3 * npt);
    dXbak_ = (double*)take(sizeof(double) * 3 * npt);
    dE_ = (EdgeDev*)take(sizeof(EdgeDev) * ne);
    dLevel_ = (uint8_t*)take(ne);
    dRobust_ = (uint8_t*)take(ne);
    dErr_ = (double*)take(sizeof(double) * 3 * ne);
    // also the landing place of the problem's upload (upload_problem), unpacked before any use
    dTerms_ = (double*)take(std::max(sizeof(double) * T_N * ne, upload_layout(ne, nkf, npt).total));
    dRc_ = (double*)take(sizeof(double) * ne);
    dHpp_ = (double*)take(sizeof(double) * 21 * nkf);
    dBp_ = (double*)take(sizeof(double) * 6 * nkf);
    dHll_ = (double*)take(sizeof(double) * 9 * npt);
    dBl_ = (double*)take(sizeof(double) * 3 * npt);
    dB_ = (double*)take(sizeof(double) * (6 * nkf + 3 * npt));
    dX2_ = (double*)take(sizeof(double) * (6 * nkf + 3 * npt));
    // dense S only for the single-workgroup solvers (n = 6 nP <= kDenseMaxN); larger systems
    // live in the block-sparse tiles of sp_ (ldlt.hip)
    const size_t nd = std::min(6 * nkf, (size_t)kDenseMaxN);
    dS_ = (double*)take(sizeof(double) * nd * nd);
    dBs_ = (double*)take(sizeof(double) * 6 * nkf);
    dDinv_ = (double*)take(sizeof(double) * 9 * npt);
    dDb_ = (double*)take(sizeof(double) * 3 * npt);
    dEmat_ = (double*)take(sizeof(double) * 18 * ne);
    dCb_ = (double*)take(sizeof(double) * 6 * ne);
    dHplA_ = (double*)take(sizeof(double) * 18 * ne);
    dScal_ = (double*)take(sizeof(double) * 16);
    dCounter_ = (unsigned*)take(sizeof(unsigned) * 16);
    dLm_ = (LmDev*)take(sizeof(LmDev));
    dKfFixed_ = (uint8_t*)take(nkf);
    dKfId_ = (int32_t*)take(sizeof(int32_t) * nkf);
    dPePos_ = (int32_t*)take(sizeof(int32_t) * ne);
    dTn_ = (Se3*)take(sizeof(Se3) * nkf);
    dXn_ = (double*)take(sizeof(double) * 3 * npt);
    dPtId_ = (int32_t*)take(sizeof(int32_t) * npt);
    {   // the one-workgroup structure builder's inputs, one block (small_in_layout)
        const SmallInLayout S = small_in_layout(ne, nkf, npt);
        char* b = (char*)take(S.total);
        dKp_ = (int32_t*)(b + S.oKp);
        dPtOrd_ = (int32_t*)(b + S.oOrd);
        dSmKid_ = (int32_t*)(b + S.oKid);
        dSmFx_ = (uint8_t*)(b + S.oFx);
        dSmallIn_ = b;
    }
    dScratch_ = (double*)take(sizeof(double) * scratchN_);
    tmpA0_ = (double*)take(sizeof(double) * tmpN);
    tmpA1_ = (double*)take(sizeof(double) * tmpN);
    tmpB0_ = (double*)take(sizeof(double) * tmpN);
    tmpB1_ = (double*)take(sizeof(double) * tmpN);
    *total = off;
    return 0;
}

// The problem as the caller holds it goes up in ONE H2D copy of the pinned staging block (poses
// as Se3, points as doubles, the edges compact: 24 B per edge and 20 B per keyframe camera, the
// vertex flags and ids) and one kernel unpacks it: the EdgeDev records (104 B) expanded here, a
// quarter of the H2D bytes of host-expanded records, and the per-edge state initialised in the same
// pass -- one copy and one launch instead of six copies and four fills on the queue.  Same
// conversions as a host expansion (float -> double, the Huber deltas as (double)(float)sqrt(th)).
__global__ void __launch_bounds__(256) k_zero2(double* a, size_t na, double* b, size_t nb) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < na) a[i] = 0.0;
    if (i < nb) b[i] = 0.0;
}

struct UploadArgs {
    const char* src;
    UploadLayout L;
    int ne, nkf, npt;
    float thMono, thStereo;
    int robust;
    Se3* T;
    double* X;
    EdgeDev* E;
    uint8_t *kfFixed, *level, *robustFlag;
    int32_t *kfId, *ptId;
    double* err;
    unsigned* counter;
};
__global__ void __launch_bounds__(256) k_unpack_upload(UploadArgs a) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const UploadLayout& L = a.L;
    if (i < a.ne) {
        const float* obs = (const float*)(a.src + L.oObs);
        EdgeDev e;
        e.pt = ((const int32_t*)(a.src + L.oPt))[i];
        e.kf = ((const int32_t*)(a.src + L.oKf))[i];
        const float o0 = obs[3 * i], o1 = obs[3 * i + 1], o2 = obs[3 * i + 2];
        e.stereo = !(o2 < 0);
        e.pad = 0;
        e.obs[0] = (double)o0;
        e.obs[1] = (double)o1;
        e.obs[2] = (double)o2;
        e.info = (double)((const float*)(a.src + L.oIs))[i];
        const float* c = (const float*)(a.src + L.oCam) + 5 * e.kf;
        e.fx = c[0];
        e.fy = c[1];
        e.cx = c[2];
        e.cy = c[3];
        e.bf = c[4];
        e.delta = (double)(e.stereo ? a.thStereo : a.thMono);
        e.dsqr = e.delta * e.delta;
        a.E[i] = e;
        a.level[i] = 0;
        a.robustFlag[i] = (uint8_t)a.robust;
        for (int k = 0; k < 3; k++) a.err[3 * i + k] = 0.0;
    }
    if (i < 8 * a.nkf) ((double*)a.T)[i] = ((const double*)(a.src + L.oT))[i];
    if (i < 3 * a.npt) a.X[i] = ((const double*)(a.src + L.oX))[i];
    if (i < a.nkf) {
        a.kfFixed[i] = ((const uint8_t*)(a.src + L.oFx))[i];
        a.kfId[i] = ((const int32_t*)(a.src + L.oKid))[i];
    }
    if (i < a.npt) a.ptId[i] = ((const int32_t*)(a.src + L.oPid))[i];
    if (i < 16) a.counter[i] = 0;
}

int BaEngine::upload_problem(const ba_problem* P) {
    nkf_ = P->n_kf;
    npt_ = P->n_pt;
    ne_ = P->n_edge;
    size_t need = 0;
    carve(false, &need);
    if (need > arenaCap_) {
        if (arena_) (void)hipFree(arena_);
        arena_ = nullptr;
        arenaCap_ = 0;
        ORB_HIP_CHECK(hipMalloc(&arena_, need + need / 4));
        arenaCap_ = need + need / 4;
    }
    carve(true, &need);

    kfId_.assign(P->kf_id, P->kf_id + nkf_);
    ptId_.assign(P->pt_id, P->pt_id + npt_);
    // the caller's edge arrays, read in place by the host structure builder during this call
    // (a global BA's 1.5 M edges are not copied)
    ePt_ = P->edge_pt;
    eKf_ = P->edge_kf;
    kfLocal_.assign(P->kf_local, P->kf_local + nkf_);
    kfFixed_.resize(nkf_);
    for (int k = 0; k < nkf_; k++)  // BundleAdjustment: every keyframe is a vertex, fixed iff mnId == 0 (Optimizer.cc:79)
        kfFixed_[k] = ((!mode_.global && !P->kf_local[k]) || P->kf_id[k] == 0) ? 1 : 0;
    if (mode_.global) kfLocal_.assign(nkf_, 1);
    ptHasEdge_.assign(npt_, 0);
    kfHasEdge_.assign(nkf_, 0);
    // poses, points, compact edges and vertex data written straight into the pinned staging block
    // (no intermediate host copy): one H2D copy, unpacked by k_unpack_upload
    const UploadLayout UL = upload_layout(ne_, nkf_, npt_);
    // the one-workgroup structure builder reads compact edge keys and the points' id order: staged
    // behind the problem and copied first (build_structure queues the problem's copy behind the
    // level-0 structure kernel)
    // (only while no other BA call runs in this process: with concurrent calls the host lists of
    // one overlap the others' GPU work -- 16 streams: 25.0-26.2 k vs 26.9-27.8 k iter/s with the
    // one-workgroup kernels, profiles/r06st_lba_streams_ab.txt)
    smallUp_ = small_struct() && g_ba_runs.load(std::memory_order_relaxed) <= 1;
    const SmallInLayout SL = small_in_layout(ne_, nkf_, npt_);
    const size_t oSm = (UL.total + 255) & ~(size_t)255;
    if (int e = stage_reserve((smallUp_ ? oSm + SL.total : UL.total) + 64)) return e;
    char* st = (char*)hStage_;
    int32_t* kpS = smallUp_ ? reinterpret_cast<int32_t*>(st + oSm + SL.oKp) : nullptr;
    Se3* Ts = reinterpret_cast<Se3*>(st + UL.oT);
    double* Xs = reinterpret_cast<double*>(st + UL.oX);
    std::memcpy(st + UL.oFx, kfFixed_.data(), nkf_);
    std::memcpy(st + UL.oKid, P->kf_id, sizeof(int32_t) * nkf_);
    std::memcpy(st + UL.oPid, P->pt_id, sizeof(int32_t) * npt_);
    std::memcpy(st + UL.oCam, P->kf_cam, sizeof(float) * 5 * nkf_);
    for (int k = 0; k < nkf_; k++) host_se3_from_Tcw(P->kf_Tcw + 16 * k, Ts[k]);
    host_parallel(npt_, [&](int a, int b) {
        for (size_t q = 3 * (size_t)a; q < 3 * (size_t)b; q++) Xs[q] = (double)P->pt_pos[q];
    });
    uint8_t* hasEdge = ptHasEdge_.data();
    uint8_t* kfEdge = kfHasEdge_.data();
    host_parallel(ne_, [&](int a, int b) {
        // (ranges share points and keyframes: the flag bytes are stored atomically, all with the
        // same value)
        for (int i = a; i < b; i++) {
            __atomic_store_n(&hasEdge[P->edge_pt[i]], (uint8_t)1, __ATOMIC_RELAXED);
            // (a few thousand keyframe flags shared by every thread: stored only while unset, so
            // the lines stay shared instead of bouncing between the cores)
            uint8_t* f = &kfEdge[P->edge_kf[i]];
            if (!__atomic_load_n(f, __ATOMIC_RELAXED)) __atomic_store_n(f, (uint8_t)1, __ATOMIC_RELAXED);
        }
        if (kpS)
            for (int i = a; i < b; i++) kpS[i] = (P->edge_kf[i] << 13) | P->edge_pt[i];
        std::memcpy(st + UL.oPt + sizeof(int32_t) * a, P->edge_pt + a, sizeof(int32_t) * (b - a));
        std::memcpy(st + UL.oKf + sizeof(int32_t) * a, P->edge_kf + a, sizeof(int32_t) * (b - a));
        std::memcpy(st + UL.oObs + sizeof(float) * 3 * (size_t)a, P->edge_obs + 3 * (size_t)a, sizeof(float) * 3 * (b - a));
        std::memcpy(st + UL.oIs + sizeof(float) * a, P->edge_inv_sigma2 + a, sizeof(float) * (b - a));
    });
    level_.assign(ne_, 0);
    hipStream_t s = stream_;
    if (smallUp_) {
        std::vector<int32_t> ord;
        ba_order_by_id(npt_, P->pt_id, &ord);
        std::memcpy(st + oSm + SL.oOrd, ord.data(), sizeof(int32_t) * npt_);
        std::memcpy(st + oSm + SL.oKid, P->kf_id, sizeof(int32_t) * nkf_);
        std::memcpy(st + oSm + SL.oFx, kfFixed_.data(), nkf_);
        ORB_HIP_CHECK(hipMemcpyAsync(dSmallIn_, st + oSm, SL.total, hipMemcpyHostToDevice, s));
    }
    char* dst = (char*)dTerms_;   // free until the first linearisation
    UploadArgs ua;
    ua.src = dst;
    ua.L = UL;
    ua.ne = ne_;
    ua.nkf = nkf_;
    ua.npt = npt_;
    // Huber deltas: LocalBundleAdjustment sqrt(5.991) (Optimizer.cc:585), BundleAdjustment sqrt(5.99) (:87)
    ua.thMono = (float)std::sqrt(mode_.global ? 5.99 : 5.991);
    ua.thStereo = (float)std::sqrt(7.815);
    ua.robust = (mode_.global && !mode_.robust) ? 0 : 1;
    ua.T = dT_;
    ua.X = dX_;
    ua.E = dE_;
    ua.kfFixed = dKfFixed_;
    ua.level = dLevel_;
    ua.robustFlag = dRobust_;
    ua.kfId = dKfId_;
    ua.ptId = dPtId_;
    ua.err = dErr_;
    ua.counter = dCounter_;
    static_assert(std::is_trivially_copyable<UploadArgs>::value, "deferred upload");
    deferArgs_.resize(sizeof(UploadArgs));
    std::memcpy(deferArgs_.data(), &ua, sizeof(UploadArgs));
    deferBytes_ = UL.total;
    deferredUpload_ = true;
    // no wait here: the host builds the structure while the copies run; the next user of the
    // staging block (stage_reserve) waits for them.  With the one-workgroup builder the problem's
    // copy and unpack are queued behind the level-0 structure kernel (build_structure)
    if (!smallUp_) return issue_upload();
    return 0;
}
int BaEngine::issue_upload() {
    if (!deferredUpload_) return 0;
    deferredUpload_ = false;
    UploadArgs ua;
    std::memcpy(&ua, deferArgs_.data(), sizeof(UploadArgs));
    ORB_HIP_CHECK(hipMemcpyAsync((void*)ua.src, hStage_, deferBytes_, hipMemcpyHostToDevice, stream_));
    const long long nthr = std::max<long long>({(long long)ne_, 8LL * nkf_, 3LL * npt_, 16LL});
    hipLaunchKernelGGL(k_unpack_upload, dim3((unsigned)((nthr + 255) / 256)), dim3(256), 0, stream_, ua);
    ORB_HIP_CHECK(hipGetLastError());
    uploadPending_ = true;
    return 0;
}

// Who builds the structure lists: the device for large problems (a global BA's millions of
// edges), the host restatement (ba_struct.cpp) below kStructGpuMinEdges, where the device
// builder's ~20 small launches cost more than the host's counting sorts (local BA, config 4:
// 1.00 vs 0.66 ms per call, gpurun_out r04d ba_timing).  ORBGPU_STRUCT_HOST=1 / 0 forces the
// host / device builder (A/B runs; both produce the same lists, tests/test_gpu_ba_struct.py).
// ORBGPU_BA_DIST=0 keeps the replicated factorisation on every rank (A/B runs)
static bool dist_enabled() {
    static const bool v = [] {
        const char* e = std::getenv("ORBGPU_BA_DIST");
        return !(e && e[0] == '0');
    }();
    return v;
}

constexpr int kStructGpuMinEdges = 100000;
static std::atomic<int> g_struct_gpu_min{kStructGpuMinEdges};   // orbgpu_unit_set_struct_gpu_min_edges
// The two builders issue different collectives (the device one all-reduces nkf and then 2
// counts, the host one nkf + 2 at once), so a sharded run must pick the same builder on every
// rank: the choice may not depend on the rank's own edge count, and sharded runs always build
// on the device.  ORBGPU_STRUCT_HOST is process-wide, hence rank-independent.
static bool struct_host(int ne, bool sharded) {
    static const int v = [] {
        const char* e = std::getenv("ORBGPU_STRUCT_HOST");
        return e ? (e[0] == '1' ? 1 : 0) : -1;
    }();
    return v < 0 ? (!sharded && ne < g_struct_gpu_min.load()) : v == 1;
}
// Local-BA sizes build their lists in one workgroup on the device (GpuStructBuilder::build_small:
// one launch and one polled count readback per level against ~0.2 ms of host counting sorts per
// level, tools/r06_lba_ab.sh).  ORBGPU_STRUCT_SMALL=0 keeps the previous choice (A/B runs);
// ORBGPU_STRUCT_HOST=1 still forces the host builder.
static bool small_struct_enabled() {
    static const bool v = [] {
        const char* e = std::getenv("ORBGPU_STRUCT_SMALL");
        const char* h = std::getenv("ORBGPU_STRUCT_HOST");
        return !(e && e[0] == '0') && !(h && h[0] == '1');
    }();
    return v;
}
bool BaEngine::small_struct() const {
    if (comm_ || !small_struct_enabled()) return false;
    int nFree = 0;
    for (int k = 0; k < nkf_; k++) nFree += kfFixed_[k] ? 0 : 1;
    return GpuStructBuilder::small_fits(nkf_, npt_, ne_, nFree);
}
bool BaEngine::host_lists() const {   // (smallUp_: this call's choice, made at upload)
    return !smallUp_ && struct_host(ne_, comm_ && comm_->size() > 1);
}
int debug_set_struct_gpu_min_edges(int v) {
    if (v < 0) return -1;
    g_struct_gpu_min.store(v);
    return 0;
}

// pose-list positions of a device-built structure: pePos[peList[j]] = j (pePos preset to -1), then
// the Schur pair lists rewritten from edges to positions
__global__ void __launch_bounds__(256) k_pe_pos(const int32_t* peList, int nPe, int32_t* pePos) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j < nPe) pePos[peList[j]] = j;
}
__global__ void __launch_bounds__(256) k_pair_pos(int32_t* pairA, int32_t* pairB, int nPair, const int32_t* pePos) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= nPair) return;
    pairA[t] = pePos[pairA[t]];
    pairB[t] = pePos[pairB[t]];
}

// ORBGPU_ND_ASYNC=0 builds the block-sparse structure before the first LM launch (A/B)
static bool nd_async() {
    static const bool v = [] {
        const char* e = getenv("ORBGPU_ND_ASYNC");
        return !(e && e[0] == '0');
    }();
    return v;
}

int BaEngine::join_sp_build() {
    if (!spBuild_.valid()) return 0;
    return spBuild_.get();
}

// initializeOptimization(level) + buildIndexMapping + BlockSolver::buildStructure
// The pose graph of the Schur pattern's off-diagonal blocks (keys i1 * nP + i2, i1 < i2; any order,
// duplicates allowed) as sorted adjacency lists: as[i] .. as[i + 1] of adj
static void pose_graph_csr(int nP, std::vector<int64_t>& all, std::vector<int>* asOut, std::vector<int>* adjOut) {
    if (!std::is_sorted(all.begin(), all.end())) std::sort(all.begin(), all.end());   // (the device list is)
    all.erase(std::unique(all.begin(), all.end()), all.end());
    std::vector<int> deg(nP + 1, 0);
    std::vector<int>& as = *asOut;
    std::vector<int>& adj = *adjOut;
    as.assign(nP + 1, 0);
    adj.assign(2 * all.size(), 0);
    for (int64_t q : all) {
        deg[q / nP]++;
        deg[q % nP]++;
    }
    for (int i = 0; i < nP; i++) as[i + 1] = as[i] + deg[i];
    // keys (i1, i2) ascending, i1 < i2: row i gets its smaller neighbours (from the keys (i1, i),
    // i1 ascending) before its larger ones (keys (i, i2), i2 ascending), so every list comes out
    // sorted without a per-row sort
    std::vector<int> fillp(as.begin(), as.end() - 1);
    bool upper = true;
    for (int64_t q : all) {
        adj[fillp[q % nP]++] = (int)(q / nP);
        upper = upper && q / nP < q % nP;
    }
    for (int64_t q : all) adj[fillp[q / nP]++] = (int)(q % nP);
    if (!upper)   // (keys below the diagonal: not the order above)
        for (int i = 0; i < nP; i++) std::sort(adj.begin() + as[i], adj.begin() + as[i + 1]);
}

// ORBGPU_EARLY_GRAPH=0 derives the pose graph from the device lists only (A/B)
static bool early_graph_enabled() {
    static const bool v = [] {
        const char* e = std::getenv("ORBGPU_EARLY_GRAPH");
        return !(e && e[0] == '0');
    }();
    return v;
}
static std::atomic<int> g_posegraph_check{0};   // orbgpu_unit_set_posegraph_check
int debug_set_posegraph_check(int on) {
    g_posegraph_check.store(on ? 1 : 0);
    return 0;
}
constexpr int kEarlyGraphMaxPoses = 4096;   // a bit matrix of nP^2 bits per host thread

// The pose graph of an unsharded global BA's first structure, from the caller's edges on the host
// (buildIndexMapping's free poses with an edge, ascending id; two poses adjacent when they share
// a map point: every pair of a point's free-pose edges), so that the nested dissection and the
// symbolic factorisation run on a helper thread WHILE the device builds the lists, instead of
// after them.  The same off-diagonal block set as the device's Schur pattern (k_gs_terms): the
// keys come out ascending from a bit matrix.  Level 0 of a global BA: every edge is active.
// Needs the points' edges in runs (validated, edgesGrouped).  build_structure adopts it when the
// device's pose count agrees and otherwise joins and discards it.
int BaEngine::start_early_pose_graph() {
    spEarlyNP_ = -1;
    std::vector<int> order;
    order.reserve(nkf_);
    for (int k = 0; k < nkf_; k++)
        if (!kfFixed_[k] && kfHasEdge_[k]) order.push_back(k);
    std::sort(order.begin(), order.end(), [&](int a, int b) { return kfId_[a] < kfId_[b]; });
    const int nP = (int)order.size();
    if (nP < kTiledMinPoses || nP > kEarlyGraphMaxPoses) return 0;
    std::vector<int32_t> poseOf(nkf_, -1);
    for (int i = 0; i < nP; i++) poseOf[order[i]] = i;
    int dev = 0;
    ORB_HIP_CHECK(hipGetDevice(&dev));
    spEarlyNP_ = nP;
    spEarlyKeys_.clear();
    const bool keep = g_posegraph_check.load() != 0;
    const int32_t* ep = ePt_;
    const int32_t* ek = eKf_;
    const int ne = ne_;
    spEarly_ = std::async(std::launch::async, [this, dev, nP, ne, ep, ek, keep, poseOf = std::move(poseOf)]() {
        if (hipSetDevice(dev) != hipSuccess) return -2;   // the current device is per thread
        const size_t nw = ((size_t)nP * nP + 63) / 64;
        const int hw = (int)std::thread::hardware_concurrency();
        const int T = ne >= (1 << 18) ? std::max(1, std::min(16, hw)) : 1;
        std::vector<std::vector<uint64_t>> bits(T);
        auto run_start = [&](int i) {   // first run start at or after i
            while (i > 0 && i < ne && ep[i] == ep[i - 1]) i++;
            return i;
        };
        auto mark = [&](int t) {   // ranges of whole runs, one bit matrix per thread
            std::vector<uint64_t>& B = bits[t];
            B.assign(nw, 0);
            const int chunk = (ne + T - 1) / T;
            const int i0 = run_start(std::min(ne, t * chunk)), i1 = run_start(std::min(ne, (t + 1) * chunk));
            int ps[64];
            for (int i = i0; i < i1;) {
                int j = i, m = 0;
                std::vector<int> big;
                for (; j < i1 && ep[j] == ep[i]; j++) {
                    const int p = poseOf[ek[j]];
                    if (p < 0) continue;
                    if (m < 64) ps[m++] = p;
                    else big.push_back(p);
                }
                if (!big.empty()) {   // (a point with more than 64 free-pose edges)
                    big.insert(big.begin(), ps, ps + m);
                    for (size_t u = 0; u < big.size(); u++)
                        for (size_t v = u + 1; v < big.size(); v++) {
                            const size_t a = std::min(big[u], big[v]), b = std::max(big[u], big[v]);
                            const size_t q = a * nP + b;
                            B[q >> 6] |= 1ull << (q & 63);
                        }
                } else {
                    for (int u = 0; u < m; u++)
                        for (int v = u + 1; v < m; v++) {
                            const size_t a = std::min(ps[u], ps[v]), b = std::max(ps[u], ps[v]);
                            const size_t q = a * nP + b;
                            B[q >> 6] |= 1ull << (q & 63);
                        }
                }
                i = j;
            }
        };
        {
            std::vector<std::thread> th;
            for (int t = 1; t < T; t++) th.emplace_back(mark, t);
            mark(0);
            for (auto& x : th) x.join();
        }
        if (T > 1) {   // OR-merge into thread 0's matrix, word ranges split over the threads
            const size_t wc = (nw + T - 1) / T;
            auto merge = [&](int t) {
                const size_t w0 = std::min(nw, t * wc), w1 = std::min(nw, (t + 1) * wc);
                for (int r = 1; r < T; r++)
                    for (size_t w = w0; w < w1; w++) bits[0][w] |= bits[r][w];
            };
            std::vector<std::thread> th;
            for (int t = 1; t < T; t++) th.emplace_back(merge, t);
            merge(0);
            for (auto& x : th) x.join();
        }
        std::vector<int64_t> keys;   // ascending: the bit index is the key i1 * nP + i2
        for (size_t w = 0; w < nw; w++)
            for (uint64_t v = bits[0][w]; v; v &= v - 1) keys.push_back((int64_t)(w * 64 + __builtin_ctzll(v)));
        if (keep) spEarlyKeys_ = keys;
        std::vector<int> as, adj;
        pose_graph_csr(nP, keys, &as, &adj);
        return sp_.build(6 * nP, 6, as, adj, true, stream_);
    });
    return 0;
}

int BaEngine::build_structure(int level) {
    if (int e = join_sp_build()) return e;   // (a previous structure's helper, if any)
    if (spEarly_.valid()) (void)spEarly_.get();
    spEarlyNP_ = -1;
    // the unsharded global BA's first structure: pose graph, nested dissection and symbolic
    // factorisation from the host edges, beside the device lists below
    if (!comm_ && mode_.global && level == 0 && edgesGrouped && ePt_ && eKf_ && nd_async() && early_graph_enabled() &&
        !host_lists())
        if (int e = start_early_pose_graph()) return e;
    using sclk = std::chrono::steady_clock;
    static const bool say = getenv("ORBGPU_BA_TIMES") != nullptr;
    auto ts0 = sclk::now();
    auto lap = [&](const char* what) {   // ORBGPU_BA_TIMES: the structure build's phases
        if (!say) return;
        const auto t = sclk::now();
        fprintf(stderr, "[ba]   structure %s %.0f us\n", what, std::chrono::duration<double, std::micro>(t - ts0).count());
        ts0 = t;
    };
    int nE = 0, nP = 0, nL = 0, nBlk = 0;
    distOk_ = false;
    std::vector<int64_t> offKeys;    // off-diagonal Schur blocks i1 * nP + i2, ascending (tiled path)
    std::vector<int32_t> blkIJ;      // blkI ++ blkJ (dense sharded path)
    if (!host_lists()) {
        // the lists built on the device from the edges already in HBM (ba_struct_gpu.hip): in one
        // workgroup at local-BA sizes (with the pose-list positions), else by the multi-launch builder
        GpuStructInfo info{};
        int r = 1;
        if (smallUp_) {
            // the first build of the call reads no levels (every edge at level 0) and queues the
            // problem's copy and unpack behind its kernel
            const bool first = deferredUpload_;
            r = gs_.build_small(level, nkf_, npt_, ne_, dKp_, dPtOrd_, first ? nullptr : dLevel_, dSmFx_, dSmKid_, dPePos_,
                                stream_, &st_, &info, [this] { return issue_upload(); });
        }
        if (int e = issue_upload()) return e;   // (not issued yet: the multi-launch builder reads the records)
        if (r == 1)
            r = gs_.build(level, nkf_, npt_, ne_, dE_, dLevel_, dKfFixed_, dKfId_, dPtId_, comm_, stream_, &st_, &info,
                          comm_ ? &blkIJ : nullptr);
        if (r == -1) return -1;
        if (r) return r;
        lap(info.posDone ? "lists (device, one workgroup)" : "lists (device)");
        nE = info.nE;
        nP = info.nP;
        nL = info.nL;
        nBlk = info.nBlk;
        nEglob_ = info.nEglob;
        nLglob_ = info.nLglob;
        if (nE && !info.posDone) {
            ORB_HIP_CHECK(hipMemsetAsync(dPePos_, 0xff, sizeof(int32_t) * nE, stream_));
            if (info.nPe)
                hipLaunchKernelGGL(k_pe_pos, dim3((info.nPe + 255) / 256), dim3(256), 0, stream_, st_.peList, info.nPe, dPePos_);
            if (info.nPair)
                hipLaunchKernelGGL(k_pair_pos, dim3((info.nPair + 255) / 256), dim3(256), 0, stream_,
                                   const_cast<int32_t*>(st_.pairA), const_cast<int32_t*>(st_.pairB), info.nPair, dPePos_);
            ORB_HIP_CHECK(hipGetLastError());
        }
        st_.pePos = dPePos_;
        st_.nPe = info.nPe;
        if (info.maxPe > 64 * kChunks || info.maxLe > 64 * 64 || info.maxBlk > 64 * kChunks) return -3;
        blkChunks_ = (info.maxBlk + 63) / 64;
        if (nE > kCsumLv * 64 * 64 || 6LL * nP + 3LL * nL > (long long)scratchN_) return -3;
        if (spEarly_.valid() && (nP != spEarlyNP_ || g_posegraph_check.load())) {
            // the device's pose set differs (not expected: then the lists' graph is used), or the
            // early keys are checked against the device's
            const int e = spEarly_.get();
            const int np = spEarlyNP_;
            spEarlyNP_ = -1;
            if (e) return e;
            if (np == nP) {
                if (int e2 = gs_.offkeys(&offKeys, stream_)) return e2;
                if (offKeys != spEarlyKeys_) {
                    fprintf(stderr, "[ba] early pose graph differs from the device's (%zu vs %zu keys)\n",
                            spEarlyKeys_.size(), offKeys.size());
                    return -2;
                }
                spEarlyNP_ = np;   // checked: sp_ holds the structure already
                spBuild_ = std::async(std::launch::deferred, [] { return 0; });
            }
        }
        if (spEarly_.valid()) {   // adopted: joined before the first Schur assembly (join_sp_build)
            spBuild_ = std::move(spEarly_);
        } else if (spEarlyNP_ == nP) {
            // checked against the device's keys above: sp_ holds the structure
        } else if (nP >= kTiledMinPoses && !comm_) {
            if (int e = gs_.offkeys(&offKeys, stream_)) return e;
        } else if (nP >= kTiledMinPoses) {
            for (int b = 0; b < nBlk; b++)
                if (blkIJ[b] != blkIJ[nBlk + b]) offKeys.push_back((int64_t)blkIJ[b] * nP + blkIJ[nBlk + b]);
        }
    } else {
        // the second pass after the outlier gating: the first pass's lists filtered (its edges are
        // a superset) instead of built again; ORBGPU_STRUCT_CHECK=1 also builds them afresh and
        // compares every list
        const bool refine = refineNext_ && !comm_ && hsValid_;
        refineNext_ = false;
        if (refine) {
            if (ba_refine_lists(hs_, level_.data(), level, &hs2_)) return -1;
            static const bool check = getenv("ORBGPU_STRUCT_CHECK") != nullptr;
            if (check) {
                BaHostStruct F;
                std::vector<uint8_t> ka, pa;
                ba_active_set(level, nkf_, npt_, ne_, eKf_, ePt_, level_.data(), &F.aE, &ka, &pa);
                if (ba_build_lists(nkf_, npt_, eKf_, ePt_, kfFixed_.data(), kfId_.data(), ptId_.data(), ka, pa, &F))
                    return -1;
                const std::vector<int32_t>* x[] = {&F.aE, &F.ePose, &F.eLand, &F.poseKf, &F.landPt, &F.peStart,
                                                   &F.peList, &F.leStart, &F.leList, &F.lpStart, &F.lpList, &F.blkI,
                                                   &F.blkJ, &F.blkStart, &F.pairA, &F.pairB};
                const std::vector<int32_t>* y[] = {&hs2_.aE, &hs2_.ePose, &hs2_.eLand, &hs2_.poseKf, &hs2_.landPt,
                                                   &hs2_.peStart, &hs2_.peList, &hs2_.leStart, &hs2_.leList,
                                                   &hs2_.lpStart, &hs2_.lpList, &hs2_.blkI, &hs2_.blkJ,
                                                   &hs2_.blkStart, &hs2_.pairA, &hs2_.pairB};
                for (int k = 0; k < 16; k++)
                    if (*x[k] != *y[k]) {
                        fprintf(stderr, "[ba] refined structure list %d differs from a fresh build\n", k);
                        return -2;
                    }
            }
            std::swap(hs_, hs2_);
        }
        BaHostStruct& H = hs_;
        std::vector<uint8_t> kfAct, ptAct;
        if (!eKf_ || !ePt_) return -1;   // only inside run(): the caller's edge arrays
        if (!refine) ba_active_set(level, nkf_, npt_, ne_, eKf_, ePt_, level_.data(), &H.aE, &kfAct, &ptAct);
        if (comm_) {
            // shards agree on the pose set: a keyframe is active if any shard has an active edge
            // on it (its pose index must be the same everywhere); also the global edge/landmark counts
            int nLloc = 0;
            for (int p = 0; p < npt_; p++) nLloc += ptAct[p];
            std::vector<double> red(nkf_ + 2);
            for (int k = 0; k < nkf_; k++) red[k] = kfAct[k];
            red[nkf_] = (double)H.aE.size();
            red[nkf_ + 1] = (double)nLloc;
            if (h2d_sync(dScratch_, red.data(), sizeof(double) * red.size())) return -2;
            if (int e = comm_->allreduce(dScratch_, red.size(), RedOp::Sum, stream_)) return e;
            if (d2h_sync(red.data(), dScratch_, sizeof(double) * red.size())) return -2;
            ORB_HIP_CHECK(hipStreamSynchronize(stream_));
            for (int k = 0; k < nkf_; k++) kfAct[k] = red[k] > 0 ? 1 : 0;
            nEglob_ = (int)red[nkf_];
            nLglob_ = (int)red[nkf_ + 1];
        }
        lap("active set");
        if (!refine &&
            ba_build_lists(nkf_, npt_, eKf_, ePt_, kfFixed_.data(), kfId_.data(), ptId_.data(), kfAct, ptAct, &H,
                           !edgesValidated))
            return -1;
        hsValid_ = true;
        lap(refine ? "lists (refined)" : "lists");
        nE = (int)H.aE.size();
        nP = (int)H.poseKf.size();
        nL = (int)H.landPt.size();
        {   // pose-list positions; the Schur pairs rewritten from edges to positions
            const int nPe = H.peStart[nP];
            hPePos_.assign(std::max(nE, 1), -1);
            for (int j = 0; j < nPe; j++) hPePos_[H.peList[j]] = j;
            const int nPair = H.blkStart[H.blkI.size()];
            for (int t = 0; t < nPair; t++) {
                H.pairA[t] = hPePos_[H.pairA[t]];
                H.pairB[t] = hPePos_[H.pairB[t]];
            }
        }
        if (!comm_) {
            nEglob_ = nE;
            nLglob_ = nL;
        }
        const std::vector<int32_t>&aE = H.aE, &ePose = H.ePose, &eLand = H.eLand, &poseKf = H.poseKf, &landPt = H.landPt,
              &peStart = H.peStart, &peList = H.peList, &leStart = H.leStart, &leList = H.leList, &lpStart = H.lpStart,
              &lpList = H.lpList, &blkI = H.blkI, &blkJ = H.blkJ, &blkStart = H.blkStart, &pairA = H.pairA,
              &pairB = H.pairB;
        nBlk = (int)blkI.size();
        for (int i = 0; i < nP; i++)
            if (peStart[i + 1] - peStart[i] > 64 * kChunks) return -3;
        for (int l = 0; l < nL; l++)
            if (leStart[l + 1] - leStart[l] > 64 * 64) return -3;
        if (nE > kCsumLv * 64 * 64 || 6LL * nP + 3LL * nL > (long long)scratchN_) return -3;
        int maxBlk = 0;
        for (int b = 0; b < nBlk; b++) maxBlk = std::max(maxBlk, blkStart[b + 1] - blkStart[b]);
        if (maxBlk > 64 * kChunks) return -3;
        blkChunks_ = (maxBlk + 63) / 64;
        // pack and upload
        std::vector<const std::vector<int32_t>*> parts = {&aE,      &ePose,   &eLand,  &poseKf, &landPt, &peStart,
                                                          &peList,  &leStart, &leList, &lpStart, &lpList, &blkI,
                                                          &blkJ,    &blkStart, &pairA, &pairB, &hPePos_};
        size_t tot = 0;
        for (auto* p : parts) tot += (p->size() + 63) & ~(size_t)63;
        if (tot * 4 > dStructCap_) {
            if (dStruct_) (void)hipFree(dStruct_);
            ORB_HIP_CHECK(hipMalloc(&dStruct_, tot * 4 * 2));
            dStructCap_ = tot * 4 * 2;
        }
        if (int e = stage2_reserve(tot * 4)) return e;   // copied below, not waited for
        // the lists packed straight into the pinned staging block (64-entry aligned sections), the
        // copy split over host threads in 64-entry groups on large systems
        int32_t* hs = reinterpret_cast<int32_t*>(hStage2_);
        std::vector<size_t> off;
        size_t o = 0;
        for (auto* p : parts) {
            off.push_back(o);
            o += (p->size() + 63) & ~(size_t)63;
        }
        host_parallel((int)(tot / 64), [&](int g0, int g1) {
            const size_t a = (size_t)g0 * 64, b = (size_t)g1 * 64;
            for (size_t k = 0; k < parts.size(); k++) {
                const size_t s0 = off[k], len = parts[k]->size(), e0 = s0 + ((len + 63) & ~(size_t)63);
                const size_t x0 = std::max(a, s0), x1 = std::min(b, e0);
                if (x0 >= x1) continue;
                const size_t d1 = std::min(x1, s0 + len);   // list entries [x0, d1), zero padding [d1, x1)
                if (x0 < d1) std::memcpy(hs + x0, parts[k]->data() + (x0 - s0), sizeof(int32_t) * (d1 - x0));
                const size_t z0 = std::max(x0, s0 + len);
                if (z0 < x1) std::memset(hs + z0, 0, sizeof(int32_t) * (x1 - z0));
            }
        }, 1 << 14);
        ORB_HIP_CHECK(hipMemcpyAsync(dStruct_, hStage2_, tot * 4, hipMemcpyHostToDevice, stream_));
        stage2Pending_ = true;
        lap("pack + upload");
        // the sharded and block-sparse set-ups below stage more uploads through the same block
        if (comm_ || nP >= kTiledMinPoses) {
            if (int e = poll_stream()) return e;
        }
        const int32_t* d = dStruct_;
        st_.nE = nE; st_.nP = nP; st_.nL = nL; st_.nBlk = nBlk;
        st_.aE = d + off[0]; st_.ePose = d + off[1]; st_.eLand = d + off[2]; st_.poseKf = d + off[3];
        st_.landPt = d + off[4]; st_.peStart = d + off[5]; st_.peList = d + off[6]; st_.leStart = d + off[7];
        st_.leList = d + off[8]; st_.lpStart = d + off[9]; st_.lpList = d + off[10]; st_.blkI = d + off[11];
        st_.blkJ = d + off[12]; st_.blkStart = d + off[13]; st_.pairA = d + off[14]; st_.pairB = d + off[15];
        st_.pePos = d + off[16]; st_.nPe = peStart[nP];
        if (nP >= kTiledMinPoses)
            for (int b = 0; b < nBlk; b++)
                if (blkI[b] != blkJ[b]) offKeys.push_back((int64_t)blkI[b] * nP + blkJ[b]);
        if (comm_) {
            blkIJ.assign(blkI.begin(), blkI.end());
            blkIJ.insert(blkIJ.end(), blkJ.begin(), blkJ.end());
        }
    }
    nTiles_ = 0;
    // at least kTiledMinPoses free poses: the block-sparse nested-dissection solver (the oracle
    // switches at the same count); below, the dense single-workgroup solvers in natural order
    tiled_ = nP >= kTiledMinPoses;
    if (!tiled_ && nP > 0 && !dense_solver(6 * nP)) return -3;
    if (tiled_ && nP > 0) {
        // block-sparse system: the pose graph (poses sharing a point; union over the shards,
        // so every rank orders and factors the same structure) -> nested-dissection order,
        // symbolic factorisation; S travels as the Schur-pattern prefix of the tiles
        std::vector<int64_t> mine = std::move(offKeys);
        if (spEarlyNP_ == nP) {
            lap("pose graph + nested dissection + symbolic factorisation started early");
        } else if (!comm_ && nd_async()) {
            // the pose graph, nested dissection and symbolic factorisation (host, ~2.5 ms at 2,000
            // keyframes) run on a helper thread while this thread queues the first LM iteration's
            // linearisation and reductions, which do not touch the block structure; lm_solve joins
            // before the Schur assembly (join_sp_build)
            int dev = 0;
            ORB_HIP_CHECK(hipGetDevice(&dev));
            spBuild_ = std::async(std::launch::async, [this, nP, dev, keys = std::move(mine)]() mutable {
                if (hipSetDevice(dev) != hipSuccess) return -2;   // the current device is per thread
                std::vector<int> as, adj;
                pose_graph_csr(nP, keys, &as, &adj);
                return sp_.build(6 * nP, 6, as, adj, true, stream_);
            });
            lap("pose graph + nested dissection + symbolic factorisation started");
        } else {
            std::vector<int64_t> all;
            if (comm_) {
                if (int e = gather_blocks(mine, &all)) return e;
            } else {
                all = std::move(mine);
            }
            std::vector<int> as, adj;
            pose_graph_csr(nP, all, &as, &adj);
            lap("pose graph");
            if (int e = sp_.build(6 * nP, 6, as, adj, true, stream_)) return e;
            lap("nested dissection + symbolic factorisation");
        }
        distOk_ = false;
        if (comm_ && comm_->size() > 1 && dist_enabled() && sp_.plan(comm_->size(), comm_->rank(), stream_) == 0) {
            // the sharded factorisation needs every rank's points inside its own subtrees and the
            // separators (Optimizer_partition_points_nd); one misaligned rank keeps the replicated
            // solve on all of them
            int* dFlag = reinterpret_cast<int*>(dCounter_ + 8);
            if (int e = sp_.align_flag(st_.ePose, nE, dFlag, stream_)) return e;
            int f = 0;
            if (d2h_sync(&f, dFlag, sizeof(int))) return -2;
            hScal_[34] = f ? 1.0 : 0.0;
            if (h2d_sync(dScratch_, hScal_ + 34, sizeof(double))) return -2;
            if (int e = comm_->allreduce(dScratch_, 1, RedOp::Max, stream_)) return e;
            if (d2h_sync(hScal_ + 34, dScratch_, sizeof(double))) return -2;
            ORB_HIP_CHECK(hipStreamSynchronize(stream_));
            distOk_ = hScal_[34] == 0.0;
            lap("sharded factorisation plan");
        }
    } else if (comm_ && nP > 0) {
        // dense system: the 64x64 tiles the Schur blocks touch (union over the shards)
        const int n = 6 * nP, nt = (n + 63) / 64;
        std::vector<double> tm((size_t)nt * nt, 0.0);
        for (int b = 0; b < nBlk; b++) {
            const int i1 = blkIJ[b], i2 = blkIJ[nBlk + b];
            for (int I = (6 * i1) / 64; I <= (6 * i1 + 5) / 64; I++)
                for (int J = (6 * i2) / 64; J <= (6 * i2 + 5) / 64; J++)
                    if (I <= J) tm[(size_t)I * nt + J] = 1.0;
        }
        if (tm.size() > scratchN_) return -3;
        if (h2d_sync(dScratch_, tm.data(), sizeof(double) * tm.size())) return -2;
        if (int e = comm_->allreduce(dScratch_, tm.size(), RedOp::Max, stream_)) return e;
        if (d2h_sync(tm.data(), dScratch_, sizeof(double) * tm.size())) return -2;
        ORB_HIP_CHECK(hipStreamSynchronize(stream_));
        std::vector<int2> tl;
        for (int I = 0; I < nt; I++)
            for (int J = I; J < nt; J++)
                if (tm[(size_t)I * nt + J] != 0.0) tl.push_back(make_int2(I, J));
        nTiles_ = (int)tl.size();
        const size_t need = sizeof(int2) * tl.size() + 256 + sizeof(double) * ((size_t)nTiles_ * 4096 + n);
        if (need > packCap_) {
            if (dPack_) (void)hipFree(dPack_);
            dPack_ = nullptr;
            packCap_ = 0;
            ORB_HIP_CHECK(hipMalloc(&dPack_, need));
            packCap_ = need;
        }
        dTiles_ = (int2*)dPack_;
        dPackBuf_ = (double*)((char*)dPack_ + ((sizeof(int2) * tl.size() + 255) & ~(size_t)255));
        if (h2d_sync(dTiles_, tl.data(), sizeof(int2) * tl.size())) return -2;
        ORB_HIP_CHECK(hipStreamSynchronize(stream_));
    }
    {   // the step vector and (dense solvers) S zeroed in one launch
        const size_t nx = 6 * (size_t)nP + 3 * (size_t)nL + 1, ns = tiled_ ? 0 : 36 * (size_t)nP * nP + 1;
        const size_t nz = std::max(nx, ns);
        hipLaunchKernelGGL(k_zero2, dim3((unsigned)((nz + 255) / 256)), dim3(256), 0, stream_, dX2_, nx, dS_, ns);
    }
    // (the structure's copy reads its own staging block, whose next user waits for it; kernels
    // queued after this are stream-ordered behind every copy and memset above)
    lap("queued");
    return 0;
}

// All-gather of the ranks' off-diagonal Schur blocks (i1 * nP + i2) through the sum
// all-reduce: every rank learns the per-rank counts, writes its own entries into its segment
// of a zeroed buffer, and the sum hands every rank the concatenation in rank order.  Once per
// structure; the values are integers below 2^53, exact in doubles.
int BaEngine::gather_blocks(const std::vector<int64_t>& mine, std::vector<int64_t>* all) {
    const int R = comm_->size(), me = comm_->rank();
    std::vector<double> h(R, 0.0);
    h[me] = (double)mine.size();
    double* d = nullptr;
    ORB_HIP_CHECK(hipMalloc(&d, sizeof(double) * std::max<size_t>(R, 1)));
    int rc = 0;
    std::vector<size_t> off(R + 1, 0);
    if (!rc && h2d_sync(d, h.data(), sizeof(double) * R)) rc = -2;
    if (!rc) rc = comm_->allreduce(d, (size_t)R, RedOp::Sum, stream_);
    if (!rc && d2h_sync(h.data(), d, sizeof(double) * R)) rc = -2;
    if (!rc && hipStreamSynchronize(stream_) != hipSuccess) rc = -2;
    (void)hipFree(d);
    if (rc) return rc;
    for (int r = 0; r < R; r++) off[r + 1] = off[r] + (size_t)h[r];
    const size_t tot = off[R];
    all->assign(tot, 0);
    if (tot == 0) return 0;
    std::vector<double> buf(tot, 0.0);
    for (size_t q = 0; q < mine.size(); q++) buf[off[me] + q] = (double)mine[q];
    ORB_HIP_CHECK(hipMalloc(&d, sizeof(double) * tot));
    if (h2d_sync(d, buf.data(), sizeof(double) * tot)) rc = -2;
    if (!rc) rc = comm_->allreduce(d, tot, RedOp::Sum, stream_);
    if (!rc && d2h_sync(buf.data(), d, sizeof(double) * tot)) rc = -2;
    if (!rc && hipStreamSynchronize(stream_) != hipSuccess) rc = -2;
    (void)hipFree(d);
    if (rc) return rc;
    for (size_t q = 0; q < tot; q++) (*all)[q] = (int64_t)buf[q];
    return 0;
}

static inline int nblk(int n, int b) { return (n + b - 1) / b; }

// computeScale in one workgroup (k_scale / k_lm_trial_end) up to this many terms, above it
// k_scale_chunks + k_csum; orbgpu_unit_set_scale_small_max lowers it so tests drive the chunked
// path (and the device LM's scale == 0 branch) at oracle-sized problems
static std::atomic<int> g_scale_small_max{2048 * 64};
// The dense single-workgroup LDL^T of a pose system of n rows: the 1,024-thread panel kernel
// (k_ldlt_reg) by default; ORBGPU_LDLT_DENSE=col / row picks the column-owner kernel (k_ldlt_col,
// n <= 96) or the row-owner kernel (k_ldlt_row) for A/B runs.  Measured per local-BA call
// (config 4, tools/ba_timing.py): panel 3.91-4.00 ms, column-owner 5.05 ms (136 us per solve
// against 77), row-owner 8.63 ms (profiles/r04b_*, r04l_*).  All perform the oracle's operation
// sequence.
enum class DenseLdlt { Col, Reg, Row, Lds, T, D2 };
static DenseLdlt dense_ldlt_kind(int n, bool use_reg) {
    static const int pick = [] {
        const char* e = std::getenv("ORBGPU_LDLT_DENSE");
        if (!e) return 1;
        if (!strcmp(e, "col")) return 0;
        if (!strcmp(e, "row")) return 2;
        if (!strcmp(e, "t")) return 3;
        if (!strcmp(e, "2d")) return 4;
        return 1;
    }();
    if (pick == 4 && n <= kLdltColMax) return DenseLdlt::D2;
    if (pick == 2 && n <= kLdltRowMax) return DenseLdlt::Row;
    if (pick == 3 && n <= kLdltColMax) return DenseLdlt::T;
    if (pick == 0 && n <= kLdltColMax) return DenseLdlt::Col;
    return use_reg ? DenseLdlt::Reg : DenseLdlt::Lds;
}
static bool scale_small(int nP, int nL) { return 6 * nP + 3 * nL <= g_scale_small_max.load(); }
int debug_set_scale_small_max(int v) {
    if (v < 0 || v > 2048 * 64) return 1;
    g_scale_small_max.store(v);
    return 0;
}

// OptimizationAlgorithmLevenberg::solve (optimization_algorithm_levenberg.cpp:59-164)
// Sharded (comm_ set): the pose rows of H and the Schur complement are sums over the shards'
// points, so each shard reduces its own edges and the exchange steps are
//   after buildSystem:  all-reduce(sum) {Hpp, b_p, chi2}           -> identical pose system
//   lambda init:        all-reduce(max) {max|diag|, lambda0}
//   per trial:          all-reduce(sum) {S, b_s} (own pose terms and lambda added by rank 0),
//                       replicated LDL^T, local back-substitution,
//                       all-reduce(sum) {chi2_new, scale (rank 0 owns the pose terms), stop}
int BaEngine::lm_solve(int iteration, const volatile bool* stop, bool* terminate) {
    hipStream_t s = stream_;
    const BaStructDev& S = st_;
    const int nE = S.nE, nP = S.nP, nL = S.nL;
    const bool own = !comm_ || comm_->rank() == 0;
    LinArgs la{S, dE_, dT_, dX_, dRobust_, dErr_, dRc_, dTerms_, dHplA_, 1, tmpA0_, dCounter_, dScal_ + 0, nullptr};
    if (comm_ && !nE) ORB_HIP_CHECK(hipMemsetAsync(dScal_, 0, 2 * sizeof(double), s));
    if (nE) {
        hipLaunchKernelGGL(k_linearize, dim3(nblk(nE, 256)), dim3(256), 0, s, la);
        hipLaunchKernelGGL(k_chi2_finish, dim3(1), dim3(256), 0, s, la);
    }
    if (nP) hipLaunchKernelGGL(k_pose_reduce, dim3(nP), dim3(kSysThreads), 0, s, S, dTerms_, dHpp_, dBp_, nullptr);
    if (nL) hipLaunchKernelGGL(k_land_reduce, dim3(nblk(12 * nL, 256)), dim3(256), 0, s, S, dTerms_, dHll_, dBl_, nullptr);
    if (comm_) {
        const RedBuf rb[3] = {{dHpp_, 21 * (size_t)nP}, {dBp_, 6 * (size_t)nP}, {dScal_, 1}};
        ORB_HIP_CHECK(hipGetLastError());
        if (int e = comm_->allreduce(rb, 3, RedOp::Sum, s)) return e;
    }
    int use_dev = 0;
    if (iteration == 0) {
        hipLaunchKernelGGL(k_lambda_init, dim3(1), dim3(1024), 0, s, nP, nL, dHpp_, dHll_, dScal_, nullptr);
        if (comm_) {
            ORB_HIP_CHECK(hipGetLastError());
            if (int e = comm_->allreduce(dScal_ + 4, 2, RedOp::Max, s)) return e;
        }
        use_dev = 1;  // lambda known on the device only until the first readback
        ni_ = 2;
        nBad_ = 0;
    }
    ORB_HIP_CHECK(hipGetLastError());
    double currentChi = 0, iniChi = 0;
    bool haveChi = false;
    double rho = 0;
    int qmax = 0;
    const int n = 6 * nP;
    const size_t ldsBytes = sizeof(double) * ((size_t)n + (size_t)n * n);
    const int in_lds = ldsBytes <= ldsMax_ ? 1 : 0;
    const size_t shm = in_lds ? ldsBytes : sizeof(double) * (size_t)n;
    const size_t regShm = ldlt_reg_shm(n);
    const bool use_reg = n < kLdltMax && regShm <= ldsMax_;   // b rides in column n
    const DenseLdlt kind = dense_ldlt_kind(n, use_reg);
    // n <= 128: register-resident single-workgroup LDL^T; S fits LDS: single-workgroup in LDS;
    // larger: block-sparse tiled LDL^T in HBM (ldlt.hip, structure from build_structure)
    if (!tiled_ && n > 0 && !use_reg && !in_lds) return -1;
    SysAddr sa{dS_, n, nullptr, nullptr, 0, nullptr};
    bool joined = false;
    do {
        // setLambda + BlockSolver::solve
        if (nE) hipLaunchKernelGGL(k_point_prep, dim3(nblk(nE, 256)), dim3(256), 0, s, S, dHll_, dBl_, dHplA_,
                                   lambda_, use_dev, dScal_, dEmat_, dCb_, nullptr);
        if (!joined) {   // the block structure, built beside the first linearisation and point prep
            if (int e = join_sp_build()) return e;
            if (tiled_) sa = sp_.addr();
            joined = true;
        }
        // the in-place LDL^T overwrites S (fill-in, L), and a shard's S holds the previous
        // trial's all-reduced blocks outside its own pattern: clear S
        if (tiled_) {
            if (int e = sp_.zero(s)) return e;
        } else if (comm_ && n) {
            ORB_HIP_CHECK(hipMemsetAsync(dS_, 0, sizeof(double) * (size_t)n * n, s));
        }
        if (S.nBlk) schur_launch(S.nBlk, blkChunks_, s, S, dEmat_, dHplA_, dCb_, dHpp_, dBp_,
                                       lambda_, use_dev, dScal_, sa, dBs_, own ? 1 : 0,
                                       distOk_ ? sp_.pose_add() : (const uint8_t*)nullptr, (const int*)nullptr);
        if (comm_ && tiled_ && distOk_) {
            // sharded factorisation: each rank's partial S and b_s go straight into it (solve_dist
            // exchanges the separator tiles and rows only)
        } else if (comm_ && tiled_) {   // all-reduce the Schur-pattern tiles of S and b_s
            ORB_HIP_CHECK(hipGetLastError());
            const RedBuf rb[2] = {{sp_.tiles(), (size_t)sp_.nA() * 4096}, {dBs_, (size_t)n}};
            if (int e = comm_->allreduce(rb, 2, RedOp::Sum, s)) return e;
        } else if (comm_ && nTiles_) {   // all-reduce the union-pattern tiles of S and b_s (packed)
            hipLaunchKernelGGL(k_tile_pack, dim3(nTiles_), dim3(256), 0, s, n, dS_, dTiles_, dPackBuf_);
            double* pb = dPackBuf_ + (size_t)nTiles_ * 4096;
            ORB_HIP_CHECK(hipMemcpyAsync(pb, dBs_, sizeof(double) * n, hipMemcpyDeviceToDevice, s));
            ORB_HIP_CHECK(hipGetLastError());
            if (int e = comm_->allreduce(dPackBuf_, (size_t)nTiles_ * 4096 + n, RedOp::Sum, s)) return e;
            hipLaunchKernelGGL(k_tile_unpack, dim3(nTiles_), dim3(256), 0, s, n, dS_, dTiles_, dPackBuf_);
            ORB_HIP_CHECK(hipMemcpyAsync(dBs_, pb, sizeof(double) * n, hipMemcpyDeviceToDevice, s));
        }
        if (tiled_ && distOk_) {
            if (int e = sp_.solve_dist(dBs_, dX2_, dScal_, s, comm_)) return e;
        } else if (tiled_) {
            if (int e = sp_.solve(dBs_, dX2_, dScal_, s)) return e;
        } else if (kind == DenseLdlt::Col) {
            hipLaunchKernelGGL(k_ldlt_col, dim3(1), dim3(256), 0, s, n, dS_, dBs_, dX2_, dScal_, nullptr);
        } else if (kind == DenseLdlt::T) {
            hipLaunchKernelGGL(k_ldlt_t, dim3(1), dim3(256), 0, s, n, dS_, dBs_, dX2_, dScal_, nullptr);
        } else if (kind == DenseLdlt::D2) {
            hipLaunchKernelGGL(k_ldlt_2d, dim3(1), dim3(256), 0, s, n, dS_, dBs_, dX2_, dScal_, nullptr);
        } else if (kind == DenseLdlt::Row) {
            hipLaunchKernelGGL(k_ldlt_row, dim3(1), dim3(128), 0, s, n, dS_, dBs_, dX2_, dScal_, nullptr);
        } else if (kind == DenseLdlt::Reg) {
            hipLaunchKernelGGL(k_ldlt_reg, dim3(1), dim3(kLdltThreads), regShm, s, n, dS_, dBs_, dX2_, dScal_, nullptr);
        } else {
            hipLaunchKernelGGL(k_ldlt, dim3(1), dim3(256), shm + 16, s, n, dS_, dBs_, dX2_, dScal_, in_lds, nullptr);
        }
        // push + update
        if (nP + nL) hipLaunchKernelGGL(k_update, dim3(nblk(nP + nL, 256)), dim3(256), 0, s, S, dT_, dTbak_, dX_,
                                        dXbak_, dX2_, dHplA_, dHll_, dBl_, lambda_, use_dev, dScal_, nullptr);
        // computeActiveErrors + activeRobustChi2 ; computeScale
        la.linearize = 0;
        la.out = dScal_ + 1;
        if (nE) {
            hipLaunchKernelGGL(k_linearize, dim3(nblk(nE, 256)), dim3(256), 0, s, la);
            hipLaunchKernelGGL(k_chi2_finish, dim3(1), dim3(256), 0, s, la);
        } else if (comm_ && qmax > 0) {   // a rank without edges: its trial chi2 is 0 (the last trial's
            ORB_HIP_CHECK(hipMemsetAsync(dScal_ + 1, 0, sizeof(double), s));   // all-reduced total otherwise)
        }
        if (scale_small(nP, nL)) {
            hipLaunchKernelGGL(k_scale, dim3(1), dim3(1024), 0, s, nP, nL, dX2_, dBp_, dBl_, lambda_, use_dev, dScal_,
                               dScal_ + 2, own ? 1 : 0, nullptr);
        } else {
            const int nv = 6 * nP + 3 * nL;
            hipLaunchKernelGGL(k_scale_chunks, dim3(nblk(nv, 256)), dim3(256), 0, s, nP, nL, dX2_, dBp_, dBl_, lambda_,
                               use_dev, dScal_, tmpA0_, own ? 1 : 0, nullptr);
            CsumList L0{tmpA0_, (nv + 63) / 64, tmpA1_, tmpA0_, dScal_ + 2};
            hipLaunchKernelGGL(k_csum, dim3(1), dim3(1024), 0, s, L0, L0, nullptr);
        }
        ORB_HIP_CHECK(hipGetLastError());
        if (comm_) {
            hScal_[32] = (stop && *stop) ? 1.0 : 0.0;
            ORB_HIP_CHECK(hipMemcpyAsync(dScal_ + 6, hScal_ + 32, sizeof(double), hipMemcpyHostToDevice, s));
            const RedBuf rb[2] = {{dScal_ + 1, 2}, {dScal_ + 6, 1}};
            if (int e = comm_->allreduce(rb, 2, RedOp::Sum, s)) return e;
        }
        ORB_HIP_CHECK(hipMemcpyAsync(hScal_, dScal_, 8 * sizeof(double), hipMemcpyDeviceToHost, s));
        if (int e = poll_stream()) return e;   // (s is stream_)
        if (comm_) stopRed_ = hScal_[6] != 0.0;
        if (!haveChi) {
            currentChi = iniChi = hScal_[0];
            haveChi = true;
        }
        if (use_dev) {
            lambda_ = hScal_[5];
            use_dev = 0;
        }
        const bool ok2 = hScal_[3] != 0.0;
        double tempChi = hScal_[1];
        if (!ok2) tempChi = DBL_MAX;
        rho = currentChi - tempChi;
        double scale = hScal_[2];
        scale += 1e-3;
        rho /= scale;
        if (rho > 0 && std::isfinite(tempChi)) {
            const double a3 = 2 * rho - 1;
            double alpha = 1. - (a3 * a3) * a3;
            alpha = std::fmin(alpha, 2. / 3.);
            const double scaleFactor = std::fmax(1. / 3., alpha);
            lambda_ *= scaleFactor;
            ni_ = 2;
            currentChi = tempChi;
        } else {
            lambda_ *= ni_;
            ni_ *= 2;
            if (nP + nL) hipLaunchKernelGGL(k_pop, dim3(nblk(nP + nL, 256)), dim3(256), 0, s, S, dT_, dTbak_, dX_,
                                            dXbak_, nullptr);
        }
        qmax++;
        last_lm[1]++;
        trace_.trial_chi2.push_back(tempChi);
        trace_.trial_lambda.push_back(lambda_);
    } while (rho < 0 && qmax < 10 && !stopped(stop));
    trace_.solve_ini_chi2.push_back(iniChi);
    trace_.solve_chi2.push_back(currentChi);
    *terminate = false;
    if (qmax == 10 || rho == 0) {
        *terminate = true;
        return 0;
    }
    if ((iniChi - currentChi) * 1e3 < iniChi) nBad_++;
    else nBad_ = 0;
    if (nBad_ >= 3) *terminate = true;
    return 0;
}

// SparseOptimizer::optimize (sparse_optimizer.cpp:354-418)
int BaEngine::optimize(int iterations, const volatile bool* stop, int* its) {
    if (device_lm(iterations)) return optimize_device(iterations, stop, its);
    *its = 0;
    bool ok = true;
    for (int i = 0; i < iterations && !stopped(stop) && ok; i++) {
        bool term = false;
        if (int e = lm_solve(i, stop, &term)) return e;
        ok = !term;
        (*its)++;
    }
    return 0;
}

// The device-resident LM (k_lm_trial_end) runs unsharded problems on the single-workgroup dense
// solvers: one queue of kernels per optimize() call, no host round trip per trial.  ORBGPU_LM_HOST=1
// keeps the host-driven loop (lm_solve) for A/B runs.
static bool lm_host_forced() {
    static const bool v = [] {
        const char* e = std::getenv("ORBGPU_LM_HOST");
        return e && e[0] == '1';
    }();
    return v;
}

// ORBGPU_STRUCT_REFINE=1 filters the second local-BA pass's lists from the first pass's
// (ba_refine_lists) instead of building them afresh.  Opt-in: equal lists, but measured slower
// at config 4 (0.47-0.50 vs 0.42-0.50 ms of structure per call, gpurun_out r05l2)
static bool refine_enabled() {
    static const bool v = [] {
        const char* e = std::getenv("ORBGPU_STRUCT_REFINE");
        return e && e[0] == '1';
    }();
    return v;
}

// ORBGPU_FUSED_PREP=0 keeps k_sys_reduce + k_point_prep on every step (A/B)
static bool fused_prep() {
    static const bool v = [] {
        const char* e = std::getenv("ORBGPU_FUSED_PREP");
        return !(e && e[0] == '0');
    }();
    return v;
}

// A one-rank group has no exchange (every all-reduce is the identity), so its sharded call is the
// unsharded call and takes the same device LM.  With more ranks the trial's all-reduces sit
// between the device steps: the host loop keeps them in order.
// Sharded runs too (enqueue_lm_step_comm): the exchanges are stream-ordered calls between the
// step's kernels, so no rank reads a trial's result back.  The block-sparse (tiled) solver keeps
// the host loop: its ~100 launches per solve take no gate, so a step queued after the run ended
// would factor once more.
bool BaEngine::device_lm(int iterations) const {
    return !tiled_ && iterations > 0 && (size_t)iterations * 10 <= (size_t)kLmTrials && !lm_host_forced() &&
           dense_solver(6 * st_.nP);
}

// the kernels of one LM step: [system: linearize, reduce, lambda init] [trial ... decide, pop]
void BaEngine::enqueue_lm_step(bool first) {
    hipStream_t s = stream_;
    const BaStructDev& S = st_;
    const int nE = S.nE, nP = S.nP, nL = S.nL;
    const int* ctl = dLm_->ctl;
    LinArgs la{S, dE_, dT_, dX_, dRobust_, dErr_, dRc_, dTerms_, dHplA_, 1, tmpA0_, dCounter_, dScal_ + 0, ctl + 1};
    // two or more edges: the chi2 totals are summed by k_lm_trial_end from chunk buffers of their own
    // (a single edge's total is its r0, which the trial's linearisation overwrites)
    const bool fuse = nE >= 2 && (nE + 63) / 64 <= kChiFuseMax;
    if (fuse) la.chunks = tmpB0_;
    if (nE) {
        hipLaunchKernelGGL(k_linearize, dim3(nblk(nE, 256)), dim3(256), 0, s, la);
        if (!fuse) hipLaunchKernelGGL(k_chi2_finish, dim3(1), dim3(256), 0, s, la);
    }
    // the first step computes lambda from the reduced system (k_lambda_init) before the point prep;
    // later steps find lambda on the device and prep inside the reduction's launch
    const bool fusedPrep = !first && fused_prep();
    if (nP + nL) {
        if (fusedPrep)
            hipLaunchKernelGGL(k_sys_reduce_prep, dim3(nP + nblk(nL, kLandBlk)), dim3(kSysThreads), 0, s, S, dTerms_,
                               dHpp_, dBp_, dHll_, dBl_, dHplA_, dScal_, dEmat_, dCb_, ctl);
        else
            hipLaunchKernelGGL(k_sys_reduce, dim3(nP + nblk(12 * nL, kSysThreads)), dim3(kSysThreads), 0, s, S, dTerms_,
                               dHpp_, dBp_, dHll_, dBl_, ctl + 1);
    }
    if (first) hipLaunchKernelGGL(k_lambda_init, dim3(1), dim3(1024), 0, s, nP, nL, dHpp_, dHll_, dScal_, ctl + 2);
    const int n = 6 * nP;
    const size_t ldsBytes = sizeof(double) * ((size_t)n + (size_t)n * n);
    const int in_lds = ldsBytes <= ldsMax_ ? 1 : 0;
    const size_t shm = in_lds ? ldsBytes : sizeof(double) * (size_t)n;
    const size_t regShm = ldlt_reg_shm(n);
    const bool use_reg = n < kLdltMax && regShm <= ldsMax_;   // b rides in column n
    const SysAddr sa{dS_, n, nullptr, nullptr, 0, nullptr};
    if (nE && !(fusedPrep && nP + nL))
        hipLaunchKernelGGL(k_point_prep, dim3(nblk(nE, 256)), dim3(256), 0, s, S, dHll_, dBl_, dHplA_, 0.0, 1, dScal_,
                           dEmat_, dCb_, ctl);
    if (S.nBlk) schur_launch(S.nBlk, blkChunks_, s, S, dEmat_, dHplA_, dCb_, dHpp_, dBp_, 0.0,
                                   1, dScal_, sa, dBs_, 1, (const uint8_t*)nullptr, ctl);
    const DenseLdlt kind = dense_ldlt_kind(n, use_reg);
    if (kind == DenseLdlt::Col) hipLaunchKernelGGL(k_ldlt_col, dim3(1), dim3(256), 0, s, n, dS_, dBs_, dX2_, dScal_, ctl);
    else if (kind == DenseLdlt::T) hipLaunchKernelGGL(k_ldlt_t, dim3(1), dim3(256), 0, s, n, dS_, dBs_, dX2_, dScal_, ctl);
    else if (kind == DenseLdlt::D2) hipLaunchKernelGGL(k_ldlt_2d, dim3(1), dim3(256), 0, s, n, dS_, dBs_, dX2_, dScal_, ctl);
    else if (kind == DenseLdlt::Row) hipLaunchKernelGGL(k_ldlt_row, dim3(1), dim3(128), 0, s, n, dS_, dBs_, dX2_, dScal_, ctl);
    else if (kind == DenseLdlt::Reg) hipLaunchKernelGGL(k_ldlt_reg, dim3(1), dim3(kLdltThreads), regShm, s, n, dS_, dBs_, dX2_, dScal_, ctl);
    else hipLaunchKernelGGL(k_ldlt, dim3(1), dim3(256), shm + 16, s, n, dS_, dBs_, dX2_, dScal_, in_lds, ctl);
    la.linearize = 0;
    la.out = dScal_ + 1;
    la.run = ctl;
    if (fuse) {
        // the update inside the trial pass: edges at the trial's poses and points, the owners'
        // values to dTn_ / dXn_ (committed by k_lm_trial_end when the trial is accepted)
        la.chunks = tmpB1_;
        la.fuse = 1;
        la.edgeBlocks = nblk(nE, 256);
        la.x = dX2_;
        la.Hll = dHll_;
        la.bl = dBl_;
        la.scal = dScal_;
        la.Tn = dTn_;
        la.Xn = dXn_;
        hipLaunchKernelGGL(k_linearize_upd, dim3(la.edgeBlocks + nblk(nP + nL, 256)), dim3(256), 0, s, la);
    } else {
        if (nP + nL) hipLaunchKernelGGL(k_update, dim3(nblk(nP + nL, 256)), dim3(256), 0, s, S, dT_, dTbak_, dX_, dXbak_,
                                        dX2_, dHplA_, dHll_, dBl_, 0.0, 1, dScal_, ctl);
        if (nE) {
            hipLaunchKernelGGL(k_linearize, dim3(nblk(nE, 256)), dim3(256), 0, s, la);
            hipLaunchKernelGGL(k_chi2_finish, dim3(1), dim3(256), 0, s, la);
        }
    }
    const bool small = scale_small(nP, nL);
    if (!small) {
        const int nv = 6 * nP + 3 * nL;
        hipLaunchKernelGGL(k_scale_chunks, dim3(nblk(nv, 256)), dim3(256), 0, s, nP, nL, dX2_, dBp_, dBl_, 0.0, 1,
                           dScal_, tmpA0_, 1, ctl);
        CsumList L0{tmpA0_, (nv + 63) / 64, tmpA1_, tmpA0_, dScal_ + 2};
        hipLaunchKernelGGL(k_csum, dim3(1), dim3(1024), 0, s, L0, L0, ctl);
    }
    hipLaunchKernelGGL(k_lm_trial_end, dim3(1), dim3(kTeThreads), 0, s, dLm_, dScal_, (volatile int*)hLm_, S, dT_, dTbak_,
                       dX_, dXbak_, dX2_, dBp_, dBl_, small ? 1 : 0,
                       fuse ? ChiFuse{tmpB0_, tmpB1_, nE} : ChiFuse{nullptr, nullptr, 0}, fuse ? dTn_ : nullptr,
                       fuse ? dXn_ : nullptr, (const double*)nullptr);
}

// the system's all-reduce staging of enqueue_lm_step_comm: dir 0 [Hpp | b_p | chi2] -> stage, dir 1
// back (gated by the system flag: on a trial of the same system the exchange still runs, on
// whatever the staging holds, and nothing is copied back)
__global__ void __launch_bounds__(256) k_lm_stage(int nP, double* Hpp, double* bp, double* scal, double* stage, int dir,
                                                  const int* run) {
    BA_GATE(run);
    const int i = blockIdx.x * blockDim.x + threadIdx.x, n1 = 21 * nP, n2 = 27 * nP;
    if (i > n2) return;
    double* p = i < n1 ? Hpp + i : i < n2 ? bp + (i - n1) : scal;
    if (dir == 0) stage[i] = *p;
    else *p = stage[i];
}
// the host's stop flag (the word the host mirrors) as a double for the ranks' all-reduce
__global__ void k_lm_stop_in(const volatile int* host, double* dst) {
    if (threadIdx.x == 0) *dst = host[0] != 0 ? 1.0 : 0.0;
}
// a rank without edges: zero chi2 partial (gated like the linearisation it replaces)
__global__ void k_lm_zero_chi(double* scal, const int* run) {
    BA_GATE(run);
    if (threadIdx.x == 0) scal[0] = 0.0;
}

// One LM step of a rank of a sharded run (dense reduced system): lm_solve's kernels for one
// trial -- the system part (linearisation, reductions and their all-reduce) gated by ctl[1], the
// trial part by ctl[0] -- with the exchanges in the same places and the decision made on the
// device by k_lm_trial_end from the all-reduced scalars (chi2s, scale, stop).  The all-reduces
// cannot be gated: every rank enqueues the same steps (optimize_device), a gated step exchanges
// scratch that nothing reads afterwards.  Same kernels, arguments and exchanges as lm_solve: the
// same bits.
int BaEngine::enqueue_lm_step_comm(bool first) {
    hipStream_t s = stream_;
    const BaStructDev& S = st_;
    const int nE = S.nE, nP = S.nP, nL = S.nL;
    const int* ctl = dLm_->ctl;
    const bool own = comm_->rank() == 0;
    LinArgs la{S, dE_, dT_, dX_, dRobust_, dErr_, dRc_, dTerms_, dHplA_, 1, tmpA0_, dCounter_, dScal_ + 0, ctl + 1};
    // system (a new iteration): chi2, Hpp, b_p, then their all-reduce through the staging
    if (!nE) hipLaunchKernelGGL(k_lm_zero_chi, dim3(1), dim3(64), 0, s, dScal_, ctl + 1);
    if (nE) {
        hipLaunchKernelGGL(k_linearize, dim3(nblk(nE, 256)), dim3(256), 0, s, la);
        hipLaunchKernelGGL(k_chi2_finish, dim3(1), dim3(256), 0, s, la);
    }
    if (nP) hipLaunchKernelGGL(k_pose_reduce, dim3(nP), dim3(kSysThreads), 0, s, S, dTerms_, dHpp_, dBp_, ctl + 1);
    if (nL) hipLaunchKernelGGL(k_land_reduce, dim3(nblk(12 * nL, 256)), dim3(256), 0, s, S, dTerms_, dHll_, dBl_, ctl + 1);
    const size_t ns = 27 * (size_t)nP + 1;
    if (ns > lmStageCap_) {
        if (dLmStage_) (void)hipFree(dLmStage_);
        dLmStage_ = nullptr;
        lmStageCap_ = 0;
        ORB_HIP_CHECK(hipMalloc(&dLmStage_, sizeof(double) * ns));
        ORB_HIP_CHECK(hipMemsetAsync(dLmStage_, 0, sizeof(double) * ns, s));
        lmStageCap_ = ns;
    }
    hipLaunchKernelGGL(k_lm_stage, dim3(nblk((int)ns, 256)), dim3(256), 0, s, nP, dHpp_, dBp_, dScal_, dLmStage_, 0, ctl + 1);
    ORB_HIP_CHECK(hipGetLastError());
    if (int e = comm_->allreduce(dLmStage_, ns, RedOp::Sum, s)) return e;
    hipLaunchKernelGGL(k_lm_stage, dim3(nblk((int)ns, 256)), dim3(256), 0, s, nP, dHpp_, dBp_, dScal_, dLmStage_, 1, ctl + 1);
    if (first) {   // computeLambdaInit, the maximum over the ranks (the first step is always live)
        hipLaunchKernelGGL(k_lambda_init, dim3(1), dim3(1024), 0, s, nP, nL, dHpp_, dHll_, dScal_, ctl + 2);
        ORB_HIP_CHECK(hipGetLastError());
        if (int e = comm_->allreduce(dScal_ + 4, 2, RedOp::Max, s)) return e;
    }
    // trial
    const int n = 6 * nP;
    const size_t ldsBytes = sizeof(double) * ((size_t)n + (size_t)n * n);
    const int in_lds = ldsBytes <= ldsMax_ ? 1 : 0;
    const size_t shm = in_lds ? ldsBytes : sizeof(double) * (size_t)n;
    const size_t regShm = ldlt_reg_shm(n);
    const bool use_reg = n < kLdltMax && regShm <= ldsMax_;
    const DenseLdlt kind = dense_ldlt_kind(n, use_reg);
    const SysAddr sa{dS_, n, nullptr, nullptr, 0, nullptr};
    if (nE) hipLaunchKernelGGL(k_point_prep, dim3(nblk(nE, 256)), dim3(256), 0, s, S, dHll_, dBl_, dHplA_, 0.0, 1, dScal_,
                               dEmat_, dCb_, ctl);
    if (n) ORB_HIP_CHECK(hipMemsetAsync(dS_, 0, sizeof(double) * (size_t)n * n, s));
    if (S.nBlk) schur_launch(S.nBlk, blkChunks_, s, S, dEmat_, dHplA_, dCb_, dHpp_, dBp_, 0.0, 1, dScal_, sa, dBs_,
                             own ? 1 : 0, (const uint8_t*)nullptr, ctl);
    if (nTiles_) {   // the union-pattern tiles of S and b_s, packed
        hipLaunchKernelGGL(k_tile_pack, dim3(nTiles_), dim3(256), 0, s, n, dS_, dTiles_, dPackBuf_);
        double* pb = dPackBuf_ + (size_t)nTiles_ * 4096;
        ORB_HIP_CHECK(hipMemcpyAsync(pb, dBs_, sizeof(double) * n, hipMemcpyDeviceToDevice, s));
        ORB_HIP_CHECK(hipGetLastError());
        if (int e = comm_->allreduce(dPackBuf_, (size_t)nTiles_ * 4096 + n, RedOp::Sum, s)) return e;
        hipLaunchKernelGGL(k_tile_unpack, dim3(nTiles_), dim3(256), 0, s, n, dS_, dTiles_, dPackBuf_);
        ORB_HIP_CHECK(hipMemcpyAsync(dBs_, pb, sizeof(double) * n, hipMemcpyDeviceToDevice, s));
    }
    if (kind == DenseLdlt::Col) hipLaunchKernelGGL(k_ldlt_col, dim3(1), dim3(256), 0, s, n, dS_, dBs_, dX2_, dScal_, ctl);
    else if (kind == DenseLdlt::T) hipLaunchKernelGGL(k_ldlt_t, dim3(1), dim3(256), 0, s, n, dS_, dBs_, dX2_, dScal_, ctl);
    else if (kind == DenseLdlt::D2) hipLaunchKernelGGL(k_ldlt_2d, dim3(1), dim3(256), 0, s, n, dS_, dBs_, dX2_, dScal_, ctl);
    else if (kind == DenseLdlt::Row) hipLaunchKernelGGL(k_ldlt_row, dim3(1), dim3(128), 0, s, n, dS_, dBs_, dX2_, dScal_, ctl);
    else if (kind == DenseLdlt::Reg) hipLaunchKernelGGL(k_ldlt_reg, dim3(1), dim3(kLdltThreads), regShm, s, n, dS_, dBs_, dX2_, dScal_, ctl);
    else hipLaunchKernelGGL(k_ldlt, dim3(1), dim3(256), shm + 16, s, n, dS_, dBs_, dX2_, dScal_, in_lds, ctl);
    if (nP + nL) hipLaunchKernelGGL(k_update, dim3(nblk(nP + nL, 256)), dim3(256), 0, s, S, dT_, dTbak_, dX_, dXbak_, dX2_,
                                    dHplA_, dHll_, dBl_, 0.0, 1, dScal_, ctl);
    la.linearize = 0;
    la.out = dScal_ + 1;
    la.run = ctl;
    if (nE) {
        hipLaunchKernelGGL(k_linearize, dim3(nblk(nE, 256)), dim3(256), 0, s, la);
        hipLaunchKernelGGL(k_chi2_finish, dim3(1), dim3(256), 0, s, la);
    } else {   // (lm_solve's memset of chi2 for a rank without edges, here per trial)
        ORB_HIP_CHECK(hipMemsetAsync(dScal_ + 1, 0, sizeof(double), s));
    }
    if (scale_small(nP, nL)) {
        hipLaunchKernelGGL(k_scale, dim3(1), dim3(1024), 0, s, nP, nL, dX2_, dBp_, dBl_, 0.0, 1, dScal_, dScal_ + 2,
                           own ? 1 : 0, ctl);
    } else {
        const int nv = 6 * nP + 3 * nL;
        hipLaunchKernelGGL(k_scale_chunks, dim3(nblk(nv, 256)), dim3(256), 0, s, nP, nL, dX2_, dBp_, dBl_, 0.0, 1,
                           dScal_, tmpA0_, own ? 1 : 0, ctl);
        CsumList L0{tmpA0_, (nv + 63) / 64, tmpA1_, tmpA0_, dScal_ + 2};
        hipLaunchKernelGGL(k_csum, dim3(1), dim3(1024), 0, s, L0, L0, ctl);
    }
    hipLaunchKernelGGL(k_lm_stop_in, dim3(1), dim3(64), 0, s, (const volatile int*)hLm_, dScal_ + 6);
    ORB_HIP_CHECK(hipGetLastError());
    {
        const RedBuf rb[2] = {{dScal_ + 1, 2}, {dScal_ + 6, 1}};
        if (int e = comm_->allreduce(rb, 2, RedOp::Sum, s)) return e;
    }
    hipLaunchKernelGGL(k_lm_trial_end, dim3(1), dim3(kTeThreads), 0, s, dLm_, dScal_, (volatile int*)hLm_, S, dT_, dTbak_,
                       dX_, dXbak_, dX2_, dBp_, dBl_, 0, ChiFuse{nullptr, nullptr, 0}, (const Se3*)nullptr,
                       (const double*)nullptr, (const double*)(dScal_ + 6));
    ORB_HIP_CHECK(hipGetLastError());
    return 0;
}

int BaEngine::optimize_device(int iterations, const volatile bool* stop, int* its) {
    *its = 0;
    if (stopped(stop)) return 0;
    hLm_[0] = stopped(stop) ? 1 : 0;
    hLm_[1] = 0;
    hLm_[2] = 0;
    hLm_[3] = 0;
    hLm_[4] = 0;
    hLm_[5] = 0;
    hipLaunchKernelGGL(k_lm_begin, dim3(1), dim3(64), 0, stream_, dLm_, iterations);
    // at most 10 trials per iteration; the host stays one step ahead of the decisions.  It learns
    // of them from the words k_lm_trial_end writes to host memory ([2] steps decided, [1] done), not
    // from an event per step: an event record is a marker packet, about 5 us of idle queue after
    // every trial (profiles/r05vlba_*).  ORBGPU_LM_EVENTS=1 keeps the events (A/B).
    const int maxSteps = 10 * iterations;
    static const bool useEvents = [] {
        const char* e = getenv("ORBGPU_LM_EVENTS");
        return e && e[0] == '1';
    }();
    // Whether the run ended with step s's decision, read once step s is decided.  Not simply the
    // latest (done, steps) pair: it may already hold step s + 1's decision, which another rank of
    // a sharded run may not have seen when it decides whether to queue step s + 2 -- and every
    // rank must queue the same steps.  The pair is one 8-byte store: steps == s + 1 means its done
    // bit is step s's; steps > s + 1 means step s + 1 was decided, so it was live and step s did
    // not end the run; steps <= s (the stream drained without deciding step s) ends the loop.
    volatile unsigned long long* hw64 = (volatile unsigned long long*)(hLm_ + 4);   // (done, steps)
    auto done_after = [&](int st) {
        const unsigned long long v = *hw64;
        const int steps = (int)(v >> 32);
        return steps == st + 1 ? (v & 0xffffffffu) != 0 : steps <= st;
    };
    static const bool say = getenv("ORBGPU_BA_TIMES") != nullptr;   // host enqueue / wait split (tools/)
    using sclk = std::chrono::steady_clock;
    double tEnq = 0, tWait = 0;
    int nSteps = 0;
    for (int j = 0; j < maxSteps; j++) {
        const auto q0 = sclk::now();
        if (comm_) {
            if (int e = enqueue_lm_step_comm(j == 0)) return e;
        } else {
            enqueue_lm_step(j == 0);
        }
        ORB_HIP_CHECK(hipGetLastError());
        const auto q1 = sclk::now();
        nSteps++;
        last_lm[0]++;
        if (useEvents) {
            ORB_HIP_CHECK(hipEventRecord(lmEv_[j & 1], stream_));
            if (j >= 1) {
                ORB_HIP_CHECK(hipEventSynchronize(lmEv_[(j - 1) & 1]));
                if (done_after(j - 1)) break;
            }
        } else if (j >= 1) {
            // step j - 1 decided (steps >= j) or the run over.  No HIP call inside the wait: a
            // stream query or event sync makes the runtime fence the next launch (a ~5 us idle
            // gap on the queue after every trial).  Only a wait past 50 ms asks whether the stream
            // drained (its writes are all visible then; the final readback checks the state).
            const auto w0 = sclk::now();
            for (unsigned spin = 1;; spin++) {
                const unsigned long long v = *hw64;
                if ((int)(v >> 32) >= j || (v & 0xffffffffu)) break;
                if ((spin & 4095) == 0 && sclk::now() - w0 > std::chrono::milliseconds(50) &&
                    hipStreamQuery(stream_) == hipSuccess)
                    break;
                __builtin_ia32_pause();
            }
            if (done_after(j - 1)) {
                tEnq += std::chrono::duration<double, std::micro>(q1 - q0).count();
                tWait += std::chrono::duration<double, std::micro>(sclk::now() - q1).count();
                break;
            }
        }
        tEnq += std::chrono::duration<double, std::micro>(q1 - q0).count();
        tWait += std::chrono::duration<double, std::micro>(sclk::now() - q1).count();
        hLm_[0] = stopped(stop) ? 1 : 0;
    }
    if (say)
        fprintf(stderr, "[ba]   LM steps queued %d: host enqueue %.1f us/step, wait %.1f us/step\n", nSteps,
                tEnq / nSteps, tWait / nSteps);
    LmDev h;
    if (int e = d2h_poll(&h, dLm_, sizeof(LmDev))) return e;   // also drains the queue
    if (!h.done) return -7;    // the step bound is the trial bound: unreachable
    *its = h.it;
    for (int t = 0; t < std::min(h.nTrial, kLmTrials); t++) {
        trace_.trial_chi2.push_back(h.trialChi[t]);
        trace_.trial_lambda.push_back(h.trialLam[t]);
    }
    for (int t = 0; t < std::min(h.nSolve, kLmSolves); t++) {
        trace_.solve_ini_chi2.push_back(h.solveIni[t]);
        trace_.solve_chi2.push_back(h.solveChi[t]);
    }
    return 0;
}

// sharded: every rank sees the same stop decision (any rank's flag stops all)
int BaEngine::reduce_stop(const volatile bool* stop) {
    if (!comm_) return 0;
    hScal_[32] = (stop && *stop) ? 1.0 : 0.0;
    ORB_HIP_CHECK(hipMemcpyAsync(dScal_ + 6, hScal_ + 32, sizeof(double), hipMemcpyHostToDevice, stream_));
    if (int e = comm_->allreduce(dScal_ + 6, 1, RedOp::Sum, stream_)) return e;
    ORB_HIP_CHECK(hipMemcpyAsync(hScal_ + 33, dScal_ + 6, sizeof(double), hipMemcpyDeviceToHost, stream_));
    ORB_HIP_CHECK(hipStreamSynchronize(stream_));
    stopRed_ = hScal_[33] != 0.0;
    return 0;
}

int BaEngine::gate_edges(int final_check, uint8_t* erase) {
    if (!ne_) return 0;
    uint8_t* dFlag = (uint8_t*)(dScratch_);  // reuse scratch (ne bytes)
    hipLaunchKernelGGL(k_gate, dim3(nblk(ne_, 256)), dim3(256), 0, stream_, ne_, dE_, dT_, dX_, dErr_, dFlag, dLevel_,
                       dRobust_, final_check ? 0 : 1);
    ORB_HIP_CHECK(hipGetLastError());
    return erase ? d2h_poll(erase, dFlag, ne_) : 0;
}

int BaEngine::run(const ba_problem* P, const volatile bool* stop, ba_result* R, Comm* comm, const BaMode* mode) {
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    // the caller's edge arrays (upload_problem) are valid during this call only: forget them on
    // every exit
    struct EdgeRefs {
        BaEngine* e;
        ~EdgeRefs() {
            (void)e->join_sp_build();   // no helper thread outlives the call (both read the
            if (e->spEarly_.valid()) (void)e->spEarly_.get();   // caller's edge arrays)
            e->ePt_ = e->eKf_ = nullptr;
        }
    } edgeRefs{this};
    struct RunCount {
        RunCount() { g_ba_runs.fetch_add(1, std::memory_order_relaxed); }
        ~RunCount() { g_ba_runs.fetch_sub(1, std::memory_order_relaxed); }
    } runCount;
    smallUp_ = false;
    trace_ = BaTrace{};
    // a one-rank group is the unsharded call: every exchange would be the identity, so none is
    // made (no collective, no host round trip per structure and stop decision)
    comm_ = comm && comm->size() > 1 ? comm : nullptr;
    mode_ = mode ? *mode : BaMode{};
    last_lm[0] = last_lm[1] = last_lm[3] = 0;
    last_lm[2] = comm_ ? 1 : 0;
    stopRed_ = false;
    hsValid_ = false;     // hs_ holds this call's lists only after its first host build
    refineNext_ = false;
    std::memcpy(R->kf_Tcw, P->kf_Tcw, sizeof(float) * 16 * P->n_kf);
    std::memcpy(R->pt_pos, P->pt_pos, sizeof(float) * 3 * P->n_pt);
    if (P->n_edge) std::memset(R->edge_erase, 0, P->n_edge);
    R->aborted = 0;
    R->iterations[0] = R->iterations[1] = 0;
    R->n_erased = 0;
    if (!comm_ && ((stop && *stop) || P->n_edge == 0)) {
        R->aborted = 1;
        return 0;
    }
    if (int e = upload_problem(P)) return e;
    const auto t_up = clk::now();
    if (comm_) {  // every shard takes the same early-return decision
        if (int e = reduce_stop(stop)) return e;
    }
    double t_struct = 0;
    auto ts = clk::now();
    if (int e = build_structure(0)) return e;
    if (int e = issue_upload()) return e;   // (already queued by every build path)
    t_struct += std::chrono::duration<double, std::milli>(clk::now() - ts).count();
    if (comm_ && (stopRed_ || nEglob_ == 0)) {  // Optimizer.cc:655-657 (and no edges at all)
        R->aborted = 1;
        return 0;
    }
    const auto t_opt0 = clk::now();
    if (mode_.global) {
        // Optimizer::BundleAdjustment: initializeOptimization(); optimize(nIterations) (Optimizer.cc:190-191)
        if (st_.nP + nLglob_ > 0)
            if (int e = optimize(mode_.iterations, stop, &R->iterations[0])) return e;
    } else {
        if (st_.nP + nLglob_ > 0)
            if (int e = optimize(5, stop, &R->iterations[0])) return e;
        if (comm_) {
            if (int e = reduce_stop(stop)) return e;
        }
        if (!stopped(stop)) {
            if (host_lists()) {   // the host builder reads the levels from the host mirror
                std::vector<uint8_t> flag(ne_);
                if (int e = gate_edges(0, flag.data())) return e;
                for (int i = 0; i < ne_; i++)
                    if (flag[i]) level_[i] = 1;
            } else {               // k_gate moved the outliers to level 1 in dLevel_ itself
                if (int e = gate_edges(0, nullptr)) return e;
            }
            ts = clk::now();
            refineNext_ = refine_enabled();
            if (int e = build_structure(0)) return e;
            t_struct += std::chrono::duration<double, std::milli>(clk::now() - ts).count();
            if (nEglob_ > 0 && st_.nP + nLglob_ > 0)
                if (int e = optimize(10, stop, &R->iterations[1])) return e;
        }
        if (int e = gate_edges(1, R->edge_erase)) return e;
        for (int i = 0; i < ne_; i++) R->n_erased += R->edge_erase[i];
    }
    const auto t_opt1 = clk::now();
    std::vector<Se3> T(nkf_);
    std::vector<double> X(3 * (size_t)npt_);
    {   // poses and points back through the staging block, one wait
        const size_t bT = sizeof(Se3) * nkf_, bX = sizeof(double) * X.size();
        if (int e = stage_reserve(bT + bX + 64)) return e;
        char* st = (char*)hStage_;
        if (bT) ORB_HIP_CHECK(hipMemcpyAsync(st, dT_, bT, hipMemcpyDeviceToHost, stream_));
        if (bX) ORB_HIP_CHECK(hipMemcpyAsync(st + bT, dX_, bX, hipMemcpyDeviceToHost, stream_));
        if (int e = poll_stream()) return e;
        std::memcpy(T.data(), st, bT);
        std::memcpy(X.data(), st + bT, bX);
    }
    for (int k = 0; k < nkf_; k++)
        if (kfLocal_[k]) host_se3_to_Tcw(T[k], R->kf_Tcw + 16 * k);
    // BundleAdjustment writes back only the points that got a vertex (vbNotIncludedMP, Optimizer.cc:217-219);
    // LocalBundleAdjustment writes back every local map point (Optimizer.cc:771-777)
    for (int p = 0; p < npt_; p++)
        if (!mode_.global || ptHasEdge_[p])
            for (int k = 0; k < 3; k++) R->pt_pos[3 * p + k] = (float)X[3 * p + k];
    last_dist[0] = distOk_ ? 1 : 0;
    last_dist[1] = distOk_ ? sp_.dist_shared_tiles() : 0;
    last_dist[2] = distOk_ ? sp_.dist_shared_rows() : 0;
    last_dist[3] = tiled_ ? sp_.nA() : 0;
    last_ms[0] = std::chrono::duration<double, std::milli>(clk::now() - t0).count();
    last_ms[1] = t_struct;
    static const bool say = getenv("ORBGPU_BA_TIMES") != nullptr;   // host-phase breakdown (tools/)
    if (say) {
        auto ms = [](clk::time_point a, clk::time_point b) {
            return std::chrono::duration<double, std::milli>(b - a).count();
        };
        fprintf(stderr, "[ba] call %.3f ms: upload %.3f, structure %.3f, optimize %.3f (incl. the second pass's "
                        "structure), readback %.3f\n", last_ms[0], ms(t0, t_up), t_struct, ms(t_opt0, t_opt1),
                ms(t_opt1, clk::now()));
    }
    comm_ = nullptr;
    return 0;
}

}  // namespace orbgpu

// ---------------------------------------------------------------- unit entry points
namespace orbgpu {
int debug_ldlt(int n, const double* S, const double* b, double* x, int variant) {
    if (variant == 2 || variant == 3) {   // block-sparse tiled solver (3: nested dissection); upper triangle read
        std::vector<double> U((size_t)n * n, 0.0);
        for (int i = 0; i < n; i++)
            for (int j = i; j < n; j++) U[(size_t)i * n + j] = S[(size_t)i * n + j];
        int ok = 0;
        if (int e = ldlt_sparse_dense(n, U.data(), b, x, &ok, nullptr, variant == 3)) return e < 0 ? e : -1;
        return ok;
    }
    if (variant == 0 && n >= kLdltMax) return -3;   // [S | b] needs a column register for b
    double *dS = nullptr, *dB = nullptr, *dX = nullptr, *dScal = nullptr;
    const size_t nn = (size_t)std::max(n, 1);
    ORB_HIP_CHECK(hipMalloc(&dS, sizeof(double) * nn * nn));
    ORB_HIP_CHECK(hipMalloc(&dB, sizeof(double) * nn));
    ORB_HIP_CHECK(hipMalloc(&dX, sizeof(double) * nn));
    ORB_HIP_CHECK(hipMalloc(&dScal, sizeof(double) * 16));
    ORB_HIP_CHECK(hipMemcpy(dS, S, sizeof(double) * n * n, hipMemcpyHostToDevice));
    ORB_HIP_CHECK(hipMemcpy(dB, b, sizeof(double) * n, hipMemcpyHostToDevice));
    ORB_HIP_CHECK(hipMemset(dX, 0, sizeof(double) * nn));
    if (variant == 5 || variant == 6 || variant == 7) {
        if (n > kLdltColMax) return -3;
        if (variant == 5) hipLaunchKernelGGL(k_ldlt_col, dim3(1), dim3(256), 0, 0, n, dS, dB, dX, dScal, nullptr);
        else if (variant == 6) hipLaunchKernelGGL(k_ldlt_t, dim3(1), dim3(256), 0, 0, n, dS, dB, dX, dScal, nullptr);
        else hipLaunchKernelGGL(k_ldlt_2d, dim3(1), dim3(256), 0, 0, n, dS, dB, dX, dScal, nullptr);
    } else if (variant == 4) {
        if (n > kLdltRowMax) return -3;
        hipLaunchKernelGGL(k_ldlt_row, dim3(1), dim3(128), 0, 0, n, dS, dB, dX, dScal, nullptr);
    } else if (variant == 0) {
        const size_t shm = ldlt_reg_shm(n);
        hipLaunchKernelGGL(k_ldlt_reg, dim3(1), dim3(kLdltThreads), shm, 0, n, dS, dB, dX, dScal, nullptr);
    } else {
        hipLaunchKernelGGL(k_ldlt, dim3(1), dim3(256), sizeof(double) * n + 16, 0, n, dS, dB, dX, dScal, 0, nullptr);
    }
    ORB_HIP_CHECK(hipGetLastError());
    double sc[16];
    ORB_HIP_CHECK(hipMemcpy(sc, dScal, sizeof(sc), hipMemcpyDeviceToHost));
    ORB_HIP_CHECK(hipMemcpy(x, dX, sizeof(double) * n, hipMemcpyDeviceToHost));
    (void)hipFree(dS); (void)hipFree(dB); (void)hipFree(dX); (void)hipFree(dScal);
    return sc[3] != 0.0 ? 1 : 0;
}

// tiled factorisation only: A (n x n, upper = S) -> d on the diagonal, L in the strict lower
// triangle, the eliminated rows above
int debug_ldlt_factor(int n, const double* S, double* out) {
    if (n <= 0) return 0;
    std::vector<double> U((size_t)n * n, 0.0), b(n, 0.0), x(n, 0.0);
    for (int i = 0; i < n; i++)
        for (int j = i; j < n; j++) U[(size_t)i * n + j] = S[(size_t)i * n + j];
    int ok = 0;
    return ldlt_sparse_dense(n, U.data(), b.data(), x.data(), &ok, out, false);
}

__global__ void k_unit_wave_tree(const double* v, double* out) {
    const double t = wave_tree(v[threadIdx.x]);
    if (threadIdx.x == 0) *out = t;
}

// SharedDiv against the plain division on n operand pairs: out[2i] = shared, out[2i + 1] = a / b
__global__ void __launch_bounds__(256) k_unit_shared_div(const double* a, const double* b, int n, double* out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const SharedDiv d(b[i]);
    out[2 * i] = d.div(a[i]);
    out[2 * i + 1] = a[i] / b[i];
}

int debug_shared_div(const double* a, const double* b, int n, double* out) {
    if (n <= 0) return 0;
    double* d = nullptr;
    ORB_HIP_CHECK(hipMalloc(&d, sizeof(double) * 4 * (size_t)n));
    ORB_HIP_CHECK(hipMemcpy(d, a, sizeof(double) * n, hipMemcpyHostToDevice));
    ORB_HIP_CHECK(hipMemcpy(d + n, b, sizeof(double) * n, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_unit_shared_div, dim3((n + 255) / 256), dim3(256), 0, 0, d, d + n, n, d + 2 * n);
    ORB_HIP_CHECK(hipGetLastError());
    ORB_HIP_CHECK(hipMemcpy(out, d + 2 * n, sizeof(double) * 2 * (size_t)n, hipMemcpyDeviceToHost));
    (void)hipFree(d);
    return 0;
}

// instrumented builds only: read and clear this unit's section timers
int debug_prof(unsigned long long* out32) {
#ifdef ORBGPU_PROF
    ORB_HIP_CHECK(hipMemcpyFromSymbol(out32, HIP_SYMBOL(g_orbgpu_prof), sizeof(unsigned long long) * 16));
    unsigned long long z[32] = {};
    ORB_HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_orbgpu_prof), z, sizeof(z)));
    return ldlt_debug_prof(out32 + 16);   // ldlt.hip's timers (slots 16-23)
#else
    (void)out32;
    return -1;
#endif
}

int debug_set_csum_lds_max(int v) {
    ORB_HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_csum_lds_max), &v, sizeof(int)));
    ORB_HIP_CHECK(hipDeviceSynchronize());
    return 0;
}

int debug_wave_tree(const double* v64, double* out) {
    double* d = nullptr;
    ORB_HIP_CHECK(hipMalloc(&d, sizeof(double) * 65));
    ORB_HIP_CHECK(hipMemcpy(d, v64, sizeof(double) * 64, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_unit_wave_tree, dim3(1), dim3(64), 0, 0, d, d + 64);
    ORB_HIP_CHECK(hipGetLastError());
    ORB_HIP_CHECK(hipMemcpy(out, d + 64, sizeof(double), hipMemcpyDeviceToHost));
    (void)hipFree(d);
    return 0;
}

int debug_csum(const double* v, int n, double* out) {
    double *dV = nullptr, *dT = nullptr;
    const size_t nn = (size_t)std::max(n, 1);
    ORB_HIP_CHECK(hipMalloc(&dV, sizeof(double) * (nn + 16)));
    ORB_HIP_CHECK(hipMalloc(&dT, sizeof(double) * (2 * (nn / 64 + 64) + 16)));
    ORB_HIP_CHECK(hipMemcpy(dV, v, sizeof(double) * n, hipMemcpyHostToDevice));
    double* o = dT + 2 * (nn / 64 + 64);
    CsumList L{dV, n, dT, dT + nn / 64 + 64, o};
    hipLaunchKernelGGL(k_csum, dim3(1), dim3(1024), 0, 0, L, L, nullptr);
    ORB_HIP_CHECK(hipGetLastError());
    ORB_HIP_CHECK(hipMemcpy(out, o, sizeof(double), hipMemcpyDeviceToHost));
    (void)hipFree(dV); (void)hipFree(dT);
    return 0;
}
}  // namespace orbgpu
