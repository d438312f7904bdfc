// epnp.hpp -- device EPnP (Lepetit et al.) as in the reference's PnPsolver
// (src/PnPsolver.cc:375-950), FP64, one thread per pose problem.
//
// The OpenCV C-API calls the reference makes are restated with OpenCV 3.2's
// scalar semantics (one-sided Jacobi SVD, SVBkSb), in the exact operation
// order of the CPU oracle so GPU and oracle agree bit for bit:
//   cvMulTransposed  -> M^T M accumulated row by row (no M is materialised)
//   cvSVD / cvSolve(CV_SVD) / cvInvert(CV_SVD) -> jacobi_t + backsubstitution
// Correspondences are read through an accessor (point k -> world xyz, pixel uv),
// so the 4-point hypotheses and the n-point Refine share one code path.
#pragma once
#include <hip/hip_runtime.h>

namespace orbgpu {
namespace epnp {

constexpr double kDblEps = 2.220446049250313e-16;
constexpr double kDblMin = 2.2250738585072014e-308;

// JacobiSVDImpl_<double> (OpenCV 3.2 lapack.cpp) for the static shapes of compute_pose (the
// 12 x 12 M^T M, the 6 x n cvSolve systems, the 3 x 3 decompositions; n1 = N): every index is
// static, so At, V and W live in registers instead of per-lane scratch memory.  WANTV false:
// the caller asked for no V (cvSVD without a V output), whose rotations are then skipped --
// V is written, never read, by the sweeps.  The descending sort swaps rows through selects
// over the static candidates.
template <int M, int N, bool WANTV>
__device__ __forceinline__ void jacobi_t(double (&At)[N][M], double (&Wo)[N], double (&Vt)[N][N]) {
    const double eps = kDblEps * 10;
    double W[N];
#pragma unroll
    for (int i = 0; i < N; i++) {
        double sd = 0;
#pragma unroll
        for (int k = 0; k < M; k++) sd += At[i][k] * At[i][k];
        W[i] = sd;
        if (WANTV)
#pragma unroll
            for (int k = 0; k < N; k++) Vt[i][k] = k == i ? 1.0 : 0.0;
    }
    const int max_iter = M > 30 ? M : 30;
    for (int iter = 0; iter < max_iter; iter++) {
        bool changed = false;
#pragma unroll
        for (int i = 0; i < N - 1; i++)
#pragma unroll
            for (int j = i + 1; j < N; j++) {
                double a = W[i], p = 0, b = W[j];
#pragma unroll
                for (int k = 0; k < M; k++) p += At[i][k] * At[j][k];
                if (fabs(p) <= eps * sqrt(a * b)) continue;
                p *= 2;
                const double beta = a - b, gamma = sqrt(p * p + beta * beta);
                double c, s;
                if (beta < 0) {
                    const double delta = (gamma - beta) * 0.5;
                    s = sqrt(delta / gamma);
                    c = p / (gamma * s * 2);
                } else {
                    c = sqrt((gamma + beta) / (gamma * 2));
                    s = p / (gamma * c * 2);
                }
                a = b = 0;
#pragma unroll
                for (int k = 0; k < M; k++) {
                    const double t0 = c * At[i][k] + s * At[j][k];
                    const double t1 = -s * At[i][k] + c * At[j][k];
                    At[i][k] = t0;
                    At[j][k] = t1;
                    a += t0 * t0;
                    b += t1 * t1;
                }
                W[i] = a;
                W[j] = b;
                changed = true;
                if (WANTV)
#pragma unroll
                    for (int k = 0; k < N; k++) {
                        const double t0 = c * Vt[i][k] + s * Vt[j][k];
                        const double t1 = -s * Vt[i][k] + c * Vt[j][k];
                        Vt[i][k] = t0;
                        Vt[j][k] = t1;
                    }
            }
        if (!changed) break;
    }
#pragma unroll
    for (int i = 0; i < N; i++) {
        double sd = 0;
#pragma unroll
        for (int k = 0; k < M; k++) sd += At[i][k] * At[i][k];
        W[i] = sqrt(sd);
    }
#pragma unroll
    for (int i = 0; i < N - 1; i++) {
        int j = i;
        double wj = W[i];
#pragma unroll
        for (int k = i + 1; k < N; k++)
            if (wj < W[k]) {
                j = k;
                wj = W[k];
            }
#pragma unroll
        for (int r = i + 1; r < N; r++) {
            const bool sw = j == r;
            const double tw = W[i];
            W[i] = sw ? W[r] : W[i];
            W[r] = sw ? tw : W[r];
#pragma unroll
            for (int k = 0; k < M; k++) {
                const double t = At[i][k];
                At[i][k] = sw ? At[r][k] : At[i][k];
                At[r][k] = sw ? t : At[r][k];
            }
            if (WANTV)
#pragma unroll
                for (int k = 0; k < N; k++) {
                    const double t = Vt[i][k];
                    Vt[i][k] = sw ? Vt[r][k] : Vt[i][k];
                    Vt[r][k] = sw ? t : Vt[r][k];
                }
        }
    }
#pragma unroll
    for (int i = 0; i < N; i++) Wo[i] = W[i];
    uint64_t rng = 0x12345678;
#pragma unroll
    for (int i = 0; i < N; i++) {
        double sd = W[i];
        for (int ii = 0; ii < 100 && sd <= kDblMin; ii++) {
            const double val0 = 1. / M;
#pragma unroll
            for (int k = 0; k < M; k++) {
                rng = (uint64_t)(unsigned)rng * 4164903690U + (unsigned)(rng >> 32);
                At[i][k] = ((unsigned)rng & 256) != 0 ? val0 : -val0;
            }
            for (int it2 = 0; it2 < 2; it2++)
#pragma unroll
                for (int j = 0; j < i; j++) {
                    sd = 0;
#pragma unroll
                    for (int k = 0; k < M; k++) sd += At[i][k] * At[j][k];
                    double asum = 0;
#pragma unroll
                    for (int k = 0; k < M; k++) {
                        const double t = At[i][k] - sd * At[j][k];
                        At[i][k] = t;
                        asum += fabs(t);
                    }
                    asum = asum > eps * 100 ? 1 / asum : 0;
#pragma unroll
                    for (int k = 0; k < M; k++) At[i][k] *= asum;
                }
            sd = 0;
#pragma unroll
            for (int k = 0; k < M; k++) sd += At[i][k] * At[i][k];
            sd = sqrt(sd);
        }
        const double scale = 1 / sd;
#pragma unroll
        for (int k = 0; k < M; k++) At[i][k] *= scale;
    }
}

// svd() for a static M x N (row-major A): Ut = A^T decomposed in registers
template <int M, int N, bool WANTV>
__device__ __forceinline__ void svd_t(const double* A, double (&w)[N], double (&Ut)[N][M], double (&Vt)[N][N]) {
#pragma unroll
    for (int i = 0; i < N; i++)
#pragma unroll
        for (int k = 0; k < M; k++) Ut[i][k] = A[k * N + i];
    jacobi_t<M, N, WANTV>(Ut, w, Vt);
}

// cvSolve(A, b, x, CV_SVD) for a static M x N A (the find_betas_approx_* systems)
template <int M, int N>
__device__ __forceinline__ void svd_solve_t(const double* A, const double* b, double* x) {
    double w[N], Ut[N][M], Vt[N][N];
    svd_t<M, N, true>(A, w, Ut, Vt);
    constexpr int nm = M < N ? M : N;
    double threshold = 0;
#pragma unroll
    for (int j = 0; j < N; j++) x[j] = 0;
#pragma unroll
    for (int i = 0; i < nm; i++) threshold += w[i];
    threshold *= kDblEps * 2;
#pragma unroll
    for (int i = 0; i < nm; i++) {
        double wi = w[i];
        if (fabs(wi) <= threshold) continue;
        wi = 1 / wi;
        double s = 0;
#pragma unroll
        for (int j = 0; j < M; j++) s += Ut[i][j] * b[j];
        s *= wi;
#pragma unroll
        for (int j = 0; j < N; j++) x[j] = x[j] + s * Vt[i][j];
    }
}


__device__ __forceinline__ void svd_invert3(const double* A, double* X) {
    double w[3], Ut[3][3], Vt[3][3], buf[3];
    svd_t<3, 3, true>(A, w, Ut, Vt);
    double threshold = 0;
#pragma unroll
    for (int i = 0; i < 9; i++) X[i] = 0;
#pragma unroll
    for (int i = 0; i < 3; i++) threshold += w[i];
    threshold *= kDblEps * 2;
#pragma unroll
    for (int i = 0; i < 3; i++) {
        double wi = w[i];
        if (fabs(wi) <= threshold) continue;
        wi = 1 / wi;
#pragma unroll
        for (int j = 0; j < 3; j++) buf[j] = Ut[i][j] * wi;
#pragma unroll
        for (int r = 0; r < 3; r++)
#pragma unroll
            for (int c = 0; c < 3; c++) X[r * 3 + c] += Vt[i][r] * buf[c];
    }
}

__device__ __forceinline__ double dot3(const double* a, const double* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
__device__ __forceinline__ double dist2(const double* p1, const double* p2) {
    return (p1[0] - p2[0]) * (p1[0] - p2[0]) + (p1[1] - p2[1]) * (p1[1] - p2[1]) + (p1[2] - p2[2]) * (p1[2] - p2[2]);
}

// Gauss-Newton step of EPnP's beta refinement (PnPsolver.cc:840-858 calls
// qr_solve, 860-950): least squares on the 6x4 Jacobian J by Householder
// reflections, held in registers (fully unrolled, static indices).
//
// Numerics that parity pins (the column scale and every sum keep the
// reference's order; the algorithm itself is the textbook one):
//  - column k is scaled by 1/m_k, m_k = max |J(r,k)| taken over rows
//    k .. 4 only: the reference's max-scan starts at the diagonal and stops
//    one row short of the last one;
//  - v = scaled column with v_k += s, s = sign(v_k)·||v||; the reflector's
//    norm term is s·v_k and the R diagonal is -m_k·s;
//  - reflections are applied to the later columns, then to the right-hand
//    side, column by column; back substitution runs bottom-up.
// Returns false (x untouched) when a column is exactly zero.
__device__ __forceinline__ bool householder_ls_6x4(double (&J)[6][4], double (&rhs)[6], double (&x)[4]) {
    double vnorm[4], rdiag[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        double m = fabs(J[k][k]);
#pragma unroll
        for (int r = k; r < 5; ++r) m = (m < fabs(J[r][k])) ? fabs(J[r][k]) : m;
        if (m == 0) return false;
        const double inv_m = 1. / m;
        double ss = 0.0;
#pragma unroll
        for (int r = k; r < 6; ++r) {
            J[r][k] *= inv_m;
            ss += J[r][k] * J[r][k];
        }
        const double s = (J[k][k] < 0) ? -sqrt(ss) : sqrt(ss);
        J[k][k] += s;
        vnorm[k] = s * J[k][k];
        rdiag[k] = -m * s;
#pragma unroll
        for (int c = k + 1; c < 4; ++c) {
            double proj = 0;
#pragma unroll
            for (int r = k; r < 6; ++r) proj += J[r][k] * J[r][c];
            const double f = proj / vnorm[k];
#pragma unroll
            for (int r = k; r < 6; ++r) J[r][c] -= f * J[r][k];
        }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        double proj = 0;
#pragma unroll
        for (int r = k; r < 6; ++r) proj += J[r][k] * rhs[r];
        proj /= vnorm[k];
#pragma unroll
        for (int r = k; r < 6; ++r) rhs[r] -= proj * J[r][k];
    }
    x[3] = rhs[3] / rdiag[3];
#pragma unroll
    for (int i = 2; i >= 0; --i) {
        double acc = 0;
#pragma unroll
        for (int c = i + 1; c < 4; ++c) acc += J[i][c] * x[c];
        x[i] = (rhs[i] - acc) / rdiag[i];
    }
    return true;
}

__device__ __forceinline__ void gauss_newton(const double* L, const double* rho, double betas[4]) {
    double A[6][4], b[6], x[4] = {0, 0, 0, 0};
    for (int k = 0; k < 5; k++) {
        for (int i = 0; i < 6; i++) {
            const double* rowL = L + i * 10;
            double* rowA = A[i];
            rowA[0] = 2 * rowL[0] * betas[0] + rowL[1] * betas[1] + rowL[3] * betas[2] + rowL[6] * betas[3];
            rowA[1] = rowL[1] * betas[0] + 2 * rowL[2] * betas[1] + rowL[4] * betas[2] + rowL[7] * betas[3];
            rowA[2] = rowL[3] * betas[0] + rowL[4] * betas[1] + 2 * rowL[5] * betas[2] + rowL[8] * betas[3];
            rowA[3] = rowL[6] * betas[0] + rowL[7] * betas[1] + rowL[8] * betas[2] + 2 * rowL[9] * betas[3];
            b[i] = rho[i] - (rowL[0] * betas[0] * betas[0] + rowL[1] * betas[0] * betas[1] + rowL[2] * betas[1] * betas[1] +
                             rowL[3] * betas[0] * betas[2] + rowL[4] * betas[1] * betas[2] + rowL[5] * betas[2] * betas[2] +
                             rowL[6] * betas[0] * betas[3] + rowL[7] * betas[1] * betas[3] + rowL[8] * betas[2] * betas[3] +
                             rowL[9] * betas[3] * betas[3]);
        }
        householder_ls_6x4(A, b, x);  // singular: x keeps its previous value
        for (int i = 0; i < 4; i++) betas[i] += x[i];
    }
}

// Point accessor: pw(k, out[3]), uv(k, &u, &v); n correspondences.
template <class Pts>
struct Solver {
    const Pts& P;
    int n;
    double fu, fv, uc, vc;
    double cws[4][3], ccs[4][3], ci[9];

    __device__ __forceinline__ Solver(const Pts& p, int n_, double fu_, double fv_, double uc_, double vc_)
        : P(p), n(n_), fu(fu_), fv(fv_), uc(uc_), vc(vc_) {}

    __device__ __forceinline__ void alphas(int i, double a[4]) const {
        double pi[3];
        P.pw(i, pi);
        for (int j = 0; j < 3; j++)
            a[1 + j] = ci[3 * j] * (pi[0] - cws[0][0]) + ci[3 * j + 1] * (pi[1] - cws[0][1]) + ci[3 * j + 2] * (pi[2] - cws[0][2]);
        a[0] = 1.0f - a[1] - a[2] - a[3];
    }
    __device__ __forceinline__ void pc(int i, double out[3]) const {
        double a[4];
        alphas(i, a);
        for (int j = 0; j < 3; j++) out[j] = a[0] * ccs[0][j] + a[1] * ccs[1][j] + a[2] * ccs[2][j] + a[3] * ccs[3][j];
    }

    __device__ __forceinline__ void choose_control_points() {
        cws[0][0] = cws[0][1] = cws[0][2] = 0;
        for (int i = 0; i < n; i++) {
            double p[3];
            P.pw(i, p);
            for (int j = 0; j < 3; j++) cws[0][j] += p[j];
        }
        for (int j = 0; j < 3; j++) cws[0][j] /= n;
        double pw0tpw0[9], dc[3], uct[3][3], vt_unused[3][3];
        for (int a = 0; a < 3; a++)
            for (int b = a; b < 3; b++) {
                double s = 0;
                for (int k = 0; k < n; k++) {
                    double p[3];
                    P.pw(k, p);
                    s += (p[a] - cws[0][a]) * (p[b] - cws[0][b]);
                }
                pw0tpw0[a * 3 + b] = s;
                pw0tpw0[b * 3 + a] = s;
            }
        svd_t<3, 3, false>(pw0tpw0, dc, uct, vt_unused);
        for (int i = 1; i < 4; i++) {
            const double k = sqrt(dc[i - 1] / n);
            for (int j = 0; j < 3; j++) cws[i][j] = cws[0][j] + k * uct[i - 1][j];
        }
    }

    __device__ __forceinline__ void barycentric() {
        double cc[9];
        for (int i = 0; i < 3; i++)
            for (int j = 1; j < 4; j++) cc[3 * i + j - 1] = cws[j][i] - cws[0][i];
        svd_invert3(cc, ci);
    }

    // cvMulTransposed(M, MtM, 1): rows of M in order 2i, 2i+1, accumulated in place.  The 78
    // upper-triangle sums stay in registers across the points (static indices) and are written
    // once.
    __device__ __forceinline__ void mtm(double (&out)[12][12]) const {
        double acc[78];
#pragma unroll
        for (int q = 0; q < 78; q++) acc[q] = 0;
        for (int i = 0; i < n; i++) {
            double a[4], u, v;
            alphas(i, a);
            P.uv(i, u, v);
            double r1[12], r2[12];
#pragma unroll
            for (int k = 0; k < 4; k++) {
                r1[3 * k] = a[k] * fu;
                r1[3 * k + 1] = 0.0;
                r1[3 * k + 2] = a[k] * (uc - u);
                r2[3 * k] = 0.0;
                r2[3 * k + 1] = a[k] * fv;
                r2[3 * k + 2] = a[k] * (vc - v);
            }
#pragma unroll
            for (int r = 0, q = 0; r < 12; r++)
#pragma unroll
                for (int c = r; c < 12; c++, q++) acc[q] += r1[r] * r1[c];
#pragma unroll
            for (int r = 0, q = 0; r < 12; r++)
#pragma unroll
                for (int c = r; c < 12; c++, q++) acc[q] += r2[r] * r2[c];
        }
#pragma unroll
        for (int r = 0, q = 0; r < 12; r++)
#pragma unroll
            for (int c = r; c < 12; c++, q++) {
                out[r][c] = acc[q];
                out[c][r] = acc[q];
            }
    }

    __device__ __forceinline__ double reprojection_error(const double R[3][3], const double t[3]) const {
        double sum2 = 0.0;
        for (int i = 0; i < n; i++) {
            double pw[3], u, v;
            P.pw(i, pw);
            P.uv(i, u, v);
            const double Xc = dot3(R[0], pw) + t[0];
            const double Yc = dot3(R[1], pw) + t[1];
            const double inv_Zc = 1.0 / (dot3(R[2], pw) + t[2]);
            const double ue = uc + fu * Xc * inv_Zc;
            const double ve = vc + fv * Yc * inv_Zc;
            sum2 += sqrt((u - ue) * (u - ue) + (v - ve) * (v - ve));
        }
        return sum2 / n;
    }

    __device__ __forceinline__ void estimate_R_and_t(double R[3][3], double t[3]) const {
        double pc0[3] = {0, 0, 0}, pw0[3] = {0, 0, 0};
        for (int i = 0; i < n; i++) {
            double pcv[3], pw[3];
            pc(i, pcv);
            P.pw(i, pw);
            for (int j = 0; j < 3; j++) {
                pc0[j] += pcv[j];
                pw0[j] += pw[j];
            }
        }
        for (int j = 0; j < 3; j++) {
            pc0[j] /= n;
            pw0[j] /= n;
        }
        double abt[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}, d[3], ut[3][3], vt[3][3];
        for (int i = 0; i < n; i++) {
            double pcv[3], pw[3];
            pc(i, pcv);
            P.pw(i, pw);
            for (int j = 0; j < 3; j++) {
                abt[3 * j] += (pcv[j] - pc0[j]) * (pw[0] - pw0[0]);
                abt[3 * j + 1] += (pcv[j] - pc0[j]) * (pw[1] - pw0[1]);
                abt[3 * j + 2] += (pcv[j] - pc0[j]) * (pw[2] - pw0[2]);
            }
        }
        svd_t<3, 3, true>(abt, d, ut, vt);
        double U[9], V[9];
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) {
                U[3 * i + j] = ut[j][i];
                V[3 * i + j] = vt[j][i];
            }
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) R[i][j] = dot3(U + 3 * i, V + 3 * j);
        const double det = R[0][0] * R[1][1] * R[2][2] + R[0][1] * R[1][2] * R[2][0] + R[0][2] * R[1][0] * R[2][1] -
                           R[0][2] * R[1][1] * R[2][0] - R[0][1] * R[1][0] * R[2][2] - R[0][0] * R[1][2] * R[2][1];
        if (det < 0) {
            R[2][0] = -R[2][0];
            R[2][1] = -R[2][1];
            R[2][2] = -R[2][2];
        }
        t[0] = pc0[0] - dot3(R[0], pw0);
        t[1] = pc0[1] - dot3(R[1], pw0);
        t[2] = pc0[2] - dot3(R[2], pw0);
    }

    // u4: rows 8..11 of Ut (the four smallest singular vectors of MtM), u4 + 12 (3 - i) = row 11 - i
    __device__ __forceinline__ double compute_R_and_t(const double* u4, const double* betas, double R[3][3], double t[3]) {
        for (int i = 0; i < 4; i++) ccs[i][0] = ccs[i][1] = ccs[i][2] = 0.0f;
        for (int i = 0; i < 4; i++) {
            const double* v = u4 + 12 * (3 - i);
            for (int j = 0; j < 4; j++)
                for (int k = 0; k < 3; k++) ccs[j][k] += betas[i] * v[3 * j + k];
        }
        // solve_for_sign: pcs of point 0; negating ccs negates every pc exactly
        double p0[3];
        pc(0, p0);
        if (p0[2] < 0.0)
            for (int i = 0; i < 4; i++)
                for (int j = 0; j < 3; j++) ccs[i][j] = -ccs[i][j];
        estimate_R_and_t(R, t);
        return reprojection_error(R, t);
    }

    // compute_pose, PnPsolver.cc:477-525
    __device__ __forceinline__ double compute_pose(double R[3][3], double t[3]) {
        choose_control_points();
        barycentric();
        // cvSVD(MtM, D, Ut, 0, CV_SVD_MODIFY_A | CV_SVD_U_T) (PnPsolver.cc:492-493): MtM is
        // symmetric, so its transpose is itself and the Jacobi sweeps run on it in place; V is
        // not requested
        // (the whole decomposition in registers; only the 4 rows compute_pose reads are kept)
        double At[12][12], d[12], v_unused[12][12], u4[48];
        mtm(At);
        jacobi_t<12, 12, false>(At, d, v_unused);
#pragma unroll
        for (int r = 0; r < 4; r++)
#pragma unroll
            for (int k = 0; k < 12; k++) u4[12 * r + k] = At[8 + r][k];
        double L[60], rho[6];
        {
            const double* v[4] = {u4 + 36, u4 + 24, u4 + 12, u4};
            double dv[4][6][3];
            for (int i = 0; i < 4; i++) {
                int a = 0, b = 1;
                for (int j = 0; j < 6; j++) {
                    dv[i][j][0] = v[i][3 * a] - v[i][3 * b];
                    dv[i][j][1] = v[i][3 * a + 1] - v[i][3 * b + 1];
                    dv[i][j][2] = v[i][3 * a + 2] - v[i][3 * b + 2];
                    b++;
                    if (b > 3) { a++; b = a + 1; }
                }
            }
            for (int i = 0; i < 6; i++) {
                double* row = L + 10 * i;
                row[0] = dot3(dv[0][i], dv[0][i]);
                row[1] = 2.0f * dot3(dv[0][i], dv[1][i]);
                row[2] = dot3(dv[1][i], dv[1][i]);
                row[3] = 2.0f * dot3(dv[0][i], dv[2][i]);
                row[4] = 2.0f * dot3(dv[1][i], dv[2][i]);
                row[5] = dot3(dv[2][i], dv[2][i]);
                row[6] = 2.0f * dot3(dv[0][i], dv[3][i]);
                row[7] = 2.0f * dot3(dv[1][i], dv[3][i]);
                row[8] = 2.0f * dot3(dv[2][i], dv[3][i]);
                row[9] = dot3(dv[3][i], dv[3][i]);
            }
            rho[0] = dist2(cws[0], cws[1]);
            rho[1] = dist2(cws[0], cws[2]);
            rho[2] = dist2(cws[0], cws[3]);
            rho[3] = dist2(cws[1], cws[2]);
            rho[4] = dist2(cws[1], cws[3]);
            rho[5] = dist2(cws[2], cws[3]);
        }
        double Betas[4][4], rep[4], Rs[4][3][3], ts[4][3];
        {  // find_betas_approx_1
            double l[24], b4[4];
            for (int i = 0; i < 6; i++) {
                l[4 * i] = L[10 * i]; l[4 * i + 1] = L[10 * i + 1]; l[4 * i + 2] = L[10 * i + 3]; l[4 * i + 3] = L[10 * i + 6];
            }
            svd_solve_t<6, 4>(l, rho, b4);
            double* be = Betas[1];
            if (b4[0] < 0) {
                be[0] = sqrt(-b4[0]); be[1] = -b4[1] / be[0]; be[2] = -b4[2] / be[0]; be[3] = -b4[3] / be[0];
            } else {
                be[0] = sqrt(b4[0]); be[1] = b4[1] / be[0]; be[2] = b4[2] / be[0]; be[3] = b4[3] / be[0];
            }
        }
        gauss_newton(L, rho, Betas[1]);
        rep[1] = compute_R_and_t(u4, Betas[1], Rs[1], ts[1]);
        {  // find_betas_approx_2
            double l[18], b3[3];
            for (int i = 0; i < 6; i++) { l[3 * i] = L[10 * i]; l[3 * i + 1] = L[10 * i + 1]; l[3 * i + 2] = L[10 * i + 2]; }
            svd_solve_t<6, 3>(l, rho, b3);
            double* be = Betas[2];
            if (b3[0] < 0) {
                be[0] = sqrt(-b3[0]);
                be[1] = (b3[2] < 0) ? sqrt(-b3[2]) : 0.0;
            } else {
                be[0] = sqrt(b3[0]);
                be[1] = (b3[2] > 0) ? sqrt(b3[2]) : 0.0;
            }
            if (b3[1] < 0) be[0] = -be[0];
            be[2] = 0.0;
            be[3] = 0.0;
        }
        gauss_newton(L, rho, Betas[2]);
        rep[2] = compute_R_and_t(u4, Betas[2], Rs[2], ts[2]);
        {  // find_betas_approx_3
            double l[30], b5[5];
            for (int i = 0; i < 6; i++)
                for (int j = 0; j < 5; j++) l[5 * i + j] = L[10 * i + j];
            svd_solve_t<6, 5>(l, rho, b5);
            double* be = Betas[3];
            if (b5[0] < 0) {
                be[0] = sqrt(-b5[0]);
                be[1] = (b5[2] < 0) ? sqrt(-b5[2]) : 0.0;
            } else {
                be[0] = sqrt(b5[0]);
                be[1] = (b5[2] > 0) ? sqrt(b5[2]) : 0.0;
            }
            if (b5[1] < 0) be[0] = -be[0];
            be[2] = b5[3] / be[0];
            be[3] = 0.0;
        }
        gauss_newton(L, rho, Betas[3]);
        rep[3] = compute_R_and_t(u4, Betas[3], Rs[3], ts[3]);
        int N = 1;
        if (rep[2] < rep[1]) N = 2;
        if (rep[3] < rep[N]) N = 3;
        for (int i = 0; i < 3; i++) {
            for (int j = 0; j < 3; j++) R[i][j] = Rs[N][i][j];
            t[i] = ts[N][i];
        }
        return rep[N];
    }
};

}  // namespace epnp
}  // namespace orbgpu
