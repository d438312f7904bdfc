// epnp.hpp -- device EPnP (Lepetit et al.) as in the reference's PnPsolver
// (src/PnPsolver.cc:375-950), FP64, one thread per pose problem.
//
// The OpenCV C-API calls the reference makes are restated with OpenCV 3.2's
// scalar semantics (one-sided Jacobi SVD, SVBkSb), in the exact operation
// order of the CPU oracle so GPU and oracle agree bit for bit:
//   cvMulTransposed  -> M^T M accumulated row by row (no M is materialised)
//   cvSVD / cvSolve(CV_SVD) / cvInvert(CV_SVD) -> jacobi_svd + backsubstitution
// Correspondences are read through an accessor (point k -> world xyz, pixel uv),
// so the 4-point hypotheses and the n-point Refine share one code path.
#pragma once
#include <hip/hip_runtime.h>

namespace orbgpu {
namespace epnp {

constexpr double kDblEps = 2.220446049250313e-16;
constexpr double kDblMin = 2.2250738585072014e-308;

// JacobiSVDImpl_<double> (OpenCV 3.2 lapack.cpp): At n x m (stride astep).
__device__ __forceinline__ void jacobi_svd(double* At, int astep, double* W_out, double* Vt, int vstep, int m, int n, int n1) {
    const double eps = kDblEps * 10;
    double W[12];
    const int max_iter = m > 30 ? m : 30;
    for (int i = 0; i < n; i++) {
        double sd = 0;
        for (int k = 0; k < m; k++) {
            const double t = At[i * astep + k];
            sd += t * t;
        }
        W[i] = sd;
        for (int k = 0; k < n; k++) Vt[i * vstep + k] = 0;
        Vt[i * vstep + i] = 1;
    }
    for (int iter = 0; iter < max_iter; iter++) {
        bool changed = false;
        for (int i = 0; i < n - 1; i++)
            for (int j = i + 1; j < n; j++) {
                double* Ai = At + i * astep;
                double* Aj = At + j * astep;
                double a = W[i], p = 0, b = W[j];
                for (int k = 0; k < m; k++) p += Ai[k] * Aj[k];
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
                for (int k = 0; k < m; k++) {
                    const double t0 = c * Ai[k] + s * Aj[k];
                    const double t1 = -s * Ai[k] + c * Aj[k];
                    Ai[k] = t0;
                    Aj[k] = t1;
                    a += t0 * t0;
                    b += t1 * t1;
                }
                W[i] = a;
                W[j] = b;
                changed = true;
                double* Vi = Vt + i * vstep;
                double* Vj = Vt + j * vstep;
                for (int k = 0; k < n; k++) {
                    const double t0 = c * Vi[k] + s * Vj[k];
                    const double t1 = -s * Vi[k] + c * Vj[k];
                    Vi[k] = t0;
                    Vj[k] = t1;
                }
            }
        if (!changed) break;
    }
    for (int i = 0; i < n; i++) {
        double sd = 0;
        for (int k = 0; k < m; k++) {
            const double t = At[i * astep + k];
            sd += t * t;
        }
        W[i] = sqrt(sd);
    }
    for (int i = 0; i < n - 1; i++) {
        int j = i;
        for (int k = i + 1; k < n; k++)
            if (W[j] < W[k]) j = k;
        if (i != j) {
            const double tw = W[i]; W[i] = W[j]; W[j] = tw;
            for (int k = 0; k < m; k++) { const double t = At[i * astep + k]; At[i * astep + k] = At[j * astep + k]; At[j * astep + k] = t; }
            for (int k = 0; k < n; k++) { const double t = Vt[i * vstep + k]; Vt[i * vstep + k] = Vt[j * vstep + k]; Vt[j * vstep + k] = t; }
        }
    }
    for (int i = 0; i < n; i++) W_out[i] = W[i];
    uint64_t rng = 0x12345678;
    for (int i = 0; i < n1; i++) {
        double sd = i < n ? W[i] : 0;
        for (int ii = 0; ii < 100 && sd <= kDblMin; ii++) {
            const double val0 = 1. / m;
            for (int k = 0; k < m; k++) {
                rng = (uint64_t)(unsigned)rng * 4164903690U + (unsigned)(rng >> 32);
                At[i * astep + k] = ((unsigned)rng & 256) != 0 ? val0 : -val0;
            }
            for (int it2 = 0; it2 < 2; it2++)
                for (int j = 0; j < i; j++) {
                    sd = 0;
                    for (int k = 0; k < m; k++) sd += At[i * astep + k] * At[j * astep + k];
                    double asum = 0;
                    for (int k = 0; k < m; k++) {
                        const double t = At[i * astep + k] - sd * At[j * astep + k];
                        At[i * astep + k] = t;
                        asum += fabs(t);
                    }
                    asum = asum > eps * 100 ? 1 / asum : 0;
                    for (int k = 0; k < m; k++) At[i * astep + k] *= asum;
                }
            sd = 0;
            for (int k = 0; k < m; k++) {
                const double t = At[i * astep + k];
                sd += t * t;
            }
            sd = sqrt(sd);
        }
        const double scale = 1 / sd;
        for (int k = 0; k < m; k++) At[i * astep + k] *= scale;
    }
}

// SVD::compute(A m x n, m >= n): w, Ut (n x m), Vt (n x n).  A is consumed as At scratch.
__device__ __forceinline__ void svd(const double* A, int m, int n, double* w, double* Ut, double* Vt) {
    for (int i = 0; i < n; i++)
        for (int k = 0; k < m; k++) Ut[i * m + k] = A[k * n + i];
    jacobi_svd(Ut, m, w, Vt, n, m, n, n);
}

__device__ __forceinline__ void svd_solve(const double* A, int m, int n, const double* b, double* x) {
    double w[6], Ut[36], Vt[36];
    svd(A, m, n, w, Ut, Vt);
    const int nm = m < n ? m : n;
    double threshold = 0;
    for (int j = 0; j < n; j++) x[j] = 0;
    for (int i = 0; i < nm; i++) threshold += w[i];
    threshold *= kDblEps * 2;
    for (int i = 0; i < nm; i++) {
        double wi = w[i];
        if (fabs(wi) <= threshold) continue;
        wi = 1 / wi;
        double s = 0;
        for (int j = 0; j < m; j++) s += Ut[i * m + j] * b[j];
        s *= wi;
        for (int j = 0; j < n; j++) x[j] = x[j] + s * Vt[i * n + j];
    }
}

__device__ __forceinline__ void svd_invert3(const double* A, double* X) {
    double w[3], Ut[9], Vt[9], buf[3];
    svd(A, 3, 3, w, Ut, Vt);
    double threshold = 0;
    for (int i = 0; i < 9; i++) X[i] = 0;
    for (int i = 0; i < 3; i++) threshold += w[i];
    threshold *= kDblEps * 2;
    for (int i = 0; i < 3; i++) {
        double wi = w[i];
        if (fabs(wi) <= threshold) continue;
        wi = 1 / wi;
        for (int j = 0; j < 3; j++) buf[j] = Ut[i * 3 + j] * wi;
        for (int r = 0; r < 3; r++)
            for (int c = 0; c < 3; c++) X[r * 3 + c] += Vt[i * 3 + r] * buf[c];
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
        double pw0tpw0[9], dc[3], uct[9], vt[9];
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
        svd(pw0tpw0, 3, 3, dc, uct, vt);
        for (int i = 1; i < 4; i++) {
            const double k = sqrt(dc[i - 1] / n);
            for (int j = 0; j < 3; j++) cws[i][j] = cws[0][j] + k * uct[3 * (i - 1) + j];
        }
    }

    __device__ __forceinline__ void barycentric() {
        double cc[9];
        for (int i = 0; i < 3; i++)
            for (int j = 1; j < 4; j++) cc[3 * i + j - 1] = cws[j][i] - cws[0][i];
        svd_invert3(cc, ci);
    }

    // cvMulTransposed(M, MtM, 1): rows of M in order 2i, 2i+1, accumulated in place.
    __device__ __forceinline__ void mtm(double* out) const {
        for (int i = 0; i < 144; i++) out[i] = 0;
        for (int i = 0; i < n; i++) {
            double a[4], u, v;
            alphas(i, a);
            P.uv(i, u, v);
            double r1[12], r2[12];
            for (int k = 0; k < 4; k++) {
                r1[3 * k] = a[k] * fu;
                r1[3 * k + 1] = 0.0;
                r1[3 * k + 2] = a[k] * (uc - u);
                r2[3 * k] = 0.0;
                r2[3 * k + 1] = a[k] * fv;
                r2[3 * k + 2] = a[k] * (vc - v);
            }
            for (int r = 0; r < 12; r++)
                for (int c = r; c < 12; c++) out[r * 12 + c] += r1[r] * r1[c];
            for (int r = 0; r < 12; r++)
                for (int c = r; c < 12; c++) out[r * 12 + c] += r2[r] * r2[c];
        }
        for (int r = 0; r < 12; r++)
            for (int c = 0; c < r; c++) out[r * 12 + c] = out[c * 12 + r];
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
        double abt[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}, d[3], ut[9], vt[9];
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
        svd(abt, 3, 3, d, ut, vt);
        double U[9], V[9];
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) {
                U[3 * i + j] = ut[3 * j + i];
                V[3 * i + j] = vt[3 * j + i];
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

    __device__ __forceinline__ double compute_R_and_t(const double* ut, const double* betas, double R[3][3], double t[3]) {
        for (int i = 0; i < 4; i++) ccs[i][0] = ccs[i][1] = ccs[i][2] = 0.0f;
        for (int i = 0; i < 4; i++) {
            const double* v = ut + 12 * (11 - i);
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
        double m[144], d[12], ut[144], vt[144];
        mtm(m);
        svd(m, 12, 12, d, ut, vt);
        double L[60], rho[6];
        {
            const double* v[4] = {ut + 12 * 11, ut + 12 * 10, ut + 12 * 9, ut + 12 * 8};
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
            svd_solve(l, 6, 4, rho, b4);
            double* be = Betas[1];
            if (b4[0] < 0) {
                be[0] = sqrt(-b4[0]); be[1] = -b4[1] / be[0]; be[2] = -b4[2] / be[0]; be[3] = -b4[3] / be[0];
            } else {
                be[0] = sqrt(b4[0]); be[1] = b4[1] / be[0]; be[2] = b4[2] / be[0]; be[3] = b4[3] / be[0];
            }
        }
        gauss_newton(L, rho, Betas[1]);
        rep[1] = compute_R_and_t(ut, Betas[1], Rs[1], ts[1]);
        {  // find_betas_approx_2
            double l[18], b3[3];
            for (int i = 0; i < 6; i++) { l[3 * i] = L[10 * i]; l[3 * i + 1] = L[10 * i + 1]; l[3 * i + 2] = L[10 * i + 2]; }
            svd_solve(l, 6, 3, rho, b3);
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
        rep[2] = compute_R_and_t(ut, Betas[2], Rs[2], ts[2]);
        {  // find_betas_approx_3
            double l[30], b5[5];
            for (int i = 0; i < 6; i++)
                for (int j = 0; j < 5; j++) l[5 * i + j] = L[10 * i + j];
            svd_solve(l, 6, 5, rho, b5);
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
        rep[3] = compute_R_and_t(ut, Betas[3], Rs[3], ts[3]);
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
