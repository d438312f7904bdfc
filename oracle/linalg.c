/*
 * linalg.c -- TEST INFRASTRUCTURE ONLY (parity oracle).
 *
 * The small dense linear algebra the reference reaches through OpenCV's C API
 * in PnPsolver.cc / Sim3Solver.cc ("parity unpinned" at this
 * boundary): restated from OpenCV 3.2 core/lapack.cpp scalar paths.
 *   ora_svd        cv::SVD::compute (JacobiSVDImpl_, one-sided Jacobi, eps = 10*DBL_EPSILON)
 *   ora_svd_solve  cv::solve(DECOMP_SVD) = SVD + SVBkSb (eps = 2*DBL_EPSILON)
 *   ora_svd_invert cv::invert(DECOMP_SVD)
 *   ora_mul_transposed_ata  cvMulTransposed(src, dst, 1) = src^T src
 * hypot(p, beta) is evaluated as sqrt(p*p + beta*beta) (both here and on the GPU).
 */
#include "orb_oracle.h"
#include <float.h>
#include <math.h>
#include <string.h>

/* cv::RNG(0x12345678).next(): multiply-with-carry */
static unsigned ora_cvrng_next(uint64_t* state)
{
    *state = (uint64_t)(unsigned)*state * 4164903690U + (unsigned)(*state >> 32);
    return (unsigned)*state;
}

/* JacobiSVDImpl_<double>: At is n x m (row stride astep), rows orthogonalised in place.
 * Outputs W (n), Vt (n x n, stride vstep, may be NULL); n1 = rows of U to normalise. */
static void jacobi_svd(double* At, int astep, double* W_out, double* Vt, int vstep, int m, int n, int n1)
{
    const double minval = DBL_MIN, eps = DBL_EPSILON * 10;
    double W[32];
    int i, j, k, iter, max_iter = m > 30 ? m : 30;
    for (i = 0; i < n; i++) {
        double sd = 0;
        for (k = 0; k < m; k++) {
            double t = At[i * astep + k];
            sd += t * t;
        }
        W[i] = sd;
        if (Vt) {
            for (k = 0; k < n; k++) Vt[i * vstep + k] = 0;
            Vt[i * vstep + i] = 1;
        }
    }
    for (iter = 0; iter < max_iter; iter++) {
        int changed = 0;
        for (i = 0; i < n - 1; i++)
            for (j = i + 1; j < n; j++) {
                double* Ai = At + i * astep;
                double* Aj = At + j * astep;
                double a = W[i], p = 0, b = W[j];
                for (k = 0; k < m; k++) p += Ai[k] * Aj[k];
                if (fabs(p) <= eps * sqrt(a * b)) continue;
                p *= 2;
                double beta = a - b, gamma = sqrt(p * p + beta * beta);
                double c, s;
                if (beta < 0) {
                    double delta = (gamma - beta) * 0.5;
                    s = sqrt(delta / gamma);
                    c = p / (gamma * s * 2);
                } else {
                    c = sqrt((gamma + beta) / (gamma * 2));
                    s = p / (gamma * c * 2);
                }
                a = b = 0;
                for (k = 0; k < m; k++) {
                    double t0 = c * Ai[k] + s * Aj[k];
                    double t1 = -s * Ai[k] + c * Aj[k];
                    Ai[k] = t0;
                    Aj[k] = t1;
                    a += t0 * t0;
                    b += t1 * t1;
                }
                W[i] = a;
                W[j] = b;
                changed = 1;
                if (Vt) {
                    double* Vi = Vt + i * vstep;
                    double* Vj = Vt + j * vstep;
                    for (k = 0; k < n; k++) {
                        double t0 = c * Vi[k] + s * Vj[k];
                        double t1 = -s * Vi[k] + c * Vj[k];
                        Vi[k] = t0;
                        Vj[k] = t1;
                    }
                }
            }
        if (!changed) break;
    }
    for (i = 0; i < n; i++) {
        double sd = 0;
        for (k = 0; k < m; k++) {
            double t = At[i * astep + k];
            sd += t * t;
        }
        W[i] = sqrt(sd);
    }
    for (i = 0; i < n - 1; i++) {
        j = i;
        for (k = i + 1; k < n; k++)
            if (W[j] < W[k]) j = k;
        if (i != j) {
            double tw = W[i]; W[i] = W[j]; W[j] = tw;
            if (Vt) {
                for (k = 0; k < m; k++) { double t = At[i * astep + k]; At[i * astep + k] = At[j * astep + k]; At[j * astep + k] = t; }
                for (k = 0; k < n; k++) { double t = Vt[i * vstep + k]; Vt[i * vstep + k] = Vt[j * vstep + k]; Vt[j * vstep + k] = t; }
            }
        }
    }
    for (i = 0; i < n; i++) W_out[i] = W[i];
    if (!Vt) return;
    uint64_t rng = 0x12345678;
    for (i = 0; i < n1; i++) {
        double sd = i < n ? W[i] : 0;
        for (int ii = 0; ii < 100 && sd <= minval; ii++) {
            const double val0 = 1. / m;
            for (k = 0; k < m; k++) At[i * astep + k] = (ora_cvrng_next(&rng) & 256) != 0 ? val0 : -val0;
            for (iter = 0; iter < 2; iter++)
                for (j = 0; j < i; j++) {
                    sd = 0;
                    for (k = 0; k < m; k++) sd += At[i * astep + k] * At[j * astep + k];
                    double asum = 0;
                    for (k = 0; k < m; k++) {
                        double t = At[i * astep + k] - sd * At[j * astep + k];
                        At[i * astep + k] = t;
                        asum += fabs(t);
                    }
                    asum = asum > eps * 100 ? 1 / asum : 0;
                    for (k = 0; k < m; k++) At[i * astep + k] *= asum;
                }
            sd = 0;
            for (k = 0; k < m; k++) {
                double t = At[i * astep + k];
                sd += t * t;
            }
            sd = sqrt(sd);
        }
        double scale = 1 / sd;
        for (k = 0; k < m; k++) At[i * astep + k] *= scale;
    }
}

/* SVD::compute(A) for m >= n (every use in the reference): w (n), Ut (n x m) =
 * transposed left vectors, Vt (n x n). */
void ora_svd(const double* A, int m, int n, double* w, double* Ut, double* Vt)
{
    double At[32 * 32], Vtmp[32 * 32];
    const int uv = (Ut || Vt) != 0;  /* SVD::compute allocates temp_v whenever u or vt is wanted */
    for (int i = 0; i < n; i++)
        for (int k = 0; k < m; k++) At[i * m + k] = A[k * n + i];
    jacobi_svd(At, m, w, uv ? Vtmp : NULL, n, m, n, uv ? n : 0);
    if (Ut) memcpy(Ut, At, sizeof(double) * n * m);
    if (Vt) memcpy(Vt, Vtmp, sizeof(double) * n * n);
}

/* SVBkSb: x (n) = V diag(1/w) U^T b, skipping w <= 2*DBL_EPSILON * sum(w). */
static void svbksb(int m, int n, const double* w, const double* Ut, const double* Vt, const double* b, double* x)
{
    const int nm = m < n ? m : n;
    double threshold = 0;
    for (int j = 0; j < n; j++) x[j] = 0;
    for (int i = 0; i < nm; i++) threshold += w[i];
    threshold *= DBL_EPSILON * 2;
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

/* cv::solve(A (m x n), b (m), x (n), DECOMP_SVD) */
void ora_svd_solve(const double* A, int m, int n, const double* b, double* x)
{
    double w[32], Ut[32 * 32], Vt[32 * 32];
    ora_svd(A, m, n, w, Ut, Vt);
    svbksb(m, n, w, Ut, Vt, b, x);
}

/* cv::invert(A (n x n), DECOMP_SVD): X = V diag(1/w) U^T */
void ora_svd_invert(const double* A, int n, double* X)
{
    double w[32], Ut[32 * 32], Vt[32 * 32], buf[32];
    ora_svd(A, n, n, w, Ut, Vt);
    double threshold = 0;
    for (int i = 0; i < n * n; i++) X[i] = 0;
    for (int i = 0; i < n; i++) threshold += w[i];
    threshold *= DBL_EPSILON * 2;
    for (int i = 0; i < n; i++) {
        double wi = w[i];
        if (fabs(wi) <= threshold) continue;
        wi = 1 / wi;
        for (int j = 0; j < n; j++) buf[j] = Ut[i * n + j] * wi;
        for (int r = 0; r < n; r++)
            for (int c = 0; c < n; c++) X[r * n + c] += Vt[i * n + r] * buf[c];
    }
}

/* cvMulTransposed(src (rows x cols), dst, order=1): dst = src^T * src */
void ora_mul_transposed_ata(const double* src, int rows, int cols, double* dst)
{
    for (int i = 0; i < cols; i++)
        for (int j = i; j < cols; j++) {
            double s = 0;
            for (int k = 0; k < rows; k++) s += src[k * cols + i] * src[k * cols + j];
            dst[i * cols + j] = s;
            dst[j * cols + i] = s;
        }
}
