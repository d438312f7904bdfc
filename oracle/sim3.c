/*
 * sim3.c -- TEST INFRASTRUCTURE ONLY (parity oracle).
 *
 * Restatement of ORB_SLAM2::Sim3Solver (reference src/Sim3Solver.cc): Horn's
 * closed-form similarity from 3 camera-frame point pairs inside RANSAC with a
 * bidirectional reprojection test.  cv::Mat float arithmetic is restated
 * expression by expression; OpenCV internals are unpinned:
 *   cv::eigen (symmetric, CV_32F)  -> OpenCV 3.2 JacobiImpl_<float> (hypot as sqrtf)
 *   cv::Rodrigues / atan2 / norm   -> double, with the deterministic det_* math below
 *   gemm / Mat::dot                -> float in, double accumulate
 * det_sincos/det_atan2 are used identically by the GPU kernels, so GPU and
 * oracle agree bit for bit; they are within a few ulp of libm (tests/test_oracle_kat.py).
 */
#include "orb_oracle.h"
#include <math.h>
#include <stdlib.h>
#include <string.h>

#define PI_D 3.14159265358979311600e+00
#define PIO2_D 1.57079632679489655800e+00

/* fdlibm kernel coefficients (__kernel_sin/__kernel_cos), |y| <= pi/4 */
void ora_det_sincos(double x, double* s_out, double* c_out)
{
    const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
                 S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
                 S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
    const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
                 C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
                 C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
    const double pio2_1 = 1.57079632673412561417e+00, pio2_1t = 6.07710050650619224932e-11;
    const double invpio2 = 6.36619772367581382433e-01;
    double fn = rint(x * invpio2);
    int n = (int)fn;
    double y = (x - fn * pio2_1) - fn * pio2_1t;
    double z = y * y;
    double r = S2 + z * (S3 + z * (S4 + z * (S5 + z * S6)));
    double s = y + (z * y) * (S1 + z * r);
    double rc = z * (C1 + z * (C2 + z * (C3 + z * (C4 + z * (C5 + z * C6)))));
    double c = 1.0 - (0.5 * z - z * rc);
    switch (n & 3) {
        case 0: *s_out = s; *c_out = c; break;
        case 1: *s_out = c; *c_out = -s; break;
        case 2: *s_out = -s; *c_out = -c; break;
        default: *s_out = -c; *c_out = s; break;
    }
}

static double det_atan01(double x) /* 0 <= x <= 1 */
{
    /* two half-angle reductions: atan(x) = 2 atan(x / (1 + sqrt(1 + x^2))) */
    x = x / (1.0 + sqrt(1.0 + x * x));
    x = x / (1.0 + sqrt(1.0 + x * x));
    double x2 = x * x, term = x, sum = x;
    for (int k = 1; k <= 14; k++) {
        term = term * x2;
        sum += ((k & 1) ? -term : term) / (2 * k + 1);
    }
    return 4.0 * sum;
}

double ora_det_atan2(double y, double x)
{
    const double ay = fabs(y), ax = fabs(x);
    double a;
    if (ax == 0 && ay == 0) a = 0;
    else if (ay <= ax) a = det_atan01(ay / ax);
    else a = PIO2_D - det_atan01(ax / ay);
    if (x < 0) a = PI_D - a;
    return y < 0 ? -a : a;
}

/* cv::eigen on a symmetric 4x4 float matrix: OpenCV 3.2 JacobiImpl_<float>.
 * A (row-major, destroyed), W eigenvalues (descending), V rows = eigenvectors. */
void ora_jacobi_eigen_f(float* A, int n, float* W, float* V)
{
    const float eps = 1.1920928955078125e-07f;
    int i, j, k, m, iters, maxIters = n * n * 30;
    int indR[8], indC[8];
    float mv = 0;
    for (i = 0; i < n; i++) {
        for (j = 0; j < n; j++) V[i * n + j] = 0;
        V[i * n + i] = 1;
    }
    for (k = 0; k < n; k++) {
        W[k] = A[(n + 1) * k];
        if (k < n - 1) {
            for (m = k + 1, mv = fabsf(A[n * k + m]), i = k + 2; i < n; i++) {
                float val = fabsf(A[n * k + i]);
                if (mv < val) mv = val, m = i;
            }
            indR[k] = m;
        }
        if (k > 0) {
            for (m = 0, mv = fabsf(A[k]), i = 1; i < k; i++) {
                float val = fabsf(A[n * i + k]);
                if (mv < val) mv = val, m = i;
            }
            indC[k] = m;
        }
    }
    if (n > 1)
        for (iters = 0; iters < maxIters; iters++) {
            for (k = 0, mv = fabsf(A[indR[0]]), i = 1; i < n - 1; i++) {
                float val = fabsf(A[n * i + indR[i]]);
                if (mv < val) mv = val, k = i;
            }
            int l = indR[k];
            for (i = 1; i < n; i++) {
                float val = fabsf(A[n * indC[i] + i]);
                if (mv < val) mv = val, k = indC[i], l = i;
            }
            float p = A[n * k + l];
            if (fabsf(p) <= eps) break;
            float y = (float)((W[l] - W[k]) * 0.5);
            float t = fabsf(y) + sqrtf(p * p + y * y);
            float s = sqrtf(p * p + t * t);
            float c = t / s;
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
                int idx = j == 0 ? k : l;
                if (idx < n - 1) {
                    for (m = idx + 1, mv = fabsf(A[n * idx + m]), i = idx + 2; i < n; i++) {
                        float val = fabsf(A[n * idx + i]);
                        if (mv < val) mv = val, m = i;
                    }
                    indR[idx] = m;
                }
                if (idx > 0) {
                    for (m = 0, mv = fabsf(A[idx]), i = 1; i < idx; i++) {
                        float val = fabsf(A[n * i + idx]);
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
            float tw = W[m]; W[m] = W[k]; W[k] = tw;
            for (i = 0; i < n; i++) { float tv = V[n * m + i]; V[n * m + i] = V[n * k + i]; V[n * k + i] = tv; }
        }
    }
}

/* cv::Rodrigues(rotation vector (float) -> 3x3 float) via double */
static void rodrigues(const float* v, float* R)
{
    double rx = v[0], ry = v[1], rz = v[2];
    double theta = sqrt(rx * rx + ry * ry + rz * rz);
    if (theta < 2.220446049250313e-16) {
        for (int i = 0; i < 9; i++) R[i] = (i % 4 == 0) ? 1.f : 0.f;
        return;
    }
    double s, c;
    ora_det_sincos(theta, &s, &c);
    double c1 = 1. - c;
    double itheta = theta ? 1. / theta : 0.;
    rx *= itheta; ry *= itheta; rz *= itheta;
    double rrt[9] = {rx * rx, rx * ry, rx * rz, rx * ry, ry * ry, ry * rz, rx * rz, ry * rz, rz * rz};
    double r_x[9] = {0, -rz, ry, rz, 0, -rx, -ry, rx, 0};
    for (int i = 0; i < 9; i++) R[i] = (float)(c * ((i % 4 == 0) ? 1.0 : 0.0) + c1 * rrt[i] + s * r_x[i]);
}

/* 3x3 float gemm rows: (float)(sum_k (double)a[i][k]*b[k][j]) */
static float gemm3(const float* A, int i, const float* B, int j, int bstride)
{
    double s = (double)A[3 * i] * B[j] + (double)A[3 * i + 1] * B[bstride + j] + (double)A[3 * i + 2] * B[2 * bstride + j];
    return (float)s;
}

typedef struct { float R[9], t[3], s, T12[16], T21[16]; } sim3_est;

/* ComputeSim3, Sim3Solver.cc:226-337.  P1, P2: 3x3 column-major sets (column i = point i). */
static void compute_sim3(const float P1[3][3], const float P2[3][3], int bFixScale, sim3_est* E)
{
    float O1[3], O2[3], Pr1[3][3], Pr2[3][3];  /* [row][col] */
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
    float M[3][3];  /* M = Pr2 * Pr1^T */
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++)
            M[i][j] = (float)((double)Pr2[i][0] * Pr1[j][0] + (double)Pr2[i][1] * Pr1[j][1] + (double)Pr2[i][2] * Pr1[j][2]);
    double N11 = M[0][0] + M[1][1] + M[2][2];
    double N12 = M[1][2] - M[2][1];
    double N13 = M[2][0] - M[0][2];
    double N14 = M[0][1] - M[1][0];
    double N22 = M[0][0] - M[1][1] - M[2][2];
    double N23 = M[0][1] + M[1][0];
    double N24 = M[2][0] + M[0][2];
    double N33 = -M[0][0] + M[1][1] - M[2][2];
    double N34 = M[1][2] + M[2][1];
    double N44 = -M[0][0] - M[1][1] + M[2][2];
    float N[16] = {(float)N11, (float)N12, (float)N13, (float)N14, (float)N12, (float)N22, (float)N23, (float)N24,
                   (float)N13, (float)N23, (float)N33, (float)N34, (float)N14, (float)N24, (float)N34, (float)N44};
    float eval[4], evec[16];
    ora_jacobi_eigen_f(N, 4, eval, evec);
    float vec[3] = {evec[1], evec[2], evec[3]};
    double nv = sqrt((double)vec[0] * vec[0] + (double)vec[1] * vec[1] + (double)vec[2] * vec[2]);
    double ang = ora_det_atan2(nv, evec[0]);
    double f = 2 * ang / nv;
    for (int i = 0; i < 3; i++) vec[i] = (float)(vec[i] * f);
    rodrigues(vec, E->R);
    float P3[3][3];  /* P3 = R * Pr2 */
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) P3[i][j] = gemm3(E->R, i, &Pr2[0][0], j, 3);
    if (!bFixScale) {
        double nom = 0, den = 0;
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) {
                nom += (double)Pr1[i][j] * P3[i][j];
                den += (float)(P3[i][j] * P3[i][j]);
            }
        E->s = (float)(nom / den);
    } else {
        E->s = 1.0f;
    }
    for (int i = 0; i < 3; i++) {
        double rO2 = (double)E->R[3 * i] * O2[0] + (double)E->R[3 * i + 1] * O2[1] + (double)E->R[3 * i + 2] * O2[2];
        E->t[i] = O1[i] - (float)(E->s * rO2);
    }
    memset(E->T12, 0, sizeof(E->T12));
    memset(E->T21, 0, sizeof(E->T21));
    E->T12[15] = E->T21[15] = 1.f;
    float sRinv[9];
    const double is = 1.0 / E->s;
    for (int i = 0; i < 3; i++) {
        for (int j = 0; j < 3; j++) {
            E->T12[4 * i + j] = (float)(E->s * (double)E->R[3 * i + j]);
            sRinv[3 * i + j] = (float)(is * (double)E->R[3 * j + i]);
            E->T21[4 * i + j] = sRinv[3 * i + j];
        }
        E->T12[4 * i + 3] = E->t[i];
    }
    for (int i = 0; i < 3; i++) {
        double v = (double)sRinv[3 * i] * E->t[0] + (double)sRinv[3 * i + 1] * E->t[1] + (double)sRinv[3 * i + 2] * E->t[2];
        E->T21[4 * i + 3] = (float)(-v);
    }
}

/* Project, 382-403 */
static void project(const float* X, const float* T, const float* K, float* uv)
{
    float p[3];
    for (int r = 0; r < 3; r++)
        p[r] = (float)((double)T[4 * r] * X[0] + (double)T[4 * r + 1] * X[1] + (double)T[4 * r + 2] * X[2] + (double)T[4 * r + 3]);
    const float invz = 1 / p[2];
    const float x = p[0] * invz, y = p[1] * invz;
    uv[0] = K[0] * x + K[2];
    uv[1] = K[1] * y + K[3];
}

struct ora_sim3 {
    int N, N1, bFixScale;
    float *X1, *X2, *p1im1, *p2im2;
    size_t *maxErr1, *maxErr2;
    int* idx1;
    float K1[4], K2[4];
    double prob;
    int minInliers, maxIts;
    int nIterations, nBestInliers;
    uint8_t *inl, *bestInl;
    sim3_est best;
    int ev_n;              /* test instrumentation: events of the last iterate() call */
    int ev[ORA_EV_CAP][2];
};

/* Sim3Solver ctor (37-112) on packed, already-filtered pairs: X1/X2 camera-frame points
 * (Rcw*X+tcw computed by the caller), sigma2 of the keypoints, index into vpMatched12. */
ora_sim3* ora_sim3_new(int N, const float* X1c, const float* X2c, const float* sigma2_1, const float* sigma2_2,
                       const int* idx1, int N1, const float* K1, const float* K2, int bFixScale)
{
    ora_sim3* S = (ora_sim3*)calloc(1, sizeof(ora_sim3));
    S->N = N; S->N1 = N1; S->bFixScale = bFixScale;
    S->X1 = (float*)malloc(sizeof(float) * 3 * (N + 1));
    S->X2 = (float*)malloc(sizeof(float) * 3 * (N + 1));
    S->p1im1 = (float*)malloc(sizeof(float) * 2 * (N + 1));
    S->p2im2 = (float*)malloc(sizeof(float) * 2 * (N + 1));
    S->maxErr1 = (size_t*)malloc(sizeof(size_t) * (N + 1));
    S->maxErr2 = (size_t*)malloc(sizeof(size_t) * (N + 1));
    S->idx1 = (int*)malloc(sizeof(int) * (N + 1));
    S->inl = (uint8_t*)calloc(N + 1, 1);
    S->bestInl = (uint8_t*)calloc(N + 1, 1);
    memcpy(S->X1, X1c, sizeof(float) * 3 * N);
    memcpy(S->X2, X2c, sizeof(float) * 3 * N);
    memcpy(S->idx1, idx1, sizeof(int) * N);
    memcpy(S->K1, K1, sizeof(float) * 4);
    memcpy(S->K2, K2, sizeof(float) * 4);
    for (int i = 0; i < N; i++) {
        S->maxErr1[i] = (size_t)(9.210 * sigma2_1[i]);
        S->maxErr2[i] = (size_t)(9.210 * sigma2_2[i]);
        /* FromCameraToImage, 405-423 */
        for (int k = 0; k < 2; k++) {
            const float* X = k ? S->X2 + 3 * i : S->X1 + 3 * i;
            const float* K = k ? S->K2 : S->K1;
            float* out = k ? S->p2im2 + 2 * i : S->p1im1 + 2 * i;
            const float invz = 1 / X[2];
            const float x = X[0] * invz, y = X[1] * invz;
            out[0] = K[0] * x + K[2];
            out[1] = K[1] * y + K[3];
        }
    }
    ora_sim3_set_ransac(S, 0.99, 6, 300);  /* the ctor's SetRansacParameters() (Sim3Solver.h:45 defaults) */
    return S;
}

void ora_sim3_free(ora_sim3* S)
{
    if (!S) return;
    free(S->X1); free(S->X2); free(S->p1im1); free(S->p2im2); free(S->maxErr1); free(S->maxErr2);
    free(S->idx1); free(S->inl); free(S->bestInl); free(S);
}

/* SetRansacParameters, 114-138 */
void ora_sim3_set_ransac(ora_sim3* S, double probability, int minInliers, int maxIterations)
{
    S->prob = probability;
    S->minInliers = minInliers;
    S->maxIts = maxIterations;
    float epsilon = (float)S->minInliers / S->N;
    int nIterations;
    if (S->minInliers == S->N) nIterations = 1;
    else nIterations = (int)ceil(log(1 - S->prob) / log(1 - pow(epsilon, 3)));
    int m = nIterations < S->maxIts ? nIterations : S->maxIts;
    S->maxIts = m > 1 ? m : 1;
    S->nIterations = 0;
}

/* CheckInliers, 340-364 */
static int check_inliers(ora_sim3* S, const sim3_est* E)
{
    int n = 0;
    for (int i = 0; i < S->N; i++) {
        float p2im1[2], p1im2[2];
        project(S->X2 + 3 * i, E->T12, S->K1, p2im1);
        project(S->X1 + 3 * i, E->T21, S->K2, p1im2);
        const float d1x = S->p1im1[2 * i] - p2im1[0], d1y = S->p1im1[2 * i + 1] - p2im1[1];
        const float d2x = p1im2[0] - S->p2im2[2 * i], d2y = p1im2[1] - S->p2im2[2 * i + 1];
        const float err1 = (float)((double)d1x * d1x + (double)d1y * d1y);
        const float err2 = (float)((double)d2x * d2x + (double)d2y * d2y);
        if (err1 < (float)S->maxErr1[i] && err2 < (float)S->maxErr2[i]) {
            S->inl[i] = 1;
            n++;
        } else {
            S->inl[i] = 0;
        }
    }
    return n;
}

/* iterate, 140-207.  Returns 1 with T12 when it returns a non-empty Mat. */
int ora_sim3_iterate(ora_sim3* S, int nIterations, ora_rng* rng, int* bNoMore, uint8_t* inliers, int* nInliers,
                     float* T12)
{
    *bNoMore = 0;
    memset(inliers, 0, S->N1);
    *nInliers = 0;
    S->ev_n = 0;
    if (S->N < S->minInliers) {
        *bNoMore = 1;
        return 0;
    }
    int* avail = (int*)malloc(sizeof(int) * (S->N + 1));
    int nCurrent = 0;
    while (S->nIterations < S->maxIts && nCurrent < nIterations) {
        nCurrent++;
        S->nIterations++;
        for (int i = 0; i < S->N; i++) avail[i] = i;
        int navail = S->N;
        float P1[3][3], P2[3][3];
        for (int i = 0; i < 3; ++i) {
            int randi = ora_rng_random_int(rng, 0, navail - 1);
            int idx = avail[randi];
            for (int r = 0; r < 3; r++) {
                P1[r][i] = S->X1[3 * idx + r];
                P2[r][i] = S->X2[3 * idx + r];
            }
            avail[randi] = avail[navail - 1];
            navail--;
        }
        sim3_est E;
        compute_sim3(P1, P2, S->bFixScale, &E);
        int ni = check_inliers(S, &E);
        if (ni >= S->nBestInliers) {
            memcpy(S->bestInl, S->inl, S->N);
            S->nBestInliers = ni;
            S->best = E;
            ora_ev_push(S->ev, &S->ev_n, nCurrent - 1, ni > S->minInliers ? 3 : 1);
            if (ni > S->minInliers) {
                *nInliers = ni;
                for (int i = 0; i < S->N; i++)
                    if (S->inl[i]) inliers[S->idx1[i]] = 1;
                memcpy(T12, E.T12, sizeof(float) * 16);
                free(avail);
                return 1;
            }
        }
    }
    free(avail);
    if (S->nIterations >= S->maxIts) *bNoMore = 1;
    return 0;
}

void ora_sim3_estimate(const ora_sim3* S, float* R, float* t, float* s)
{
    memcpy(R, S->best.R, sizeof(float) * 9);
    memcpy(t, S->best.t, sizeof(float) * 3);
    *s = S->best.s;
}

int ora_sim3_iterations(const ora_sim3* S) { return S->nIterations; }

int ora_sim3_events(const ora_sim3* S, int* out, int cap)
{
    const int n = S->ev_n < ORA_EV_CAP ? S->ev_n : ORA_EV_CAP;
    for (int i = 0; i < n && i < cap; i++) { out[2 * i] = S->ev[i][0]; out[2 * i + 1] = S->ev[i][1]; }
    return S->ev_n;
}
