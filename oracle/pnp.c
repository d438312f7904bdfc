/*
 * pnp.c -- TEST INFRASTRUCTURE ONLY (parity oracle).
 *
 * Restatement of ORB_SLAM2::PnPsolver (reference src/PnPsolver.cc, the EPnP
 * of Lepetit et al. inside a RANSAC loop).  FP64 EPnP with the OpenCV C-API
 * calls restated in linalg.c; the RANSAC control flow (|| loop condition,
 * best-so-far Refine, early return) kept line for line.
 */
#include "orb_oracle.h"
#include <math.h>
#include <stdlib.h>
#include <string.h>

void ora_svd(const double* A, int m, int n, double* w, double* Ut, double* Vt);
void ora_svd_solve(const double* A, int m, int n, const double* b, double* x);
void ora_svd_invert(const double* A, int n, double* X);
void ora_mul_transposed_ata(const double* src, int rows, int cols, double* dst);

/* ---------------------------------------------------------------- EPnP core */
typedef struct {
    double uc, vc, fu, fv;
    int n;                 /* number_of_correspondences */
    const double* pws;     /* 3n */
    const double* us;      /* 2n */
    double* alphas;        /* 4n */
    double* pcs;           /* 3n */
    double cws[4][3], ccs[4][3];
} epnp_t;

static double dot3(const double* a, const double* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
static double dist2(const double* p1, const double* p2)
{
    return (p1[0] - p2[0]) * (p1[0] - p2[0]) + (p1[1] - p2[1]) * (p1[1] - p2[1]) + (p1[2] - p2[2]) * (p1[2] - p2[2]);
}

/* choose_control_points, PnPsolver.cc:375-409 */
static void choose_control_points(epnp_t* E)
{
    const int n = E->n;
    E->cws[0][0] = E->cws[0][1] = E->cws[0][2] = 0;
    for (int i = 0; i < n; i++)
        for (int j = 0; j < 3; j++) E->cws[0][j] += E->pws[3 * i + j];
    for (int j = 0; j < 3; j++) E->cws[0][j] /= n;
    double* PW0 = (double*)malloc(sizeof(double) * 3 * n);
    double pw0tpw0[9], dc[3], uct[9];
    for (int i = 0; i < n; i++)
        for (int j = 0; j < 3; j++) PW0[3 * i + j] = E->pws[3 * i + j] - E->cws[0][j];
    ora_mul_transposed_ata(PW0, n, 3, pw0tpw0);
    ora_svd(pw0tpw0, 3, 3, dc, uct, NULL);
    free(PW0);
    for (int i = 1; i < 4; i++) {
        double k = sqrt(dc[i - 1] / n);
        for (int j = 0; j < 3; j++) E->cws[i][j] = E->cws[0][j] + k * uct[3 * (i - 1) + j];
    }
}

/* compute_barycentric_coordinates, 411-434 */
static void compute_barycentric_coordinates(epnp_t* E)
{
    double cc[9], ci[9];
    for (int i = 0; i < 3; i++)
        for (int j = 1; j < 4; j++) cc[3 * i + j - 1] = E->cws[j][i] - E->cws[0][i];
    ora_svd_invert(cc, 3, ci);
    for (int i = 0; i < E->n; i++) {
        const double* pi = E->pws + 3 * i;
        double* a = E->alphas + 4 * i;
        for (int j = 0; j < 3; j++)
            a[1 + j] = ci[3 * j] * (pi[0] - E->cws[0][0]) + ci[3 * j + 1] * (pi[1] - E->cws[0][1]) +
                       ci[3 * j + 2] * (pi[2] - E->cws[0][2]);
        a[0] = 1.0f - a[1] - a[2] - a[3];
    }
}

/* fill_M, 436-451 */
static void fill_M(const epnp_t* E, double* M, int row, const double* as, double u, double v)
{
    double* M1 = M + row * 12;
    double* M2 = M1 + 12;
    for (int i = 0; i < 4; i++) {
        M1[3 * i] = as[i] * E->fu;
        M1[3 * i + 1] = 0.0;
        M1[3 * i + 2] = as[i] * (E->uc - u);
        M2[3 * i] = 0.0;
        M2[3 * i + 1] = as[i] * E->fv;
        M2[3 * i + 2] = as[i] * (E->vc - v);
    }
}

static void compute_ccs(epnp_t* E, const double* betas, const double* ut)
{
    for (int i = 0; i < 4; i++) E->ccs[i][0] = E->ccs[i][1] = E->ccs[i][2] = 0.0f;
    for (int i = 0; i < 4; i++) {
        const double* v = ut + 12 * (11 - i);
        for (int j = 0; j < 4; j++)
            for (int k = 0; k < 3; k++) E->ccs[j][k] += betas[i] * v[3 * j + k];
    }
}

static void compute_pcs(epnp_t* E)
{
    for (int i = 0; i < E->n; i++) {
        const double* a = E->alphas + 4 * i;
        double* pc = E->pcs + 3 * i;
        for (int j = 0; j < 3; j++)
            pc[j] = a[0] * E->ccs[0][j] + a[1] * E->ccs[1][j] + a[2] * E->ccs[2][j] + a[3] * E->ccs[3][j];
    }
}

static double reprojection_error(const epnp_t* E, const double R[3][3], const double t[3])
{
    double sum2 = 0.0;
    for (int i = 0; i < E->n; i++) {
        const double* pw = E->pws + 3 * i;
        double Xc = dot3(R[0], pw) + t[0];
        double Yc = dot3(R[1], pw) + t[1];
        double inv_Zc = 1.0 / (dot3(R[2], pw) + t[2]);
        double ue = E->uc + E->fu * Xc * inv_Zc;
        double ve = E->vc + E->fv * Yc * inv_Zc;
        double u = E->us[2 * i], v = E->us[2 * i + 1];
        sum2 += sqrt((u - ue) * (u - ue) + (v - ve) * (v - ve));
    }
    return sum2 / E->n;
}

/* estimate_R_and_t, 569-627 */
static void estimate_R_and_t(const epnp_t* E, double R[3][3], double t[3])
{
    double pc0[3] = {0, 0, 0}, pw0[3] = {0, 0, 0};
    for (int i = 0; i < E->n; i++) {
        const double* pc = E->pcs + 3 * i;
        const double* pw = E->pws + 3 * i;
        for (int j = 0; j < 3; j++) {
            pc0[j] += pc[j];
            pw0[j] += pw[j];
        }
    }
    for (int j = 0; j < 3; j++) {
        pc0[j] /= E->n;
        pw0[j] /= E->n;
    }
    double abt[9] = {0}, abt_d[3], abt_ut[9], abt_vt[9];
    for (int i = 0; i < E->n; i++) {
        const double* pc = E->pcs + 3 * i;
        const double* pw = E->pws + 3 * i;
        for (int j = 0; j < 3; j++) {
            abt[3 * j] += (pc[j] - pc0[j]) * (pw[0] - pw0[0]);
            abt[3 * j + 1] += (pc[j] - pc0[j]) * (pw[1] - pw0[1]);
            abt[3 * j + 2] += (pc[j] - pc0[j]) * (pw[2] - pw0[2]);
        }
    }
    ora_svd(abt, 3, 3, abt_d, abt_ut, abt_vt);
    /* cvSVD(ABt, D, U, V): U = abt_ut^T, V = abt_vt^T; R[i][j] = dot(U row i, V row j) */
    double U[9], V[9];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
            U[3 * i + j] = abt_ut[3 * j + i];
            V[3 * i + j] = abt_vt[3 * j + i];
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

static void solve_for_sign(epnp_t* E)
{
    if (E->pcs[2] < 0.0) {
        for (int i = 0; i < 4; i++)
            for (int j = 0; j < 3; j++) E->ccs[i][j] = -E->ccs[i][j];
        for (int i = 0; i < E->n; i++) {
            E->pcs[3 * i] = -E->pcs[3 * i];
            E->pcs[3 * i + 1] = -E->pcs[3 * i + 1];
            E->pcs[3 * i + 2] = -E->pcs[3 * i + 2];
        }
    }
}

static double compute_R_and_t(epnp_t* E, const double* ut, const double* betas, double R[3][3], double t[3])
{
    compute_ccs(E, betas, ut);
    compute_pcs(E);
    solve_for_sign(E);
    estimate_R_and_t(E, R, t);
    return reprojection_error(E, R, t);
}

static void find_betas_approx_1(const double* L, const double* rho, double* betas)
{
    double l[6 * 4], b4[4];
    for (int i = 0; i < 6; i++) {
        l[4 * i] = L[10 * i]; l[4 * i + 1] = L[10 * i + 1]; l[4 * i + 2] = L[10 * i + 3]; l[4 * i + 3] = L[10 * i + 6];
    }
    ora_svd_solve(l, 6, 4, rho, b4);
    if (b4[0] < 0) {
        betas[0] = sqrt(-b4[0]);
        betas[1] = -b4[1] / betas[0];
        betas[2] = -b4[2] / betas[0];
        betas[3] = -b4[3] / betas[0];
    } else {
        betas[0] = sqrt(b4[0]);
        betas[1] = b4[1] / betas[0];
        betas[2] = b4[2] / betas[0];
        betas[3] = b4[3] / betas[0];
    }
}

static void find_betas_approx_2(const double* L, const double* rho, double* betas)
{
    double l[6 * 3], b3[3];
    for (int i = 0; i < 6; i++) { l[3 * i] = L[10 * i]; l[3 * i + 1] = L[10 * i + 1]; l[3 * i + 2] = L[10 * i + 2]; }
    ora_svd_solve(l, 6, 3, rho, b3);
    if (b3[0] < 0) {
        betas[0] = sqrt(-b3[0]);
        betas[1] = (b3[2] < 0) ? sqrt(-b3[2]) : 0.0;
    } else {
        betas[0] = sqrt(b3[0]);
        betas[1] = (b3[2] > 0) ? sqrt(b3[2]) : 0.0;
    }
    if (b3[1] < 0) betas[0] = -betas[0];
    betas[2] = 0.0;
    betas[3] = 0.0;
}

static void find_betas_approx_3(const double* L, const double* rho, double* betas)
{
    double l[6 * 5], b5[5];
    for (int i = 0; i < 6; i++)
        for (int j = 0; j < 5; j++) l[5 * i + j] = L[10 * i + j];
    ora_svd_solve(l, 6, 5, rho, b5);
    if (b5[0] < 0) {
        betas[0] = sqrt(-b5[0]);
        betas[1] = (b5[2] < 0) ? sqrt(-b5[2]) : 0.0;
    } else {
        betas[0] = sqrt(b5[0]);
        betas[1] = (b5[2] > 0) ? sqrt(b5[2]) : 0.0;
    }
    if (b5[1] < 0) betas[0] = -betas[0];
    betas[2] = b5[3] / betas[0];
    betas[3] = 0.0;
}

static void compute_L_6x10(const double* ut, double* l_6x10)
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
        double* row = l_6x10 + 10 * i;
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
}

static void compute_rho(const epnp_t* E, double* rho)
{
    rho[0] = dist2(E->cws[0], E->cws[1]);
    rho[1] = dist2(E->cws[0], E->cws[2]);
    rho[2] = dist2(E->cws[0], E->cws[3]);
    rho[3] = dist2(E->cws[1], E->cws[2]);
    rho[4] = dist2(E->cws[1], E->cws[3]);
    rho[5] = dist2(E->cws[2], E->cws[3]);
}

/* qr_solve, 860-950 (Householder); returns 0 when A is singular (X untouched) */
static int qr_solve(double* A, int nr, int nc, double* b, double* X)
{
    double A1[16], A2[16];
    double* pA = A;
    double* ppAkk = pA;
    for (int k = 0; k < nc; k++) {
        double* ppAik = ppAkk;
        double eta = fabs(*ppAik);
        for (int i = k + 1; i < nr; i++) {
            double elt = fabs(*ppAik);
            if (eta < elt) eta = elt;
            ppAik += nc;
        }
        if (eta == 0) {
            A1[k] = A2[k] = 0.0;
            return 0;
        } else {
            double* pp = ppAkk;
            double sum = 0.0, inv_eta = 1. / eta;
            for (int i = k; i < nr; i++) {
                *pp *= inv_eta;
                sum += *pp * *pp;
                pp += nc;
            }
            double sigma = sqrt(sum);
            if (*ppAkk < 0) sigma = -sigma;
            *ppAkk += sigma;
            A1[k] = sigma * *ppAkk;
            A2[k] = -eta * sigma;
            for (int j = k + 1; j < nc; j++) {
                double* p2 = ppAkk;
                double s2 = 0;
                for (int i = k; i < nr; i++) {
                    s2 += *p2 * p2[j - k];
                    p2 += nc;
                }
                double tau = s2 / A1[k];
                p2 = ppAkk;
                for (int i = k; i < nr; i++) {
                    p2[j - k] -= tau * *p2;
                    p2 += nc;
                }
            }
        }
        ppAkk += nc + 1;
    }
    double* ppAjj = pA;
    double* pb = b;
    for (int j = 0; j < nc; j++) {
        double* ppAij = ppAjj;
        double tau = 0;
        for (int i = j; i < nr; i++) {
            tau += *ppAij * pb[i];
            ppAij += nc;
        }
        tau /= A1[j];
        ppAij = ppAjj;
        for (int i = j; i < nr; i++) {
            pb[i] -= tau * *ppAij;
            ppAij += nc;
        }
        ppAjj += nc + 1;
    }
    double* pX = X;
    pX[nc - 1] = pb[nc - 1] / A2[nc - 1];
    for (int i = nc - 2; i >= 0; i--) {
        double* ppAij = pA + i * nc + (i + 1);
        double sum = 0;
        for (int j = i + 1; j < nc; j++) {
            sum += *ppAij * pX[j];
            ppAij++;
        }
        pX[i] = (pb[i] - sum) / A2[i];
    }
    return 1;
}

static void gauss_newton(const double* L, const double* rho, double betas[4])
{
    double A[24], b[6], x[4] = {0, 0, 0, 0};
    for (int k = 0; k < 5; k++) {
        for (int i = 0; i < 6; i++) {
            const double* rowL = L + i * 10;
            double* rowA = A + i * 4;
            rowA[0] = 2 * rowL[0] * betas[0] + rowL[1] * betas[1] + rowL[3] * betas[2] + rowL[6] * betas[3];
            rowA[1] = rowL[1] * betas[0] + 2 * rowL[2] * betas[1] + rowL[4] * betas[2] + rowL[7] * betas[3];
            rowA[2] = rowL[3] * betas[0] + rowL[4] * betas[1] + 2 * rowL[5] * betas[2] + rowL[8] * betas[3];
            rowA[3] = rowL[6] * betas[0] + rowL[7] * betas[1] + rowL[8] * betas[2] + 2 * rowL[9] * betas[3];
            b[i] = rho[i] - (rowL[0] * betas[0] * betas[0] + rowL[1] * betas[0] * betas[1] + rowL[2] * betas[1] * betas[1] +
                             rowL[3] * betas[0] * betas[2] + rowL[4] * betas[1] * betas[2] + rowL[5] * betas[2] * betas[2] +
                             rowL[6] * betas[0] * betas[3] + rowL[7] * betas[1] * betas[3] + rowL[8] * betas[2] * betas[3] +
                             rowL[9] * betas[3] * betas[3]);
        }
        qr_solve(A, 6, 4, b, x);  /* singular A: x keeps its last value (reference: stale stack) */
        for (int i = 0; i < 4; i++) betas[i] += x[i];
    }
}

/* compute_pose, 477-525 */
double ora_epnp_compute_pose(const double* pws, const double* us, int n, double fu, double fv, double uc,
                             double vc, double R[3][3], double t[3])
{
    epnp_t E;
    E.uc = uc; E.vc = vc; E.fu = fu; E.fv = fv;
    E.n = n; E.pws = pws; E.us = us;
    E.alphas = (double*)malloc(sizeof(double) * 4 * n);
    E.pcs = (double*)malloc(sizeof(double) * 3 * n);
    choose_control_points(&E);
    compute_barycentric_coordinates(&E);
    double* M = (double*)malloc(sizeof(double) * 24 * n);
    for (int i = 0; i < n; i++) fill_M(&E, M, 2 * i, E.alphas + 4 * i, us[2 * i], us[2 * i + 1]);
    double mtm[144], d[12], ut[144];
    ora_mul_transposed_ata(M, 2 * n, 12, mtm);
    ora_svd(mtm, 12, 12, d, ut, NULL);
    free(M);
    double L[60], rho[6];
    compute_L_6x10(ut, L);
    compute_rho(&E, rho);
    double Betas[4][4], rep_errors[4], Rs[4][3][3], ts[4][3];
    find_betas_approx_1(L, rho, Betas[1]);
    gauss_newton(L, rho, Betas[1]);
    rep_errors[1] = compute_R_and_t(&E, ut, Betas[1], Rs[1], ts[1]);
    find_betas_approx_2(L, rho, Betas[2]);
    gauss_newton(L, rho, Betas[2]);
    rep_errors[2] = compute_R_and_t(&E, ut, Betas[2], Rs[2], ts[2]);
    find_betas_approx_3(L, rho, Betas[3]);
    gauss_newton(L, rho, Betas[3]);
    rep_errors[3] = compute_R_and_t(&E, ut, Betas[3], Rs[3], ts[3]);
    int N = 1;
    if (rep_errors[2] < rep_errors[1]) N = 2;
    if (rep_errors[3] < rep_errors[N]) N = 3;
    memcpy(R, Rs[N], sizeof(double) * 9);
    memcpy(t, ts[N], sizeof(double) * 3);
    free(E.alphas);
    free(E.pcs);
    return rep_errors[N];
}

/* ---------------------------------------------------------------- RANSAC */
struct ora_pnp {
    int N, nMatches;
    float* p3d;        /* mvP3Dw (N x 3) */
    float* p2d;        /* mvP2D (N x 2) */
    float* maxErr;     /* mvMaxError */
    int* kpIdx;        /* mvKeyPointIndices */
    double fu, fv, uc, vc;
    /* ransac params */
    double prob;
    int minInliers, maxIts, minSet;
    float epsilon;
    /* state across iterate() calls */
    int nIterations, nBestInliers;
    uint8_t* bestInliers;
    float bestTcw[16];
    double Ri[3][3], ti[3];
    int nInliersi;
    uint8_t* inliersi;
    int nRefined;
    uint8_t* refinedInliers;
    float refinedTcw[16];
    /* test instrumentation (no reference counterpart): the events of the last iterate() call,
     * (hypothesis index within the call, kind) with kind 1 = best update, 2 = Refine failed,
     * 3 = Refine succeeded; the first ORA_EV_CAP are kept, ev_n counts them all */
    int ev_n;
    int ev[ORA_EV_CAP][2];
};

/* PnPsolver ctor (67-110) on already-packed correspondences + SetRansacParameters defaults */
ora_pnp* ora_pnp_new(int N, const float* p3d, const float* p2d, const float* sigma2, const int* kpIdx, int nMatches,
                     float fx, float fy, float cx, float cy)
{
    ora_pnp* P = (ora_pnp*)calloc(1, sizeof(ora_pnp));
    P->N = N;
    P->nMatches = nMatches;
    P->p3d = (float*)malloc(sizeof(float) * 3 * (N + 1));
    P->p2d = (float*)malloc(sizeof(float) * 2 * (N + 1));
    P->maxErr = (float*)malloc(sizeof(float) * (N + 1));
    P->kpIdx = (int*)malloc(sizeof(int) * (N + 1));
    P->bestInliers = (uint8_t*)calloc(N + 1, 1);
    P->inliersi = (uint8_t*)calloc(N + 1, 1);
    P->refinedInliers = (uint8_t*)calloc(N + 1, 1);
    memcpy(P->p3d, p3d, sizeof(float) * 3 * N);
    memcpy(P->p2d, p2d, sizeof(float) * 2 * N);
    memcpy(P->kpIdx, kpIdx, sizeof(int) * N);
    for (int i = 0; i < N; i++) P->maxErr[i] = sigma2[i];  /* times th2 in set_ransac */
    P->fu = fx; P->fv = fy; P->uc = cx; P->vc = cy;
    return P;
}

void ora_pnp_free(ora_pnp* P)
{
    if (!P) return;
    free(P->p3d); free(P->p2d); free(P->maxErr); free(P->kpIdx);
    free(P->bestInliers); free(P->inliersi); free(P->refinedInliers);
    free(P);
}

/* SetRansacParameters, 121-157; sigma2 was stored in maxErr by ora_pnp_new */
void ora_pnp_set_ransac(ora_pnp* P, double probability, int minInliers, int maxIterations, int minSet,
                        float epsilon, float th2)
{
    P->prob = probability;
    P->minInliers = minInliers;
    P->maxIts = maxIterations;
    P->epsilon = epsilon;
    P->minSet = minSet;
    const int N = P->N;
    int nMinInliers = (int)(N * P->epsilon);
    if (nMinInliers < P->minInliers) nMinInliers = P->minInliers;
    if (nMinInliers < minSet) nMinInliers = minSet;
    P->minInliers = nMinInliers;
    if (P->epsilon < (float)P->minInliers / N) P->epsilon = (float)P->minInliers / N;
    int nIterations;
    if (P->minInliers == N) nIterations = 1;
    else nIterations = (int)ceil(log(1 - P->prob) / log(1 - pow(P->epsilon, 3)));
    P->maxIts = 1 > (nIterations < P->maxIts ? nIterations : P->maxIts) ? 1
                                                                           : (nIterations < P->maxIts ? nIterations : P->maxIts);
    for (int i = 0; i < N; i++) P->maxErr[i] = P->maxErr[i] * th2;
}

int ora_pnp_max_its(const ora_pnp* P) { return P->maxIts; }
int ora_pnp_min_inliers(const ora_pnp* P) { return P->minInliers; }

/* CheckInliers, 308-339 (float/double mix kept) */
static void check_inliers(ora_pnp* P)
{
    P->nInliersi = 0;
    for (int i = 0; i < P->N; i++) {
        const float X = P->p3d[3 * i], Y = P->p3d[3 * i + 1], Z = P->p3d[3 * i + 2];
        const float Xc = (float)(P->Ri[0][0] * X + P->Ri[0][1] * Y + P->Ri[0][2] * Z + P->ti[0]);
        const float Yc = (float)(P->Ri[1][0] * X + P->Ri[1][1] * Y + P->Ri[1][2] * Z + P->ti[1]);
        const float invZc = (float)(1 / (P->Ri[2][0] * X + P->Ri[2][1] * Y + P->Ri[2][2] * Z + P->ti[2]));
        const double ue = P->uc + P->fu * Xc * invZc;
        const double ve = P->vc + P->fv * Yc * invZc;
        const float distX = (float)(P->p2d[2 * i] - ue);
        const float distY = (float)(P->p2d[2 * i + 1] - ve);
        const float error2 = distX * distX + distY * distY;
        if (error2 < P->maxErr[i]) {
            P->inliersi[i] = 1;
            P->nInliersi++;
        } else {
            P->inliersi[i] = 0;
        }
    }
}

static void pose_to_tcw(const double R[3][3], const double t[3], float* T)
{
    memset(T, 0, sizeof(float) * 16);
    for (int i = 0; i < 3; i++) {
        for (int j = 0; j < 3; j++) T[4 * i + j] = (float)R[i][j];
        T[4 * i + 3] = (float)t[i];
    }
    T[15] = 1.0f;
}

static void compute_pose_on(ora_pnp* P, const int* idx, int n)
{
    double* pws = (double*)malloc(sizeof(double) * 3 * n);
    double* us = (double*)malloc(sizeof(double) * 2 * n);
    for (int k = 0; k < n; k++) {
        const int i = idx[k];
        pws[3 * k] = P->p3d[3 * i]; pws[3 * k + 1] = P->p3d[3 * i + 1]; pws[3 * k + 2] = P->p3d[3 * i + 2];
        us[2 * k] = P->p2d[2 * i]; us[2 * k + 1] = P->p2d[2 * i + 1];
    }
    ora_epnp_compute_pose(pws, us, n, P->fu, P->fv, P->uc, P->vc, P->Ri, P->ti);
    free(pws);
    free(us);
}

/* Refine, 260-305 (uses the best-so-far inliers) */
static int refine(ora_pnp* P)
{
    int* idx = (int*)malloc(sizeof(int) * (P->N + 1));
    int n = 0;
    for (int i = 0; i < P->N; i++)
        if (P->bestInliers[i]) idx[n++] = i;
    compute_pose_on(P, idx, n);
    free(idx);
    check_inliers(P);
    P->nRefined = P->nInliersi;
    memcpy(P->refinedInliers, P->inliersi, P->N);
    if (P->nInliersi > P->minInliers) {
        pose_to_tcw(P->Ri, P->ti, P->refinedTcw);
        return 1;
    }
    return 0;
}

/* iterate, 165-258.  inliers_out: nMatches bytes (vbInliers), Tcw 16 floats.
 * Returns 1 if a pose is returned (non-empty Mat), 0 otherwise. */
int ora_pnp_iterate(ora_pnp* P, int nIterations, ora_rng* rng, int* bNoMore, uint8_t* inliers_out,
                    int* nInliers, float* Tcw)
{
    *bNoMore = 0;
    *nInliers = 0;
    P->ev_n = 0;
    memset(inliers_out, 0, P->nMatches);
    if (P->N < P->minInliers) {
        *bNoMore = 1;
        return 0;
    }
    int* avail = (int*)malloc(sizeof(int) * (P->N + 1));
    int nCurrentIterations = 0;
    int sel[64];
    while (P->nIterations < P->maxIts || nCurrentIterations < nIterations) {
        nCurrentIterations++;
        P->nIterations++;
        for (int i = 0; i < P->N; i++) avail[i] = i;
        int navail = P->N;
        for (int i = 0; i < P->minSet; ++i) {
            int randi = ora_rng_random_int(rng, 0, navail - 1);
            sel[i] = avail[randi];
            avail[randi] = avail[navail - 1];
            navail--;
        }
        compute_pose_on(P, sel, P->minSet);
        check_inliers(P);
        if (P->nInliersi >= P->minInliers) {
            if (P->nInliersi > P->nBestInliers) {
                memcpy(P->bestInliers, P->inliersi, P->N);
                P->nBestInliers = P->nInliersi;
                pose_to_tcw(P->Ri, P->ti, P->bestTcw);
                ora_ev_push(P->ev, &P->ev_n, nCurrentIterations - 1, 1);
            }
            const int ok = refine(P);
            ora_ev_push(P->ev, &P->ev_n, nCurrentIterations - 1, ok ? 3 : 2);
            if (ok) {
                *nInliers = P->nRefined;
                for (int i = 0; i < P->N; i++)
                    if (P->refinedInliers[i]) inliers_out[P->kpIdx[i]] = 1;
                memcpy(Tcw, P->refinedTcw, sizeof(float) * 16);
                free(avail);
                return 1;
            }
        }
    }
    free(avail);
    if (P->nIterations >= P->maxIts) {
        *bNoMore = 1;
        if (P->nBestInliers >= P->minInliers) {
            *nInliers = P->nBestInliers;
            for (int i = 0; i < P->N; i++)
                if (P->bestInliers[i]) inliers_out[P->kpIdx[i]] = 1;
            memcpy(Tcw, P->bestTcw, sizeof(float) * 16);
            return 1;
        }
    }
    return 0;
}

int ora_pnp_iterations(const ora_pnp* P) { return P->nIterations; }

int ora_pnp_events(const ora_pnp* P, int* out, int cap)
{
    const int n = P->ev_n < ORA_EV_CAP ? P->ev_n : ORA_EV_CAP;
    for (int i = 0; i < n && i < cap; i++) { out[2 * i] = P->ev[i][0]; out[2 * i + 1] = P->ev[i][1]; }
    return P->ev_n;
}
