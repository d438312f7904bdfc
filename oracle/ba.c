/*
 * ba.c -- TEST INFRASTRUCTURE ONLY (parity oracle).
 *
 * Restatement of ORB_SLAM2::Optimizer::LocalBundleAdjustment (reference
 * src/Optimizer.cc:453-778) and the g2o pieces it runs on:
 *   SE3Quat (Thirdparty/g2o/g2o/types/se3quat.h: ctor 58-60, operator* 92-98,
 *     map 217-220, exp 223-257, normalizeRotation 280-285) with Eigen 3
 *     Quaterniond semantics (from-matrix, toRotationMatrix, _transformVector,
 *     scalar quaternion product);
 *   EdgeSE3ProjectXYZ / EdgeStereoSE3ProjectXYZ (types_six_dof_expmap.h:80-141,
 *     .cpp:103-234; the stereo cam_project's float invz and float bf*invz);
 *   BaseBinaryEdge::constructQuadraticForm (base_binary_edge.hpp:55-120),
 *     BaseEdge::chi2 / robustInformation (base_edge.h:58-61, 96-102),
 *     RobustKernelHuber::robustify (robust_kernel_impl.cpp:78-91);
 *   BlockSolver<6,3> buildStructure/buildSystem/setLambda/solve
 *     (block_solver.hpp:142-604), SparseOptimizer active set / index map /
 *     update / push-pop (sparse_optimizer.cpp:61-114, 166-267, 354-435),
 *     OptimizationAlgorithmLevenberg::solve / computeLambdaInit / computeScale
 *     (optimization_algorithm_levenberg.cpp:59-189);
 *   Converter::toSE3Quat / toCvMat (Converter.cc:37-68).
 *
 * Choices where the reference's arithmetic is unpinned (Eigen):
 *   - every accumulation that g2o/Eigen performs as a running "+=" over edges,
 *     landmarks or vector entries is evaluated, by default, in the CANONICAL order
 *     below (ora_csum: 64-wide pairwise tree, recursively), identically on the GPU
 *     (bit-identical tests); ora_ba_set_order(ORA_BA_G2O) switches the oracle to the
 *     reference's own sequential order (g2o block_solver.hpp:353-560,
 *     sparse_optimizer.cpp:61-114), which the GPU is held to at 1e-5;
 *   - the pose system is factorised by a right-looking LDL^T on the upper
 *     triangle (SimplicialLDLT+AMD in the reference): in natural pose order
 *     below ORA_TILED_MIN_POSES free poses, above in the nested-dissection
 *     order of the pose graph (ordering.c); failure = an exactly zero pivot,
 *     like Eigen's LDLT;
 *   - sin/cos in SE3Quat::exp use ora_det_sincos (sim3.c); pow(theta,3) in
 *     exp and pow(2*rho-1,3) in the LM step are (a*a)*a;
 *   - small fixed-size products sum their terms left to right.
 * Map points are never isBad() inside the call (the adapter's view).
 */
#include "orb_oracle.h"
#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

/* ---- canonical reduction ---------------------------------------------- */
/* Sum of v[0..n) (destroys v): split into chunks of 64, reduce each chunk by
 * the tree a[i] += a[i+off] for off = 32,16,..,1 (zero padded), recurse on the
 * chunk sums.  This is exactly a wave64 shuffle-down reduction per level. */
double ora_csum(double* v, int n)
{
    if (n <= 0) return 0.0;
    while (n > 1) {
        int m = (n + 63) / 64;
        for (int c = 0; c < m; c++) {
            double a[64];
            for (int i = 0; i < 64; i++) a[i] = (c * 64 + i < n) ? v[c * 64 + i] : 0.0;
            for (int off = 32; off >= 1; off >>= 1)
                for (int i = 0; i < off; i++) a[i] += a[i + off];
            v[c] = a[0];
        }
        n = m;
    }
    return v[0];
}

/* Accumulation order of the BA / PoseOptimization restatement.
 *   ORA_BA_CANONICAL (default): every running sum in the canonical tree order above, which the
 *     GPU kernels also use -> bit-identical parity tests;
 *   ORA_BA_G2O: the reference's own order -- g2o accumulates each vertex's Hessian block and
 *     b as "+=" over its edges in active-edge (internalId) order (BlockSolver::buildSystem,
 *     block_solver.hpp:502-560, via BaseBinaryEdge::constructQuadraticForm), the Schur
 *     complement as Hpp - BDinv_1 B_1^T - BDinv_2 B_2^T - ... in landmark order and b_schur
 *     as b - (sum of B db in landmark order) (BlockSolver::solve, block_solver.hpp:353-430),
 *     and chi2 / computeScale as sequential sums (sparse_optimizer.cpp:61-114,
 *     optimization_algorithm_levenberg.cpp:182-189).  The GPU is held to this mode at the
 *     north star's 1e-5 tolerance (tests/test_gpu_ba_g2o_order.py). */
static int g_ba_order = ORA_BA_CANONICAL;
void ora_ba_set_order(int mode) { g_ba_order = mode; }
int ora_ba_get_order(void) { return g_ba_order; }

static double ba_sum(double* v, int n)
{
    if (g_ba_order == ORA_BA_CANONICAL) return ora_csum(v, n);
    double s = 0.0;
    for (int i = 0; i < n; i++) s += v[i];
    return s;
}

/* h - (v[0] + ... + v[n-1]) canonically, or ((h - v[0]) - v[1]) - ... (g2o's "-=" per term) */
static double ba_sub_terms(double h, double* v, int n)
{
    if (g_ba_order == ORA_BA_CANONICAL) return h - ora_csum(v, n);
    for (int i = 0; i < n; i++) h -= v[i];
    return h;
}

/* ---- SE3Quat ------------------------------------------------------------ */
typedef struct { double q[4]; double t[3]; } se3q; /* q = (x, y, z, w) like Eigen coeffs() */

static void quat_normalize(double* q)
{
    double z = ((q[0] * q[0] + q[1] * q[1]) + q[2] * q[2]) + q[3] * q[3];
    if (z > 0) {
        double n = sqrt(z);
        for (int i = 0; i < 4; i++) q[i] = q[i] / n;
    }
}

static void se3_normalize(se3q* T) /* normalizeRotation */
{
    if (T->q[3] < 0)
        for (int i = 0; i < 4; i++) T->q[i] *= -1;
    quat_normalize(T->q);
}

static void quat_from_R(const double* m, double* q) /* Quaterniond(const Matrix3d&) */
{
    double t = (m[0] + m[4]) + m[8];
    if (t > 0) {
        t = sqrt(t + 1.0);
        q[3] = 0.5 * t;
        t = 0.5 / t;
        q[0] = (m[7] - m[5]) * t;
        q[1] = (m[2] - m[6]) * t;
        q[2] = (m[3] - m[1]) * t;
    } else {
        int i = 0;
        if (m[4] > m[0]) i = 1;
        if (m[8] > m[i * 4]) i = 2;
        int j = (i + 1) % 3, k = (j + 1) % 3;
        t = sqrt(((m[i * 4] - m[j * 4]) - m[k * 4]) + 1.0);
        q[i] = 0.5 * t;
        t = 0.5 / t;
        q[3] = (m[k * 3 + j] - m[j * 3 + k]) * t;
        q[j] = (m[j * 3 + i] + m[i * 3 + j]) * t;
        q[k] = (m[k * 3 + i] + m[i * 3 + k]) * t;
    }
}

static void quat_to_R(const double* q, double* R) /* toRotationMatrix */
{
    const double x = q[0], y = q[1], z = q[2], w = q[3];
    const double tx = 2.0 * x, ty = 2.0 * y, tz = 2.0 * z;
    const double twx = tx * w, twy = ty * w, twz = tz * w;
    const double txx = tx * x, txy = ty * x, txz = tz * x;
    const double tyy = ty * y, tyz = tz * y, tzz = tz * z;
    R[0] = 1.0 - (tyy + tzz); R[1] = txy - twz;         R[2] = txz + twy;
    R[3] = txy + twz;         R[4] = 1.0 - (txx + tzz); R[5] = tyz - twx;
    R[6] = txz - twy;         R[7] = tyz + twx;         R[8] = 1.0 - (txx + tyy);
}

static void cross3(const double* a, const double* b, double* c)
{
    c[0] = a[1] * b[2] - a[2] * b[1];
    c[1] = a[2] * b[0] - a[0] * b[2];
    c[2] = a[0] * b[1] - a[1] * b[0];
}

static void quat_rotate(const double* q, const double* v, double* out) /* _transformVector */
{
    double uv[3], c[3];
    cross3(q, v, uv);
    for (int i = 0; i < 3; i++) uv[i] += uv[i];
    cross3(q, uv, c);
    for (int i = 0; i < 3; i++) out[i] = (v[i] + q[3] * uv[i]) + c[i];
}

static void quat_mul(const double* a, const double* b, double* o) /* quat_product (scalar path) */
{
    double r[4];
    r[3] = ((a[3] * b[3] - a[0] * b[0]) - a[1] * b[1]) - a[2] * b[2];
    r[0] = ((a[3] * b[0] + a[0] * b[3]) + a[1] * b[2]) - a[2] * b[1];
    r[1] = ((a[3] * b[1] + a[1] * b[3]) + a[2] * b[0]) - a[0] * b[2];
    r[2] = ((a[3] * b[2] + a[2] * b[3]) + a[0] * b[1]) - a[1] * b[0];
    memcpy(o, r, sizeof(r));
}

static void se3_map(const se3q* T, const double* X, double* out) /* map */
{
    double r[3];
    quat_rotate(T->q, X, r);
    for (int i = 0; i < 3; i++) out[i] = r[i] + T->t[i];
}

static void se3_mul(const se3q* a, const se3q* b, se3q* o) /* operator* */
{
    se3q r;
    double rt[3];
    quat_rotate(a->q, b->t, rt);
    for (int i = 0; i < 3; i++) r.t[i] = a->t[i] + rt[i];
    quat_mul(a->q, b->q, r.q);
    se3_normalize(&r);
    *o = r;
}

static void mat3_mul(const double* A, const double* B, double* C)
{
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++)
            C[i * 3 + j] = (A[i * 3] * B[j] + A[i * 3 + 1] * B[3 + j]) + A[i * 3 + 2] * B[6 + j];
}

static void se3_exp(const double* upd, se3q* out) /* SE3Quat::exp */
{
    const double* w = upd;
    const double* u = upd + 3;
    double theta = sqrt((w[0] * w[0] + w[1] * w[1]) + w[2] * w[2]);
    double Om[9] = {0, -w[2], w[1], w[2], 0, -w[0], -w[1], w[0], 0};
    double Om2[9], R[9], V[9];
    mat3_mul(Om, Om, Om2);
    if (theta < 0.00001) {
        for (int i = 0; i < 9; i++) R[i] = (((i % 4) == 0 ? 1.0 : 0.0) + Om[i]) + Om2[i];
        memcpy(V, R, sizeof(R));
    } else {
        double s, c;
        ora_det_sincos(theta, &s, &c);
        const double a = s / theta, b = (1 - c) / (theta * theta);
        const double cc = (theta - s) / ((theta * theta) * theta);
        for (int i = 0; i < 9; i++) {
            const double I = (i % 4) == 0 ? 1.0 : 0.0;
            R[i] = (I + a * Om[i]) + b * Om2[i];
            V[i] = (I + b * Om[i]) + cc * Om2[i];
        }
    }
    quat_from_R(R, out->q);
    for (int i = 0; i < 3; i++) out->t[i] = (V[i * 3] * u[0] + V[i * 3 + 1] * u[1]) + V[i * 3 + 2] * u[2];
    se3_normalize(out);
}

static void se3_from_Tcw(const float* T, se3q* o) /* Converter::toSE3Quat */
{
    double R[9];
    for (int r = 0; r < 3; r++)
        for (int c = 0; c < 3; c++) R[r * 3 + c] = (double)T[r * 4 + c];
    quat_from_R(R, o->q);
    for (int r = 0; r < 3; r++) o->t[r] = (double)T[r * 4 + 3];
    se3_normalize(o);
}

static void se3_to_Tcw(const se3q* s, float* T) /* Converter::toCvMat(SE3Quat) */
{
    double R[9];
    quat_to_R(s->q, R);
    for (int r = 0; r < 3; r++) {
        for (int c = 0; c < 3; c++) T[r * 4 + c] = (float)R[r * 3 + c];
        T[r * 4 + 3] = (float)s->t[r];
    }
    T[12] = T[13] = T[14] = 0.f;
    T[15] = 1.f;
}

/* ---- edges ---------------------------------------------------------------- */
typedef struct {
    int pt, kf, stereo;
    double obs[3], info, fx, fy, cx, cy, bf;
    double delta, dsqr;   /* Huber, delta = (double)(float)sqrt(th) */
    int robust, level;
    double err[3];        /* _error as last computed */
} ba_edge;

/* computeError: EdgeSE3ProjectXYZ (h:94-99) / EdgeStereoSE3ProjectXYZ (h:126-131) */
static void edge_error(ba_edge* e, const se3q* T, const double* X)
{
    double p[3];
    se3_map(T, X, p);
    if (!e->stereo) {
        const double px = p[0] / p[2], py = p[1] / p[2];
        e->err[0] = e->obs[0] - (px * e->fx + e->cx);
        e->err[1] = e->obs[1] - (py * e->fy + e->cy);
        e->err[2] = 0;
    } else {
        const float invz = (float)(1.0 / p[2]);
        const float bf = (float)e->bf;
        const double u = (p[0] * (double)invz) * e->fx + e->cx;
        const double v = (p[1] * (double)invz) * e->fy + e->cy;
        e->err[0] = e->obs[0] - u;
        e->err[1] = e->obs[1] - v;
        e->err[2] = e->obs[2] - (u - (double)(bf * invz));
    }
}

static double edge_chi2(const ba_edge* e)
{
    const int D = e->stereo ? 3 : 2;
    double s = 0;
    for (int j = 0; j < D; j++) s += e->err[j] * (e->info * e->err[j]);
    return s;
}

static void huber(const ba_edge* e, double chi, double* rho0, double* rho1)
{
    if (chi <= e->dsqr) {
        *rho0 = chi;
        *rho1 = 1.;
    } else {
        const double sq = sqrt(chi);
        *rho0 = (2 * sq) * e->delta - e->dsqr;
        *rho1 = e->delta / sq;
    }
}

static double edge_robust_chi2(const ba_edge* e)
{
    double c = edge_chi2(e), r0, r1;
    if (!e->robust) return c;
    huber(e, c, &r0, &r1);
    return r0;
}

static int edge_depth_positive(const ba_edge* e, const se3q* T, const double* X)
{
    double p[3];
    se3_map(T, X, p);
    return p[2] > 0.0;
}

/* linearizeOplus (.cpp:103-147 mono, 188-234 stereo): A = d e / d point (Dx3), B = d e / d pose (Dx6) */
static void edge_jacobians(const ba_edge* e, const se3q* T, const double* X, double* A, double* B)
{
    double p[3], R[9];
    se3_map(T, X, p);
    quat_to_R(T->q, R);
    const double x = p[0], y = p[1], z = p[2], z_2 = z * z;
    const double fx = e->fx, fy = e->fy;
    if (!e->stereo) {
        double tmp[6] = {fx, 0, ((-x) / z) * fx, 0, fy, ((-y) / z) * fy};
        const double s = -1. / z;
        double st[6];
        for (int i = 0; i < 6; i++) st[i] = s * tmp[i];
        for (int i = 0; i < 2; i++)
            for (int j = 0; j < 3; j++)
                A[i * 3 + j] = (st[i * 3] * R[j] + st[i * 3 + 1] * R[3 + j]) + st[i * 3 + 2] * R[6 + j];
    } else {
        const double bf = e->bf;
        for (int j = 0; j < 3; j++) {
            A[0 * 3 + j] = ((-fx) * R[0 * 3 + j]) / z + ((fx * x) * R[2 * 3 + j]) / z_2;
            A[1 * 3 + j] = ((-fy) * R[1 * 3 + j]) / z + ((fy * y) * R[2 * 3 + j]) / z_2;
            A[2 * 3 + j] = A[0 * 3 + j] - (bf * R[2 * 3 + j]) / z_2;
        }
    }
    B[0] = ((x * y) / z_2) * fx;
    B[1] = (-(1 + ((x * x) / z_2))) * fx;
    B[2] = (y / z) * fx;
    B[3] = (-1. / z) * fx;
    B[4] = 0;
    B[5] = (x / z_2) * fx;
    B[6] = (1 + ((y * y) / z_2)) * fy;
    B[7] = ((-x) * y / z_2) * fy;
    B[8] = ((-x) / z) * fy;
    B[9] = 0;
    B[10] = (-1. / z) * fy;
    B[11] = (y / z_2) * fy;
    if (e->stereo) {
        const double bf = e->bf;
        B[12] = B[0] - (bf * y) / z_2;
        B[13] = B[1] + (bf * x) / z_2;
        B[14] = B[2];
        B[15] = B[3];
        B[16] = 0;
        B[17] = B[5] - bf / z_2;
    }
}

/* per-edge quadratic-form terms (constructQuadraticForm), summed canonically by vertex */
typedef struct {
    double Hpp[21];  /* upper triangle r<=c of B^T W B, row-major packed */
    double bp[6];
    double Hpl[18];  /* 6x3 */
    double Hll[9];   /* full 3x3 */
    double bl[3];
} edge_terms;

static void edge_quadratic(const ba_edge* e, const double* A, const double* B, int poseFree, edge_terms* o)
{
    const int D = e->stereo ? 3 : 2;
    const double chi = edge_chi2(e);
    double rho1 = 1.0, r0;
    if (e->robust) huber(e, chi, &r0, &rho1);
    const double w = e->robust ? rho1 * e->info : e->info;
    double omr[3];
    for (int k = 0; k < D; k++) {
        omr[k] = -(e->info * e->err[k]);
        if (e->robust) omr[k] *= rho1;
    }
    /* point (from) */
    for (int r = 0; r < 3; r++) {
        double s = 0;
        for (int k = 0; k < D; k++) s += A[k * 3 + r] * omr[k];
        o->bl[r] = s;
        for (int c = 0; c < 3; c++) {
            double h = 0;
            for (int k = 0; k < D; k++) h += (A[k * 3 + r] * w) * A[k * 3 + c];
            o->Hll[r * 3 + c] = h;
        }
    }
    if (!poseFree) return;
    int idx = 0;
    for (int r = 0; r < 6; r++) {
        double s = 0;
        for (int k = 0; k < D; k++) s += B[k * 6 + r] * omr[k];
        o->bp[r] = s;
        for (int c = r; c < 6; c++) {
            double h = 0;
            for (int k = 0; k < D; k++) h += (B[k * 6 + r] * w) * B[k * 6 + c];
            o->Hpp[idx++] = h;
        }
        for (int c = 0; c < 3; c++) {
            double h = 0;
            if (e->robust)   /* B^T * weightedOmega * A */
                for (int k = 0; k < D; k++) h += (B[k * 6 + r] * w) * A[k * 3 + c];
            else             /* B^T * AtO^T */
                for (int k = 0; k < D; k++) h += B[k * 6 + r] * (A[k * 3 + c] * e->info);
            o->Hpl[r * 3 + c] = h;
        }
    }
}

/* Eigen 3x3 inverse (cofactors, InverseImpl.h compute_inverse_size3) */
static void inv3(const double* m, double* r)
{
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

/* Dense LDL^T on the upper triangle (row-major n x n, only r<=c read), in place.
 * Returns 0 on an exactly zero pivot. */
int ora_ldlt_solve(double* S, int n, const double* b, double* x)
{
    double* l = (double*)malloc(sizeof(double) * (n + 1));
    for (int k = 0; k < n; k++) {
        const double d = S[(size_t)k * n + k];
        if (d == 0.0) { free(l); return 0; }
        for (int i = k + 1; i < n; i++) l[i] = S[(size_t)k * n + i] / d;
        for (int i = k + 1; i < n; i++) {
            if (l[i] == 0.0) continue;   /* envelope skip: S[i][j] - 0*S[k][j] == S[i][j] (up to the sign of 0) */
            for (int j = i; j < n; j++) S[(size_t)i * n + j] -= l[i] * S[(size_t)k * n + j];
        }
        for (int i = k + 1; i < n; i++) S[(size_t)k * n + i] = l[i];   /* row k now holds L^T */
    }
    double* y = (double*)malloc(sizeof(double) * (n + 1));
    memcpy(y, b, sizeof(double) * n);
    for (int k = 0; k < n; k++)          /* L y = b (column sweep) */
        for (int i = k + 1; i < n; i++) y[i] -= S[(size_t)k * n + i] * y[k];
    for (int k = 0; k < n; k++) y[k] = y[k] / S[(size_t)k * n + k];
    for (int k = n - 1; k >= 0; k--)     /* L^T x = z (column sweep) */
        for (int i = 0; i < k; i++) y[i] -= S[(size_t)i * n + k] * y[k];
    memcpy(x, y, sizeof(double) * n);
    free(y);
    free(l);
    return 1;
}

/* The same solve on envelope (profile) storage of the upper triangle, for large pose systems
 * (a 16k-keyframe map has n = 96k: 74 GB dense).  Column c holds rows f[c]..c; f is the
 * nondecreasing hull of the first structurally nonzero row of each column, so the LDL^T fill
 * stays inside and row k reaches exactly the columns (k, last[k]].  Per element the operation
 * sequence is ora_ldlt_solve's: the entries it skips are the exact zeros outside the envelope,
 * which the dense version subtracts as 0 * S[k][j] (equal up to the sign of a zero). */
typedef struct { int n; int* f; int* last; size_t* cs; double* v; } env_mat;
#define ENV(E, r, c) ((E)->v[(E)->cs[c] + (size_t)((r) - (E)->f[c])])

/* f: first row per column (f[c] <= c), made monotone here; allocates the zeroed storage */
static int env_init(env_mat* E, int n, int* f)
{
    E->n = n;
    E->f = f;
    for (int c = n - 2; c >= 0; c--) if (f[c + 1] < f[c]) f[c] = f[c + 1];
    E->cs = (size_t*)malloc(sizeof(size_t) * (n + 1));
    E->last = (int*)malloc(sizeof(int) * (n + 1));
    size_t t = 0;
    for (int c = 0; c < n; c++) { E->cs[c] = t; t += (size_t)(c - f[c] + 1); }
    E->cs[n] = t;
    E->v = (double*)calloc(t + 1, sizeof(double));
    int j = 0;
    for (int k = 0; k < n; k++) {
        if (j < k) j = k;
        while (j + 1 < n && f[j + 1] <= k) j++;
        E->last[k] = j;
    }
    return E->v != NULL;
}

static void env_free(env_mat* E) { free(E->cs); free(E->last); free(E->v); }

static int ora_env_ldlt_solve(env_mat* E, const double* b, double* x)
{
    const int n = E->n;
    double* l = (double*)malloc(sizeof(double) * (n + 1));
    for (int k = 0; k < n; k++) {
        const double d = ENV(E, k, k);
        if (d == 0.0) { free(l); return 0; }
        const int hi = E->last[k];
        for (int i = k + 1; i <= hi; i++) l[i] = ENV(E, k, i) / d;
        for (int i = k + 1; i <= hi; i++) {
            if (l[i] == 0.0) continue;
            for (int j = i; j <= hi; j++) ENV(E, i, j) -= l[i] * ENV(E, k, j);
        }
        for (int i = k + 1; i <= hi; i++) ENV(E, k, i) = l[i];   /* row k now holds L^T */
    }
    double* y = (double*)malloc(sizeof(double) * (n + 1));
    memcpy(y, b, sizeof(double) * n);
    for (int k = 0; k < n; k++)          /* L y = b (column sweep) */
        for (int i = k + 1; i <= E->last[k]; i++) y[i] -= ENV(E, k, i) * y[k];
    for (int k = 0; k < n; k++) y[k] = y[k] / ENV(E, k, k);
    for (int k = n - 1; k >= 0; k--)     /* L^T x = z (column sweep) */
        for (int i = E->f[k]; i < k; i++) y[i] -= ENV(E, i, k) * y[k];
    memcpy(x, y, sizeof(double) * n);
    free(y);
    free(l);
    return 1;
}

/* ---- the optimizer -------------------------------------------------------- */
typedef struct {
    int nkf, npt, ne;
    se3q *T, *Tbak;
    double *X, *Xbak;
    int *kfFixed, *kfId, *ptId;
    ba_edge* E;
    /* active structure */
    int nE, nP, nL;          /* active edges, free poses, active points */
    int *aE;                 /* active edge list (edge order) */
    int *poseIdx, *ptIdx;    /* kf -> pose index or -1; pt -> landmark index or -1 */
    int *poseOf, *ptOf;      /* pose index -> kf; landmark -> pt */
    int *peStart, *peList;   /* per pose: active edges (edge order) */
    int *leStart, *leList;   /* per landmark: active edges (edge order) */
    /* system */
    edge_terms* terms;       /* per active edge */
    double *Hpp, *bp, *Hll, *bl;   /* Hpp 21 per pose, Hll 9 per landmark */
    double *x, *b;           /* vector: poses (6 nP) then landmarks (3 nL) */
    double lambda, ni;
    int nBad;
    double* scratch;
    int scratchN;
    ora_ba_trace* trace;
} ba_ctx;

static double* scratch(ba_ctx* c, int n)
{
    if (n > c->scratchN) {
        free(c->scratch);
        c->scratch = (double*)malloc(sizeof(double) * (n + 64));
        c->scratchN = n;
    }
    return c->scratch;
}

static const int* g_keys;
static int cmp_idx(const void* a, const void* b)
{
    int ka = g_keys[*(const int*)a], kb = g_keys[*(const int*)b];
    return ka < kb ? -1 : ka > kb;
}

/* initializeOptimization(level) + buildIndexMapping + BlockSolver::buildStructure */
static void build_structure(ba_ctx* c, int level)
{
    int* kfAct = (int*)calloc(c->nkf, sizeof(int));
    int* ptAct = (int*)calloc(c->npt, sizeof(int));
    c->nE = 0;
    for (int i = 0; i < c->ne; i++)
        if (c->E[i].level == level) {   /* allVerticesFixed never holds: points are free */
            c->aE[c->nE++] = i;
            kfAct[c->E[i].kf] = 1;
            ptAct[c->E[i].pt] = 1;
        }
    /* poses: active, not fixed, sorted by id; landmarks: active, sorted by id */
    int* ord = (int*)malloc(sizeof(int) * (c->nkf + c->npt + 1));
    int n = 0;
    for (int k = 0; k < c->nkf; k++)
        if (kfAct[k] && !c->kfFixed[k]) ord[n++] = k;
    g_keys = c->kfId;
    qsort(ord, n, sizeof(int), cmp_idx);
    c->nP = n;
    for (int k = 0; k < c->nkf; k++) c->poseIdx[k] = -1;
    for (int i = 0; i < n; i++) { c->poseOf[i] = ord[i]; c->poseIdx[ord[i]] = i; }
    n = 0;
    for (int p = 0; p < c->npt; p++)
        if (ptAct[p]) ord[n++] = p;
    g_keys = c->ptId;
    qsort(ord, n, sizeof(int), cmp_idx);
    c->nL = n;
    for (int p = 0; p < c->npt; p++) c->ptIdx[p] = -1;
    for (int i = 0; i < n; i++) { c->ptOf[i] = ord[i]; c->ptIdx[ord[i]] = i; }
    free(ord);
    /* CSR edge lists in active-edge order */
    memset(c->peStart, 0, sizeof(int) * (c->nP + 1));
    memset(c->leStart, 0, sizeof(int) * (c->nL + 1));
    for (int a = 0; a < c->nE; a++) {
        const ba_edge* e = &c->E[c->aE[a]];
        if (c->poseIdx[e->kf] >= 0) c->peStart[c->poseIdx[e->kf] + 1]++;
        c->leStart[c->ptIdx[e->pt] + 1]++;
    }
    for (int i = 0; i < c->nP; i++) c->peStart[i + 1] += c->peStart[i];
    for (int i = 0; i < c->nL; i++) c->leStart[i + 1] += c->leStart[i];
    int* fp = (int*)malloc(sizeof(int) * (c->nP + 1));
    int* fl = (int*)malloc(sizeof(int) * (c->nL + 1));
    memcpy(fp, c->peStart, sizeof(int) * (c->nP + 1));
    memcpy(fl, c->leStart, sizeof(int) * (c->nL + 1));
    for (int a = 0; a < c->nE; a++) {
        const ba_edge* e = &c->E[c->aE[a]];
        if (c->poseIdx[e->kf] >= 0) c->peList[fp[c->poseIdx[e->kf]]++] = a;
        c->leList[fl[c->ptIdx[e->pt]]++] = a;
    }
    free(fp);
    free(fl);
    free(kfAct);
    free(ptAct);
    memset(c->x, 0, sizeof(double) * (6 * c->nP + 3 * c->nL + 1));
}

static void compute_active_errors(ba_ctx* c)
{
    for (int a = 0; a < c->nE; a++) {
        ba_edge* e = &c->E[c->aE[a]];
        edge_error(e, &c->T[e->kf], &c->X[3 * e->pt]);
    }
}

static double active_robust_chi2(ba_ctx* c)
{
    double* v = scratch(c, c->nE);
    for (int a = 0; a < c->nE; a++) v[a] = edge_robust_chi2(&c->E[c->aE[a]]);
    return ba_sum(v, c->nE);
}

/* BlockSolver::buildSystem */
static void build_system(ba_ctx* c)
{
    for (int a = 0; a < c->nE; a++) {
        const ba_edge* e = &c->E[c->aE[a]];
        double A[9], B[18];
        edge_jacobians(e, &c->T[e->kf], &c->X[3 * e->pt], A, B);
        edge_quadratic(e, A, B, c->poseIdx[e->kf] >= 0, &c->terms[a]);
    }
    int maxn = 1;
    for (int i = 0; i < c->nP; i++) if (c->peStart[i + 1] - c->peStart[i] > maxn) maxn = c->peStart[i + 1] - c->peStart[i];
    double* v = scratch(c, maxn);
    for (int i = 0; i < c->nP; i++) {
        const int s = c->peStart[i], n = c->peStart[i + 1] - s;
        for (int q = 0; q < 21; q++) {
            for (int j = 0; j < n; j++) v[j] = c->terms[c->peList[s + j]].Hpp[q];
            c->Hpp[21 * i + q] = ba_sum(v, n);
        }
        for (int q = 0; q < 6; q++) {
            for (int j = 0; j < n; j++) v[j] = c->terms[c->peList[s + j]].bp[q];
            c->bp[6 * i + q] = ba_sum(v, n);
        }
    }
    for (int i = 0; i < c->nL; i++) {
        const int s = c->leStart[i], n = c->leStart[i + 1] - s;
        double w[64];
        double* vv = n <= 64 ? w : scratch(c, n);
        for (int q = 0; q < 9; q++) {
            for (int j = 0; j < n; j++) vv[j] = c->terms[c->leList[s + j]].Hll[q];
            c->Hll[9 * i + q] = ba_sum(vv, n);
        }
        for (int q = 0; q < 3; q++) {
            for (int j = 0; j < n; j++) vv[j] = c->terms[c->leList[s + j]].bl[q];
            c->bl[3 * i + q] = ba_sum(vv, n);
        }
    }
    for (int i = 0; i < c->nP; i++)
        for (int q = 0; q < 6; q++) c->b[6 * i + q] = c->bp[6 * i + q];
    for (int i = 0; i < c->nL; i++)
        for (int q = 0; q < 3; q++) c->b[6 * c->nP + 3 * i + q] = c->bl[3 * i + q];
}

static const int DIAG21[6] = {0, 6, 11, 15, 18, 20};

static double lambda_init(ba_ctx* c)
{
    double m = 0.;
    for (int i = 0; i < c->nP; i++)
        for (int j = 0; j < 6; j++) m = fmax(fabs(c->Hpp[21 * i + DIAG21[j]]), m);
    for (int i = 0; i < c->nL; i++)
        for (int j = 0; j < 3; j++) m = fmax(fabs(c->Hll[9 * i + 4 * j]), m);
    return 1e-5 * m;
}

/* BlockSolver::solve with lambda on the diagonals (setLambda .. restoreDiagonal) */
static int schur_solve(ba_ctx* c, double lambda)
{
    const int nP = c->nP, nL = c->nL, n = 6 * nP;
    double* Dinv = (double*)malloc(sizeof(double) * 9 * (nL + 1));
    double* db = (double*)malloc(sizeof(double) * 3 * (nL + 1));
    /* per active edge with a free pose: BDinv (6x3) and B*db (6) */
    double* E = (double*)malloc(sizeof(double) * 18 * (c->nE + 1));
    double* cb = (double*)malloc(sizeof(double) * 6 * (c->nE + 1));
    for (int l = 0; l < nL; l++) {
        double D[9];
        memcpy(D, &c->Hll[9 * l], sizeof(D));
        for (int j = 0; j < 3; j++) D[4 * j] += lambda;
        inv3(D, &Dinv[9 * l]);
        const double* Di = &Dinv[9 * l];
        const double* bl = &c->bl[3 * l];
        for (int r = 0; r < 3; r++) db[3 * l + r] = (Di[r * 3] * bl[0] + Di[r * 3 + 1] * bl[1]) + Di[r * 3 + 2] * bl[2];
        for (int j = c->leStart[l]; j < c->leStart[l + 1]; j++) {
            const int a = c->leList[j];
            if (c->poseIdx[c->E[c->aE[a]].kf] < 0) continue;
            const double* Bi = c->terms[a].Hpl;
            for (int r = 0; r < 6; r++) {
                for (int k = 0; k < 3; k++)
                    E[18 * a + r * 3 + k] = (Bi[r * 3] * Di[k] + Bi[r * 3 + 1] * Di[3 + k]) + Bi[r * 3 + 2] * Di[6 + k];
                cb[6 * a + r] = (Bi[r * 3] * db[3 * l] + Bi[r * 3 + 1] * db[3 * l + 1]) + Bi[r * 3 + 2] * db[3 * l + 2];
            }
        }
    }
    /* S (upper) and b_schur: terms in landmark order.  Per landmark its pose edges sorted by
     * pose (g2o's per-landmark block list); Schur block (i1 <= i2) -> its (a1, a2) pairs in
     * landmark order, so the cost is sum_l k_l^2 like the reference's BlockSolver::solve. */
    double* bs = (double*)malloc(sizeof(double) * (n + 1));
    int* lpStart = (int*)calloc(nL + 2, sizeof(int));
    int* lpList = (int*)malloc(sizeof(int) * (c->nE + 1));
    for (int l = 0; l < nL; l++) {
        lpStart[l + 1] = lpStart[l];
        for (int j = c->leStart[l]; j < c->leStart[l + 1]; j++) {
            const int a = c->leList[j];
            const int pi = c->poseIdx[c->E[c->aE[a]].kf];
            if (pi < 0) continue;
            int q = lpStart[l + 1]++;   /* insertion sort by pose index (k_l is small) */
            while (q > lpStart[l] && c->poseIdx[c->E[c->aE[lpList[q - 1]]].kf] > pi) {
                lpList[q] = lpList[q - 1];
                q--;
            }
            lpList[q] = a;
        }
    }
#define POSE_OF(a) (c->poseIdx[c->E[c->aE[(a)]].kf])
    int* blkOf = (int*)malloc(sizeof(int) * ((size_t)nP * nP + 1));
    for (size_t q = 0; q < (size_t)nP * nP; q++) blkOf[q] = -1;
    int nBlk = 0;
    for (int l = 0; l < nL; l++)
        for (int u = lpStart[l]; u < lpStart[l + 1]; u++)
            for (int w = u; w < lpStart[l + 1]; w++) {
                int* bo = &blkOf[(size_t)POSE_OF(lpList[u]) * nP + POSE_OF(lpList[w])];
                if (*bo < 0) *bo = nBlk++;
            }
    int* bStart = (int*)calloc(nBlk + 2, sizeof(int));
    for (int l = 0; l < nL; l++)
        for (int u = lpStart[l]; u < lpStart[l + 1]; u++)
            for (int w = u; w < lpStart[l + 1]; w++)
                bStart[blkOf[(size_t)POSE_OF(lpList[u]) * nP + POSE_OF(lpList[w])] + 1]++;
    for (int q = 0; q < nBlk; q++) bStart[q + 1] += bStart[q];
    const int nPair = bStart[nBlk];
    int* pA = (int*)malloc(sizeof(int) * (nPair + 1));
    int* pB = (int*)malloc(sizeof(int) * (nPair + 1));
    int* fill = (int*)malloc(sizeof(int) * (nBlk + 1));
    memcpy(fill, bStart, sizeof(int) * (nBlk + 1));
    for (int l = 0; l < nL; l++)
        for (int u = lpStart[l]; u < lpStart[l + 1]; u++)
            for (int w = u; w < lpStart[l + 1]; w++) {
                const int q = fill[blkOf[(size_t)POSE_OF(lpList[u]) * nP + POSE_OF(lpList[w])]]++;
                pA[q] = lpList[u];
                pB[q] = lpList[w];
            }
    /* Storage of S.  nP < ORA_TILED_MIN_POSES: natural order in an envelope (the GPU's dense
     * single-workgroup solvers); otherwise the nested-dissection order of the pose graph and
     * the block-sparse factor (ordering.c; the GPU's tiled solver) */
    const int use_nd = nP >= ORA_TILED_MIN_POSES;
    int* fcol = NULL;
    env_mat Env;
    memset(&Env, 0, sizeof(Env));
    ora_sp* SP = NULL;
    if (use_nd) {
        int* as = (int*)calloc(nP + 1, sizeof(int));
        for (int i1 = 0; i1 < nP; i1++)
            for (int i2 = i1 + 1; i2 < nP; i2++)
                if (blkOf[(size_t)i1 * nP + i2] >= 0) { as[i1 + 1]++; as[i2 + 1]++; }
        for (int i = 0; i < nP; i++) as[i + 1] += as[i];
        int* adj = (int*)malloc(sizeof(int) * (as[nP] + 1));
        int* f = (int*)malloc(sizeof(int) * (nP + 1));
        memcpy(f, as, sizeof(int) * nP);
        for (int i1 = 0; i1 < nP; i1++)   /* lists sorted: i1 ascending, then i2 ascending */
            for (int i2 = 0; i2 < nP; i2++)
                if (i1 != i2 && blkOf[(size_t)(i1 < i2 ? i1 : i2) * nP + (i1 < i2 ? i2 : i1)] >= 0) adj[f[i1]++] = i2;
        int* perm = (int*)malloc(sizeof(int) * (nP + 1));
        ora_nd_order(nP, as, adj, ORA_ND_LEAF, perm);
        SP = ora_sp_create(n, 6, as, adj, perm);
        free(perm); free(f); free(adj); free(as);
    } else {
        /* the envelope of S: per column the first row any Schur block (or the diagonal) reaches */
        fcol = (int*)malloc(sizeof(int) * (n + 1));
        for (int c = 0; c < n; c++) fcol[c] = 6 * (c / 6);
        for (int l = 0; l < nL; l++)
            for (int u = lpStart[l]; u < lpStart[l + 1]; u++)
                for (int w = u; w < lpStart[l + 1]; w++) {
                    const int i1 = POSE_OF(lpList[u]), i2 = POSE_OF(lpList[w]);
                    for (int cc = 0; cc < 6; cc++)
                        if (6 * i1 < fcol[6 * i2 + cc]) fcol[6 * i2 + cc] = 6 * i1;
                }
        env_init(&Env, n, fcol);
    }
    int maxM = 1;
    for (int q = 0; q < nBlk; q++) if (bStart[q + 1] - bStart[q] > maxM) maxM = bStart[q + 1] - bStart[q];
    double* v = (double*)malloc(sizeof(double) * (maxM + nL + 1));
    for (int i1 = 0; i1 < nP; i1++)
        for (int i2 = i1; i2 < nP; i2++) {
            const int bq = blkOf[(size_t)i1 * nP + i2];
            const int s0 = bq < 0 ? 0 : bStart[bq], m = bq < 0 ? 0 : bStart[bq + 1] - s0;
            if (bq < 0 && i1 != i2) continue;   /* structurally zero block (calloc) */
            for (int r = 0; r < 6; r++)
                for (int cc = (i1 == i2 ? r : 0); cc < 6; cc++) {
                    for (int t = 0; t < m; t++) {
                        const double* Ei = &E[18 * pA[s0 + t] + r * 3];
                        const double* Bj = &c->terms[pB[s0 + t]].Hpl[cc * 3];
                        v[t] = (Ei[0] * Bj[0] + Ei[1] * Bj[1]) + Ei[2] * Bj[2];
                    }
                    double h = 0;
                    if (i1 == i2) {
                        h = c->Hpp[21 * i1 + DIAG21[r] + (cc - r)];
                        if (cc == r) h += lambda;
                    }
                    const double val = ba_sub_terms(h, v, m);
                    if (use_nd) *ora_sp_at(SP, 6 * i1 + r, 6 * i2 + cc) = val;
                    else ENV(&Env, 6 * i1 + r, 6 * i2 + cc) = val;
                }
        }
    /* b_schur: per pose, its landmarks' terms in landmark order */
    {
        int* psStart = (int*)calloc(nP + 2, sizeof(int));
        int* psList = (int*)malloc(sizeof(int) * (c->nE + 1));
        for (int l = 0; l < nL; l++)
            for (int u = lpStart[l]; u < lpStart[l + 1]; u++) psStart[POSE_OF(lpList[u]) + 1]++;
        for (int i = 0; i < nP; i++) psStart[i + 1] += psStart[i];
        int* pf = (int*)malloc(sizeof(int) * (nP + 1));
        memcpy(pf, psStart, sizeof(int) * (nP + 1));
        for (int l = 0; l < nL; l++)
            for (int u = lpStart[l]; u < lpStart[l + 1]; u++) psList[pf[POSE_OF(lpList[u])]++] = lpList[u];
        for (int i = 0; i < nP; i++)
            for (int r = 0; r < 6; r++) {
                const int m = psStart[i + 1] - psStart[i];
                for (int t = 0; t < m; t++) v[t] = cb[6 * psList[psStart[i] + t] + r];
                bs[6 * i + r] = c->bp[6 * i + r] - ba_sum(v, m);
            }
        free(psStart); free(psList); free(pf);
    }
    double* xp = (double*)malloc(sizeof(double) * (n + 1));
    int ok = n == 0 ? 1 : (use_nd ? ora_sp_solve(SP, bs, xp) : ora_env_ldlt_solve(&Env, bs, xp));
    if (ok) {
        memcpy(c->x, xp, sizeof(double) * n);
        /* xl = Dinv (bl - sum_i B_i^T xp_i); rightMultiply over the landmark's blocks in pose order */
        for (int l = 0; l < nL; l++) {
            double cl[3] = {c->bl[3 * l], c->bl[3 * l + 1], c->bl[3 * l + 2]};
            for (int u = lpStart[l]; u < lpStart[l + 1]; u++) {
                const int a = lpList[u];
                const double* B = c->terms[a].Hpl;
                const double* cp = &xp[6 * POSE_OF(a)];
                for (int k = 0; k < 3; k++) {
                    double s = 0;
                    for (int r = 0; r < 6; r++) s += B[r * 3 + k] * (-cp[r]);
                    cl[k] += s;
                }
            }
            const double* Di = &Dinv[9 * l];
            for (int r = 0; r < 3; r++)
                c->x[6 * nP + 3 * l + r] = (Di[r * 3] * cl[0] + Di[r * 3 + 1] * cl[1]) + Di[r * 3 + 2] * cl[2];
        }
    }
#undef POSE_OF
    free(lpStart); free(lpList); free(blkOf); free(bStart); free(pA); free(pB); free(fill);
    if (use_nd) ora_sp_free(SP);
    else { env_free(&Env); free(fcol); }
    free(xp); free(v); free(bs); free(E); free(cb); free(Dinv); free(db);
    return ok;
}

static void push_state(ba_ctx* c)
{
    memcpy(c->Tbak, c->T, sizeof(se3q) * c->nkf);
    memcpy(c->Xbak, c->X, sizeof(double) * 3 * c->npt);
}

static void pop_state(ba_ctx* c)
{
    memcpy(c->T, c->Tbak, sizeof(se3q) * c->nkf);
    memcpy(c->X, c->Xbak, sizeof(double) * 3 * c->npt);
}

static void apply_update(ba_ctx* c) /* SparseOptimizer::update in _ivMap order */
{
    for (int i = 0; i < c->nP; i++) {
        se3q d, r;
        se3_exp(&c->x[6 * i], &d);
        se3_mul(&d, &c->T[c->poseOf[i]], &r);
        c->T[c->poseOf[i]] = r;
    }
    for (int l = 0; l < c->nL; l++)
        for (int k = 0; k < 3; k++) c->X[3 * c->ptOf[l] + k] += c->x[6 * c->nP + 3 * l + k];
}

static double compute_scale(ba_ctx* c)
{
    const int n = 6 * c->nP + 3 * c->nL;
    double* v = scratch(c, n);
    for (int j = 0; j < n; j++) v[j] = c->x[j] * (c->lambda * c->x[j] + c->b[j]);
    return ba_sum(v, n);
}

static int stop_set(const volatile int* stop) { return stop && *stop; }

enum { SOLVE_OK = 0, SOLVE_TERMINATE = 1 };

/* OptimizationAlgorithmLevenberg::solve */
static int lm_solve(ba_ctx* c, int iteration, const volatile int* stop)
{
    compute_active_errors(c);
    double currentChi = active_robust_chi2(c);
    const double iniChi = currentChi;
    build_system(c);
    if (iteration == 0) {
        c->lambda = lambda_init(c);
        c->ni = 2;
        c->nBad = 0;
    }
    double rho = 0;
    int qmax = 0;
    do {
        push_state(c);
        const int ok2 = schur_solve(c, c->lambda);
        apply_update(c);
        compute_active_errors(c);
        double tempChi = active_robust_chi2(c);
        if (!ok2) tempChi = DBL_MAX;
        rho = currentChi - tempChi;
        double scale = compute_scale(c);
        scale += 1e-3;
        rho /= scale;
        if (rho > 0 && isfinite(tempChi)) {
            const double a3 = 2 * rho - 1;
            double alpha = 1. - (a3 * a3) * a3;
            alpha = fmin(alpha, 2. / 3.);
            const double scaleFactor = fmax(1. / 3., alpha);
            c->lambda *= scaleFactor;
            c->ni = 2;
            currentChi = tempChi;
        } else {
            c->lambda *= c->ni;
            c->ni *= 2;
            pop_state(c);
        }
        qmax++;
        if (c->trace && c->trace->n_trials < ORA_BA_TRACE_MAX) {
            ora_ba_trace* t = c->trace;
            t->trial_chi2[t->n_trials] = tempChi;
            t->trial_lambda[t->n_trials] = c->lambda;
            t->n_trials++;
        }
    } while (rho < 0 && qmax < 10 && !stop_set(stop));
    if (c->trace && c->trace->n_solves < ORA_BA_TRACE_MAX) {
        c->trace->solve_ini_chi2[c->trace->n_solves] = iniChi;
        c->trace->solve_chi2[c->trace->n_solves] = currentChi;
        c->trace->n_solves++;
    }
    if (qmax == 10 || rho == 0) return SOLVE_TERMINATE;
    if ((iniChi - currentChi) * 1e3 < iniChi) c->nBad++;
    else c->nBad = 0;
    if (c->nBad >= 3) return SOLVE_TERMINATE;
    return SOLVE_OK;
}

/* SparseOptimizer::optimize(iterations) */
static int optimize(ba_ctx* c, int iterations, const volatile int* stop)
{
    int it = 0, ok = 1;
    for (int i = 0; i < iterations && !stop_set(stop) && ok; i++) {
        ok = lm_solve(c, i, stop) == SOLVE_OK;
        it++;
    }
    return it;
}

/* global = 0: Optimizer::LocalBundleAdjustment (Optimizer.cc:453-778);
 * global = 1: Optimizer::BundleAdjustment (Optimizer.cc:49-237) with nIterations / bRobust. */
static int ba_run(const ora_ba_problem* P, int global, int nIterations, int bRobust, const volatile int* stop,
                  ora_ba_result* R, ora_ba_trace* trace)
{
    ba_ctx C;
    memset(&C, 0, sizeof(C));
    ba_ctx* c = &C;
    c->nkf = P->n_kf; c->npt = P->n_pt; c->ne = P->n_edge;
    c->trace = trace;
    if (trace) memset(trace, 0, sizeof(*trace));
    c->T = (se3q*)malloc(sizeof(se3q) * (c->nkf + 1));
    c->Tbak = (se3q*)malloc(sizeof(se3q) * (c->nkf + 1));
    c->X = (double*)malloc(sizeof(double) * 3 * (c->npt + 1));
    c->Xbak = (double*)malloc(sizeof(double) * 3 * (c->npt + 1));
    c->kfFixed = (int*)malloc(sizeof(int) * (c->nkf + 1));
    c->kfId = (int*)malloc(sizeof(int) * (c->nkf + 1));
    c->ptId = (int*)malloc(sizeof(int) * (c->npt + 1));
    c->E = (ba_edge*)calloc(c->ne + 1, sizeof(ba_edge));
    c->aE = (int*)malloc(sizeof(int) * (c->ne + 1));
    c->poseIdx = (int*)malloc(sizeof(int) * (c->nkf + 1));
    c->poseOf = (int*)malloc(sizeof(int) * (c->nkf + 1));
    c->ptIdx = (int*)malloc(sizeof(int) * (c->npt + 1));
    c->ptOf = (int*)malloc(sizeof(int) * (c->npt + 1));
    c->peStart = (int*)malloc(sizeof(int) * (c->nkf + 2));
    c->leStart = (int*)malloc(sizeof(int) * (c->npt + 2));
    c->peList = (int*)malloc(sizeof(int) * (c->ne + 1));
    c->leList = (int*)malloc(sizeof(int) * (c->ne + 1));
    c->terms = (edge_terms*)calloc(c->ne + 1, sizeof(edge_terms));
    c->Hpp = (double*)malloc(sizeof(double) * 21 * (c->nkf + 1));
    c->bp = (double*)malloc(sizeof(double) * 6 * (c->nkf + 1));
    c->Hll = (double*)malloc(sizeof(double) * 9 * (c->npt + 1));
    c->bl = (double*)malloc(sizeof(double) * 3 * (c->npt + 1));
    c->x = (double*)calloc(6 * c->nkf + 3 * c->npt + 1, sizeof(double));
    c->b = (double*)calloc(6 * c->nkf + 3 * c->npt + 1, sizeof(double));

    for (int k = 0; k < c->nkf; k++) {
        se3_from_Tcw(&P->kf_Tcw[16 * k], &c->T[k]);
        c->kfId[k] = P->kf_id[k];
        c->kfFixed[k] = (!global && !P->kf_local[k]) || P->kf_id[k] == 0;   /* Optimizer.cc:79 / 524, 547 */
    }
    for (int p = 0; p < c->npt; p++) {
        c->ptId[p] = P->pt_id[p];
        for (int j = 0; j < 3; j++) c->X[3 * p + j] = (double)P->pt_pos[3 * p + j];
    }
    /* Huber deltas: sqrt(5.991) in LocalBundleAdjustment (585), sqrt(5.99) in BundleAdjustment (87) */
    const float thMono = (float)sqrt(global ? 5.99 : 5.991), thStereo = (float)sqrt(7.815);
    for (int i = 0; i < c->ne; i++) {
        ba_edge* e = &c->E[i];
        e->pt = P->edge_pt[i];
        e->kf = P->edge_kf[i];
        e->stereo = !(P->edge_obs[3 * i + 2] < 0);
        for (int j = 0; j < 3; j++) e->obs[j] = (double)P->edge_obs[3 * i + j];
        e->info = (double)P->edge_inv_sigma2[i];
        const float* cam = &P->kf_cam[5 * e->kf];
        e->fx = cam[0]; e->fy = cam[1]; e->cx = cam[2]; e->cy = cam[3]; e->bf = cam[4];
        e->delta = (double)(e->stereo ? thStereo : thMono);
        e->dsqr = e->delta * e->delta;
        e->robust = global ? (bRobust != 0) : 1;
        e->level = 0;
    }
    /* outputs default to the inputs (early abort writes nothing back) */
    memcpy(R->kf_Tcw, P->kf_Tcw, sizeof(float) * 16 * c->nkf);
    memcpy(R->pt_pos, P->pt_pos, sizeof(float) * 3 * c->npt);
    memset(R->edge_erase, 0, c->ne);
    R->aborted = 0;
    R->iterations[0] = R->iterations[1] = 0;
    R->n_erased = 0;
    if (stop_set(stop) || c->ne == 0) {
        R->aborted = 1;
        goto done;
    }

    build_structure(c, 0);
    if (global) {   /* initializeOptimization(); optimize(nIterations); no gating (Optimizer.cc:190-191) */
        if (c->nP + c->nL > 0) R->iterations[0] = optimize(c, nIterations, stop);
        for (int k = 0; k < c->nkf; k++) se3_to_Tcw(&c->T[k], &R->kf_Tcw[16 * k]);
        for (int p = 0; p < c->npt; p++)
            if (c->ptIdx[p] >= 0)   /* vbNotIncludedMP points keep their position (217-219) */
                for (int j = 0; j < 3; j++) R->pt_pos[3 * p + j] = (float)c->X[3 * p + j];
        goto done;
    }
    if (c->nP + c->nL > 0) R->iterations[0] = optimize(c, 5, stop);
    if (!stop_set(stop)) {
        for (int i = 0; i < c->ne; i++) {   /* Optimizer.cc:674-706 */
            ba_edge* e = &c->E[i];
            const double th = e->stereo ? 7.815 : 5.991;
            if (edge_chi2(e) > th || !edge_depth_positive(e, &c->T[e->kf], &c->X[3 * e->pt])) e->level = 1;
            e->robust = 0;
        }
        build_structure(c, 0);
        if (c->nE > 0 && c->nP + c->nL > 0) R->iterations[1] = optimize(c, 10, stop);
    }
    for (int i = 0; i < c->ne; i++) {       /* Optimizer.cc:714-746 */
        const ba_edge* e = &c->E[i];
        const double th = e->stereo ? 7.815 : 5.991;
        if (edge_chi2(e) > th || !edge_depth_positive(e, &c->T[e->kf], &c->X[3 * e->pt])) {
            R->edge_erase[i] = 1;
            R->n_erased++;
        }
    }
    for (int k = 0; k < c->nkf; k++)
        if (P->kf_local[k]) se3_to_Tcw(&c->T[k], &R->kf_Tcw[16 * k]);
    for (int p = 0; p < c->npt; p++)
        for (int j = 0; j < 3; j++) R->pt_pos[3 * p + j] = (float)c->X[3 * p + j];
done:
    free(c->T); free(c->Tbak); free(c->X); free(c->Xbak); free(c->kfFixed); free(c->kfId); free(c->ptId);
    free(c->E); free(c->aE); free(c->poseIdx); free(c->poseOf); free(c->ptIdx); free(c->ptOf);
    free(c->peStart); free(c->leStart); free(c->peList); free(c->leList); free(c->terms);
    free(c->Hpp); free(c->bp); free(c->Hll); free(c->bl); free(c->x); free(c->b); free(c->scratch);
    return 0;
}

int ora_local_ba(const ora_ba_problem* P, const volatile int* stop, ora_ba_result* R, ora_ba_trace* trace)
{
    return ba_run(P, 0, 0, 1, stop, R, trace);
}

int ora_global_ba(const ora_ba_problem* P, int nIterations, int bRobust, const volatile int* stop, ora_ba_result* R,
                  ora_ba_trace* trace)
{
    return ba_run(P, 1, nIterations, bRobust, stop, R, trace);
}


/* ======================================================================
 * Optimizer::PoseOptimization (Optimizer.cc:239-451): one SE3 vertex, unary
 * EdgeSE3ProjectXYZOnlyPose / EdgeStereoSE3ProjectXYZOnlyPose edges
 * (types_six_dof_expmap.cpp:266-364), LinearSolverDense (Eigen LDLT with
 * diagonal pivoting, linear_solver_dense.h:65-113), 4 rounds of optimize(10)
 * each restarted from pFrame->mTcw, outlier classification after every round.
 * ====================================================================== */
typedef struct {
    double Xw[3], obs[3], info, delta, dsqr, err[3];
    int stereo, level, robust, kp;
} pose_edge;

static void pose_edge_error(pose_edge* e, const se3q* T, const ora_pose_problem* P)
{
    double p[3];
    se3_map(T, e->Xw, p);
    const double fx = P->fx, fy = P->fy, cx = P->cx, cy = P->cy;
    if (!e->stereo) {
        const double px = p[0] / p[2], py = p[1] / p[2];
        e->err[0] = e->obs[0] - (px * fx + cx);
        e->err[1] = e->obs[1] - (py * fy + cy);
        e->err[2] = 0;
    } else {
        const float invz = (float)(1.0 / p[2]);
        const double u = (p[0] * (double)invz) * fx + cx;
        const double v = (p[1] * (double)invz) * fy + cy;
        e->err[0] = e->obs[0] - u;
        e->err[1] = e->obs[1] - v;
        e->err[2] = e->obs[2] - (u - (double)P->bf * (double)invz);
    }
}

static double pose_edge_chi2(const pose_edge* e)
{
    const int D = e->stereo ? 3 : 2;
    double s = 0;
    for (int j = 0; j < D; j++) s += e->err[j] * (e->info * e->err[j]);
    return s;
}

/* Jacobian d e / d pose (D x 6), linearizeOplus of the OnlyPose edges */
static void pose_edge_jacobian(const pose_edge* e, const se3q* T, const ora_pose_problem* P, double* J)
{
    double p[3];
    se3_map(T, e->Xw, p);
    const double x = p[0], y = p[1], invz = 1.0 / p[2], invz_2 = invz * invz;
    const double fx = P->fx, fy = P->fy, bf = P->bf;
    J[0] = ((x * y) * invz_2) * fx;
    J[1] = (-(1 + ((x * x) * invz_2))) * fx;
    J[2] = (y * invz) * fx;
    J[3] = (-invz) * fx;
    J[4] = 0;
    J[5] = (x * invz_2) * fx;
    J[6] = (1 + ((y * y) * invz_2)) * fy;
    J[7] = (((-x) * y) * invz_2) * fy;
    J[8] = ((-x) * invz) * fy;
    J[9] = 0;
    J[10] = (-invz) * fy;
    J[11] = (y * invz_2) * fy;
    if (e->stereo) {
        J[12] = J[0] - ((bf * y) * invz_2);
        J[13] = J[1] + ((bf * x) * invz_2);
        J[14] = J[2];
        J[15] = J[3];
        J[16] = 0;
        J[17] = J[5] - (bf * invz_2);
    }
}

/* Eigen::LDLT<MatrixXd> (Lower) compute + solve, diagonal pivoting, sequential dot products.
 * H: n x n symmetric (both triangles), destroyed.  Returns isPositive(). */
int ora_ldlt_pivot_solve(double* H, int n, const double* b, double* x)
{
    int tr[64];
    double tmp[64], y[64];
    int sign = 0;   /* 0 ZeroSign, 1 PositiveSemiDef, 2 NegativeSemiDef, 3 Indefinite */
    if (n > 64) return 0;
#define M(i, j) H[(i) * n + (j)]
    for (int k = 0; k < n; k++) {
        int idx = k;
        double big = fabs(M(k, k));
        for (int i = k + 1; i < n; i++)
            if (fabs(M(i, i)) > big) { big = fabs(M(i, i)); idx = i; }
        tr[k] = idx;
        if (idx != k) {
            for (int j = 0; j < k; j++) { const double t = M(k, j); M(k, j) = M(idx, j); M(idx, j) = t; }
            for (int i = idx + 1; i < n; i++) { const double t = M(i, k); M(i, k) = M(i, idx); M(i, idx) = t; }
            { const double t = M(k, k); M(k, k) = M(idx, idx); M(idx, idx) = t; }
            for (int i = k + 1; i < idx; i++) { const double t = M(i, k); M(i, k) = M(idx, i); M(idx, i) = t; }
        }
        if (k > 0) {
            for (int j = 0; j < k; j++) tmp[j] = M(j, j) * M(k, j);
            double s = 0;
            for (int j = 0; j < k; j++) s += M(k, j) * tmp[j];
            M(k, k) -= s;
            for (int i = k + 1; i < n; i++) {
                double t = 0;
                for (int j = 0; j < k; j++) t += M(i, j) * tmp[j];
                M(i, k) -= t;
            }
        }
        const double akk = M(k, k);
        const int valid = fabs(akk) > 0.0;
        if (k == 0 && !valid) {   /* the whole diagonal is zero */
            for (int j = k; j < n; j++) tr[j] = j;
            sign = 0;
            break;
        }
        if (valid)
            for (int i = k + 1; i < n; i++) M(i, k) /= akk;
        if (sign == 1) { if (akk < 0) sign = 3; }
        else if (sign == 2) { if (akk > 0) sign = 3; }
        else if (sign == 0) { if (akk > 0) sign = 1; else if (akk < 0) sign = 2; }
    }
    if (!(sign == 1 || sign == 0)) return 0;
    for (int i = 0; i < n; i++) y[i] = b[i];
    for (int k = 0; k < n; k++) { const double t = y[k]; y[k] = y[tr[k]]; y[tr[k]] = t; }   /* P b */
    for (int i = 0; i < n; i++)                                                          /* L y */
        for (int j = 0; j < i; j++) y[i] -= M(i, j) * y[j];
    for (int i = 0; i < n; i++)                                                          /* D */
        y[i] = fabs(M(i, i)) > DBL_MIN ? y[i] / M(i, i) : 0.0;
    for (int i = n - 1; i >= 0; i--)                                                     /* L^T x */
        for (int j = n - 1; j > i; j--) y[i] -= M(j, i) * y[j];
    for (int k = n - 1; k >= 0; k--) { const double t = y[k]; y[k] = y[tr[k]]; y[tr[k]] = t; }  /* P^T */
    for (int i = 0; i < n; i++) x[i] = y[i];
#undef M
    return 1;
}

static const int DIAG21P[6] = {0, 6, 11, 15, 18, 20};

/* one OptimizationAlgorithmLevenberg::solve on the single pose */
static int pose_lm_solve(pose_edge* E, int ne, se3q* T, const ora_pose_problem* P, int iteration, double* lambda,
                         double* ni, int* nBadLM, double* scratch, double* xs, ora_ba_trace* tr)
{
    int nA = 0;
    double* v = scratch;
    for (int i = 0; i < ne; i++)
        if (E[i].level == 0) {
            pose_edge_error(&E[i], T, P);
            const double c = pose_edge_chi2(&E[i]);
            double r0 = c;
            if (E[i].robust && !(c <= E[i].dsqr)) { const double sq = sqrt(c); r0 = (2 * sq) * E[i].delta - E[i].dsqr; }
            v[nA++] = r0;
        }
    double currentChi = ba_sum(v, nA);
    const double iniChi = currentChi;
    /* buildSystem: terms per active edge, canonical sums in edge order */
    double H[21], bvec[6];
    {
        double* terms = scratch + ne + 64;   /* 27 x nA */
        int a = 0;
        for (int i = 0; i < ne; i++) {
            if (E[i].level != 0) continue;
            pose_edge* e = &E[i];
            double J[18];
            pose_edge_jacobian(e, T, P, J);
            const int D = e->stereo ? 3 : 2;
            const double c = pose_edge_chi2(e);
            double r1 = 1.;
            if (e->robust && !(c <= e->dsqr)) r1 = e->delta / sqrt(c);
            const double w = e->robust ? r1 * e->info : e->info;
            double omr[3] = {0, 0, 0};
            for (int k = 0; k < D; k++) {
                omr[k] = -(e->info * e->err[k]);
                if (e->robust) omr[k] *= r1;
            }
            int q = 0;
            for (int r = 0; r < 6; r++) {
                double s = 0;
                for (int k = 0; k < D; k++) s += J[k * 6 + r] * omr[k];
                terms[(21 + r) * nA + a] = s;
                for (int cc = r; cc < 6; cc++) {
                    double h = 0;
                    for (int k = 0; k < D; k++) h += (J[k * 6 + r] * w) * J[k * 6 + cc];
                    terms[q * nA + a] = h;
                    q++;
                }
            }
            a++;
        }
        for (int q = 0; q < 27; q++) {
            for (int j = 0; j < nA; j++) v[j] = terms[q * nA + j];
            const double s = ba_sum(v, nA);
            if (q < 21) H[q] = s; else bvec[q - 21] = s;
        }
    }
    if (iteration == 0) {
        double m = 0.;
        for (int j = 0; j < 6; j++) m = fmax(fabs(H[DIAG21P[j]]), m);
        *lambda = 1e-5 * m;
        *ni = 2;
        *nBadLM = 0;
    }
    double rho = 0;
    int qmax = 0;
    do {
        const se3q Tbak = *T;
        double Hd[36], x[6];
        for (int r = 0, q = 0; r < 6; r++)
            for (int cc = r; cc < 6; cc++, q++) {
                double h = H[q];
                if (cc == r) h += *lambda;
                Hd[r * 6 + cc] = h;
                Hd[cc * 6 + r] = h;
            }
        const int ok2 = ora_ldlt_pivot_solve(Hd, 6, bvec, x);
        if (ok2) memcpy(xs, x, sizeof(x));   /* a failed solve leaves the solver's _x as it was */
        {
            se3q d, r;
            se3_exp(xs, &d);
            se3_mul(&d, T, &r);
            *T = r;
        }
        int nB = 0;
        for (int i = 0; i < ne; i++)
            if (E[i].level == 0) {
                pose_edge_error(&E[i], T, P);
                const double c = pose_edge_chi2(&E[i]);
                double r0 = c;
                if (E[i].robust && !(c <= E[i].dsqr)) { const double sq = sqrt(c); r0 = (2 * sq) * E[i].delta - E[i].dsqr; }
                v[nB++] = r0;
            }
        double tempChi = ba_sum(v, nB);
        if (!ok2) tempChi = DBL_MAX;
        rho = currentChi - tempChi;
        for (int j = 0; j < 6; j++) v[j] = xs[j] * (*lambda * xs[j] + bvec[j]);
        double scale = ba_sum(v, 6);
        scale += 1e-3;
        rho /= scale;
        if (rho > 0 && isfinite(tempChi)) {
            const double a3 = 2 * rho - 1;
            double alpha = 1. - (a3 * a3) * a3;
            alpha = fmin(alpha, 2. / 3.);
            const double scaleFactor = fmax(1. / 3., alpha);
            *lambda *= scaleFactor;
            *ni = 2;
            currentChi = tempChi;
        } else {
            *lambda *= *ni;
            *ni *= 2;
            *T = Tbak;
        }
        qmax++;
        if (tr && tr->n_trials < ORA_BA_TRACE_MAX) {
            tr->trial_chi2[tr->n_trials] = tempChi;
            tr->trial_lambda[tr->n_trials] = *lambda;
            tr->n_trials++;
        }
    } while (rho < 0 && qmax < 10);
    if (tr && tr->n_solves < ORA_BA_TRACE_MAX) {
        tr->solve_ini_chi2[tr->n_solves] = iniChi;
        tr->solve_chi2[tr->n_solves] = currentChi;
        tr->n_solves++;
    }
    if (qmax == 10 || rho == 0) return 1;
    if ((iniChi - currentChi) * 1e3 < iniChi) (*nBadLM)++;
    else *nBadLM = 0;
    return *nBadLM >= 3;
}

int ora_pose_optimization(const ora_pose_problem* P, float* Tcw_out, uint8_t* outlier, ora_ba_trace* tr)
{
    const int N = P->N;
    if (tr) memset(tr, 0, sizeof(*tr));
    memcpy(Tcw_out, P->Tcw, sizeof(float) * 16);
    pose_edge* E = (pose_edge*)calloc(N + 1, sizeof(pose_edge));
    const float deltaMono = (float)sqrt(5.991), deltaStereo = (float)sqrt(7.815);
    int ne = 0;
    for (int i = 0; i < N; i++) {
        if (!P->has_mp[i]) continue;
        outlier[i] = 0;
        pose_edge* e = &E[ne++];
        e->kp = i;
        e->stereo = !(P->obs[3 * i + 2] < 0);
        for (int j = 0; j < 3; j++) { e->Xw[j] = (double)P->Xw[3 * i + j]; e->obs[j] = (double)P->obs[3 * i + j]; }
        e->info = (double)P->inv_sigma2[i];
        e->delta = (double)(e->stereo ? deltaStereo : deltaMono);
        e->dsqr = e->delta * e->delta;
        e->robust = 1;
        e->level = 0;
    }
    const int nInitial = ne;
    if (nInitial < 3) { free(E); return 0; }
    double* scratch = (double*)malloc(sizeof(double) * (28 * (size_t)ne + 128));
    const float chi2Mono = 5.991f, chi2Stereo = 7.815f;
    int nBad = 0;
    se3q T;
    for (int it = 0; it < 4; it++) {
        se3_from_Tcw(P->Tcw, &T);            /* vSE3->setEstimate(toSE3Quat(pFrame->mTcw)) */
        double xs[6] = {0, 0, 0, 0, 0, 0};   /* BlockSolver::_x, (re)allocated by buildStructure */
        int nAct = 0;
        for (int i = 0; i < ne; i++) nAct += E[i].level == 0;
        if (nAct > 0) {   /* optimize(10): no active edge -> no vertex to optimise (returns -1) */
            double lambda = 0, ni = 2;
            int nBadLM = 0;
            for (int k = 0; k < 10; k++)
                if (pose_lm_solve(E, ne, &T, P, k, &lambda, &ni, &nBadLM, scratch, xs, tr)) break;
        }
        nBad = 0;
        for (int i = 0; i < ne; i++) {
            pose_edge* e = &E[i];
            if (outlier[e->kp]) pose_edge_error(e, &T, P);
            const float chi2 = (float)pose_edge_chi2(e);
            if (chi2 > (e->stereo ? chi2Stereo : chi2Mono)) {
                outlier[e->kp] = 1;
                e->level = 1;
                nBad++;
            } else {
                outlier[e->kp] = 0;
                e->level = 0;
            }
            if (it == 2) e->robust = 0;
        }
        if (ne < 10) break;
    }
    se3_to_Tcw(&T, Tcw_out);
    free(scratch);
    free(E);
    return nInitial - nBad;
}

/* ======================================================================
 * Optimizer::OptimizeSim3 (reference src/Optimizer.cc:1046-1241).
 * One VertexSim3Expmap (types_seven_dof_expmap.h:48-94: oplus = Sim3(update)*estimate,
 * update[6] zeroed IN PLACE when _fix_scale -- it is the solver's _x), fixed point
 * vertices, EdgeSim3ProjectXYZ / EdgeInverseSim3ProjectXYZ (130-171) with the default
 * numeric Jacobian of BaseBinaryEdge::linearizeOplus (base_binary_edge.hpp:131-204:
 * delta 1e-9, central difference, push/oplus/computeError/pop per column), Huber
 * sqrt(th2) on both edges, BlockSolverX + LinearSolverDense (pivoted LDL^T of the 7x7
 * block), optimize(5), chi2 gating, optimize(10 | 5) on the inliers.
 * g2o::Sim3 (sim3.h): ctor from update 64-146, map 148-150, inverse 235-238,
 * operator* 264-270.  exp uses ora_det_exp / ora_det_sincos; 3x3 products and norms
 * sum their terms left to right; the canonical sums of the LM are those of the pose
 * optimisation above.
 * ====================================================================== */

/* fdlibm __ieee754_exp, as IEEE operation sequence (deterministic on CPU and GPU) */
double ora_det_exp(double x)
{
    const double halF[2] = {0.5, -0.5};
    const double ln2HI[2] = {6.93147180369123816490e-01, -6.93147180369123816490e-01};
    const double ln2LO[2] = {1.90821492927058770002e-10, -1.90821492927058770002e-10};
    const double invln2 = 1.44269504088896338700e+00;
    const double P1 = 1.66666666666666019037e-01, P2 = -2.77777777770155933842e-03,
                 P3 = 6.61375632143793436117e-05, P4 = -1.65339022054652515390e-06,
                 P5 = 4.13813679705723846039e-08;
    if (x != x) return x;
    if (x > 7.09782712893383973096e+02) return HUGE_VAL;
    if (x < -7.45133219101941108420e+02) return 0.0;
    const int xsb = x < 0;
    const double ax = fabs(x);
    double hi = 0, lo = 0;
    int k = 0;
    if (ax > 0.5 * 6.93147180559945286227e-01) {
        if (ax < 1.5 * 6.93147180559945286227e-01) {
            hi = x - ln2HI[xsb];
            lo = ln2LO[xsb];
            k = 1 - xsb - xsb;
        } else {
            k = (int)(invln2 * x + halF[xsb]);
            const double t = k;
            hi = x - t * ln2HI[0];
            lo = t * ln2LO[0];
        }
        x = hi - lo;
    } else if (ax < 3.7252902984e-09) { /* 2^-28 */
        return 1.0 + x;
    }
    const double t = x * x;
    const double c = x - t * (P1 + t * (P2 + t * (P3 + t * (P4 + t * P5))));
    if (k == 0) return 1.0 - ((x * c) / (c - 2.0) - x);
    const double y = 1.0 - ((lo - (x * c) / (2.0 - c)) - hi);
    return ldexp(y, k);
}

typedef struct { double q[4]; double t[3]; double s; } sim3q;

static void sim3_exp(const double* upd, sim3q* o) /* Sim3(const Vector7d&) sim3.h:64-146 */
{
    const double w[3] = {upd[0], upd[1], upd[2]};
    const double u[3] = {upd[3], upd[4], upd[5]};
    const double sigma = upd[6];
    const double theta = sqrt((w[0] * w[0] + w[1] * w[1]) + w[2] * w[2]);
    const double Om[9] = {0, -w[2], w[1], w[2], 0, -w[0], -w[1], w[0], 0};
    double Om2[9], R[9], W[9];
    mat3_mul(Om, Om, Om2);
    const double s = ora_det_exp(sigma);
    const double eps = 0.00001;
    double A, B, C;
    if (fabs(sigma) < eps) {
        C = 1;
        if (theta < eps) {
            A = 1. / 2.;
            B = 1. / 6.;
            for (int i = 0; i < 9; i++) R[i] = (((i % 4) == 0 ? 1.0 : 0.0) + Om[i]) + Om2[i];
        } else {
            double sn, cs;
            ora_det_sincos(theta, &sn, &cs);
            const double theta2 = theta * theta;
            A = (1 - cs) / theta2;
            B = (theta - sn) / (theta2 * theta);
            const double a = sn / theta, b = (1 - cs) / (theta * theta);
            for (int i = 0; i < 9; i++) R[i] = (((i % 4) == 0 ? 1.0 : 0.0) + a * Om[i]) + b * Om2[i];
        }
    } else {
        C = (s - 1) / sigma;
        if (theta < eps) {
            const double sigma2 = sigma * sigma;
            A = ((sigma - 1) * s + 1) / sigma2;
            B = ((0.5 * sigma2 - sigma + 1) * s) / (sigma2 * sigma);
            for (int i = 0; i < 9; i++) R[i] = (((i % 4) == 0 ? 1.0 : 0.0) + Om[i]) + Om2[i];
        } else {
            double sn, cs;
            ora_det_sincos(theta, &sn, &cs);
            const double ra = sn / theta, rb = (1 - cs) / (theta * theta);
            for (int i = 0; i < 9; i++) R[i] = (((i % 4) == 0 ? 1.0 : 0.0) + ra * Om[i]) + rb * Om2[i];
            const double a = s * sn, b = s * cs;
            const double theta2 = theta * theta, sigma2 = sigma * sigma;
            const double c = theta2 + sigma2;
            A = (a * sigma + (1 - b) * theta) / (theta * c);
            B = (C - ((b - 1) * sigma + a * theta) / c) * 1. / theta2;
        }
    }
    quat_from_R(R, o->q);
    for (int i = 0; i < 9; i++) W[i] = (A * Om[i] + B * Om2[i]) + C * ((i % 4) == 0 ? 1.0 : 0.0);
    for (int i = 0; i < 3; i++) o->t[i] = (W[i * 3] * u[0] + W[i * 3 + 1] * u[1]) + W[i * 3 + 2] * u[2];
    o->s = s;
}

static void sim3_mul(const sim3q* a, const sim3q* b, sim3q* o) /* operator* sim3.h:264-270 */
{
    sim3q r;
    double rt[3];
    quat_mul(a->q, b->q, r.q);
    quat_rotate(a->q, b->t, rt);
    for (int i = 0; i < 3; i++) r.t[i] = a->s * rt[i] + a->t[i];
    r.s = a->s * b->s;
    *o = r;
}

static void sim3_map(const sim3q* T, const double* X, double* out) /* map sim3.h:148-150 */
{
    double r[3];
    quat_rotate(T->q, X, r);
    for (int i = 0; i < 3; i++) out[i] = T->s * r[i] + T->t[i];
}

static void sim3_inverse(const sim3q* T, sim3q* o) /* inverse sim3.h:235-238 */
{
    sim3q r;
    r.q[0] = -T->q[0]; r.q[1] = -T->q[1]; r.q[2] = -T->q[2]; r.q[3] = T->q[3];
    const double ms = -1. / T->s;
    const double v[3] = {ms * T->t[0], ms * T->t[1], ms * T->t[2]};
    quat_rotate(r.q, v, r.t);
    r.s = 1. / T->s;
    *o = r;
}

/* g2o::Sim3(Converter::toMatrix3d(R), toVector3d(t), s) (LoopClosing.cc:317) */
void ora_sim3_from_Rts(const float* R, const float* t, float s, double* S12)
{
    double Rd[9];
    for (int i = 0; i < 9; i++) Rd[i] = (double)R[i];
    quat_from_R(Rd, S12);
    for (int i = 0; i < 3; i++) S12[4 + i] = (double)t[i];
    S12[7] = (double)s;
}

typedef struct {
    double X[3], obs[2], info, err[2];
    int inv;        /* 0: EdgeSim3ProjectXYZ (X = point 2, camera 1), 1: inverse edge */
    int level;      /* 0 active, 1 removed */
} s3_edge;

typedef struct { double f1[2], p1[2], f2[2], p2[2]; } s3_cam;

/* computeError with the Sim3 estimate T and its inverse Ti */
static void s3_error(const s3_edge* e, const sim3q* T, const sim3q* Ti, const s3_cam* K, double* err)
{
    double p[3];
    if (!e->inv) {
        sim3_map(T, e->X, p);
        const double px = p[0] / p[2], py = p[1] / p[2];
        err[0] = e->obs[0] - (px * K->f1[0] + K->p1[0]);
        err[1] = e->obs[1] - (py * K->f1[1] + K->p1[1]);
    } else {
        sim3_map(Ti, e->X, p);
        const double px = p[0] / p[2], py = p[1] / p[2];
        err[0] = e->obs[0] - (px * K->f2[0] + K->p2[0]);
        err[1] = e->obs[1] - (py * K->f2[1] + K->p2[1]);
    }
}

static double s3_chi2(const double* err, double info) { return err[0] * (info * err[0]) + err[1] * (info * err[1]); }

static double s3_rho0(double c, double delta, double dsqr)
{
    if (c <= dsqr) return c;
    const double sq = sqrt(c);
    return (2 * sq) * delta - dsqr;
}

static const int DIAG28[7] = {0, 7, 13, 18, 22, 25, 27};

/* the 14 perturbed estimates of linearizeOplus: Sim3(+-delta e_d) * T and their inverses */
static void s3_perturbed(const sim3q* T, int fixScale, sim3q* Tp, sim3q* Tpi)
{
    const double delta = 1e-9;
    for (int d = 0; d < 7; d++)
        for (int sgn = 0; sgn < 2; sgn++) {
            double add[7] = {0, 0, 0, 0, 0, 0, 0};
            add[d] = sgn ? -delta : delta;
            if (fixScale) add[6] = 0;
            sim3q U;
            sim3_exp(add, &U);
            sim3_mul(&U, T, &Tp[2 * d + sgn]);
            sim3_inverse(&Tp[2 * d + sgn], &Tpi[2 * d + sgn]);
        }
}

/* one OptimizationAlgorithmLevenberg::solve on the Sim3 vertex */
static int s3_lm_solve(s3_edge* E, int ne, sim3q* T, const s3_cam* K, int fixScale, double delta, int iteration,
                       double* lambda, double* ni, int* nBadLM, double* scratch, double* xs, ora_ba_trace* tr)
{
    const double dsqr = delta * delta;
    double* v = scratch;
    sim3q Ti;
    sim3_inverse(T, &Ti);
    int nA = 0;
    for (int i = 0; i < ne; i++)
        if (E[i].level == 0) {
            s3_error(&E[i], T, &Ti, K, E[i].err);
            v[nA++] = s3_rho0(s3_chi2(E[i].err, E[i].info), delta, dsqr);
        }
    double currentChi = ora_csum(v, nA);
    const double iniChi = currentChi;
    double H[28], bvec[7];
    {
        sim3q Tp[14], Tpi[14];
        s3_perturbed(T, fixScale, Tp, Tpi);
        const double scalar = 1.0 / (2 * 1e-9);
        double* terms = scratch + ne + 64; /* 35 x nA */
        int a = 0;
        for (int i = 0; i < ne; i++) {
            s3_edge* e = &E[i];
            if (e->level != 0) continue;
            double J[14]; /* 2 x 7 row-major */
            for (int d = 0; d < 7; d++) {
                double ep[2], em[2];
                s3_error(e, &Tp[2 * d], &Tpi[2 * d], K, ep);
                s3_error(e, &Tp[2 * d + 1], &Tpi[2 * d + 1], K, em);
                J[d] = scalar * (ep[0] - em[0]);
                J[7 + d] = scalar * (ep[1] - em[1]);
            }
            const double c = s3_chi2(e->err, e->info);
            double r1 = 1.;
            if (!(c <= dsqr)) r1 = delta / sqrt(c);
            const double w = r1 * e->info;
            double omr[2];
            for (int k = 0; k < 2; k++) omr[k] = -(e->info * e->err[k]) * r1;
            int q = 0;
            for (int r = 0; r < 7; r++) {
                terms[(28 + r) * nA + a] = J[r] * omr[0] + J[7 + r] * omr[1];
                for (int cc = r; cc < 7; cc++) {
                    terms[q * nA + a] = (J[r] * w) * J[cc] + (J[7 + r] * w) * J[7 + cc];
                    q++;
                }
            }
            a++;
        }
        for (int q = 0; q < 35; q++) {
            for (int j = 0; j < nA; j++) v[j] = terms[q * nA + j];
            const double s = ora_csum(v, nA);
            if (q < 28) H[q] = s; else bvec[q - 28] = s;
        }
    }
    if (iteration == 0) {
        double m = 0.;
        for (int j = 0; j < 7; j++) m = fmax(fabs(H[DIAG28[j]]), m);
        *lambda = 1e-5 * m;
        *ni = 2;
        *nBadLM = 0;
    }
    double rho = 0;
    int qmax = 0;
    do {
        const sim3q Tbak = *T;
        double Hd[49], x[7];
        for (int r = 0, q = 0; r < 7; r++)
            for (int cc = r; cc < 7; cc++, q++) {
                double h = H[q];
                if (cc == r) h += *lambda;
                Hd[r * 7 + cc] = h;
                Hd[cc * 7 + r] = h;
            }
        const int ok2 = ora_ldlt_pivot_solve(Hd, 7, bvec, x);
        if (ok2) memcpy(xs, x, sizeof(x));
        if (fixScale) xs[6] = 0; /* oplusImpl writes through the Map of the solver's _x */
        {
            sim3q U, r;
            sim3_exp(xs, &U);
            sim3_mul(&U, T, &r);
            *T = r;
        }
        sim3_inverse(T, &Ti);
        int nB = 0;
        for (int i = 0; i < ne; i++)
            if (E[i].level == 0) {
                s3_error(&E[i], T, &Ti, K, E[i].err);
                v[nB++] = s3_rho0(s3_chi2(E[i].err, E[i].info), delta, dsqr);
            }
        double tempChi = ora_csum(v, nB);
        if (!ok2) tempChi = DBL_MAX;
        rho = currentChi - tempChi;
        for (int j = 0; j < 7; j++) v[j] = xs[j] * (*lambda * xs[j] + bvec[j]);
        double scale = ora_csum(v, 7);
        scale += 1e-3;
        rho /= scale;
        if (rho > 0 && isfinite(tempChi)) {
            const double a3 = 2 * rho - 1;
            double alpha = 1. - (a3 * a3) * a3;
            alpha = fmin(alpha, 2. / 3.);
            const double scaleFactor = fmax(1. / 3., alpha);
            *lambda *= scaleFactor;
            *ni = 2;
            currentChi = tempChi;
        } else {
            *lambda *= *ni;
            *ni *= 2;
            *T = Tbak;
        }
        qmax++;
        if (tr && tr->n_trials < ORA_BA_TRACE_MAX) {
            tr->trial_chi2[tr->n_trials] = tempChi;
            tr->trial_lambda[tr->n_trials] = *lambda;
            tr->n_trials++;
        }
    } while (rho < 0 && qmax < 10);
    if (tr && tr->n_solves < ORA_BA_TRACE_MAX) {
        tr->solve_ini_chi2[tr->n_solves] = iniChi;
        tr->solve_chi2[tr->n_solves] = currentChi;
        tr->n_solves++;
    }
    if (qmax == 10 || rho == 0) return 1;
    if ((iniChi - currentChi) * 1e3 < iniChi) (*nBadLM)++;
    else *nBadLM = 0;
    return *nBadLM >= 3;
}

static void s3_optimize(s3_edge* E, int ne, sim3q* T, const s3_cam* K, int fixScale, double delta, int its,
                        double* scratch, ora_ba_trace* tr)
{
    double xs[7] = {0, 0, 0, 0, 0, 0, 0}; /* BlockSolver::_x after buildStructure */
    double lambda = 0, ni = 2;
    int nBadLM = 0;
    int nAct = 0;
    for (int i = 0; i < ne; i++) nAct += E[i].level == 0;
    if (nAct == 0) return; /* no active edge: the Sim3 vertex is not in the index map (optimize returns -1) */
    for (int k = 0; k < its; k++)
        if (s3_lm_solve(E, ne, T, K, fixScale, delta, k, &lambda, &ni, &nBadLM, scratch, xs, tr)) break;
}

int ora_optimize_sim3(const ora_sim3opt_problem* P, double* S12, uint8_t* erased, ora_ba_trace* tr)
{
    const int N = P->N;
    if (tr) memset(tr, 0, sizeof(*tr));
    for (int i = 0; i < N; i++) erased[i] = 0;
    s3_cam K;
    K.f1[0] = P->K1[0]; K.f1[1] = P->K1[1]; K.p1[0] = P->K1[2]; K.p1[1] = P->K1[3];
    K.f2[0] = P->K2[0]; K.f2[1] = P->K2[1]; K.p2[0] = P->K2[2]; K.p2[1] = P->K2[3];
    s3_edge* E = (s3_edge*)calloc(2 * (size_t)N + 1, sizeof(s3_edge));
    int* corr = (int*)malloc(sizeof(int) * ((size_t)N + 1));
    int nc = 0;
    for (int i = 0; i < N; i++) {
        if (!P->valid[i]) continue;
        s3_edge* e12 = &E[2 * nc];
        s3_edge* e21 = &E[2 * nc + 1];
        for (int j = 0; j < 3; j++) { e12->X[j] = (double)P->X2c[3 * i + j]; e21->X[j] = (double)P->X1c[3 * i + j]; }
        e12->obs[0] = P->obs1[2 * i]; e12->obs[1] = P->obs1[2 * i + 1];
        e21->obs[0] = P->obs2[2 * i]; e21->obs[1] = P->obs2[2 * i + 1];
        e12->info = (double)P->inv_sigma2_1[i];
        e21->info = (double)P->inv_sigma2_2[i];
        e12->inv = 0; e21->inv = 1;
        corr[nc++] = i;
    }
    const int ne = 2 * nc;
    const float deltaHuberF = sqrtf(P->th2);
    const double delta = (double)deltaHuberF;
    const double th2 = (double)P->th2;
    double* scratch = (double*)malloc(sizeof(double) * (36 * (size_t)ne + 192));
    sim3q T;
    memcpy(T.q, S12, 4 * sizeof(double));
    memcpy(T.t, S12 + 4, 3 * sizeof(double));
    T.s = S12[7];
    s3_optimize(E, ne, &T, &K, P->bFixScale, delta, 5, scratch, tr);
    int nBad = 0;
    for (int c = 0; c < nc; c++) {
        s3_edge* a = &E[2 * c];
        s3_edge* b = &E[2 * c + 1];
        if (s3_chi2(a->err, a->info) > th2 || s3_chi2(b->err, b->info) > th2) {
            erased[corr[c]] = 1;
            a->level = b->level = 1;
            nBad++;
        }
    }
    const int nMoreIterations = nBad > 0 ? 10 : 5;
    int nIn = 0;
    if (nc - nBad >= 10) {
        s3_optimize(E, ne, &T, &K, P->bFixScale, delta, nMoreIterations, scratch, tr);
        for (int c = 0; c < nc; c++) {
            s3_edge* a = &E[2 * c];
            s3_edge* b = &E[2 * c + 1];
            if (a->level) continue;
            if (s3_chi2(a->err, a->info) > th2 || s3_chi2(b->err, b->info) > th2) erased[corr[c]] = 1;
            else nIn++;
        }
        memcpy(S12, T.q, 4 * sizeof(double));
        memcpy(S12 + 4, T.t, 3 * sizeof(double));
        S12[7] = T.s;
    }
    free(scratch);
    free(corr);
    free(E);
    return nIn;
}
