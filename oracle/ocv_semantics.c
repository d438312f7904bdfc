/*
 * ocv_semantics.c -- TEST INFRASTRUCTURE ONLY (parity oracle).
 *
 * Restatements of the third-party arithmetic the reference calls at its
 * ORB-extraction call sites.  OpenCV is NOT vendored in the
 * reference and is absent from this image; each routine restates the scalar
 * code path of OpenCV 3.2 (the version README.md:68 says the reference was
 * tested with).  "parity unpinned" at this boundary -- see DESIGN.md.
 *
 *   cvRound          -> lrint/lrintf (round-half-even)          ORBextractor.cc:81,115,119-120,442,1112
 *   fastAtan2        -> OpenCV 3.2 core/mathfuncs.cpp polynomial ORBextractor.cc:103
 *   sinf / cosf      -> glibc 2.35 sincosf (pinned exhaustively) ORBextractor.cc:112
 *   FAST_t<16>       -> features2d/fast.cpp + fast_score.cpp     ORBextractor.cc:809,814
 *   resize LINEAR 8U -> imgproc/imgwarp.cpp fixed point (11 bit) ORBextractor.cc:1120
 *   GaussianBlur 8U  -> imgproc/smooth.cpp + filter.cpp 8-bit fixed-point separable
 *                       filter, scalar (non-SSE) column cast      ORBextractor.cc:1086
 *   undistortPoints  -> imgproc/undistort.cpp cvUndistortPoints  Frame.cc:404-464
 */
#include "orb_oracle.h"
#include <math.h>
#include <string.h>
#include <stdlib.h>
#include <float.h>

int ora_cvRound_f(float v) { return (int)lrintf(v); }
int ora_cvRound_d(double v) { return (int)lrint(v); }

/* OpenCV 3.2 fastAtan2 (degrees, [0,360)) */
static const float atan2_p1 = 0.9997878412794807f * (float)(180 / 3.14159265358979323846);
static const float atan2_p3 = -0.3258083974640975f * (float)(180 / 3.14159265358979323846);
static const float atan2_p5 = 0.1555786518463281f * (float)(180 / 3.14159265358979323846);
static const float atan2_p7 = -0.04432655554792128f * (float)(180 / 3.14159265358979323846);

float ora_fastAtan2(float y, float x)
{
    float ax = fabsf(x), ay = fabsf(y);
    float a, c, c2;
    if (ax >= ay) {
        c = ay / (ax + (float)DBL_EPSILON);
        c2 = c * c;
        a = (((atan2_p7 * c2 + atan2_p5) * c2 + atan2_p3) * c2 + atan2_p1) * c;
    } else {
        c = ax / (ay + (float)DBL_EPSILON);
        c2 = c * c;
        a = 90.f - (((atan2_p7 * c2 + atan2_p5) * c2 + atan2_p3) * c2 + atan2_p1) * c;
    }
    if (x < 0) a = 180.f - a;
    if (y < 0) a = 360.f - a;
    return a;
}

/* glibc 2.35 sysdeps/ieee754/flt-32 sinf/cosf (Szabolcs Nagy's sincosf),
 * restated for |x| < 120 (the descriptor only needs [0, 2*pi]).  Verified
 * bit-for-bit against the host libm over every float in [0, 6.2832]. */
typedef struct { double sign[4], hpi_inv, hpi, c0, c1, c2, c3, c4, s1, s2, s3; } sc_tab;
static const sc_tab SCT[2] = {
    {{1.0, -1.0, -1.0, 1.0}, 0x1.45F306DC9C883p+23, 0x1.921FB54442D18p0, 0x1p0,
     -0x1.ffffffd0c621cp-2, 0x1.55553e1068f19p-5, -0x1.6c087e89a359dp-10, 0x1.99343027bf8c3p-16,
     -0x1.555545995a603p-3, 0x1.1107605230bc4p-7, -0x1.994eb3774cf24p-13},
    {{1.0, -1.0, -1.0, 1.0}, 0x1.45F306DC9C883p+23, 0x1.921FB54442D18p0, -0x1p0,
     0x1.ffffffd0c621cp-2, -0x1.55553e1068f19p-5, 0x1.6c087e89a359dp-10, -0x1.99343027bf8c3p-16,
     -0x1.555545995a603p-3, 0x1.1107605230bc4p-7, -0x1.994eb3774cf24p-13}};

static inline uint32_t f2u(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static inline uint32_t top12(float f) { return (f2u(f) >> 20) & 0x7ff; }

static inline float sc_poly(double x, double x2, const sc_tab* p, int n)
{
    if ((n & 1) == 0) {
        double x3 = x * x2;
        double s1 = p->s2 + x2 * p->s3;
        double x7 = x3 * x2;
        double s = x + x3 * p->s1;
        return (float)(s + x7 * s1);
    } else {
        double x4 = x2 * x2;
        double c2 = p->c3 + x2 * p->c4;
        double c1 = p->c0 + x2 * p->c1;
        double x6 = x4 * x2;
        double c = c1 + x4 * p->c2;
        return (float)(c + x6 * c2);
    }
}

static inline double sc_reduce(double x, const sc_tab* p, int* np)
{
    double r = x * p->hpi_inv;
    int n = ((int32_t)r + 0x800000) >> 24;
    *np = n;
    return x - n * p->hpi;
}

float ora_cosf(float y)
{
    double x = y, s;
    const sc_tab* p = &SCT[0];
    int n;
    if (top12(y) < top12(0x1.921FB6p-1f)) {
        double x2 = x * x;
        if (top12(y) < top12(0x1p-12f)) return 1.0f;
        return sc_poly(x, x2, p, 1);
    }
    x = sc_reduce(x, p, &n);
    s = p->sign[n & 3];
    if (n & 2) p = &SCT[1];
    return sc_poly(x * s, x * x, p, n ^ 1);
}

float ora_sinf(float y)
{
    double x = y, s;
    const sc_tab* p = &SCT[0];
    int n;
    if (top12(y) < top12(0x1.921FB6p-1f)) {
        s = x * x;
        if (top12(y) < top12(0x1p-12f)) return y;
        return sc_poly(x, s, p, 0);
    }
    x = sc_reduce(x, p, &n);
    s = p->sign[n & 3];
    if (n & 2) p = &SCT[1];
    return sc_poly(x * s, x * x, p, n);
}

/* ---- FAST-9/16 ------------------------------------------------------------
 * Circle order of OpenCV makeOffsets(pixel, step, 16). */
static const int FAST_OFS[16][2] = {
    {0, 3}, {1, 3}, {2, 2}, {3, 1}, {3, 0}, {3, -1}, {2, -2}, {1, -3},
    {0, -3}, {-1, -3}, {-2, -2}, {-3, -1}, {-3, 0}, {-3, 1}, {-2, 2}, {-1, 3}};

/* cornerScore<16> (fast_score.cpp): returns max(threshold, A, B) - 1 where A/B
 * are the best dark/bright contiguous-9 contrasts.  With threshold 0 passed in
 * it is S = max(0,A,B)-1; a pixel is a FAST corner at threshold t iff A>t||B>t
 * iff max(A,B)-1 >= t, and its stored score is then exactly max(A,B)-1. */
int ora_fast_score(const uint8_t* p, int step)
{
    int v = p[0];
    int d[25];
    for (int k = 0; k < 25; k++) {
        int kk = k & 15;
        d[k] = v - p[FAST_OFS[kk][0] + FAST_OFS[kk][1] * step];
    }
    int A = -1000, B = -1000;
    for (int k = 0; k < 16; k++) {
        int mn = 1000, mx = -1000;
        for (int j = 0; j < 9; j++) {
            int dv = d[k + j];
            if (dv < mn) mn = dv;
            if (dv > mx) mx = dv;
        }
        if (mn > A) A = mn;      /* dark arc: all d >= mn */
        if (-mx > B) B = -mx;    /* bright arc: all -d >= -mx */
    }
    return (A > B ? A : B) - 1;
}

/* FAST_t<16>(roi, kps, threshold, nonmax=true), features2d/fast.cpp:
 * detection on rows/cols [3, n-3) of the ROI, scores of non-corners are 0,
 * a corner survives if its score is strictly greater than all 8 neighbours.
 * Output is raster order (row, then column). */
int ora_fast_roi(const uint8_t* roi, int step, int cols, int rows, int th,
                 int* xs, int* ys, int* scores, int cap)
{
    if (th < 0) th = 0;
    if (th > 255) th = 255;
    if (rows < 7 || cols < 7) return 0;
    int pix[25];
    for (int k = 0; k < 25; k++) pix[k] = FAST_OFS[k & 15][0] + FAST_OFS[k & 15][1] * step;
    /* threshold_tab of FAST_t: 1 = darker than v-th, 2 = brighter than v+th */
    uint8_t tab_mem[512];
    for (int i = -255; i <= 255; i++) tab_mem[i + 255] = (uint8_t)(i < -th ? 1 : (i > th ? 2 : 0));
    int* sc = (int*)calloc((size_t)rows * cols, sizeof(int));
    for (int i = 3; i < rows - 3; i++) {
        const uint8_t* ptr = roi + (size_t)i * step;
        for (int j = 3; j < cols - 3; j++) {
            const uint8_t* p = ptr + j;
            const int v = p[0];
            const uint8_t* tab = tab_mem - v + 255;
            int d = tab[p[pix[0]]] | tab[p[pix[8]]];
            if (d == 0) continue;
            d &= tab[p[pix[2]]] | tab[p[pix[10]]];
            d &= tab[p[pix[4]]] | tab[p[pix[12]]];
            d &= tab[p[pix[6]]] | tab[p[pix[14]]];
            if (d == 0) continue;
            d &= tab[p[pix[1]]] | tab[p[pix[9]]];
            d &= tab[p[pix[3]]] | tab[p[pix[11]]];
            d &= tab[p[pix[5]]] | tab[p[pix[13]]];
            d &= tab[p[pix[7]]] | tab[p[pix[15]]];
            int corner = 0;
            if (d & 1) {
                int vt = v - th, count = 0;
                for (int k = 0; k < 25; k++) {
                    if (p[pix[k]] < vt) { if (++count > 8) { corner = 1; break; } }
                    else count = 0;
                }
            }
            if (!corner && (d & 2)) {
                int vt = v + th, count = 0;
                for (int k = 0; k < 25; k++) {
                    if (p[pix[k]] > vt) { if (++count > 8) { corner = 1; break; } }
                    else count = 0;
                }
            }
            if (corner) sc[i * cols + j] = ora_fast_score(p, step);
        }
    }
    int n = 0;
    for (int i = 3; i < rows - 3; i++)
        for (int j = 3; j < cols - 3; j++) {
            int s = sc[i * cols + j];
            if (!s) continue;
            const int* r0 = sc + (i - 1) * cols + j;
            const int* r1 = sc + i * cols + j;
            const int* r2 = sc + (i + 1) * cols + j;
            if (s > r0[-1] && s > r0[0] && s > r0[1] && s > r1[-1] && s > r1[1] &&
                s > r2[-1] && s > r2[0] && s > r2[1]) {
                if (n < cap) { xs[n] = j; ys[n] = i; scores[n] = s; }
                n++;
            }
        }
    free(sc);
    return n;
}

/* ---- resize(INTER_LINEAR) for CV_8U (imgwarp.cpp, OpenCV 3.2) ------------ */
#define RCOEF_BITS 11
#define RCOEF_SCALE (1 << RCOEF_BITS)

static inline short sat_short_f(float v)
{
    int i = (int)lrintf(v);
    return (short)(i < -32768 ? -32768 : (i > 32767 ? 32767 : i));
}

void ora_resize_linear_u8(const uint8_t* src, int sstep, int sw, int sh,
                          uint8_t* dst, int dstep, int dw, int dh)
{
    double inv_scale_x = (double)dw / sw, inv_scale_y = (double)dh / sh;
    double scale_x = 1. / inv_scale_x, scale_y = 1. / inv_scale_y;
    int* xofs = (int*)malloc(sizeof(int) * dw);
    short* ialpha = (short*)malloc(sizeof(short) * 2 * dw);
    int* yofs = (int*)malloc(sizeof(int) * dh);
    short* ibeta = (short*)malloc(sizeof(short) * 2 * dh);
    int xmax = dw;
    for (int dx = 0; dx < dw; dx++) {
        float fx = (float)((dx + 0.5) * scale_x - 0.5);
        int sx = (int)floorf(fx);
        fx -= sx;
        if (sx < 0) { fx = 0; sx = 0; }
        if (sx + 1 >= sw) {
            if (dx < xmax) xmax = dx;
            if (sx >= sw - 1) { fx = 0; sx = sw - 1; }
        }
        xofs[dx] = sx;
        ialpha[dx * 2] = sat_short_f((1.f - fx) * RCOEF_SCALE);
        ialpha[dx * 2 + 1] = sat_short_f(fx * RCOEF_SCALE);
    }
    for (int dy = 0; dy < dh; dy++) {
        float fy = (float)((dy + 0.5) * scale_y - 0.5);
        int sy = (int)floorf(fy);
        fy -= sy;
        yofs[dy] = sy;
        ibeta[dy * 2] = sat_short_f((1.f - fy) * RCOEF_SCALE);
        ibeta[dy * 2 + 1] = sat_short_f(fy * RCOEF_SCALE);
    }
    int* D0 = (int*)malloc(sizeof(int) * dw);
    int* D1 = (int*)malloc(sizeof(int) * dw);
    for (int dy = 0; dy < dh; dy++) {
        int sy0 = yofs[dy];
        int r0 = sy0 < 0 ? 0 : (sy0 >= sh ? sh - 1 : sy0);
        int r1 = sy0 + 1 < 0 ? 0 : (sy0 + 1 >= sh ? sh - 1 : sy0 + 1);
        for (int k = 0; k < 2; k++) {
            const uint8_t* S = src + (size_t)(k ? r1 : r0) * sstep;
            int* D = k ? D1 : D0;
            for (int dx = 0; dx < dw; dx++) {
                int sx = xofs[dx];
                if (dx < xmax) D[dx] = S[sx] * ialpha[dx * 2] + S[sx + 1] * ialpha[dx * 2 + 1];
                else D[dx] = S[sx] * RCOEF_SCALE;
            }
        }
        int b0 = ibeta[dy * 2], b1 = ibeta[dy * 2 + 1];
        uint8_t* drow = dst + (size_t)dy * dstep;
        for (int dx = 0; dx < dw; dx++)
            drow[dx] = (uint8_t)((((b0 * (D0[dx] >> 4)) >> 16) + ((b1 * (D1[dx] >> 4)) >> 16) + 2) >> 2);
    }
    free(D0); free(D1); free(xofs); free(ialpha); free(yofs); free(ibeta);
}

/* ---- GaussianBlur(7x7, sigma 2) on CV_8U ------------------------------------
 * getGaussianKernel(7, 2, CV_32F) (float taps, double normalisation), then
 * createSeparableLinearFilter's 8U path: taps*256 -> int (cvRound), int row
 * pass, int column pass, FixedPtCastEx<int,uchar>(16): (v + 2^15) >> 16. */
void ora_gaussian7_taps(int taps[7])
{
    float cf[7];
    double sum = 0, scale2X = -0.5 / (2.0 * 2.0);
    for (int i = 0; i < 7; i++) {
        double x = i - 3.0;
        cf[i] = (float)exp(scale2X * x * x);
        sum += cf[i];
    }
    sum = 1. / sum;
    for (int i = 0; i < 7; i++) {
        cf[i] = (float)(cf[i] * sum);
        taps[i] = (int)lrintf(cf[i] * 256.0f);
    }
}

static inline int refl101(int p, int len)
{
    if (len == 1) return 0;
    while (p < 0 || p >= len) {
        if (p < 0) p = -p;
        else p = 2 * len - p - 2;
    }
    return p;
}

void ora_gaussian7_u8(const uint8_t* src, int sstep, int w, int h, uint8_t* dst, int dstep)
{
    int K[7];
    ora_gaussian7_taps(K);
    int* tmp = (int*)malloc(sizeof(int) * (size_t)w * h);
    for (int y = 0; y < h; y++)
        for (int x = 0; x < w; x++) {
            int s = 0;
            for (int k = -3; k <= 3; k++) s += K[k + 3] * src[(size_t)y * sstep + refl101(x + k, w)];
            tmp[(size_t)y * w + x] = s;
        }
    for (int y = 0; y < h; y++)
        for (int x = 0; x < w; x++) {
            int s = 0;
            for (int k = -3; k <= 3; k++) s += K[k + 3] * tmp[(size_t)refl101(y + k, h) * w + x];
            int v = (s + (1 << 15)) >> 16;
            dst[(size_t)y * dstep + x] = (uint8_t)(v > 255 ? 255 : (v < 0 ? 0 : v));
        }
    free(tmp);
}

/* Test helper: count floats in [lo, hi] where the sinf/cosf restatement and
 * the host libm differ (pins the restatement; tests/test_oracle_kat.py). */
long ora_check_sincos_vs_libm(float lo, float hi, long stride)
{
    long bad = 0;
    uint32_t u = f2u(lo);
    const uint32_t uhi = f2u(hi);
    if (stride < 1) stride = 1;
    for (; u <= uhi; u += (uint32_t)stride) {
        float f;
        memcpy(&f, &u, 4);
        volatile float vf = f;
        float c = cosf(vf), s = sinf(vf);
        if (f2u(c) != f2u(ora_cosf(f)) || f2u(s) != f2u(ora_sinf(f))) bad++;
        if (uhi - u < (uint32_t)stride) break;
    }
    return bad;
}

/* cv::undistortPoints(src, dst, K, D, noArray(), K) for CV_32FC2 points (OpenCV 3.2
 * imgproc/undistort.cpp, cvUndistortPoints), as Frame::UndistortKeyPoints and
 * Frame::ComputeImageBounds call it (Frame.cc:418-419, 445-447).  The camera matrix and the
 * coefficients are converted to double (cvConvert); with coefficients the distortion is
 * compensated by 5 fixed-point iterations (iters = 5); R is the identity and the new camera
 * matrix P = K enters as RR = P * I (cvMatMul, exact: every product by 0 or 1 is exact and
 * every added term +-0).  The tilt (k[12], k[13]) and thin-prism (k[8..11]) terms of the
 * 12/14-coefficient models are 0 for the 4/5/8-coefficient vectors ORB-SLAM2 passes; with an
 * identity tilt matrix the untilt step is exact, and their +0 terms are exact, so they are
 * not restated.  k: 8 doubles (k1 k2 p1 p2 k3 k4 k5 k6), zero-filled beyond the given count. */
void ora_undistort_points(const float* src, int n, const float K[9], const double k[8], int has_dist, float* dst)
{
    double A[3][3], RR[3][3];
    for (int r = 0; r < 3; r++)
        for (int c = 0; c < 3; c++) A[r][c] = (double)K[r * 3 + c];
    for (int r = 0; r < 3; r++)
        for (int c = 0; c < 3; c++) RR[r][c] = A[r][c];
    const int iters = has_dist ? 5 : 1;
    const double fx = A[0][0], fy = A[1][1];
    const double ifx = 1. / fx, ify = 1. / fy;
    const double cx = A[0][2], cy = A[1][2];
    for (int i = 0; i < n; i++) {
        double x = src[2 * i], y = src[2 * i + 1], x0, y0;
        x0 = x = (x - cx) * ifx;
        y0 = y = (y - cy) * ify;
        for (int j = 0; j < iters; j++) {
            double r2 = x * x + y * y;
            double icdist = (1 + ((k[7] * r2 + k[6]) * r2 + k[5]) * r2) / (1 + ((k[4] * r2 + k[1]) * r2 + k[0]) * r2);
            double deltaX = 2 * k[2] * x * y + k[3] * (r2 + 2 * x * x);
            double deltaY = k[2] * (r2 + 2 * y * y) + 2 * k[3] * x * y;
            x = (x0 - deltaX) * icdist;
            y = (y0 - deltaY) * icdist;
        }
        double xx = RR[0][0] * x + RR[0][1] * y + RR[0][2];
        double yy = RR[1][0] * x + RR[1][1] * y + RR[1][2];
        double ww = 1. / (RR[2][0] * x + RR[2][1] * y + RR[2][2]);
        x = xx * ww;
        y = yy * ww;
        dst[2 * i] = (float)x;
        dst[2 * i + 1] = (float)y;
    }
}
