/*
 * matchers2.c -- TEST INFRASTRUCTURE ONLY (see orb_oracle.h).
 * CPU restatement of the remaining ORBmatcher searches (reference src/ORBmatcher.cc):
 *   SearchByProjection(Frame&, KeyFrame*, set, th, ORBdist)   1472-1599  (relocalization)
 *   SearchByBoW(KeyFrame*, Frame&, vector<MapPoint*>&)          159-288
 *   SearchByBoW(KeyFrame*, KeyFrame*, vector<MapPoint*>&)       522-655
 *   SearchForInitialization(F1, F2, vbPrevMatched, vnMatches12, windowSize)  405-520
 *   SearchForTriangulation(KF1, KF2, F12, vMatchedPairs, bOnlyStereo)        657-823
 * Each is the reference loop written out sequentially over plain arrays.
 */
#include <limits.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "orb_oracle.h"

#define HISTO 30
#define TH_LOW 50

/* ComputeThreeMaxima (ORBmatcher.cc:1601-1642) over histogram bin counts */
static void three_maxima(const int* cnt, int* i1, int* i2, int* i3)
{
    int m1 = 0, m2 = 0, m3 = 0;
    *i1 = *i2 = *i3 = -1;
    for (int i = 0; i < HISTO; i++) {
        const int s = cnt[i];
        if (s > m1) { m3 = m2; m2 = m1; m1 = s; *i3 = *i2; *i2 = *i1; *i1 = i; }
        else if (s > m2) { m3 = m2; m2 = s; *i3 = *i2; *i2 = i; }
        else if (s > m3) { m3 = s; *i3 = i; }
    }
    if (m2 < 0.1f * (float)m1) { *i2 = -1; *i3 = -1; }
    else if (m3 < 0.1f * (float)m1) { *i3 = -1; }
}

static int rot_bin(float a1, float a2)
{
    const float factor = 1.0f / HISTO;
    float rot = a1 - a2;
    if (rot < 0.0) rot += 360.0f;
    int bin = (int)roundf(rot * factor);
    if (bin == HISTO) bin = 0;
    return bin;
}

/* histogram as (bin, value) records in insertion order */
typedef struct { int* bin; int* val; int n; int cnt[HISTO]; } hist_t;

static void hist_init(hist_t* h, int cap)
{
    h->bin = (int*)malloc(sizeof(int) * (cap + 1));
    h->val = (int*)malloc(sizeof(int) * (cap + 1));
    h->n = 0;
    memset(h->cnt, 0, sizeof(h->cnt));
}

static void hist_push(hist_t* h, int bin, int v)
{
    h->bin[h->n] = bin;
    h->val[h->n++] = v;
    h->cnt[bin]++;
}

static void hist_free(hist_t* h) { free(h->bin); free(h->val); }

/* Rcw*X + tcw as one cv::gemm: f64 accumulation, one rounding */
static float gemm_row3(const float* T, int r, const float* X)
{
    double s = (double)T[r * 4 + 0] * X[0] + (double)T[r * 4 + 1] * X[1] + (double)T[r * 4 + 2] * X[2];
    return (float)(s + (double)T[r * 4 + 3]);
}

/* -Rcw.t()*tcw (camera centre) as one cv::gemm with alpha = -1 */
static void camera_center(const float* T, float* O)
{
    for (int i = 0; i < 3; i++) {
        double s = (double)T[0 * 4 + i] * T[3] + (double)T[1 * 4 + i] * T[7] + (double)T[2 * 4 + i] * T[11];
        O[i] = (float)(s * -1.0);
    }
}

/* fdlibm __ieee754_log as an IEEE operation sequence (the GPU's detmath::log_d, same order):
 * the device's stand-in for glibc logf in PredictScale; ora_predict_scale_mismatches checks
 * the two agree on every float of a range. */
double ora_det_log(double x)
{
    const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10;
    const double Lg1 = 6.666666666666735130e-01, Lg2 = 3.999999999940941908e-01, Lg3 = 2.857142874366239149e-01,
                 Lg4 = 2.222219843214978396e-01, Lg5 = 1.818357216161805012e-01, Lg6 = 1.531383769920937332e-01,
                 Lg7 = 1.479819860511658591e-01;
    if (!(x > 0.0)) return x == 0.0 ? -HUGE_VAL : (x - x) / 0.0;
    if (x > 1.79769313486231570815e+308) return x;
    unsigned long long bits;
    memcpy(&bits, &x, 8);
    int hx = (int)(bits >> 32);
    int k = 0;
    if (hx < 0x00100000) {
        x *= 1.80143985094819840000e+16;
        k -= 54;
        memcpy(&bits, &x, 8);
        hx = (int)(bits >> 32);
    }
    k += (hx >> 20) - 1023;
    hx &= 0x000fffff;
    const int i0 = (hx + 0x95f64) & 0x100000;
    bits = ((unsigned long long)(unsigned)(hx | (i0 ^ 0x3ff00000)) << 32) | (bits & 0xffffffffull);
    memcpy(&x, &bits, 8);
    k += (i0 >> 20);
    const double f = x - 1.0;
    const double dk = (double)k;
    if ((0x000fffff & (2 + hx)) < 3) {
        if (f == 0.0) return k == 0 ? 0.0 : dk * ln2_hi + dk * ln2_lo;
        const double R = f * f * (0.5 - 0.33333333333333333 * f);
        return k == 0 ? f - R : dk * ln2_hi - ((R - dk * ln2_lo) - f);
    }
    const double s = f / (2.0 + f);
    const double z = s * s;
    int i = hx - 0x6147a;
    const double w = z * z;
    const int j = 0x6b851 - hx;
    const double t1 = w * (Lg2 + w * (Lg4 + w * Lg6));
    const double t2 = z * (Lg1 + w * (Lg3 + w * (Lg5 + w * Lg7)));
    i |= j;
    const double R = t2 + t1;
    if (i > 0) {
        const double hfsq = 0.5 * f * f;
        return k == 0 ? f - (hfsq - s * (hfsq + R)) : dk * ln2_hi - ((hfsq - (s * (hfsq + R) + dk * ln2_lo)) - f);
    }
    return k == 0 ? f - s * (f - R) : dk * ln2_hi - ((s * (f - R) - dk * ln2_lo) - f);
}

/* Every float r in [lo, hi]: ceilf(logf(r) / lsf) (glibc, the reference's PredictScale) vs
 * ceilf((float)ora_det_log(r) / lsf); returns the number of r where the levels differ. */
long long ora_predict_scale_mismatches(float lo, float hi, float lsf, long long* n_checked, long long* n_logf_diff)
{
    long long bad = 0, n = 0, d = 0;
    for (float r = lo; r <= hi; r = nextafterf(r, INFINITY)) {
        const float a = logf(r), b = (float)ora_det_log((double)r);
        if (a != b) d++;
        if (ceilf(a / lsf) != ceilf(b / lsf)) bad++;
        n++;
    }
    *n_checked = n;
    *n_logf_diff = d;
    return bad;
}

/* MapPoint::PredictScale (MapPoint.cc:402-417) */
static int predict_scale(float maxDistance, float currentDist, float logScaleFactor, int nlevels)
{
    const float ratio = maxDistance / currentDist;
    int nScale = (int)ceilf(logf(ratio) / logScaleFactor);
    if (nScale < 0) nScale = 0;
    else if (nScale >= nlevels) nScale = nlevels - 1;
    return nScale;
}

/* Frame::isInFrustum(pMP, viewingCosLimit) (Frame.cc:269-325) for n map points, with
 * MapPoint::GetMax/MinDistanceInvariance (1.2f / 0.8f, MapPoint.cc:373-383) and PredictScale
 * (glibc logf, as the reference).  Pc and mOw as one cv::gemm each (f64 accumulation, one
 * rounding), cv::norm and Mat::dot accumulated in double.  Returns the points in view. */
int ora_is_in_frustum(const float* Tcw, float fx, float fy, float cx, float cy, float mbf, float minX, float maxX,
                      float minY, float maxY, int nlevels, float logScaleFactor, int n, const float* pos,
                      const float* maxDist, const float* minDist, const float* normal, const uint8_t* skip,
                      float viewingCosLimit, uint8_t* inView, float* projX, float* projXR, float* projY, int* level,
                      float* viewCos)
{
    float Ow[3];
    camera_center(Tcw, Ow);
    int nv = 0;
    for (int j = 0; j < n; j++) {
        inView[j] = 0;
        if (skip[j]) continue;
        const float* P = pos + 3 * (size_t)j;
        const float PcX = gemm_row3(Tcw, 0, P), PcY = gemm_row3(Tcw, 1, P), PcZ = gemm_row3(Tcw, 2, P);
        if (PcZ < 0.0f) continue;
        const float invz = 1.0f / PcZ;
        const float u = fx * PcX * invz + cx;
        const float v = fy * PcY * invz + cy;
        if (u < minX || u > maxX) continue;
        if (v < minY || v > maxY) continue;
        const float maxDistance = 1.2f * maxDist[j];
        const float minDistance = 0.8f * minDist[j];
        const float PO[3] = {P[0] - Ow[0], P[1] - Ow[1], P[2] - Ow[2]};
        const double s2 = ((double)PO[0] * PO[0] + (double)PO[1] * PO[1]) + (double)PO[2] * PO[2];
        const float dist = (float)sqrt(s2);
        if (dist < minDistance || dist > maxDistance) continue;
        const float* Pn = normal + 3 * (size_t)j;
        const double dot = ((double)PO[0] * Pn[0] + (double)PO[1] * Pn[1]) + (double)PO[2] * Pn[2];
        const float vc = (float)(dot / (double)dist);
        if (vc < viewingCosLimit) continue;
        inView[j] = 1;
        projX[j] = u;
        projXR[j] = u - mbf * invz;
        projY[j] = v;
        level[j] = predict_scale(maxDist[j], dist, logScaleFactor, nlevels);
        viewCos[j] = vc;
        nv++;
    }
    return nv;
}

int ora_search_by_projection_kf(const ora_frame* F, const float* Tcw, const float* K, int* curMP, int n, const int* kfMP,
                                const uint8_t* skip, const float* kfAngle, const float* mpPos, const uint8_t* mpDesc,
                                const float* mpMaxDist, const float* mpMinDist, float logScaleFactor, float th,
                                int ORBdist, int checkOri)
{
    int nmatches = 0;
    float Ow[3];
    camera_center(Tcw, Ow);
    hist_t H;
    hist_init(&H, n);
    int* cand = (int*)malloc(sizeof(int) * (F->N + 1));
    for (int i = 0; i < n; i++) {
        const int mp = kfMP[i];
        if (mp < 0 || skip[i]) continue;
        const float* X = mpPos + 3 * (size_t)mp;
        const float xc = gemm_row3(Tcw, 0, X), yc = gemm_row3(Tcw, 1, X), zc = gemm_row3(Tcw, 2, X);
        const float invzc = (float)(1.0 / (double)zc);
        const float u = K[0] * xc * invzc + K[2];
        const float v = K[1] * yc * invzc + K[3];
        if (u < F->minX || u > F->maxX) continue;
        if (v < F->minY || v > F->maxY) continue;
        const float PO[3] = {X[0] - Ow[0], X[1] - Ow[1], X[2] - Ow[2]};
        double s2 = 0;
        for (int k = 0; k < 3; k++) s2 += (double)PO[k] * (double)PO[k];
        const float dist3D = (float)sqrt(s2);
        const float maxDistance = 1.2f * mpMaxDist[mp], minDistance = 0.8f * mpMinDist[mp];
        if (dist3D < minDistance || dist3D > maxDistance) continue;
        const int nPredictedLevel = predict_scale(mpMaxDist[mp], dist3D, logScaleFactor, F->nlevels);
        const float radius = th * F->scaleFactors[nPredictedLevel];
        const int nc = ora_frame_features_in_area(F, u, v, radius, nPredictedLevel - 1, nPredictedLevel + 1, cand,
                                                  F->N);
        if (nc == 0) continue;
        const uint8_t* dMP = mpDesc + 32 * (size_t)mp;
        int bestDist = 256, bestIdx2 = -1;
        for (int c = 0; c < nc; c++) {
            const int i2 = cand[c];
            if (curMP[i2] >= 0) continue;
            const int dist = ora_descriptor_distance(dMP, F->desc + 32 * (size_t)i2);
            if (dist < bestDist) { bestDist = dist; bestIdx2 = i2; }
        }
        if (bestDist <= ORBdist) {
            curMP[bestIdx2] = mp;
            nmatches++;
            if (checkOri) hist_push(&H, rot_bin(kfAngle[i], F->kpsUn[bestIdx2].angle), bestIdx2);
        }
    }
    if (checkOri) {
        int i1, i2, i3;
        three_maxima(H.cnt, &i1, &i2, &i3);
        for (int k = 0; k < H.n; k++)
            if (H.bin[k] != i1 && H.bin[k] != i2 && H.bin[k] != i3) { curMP[H.val[k]] = -1; nmatches--; }
    }
    hist_free(&H);
    free(cand);
    return nmatches;
}

/* The two SearchByBoW loops share one shape: node merge, queries (side 1) in node order,
 * candidates (side 2) in node order, best / second, greedy occupancy of side 2. */
static int bow_common(const ora_featvec* fv1, const uint8_t* ok1, const uint8_t* desc1, const float* ang1,
                      const ora_featvec* fv2, const uint8_t* ok2, const uint8_t* desc2, const float* ang2, int n1,
                      int n2, int le_low, float nnratio, int checkOri, int* out12, int* taken2)
{
    int nmatches = 0;
    hist_t H;
    hist_init(&H, n1 + n2);
    int a = 0, b = 0;
    while (a < fv1->n_nodes && b < fv2->n_nodes) {
        if (fv1->node_id[a] == fv2->node_id[b]) {
            for (int q = fv1->start[a]; q < fv1->start[a + 1]; q++) {
                const int idx1 = fv1->feat[q];
                if (!ok1[idx1]) continue;
                const uint8_t* d1 = desc1 + 32 * (size_t)idx1;
                int best1 = 256, best2 = 256, bestIdx2 = -1;
                for (int c = fv2->start[b]; c < fv2->start[b + 1]; c++) {
                    const int idx2 = fv2->feat[c];
                    if (taken2[idx2] || !ok2[idx2]) continue;
                    const int dist = ora_descriptor_distance(d1, desc2 + 32 * (size_t)idx2);
                    if (dist < best1) { best2 = best1; best1 = dist; bestIdx2 = idx2; }
                    else if (dist < best2) best2 = dist;
                }
                const int pass = le_low ? (best1 <= TH_LOW) : (best1 < TH_LOW);
                if (pass && (float)best1 < nnratio * (float)best2) {
                    out12[idx1] = bestIdx2;
                    taken2[bestIdx2] = 1;
                    if (checkOri) hist_push(&H, rot_bin(ang1[idx1], ang2[bestIdx2]), idx1);
                    nmatches++;
                }
            }
            a++;
            b++;
        } else if (fv1->node_id[a] < fv2->node_id[b]) {
            a++;
        } else {
            b++;
        }
    }
    if (checkOri) {
        int i1, i2, i3;
        three_maxima(H.cnt, &i1, &i2, &i3);
        for (int k = 0; k < H.n; k++)
            if (H.bin[k] != i1 && H.bin[k] != i2 && H.bin[k] != i3) { out12[H.val[k]] = -1; nmatches--; }
    }
    hist_free(&H);
    (void)n2;
    return nmatches;
}

int ora_search_by_bow_frame(const ora_featvec* fvKF, const int* kfMP, const uint8_t* kfMPbad, const uint8_t* kfDesc,
                            const float* kfAngle, int nKF, const ora_featvec* fvF, const uint8_t* fDesc,
                            const float* fAngle, int NF, float nnratio, int checkOri, int* matchesF)
{
    /* queries: keyframe features with a good map point; candidates: every frame feature;
     * output indexed by the frame feature (vpMapPointMatches[bestIdxF] = pMP) */
    uint8_t* ok1 = (uint8_t*)malloc(nKF + 1);
    uint8_t* ok2 = (uint8_t*)malloc(NF + 1);
    int* m12 = (int*)malloc(sizeof(int) * (nKF + 1));
    int* taken = (int*)calloc(NF + 1, sizeof(int));
    for (int i = 0; i < nKF; i++) { ok1[i] = kfMP[i] >= 0 && !kfMPbad[i]; m12[i] = -1; }
    for (int i = 0; i < NF; i++) ok2[i] = 1;
    /* KF->F orientation uses kp.angle - F.mvKeys[bestIdxF].angle (ORBmatcher.cc:231) */
    const int n = bow_common(fvKF, ok1, kfDesc, kfAngle, fvF, ok2, fDesc, fAngle, nKF, NF, 1, nnratio, checkOri, m12,
                             taken);
    for (int i = 0; i < NF; i++) matchesF[i] = -1;
    for (int i = 0; i < nKF; i++)
        if (m12[i] >= 0) matchesF[m12[i]] = kfMP[i];
    free(ok1); free(ok2); free(m12); free(taken);
    return n;
}

int ora_search_by_bow_kf(const ora_featvec* fv1, const int* mp1, const uint8_t* bad1, const uint8_t* desc1,
                         const float* ang1, int n1, const ora_featvec* fv2, const int* mp2, const uint8_t* bad2,
                         const uint8_t* desc2, const float* ang2, int n2, float nnratio, int checkOri, int* matches12)
{
    uint8_t* ok1 = (uint8_t*)malloc(n1 + 1);
    uint8_t* ok2 = (uint8_t*)malloc(n2 + 1);
    int* m12 = (int*)malloc(sizeof(int) * (n1 + 1));
    int* taken = (int*)calloc(n2 + 1, sizeof(int));
    for (int i = 0; i < n1; i++) { ok1[i] = mp1[i] >= 0 && !bad1[i]; m12[i] = -1; }
    for (int i = 0; i < n2; i++) ok2[i] = mp2[i] >= 0 && !bad2[i];
    const int n = bow_common(fv1, ok1, desc1, ang1, fv2, ok2, desc2, ang2, n1, n2, 0, nnratio, checkOri, m12, taken);
    for (int i = 0; i < n1; i++) matches12[i] = m12[i] >= 0 ? mp2[m12[i]] : -1;
    free(ok1); free(ok2); free(m12); free(taken);
    return n;
}

int ora_search_for_initialization(const ora_frame* F1, const ora_frame* F2, float* prevMatched, int* matches12,
                                  int windowSize, float nnratio, int checkOri)
{
    const int N1 = F1->N, N2 = F2->N;
    int nmatches = 0;
    int* dist21 = (int*)malloc(sizeof(int) * (N2 + 1));
    int* m21 = (int*)malloc(sizeof(int) * (N2 + 1));
    int* cand = (int*)malloc(sizeof(int) * (N2 + 1));
    for (int i = 0; i < N2; i++) { dist21[i] = INT_MAX; m21[i] = -1; }
    for (int i = 0; i < N1; i++) matches12[i] = -1;
    hist_t H;
    hist_init(&H, N1);
    for (int i1 = 0; i1 < N1; i1++) {
        const int level1 = F1->kpsUn[i1].octave;
        if (level1 > 0) continue;
        const int nc = ora_frame_features_in_area(F2, prevMatched[2 * i1], prevMatched[2 * i1 + 1], (float)windowSize,
                                                  level1, level1, cand, N2);
        if (nc == 0) continue;
        const uint8_t* d1 = F1->desc + 32 * (size_t)i1;
        int bestDist = INT_MAX, bestDist2 = INT_MAX, bestIdx2 = -1;
        for (int c = 0; c < nc; c++) {
            const int i2 = cand[c];
            const int dist = ora_descriptor_distance(d1, F2->desc + 32 * (size_t)i2);
            if (dist21[i2] <= dist) continue;
            if (dist < bestDist) { bestDist2 = bestDist; bestDist = dist; bestIdx2 = i2; }
            else if (dist < bestDist2) bestDist2 = dist;
        }
        if (bestDist <= TH_LOW) {
            if (bestDist < (float)bestDist2 * nnratio) {
                if (m21[bestIdx2] >= 0) { matches12[m21[bestIdx2]] = -1; nmatches--; }
                matches12[i1] = bestIdx2;
                m21[bestIdx2] = i1;
                dist21[bestIdx2] = bestDist;
                nmatches++;
                if (checkOri) hist_push(&H, rot_bin(F1->kpsUn[i1].angle, F2->kpsUn[bestIdx2].angle), i1);
            }
        }
    }
    if (checkOri) {
        int i1, i2, i3;
        three_maxima(H.cnt, &i1, &i2, &i3);
        for (int k = 0; k < H.n; k++) {
            if (H.bin[k] == i1 || H.bin[k] == i2 || H.bin[k] == i3) continue;
            const int idx1 = H.val[k];
            if (matches12[idx1] >= 0) { matches12[idx1] = -1; nmatches--; }
        }
    }
    for (int i1 = 0; i1 < N1; i1++)
        if (matches12[i1] >= 0) {
            prevMatched[2 * i1] = F2->kpsUn[matches12[i1]].x;
            prevMatched[2 * i1 + 1] = F2->kpsUn[matches12[i1]].y;
        }
    hist_free(&H);
    free(dist21); free(m21); free(cand);
    return nmatches;
}

/* CheckDistEpipolarLine (ORBmatcher.cc:140-157) */
static int epipolar_ok(const ora_kp* kp1, const ora_kp* kp2, const float* F12, float sigma2)
{
    const float a = kp1->x * F12[0 * 3 + 0] + kp1->y * F12[1 * 3 + 0] + F12[2 * 3 + 0];
    const float b = kp1->x * F12[0 * 3 + 1] + kp1->y * F12[1 * 3 + 1] + F12[2 * 3 + 1];
    const float c = kp1->x * F12[0 * 3 + 2] + kp1->y * F12[1 * 3 + 2] + F12[2 * 3 + 2];
    const float num = a * kp2->x + b * kp2->y + c;
    const float den = a * a + b * b;
    if (den == 0) return 0;
    const float dsqr = num * num / den;
    return dsqr < 3.84 * sigma2;
}

int ora_search_for_triangulation(const ora_featvec* fv1, const ora_kp* k1, const uint8_t* d1, const float* uR1,
                                 const uint8_t* hasMP1, int n1, const float* Tcw1, const ora_featvec* fv2,
                                 const ora_kp* k2, const uint8_t* d2, const float* uR2, const uint8_t* hasMP2, int n2,
                                 const float* Tcw2, const float* K2, const float* scale2, const float* sigma2_2,
                                 const float* F12, int bOnlyStereo, int checkOri, int* pairs, int cap)
{
    float Cw[3], C2[3];
    camera_center(Tcw1, Cw);
    for (int r = 0; r < 3; r++) C2[r] = gemm_row3(Tcw2, r, Cw);
    const float invz = 1.0f / C2[2];
    const float ex = K2[0] * C2[0] * invz + K2[2];
    const float ey = K2[1] * C2[1] * invz + K2[3];
    int nmatches = 0;
    int* m12 = (int*)malloc(sizeof(int) * (n1 + 1));
    for (int i = 0; i < n1; i++) m12[i] = -1;
    hist_t H;
    hist_init(&H, n1);
    int a = 0, b = 0;
    while (a < fv1->n_nodes && b < fv2->n_nodes) {
        if (fv1->node_id[a] == fv2->node_id[b]) {
            for (int q = fv1->start[a]; q < fv1->start[a + 1]; q++) {
                const int idx1 = fv1->feat[q];
                if (hasMP1[idx1]) continue;
                const int bStereo1 = uR1[idx1] >= 0;
                if (bOnlyStereo && !bStereo1) continue;
                const ora_kp* kp1 = &k1[idx1];
                int bestDist = TH_LOW, bestIdx2 = -1;
                for (int c = fv2->start[b]; c < fv2->start[b + 1]; c++) {
                    const int idx2 = fv2->feat[c];
                    if (hasMP2[idx2]) continue;   /* vbMatched2 is never set (reference quirk) */
                    const int bStereo2 = uR2[idx2] >= 0;
                    if (bOnlyStereo && !bStereo2) continue;
                    const int dist = ora_descriptor_distance(d1 + 32 * (size_t)idx1, d2 + 32 * (size_t)idx2);
                    if (dist > TH_LOW || dist > bestDist) continue;
                    const ora_kp* kp2 = &k2[idx2];
                    if (!bStereo1 && !bStereo2) {
                        const float distex = ex - kp2->x, distey = ey - kp2->y;
                        if (distex * distex + distey * distey < 100 * scale2[kp2->octave]) continue;
                    }
                    if (epipolar_ok(kp1, kp2, F12, sigma2_2[kp2->octave])) { bestIdx2 = idx2; bestDist = dist; }
                }
                if (bestIdx2 >= 0) {
                    m12[idx1] = bestIdx2;
                    nmatches++;
                    if (checkOri) hist_push(&H, rot_bin(kp1->angle, k2[bestIdx2].angle), idx1);
                }
            }
            a++;
            b++;
        } else if (fv1->node_id[a] < fv2->node_id[b]) {
            a++;
        } else {
            b++;
        }
    }
    if (checkOri) {
        int i1, i2, i3;
        three_maxima(H.cnt, &i1, &i2, &i3);
        for (int k = 0; k < H.n; k++)
            if (H.bin[k] != i1 && H.bin[k] != i2 && H.bin[k] != i3) { m12[H.val[k]] = -1; nmatches--; }
    }
    int np = 0;
    for (int i = 0; i < n1; i++)
        if (m12[i] >= 0) {
            if (np < cap) { pairs[2 * np] = i; pairs[2 * np + 1] = m12[i]; }
            np++;
        }
    hist_free(&H);
    free(m12);
    return nmatches;
}
