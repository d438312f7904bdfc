/*
 * matchers3.c -- TEST INFRASTRUCTURE ONLY (parity oracle).
 *
 * Restatement of the LocalMapping / LoopClosing projection searches of
 * ORB_SLAM2::ORBmatcher (reference src/ORBmatcher.cc):
 *   SearchByProjection(KeyFrame*, Scw, vpPoints, vpMatched, th)      290-403
 *   Fuse(KeyFrame*, vpMapPoints, th)                                 825-975
 *   Fuse(KeyFrame*, Scw, vpPoints, th, vpReplacePoint)               977-1100
 *   SearchBySim3(pKF1, pKF2, vpMatches12, s12, R12, t12, th)         1102-1326
 * KeyFrame::GetFeaturesInArea (KeyFrame.cc:569-608) has no level filter; the
 * [pred-1, pred] octave test of every search is applied in the candidate loop.
 * cv::Mat semantics (unpinned; the same ones as sim3.c / matchers2.c):
 *   A*x + b (gemm)   -> double accumulation, one rounding to float
 *   -A.t()*b         -> gemm with alpha = -1
 *   Mat / s, s * Mat -> convertTo: float multiply by (float)(1.0 / s) resp. (float)s
 *   Mat::dot, norm   -> double accumulation of double products
 * Fuse's map mutation (951-970) is the caller's: the oracle returns, per map
 * point, the keyframe keypoint the reference would fuse it with (or -1); the
 * selection never depends on the mutation (no occupancy test in Fuse).
 */
#include "orb_oracle.h"
#include <limits.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

#define TH_LOW 50
#define TH_HIGH 100

typedef struct {
    float R[9], t[3], O[3];
} simpose;

static float gemm3(const float* R, const float* t, int r, const float* X)
{
    double s = (double)R[r * 3 + 0] * X[0] + (double)R[r * 3 + 1] * X[1] + (double)R[r * 3 + 2] * X[2];
    return (float)(s + (double)t[r]);
}

static void center_of(simpose* P)
{
    for (int i = 0; i < 3; i++) {
        double s = (double)P->R[0 * 3 + i] * P->t[0] + (double)P->R[1 * 3 + i] * P->t[1] +
                   (double)P->R[2 * 3 + i] * P->t[2];
        P->O[i] = (float)(s * -1.0);
    }
}

/* Rcw, tcw of a 4x4 pose, Ow = -Rcw^T tcw (KeyFrame::SetPose) */
static void pose_of_T(const float* T, simpose* P)
{
    for (int r = 0; r < 3; r++) {
        for (int c = 0; c < 3; c++) P->R[r * 3 + c] = T[r * 4 + c];
        P->t[r] = T[r * 4 + 3];
    }
    center_of(P);
}

/* ORBmatcher.cc:298-303: scw = sqrt(row0 . row0), Rcw = sRcw / scw, tcw = t / scw */
static void pose_of_Scw(const float* S, simpose* P)
{
    const double d = (double)S[0] * S[0] + (double)S[1] * S[1] + (double)S[2] * S[2];
    const float scw = (float)sqrt(d);
    const float a = (float)(1.0 / (double)scw);
    for (int r = 0; r < 3; r++) {
        for (int c = 0; c < 3; c++) P->R[r * 3 + c] = S[r * 4 + c] * a + 0.0f;
        P->t[r] = S[r * 4 + 3] * a + 0.0f;
    }
    center_of(P);
}

static int predict_scale(float maxDistance, float currentDist, float logScaleFactor, int nlevels)
{
    const float ratio = maxDistance / currentDist;
    int nScale = (int)ceilf(logf(ratio) / logScaleFactor);
    if (nScale < 0) nScale = 0;
    else if (nScale >= nlevels) nScale = nlevels - 1;
    return nScale;
}

static int in_image(const ora_frame* F, float u, float v)
{
    return u >= F->minX && u < F->maxX && v >= F->minY && v < F->maxY;   /* KeyFrame::IsInImage */
}

static float norm3(const float* v)
{
    double s = 0;
    for (int k = 0; k < 3; k++) s += (double)v[k] * (double)v[k];
    return (float)sqrt(s);
}

static double dot3d(const float* a, const float* b)
{
    return (double)a[0] * b[0] + (double)a[1] * b[1] + (double)a[2] * b[2];
}

int ora_search_by_projection_sim3(const ora_frame* KF, const float* K, const float* Scw, int np, const float* pos,
                                  const uint8_t* desc, const float* maxD, const float* minD, const float* normal,
                                  const uint8_t* skip, float logScaleFactor, int th, int* matched)
{
    simpose P;
    pose_of_Scw(Scw, &P);
    int* cand = (int*)malloc(sizeof(int) * (KF->N + 1));
    int nmatches = 0;
    for (int i = 0; i < np; i++) {
        if (skip[i]) continue;
        const float* X = pos + 3 * (size_t)i;
        const float xc = gemm3(P.R, P.t, 0, X), yc = gemm3(P.R, P.t, 1, X), zc = gemm3(P.R, P.t, 2, X);
        if (zc < 0.0) continue;
        const float invz = 1 / zc;
        const float x = xc * invz, y = yc * invz;
        const float u = K[0] * x + K[2], v = K[1] * y + K[3];
        if (!in_image(KF, u, v)) continue;
        const float maxDistance = 1.2f * maxD[i], minDistance = 0.8f * minD[i];
        const float PO[3] = {X[0] - P.O[0], X[1] - P.O[1], X[2] - P.O[2]};
        const float dist = norm3(PO);
        if (dist < minDistance || dist > maxDistance) continue;
        if (dot3d(PO, normal + 3 * (size_t)i) < 0.5 * dist) continue;
        const int lvl = predict_scale(maxD[i], dist, logScaleFactor, KF->nlevels);
        const float radius = th * KF->scaleFactors[lvl];
        const int nc = ora_frame_features_in_area(KF, u, v, radius, -1, -1, cand, KF->N);
        if (nc == 0) continue;
        int bestDist = 256, bestIdx = -1;
        for (int k = 0; k < nc; k++) {
            const int idx = cand[k];
            if (matched[idx] >= 0) continue;
            const int kpLevel = KF->kpsUn[idx].octave;
            if (kpLevel < lvl - 1 || kpLevel > lvl) continue;
            const int d = ora_descriptor_distance(desc + 32 * (size_t)i, KF->desc + 32 * (size_t)idx);
            if (d < bestDist) { bestDist = d; bestIdx = idx; }
        }
        if (bestDist <= TH_LOW) {
            matched[bestIdx] = i;
            nmatches++;
        }
    }
    free(cand);
    return nmatches;
}

/* shared body of the two Fuse variants: best keypoint per point or -1 */
static int fuse_body(const ora_frame* KF, const float* K5, const simpose* P, int sim3, int np, const float* pos,
                     const uint8_t* desc, const float* maxD, const float* minD, const float* normal,
                     const uint8_t* skip, float logScaleFactor, float th, int* best)
{
    int* cand = (int*)malloc(sizeof(int) * (KF->N + 1));
    int nFused = 0;
    for (int i = 0; i < np; i++) {
        best[i] = -1;
        if (skip[i]) continue;
        const float* X = pos + 3 * (size_t)i;
        const float xc = gemm3(P->R, P->t, 0, X), yc = gemm3(P->R, P->t, 1, X), zc = gemm3(P->R, P->t, 2, X);
        if (zc < 0.0f) continue;
        const float invz = sim3 ? (float)(1.0 / (double)zc) : 1 / zc;
        const float x = xc * invz, y = yc * invz;
        const float u = K5[0] * x + K5[2], v = K5[1] * y + K5[3];
        if (!in_image(KF, u, v)) continue;
        const float ur = u - K5[4] * invz;
        const float maxDistance = 1.2f * maxD[i], minDistance = 0.8f * minD[i];
        const float PO[3] = {X[0] - P->O[0], X[1] - P->O[1], X[2] - P->O[2]};
        const float dist3D = norm3(PO);
        if (dist3D < minDistance || dist3D > maxDistance) continue;
        if (dot3d(PO, normal + 3 * (size_t)i) < 0.5 * dist3D) continue;
        const int lvl = predict_scale(maxD[i], dist3D, logScaleFactor, KF->nlevels);
        const float radius = th * KF->scaleFactors[lvl];
        const int nc = ora_frame_features_in_area(KF, u, v, radius, -1, -1, cand, KF->N);
        if (nc == 0) continue;
        int bestDist = sim3 ? INT_MAX : 256, bestIdx = -1;
        for (int k = 0; k < nc; k++) {
            const int idx = cand[k];
            const ora_kp* kp = &KF->kpsUn[idx];
            const int kpLevel = kp->octave;
            if (kpLevel < lvl - 1 || kpLevel > lvl) continue;
            if (!sim3) {   /* reprojection gate, ORBmatcher.cc:914-938 */
                const float s2 = KF->scaleFactors[kpLevel] * KF->scaleFactors[kpLevel];
                const float invSigma2 = 1.0f / s2;
                const float ex = u - kp->x, ey = v - kp->y;
                if (KF->uRight && KF->uRight[idx] >= 0) {
                    const float er = ur - KF->uRight[idx];
                    const float e2 = ex * ex + ey * ey + er * er;
                    if (e2 * invSigma2 > 7.8) continue;
                } else {
                    const float e2 = ex * ex + ey * ey;
                    if (e2 * invSigma2 > 5.99) continue;
                }
            }
            const int d = ora_descriptor_distance(desc + 32 * (size_t)i, KF->desc + 32 * (size_t)idx);
            if (d < bestDist) { bestDist = d; bestIdx = idx; }
        }
        if (bestDist <= TH_LOW) {
            best[i] = bestIdx;
            nFused++;
        }
    }
    free(cand);
    return nFused;
}

int ora_fuse(const ora_frame* KF, const float* Tcw, const float* K5, int np, const float* pos, const uint8_t* desc,
             const float* maxD, const float* minD, const float* normal, const uint8_t* skip, float logScaleFactor,
             float th, int* best)
{
    simpose P;
    pose_of_T(Tcw, &P);
    return fuse_body(KF, K5, &P, 0, np, pos, desc, maxD, minD, normal, skip, logScaleFactor, th, best);
}

int ora_fuse_sim3(const ora_frame* KF, const float* K4, const float* Scw, int np, const float* pos,
                  const uint8_t* desc, const float* maxD, const float* minD, const float* normal, const uint8_t* skip,
                  float logScaleFactor, float th, int* best)
{
    simpose P;
    pose_of_Scw(Scw, &P);
    const float K5[5] = {K4[0], K4[1], K4[2], K4[3], 0.0f};
    return fuse_body(KF, K5, &P, 1, np, pos, desc, maxD, minD, normal, skip, logScaleFactor, th, best);
}

/* one direction of SearchBySim3: points of side A (pose Aw), mapped by (sR, t) into side B */
static void sim3_direction(const ora_frame* B, const float* K, const simpose* Aw, const float* sR, const float* t,
                           int NA, const int* mpA, const uint8_t* matchedA, const float* pos, const uint8_t* desc,
                           const float* maxD, const float* minD, const uint8_t* bad, float logScaleFactor, float th,
                           int* vnMatch, int* cand)
{
    for (int i = 0; i < NA; i++) {
        vnMatch[i] = -1;
        const int mp = mpA[i];
        if (mp < 0 || matchedA[i]) continue;
        if (bad[mp]) continue;
        const float* X = pos + 3 * (size_t)mp;
        float c1[3], c2[3];
        for (int r = 0; r < 3; r++) c1[r] = gemm3(Aw->R, Aw->t, r, X);
        for (int r = 0; r < 3; r++) c2[r] = gemm3(sR, t, r, c1);
        if (c2[2] < 0.0) continue;
        const float invz = (float)(1.0 / (double)c2[2]);
        const float x = c2[0] * invz, y = c2[1] * invz;
        const float u = K[0] * x + K[2], v = K[1] * y + K[3];
        if (!in_image(B, u, v)) continue;
        const float maxDistance = 1.2f * maxD[mp], minDistance = 0.8f * minD[mp];
        const float dist3D = norm3(c2);
        if (dist3D < minDistance || dist3D > maxDistance) continue;
        const int lvl = predict_scale(maxD[mp], dist3D, logScaleFactor, B->nlevels);
        const float radius = th * B->scaleFactors[lvl];
        const int nc = ora_frame_features_in_area(B, u, v, radius, -1, -1, cand, B->N);
        if (nc == 0) continue;
        int bestDist = INT_MAX, bestIdx = -1;
        for (int k = 0; k < nc; k++) {
            const int idx = cand[k];
            const int oct = B->kpsUn[idx].octave;
            if (oct < lvl - 1 || oct > lvl) continue;
            const int d = ora_descriptor_distance(desc + 32 * (size_t)mp, B->desc + 32 * (size_t)idx);
            if (d < bestDist) { bestDist = d; bestIdx = idx; }
        }
        if (bestDist <= TH_HIGH) vnMatch[i] = bestIdx;
    }
}

/* matches12 (N1, in/out): -1 none; >= 0 KF2 keypoint index of the matched map point;
 * -2 matched to a point not observed in KF2.  New agreements write the KF2 index. */
int ora_search_by_sim3(const ora_frame* KF1, const float* T1w, const int* mp1, const ora_frame* KF2, const float* T2w,
                       const int* mp2, const float* K, const float* pos, const uint8_t* desc, const float* maxD,
                       const float* minD, const uint8_t* bad, int* matches12, float s12, const float* R12,
                       const float* t12, float logScaleFactor, float th)
{
    const int N1 = KF1->N, N2 = KF2->N;
    simpose P1, P2;
    pose_of_T(T1w, &P1);
    pose_of_T(T2w, &P2);
    /* sR12 = s12*R12, sR21 = (1.0/s12)*R12.t(), t21 = -sR21*t12 (ORBmatcher.cc:1119-1121) */
    float sR12[9], sR21[9], t21[3];
    const float a21 = (float)(1.0 / (double)s12);
    for (int r = 0; r < 3; r++)
        for (int c = 0; c < 3; c++) {
            sR12[r * 3 + c] = R12[r * 3 + c] * s12 + 0.0f;
            sR21[r * 3 + c] = R12[c * 3 + r] * a21 + 0.0f;
        }
    for (int r = 0; r < 3; r++) {
        double s = (double)sR21[r * 3 + 0] * t12[0] + (double)sR21[r * 3 + 1] * t12[1] + (double)sR21[r * 3 + 2] * t12[2];
        t21[r] = (float)(s * -1.0);
    }
    uint8_t* am1 = (uint8_t*)calloc(N1 + 1, 1);
    uint8_t* am2 = (uint8_t*)calloc(N2 + 1, 1);
    for (int i = 0; i < N1; i++)
        if (matches12[i] != -1) {
            am1[i] = 1;
            const int idx2 = matches12[i];
            if (idx2 >= 0 && idx2 < N2) am2[idx2] = 1;
        }
    int* vn1 = (int*)malloc(sizeof(int) * (N1 + 1));
    int* vn2 = (int*)malloc(sizeof(int) * (N2 + 1));
    int* cand = (int*)malloc(sizeof(int) * ((N1 > N2 ? N1 : N2) + 1));
    sim3_direction(KF2, K, &P1, sR21, t21, N1, mp1, am1, pos, desc, maxD, minD, bad, logScaleFactor, th, vn1, cand);
    sim3_direction(KF1, K, &P2, sR12, t12, N2, mp2, am2, pos, desc, maxD, minD, bad, logScaleFactor, th, vn2, cand);
    int nFound = 0;
    for (int i1 = 0; i1 < N1; i1++) {
        const int idx2 = vn1[i1];
        if (idx2 >= 0 && vn2[idx2] == i1) {
            matches12[i1] = idx2;
            nFound++;
        }
    }
    free(am1); free(am2); free(vn1); free(vn2); free(cand);
    return nFound;
}
