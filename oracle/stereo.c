/*
 * stereo.c -- TEST INFRASTRUCTURE ONLY (see orb_oracle.h).
 * CPU restatement of Frame::ComputeStereoMatches (reference src/Frame.cc:466-640).
 *
 * cv::Mat windows are read from the padded pyramid levels of the two extractors
 * (ora_extractor_level: 19-px REFLECT_101 border), so a window that would leave the
 * unpadded level reads the border (the reference's cv::Mat::colRange would assert
 * there; keypoints sit >= 16 px inside each level, so it does not happen in practice).
 * cv::norm(IL, IR, NORM_L1) of the centred CV_32F windows is an exact integer (pixel
 * differences of integers), so it is summed in int here.
 */
#include <limits.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "orb_oracle.h"

#define EDGE 19

typedef struct { const uint8_t* data; int pw, ph, step; } lvl_t;

static int px(const lvl_t* L, int x, int y) { return L->data[(size_t)(y + EDGE) * L->step + (x + EDGE)]; }

static int cmp_pair(const void* a, const void* b)
{
    const int* p = (const int*)a;
    const int* q = (const int*)b;
    if (p[0] != q[0]) return p[0] < q[0] ? -1 : 1;
    return p[1] < q[1] ? -1 : (p[1] > q[1]);
}

int ora_compute_stereo_matches(const ora_kp* kL, const uint8_t* dL, int NL, const ora_kp* kR, const uint8_t* dR,
                               int NR, const ora_extractor* exL, const ora_extractor* exR, int rows0, float mbf,
                               float mb, float* uRight, float* depth)
{
    float scale[32], invScale[32], s2[32], is2[32];
    int nper[32], umax[16];
    ora_extractor_tables(exL, scale, invScale, s2, is2, nper, umax);
    const int nlev = ora_extractor_nlevels(exL);
    lvl_t PL[32], PR[32];
    for (int l = 0; l < nlev; l++) {
        ora_extractor_level(exL, l, &PL[l].data, &PL[l].pw, &PL[l].ph, &PL[l].step);
        ora_extractor_level(exR, l, &PR[l].data, &PR[l].pw, &PR[l].ph, &PR[l].step);
    }
    for (int i = 0; i < NL; i++) { uRight[i] = -1.0f; depth[i] = -1.0f; }   /* 468-469 */
    const int thOrbDist = (100 + 50) / 2;                                      /* 471 */
    const int nRows = rows0;
    /* row table (475-493): row -> right keypoints in iR order */
    int* rcnt = (int*)calloc(nRows + 1, sizeof(int));
    for (int iR = 0; iR < NR; iR++) {
        const float kpY = kR[iR].y;
        const float r = 2.0f * scale[kR[iR].octave];
        const int maxr = (int)ceilf(kpY + r), minr = (int)floorf(kpY - r);
        for (int yi = minr; yi <= maxr; yi++)
            if (yi >= 0 && yi < nRows) rcnt[yi + 1]++;
    }
    for (int y = 0; y < nRows; y++) rcnt[y + 1] += rcnt[y];
    int* ridx = (int*)malloc(sizeof(int) * (rcnt[nRows] + 1));
    int* fill = (int*)malloc(sizeof(int) * (nRows + 1));
    memcpy(fill, rcnt, sizeof(int) * (nRows + 1));
    for (int iR = 0; iR < NR; iR++) {
        const float kpY = kR[iR].y;
        const float r = 2.0f * scale[kR[iR].octave];
        const int maxr = (int)ceilf(kpY + r), minr = (int)floorf(kpY - r);
        for (int yi = minr; yi <= maxr; yi++)
            if (yi >= 0 && yi < nRows) ridx[fill[yi]++] = iR;
    }
    const float minZ = mb, minD = 0, maxD = mbf / minZ;                       /* 496-498 */
    int* vd = (int*)malloc(sizeof(int) * 2 * (NL + 1));
    int nvd = 0;
    for (int iL = 0; iL < NL; iL++) {
        const ora_kp* kpL = &kL[iL];
        const int levelL = kpL->octave;
        const float vL = kpL->y, uL = kpL->x;
        const int row = (int)vL;                                               /* vRowIndices[vL] */
        if (row < 0 || row >= nRows) continue;
        const int c0 = rcnt[row], c1 = rcnt[row + 1];
        if (c0 == c1) continue;
        const float minU = uL - maxD, maxU = uL - minD;
        if (maxU < 0) continue;
        int bestDist = 100, bestIdxR = 0;                                      /* TH_HIGH */
        for (int c = c0; c < c1; c++) {
            const int iR = ridx[c];
            const ora_kp* kpR = &kR[iR];
            if (kpR->octave < levelL - 1 || kpR->octave > levelL + 1) continue;
            const float uR = kpR->x;
            if (uR >= minU && uR <= maxU) {
                const int dist = ora_descriptor_distance(dL + 32 * (size_t)iL, dR + 32 * (size_t)iR);
                if (dist < bestDist) { bestDist = dist; bestIdxR = iR; }
            }
        }
        if (!(bestDist < thOrbDist)) continue;
        /* subpixel match by correlation (551-605) */
        const float uR0 = kR[bestIdxR].x;
        const float scaleFactor = invScale[kpL->octave];
        const float scaleduL = roundf(kpL->x * scaleFactor);
        const float scaledvL = roundf(kpL->y * scaleFactor);
        const float scaleduR0 = roundf(uR0 * scaleFactor);
        const int w = 5, L = 5;
        const lvl_t* IL = &PL[kpL->octave];
        const lvl_t* IR = &PR[kpL->octave];
        const int yL = (int)scaledvL, xL = (int)scaleduL;
        const int cL = px(IL, xL, yL);
        const float iniu = scaleduR0 + L - w, endu = scaleduR0 + L + w + 1;
        if (iniu < 0 || endu >= IR->pw - 2 * EDGE) continue;
        int bestD = INT_MAX, bestincR = 0;
        int vDists[11];
        for (int incR = -L; incR <= L; incR++) {
            const int xR = (int)scaleduR0 + incR;
            const int cR = px(IR, xR, yL);
            int dist = 0;
            for (int dy = -w; dy <= w; dy++)
                for (int dx = -w; dx <= w; dx++) {
                    const int a = px(IL, xL + dx, yL + dy) - cL;
                    const int b = px(IR, xR + dx, yL + dy) - cR;
                    dist += abs(a - b);
                }
            if (dist < bestD) { bestD = dist; bestincR = incR; }
            vDists[L + incR] = dist;
        }
        if (bestincR == -L || bestincR == L) continue;
        const float dist1 = (float)vDists[L + bestincR - 1];
        const float dist2 = (float)vDists[L + bestincR];
        const float dist3 = (float)vDists[L + bestincR + 1];
        const float deltaR = (dist1 - dist3) / (2.0f * (dist1 + dist3 - 2.0f * dist2));
        if (deltaR < -1 || deltaR > 1) continue;
        float bestuR = scale[kpL->octave] * ((float)scaleduR0 + (float)bestincR + deltaR);
        float disparity = (uL - bestuR);
        if (disparity >= minD && disparity < maxD) {
            if (disparity <= 0) {
                disparity = 0.01;
                bestuR = uL - 0.01;
            }
            depth[iL] = mbf / disparity;
            uRight[iL] = bestuR;
            vd[2 * nvd] = bestD;
            vd[2 * nvd + 1] = iL;
            nvd++;
        }
    }
    /* median filter (624-639); an empty vDistIdx is UB in the reference: nothing to filter */
    int kept = nvd;
    if (nvd > 0) {
        qsort(vd, nvd, 2 * sizeof(int), cmp_pair);
        const float median = (float)vd[2 * (nvd / 2)];
        const float thDist = 1.5f * 1.4f * median;
        for (int i = nvd - 1; i >= 0; i--) {
            if ((float)vd[2 * i] < thDist) break;
            uRight[vd[2 * i + 1]] = -1;
            depth[vd[2 * i + 1]] = -1;
            kept--;
        }
    }
    free(rcnt); free(ridx); free(fill); free(vd);
    return kept;
}

/* Frame::UnprojectStereo, Frame.cc:666-680.  mRwc*x3Dc+mOw is one cv::gemm (3x3 by 3x1 plus
 * 3x1), evaluated as the rest of this oracle evaluates that product: f64 accumulation of the
 * f32 products, one rounding to float (matchers2.c gemm_row3). */
void ora_unproject_stereo(const ora_kp* kps, const float* depth, int N, const float* Twc, float fx, float fy,
                          float cx, float cy, float* x3D, int* mp) {
    const float invfx = 1.0f / fx, invfy = 1.0f / fy;
    for (int i = 0; i < N; i++) {
        const float z = depth[i];
        if (mp) mp[i] = z > 0 ? i : -1;
        if (!(z > 0)) continue;
        const float u = kps[i].x, v = kps[i].y;
        const float x = (u - cx) * z * invfx;
        const float y = (v - cy) * z * invfy;
        for (int r = 0; r < 3; r++) {
            const double acc = (double)Twc[r * 4 + 0] * x + (double)Twc[r * 4 + 1] * y + (double)Twc[r * 4 + 2] * z;
            x3D[3 * i + r] = (float)(acc + (double)Twc[r * 4 + 3]);
        }
    }
}

/* mDistCoef (4, 5 or 8 floats) -> the double k[8] cvUndistortPoints works with (cvConvert). */
static void dist_to_k(const float* dist, int ndist, double k[8])
{
    for (int i = 0; i < 8; i++) k[i] = i < ndist ? (double)dist[i] : 0.0;
}

/* Frame::UndistortKeyPoints, Frame.cc:404-430: mvKeysUn = mvKeys when mDistCoef.at<float>(0)
 * is 0 (the other coefficients are not looked at); otherwise every keypoint's pt goes through
 * cv::undistortPoints(mat, mat, mK, mDistCoef, Mat(), mK) and the rest of the KeyPoint is
 * copied. */
void ora_undistort_keypoints(const ora_kp* keys, int N, const float K[9], const float* dist, int ndist,
                             ora_kp* keysUn)
{
    for (int i = 0; i < N; i++) keysUn[i] = keys[i];
    if (dist[0] == 0.0f) return;
    double k[8];
    dist_to_k(dist, ndist, k);
    for (int i = 0; i < N; i++) {
        const float src[2] = {keys[i].x, keys[i].y};
        float dst[2];
        ora_undistort_points(src, 1, K, k, 1, dst);
        keysUn[i].x = dst[0];
        keysUn[i].y = dst[1];
    }
}

/* Frame::ComputeImageBounds, Frame.cc:432-464, and the grid factors of the Frame constructors
 * (mfGridElementWidthInv = FRAME_GRID_COLS / (mnMaxX - mnMinX), Frame.cc:97-98): bounds[0..5] =
 * mnMinX, mnMaxX, mnMinY, mnMaxY, mfGridElementWidthInv, mfGridElementHeightInv. */
void ora_compute_image_bounds(int cols, int rows, const float K[9], const float* dist, int ndist, float bounds[6])
{
    if (dist[0] != 0.0f) {
        const float c[8] = {0.0f, 0.0f, (float)cols, 0.0f, 0.0f, (float)rows, (float)cols, (float)rows};
        float u[8];
        double k[8];
        dist_to_k(dist, ndist, k);
        ora_undistort_points(c, 4, K, k, 1, u);
        /* std::min(a, b) = b < a ? b : a; std::max(a, b) = a < b ? b : a */
        bounds[0] = u[4] < u[0] ? u[4] : u[0];
        bounds[1] = u[2] < u[6] ? u[6] : u[2];
        bounds[2] = u[3] < u[1] ? u[3] : u[1];
        bounds[3] = u[5] < u[7] ? u[7] : u[5];
    } else {
        bounds[0] = 0.0f;
        bounds[1] = (float)cols;
        bounds[2] = 0.0f;
        bounds[3] = (float)rows;
    }
    bounds[4] = (float)64 / (float)(bounds[1] - bounds[0]);
    bounds[5] = (float)48 / (float)(bounds[3] - bounds[2]);
}
