/*
 * orb_match.c -- TEST INFRASTRUCTURE ONLY (parity oracle).
 *
 * Restatement of the guided matchers of ORB_SLAM2::ORBmatcher
 * (reference src/ORBmatcher.cc) and the Frame grid they query
 * (src/Frame.cc:230-245, 327-392; include/Frame.h:37-38).
 *
 * cv::Mat products in the projections (`Rcw*x3Dw+tcw`) are restated as
 * cv::gemm's GEMMSingleMul<float,double>: float operands, double
 * accumulation, one rounding to float ("parity unpinned" at OpenCV).
 */
#include "orb_oracle.h"
#include <math.h>
#include <stdlib.h>
#include <string.h>

#define TH_HIGH 100
#define TH_LOW 50
#define HISTO_LENGTH 30

/* DescriptorDistance, ORBmatcher.cc:1647-1663 (SWAR popcount of 8 int32 words) */
int ora_descriptor_distance(const uint8_t* a, const uint8_t* b)
{
    int dist = 0;
    for (int i = 0; i < 8; i++) {
        uint32_t pa, pb;
        memcpy(&pa, a + 4 * i, 4);
        memcpy(&pb, b + 4 * i, 4);
        uint32_t v = pa ^ pb;
        v = v - ((v >> 1) & 0x55555555u);
        v = (v & 0x33333333u) + ((v >> 2) & 0x33333333u);
        dist += (int)((((v + (v >> 4)) & 0xF0F0F0Fu) * 0x1010101u) >> 24);
    }
    return dist;
}

/* PosInGrid Frame.cc:382-392 + AssignFeaturesToGrid 230-245 (cell = ix*48+iy, insertion order) */
void ora_frame_build_grid(ora_frame* f)
{
    const int NC = ORA_GRID_COLS * ORA_GRID_ROWS;
    int* cnt = (int*)calloc(NC + 1, sizeof(int));
    int* cellOf = (int*)malloc(sizeof(int) * (f->N > 0 ? f->N : 1));
    for (int i = 0; i < f->N; i++) {
        int px = (int)roundf((f->kpsUn[i].x - f->minX) * f->gridWInv);
        int py = (int)roundf((f->kpsUn[i].y - f->minY) * f->gridHInv);
        if (px < 0 || px >= ORA_GRID_COLS || py < 0 || py >= ORA_GRID_ROWS) { cellOf[i] = -1; continue; }
        cellOf[i] = px * ORA_GRID_ROWS + py;
        cnt[cellOf[i] + 1]++;
    }
    f->cellStart[0] = 0;
    for (int c = 0; c < NC; c++) f->cellStart[c + 1] = f->cellStart[c] + cnt[c + 1];
    memset(cnt, 0, sizeof(int) * (NC + 1));
    for (int i = 0; i < f->N; i++)
        if (cellOf[i] >= 0) f->cellIdx[f->cellStart[cellOf[i]] + cnt[cellOf[i]]++] = i;
    free(cnt);
    free(cellOf);
}

/* Frame::GetFeaturesInArea, Frame.cc:327-380 */
int ora_frame_features_in_area(const ora_frame* f, float x, float y, float r,
                               int minLevel, int maxLevel, int* out, int cap)
{
    int n = 0;
    int a = (int)floorf((x - f->minX - r) * f->gridWInv);
    const int nMinCellX = a > 0 ? a : 0;
    if (nMinCellX >= ORA_GRID_COLS) return 0;
    a = (int)ceilf((x - f->minX + r) * f->gridWInv);
    const int nMaxCellX = a < ORA_GRID_COLS - 1 ? a : ORA_GRID_COLS - 1;
    if (nMaxCellX < 0) return 0;
    a = (int)floorf((y - f->minY - r) * f->gridHInv);
    const int nMinCellY = a > 0 ? a : 0;
    if (nMinCellY >= ORA_GRID_ROWS) return 0;
    a = (int)ceilf((y - f->minY + r) * f->gridHInv);
    const int nMaxCellY = a < ORA_GRID_ROWS - 1 ? a : ORA_GRID_ROWS - 1;
    if (nMaxCellY < 0) return 0;
    const int bCheckLevels = (minLevel > 0) || (maxLevel >= 0);
    for (int ix = nMinCellX; ix <= nMaxCellX; ix++)
        for (int iy = nMinCellY; iy <= nMaxCellY; iy++) {
            int c = ix * ORA_GRID_ROWS + iy;
            for (int j = f->cellStart[c]; j < f->cellStart[c + 1]; j++) {
                const ora_kp* kp = &f->kpsUn[f->cellIdx[j]];
                if (bCheckLevels) {
                    if (kp->octave < minLevel) continue;
                    if (maxLevel >= 0 && kp->octave > maxLevel) continue;
                }
                const float distx = kp->x - x, disty = kp->y - y;
                if (fabsf(distx) < r && fabsf(disty) < r) {
                    if (n < cap) out[n] = f->cellIdx[j];
                    n++;
                }
            }
        }
    return n;
}

/* ComputeThreeMaxima, ORBmatcher.cc:1601-1642 */
void ora_compute_three_maxima(const int* histo, int L, int* ind1, int* ind2, int* ind3)
{
    int max1 = 0, max2 = 0, max3 = 0;
    *ind1 = *ind2 = *ind3 = -1;
    for (int i = 0; i < L; i++) {
        const int s = histo[i];
        if (s > max1) {
            max3 = max2; max2 = max1; max1 = s;
            *ind3 = *ind2; *ind2 = *ind1; *ind1 = i;
        } else if (s > max2) {
            max3 = max2; max2 = s;
            *ind3 = *ind2; *ind2 = i;
        } else if (s > max3) {
            max3 = s; *ind3 = i;
        }
    }
    if (max2 < 0.1f * (float)max1) { *ind2 = -1; *ind3 = -1; }
    else if (max3 < 0.1f * (float)max1) { *ind3 = -1; }
}

/* Rcw*X + t as one cv::gemm: float in, double accumulate, float out */
static inline float gemm_row(const float* T, int r, const float* X)
{
    double s = (double)T[r * 4 + 0] * X[0] + (double)T[r * 4 + 1] * X[1] + (double)T[r * 4 + 2] * X[2];
    return (float)(s + (double)T[r * 4 + 3]);
}

/* SearchByProjection(Frame& Cur, const Frame& Last, th, bMono), ORBmatcher.cc:1328-1470 */
int ora_search_by_projection_last(const ora_frame* cur, int* curMP, const ora_lastframe* L,
                                  float th, int bMono, float nnratio, int checkOri)
{
    (void)nnratio;
    int nmatches = 0;
    const float factor = 1.0f / HISTO_LENGTH;
    const float* Tc = L->Tcw_cur;
    const float* Tl = L->Tcw_last;
    /* twc = -Rcw.t()*tcw ; tlc = Rlw*twc + tlw */
    float twc[3], tlc[3];
    for (int i = 0; i < 3; i++) {
        double s = (double)Tc[0 * 4 + i] * Tc[3] + (double)Tc[1 * 4 + i] * Tc[7] + (double)Tc[2 * 4 + i] * Tc[11];
        twc[i] = (float)(s * -1.0);
    }
    for (int i = 0; i < 3; i++) tlc[i] = gemm_row(Tl, i, twc);
    const int bForward = tlc[2] > L->mb && !bMono;
    const int bBackward = -tlc[2] > L->mb && !bMono;

    int* hbin = (int*)malloc(sizeof(int) * (L->lastN + 1));
    int* hidx = (int*)malloc(sizeof(int) * (L->lastN + 1));
    int nh = 0;
    int* cand = (int*)malloc(sizeof(int) * (cur->N + 1));

    for (int i = 0; i < L->lastN; i++) {
        int mp = L->lastMP[i];
        if (mp < 0) continue;
        if (L->lastOutlier[i]) continue;
        const float* X = L->mpPos + 3 * mp;
        const float xc = gemm_row(Tc, 0, X), yc = gemm_row(Tc, 1, X), zc = gemm_row(Tc, 2, X);
        const float invzc = (float)(1.0 / zc);
        if (invzc < 0) continue;
        float u = L->fx * xc * invzc + L->cx;
        float v = L->fy * yc * invzc + L->cy;
        if (u < cur->minX || u > cur->maxX) continue;
        if (v < cur->minY || v > cur->maxY) continue;
        int nLastOctave = L->lastKeys[i].octave;
        float radius = th * cur->scaleFactors[nLastOctave];
        int nc;
        if (bForward) nc = ora_frame_features_in_area(cur, u, v, radius, nLastOctave, -1, cand, cur->N);
        else if (bBackward) nc = ora_frame_features_in_area(cur, u, v, radius, 0, nLastOctave, cand, cur->N);
        else nc = ora_frame_features_in_area(cur, u, v, radius, nLastOctave - 1, nLastOctave + 1, cand, cur->N);
        if (nc == 0) continue;
        const uint8_t* dMP = L->mpDesc + 32 * (size_t)mp;
        int bestDist = 256, bestIdx2 = -1;
        for (int k = 0; k < nc; k++) {
            const int i2 = cand[k];
            if (curMP[i2] >= 0 && L->mpObs[curMP[i2]] > 0) continue;
            if (cur->uRight && cur->uRight[i2] > 0) {
                const float ur = u - L->mbf * invzc;
                const float er = fabsf(ur - cur->uRight[i2]);
                if (er > radius) continue;
            }
            const int dist = ora_descriptor_distance(dMP, cur->desc + 32 * (size_t)i2);
            if (dist < bestDist) { bestDist = dist; bestIdx2 = i2; }
        }
        if (bestDist <= TH_HIGH) {
            curMP[bestIdx2] = mp;
            nmatches++;
            if (checkOri) {
                float rot = L->lastKeysUn[i].angle - cur->kpsUn[bestIdx2].angle;
                if (rot < 0.0) rot += 360.0f;
                int bin = (int)roundf(rot * factor);
                if (bin == HISTO_LENGTH) bin = 0;
                hbin[nh] = bin; hidx[nh] = bestIdx2; nh++;
            }
        }
    }
    if (checkOri) {
        int sizes[HISTO_LENGTH] = {0};
        for (int k = 0; k < nh; k++) sizes[hbin[k]]++;
        int i1, i2, i3;
        ora_compute_three_maxima(sizes, HISTO_LENGTH, &i1, &i2, &i3);
        for (int b = 0; b < HISTO_LENGTH; b++) {
            if (b == i1 || b == i2 || b == i3) continue;
            for (int k = 0; k < nh; k++)
                if (hbin[k] == b) { curMP[hidx[k]] = -1; nmatches--; }
        }
    }
    free(hbin); free(hidx); free(cand);
    return nmatches;
}

/* SearchByProjection(Frame& F, const vector<MapPoint*>&, th), ORBmatcher.cc:45-129
 * (+ RadiusByViewingCos 131-137) */
int ora_search_by_projection_local(const ora_frame* F, int* curMP, const int* mpObs,
                                   const ora_localmaps* m, float th, float nnratio)
{
    int nmatches = 0;
    const int bFactor = th != 1.0;
    int* cand = (int*)malloc(sizeof(int) * (F->N + 1));
    for (int iMP = 0; iMP < m->n; iMP++) {
        if (!m->inView[iMP]) continue;
        const int nPredictedLevel = m->level[iMP];
        float r = m->viewCos[iMP] > 0.998 ? 2.5f : 4.0f;
        if (bFactor) r *= th;
        const float rs = r * F->scaleFactors[nPredictedLevel];
        int nc = ora_frame_features_in_area(F, m->projX[iMP], m->projY[iMP], rs,
                                            nPredictedLevel - 1, nPredictedLevel, cand, F->N);
        if (nc == 0) continue;
        const uint8_t* d0 = m->desc + 32 * (size_t)iMP;
        int bestDist = 256, bestLevel = -1, bestDist2 = 256, bestLevel2 = -1, bestIdx = -1;
        for (int k = 0; k < nc; k++) {
            const int idx = cand[k];
            if (curMP[idx] >= 0 && mpObs[curMP[idx]] > 0) continue;
            if (F->uRight && F->uRight[idx] > 0) {
                const float er = fabsf(m->projXR[iMP] - F->uRight[idx]);
                if (er > r * F->scaleFactors[nPredictedLevel]) continue;
            }
            const int dist = ora_descriptor_distance(d0, F->desc + 32 * (size_t)idx);
            if (dist < bestDist) {
                bestDist2 = bestDist; bestDist = dist;
                bestLevel2 = bestLevel; bestLevel = F->kpsUn[idx].octave;
                bestIdx = idx;
            } else if (dist < bestDist2) {
                bestLevel2 = F->kpsUn[idx].octave;
                bestDist2 = dist;
            }
        }
        if (bestDist <= TH_HIGH) {
            if (bestLevel == bestLevel2 && bestDist > nnratio * bestDist2) continue;
            curMP[bestIdx] = m->mpId[iMP];
            nmatches++;
        }
    }
    free(cand);
    return nmatches;
}
