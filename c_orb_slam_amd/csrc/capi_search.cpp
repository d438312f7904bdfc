// capi_search.cpp -- extern "C" entry points of the remaining ORBmatcher searches
// (include/orbslam_gpu.h), reference src/ORBmatcher.cc:
//   SearchByProjection(Frame&, KeyFrame*, set, th, ORBdist)   1472-1599  (relocalization)
//   SearchForInitialization(F1, F2, vbPrevMatched, vnMatches12, windowSize)   405-520
//   SearchByBoW(KeyFrame*, Frame&, vpMapPointMatches)           159-288
//   SearchByBoW(KeyFrame*, KeyFrame*, vpMatches12)              522-655
//   SearchForTriangulation(KF1, KF2, F12, vMatchedPairs, bOnlyStereo)         657-823
//   SearchByProjection(KeyFrame*, Scw, vpPoints, vpMatched, th)  290-403   (loop closing)
//   Fuse(KeyFrame*, vpMapPoints, th)                             825-975   (local mapping)
//   Fuse(KeyFrame*, Scw, vpPoints, th, vpReplacePoint)           977-1100  (loop closing)
//   SearchBySim3(pKF1, pKF2, vpMatches12, s12, R12, t12, th)     1102-1326 (loop detection)
//
// Split of the work: the device enumerates every candidate of every query and its 256-bit
// Hamming distance (the window engine Matcher::area_candidates over the frame grid, or the
// CSR engine k_csr_hamming for vocabulary-node candidates); the host computes the per-query
// projections (float, the reference's expression order) and replays the order-dependent
// selection (occupancy, best / second, ratio, rotation histogram) over those lists.
#include <algorithm>
#include <climits>
#include <cmath>
#include <cstring>
#include <vector>

#include "capi_handles.hpp"

using orbgpu::AreaQuery;
using orbgpu::Matcher;
using orbgpu::SearchDev;

namespace {

constexpr int kHisto = 30;
constexpr int kThLow = 50;

size_t al(size_t n) { return (n + 255) & ~(size_t)255; }

template <class T>
T* up(Matcher* m, const T* src, size_t count, hipStream_t s, int* err) {
    if (!src || count == 0) return nullptr;
    void* d = m->arena_alloc(count * sizeof(T));
    if (!d || hipMemcpyAsync(d, src, count * sizeof(T), hipMemcpyHostToDevice, s) != hipSuccess) {
        *err = ORB_E_HIP;
        return nullptr;
    }
    return (T*)d;
}

// rotation-consistency histogram (ORBmatcher.cc:1601-1642 ComputeThreeMaxima)
struct RotHist {
    std::vector<std::pair<int, int>> rec;   // (bin, value) in insertion order
    int cnt[kHisto] = {};
    void push(float a1, float a2, int v) {
        const float factor = 1.0f / kHisto;
        float rot = a1 - a2;
        if (rot < 0.0) rot += 360.0f;
        int bin = (int)std::round(rot * factor);
        if (bin == kHisto) bin = 0;
        rec.emplace_back(bin, v);
        cnt[bin]++;
    }
    void maxima(int& i1, int& i2, int& i3) const {
        int m1 = 0, m2 = 0, m3 = 0;
        i1 = i2 = i3 = -1;
        for (int i = 0; i < kHisto; i++) {
            const int s = cnt[i];
            if (s > m1) {
                m3 = m2; m2 = m1; m1 = s;
                i3 = i2; i2 = i1; i1 = i;
            } else if (s > m2) {
                m3 = m2; m2 = s;
                i3 = i2; i2 = i;
            } else if (s > m3) {
                m3 = s;
                i3 = i;
            }
        }
        if (m2 < 0.1f * (float)m1) {
            i2 = -1;
            i3 = -1;
        } else if (m3 < 0.1f * (float)m1) {
            i3 = -1;
        }
    }
    // visit every recorded value outside the three dominant bins
    template <class F>
    void reject(F f) const {
        int i1, i2, i3;
        maxima(i1, i2, i3);
        for (const auto& r : rec)
            if (r.first != i1 && r.first != i2 && r.first != i3) f(r.second);
    }
};

// Rcw*X + tcw as one cv::gemm (f64 accumulate, one rounding)
inline float gemm_row(const float* T, int r, const float* X) {
    const double s = (double)T[r * 4 + 0] * X[0] + (double)T[r * 4 + 1] * X[1] + (double)T[r * 4 + 2] * X[2];
    return (float)(s + (double)T[r * 4 + 3]);
}

// -Rcw.t()*tcw as one cv::gemm with alpha -1 (Frame/KeyFrame camera centre)
inline void camera_center(const float* T, float* O) {
    for (int i = 0; i < 3; i++) {
        const double s = (double)T[0 * 4 + i] * T[3] + (double)T[1 * 4 + i] * T[7] + (double)T[2 * 4 + i] * T[11];
        O[i] = (float)(s * -1.0);
    }
}

bool frame_ok(const orb_frame* f) {
    return f && f->N >= 0 && f->N <= orbgpu::kMaxFrameKeys && (f->N == 0 || (f->keysUn && f->desc)) &&
           f->scaleFactors && f->nlevels > 0;
}

bool featvec_ok(const orb_featvec* v, int n) {
    if (!v || v->n_nodes < 0) return false;
    if (v->n_nodes == 0) return true;
    if (!v->node_id || !v->start || !v->feat || v->start[0] != 0) return false;
    for (int a = 0; a < v->n_nodes; a++) {
        if (v->start[a + 1] < v->start[a]) return false;
        if (a && v->node_id[a] <= v->node_id[a - 1]) return false;
    }
    for (int k = 0; k < v->start[v->n_nodes]; k++)
        if (v->feat[k] < 0 || v->feat[k] >= n) return false;
    return true;
}

// Upload a frame's keypoints / descriptors and describe it as the engine's "cur" frame.
SearchDev frame_dev(Matcher* m, const orb_frame* f, hipStream_t s, int* err) {
    SearchDev P;
    std::memset(&P, 0, sizeof(P));
    P.cur.N = f->N;
    P.cur.minX = f->minX; P.cur.maxX = f->maxX; P.cur.minY = f->minY; P.cur.maxY = f->maxY;
    P.cur.gridWInv = f->gridWInv; P.cur.gridHInv = f->gridHInv;
    P.cur.nlevels = f->nlevels;
    P.cur.keysUn = (const orbgpu::orb_kp_dev*)up(m, f->keysUn, (size_t)f->N, s, err);
    P.cur.desc = up(m, f->desc, (size_t)f->N * 32, s, err);
    return P;
}

// vocabulary-node candidate lists: queries = side-1 features of every common node (node order),
// candidates = side-2 features of that node passing `ok2` (static flags), all distances on device
struct NodeLists {
    std::vector<int> qidx, off, cand, dist;
};

int node_lists(Matcher* m, const orb_featvec* fv1, const uint8_t* ok1, const uint8_t* desc1, int n1,
               const orb_featvec* fv2, const uint8_t* ok2, const uint8_t* desc2, int n2, NodeLists& L) {
    L.qidx.clear();
    L.cand.clear();
    L.off.assign(1, 0);
    int a = 0, b = 0;
    while (a < fv1->n_nodes && b < fv2->n_nodes) {
        if (fv1->node_id[a] == fv2->node_id[b]) {
            for (int q = fv1->start[a]; q < fv1->start[a + 1]; q++) {
                const int idx1 = fv1->feat[q];
                if (!ok1[idx1]) continue;
                L.qidx.push_back(idx1);
                for (int c = fv2->start[b]; c < fv2->start[b + 1]; c++)
                    if (ok2[fv2->feat[c]]) L.cand.push_back(fv2->feat[c]);
                L.off.push_back((int)L.cand.size());
            }
            a++;
            b++;
        } else if (fv1->node_id[a] < fv2->node_id[b]) {
            a++;
        } else {
            b++;
        }
    }
    const int nq = (int)L.qidx.size(), nc = (int)L.cand.size();
    L.dist.assign((size_t)std::max(nc, 1), 0);
    if (nq == 0 || nc == 0) return 0;
    hipStream_t s = m->stream();
    if (m->arena_reserve(al((size_t)n1 * 32) + al((size_t)n2 * 32) + al((size_t)nq * 32) + 2 * al((size_t)nc * 4) +
                         al(((size_t)nq + 1) * 4) + 3 * al((size_t)nq * 4) + 4096))
        return ORB_E_HIP;
    int err = 0;
    std::vector<uint8_t> qd((size_t)nq * 32);
    for (int i = 0; i < nq; i++) std::memcpy(&qd[(size_t)i * 32], desc1 + 32 * (size_t)L.qidx[i], 32);
    const uint8_t* dq = up(m, qd.data(), qd.size(), s, &err);
    const uint8_t* dt = up(m, desc2, (size_t)n2 * 32, s, &err);
    const int* doff = up(m, L.off.data(), L.off.size(), s, &err);
    const int* dc = up(m, L.cand.data(), L.cand.size(), s, &err);
    int* dd = (int*)m->arena_alloc((size_t)nc * 4);
    int* dbi = (int*)m->arena_alloc((size_t)nq * 4);
    int* dbd = (int*)m->arena_alloc((size_t)nq * 4);
    int* dsd = (int*)m->arena_alloc((size_t)nq * 4);
    if (err || !dd || !dbi || !dbd || !dsd) return ORB_E_HIP;
    if (m->candidates(dq, nq, dt, n2, doff, dc, dd, dbi, dbd, dsd)) return ORB_E_HIP;
    if (hipMemcpyAsync(L.dist.data(), dd, (size_t)nc * 4, hipMemcpyDeviceToHost, s) != hipSuccess) return ORB_E_HIP;
    return orbgpu::stream_wait(s) == hipSuccess ? ORB_OK : ORB_E_HIP;
}


// ---- similarity-pose projection searches (ORBmatcher.cc:290-403, 825-1326) -----------------
struct SimPose {
    float R[9], t[3], O[3];
};

inline float gemm3(const float* R, const float* t, int r, const float* X) {
    const double s = (double)R[r * 3 + 0] * X[0] + (double)R[r * 3 + 1] * X[1] + (double)R[r * 3 + 2] * X[2];
    return (float)(s + (double)t[r]);
}

inline void pose_center(SimPose& P) {   // -Rcw.t()*tcw: gemm with alpha -1
    for (int i = 0; i < 3; i++) {
        const double s = (double)P.R[i] * P.t[0] + (double)P.R[3 + i] * P.t[1] + (double)P.R[6 + i] * P.t[2];
        P.O[i] = (float)(s * -1.0);
    }
}

inline SimPose pose_T(const float* T) {
    SimPose P;
    for (int r = 0; r < 3; r++) {
        for (int c = 0; c < 3; c++) P.R[r * 3 + c] = T[r * 4 + c];
        P.t[r] = T[r * 4 + 3];
    }
    pose_center(P);
    return P;
}

// ORBmatcher.cc:298-303: scw = sqrt(row0.row0); Rcw = sRcw/scw, tcw = t/scw (convertTo: float
// multiply by (float)(1/scw)); Ow = -Rcw.t()*tcw
inline SimPose pose_Scw(const float* S) {
    SimPose P;
    const double d = (double)S[0] * S[0] + (double)S[1] * S[1] + (double)S[2] * S[2];
    const float scw = (float)std::sqrt(d);
    const float a = (float)(1.0 / (double)scw);
    for (int r = 0; r < 3; r++) {
        for (int c = 0; c < 3; c++) P.R[r * 3 + c] = S[r * 4 + c] * a + 0.0f;
        P.t[r] = S[r * 4 + 3] * a + 0.0f;
    }
    pose_center(P);
    return P;
}

inline int predict_scale(float maxDistance, float dist, float logScaleFactor, int nlevels) {   // MapPoint.cc:385-400
    const float ratio = maxDistance / dist;
    int n = (int)std::ceil(std::log(ratio) / logScaleFactor);
    return n < 0 ? 0 : (n >= nlevels ? nlevels - 1 : n);
}

inline bool kf_in_image(const orb_frame* F, float u, float v) {   // KeyFrame::IsInImage
    return u >= F->minX && u < F->maxX && v >= F->minY && v < F->maxY;
}

inline float norm3f(const float* v) {
    double s = 0;
    for (int k = 0; k < 3; k++) s += (double)v[k] * (double)v[k];
    return (float)std::sqrt(s);
}

bool geo_ok(const orb_mappoints* p, const orb_mappoint_geo* g, bool normal) {
    if (!p || p->n < 0) return false;
    if (p->n == 0) return true;
    return p->pos && p->desc && g && g->max_dist && g->min_dist && (!normal || g->normal);
}

// Queries of one projection pass -> every in-window candidate (KeyFrame::GetFeaturesInArea,
// octave range [pred-1, pred] applied on device) with its Hamming distance.
struct ProjPass {
    std::vector<AreaQuery> q;
    std::vector<uint8_t> qdesc;
    std::vector<float> u, v, ur;   // projections for the host gates
    std::vector<int> off;
    std::vector<int2> cand;
    void add(float x, float y, float r, int lvl, const uint8_t* d, float uu, float vv, float uur, size_t i) {
        AreaQuery& a = q[i];
        a.x = x;
        a.y = y;
        a.r = r;
        a.minLevel = lvl - 1;
        a.maxLevel = lvl;
        a.qd = (int)(qdesc.size() / 32);
        qdesc.insert(qdesc.end(), d, d + 32);
        u[i] = uu;
        v[i] = vv;
        ur[i] = uur;
    }
    void reset(int n) {
        q.assign((size_t)n, AreaQuery{0, 0, 0, -1, -1, -1});
        qdesc.clear();
        u.assign((size_t)n, 0.f);
        v.assign((size_t)n, 0.f);
        ur.assign((size_t)n, 0.f);
    }
    int run(Matcher* m, const orb_frame* F) {
        const size_t n = q.size();
        if (m->arena_reserve(al((size_t)F->N * 28) + al((size_t)F->N * 32) + al(n * sizeof(AreaQuery)) +
                             al(qdesc.size()) + 4096))
            return ORB_E_HIP;
        int err = 0;
        hipStream_t s = m->stream();
        SearchDev P = frame_dev(m, F, s, &err);
        const AreaQuery* dq = up(m, q.data(), n, s, &err);
        const uint8_t* dd = up(m, qdesc.data(), qdesc.size(), s, &err);
        if (err) return err;
        if (n == 0) {
            off.assign(1, 0);
            return ORB_OK;
        }
        return m->area_candidates(P, dq, (int)n, dd, off, cand) ? ORB_E_HIP : ORB_OK;
    }
};

// Projection of map point i for SearchByProjection(KF,Scw) / Fuse / Fuse(Scw) (shared gates):
// returns the predicted level or -1 when a gate rejects the point.
int project_point(const orb_frame* KF, const SimPose& P, const float* X, float maxD, float minD, const float* Pn,
                  float logScaleFactor, int invz_mode, float bf, float* u, float* v, float* ur) {
    const float xc = gemm3(P.R, P.t, 0, X), yc = gemm3(P.R, P.t, 1, X), zc = gemm3(P.R, P.t, 2, X);
    if (zc < 0.0f) return -1;
    const float invz = invz_mode ? (float)(1.0 / (double)zc) : 1 / zc;   // `1.0/z` vs `1/z`
    const float x = xc * invz, y = yc * invz;
    *u = KF->fx * x + KF->cx;
    *v = KF->fy * y + KF->cy;
    if (!kf_in_image(KF, *u, *v)) return -1;
    *ur = *u - bf * invz;
    const float PO[3] = {X[0] - P.O[0], X[1] - P.O[1], X[2] - P.O[2]};
    const float dist = norm3f(PO);
    if (dist < 0.8f * minD || dist > 1.2f * maxD) return -1;
    const double dot = (double)PO[0] * Pn[0] + (double)PO[1] * Pn[1] + (double)PO[2] * Pn[2];
    if (dot < 0.5 * dist) return -1;
    return predict_scale(maxD, dist, logScaleFactor, KF->nlevels);
}

int fuse_common(Matcher* m, const orb_frame* KF, const SimPose& P, bool sim3, const orb_mappoints* pts,
                const orb_mappoint_geo* geo, const uint8_t* skip, float logScaleFactor, float th, int32_t* best,
                int* nfused) {
    const int n = pts->n;
    ProjPass pp;
    pp.reset(n);
    for (int i = 0; i < n; i++) {
        best[i] = -1;
        if (skip[i]) continue;
        float u, v, ur;
        const int lvl = project_point(KF, P, pts->pos + 3 * (size_t)i, geo->max_dist[i], geo->min_dist[i],
                                      geo->normal + 3 * (size_t)i, logScaleFactor, sim3 ? 1 : 0, sim3 ? 0.f : KF->bf,
                                      &u, &v, &ur);
        if (lvl < 0) continue;
        pp.add(u, v, th * KF->scaleFactors[lvl], lvl, pts->desc + 32 * (size_t)i, u, v, ur, (size_t)i);
    }
    if (int e = pp.run(m, KF)) return e;
    int nf = 0;
    for (int i = 0; i < n; i++) {
        if (pp.q[i].qd < 0) continue;
        int bestDist = sim3 ? INT_MAX : 256, bestIdx = -1;
        for (int k = pp.off[i]; k < pp.off[i + 1]; k++) {
            const int idx = pp.cand[k].x;
            if (!sim3) {   // reprojection gate (ORBmatcher.cc:914-938)
                const orb_kp& kp = KF->keysUn[idx];
                const float s2 = KF->scaleFactors[kp.octave] * KF->scaleFactors[kp.octave];
                const float invSigma2 = 1.0f / s2;
                const float ex = pp.u[i] - kp.x, ey = pp.v[i] - kp.y;
                if (KF->uRight && KF->uRight[idx] >= 0) {
                    const float er = pp.ur[i] - KF->uRight[idx];
                    const float e2 = ex * ex + ey * ey + er * er;
                    if (e2 * invSigma2 > 7.8) continue;
                } else {
                    const float e2 = ex * ex + ey * ey;
                    if (e2 * invSigma2 > 5.99) continue;
                }
            }
            if (pp.cand[k].y < bestDist) {
                bestDist = pp.cand[k].y;
                bestIdx = idx;
            }
        }
        if (bestDist <= kThLow) {
            best[i] = bestIdx;
            nf++;
        }
    }
    *nfused = nf;
    return ORB_OK;
}

}  // namespace

extern "C" {

int ORBmatcher_SearchByProjection_KeyFrame(ORBmatcher_h h, const orb_frame* F, int32_t* cur_mp, int n,
                                           const int32_t* kf_mp, const uint8_t* skip, const float* kf_angle,
                                           const orb_mappoints* mps, const float* mp_max_dist,
                                           const float* mp_min_dist, float logScaleFactor, float th, int ORBdist,
                                           int* nmatches) {
    if (!h || !frame_ok(F) || !F->Tcw || !cur_mp || n < 0 || !mps || !nmatches) return ORB_E_INVALID;
    if (n > 0 && (!kf_mp || !skip || !kf_angle)) return ORB_E_INVALID;
    if (mps->n > 0 && (!mps->pos || !mps->desc || !mp_max_dist || !mp_min_dist)) return ORB_E_INVALID;
    Matcher* m = h->m;
    if (m->device_pointers()) return ORB_E_INVALID;   // host arrays only
    for (int i = 0; i < n; i++)
        if (kf_mp[i] >= mps->n) return ORB_E_INVALID;
    for (int i = 0; i < F->N; i++)
        if (cur_mp[i] >= mps->n) return ORB_E_INVALID;
    hipStream_t s = m->stream();
    // projection / scale prediction (ORBmatcher.cc:1478-1525), host float in the reference's order
    const float* T = F->Tcw;
    float Ow[3];
    camera_center(T, Ow);
    std::vector<AreaQuery> q((size_t)n);
    std::vector<uint8_t> qdesc;
    for (int i = 0; i < n; i++) {
        AreaQuery& a = q[i];
        a.qd = -1;
        const int mp = kf_mp[i];
        if (mp < 0 || skip[i]) continue;
        const float* X = mps->pos + 3 * (size_t)mp;
        const float xc = gemm_row(T, 0, X), yc = gemm_row(T, 1, X), zc = gemm_row(T, 2, X);
        const float invzc = (float)(1.0 / (double)zc);
        const float u = F->fx * xc * invzc + F->cx;
        const float v = F->fy * yc * invzc + F->cy;
        if (u < F->minX || u > F->maxX || v < F->minY || v > F->maxY) continue;
        const float PO[3] = {X[0] - Ow[0], X[1] - Ow[1], X[2] - Ow[2]};
        double s2 = 0;
        for (int k = 0; k < 3; k++) s2 += (double)PO[k] * (double)PO[k];
        const float dist3D = (float)std::sqrt(s2);
        if (dist3D < 0.8f * mp_min_dist[mp] || dist3D > 1.2f * mp_max_dist[mp]) continue;
        const float ratio = mp_max_dist[mp] / dist3D;   // MapPoint::PredictScale
        int lvl = (int)std::ceil(std::log(ratio) / logScaleFactor);
        lvl = lvl < 0 ? 0 : (lvl >= F->nlevels ? F->nlevels - 1 : lvl);
        a.x = u;
        a.y = v;
        a.r = th * F->scaleFactors[lvl];
        a.minLevel = lvl - 1;
        a.maxLevel = lvl + 1;
        a.qd = (int)(qdesc.size() / 32);
        qdesc.insert(qdesc.end(), mps->desc + 32 * (size_t)mp, mps->desc + 32 * (size_t)mp + 32);
    }
    if (m->arena_reserve(al((size_t)F->N * 28) + al((size_t)F->N * 32) + al(q.size() * sizeof(AreaQuery)) +
                         al(qdesc.size()) + 4096))
        return ORB_E_HIP;
    int err = 0;
    SearchDev P = frame_dev(m, F, s, &err);
    const AreaQuery* dq = up(m, q.data(), q.size(), s, &err);
    const uint8_t* dd = up(m, qdesc.data(), qdesc.size(), s, &err);
    if (err) return err;
    std::vector<int> off;
    std::vector<int2> cand;
    if (m->area_candidates(P, dq, n, dd, off, cand)) return ORB_E_HIP;
    // greedy replay (ORBmatcher.cc:1526-1567) + rotation check (1570-1596)
    int nm = 0;
    RotHist H;
    for (int i = 0; i < n; i++) {
        if (q[i].qd < 0 || off[i] == off[i + 1]) continue;
        int bestDist = 256, bestIdx2 = -1;
        for (int k = off[i]; k < off[i + 1]; k++) {
            const int i2 = cand[k].x;
            if (cur_mp[i2] >= 0) continue;
            if (cand[k].y < bestDist) {
                bestDist = cand[k].y;
                bestIdx2 = i2;
            }
        }
        if (bestDist <= ORBdist) {
            cur_mp[bestIdx2] = kf_mp[i];
            nm++;
            if (m->check_ori()) H.push(kf_angle[i], F->keysUn[bestIdx2].angle, bestIdx2);
        }
    }
    if (m->check_ori())
        H.reject([&](int i2) {
            cur_mp[i2] = -1;
            nm--;
        });
    *nmatches = nm;
    return ORB_OK;
}

int ORBmatcher_SearchForInitialization(ORBmatcher_h h, const orb_frame* F1, const orb_frame* F2, float* prev_matched,
                                       int32_t* matches12, int windowSize, int* nmatches) {
    if (!h || !frame_ok(F1) || !frame_ok(F2) || !nmatches || (F1->N && (!prev_matched || !matches12)))
        return ORB_E_INVALID;
    Matcher* m = h->m;
    if (m->device_pointers()) return ORB_E_INVALID;
    hipStream_t s = m->stream();
    const int N1 = F1->N, N2 = F2->N;
    std::vector<AreaQuery> q((size_t)N1);
    for (int i1 = 0; i1 < N1; i1++) {   // level-0 keypoints, window around vbPrevMatched (429-436)
        AreaQuery& a = q[i1];
        const int level1 = F1->keysUn[i1].octave;
        a.qd = level1 > 0 ? -1 : i1;
        a.x = prev_matched[2 * i1];
        a.y = prev_matched[2 * i1 + 1];
        a.r = (float)windowSize;
        a.minLevel = level1;
        a.maxLevel = level1;
    }
    if (m->arena_reserve(al((size_t)N2 * 28) + al((size_t)N2 * 32) + al(q.size() * sizeof(AreaQuery)) +
                         al((size_t)N1 * 32) + 4096))
        return ORB_E_HIP;
    int err = 0;
    SearchDev P = frame_dev(m, F2, s, &err);
    const AreaQuery* dq = up(m, q.data(), q.size(), s, &err);
    const uint8_t* dd = up(m, F1->desc, (size_t)N1 * 32, s, &err);
    if (err) return err;
    std::vector<int> off;
    std::vector<int2> cand;
    if (m->area_candidates(P, dq, N1, dd, off, cand)) return ORB_E_HIP;
    // replay (438-502): vMatchedDistance / vnMatches21 make it order dependent
    std::vector<int> dist21((size_t)N2, INT_MAX), m21((size_t)N2, -1);
    for (int i = 0; i < N1; i++) matches12[i] = -1;
    int nm = 0;
    RotHist H;
    const float nnratio = m->nnratio();
    for (int i1 = 0; i1 < N1; i1++) {
        if (q[i1].qd < 0 || off[i1] == off[i1 + 1]) continue;
        int bestDist = INT_MAX, bestDist2 = INT_MAX, bestIdx2 = -1;
        for (int k = off[i1]; k < off[i1 + 1]; k++) {
            const int i2 = cand[k].x, dist = cand[k].y;
            if (dist21[i2] <= dist) continue;
            if (dist < bestDist) {
                bestDist2 = bestDist;
                bestDist = dist;
                bestIdx2 = i2;
            } else if (dist < bestDist2) {
                bestDist2 = dist;
            }
        }
        if (bestDist <= kThLow && bestDist < (float)bestDist2 * nnratio) {
            if (m21[bestIdx2] >= 0) {
                matches12[m21[bestIdx2]] = -1;
                nm--;
            }
            matches12[i1] = bestIdx2;
            m21[bestIdx2] = i1;
            dist21[bestIdx2] = bestDist;
            nm++;
            if (m->check_ori()) H.push(F1->keysUn[i1].angle, F2->keysUn[bestIdx2].angle, i1);
        }
    }
    if (m->check_ori())
        H.reject([&](int i1) {
            if (matches12[i1] >= 0) {
                matches12[i1] = -1;
                nm--;
            }
        });
    for (int i1 = 0; i1 < N1; i1++)
        if (matches12[i1] >= 0) {
            prev_matched[2 * i1] = F2->keysUn[matches12[i1]].x;
            prev_matched[2 * i1 + 1] = F2->keysUn[matches12[i1]].y;
        }
    *nmatches = nm;
    return ORB_OK;
}

// shared replay of the two SearchByBoW loops (node order, best / second, greedy side-2 occupancy)
static int bow_replay(Matcher* m, const NodeLists& L, const float* ang1, const float* ang2, int n1, int n2,
                      bool le_low, std::vector<int>& m12) {
    m12.assign((size_t)n1, -1);
    std::vector<uint8_t> taken((size_t)n2, 0);
    int nm = 0;
    RotHist H;
    const float nnratio = m->nnratio();
    for (size_t q = 0; q < L.qidx.size(); q++) {
        const int idx1 = L.qidx[q];
        int best1 = 256, best2 = 256, bestIdx2 = -1;
        for (int k = L.off[q]; k < L.off[q + 1]; k++) {
            const int idx2 = L.cand[k];
            if (taken[idx2]) continue;
            const int dist = L.dist[k];
            if (dist < best1) {
                best2 = best1;
                best1 = dist;
                bestIdx2 = idx2;
            } else if (dist < best2) {
                best2 = dist;
            }
        }
        const bool pass = le_low ? best1 <= kThLow : best1 < kThLow;
        if (pass && (float)best1 < nnratio * (float)best2) {
            m12[idx1] = bestIdx2;
            taken[bestIdx2] = 1;
            if (m->check_ori()) H.push(ang1[idx1], ang2[bestIdx2], idx1);
            nm++;
        }
    }
    if (m->check_ori())
        H.reject([&](int idx1) {
            m12[idx1] = -1;
            nm--;
        });
    return nm;
}

int ORBmatcher_SearchByBoW_Frame(ORBmatcher_h h, int nKF, const uint8_t* kf_desc, const float* kf_angle,
                                 const int32_t* kf_mp, const uint8_t* kf_mp_bad, const orb_featvec* fvKF, int NF,
                                 const uint8_t* f_desc, const float* f_angle, const orb_featvec* fvF,
                                 int32_t* matches, int* nmatches) {
    if (!h || nKF < 0 || NF < 0 || !nmatches || !featvec_ok(fvKF, nKF) || !featvec_ok(fvF, NF)) return ORB_E_INVALID;
    if ((nKF && (!kf_desc || !kf_angle || !kf_mp || !kf_mp_bad)) || (NF && (!f_desc || !f_angle || !matches)))
        return ORB_E_INVALID;
    Matcher* m = h->m;
    if (m->device_pointers()) return ORB_E_INVALID;
    std::vector<uint8_t> ok1((size_t)nKF), ok2((size_t)NF, 1);
    for (int i = 0; i < nKF; i++) ok1[i] = kf_mp[i] >= 0 && !kf_mp_bad[i];
    NodeLists L;
    if (int e = node_lists(m, fvKF, ok1.data(), kf_desc, nKF, fvF, ok2.data(), f_desc, NF, L)) return e;
    std::vector<int> m12;
    const int nm = bow_replay(m, L, kf_angle, f_angle, nKF, NF, true, m12);
    for (int i = 0; i < NF; i++) matches[i] = -1;
    for (int i = 0; i < nKF; i++)
        if (m12[i] >= 0) matches[m12[i]] = kf_mp[i];
    *nmatches = nm;
    return ORB_OK;
}

int ORBmatcher_SearchByBoW_KeyFrames(ORBmatcher_h h, int n1, const uint8_t* desc1, const float* angle1,
                                     const int32_t* mp1, const uint8_t* bad1, const orb_featvec* fv1, int n2,
                                     const uint8_t* desc2, const float* angle2, const int32_t* mp2,
                                     const uint8_t* bad2, const orb_featvec* fv2, int32_t* matches12,
                                     int* nmatches) {
    if (!h || n1 < 0 || n2 < 0 || !nmatches || !featvec_ok(fv1, n1) || !featvec_ok(fv2, n2)) return ORB_E_INVALID;
    if ((n1 && (!desc1 || !angle1 || !mp1 || !bad1 || !matches12)) || (n2 && (!desc2 || !angle2 || !mp2 || !bad2)))
        return ORB_E_INVALID;
    Matcher* m = h->m;
    if (m->device_pointers()) return ORB_E_INVALID;
    std::vector<uint8_t> ok1((size_t)n1), ok2((size_t)n2);
    for (int i = 0; i < n1; i++) ok1[i] = mp1[i] >= 0 && !bad1[i];
    for (int i = 0; i < n2; i++) ok2[i] = mp2[i] >= 0 && !bad2[i];
    NodeLists L;
    if (int e = node_lists(m, fv1, ok1.data(), desc1, n1, fv2, ok2.data(), desc2, n2, L)) return e;
    std::vector<int> m12;
    const int nm = bow_replay(m, L, angle1, angle2, n1, n2, false, m12);
    for (int i = 0; i < n1; i++) matches12[i] = m12[i] >= 0 ? mp2[m12[i]] : -1;
    *nmatches = nm;
    return ORB_OK;
}

int ORBmatcher_SearchForTriangulation(ORBmatcher_h h, const orb_frame* KF1, const uint8_t* has_mp1,
                                      const orb_featvec* fv1, const orb_frame* KF2, const uint8_t* has_mp2,
                                      const orb_featvec* fv2, const float* levelSigma2_2, const float* F12,
                                      int bOnlyStereo, int32_t* pairs, int cap, int* npairs) {
    if (!h || !frame_ok(KF1) || !frame_ok(KF2) || !KF1->Tcw || !KF2->Tcw || !levelSigma2_2 || !F12 || !npairs ||
        cap < 0 || (cap && !pairs))
        return ORB_E_INVALID;
    const int n1 = KF1->N, n2 = KF2->N;
    if (!featvec_ok(fv1, n1) || !featvec_ok(fv2, n2) || (n1 && !has_mp1) || (n2 && !has_mp2)) return ORB_E_INVALID;
    Matcher* m = h->m;
    if (m->device_pointers()) return ORB_E_INVALID;
    // epipole in the second image (ORBmatcher.cc:664-671)
    float Cw[3], C2[3];
    camera_center(KF1->Tcw, Cw);
    for (int r = 0; r < 3; r++) C2[r] = gemm_row(KF2->Tcw, r, Cw);
    const float invz = 1.0f / C2[2];
    const float ex = KF2->fx * C2[0] * invz + KF2->cx;
    const float ey = KF2->fy * C2[1] * invz + KF2->cy;
    auto stereo1 = [&](int i) { return KF1->uRight && KF1->uRight[i] >= 0; };
    auto stereo2 = [&](int i) { return KF2->uRight && KF2->uRight[i] >= 0; };
    std::vector<uint8_t> ok1((size_t)n1), ok2((size_t)n2);
    for (int i = 0; i < n1; i++) ok1[i] = !has_mp1[i] && (!bOnlyStereo || stereo1(i));
    for (int i = 0; i < n2; i++) ok2[i] = !has_mp2[i] && (!bOnlyStereo || stereo2(i));   // vbMatched2 never set
    NodeLists L;
    if (int e = node_lists(m, fv1, ok1.data(), KF1->desc, n1, fv2, ok2.data(), KF2->desc, n2, L)) return e;
    std::vector<int> m12((size_t)n1, -1);
    int nm = 0;
    RotHist H;
    for (size_t q = 0; q < L.qidx.size(); q++) {
        const int idx1 = L.qidx[q];
        const orb_kp& kp1 = KF1->keysUn[idx1];
        const bool bStereo1 = stereo1(idx1);
        // CheckDistEpipolarLine line coefficients (140-145)
        const float a = kp1.x * F12[0] + kp1.y * F12[3] + F12[6];
        const float b = kp1.x * F12[1] + kp1.y * F12[4] + F12[7];
        const float c = kp1.x * F12[2] + kp1.y * F12[5] + F12[8];
        int bestDist = kThLow, bestIdx2 = -1;
        for (int k = L.off[q]; k < L.off[q + 1]; k++) {
            const int idx2 = L.cand[k], dist = L.dist[k];
            if (dist > kThLow || dist > bestDist) continue;   // later candidates win ties
            const orb_kp& kp2 = KF2->keysUn[idx2];
            if (!bStereo1 && !stereo2(idx2)) {
                const float distex = ex - kp2.x, distey = ey - kp2.y;
                if (distex * distex + distey * distey < 100 * KF2->scaleFactors[kp2.octave]) continue;
            }
            const float num = a * kp2.x + b * kp2.y + c;
            const float den = a * a + b * b;
            if (den == 0) continue;
            const float dsqr = num * num / den;
            if (dsqr < 3.84 * levelSigma2_2[kp2.octave]) {
                bestIdx2 = idx2;
                bestDist = dist;
            }
        }
        if (bestIdx2 >= 0) {
            m12[idx1] = bestIdx2;
            nm++;
            if (m->check_ori()) H.push(kp1.angle, KF2->keysUn[bestIdx2].angle, idx1);
        }
    }
    if (m->check_ori())
        H.reject([&](int idx1) {
            m12[idx1] = -1;
            nm--;
        });
    int np = 0;
    for (int i = 0; i < n1; i++)
        if (m12[i] >= 0) {
            if (np < cap) {
                pairs[2 * np] = i;
                pairs[2 * np + 1] = m12[i];
            }
            np++;
        }
    *npairs = np;
    return np > cap ? ORB_E_CAPACITY : ORB_OK;
}

int ORBmatcher_SearchByProjection_Sim3(ORBmatcher_h h, const orb_frame* KF, const float* Scw,
                                       const orb_mappoints* pts, const orb_mappoint_geo* geo, const uint8_t* skip,
                                       float logScaleFactor, int th, int32_t* matched, int* nmatches) {
    if (!h || !frame_ok(KF) || !Scw || !geo_ok(pts, geo, true) || (pts->n && !skip) || !nmatches ||
        (KF->N && !matched))
        return ORB_E_INVALID;
    Matcher* m = h->m;
    if (m->device_pointers()) return ORB_E_INVALID;
    const SimPose P = pose_Scw(Scw);
    const int n = pts->n;
    ProjPass pp;
    pp.reset(n);
    for (int i = 0; i < n; i++) {
        if (skip[i]) continue;
        float u, v, ur;
        const int lvl = project_point(KF, P, pts->pos + 3 * (size_t)i, geo->max_dist[i], geo->min_dist[i],
                                      geo->normal + 3 * (size_t)i, logScaleFactor, 0, 0.f, &u, &v, &ur);
        if (lvl < 0) continue;
        pp.add(u, v, th * KF->scaleFactors[lvl], lvl, pts->desc + 32 * (size_t)i, u, v, ur, (size_t)i);
    }
    if (int e = pp.run(m, KF)) return e;
    // greedy replay in vpPoints order: vpMatched occupancy grows as points are matched (375, 396)
    int nm = 0;
    for (int i = 0; i < n; i++) {
        if (pp.q[i].qd < 0) continue;
        int bestDist = 256, bestIdx = -1;
        for (int k = pp.off[i]; k < pp.off[i + 1]; k++) {
            const int idx = pp.cand[k].x;
            if (matched[idx] >= 0) continue;
            if (pp.cand[k].y < bestDist) {
                bestDist = pp.cand[k].y;
                bestIdx = idx;
            }
        }
        if (bestDist <= kThLow) {
            matched[bestIdx] = i;
            nm++;
        }
    }
    *nmatches = nm;
    return ORB_OK;
}

int ORBmatcher_Fuse(ORBmatcher_h h, const orb_frame* KF, const orb_mappoints* pts, const orb_mappoint_geo* geo,
                    const uint8_t* skip, float logScaleFactor, float th, int32_t* best, int* nfused) {
    if (!h || !frame_ok(KF) || !KF->Tcw || !geo_ok(pts, geo, true) || (pts->n && (!skip || !best)) || !nfused)
        return ORB_E_INVALID;
    if (h->m->device_pointers()) return ORB_E_INVALID;
    return fuse_common(h->m, KF, pose_T(KF->Tcw), false, pts, geo, skip, logScaleFactor, th, best, nfused);
}

int ORBmatcher_Fuse_Sim3(ORBmatcher_h h, const orb_frame* KF, const float* Scw, const orb_mappoints* pts,
                         const orb_mappoint_geo* geo, const uint8_t* skip, float logScaleFactor, float th,
                         int32_t* best, int* nfused) {
    if (!h || !frame_ok(KF) || !Scw || !geo_ok(pts, geo, true) || (pts->n && (!skip || !best)) || !nfused)
        return ORB_E_INVALID;
    if (h->m->device_pointers()) return ORB_E_INVALID;
    return fuse_common(h->m, KF, pose_Scw(Scw), true, pts, geo, skip, logScaleFactor, th, best, nfused);
}

int ORBmatcher_SearchBySim3(ORBmatcher_h h, const orb_frame* KF1, const int32_t* mp1, const orb_frame* KF2,
                            const int32_t* mp2, const orb_mappoints* pts, const orb_mappoint_geo* geo,
                            const uint8_t* bad, float s12, const float* R12, const float* t12, float logScaleFactor,
                            float th, int32_t* matches12, int* nfound) {
    if (!h || !frame_ok(KF1) || !frame_ok(KF2) || !KF1->Tcw || !KF2->Tcw || !geo_ok(pts, geo, false) ||
        (pts->n && !bad) || !R12 || !t12 || !nfound || (KF1->N && (!mp1 || !matches12)) || (KF2->N && !mp2))
        return ORB_E_INVALID;
    Matcher* m = h->m;
    if (m->device_pointers()) return ORB_E_INVALID;
    const int N1 = KF1->N, N2 = KF2->N;
    for (int i = 0; i < N1; i++)
        if (mp1[i] >= pts->n || matches12[i] < -2 || matches12[i] >= N2) return ORB_E_INVALID;
    for (int i = 0; i < N2; i++)
        if (mp2[i] >= pts->n) return ORB_E_INVALID;
    const SimPose P1 = pose_T(KF1->Tcw), P2 = pose_T(KF2->Tcw);
    // sR12 = s12*R12, sR21 = (1.0/s12)*R12.t(), t21 = -sR21*t12 (ORBmatcher.cc:1119-1121)
    float sR12[9], sR21[9], t21[3];
    const float a21 = (float)(1.0 / (double)s12);
    for (int r = 0; r < 3; r++)
        for (int c = 0; c < 3; c++) {
            sR12[r * 3 + c] = R12[r * 3 + c] * s12 + 0.0f;
            sR21[r * 3 + c] = R12[c * 3 + r] * a21 + 0.0f;
        }
    for (int r = 0; r < 3; r++) {
        const double sacc = (double)sR21[r * 3] * t12[0] + (double)sR21[r * 3 + 1] * t12[1] + (double)sR21[r * 3 + 2] * t12[2];
        t21[r] = (float)(sacc * -1.0);
    }
    std::vector<uint8_t> am1((size_t)N1), am2((size_t)N2);
    for (int i = 0; i < N1; i++)
        if (matches12[i] != -1) {
            am1[i] = 1;
            if (matches12[i] >= 0) am2[matches12[i]] = 1;
        }
    // one direction: side A's points through A's pose and (sR, t) into side B (1148-1225 / 1228-1305)
    auto direction = [&](const orb_frame* B, const SimPose& Aw, const float* sR, const float* t, int NA,
                         const int32_t* mpA, const std::vector<uint8_t>& amA, std::vector<int>& vn) -> int {
        ProjPass pp;
        pp.reset(NA);
        vn.assign((size_t)NA, -1);
        for (int i = 0; i < NA; i++) {
            const int mp = mpA[i];
            if (mp < 0 || amA[i] || bad[mp]) continue;
            const float* X = pts->pos + 3 * (size_t)mp;
            float c1[3], c2[3];
            for (int r = 0; r < 3; r++) c1[r] = gemm3(Aw.R, Aw.t, r, X);
            for (int r = 0; r < 3; r++) c2[r] = gemm3(sR, t, r, c1);
            if (c2[2] < 0.0) continue;
            const float invz = (float)(1.0 / (double)c2[2]);
            const float x = c2[0] * invz, y = c2[1] * invz;
            const float u = KF1->fx * x + KF1->cx, v = KF1->fy * y + KF1->cy;   // pKF1's intrinsics
            if (!kf_in_image(B, u, v)) continue;
            const float dist3D = norm3f(c2);
            if (dist3D < 0.8f * geo->min_dist[mp] || dist3D > 1.2f * geo->max_dist[mp]) continue;
            const int lvl = predict_scale(geo->max_dist[mp], dist3D, logScaleFactor, B->nlevels);
            pp.add(u, v, th * B->scaleFactors[lvl], lvl, pts->desc + 32 * (size_t)mp, u, v, 0.f, (size_t)i);
        }
        if (int e = pp.run(m, B)) return e;
        for (int i = 0; i < NA; i++) {
            if (pp.q[i].qd < 0) continue;
            int bestDist = INT_MAX, bestIdx = -1;
            for (int k = pp.off[i]; k < pp.off[i + 1]; k++)
                if (pp.cand[k].y < bestDist) {
                    bestDist = pp.cand[k].y;
                    bestIdx = pp.cand[k].x;
                }
            if (bestDist <= 100) vn[i] = bestIdx;   // TH_HIGH
        }
        return ORB_OK;
    };
    std::vector<int> vn1, vn2;
    if (int e = direction(KF2, P1, sR21, t21, N1, mp1, am1, vn1)) return e;
    if (int e = direction(KF1, P2, sR12, t12, N2, mp2, am2, vn2)) return e;
    int nf = 0;
    for (int i1 = 0; i1 < N1; i1++) {
        const int idx2 = vn1[i1];
        if (idx2 >= 0 && vn2[idx2] == i1) {
            matches12[i1] = idx2;
            nf++;
        }
    }
    *nfound = nf;
    return ORB_OK;
}

}  // extern "C"
