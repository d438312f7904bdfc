// capi_stereo.cpp -- extern "C" ORBmatcher_ComputeStereoMatches[_batch] (include/orbslam_gpu.h).
// Replaces ORB_SLAM2::Frame::ComputeStereoMatches (reference src/Frame.cc:466-640).
#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "capi_handles.hpp"
#include "stereo.hpp"

namespace {
size_t al(size_t n) { return (n + 255) & ~(size_t)255; }

template <class T>
T* up(orbgpu::Matcher* m, const T* src, size_t count, hipStream_t s, int* err) {
    if (!src || count == 0) return nullptr;
    void* d = m->arena_alloc(count * sizeof(T));
    if (!d || hipMemcpyAsync(d, src, count * sizeof(T), hipMemcpyHostToDevice, s) != hipSuccess) {
        *err = ORB_E_HIP;
        return nullptr;
    }
    return (T*)d;
}
}  // namespace

extern "C" {

int ORBmatcher_ComputeStereoMatches_batch(ORBmatcher_h h, ORBextractor_h left, ORBextractor_h right, int npairs,
                                          const int* NL, const orb_kp* const* keysL, const uint8_t* const* descL,
                                          const int* NR, const orb_kp* const* keysR,
                                          const uint8_t* const* descR, float mbf, float mb,
                                          float* const* uRight, float* const* depth, int* nmatches) {
    return ORBmatcher_ComputeStereoMatches_batch_at(h, left, 0, right, 0, npairs, NL, keysL, descL, NR, keysR, descR,
                                                    mbf, mb, uRight, depth, nmatches);
}

int ORBmatcher_ComputeStereoMatches_batch_at(ORBmatcher_h h, ORBextractor_h left, int first_left,
                                             ORBextractor_h right, int first_right, int npairs, const int* NL,
                                             const orb_kp* const* keysL, const uint8_t* const* descL, const int* NR,
                                             const orb_kp* const* keysR, const uint8_t* const* descR, float mbf,
                                             float mb, float* const* uRight, float* const* depth, int* nmatches) {
    if (!h || !left || !right || npairs < 0 || first_left < 0 || first_right < 0 || !NL || !keysL || !descL || !NR ||
        !keysR || !descR || !uRight || !depth || !nmatches)
        return ORB_E_INVALID;
    if (npairs == 0) return ORB_OK;
    const orbgpu::Extractor* EL = left->ex;
    const orbgpu::Extractor* ER = right->ex;
    if (!EL->pyramid_base() || !ER->pyramid_base() || first_left + npairs > EL->last_batch() ||
        first_right + npairs > ER->last_batch())
        return ORB_E_INVALID;   // images first + p of the last extract() of the extractors
    const auto& LL = EL->levels();
    const auto& LR = ER->levels();
    if (LL.size() != LR.size() || (int)LL.size() > orbgpu::kStereoMaxLevels) return ORB_E_INVALID;
    for (size_t l = 0; l < LL.size(); l++)
        if (LL[l].w != LR[l].w || LL[l].h != LR[l].h || LL[l].pitch != LR[l].pitch || LL[l].off != LR[l].off)
            return ORB_E_INVALID;   // a rectified pair: equal image geometry
    if (!(mb > 0.0f)) return ORB_E_INVALID;
    for (int p = 0; p < npairs; p++) {
        if (NL[p] < 0 || NR[p] < 0 || NL[p] > orbgpu::kStereoMaxKeys || NR[p] > 65535) return ORB_E_INVALID;
        if ((NL[p] && (!keysL[p] || !descL[p] || !uRight[p] || !depth[p])) || (NR[p] && (!keysR[p] || !descR[p])))
            return ORB_E_INVALID;
    }
    orbgpu::Matcher* m = h->m;
    const bool dev = m->device_pointers();
    hipStream_t s = m->stream();
    // the pyramids are produced on the extractors' streams
    if (orbgpu::stream_wait(EL->stream()) != hipSuccess ||
        (ER != EL && orbgpu::stream_wait(ER->stream()) != hipSuccess))
        return ORB_E_HIP;
    orbgpu::StereoParams P;
    std::memset(&P, 0, sizeof(P));
    for (size_t l = 0; l < LL.size(); l++) {
        P.lv[l].off = (long long)LL[l].off;
        P.lv[l].pitch = LL[l].pitch;
        P.lv[l].w = LL[l].w;
        P.lv[l].h = LL[l].h;
        P.scale[l] = EL->scale()[l];
        P.invScale[l] = EL->inv_scale()[l];
    }
    P.mbf = mbf;
    P.mb = mb;
    P.rows0 = LL[0].h;
    if (P.rows0 > orbgpu::kStereoMaxRows) return ORB_E_INVALID;
    // rows a right keypoint covers: ceil(y + r) - floor(y - r) + 1 <= 2r + 3, r = 2 * scale
    const int band = (int)std::ceil(4.0f * EL->scale()[LL.size() - 1]) + 3;
    size_t need = al(sizeof(orbgpu::StereoDev) * npairs) + al(4 * (size_t)npairs);
    int maxNL = 0;
    for (int p = 0; p < npairs; p++) {
        need += al(4 * (size_t)NL[p]) + al(4 * ((size_t)P.rows0 + 1)) + al(8 * (size_t)NR[p] * band + 8);
        if (!dev) need += al(28 * (size_t)NL[p]) + al(32 * (size_t)NL[p]) + al(28 * (size_t)NR[p]) +
                          al(32 * (size_t)NR[p]) + 2 * al(4 * (size_t)NL[p]);
        maxNL = std::max(maxNL, NL[p]);
    }
    if (m->arena_reserve(need + 4096)) return ORB_E_HIP;
    int err = 0;
    std::vector<orbgpu::StereoDev> probs(npairs);
    int* d_kept = (int*)(dev ? m->count_buf(4 * (size_t)npairs) : m->arena_alloc(4 * (size_t)npairs));
    for (int p = 0; p < npairs; p++) {
        orbgpu::StereoDev& S = probs[p];
        S.NL = NL[p];
        S.NR = NR[p];
        S.pyrL = EL->pyramid_base() + (size_t)(first_left + p) * EL->pyramid_image_bytes();
        S.pyrR = ER->pyramid_base() + (size_t)(first_right + p) * ER->pyramid_image_bytes();
        S.sad = (int*)m->arena_alloc(4 * (size_t)NL[p] + 4);
        S.rowStart = (int*)m->arena_alloc(4 * ((size_t)P.rows0 + 1));
        S.rowIdx = (int2*)m->arena_alloc(8 * (size_t)NR[p] * band + 8);
        if (!S.sad || !S.rowStart || !S.rowIdx) return ORB_E_HIP;
        S.kept = d_kept + p;
        if (dev) {
            S.kL = (const orbgpu::orb_kp_dev*)keysL[p];
            S.dL = descL[p];
            S.kR = (const orbgpu::orb_kp_dev*)keysR[p];
            S.dR = descR[p];
            S.uRight = uRight[p];
            S.depth = depth[p];
        } else {
            S.kL = (const orbgpu::orb_kp_dev*)up(m, keysL[p], (size_t)NL[p], s, &err);
            S.dL = up(m, descL[p], 32 * (size_t)NL[p], s, &err);
            S.kR = (const orbgpu::orb_kp_dev*)up(m, keysR[p], (size_t)NR[p], s, &err);
            S.dR = up(m, descR[p], 32 * (size_t)NR[p], s, &err);
            S.uRight = (float*)m->arena_alloc(4 * (size_t)NL[p] + 4);
            S.depth = (float*)m->arena_alloc(4 * (size_t)NL[p] + 4);
        }
    }
    if (err || !d_kept) return ORB_E_HIP;
    auto* d_probs = (orbgpu::StereoDev*)m->arena_alloc(sizeof(orbgpu::StereoDev) * npairs);
    if (!d_probs) return ORB_E_HIP;
    if (hipMemcpyAsync(d_probs, m->h2d_src(probs.data(), sizeof(orbgpu::StereoDev) * npairs),
                       sizeof(orbgpu::StereoDev) * npairs, hipMemcpyHostToDevice, s) != hipSuccess)
        return ORB_E_HIP;
    if (orbgpu::stereo_launch(d_probs, npairs, maxNL, P, s, m)) return ORB_E_HIP;
    if (dev) {   // device mode may be deferred (ORBmatcher_set_deferred)
        if (m->d2h_counts(nmatches, d_kept, 4 * (size_t)npairs)) return ORB_E_HIP;
        return m->end_call() ? ORB_E_HIP : ORB_OK;
    }
    if (hipMemcpyAsync(nmatches, d_kept, 4 * (size_t)npairs, hipMemcpyDeviceToHost, s) != hipSuccess)
        return ORB_E_HIP;
    if (!dev)
        for (int p = 0; p < npairs; p++)
            if (NL[p] && (hipMemcpyAsync(uRight[p], probs[p].uRight, 4 * (size_t)NL[p], hipMemcpyDeviceToHost, s) !=
                              hipSuccess ||
                          hipMemcpyAsync(depth[p], probs[p].depth, 4 * (size_t)NL[p], hipMemcpyDeviceToHost, s) !=
                              hipSuccess))
                return ORB_E_HIP;
    return orbgpu::stream_wait(s) == hipSuccess ? ORB_OK : ORB_E_HIP;
}

int ORBmatcher_ComputeStereoMatches(ORBmatcher_h h, ORBextractor_h left, ORBextractor_h right, int index, int NL,
                                    const orb_kp* keysL, const uint8_t* descL, int NR, const orb_kp* keysR,
                                    const uint8_t* descR, float mbf, float mb, float* uRight, float* depth,
                                    int* nmatches) {
    if (!h || !left || !right || index < 0) return ORB_E_INVALID;
    if (index != 0) return ORB_E_INVALID;   // single form: image 0 of the last extract() call
    return ORBmatcher_ComputeStereoMatches_batch(h, left, right, 1, &NL, &keysL, &descL, &NR, &keysR, &descR, mbf,
                                                 mb, &uRight, &depth, nmatches);
}

int Frame_UnprojectStereo_batch_device(ORBmatcher_h h, int count, const orb_unproject* U) {
    if (!h || count < 0 || (count > 0 && !U)) return ORB_E_INVALID;
    if (count == 0) return ORB_OK;
    std::vector<orbgpu::UnprojDev> P((size_t)count);
    int maxN = 0;
    for (int f = 0; f < count; f++) {
        const orb_unproject& Q = U[f];
        if (Q.N < 0 || (Q.N > 0 && (!Q.keysUn || !Q.depth || !Q.Twc || !Q.x3D))) return ORB_E_INVALID;
        orbgpu::UnprojDev& d = P[f];
        d.N = Q.N;
        d.keys = (const orbgpu::orb_kp_dev*)Q.keysUn;
        d.depth = Q.depth;
        d.Twc = Q.Twc;
        d.fx = Q.fx; d.fy = Q.fy; d.cx = Q.cx; d.cy = Q.cy;
        d.invfx = 1.0f / Q.fx;   // Frame.cc:108-109
        d.invfy = 1.0f / Q.fy;
        d.x3D = Q.x3D;
        d.mp = Q.mp;
        maxN = std::max(maxN, Q.N);
    }
    (void)maxN;
    return orbgpu::unproject_batch(P.data(), count, h->m->stream()) ? ORB_E_HIP : ORB_OK;
}

static int fill_undist(const orb_undistort& q, orbgpu::UndistDev& d) {
    if (q.N < 0 || q.N > (1 << 24) || (q.N > 0 && (!q.keys || !q.keysUn))) return ORB_E_INVALID;
    if (q.ndist != 4 && q.ndist != 5 && q.ndist != 8) return ORB_E_INVALID;   // cv::undistortPoints sizes ORB-SLAM2 reads
    std::memset(&d, 0, sizeof(d));
    d.N = q.N;
    d.keys = (const orbgpu::orb_kp_dev*)q.keys;
    d.keysUn = (orbgpu::orb_kp_dev*)q.keysUn;
    d.has_dist = q.dist[0] != 0.0f;   // Frame.cc:406: mDistCoef.at<float>(0)==0.0 -> mvKeysUn = mvKeys
    for (int i = 0; i < 9; i++) d.A[i] = (double)q.K[i];
    for (int i = 0; i < 8; i++) d.k[i] = i < q.ndist ? (double)q.dist[i] : 0.0;
    return ORB_OK;
}

int Frame_UndistortKeyPoints_batch(ORBmatcher_h h, int count, const orb_undistort* U) {
    if (!h || count < 0 || (count > 0 && !U)) return ORB_E_INVALID;
    if (count == 0) return ORB_OK;
    std::vector<orbgpu::UndistDev> P((size_t)count);
    for (int f = 0; f < count; f++)
        if (int e = fill_undist(U[f], P[f])) return e;
    hipStream_t s = h->m->stream();
    if (h->m->device_pointers()) return orbgpu::undistort_batch(P.data(), count, s) ? ORB_E_HIP : ORB_OK;
    // host arrays: one device block holding every frame's keys and results, copied per call
    size_t tot = 0;
    for (int f = 0; f < count; f++) tot += (size_t)P[f].N;
    if (tot == 0) return ORB_OK;
    void* d = nullptr;
    if (hipMalloc(&d, 2 * tot * sizeof(orb_kp)) != hipSuccess) return ORB_E_HIP;
    orbgpu::orb_kp_dev* dk = (orbgpu::orb_kp_dev*)d;
    int rc = ORB_OK;
    size_t o = 0;
    for (int f = 0; f < count && rc == ORB_OK; f++) {
        if (P[f].N && hipMemcpyAsync(dk + o, U[f].keys, P[f].N * sizeof(orb_kp), hipMemcpyHostToDevice, s) != hipSuccess)
            rc = ORB_E_HIP;
        P[f].keys = dk + o;
        P[f].keysUn = dk + tot + o;
        o += (size_t)P[f].N;
    }
    if (rc == ORB_OK && orbgpu::undistort_batch(P.data(), count, s)) rc = ORB_E_HIP;
    o = 0;
    for (int f = 0; f < count && rc == ORB_OK; f++) {
        if (P[f].N && hipMemcpyAsync(U[f].keysUn, dk + tot + o, P[f].N * sizeof(orb_kp), hipMemcpyDeviceToHost, s) !=
                          hipSuccess)
            rc = ORB_E_HIP;
        o += (size_t)P[f].N;
    }
    if (orbgpu::stream_wait(s) != hipSuccess) rc = ORB_E_HIP;
    (void)hipFree(d);
    return rc;
}

int Frame_UndistortKeyPoints(ORBmatcher_h h, const orb_undistort* U) {
    if (!h || !U) return ORB_E_INVALID;
    if (h->m->device_pointers()) {   // the single form is synchronous in either pointer space
        const int e = Frame_UndistortKeyPoints_batch(h, 1, U);
        if (e) return e;
        return orbgpu::stream_wait(h->m->stream()) == hipSuccess ? ORB_OK : ORB_E_HIP;
    }
    return Frame_UndistortKeyPoints_batch(h, 1, U);
}

int Frame_ComputeImageBounds(ORBmatcher_h h, int cols, int rows, const float* K, const float* dist, int ndist,
                             float* bounds) {
    if (!h || !K || !dist || !bounds || cols <= 0 || rows <= 0) return ORB_E_INVALID;
    if (ndist != 4 && ndist != 5 && ndist != 8) return ORB_E_INVALID;
    if (dist[0] != 0.0f) {   // Frame.cc:438-455: the four image corners through cv::undistortPoints
        orb_kp c[4];
        std::memset(c, 0, sizeof(c));
        c[1].x = (float)cols;
        c[2].y = (float)rows;
        c[3].x = (float)cols; c[3].y = (float)rows;
        orb_kp u[4];
        orb_undistort q;
        std::memset(&q, 0, sizeof(q));
        q.N = 4;
        q.keys = c;
        q.keysUn = u;
        std::memcpy(q.K, K, sizeof(q.K));
        for (int i = 0; i < ndist; i++) q.dist[i] = dist[i];
        q.ndist = ndist;
        const bool dev = h->m->device_pointers();
        h->m->set_device_pointers(false);   // the corners are host values
        const int e = Frame_UndistortKeyPoints_batch(h, 1, &q);
        h->m->set_device_pointers(dev);
        if (e) return e;
        bounds[0] = std::min(u[0].x, u[2].x);   // mnMinX = min(mat(0,0), mat(2,0))
        bounds[1] = std::max(u[1].x, u[3].x);
        bounds[2] = std::min(u[0].y, u[1].y);
        bounds[3] = std::max(u[2].y, u[3].y);
    } else {
        bounds[0] = 0.0f;
        bounds[1] = (float)cols;
        bounds[2] = 0.0f;
        bounds[3] = (float)rows;
    }
    // Frame.cc:155-156 (FRAME_GRID_COLS / ROWS = 64 / 48)
    bounds[4] = static_cast<float>(64) / static_cast<float>(bounds[1] - bounds[0]);
    bounds[5] = static_cast<float>(48) / static_cast<float>(bounds[3] - bounds[2]);
    return ORB_OK;
}

int MapPoint_CreateStereo_batch_device(ORBmatcher_h h, int count, const orb_newpoints* Q) {
    if (!h || count < 0 || (count > 0 && !Q)) return ORB_E_INVALID;
    if (count == 0) return ORB_OK;
    std::vector<orbgpu::UnprojDev> P((size_t)count);
    for (int f = 0; f < count; f++) {
        const orb_newpoints& q = Q[f];
        if (q.N < 0 || (q.N > 0 && (!q.keysUn || !q.depth || !q.Twc || !q.x3D || !q.row || !q.normal ||
                                    !q.max_dist || !q.min_dist || !q.scaleFactors || q.nlevels <= 0)))
            return ORB_E_INVALID;
        orbgpu::UnprojDev& d = P[f];
        std::memset(&d, 0, sizeof(d));
        d.N = q.N;
        d.keys = (const orbgpu::orb_kp_dev*)q.keysUn;
        d.depth = q.depth;
        d.Twc = q.Twc;
        d.fx = q.fx; d.fy = q.fy; d.cx = q.cx; d.cy = q.cy;
        d.invfx = 1.0f / q.fx;
        d.invfy = 1.0f / q.fy;
        d.x3D = q.x3D;
        d.mp = q.row;
        d.mp_base = q.row_base;
        d.normal = q.normal;
        d.maxDist = q.max_dist;
        d.minDist = q.min_dist;
        d.scale = q.scaleFactors;
        d.nlevels = q.nlevels;
    }
    return orbgpu::unproject_batch(P.data(), count, h->m->stream()) ? ORB_E_HIP : ORB_OK;
}

int Tracking_PrepareLocalSearch_batch_device(ORBmatcher_h h, int count, const orb_localprep* Q) {
    if (!h || count < 0 || (count > 0 && !Q)) return ORB_E_INVALID;
    if (count == 0) return ORB_OK;
    orbgpu::Matcher* m = h->m;
    std::vector<orbgpu::LocalPrepDev> P((size_t)count);
    for (int f = 0; f < count; f++) {
        const orb_localprep& q = Q[f];
        if (q.N < 0 || q.n < 0 || (q.N > 0 && (!q.cur_mp || !q.outlier)) || (q.n > 0 && (!q.row || !q.skip)))
            return ORB_E_INVALID;
        P[f] = orbgpu::LocalPrepDev{q.N, q.cur_mp, q.outlier, q.n, q.row, q.skip};
    }
    if (m->arena_reserve(sizeof(orbgpu::LocalPrepDev) * count + 256)) return ORB_E_HIP;
    void* d = m->arena_alloc(sizeof(orbgpu::LocalPrepDev) * count);
    hipStream_t s = m->stream();
    if (!d || hipMemcpyAsync(d, m->h2d_src(P.data(), sizeof(orbgpu::LocalPrepDev) * count),
                             sizeof(orbgpu::LocalPrepDev) * count, hipMemcpyHostToDevice, s) != hipSuccess)
        return ORB_E_HIP;
    if (orbgpu::local_prep_batch((const orbgpu::LocalPrepDev*)d, count, s)) return ORB_E_HIP;
    // outside deferred mode the staging copy is pageable: finish before the host vector goes
    return m->end_call() ? ORB_E_HIP : ORB_OK;
}

}  // extern "C"
