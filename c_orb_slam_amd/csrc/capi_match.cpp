// capi_match.cpp -- extern "C" ORBmatcher_* entry points (include/orbslam_gpu.h).
// Each replaces a member of ORB_SLAM2::ORBmatcher (reference include/ORBmatcher.h:41-103).
#include <cstring>
#include <new>
#include <vector>

#include "capi_handles.hpp"

using orbgpu::FrameDev;
using orbgpu::Matcher;
using orbgpu::SearchDev;


namespace {

size_t al(size_t n) { return (n + 255) & ~(size_t)255; }

// Host-pointer mode: copy one host array into the arena, return its device address.
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

size_t frame_bytes(const orb_frame* f) {
    if (!f) return 0;
    return al((size_t)f->N * 28) + al((size_t)f->N * 32) + (f->uRight ? al((size_t)f->N * 4) : 0) +
           al((size_t)f->nlevels * 4) + al(64);
}

FrameDev frame_dev(Matcher* m, const orb_frame* f, bool dev, hipStream_t s, int* err) {
    FrameDev d;
    memset(&d, 0, sizeof(d));
    if (!f) return d;
    d.N = f->N;
    d.minX = f->minX; d.maxX = f->maxX; d.minY = f->minY; d.maxY = f->maxY;
    d.gridWInv = f->gridWInv; d.gridHInv = f->gridHInv;
    d.nlevels = f->nlevels;
    d.fx = f->fx; d.fy = f->fy; d.cx = f->cx; d.cy = f->cy; d.bf = f->bf; d.b = f->b;
    if (dev) {
        d.keysUn = (const orbgpu::orb_kp_dev*)f->keysUn;
        d.desc = f->desc;
        d.uRight = f->uRight;
        d.scale = f->scaleFactors;
        d.Tcw = f->Tcw;
    } else {
        d.keysUn = (const orbgpu::orb_kp_dev*)up(m, f->keysUn, (size_t)f->N, s, err);
        d.desc = up(m, f->desc, (size_t)f->N * 32, s, err);
        d.uRight = up(m, f->uRight, f->uRight ? (size_t)f->N : 0, s, err);
        d.scale = up(m, f->scaleFactors, (size_t)f->nlevels, s, err);
        d.Tcw = up(m, f->Tcw, 16, s, err);
    }
    return d;
}

bool frame_ok(const orb_frame* f) {
    return f && f->N >= 0 && f->N <= orbgpu::kMaxFrameKeys && (f->N == 0 || (f->keysUn && f->desc)) &&
           f->scaleFactors && f->Tcw && f->nlevels > 0;
}

}  // namespace

extern "C" {

int ORBmatcher_create(float nnratio, int checkOri, ORBmatcher_h* out) {
    if (!out) return ORB_E_INVALID;
    *out = nullptr;
    auto* m = new (std::nothrow) Matcher(nnratio, checkOri != 0);
    if (!m) return ORB_E_INVALID;
    int rc = m->init_device();
    if (rc) {
        delete m;
        return rc == -4 ? ORB_E_NODEVICE : ORB_E_HIP;
    }
    *out = new ORBmatcher_t{m};
    return ORB_OK;
}

int ORBmatcher_destroy(ORBmatcher_h h) {
    if (!h) return ORB_E_INVALID;
    delete h->m;
    delete h;
    return ORB_OK;
}

int ORBmatcher_set_device_pointers(ORBmatcher_h h, int on) {
    if (!h) return ORB_E_INVALID;
    h->m->set_device_pointers(on != 0);
    return ORB_OK;
}

void* ORBmatcher_stream(ORBmatcher_h h) { return h ? (void*)h->m->stream() : nullptr; }

int ORBmatcher_enable_timing(ORBmatcher_h h, int on) {
    if (!h) return ORB_E_INVALID;
    return h->m->set_timing(on != 0) ? ORB_E_HIP : ORB_OK;
}

int ORBmatcher_set_deferred(ORBmatcher_h h, int on) {
    if (!h || !h->m->device_pointers()) return ORB_E_INVALID;   // device-resident batches only
    if (!on && h->m->chain().on() && h->m->chain().finish(h->m->stream())) return ORB_E_HIP;
    h->m->chain().set(on != 0);
    return ORB_OK;
}

int ORBmatcher_finish(ORBmatcher_h h) {
    if (!h) return ORB_E_INVALID;
    return h->m->chain().finish(h->m->stream()) ? ORB_E_HIP : ORB_OK;
}

int ORBmatcher_chain_close(ORBmatcher_h h, long long* epoch) {
    if (!h || !epoch || !h->m->chain().on()) return ORB_E_INVALID;
    return h->m->chain().close(h->m->stream(), epoch) ? ORB_E_HIP : ORB_OK;
}

int ORBmatcher_chain_wait(ORBmatcher_h h, long long epoch) {
    if (!h) return ORB_E_INVALID;
    return h->m->chain().wait(epoch) ? ORB_E_HIP : ORB_OK;
}

int ORBmatcher_chain_finish(ORBmatcher_h h, long long epoch) {
    if (!h) return ORB_E_INVALID;
    return h->m->chain().finish_upto(epoch) ? ORB_E_HIP : ORB_OK;
}

int ORBmatcher_last_timings(ORBmatcher_h h, float* ms8, long long* counts8) {
    if (!h || !ms8 || !counts8) return ORB_E_INVALID;
    return h->m->timings(ms8, counts8) ? ORB_E_HIP : ORB_OK;
}

// ORBmatcher.cc:1647-1663 (SWAR popcount == popcount)
int ORBmatcher_DescriptorDistance(const uint8_t* a, const uint8_t* b) {
    if (!a || !b) return ORB_E_INVALID;
    int dist = 0;
    for (int i = 0; i < 8; i++) {
        uint32_t pa, pb;
        memcpy(&pa, a + 4 * i, 4);
        memcpy(&pb, b + 4 * i, 4);
        dist += __builtin_popcount(pa ^ pb);
    }
    return dist;
}

int ORBmatcher_SearchByProjection_LastFrame_batch(ORBmatcher_h h, int npairs, const orb_frame* cur,
                                                  int32_t* const* cur_mp, const orb_frame* last,
                                                  const orb_kp* const* last_keys, const int32_t* const* last_mp,
                                                  const uint8_t* const* last_outlier, const orb_mappoints* mps,
                                                  float th, int bMono, int* nmatches) {
    if (!h || npairs < 0 || !cur || !cur_mp || !last || !last_keys || !last_mp || !last_outlier || !mps || !nmatches)
        return ORB_E_INVALID;
    Matcher* m = h->m;
    const bool dev = m->device_pointers();
    hipStream_t s = m->stream();
    for (int p = 0; p < npairs; p++) {
        if (!frame_ok(&cur[p]) || !last[p].Tcw || last[p].N < 0 || (last[p].N > 0 && !last[p].keysUn)) return ORB_E_INVALID;
        if (last[p].N > 0 && (!last_keys[p] || !last_mp[p] || !last_outlier[p])) return ORB_E_INVALID;
        if (mps[p].n > 0 && (!mps[p].pos || !mps[p].desc || !mps[p].observations)) return ORB_E_INVALID;
        if (!dev) {  // host mode: validate map point indices (device mode trusts the caller)
            for (int i = 0; i < last[p].N; i++)
                if (last_mp[p][i] >= mps[p].n) return ORB_E_INVALID;
            for (int i = 0; i < cur[p].N; i++)
                if (cur_mp[p][i] >= mps[p].n) return ORB_E_INVALID;
        }
    }
    int err = 0;
    std::vector<SearchDev> probs(npairs);
    if (!dev) {
        size_t need = 0;
        for (int p = 0; p < npairs; p++) {
            const int nl = last[p].N;
            need += frame_bytes(&cur[p]) + al((size_t)nl * 28) * 2 + al(64) + al((size_t)nl * 4) + al((size_t)nl) +
                    al((size_t)mps[p].n * 12) + al((size_t)mps[p].n * 32) + al((size_t)mps[p].n * 4) +
                    al((size_t)cur[p].N * 4) + al(4);
        }
        if (m->arena_reserve(need + (size_t)npairs * 4 + 4096)) return ORB_E_HIP;
    }
    if (dev && m->arena_reserve((size_t)npairs * 4 + 256)) return ORB_E_HIP;
    int* d_nm = nullptr;
    std::vector<int*> nm_dev(npairs, nullptr);
    for (int p = 0; p < npairs; p++) {
        SearchDev& P = probs[p];
        memset(&P, 0, sizeof(P));
        P.cur = frame_dev(m, &cur[p], dev, s, &err);
        const int nl = last[p].N;
        P.nq = nl;
        P.last.N = nl;
        if (dev) {
            P.last.keysUn = (const orbgpu::orb_kp_dev*)last[p].keysUn;
            P.last.Tcw = last[p].Tcw;
            P.lastKeys = (const orbgpu::orb_kp_dev*)last_keys[p];
            P.lastMP = last_mp[p];
            P.lastOutlier = last_outlier[p];
            P.mpPos = mps[p].pos;
            P.mpDesc = mps[p].desc;
            P.mpObs = mps[p].observations;
            P.curMP = cur_mp[p];
        } else {
            P.last.keysUn = (const orbgpu::orb_kp_dev*)up(m, last[p].keysUn, (size_t)nl, s, &err);
            P.last.Tcw = up(m, last[p].Tcw, 16, s, &err);
            P.lastKeys = (const orbgpu::orb_kp_dev*)up(m, last_keys[p], (size_t)nl, s, &err);
            P.lastMP = up(m, last_mp[p], (size_t)nl, s, &err);
            P.lastOutlier = up(m, last_outlier[p], (size_t)nl, s, &err);
            P.mpPos = up(m, mps[p].pos, (size_t)mps[p].n * 3, s, &err);
            P.mpDesc = up(m, mps[p].desc, (size_t)mps[p].n * 32, s, &err);
            P.mpObs = up(m, mps[p].observations, (size_t)mps[p].n, s, &err);
            P.curMP = (int*)m->arena_alloc((size_t)cur[p].N * 4 + 4);
            if (cur[p].N > 0 && hipMemcpyAsync(P.curMP, cur_mp[p], (size_t)cur[p].N * 4, hipMemcpyHostToDevice, s) != hipSuccess)
                err = ORB_E_HIP;
        }
        nm_dev[p] = nullptr;
    }
    if (err) return err;
    // nmatches: small device array
    {
        void* d = dev ? m->count_buf((size_t)npairs * 4 + 4) : m->arena_alloc((size_t)npairs * 4 + 4);
        if (!d) return ORB_E_HIP;
        d_nm = (int*)d;
        for (int p = 0; p < npairs; p++) probs[p].nmatches = d_nm + p;
    }
    int rc = m->search_last(probs, th, bMono != 0);
    if (rc) return rc == -1 ? ORB_E_INVALID : ORB_E_HIP;
    if (dev) {   // device mode may be deferred (ORBmatcher_set_deferred)
        if (m->d2h_counts(nmatches, d_nm, (size_t)npairs * 4)) return ORB_E_HIP;
        return m->end_call() ? ORB_E_HIP : ORB_OK;
    }
    if (hipMemcpyAsync(nmatches, d_nm, (size_t)npairs * 4, hipMemcpyDeviceToHost, s) != hipSuccess) return ORB_E_HIP;
    {
        for (int p = 0; p < npairs; p++)
            if (cur[p].N > 0 &&
                hipMemcpyAsync(cur_mp[p], probs[p].curMP, (size_t)cur[p].N * 4, hipMemcpyDeviceToHost, s) != hipSuccess)
                return ORB_E_HIP;
    }
    if (orbgpu::stream_wait(s) != hipSuccess) return ORB_E_HIP;
    return ORB_OK;
}

int ORBmatcher_SearchByProjection_LastFrame(ORBmatcher_h h, const orb_frame* cur, int32_t* cur_mp,
                                            const orb_frame* last, const orb_kp* last_keys, const int32_t* last_mp,
                                            const uint8_t* last_outlier, const orb_mappoints* mps, float th, int bMono,
                                            int* nmatches) {
    return ORBmatcher_SearchByProjection_LastFrame_batch(h, 1, cur, &cur_mp, last, &last_keys, &last_mp, &last_outlier,
                                                         mps, th, bMono, nmatches);
}

int ORBmatcher_SearchByProjection_MapPoints(ORBmatcher_h h, const orb_frame* F, int32_t* cur_mp, int n,
                                            const uint8_t* track_in_view, const float* proj_x, const float* proj_xr,
                                            const float* proj_y, const int32_t* level, const float* view_cos,
                                            const int32_t* mp_index, const orb_mappoints* mps, float th,
                                            int* nmatches) {
    if (!h || !frame_ok(F) || !cur_mp || n < 0 || !mps || !nmatches) return ORB_E_INVALID;
    if (n > 0 && (!track_in_view || !proj_x || !proj_xr || !proj_y || !level || !view_cos || !mp_index))
        return ORB_E_INVALID;
    Matcher* m = h->m;
    const bool dev = m->device_pointers();
    hipStream_t s = m->stream();
    if (!dev) {
        for (int j = 0; j < n; j++)
            if (track_in_view[j] && (mp_index[j] < 0 || mp_index[j] >= mps->n || level[j] < 0 || level[j] >= F->nlevels))
                return ORB_E_INVALID;
        for (int i = 0; i < F->N; i++)
            if (cur_mp[i] >= mps->n) return ORB_E_INVALID;
        size_t need = frame_bytes(F) + al((size_t)n) + 4 * al((size_t)n * 4) + al((size_t)n * 4) * 2 +
                      al((size_t)mps->n * 12) + al((size_t)mps->n * 32) + al((size_t)mps->n * 4) +
                      al((size_t)F->N * 4) + al(8);
        if (m->arena_reserve(need + 4096)) return ORB_E_HIP;
    } else {
        if (m->arena_reserve(4096)) return ORB_E_HIP;
    }
    int err = 0;
    std::vector<SearchDev> probs(1);
    SearchDev& P = probs[0];
    memset(&P, 0, sizeof(P));
    P.cur = frame_dev(m, F, dev, s, &err);
    P.nq = n;
    if (dev) {
        P.inView = track_in_view; P.projX = proj_x; P.projXR = proj_xr; P.projY = proj_y;
        P.level = level; P.viewCos = view_cos; P.mpIndex = mp_index;
        P.mpPos = mps->pos; P.mpDesc = mps->desc; P.mpObs = mps->observations;
        P.curMP = cur_mp;
    } else {
        P.inView = up(m, track_in_view, (size_t)n, s, &err);
        P.projX = up(m, proj_x, (size_t)n, s, &err);
        P.projXR = up(m, proj_xr, (size_t)n, s, &err);
        P.projY = up(m, proj_y, (size_t)n, s, &err);
        P.level = up(m, level, (size_t)n, s, &err);
        P.viewCos = up(m, view_cos, (size_t)n, s, &err);
        P.mpIndex = up(m, mp_index, (size_t)n, s, &err);
        P.mpPos = up(m, mps->pos, (size_t)mps->n * 3, s, &err);
        P.mpDesc = up(m, mps->desc, (size_t)mps->n * 32, s, &err);
        P.mpObs = up(m, mps->observations, (size_t)mps->n, s, &err);
        P.curMP = (int*)m->arena_alloc((size_t)F->N * 4 + 4);
        if (F->N > 0 && hipMemcpyAsync(P.curMP, cur_mp, (size_t)F->N * 4, hipMemcpyHostToDevice, s) != hipSuccess)
            err = ORB_E_HIP;
    }
    if (err) return err;
    int* d_nm = (int*)m->arena_alloc(8);
    P.nmatches = d_nm;
    int rc = m->search_local(probs, th);
    if (rc) return rc == -1 ? ORB_E_INVALID : ORB_E_HIP;
    if (hipMemcpyAsync(nmatches, d_nm, 4, hipMemcpyDeviceToHost, s) != hipSuccess) return ORB_E_HIP;
    if (!dev && F->N > 0 && hipMemcpyAsync(cur_mp, P.curMP, (size_t)F->N * 4, hipMemcpyDeviceToHost, s) != hipSuccess)
        return ORB_E_HIP;
    if (orbgpu::stream_wait(s) != hipSuccess) return ORB_E_HIP;
    return ORB_OK;
}

int Frame_isInFrustum_batch(ORBmatcher_h h, int count, const orb_frame* F, const orb_localmap* maps,
                            float viewingCosLimit, float logScaleFactor, uint8_t* const* in_view,
                            float* const* proj_x, float* const* proj_xr, float* const* proj_y, int32_t* const* level,
                            float* const* view_cos, int* nvisible) {
    if (!h || count < 0 || (count > 0 && (!F || !maps || !in_view || !proj_x || !proj_xr || !proj_y || !level ||
                                          !view_cos || !nvisible)))
        return ORB_E_INVALID;
    if (count == 0) return ORB_OK;
    Matcher* m = h->m;
    if (!m->device_pointers()) return ORB_E_INVALID;
    hipStream_t s = m->stream();
    size_t need = al((size_t)count * 4) + al(sizeof(orbgpu::FrustumDev) * count) + 4096;
    for (int p = 0; p < count; p++) {
        const orb_localmap& M = maps[p];
        if (!frame_ok(&F[p]) || !F[p].Tcw || M.n < 0) return ORB_E_INVALID;
        if (M.n > 0 && (!M.pos || !M.max_dist || !M.min_dist || !M.normal || !M.skip || !in_view[p] || !proj_x[p] ||
                        !proj_xr[p] || !proj_y[p] || !level[p] || !view_cos[p]))
            return ORB_E_INVALID;
        need += al((size_t)M.n * 4);
    }
    if (m->arena_reserve(need)) return ORB_E_HIP;
    int err = 0;
    int* d_nv = (int*)m->arena_alloc((size_t)count * 4);
    if (!d_nv || hipMemsetAsync(d_nv, 0, (size_t)count * 4, s) != hipSuccess) return ORB_E_HIP;
    std::vector<SearchDev> probs(count);
    std::vector<orbgpu::FrustumDev> fr(count);
    for (int p = 0; p < count; p++) {
        SearchDev& P = probs[p];
        memset(&P, 0, sizeof(P));
        P.cur = frame_dev(m, &F[p], true, s, &err);
        P.nq = maps[p].n;
        P.mpPos = maps[p].pos;
        orbgpu::FrustumDev& f = fr[p];
        f.maxDist = maps[p].max_dist;
        f.minDist = maps[p].min_dist;
        f.normal = maps[p].normal;
        f.skip = maps[p].skip;
        f.inView = in_view[p];
        f.projX = proj_x[p];
        f.projXR = proj_xr[p];
        f.projY = proj_y[p];
        f.level = level[p];
        f.viewCos = view_cos[p];
        f.mpIndex = (int*)m->arena_alloc((size_t)std::max(maps[p].n, 1) * 4);
        f.nvisible = d_nv + p;
        if (!f.mpIndex) return ORB_E_HIP;
    }
    if (err) return err;
    if (m->frustum(probs, fr, viewingCosLimit, logScaleFactor)) return ORB_E_HIP;
    if (hipMemcpyAsync(nvisible, d_nv, (size_t)count * 4, hipMemcpyDeviceToHost, s) != hipSuccess) return ORB_E_HIP;
    return orbgpu::stream_wait(s) == hipSuccess ? ORB_OK : ORB_E_HIP;
}

int ORBmatcher_SearchLocalPoints_batch(ORBmatcher_h h, int count, const orb_frame* F, int32_t* const* cur_mp,
                                       const orb_localmap* maps, float logScaleFactor, float th, float nnratio,
                                       int* nmatches, int* nvisible) {
    if (!h || count < 0 || (count > 0 && (!F || !cur_mp || !maps || !nmatches || !nvisible))) return ORB_E_INVALID;
    if (count == 0) return ORB_OK;
    Matcher* m = h->m;
    if (!m->device_pointers()) return ORB_E_INVALID;   // device-resident tracking path only
    hipStream_t s = m->stream();
    size_t need = al((size_t)count * 8) + al(sizeof(orbgpu::FrustumDev) * count) + 4096;
    for (int p = 0; p < count; p++) {
        const orb_localmap& M = maps[p];
        if (!frame_ok(&F[p]) || !F[p].Tcw || M.n < 0 || !cur_mp[p]) return ORB_E_INVALID;
        if (M.n > 0 && (!M.pos || !M.desc || !M.observations || !M.max_dist || !M.min_dist || !M.normal || !M.skip))
            return ORB_E_INVALID;
        need += 7 * al((size_t)M.n * 4) + 256;
    }
    if (m->arena_reserve(need)) return ORB_E_HIP;
    int err = 0;
    int* d_cnt = (int*)m->count_buf((size_t)count * 8);
    if (!d_cnt) return ORB_E_HIP;
    if (hipMemsetAsync(d_cnt, 0, (size_t)count * 8, s) != hipSuccess) return ORB_E_HIP;
    std::vector<SearchDev> probs(count);
    std::vector<orbgpu::FrustumDev> fr(count);
    for (int p = 0; p < count; p++) {
        SearchDev& P = probs[p];
        memset(&P, 0, sizeof(P));
        P.cur = frame_dev(m, &F[p], true, s, &err);
        P.nq = maps[p].n;
        P.mpPos = maps[p].pos;
        P.mpDesc = maps[p].desc;
        P.mpObs = maps[p].observations;
        P.curMP = cur_mp[p];
        P.nmatches = d_cnt + p;
        orbgpu::FrustumDev& f = fr[p];
        memset(&f, 0, sizeof(f));
        f.maxDist = maps[p].max_dist;
        f.minDist = maps[p].min_dist;
        f.normal = maps[p].normal;
        f.skip = maps[p].skip;
        f.nvisible = d_cnt + count + p;
    }
    if (err) return err;
    const int rc = m->search_local_points(probs, fr, 0.5f, logScaleFactor, th, nnratio > 0.f ? nnratio : m->nnratio());
    if (rc) return rc == -1 ? ORB_E_INVALID : ORB_E_HIP;
    if (m->d2h_counts(nmatches, d_cnt, (size_t)count * 4) || m->d2h_counts(nvisible, d_cnt + count, (size_t)count * 4))
        return ORB_E_HIP;
    (void)s;
    return m->end_call() ? ORB_E_HIP : ORB_OK;
}

int ORBmatcher_SearchDense_batch(ORBmatcher_h h, int count, const uint8_t* const* qdesc, const int* nq,
                                 const uint8_t* const* tdesc, const int* nt, int32_t* const* best_idx,
                                 int32_t* const* best_dist, int32_t* const* second_dist) {
    if (!h || count < 0 || (count > 0 && (!qdesc || !nq || !tdesc || !nt || !best_idx || !best_dist || !second_dist)))
        return ORB_E_INVALID;
    for (int p = 0; p < count; p++) {
        if (nq[p] < 0 || nt[p] < 0) return ORB_E_INVALID;
        if (nq[p] > 0 && (!qdesc[p] || !best_idx[p] || !best_dist[p] || !second_dist[p])) return ORB_E_INVALID;
        if (nt[p] > 0 && !tdesc[p]) return ORB_E_INVALID;
    }
    if (count == 0) return ORB_OK;
    Matcher* m = h->m;
    const bool dev = m->device_pointers();
    hipStream_t s = m->stream();
    std::vector<orbgpu::DenseDev> probs;
    if (!dev) {
        size_t need = 4096;
        for (int p = 0; p < count; p++) need += al((size_t)nq[p] * 32) + al((size_t)nt[p] * 32) + 3 * al((size_t)nq[p] * 4);
        if (m->arena_reserve(need)) return ORB_E_HIP;
    }
    int err = 0;
    for (int p = 0; p < count; p++) {
        if (nq[p] == 0) continue;
        orbgpu::DenseDev d;
        d.nq = nq[p];
        d.nt = nt[p];
        if (dev) {
            d.q = qdesc[p];
            d.t = tdesc[p];
            d.best_idx = best_idx[p];
            d.best_dist = best_dist[p];
            d.second_dist = second_dist[p];
        } else {
            d.q = up(m, qdesc[p], (size_t)nq[p] * 32, s, &err);
            d.t = nt[p] ? up(m, tdesc[p], (size_t)nt[p] * 32, s, &err) : nullptr;
            d.best_idx = (int*)m->arena_alloc((size_t)nq[p] * 4);
            d.best_dist = (int*)m->arena_alloc((size_t)nq[p] * 4);
            d.second_dist = (int*)m->arena_alloc((size_t)nq[p] * 4);
            if (!d.best_idx || !d.best_dist || !d.second_dist) err = ORB_E_HIP;
        }
        probs.push_back(d);
    }
    if (err) return err;
    if (m->dense(probs)) return ORB_E_HIP;
    if (dev) return m->end_call() ? ORB_E_HIP : ORB_OK;
    for (int p = 0, k = 0; p < count; p++) {
        if (nq[p] == 0) continue;
        const orbgpu::DenseDev& d = probs[k++];
        if (hipMemcpyAsync(best_idx[p], d.best_idx, (size_t)nq[p] * 4, hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipMemcpyAsync(best_dist[p], d.best_dist, (size_t)nq[p] * 4, hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipMemcpyAsync(second_dist[p], d.second_dist, (size_t)nq[p] * 4, hipMemcpyDeviceToHost, s) != hipSuccess)
            return ORB_E_HIP;
    }
    return orbgpu::stream_wait(s) == hipSuccess ? ORB_OK : ORB_E_HIP;
}

int ORBmatcher_last_dense_timing(ORBmatcher_h h, float* ms, long long* pairs) {
    if (!h || !ms || !pairs) return ORB_E_INVALID;
    return h->m->dense_timing(ms, pairs) ? ORB_E_HIP : ORB_OK;
}

int ORBmatcher_SearchCandidates(ORBmatcher_h h, const uint8_t* qdesc, int nq, const uint8_t* tdesc, int nt,
                                const int32_t* off, const int32_t* cand, int32_t* dist, int32_t* best_idx,
                                int32_t* best_dist, int32_t* second_dist) {
    if (!h || nq < 0 || nt < 0 || !off) return ORB_E_INVALID;
    if (nq == 0) return ORB_OK;
    if (!qdesc || !best_idx || !best_dist || !second_dist) return ORB_E_INVALID;
    Matcher* m = h->m;
    const bool dev = m->device_pointers();
    hipStream_t s = m->stream();
    if (dev) {
        int rc = m->candidates(qdesc, nq, tdesc, nt, off, cand, dist, best_idx, best_dist, second_dist);
        if (rc) return ORB_E_HIP;
        return orbgpu::stream_wait(s) == hipSuccess ? ORB_OK : ORB_E_HIP;
    }
    const int ncand = off[nq];
    if (off[0] != 0 || ncand < 0) return ORB_E_INVALID;
    for (int q = 0; q < nq; q++)
        if (off[q + 1] < off[q]) return ORB_E_INVALID;
    for (int k = 0; k < ncand; k++)
        if (cand[k] < 0 || cand[k] >= nt) return ORB_E_INVALID;
    size_t need = al((size_t)nq * 32) + al((size_t)nt * 32) + al((size_t)(nq + 1) * 4) + 2 * al((size_t)ncand * 4 + 4) +
                  3 * al((size_t)nq * 4);
    if (m->arena_reserve(need + 4096)) return ORB_E_HIP;
    int err = 0;
    const uint8_t* dq = up(m, qdesc, (size_t)nq * 32, s, &err);
    const uint8_t* dt = up(m, tdesc, (size_t)nt * 32, s, &err);
    const int* doff = up(m, off, (size_t)nq + 1, s, &err);
    const int* dc = up(m, cand, (size_t)ncand, s, &err);
    int* dd = (int*)m->arena_alloc((size_t)ncand * 4 + 4);
    int* dbi = (int*)m->arena_alloc((size_t)nq * 4);
    int* dbd = (int*)m->arena_alloc((size_t)nq * 4);
    int* dsd = (int*)m->arena_alloc((size_t)nq * 4);
    if (err || !dd || !dbi || !dbd || !dsd) return ORB_E_HIP;
    if (m->candidates(dq, nq, dt, nt, doff, dc, dd, dbi, dbd, dsd)) return ORB_E_HIP;
    if (dist && ncand > 0 && hipMemcpyAsync(dist, dd, (size_t)ncand * 4, hipMemcpyDeviceToHost, s) != hipSuccess)
        return ORB_E_HIP;
    if (hipMemcpyAsync(best_idx, dbi, (size_t)nq * 4, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipMemcpyAsync(best_dist, dbd, (size_t)nq * 4, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipMemcpyAsync(second_dist, dsd, (size_t)nq * 4, hipMemcpyDeviceToHost, s) != hipSuccess)
        return ORB_E_HIP;
    return orbgpu::stream_wait(s) == hipSuccess ? ORB_OK : ORB_E_HIP;
}

}  // extern "C"
