// capi_vocab.cpp -- extern "C" ORBvocabulary_* (include/orbslam_gpu.h): the ORBVocabulary
// (DBoW2::TemplatedVocabulary<FORB::TDescriptor, FORB>, reference include/ORBVocabulary.h) as used
// by Frame::ComputeBoW / KeyFrame::ComputeBoW (src/Frame.cc:395-402, src/KeyFrame.cc:59-67) and
// KeyFrameDatabase's scoring (src/KeyFrameDatabase.cc:133, 249).
#include <algorithm>
#include <cstring>
#include <new>
#include <vector>

#include "../../include/orbslam_gpu.h"
#include "vocab.hpp"

struct ORBvocabulary_t {
    orbgpu::Vocabulary* v = nullptr;
    hipStream_t s = nullptr;
    bool uploaded = false;
    void* arena = nullptr;
    size_t cap = 0;
};

namespace {

size_t al(size_t n) { return (n + 255) & ~(size_t)255; }

// device stream + tree on first use; ORB_E_NODEVICE without a gfx950 device
int ensure_device(ORBvocabulary_t* h) {
    if (!h->s) {
        int n = 0;
        if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return ORB_E_NODEVICE;
        if (hipStreamCreateWithFlags(&h->s, hipStreamNonBlocking) != hipSuccess) return ORB_E_HIP;
    }
    if (!h->uploaded) {
        if (h->v->upload()) return ORB_E_HIP;
        h->uploaded = true;
    }
    return ORB_OK;
}

int reserve(ORBvocabulary_t* h, size_t bytes) {
    if (bytes <= h->cap) return ORB_OK;
    if (h->arena) (void)hipFree(h->arena);
    h->arena = nullptr;
    h->cap = 0;
    if (hipMalloc(&h->arena, bytes) != hipSuccess) return ORB_E_HIP;
    h->cap = bytes;
    return ORB_OK;
}

size_t frame_bytes(int N) {
    const size_t n = (size_t)std::max(N, 1);
    return al(32 * n) + 3 * al(4 * n) + 2 * al(8 * n) + 2 * al(4 * n) + al(4 * (n + 1)) + al(8);
}

// carve one frame's device buffers from p
orbgpu::BowJob carve(char*& p, const uint8_t* d_desc_src, int N) {
    const size_t n = (size_t)std::max(N, 1);
    orbgpu::BowJob J;
    J.N = N;
    J.desc = (const uint8_t*)p;
    (void)d_desc_src;
    p += al(32 * n);
    J.feat_word = (uint32_t*)p; p += al(4 * n);
    J.feat_node = (uint32_t*)p; p += al(4 * n);
    J.bow_word = (uint32_t*)p; p += al(4 * n);
    J.feat_weight = (double*)p; p += al(8 * n);
    J.bow_value = (double*)p; p += al(8 * n);
    J.fv_node = (uint32_t*)p; p += al(4 * n);
    J.fv_feat = (int*)p; p += al(4 * n);
    J.fv_start = (int*)p; p += al(4 * (n + 1));
    J.counts = (int*)p; p += al(8);
    return J;
}

int run_frames(ORBvocabulary_t* h, int count, const uint8_t* const* desc, const int* N, int levelsup, bool assemble,
               std::vector<orbgpu::BowJob>& jobs) {
    size_t need = al(sizeof(orbgpu::BowJob) * (size_t)count);
    int maxN = 0;
    for (int f = 0; f < count; f++) {
        need += frame_bytes(N[f]);
        maxN = std::max(maxN, N[f]);
    }
    if (int e = reserve(h, need)) return e;
    char* p = (char*)h->arena;
    orbgpu::BowJob* d_jobs = (orbgpu::BowJob*)p;
    p += al(sizeof(orbgpu::BowJob) * (size_t)count);
    jobs.resize(count);
    for (int f = 0; f < count; f++) {
        jobs[f] = carve(p, desc[f], N[f]);
        if (N[f] > 0 &&
            hipMemcpyAsync((void*)jobs[f].desc, desc[f], 32 * (size_t)N[f], hipMemcpyHostToDevice, h->s) != hipSuccess)
            return ORB_E_HIP;
    }
    if (hipMemcpyAsync(d_jobs, jobs.data(), sizeof(orbgpu::BowJob) * (size_t)count, hipMemcpyHostToDevice, h->s) !=
        hipSuccess)
        return ORB_E_HIP;
    if (h->v->transform(d_jobs, count, maxN, levelsup, assemble, h->s)) return ORB_E_HIP;
    return ORB_OK;
}

}  // namespace

extern "C" {

int ORBvocabulary_create(ORBvocabulary_h* out) {
    if (!out) return ORB_E_INVALID;
    *out = nullptr;
    auto* h = new (std::nothrow) ORBvocabulary_t;
    if (!h) return ORB_E_INVALID;
    h->v = new (std::nothrow) orbgpu::Vocabulary;
    if (!h->v) {
        delete h;
        return ORB_E_INVALID;
    }
    *out = h;
    return ORB_OK;
}

int ORBvocabulary_destroy(ORBvocabulary_h h) {
    if (!h) return ORB_E_INVALID;
    if (h->s) (void)hipStreamSynchronize(h->s);
    if (h->arena) (void)hipFree(h->arena);
    if (h->s) (void)hipStreamDestroy(h->s);
    delete h->v;
    delete h;
    return ORB_OK;
}

int ORBvocabulary_loadFromTextFile(ORBvocabulary_h h, const char* path) {
    if (!h || !path) return ORB_E_INVALID;
    auto* v = new (std::nothrow) orbgpu::Vocabulary;
    if (!v) return ORB_E_INVALID;
    if (v->load_text(path)) {
        delete v;
        return ORB_E_INVALID;   // the reference returns false (and keeps whatever it had parsed)
    }
    if (h->s) (void)hipStreamSynchronize(h->s);
    delete h->v;
    h->v = v;
    h->uploaded = false;
    return ORB_OK;
}

int ORBvocabulary_info(ORBvocabulary_h h, int* k, int* L, int* scoring, int* weighting, int* n_nodes, int* n_words) {
    if (!h) return ORB_E_INVALID;
    if (k) *k = h->v->k();
    if (L) *L = h->v->L();
    if (scoring) *scoring = h->v->scoring();
    if (weighting) *weighting = h->v->weighting();
    if (n_nodes) *n_nodes = h->v->nnodes();
    if (n_words) *n_words = h->v->nwords();
    return ORB_OK;
}

int ORBvocabulary_transform_batch(ORBvocabulary_h h, int count, const uint8_t* const* desc, const int* N, int levelsup,
                                  orb_bow* out) {
    if (!h || count < 0 || (count > 0 && (!desc || !N || !out))) return ORB_E_INVALID;
    for (int f = 0; f < count; f++) {
        if (N[f] < 0 || (N[f] > 0 && !desc[f])) return ORB_E_INVALID;
        if (!out[f].word || !out[f].value || !out[f].fv_node || !out[f].fv_start || !out[f].fv_feat)
            return ORB_E_INVALID;
        if (N[f] > orbgpu::kVocMaxFeatures || out[f].cap < N[f]) return ORB_E_CAPACITY;
    }
    if (count == 0) return ORB_OK;
    if (h->v->empty()) {   // transform() clears both vectors and returns (TemplatedVocabulary.h:1134-1137)
        for (int f = 0; f < count; f++) {
            out[f].n_words = out[f].n_nodes = 0;
            out[f].fv_start[0] = 0;
        }
        return ORB_OK;
    }
    if (int e = ensure_device(h)) return e;
    std::vector<orbgpu::BowJob> jobs;
    if (int e = run_frames(h, count, desc, N, levelsup, true, jobs)) return e;
    std::vector<int> cnt(2 * (size_t)count);
    for (int f = 0; f < count; f++)
        if (hipMemcpyAsync(&cnt[2 * f], jobs[f].counts, 8, hipMemcpyDeviceToHost, h->s) != hipSuccess) return ORB_E_HIP;
    if (hipStreamSynchronize(h->s) != hipSuccess) return ORB_E_HIP;
    for (int f = 0; f < count; f++) {
        const int nb = cnt[2 * f], nf = cnt[2 * f + 1], m = N[f];
        out[f].n_words = nb;
        out[f].n_nodes = nf;
        if (nb > 0 && (hipMemcpyAsync(out[f].word, jobs[f].bow_word, 4 * (size_t)nb, hipMemcpyDeviceToHost, h->s) !=
                           hipSuccess ||
                       hipMemcpyAsync(out[f].value, jobs[f].bow_value, 8 * (size_t)nb, hipMemcpyDeviceToHost, h->s) !=
                           hipSuccess))
            return ORB_E_HIP;
        if (hipMemcpyAsync(out[f].fv_start, jobs[f].fv_start, 4 * ((size_t)nf + 1), hipMemcpyDeviceToHost, h->s) !=
            hipSuccess)
            return ORB_E_HIP;
        if (nf > 0 && (hipMemcpyAsync(out[f].fv_node, jobs[f].fv_node, 4 * (size_t)nf, hipMemcpyDeviceToHost, h->s) !=
                           hipSuccess ||
                       hipMemcpyAsync(out[f].fv_feat, jobs[f].fv_feat, 4 * (size_t)m, hipMemcpyDeviceToHost, h->s) !=
                           hipSuccess))
            return ORB_E_HIP;
    }
    return hipStreamSynchronize(h->s) == hipSuccess ? ORB_OK : ORB_E_HIP;
}

int ORBvocabulary_transform(ORBvocabulary_h h, const uint8_t* desc, int N, int levelsup, orb_bow* out) {
    return ORBvocabulary_transform_batch(h, 1, &desc, &N, levelsup, out);
}

int ORBvocabulary_transform_features(ORBvocabulary_h h, const uint8_t* desc, int N, int levelsup, uint32_t* word,
                                     double* weight, uint32_t* node) {
    if (!h || N < 0 || (N > 0 && (!desc || !word || !weight || !node))) return ORB_E_INVALID;
    if (N > orbgpu::kVocMaxFeatures) return ORB_E_CAPACITY;
    if (N == 0) return ORB_OK;
    if (h->v->empty()) return ORB_E_INVALID;   // no tree to descend
    if (int e = ensure_device(h)) return e;
    std::vector<orbgpu::BowJob> jobs;
    if (int e = run_frames(h, 1, &desc, &N, levelsup, false, jobs)) return e;
    if (hipMemcpyAsync(word, jobs[0].feat_word, 4 * (size_t)N, hipMemcpyDeviceToHost, h->s) != hipSuccess ||
        hipMemcpyAsync(weight, jobs[0].feat_weight, 8 * (size_t)N, hipMemcpyDeviceToHost, h->s) != hipSuccess ||
        hipMemcpyAsync(node, jobs[0].feat_node, 4 * (size_t)N, hipMemcpyDeviceToHost, h->s) != hipSuccess)
        return ORB_E_HIP;
    return hipStreamSynchronize(h->s) == hipSuccess ? ORB_OK : ORB_E_HIP;
}

int ORBvocabulary_score(ORBvocabulary_h h, const uint32_t* qw, const double* qv, int nq, int count,
                        const int32_t* cstart, const uint32_t* cw, const double* cv, double* scores) {
    if (!h || nq < 0 || count < 0 || (nq > 0 && (!qw || !qv)) || (count > 0 && (!cstart || !scores)))
        return ORB_E_INVALID;
    if (count == 0) return ORB_OK;
    const int tot = cstart[count] - cstart[0];
    if (cstart[0] != 0 || tot < 0 || (tot > 0 && (!cw || !cv))) return ORB_E_INVALID;
    for (int c = 0; c < count; c++)
        if (cstart[c + 1] < cstart[c]) return ORB_E_INVALID;
    if (h->v->scoring() != 0) return ORB_E_INVALID;   // L1Scoring only (ORBvoc.txt: L1_NORM)
    if (int e = ensure_device(h)) return e;
    const size_t nqs = (size_t)std::max(nq, 1), ts = (size_t)std::max(tot, 1);
    const size_t need = al(4 * nqs) + al(8 * nqs) + al(4 * ((size_t)count + 1)) + al(4 * ts) + al(8 * ts) +
                        al(8 * (size_t)count);
    if (int e = reserve(h, need)) return e;
    char* p = (char*)h->arena;
    uint32_t* d_qw = (uint32_t*)p; p += al(4 * nqs);
    double* d_qv = (double*)p; p += al(8 * nqs);
    int* d_cs = (int*)p; p += al(4 * ((size_t)count + 1));
    uint32_t* d_cw = (uint32_t*)p; p += al(4 * ts);
    double* d_cv = (double*)p; p += al(8 * ts);
    double* d_out = (double*)p;
    auto H2D = [&](void* d, const void* s, size_t b) {
        return b == 0 || hipMemcpyAsync(d, s, b, hipMemcpyHostToDevice, h->s) == hipSuccess;
    };
    if (!H2D(d_qw, qw, 4 * (size_t)nq) || !H2D(d_qv, qv, 8 * (size_t)nq) ||
        !H2D(d_cs, cstart, 4 * ((size_t)count + 1)) || !H2D(d_cw, cw, 4 * (size_t)tot) ||
        !H2D(d_cv, cv, 8 * (size_t)tot))
        return ORB_E_HIP;
    if (h->v->score_l1(d_qw, d_qv, nq, d_cs, d_cw, d_cv, count, d_out, h->s)) return ORB_E_HIP;
    if (hipMemcpyAsync(scores, d_out, 8 * (size_t)count, hipMemcpyDeviceToHost, h->s) != hipSuccess) return ORB_E_HIP;
    return hipStreamSynchronize(h->s) == hipSuccess ? ORB_OK : ORB_E_HIP;
}

}  // extern "C"
