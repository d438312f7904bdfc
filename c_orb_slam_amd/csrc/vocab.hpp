// vocab.hpp -- gfx950 DBoW2 vocabulary (ORBVocabulary = TemplatedVocabulary<FORB::TDescriptor, FORB>):
// the text loader on the host, the tree descent and the BowVector / FeatureVector assembly on
// the device (see vocab.hip).  Reference Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

#include "orb_common.hpp"

namespace orbgpu {

constexpr int kVocMaxFeatures = 4096;   // per frame (the assembly sorts in LDS)

// Device view of the tree: the children of node p are the slots [cbeg[p], cbeg[p] + ccnt[p])
// in insertion order; slot s holds the child's node id and its 32-byte descriptor.
struct VocDev {
    const int* cbeg;
    const int* ccnt;
    const int* slot_node;
    const uint4* slot_desc;   // 2 x uint4 per slot
    const int* word_id;       // per node
    const double* weight;     // per node
    int L, scoring, weighting, nwords;
};

// One frame of a transform batch (device pointers).
struct BowJob {
    const uint8_t* desc;      // N x 32
    int N;
    uint32_t* feat_word;      // scratch N: per-feature word id
    double* feat_weight;      // scratch N
    uint32_t* feat_node;      // scratch N
    uint32_t* bow_word;       // out: <= N
    double* bow_value;        // out
    uint32_t* fv_node;        // out: <= N
    int* fv_start;            // out: <= N + 1
    int* fv_feat;             // out: N
    int* counts;              // out: [n_words, n_nodes]
};

class Vocabulary {
public:
    ~Vocabulary();
    // TemplatedVocabulary::loadFromTextFile (1338-1424); 0 ok, -1 unreadable, -2 bad header, -3 bad parent
    int load_text(const char* path);
    int upload();   // copy the tree to the device (after load_text)
    bool empty() const { return nwords_ == 0; }
    int k() const { return k_; }
    int L() const { return L_; }
    int scoring() const { return scoring_; }
    int weighting() const { return weighting_; }
    int nnodes() const { return (int)parent_.size(); }
    int nwords() const { return nwords_; }
    // transform of `count` frames; jobs in device memory (d_jobs), maxN = max N over the jobs
    int transform(const BowJob* d_jobs, int count, int maxN, int levelsup, bool assemble, hipStream_t s);
    const VocDev& dev() const { return dv_; }
    // L1Scoring::score of query q against `count` candidates (device CSR inputs)
    int score_l1(const uint32_t* qw, const double* qv, int nq, const int* cstart, const uint32_t* cw,
                 const double* cv, int count, double* out, hipStream_t s);

private:
    int k_ = 0, L_ = 0, scoring_ = 0, weighting_ = 0, nwords_ = 0, maxc_ = 0;
    std::vector<int> parent_, word_;
    std::vector<std::vector<int>> children_;
    std::vector<uint8_t> desc_;   // 32 per node
    std::vector<double> weight_;
    void* d_mem_ = nullptr;
    VocDev dv_ = {};
};

}  // namespace orbgpu
