// vocab.hip -- gfx950 DBoW2 vocabulary: TemplatedVocabulary<FORB::TDescriptor, FORB>
// (reference Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h) behind Frame::ComputeBoW
// (src/Frame.cc:395-402) and KeyFrame::ComputeBoW (src/KeyFrame.cc:59-67).
//
//   host          loadFromTextFile (1338-1424) into a child-slot layout
//   k_voc_words   transform(feature, word, weight, nid, levelsup) (1217-1256): a group of
//                 G lanes per descriptor walks the tree; lane c scores child slots c, c+G, ...
//                 (8-dword popcount, the FORB::distance of FORB.cpp:83-101) and a group min
//                 over (dist, child position) keeps the reference's first strict minimum
//   k_voc_vectors transform(features, BowVector, FeatureVector, levelsup) (1126-1197): one
//                 workgroup per frame sorts (word, feature) and (node, feature) keys in LDS,
//                 sums the weights of each word in feature order (BowVector::addWeight),
//                 normalises with the scoring's norm (BowVector::normalize, BowVector.cpp:62-84;
//                 the norm is one sequential sum in ascending word order, as std::map iterates)
//                 and emits the FeatureVector as CSR (FeatureVector::addFeature order)
//   k_voc_score   L1Scoring::score (ScoringObject.cpp:21-66): one thread per (query, candidate)
//                 BowVector pair, the reference's merge order
//
// HBM layout: per node child-slot range (cbeg, ccnt); per slot the child id and its 32-byte
// descriptor, so the children of one node are one contiguous 32*k-byte read.
#include "vocab.hpp"

#include <algorithm>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>

namespace orbgpu {

// ------------------------------------------------------------------ host: loader
int Vocabulary::load_text(const char* path) {
    std::ifstream f(path);
    if (!f.is_open()) return -1;
    if (f.eof()) return -1;
    std::string s;
    std::getline(f, s);
    std::stringstream ss;
    ss << s;
    int k = -1, L = -1, n1 = -1, n2 = -1;
    ss >> k >> L >> n1 >> n2;
    if (k < 0 || k > 20 || L < 1 || L > 10 || n1 < 0 || n1 > 5 || n2 < 0 || n2 > 3) return -2;
    k_ = k; L_ = L; scoring_ = n1; weighting_ = n2;
    parent_.assign(1, 0);
    word_.assign(1, 0);
    children_.assign(1, {});
    desc_.assign(32, 0);
    weight_.assign(1, 0.0);
    nwords_ = 0;
    // node lines while(!f.eof()), the trailing empty line included.  A line whose parent
    // (or leaf flag) does not extract is the reference's undefined behaviour; realised as the
    // previous line's values (oracle/dbow2.c header).
    int prev_pid = 0, prev_leaf = 0;
    while (!f.eof()) {
        std::string snode;
        std::getline(f, snode);
        std::stringstream ssnode;
        ssnode << snode;
        int pid = prev_pid, isLeaf = prev_leaf;
        bool ok = static_cast<bool>(ssnode >> pid);
        if (ok) ok = static_cast<bool>(ssnode >> isLeaf);
        if (!ok) { pid = prev_pid; isLeaf = prev_leaf; }
        if (pid < 0 || pid >= (int)parent_.size()) return -3;
        const int nid = (int)parent_.size();
        parent_.push_back(pid);
        children_.push_back({});
        children_[pid].push_back(nid);
        desc_.resize(desc_.size() + 32, 0);
        double w = 0.0;
        if (ok) {
            for (int d = 0; d < 32; d++) {   // FORB::fromString: a byte that does not parse stays 0
                std::string e;
                if (!(ssnode >> e)) continue;
                char* end = nullptr;
                const long v = std::strtol(e.c_str(), &end, 10);
                if (end != e.c_str()) desc_[32 * (size_t)nid + d] = (uint8_t)v;
            }
            std::string ws;
            if (ssnode >> ws) w = std::strtod(ws.c_str(), nullptr);
        }
        weight_.push_back(w);
        word_.push_back(isLeaf > 0 ? nwords_++ : 0);
        prev_pid = pid;
        prev_leaf = isLeaf;
    }
    return 0;
}

Vocabulary::~Vocabulary() {
    if (d_mem_) (void)hipFree(d_mem_);
}

int Vocabulary::upload() {
    const int n = nnodes();
    std::vector<int> cbeg(n), ccnt(n), slot_node;
    std::vector<uint8_t> slot_desc;
    slot_node.reserve(n);
    slot_desc.reserve((size_t)32 * n);
    for (int p = 0; p < n; p++) {
        cbeg[p] = (int)slot_node.size();
        ccnt[p] = (int)children_[p].size();
        for (int c : children_[p]) {
            slot_node.push_back(c);
            slot_desc.insert(slot_desc.end(), desc_.begin() + 32 * (size_t)c, desc_.begin() + 32 * (size_t)c + 32);
        }
    }
    const size_t ns = std::max<size_t>(slot_node.size(), 1);
    auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
    const size_t b_cb = al(4 * (size_t)n), b_sn = al(4 * ns), b_sd = al(32 * ns), b_w = al(8 * (size_t)n);
    if (d_mem_) (void)hipFree(d_mem_);
    d_mem_ = nullptr;
    ORB_HIP_CHECK(hipMalloc(&d_mem_, 3 * b_cb + b_sn + b_sd + b_w));
    char* p = (char*)d_mem_;
    int* d_cbeg = (int*)p; p += b_cb;
    int* d_ccnt = (int*)p; p += b_cb;
    int* d_word = (int*)p; p += b_cb;
    int* d_sn = (int*)p; p += b_sn;
    uint4* d_sd = (uint4*)p; p += b_sd;
    double* d_w = (double*)p;
    ORB_HIP_CHECK(hipMemcpy(d_cbeg, cbeg.data(), 4 * (size_t)n, hipMemcpyHostToDevice));
    ORB_HIP_CHECK(hipMemcpy(d_ccnt, ccnt.data(), 4 * (size_t)n, hipMemcpyHostToDevice));
    ORB_HIP_CHECK(hipMemcpy(d_word, word_.data(), 4 * (size_t)n, hipMemcpyHostToDevice));
    if (!slot_node.empty()) {
        ORB_HIP_CHECK(hipMemcpy(d_sn, slot_node.data(), 4 * slot_node.size(), hipMemcpyHostToDevice));
        ORB_HIP_CHECK(hipMemcpy(d_sd, slot_desc.data(), slot_desc.size(), hipMemcpyHostToDevice));
    }
    ORB_HIP_CHECK(hipMemcpy(d_w, weight_.data(), 8 * (size_t)n, hipMemcpyHostToDevice));
    dv_.cbeg = d_cbeg; dv_.ccnt = d_ccnt; dv_.word_id = d_word; dv_.slot_node = d_sn; dv_.slot_desc = d_sd;
    dv_.weight = d_w;
    dv_.L = L_; dv_.scoring = scoring_; dv_.weighting = weighting_; dv_.nwords = nwords_;
    maxc_ = 0;
    for (int c : ccnt) maxc_ = std::max(maxc_, c);
    return 0;
}

// ------------------------------------------------------------------ kernels
template <int G>
__global__ void __launch_bounds__(256) k_voc_words(VocDev V, const BowJob* __restrict__ jobs, int levelsup) {
    const BowJob J = jobs[blockIdx.y];
    const int g = threadIdx.x / G, l = threadIdx.x % G;
    const int f = blockIdx.x * (256 / G) + g;
    if (f >= J.N) return;   // f is uniform in a group: groups leave whole
    const uint32_t* q32 = reinterpret_cast<const uint32_t*>(J.desc + 32 * (size_t)f);
    uint32_t q[8];
#pragma unroll
    for (int k = 0; k < 8; k++) q[k] = q32[k];
    const int nid_level = V.L - levelsup;
    int node = 0, level = 0, nd = 0;
    bool set = nid_level <= 0;
    for (;;) {
        const int cnt = V.ccnt[node];
        if (cnt == 0) break;
        ++level;
        const int beg = V.cbeg[node];
        unsigned best = 0xffffffffu;
        for (int c = l; c < cnt; c += G) {
            const uint4 a = V.slot_desc[2 * (size_t)(beg + c)], b = V.slot_desc[2 * (size_t)(beg + c) + 1];
            const int d = __popc(q[0] ^ a.x) + __popc(q[1] ^ a.y) + __popc(q[2] ^ a.z) + __popc(q[3] ^ a.w) +
                          __popc(q[4] ^ b.x) + __popc(q[5] ^ b.y) + __popc(q[6] ^ b.z) + __popc(q[7] ^ b.w);
            best = min(best, ((unsigned)d << 16) | (unsigned)c);   // first strict minimum in child order
        }
#pragma unroll
        for (int o = G / 2; o >= 1; o >>= 1) best = min(best, (unsigned)__shfl_xor((int)best, o, 64));
        node = V.slot_node[beg + (int)(best & 0xffffu)];
        if (level == nid_level) {
            nd = node;
            set = true;
        }
    }
    if (!set) nd = node;   // a leaf above the nid level (the reference leaves nid unset)
    if (l == 0) {
        J.feat_word[f] = (uint32_t)V.word_id[node];
        J.feat_weight[f] = V.weight[node];
        J.feat_node[f] = (uint32_t)nd;
    }
}

constexpr int VV_T = 1024;

// exclusive scan of flag(i) over i < n (n <= 4 * VV_T); out[i] = rank of flagged i; returns total
template <class Flag>
__device__ __forceinline__ int vv_scan(int n, Flag flag, int* out, int* s_w) {
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    int f[4], loc = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int i = 4 * tid + k;
        f[k] = (i < n && flag(i)) ? 1 : 0;
        loc += f[k];
    }
    int incl = loc;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(incl, o, 64);
        if (lane >= o) incl += y;
    }
    if (lane == 63) s_w[wid] = incl;
    __syncthreads();
    int off = 0, tot = 0;
    for (int w = 0; w < VV_T / 64; w++) {
        const int v = s_w[w];
        if (w < wid) off += v;
        tot += v;
    }
    int r = off + incl - loc;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int i = 4 * tid + k;
        if (i < n && f[k]) out[i] = r++;
    }
    __syncthreads();
    return tot;
}

__device__ __forceinline__ void vv_sort(unsigned long long* key, int P) {
    for (int k = 2; k <= P; k <<= 1)
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = threadIdx.x; i < P; i += VV_T) {
                const int ix = i ^ j;
                if (ix > i) {
                    const unsigned long long a = key[i], b = key[ix];
                    if ((a > b) == ((i & k) == 0)) {
                        key[i] = b;
                        key[ix] = a;
                    }
                }
            }
            __syncthreads();
        }
}

__global__ void __launch_bounds__(VV_T) k_voc_vectors(VocDev V, const BowJob* __restrict__ jobs) {
    __shared__ unsigned long long s_key[kVocMaxFeatures];
    __shared__ double s_val[kVocMaxFeatures];
    __shared__ int s_pos[kVocMaxFeatures];
    __shared__ int s_w[VV_T / 64];
    __shared__ double s_norm;
    const BowJob J = jobs[blockIdx.x];
    const int N = J.N, tid = threadIdx.x;
    int P = 1;
    while (P < N) P <<= 1;
    const unsigned long long NONE = ~0ull;
    auto hi = [&](int i) { return (uint32_t)(s_key[i] >> 32); };
    auto lo = [&](int i) { return (int)(uint32_t)s_key[i]; };
    // ---- BowVector: (word, feature) for every feature with weight > 0 (not stopped)
    for (int i = tid; i < P; i += VV_T)
        s_key[i] = (i < N && J.feat_weight[i] > 0) ? (((unsigned long long)J.feat_word[i] << 32) | (unsigned)i) : NONE;
    __syncthreads();
    vv_sort(s_key, P);
    const int m = vv_scan(P, [&](int i) { return s_key[i] != NONE; }, s_pos, s_w);
    const int nb = vv_scan(m, [&](int i) { return i == 0 || hi(i) != hi(i - 1); }, s_pos, s_w);
    const bool tf = V.weighting == 0 || V.weighting == 1;   // TF_IDF, TF: addWeight; IDF, BINARY: addIfNotExist
    for (int i = tid; i < m; i += VV_T) {
        if (!(i == 0 || hi(i) != hi(i - 1))) continue;
        double s = J.feat_weight[lo(i)];
        if (tf)
            for (int j = i + 1; j < m && hi(j) == hi(i); j++) s += J.feat_weight[lo(j)];
        const int r = s_pos[i];
        s_val[r] = s;
        J.bow_word[r] = hi(i);
    }
    __syncthreads();
    const bool must = V.scoring != 5;   // every scoring but DOT_PRODUCT normalises (ScoringObject.h:73-89)
    if (tf && !must && nb > 0) {
        for (int r = tid; r < nb; r += VV_T) s_val[r] /= (double)nb;
        __syncthreads();
    }
    if (must) {
        if (tid == 0) {
            double norm = 0.0;
            if (V.scoring != 1) {
                for (int r = 0; r < nb; r++) norm += fabs(s_val[r]);
            } else {
                for (int r = 0; r < nb; r++) norm += s_val[r] * s_val[r];
                norm = sqrt(norm);
            }
            s_norm = norm;
        }
        __syncthreads();
        const double norm = s_norm;
        if (norm > 0.0)
            for (int r = tid; r < nb; r += VV_T) s_val[r] /= norm;
        __syncthreads();
    }
    for (int r = tid; r < nb; r += VV_T) J.bow_value[r] = s_val[r];
    __syncthreads();
    // ---- FeatureVector: (node, feature) of the same features
    for (int i = tid; i < P; i += VV_T)
        s_key[i] = (i < N && J.feat_weight[i] > 0) ? (((unsigned long long)J.feat_node[i] << 32) | (unsigned)i) : NONE;
    __syncthreads();
    vv_sort(s_key, P);
    const int nf = vv_scan(m, [&](int i) { return i == 0 || hi(i) != hi(i - 1); }, s_pos, s_w);
    for (int i = tid; i < m; i += VV_T) {
        J.fv_feat[i] = lo(i);
        if (i == 0 || hi(i) != hi(i - 1)) {
            J.fv_node[s_pos[i]] = hi(i);
            J.fv_start[s_pos[i]] = i;
        }
    }
    if (tid == 0) {
        J.fv_start[nf] = m;
        J.counts[0] = nb;
        J.counts[1] = nf;
    }
}

// L1Scoring::score: one thread per candidate, the reference's merge and summation order
__global__ void __launch_bounds__(256) k_voc_score(const uint32_t* __restrict__ qw, const double* __restrict__ qv,
                                                   int nq, const int* __restrict__ cstart,
                                                   const uint32_t* __restrict__ cw, const double* __restrict__ cv,
                                                   int count, double* __restrict__ out) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= count) return;
    const int b0 = cstart[c], n2 = cstart[c + 1] - b0;
    const uint32_t* w2 = cw + b0;
    const double* v2 = cv + b0;
    double score = 0;
    int a = 0, b = 0;
    while (a < nq && b < n2) {
        const uint32_t x = qw[a], y = w2[b];
        if (x == y) {
            const double vi = qv[a], wi = v2[b];
            score += fabs(vi - wi) - fabs(vi) - fabs(wi);
            ++a;
            ++b;
        } else if (x < y) {
            ++a;   // v1.lower_bound(v2_it->first), one step at a time
        } else {
            ++b;
        }
    }
    out[c] = -score / 2.0;
}

// ------------------------------------------------------------------ host: launches
int Vocabulary::transform(const BowJob* d_jobs, int count, int maxN, int levelsup, bool assemble, hipStream_t s) {
    if (count <= 0) return 0;
    if (maxN > 0) {
        const int g = maxc_ <= 8 ? 8 : maxc_ <= 16 ? 16 : maxc_ <= 32 ? 32 : 64;
        const unsigned gx = (unsigned)((maxN + 256 / g - 1) / (256 / g));
        switch (g) {
            case 8: hipLaunchKernelGGL(k_voc_words<8>, dim3(gx, count), dim3(256), 0, s, dv_, d_jobs, levelsup); break;
            case 16: hipLaunchKernelGGL(k_voc_words<16>, dim3(gx, count), dim3(256), 0, s, dv_, d_jobs, levelsup); break;
            case 32: hipLaunchKernelGGL(k_voc_words<32>, dim3(gx, count), dim3(256), 0, s, dv_, d_jobs, levelsup); break;
            default: hipLaunchKernelGGL(k_voc_words<64>, dim3(gx, count), dim3(256), 0, s, dv_, d_jobs, levelsup); break;
        }
    }
    if (assemble) hipLaunchKernelGGL(k_voc_vectors, dim3(count), dim3(VV_T), 0, s, dv_, d_jobs);
    ORB_HIP_CHECK(hipGetLastError());
    return 0;
}

int Vocabulary::score_l1(const uint32_t* qw, const double* qv, int nq, const int* cstart, const uint32_t* cw,
                         const double* cv, int count, double* out, hipStream_t s) {
    if (count <= 0) return 0;
    hipLaunchKernelGGL(k_voc_score, dim3((count + 255) / 256), dim3(256), 0, s, qw, qv, nq, cstart, cw, cv, count, out);
    ORB_HIP_CHECK(hipGetLastError());
    return 0;
}

}  // namespace orbgpu
