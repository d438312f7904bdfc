// orb_match.hpp -- gfx950 guided Hamming matching (see orb_match.hip).
#pragma once
#include <cstdint>
#include <vector>

#include "orb_common.hpp"
#include "orb_extract.hpp"

namespace orbgpu {

constexpr int kGridCols = 64;   // FRAME_GRID_COLS, Frame.h:37
constexpr int kGridRows = 48;   // FRAME_GRID_ROWS, Frame.h:38
constexpr int kGridCells = kGridCols * kGridRows;
constexpr int kTopK = 8;        // candidates kept per query for the greedy replay
constexpr int kMaxFrameKeys = 4096;

struct FrameDev {
    int N;
    const orb_kp_dev* keysUn;
    const uint8_t* desc;
    const float* uRight;  // may be null
    float minX, maxX, minY, maxY, gridWInv, gridHInv;
    const float* scale;
    int nlevels;
    float fx, fy, cx, cy, bf, b;
    const float* Tcw;
};

// One SearchByProjection problem (one (cur, last) pair, or one (F, map points) set).
struct SearchDev {
    FrameDev cur;
    // LastFrame mode
    FrameDev last;
    const orb_kp_dev* lastKeys;
    const int* lastMP;
    const uint8_t* lastOutlier;
    // MapPoints mode (per query arrays)
    const uint8_t* inView;
    const float* projX;
    const float* projXR;
    const float* projY;
    const int* level;
    const float* viewCos;
    const int* mpIndex;
    int nq;
    // map point table
    const float* mpPos;
    const uint8_t* mpDesc;
    const int* mpObs;
    // in/out
    int* curMP;
    int* nmatches;
    // scratch (device)
    int* gridStart;   // kGridCells+1
    int* gridIdx;     // cur.N
    int2* topk;       // nq * kTopK  (x = dist, y = candidate index)
    int4* qinfo;      // nq: x = ncand (-1 skip), y = bits(u), z = bits(v), w = bits(radius/r)
    int2* hist;       // nq (bin, idx)
    // SearchLocalPoints: k_frustum lists the in-view queries (any order) so that k_candidates'
    // waves are dense in queries with a window; null otherwise
    int* visList;     // nq
    int* visCount;    // 1
};

// Frame::isInFrustum inputs / outputs of one SearchLocalPoints problem (Tracking.cc:1143-1193):
// the local map points are the problem's map point table (SearchDev mpPos / mpDesc / mpObs)
struct FrustumDev {
    const float* maxDist;   // MapPoint::mfMaxDistance
    const float* minDist;   // mfMinDistance
    const float* normal;    // GetNormal() (3 per point)
    const uint8_t* skip;    // mnLastFrameSeen == CurrentFrame.mnId or isBad()
    uint8_t* inView;        // outputs: mbTrackInView, mTrackProjX / XR / Y, mnTrackScaleLevel,
    float* projX;           //          mTrackViewCos
    float* projXR;
    float* projY;
    int* level;
    float* viewCos;
    int* mpIndex;
    int* nvisible;          // IncreaseVisible() count (nToMatch)
};

// One brute-force matching problem (ORBmatcher_SearchDense_batch): device descriptor arrays,
// per-query outputs
struct DenseDev {
    const uint8_t* q;
    const uint8_t* t;
    int nq, nt;
    int* best_idx;
    int* best_dist;
    int* second_dist;
};

// one GetFeaturesInArea query of the area-candidate engine; qd = query descriptor row (-1 = none)
struct AreaQuery {
    float x, y, r;
    int minLevel, maxLevel;
    int qd;
};

constexpr int kCountSlots = 64;   // measurement counters: kCountSlots addresses per counter

class Matcher {
public:
    Matcher(float nnratio, bool checkOri) : nnratio_(nnratio), checkOri_(checkOri) {}
    ~Matcher();
    int init_device();
    void set_device_pointers(bool on) { device_ptrs_ = on; }
    bool device_pointers() const { return device_ptrs_; }
    // Runs `n` SearchByProjection(Cur, Last) problems in one set of launches.
    int search_last(std::vector<SearchDev>& probs, float th, bool bMono);
    int search_local(std::vector<SearchDev>& probs, float th);
    // Tracking::SearchLocalPoints: isInFrustum(pMP, viewingCosLimit) on the device for every
    // local map point of each problem, then SearchByProjection(F, vpLocalMapPoints, th) with
    // ratio `nnratio` (the reference's SearchLocalPoints builds its own ORBmatcher(0.8))
    int search_local_points(std::vector<SearchDev>& probs, std::vector<FrustumDev>& fr, float viewingCosLimit,
                            float logScaleFactor, float th, float nnratio);
    // Frame::isInFrustum only (outputs in fr's device arrays; arena-allocated problem copy)
    int frustum(std::vector<SearchDev>& probs, const std::vector<FrustumDev>& fr, float viewingCosLimit,
                float logScaleFactor);
    int candidates(const uint8_t* q, int nq, const uint8_t* t, int nt, const int* off, const int* cand, int* dist,
                   int* best_idx, int* best_dist, int* second_dist);
    // brute force: every query of each problem against every train row (LDS-resident blocks)
    int dense(const std::vector<DenseDev>& probs);
    int dense_timing(float* ms, long long* pairs);
    hipStream_t stream() const { return stream_; }
    // deferred mode (ORBmatcher_set_deferred): batch device calls return without a stream sync
    DeferredChain& chain() { return chain_; }
    // H2D source: the caller's host bytes, or a pinned copy of them in deferred mode
    const void* h2d_src(const void* host, size_t bytes) { return chain_.on() ? chain_.stage(host, bytes) : host; }
    // Device memory for a call's counts: the arena, or in deferred mode the chain's count
    // blocks (they outlive the call: the copy happens when the chain closes)
    void* count_buf(size_t bytes) { return chain_.on() ? chain_.dev_counts(bytes) : arena_alloc(bytes); }
    // D2H of device counts (from count_buf) into `user`: now, or in deferred mode at the
    // chain's close (one copy for the epoch, landing at finish())
    int d2h_counts(void* user, const void* dev, size_t bytes) {
        if (chain_.on()) {
            chain_.land_dev(user, dev, bytes);
            return 0;
        }
        ORB_HIP_CHECK(hipMemcpyAsync(user, dev, bytes, hipMemcpyDeviceToHost, stream_));
        return 0;
    }
    // end of a call: sync unless deferred
    int end_call() {
        if (chain_.on()) return 0;
        ORB_HIP_CHECK(hipStreamSynchronize(stream_));
        return 0;
    }
    float nnratio() const { return nnratio_; }
    bool check_ori() const { return checkOri_; }

    // Every GetFeaturesInArea candidate (idx, Hamming distance) of each query over `frame`
    // (its cur frame: device keysUn/desc + grid geometry), CSR in reference order, to host.
    int area_candidates(const SearchDev& frame, const AreaQuery* d_q, int nq, const uint8_t* d_qdesc,
                        std::vector<int>& off, std::vector<int2>& cand);
    // device arena for host-pointer mode: reserve() resets it, alloc() carves it
    int arena_reserve(size_t bytes);
    void* arena_alloc(size_t bytes);

    // Measurement (bench roofline): with timing on, the search / stereo / CSR launches record
    // HIP events on stream() around each kernel and count their work units on the device.
    //   ms[0..7]:  k_build_grid, k_candidates, k_select, k_stereo_rows, k_stereo_match,
    //              k_stereo_filter, k_csr_hamming, k_frustum
    //   cnt[0..7]: search (query, candidate) pairs scored, search queries with a window,
    //              stereo (left, right) pairs scored, stereo left keypoints, CSR pairs, CSR queries
    int set_timing(bool on);
    bool timing() const { return timing_; }
    int timings(float* ms8, long long* cnt8);
    void mark(int i);   // record event i on stream() (timing on)
    unsigned long long* counters() const { return timing_ ? d_count_ : nullptr; }
    int zero_counters(int first, int n);

private:
    int run(std::vector<SearchDev>& probs, float th, bool bMono, bool lastMode, float nnratio);
    float nnratio_;
    bool checkOri_;
    bool device_ptrs_ = false;
    hipStream_t stream_ = nullptr;
    DeferredChain chain_;
    void* d_scratch_ = nullptr;
    size_t scratch_cap_ = 0;
    void* d_probs_ = nullptr;
    size_t probs_cap_ = 0;
    void* d_arena_ = nullptr;
    size_t arena_cap_ = 0, arena_used_ = 0;
    void* d_cand_ = nullptr;
    size_t cand_cap_ = 0;
    void* d_dense_ = nullptr;
    size_t dense_cap_ = 0;
    bool timing_ = false;
    const FrustumDev* frustum_ = nullptr;   // pending k_frustum of search_local_points
    float frustumCos_ = 0.5f, frustumLsf_ = 0.f;
    hipEvent_t ev_[16] = {};
    bool evSet_[16] = {};
    unsigned long long* d_count_ = nullptr;
};

int debug_prof_match(unsigned long long* out32);   // section timers of k_select (prof builds)

}  // namespace orbgpu
