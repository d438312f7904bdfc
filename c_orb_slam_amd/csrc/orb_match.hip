// orb_match.hip -- gfx950 guided 256-bit Hamming matching (reference src/ORBmatcher.cc).
//
// The reference matchers are greedy: a query may not take a candidate that an
// earlier query already took (`if(F.mvpMapPoints[idx]) ... continue`,
// ORBmatcher.cc:87-89, 1403-1405).  So the work is split in two launches:
//   k_candidates  (one thread per query, all queries of all problems in
//                 parallel): projection, Frame::GetFeaturesInArea window over
//                 the device grid, static filters, popcount distances, and the
//                 kTopK smallest (dist, enumeration order) candidates;
//   k_select_r    (one workgroup per problem): the sequential greedy replay,
//                 solved as a parallel fixed-point iteration over the queries
//                 (occupancy owners in LDS), with a full rescan only when every
//                 kept candidate is already taken, then the rotation-consistency
//                 histogram (ORBmatcher.cc:1447-1467).
// k_build_grid rebuilds Frame::mGrid (AssignFeaturesToGrid, Frame.cc:230-245)
// as a CSR in cell order (ix-major) with keypoint order kept inside a cell.
#define ORBGPU_PROF_BLOCK 20   // prof builds: k_select_r sections of a mid-batch frame (full local map)
#include "orb_match.hpp"

#include <chrono>
#include <cstdlib>

#include <cstring>

#include "detmath.hpp"

namespace orbgpu {

constexpr int TH_HIGH = 100;  // ORBmatcher.cc:37
constexpr int kSelectLocalThreads = 1024;
constexpr int HISTO_LENGTH = 30;

__device__ __forceinline__ int hamming32(const uint8_t* a, const uint8_t* b) {
    const uint4* pa = reinterpret_cast<const uint4*>(a);
    const uint4* pb = reinterpret_cast<const uint4*>(b);
    const uint4 a0 = pa[0], a1 = pa[1], b0 = pb[0], b1 = pb[1];
    return __popc(a0.x ^ b0.x) + __popc(a0.y ^ b0.y) + __popc(a0.z ^ b0.z) + __popc(a0.w ^ b0.w) +
           __popc(a1.x ^ b1.x) + __popc(a1.y ^ b1.y) + __popc(a1.z ^ b1.z) + __popc(a1.w ^ b1.w);
}

// the query's descriptor held in registers across its candidates
struct Desc32 {
    uint4 a0, a1;
    __device__ __forceinline__ explicit Desc32(const uint8_t* a) {
        a0 = reinterpret_cast<const uint4*>(a)[0];
        a1 = reinterpret_cast<const uint4*>(a)[1];
    }
    __device__ __forceinline__ int dist(const uint8_t* b) const {
        const uint4* pb = reinterpret_cast<const uint4*>(b);
        const uint4 b0 = pb[0], b1 = pb[1];
        return __popc(a0.x ^ b0.x) + __popc(a0.y ^ b0.y) + __popc(a0.z ^ b0.z) + __popc(a0.w ^ b0.w) +
               __popc(a1.x ^ b1.x) + __popc(a1.y ^ b1.y) + __popc(a1.z ^ b1.z) + __popc(a1.w ^ b1.w);
    }
};

// Rcw*X + tcw as one cv::gemm (GEMMSingleMul<float,double>): f64 accumulate, one rounding.
__device__ __forceinline__ float gemm_row(const float* T, int r, float X0, float X1, float X2) {
    double s = (double)T[r * 4 + 0] * X0 + (double)T[r * 4 + 1] * X1 + (double)T[r * 4 + 2] * X2;
    return (float)(s + (double)T[r * 4 + 3]);
}

// ---------------------------------------------------------------- grid build

// Frame::AssignFeaturesToGrid (Frame.cc:230-245) as a counting sort: gridIdx lists every cell's
// keypoints in index order, cells in x-major order (cell = px * 48 + py), gridStart[c] its
// offset; keypoints outside the grid follow as 4095.  Everything stays in LDS until the final
// scattered store: per-cell counts, starts and cursors are packed 16-bit pairs (a cell holds at
// most N <= 4096 keypoints), the keypoints are scattered into their cell segments by LDS
// atomics (arbitrary order inside a segment), and each keypoint's final slot is its segment
// start plus the number of smaller indices in its segment (a stable order with no serial sort:
// O(sum of squared cell sizes / 256) LDS reads, a few per keypoint for ordinary frames, and still
// spread over the whole workgroup when every keypoint lands in one cell).
inline size_t grid_lds_bytes(int maxN) { return (((size_t)std::max(maxN, 1) * 4 + 4 + 15) & ~(size_t)15); }
inline size_t select_lds_bytes(int maxN) { return ((size_t)std::max(maxN, 1) * 11 + 15) & ~(size_t)15; }

__device__ __forceinline__ int packed16(const uint32_t* a, int c) { return (int)((a[c >> 1] >> (16 * (c & 1))) & 0xffffu); }

// dropOccupied (the greedy searches of run()): keypoints whose slot already holds a map point
// with Observations() > 0 when the call starts are left out of the cells.  The reference skips
// them as candidates (ORBmatcher.cc:87-89, 1403-1405), and a slot occupied at the start stays
// occupied (the loops only fill empty or observation-less slots), so no query of the call can
// take them; the remaining candidates keep their enumeration order.
__global__ void k_stream_signal(volatile int* w, int v) {
    if (threadIdx.x == 0) *w = v;
}

// The calling thread's pinned signal word, freed when the thread ends (thread pools that create and
// drop threads do not leak pinned pages).
struct SignalWord {
    volatile int* word = nullptr;
    int seq = 0;
    bool tried = false;
    ~SignalWord() {
        if (word) (void)hipHostFree((void*)word);
    }
};

// Drains stream s by spinning on a word a one-thread kernel writes behind the queued work: the
// calling thread spins one CPU core for up to 50 ms per call (then falls back to a blocking
// hipStreamSynchronize).  A blocking sync woke 20-40 us late.  Once the word is seen,
// hipStreamQuery reports an asynchronous failure of the drained work, as hipStreamSynchronize would.
hipError_t stream_wait(hipStream_t s) {
    thread_local SignalWord sw;
    static const bool blocking = [] {   // ORBGPU_SYNC_BLOCKING=1: plain hipStreamSynchronize (A/B)
        const char* e = std::getenv("ORBGPU_SYNC_BLOCKING");
        return e && e[0] == '1';
    }();
    if (blocking) return hipStreamSynchronize(s);
    if (!sw.word && !sw.tried) {
        sw.tried = true;
        void* p = nullptr;
        if (hipHostMalloc(&p, 64, hipHostMallocCoherent) == hipSuccess) {
            std::memset(p, 0, 64);
            sw.word = (volatile int*)p;
        }
    }
    if (!sw.word) return hipStreamSynchronize(s);
    const int v = ++sw.seq;
    hipLaunchKernelGGL(k_stream_signal, dim3(1), dim3(64), 0, s, sw.word, v);
    if (hipError_t e = hipGetLastError()) return e;
    const auto t0 = std::chrono::steady_clock::now();
    for (unsigned spin = 1; *sw.word != v; spin++) {
        if ((spin & 4095) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(50))
            return hipStreamSynchronize(s);
        __builtin_ia32_pause();
    }
    const hipError_t q = hipStreamQuery(s);   // the signal kernel has run: only a sticky error remains
    return q == hipErrorNotReady ? hipSuccess : q;
}

__global__ void __launch_bounds__(256) k_build_grid(SearchDev* probs, int dropOccupied) {
    ORBGPU_LATENCY_WAVE();
    constexpr int kPer = kGridCells / 256;   // 12 cells per thread in the scan
    static_assert(kGridCells % 512 == 0, "packed pairs per thread");
    __shared__ uint32_t s_cnt[kGridCells / 2];   // counts, then cursors
    __shared__ uint32_t s_beg[kGridCells / 2];   // segment starts
    __shared__ int s_wsum[4];
    extern __shared__ int s_dyn32[];
    int16_t* s_dyn = reinterpret_cast<int16_t*>(s_dyn32);
    SearchDev& P = probs[blockIdx.x];
    const FrameDev& F = P.cur;
    const int N = F.N, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    int16_t* s_cell = s_dyn;                       // N: cell of keypoint i or -1
    int16_t* s_idx = s_dyn + ((N + 1) & ~1);       // total: keypoints in cell order (unordered inside)
    for (int w = tid; w < kGridCells / 2; w += 256) s_cnt[w] = 0u;
    __syncthreads();
    for (int i = tid; i < N; i += 256) {
        const orb_kp_dev kp = F.keysUn[i];
        const int px = (int)roundf((kp.x - F.minX) * F.gridWInv);
        const int py = (int)roundf((kp.y - F.minY) * F.gridHInv);
        int cell = -1;
        bool occ = false;
        if (dropOccupied) {
            const int m = P.curMP[i];
            occ = m >= 0 && P.mpObs[m] > 0;
        }
        if (!(px < 0 || px >= kGridCols || py < 0 || py >= kGridRows) && !occ) {
            cell = px * kGridRows + py;
            atomicAdd(&s_cnt[cell >> 1], 1u << (16 * (cell & 1)));
        }
        s_cell[i] = (int16_t)cell;
    }
    __syncthreads();
    // exclusive scan of the counts: thread t owns cells [kPer t, kPer t + kPer)
    int cnt[kPer], tot = 0;
#pragma unroll
    for (int k = 0; k < kPer; k += 2) {
        const uint32_t w = s_cnt[(kPer * tid + k) >> 1];
        cnt[k] = (int)(w & 0xffffu);
        cnt[k + 1] = (int)(w >> 16);
        tot += cnt[k] + cnt[k + 1];
    }
    int incl = tot;
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(incl, o, 64);
        if (lane >= o) incl += y;
    }
    if (lane == 63) s_wsum[wid] = incl;
    __syncthreads();
    int run = incl - tot;
    for (int w = 0; w < wid; w++) run += s_wsum[w];
    const int total = s_wsum[0] + s_wsum[1] + s_wsum[2] + s_wsum[3];
#pragma unroll
    for (int k = 0; k < kPer; k += 2) {
        const int c = kPer * tid + k;
        P.gridStart[c] = run;
        P.gridStart[c + 1] = run + cnt[k];
        const uint32_t pr = (uint32_t)run | ((uint32_t)(run + cnt[k]) << 16);
        s_cnt[c >> 1] = pr;   // cursors
        s_beg[c >> 1] = pr;   // starts
        run += cnt[k] + cnt[k + 1];
    }
    if (tid == 255) P.gridStart[kGridCells] = total;
    __syncthreads();
    for (int i = tid; i < N; i += 256) {
        const int cell = s_cell[i];
        if (cell >= 0) {
            const int sh = 16 * (cell & 1);
            const int pos = (int)((atomicAdd(&s_cnt[cell >> 1], 1u << sh) >> sh) & 0xffffu);
            s_idx[pos] = (int16_t)i;
        }
    }
    for (int i = total + tid; i < N; i += 256) P.gridIdx[i] = 4095;
    __syncthreads();
    // stable slot of every placed keypoint: its segment start + the smaller indices in the segment
    for (int p = tid; p < total; p += 256) {
        const int i = s_idx[p], c = s_cell[i];
        const int b0 = packed16(s_beg, c), b1 = c + 1 < kGridCells ? packed16(s_beg, c + 1) : total;
        int r = 0;
        for (int q = b0; q < b1; q++) r += (int)s_idx[q] < i;
        P.gridIdx[b0 + r] = i;
    }
}

// ------------------------------------------------------- candidate enumeration
struct QueryWin {
    float x, y, r;
    int minLevel, maxLevel;
};

// Where a search reads the current frame's grid, keypoints and descriptors: HBM (GView), or
// the LDS copy a k_candidates workgroup stages once for its queries (LView).
struct GView {
    const SearchDev& P;
    __device__ __forceinline__ int start(int c) const { return P.gridStart[c]; }
    __device__ __forceinline__ int idx(int j) const { return P.gridIdx[j]; }
    __device__ __forceinline__ void kp(int i, float& x, float& y, int& oct) const {
        const orb_kp_dev k = P.cur.keysUn[i];
        x = k.x;
        y = k.y;
        oct = k.octave;
    }
    __device__ __forceinline__ int dist(const Desc32& d, int i) const { return d.dist(P.cur.desc + 32 * (size_t)i); }
};
struct LView {
    const uint16_t* gs;   // gridStart (kGridCells + 1)
    const uint16_t* gi;   // gridIdx (N)
    const float2* xy;     // keysUn x, y (N)
    const uint8_t* oct;   // keysUn octave (N)
    const uint4* desc;    // descriptors (2 per keypoint)
    __device__ __forceinline__ int start(int c) const { return gs[c]; }
    __device__ __forceinline__ int idx(int j) const { return gi[j]; }
    __device__ __forceinline__ void kp(int i, float& x, float& y, int& o) const {
        const float2 v = xy[i];
        x = v.x;
        y = v.y;
        o = oct[i];
    }
    __device__ __forceinline__ int dist(const Desc32& d, int i) const {
        const uint4 b0 = desc[2 * i], b1 = desc[2 * i + 1];
        return __popc(d.a0.x ^ b0.x) + __popc(d.a0.y ^ b0.y) + __popc(d.a0.z ^ b0.z) + __popc(d.a0.w ^ b0.w) +
               __popc(d.a1.x ^ b1.x) + __popc(d.a1.y ^ b1.y) + __popc(d.a1.z ^ b1.z) + __popc(d.a1.w ^ b1.w);
    }
};

// Frame::GetFeaturesInArea (Frame.cc:327-380) over the CSR grid, calling
// visit(idx) in the reference's enumeration order.
template <class View, class Visit>
__device__ __forceinline__ void for_features_in_area(const SearchDev& P, const View& V, const QueryWin& w, Visit visit) {
    const FrameDev& F = P.cur;
    const int nMinCellX = max(0, (int)floorf((w.x - F.minX - w.r) * F.gridWInv));
    if (nMinCellX >= kGridCols) return;
    const int nMaxCellX = min(kGridCols - 1, (int)ceilf((w.x - F.minX + w.r) * F.gridWInv));
    if (nMaxCellX < 0) return;
    const int nMinCellY = max(0, (int)floorf((w.y - F.minY - w.r) * F.gridHInv));
    if (nMinCellY >= kGridRows) return;
    const int nMaxCellY = min(kGridRows - 1, (int)ceilf((w.y - F.minY + w.r) * F.gridHInv));
    if (nMaxCellY < 0) return;
    const bool bCheckLevels = (w.minLevel > 0) || (w.maxLevel >= 0);
    for (int ix = nMinCellX; ix <= nMaxCellX; ix++)
        for (int iy = nMinCellY; iy <= nMaxCellY; iy++) {
            const int c = ix * kGridRows + iy;
            const int e = V.start(c + 1);
            for (int j = V.start(c); j < e; j++) {
                const int idx = V.idx(j);
                float kx, ky;
                int ko;
                V.kp(idx, kx, ky, ko);
                if (bCheckLevels) {
                    if (ko < w.minLevel) continue;
                    if (w.maxLevel >= 0 && ko > w.maxLevel) continue;
                }
                const float distx = kx - w.x, disty = ky - w.y;
                if (fabsf(distx) < w.r && fabsf(disty) < w.r) visit(idx);
            }
        }
}
template <class Visit>
__device__ __forceinline__ void for_features_in_area(const SearchDev& P, const QueryWin& w, Visit visit) {
    for_features_in_area(P, GView{P}, w, visit);
}

// The K best (dist, idx) of a query's candidates, sorted by dist, equal distances in visit
// order (later after earlier), held in registers: an unrolled compare-and-shift network with
// static slot indices (a dynamically indexed private array lives in scratch memory).  Empty
// slots hold dist INT_MAX, so a full list's cut-off test `dist >= t[K-1].x` covers both cases.
template <int K>
struct TopK {
    int2 t[K];
    __device__ __forceinline__ TopK() {
#pragma unroll
        for (int p = 0; p < K; p++) t[p] = make_int2(INT_MAX, -1);
    }
    __device__ __forceinline__ void insert(int dist, int idx) {
        if (dist >= t[K - 1].x) return;
#pragma unroll
        for (int p = K - 1; p > 0; p--) {
            const bool sh = t[p - 1].x > dist;   // slot p takes its predecessor
            const bool at = !sh && t[p].x > dist;   // the insertion point
            t[p] = sh ? t[p - 1] : at ? make_int2(dist, idx) : t[p];
        }
        if (t[0].x > dist) t[0] = make_int2(dist, idx);
    }
};

struct LastQuery {
    bool valid;
    QueryWin w;
    float u, invzc, radius;
    int mp;
};

// Projection part of SearchByProjection(Cur, Last), ORBmatcher.cc:1358-1395
__device__ __forceinline__ LastQuery last_query(const SearchDev& P, int i, float th, bool bFwd, bool bBwd) {
    LastQuery q;
    q.valid = false;
    const int mp = P.lastMP[i];
    if (mp < 0 || P.lastOutlier[i]) return q;
    const float* X = P.mpPos + 3 * (size_t)mp;
    const float* T = P.cur.Tcw;
    const float xc = gemm_row(T, 0, X[0], X[1], X[2]);
    const float yc = gemm_row(T, 1, X[0], X[1], X[2]);
    const float zc = gemm_row(T, 2, X[0], X[1], X[2]);
    const float invzc = (float)(1.0 / (double)zc);
    if (invzc < 0) return q;
    const float u = P.cur.fx * xc * invzc + P.cur.cx;
    const float v = P.cur.fy * yc * invzc + P.cur.cy;
    if (u < P.cur.minX || u > P.cur.maxX) return q;
    if (v < P.cur.minY || v > P.cur.maxY) return q;
    const int nLastOctave = P.lastKeys[i].octave;
    const float radius = th * P.cur.scale[nLastOctave];
    q.w.x = u;
    q.w.y = v;
    q.w.r = radius;
    if (bFwd) { q.w.minLevel = nLastOctave; q.w.maxLevel = -1; }
    else if (bBwd) { q.w.minLevel = 0; q.w.maxLevel = nLastOctave; }
    else { q.w.minLevel = nLastOctave - 1; q.w.maxLevel = nLastOctave + 1; }
    q.u = u;
    q.invzc = invzc;
    q.radius = radius;
    q.mp = mp;
    q.valid = true;
    return q;
}

__device__ __forceinline__ void fwd_bwd(const SearchDev& P, bool bMono, bool& bFwd, bool& bBwd) {
    const float* Tc = P.cur.Tcw;
    const float* Tl = P.last.Tcw;
    float twc[3];
    for (int i = 0; i < 3; i++) {
        double s = (double)Tc[0 * 4 + i] * Tc[3] + (double)Tc[1 * 4 + i] * Tc[7] + (double)Tc[2 * 4 + i] * Tc[11];
        twc[i] = (float)(s * -1.0);
    }
    const float tlc2 = gemm_row(Tl, 2, twc[0], twc[1], twc[2]);
    bFwd = tlc2 > P.cur.b && !bMono;
    bBwd = -tlc2 > P.cur.b && !bMono;
}

// Enumerate a LastFrame query's passing candidates; `blocked(i2)` models occupancy.
template <class Blocked, class Top, class View = GView>
__device__ int scan_last(const SearchDev& P, const LastQuery& q, Blocked blocked, Top& top, const View& V) {
    int cnt = 0;
    const Desc32 dMP(P.mpDesc + 32 * (size_t)q.mp);
    for_features_in_area(P, V, q.w, [&](int i2) {
        if (blocked(i2)) return;
        if (P.cur.uRight && P.cur.uRight[i2] > 0) {
            const float ur = q.u - P.cur.bf * q.invzc;
            const float er = fabsf(ur - P.cur.uRight[i2]);
            if (er > q.radius) return;
        }
        top.insert(V.dist(dMP, i2), i2);
        cnt++;
    });
    return cnt;
}
template <class Blocked, class Top>
__device__ int scan_last(const SearchDev& P, const LastQuery& q, Blocked blocked, Top& top) {
    return scan_last(P, q, blocked, top, GView{P});
}

struct LocalQuery {
    bool valid;
    QueryWin w;
    float r, projXR;
    int level, mp;
};

// SearchByProjection(F, vpMapPoints, th) window, ORBmatcher.cc:51-71
__device__ __forceinline__ LocalQuery local_query(const SearchDev& P, int j, float th) {
    LocalQuery q;
    q.valid = false;
    if (!P.inView[j]) return q;
    const int lvl = P.level[j];
    float r = P.viewCos[j] > 0.998f ? 2.5f : 4.0f;  // RadiusByViewingCos, 131-137
    if (th != 1.0f) r *= th;
    q.w.x = P.projX[j];
    q.w.y = P.projY[j];
    q.w.r = r * P.cur.scale[lvl];
    q.w.minLevel = lvl - 1;
    q.w.maxLevel = lvl;
    q.r = r;
    q.projXR = P.projXR[j];
    q.level = lvl;
    q.mp = P.mpIndex[j];
    q.valid = true;
    return q;
}

template <class Blocked, class Top, class View = GView>
__device__ int scan_local(const SearchDev& P, const LocalQuery& q, Blocked blocked, Top& top, const View& V) {
    int cnt = 0;
    const Desc32 d0(P.mpDesc + 32 * (size_t)q.mp);
    for_features_in_area(P, V, q.w, [&](int idx) {
        if (blocked(idx)) return;
        if (P.cur.uRight && P.cur.uRight[idx] > 0) {
            const float er = fabsf(q.projXR - P.cur.uRight[idx]);
            if (er > q.r * P.cur.scale[q.level]) return;
        }
        top.insert(V.dist(d0, idx), idx);
        cnt++;
    });
    return cnt;
}
template <class Blocked, class Top>
__device__ int scan_local(const SearchDev& P, const LocalQuery& q, Blocked blocked, Top& top) {
    return scan_local(P, q, blocked, top, GView{P});
}

// Parallel phase: one thread per query.  STAGE: each 1024-thread workgroup first copies the
// current frame's grid, keypoint positions / octaves and descriptors into LDS (every problem has
// N <= kStageMaxN), then walks its 1024 queries, so the window walks -- cell start -> keypoint
// index -> keypoint -> descriptor, a chain of dependent loads per candidate -- read LDS, and the
// frame is read from HBM once per 1024 queries.
constexpr int kStageMaxN = 1536;
constexpr int kStageThreads = 1024;
// ORBGPU_CAND_NT=256: the staged candidate search in 256-thread workgroups (each stages the
// frame itself; 4x the workgroups over more CUs) instead of 1024 (A/B runs)
// ORBGPU_SELECT_LOCAL_NT=512: SearchLocalPoints' selection in 512-thread workgroups (8 query
// slots per thread, the same 4,096 per problem) instead of 1,024 (A/B runs): a workgroup then
// needs 8 free wave slots on a CU, not 16, beside the extraction grids
static int select_local_threads() {
    static const int v = [] {
        const char* e = std::getenv("ORBGPU_SELECT_LOCAL_NT");
        return e && std::atoi(e) == 512 ? 512 : kSelectLocalThreads;
    }();
    return v;
}
// ORBGPU_CAND_LOCAL_STAGE=0: SearchLocalPoints' candidate search without the LDS-staged frame
// (no LDS, so its workgroups are not held back by the extraction grids' LDS use; A/B runs)
static bool cand_local_stage() {
    static const bool v = [] {
        const char* e = std::getenv("ORBGPU_CAND_LOCAL_STAGE");
        return !(e && std::atoi(e) == 0);
    }();
    return v;
}
static int stage_threads() {
    static const int v = [] {
        const char* e = std::getenv("ORBGPU_CAND_NT");
        return e && std::atoi(e) == 256 ? 256 : kStageThreads;
    }();
    return v;
}
constexpr size_t kStageLds = sizeof(uint16_t) * (kGridCells + 2) + sizeof(uint16_t) * kStageMaxN +
                             sizeof(float2) * kStageMaxN + kStageMaxN + 32 * (size_t)kStageMaxN + 64;
template <bool LAST, bool STAGE, int NT>
__global__ void __launch_bounds__(NT) k_candidates(const SearchDev* __restrict__ probs, int np, int gx, float th,
                                                   int bMono, unsigned long long* counters) {
    ORBGPU_LATENCY_WAVE();
    // XCD-aware order (xcd_problem_block): every block of a problem runs on one XCD and the
    // frame it stages is fetched into one L2
    int by, bx;
    if (!xcd_problem_block(np, gx, by, bx)) return;
    const SearchDev P = probs[by];
    int nvis = P.nq;
    if (!LAST && P.visList) nvis = *P.visCount;   // SearchLocalPoints: the t-th in-view query
    // a workgroup with no query of its own stages nothing (SearchLocalPoints' in-view count is
    // known on the device only: the grid covers every local map point)
    if (!counters && bx * NT >= nvis) return;
    const int tBegin = bx * NT + (int)threadIdx.x;
    const int tStride = gx * NT;
    LView V{};
    if constexpr (STAGE) {
        extern __shared__ __align__(16) unsigned char s_stage[];
        uint4* s_desc = reinterpret_cast<uint4*>(s_stage);                              // 32 N
        float2* s_xy = reinterpret_cast<float2*>(s_stage + 32 * (size_t)kStageMaxN);   // 8 N
        uint16_t* s_gs = reinterpret_cast<uint16_t*>(s_xy + kStageMaxN);               // cells + 1
        uint16_t* s_gi = s_gs + kGridCells + 2;                                         // N
        uint8_t* s_oct = reinterpret_cast<uint8_t*>(s_gi + kStageMaxN);                // N
        const int N = P.cur.N, tid = threadIdx.x;
        const uint4* gd = reinterpret_cast<const uint4*>(P.cur.desc);
        for (int k = tid; k < 2 * N; k += NT) s_desc[k] = gd[k];
        for (int k = tid; k < N; k += NT) {
            const orb_kp_dev kp = P.cur.keysUn[k];
            s_xy[k] = make_float2(kp.x, kp.y);
            s_oct[k] = (uint8_t)kp.octave;
            s_gi[k] = (uint16_t)P.gridIdx[k];
        }
        for (int c = tid; c <= kGridCells; c += NT) s_gs[c] = (uint16_t)P.gridStart[c];
        __syncthreads();
        V = LView{s_gs, s_gi, s_xy, s_oct, s_desc};
    }
    bool bF = false, bB = false;
    if (LAST) fwd_bwd(P, bMono != 0, bF, bB);
    unsigned long long pr = 0, nqv = 0;
    auto never = [](int) { return false; };
    for (int t = tBegin; t < nvis; t += tStride) {
        const int q = (!LAST && P.visList) ? P.visList[t] : t;
        if (q >= P.nq) continue;
        TopK<kTopK> top;
        int cnt = -1;
        if (LAST) {
            const LastQuery lq = last_query(P, q, th, bF, bB);
            if (lq.valid) cnt = STAGE ? scan_last(P, lq, never, top, V) : scan_last(P, lq, never, top);
        } else {
            const LocalQuery lq = local_query(P, q, th);
            if (lq.valid) cnt = STAGE ? scan_local(P, lq, never, top, V) : scan_local(P, lq, never, top);
        }
        P.qinfo[q] = make_int4(cnt, 0, 0, 0);
        const int kk = cnt < kTopK ? cnt : kTopK;
#pragma unroll
        for (int k = 0; k < kTopK; k++)
            if (k < kk) P.topk[(size_t)q * kTopK + k] = top.t[k];
        if (cnt > 0) pr += (unsigned long long)cnt;
        if (cnt >= 0) nqv++;
    }
    if (counters) {   // measurement: scored pairs and windowed queries
        pr = wave_sum_u64(pr);
        nqv = wave_sum_u64(nqv);
        if ((threadIdx.x & 63) == 0) {
            const int sl = (bx + by * 7 + (threadIdx.x >> 6)) & (kCountSlots - 1);
            atomicAdd(&counters[0 * kCountSlots + sl], pr);
            atomicAdd(&counters[1 * kCountSlots + sl], nqv);
        }
    }
}

// Frame::isInFrustum(pMP, viewingCosLimit) (Frame.cc:269-325), one thread per local map point.
// Float evaluation as the reference writes it: Pc = Rcw P + tcw and mOw = -Rcw^T tcw as one
// cv::gemm each (f64 accumulation, one rounding), invz = 1.0f / PcZ,
// dist = cv::norm(PO) and PO.dot(Pn) accumulated in double, PredictScale through
// detmath::predict_scale (glibc logf's levels on every input, tests/test_oracle_kat.py).
__global__ void __launch_bounds__(256) k_frustum(const SearchDev* __restrict__ probs, const FrustumDev* __restrict__ frs,
                                                 float viewingCosLimit, float logScaleFactor, int np, int gx) {
    ORBGPU_LATENCY_WAVE();
    // XCD-aware order (as k_candidates): problem p's blocks run on XCD p % 8, where its
    // candidate search and selection then read the query arrays this kernel writes
    int by, bx;
    if (!xcd_problem_block(np, gx, by, bx)) return;
    const SearchDev& P = probs[by];
    const FrustumDev& Fq = frs[by];
    const int j = bx * blockDim.x + threadIdx.x;
    const bool on = j < P.nq;
    int vis = 0;
    if (on) {
        Fq.mpIndex[j] = j;
        const FrameDev& F = P.cur;
        if (!Fq.skip[j]) {
            const float* T = F.Tcw;
            const float* X = P.mpPos + 3 * (size_t)j;
            const float PcX = gemm_row(T, 0, X[0], X[1], X[2]);
            const float PcY = gemm_row(T, 1, X[0], X[1], X[2]);
            const float PcZ = gemm_row(T, 2, X[0], X[1], X[2]);
            if (!(PcZ < 0.0f)) {
                const float invz = 1.0f / PcZ;
                const float u = F.fx * PcX * invz + F.cx;
                const float v = F.fy * PcY * invz + F.cy;
                if (!(u < F.minX || u > F.maxX) && !(v < F.minY || v > F.maxY)) {
                    const float maxDistance = 1.2f * Fq.maxDist[j];   // GetMaxDistanceInvariance
                    const float minDistance = 0.8f * Fq.minDist[j];   // GetMinDistanceInvariance
                    float Ow[3];
                    for (int i = 0; i < 3; i++) {
                        const double s = (double)T[0 * 4 + i] * T[3] + (double)T[1 * 4 + i] * T[7] +
                                         (double)T[2 * 4 + i] * T[11];
                        Ow[i] = (float)(s * -1.0);
                    }
                    const float PO[3] = {X[0] - Ow[0], X[1] - Ow[1], X[2] - Ow[2]};
                    const double s2 = ((double)PO[0] * PO[0] + (double)PO[1] * PO[1]) + (double)PO[2] * PO[2];
                    const float dist = (float)sqrt(s2);
                    if (!(dist < minDistance || dist > maxDistance)) {
                        const float* Pn = Fq.normal + 3 * (size_t)j;
                        const double dot = ((double)PO[0] * Pn[0] + (double)PO[1] * Pn[1]) + (double)PO[2] * Pn[2];
                        const float viewCos = (float)(dot / (double)dist);
                        if (!(viewCos < viewingCosLimit)) {
                            vis = 1;
                            Fq.projX[j] = u;
                            Fq.projXR[j] = u - F.bf * invz;
                            Fq.projY[j] = v;
                            Fq.level[j] = detmath::predict_scale(Fq.maxDist[j], dist, logScaleFactor, F.nlevels);
                            Fq.viewCos[j] = viewCos;
                        }
                    }
                }
            }
        }
        Fq.inView[j] = (uint8_t)vis;
        if (!vis && P.qinfo) P.qinfo[j] = make_int4(-1, 0, 0, 0);   // no window: k_candidates skips it
    }
    const unsigned long long vm = __ballot(vis != 0);
    const int nv = (int)__popcll(vm);
    if (P.visList && nv) {   // compact the in-view queries, one atomic per wave
        int base = 0;
        if ((threadIdx.x & 63) == 0) base = atomicAdd(P.visCount, nv);
        base = __shfl(base, 0, 64);
        if (vis) P.visList[base + (int)__popcll(vm & ((1ull << (threadIdx.x & 63)) - 1ull))] = j;
    }
    if ((threadIdx.x & 63) == 0 && nv) atomicAdd(Fq.nvisible, nv);
}

// Greedy replay as a fixed-point iteration (one workgroup per problem).
// The reference loop is sequential: query q may not take a keypoint that an earlier
// query q' < q already took with Observations() > 0 (ORBmatcher.cc:87-89, 1403-1405).
// Its outcome is the unique solution of
//     choice(q) = decide(q, occupied = occ0 U { choice(q') : q' < q, take(q'), obs(q') })
// and since choice(q) depends only on earlier queries, Jacobi iteration over all queries
// in parallel reaches it: after round r every query whose dependency chain is shorter
// than r is final, and a round that changes nothing is the fixed point.  Conflicts are
// rare, so it converges in a few rounds (about 4 for SearchLocalPoints, 12 for the
// last-frame search of the bench); each round is one owner[]
// rebuild (atomicMin of the claiming query per keypoint, in LDS) plus one decide() per
// query against the kTopK list, with a full rescan only when every kept candidate is
// taken.  Overwrites (a later query re-taking a keypoint whose earlier taker has no
// observations) keep the latest taker, as the reference's sequential assignment does.
constexpr int kSelQLast = 8, kSelQLocal = 4;   // register slots per thread of k_select_r
static_assert(512 * kSelQLast >= kMaxFrameKeys, "LAST mode: every query of a frame in a register slot");

// decide(q) from global memory only (the whole top-K list, then the rescan with occupancy): the
// rare path of k_select_r, kept out of line so that its unrolled slots stay small
template <bool LAST>
__device__ __noinline__ int select_slow(const SearchDev* __restrict__ Pp, int q, int c, const uint8_t* s_occ0,
                                        const int* s_owner, const uint8_t* s_oct, float th, int bF, int bB,
                                        float nnratio) {
    const SearchDev& P = *Pp;
    auto occupied = [&](int idx) { return s_occ0[idx] != 0 || s_owner[idx] < q; };
    const int kk = c < kTopK ? c : kTopK;
    const int2* top = P.topk + (size_t)q * kTopK;
    constexpr int need = LAST ? 1 : 2;
    int bestDist = 256, bestIdx = -1, bestDist2 = 256, idx2 = -1, nfree = 0;
    for (int k = 0; k < kk && nfree < need; k++) {
        const int2 e = top[k];
        if (occupied(e.y)) continue;
        if (nfree == 0) { bestDist = e.x; bestIdx = e.y; }
        else { bestDist2 = e.x; idx2 = e.y; }
        nfree++;
    }
    if (nfree < need && c > kTopK) {
        bestDist = bestDist2 = 256;
        bestIdx = idx2 = -1;
        if (LAST) {
            TopK<1> top2;
            const LastQuery lq = last_query(P, q, th, bF != 0, bB != 0);
            if (scan_last(P, lq, occupied, top2) > 0) { bestDist = top2.t[0].x; bestIdx = top2.t[0].y; }
        } else {
            TopK<2> top2;
            const LocalQuery lq = local_query(P, q, th);
            const int c2 = scan_local(P, lq, occupied, top2);
            if (c2 > 0) { bestDist = top2.t[0].x; bestIdx = top2.t[0].y; }
            if (c2 > 1) { bestDist2 = top2.t[1].x; idx2 = top2.t[1].y; }
        }
    }
    if (bestDist > TH_HIGH) return -1;
    if (!LAST) {
        const int bestLevel = s_oct[bestIdx];
        const int bestLevel2 = idx2 >= 0 ? (int)s_oct[idx2] : -1;
        if (bestLevel == bestLevel2 && (float)bestDist > nnratio * (float)bestDist2) return -1;
    }
    return bestIdx;
}

// k_select_r: the fixed point above with the query state in registers.  The queries (all of
// them, or SearchLocalPoints' in-view list) are dealt to the threads, Q per thread (slot s of
// thread t = list entry t + s * NT); each slot holds its query's candidate count, observation
// flag, current choice and first 4 kept candidates (dist << 16 | index), loaded once, so a
// round touches only LDS (owners, initial occupancy, octaves).  A query whose first 4
// candidates are all taken, and list entries beyond NT * Q, go through select_slow (global
// memory).  A query's choice depends on the query order only through `owner < q`, so dealing
// the queries to threads in any order is the same iteration.
template <bool LAST, int NT, int Q>
__global__ void __launch_bounds__(NT) k_select_r(const SearchDev* __restrict__ probs, float th, int bMono,
                                                  float nnratio, int checkOri, int Nmax) {
    ORBGPU_LATENCY_WAVE();
    extern __shared__ int s_dyn[];
    int* s_owner = s_dyn;                                           // earliest claiming query with Observations() > 0
    int* s_lastq = s_dyn + Nmax;                                    // latest claiming query (any)
    uint8_t* s_occ0 = reinterpret_cast<uint8_t*>(s_dyn + 2 * Nmax); // occupancy before this call
    uint8_t* s_rm = s_occ0 + Nmax;                                  // slot cleared by the rotation check
    uint8_t* s_oct = s_rm + Nmax;                                   // keypoint octave
    __shared__ int s_hsz[HISTO_LENGTH];
    __shared__ int s_ind[3];
    __shared__ int s_changed, s_nm, s_rmcnt;
    ORBGPU_PROF_START;
    const SearchDev* Pp = probs + blockIdx.x;
    const SearchDev& P = *Pp;
    const int tid = threadIdx.x;
    const int N = P.cur.N, nq = P.nq;
    const int* list = (!LAST && P.visList) ? P.visList : nullptr;
    const int nact = list ? *P.visCount : nq;
    for (int i = tid; i < N; i += NT) {
        const int m = P.curMP[i];
        s_occ0[i] = (m >= 0 && P.mpObs[m] > 0) ? 1 : 0;
        s_owner[i] = INT_MAX;
        s_lastq[i] = -1;
        s_rm[i] = 0;
        if (!LAST) s_oct[i] = (uint8_t)P.cur.keysUn[i].octave;
    }
    if (tid < HISTO_LENGTH) s_hsz[tid] = 0;
    if (tid == 0) { s_nm = 0; s_rmcnt = 0; }
    bool bF = false, bB = false;
    if (LAST) fwd_bwd(P, bMono != 0, bF, bB);
    uint32_t tk[Q][4];
    int qs[Q], cnt[Q], ch[Q];
    uint32_t obsm = 0;
    auto obs_of = [&](int q) {
        const int mp = LAST ? P.lastMP[q] : P.mpIndex[q];
        return mp >= 0 && P.mpObs[mp] > 0;
    };
#pragma unroll
    for (int s = 0; s < Q; s++) {
        const int k = tid + s * NT;
        qs[s] = k < nact ? (list ? list[k] : k) : -1;
        cnt[s] = -1;
        ch[s] = -1;
#pragma unroll
        for (int j = 0; j < 4; j++) tk[s][j] = 0u;
        if (qs[s] >= 0) {
            const int q = qs[s];
            const int c = P.qinfo[q].x;
            cnt[s] = c;
            if (c > 0) {
                if (obs_of(q)) obsm |= 1u << s;
                const int4* t4 = reinterpret_cast<const int4*>(P.topk + (size_t)q * kTopK);
                const int4 a = t4[0], b = t4[1];   // entries >= min(c, kTopK) are never read
                tk[s][0] = ((uint32_t)a.x << 16) | (uint32_t)a.y;
                tk[s][1] = ((uint32_t)a.z << 16) | (uint32_t)a.w;
                tk[s][2] = ((uint32_t)b.x << 16) | (uint32_t)b.y;
                tk[s][3] = ((uint32_t)b.z << 16) | (uint32_t)b.w;
            }
        }
    }
    __syncthreads();
    ORBGPU_PROF_MARK(LAST ? 0 : 8);
    constexpr int need = LAST ? 1 : 2;
    auto decide = [&](int s) -> int {   // decide(q) for slot s
        const int q = qs[s];
        const int c = cnt[s];
        if (c <= 0) return -1;
        const int kk = c < kTopK ? c : kTopK;
        int bestDist = 256, bestIdx = -1, bestDist2 = 256, idx2 = -1, nfree = 0;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            if (j < kk && nfree < need) {
                const int idx = (int)(tk[s][j] & 0xffffu), d = (int)(tk[s][j] >> 16);
                if (!(s_occ0[idx] != 0 || s_owner[idx] < q)) {
                    if (nfree == 0) { bestDist = d; bestIdx = idx; }
                    else { bestDist2 = d; idx2 = idx; }
                    nfree++;
                }
            }
        }
        if (nfree < need && kk > 4)   // the first 4 kept candidates are taken: the rest of the list
            return select_slow<LAST>(Pp, q, c, s_occ0, s_owner, s_oct, th, bF, bB, nnratio);
        if (bestDist > TH_HIGH) return -1;
        if (!LAST) {
            const int bestLevel = s_oct[bestIdx];
            const int bestLevel2 = idx2 >= 0 ? (int)s_oct[idx2] : -1;
            if (bestLevel == bestLevel2 && (float)bestDist > nnratio * (float)bestDist2) return -1;
        }
        return bestIdx;
    };
    // list entries beyond the register slots: choice in qinfo.y, obs flag in qinfo.z
    auto decide_g = [&](int q) -> int {
        const int c = P.qinfo[q].x;
        return c > 0 ? select_slow<LAST>(Pp, q, c, s_occ0, s_owner, s_oct, th, bF, bB, nnratio) : -1;
    };
    for (int k = NT * Q + tid; k < nact; k += NT) {
        const int q = list ? list[k] : k;
        P.qinfo[q].z = (P.qinfo[q].x > 0 && obs_of(q)) ? 1 : 0;
        P.qinfo[q].y = decide_g(q);
    }
#pragma unroll
    for (int s = 0; s < Q; s++) ch[s] = decide(s);   // round 0: nothing claimed yet
    for (int round = 0; round <= nq; round++) {
        __syncthreads();
        for (int i = tid; i < N; i += NT) s_owner[i] = INT_MAX;
        if (tid == 0) s_changed = 0;
        __syncthreads();
#pragma unroll
        for (int s = 0; s < Q; s++)
            if (ch[s] >= 0 && ((obsm >> s) & 1u)) atomicMin(&s_owner[ch[s]], qs[s]);
        for (int k = NT * Q + tid; k < nact; k += NT) {
            const int q = list ? list[k] : k;
            const int4 qi = P.qinfo[q];
            if (qi.y >= 0 && qi.z) atomicMin(&s_owner[qi.y], q);
        }
        __syncthreads();
        bool chg = false;
#pragma unroll
        for (int s = 0; s < Q; s++) {
            const int c = decide(s);
            if (c != ch[s]) { ch[s] = c; chg = true; }
        }
        for (int k = NT * Q + tid; k < nact; k += NT) {
            const int q = list ? list[k] : k;
            const int c = decide_g(q);
            if (c != P.qinfo[q].y) { P.qinfo[q].y = c; chg = true; }
        }
        if (chg) s_changed = 1;
        __syncthreads();
        ORBGPU_PROF_COUNT(LAST ? 6 : 14);
        if (!s_changed) break;
    }
    ORBGPU_PROF_MARK(LAST ? 1 : 9);
    int nm = 0;
#pragma unroll
    for (int s = 0; s < Q; s++)
        if (ch[s] >= 0) { atomicMax(&s_lastq[ch[s]], qs[s]); nm++; }
    for (int k = NT * Q + tid; k < nact; k += NT) {
        const int q = list ? list[k] : k;
        const int c = P.qinfo[q].y;
        if (c >= 0) { atomicMax(&s_lastq[c], q); nm++; }
    }
    atomicAdd(&s_nm, nm);
    __syncthreads();
    if (LAST && checkOri) {
        // rotation-consistency histogram over the matches (ORBmatcher.cc:1422-1467); LAST mode
        // has no list beyond the slots (nq <= kMaxFrameKeys <= NT * Q, checked by the host)
        int bins[Q];
#pragma unroll
        for (int s = 0; s < Q; s++) {
            bins[s] = -1;
            const int bi = ch[s];
            if (bi < 0) continue;
            float rot = P.last.keysUn[qs[s]].angle - P.cur.keysUn[bi].angle;
            if (rot < 0.0f) rot += 360.0f;
            int bin = (int)roundf(rot * (1.0f / HISTO_LENGTH));
            if (bin == HISTO_LENGTH) bin = 0;
            atomicAdd(&s_hsz[bin], 1);
            bins[s] = bin;
        }
        __syncthreads();
        if (tid == 0) {
            // ComputeThreeMaxima, ORBmatcher.cc:1601-1642
            int max1 = 0, max2 = 0, max3 = 0, ind1 = -1, ind2 = -1, ind3 = -1;
            for (int i = 0; i < HISTO_LENGTH; i++) {
                const int sz = s_hsz[i];
                if (sz > max1) { max3 = max2; max2 = max1; max1 = sz; ind3 = ind2; ind2 = ind1; ind1 = i; }
                else if (sz > max2) { max3 = max2; max2 = sz; ind3 = ind2; ind2 = i; }
                else if (sz > max3) { max3 = sz; ind3 = i; }
            }
            if (max2 < 0.1f * (float)max1) { ind2 = -1; ind3 = -1; }
            else if (max3 < 0.1f * (float)max1) { ind3 = -1; }
            s_ind[0] = ind1;
            s_ind[1] = ind2;
            s_ind[2] = ind3;
        }
        __syncthreads();
        const int ind1 = s_ind[0], ind2 = s_ind[1], ind3 = s_ind[2];
        int removed = 0;
#pragma unroll
        for (int s = 0; s < Q; s++) {
            if (ch[s] < 0) continue;
            const int b = bins[s];
            if (b != ind1 && b != ind2 && b != ind3) {
                s_rm[ch[s]] = 1;
                removed++;
            }
        }
        atomicAdd(&s_rmcnt, removed);
    }
    __syncthreads();
    ORBGPU_PROF_MARK(LAST ? 2 : 10);
    for (int i = tid; i < N; i += NT) {
        const int lq = s_lastq[i];
        if (s_rm[i]) P.curMP[i] = -1;
        else if (lq >= 0) P.curMP[i] = LAST ? P.lastMP[lq] : P.mpIndex[lq];
    }
    if (tid == 0) *P.nmatches = s_nm - s_rmcnt;
    ORBGPU_PROF_MARK(LAST ? 3 : 11);
}

// CSR candidate mode: one wave per query, lanes over candidates; (dist<<20 | k)
// keys make the wave min pick the earliest candidate among equal distances.
__global__ void __launch_bounds__(256) k_csr_hamming(const uint8_t* __restrict__ q, int nq, const uint8_t* __restrict__ t,
                                                     const int* __restrict__ off, const int* __restrict__ cand,
                                                     int* __restrict__ dist, int* __restrict__ best_idx,
                                                     int* __restrict__ best_dist, int* __restrict__ second_dist,
                                                     unsigned long long* counters) {
    const int lane = threadIdx.x & 63;
    const int qi = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (qi >= nq) return;
    const int b = off[qi], e = off[qi + 1];
    const uint8_t* qd = q + 32 * (size_t)qi;
    unsigned long long k1 = ~0ull, k2 = ~0ull;
    for (int k = b + lane; k < e; k += 64) {
        const int d = hamming32(qd, t + 32 * (size_t)cand[k]);
        if (dist) dist[k] = d;   // best / second need no per-pair store
        const unsigned long long key = ((unsigned long long)d << 32) | (unsigned)(k - b);
        if (key < k1) { k2 = k1; k1 = key; }
        else if (key < k2) k2 = key;
    }
    for (int o = 32; o > 0; o >>= 1) {
        const unsigned long long o1 = __shfl_xor(k1, o, 64), o2 = __shfl_xor(k2, o, 64);
        const unsigned long long n1 = o1 < k1 ? o1 : k1;
        const unsigned long long hi = o1 < k1 ? k1 : o1;
        unsigned long long n2 = o2 < k2 ? o2 : k2;
        n2 = hi < n2 ? hi : n2;
        k1 = n1;
        k2 = n2;
    }
    if (lane == 0) {
        if (counters) {
            const int sl = blockIdx.x & (kCountSlots - 1);
            atomicAdd(&counters[4 * kCountSlots + sl], (unsigned long long)(e - b));
            atomicAdd(&counters[5 * kCountSlots + sl], 1ull);
        }
        best_idx[qi] = k1 == ~0ull ? -1 : cand[b + (int)(k1 & 0xffffffffu)];
        best_dist[qi] = k1 == ~0ull ? 256 : (int)(k1 >> 32);
        second_dist[qi] = k2 == ~0ull ? 256 : (int)(k2 >> 32);
    }
}

// ------------------------------------------------------- dense (brute-force) matching
// Every query of a problem against every train descriptor of it, best / second distance with the
// reference loops' rule (distance strictly below the best: earliest index wins ties; ORBmatcher.cc
// e.g. 1411-1423, 1647-1663).  A workgroup takes 256 queries (one per thread, descriptor in
// registers) x one block of kDenseBlock train descriptors staged in LDS: every wave reads the
// same train descriptor (an LDS broadcast) per step, so a pair costs 8 XOR + 8 popcount-adds and
// no memory traffic.  The blocks' (best, second) keys (distance << 32 | index) merge exactly:
// the minimum key is the sequential loop's best, the second-smallest key's distance its second.
constexpr int kDenseBlock = 256;
constexpr int kDenseQ = 256;

struct DenseJob {
    int prob, q0, t0, part;   // problem, first query, first train row, partial slot
};

template <int TB>
__global__ void __launch_bounds__(kDenseQ) k_dense_hamming(const DenseDev* __restrict__ probs,
                                                           const DenseJob* __restrict__ jobs,
                                                           unsigned long long* __restrict__ part,
                                                           unsigned long long* counters) {
    __shared__ uint4 tl[TB * 2];
    const DenseJob J = jobs[blockIdx.x];
    const DenseDev P = probs[J.prob];
    const int tid = threadIdx.x;
    const int nt = min(TB, P.nt - J.t0);
    const uint4* src = reinterpret_cast<const uint4*>(P.t + 32 * (size_t)J.t0);
    for (int k = tid; k < 2 * nt; k += kDenseQ) tl[k] = src[k];
    const int qi = J.q0 + tid;
    uint4 a0 = make_uint4(0, 0, 0, 0), a1 = a0;
    if (qi < P.nq) {
        a0 = reinterpret_cast<const uint4*>(P.q + 32 * (size_t)qi)[0];
        a1 = reinterpret_cast<const uint4*>(P.q + 32 * (size_t)qi)[1];
    }
    __syncthreads();
    // keys d << 16 | j (d <= 256, j < kDenseBlock): in j order, the reference's strict
    // `dist < bestDist` / `dist < bestDist2` updates are b1 = min(b1, key) and
    // b2 = min(b2, max(b1, key)) on the keys (b1 <= b2; an equal distance later in j is a larger key,
    // so it never displaces the best and does become the second).  Four train rows per step:
    // their LDS broadcasts are issued together and the four popcount chains are independent.
    unsigned b1 = 0xffffffffu, b2 = 0xffffffffu;
    auto dist = [&](const uint4& t0, const uint4& t1) {
        return __popc(a0.x ^ t0.x) + __popc(a0.y ^ t0.y) + __popc(a0.z ^ t0.z) + __popc(a0.w ^ t0.w) +
               __popc(a1.x ^ t1.x) + __popc(a1.y ^ t1.y) + __popc(a1.z ^ t1.z) + __popc(a1.w ^ t1.w);
    };
    auto take = [&](unsigned key) {
        b2 = min(b2, max(b1, key));   // (b1 <= b2): the median of b1, b2, key
        b1 = min(b1, key);
    };
    int j = 0;
    for (; j + 4 <= nt; j += 4) {
        const uint4 t0 = tl[2 * j], t1 = tl[2 * j + 1], t2 = tl[2 * j + 2], t3 = tl[2 * j + 3];
        const uint4 t4 = tl[2 * j + 4], t5 = tl[2 * j + 5], t6 = tl[2 * j + 6], t7 = tl[2 * j + 7];
        const unsigned d0 = dist(t0, t1), d1 = dist(t2, t3), d2 = dist(t4, t5), d3 = dist(t6, t7);
        take((d0 << 16) | (unsigned)j);
        take((d1 << 16) | (unsigned)(j + 1));
        take((d2 << 16) | (unsigned)(j + 2));
        take((d3 << 16) | (unsigned)(j + 3));
    }
    for (; j < nt; j++) take((dist(tl[2 * j], tl[2 * j + 1]) << 16) | (unsigned)j);
    if (qi < P.nq) {
        unsigned long long* o = part + 2 * ((size_t)J.part * kDenseQ + tid);
        o[0] = b1 == 0xffffffffu ? ~0ull : ((unsigned long long)(b1 >> 16) << 32) | (unsigned)(J.t0 + (int)(b1 & 0xffffu));
        // the block's second-smallest key: its distance is b2; any index past the best keeps
        // the merge's ordering of equal distances irrelevant to second_dist
        o[1] = b2 == 0xffffffffu ? ~0ull : ((unsigned long long)(b2 >> 16) << 32) | 0xffffffffu;
    }
    if (counters && tid == 0) {
        const int sl = blockIdx.x & (kCountSlots - 1);
        atomicAdd(&counters[6 * kCountSlots + sl], (unsigned long long)nt * (unsigned long long)min(kDenseQ, P.nq - J.q0));
    }
}

// Merge the train blocks' partial keys of every query (one thread per query).
__global__ void __launch_bounds__(256) k_dense_merge(const DenseDev* __restrict__ probs, const int* __restrict__ qjob,
                                                     const DenseJob* __restrict__ jobs, int nblk_per_q,
                                                     const unsigned long long* __restrict__ part, int nq_blocks,
                                                     int njobs) {
    const int g = blockIdx.x * blockDim.x + threadIdx.x;   // (query block, thread)
    const int qb = g / kDenseQ, tq = g % kDenseQ;
    if (qb >= nq_blocks) return;
    const DenseJob J0 = jobs[qjob[qb]];
    const DenseDev P = probs[J0.prob];
    const int qi = J0.q0 + tq;
    if (qi >= P.nq) return;
    unsigned long long k1 = ~0ull, k2 = ~0ull;
    for (int b = 0; b < nblk_per_q && qjob[qb] + b < njobs; b++) {
        const DenseJob J = jobs[qjob[qb] + b];
        if (J.prob != J0.prob || J.q0 != J0.q0) break;
        const unsigned long long* o = part + 2 * ((size_t)J.part * kDenseQ + tq);
        const unsigned long long o1 = o[0], o2 = o[1];
        const unsigned long long n1 = o1 < k1 ? o1 : k1, hi = o1 < k1 ? k1 : o1;
        unsigned long long n2 = o2 < k2 ? o2 : k2;
        n2 = hi < n2 ? hi : n2;
        k1 = n1;
        k2 = n2;
    }
    P.best_idx[qi] = k1 == ~0ull ? -1 : (int)(k1 & 0xffffffffu);
    P.best_dist[qi] = k1 == ~0ull ? 256 : (int)(k1 >> 32);
    P.second_dist[qi] = k2 == ~0ull ? 256 : (int)(k2 >> 32);
}

// ------------------------------------------------------- area-candidate engine
// Frame::GetFeaturesInArea windows of arbitrary queries over one frame grid, every candidate
// with its Hamming distance, in the reference's enumeration order (CSR).  The order-dependent
// selection of the remaining ORBmatcher searches is replayed on the host from these lists.
__global__ void __launch_bounds__(256) k_area_count(const SearchDev* __restrict__ probs, const AreaQuery* __restrict__ q,
                                                    int nq, int* __restrict__ cnt) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nq) return;
    const AreaQuery a = q[i];
    int c = 0;
    if (a.qd >= 0) {
        QueryWin w{a.x, a.y, a.r, a.minLevel, a.maxLevel};
        for_features_in_area(probs[0], w, [&](int) { c++; });
    }
    cnt[i] = c;
}

__global__ void __launch_bounds__(256) k_area_fill(const SearchDev* __restrict__ probs, const AreaQuery* __restrict__ q,
                                                   int nq, const uint8_t* __restrict__ qdesc, const int* __restrict__ off,
                                                   int2* __restrict__ out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nq) return;
    const AreaQuery a = q[i];
    if (a.qd < 0) return;
    const SearchDev& P = probs[0];
    const uint8_t* d0 = qdesc + 32 * (size_t)a.qd;
    int k = off[i];
    QueryWin w{a.x, a.y, a.r, a.minLevel, a.maxLevel};
    for_features_in_area(P, w, [&](int idx) { out[k++] = make_int2(idx, hamming32(d0, P.cur.desc + 32 * (size_t)idx)); });
}

int Matcher::area_candidates(const SearchDev& frame, const AreaQuery* d_q, int nq, const uint8_t* d_qdesc,
                             std::vector<int>& off, std::vector<int2>& cand) {
    off.assign((size_t)nq + 1, 0);
    cand.clear();
    if (frame.cur.N > kMaxFrameKeys || frame.cur.N < 0) return -1;
    const size_t grid = ((size_t)(kGridCells + 1 + frame.cur.N) * 4 + 255) & ~(size_t)255;
    const size_t need = grid + 2 * (((size_t)nq + 1) * 4 + 256) + sizeof(SearchDev) + 256;
    if (need > scratch_cap_) {
        if (d_scratch_) (void)hipFree(d_scratch_);
        scratch_cap_ = need * 2;
        ORB_HIP_CHECK(hipMalloc(&d_scratch_, scratch_cap_));
    }
    char* s = (char*)d_scratch_;
    SearchDev P = frame;
    P.gridStart = (int*)s;
    P.gridIdx = P.gridStart + kGridCells + 1;
    s += grid;
    int* d_cnt = (int*)s;
    s += (((size_t)nq + 1) * 4 + 255) & ~(size_t)255;
    int* d_off = (int*)s;
    s += (((size_t)nq + 1) * 4 + 255) & ~(size_t)255;
    SearchDev* dp = (SearchDev*)s;
    ORB_HIP_CHECK(hipMemcpyAsync(dp, &P, sizeof(SearchDev), hipMemcpyHostToDevice, stream_));
    hipLaunchKernelGGL(k_build_grid, dim3(1), dim3(256), grid_lds_bytes(frame.cur.N), stream_, dp, 0);
    if (nq == 0) return stream_wait(stream_) == hipSuccess ? 0 : -2;
    hipLaunchKernelGGL(k_area_count, dim3((nq + 255) / 256), dim3(256), 0, stream_, dp, d_q, nq, d_cnt);
    ORB_HIP_CHECK(hipGetLastError());
    ORB_HIP_CHECK(hipMemcpyAsync(off.data() + 1, d_cnt, sizeof(int) * nq, hipMemcpyDeviceToHost, stream_));
    ORB_HIP_CHECK(stream_wait(stream_));
    for (int i = 0; i < nq; i++) off[i + 1] += off[i];
    const int total = off[nq];
    cand.resize((size_t)std::max(total, 1));
    if (total == 0) return 0;
    if ((size_t)total * sizeof(int2) > cand_cap_) {
        if (d_cand_) (void)hipFree(d_cand_);
        cand_cap_ = (size_t)total * sizeof(int2) * 2;
        ORB_HIP_CHECK(hipMalloc(&d_cand_, cand_cap_));
    }
    ORB_HIP_CHECK(hipMemcpyAsync(d_off, off.data(), sizeof(int) * ((size_t)nq + 1), hipMemcpyHostToDevice, stream_));
    hipLaunchKernelGGL(k_area_fill, dim3((nq + 255) / 256), dim3(256), 0, stream_, dp, d_q, nq, d_qdesc, d_off,
                       (int2*)d_cand_);
    ORB_HIP_CHECK(hipGetLastError());
    ORB_HIP_CHECK(hipMemcpyAsync(cand.data(), d_cand_, sizeof(int2) * (size_t)total, hipMemcpyDeviceToHost, stream_));
    ORB_HIP_CHECK(stream_wait(stream_));
    return 0;
}

// --------------------------------------------------------------------- host
Matcher::~Matcher() {
    for (int i = 0; i < 16; i++)
        if (ev_[i]) (void)hipEventDestroy(ev_[i]);
    if (d_count_) (void)hipFree(d_count_);
    if (d_cand_) (void)hipFree(d_cand_);
    if (d_dense_) (void)hipFree(d_dense_);
    if (d_scratch_) (void)hipFree(d_scratch_);
    if (d_probs_) (void)hipFree(d_probs_);
    if (d_arena_) (void)hipFree(d_arena_);
    if (stream_) (void)hipStreamDestroy(stream_);
}

int Matcher::init_device() {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return -4;
    // ORBGPU_MATCH_STREAM_PRIO=1: the tracking lane's stream at the device's highest priority
    // (A/B runs of the pipelined bench; the reference has no counterpart)
    const char* pe = std::getenv("ORBGPU_MATCH_STREAM_PRIO");
    if (pe && pe[0] == '1') {
        int lo = 0, hi = 0;
        ORB_HIP_CHECK(hipDeviceGetStreamPriorityRange(&lo, &hi));
        ORB_HIP_CHECK(hipStreamCreateWithPriority(&stream_, hipStreamNonBlocking, hi));
    } else {
        ORB_HIP_CHECK(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
    }
    return 0;
}

int Matcher::arena_reserve(size_t bytes) {
    arena_used_ = 0;
    if (bytes <= arena_cap_) return 0;
    if (d_arena_) (void)hipFree(d_arena_);
    d_arena_ = nullptr;
    arena_cap_ = 0;
    ORB_HIP_CHECK(hipMalloc(&d_arena_, bytes));
    arena_cap_ = bytes;
    return 0;
}

void* Matcher::arena_alloc(size_t bytes) {
    bytes = (bytes + 255) & ~(size_t)255;
    if (arena_used_ + bytes > arena_cap_) return nullptr;
    void* p = (char*)d_arena_ + arena_used_;
    arena_used_ += bytes;
    return p;
}

// k_candidates' XCD-aware 1-D grid: gx blocks per problem, problems dealt to the 8 XCDs
static inline int cand_gx(int maxq, int nt) { return (maxq + nt - 1) / nt; }
static inline dim3 cand_grid(int maxq, int nt, int np) { return xcd_grid(cand_gx(maxq, nt), np); }

int Matcher::run(std::vector<SearchDev>& probs, float th, bool bMono, bool lastMode, float nnratio) {
    const int np = (int)probs.size();
    if (np == 0) return 0;
    size_t need = 0;
    int maxq = 0, maxN = 1;
    const bool vis = frustum_ != nullptr;   // SearchLocalPoints: in-view query lists
    for (auto& p : probs) {
        if (p.cur.N > kMaxFrameKeys || p.cur.N < 0 || p.nq < 0) return -1;
        maxN = std::max(maxN, p.cur.N);
        need += ((size_t)(kGridCells + 1 + p.cur.N) * 4 + 255) & ~(size_t)255;
        need += ((size_t)p.nq * (kTopK * 8 + 16 + 8) + 255) & ~(size_t)255;
        if (vis) need += ((size_t)p.nq * 4 + 255) & ~(size_t)255;
        maxq = std::max(maxq, p.nq);
    }
    if (vis) need += ((size_t)np * 4 + 255) & ~(size_t)255;
    if (need > scratch_cap_) {
        if (d_scratch_) (void)hipFree(d_scratch_);
        scratch_cap_ = need * 2;
        ORB_HIP_CHECK(hipMalloc(&d_scratch_, scratch_cap_));
    }
    char* s = (char*)d_scratch_;
    int* visCounts = nullptr;
    if (vis) {
        visCounts = (int*)s;
        s += ((size_t)np * 4 + 255) & ~(size_t)255;
    }
    for (size_t k = 0; k < probs.size(); k++) {
        SearchDev& p = probs[k];
        p.gridStart = (int*)s;
        p.gridIdx = p.gridStart + kGridCells + 1;
        s += ((size_t)(kGridCells + 1 + p.cur.N) * 4 + 255) & ~(size_t)255;
        p.topk = (int2*)s;
        p.qinfo = (int4*)(p.topk + (size_t)p.nq * kTopK);
        p.hist = (int2*)(p.qinfo + p.nq);
        s += ((size_t)p.nq * (kTopK * 8 + 16 + 8) + 255) & ~(size_t)255;
        p.visList = nullptr;
        p.visCount = nullptr;
        if (vis) {
            p.visList = (int*)s;
            p.visCount = visCounts + k;
            s += ((size_t)p.nq * 4 + 255) & ~(size_t)255;
        }
    }
    if (vis) ORB_HIP_CHECK(hipMemsetAsync(visCounts, 0, (size_t)np * 4, stream_));
    const size_t pb = sizeof(SearchDev) * np;
    if (pb > probs_cap_) {
        if (d_probs_) (void)hipFree(d_probs_);
        probs_cap_ = pb * 2;
        ORB_HIP_CHECK(hipMalloc(&d_probs_, probs_cap_));
    }
    ORB_HIP_CHECK(hipMemcpyAsync(d_probs_, h2d_src(probs.data(), pb), pb, hipMemcpyHostToDevice, stream_));
    SearchDev* dp = (SearchDev*)d_probs_;
    if (frustum_ && maxq > 0) {   // SearchLocalPoints: Frame::isInFrustum fills the query arrays first
        mark(8);
        hipLaunchKernelGGL(k_frustum, cand_grid(maxq, 256, np), dim3(256), 0, stream_, (const SearchDev*)dp,
                           frustum_, frustumCos_, frustumLsf_, np, cand_gx(maxq, 256));
        mark(9);
    }
    if (timing_) {
        if (int e = zero_counters(0, 2)) return e;
        mark(0);
    }
    hipLaunchKernelGGL(k_build_grid, dim3(np), dim3(256), grid_lds_bytes(maxN), stream_, dp, 1);
    mark(1);
    if (maxq > 0) {
        if (lastMode) {
            if (maxN <= kStageMaxN && stage_threads() == 256)
                hipLaunchKernelGGL((k_candidates<true, true, 256>), cand_grid(maxq, 256, np), dim3(256), kStageLds,
                                   stream_, dp, np, cand_gx(maxq, 256), th, (int)bMono, counters());
            else if (maxN <= kStageMaxN)
                hipLaunchKernelGGL((k_candidates<true, true, kStageThreads>), cand_grid(maxq, kStageThreads, np),
                                   dim3(kStageThreads), kStageLds,
                                   stream_, dp, np, cand_gx(maxq, kStageThreads), th, (int)bMono, counters());
            else
                hipLaunchKernelGGL((k_candidates<true, false, 256>), cand_grid(maxq, 256, np), dim3(256), 0, stream_, dp,
                                   np, cand_gx(maxq, 256), th, (int)bMono, counters());
            mark(2);
            // nq = the last frame's N <= kMaxFrameKeys = 512 * kSelQLast: every query in a slot
            hipLaunchKernelGGL((k_select_r<true, 512, kSelQLast>), dim3(np), dim3(512), select_lds_bytes(maxN), stream_, dp,
                               th, (int)bMono, nnratio, (int)checkOri_, maxN);
        } else {
            if (maxN <= kStageMaxN && cand_local_stage() && stage_threads() == 256)
                hipLaunchKernelGGL((k_candidates<false, true, 256>), cand_grid(maxq, 256, np), dim3(256), kStageLds,
                                   stream_, dp, np, cand_gx(maxq, 256), th, 0, counters());
            else if (maxN <= kStageMaxN && cand_local_stage())
                hipLaunchKernelGGL((k_candidates<false, true, kStageThreads>), cand_grid(maxq, kStageThreads, np),
                                   dim3(kStageThreads), kStageLds,
                                   stream_, dp, np, cand_gx(maxq, kStageThreads), th, 0, counters());
            else
                hipLaunchKernelGGL((k_candidates<false, false, 256>), cand_grid(maxq, 256, np), dim3(256), 0, stream_, dp,
                                   np, cand_gx(maxq, 256), th, 0, counters());
            mark(2);
            // SearchLocalPoints-sized query sets (thousands of local map points, long occupancy
            // chains between duplicated points): 16 waves per round of the fixed point
            if (select_local_threads() == 512)
                hipLaunchKernelGGL((k_select_r<false, 512, 2 * kSelQLocal>), dim3(np), dim3(512), select_lds_bytes(maxN),
                                   stream_, dp, th, 0, nnratio, 0, maxN);
            else
                hipLaunchKernelGGL((k_select_r<false, kSelectLocalThreads, kSelQLocal>), dim3(np),
                                   dim3(kSelectLocalThreads), select_lds_bytes(maxN), stream_, dp, th, 0, nnratio, 0, maxN);
        }
    } else {
        mark(2);
    }
    mark(3);
    ORB_HIP_CHECK(hipGetLastError());
    return 0;
}

int Matcher::search_last(std::vector<SearchDev>& probs, float th, bool bMono) {
    return run(probs, th, bMono, true, nnratio_);
}

int Matcher::frustum(std::vector<SearchDev>& probs, const std::vector<FrustumDev>& fr, float viewingCosLimit,
                     float logScaleFactor) {
    const int np = (int)probs.size();
    int maxq = 0;
    for (auto& p : probs) maxq = std::max(maxq, p.nq);
    if (np == 0 || maxq == 0) return 0;
    const size_t pb = sizeof(SearchDev) * np;
    if (pb > probs_cap_) {
        if (d_probs_) (void)hipFree(d_probs_);
        probs_cap_ = pb * 2;
        ORB_HIP_CHECK(hipMalloc(&d_probs_, probs_cap_));
    }
    FrustumDev* dfr = (FrustumDev*)arena_alloc(sizeof(FrustumDev) * np);
    if (!dfr) return -2;
    ORB_HIP_CHECK(hipMemcpyAsync(d_probs_, probs.data(), pb, hipMemcpyHostToDevice, stream_));
    ORB_HIP_CHECK(hipMemcpyAsync(dfr, fr.data(), sizeof(FrustumDev) * np, hipMemcpyHostToDevice, stream_));
    mark(8);
    hipLaunchKernelGGL(k_frustum, cand_grid(maxq, 256, np), dim3(256), 0, stream_, (const SearchDev*)d_probs_, dfr,
                       viewingCosLimit, logScaleFactor, np, cand_gx(maxq, 256));
    mark(9);
    ORB_HIP_CHECK(hipGetLastError());
    return 0;
}

int Matcher::search_local_points(std::vector<SearchDev>& probs, std::vector<FrustumDev>& fr, float viewingCosLimit,
                                 float logScaleFactor, float th, float nnratio) {
    const int np = (int)probs.size();
    if (np == 0) return 0;
    int maxq = 0;
    for (auto& p : probs) maxq = std::max(maxq, p.nq);
    if (maxq > 0) {
        // per-problem isInFrustum outputs (inView 1 B, projX/XR/Y/viewCos 4 B, level/mpIndex 4 B)
        size_t need = sizeof(FrustumDev) * np + 256;
        for (auto& p : probs) need += 7 * ((((size_t)p.nq * 4) + 255) & ~(size_t)255);
        char* base = (char*)arena_alloc(need);
        if (!base) return -2;
        char* o = base + ((sizeof(FrustumDev) * np + 255) & ~(size_t)255);
        for (int k = 0; k < np; k++) {
            const size_t b = (((size_t)probs[k].nq * 4) + 255) & ~(size_t)255;
            FrustumDev& f = fr[k];
            f.inView = (uint8_t*)o; o += b;
            f.projX = (float*)o; o += b;
            f.projXR = (float*)o; o += b;
            f.projY = (float*)o; o += b;
            f.level = (int*)o; o += b;
            f.viewCos = (float*)o; o += b;
            f.mpIndex = (int*)o; o += b;
            SearchDev& P = probs[k];
            P.inView = f.inView; P.projX = f.projX; P.projXR = f.projXR; P.projY = f.projY;
            P.level = f.level; P.viewCos = f.viewCos; P.mpIndex = f.mpIndex;
        }
        ORB_HIP_CHECK(hipMemcpyAsync(base, h2d_src(fr.data(), sizeof(FrustumDev) * np), sizeof(FrustumDev) * np,
                                     hipMemcpyHostToDevice, stream_));
        frustum_ = (const FrustumDev*)base;   // launched by run() once the problems are on the device
        frustumCos_ = viewingCosLimit;
        frustumLsf_ = logScaleFactor;
    }
    const int rc = run(probs, th, false, false, nnratio);
    frustum_ = nullptr;
    return rc;
}
int Matcher::search_local(std::vector<SearchDev>& probs, float th) { return run(probs, th, false, false, nnratio_); }

int Matcher::candidates(const uint8_t* q, int nq, const uint8_t* t, int nt, const int* off, const int* cand, int* dist,
                        int* best_idx, int* best_dist, int* second_dist) {
    (void)nt;
    if (nq <= 0) return 0;
    if (timing_) {
        if (int e = zero_counters(4, 2)) return e;
        mark(12);
    }
    hipLaunchKernelGGL(k_csr_hamming, dim3((nq + 3) / 4), dim3(256), 0, stream_, q, nq, t, off, cand, dist, best_idx,
                       best_dist, second_dist, counters());
    mark(13);
    ORB_HIP_CHECK(hipGetLastError());
    return 0;
}

// train rows per k_dense_hamming workgroup: 256, or 128 / 64 (ORBGPU_DENSE_TB) for more
// workgroups (and waves per SIMD) over the same tiles, at more partial keys for the merge
static int dense_block() {
    static const int v = [] {
        const char* e = std::getenv("ORBGPU_DENSE_TB");
        const int b = e ? std::atoi(e) : kDenseBlock;
        return b == 64 || b == 128 ? b : kDenseBlock;
    }();
    return v;
}

int Matcher::dense(const std::vector<DenseDev>& probs) {
    const int np = (int)probs.size();
    if (np == 0) return 0;
    const int TB = dense_block();
    std::vector<DenseJob> jobs;
    std::vector<int> qjob;   // first job of each query block (its train blocks follow it)
    int maxBlk = 0;
    for (int p = 0; p < np; p++) {
        // a problem without train rows still runs one (empty) block: its queries get (-1, 256, 256)
        const int nb = std::max(1, (probs[p].nt + TB - 1) / TB);
        maxBlk = std::max(maxBlk, nb);
        for (int q0 = 0; q0 < probs[p].nq; q0 += kDenseQ) {
            qjob.push_back((int)jobs.size());
            for (int b = 0; b < nb; b++) jobs.push_back(DenseJob{p, q0, b * TB, (int)jobs.size()});
        }
    }
    const size_t bP = (sizeof(DenseDev) * np + 255) & ~(size_t)255, bJ = (sizeof(DenseJob) * jobs.size() + 255) & ~(size_t)255;
    const size_t bQ = (sizeof(int) * qjob.size() + 255) & ~(size_t)255;
    const size_t bPart = sizeof(unsigned long long) * 2 * kDenseQ * std::max<size_t>(jobs.size(), 1);
    const size_t need = bP + bJ + bQ + bPart;
    if (need > dense_cap_) {
        if (d_dense_) (void)hipFree(d_dense_);
        d_dense_ = nullptr;
        dense_cap_ = 0;
        ORB_HIP_CHECK(hipMalloc(&d_dense_, need * 2));
        dense_cap_ = need * 2;
    }
    char* b = (char*)d_dense_;
    DenseDev* dP = (DenseDev*)b;
    DenseJob* dJ = (DenseJob*)(b + bP);
    int* dQ = (int*)(b + bP + bJ);
    unsigned long long* dPart = (unsigned long long*)(b + bP + bJ + bQ);
    // one staging copy: problems | jobs | query-block index
    std::vector<char> h(bP + bJ + bQ, 0);
    std::memcpy(h.data(), probs.data(), sizeof(DenseDev) * np);
    if (!jobs.empty()) std::memcpy(h.data() + bP, jobs.data(), sizeof(DenseJob) * jobs.size());
    if (!qjob.empty()) std::memcpy(h.data() + bP + bJ, qjob.data(), sizeof(int) * qjob.size());
    ORB_HIP_CHECK(hipMemcpyAsync(b, h2d_src(h.data(), h.size()), h.size(), hipMemcpyHostToDevice, stream_));
    if (timing_) {
        if (int e = zero_counters(6, 1)) return e;
        mark(14);
    }
    if (!jobs.empty()) {
        if (TB == 64)
            hipLaunchKernelGGL(k_dense_hamming<64>, dim3((unsigned)jobs.size()), dim3(kDenseQ), 0, stream_,
                               (const DenseDev*)dP, (const DenseJob*)dJ, dPart, counters());
        else if (TB == 128)
            hipLaunchKernelGGL(k_dense_hamming<128>, dim3((unsigned)jobs.size()), dim3(kDenseQ), 0, stream_,
                               (const DenseDev*)dP, (const DenseJob*)dJ, dPart, counters());
        else
            hipLaunchKernelGGL(k_dense_hamming<kDenseBlock>, dim3((unsigned)jobs.size()), dim3(kDenseQ), 0, stream_,
                               (const DenseDev*)dP, (const DenseJob*)dJ, dPart, counters());
    }
    if (!qjob.empty())
        hipLaunchKernelGGL(k_dense_merge, dim3((unsigned)((qjob.size() * kDenseQ + 255) / 256)), dim3(256), 0, stream_,
                           (const DenseDev*)dP, (const int*)dQ, (const DenseJob*)dJ, maxBlk, dPart, (int)qjob.size(),
                           (int)jobs.size());
    mark(15);
    ORB_HIP_CHECK(hipGetLastError());
    if (!chain_.on()) ORB_HIP_CHECK(stream_wait(stream_));   // the pageable staging vector
    return 0;
}

int Matcher::dense_timing(float* ms, long long* pairs) {
    *ms = -1.0f;
    *pairs = -1;
    if (!d_count_) return 0;
    ORB_HIP_CHECK(stream_wait(stream_));
    if (evSet_[14] && evSet_[15]) (void)hipEventElapsedTime(ms, ev_[14], ev_[15]);
    std::vector<unsigned long long> c(kCountSlots);
    ORB_HIP_CHECK(hipMemcpy(c.data(), d_count_ + 6 * kCountSlots, sizeof(unsigned long long) * kCountSlots,
                            hipMemcpyDeviceToHost));
    *pairs = 0;
    for (unsigned long long v : c) *pairs += (long long)v;
    return 0;
}

int Matcher::set_timing(bool on) {
    if (on && !d_count_) {
        for (int i = 0; i < 16; i++) ORB_HIP_CHECK(hipEventCreate(&ev_[i]));
        ORB_HIP_CHECK(hipMalloc(&d_count_, sizeof(unsigned long long) * 8 * kCountSlots));
        ORB_HIP_CHECK(hipMemset(d_count_, 0, sizeof(unsigned long long) * 8 * kCountSlots));
    }
    timing_ = on;
    return 0;
}

void Matcher::mark(int i) {
    if (!timing_) return;
    (void)hipEventRecord(ev_[i], stream_);
    evSet_[i] = true;
}

int Matcher::zero_counters(int first, int n) {
    ORB_HIP_CHECK(hipMemsetAsync(d_count_ + (size_t)first * kCountSlots, 0, sizeof(unsigned long long) * n * kCountSlots,
                                 stream_));
    return 0;
}

// events: search 0..3 (grid | candidates | select), stereo 4..7 (rows | match | filter), CSR 12..13,
// isInFrustum 8..9
int Matcher::timings(float* ms8, long long* cnt8) {
    for (int i = 0; i < 8; i++) {
        ms8[i] = -1.0f;
        cnt8[i] = -1;
    }
    if (!d_count_) return 0;
    ORB_HIP_CHECK(stream_wait(stream_));
    const int pairs[8][2] = {{0, 1}, {1, 2}, {2, 3}, {4, 5}, {5, 6}, {6, 7}, {12, 13}, {8, 9}};
    for (int k = 0; k < 8; k++) {
        const int a = pairs[k][0], b = pairs[k][1];
        if (evSet_[a] && evSet_[b]) (void)hipEventElapsedTime(&ms8[k], ev_[a], ev_[b]);
    }
    std::vector<unsigned long long> c(8 * kCountSlots);
    ORB_HIP_CHECK(hipMemcpy(c.data(), d_count_, sizeof(unsigned long long) * c.size(), hipMemcpyDeviceToHost));
    for (int i = 0; i < 8; i++) {
        cnt8[i] = 0;
        for (int k = 0; k < kCountSlots; k++) cnt8[i] += (long long)c[(size_t)i * kCountSlots + k];
    }
    return 0;
}

int debug_prof_match(unsigned long long* out32) {
#ifdef ORBGPU_PROF
    ORB_HIP_CHECK(hipMemcpyFromSymbol(out32, HIP_SYMBOL(g_orbgpu_prof), sizeof(unsigned long long) * 32));
    unsigned long long z[32] = {};
    ORB_HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_orbgpu_prof), z, sizeof(z)));
    return 0;
#else
    (void)out32;
    return -1;
#endif
}

}  // namespace orbgpu
