// ba_struct_gpu.hip -- the BA structure of one optimisation level built on the device
// (see ba_struct_gpu.hpp).  Reference: g2o sparse_optimizer.cpp:198-287 (initializeOptimization:
// the active edges of a level, the vertices they touch; buildIndexMapping: vertices by id),
// block_solver.hpp:139-216 (buildStructure: per-vertex edge lists, the Schur pattern).
//
// The host restatement (ba_struct.cpp) defines every order; each list here is the same list:
//   aE            stream compaction of the level's edges (edge order)
//   poseKf/landPt stable radix sort of the active vertices by mnId
//   peList/leList stable sort of the active edges by pose / landmark (edge order inside)
//   lpList        sort by (landmark, pose): each landmark's free-pose edges in pose order; two
//                 equal keys = two edges between one (pose, landmark) pair (an error, as on host)
//   Schur terms   every (landmark, u <= v) pair of a landmark's lpList, numbered in the host's
//                 walk order (landmark, u, v); a stable sort by block key (i1, i2) groups each
//                 block's terms in landmark order; off-diagonal blocks are numbered by their first
//                 term (first use), after the nP diagonal blocks -- a scan of first-term flags.
#include "ba_struct_gpu.hpp"

#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>

#include "ba_struct.hpp"
#include "comm.hpp"
#include "orb_common.hpp"

namespace orbgpu {

namespace {
enum Slot {
    S_FLAG, S_AE, S_KFACT, S_PTACT, S_KFKEY, S_KFKEY2, S_KFIDX, S_POSEKF, S_PTKEY, S_PTKEY2, S_PTIDX, S_LANDPT,
    S_POSEIDX, S_LANDIDX, S_EPOSE, S_ELAND, S_KPE, S_KPE2, S_VA, S_PELIST, S_KLE, S_KLE2, S_LELIST, S_KLP, S_KLP2,
    S_LPLIST, S_PECNT, S_PESTART, S_LECNT, S_LESTART, S_LPCNT, S_LPSTART, S_TC, S_TSTART, S_BKEY, S_BKEY2, S_TIDX,
    S_TIDX2, S_TA, S_TB, S_FIRST, S_RANK, S_HEAD, S_SEG, S_BCNT, S_BSTART, S_BLKI, S_BLKJ, S_BOF, S_PA, S_PB, S_SC,
    S_ACTD, S_OFFKEY, S_TEMP, S_COUNT
};
static_assert(S_COUNT <= 64, "slots");

// scalar block (device, mirrored to pinned host memory)
enum Sc { C_NE, C_NP, C_NL, C_NPAIR, C_NLP, C_NPE, C_NLE, C_ERR, C_MAXPE, C_MAXLE, C_MAXBLK, C_NOFF, C_NEG, C_NLG, C_N };

constexpr int kT = 256;
inline unsigned nb(long long n) { return (unsigned)std::max<long long>(1, (n + kT - 1) / kT); }

// Counters and maxima over many threads into one word: one atomic per wave (a wave-wide max / sum
// first), not one per thread -- thousands of same-address atomics serialise at the L2.
__device__ __forceinline__ int wave_max_i(int v) {
    for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o));
    return v;
}

__global__ void k_gs_active(int ne, const EdgeDev* __restrict__ E, const uint8_t* __restrict__ lv, int level,
                            int* flag, int* kfAct, int* ptAct) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= ne) return;
    const bool a = lv[i] == level;
    flag[i] = a ? 1 : 0;
    if (a) {
        kfAct[E[i].kf] = 1;
        ptAct[E[i].pt] = 1;
    }
}

__global__ void k_gs_act_to_d(int n, const int* a, double* d) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) d[i] = (double)a[i];
}
__global__ void k_gs_d_to_act(int n, const double* d, int* a) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) a[i] = d[i] > 0 ? 1 : 0;
}

// vertex sort keys: active (and free, for poses) first, then by id (signed -> order-preserving
// unsigned); the active count into sc[slot]
__global__ void k_gs_vkeys(int n, const int* act, const uint8_t* fixed, const int32_t* id, unsigned long long* key,
                           int* idx, int* sc, int slot) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    const bool a = k < n && act[k] && !(fixed && fixed[k]);
    if (k < n) {
        key[k] = (a ? 0ull : (1ull << 32)) | (unsigned long long)((uint32_t)id[k] ^ 0x80000000u);
        idx[k] = k;
    }
    const int c = __popcll(__ballot(a));
    if ((threadIdx.x & 63) == 0 && c) atomicAdd(sc + slot, c);
}

__global__ void k_gs_index(int n, const int* __restrict__ sc, int slot, const int* __restrict__ sorted, int* map) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n && i < sc[slot]) map[sorted[i]] = i;
}

__global__ void k_gs_edges(int ne, const int* __restrict__ sc, const int* __restrict__ aE, const EdgeDev* __restrict__ E,
                           const int* __restrict__ poseIdx, const int* __restrict__ landIdx, int nkf, int* ePose,
                           int* eLand, uint32_t* kPe, uint32_t* kLe, unsigned long long* kLp, int* vA) {
    const int a = blockIdx.x * blockDim.x + threadIdx.x;
    if (a >= ne) return;
    vA[a] = a;
    if (a < sc[C_NE]) {
        const int e = aE[a], p = poseIdx[E[e].kf], l = landIdx[E[e].pt];
        ePose[a] = p;
        eLand[a] = l;
        kPe[a] = p >= 0 ? (uint32_t)p : 0xffffffffu;
        kLe[a] = (uint32_t)l;
        kLp[a] = p >= 0 ? (unsigned long long)l * (unsigned long long)nkf + (unsigned long long)p : ~0ull;
    } else {
        kPe[a] = 0xffffffffu;
        kLe[a] = 0xffffffffu;
        kLp[a] = ~0ull;
    }
}

// first position of a key >= v in a sorted key array (the lists' segment starts)
template <class K>
__device__ __forceinline__ int lower_bound_k(const K* __restrict__ k, int n, K v) {
    int lo = 0, hi = n;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (k[mid] < v) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}
// The per-pose / per-landmark segment starts and counts of the three sorted edge lists: the start
// of pose p is the number of sorted keys below p (invalid keys sort last), so the starts equal the
// exclusive sums of the per-vertex counts -- without a same-address atomic per edge (1.5 M of them
// onto 2,000 pose counters serialised at the L2: 0.3 ms per config-5 build).
__global__ void k_gs_starts(int ne, int nkf, int npt, const uint32_t* __restrict__ kPe2, const uint32_t* __restrict__ kLe2,
                            const unsigned long long* __restrict__ kLp2, int* peStart, int* peCnt, int* leStart,
                            int* leCnt, int* lpStart, int* lpCnt) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i <= nkf) {
        const int a = lower_bound_k(kPe2, ne, (uint32_t)i);
        peStart[i] = a;
        peCnt[i] = i < nkf ? lower_bound_k(kPe2, ne, (uint32_t)(i + 1)) - a : 0;
    }
    if (i <= npt) {
        const int a = lower_bound_k(kLe2, ne, (uint32_t)i);
        leStart[i] = a;
        leCnt[i] = i < npt ? lower_bound_k(kLe2, ne, (uint32_t)(i + 1)) - a : 0;
        const unsigned long long nk = (unsigned long long)nkf;
        const int b = lower_bound_k(kLp2, ne, (unsigned long long)i * nk);
        lpStart[i] = b;
        lpCnt[i] = i < npt ? lower_bound_k(kLp2, ne, (unsigned long long)(i + 1) * nk) - b : 0;
    }
}

// the per-landmark Schur term counts m (m + 1) / 2 and the list maxima
__global__ void k_gs_counts(int npt, int nkf, const int* __restrict__ sc_in, const int* __restrict__ peCnt,
                            const int* __restrict__ leCnt, const int* __restrict__ lpCnt, long long* tc, int* sc) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const int nP = sc_in[C_NP], nL = sc_in[C_NL];
    if (i <= npt) {
        const long long m = i < nL ? lpCnt[i] : 0;
        tc[i] = m * (m + 1) / 2;
    }
    const int le = wave_max_i(i < nL ? leCnt[i] : 0);
    const int pe = wave_max_i(i < nP && i < nkf ? peCnt[i] : 0);
    if ((threadIdx.x & 63) == 0) {
        if (le) atomicMax(sc + C_MAXLE, le);
        if (pe) atomicMax(sc + C_MAXPE, pe);
    }
}

// one (pose, landmark) pair per edge: adjacent equal (landmark, pose) keys are an error
__global__ void k_gs_dup(int ne, const int* __restrict__ sc_in, const unsigned long long* __restrict__ k, int* sc) {
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= 1 && q < ne && k[q] != ~0ull && k[q] == k[q - 1]) atomicOr(sc + C_ERR, 1);
}

__global__ void k_gs_scalars(const int* peStart, const int* leStart, const int* lpStart, const long long* tStart,
                             int* sc) {
    const int nP = sc[C_NP], nL = sc[C_NL];
    sc[C_NPE] = peStart[nP];
    sc[C_NLE] = leStart[nL];
    sc[C_NLP] = lpStart[nL];
    // the Schur-term count must fit the int the buffers are sized from: flag it
    // and report capacity instead of writing past them at 64-bit tStart offsets
    if (tStart[nL] > 0x7fffffffLL) atomicOr(sc + C_ERR, 2);
    sc[C_NPAIR] = tStart[nL] > 0x7fffffffLL ? 0 : (int)tStart[nL];
}

// every Schur term (u <= v over the landmark's lpList), numbered in the host walk's order
// One thread per Schur term t (coalesced stores): its landmark l is the last with tStart[l] <= t,
// then (u, v) the (t - tStart[l])-th pair u <= v of the landmark's lpList in the host's walk order
__global__ void k_gs_terms(int npt, int nkf, const int* __restrict__ sc, const int* __restrict__ lpStart,
                           const int* __restrict__ lpList, const unsigned long long* __restrict__ kLp,
                           const long long* __restrict__ tStart, unsigned long long* bkey, int* tidx, int* tA, int* tB) {
    const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const int nL = min(npt, sc[C_NL]);
    if (t >= tStart[nL]) return;
    int lo = 0, hi = nL;   // the last l in [0, nL) with tStart[l] <= t
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (tStart[mid] <= t) lo = mid;
        else hi = mid;
    }
    const int l = lo;
    const int b0 = lpStart[l], m = lpStart[l + 1] - b0;
    long long r = t - tStart[l];
    int u = 0;
    while (r >= m - u) {
        r -= m - u;
        u++;
    }
    const int v = u + (int)r;
    const unsigned long long pu = kLp[b0 + u] % (unsigned long long)nkf;
    const unsigned long long pv = kLp[b0 + v] % (unsigned long long)nkf;
    bkey[t] = pu * (unsigned long long)nkf + pv;
    tidx[t] = (int)t;
    tA[t] = lpList[b0 + u];
    tB[t] = lpList[b0 + v];
}

__global__ void k_gs_heads(int nPair, int nkf, const unsigned long long* __restrict__ k, const int* __restrict__ st,
                           int* first, int* headPos, int* offFlag) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nPair) return;
    const bool head = i == 0 || k[i] != k[i - 1];
    const bool off = (k[i] / (unsigned long long)nkf) != (k[i] % (unsigned long long)nkf);
    if (head && off) first[st[i]] = 1;
    headPos[i] = head ? i : 0;
    offFlag[i] = head && off ? 1 : 0;
}

__global__ void k_gs_diag(int nP, int* blkI, int* blkJ) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p < nP) {
        blkI[p] = p;
        blkJ[p] = p;
    }
}

__global__ void k_gs_blocks(int nPair, int nkf, int nP, const unsigned long long* __restrict__ k,
                            const int* __restrict__ st, const int* __restrict__ seg, const int* __restrict__ rank,
                            int* bOf, int* bCnt, int* blkI, int* blkJ) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nPair) return;
    const int s0 = seg[i];
    const int pu = (int)(k[i] / (unsigned long long)nkf), pv = (int)(k[i] % (unsigned long long)nkf);
    const int b = pu == pv ? pu : nP + rank[st[s0]];
    bOf[i] = b;
    // a block's terms are one segment of the sorted keys: its last term stores the count
    if (i + 1 == nPair || k[i + 1] != k[i]) bCnt[b] = i - s0 + 1;
    if (i == s0) {
        blkI[b] = pu;
        blkJ[b] = pv;
    }
}

__global__ void k_gs_fill(int nPair, const int* __restrict__ st, const int* __restrict__ seg,
                          const int* __restrict__ bOf, const int* __restrict__ bStart, const int* __restrict__ tA,
                          const int* __restrict__ tB, int* pA, int* pB) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nPair) return;
    const int q = bStart[bOf[i]] + (i - seg[i]);
    pA[q] = tA[st[i]];
    pB[q] = tB[st[i]];
}

__global__ void k_gs_blkmax(int nBlk, const int* __restrict__ bCnt, int* sc) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    const int m = wave_max_i(b < nBlk ? bCnt[b] : 0);
    if ((threadIdx.x & 63) == 0 && m) atomicMax(sc + C_MAXBLK, m);
}

__global__ void k_gs_offkey(int nOffMax, const int* __restrict__ sc, const unsigned long long* __restrict__ k, int nkf,
                            int nP, long long* out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nOffMax || i >= sc[C_NOFF]) return;
    out[i] = (long long)(k[i] / (unsigned long long)nkf) * nP + (long long)(k[i] % (unsigned long long)nkf);
}

__global__ void k_gs_glob_in(const int* sc, double* d) {
    d[0] = (double)sc[C_NE];
    d[1] = (double)sc[C_NL];
}
__global__ void k_gs_glob_out(const double* d, int* sc) {
    sc[C_NEG] = (int)d[0];
    sc[C_NLG] = (int)d[1];
}

struct Max {
    __device__ __forceinline__ int operator()(int a, int b) const { return a > b ? a : b; }
};

// ---------------------------------------------------------------- one workgroup, small problems
// A local BA (SURVEY config 4: 30 keyframes, 3,000 points, 15 k edges) is too small for the
// multi-launch builder above: its ~40 launches and two readbacks cost more than the host's
// counting sorts.  k_gs_small builds the same sixteen lists in ONE 1024-thread workgroup.  Global
// memory is read once at the start (each thread a contiguous chunk of edges, its loads independent)
// and written as results; every intermediate list lives in LDS (16-bit positions), because a
// chain of dependent global loads per thread costs ~0.5-1 us a link in a single workgroup (the
// first version, which kept the lists in global memory, took 330-380 us per level).  The counts
// reach the host through pinned memory (one poll, no copy).  Every list is the host's
// (ba_struct.cpp) by construction:
//   aE            per-thread chunks compacted with one workgroup scan: edge order
//   poseKf        the free active keyframes ranked by (mnId, index) -- at most kSmMaxP of them
//   landPt        the active points compacted in the host's (mnId, index) order of all points
//   le/lp counts  one packed counter per landmark (edges low, free-pose edges high), one scan
//   leList        LDS cursors, then each landmark's (short) segment sorted by edge position
//   lpList        a landmark's free-pose edges placed by the rank of their pose in the landmark's
//                 pose bitmask: pose order without a sort; a pose seen twice = duplicate edge
//   peList        per wave a contiguous range of active edges (counted per pose in the edge
//                 pass), split by pose with ballots (stable: edge order inside a pose), bases
//                 scanned pose-major over the waves
//   Schur blocks  a landmark's terms are the pose pairs (i <= j) of its bitmask; an off-diagonal
//                 block's first use is its first landmark, then (i, j) -- the host walk's order
//                 (landmark, u, v) because a landmark's lp entries are in pose order; each block's
//                 terms placed in landmark order by the same wave-range ballot split
// Anything outside the limits (more free poses, a longer landmark segment) is reported as
// "fallback" and the multi-launch builder runs instead.  Inputs: the compact per-edge keys
// (keyframe << 13 | point) and the points' (mnId, index) order, both written at upload.
constexpr int kSmT = 1024, kSmW = kSmT / 64;
constexpr int kSmMaxPt = 8192, kSmMaxKf = 1024, kSmMaxE = 16384;
constexpr int kSmPer = kSmMaxE / kSmT;                       // edges per thread
constexpr int kSmPtPer = kSmMaxPt / kSmT;                    // points per thread
constexpr int kSmSteps = kSmMaxPt / kSmW / 64;               // 64-landmark steps per wave
constexpr int kSmMaxP = 23;                                  // free poses (the dense solvers' range)
constexpr int kSmTri = (kSmMaxP + 1) * (kSmMaxP + 2) / 2;    // pose pairs i <= j: j (j + 1) / 2 + i
constexpr int kSmMaxLe = 256;
// the LDS pool, by phase (bytes)
constexpr int kOffA = 0;                              // ePose8[e]                 | Schur: per-wave pair counters (A+B)
constexpr int kOffB = kOffA + kSmMaxE;                // leStart16[l]
constexpr int kOffC = kOffB + 2 * (kSmMaxPt + 32);    // free keyframes (poses) -> lpList16[q]
constexpr int kOffD = kOffC + 2 * kSmMaxE;            // packed counts int[l] -> leList16[j] -> pePos16[a] -> Schur ballots
constexpr int kOffE = kOffD + 4 * (kSmMaxPt + 16);    // point flags (P1-P2) -> lpStart16[l]
constexpr int kOffF = kOffE + 2 * (kSmMaxPt + 32);    // landIdx16[p] -> le cursors int[l] -> mask32[l]
constexpr int kPool = kOffF + 4 * (kSmMaxPt + 16);
static_assert(4 * kSmW * kSmTri <= kOffC, "the pair counters overlap A+B only");
static_assert(8 * kSmW * (kSmMaxPt / kSmW / 64) * 23 <= kOffE - kOffD, "the Schur step ballots fit D");
static_assert(4 * kSmMaxKf <= 2 * kSmMaxE, "the free keyframes fit C");
enum SmSc { SM_NE, SM_NP, SM_NL, SM_NBLK, SM_NPAIR, SM_NPE, SM_NLP, SM_MAXPE, SM_MAXLE, SM_MAXBLK, SM_ERR, SM_FALLBACK,
            SM_SEQ, SM_N };

struct SmallArgs {
    int level, nkf, npt, ne, seq;
    const int32_t* kp;        // per edge (keyframe << 13) | point (k_unpack_upload)
    const int32_t* ptOrd;     // the points by (mnId, index) (host, once per call)
    const uint8_t* lv;        // null: every edge at `level` (the first build of a call)
    const uint8_t* kfFixed;
    const int32_t* kfId;
    int *aE, *ePose, *eLand, *poseKf, *landPt, *peStart, *peList, *leStart, *leList, *lpStart, *lpList, *blkI, *blkJ,
        *blkStart, *pairA, *pairB;
    int* pePos;           // null: pairs hold active-edge positions; else pePos and pairs as pose-list positions
    int* sc;              // device copy of the counts
    volatile int* hSc;    // pinned coherent: the counts, then the sequence word
    volatile long long* ts;   // ORBGPU_BA_TIMES: phase timestamps (wall clock, 100 MHz) or null
};

__device__ __forceinline__ unsigned long long lanes_below() {
    return (1ull << (threadIdx.x & 63)) - 1ull;
}
__device__ __forceinline__ int wave_incl_scan(int v) {
    const int lane = threadIdx.x & 63;
    for (int o = 1; o < 64; o <<= 1) {
        const int t = __shfl_up(v, o);
        if (lane >= o) v += t;
    }
    return v;
}
// exclusive prefix of v over the workgroup, *tot the sum (ws: 32 ints of LDS)
__device__ __forceinline__ int block_excl(int v, int* ws, int* tot) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int inc = wave_incl_scan(v);
    if (lane == 63) ws[w] = inc;
    __syncthreads();
    if (w == 0) {
        const int t = lane < kSmW ? ws[lane] : 0;
        const int it = wave_incl_scan(t);
        if (lane < kSmW) ws[kSmW + lane] = it;
    }
    __syncthreads();
    const int base = w ? ws[kSmW + w - 1] : 0;
    *tot = ws[2 * kSmW - 1];
    __syncthreads();
    return base + inc - v;
}
__device__ __forceinline__ int block_max(int v, int* ws) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o));
    if (lane == 0) ws[w] = v;
    __syncthreads();
    int m = 0;
    for (int k = 0; k < kSmW; k++) m = max(m, ws[k]);
    __syncthreads();
    return m;
}
// in-place exclusive scan of a[0, n) in LDS (contiguous chunks per thread); returns the total
__device__ int block_scan_inplace(int* a, int n, int* ws) {
    const int per = (n + kSmT - 1) / kSmT;
    const int c0 = min(n, (int)threadIdx.x * per), c1 = min(n, c0 + per);
    int s = 0;
    for (int i = c0; i < c1; i++) s += a[i];
    int tot;
    int base = block_excl(s, ws, &tot);
    for (int i = c0; i < c1; i++) {
        const int v = a[i];
        a[i] = base;
        base += v;
    }
    __syncthreads();
    return tot;
}
// the lanes whose `key` equals this lane's (valid lanes only; keys below 2^bits)
__device__ __forceinline__ unsigned long long same_key(int key, bool valid, int bits) {
    unsigned long long m = __ballot(valid);
    for (int b = 0; b < bits; b++) {
        const bool on = (key >> b) & 1;
        const unsigned long long t = __ballot(valid && on);
        m &= on ? t : ~t;
    }
    return m;
}

__global__ void __launch_bounds__(kSmT) k_gs_small(SmallArgs A) {
    __shared__ __attribute__((aligned(16))) unsigned char pool[kPool];
    __shared__ uint8_t sKfAct[kSmMaxKf];
    __shared__ int8_t sPoseIdx[kSmMaxKf];
    __shared__ int sPe[kSmW * kSmMaxP];
    __shared__ int sFirst[kSmTri], sTot[kSmTri], sBlk[kSmTri], sBcnt[kSmTri + 1];
    __shared__ int sFreeId[kSmMaxP + 1];
    __shared__ int sWs[2 * kSmW];
    int8_t* const ePose8 = reinterpret_cast<int8_t*>(pool + kOffA);
    uint16_t* const leStart16 = reinterpret_cast<uint16_t*>(pool + kOffB);
    int* const sFree = reinterpret_cast<int*>(pool + kOffC);
    uint16_t* const lpList16 = reinterpret_cast<uint16_t*>(pool + kOffC);
    int* const cnt = reinterpret_cast<int*>(pool + kOffD);
    uint16_t* const leList16 = reinterpret_cast<uint16_t*>(pool + kOffD);
    uint16_t* const pePos16 = reinterpret_cast<uint16_t*>(pool + kOffD);
    uint8_t* const ptAct = pool + kOffE;
    uint16_t* const lpStart16 = reinterpret_cast<uint16_t*>(pool + kOffE);
    uint16_t* const landIdx16 = reinterpret_cast<uint16_t*>(pool + kOffF);
    int* const cur = reinterpret_cast<int*>(pool + kOffF);
    uint32_t* const mask = reinterpret_cast<uint32_t*>(pool + kOffF);
    int* const sBc = reinterpret_cast<int*>(pool);   // per wave, per pose pair: term count, then next slot

    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int ne = A.ne, nkf = A.nkf, npt = A.npt;
#define SM_TS(k) \
    if (A.ts && tid == 0) A.ts[k] = (long long)wall_clock64()
    SM_TS(0);
    int nE = 0, nP = 0, nL = 0, nBlk = 0, nPair = 0, nPe = 0, nLp = 0, maxPe = 0, maxLe = 0, maxBlk = 0, err = 0,
        fallback = 0, pw = 1;

    for (int i = tid; i < npt; i += kSmT) ptAct[i] = 0;
    for (int i = tid; i < nkf; i += kSmT) {
        sKfAct[i] = 0;
        sPoseIdx[i] = -1;
    }
    for (int i = tid; i <= npt; i += kSmT) cnt[i] = 0;
    for (int i = tid; i < kSmW * kSmMaxP; i += kSmT) sPe[i] = 0;
    // 1. initializeOptimization(level): this thread's chunk of kSmPer edges [c0, c1) as four
    // 16-byte key loads and one 16-byte level load (the compact per-edge keys, not the records)
    const int c0 = min(ne, tid * kSmPer), c1 = min(ne, c0 + kSmPer);
    int kp[kSmPer];        // active: (keyframe << 13) | point; later (landmark << 5) | (pose + 1)
    uint32_t act = 0;
    if (c1 - c0 == kSmPer) {
        const int4* k4 = reinterpret_cast<const int4*>(A.kp + c0);
        const uint4 l4 = A.lv ? *reinterpret_cast<const uint4*>(A.lv + c0) : make_uint4(0, 0, 0, 0);
        const uint32_t lw[4] = {l4.x, l4.y, l4.z, l4.w};
#pragma unroll
        for (int v = 0; v < 4; v++) {
            const int4 q = k4[v];
            kp[4 * v] = q.x;
            kp[4 * v + 1] = q.y;
            kp[4 * v + 2] = q.z;
            kp[4 * v + 3] = q.w;
        }
#pragma unroll
        for (int k = 0; k < kSmPer; k++) act |= ((lw[k >> 2] >> (8 * (k & 3))) & 0xffu) == (uint32_t)A.level ? 1u << k : 0u;
    } else if (c0 < c1) {
#pragma unroll
        for (int k = 0; k < kSmPer; k++) {
            const int i = min(c0 + k, c1 - 1);
            kp[k] = A.kp[i];
            act |= (c0 + k < c1 && (A.lv ? A.lv[i] : 0) == A.level) ? 1u << k : 0u;
        }
    }
    __syncthreads();   // (the flags are cleared)
#pragma unroll
    for (int k = 0; k < kSmPer; k++)
        if ((act >> k) & 1u) {
            ptAct[kp[k] & 8191] = 1;
            sKfAct[kp[k] >> 13] = 1;
        }
    int aBase;   // this thread's first active-edge position
    {
        int tot;
        aBase = block_excl(__popc(act), sWs, &tot);
        nE = tot;
        int q = aBase;
#pragma unroll
        for (int k = 0; k < kSmPer; k++)
            if ((act >> k) & 1u) A.aE[q++] = c0 + k;
    }
    SM_TS(1);
    // 2. buildIndexMapping: the free active keyframes by (mnId, index)
    for (int b = 0; b < nkf; b += kSmT) {
        const int k = b + tid;
        const bool f = k < nkf && sKfAct[k] && !A.kfFixed[k];
        int tot;
        const int pos = block_excl(f ? 1 : 0, sWs, &tot);
        if (f) sFree[nP + pos] = k;
        nP += tot;
    }
    __syncthreads();
    if (nP > kSmMaxP) {
        fallback = 1;
        goto done;
    }
    if (tid < nP) sFreeId[tid] = A.kfId[sFree[tid]];
    __syncthreads();
    if (tid < nP) {
        const int k = sFree[tid];
        const int32_t id = sFreeId[tid];
        int r = 0;
        for (int q = 0; q < nP; q++) {
            const int32_t id2 = sFreeId[q];
            r += (id2 < id || (id2 == id && sFree[q] < k)) ? 1 : 0;
        }
        A.poseKf[r] = k;
        sPoseIdx[k] = (int8_t)r;
    }
    SM_TS(2);
    {   // the active points in (mnId, index) order: the host's order of all points, compacted
        const int r0 = min(npt, tid * kSmPtPer), r1 = min(npt, r0 + kSmPtPer);
        int pp[kSmPtPer];
        uint32_t pa = 0;
#pragma unroll
        for (int k = 0; k < kSmPtPer; k++) {
            const int r = r0 + k;
            pp[k] = r < r1 ? A.ptOrd[r] : 0;
        }
#pragma unroll
        for (int k = 0; k < kSmPtPer; k++) pa |= (r0 + k < r1 && ptAct[pp[k]]) ? 1u << k : 0u;
        int tot;
        int q = block_excl(__popc(pa), sWs, &tot);
        nL = tot;
#pragma unroll
        for (int k = 0; k < kSmPtPer; k++)
            if ((pa >> k) & 1u) {
                A.landPt[q] = pp[k];
                landIdx16[pp[k]] = (uint16_t)q;
                q++;
            }
    }
    __syncthreads();
    SM_TS(3);
    SM_TS(4);
    // 3. per active edge: its pose / landmark index; per landmark one packed counter
    pw = max(1, (nE + kSmW - 1) / kSmW);   // the pose lists' per-wave ranges of active edges
    {
        int q = aBase;
#pragma unroll
        for (int k = 0; k < kSmPer; k++)
            if ((act >> k) & 1u) {
                const int p = sPoseIdx[kp[k] >> 13], l = landIdx16[kp[k] & 8191];
                ePose8[q] = (int8_t)p;
                A.ePose[q] = p;
                A.eLand[q] = l;
                atomicAdd(&cnt[l], p >= 0 ? 0x10001 : 1);
                if (p >= 0) atomicAdd(&sPe[(q / pw) * kSmMaxP + p], 1);   // (order-free counts)
                kp[k] = (l << 5) | (p + 1);
                q++;
            }
    }
    __syncthreads();
    {
        int m = 0;
        for (int i = tid; i < nL; i += kSmT) m = max(m, cnt[i] & 0xffff);
        maxLe = block_max(m, sWs);
        if (maxLe > kSmMaxLe) {
            fallback = 1;
            goto done;
        }
        // both scans at once: the low halves sum to nE < 2^16, so nothing carries into the high ones
        const int tot = block_scan_inplace(cnt, nL + 1, sWs);
        nLp = tot >> 16;
        for (int i = tid; i <= nL; i += kSmT) {
            const int v = cnt[i], le = v & 0xffff, lp = v >> 16;
            leStart16[i] = (uint16_t)le;
            lpStart16[i] = (uint16_t)lp;
            cur[i] = le;
            A.leStart[i] = le;
            A.lpStart[i] = lp;
        }
    }
    __syncthreads();
    SM_TS(5);
    {   // each landmark's edges through the cursors (then sorted per landmark below)
        int q = aBase;
#pragma unroll
        for (int k = 0; k < kSmPer; k++)
            if ((act >> k) & 1u) leList16[atomicAdd(&cur[kp[k] >> 5], 1)] = (uint16_t)q++;
    }
    __syncthreads();
    {
        int dup = 0;
        for (int l = tid; l < nL; l += kSmT) {
            const int s0 = leStart16[l], s1 = leStart16[l + 1];
            for (int j = s0 + 1; j < s1; j++) {
                const uint16_t v = leList16[j];
                int k = j - 1;
                while (k >= s0 && leList16[k] > v) {
                    leList16[k + 1] = leList16[k];
                    k--;
                }
                leList16[k + 1] = v;
            }
            // the free-pose edges in pose order: an edge's slot is its pose's rank in the bitmask
            uint32_t M = 0;
            for (int j = s0; j < s1; j++) {
                const int a = leList16[j], p = ePose8[a];
                A.leList[j] = a;
                if (p < 0) continue;
                dup |= (M >> p) & 1u;
                M |= 1u << p;
            }
            const int q0 = lpStart16[l];
            for (int j = s0; j < s1; j++) {
                const int a = leList16[j], p = ePose8[a];
                if (p >= 0) {
                    const int q = q0 + __popc(M & ((1u << p) - 1u));
                    lpList16[q] = (uint16_t)a;
                    A.lpList[q] = a;
                }
            }
            mask[l] = M;
        }
        if (__syncthreads_or(dup)) {
            err = 1;
            goto done;
        }
    }
    SM_TS(6);
    {   // 4. the pose lists: per wave a contiguous range of active edges, split by pose
        // (the per-wave, per-pose counts came from the edge pass)
        const int e0 = min(nE, wv * pw), e1 = min(nE, e0 + pw);
        volatile int* const pe = sPe + wv * kSmMaxP;
        if (wv == 0) {   // per pose: its total, its start, the waves' bases in wave order
            int t = 0;
            if (lane < nP)
                for (int w = 0; w < kSmW; w++) t += sPe[w * kSmMaxP + lane];
            const int inc = wave_incl_scan(t);
            if (lane < nP) {
                int run = inc - t;
                A.peStart[lane] = run;
                for (int w = 0; w < kSmW; w++) {
                    const int c = sPe[w * kSmMaxP + lane];
                    sPe[w * kSmMaxP + lane] = run;
                    run += c;
                }
            }
            int mx = t;
            for (int o = 32; o > 0; o >>= 1) mx = max(mx, __shfl_xor(mx, o));
            const int tot = __shfl(inc, 63);
            if (lane == 0) {
                sWs[0] = mx;
                sWs[1] = tot;
                A.peStart[nP] = tot;
            }
        }
        __syncthreads();
        maxPe = sWs[0];
        nPe = sWs[1];
        for (int b = e0; b < e1; b += 64) {
            const int a = b + lane;
            const int p = a < e1 ? ePose8[a] : -1;
            const unsigned long long m = same_key(p, p >= 0, 5);
            if (p >= 0) {
                const int pos = pe[p] + __popcll(m & lanes_below());
                A.peList[pos] = a;
                pePos16[a] = (uint16_t)pos;
                if (A.pePos) A.pePos[a] = pos;
                if ((m & lanes_below()) == 0) pe[p] += __popcll(m);
            } else if (a < e1) {
                pePos16[a] = 0xffff;
                if (A.pePos) A.pePos[a] = -1;
            }
        }
        __syncthreads();
    }
    SM_TS(7);
    if (A.pePos) {   // the pairs are written as pose-list positions: map the lp entries once
        for (int q = tid; q < nLp; q += kSmT) lpList16[q] = pePos16[lpList16[q]];
        __syncthreads();
    }
    {   // 5. buildStructure's Schur pattern over the pose pairs s = j (j + 1) / 2 + i, i <= j.
        // Each wave owns a contiguous range of landmarks in up to kSmSteps steps of 64 (lane =
        // landmark, its pose bitmask in a register).  Per step and pose one ballot ("which lanes
        // see pose p") goes to LDS; a pair's count, first use and every term's slot follow from
        // ANDs and popcounts of two of them.  Each lane places only its own landmark's terms.
        const int nTri = nP * (nP + 1) / 2;
        unsigned long long* const Bt = reinterpret_cast<unsigned long long*>(pool + kOffD) + wv * kSmSteps * kSmMaxP;
        for (int s = tid; s < kSmTri; s += kSmT) sFirst[s] = 0x7fffffff;
        for (int s = tid; s <= kSmTri; s += kSmT) sBcnt[s] = 0;
        const int pl = (nL + kSmW - 1) / kSmW, l0 = min(nL, wv * pl), l1 = min(nL, l0 + pl);
        const int nst = (l1 - l0 + 63) / 64;
        uint32_t Ms[kSmSteps];
        int Q0[kSmSteps];
#pragma unroll
        for (int st = 0; st < kSmSteps; st++) {
            const int l = l0 + st * 64 + lane;
            const bool ok = st < nst && l < l1;
            Ms[st] = ok ? mask[l] : 0u;
            Q0[st] = ok ? lpStart16[l] : 0;
            if (st < nst)
                for (int p = 0; p < nP; p++) {
                    const unsigned long long m = __ballot((Ms[st] >> p) & 1u);
                    if (lane == 0) Bt[st * kSmMaxP + p] = m;
                }
        }
        __syncthreads();   // (the first-use keys are reset; the ballots are published)
        // per pair (lane-strided): the wave's term count and its first landmark
        for (int s = lane; s < nTri; s += 64) {
            int j = 0;
            while ((j + 1) * (j + 2) / 2 <= s) j++;
            const int i = s - j * (j + 1) / 2;
            int c = 0, first = 0x7fffffff;
            for (int st = 0; st < nst; st++) {
                const unsigned long long x = Bt[st * kSmMaxP + i] & Bt[st * kSmMaxP + j];
                if (x && first == 0x7fffffff) first = l0 + st * 64 + (int)__builtin_ctzll(x);
                c += __popcll(x);
            }
            sBc[wv * kSmTri + s] = c;
            if (i != j && c) atomicMin(&sFirst[s], first);
        }
        __syncthreads();
        // per pair: its term count; a used off-diagonal pair's first use as one ordered key
        // (first landmark, i, j) -- sFirst < kSmMaxPt, so the key fits an int
        int nOffMine = 0;
        for (int s = tid; s < nTri; s += kSmT) {
            int j = 0;
            while ((j + 1) * (j + 2) / 2 <= s) j++;
            const int i = s - j * (j + 1) / 2;
            int t = 0;
            for (int w = 0; w < kSmW; w++) t += sBc[w * kSmTri + s];
            sTot[s] = t;
            const bool off = i != j && t > 0;
            sFirst[s] = off ? sFirst[s] * 1024 + i * 32 + j : 0x7fffffff;
            nOffMine += off ? 1 : 0;
        }
        {
            int tot;
            (void)block_excl(nOffMine, sWs, &tot);   // (its barriers publish sTot / sFirst)
            nBlk = nP + tot;
        }
        // block numbers: diagonal blocks 0..nP-1, then the used off-diagonal ones by first use
        for (int s = tid; s < nTri; s += kSmT) {
            int j = 0;
            while ((j + 1) * (j + 2) / 2 <= s) j++;
            const int i = s - j * (j + 1) / 2;
            const int key = sFirst[s];
            int num = -1;
            if (i == j) {
                num = i;
            } else if (key != 0x7fffffff) {
                int r = 0;
                for (int s2 = 0; s2 < nTri; s2++) r += sFirst[s2] < key ? 1 : 0;
                num = nP + r;
            }
            sBlk[s] = num;
            if (num >= 0) {
                sBcnt[num] = sTot[s];
                A.blkI[num] = i;
                A.blkJ[num] = j;
            }
        }
        __syncthreads();
        int mb = 0;
        for (int b = tid; b < nBlk; b += kSmT) mb = max(mb, sBcnt[b]);
        maxBlk = block_max(mb, sWs);
        nPair = block_scan_inplace(sBcnt, nBlk + 1, sWs);
        for (int b = tid; b <= nBlk; b += kSmT) A.blkStart[b] = sBcnt[b];
        for (int s = tid; s < nTri; s += kSmT)
            if (sBlk[s] >= 0) {
                int run = sBcnt[sBlk[s]];
                for (int w = 0; w < kSmW; w++) {
                    const int c = sBc[w * kSmTri + s];
                    sBc[w * kSmTri + s] = run;
                    run += c;
                }
            }
        __syncthreads();
        // the terms: a term's slot is its wave's base for the pair, plus the wave's earlier steps'
        // terms of the pair, plus the lanes below it in its step with the pair -- landmark order
#pragma unroll
        for (int st = 0; st < kSmSteps; st++) {
            if (st >= nst) break;
            const uint32_t M = Ms[st];
            const int q0 = Q0[st];
            const unsigned long long* const Bs = Bt + st * kSmMaxP;
            for (uint32_t mu = M; mu; mu &= mu - 1) {
                const int i = __builtin_ctz(mu);
                const int ai = lpList16[q0 + __popc(M & ((1u << i) - 1u))];
                const unsigned long long bi = Bs[i];
                for (uint32_t mv = mu; mv; mv &= mv - 1) {
                    const int j = __builtin_ctz(mv);
                    const int s = j * (j + 1) / 2 + i;
                    int pos = sBc[wv * kSmTri + s] + __popcll(bi & Bs[j] & lanes_below());
                    for (int st2 = 0; st2 < st; st2++) pos += __popcll(Bt[st2 * kSmMaxP + i] & Bt[st2 * kSmMaxP + j]);
                    A.pairA[pos] = ai;
                    A.pairB[pos] = lpList16[q0 + __popc(M & ((1u << j) - 1u))];
                }
            }
        }
    }
done:
    __syncthreads();
    SM_TS(8);
    if (tid == 0) {
        int v[SM_N];
        v[SM_NE] = nE;
        v[SM_NP] = nP;
        v[SM_NL] = nL;
        v[SM_NBLK] = nBlk;
        v[SM_NPAIR] = nPair;
        v[SM_NPE] = nPe;
        v[SM_NLP] = nLp;
        v[SM_MAXPE] = maxPe;
        v[SM_MAXLE] = maxLe;
        v[SM_MAXBLK] = maxBlk;
        v[SM_ERR] = err;
        v[SM_FALLBACK] = fallback;
        v[SM_SEQ] = A.seq;
        for (int k = 0; k < SM_SEQ; k++) {
            A.sc[k] = v[k];
            A.hSc[k] = v[k];
        }
        __threadfence_system();
        A.hSc[SM_SEQ] = A.seq;
    }
#undef SM_TS
}
}  // namespace

GpuStructBuilder::~GpuStructBuilder() {
    for (auto& p : p_)
        if (p) (void)hipFree(p);
    if (hSc_) (void)hipHostFree(hSc_);
    if (hSig_) (void)hipHostFree((void*)hSig_);
}

void* GpuStructBuilder::buf(int slot, size_t bytes) {
    bytes = std::max<size_t>(bytes, 256);
    if (bytes > cap_[slot]) {
        if (p_[slot]) (void)hipFree(p_[slot]);
        p_[slot] = nullptr;
        cap_[slot] = 0;
        if (hipMalloc(&p_[slot], bytes + bytes / 4) != hipSuccess) return nullptr;
        cap_[slot] = bytes + bytes / 4;
    }
    return p_[slot];
}

#define GS_CHECK(expr)                          \
    do {                                        \
        if ((expr) != hipSuccess) return -2;    \
    } while (0)
#define GS_PTR(T, name, slot, count)                          \
    T* name = (T*)buf(slot, sizeof(T) * (size_t)(count));    \
    if (!name) return -2

int GpuStructBuilder::build(int level, int nkf, int npt, int ne, const EdgeDev* dE, const uint8_t* dLevel,
                            const uint8_t* dKfFixed, const int32_t* dKfId, const int32_t* dPtId, Comm* comm,
                            hipStream_t s, BaStructDev* st, GpuStructInfo* info, std::vector<int32_t>* blkIJ) {
    if (!hSc_ && hipHostMalloc((void**)&hSc_, sizeof(int) * 64) != hipSuccess) return -2;
    const int nE0 = std::max(ne, 1);
    // hipcub: size query, then the call, on one grow-only temporary
    auto cub = [&](auto fn) -> int {
        size_t bytes = 0;
        GS_CHECK(fn(nullptr, bytes));
        void* t = buf(S_TEMP, bytes);
        if (!t) return -2;
        GS_CHECK(fn(t, bytes));
        return 0;
    };
    GS_PTR(int, sc, S_SC, 64);
    GS_PTR(int, flag, S_FLAG, nE0);
    GS_PTR(int, aE, S_AE, nE0);
    GS_PTR(int, kfAct, S_KFACT, nkf + 1);
    GS_PTR(int, ptAct, S_PTACT, npt + 1);
    GS_CHECK(hipMemsetAsync(sc, 0, sizeof(int) * 64, s));
    GS_CHECK(hipMemsetAsync(kfAct, 0, sizeof(int) * (nkf + 1), s));
    GS_CHECK(hipMemsetAsync(ptAct, 0, sizeof(int) * (npt + 1), s));
    // 1. initializeOptimization(level): the active edges, the vertices they touch
    if (ne) hipLaunchKernelGGL(k_gs_active, dim3(nb(ne)), dim3(kT), 0, s, ne, dE, dLevel, level, flag, kfAct, ptAct);
    if (int e = cub([&](void* t, size_t& b) {
            return hipcub::DeviceSelect::Flagged(t, b, hipcub::CountingInputIterator<int>(0), flag, aE, sc + C_NE, ne, s);
        }))
        return e;
    if (comm) {   // a keyframe is active if any shard has an active edge on it
        GS_PTR(double, actd, S_ACTD, nkf + 2);
        if (nkf) hipLaunchKernelGGL(k_gs_act_to_d, dim3(nb(nkf)), dim3(kT), 0, s, nkf, kfAct, actd);
        if (int e = comm->allreduce(actd, (size_t)nkf, RedOp::Sum, s)) return e;
        if (nkf) hipLaunchKernelGGL(k_gs_d_to_act, dim3(nb(nkf)), dim3(kT), 0, s, nkf, actd, kfAct);
    }
    // 2. buildIndexMapping: free active poses and active landmarks, ascending by id
    GS_PTR(unsigned long long, kfKey, S_KFKEY, nkf + 1);
    GS_PTR(unsigned long long, kfKey2, S_KFKEY2, nkf + 1);
    GS_PTR(int, kfIdx, S_KFIDX, nkf + 1);
    GS_PTR(int, poseKf, S_POSEKF, nkf + 1);
    GS_PTR(unsigned long long, ptKey, S_PTKEY, npt + 1);
    GS_PTR(unsigned long long, ptKey2, S_PTKEY2, npt + 1);
    GS_PTR(int, ptIdx, S_PTIDX, npt + 1);
    GS_PTR(int, landPt, S_LANDPT, npt + 1);
    GS_PTR(int, poseIdx, S_POSEIDX, nkf + 1);
    GS_PTR(int, landIdx, S_LANDIDX, npt + 1);
    if (nkf) {
        hipLaunchKernelGGL(k_gs_vkeys, dim3(nb(nkf)), dim3(kT), 0, s, nkf, kfAct, dKfFixed, dKfId, kfKey, kfIdx, sc, (int)C_NP);
        if (int e = cub([&](void* t, size_t& b) {
                return hipcub::DeviceRadixSort::SortPairs(t, b, kfKey, kfKey2, kfIdx, poseKf, nkf, 0, 33, s);
            }))
            return e;
    }
    if (npt) {
        hipLaunchKernelGGL(k_gs_vkeys, dim3(nb(npt)), dim3(kT), 0, s, npt, ptAct, (const uint8_t*)nullptr, dPtId, ptKey,
                           ptIdx, sc, (int)C_NL);
        if (int e = cub([&](void* t, size_t& b) {
                return hipcub::DeviceRadixSort::SortPairs(t, b, ptKey, ptKey2, ptIdx, landPt, npt, 0, 33, s);
            }))
            return e;
    }
    GS_CHECK(hipMemsetAsync(poseIdx, 0xff, sizeof(int) * (nkf + 1), s));
    GS_CHECK(hipMemsetAsync(landIdx, 0xff, sizeof(int) * (npt + 1), s));
    if (nkf) hipLaunchKernelGGL(k_gs_index, dim3(nb(nkf)), dim3(kT), 0, s, nkf, sc, (int)C_NP, poseKf, poseIdx);
    if (npt) hipLaunchKernelGGL(k_gs_index, dim3(nb(npt)), dim3(kT), 0, s, npt, sc, (int)C_NL, landPt, landIdx);
    // 3. per active edge: pose / landmark index; the three edge lists by stable sorts
    GS_PTR(int, ePose, S_EPOSE, nE0);
    GS_PTR(int, eLand, S_ELAND, nE0);
    GS_PTR(uint32_t, kPe, S_KPE, nE0);
    GS_PTR(uint32_t, kPe2, S_KPE2, nE0);
    GS_PTR(int, vA, S_VA, nE0);
    GS_PTR(int, peList, S_PELIST, nE0);
    GS_PTR(uint32_t, kLe, S_KLE, nE0);
    GS_PTR(uint32_t, kLe2, S_KLE2, nE0);
    GS_PTR(int, leList, S_LELIST, nE0);
    GS_PTR(unsigned long long, kLp, S_KLP, nE0);
    GS_PTR(unsigned long long, kLp2, S_KLP2, nE0);
    GS_PTR(int, lpList, S_LPLIST, nE0);
    GS_PTR(int, peCnt, S_PECNT, nkf + 1);
    GS_PTR(int, peStart, S_PESTART, nkf + 1);
    GS_PTR(int, leCnt, S_LECNT, npt + 1);
    GS_PTR(int, leStart, S_LESTART, npt + 1);
    GS_PTR(int, lpCnt, S_LPCNT, npt + 1);
    GS_PTR(int, lpStart, S_LPSTART, npt + 1);
    GS_PTR(long long, tc, S_TC, npt + 1);
    GS_PTR(long long, tStart, S_TSTART, npt + 1);
    if (ne) {
        hipLaunchKernelGGL(k_gs_edges, dim3(nb(ne)), dim3(kT), 0, s, ne, sc, aE, dE, poseIdx, landIdx, nkf, ePose, eLand,
                           kPe, kLe, kLp, vA);
        if (int e = cub([&](void* t, size_t& b) {
                return hipcub::DeviceRadixSort::SortPairs(t, b, kPe, kPe2, vA, peList, ne, 0, 32, s);
            }))
            return e;
        if (int e = cub([&](void* t, size_t& b) {
                return hipcub::DeviceRadixSort::SortPairs(t, b, kLe, kLe2, vA, leList, ne, 0, 32, s);
            }))
            return e;
        if (int e = cub([&](void* t, size_t& b) {
                return hipcub::DeviceRadixSort::SortPairs(t, b, kLp, kLp2, vA, lpList, ne, 0, 64, s);
            }))
            return e;
        hipLaunchKernelGGL(k_gs_dup, dim3(nb(ne)), dim3(kT), 0, s, ne, sc, kLp2, sc);
    }
    {   // segment starts and counts of the sorted lists (no edges: every start 0)
        const uint32_t* kPe2s = ne ? kPe2 : kPe;   // (unsorted, unused at ne = 0)
        const uint32_t* kLe2s = ne ? kLe2 : kLe;
        const unsigned long long* kLp2s = ne ? kLp2 : kLp;
        hipLaunchKernelGGL(k_gs_starts, dim3(nb((long long)std::max(nkf, npt) + 1)), dim3(kT), 0, s, ne, nkf, npt, kPe2s,
                           kLe2s, kLp2s, peStart, peCnt, leStart, leCnt, lpStart, lpCnt);
    }
    hipLaunchKernelGGL(k_gs_counts, dim3(nb((long long)std::max(nkf, npt) + 1)), dim3(kT), 0, s, npt, nkf, sc, peCnt,
                       leCnt, lpCnt, tc, sc);
    if (int e = cub([&](void* t, size_t& b) { return hipcub::DeviceScan::ExclusiveSum(t, b, tc, tStart, npt + 1, s); }))
        return e;
    hipLaunchKernelGGL(k_gs_scalars, dim3(1), dim3(1), 0, s, peStart, leStart, lpStart, tStart, sc);
    if (comm) {   // the global edge / landmark counts
        GS_PTR(double, gd, S_ACTD, std::max(nkf + 2, 2));
        hipLaunchKernelGGL(k_gs_glob_in, dim3(1), dim3(1), 0, s, sc, gd);
        if (int e = comm->allreduce(gd, 2, RedOp::Sum, s)) return e;
        hipLaunchKernelGGL(k_gs_glob_out, dim3(1), dim3(1), 0, s, gd, sc);
    }
    GS_CHECK(hipGetLastError());
    GS_CHECK(hipMemcpyAsync(hSc_, sc, sizeof(int) * C_N, hipMemcpyDeviceToHost, s));
    GS_CHECK(stream_wait(s));
    const int nE = hSc_[C_NE], nP = hSc_[C_NP], nL = hSc_[C_NL];
    const long long nPairL = hSc_[C_NPAIR];
    if (hSc_[C_ERR]) {
        info->err = hSc_[C_ERR];
        return (hSc_[C_ERR] & 2) ? -3 : -1;   // 2: more Schur terms than an int counts (capacity)
    }
    const int nPair = (int)nPairL;
    // 4. buildStructure's Schur pattern
    const int nPair0 = std::max(nPair, 1);
    GS_PTR(unsigned long long, bkey, S_BKEY, nPair0);
    GS_PTR(unsigned long long, bkey2, S_BKEY2, nPair0);
    GS_PTR(int, tidx, S_TIDX, nPair0);
    GS_PTR(int, tidx2, S_TIDX2, nPair0);
    GS_PTR(int, tA, S_TA, nPair0);
    GS_PTR(int, tB, S_TB, nPair0);
    GS_PTR(int, first, S_FIRST, nPair0 + 1);
    GS_PTR(int, rank, S_RANK, nPair0 + 1);
    GS_PTR(int, headPos, S_HEAD, nPair0);
    GS_PTR(int, seg, S_SEG, nPair0);
    GS_PTR(int, bCnt, S_BCNT, (size_t)nP + nPair0 + 1);
    GS_PTR(int, bStart, S_BSTART, (size_t)nP + nPair0 + 1);
    GS_PTR(int, blkI, S_BLKI, (size_t)nP + nPair0);
    GS_PTR(int, blkJ, S_BLKJ, (size_t)nP + nPair0);
    GS_PTR(int, bOf, S_BOF, nPair0);
    GS_PTR(int, pA, S_PA, nPair0);
    GS_PTR(int, pB, S_PB, nPair0);
    GS_PTR(int, offFlag, S_OFFKEY, nPair0);
    GS_CHECK(hipMemsetAsync(first, 0, sizeof(int) * (nPair0 + 1), s));
    GS_CHECK(hipMemsetAsync(bCnt, 0, sizeof(int) * ((size_t)nP + nPair0 + 1), s));
    if (nP) hipLaunchKernelGGL(k_gs_diag, dim3(nb(nP)), dim3(kT), 0, s, nP, blkI, blkJ);
    int nOff = 0;
    if (nPair > 0) {
        hipLaunchKernelGGL(k_gs_terms, dim3(nb(nPair)), dim3(kT), 0, s, npt, nkf, sc, lpStart, lpList, kLp2, tStart, bkey,
                           tidx, tA, tB);
        int endbit = 1;
        while (endbit < 64 && ((unsigned long long)nkf * (unsigned long long)nkf >> endbit) != 0) endbit++;
        if (int e = cub([&](void* t, size_t& b) {
                return hipcub::DeviceRadixSort::SortPairs(t, b, bkey, bkey2, tidx, tidx2, nPair, 0, endbit, s);
            }))
            return e;
        hipLaunchKernelGGL(k_gs_heads, dim3(nb(nPair)), dim3(kT), 0, s, nPair, nkf, bkey2, tidx2, first, headPos, offFlag);
        if (int e = cub([&](void* t, size_t& b) { return hipcub::DeviceScan::ExclusiveSum(t, b, first, rank, nPair + 1, s); }))
            return e;
        if (int e = cub([&](void* t, size_t& b) {
                return hipcub::DeviceScan::InclusiveScan(t, b, headPos, seg, Max(), nPair, s);
            }))
            return e;
        GS_CHECK(hipMemcpyAsync(sc + C_NOFF, rank + nPair, sizeof(int), hipMemcpyDeviceToDevice, s));
        hipLaunchKernelGGL(k_gs_blocks, dim3(nb(nPair)), dim3(kT), 0, s, nPair, nkf, nP, bkey2, tidx2, seg, rank, bOf,
                           bCnt, blkI, blkJ);
    }
    if (int e = cub([&](void* t, size_t& b) {
            return hipcub::DeviceScan::ExclusiveSum(t, b, bCnt, bStart, nP + nPair + 1, s);
        }))
        return e;
    if (nPair > 0) {
        hipLaunchKernelGGL(k_gs_fill, dim3(nb(nPair)), dim3(kT), 0, s, nPair, tidx2, seg, bOf, bStart, tA, tB, pA, pB);
        hipLaunchKernelGGL(k_gs_blkmax, dim3(nb((long long)nP + nPair)), dim3(kT), 0, s, nP + nPair, bCnt, sc);
    } else if (nP) {
        hipLaunchKernelGGL(k_gs_blkmax, dim3(nb(nP)), dim3(kT), 0, s, nP, bCnt, sc);
    }
    GS_CHECK(hipGetLastError());
    GS_CHECK(hipMemcpyAsync(hSc_ + C_MAXBLK, sc + C_MAXBLK, sizeof(int) * 2, hipMemcpyDeviceToHost, s));
    GS_CHECK(stream_wait(s));
    nOff = nPair > 0 ? hSc_[C_NOFF] : 0;
    const int nBlk = nP + nOff;
    info->nE = nE;
    info->nP = nP;
    info->nL = nL;
    info->nBlk = nBlk;
    info->nPair = nPair;
    info->nLp = hSc_[C_NLP];
    info->nPe = hSc_[C_NPE];
    info->nLe = hSc_[C_NLE];
    info->err = 0;
    info->maxPe = hSc_[C_MAXPE];
    info->maxLe = hSc_[C_MAXLE];
    info->maxBlk = hSc_[C_MAXBLK];
    info->nEglob = comm ? hSc_[C_NEG] : nE;
    info->nLglob = comm ? hSc_[C_NLG] : nL;
    info->posDone = 0;
    st->nE = nE;
    st->nP = nP;
    st->nL = nL;
    st->nBlk = nBlk;
    st->aE = aE;
    st->ePose = ePose;
    st->eLand = eLand;
    st->poseKf = poseKf;
    st->landPt = landPt;
    st->peStart = peStart;
    st->peList = peList;
    st->leStart = leStart;
    st->leList = leList;
    st->lpStart = lpStart;
    st->lpList = lpList;
    st->blkI = blkI;
    st->blkJ = blkJ;
    st->blkStart = bStart;
    st->pairA = pA;
    st->pairB = pB;
    last_ = *st;
    nkf_ = nkf;
    nP_ = nP;
    nPair_ = nPair;
    nOff_ = nOff;
    if (blkIJ) {
        blkIJ->assign(2 * (size_t)nBlk, 0);
        if (nBlk) {
            GS_CHECK(hipMemcpyAsync(blkIJ->data(), blkI, sizeof(int) * nBlk, hipMemcpyDeviceToHost, s));
            GS_CHECK(hipMemcpyAsync(blkIJ->data() + nBlk, blkJ, sizeof(int) * nBlk, hipMemcpyDeviceToHost, s));
            GS_CHECK(stream_wait(s));
        }
    }
    return 0;
}

bool small_inputs_fit(int nkf, int npt, int ne) {
    return nkf <= kSmMaxKf && npt <= kSmMaxPt && ne <= kSmMaxE;
}
bool GpuStructBuilder::small_fits(int nkf, int npt, int ne, int nFreeKf) {
    return small_inputs_fit(nkf, npt, ne) && nFreeKf <= kSmMaxP;
}

int GpuStructBuilder::build_small(int level, int nkf, int npt, int ne, const int32_t* dKp, const int32_t* dPtOrd,
                                  const uint8_t* dLevel, const uint8_t* dKfFixed, const int32_t* dKfId, int32_t* pePos,
                                  hipStream_t s, BaStructDev* st, GpuStructInfo* info,
                                  const std::function<int()>& afterLaunch) {
    if (!small_inputs_fit(nkf, npt, ne)) return 1;
    if (!hSig_) {
        if (hipHostMalloc((void**)&hSig_, sizeof(int) * 64, hipHostMallocCoherent) != hipSuccess) return -2;
        std::memset((void*)hSig_, 0, sizeof(int) * 64);
    }
    const int nE0 = std::max(ne, 1);
    SmallArgs A{};
    A.level = level;
    A.nkf = nkf;
    A.npt = npt;
    A.ne = ne;
    A.seq = ++sigSeq_;
    A.kp = dKp;
    A.ptOrd = dPtOrd;
    A.lv = dLevel;
    A.kfFixed = dKfFixed;
    A.kfId = dKfId;
    // the slots of the multi-launch builder (download() and the engine read the same pointers);
    // the Schur terms are at most kSmMaxP + 1 choose 2 per landmark, i.e. 12 per free-pose edge
    GS_PTR(int, sc, S_SC, 64);
    GS_PTR(int, aE, S_AE, nE0);
    GS_PTR(int, ePose, S_EPOSE, nE0);
    GS_PTR(int, eLand, S_ELAND, nE0);
    GS_PTR(int, poseKf, S_POSEKF, nkf + 1);
    GS_PTR(int, landPt, S_LANDPT, npt + 1);
    GS_PTR(int, peStart, S_PESTART, nkf + 1);
    GS_PTR(int, peList, S_PELIST, nE0);
    GS_PTR(int, leStart, S_LESTART, npt + 1);
    GS_PTR(int, leList, S_LELIST, nE0);
    GS_PTR(int, lpStart, S_LPSTART, npt + 1);
    GS_PTR(int, lpList, S_LPLIST, nE0);
    GS_PTR(int, blkI, S_BLKI, kSmTri + 1);
    GS_PTR(int, blkJ, S_BLKJ, kSmTri + 1);
    GS_PTR(int, bStart, S_BSTART, kSmTri + 1);
    GS_PTR(int, pA, S_PA, (size_t)(kSmMaxP + 1) / 2 * nE0 + 1);
    GS_PTR(int, pB, S_PB, (size_t)(kSmMaxP + 1) / 2 * nE0 + 1);
    A.aE = aE; A.ePose = ePose; A.eLand = eLand; A.poseKf = poseKf; A.landPt = landPt; A.peStart = peStart;
    A.peList = peList; A.leStart = leStart; A.leList = leList; A.lpStart = lpStart; A.lpList = lpList; A.blkI = blkI;
    A.blkJ = blkJ; A.blkStart = bStart; A.pairA = pA; A.pairB = pB; A.pePos = pePos; A.sc = sc;
    A.hSc = hSig_;
    static const bool say = getenv("ORBGPU_BA_TIMES") != nullptr;
    A.ts = say ? reinterpret_cast<volatile long long*>(hSig_ + 32) : nullptr;
    hipLaunchKernelGGL(k_gs_small, dim3(1), dim3(kSmT), 0, s, A);
    GS_CHECK(hipGetLastError());
    if (afterLaunch)   // work the caller queues behind the kernel while the host waits for its counts
        if (int e = afterLaunch()) return e;
    // the counts arrive in pinned memory behind the lists: spin on the sequence word (a stream
    // sync wakes tens of us late); past 50 ms, a stream sync
    volatile int* w = hSig_ + SM_SEQ;
    const auto t0 = std::chrono::steady_clock::now();
    for (unsigned spin = 1; *w != A.seq; spin++) {
        if ((spin & 4095) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(50)) {
            GS_CHECK(hipStreamSynchronize(s));
            if (*w != A.seq) return -2;
            break;
        }
        __builtin_ia32_pause();
    }
    const hipError_t q = hipStreamQuery(s);   // a sticky error of the drained work
    if (q != hipSuccess && q != hipErrorNotReady) return -2;
    int v[SM_N];
    for (int k = 0; k < SM_SEQ; k++) v[k] = hSig_[k];
    if (say) {
        const volatile long long* t = reinterpret_cast<const volatile long long*>(hSig_ + 32);
        fprintf(stderr, "[ba]     one-workgroup lists (us): edges %.1f  poses %.1f  points %.1f  -- %.1f  "
                "counts %.1f  landmark lists %.1f  pose lists %.1f  Schur %.1f  (total %.1f)\n",
                (t[1] - t[0]) * 0.01, (t[2] - t[1]) * 0.01, (t[3] - t[2]) * 0.01, (t[4] - t[3]) * 0.01,
                (t[5] - t[4]) * 0.01, (t[6] - t[5]) * 0.01, (t[7] - t[6]) * 0.01, (t[8] - t[7]) * 0.01,
                (t[8] - t[0]) * 0.01);
    }
    if (v[SM_FALLBACK]) return 1;
    if (v[SM_ERR]) {
        info->err = v[SM_ERR];
        return -1;
    }
    const int nE = v[SM_NE], nP = v[SM_NP], nL = v[SM_NL], nBlk = v[SM_NBLK], nPair = v[SM_NPAIR];
    info->nE = nE;
    info->nP = nP;
    info->nL = nL;
    info->nBlk = nBlk;
    info->nPair = nPair;
    info->nLp = v[SM_NLP];
    info->nPe = v[SM_NPE];
    info->nLe = nE;
    info->err = 0;
    info->maxPe = v[SM_MAXPE];
    info->maxLe = v[SM_MAXLE];
    info->maxBlk = v[SM_MAXBLK];
    info->nEglob = nE;
    info->nLglob = nL;
    info->posDone = pePos ? 1 : 0;
    st->nE = nE;
    st->nP = nP;
    st->nL = nL;
    st->nBlk = nBlk;
    st->aE = aE;
    st->ePose = ePose;
    st->eLand = eLand;
    st->poseKf = poseKf;
    st->landPt = landPt;
    st->peStart = peStart;
    st->peList = peList;
    st->leStart = leStart;
    st->leList = leList;
    st->lpStart = lpStart;
    st->lpList = lpList;
    st->blkI = blkI;
    st->blkJ = blkJ;
    st->blkStart = bStart;
    st->pairA = pA;
    st->pairB = pB;
    last_ = *st;
    nkf_ = nkf;
    nP_ = nP;
    nPair_ = nPair;
    nOff_ = -1;   // no sorted block keys behind this build (offkeys() refuses)
    return 0;
}

int GpuStructBuilder::offkeys(std::vector<int64_t>* out, hipStream_t s) {
    if (nOff_ < 0) return -2;   // the one-workgroup build keeps no block keys (dense systems only)
    out->assign(nOff_, 0);
    if (!nOff_) return 0;
    // the sorted block keys at the off-diagonal segment heads, compacted (ascending (i1, i2))
    auto cub = [&](auto fn) -> int {
        size_t bytes = 0;
        GS_CHECK(fn(nullptr, bytes));
        void* t = buf(S_TEMP, bytes);
        if (!t) return -2;
        GS_CHECK(fn(t, bytes));
        return 0;
    };
    const unsigned long long* bkey2 = (const unsigned long long*)p_[S_BKEY2];
    const int* offFlag = (const int*)p_[S_OFFKEY];
    int* sc = (int*)p_[S_SC];
    GS_PTR(unsigned long long, ok, S_KFKEY2, std::max(nPair_, 1));
    GS_PTR(long long, okl, S_TIDX, nOff_);   // tidx is free once the pairs are filled
    const int nPair = nPair_, nkf = nkf_, nP = nP_;
    if (int e = cub([&](void* t, size_t& b) {
            return hipcub::DeviceSelect::Flagged(t, b, bkey2, offFlag, ok, sc + C_NOFF, nPair, s);
        }))
        return e;
    hipLaunchKernelGGL(k_gs_offkey, dim3(nb(nOff_)), dim3(kT), 0, s, nOff_, sc, ok, nkf, nP, okl);
    GS_CHECK(hipGetLastError());
    GS_CHECK(hipMemcpyAsync(out->data(), okl, sizeof(long long) * nOff_, hipMemcpyDeviceToHost, s));
    GS_CHECK(stream_wait(s));
    return 0;
}

int GpuStructBuilder::download(const GpuStructInfo& I, std::vector<int32_t>* out, hipStream_t s) {
    const BaStructDev& S = last_;
    const struct {
        const int32_t* p;
        size_t n;
    } parts[] = {{S.aE, (size_t)I.nE},          {S.ePose, (size_t)I.nE},       {S.eLand, (size_t)I.nE},
                 {S.poseKf, (size_t)I.nP},      {S.landPt, (size_t)I.nL},      {S.peStart, (size_t)I.nP + 1},
                 {S.peList, (size_t)I.nPe},     {S.leStart, (size_t)I.nL + 1}, {S.leList, (size_t)I.nLe},
                 {S.lpStart, (size_t)I.nL + 1}, {S.lpList, (size_t)I.nLp},     {S.blkI, (size_t)I.nBlk},
                 {S.blkJ, (size_t)I.nBlk},      {S.blkStart, (size_t)I.nBlk + 1}, {S.pairA, (size_t)I.nPair},
                 {S.pairB, (size_t)I.nPair}};
    size_t tot = 0;
    for (auto& q : parts) tot += q.n;
    out->assign(tot, 0);
    size_t o = 0;
    for (auto& q : parts) {
        if (q.n) GS_CHECK(hipMemcpyAsync(out->data() + o, q.p, sizeof(int32_t) * q.n, hipMemcpyDeviceToHost, s));
        o += q.n;
    }
    GS_CHECK(hipStreamSynchronize(s));
    return 0;
}

}  // namespace orbgpu

// ---------------------------------------------------------------- unit entry (parity tests)
namespace orbgpu {
// Both builders on one level of a problem given as plain arrays; out = [nE nP nL nBlk nPair nPe nLe
// nLp | the 16 lists in download() order].  gpu = 0: the host restatement (ba_struct.cpp), 1 build(), 2 build_small().
int debug_struct_all(int nkf, int npt, int ne, const int32_t* eKf, const int32_t* ePt, const uint8_t* lv,
                     const uint8_t* kfFixed, const int32_t* kfId, const int32_t* ptId, int level, int gpu,
                     std::vector<int32_t>* out) {
    out->clear();
    if (!gpu) {
        BaHostStruct S;
        std::vector<uint8_t> kfAct, ptAct;
        ba_active_set(level, nkf, npt, ne, eKf, ePt, lv, &S.aE, &kfAct, &ptAct);
        if (ba_build_lists(nkf, npt, eKf, ePt, kfFixed, kfId, ptId, kfAct, ptAct, &S)) return -1;
        const int nP = (int)S.poseKf.size(), nL = (int)S.landPt.size(), nBlk = (int)S.blkI.size();
        *out = {(int)S.aE.size(), nP, nL, nBlk, S.blkStart[nBlk], S.peStart[nP], S.leStart[nL], S.lpStart[nL]};
        const std::vector<int32_t>* parts[] = {&S.aE,     &S.ePose,  &S.eLand,  &S.poseKf,   &S.landPt, &S.peStart,
                                               &S.peList, &S.leStart, &S.leList, &S.lpStart, &S.lpList, &S.blkI,
                                               &S.blkJ,   &S.blkStart, &S.pairA, &S.pairB};
        const size_t n[] = {S.aE.size(), S.aE.size(), S.aE.size(), (size_t)nP, (size_t)nL, (size_t)nP + 1,
                            (size_t)S.peStart[nP], (size_t)nL + 1, (size_t)S.leStart[nL], (size_t)nL + 1,
                            (size_t)S.lpStart[nL], (size_t)nBlk, (size_t)nBlk, (size_t)nBlk + 1,
                            (size_t)S.blkStart[nBlk], (size_t)S.blkStart[nBlk]};
        for (int k = 0; k < 16; k++) out->insert(out->end(), parts[k]->begin(), parts[k]->begin() + n[k]);
        return 0;
    }
    hipStream_t s = nullptr;
    GS_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    std::vector<EdgeDev> E(std::max(ne, 1));
    std::memset(E.data(), 0, sizeof(EdgeDev) * E.size());
    for (int i = 0; i < ne; i++) {
        E[i].pt = ePt[i];
        E[i].kf = eKf[i];
    }
    EdgeDev* dE = nullptr;
    uint8_t *dLv = nullptr, *dFx = nullptr;
    int32_t *dKid = nullptr, *dPid = nullptr;
    int rc = 0;
    if (hipMalloc(&dE, sizeof(EdgeDev) * E.size()) != hipSuccess || hipMalloc(&dLv, std::max(ne, 1)) != hipSuccess ||
        hipMalloc(&dFx, std::max(nkf, 1)) != hipSuccess || hipMalloc(&dKid, 4 * std::max(nkf, 1)) != hipSuccess ||
        hipMalloc(&dPid, 4 * std::max(npt, 1)) != hipSuccess)
        rc = -2;
    if (!rc && (hipMemcpy(dE, E.data(), sizeof(EdgeDev) * E.size(), hipMemcpyHostToDevice) != hipSuccess ||
                (ne && hipMemcpy(dLv, lv, ne, hipMemcpyHostToDevice) != hipSuccess) ||
                (nkf && hipMemcpy(dFx, kfFixed, nkf, hipMemcpyHostToDevice) != hipSuccess) ||
                (nkf && hipMemcpy(dKid, kfId, 4 * nkf, hipMemcpyHostToDevice) != hipSuccess) ||
                (npt && hipMemcpy(dPid, ptId, 4 * npt, hipMemcpyHostToDevice) != hipSuccess)))
        rc = -2;
    if (!rc) {
        GpuStructBuilder b;
        BaStructDev st{};
        GpuStructInfo info{};
        rc = 1;   // gpu = 2: the one-workgroup builder (the multi-launch one outside its limits)
        if (gpu == 2 && small_inputs_fit(nkf, npt, ne)) {
            // its inputs as the engine's upload makes them: the compact edge keys, the point order
            std::vector<int32_t> kp(std::max(ne, 1)), ord;
            for (int i = 0; i < ne; i++) kp[i] = (eKf[i] << 13) | ePt[i];
            ba_order_by_id(npt, ptId, &ord);
            ord.resize(std::max(npt, 1));
            int32_t *dKp = nullptr, *dOrd = nullptr;
            if (hipMalloc(&dKp, 4 * kp.size()) != hipSuccess || hipMalloc(&dOrd, 4 * ord.size()) != hipSuccess ||
                hipMemcpy(dKp, kp.data(), 4 * kp.size(), hipMemcpyHostToDevice) != hipSuccess ||
                hipMemcpy(dOrd, ord.data(), 4 * ord.size(), hipMemcpyHostToDevice) != hipSuccess)
                rc = -2;
            else
                rc = b.build_small(level, nkf, npt, ne, dKp, dOrd, dLv, dFx, dKid, nullptr, s, &st, &info);
            (void)hipFree(dKp);
            (void)hipFree(dOrd);
        }
        if (rc == 1) rc = b.build(level, nkf, npt, ne, dE, dLv, dFx, dKid, dPid, nullptr, s, &st, &info);
        std::vector<int32_t> lists;
        if (!rc) rc = b.download(info, &lists, s);
        if (!rc) {
            *out = {info.nE, info.nP, info.nL, info.nBlk, info.nPair, info.nPe, info.nLe, info.nLp};
            out->insert(out->end(), lists.begin(), lists.end());
        }
    }
    (void)hipFree(dE);
    (void)hipFree(dLv);
    (void)hipFree(dFx);
    (void)hipFree(dKid);
    (void)hipFree(dPid);
    (void)hipStreamDestroy(s);
    return rc;
}
}  // namespace orbgpu
