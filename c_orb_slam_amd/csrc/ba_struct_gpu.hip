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
}  // namespace

GpuStructBuilder::~GpuStructBuilder() {
    for (auto& p : p_)
        if (p) (void)hipFree(p);
    if (hSc_) (void)hipHostFree(hSc_);
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

int GpuStructBuilder::offkeys(std::vector<int64_t>* out, hipStream_t s) {
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
// nLp | the 16 lists in download() order].  gpu = 0: the host restatement (ba_struct.cpp).
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
        rc = b.build(level, nkf, npt, ne, dE, dLv, dFx, dKid, dPid, nullptr, s, &st, &info);
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
