// octree.hip -- gfx950 ORBextractor::DistributeOctTree (reference src/ORBextractor.cc:481-763).
//
// One workgroup per (image, level) job, all jobs of a batch in one launch, straight after
// k_fast_cells (each job compacts its own level's cell outputs first): no host round trip
// between FAST and the descriptor kernel.
//
// The std::list algorithm is restated over two observations:
//  * keys inside a node are always a subsequence of the input order, and the only
//    order-dependent use of that order is "first key wins response ties" -- so per-node key
//    sets are kept order-free (node id per key, or an unordered arena slice) and the tie is
//    resolved as (max response, min input index);
//  * the phase-1 loop (divide every node with > 1 key, children pushed to the FRONT in
//    n1..n4 order, parents erased) is a pure function of the list order, so the new list is
//    [children in reverse push order] ++ [the 1-key nodes in old order], built with block
//    scans; node id == list position.
// Phase 2 (size + 3 * nToExpand > N: divide the previous round's nodes largest-first,
// stop at N) is the reference's sequential loop: an index-linked list, one divide at a time
// with the workgroup partitioning the node's arena slice.  The reference sorts
// pair<int, ExtractorNode*> and so breaks size ties by heap address; this (like the host
// oracle) breaks them by node creation order -- DESIGN.md Appendix, quirk Q1.
#include "octree.hpp"

#include <cstdlib>

namespace orbgpu {

constexpr int OCT_TMAX = 1024;   // largest workgroup instance (k_octree<256|512|1024>)
constexpr int kOctCellsMax = kOctKMax / 2;   // FAST cells of one level (a job's compaction; in S.tmp)

struct OctShared {
    int16_t x0[2 * kOctNMax], y0[2 * kOctNMax], x1[2 * kOctNMax], y1[2 * kOctNMax];
    uint16_t cnt[2 * kOctNMax], seq[2 * kOctNMax], kbeg[2 * kOctNMax];
    int16_t prv[2 * kOctNMax], nxt[2 * kOctNMax];
    int ia[4 * kOctNMax];          // counters (phase 1 per virtual child, phase 2 per quadrant); best keys
    uint16_t vpos[4 * kOctNMax];   // virtual child -> push index -> list position
    uint16_t er[kOctNMax], eidx[kOctNMax];
    uint16_t vs[kOctNMax], vs2[kOctNMax];
    uint32_t sk[kOctNMax];         // phase-2 sort keys (size << 16 | creation order)
    uint16_t knode[kOctKMax], arena[kOctKMax];
    alignas(16) uint16_t tmp[kOctKMax];   // also the compaction's int cell deltas
    int wsum[OCT_TMAX / 64];
    int head, size, nfree, m, newm, seqctr, flag;
};

// Block-wide exclusive scan of flag(i) over i < n; put(i, rank) for flagged i.  Returns the
// total.  Every thread of the block calls it (two barriers).
template <int T, class Flag, class Put>
__device__ __forceinline__ int oct_scan(int n, Flag flag, Put put, int* wsum) {
    const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
    const int per = (n + T - 1) / T;
    const int a = min(n, t * per), e = min(n, a + per);
    int local = 0;
    for (int i = a; i < e; i++) local += flag(i) ? 1 : 0;
    int incl = local;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(incl, o, 64);
        if (lane >= o) incl += y;
    }
    if (lane == 63) wsum[wid] = incl;
    __syncthreads();
    int off = 0, total = 0;
#pragma unroll
    for (int w = 0; w < T / 64; w++) {
        const int s = wsum[w];
        if (w < wid) off += s;
        total += s;
    }
    int ex = off + incl - local;
    for (int i = a; i < e; i++)
        if (flag(i)) put(i, ex++);
    __syncthreads();
    return total;
}

// Block-wide exclusive scan of val(i) over i < n; put(i, prefix) for every i.  Returns the
// total.  Every thread of the block calls it (two barriers).
template <int T, class Val, class Put>
__device__ __forceinline__ int oct_scan_val(int n, Val val, Put put, int* wsum) {
    const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
    const int per = (n + T - 1) / T;
    const int a = min(n, t * per), e = min(n, a + per);
    int local = 0;
    for (int i = a; i < e; i++) local += val(i);
    int incl = local;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(incl, o, 64);
        if (lane >= o) incl += y;
    }
    if (lane == 63) wsum[wid] = incl;
    __syncthreads();
    int off = 0, total = 0;
#pragma unroll
    for (int w = 0; w < T / 64; w++) {
        const int s = wsum[w];
        if (w < wid) off += s;
        total += s;
    }
    int ex = off + incl - local;
    for (int i = a; i < e; i++) {
        put(i, ex);
        ex += val(i);
    }
    __syncthreads();
    return total;
}

__device__ __forceinline__ void oct_child_rect(const OctShared& S, int p, int q, int& a0, int& b0, int& a1, int& b1) {
    const int X0 = S.x0[p], Y0 = S.y0[p], X1 = S.x1[p], Y1 = S.y1[p];
    const int halfX = (int)ceilf((float)(X1 - X0) / 2), halfY = (int)ceilf((float)(Y1 - Y0) / 2);
    const int mx = X0 + halfX, my = Y0 + halfY;
    a0 = (q & 1) ? mx : X0;
    a1 = (q & 1) ? X1 : mx;
    b0 = (q & 2) ? my : Y0;
    b1 = (q & 2) ? Y1 : my;
}

// ExtractorNode::DivideNode child of a key: n1 (0) / n2 (1) / n3 (2) / n4 (3)
__device__ __forceinline__ int oct_quadrant(const OctShared& S, int p, uint32_t pk) {
    const int halfX = (int)ceilf((float)(S.x1[p] - S.x0[p]) / 2), halfY = (int)ceilf((float)(S.y1[p] - S.y0[p]) / 2);
    const int mx = S.x0[p] + halfX, my = S.y0[p] + halfY;
    const int x = (int)(pk & 0xfff), y = (int)((pk >> 12) & 0xfff);
    return (x < mx) ? (y < my ? 0 : 2) : (y < my ? 1 : 3);
}

__device__ __forceinline__ int oct_best_key(uint32_t pk, int k) { return (int)((pk >> 24) << 16) | (0xffff - k); }

template <int T>
__global__ void __launch_bounds__(T) k_octree(OctInput in, int nlevels, const OctLevelDev* __restrict__ lv,
                                                 uint32_t* __restrict__ jobsel, int* __restrict__ jobcnt, int jcap,
                                                 uint16_t* __restrict__ gscratch, size_t gstride, int* __restrict__ err) {
    __shared__ OctShared S;
    ORBGPU_PROF_START;
#ifdef ORBGPU_PROF
    // every job's duration (instrumented builds): slot 10 = max (cycles << 4 | level), slot 11 =
    // the sum, slot 12 = the job count, written on every return path by the destructor
    struct JobTimer {
        unsigned long long t0;
        int lvl;
        __device__ ~JobTimer() {
            if (threadIdx.x == 0) {
                const unsigned long long c = clock64() - t0;
                atomicMax(&g_orbgpu_prof[10], (c << 4) | (unsigned long long)lvl);
                atomicAdd(&g_orbgpu_prof[11], c);
                atomicAdd(&g_orbgpu_prof[12], 1ull);
            }
        }
    } jt{(unsigned long long)clock64(), (int)blockIdx.x / ((int)gridDim.x / nlevels)};
#endif
    // level-major dispatch order: the long jobs (level 0: the most candidates and features) of
    // every image start first and the short ones fill in behind them
    const int B = (int)gridDim.x / nlevels;
    const int l = (int)blockIdx.x / B, b = (int)blockIdx.x - l * B, job = b * nlevels + l;
    const int tid = threadIdx.x;
    // ---- the level's FAST candidates in cell order (ORBextractor.cc:776-829's push order):
    //      cell offsets by a block scan of the counts (S.ia), then a thread per candidate finds
    //      its cell (binary search over the offsets) and copies it from the cell's slot run to the
    //      level's own range of `packed` (read back below by this workgroup only); the copies of
    //      a thread are independent, so their loads are in flight together
    const int cb = in.lcb[l], nc = in.lcb[l + 1] - cb;
    const int* cnt = in.counts + (size_t)b * in.ncells + cb;
    if (nc + 1 > 4 * kOctNMax || nc > kOctCellsMax) {
        if (tid == 0) {
            jobcnt[job] = 0;
            atomicOr(err, 2);
        }
        return;
    }
    // the cell deltas live in S.tmp (free until phase 1; kOctCellsMax ints)
    int* cdelta = reinterpret_cast<int*>(S.tmp);
    const int n = oct_scan_val<T>(
        nc, [&](int i) { return cnt[i]; },
        [&](int i, int o) {
            S.ia[i] = o;
            cdelta[i] = in.cell_slot[cb + i] - in.cell_slot[cb] - o;
        },
        S.wsum);
    const size_t base = (size_t)b * in.slots_per_image + (size_t)in.cell_slot[cb];
    if (n <= 0 || n > 0xffff) {
        if (tid == 0) {
            jobcnt[job] = 0;
            if (n > 0xffff) atomicOr(err, 2);
        }
        return;
    }
    {
        const uint32_t* sl = in.slots + base;   // cell c's run starts at sl[ia[c] + cdelta[c]]
        uint32_t* dst = in.packed + base;
        constexpr int U = 4;
        for (int k0 = tid; k0 < n; k0 += U * T) {
            uint32_t v[U];
#pragma unroll
            for (int u = 0; u < U; u++) {
                const int k = k0 + u * T;
                if (k < n) {
                    int lo = 0, hi = nc - 1;   // the last cell whose offset is <= k (it holds k)
                    while (lo < hi) {
                        const int mid = (lo + hi + 1) >> 1;
                        if (S.ia[mid] <= k) lo = mid;
                        else hi = mid - 1;
                    }
                    v[u] = sl[k + cdelta[lo]];
                }
            }
#pragma unroll
            for (int u = 0; u < U; u++)
                if (k0 + u * T < n) dst[k0 + u * T] = v[u];
        }
        if (tid == 0) atomicAdd(in.g_total, n);
    }
    __syncthreads();
    const uint32_t* src = in.packed + base;
    const OctLevelDev L = lv[l];
    const int N = L.N;
    // keys: node / arena / scratch indices in LDS, or in the global scratch for big jobs
    uint16_t* knode = S.knode;
    uint16_t* arena = S.arena;
    uint16_t* tmp = S.tmp;
    if (n > kOctKMax) {
        knode = gscratch + base;
        arena = knode + gstride;
        tmp = arena + gstride;
    }
    // ---- initial nodes (ORBextractor.cc:543-585)
    const int W = L.maxX - L.minX, Hh = L.maxY - L.minY;
    const int nIni = (int)roundf((float)W / (float)Hh);
    if (nIni < 1 || nIni > kOctNMax) {
        if (tid == 0) {
            jobcnt[job] = 0;
            atomicOr(err, 4);
        }
        return;
    }
    const float hX = (float)W / (float)nIni;
    for (int i = tid; i < nIni; i += T) S.ia[i] = 0;
    __syncthreads();
    for (int k = tid; k < n; k += T) {
        const uint32_t pk = src[k];
        int ib = (int)((float)(pk & 0xfff) / hX);
        ib = min(ib, nIni - 1);
        knode[k] = (uint16_t)ib;
        atomicAdd(&S.ia[ib], 1);
    }
    __syncthreads();
    // list = non-empty initial nodes in order (buffer 0), node id == position
    int cur = 0;
    int Sz = oct_scan<T>(
        nIni, [&](int i) { return S.ia[i] > 0; },
        [&](int i, int r) {
            S.x0[r] = (int16_t)(int)(hX * (float)i);
            S.x1[r] = (int16_t)(int)(hX * (float)(i + 1));
            S.y0[r] = 0;
            S.y1[r] = (int16_t)Hh;
            S.cnt[r] = (uint16_t)S.ia[i];
            S.seq[r] = (uint16_t)i;
            S.er[i] = (uint16_t)r;
        },
        S.wsum);
    for (int k = tid; k < n; k += T) knode[k] = S.er[knode[k]];
    int seqbase = nIni;
    int phase2 = 0, m = 0;
    __syncthreads();
    ORBGPU_PROF_MARK(0);   // initial nodes
    // ---- phase 1 (ORBextractor.cc:594-673)
    for (;;) {
        const int prevSize = Sz;
        const int nE = oct_scan<T>(
            Sz, [&](int i) { return S.cnt[cur + i] > 1; },
            [&](int i, int r) {
                S.er[i] = (uint16_t)r;
                S.eidx[r] = (uint16_t)i;
            },
            S.wsum);
        ORBGPU_PROF_COUNT(9);
        if (nE == 0) break;   // every node holds one key: size == prevSize
        for (int v = tid; v < 4 * nE; v += T) S.ia[v] = 0;
        __syncthreads();
        for (int k = tid; k < n; k += T) {
            const int p = knode[k];
            if (S.cnt[cur + p] > 1) {
                const int v = 4 * S.er[p] + oct_quadrant(S, cur + p, src[k]);
                tmp[k] = (uint16_t)v;
                atomicAdd(&S.ia[v], 1);
            } else {
                tmp[k] = 0xffff;
            }
        }
        __syncthreads();
        // push order of the non-empty children: parents in list order, n1..n4
        const int nC = oct_scan<T>(
            4 * nE, [&](int v) { return S.ia[v] > 0; }, [&](int v, int r) { S.vpos[v] = (uint16_t)r; }, S.wsum);
        const int nb = kOctNMax - cur;
        // 1-key nodes keep their relative order behind the children
        const int nNM = oct_scan<T>(
            Sz, [&](int i) { return S.cnt[cur + i] == 1; }, [&](int i, int r) { S.er[i] = (uint16_t)(nC + r); },
            S.wsum);
        if (nC + nNM > kOctNMax) {
            if (tid == 0) {
                jobcnt[job] = 0;
                atomicOr(err, 8);
            }
            return;
        }
        for (int v = tid; v < 4 * nE; v += T) {
            const int c = S.ia[v];
            if (c > 0) {
                const int t = S.vpos[v], pos = nC - 1 - t, parent = cur + S.eidx[v >> 2];
                int a0, b0, a1, b1;
                oct_child_rect(S, parent, v & 3, a0, b0, a1, b1);
                S.x0[nb + pos] = (int16_t)a0;
                S.y0[nb + pos] = (int16_t)b0;
                S.x1[nb + pos] = (int16_t)a1;
                S.y1[nb + pos] = (int16_t)b1;
                S.cnt[nb + pos] = (uint16_t)c;
                S.seq[nb + pos] = (uint16_t)(seqbase + t);
                S.vpos[v] = (uint16_t)pos;
            }
        }
        for (int i = tid; i < Sz; i += T)
            if (S.cnt[cur + i] == 1) {
                const int pos = S.er[i];
                S.x0[nb + pos] = S.x0[cur + i];
                S.y0[nb + pos] = S.y0[cur + i];
                S.x1[nb + pos] = S.x1[cur + i];
                S.y1[nb + pos] = S.y1[cur + i];
                S.cnt[nb + pos] = 1;
                S.seq[nb + pos] = S.seq[cur + i];
            }
        __syncthreads();
        // vSizeAndPointerToNode: children with > 1 key, push order
        const int nToExpand = oct_scan<T>(
            4 * nE, [&](int v) { return S.ia[v] > 1; }, [&](int v, int r) { S.vs[r] = (uint16_t)S.vpos[v]; },
            S.wsum);
        for (int k = tid; k < n; k += T) {
            const int v = tmp[k];
            knode[k] = v != 0xffff ? S.vpos[v] : S.er[knode[k]];
        }
        seqbase += nC;
        cur = nb;
        Sz = nC + nNM;
        __syncthreads();
        if (Sz >= N || Sz == prevSize) break;
        if (Sz + nToExpand * 3 > N) {
            phase2 = 1;
            m = nToExpand;
            break;
        }
    }
    ORBGPU_PROF_MARK(1);   // phase 1
    if (phase2) {
        // ---- phase 2 (ORBextractor.cc:673-738): arena slices, linked list, largest first
        const int nb = kOctNMax - cur;
        // kbeg = exclusive scan of cnt in list order; the list linked in position order
        {
            oct_scan_val<T>(
                Sz, [&](int i) { return (int)S.cnt[cur + i]; }, [&](int i, int ex) { S.kbeg[cur + i] = (uint16_t)ex; },
                S.wsum);
            for (int i = tid; i < Sz; i += T) {
                S.ia[i] = 0;
                S.prv[cur + i] = (int16_t)(i > 0 ? cur + i - 1 : -1);
                S.nxt[cur + i] = (int16_t)(i + 1 < Sz ? cur + i + 1 : -1);
            }
            if (tid == 0) {
                S.head = Sz > 0 ? cur : -1;
                S.size = Sz;
                S.nfree = nb;
                S.seqctr = seqbase;
                S.m = m;
                S.flag = 0;
            }
            for (int i = tid; i < m; i += T) S.vs[i] = (uint16_t)(cur + S.vs[i]);
            __syncthreads();
            for (int k = tid; k < n; k += T) {
                const int p = knode[k];
                arena[S.kbeg[cur + p] + atomicAdd(&S.ia[p], 1)] = (uint16_t)k;
            }
            __syncthreads();
        }
        ORBGPU_PROF_MARK(2);   // phase-2 set-up
        for (;;) {
            ORBGPU_PROF_COUNT(8);
            const int prevSize = S.size;
            const int mm = S.m;
            // sort ascending by (size, creation order): rank sort, keys unique
            for (int i = tid; i < mm; i += T) {
                const int id = S.vs[i];
                S.sk[i] = ((uint32_t)S.cnt[id] << 16) | S.seq[id];
            }
            __syncthreads();
            for (int i = tid; i < mm; i += T) {
                const uint32_t ki = S.sk[i];
                int r = 0;
                for (int j = 0; j < mm; j++) r += S.sk[j] < ki ? 1 : 0;
                S.vs2[r] = S.vs[i];
            }
            for (int i = tid; i < 4 * mm; i += T) S.ia[i] = 0;
            if (tid == 0) S.newm = 0;
            __syncthreads();
            ORBGPU_PROF_MARK(3);   // rank sort
            // The round's divides (largest first, ORBextractor.cc:700-736) are sequential only in
            // their bookkeeping (push_front order, node ids, the size >= N stop): the keys of
            // every node of the round are partitioned into its quadrants at once.  A node the
            // stop leaves undivided keeps its key SET (its slice is only reordered, and every
            // later use of a slice is order-free: best key = max response, then min index).
            // er[j] = first flattened key position of vs2[j]
            const int tot = oct_scan_val<T>(
                mm, [&](int j) { return (int)S.cnt[S.vs2[j]]; }, [&](int j, int ex) { S.er[j] = (uint16_t)ex; },
                S.wsum);
            auto owner = [&](int t) {   // largest j with er[j] <= t
                int lo = 0, hi = mm - 1;
                while (lo < hi) {
                    const int mid = (lo + hi + 1) >> 1;
                    if ((int)S.er[mid] <= t) lo = mid;
                    else hi = mid - 1;
                }
                return lo;
            };
            // (flattened position t: its key in tmp[t], its (node, quadrant) in knode[t])
            for (int t = tid; t < tot; t += T) {
                const int j = owner(t), p = S.vs2[j], pos = S.kbeg[p] + (t - S.er[j]);
                const int k = arena[pos];
                const int q = oct_quadrant(S, p, src[k]);
                tmp[t] = (uint16_t)k;
                knode[t] = (uint16_t)(4 * j + q);
                atomicAdd(&S.ia[4 * j + q], 1);
            }
            __syncthreads();
            // quadrant starts inside each node's slice (children n1..n4 take consecutive
            // sub-slices); ia becomes the scatter cursors
            for (int j = tid; j < mm; j += T) {
                int start = S.kbeg[S.vs2[j]];
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    S.vpos[4 * j + q] = (uint16_t)start;
                    start += S.ia[4 * j + q];
                    S.ia[4 * j + q] = 0;
                }
            }
            __syncthreads();
            for (int t = tid; t < tot; t += T) {
                const int v = knode[t];
                arena[S.vpos[v] + atomicAdd(&S.ia[v], 1)] = tmp[t];
            }
            __syncthreads();
            ORBGPU_PROF_MARK(4);   // key partition
            // the reference's sequential loop over the round's nodes: children pushed to the
            // front (n1..n4), the parent erased, stop as soon as the list reaches N
            // (list scalars in registers; an erased node is marked prv = -2)
            if (tid == 0) {
                int head = S.head, size = S.size, nfree = S.nfree, seqctr = S.seqctr, newm = 0, flag = 0;
                for (int j = mm - 1; j >= 0; j--) {
                    const int p = S.vs2[j];
                    int c4[4];
#pragma unroll
                    for (int q = 0; q < 4; q++) c4[q] = S.ia[4 * j + q];
                    for (int q = 0; q < 4; q++) {
                        const int c = c4[q];
                        if (c > 0) {
                            const int id = nfree++;
                            if (nfree > 2 * kOctNMax || id == cur) {
                                flag = 1;
                                break;
                            }
                            int a0, b0, a1, b1;
                            oct_child_rect(S, p, q, a0, b0, a1, b1);
                            S.x0[id] = (int16_t)a0;
                            S.y0[id] = (int16_t)b0;
                            S.x1[id] = (int16_t)a1;
                            S.y1[id] = (int16_t)b1;
                            S.cnt[id] = (uint16_t)c;
                            S.seq[id] = (uint16_t)(seqctr++);
                            S.kbeg[id] = S.vpos[4 * j + q];
                            // lNodes.push_front
                            S.prv[id] = -1;
                            S.nxt[id] = (int16_t)head;
                            if (head >= 0) S.prv[head] = (int16_t)id;
                            head = id;
                            size++;
                            if (c > 1) S.vs[newm++] = (uint16_t)id;
                        }
                    }
                    if (flag) break;
                    // lNodes.erase(parent)
                    const int pp = S.prv[p], pn = S.nxt[p];
                    if (pp >= 0) S.nxt[pp] = (int16_t)pn;
                    else head = pn;
                    if (pn >= 0) S.prv[pn] = (int16_t)pp;
                    S.prv[p] = -2;
                    size--;
                    if (size >= N) break;
                }
                S.head = head;
                S.size = size;
                S.nfree = nfree;
                S.seqctr = seqctr;
                S.newm = newm;
                S.flag = flag;
            }
            __syncthreads();
            ORBGPU_PROF_MARK(5);   // serial list update
            if (S.flag) {
                if (tid == 0) {
                    jobcnt[job] = 0;
                    atomicOr(err, 8);
                }
                return;
            }
            if (S.size >= N || S.size == prevSize) break;
            if (tid == 0) S.m = S.newm;
            __syncthreads();
        }
        // final list order: every divide pushed its children to the front, so the list is the
        // live phase-2 nodes newest first (ids nfree-1 down to nb), then the live nodes phase 1
        // left (ids cur.. in list position order)
        const int n2 = S.nfree - nb;
        const int sz = oct_scan<T>(
            n2 + Sz,
            [&](int u) {
                const int id = u < n2 ? nb + n2 - 1 - u : cur + (u - n2);
                return S.prv[id] != -2;
            },
            [&](int u, int r) { S.vpos[r] = (uint16_t)(u < n2 ? nb + n2 - 1 - u : cur + (u - n2)); }, S.wsum);
        if (sz > jcap) {
            if (tid == 0) {
                jobcnt[job] = 0;
                atomicOr(err, 16);
            }
            return;
        }
        // the best key of each node over its slice (max response, then min index): the live
        // slices partition the arena, so each position names its node (tmp) and the keys
        // meet in one atomic max per node
        for (int i = tid; i < sz; i += T) {
            const int id = S.vpos[i];
            const int kb = S.kbeg[id], kc = S.cnt[id];
            for (int t = 0; t < kc; t++) tmp[kb + t] = (uint16_t)i;
            S.ia[i] = -1;
        }
        __syncthreads();
        for (int pos = tid; pos < n; pos += T) {
            const int k = arena[pos];
            atomicMax(&S.ia[tmp[pos]], oct_best_key(src[k], k));
        }
        __syncthreads();
        for (int i = tid; i < sz; i += T) {
            const int k = 0xffff - (S.ia[i] & 0xffff);
            jobsel[(size_t)job * jcap + i] = src[k];
        }
        if (tid == 0) jobcnt[job] = sz;
        ORBGPU_PROF_MARK(6);   // final walk + best keys
        return;
    }
    // ---- phase 1 finished: list = positions 0..Sz-1 of buffer `cur`
    if (Sz > jcap) {
        if (tid == 0) {
            jobcnt[job] = 0;
            atomicOr(err, 16);
        }
        return;
    }
    for (int i = tid; i < Sz; i += T) S.ia[i] = -1;
    __syncthreads();
    for (int k = tid; k < n; k += T) atomicMax(&S.ia[knode[k]], oct_best_key(src[k], k));
    __syncthreads();
    for (int i = tid; i < Sz; i += T) {
        const int k = 0xffff - (S.ia[i] & 0xffff);
        jobsel[(size_t)job * jcap + i] = src[k];
    }
    if (tid == 0) jobcnt[job] = Sz;
    ORBGPU_PROF_MARK(7);   // phase-1 best keys
}

// Per image: level-major concatenation of the job lists -> (packed, b<<20 | l<<16 | k) at
// sel[b * selcap + k], n_out[b] (the reference's allKeypoints order, ORBextractor.cc:1065-1101).
__global__ void __launch_bounds__(64) k_sel_build(const uint32_t* __restrict__ jobsel, const int* __restrict__ jobcnt,
                                                  int nlevels, int jcap, int cap, int2* __restrict__ sel, int selcap,
                                                  int* __restrict__ nout, int* __restrict__ err) {
    const int b = blockIdx.x, lane = threadIdx.x;
    const int c = lane < nlevels ? jobcnt[b * nlevels + lane] : 0;
    int incl = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(incl, o, 64);
        if (lane >= o) incl += y;
    }
    const int total = __shfl(incl, 63, 64);
    if (lane == 0) {
        nout[b] = total;
        if (total > cap || total > selcap) atomicOr(err, 1);
    }
    if (total > cap || total > selcap) return;
    for (int l = 0; l < nlevels; l++) {
        const int cl = __shfl(c, l, 64), off = __shfl(incl - c, l, 64);
        const uint32_t* js = jobsel + (size_t)(b * nlevels + l) * jcap;
        for (int i = lane; i < cl; i += 64)
            sel[(size_t)b * selcap + off + i] = make_int2((int)js[i], (b << 20) | (l << 16) | (off + i));
    }
}

int octree_prof_read(unsigned long long* out16) {
#ifdef ORBGPU_PROF
    unsigned long long v[32];
    ORB_HIP_CHECK(hipMemcpyFromSymbol(v, HIP_SYMBOL(g_orbgpu_prof), sizeof(v)));
    for (int i = 0; i < 16; i++) out16[i] = v[i];
    unsigned long long z[32] = {};
    ORB_HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_orbgpu_prof), z, sizeof(z)));
    return 0;
#else
    (void)out16;
    return -1;
#endif
}

int octree_launch(const OctInput& in, int B, int nlevels, const OctLevelDev* lv, uint32_t* jobsel, int* jobcnt, int jcap,
                  uint16_t* gscratch, size_t gstride, int cap, int2* sel, int selcap, int* nout, int* err,
                  hipStream_t s) {
    static const int nt = [] {
        const char* e = getenv("ORBGPU_OCT_T");
        const int v = e ? atoi(e) : 512;   // 512: 0.139 -> 0.137 ms (128 images), 0.101 -> 0.093 (2)
        return v == 256 || v == 1024 ? v : 512;
    }();
    if (nt == 1024)
        hipLaunchKernelGGL(k_octree<1024>, dim3(B * nlevels), dim3(1024), 0, s, in, nlevels, lv, jobsel, jobcnt,
                           jcap, gscratch, gstride, err);
    else if (nt == 512)
        hipLaunchKernelGGL(k_octree<512>, dim3(B * nlevels), dim3(512), 0, s, in, nlevels, lv, jobsel, jobcnt,
                           jcap, gscratch, gstride, err);
    else
        hipLaunchKernelGGL(k_octree<256>, dim3(B * nlevels), dim3(256), 0, s, in, nlevels, lv, jobsel, jobcnt,
                           jcap, gscratch, gstride, err);
    hipLaunchKernelGGL(k_sel_build, dim3(B), dim3(64), 0, s, (const uint32_t*)jobsel, (const int*)jobcnt, nlevels,
                       jcap, cap, sel, selcap, nout, err);
    ORB_HIP_CHECK(hipGetLastError());
    return 0;
}

}  // namespace orbgpu
