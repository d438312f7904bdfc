// ba_struct.cpp -- host index maps and lists of one BA optimisation level (ba_struct.hpp).
// Every list comes out in the order the reference's structures imply:
//   vertices ascending by mnId (g2o's _ivMap is sorted by vertex id, sparse_optimizer.cpp:
//   buildIndexMapping; poses below landmarks by the Optimizer's id scheme, Optimizer.cc:
//   561-627), per-vertex edge lists in edge insertion order, and each landmark's pose terms
//   in pose order (BlockSolver::buildStructure walks the landmark's edges per pose,
//   block_solver.hpp:139-168).  Counting sorts throughout: O(edges + vertices) per call.
#include "ba_struct.hpp"

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <numeric>
#include <thread>

namespace orbgpu {

void ba_active_set(int level, int nkf, int npt, int ne, const int32_t* eKf, const int32_t* ePt, const uint8_t* edgeLevel,
                   std::vector<int32_t>* aE, std::vector<uint8_t>* kfAct, std::vector<uint8_t>* ptAct) {
    aE->clear();
    aE->reserve(ne);
    kfAct->assign(nkf, 0);
    ptAct->assign(npt, 0);
    for (int i = 0; i < ne; i++)
        if (edgeLevel[i] == level) {
            aE->push_back(i);
            (*kfAct)[eKf[i]] = 1;
            (*ptAct)[ePt[i]] = 1;
        }
}

// indices i with flag[i] set, ascending by id[i] (ids are distinct): an LSD radix sort of 64-bit
// keys (the id, sign-flipped so unsigned order is signed order, above the index), three 11-bit
// passes over the id -- a landmark set of thousands sorts in O(n) instead of a comparison sort's
// n log n indirect compares
static void by_id(int n, const uint8_t* flag, const int32_t* id, std::vector<int32_t>* out) {
    out->clear();
    thread_local std::vector<uint64_t> keys, tmp;
    keys.clear();
    bool sorted = true;
    int32_t last = 0;
    for (int i = 0; i < n; i++)
        if (flag[i]) {
            if (!keys.empty() && id[i] <= last) sorted = false;
            last = id[i];
            keys.push_back(((uint64_t)((uint32_t)id[i] ^ 0x80000000u) << 32) | (uint32_t)i);
        }
    const size_t m = keys.size();
    if (!sorted) {
        if (m < 64) {
            std::sort(keys.begin(), keys.end());
        } else {
            tmp.resize(m);
            uint32_t cnt[2048];
            for (int pass = 0; pass < 3; pass++) {
                const int sh = 32 + 11 * pass;
                std::fill(cnt, cnt + 2048, 0u);
                for (size_t k = 0; k < m; k++) cnt[(keys[k] >> sh) & 2047]++;
                uint32_t acc = 0;
                for (int b = 0; b < 2048; b++) {
                    const uint32_t c = cnt[b];
                    cnt[b] = acc;
                    acc += c;
                }
                for (size_t k = 0; k < m; k++) tmp[cnt[(keys[k] >> sh) & 2047]++] = keys[k];
                keys.swap(tmp);
            }
        }
    }
    out->resize(m);
    for (size_t k = 0; k < m; k++) (*out)[k] = (int32_t)(keys[k] & 0xffffffffu);
}

void ba_order_by_id(int n, const int32_t* id, std::vector<int32_t>* out) {
    std::vector<uint8_t> all((size_t)std::max(n, 1), 1);
    by_id(n, all.data(), id, out);
}

// The Schur pattern of a structure whose lpStart / lpList (landmark -> free-pose edges, pose
// order) and their poses qp are built: blocks numbered (diagonal first, then first use in the
// (landmark, u <= v) walk), each block's terms in landmark order.
int ba_build_blocks(int nP, int nL, const int32_t* __restrict__ qs, const int32_t* __restrict__ ql,
                    const int32_t* __restrict__ qp, BaHostStruct* S) {
    static const bool say = getenv("ORBGPU_BA_TIMES") != nullptr;
    using sclk = std::chrono::steady_clock;
    auto ts0 = sclk::now();
    auto lap = [&](const char* what) {
        if (!say) return;
        const auto t = sclk::now();
        fprintf(stderr, "[ba]     lists: %s %.1f us\n", what, std::chrono::duration<double, std::micro>(t - ts0).count());
        ts0 = t;
    };
    // Schur pattern: diagonal blocks first, then blocks in order of first use (landmark order,
    // pose pairs u <= v); one pass numbers and counts, one pass fills
    std::vector<int32_t> blkOf((size_t)nP * nP, -1), bi, bj, cnt;
    for (int i = 0; i < nP; i++) {
        blkOf[(size_t)i * nP + i] = i;
        bi.push_back(i);
        bj.push_back(i);
        cnt.push_back(0);
    }
    {
        int32_t* __restrict__ bo = blkOf.data();
        for (int l = 0; l < nL; l++) {
            const int b0 = qs[l], b1 = qs[l + 1];
            for (int u = b0; u < b1; u++) {
                int32_t* __restrict__ row = bo + (size_t)qp[u] * nP;
                for (int v = u; v < b1; v++) {
                    int b = row[qp[v]];
                    if (b < 0) {
                        b = row[qp[v]] = (int)bi.size();
                        bi.push_back(qp[u]);
                        bj.push_back(qp[v]);
                        cnt.push_back(0);
                    }
                    cnt[b]++;
                }
            }
        }
    }
    lap("block numbering + counts");
    const int nBlk = (int)bi.size();
    S->blkI.swap(bi);
    S->blkJ.swap(bj);
    S->blkStart.assign(nBlk + 1, 0);
    for (int b = 0; b < nBlk; b++) S->blkStart[b + 1] = S->blkStart[b] + cnt[b];
    const int nPair = S->blkStart[nBlk];
    S->pairA.resize(std::max(nPair, 1));
    S->pairB.resize(std::max(nPair, 1));
    // fill: each block's terms in landmark order.  Large systems (a global BA) split the landmarks
    // into T contiguous ranges: per-range block counts, per-block prefix over the ranges (range t
    // starts after ranges < t), then every range fills its own slots -- the same order.
    {
        int32_t* __restrict__ pa = S->pairA.data();
        int32_t* __restrict__ pb = S->pairB.data();
        const int32_t* __restrict__ bo = blkOf.data();
        const char* env = getenv("ORBGPU_STRUCT_THREADS");
        const int hw = (int)std::thread::hardware_concurrency();
        int T = env ? atoi(env) : (nPair >= (1 << 18) ? std::min(16, std::max(1, hw)) : 1);
        T = std::max(1, std::min(T, std::max(1, nL)));
        auto walk = [&](int l0, int l1, int32_t* cur, bool fill) {
            for (int l = l0; l < l1; l++) {
                const int b0 = qs[l], b1 = qs[l + 1];
                for (int u = b0; u < b1; u++) {
                    const int32_t* __restrict__ row = bo + (size_t)qp[u] * nP;
                    const int au = ql[u];
                    for (int v = u; v < b1; v++) {
                        const int b = row[qp[v]];
                        if (fill) {
                            const int q = cur[b]++;
                            pa[q] = au;
                            pb[q] = ql[v];
                        } else {
                            cur[b]++;
                        }
                    }
                }
            }
        };
        if (T == 1) {
            std::vector<int32_t> fb(S->blkStart.begin(), S->blkStart.end() - 1);
            walk(0, nL, fb.data(), true);
        } else {
            const int chunk = (nL + T - 1) / T;
            std::vector<std::vector<int32_t>> cur(T, std::vector<int32_t>(nBlk, 0));
            auto par = [&](auto f) {
                std::vector<std::thread> th;
                for (int t = 1; t < T; t++) th.emplace_back([&f, t] { f(t); });
                f(0);
                for (auto& x : th) x.join();
            };
            par([&](int t) { walk(std::min(nL, t * chunk), std::min(nL, (t + 1) * chunk), cur[t].data(), false); });
            par([&](int t) {   // blocks [t * bc, (t + 1) * bc): counts -> starting slots per range
                const int bc = (nBlk + T - 1) / T;
                for (int b = std::min(nBlk, t * bc); b < std::min(nBlk, (t + 1) * bc); b++) {
                    int base = S->blkStart[b];
                    for (int r = 0; r < T; r++) {
                        const int c = cur[r][b];
                        cur[r][b] = base;
                        base += c;
                    }
                }
            });
            par([&](int t) { walk(std::min(nL, t * chunk), std::min(nL, (t + 1) * chunk), cur[t].data(), true); });
        }
    }
    lap("pair fill");
    return 0;
}

int ba_build_lists(int nkf, int npt, const int32_t* eKf, const int32_t* ePt, const uint8_t* kfFixed,
                   const int32_t* kfId, const int32_t* ptId, const std::vector<uint8_t>& kfAct,
                   const std::vector<uint8_t>& ptAct, BaHostStruct* S, bool checkDup) {
    static const bool say = getenv("ORBGPU_BA_TIMES") != nullptr;   // the phases below (tools/)
    using sclk = std::chrono::steady_clock;
    auto ts0 = sclk::now();
    auto lap = [&](const char* what) {
        if (!say) return;
        const auto t = sclk::now();
        fprintf(stderr, "[ba]     lists: %s %.1f us\n", what, std::chrono::duration<double, std::micro>(t - ts0).count());
        ts0 = t;
    };
    std::vector<uint8_t> freeKf(nkf);
    for (int k = 0; k < nkf; k++) freeKf[k] = kfAct[k] && !kfFixed[k];
    by_id(nkf, freeKf.data(), kfId, &S->poseKf);
    by_id(npt, ptAct.data(), ptId, &S->landPt);
    const std::vector<int32_t>& aE = S->aE;
    const int nE = (int)aE.size(), nP = (int)S->poseKf.size(), nL = (int)S->landPt.size();
    std::vector<int32_t> poseIdx(nkf, -1), landIdx(npt, -1);
    for (int i = 0; i < nP; i++) poseIdx[S->poseKf[i]] = i;
    for (int i = 0; i < nL; i++) landIdx[S->landPt[i]] = i;
    // raw pointers below: stores through S's vectors would otherwise alias every load
    S->ePose.resize(nE);
    S->eLand.resize(nE);
    S->peStart.assign(nP + 1, 0);
    S->leStart.assign(nL + 1, 0);
    S->lpStart.assign(nL + 1, 0);
    {
        int32_t* __restrict__ eP = S->ePose.data();
        int32_t* __restrict__ eL = S->eLand.data();
        int32_t* __restrict__ ps = S->peStart.data();
        int32_t* __restrict__ ls = S->leStart.data();
        int32_t* __restrict__ qs = S->lpStart.data();
        const int32_t* __restrict__ pi = poseIdx.data();
        const int32_t* __restrict__ li = landIdx.data();
        const int32_t* __restrict__ ae = aE.data();
        for (int a = 0; a < nE; a++) {
            const int e = ae[a], p = pi[eKf[e]], l = li[ePt[e]];
            eP[a] = p;
            eL[a] = l;
            const int32_t f = p >= 0;   // branch-free: fixed-pose edges count 0 (into ps[0] += 0)
            ls[l + 1]++;
            ps[p + 1] += f;
            qs[l + 1] += f;
        }
        for (int i = 0; i < nP; i++) ps[i + 1] += ps[i];
        for (int i = 0; i < nL; i++) {
            ls[i + 1] += ls[i];
            qs[i + 1] += qs[i];
        }
    }
    lap("index maps + counts");
    const int nPe = S->peStart[nP], nLe = S->leStart[nL], nLp = S->lpStart[nL];
    S->peList.resize(std::max(nPe, 1));
    S->leList.resize(std::max(nLe, 1));
    S->lpList.resize(std::max(nLp, 1));
    std::vector<int32_t> lpPose(std::max(nLp, 1));
    {
        const int32_t* __restrict__ eP = S->ePose.data();
        const int32_t* __restrict__ eL = S->eLand.data();
        const int32_t* __restrict__ ps = S->peStart.data();
        int32_t* __restrict__ pl = S->peList.data();
        int32_t* __restrict__ ll = S->leList.data();
        int32_t* __restrict__ ql = S->lpList.data();
        int32_t* __restrict__ qp = lpPose.data();
        std::vector<int32_t> fp(S->peStart.begin(), S->peStart.end() - 1), fl(S->leStart.begin(), S->leStart.end() - 1),
            fq(S->lpStart.begin(), S->lpStart.end() - 1);
        int32_t* __restrict__ fpp = fp.data();
        int32_t* __restrict__ flp = fl.data();
        int32_t* __restrict__ fqp = fq.data();
        for (int a = 0; a < nE; a++) {
            if (eP[a] >= 0) pl[fpp[eP[a]]++] = a;
            ll[flp[eL[a]]++] = a;
        }
        // landmark buckets filled pose by pose: each comes out in ascending pose order
        for (int p = 0; p < nP; p++)
            for (int j = ps[p]; j < ps[p + 1]; j++) {
                const int a = pl[j], q = fqp[eL[a]]++;
                ql[q] = a;
                qp[q] = p;
            }
    }
    lap("edge lists");
    const int32_t* __restrict__ qs = S->lpStart.data();
    const int32_t* __restrict__ ql = S->lpList.data();
    const int32_t* __restrict__ qp = lpPose.data();
    if (checkDup) {   // one edge per (pose, landmark); (the C ABI validated its callers' edges)
        for (int l = 0; l < nL; l++)
            for (int j = qs[l] + 1; j < qs[l + 1]; j++)
                if (qp[j] == qp[j - 1]) return -1;
        lap("duplicate check");
    }
    return ba_build_blocks(nP, nL, qs, ql, qp, S);
}


// The lists of a level whose active edges are a subset of an earlier structure's (A: the same
// problem, its edges of another level set or gated since): every list of A filtered to the edges
// now at `level`, in A's order -- edge order, id order and pose order all survive a filter -- and
// a vertex kept while one of its edges is.  The Schur pattern is numbered again (a block's first
// use can move).  Equal to ba_active_set + ba_build_lists on the same level (no duplicate check:
// A's edges had none).
int ba_refine_lists(const BaHostStruct& A, const uint8_t* edgeLevel, int level, BaHostStruct* S) {
    const int nE1 = (int)A.aE.size(), nP1 = (int)A.poseKf.size(), nL1 = (int)A.landPt.size();
    std::vector<int32_t> a2(std::max(nE1, 1), -1);
    S->aE.clear();
    for (int a = 0; a < nE1; a++)
        if (edgeLevel[A.aE[a]] == level) {
            a2[a] = (int)S->aE.size();
            S->aE.push_back(A.aE[a]);
        }
    const int nE = (int)S->aE.size();
    // vertices: kept while an edge of theirs is (a free pose's edges are its peList segment)
    std::vector<int32_t> pMap(std::max(nP1, 1), -1), lMap(std::max(nL1, 1), -1);
    S->poseKf.clear();
    for (int i = 0; i < nP1; i++)
        for (int j = A.peStart[i]; j < A.peStart[i + 1]; j++)
            if (a2[A.peList[j]] >= 0) {
                pMap[i] = (int)S->poseKf.size();
                S->poseKf.push_back(A.poseKf[i]);
                break;
            }
    S->landPt.clear();
    for (int l = 0; l < nL1; l++)
        for (int j = A.leStart[l]; j < A.leStart[l + 1]; j++)
            if (a2[A.leList[j]] >= 0) {
                lMap[l] = (int)S->landPt.size();
                S->landPt.push_back(A.landPt[l]);
                break;
            }
    const int nP = (int)S->poseKf.size(), nL = (int)S->landPt.size();
    S->ePose.resize(nE);
    S->eLand.resize(nE);
    for (int a = 0; a < nE1; a++)
        if (a2[a] >= 0) {
            S->ePose[a2[a]] = A.ePose[a] >= 0 ? pMap[A.ePose[a]] : -1;
            S->eLand[a2[a]] = lMap[A.eLand[a]];
        }
    // a filter of each vertex's segment, the vertices in their (kept) order
    auto filter = [&](const std::vector<int32_t>& st, const std::vector<int32_t>& li, int n1,
                      const std::vector<int32_t>& vmap, std::vector<int32_t>* st2, std::vector<int32_t>* li2,
                      std::vector<int32_t>* pose2) {
        st2->assign(1, 0);
        li2->clear();
        if (pose2) pose2->clear();
        for (int v = 0; v < n1; v++) {
            if (vmap[v] < 0) continue;
            for (int j = st[v]; j < st[v + 1]; j++) {
                const int a = a2[li[j]];
                if (a < 0) continue;
                li2->push_back(a);
                if (pose2) pose2->push_back(S->ePose[a]);
            }
            st2->push_back((int)li2->size());
        }
        if (li2->empty()) li2->push_back(0);   // the sizes ba_build_lists leaves (>= 1)
    };
    filter(A.peStart, A.peList, nP1, pMap, &S->peStart, &S->peList, nullptr);
    filter(A.leStart, A.leList, nL1, lMap, &S->leStart, &S->leList, nullptr);
    std::vector<int32_t> lpPose;
    filter(A.lpStart, A.lpList, nL1, lMap, &S->lpStart, &S->lpList, &lpPose);
    if (lpPose.empty()) lpPose.push_back(0);
    return ba_build_blocks(nP, nL, S->lpStart.data(), S->lpList.data(), lpPose.data(), S);
}

}  // namespace orbgpu
