// capi_ba.cpp -- extern "C" Optimizer_LocalBundleAdjustment (include/orbslam_gpu.h).
// Replaces ORB_SLAM2::Optimizer::LocalBundleAdjustment (reference src/Optimizer.cc:453-778).
#include <algorithm>
#include <atomic>
#include <cstring>
#include <new>
#include <vector>

#include "ba.hpp"
#include "ba_struct.hpp"
#include "ba_struct_gpu.hpp"
#include "capi_handles.hpp"
#include "host_par.hpp"
#include "ordering.hpp"
#include "orb_match.hpp"
#include "sim3opt.hpp"
#include "orb_extract.hpp"
#include "orb_match.hpp"

namespace {
orbgpu::BaEngine* engine(int* rc) {
    thread_local orbgpu::BaEngine* e = nullptr;
    thread_local int erc = 0;
    if (!e) {
        e = new orbgpu::BaEngine();
        erc = e->init();
    }
    *rc = erc;
    return e;
}

// Edges grouped by map point: 0 valid, 1 invalid (an index out of range, or a repeated keyframe
// inside a point's run), 2 some point starts two runs (the caller buckets).  Large problems run
// on up to 16 threads over ranges of whole runs (a range starts at the first run that starts in
// it); a run start claims its point with an atomic exchange, so a point met twice is seen by
// whichever range comes second.
int grouped_pairs(const ba_problem* P) {
    const int ne = P->n_edge;
    const int32_t* ep = P->edge_pt;
    const int32_t* ek = P->edge_kf;
    const uint32_t npt = (uint32_t)P->n_pt, nkf = (uint32_t)P->n_kf;
    std::vector<uint8_t> seen(std::max(P->n_pt, 1), 0);
    std::atomic<int> bad{0}, rep{0};
    const auto run_start = [&](int i) {   // first run start at or after i
        while (i > 0 && i < ne && ep[i] == ep[i - 1]) i++;
        return i;
    };
    orbgpu::host_parallel(ne, [&](int a, int b) {
        const int i0 = run_start(a), i1 = run_start(b);
        if (i0 >= i1) return;
        std::vector<int32_t> stamp(std::max(P->n_kf, 1), -1);
        int32_t cur = -1, run = -1;
        bool dup = false, again = false;
        for (int i = i0; i < i1; i++) {
            const int32_t pt = ep[i], kf = ek[i];
            if ((uint32_t)pt >= npt || (uint32_t)kf >= nkf) {
                dup = true;
                break;
            }
            if (pt != cur) {
                again |= __atomic_exchange_n(&seen[pt], (uint8_t)1, __ATOMIC_RELAXED) != 0;
                cur = pt;
                run++;
            }
            dup |= stamp[kf] == run;
            stamp[kf] = run;
        }
        if (dup) bad.store(1, std::memory_order_relaxed);
        if (again) rep.store(1, std::memory_order_relaxed);
    });
    return bad.load() ? 1 : rep.load() ? 2 : 0;
}

// grouped (optional): set when every map point's edges are one run (the Optimizer's order; the
// engine can then walk a point's edges without bucketing them)
int validate(const ba_problem* P, const ba_result* R, bool* grouped = nullptr) {
    if (grouped) *grouped = false;
    if (!P || !R || P->n_kf < 0 || P->n_pt < 0 || P->n_edge < 0) return ORB_E_INVALID;
    if (P->n_kf && (!P->kf_id || !P->kf_Tcw || !P->kf_local || !P->kf_cam || !R->kf_Tcw)) return ORB_E_INVALID;
    if (P->n_pt && (!P->pt_id || !P->pt_pos || !R->pt_pos)) return ORB_E_INVALID;
    if (P->n_edge && (!P->edge_pt || !P->edge_kf || !P->edge_obs || !P->edge_inv_sigma2 || !R->edge_erase))
        return ORB_E_INVALID;
    // distinct ids (sorted copies) and one edge per (map point, keyframe): the edges bucketed by
    // point, a keyframe stamp per bucket -- O(edges), no hashing (validation runs on every call)
    // (ids sorted by an LSD radix sort of the sign-flipped keys, three 11-bit passes: O(n))
    auto distinct = [](const int32_t* v, int n) {
        if (n < 2) return true;
        int i0 = 1;   // ids in ascending order (the usual mnId order): distinct by one scan
        while (i0 < n && v[i0 - 1] < v[i0]) i0++;
        if (i0 == n) return true;
        std::vector<uint32_t> c(n), t(n);
        for (int i = 0; i < n; i++) c[i] = (uint32_t)v[i] ^ 0x80000000u;
        uint32_t cnt[2048];
        for (int sh = 0; sh < 32; sh += 11) {
            std::fill(cnt, cnt + 2048, 0u);
            for (int i = 0; i < n; i++) cnt[(c[i] >> sh) & 2047]++;
            uint32_t acc = 0;
            for (int b = 0; b < 2048; b++) {
                const uint32_t k = cnt[b];
                cnt[b] = acc;
                acc += k;
            }
            for (int i = 0; i < n; i++) t[cnt[(c[i] >> sh) & 2047]++] = c[i];
            c.swap(t);
        }
        return std::adjacent_find(c.begin(), c.end()) == c.end();
    };
    if (!distinct(P->kf_id, P->n_kf) || !distinct(P->pt_id, P->n_pt)) return ORB_E_INVALID;
    if (P->n_kf > 32768) return ORB_E_CAPACITY;   // block-sparse pose system: tile map (n_kf / 10.7)^2 ints
    {   // the Optimizer adds each map point's edges together (Optimizer.cc:99-160, 536-627): then one
        // pass with a keyframe stamp per run of equal points checks the pairs; a point met in two
        // runs falls through to the bucketing below
        const int g = grouped_pairs(P);
        if (g == 1) return ORB_E_INVALID;
        if (g == 0) {
            if (grouped) *grouped = true;
            return ORB_OK;
        }
    }
    std::vector<int32_t> start((size_t)P->n_pt + 1, 0);
    for (int i = 0; i < P->n_edge; i++) {
        const int32_t pt = P->edge_pt[i], kf = P->edge_kf[i];
        if (pt < 0 || pt >= P->n_pt || kf < 0 || kf >= P->n_kf) return ORB_E_INVALID;
        start[pt + 1]++;
    }
    for (int p = 0; p < P->n_pt; p++) start[p + 1] += start[p];
    std::vector<int32_t> kfs(std::max(P->n_edge, 1)), fill(start.begin(), start.end() - 1);
    for (int i = 0; i < P->n_edge; i++) kfs[fill[P->edge_pt[i]]++] = P->edge_kf[i];
    std::vector<int32_t> stamp(std::max(P->n_kf, 1), -1);
    for (int p = 0; p < P->n_pt; p++)
        for (int j = start[p]; j < start[p + 1]; j++) {
            if (stamp[kfs[j]] == p) return ORB_E_INVALID;
            stamp[kfs[j]] = p;
        }
    return ORB_OK;
}

int run_ba(const ba_problem* P, const volatile bool* stop, ba_result* R, orbgpu::Comm* comm,
           const orbgpu::BaMode* mode) {
    bool grouped = false;
    if (int v = validate(P, R, &grouped)) return v;
    int rc = 0;
    orbgpu::BaEngine* e = engine(&rc);
    if (rc) return rc == -4 ? ORB_E_NODEVICE : ORB_E_HIP;
    e->edgesGrouped = grouped;
    e->edgesValidated = true;
    const int r = e->run(P, stop, R, comm, mode);
    if (r == -1) return ORB_E_INVALID;
    if (r == -3) return ORB_E_CAPACITY;
    if (r == ORB_E_NODEVICE || r == ORB_E_HIP) return r;
    return r ? ORB_E_HIP : ORB_OK;
}

orbgpu::PoseEngine* pose_engine(int* rc) {
    thread_local orbgpu::PoseEngine* e = nullptr;
    thread_local int erc = 0;
    if (!e) {
        e = new orbgpu::PoseEngine();
        erc = e->init();
    }
    *rc = erc;
    return e;
}
}  // namespace

struct orbgpu_comm_t {};  // opaque: a handle is an orbgpu::Comm*

static orbgpu::Comm* as_comm(orbgpu_comm_h h) { return reinterpret_cast<orbgpu::Comm*>(h); }

extern "C" {

int Optimizer_LocalBundleAdjustment(const ba_problem* P, const volatile bool* stop, ba_result* R) {
    return run_ba(P, stop, R, nullptr, nullptr);
}

int Optimizer_BundleAdjustment(const ba_problem* P, int nIterations, int bRobust, const volatile bool* stop,
                               ba_result* R) {
    if (nIterations < 0) return ORB_E_INVALID;
    orbgpu::BaMode m;
    m.global = true;
    m.iterations = nIterations;
    m.robust = bRobust != 0;
    return run_ba(P, stop, R, nullptr, &m);
}

int Optimizer_LocalBundleAdjustment_sharded(const ba_problem* shard, orbgpu_comm_h comm, const volatile bool* stop,
                                            ba_result* R) {
    if (!comm) return ORB_E_INVALID;
    return run_ba(shard, stop, R, as_comm(comm), nullptr);
}

int Optimizer_BundleAdjustment_sharded(const ba_problem* shard, orbgpu_comm_h comm, int nIterations, int bRobust,
                                       const volatile bool* stop, ba_result* R) {
    if (!comm || nIterations < 0) return ORB_E_INVALID;
    orbgpu::BaMode m;
    m.global = true;
    m.iterations = nIterations;
    m.robust = bRobust != 0;
    return run_ba(shard, stop, R, as_comm(comm), &m);
}

int Optimizer_PoseOptimization_batch(int count, const pose_problem* P, float* Tcw_out, uint8_t* const* outlier,
                                     int* ninliers) {
    if (count < 0 || (count > 0 && (!P || !Tcw_out || !outlier || !ninliers))) return ORB_E_INVALID;
    for (int f = 0; f < count; f++) {
        const pose_problem& Q = P[f];
        if (Q.N < 0 || !Q.Tcw || (!outlier[f] && Q.N > 0)) return ORB_E_INVALID;
        if (Q.N > 0 && (!Q.has_mp || !Q.Xw || !Q.obs || !Q.inv_sigma2)) return ORB_E_INVALID;
    }
    if (count == 0) return ORB_OK;
    int rc = 0;
    orbgpu::PoseEngine* e = pose_engine(&rc);
    if (rc) return rc == -4 ? ORB_E_NODEVICE : ORB_E_HIP;
    const int r = e->run(count, P, Tcw_out, outlier, ninliers);
    if (r == -3) return ORB_E_CAPACITY;
    return r ? ORB_E_HIP : ORB_OK;
}

int Optimizer_PoseOptimization_batch_device(int count, const pose_problem* P, float* const* Tcw_out,
                                            uint8_t* const* outlier, int* ninliers) {
    if (count < 0 || (count > 0 && (!P || !Tcw_out || !outlier || !ninliers))) return ORB_E_INVALID;
    for (int f = 0; f < count; f++) {
        const pose_problem& Q = P[f];
        if (Q.N < 0 || !Q.Tcw || !Tcw_out[f] || (Q.N > 0 && (!outlier[f] || !Q.has_mp || !Q.Xw || !Q.obs ||
                                                             !Q.inv_sigma2)))
            return ORB_E_INVALID;
    }
    if (count == 0) return ORB_OK;
    int rc = 0;
    orbgpu::PoseEngine* e = pose_engine(&rc);
    if (rc) return rc == -4 ? ORB_E_NODEVICE : ORB_E_HIP;
    const int r = e->run_device(count, P, Tcw_out, outlier, ninliers);
    if (r == -3) return ORB_E_CAPACITY;
    return r ? ORB_E_HIP : ORB_OK;
}

int Optimizer_pose_timing(int enable, float* last_ms) {
    int rc = 0;
    orbgpu::PoseEngine* e = pose_engine(&rc);
    if (rc) return rc == -4 ? ORB_E_NODEVICE : ORB_E_HIP;
    if (enable >= 0) e->set_timing(enable != 0);
    if (last_ms) {
        const int r = e->last_timing(last_ms);
        if (r == -1) return ORB_E_INVALID;   // nothing timed yet
        if (r) return ORB_E_HIP;
    }
    return ORB_OK;
}

int Optimizer_PoseOptimization_frames_device(int count, const pose_frame* F, float* const* Tcw_out,
                                             uint8_t* const* outlier, int* ninliers) {
    if (count < 0 || (count > 0 && (!F || !Tcw_out || !outlier || !ninliers))) return ORB_E_INVALID;
    for (int f = 0; f < count; f++) {
        const pose_frame& Q = F[f];
        if (Q.N < 0 || !Q.Tcw || !Tcw_out[f]) return ORB_E_INVALID;
        if (Q.N > 0 && (!outlier[f] || !Q.mp || !Q.mp_pos || !Q.keysUn || !Q.uRight || !Q.invLevelSigma2 ||
                        Q.nlevels <= 0))
            return ORB_E_INVALID;
    }
    if (count == 0) return ORB_OK;
    int rc = 0;
    orbgpu::PoseEngine* e = pose_engine(&rc);
    if (rc) return rc == -4 ? ORB_E_NODEVICE : ORB_E_HIP;
    const int r = e->run_frames_device(count, F, Tcw_out, outlier, ninliers);
    if (r == -3) return ORB_E_CAPACITY;
    return r ? ORB_E_HIP : ORB_OK;
}

int Optimizer_PoseOptimization_frames_device_deferred(ORBmatcher_h chain, int count, const pose_frame* F,
                                                      float* const* Tcw_out, uint8_t* const* outlier,
                                                      int* ninliers) {
    if (!chain || !chain->m->chain().on()) return ORB_E_INVALID;
    if (count < 0 || (count > 0 && (!F || !Tcw_out || !outlier || !ninliers))) return ORB_E_INVALID;
    for (int f = 0; f < count; f++) {
        const pose_frame& Q = F[f];
        if (Q.N < 0 || !Q.Tcw || !Tcw_out[f]) return ORB_E_INVALID;
        if (Q.N > 0 && (!outlier[f] || !Q.mp || !Q.mp_pos || !Q.keysUn || !Q.uRight || !Q.invLevelSigma2 ||
                        Q.nlevels <= 0))
            return ORB_E_INVALID;
    }
    if (count == 0) return ORB_OK;
    int rc = 0;
    orbgpu::PoseEngine* e = pose_engine(&rc);
    if (rc) return rc == -4 ? ORB_E_NODEVICE : ORB_E_HIP;
    orbgpu::Matcher* m = chain->m;
    return e->run_frames_device(count, F, Tcw_out, outlier, ninliers, m->stream(), &m->chain()) ? ORB_E_HIP : ORB_OK;
}

int Optimizer_OptimizeSim3_batch(int count, const sim3opt_problem* P, double* S12, uint8_t* const* erased,
                                 int* nIn) {
    if (count < 0 || (count > 0 && (!P || !S12 || !erased || !nIn))) return ORB_E_INVALID;
    for (int f = 0; f < count; f++) {
        const sim3opt_problem& Q = P[f];
        if (Q.N < 0 || (Q.N > 0 && (!erased[f] || !Q.valid || !Q.X1c || !Q.X2c || !Q.obs1 || !Q.obs2 ||
                                    !Q.inv_sigma2_1 || !Q.inv_sigma2_2)))
            return ORB_E_INVALID;
        if (!(Q.th2 >= 0.f)) return ORB_E_INVALID;
    }
    if (count == 0) return ORB_OK;
    const int r = orbgpu::sim3opt_run(count, P, S12, erased, nIn);
    if (r == -3) return ORB_E_CAPACITY;
    if (r == -4) return ORB_E_NODEVICE;
    return r ? ORB_E_HIP : ORB_OK;
}

int Optimizer_OptimizeSim3(const sim3opt_problem* P, double* S12, uint8_t* erased, int* nIn) {
    uint8_t* e[1] = {erased};
    return Optimizer_OptimizeSim3_batch(1, P, S12, e, nIn);
}

int Optimizer_PoseOptimization(const pose_problem* P, float* Tcw_out, uint8_t* outlier, int* ninliers) {
    if (!P || !Tcw_out || !ninliers) return ORB_E_INVALID;
    uint8_t* const o[1] = {outlier};
    return Optimizer_PoseOptimization_batch(1, P, Tcw_out, o, ninliers);
}

static int block_partition(const ba_problem* P, int nranks, int32_t* pt_rank, std::vector<int32_t>* kfRankOut);

int Optimizer_partition_points(const ba_problem* P, int nranks, int32_t* pt_rank) {
    return block_partition(P, nranks, pt_rank, nullptr);
}

// the keyframe-block partition; kfRankOut (optional) receives every keyframe's block
static int block_partition(const ba_problem* P, int nranks, int32_t* pt_rank, std::vector<int32_t>* kfRankOut) {
    if (!P || nranks < 1 || P->n_kf < 0 || P->n_pt < 0 || P->n_edge < 0) return ORB_E_INVALID;
    if (P->n_pt && !pt_rank) return ORB_E_INVALID;
    if (P->n_edge && (!P->edge_pt || !P->edge_kf)) return ORB_E_INVALID;
    if (P->n_kf && !P->kf_id) return ORB_E_INVALID;
    // reference keyframe of a point = keyframe of its first observation (edge order);
    // keyframe weight = edges of the points it references
    std::vector<int32_t> ref(P->n_pt, -1), nedge(P->n_pt, 0);
    for (int i = 0; i < P->n_edge; i++) {
        const int pt = P->edge_pt[i], kf = P->edge_kf[i];
        if (pt < 0 || pt >= P->n_pt || kf < 0 || kf >= P->n_kf) return ORB_E_INVALID;
        if (ref[pt] < 0) ref[pt] = kf;
        nedge[pt]++;
    }
    std::vector<int64_t> w(P->n_kf, 0);
    int64_t W = 0;
    for (int p = 0; p < P->n_pt; p++)
        if (ref[p] >= 0) {
            w[ref[p]] += nedge[p];
            W += nedge[p];
        }
    // contiguous keyframe blocks in mnId order with ~equal edge weight
    std::vector<int32_t> order(P->n_kf);
    for (int k = 0; k < P->n_kf; k++) order[k] = k;
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return P->kf_id[a] < P->kf_id[b]; });
    std::vector<int32_t> kfRank(P->n_kf, 0);
    int64_t acc = 0;
    for (int32_t k : order) {
        // block of the keyframe = where the middle of its weight falls
        const int64_t mid2 = 2 * acc + w[k];
        int r = W > 0 ? (int)((mid2 * nranks) / (2 * W)) : 0;
        kfRank[k] = std::min(std::max(r, 0), nranks - 1);
        acc += w[k];
    }
    for (int p = 0; p < P->n_pt; p++) pt_rank[p] = ref[p] >= 0 ? kfRank[ref[p]] : 0;
    if (kfRankOut) *kfRankOut = std::move(kfRank);
    return ORB_OK;
}

int Optimizer_partition_points_nd(const ba_problem* P, int nranks, int32_t* pt_rank, int32_t* kf_owner) {
    if (!P || nranks < 1 || P->n_kf < 0 || P->n_pt < 0 || P->n_edge < 0) return ORB_E_INVALID;
    if (P->n_pt && !pt_rank) return ORB_E_INVALID;
    if (P->n_edge && (!P->edge_pt || !P->edge_kf)) return ORB_E_INVALID;
    if (P->n_kf && !P->kf_id) return ORB_E_INVALID;
    if (P->n_pt && !P->pt_id) return ORB_E_INVALID;
    const int nkf = P->n_kf, npt = P->n_pt, ne = P->n_edge;
    for (int i = 0; i < ne; i++)
        if (P->edge_pt[i] < 0 || P->edge_pt[i] >= npt || P->edge_kf[i] < 0 || P->edge_kf[i] >= nkf)
            return ORB_E_INVALID;
    // BundleAdjustment's structure at level 0 (every keyframe a vertex, fixed iff mnId == 0):
    // the pose numbering and Schur blocks every rank's engine derives from the union of shards
    std::vector<int32_t> eKf(P->edge_kf, P->edge_kf + ne), ePt(P->edge_pt, P->edge_pt + ne);
    std::vector<int32_t> kfId(P->kf_id, P->kf_id + nkf), ptId(P->pt_id, P->pt_id + npt);
    std::vector<uint8_t> kfFixed(nkf), level(ne, 0), kfAct, ptAct;
    for (int k = 0; k < nkf; k++) kfFixed[k] = P->kf_id[k] == 0 ? 1 : 0;
    orbgpu::BaHostStruct H;
    orbgpu::ba_active_set(0, nkf, npt, ne, eKf.data(), ePt.data(), level.data(), &H.aE, &kfAct, &ptAct);
    if (orbgpu::ba_build_lists(nkf, npt, eKf.data(), ePt.data(), kfFixed.data(), kfId.data(), ptId.data(), kfAct, ptAct,
                               &H))
        return ORB_E_INVALID;
    const int nP = (int)H.poseKf.size();
    if (kf_owner)
        for (int k = 0; k < nkf; k++) kf_owner[k] = -2;   // not a free pose of the structure
    if (nranks == 1 || nP < orbgpu::kBaTiledMinPoses) {   // no block-sparse factorisation to shard:
        std::vector<int32_t> kfRank;                       // the keyframe-block partition, and a
        if (int e = block_partition(P, nranks, pt_rank, &kfRank)) return e;   // free pose's owner
        if (kf_owner)                                      // is its keyframe's block
            for (int32_t k : H.poseKf) kf_owner[k] = kfRank[k];
        return ORB_OK;
    }
    // the pose graph of the Schur blocks, as BaEngine::build_structure forms it
    std::vector<int64_t> keys;
    for (size_t b = 0; b < H.blkI.size(); b++)
        if (H.blkI[b] != H.blkJ[b]) keys.push_back((int64_t)H.blkI[b] * nP + H.blkJ[b]);
    std::sort(keys.begin(), keys.end());
    keys.erase(std::unique(keys.begin(), keys.end()), keys.end());
    std::vector<int> deg(nP + 1, 0), as(nP + 1, 0), adj(2 * keys.size());
    for (int64_t q : keys) {
        deg[q / nP]++;
        deg[q % nP]++;
    }
    for (int i = 0; i < nP; i++) as[i + 1] = as[i] + deg[i];
    std::vector<int> fillp(as.begin(), as.end() - 1);
    for (int64_t q : keys) adj[fillp[q / nP]++] = (int)(q % nP);
    for (int64_t q : keys) adj[fillp[q % nP]++] = (int)(q / nP);
    for (int i = 0; i < nP; i++) std::sort(adj.begin() + as[i], adj.begin() + as[i + 1]);
    orbgpu::NdTree tree;
    orbgpu::nd_order(nP, as, adj, orbgpu::kNdLeafPoses, &tree);
    std::vector<int> owner;
    orbgpu::nd_assign(tree, nranks, &owner);
    std::vector<int> poseOwner(nP, -1);
    for (size_t k = 0; k < tree.start.size(); k++)
        for (int q = tree.start[k]; q < tree.end[k]; q++) poseOwner[tree.perm[q]] = owner[k];
    if (kf_owner)
        for (int q = 0; q < nP; q++) kf_owner[H.poseKf[q]] = poseOwner[q];
    // a point goes to the rank of the first subtree pose it observes (all of its poses are in
    // that subtree or the separators above it); a point of separator poses only, round robin
    std::vector<int32_t> landOf(npt, -1);
    for (size_t l = 0; l < H.landPt.size(); l++) landOf[H.landPt[l]] = (int32_t)l;
    int rr = 0;
    for (int p = 0; p < npt; p++) {
        int r = -1;
        const int l = landOf[p];
        if (l >= 0)
            for (int q = H.lpStart[l]; q < H.lpStart[l + 1] && r < 0; q++) {
                const int pose = H.ePose[H.lpList[q]];
                if (pose >= 0) r = poseOwner[pose];
            }
        if (r < 0) r = rr++ % nranks;
        pt_rank[p] = r;
    }
    return ORB_OK;
}

int orbgpu_comm_unique_id(uint8_t* id) {
    if (!id) return ORB_E_INVALID;
    return orbgpu::rccl_unique_id(id);
}

int orbgpu_comm_init_rccl(int nranks, int rank, const uint8_t* id, orbgpu_comm_h* out) {
    if (!id || !out || nranks < 1 || rank < 0 || rank >= nranks) return ORB_E_INVALID;
    int rc = 0;
    orbgpu::Comm* c = orbgpu::rccl_comm_create(nranks, rank, id, &rc);
    *out = reinterpret_cast<orbgpu_comm_h>(c);
    return rc;
}

int orbgpu_comm_init_local(int nranks, orbgpu_comm_h* out) {
    if (!out || nranks < 1 || nranks > 64) return ORB_E_INVALID;
    std::vector<orbgpu::Comm*> v = orbgpu::local_comm_group(nranks);
    for (int r = 0; r < nranks; r++) out[r] = reinterpret_cast<orbgpu_comm_h>(v[r]);
    return ORB_OK;
}

int orbgpu_comm_init_shm(const char* name, int nranks, int rank, size_t max_doubles, orbgpu_comm_h* out) {
    if (!out) return ORB_E_INVALID;
    int rc = 0;
    orbgpu::Comm* c = orbgpu::shm_comm_create(name, nranks, rank, max_doubles, &rc);
    *out = reinterpret_cast<orbgpu_comm_h>(c);
    return rc;
}

int orbgpu_comm_rank(orbgpu_comm_h h, int* rank, int* size) {
    if (!h) return ORB_E_INVALID;
    if (rank) *rank = as_comm(h)->rank();
    if (size) *size = as_comm(h)->size();
    return ORB_OK;
}

int orbgpu_comm_destroy(orbgpu_comm_h h) {
    delete as_comm(h);
    return ORB_OK;
}

int Optimizer_last_trace(double* solve_ini_chi2, double* solve_chi2, int solve_cap, int* n_solves,
                         double* trial_chi2, double* trial_lambda, int trial_cap, int* n_trials) {
    int rc = 0;
    orbgpu::BaEngine* e = engine(&rc);
    if (rc) return rc == -4 ? ORB_E_NODEVICE : ORB_E_HIP;
    const orbgpu::BaTrace& t = e->trace();
    const int ns = (int)t.solve_chi2.size(), nt = (int)t.trial_chi2.size();
    if (n_solves) *n_solves = ns;
    if (n_trials) *n_trials = nt;
    for (int i = 0; i < std::min(ns, solve_cap); i++) {
        if (solve_ini_chi2) solve_ini_chi2[i] = t.solve_ini_chi2[i];
        if (solve_chi2) solve_chi2[i] = t.solve_chi2[i];
    }
    for (int i = 0; i < std::min(nt, trial_cap); i++) {
        if (trial_chi2) trial_chi2[i] = t.trial_chi2[i];
        if (trial_lambda) trial_lambda[i] = t.trial_lambda[i];
    }
    return ORB_OK;
}

int Optimizer_last_sharding(int* info4) {
    if (!info4) return ORB_E_INVALID;
    int rc = 0;
    orbgpu::BaEngine* e = engine(&rc);
    if (rc) return rc == -4 ? ORB_E_NODEVICE : ORB_E_HIP;
    for (int i = 0; i < 4; i++) info4[i] = e->last_dist[i];
    return ORB_OK;
}

int Optimizer_last_lm_path(int* info4) {
    if (!info4) return ORB_E_INVALID;
    int rc = 0;
    orbgpu::BaEngine* e = engine(&rc);
    if (rc) return rc == -4 ? ORB_E_NODEVICE : ORB_E_HIP;
    for (int i = 0; i < 4; i++) info4[i] = e->last_lm[i];
    return ORB_OK;
}

int Optimizer_last_timings(double* ms2) {
    if (!ms2) return ORB_E_INVALID;
    int rc = 0;
    orbgpu::BaEngine* e = engine(&rc);
    if (rc) return rc == -4 ? ORB_E_NODEVICE : ORB_E_HIP;
    ms2[0] = e->last_ms[0];
    ms2[1] = e->last_ms[1];
    return ORB_OK;
}

int orbgpu_unit_ldlt_solve(int n, const double* S, const double* b, double* x, int variant, int* ok) {
    if (n < 0 || (n > 0 && (!S || !b || !x)) || !ok) return ORB_E_INVALID;
    int rc = 0;
    engine(&rc);
    if (rc) return rc == -4 ? ORB_E_NODEVICE : ORB_E_HIP;
    const int r = orbgpu::debug_ldlt(n, S, b, x, variant);
    if (r < 0) return r == -3 ? ORB_E_CAPACITY : ORB_E_HIP;
    *ok = r;
    return ORB_OK;
}

int orbgpu_unit_ldlt_factor(int n, const double* S, double* out) {
    if (n < 0 || (n > 0 && (!S || !out))) return ORB_E_INVALID;
    int rc = 0;
    engine(&rc);
    if (rc) return rc == -4 ? ORB_E_NODEVICE : ORB_E_HIP;
    return orbgpu::debug_ldlt_factor(n, S, out) ? ORB_E_HIP : ORB_OK;
}

int orbgpu_debug_prof(unsigned long long* out32) { return out32 ? orbgpu::debug_prof(out32) : ORB_E_INVALID; }
int orbgpu_debug_prof_extract(unsigned long long* out32) {
    return out32 ? orbgpu::debug_prof_extract(out32) : ORB_E_INVALID;
}
int orbgpu_debug_prof_match(unsigned long long* out32) {
    return out32 ? orbgpu::debug_prof_match(out32) : ORB_E_INVALID;
}

int orbgpu_unit_nd_order(int n, const int32_t* adjStart, const int32_t* adj, int leaf, int32_t* perm,
                         int32_t* n_nodes, int32_t* height) {
    if (n < 0 || leaf < 1 || (n > 0 && (!adjStart || !adj || !perm))) return ORB_E_INVALID;
    // the lists must be a well-formed CSR graph: offsets from 0, non-decreasing, every neighbour
    // in [0, n) and no self loop (nd_order indexes its marks with them unchecked)
    if (n > 0) {
        if (adjStart[0] != 0) return ORB_E_INVALID;
        for (int i = 0; i < n; i++) {
            if (adjStart[i + 1] < adjStart[i]) return ORB_E_INVALID;
            for (int e = adjStart[i]; e < adjStart[i + 1]; e++)
                if (adj[e] < 0 || adj[e] >= n || adj[e] == i) return ORB_E_INVALID;
        }
    }
    std::vector<int> as(adjStart, adjStart + n + 1), ad(adj, adj + (n > 0 ? adjStart[n] : 0));
    orbgpu::NdTree t;
    orbgpu::nd_order(n, as, ad, leaf, &t);
    for (int i = 0; i < n; i++) perm[i] = t.perm[i];
    if (n_nodes) *n_nodes = (int32_t)t.start.size();
    if (height) {
        int h = 0;
        for (int v : t.height) h = std::max(h, v);
        *height = h;
    }
    return ORB_OK;
}

int orbgpu_unit_set_csum_lds_max(int m2_max) {
    if (m2_max < 0 || m2_max > 1024) return ORB_E_INVALID;
    return orbgpu::debug_set_csum_lds_max(m2_max) ? ORB_E_HIP : ORB_OK;
}

int orbgpu_unit_set_scale_small_max(int terms) {
    return orbgpu::debug_set_scale_small_max(terms) ? ORB_E_INVALID : ORB_OK;
}
int orbgpu_unit_set_posegraph_check(int on) {
    return orbgpu::debug_set_posegraph_check(on);
}

int orbgpu_unit_set_struct_gpu_min_edges(int edges) {
    return orbgpu::debug_set_struct_gpu_min_edges(edges) ? ORB_E_INVALID : ORB_OK;
}

int orbgpu_unit_ba_struct(int nkf, int npt, int ne, const int32_t* edge_kf, const int32_t* edge_pt,
                          const uint8_t* edge_level, const uint8_t* kf_fixed, const int32_t* kf_id,
                          const int32_t* pt_id, int level, int32_t* out, long long cap) {
    if (nkf < 0 || npt < 0 || ne < 0 || !out || cap < 5) return ORB_E_INVALID;
    if ((ne && (!edge_kf || !edge_pt || !edge_level)) || (nkf && (!kf_fixed || !kf_id)) || (npt && !pt_id))
        return ORB_E_INVALID;
    for (int i = 0; i < ne; i++)
        if (edge_kf[i] < 0 || edge_kf[i] >= nkf || edge_pt[i] < 0 || edge_pt[i] >= npt) return ORB_E_INVALID;
    orbgpu::BaHostStruct S;
    std::vector<uint8_t> kfAct, ptAct;
    orbgpu::ba_active_set(level, nkf, npt, ne, edge_kf, edge_pt, edge_level, &S.aE, &kfAct, &ptAct);
    if (orbgpu::ba_build_lists(nkf, npt, edge_kf, edge_pt, kf_fixed, kf_id, pt_id, kfAct, ptAct, &S)) return ORB_E_INVALID;
    const int nE = (int)S.aE.size(), nP = (int)S.poseKf.size(), nL = (int)S.landPt.size();
    const int nBlk = (int)S.blkI.size(), nPair = S.blkStart[nBlk];
    // [nE nP nL nBlk nPair | poseKf | landPt | ePose | eLand | lpStart | lpList | blkI | blkJ | blkStart | pairA | pairB]
    const long long need = 5LL + nP + nL + 2LL * nE + (nL + 1) + S.lpStart[nL] + 2LL * nBlk + (nBlk + 1) + 2LL * nPair;
    if (need > cap) return ORB_E_CAPACITY;
    int32_t* o = out;
    *o++ = nE; *o++ = nP; *o++ = nL; *o++ = nBlk; *o++ = nPair;
    auto put = [&](const std::vector<int32_t>& v, size_t n) { o = std::copy(v.begin(), v.begin() + n, o); };
    put(S.poseKf, nP); put(S.landPt, nL); put(S.ePose, nE); put(S.eLand, nE); put(S.lpStart, nL + 1);
    put(S.lpList, S.lpStart[nL]); put(S.blkI, nBlk); put(S.blkJ, nBlk); put(S.blkStart, nBlk + 1);
    put(S.pairA, nPair); put(S.pairB, nPair);
    return ORB_OK;
}

int orbgpu_unit_ba_struct_all(int nkf, int npt, int ne, const int32_t* edge_kf, const int32_t* edge_pt,
                              const uint8_t* edge_level, const uint8_t* kf_fixed, const int32_t* kf_id,
                              const int32_t* pt_id, int level, int gpu, int32_t* out, long long cap, long long* n_out) {
    if (nkf < 0 || npt < 0 || ne < 0 || !out || !n_out) return ORB_E_INVALID;
    if ((ne && (!edge_kf || !edge_pt || !edge_level)) || (nkf && (!kf_fixed || !kf_id)) || (npt && !pt_id))
        return ORB_E_INVALID;
    for (int i = 0; i < ne; i++)
        if (edge_kf[i] < 0 || edge_kf[i] >= nkf || edge_pt[i] < 0 || edge_pt[i] >= npt) return ORB_E_INVALID;
    if (gpu) {
        int rc = 0;
        engine(&rc);
        if (rc) return rc == -4 ? ORB_E_NODEVICE : ORB_E_HIP;
    }
    std::vector<int32_t> v;
    const int r = orbgpu::debug_struct_all(nkf, npt, ne, edge_kf, edge_pt, edge_level, kf_fixed, kf_id, pt_id, level,
                                           gpu, &v);
    if (r == -1) return ORB_E_INVALID;
    if (r) return ORB_E_HIP;
    *n_out = (long long)v.size();
    if ((long long)v.size() > cap) return ORB_E_CAPACITY;
    std::copy(v.begin(), v.end(), out);
    return ORB_OK;
}

int orbgpu_unit_wave_tree(const double* v64, double* out) {
    if (!v64 || !out) return ORB_E_INVALID;
    int rc = 0;
    engine(&rc);
    if (rc) return rc == -4 ? ORB_E_NODEVICE : ORB_E_HIP;
    return orbgpu::debug_wave_tree(v64, out) ? ORB_E_HIP : ORB_OK;
}

int orbgpu_unit_shared_div(const double* a, const double* b, int n, double* out) {
    if (!a || !b || !out || n < 0) return ORB_E_INVALID;
    int rc = 0;
    engine(&rc);
    if (rc) return rc == -4 ? ORB_E_NODEVICE : ORB_E_HIP;
    return orbgpu::debug_shared_div(a, b, n, out) ? ORB_E_HIP : ORB_OK;
}

int orbgpu_unit_csum(const double* v, int n, double* out) {
    if (n < 0 || (n > 0 && !v) || !out) return ORB_E_INVALID;
    int rc = 0;
    engine(&rc);
    if (rc) return rc == -4 ? ORB_E_NODEVICE : ORB_E_HIP;
    return orbgpu::debug_csum(v, n, out) ? ORB_E_HIP : ORB_OK;
}

}  // extern "C"
