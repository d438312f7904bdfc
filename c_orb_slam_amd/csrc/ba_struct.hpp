// ba_struct.hpp -- host side of initializeOptimization(level) + buildIndexMapping +
// BlockSolver::buildStructure (g2o sparse_optimizer.cpp:198-287, block_solver.hpp:73-216):
// the active edge set of one optimisation level, vertex index maps and every list the BA
// kernels walk (ba.hip).  Pure C++, no device calls: BaEngine::build_structure packs the
// result and uploads it once per structure.
#pragma once
#include <cstdint>
#include <vector>

namespace orbgpu {

struct BaHostStruct {
    // aE: active edge -> edge; ePose / eLand: active edge -> pose index (-1 fixed) / landmark
    // poseKf / landPt: index -> keyframe / point (ascending mnId)
    // peStart/peList: pose -> active edges (edge order); leStart/leList: landmark -> active
    // edges (edge order); lpStart/lpList: landmark -> active edges with a free pose (pose order)
    // blkI/blkJ: Schur blocks (diagonal first, then first use in landmark order);
    // blkStart/pairA/pairB: per block, the landmark terms (landmark order)
    std::vector<int32_t> aE, ePose, eLand, poseKf, landPt, peStart, peList, leStart, leList, lpStart, lpList, blkI,
        blkJ, blkStart, pairA, pairB;
};

// Active edges of `level` and the vertices they touch.
void ba_active_set(int level, int nkf, int npt, int ne, const int32_t* eKf, const int32_t* ePt, const uint8_t* edgeLevel,
                   std::vector<int32_t>* aE, std::vector<uint8_t>* kfAct, std::vector<uint8_t>* ptAct);

// The index maps and lists of an active set.  kfAct may be the union over shards.  Returns 0,
// or -1 when a landmark has two edges to one pose (g2o would build a duplicate Hpl block).
// every index 0..n-1 ascending by (id[i], i): the vertex order of buildIndexMapping before the
// active-set filter (the one-workgroup device builder's input)
void ba_order_by_id(int n, const int32_t* id, std::vector<int32_t>* out);

int ba_build_lists(int nkf, int npt, const int32_t* eKf, const int32_t* ePt, const uint8_t* kfFixed,
                   const int32_t* kfId, const int32_t* ptId, const std::vector<uint8_t>& kfAct,
                   const std::vector<uint8_t>& ptAct, BaHostStruct* S, bool checkDup = true);

// The Schur pattern from built lp lists (ba_build_lists' last phases).
int ba_build_blocks(int nP, int nL, const int32_t* qs, const int32_t* ql, const int32_t* qp, BaHostStruct* S);

// The lists of `level` from an earlier structure A of the same problem whose active edges are a
// superset (the second LocalBundleAdjustment pass after the outlier gating): A's lists filtered,
// the Schur pattern renumbered.  Same lists as ba_active_set + ba_build_lists.
int ba_refine_lists(const BaHostStruct& A, const uint8_t* edgeLevel, int level, BaHostStruct* S);

}  // namespace orbgpu
