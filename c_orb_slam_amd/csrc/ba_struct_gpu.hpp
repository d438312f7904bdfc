// ba_struct_gpu.hpp -- initializeOptimization(level) + buildIndexMapping +
// BlockSolver::buildStructure (g2o sparse_optimizer.cpp:198-287, block_solver.hpp:139-216) on the
// device: every list BaStructDev points at, identical to the host restatement (ba_struct.cpp),
// built from the edges already in HBM with stable radix sorts, scans and compactions.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

#include "ba_types.hpp"

namespace orbgpu {

class Comm;

struct GpuStructInfo {
    int nE, nP, nL, nBlk, nPair, nLp, nPe, nLe;
    int err;                    // bit 0: a landmark with two edges to one pose
    int maxPe, maxLe, maxBlk;   // longest per-pose / per-landmark / per-block list
    int nEglob, nLglob;         // over the shards (comm); == nE, nL otherwise
};

class GpuStructBuilder {
public:
    ~GpuStructBuilder();
    // Lists of the active edges of `level` into this builder's buffers; *st gets their device
    // pointers and counts.  comm: the keyframe activity and the global counts are reduced over
    // the shards (every shard orders the same pose set).  blkIJ (optional): blkI ++ blkJ on the
    // host.  Returns 0, -1 (a landmark with two edges to one pose) or -2 (HIP).
    int build(int level, int nkf, int npt, int ne, const EdgeDev* dE, const uint8_t* dLevel, const uint8_t* dKfFixed,
              const int32_t* dKfId, const int32_t* dPtId, Comm* comm, hipStream_t s, BaStructDev* st,
              GpuStructInfo* info, std::vector<int32_t>* blkIJ = nullptr);
    // after build(): the off-diagonal Schur blocks as i1 * nP + i2, ascending (the pose graph)
    int offkeys(std::vector<int64_t>* out, hipStream_t s);
    // the lists of the last build, back on the host, in one buffer:
    // [aE | ePose | eLand | poseKf | landPt | peStart | peList | leStart | leList | lpStart | lpList |
    //  blkI | blkJ | blkStart | pairA | pairB]
    int download(const GpuStructInfo& info, std::vector<int32_t>* out, hipStream_t s);

private:
    void* buf(int slot, size_t bytes);
    static constexpr int kSlots = 64;
    void* p_[kSlots] = {};
    size_t cap_[kSlots] = {};
    int* hSc_ = nullptr;   // pinned scalar mirror
    BaStructDev last_{};
    int nkf_ = 0, nP_ = 0, nPair_ = 0, nOff_ = 0;
};

// both builders on one level (unit entry orbgpu_unit_ba_struct_all): [nE nP nL nBlk nPair nPe nLe nLp |
// the 16 lists]; gpu = 0: the host restatement.  0, -1 (duplicate edge) or -2 (HIP).
int debug_struct_all(int nkf, int npt, int ne, const int32_t* eKf, const int32_t* ePt, const uint8_t* lv,
                     const uint8_t* kfFixed, const int32_t* kfId, const int32_t* ptId, int level, int gpu,
                     std::vector<int32_t>* out);

}  // namespace orbgpu
