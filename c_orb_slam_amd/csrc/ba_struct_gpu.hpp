// ba_struct_gpu.hpp -- initializeOptimization(level) + buildIndexMapping +
// BlockSolver::buildStructure (g2o sparse_optimizer.cpp:198-287, block_solver.hpp:139-216) on the
// device: every list BaStructDev points at, identical to the host restatement (ba_struct.cpp),
// built from the edges already in HBM with stable radix sorts, scans and compactions.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <functional>
#include <vector>

#include "ba_types.hpp"

namespace orbgpu {

class Comm;

struct GpuStructInfo {
    int nE, nP, nL, nBlk, nPair, nLp, nPe, nLe;
    int err;                    // bit 0: a landmark with two edges to one pose
    int maxPe, maxLe, maxBlk;   // longest per-pose / per-landmark / per-block list
    int nEglob, nLglob;         // over the shards (comm); == nE, nL otherwise
    int posDone;                // build_small with pePos: pePos written, pairs are pose-list positions
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
    // The same lists from ONE workgroup (local-BA sizes: <= 1,024 keyframes, <= 8,192 points,
    // <= 16,384 edges, <= 23 free active poses, <= 256 edges per landmark), the counts polled from
    // pinned memory.  pePos (optional, >= ne entries): the pose-list position of every active edge
    // (-1 on fixed keyframes) written too, and pairA / pairB as pose-list positions.  Returns 0,
    // 1 (outside the limits: nothing usable, run build()), -1 (duplicate edge) or -2 (HIP).
    // Unsharded only.
    // Inputs: dKp[e] = (keyframe << 13) | point per edge, dPtOrd = every point by (mnId, index)
    // (ba_order_by_id); dLevel null = every edge at `level`.  afterLaunch (optional) runs right
    // after the kernel is queued, before the wait for its counts.
    int build_small(int level, int nkf, int npt, int ne, const int32_t* dKp, const int32_t* dPtOrd,
                    const uint8_t* dLevel, const uint8_t* dKfFixed, const int32_t* dKfId, int32_t* pePos, hipStream_t s,
                    BaStructDev* st, GpuStructInfo* info, const std::function<int()>& afterLaunch = nullptr);
    static bool small_fits(int nkf, int npt, int ne, int nFreeKf);
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
    volatile int* hSig_ = nullptr;   // pinned coherent: build_small's counts and sequence word
    int sigSeq_ = 0;
    BaStructDev last_{};
    int nkf_ = 0, nP_ = 0, nPair_ = 0, nOff_ = 0;
};

// build_small's size limits without the pose count (<= 1,024 keyframes, <= 8,192 points, <= 16,384 edges)
bool small_inputs_fit(int nkf, int npt, int ne);

// both builders on one level (unit entry orbgpu_unit_ba_struct_all): [nE nP nL nBlk nPair nPe nLe nLp |
// the 16 lists]; gpu = 0: the host restatement, 1: build(), 2: build_small() (build() outside
// its limits).  0, -1 (duplicate edge) or -2 (HIP).
int debug_struct_all(int nkf, int npt, int ne, const int32_t* eKf, const int32_t* ePt, const uint8_t* lv,
                     const uint8_t* kfFixed, const int32_t* kfId, const int32_t* ptId, int level, int gpu,
                     std::vector<int32_t>* out);

}  // namespace orbgpu
