// ba_types.hpp -- the BA problem's edge record and the per-level structure the kernels walk
// (shared by ba.hip and the device structure builder, ba_struct_gpu.hip).
#pragma once
#include <cstdint>

namespace orbgpu {

struct alignas(16) EdgeDev {  // one g2o edge (vertex 0 = point, vertex 1 = keyframe pose); 16-B aligned: 16-B loads
    double obs[3];
    double info;            // invSigma2 (float -> double)
    double fx, fy, cx, cy, bf;
    double delta, dsqr;     // RobustKernelHuber: delta = (double)(float)sqrt(th)
    int32_t pt, kf;
    int32_t stereo, pad;
};

// per-phase active structure (initializeOptimization + buildIndexMapping + buildStructure)
struct BaStructDev {
    int nE, nP, nL, nBlk;
    const int32_t* aE;        // active edge -> edge
    const int32_t* ePose;     // active edge -> pose index or -1 (fixed keyframe)
    const int32_t* eLand;     // active edge -> landmark index
    const int32_t* poseKf;    // pose index -> keyframe
    const int32_t* landPt;    // landmark index -> point
    const int32_t* peStart;   // pose -> active edges (edge order)
    const int32_t* peList;
    const int32_t* leStart;   // landmark -> active edges (edge order)
    const int32_t* leList;
    const int32_t* lpStart;   // landmark -> active edges with a free pose (pose order)
    const int32_t* lpList;
    const int32_t* blkI;      // Schur blocks (i1 <= i2), diagonal blocks always present
    const int32_t* blkJ;
    const int32_t* blkStart;  // block -> pair terms (landmark order)
    const int32_t* pairA;     // active edge of the landmark to pose i1 (BaEngine: its pose-list position)
    const int32_t* pairB;     // active edge of the landmark to pose i2 (BaEngine: its pose-list position)
    // BaEngine only: active edge -> its position in peList (-1: fixed pose), and nPe = peStart[nP].
    // A free-pose edge's pose terms, Hpl, Emat and c_b live at that position, so every per-pose
    // walk (the pose reduction, a Schur block's terms in landmark order) reads consecutive records.
    const int32_t* pePos;
    int nPe;
};

}  // namespace orbgpu
