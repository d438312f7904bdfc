// octree.hpp -- gfx950 DistributeOctTree (see octree.hip).  Reference: src/ORBextractor.cc:481-763.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "orb_common.hpp"

namespace orbgpu {

constexpr int kOctNMax = 640;    // live octree nodes per (image, level): nFeaturesPerLevel + 8 <= kOctNMax
constexpr int kOctKMax = 4096;   // keys per job held in LDS; larger jobs use the global scratch

struct OctLevelDev {   // DistributeOctTree(vToDistributeKeys, minX, maxX, minY, maxY, N, level)
    int minX, maxX, minY, maxY, N;
};

// k_octree over B * nlevels jobs, then k_sel_build: sel[b * selcap + k] = (packed, b<<20|l<<16|k),
// nout[b].  err bits: 1 capacity (cap / selcap), 2 > 65535 keys, 4 bad geometry, 8 node pool,
// 16 job capacity.
// instrumented builds (make prof): k_octree section cycles of job 0 into out16, then reset
int octree_prof_read(unsigned long long* out16);

// The FAST output a job reads (k_fast_cells): cell c of image b holds counts[b * ncells + c]
// candidates at slots[b * slots_per_image + cell_slot[c]]; level l's cells are [lcb[l], lcb[l+1]).
// Each job compacts its level's cells, in cell order (the reference's vToDistributeKeys order),
// into packed at the level's own slot range (disjoint per job), and adds its count to g_total.
struct OctInput {
    const uint32_t* slots;
    size_t slots_per_image;
    const int* counts;
    const int* cell_slot;
    const int* lcb;
    int ncells;
    uint32_t* packed;
    int* g_total;
};

int octree_launch(const OctInput& in, int B, int nlevels, const OctLevelDev* lv, uint32_t* jobsel, int* jobcnt, int jcap,
                  uint16_t* gscratch, size_t gstride, int cap, int2* sel, int selcap, int* nout, int* err,
                  hipStream_t s);

}  // namespace orbgpu
