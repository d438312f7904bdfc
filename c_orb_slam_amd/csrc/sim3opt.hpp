// sim3opt.hpp -- Optimizer::OptimizeSim3 (reference src/Optimizer.cc:1046-1241) on gfx950.
#pragma once
#include <cstdint>

#include "../../include/orbslam_gpu.h"

namespace orbgpu {
// 0 ok, -3 capacity (> 2048 valid correspondences), -4 no device, other < 0: HIP error
int sim3opt_run(int count, const sim3opt_problem* P, double* S12, uint8_t* const* erased, int* nIn);
}  // namespace orbgpu
