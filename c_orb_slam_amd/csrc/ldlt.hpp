// ldlt.hpp -- tiled multi-workgroup LDL^T solve of the reduced pose system (see ldlt.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>

namespace orbgpu {
size_t ldlt_tiled_workspace(int n);
// A: n x n row-major (upper = S, strict lower must be 0), factorised in place.
// scal[3] = 1 on success (x written), 0 on a zero pivot (x untouched).
int ldlt_tiled_solve(int n, double* A, const double* b, double* x, double* scal, void* ws, hipStream_t s);
}  // namespace orbgpu
