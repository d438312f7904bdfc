// ldlt.hip -- tiled multi-workgroup dense LDL^T solve of the reduced pose system S x = b_s
// for large bundle adjustments (reference: g2o LinearSolverEigen, SimplicialLDLT,
// Thirdparty/g2o/g2o/solvers/linear_solver_eigen.h:104; restated in oracle/ba.c
// ora_ldlt_solve).
//
// Per-element operation sequence is the oracle's: pivot k ascending, d_k = A[k][k],
// l_i = A[k][i] / d_k, A[i][j] -= l_i * A[k][j] (j >= i), no FMA contraction; forward
// y_i -= L[i][k] y_k in k order, y_k /= d_k, backward y_i -= L[k][i] y_k in descending k.
// Work is skipped at 64x64-tile granularity where the L tile is exactly zero, which is the
// oracle's `l == 0` envelope skip (exact up to the sign of zero): a banded / block-sparse
// Schur complement (keyframes observe nearby keyframes' points) costs O(n bw^2), not n^3/3.
//
// Layout: A row-major n x n in HBM, upper triangle = S on entry; on exit the diagonal holds
// d, the strict lower triangle holds L, the upper triangle the eliminated rows.  Per panel p
// (64 pivots):
//   k_ldlt_panel  grid = column tiles J >= p: every workgroup refactors the 64x64 diagonal
//                 block in LDS (redundantly), applies the panel pivots to its 64-column
//                 chunk of the panel rows, writes L for its chunk and the tile's nonzero flag;
//   k_ldlt_trail  grid = trailing tiles (I <= J): A[I][J] -= L[I][p] U[p][J], k in order,
//                 4x4 register micro-tiles over LDS-staged L / U tiles; zero tiles exit.
// Solves: one launch each, a workgroup (one wave) per 64-row block; a block consumes the
// finished blocks it depends on in order, spinning on their done flags (blocks are
// dispatched in dependency order, so a waiting block's producers are resident or done).
#include <hip/hip_runtime.h>

#include <cstdint>

#include "ldlt.hpp"
#include "orb_common.hpp"

namespace orbgpu {

constexpr int LT = 64;          // tile edge
constexpr int LP = LT + 1;      // LDS row pitch (doubles)

__device__ __forceinline__ double rdlane(double v, int l) {
    const unsigned long long u = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)(u & 0xffffffffu), l);
    const int hi = __builtin_amdgcn_readlane((int)(u >> 32), l);
    return __longlong_as_double(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}

// One wave per workgroup; lane j owns column j of a 64-row block in registers.
// Phase 1 (every workgroup, redundantly): factorise the diagonal block -- at pivot k lane i
// forms l_ik = D[k][i] / d_k from its own column, and lane j applies D[i][j] -= l_i D[k][j]
// to its column (rows k < i <= j) with l_i broadcast by readlane.  Phase 2 (J > p): the
// same pivots on the chunk columns, l_ik broadcast from LDS (uniform `l != 0` skip).
__global__ void __launch_bounds__(64) k_ldlt_panel(int n, int p, double* __restrict__ A, uint8_t* nz, int nt,
                                                   int* fail, double* dstage) {
    __shared__ double Ls[LT * LP];   // Ls[k * LP + i] = l_ik ; reused as the L transpose buffer
    __shared__ double dvs[LT];
    if (*fail) return;
    const int lane = threadIdx.x;
    const int p0 = p * LT, pw = min(LT, n - p0);
    const int J = p + blockIdx.x, J0 = J * LT, cw = min(LT, n - J0);
    const bool diag = J == p;
    double* Ap = A + (size_t)p0 * n;   // panel rows
    if (!diag) {   // an all-zero chunk stays zero and its L stays zero (A is pre-cleared)
        bool nzc = false;
        for (int r0 = 0; r0 < pw; r0 += 16) {
            double v[16];
#pragma unroll
            for (int u = 0; u < 16; u++) v[u] = (r0 + u < pw && lane < cw) ? Ap[(size_t)(r0 + u) * n + J0 + lane] : 0.0;
#pragma unroll
            for (int u = 0; u < 16; u++) nzc |= v[u] != 0.0;
        }
        if (!__any(nzc)) {
            if (lane == 0) nz[(size_t)J * nt + p] = 0;
            return;
        }
    }
    double col[LT];
#pragma unroll
    for (int r = 0; r < LT; r++)
        col[r] = (r < pw && lane < pw && r <= lane) ? Ap[(size_t)r * n + p0 + lane] : 0.0;
    bool bad = false;
#pragma unroll
    for (int k = 0; k < LT; k++) {
        if (k < pw && !bad) {
            const double d = rdlane(col[k], k);
            if (d == 0.0) {
                bad = true;
            } else {
                const double li = (lane > k && lane < pw) ? col[k] / d : 0.0;
                Ls[k * LP + lane] = li;
                if (lane == k) dvs[k] = d;
                const double dkj = col[k];
#pragma unroll
                for (int i = k + 1; i < LT; i++) {
                    const double l = rdlane(li, i);
                    if (i < pw && i <= lane && l != 0.0) col[i] -= l * dkj;
                }
            }
        }
    }
    if (bad) {
        if (lane == 0) atomicExch(fail, 1);
        return;
    }
    __syncthreads();
    if (diag) {   // the other workgroups of this launch still read A's diagonal block: stage it
#pragma unroll
        for (int r = 0; r < LT; r++) dstage[r * LT + lane] = lane >= r ? col[r] : Ls[lane * LP + r];
        if (lane == 0) nz[(size_t)p * nt + p] = 1;
        return;
    }
    // phase 2: this workgroup's chunk of the panel rows
#pragma unroll
    for (int r = 0; r < LT; r++) col[r] = (r < pw && lane < cw) ? Ap[(size_t)r * n + J0 + lane] : 0.0;
#pragma unroll
    for (int k = 0; k < LT; k++) {
        if (k < pw) {
            const double ckj = col[k];
#pragma unroll
            for (int i = k + 1; i < LT; i++) {
                const double l = Ls[k * LP + i];   // uniform
                if (i < pw && l != 0.0) col[i] -= l * ckj;
            }
        }
    }
    bool nzl = false;
#pragma unroll
    for (int r = 0; r < LT; r++) {
        if (r < pw && lane < cw) Ap[(size_t)r * n + J0 + lane] = col[r];
        nzl |= col[r] != 0.0;
    }
    // flag = some eliminated U[k][j] != 0, a superset of "some l != 0": skipping on it is exact
    __syncthreads();   // everyone is done reading Ls
#pragma unroll
    for (int k = 0; k < LT; k++) Ls[lane * LP + k] = k < pw ? col[k] / dvs[k] : 0.0;   // row J0+lane of L
    __syncthreads();
    for (int jj = 0; jj < cw; jj++)
        if (lane < pw) A[(size_t)(J0 + jj) * n + p0 + lane] = Ls[jj * LP + lane];
    const bool anyl = __any(nzl);   // wave-wide vote outside the lane-0 branch
    if (lane == 0) nz[(size_t)J * nt + p] = anyl ? 1 : 0;
}

// grid = m*m + 1 (m = trailing tiles): block m*m stores the staged diagonal block of panel p.
__global__ void __launch_bounds__(256) k_ldlt_trail(int n, int p, double* __restrict__ A, const uint8_t* nz, int nt,
                                                    const int* fail, const double* dstage) {
    if (*fail) return;
    const int m = nt - p - 1;
    if ((int)blockIdx.x == m * m) {
        const int p0 = p * LT, pw = min(LT, n - p0);
        for (int q = threadIdx.x; q < LT * LT; q += 256) {
            const int i = q >> 6, j = q & 63;
            if (i < pw && j < pw) A[(size_t)(p0 + i) * n + p0 + j] = dstage[q];  // U upper, d, L lower
        }
        return;
    }
    const int I = p + 1 + (int)blockIdx.x / m, J = p + 1 + (int)blockIdx.x % m;
    if (I > J) return;
    if (!nz[(size_t)I * nt + p] || !nz[(size_t)J * nt + p]) return;   // L[I][p] or U[p][J] is zero
    __shared__ double Lt[LT * LP];   // Lt[k][i] = L[I0+i][p0+k]
    __shared__ double Ut[LT * LP];   // Ut[k][j] = U[p0+k][J0+j]
    const int tid = threadIdx.x;
    const int p0 = p * LT, pw = min(LT, n - p0);
    const int I0 = I * LT, J0 = J * LT, ih = min(LT, n - I0), jw = min(LT, n - J0);
    for (int q = tid; q < LT * LT; q += 256) {
        const int r = q >> 6, c = q & 63;
        Lt[c * LP + r] = (r < ih && c < pw) ? A[(size_t)(I0 + r) * n + p0 + c] : 0.0;
        Ut[r * LP + c] = (r < pw && c < jw) ? A[(size_t)(p0 + r) * n + J0 + c] : 0.0;
    }
    __syncthreads();
    const int ty = tid >> 4, tx = tid & 15;
    double acc[4][4];
#pragma unroll
    for (int a = 0; a < 4; a++)
#pragma unroll
        for (int b = 0; b < 4; b++) {
            const int i = ty + 16 * a, j = tx + 16 * b;
            acc[a][b] = (i < ih && j < jw) ? A[(size_t)(I0 + i) * n + J0 + j] : 0.0;
        }
    for (int k = 0; k < pw; k++) {
        double l[4], u[4];
#pragma unroll
        for (int a = 0; a < 4; a++) l[a] = Lt[k * LP + ty + 16 * a];
#pragma unroll
        for (int b = 0; b < 4; b++) u[b] = Ut[k * LP + tx + 16 * b];
#pragma unroll
        for (int a = 0; a < 4; a++)
#pragma unroll
            for (int b = 0; b < 4; b++) acc[a][b] -= l[a] * u[b];
    }
#pragma unroll
    for (int a = 0; a < 4; a++)
#pragma unroll
        for (int b = 0; b < 4; b++) {
            const int i = ty + 16 * a, j = tx + 16 * b;
            if (i < ih && j < jw && (I != J || i <= j)) A[(size_t)(I0 + i) * n + J0 + j] = acc[a][b];
        }
}

__device__ __forceinline__ void wait_flag(const int* f) {
    while (__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == 0) __builtin_amdgcn_s_sleep(1);
}

__device__ __forceinline__ void set_flag(int* f) {
    __hip_atomic_store(f, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}

// Stage rows [0, rows) of a 64-column tile (row r at src + r * n, column = lane) into
// Lt[r * LP + lane], 16 independent loads in flight per batch.
__device__ __forceinline__ void stage_rows(double* Lt, const double* __restrict__ src, size_t n, int rows, int lane,
                                           bool col_ok) {
    for (int r0 = 0; r0 < rows; r0 += 16) {
        double v[16];
#pragma unroll
        for (int u = 0; u < 16; u++) v[u] = (r0 + u < rows && col_ok) ? src[(size_t)(r0 + u) * n + lane] : 0.0;
#pragma unroll
        for (int u = 0; u < 16; u++)
            if (r0 + u < rows) Lt[(r0 + u) * LP + lane] = v[u];
    }
}

// L y = b (column-sweep order per element): block I = blockIdx.x, one wave.
__global__ void __launch_bounds__(64) k_ldlt_fwd(int n, const double* __restrict__ A, const double* b, double* y,
                                                 const uint8_t* nz, int nt, const int* fail, int* done,
                                                 double* scal) {
    __shared__ double Lt[LT * LP];
    const int I = blockIdx.x, lane = threadIdx.x;
    if (I == 0 && lane == 0) scal[3] = *fail ? 0.0 : 1.0;
    if (*fail) return;
    const int I0 = I * LT, ih = min(LT, n - I0), i = I0 + lane;
    const bool on = lane < ih;
    double acc = on ? b[i] : 0.0;
    for (int K = 0; K < I; K++) {
        if (!nz[(size_t)I * nt + K]) continue;
        const int K0 = K * LT;
        stage_rows(Lt, A + (size_t)I0 * n + K0, n, ih, lane, true);
        if (lane == 0) wait_flag(done + K);
        __syncthreads();
        __atomic_thread_fence(__ATOMIC_ACQUIRE);
        const double yk_l = y[K0 + lane];
        for (int k = 0; k < LT; k++) {
            const double yk = rdlane(yk_l, k);
            if (on) acc -= Lt[lane * LP + k] * yk;
        }
    }
    // diagonal block: y_k final when all k' < k applied
    stage_rows(Lt, A + (size_t)I0 * n + I0, n, ih, lane, lane < ih);
    __syncthreads();
    for (int k = 0; k < ih; k++) {
        const double yk = rdlane(acc, k);
        if (on && lane > k) acc -= Lt[lane * LP + k] * yk;
    }
    if (on) y[i] = acc;   // undivided: later blocks' forward updates use it
    __atomic_thread_fence(__ATOMIC_RELEASE);
    __syncthreads();
    if (lane == 0) set_flag(done + I);
}

// y_i /= d_i (the oracle's middle sweep), then L^T x = y with k descending.
__global__ void __launch_bounds__(64) k_ldlt_bwd(int n, const double* __restrict__ A, double* y, double* x,
                                                 const uint8_t* nz, int nt, const int* fail, int* done) {
    __shared__ double Lt[LT * LP];
    if (*fail) return;
    const int I = nt - 1 - blockIdx.x, lane = threadIdx.x;
    const int I0 = I * LT, ih = min(LT, n - I0), i = I0 + lane;
    const bool on = lane < ih;
    double acc = on ? y[i] / A[(size_t)i * n + i] : 0.0;
    for (int K = nt - 1; K > I; K--) {
        if (!nz[(size_t)K * nt + I]) continue;   // L[K block][I block] == 0
        const int K0 = K * LT, kh = min(LT, n - K0);
        // Lt[k][i] = L[K0+k][I0+i] = A[(K0+k) n + I0+i] (coalesced over i)
        stage_rows(Lt, A + (size_t)K0 * n + I0, n, kh, lane, on);
        if (lane == 0) wait_flag(done + K);
        __syncthreads();
        __atomic_thread_fence(__ATOMIC_ACQUIRE);
        const double xk_l = lane < kh ? x[K0 + lane] : 0.0;
        for (int k = kh - 1; k >= 0; k--) {
            const double xk = rdlane(xk_l, k);
            if (on) acc -= Lt[k * LP + lane] * xk;
        }
    }
    stage_rows(Lt, A + (size_t)I0 * n + I0, n, ih, lane, on);
    __syncthreads();
    for (int k = ih - 1; k >= 0; k--) {
        const double xk = rdlane(acc, k);
        if (on && lane < k) acc -= Lt[k * LP + lane] * xk;
    }
    if (on) x[i] = acc;
    __atomic_thread_fence(__ATOMIC_RELEASE);
    __syncthreads();
    if (lane == 0) set_flag(done + I);
}

static inline size_t al256(size_t b) { return (b + 255) & ~(size_t)255; }

size_t ldlt_tiled_workspace(int n) {
    const size_t nt = (size_t)(n + LT - 1) / LT;
    return al256(nt * nt) + al256(sizeof(int) * (64 + 2 * nt)) + al256(sizeof(double) * (size_t)n) +
           sizeof(double) * LT * LT;
}

// ws: ldlt_tiled_workspace(n) bytes.  x is written only if the factorisation succeeds
// (scal[3] = 1), like ora_ldlt_solve's caller keeps the previous x on failure.
int ldlt_tiled_solve(int n, double* A, const double* b, double* x, double* scal, void* ws, hipStream_t s) {
    if (n <= 0) return 0;
    const int nt = (n + LT - 1) / LT;
    char* w = (char*)ws;
    uint8_t* nz = (uint8_t*)w;
    int* flags = (int*)(w + al256((size_t)nt * nt));
    int* fail = flags;            // [0]
    int* done = flags + 64;       // fwd [0, nt), bwd [nt, 2 nt)
    double* y = (double*)(w + al256((size_t)nt * nt) + al256(sizeof(int) * (64 + 2 * (size_t)nt)));
    double* dstage = (double*)((char*)y + al256(sizeof(double) * (size_t)n));
    ORB_HIP_CHECK(hipMemsetAsync(flags, 0, sizeof(int) * (64 + 2 * nt), s));
    for (int p = 0; p < nt; p++) {
        const int m = nt - p - 1;
        hipLaunchKernelGGL(k_ldlt_panel, dim3(nt - p), dim3(64), 0, s, n, p, A, nz, nt, fail, dstage);
        hipLaunchKernelGGL(k_ldlt_trail, dim3(m * m + 1), dim3(256), 0, s, n, p, A, nz, nt, fail, dstage);
    }
    hipLaunchKernelGGL(k_ldlt_fwd, dim3(nt), dim3(64), 0, s, n, A, b, y, nz, nt, fail, done, scal);
    hipLaunchKernelGGL(k_ldlt_bwd, dim3(nt), dim3(64), 0, s, n, A, y, x, nz, nt, fail, done + nt);
    ORB_HIP_CHECK(hipGetLastError());
    return 0;
}

}  // namespace orbgpu
