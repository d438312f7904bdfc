// ldlt.hip -- tiled multi-workgroup dense LDL^T solve of the reduced pose system S x = b_s
// for large bundle adjustments (reference: g2o LinearSolverEigen, SimplicialLDLT,
// Thirdparty/g2o/g2o/solvers/linear_solver_eigen.h:104; restated in oracle/ba.c
// ora_ldlt_solve).
//
// Per-element operation sequence is the oracle's: pivot k ascending, d_k = A[k][k],
// l_i = A[k][i] / d_k, A[i][j] -= l_i * A[k][j] (j >= i), no FMA contraction; forward
// y_i -= L[i][k] y_k in k order, y_k /= d_k, backward y_i -= L[k][i] y_k in descending k.
// Work is skipped at 64x64-tile granularity where a tile is exactly zero, which is the
// oracle's `l == 0` envelope skip (exact up to the sign of zero): a banded / block-sparse
// Schur complement (keyframes observe nearby keyframes' points) costs O(n bw^2), not n^3/3.
//
// Layout: A row-major n x n in HBM, upper triangle = S on entry (strict lower = 0); on exit
// the diagonal holds d, the strict lower triangle L, the upper triangle the eliminated rows.
// Tile maps (nt = ceil(n/64)): mask[I*nt+J] = tile (I<=J) of the working matrix may be
// nonzero (initial scan + fill-in), lnz[K*nt+I] = L tile (I, K) may be nonzero.
// Per panel p (64 pivots), three launches:
//   k_ldlt_diag    one wave: the 64x64 diagonal block, lane j = column j in registers,
//                  l_i broadcast by readlane; writes U / d / L of the block;
//   k_ldlt_chunks  persistent workgroups over the nonzero chunks J > p of the panel rows:
//                  left-looking per column (same per-element k order), the l_ik of the
//                  diagonal block are wave-uniform loads (scalar cache), L written through
//                  an LDS transpose, lnz[p][J] set;
//   k_ldlt_trail   persistent workgroups over the tile pairs (I <= J) of the nonzero L tiles
//                  of panel p: A[I][J] -= L[I][p] U[p][J], k in order, 4x4 register
//                  micro-tiles over LDS-staged L / U; marks fill-in in mask.
// Solves: one launch each, a workgroup (one wave) per 64-row block; a block consumes the
// finished blocks it depends on in order, spinning on their done flags (blocks are
// dispatched in dependency order, so a waiting block's producers are resident or done);
// the L rows it needs are staged into registers so the dependent chain never waits on LDS.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include "ldlt.hpp"
#include "orb_common.hpp"

namespace orbgpu {

constexpr int LT = 64;          // tile edge
constexpr int LP = LT + 1;      // LDS row pitch (doubles)
constexpr int kChunkWGs = 128;  // persistent workgroups of k_ldlt_chunks
constexpr int kTrailWGs = 512;  // persistent workgroups of k_ldlt_trail

__device__ __forceinline__ double rdlane(double v, int l) {
    const unsigned long long u = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)(u & 0xffffffffu), l);
    const int hi = __builtin_amdgcn_readlane((int)(u >> 32), l);
    return __longlong_as_double(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}

// mask[I][J] (I <= J) = some entry of the tile is nonzero
__global__ void __launch_bounds__(256) k_ldlt_mask(int n, const double* __restrict__ A, uint8_t* mask, int nt) {
    const int I = blockIdx.y, J = blockIdx.x;
    if (I > J) return;
    const int I0 = I * LT, J0 = J * LT, ih = min(LT, n - I0), jw = min(LT, n - J0);
    bool any = false;
    for (int q = threadIdx.x; q < LT * LT; q += 256) {
        const int r = q >> 6, c = q & 63;
        if (r < ih && c < jw && (I != J || r <= c)) any |= A[(size_t)(I0 + r) * n + J0 + c] != 0.0;
    }
    any = __syncthreads_or(any);
    if (threadIdx.x == 0) mask[(size_t)I * nt + J] = (any || I == J) ? 1 : 0;
}

// Diagonal block of panel p, one wave: lane j owns column j (rows 0..63) in registers.
__global__ void __launch_bounds__(64) k_ldlt_diag(int n, int p, double* __restrict__ A, uint8_t* lnz, int nt,
                                                  int* fail) {
    __shared__ double Ls[LT * LP];   // Ls[k * LP + i] = l_ik
    if (*fail) return;
    const int lane = threadIdx.x;
    const int p0 = p * LT, pw = min(LT, n - p0);
    double* Ad = A + (size_t)p0 * n + p0;
    for (int J = p + 1 + lane; J < nt; J += 64) lnz[(size_t)p * nt + J] = 0;   // set by k_ldlt_chunks
    if (lane == 0) lnz[(size_t)p * nt + p] = 1;
    double col[LT];
#pragma unroll
    for (int r = 0; r < LT; r++) col[r] = (r < pw && lane < pw && r <= lane) ? Ad[(size_t)r * n + lane] : 0.0;
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
                // lanes j < i update their (never stored) lower-triangle slot too: no per-lane
                // predicate, and the oracle's `l == 0` row skip is a wave-uniform branch
                const double dkj = col[k];
#pragma unroll
                for (int i = k + 1; i < LT; i++) {
                    const double l = rdlane(li, i);
                    if (l != 0.0) col[i] -= l * dkj;
                }
            }
        }
    }
    if (bad) {
        if (lane == 0) atomicExch(fail, 1);
        return;
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < LT; r++)
        if (r < pw && lane < pw) Ad[(size_t)r * n + lane] = lane >= r ? col[r] : Ls[lane * LP + r];
}

// Nonzero chunks J > p of the panel rows: persistent workgroups (one wave each).
__global__ void __launch_bounds__(64) k_ldlt_chunks(int n, int p, double* __restrict__ A,
                                                    const double* __restrict__ Ld, const uint8_t* mask,
                                                    uint8_t* lnz, int nt, const int* fail) {
    __shared__ int list[2048];
    __shared__ double T[LT * LP];
    __shared__ int cnt;
    if (*fail) return;
    const int lane = threadIdx.x;
    const int p0 = p * LT, pw = min(LT, n - p0);
    // compact the nonzero chunks of row p of the tile mask (contiguous scan)
    if (lane == 0) cnt = 0;
    __syncthreads();
    for (int J0 = p + 1; J0 < nt; J0 += 64) {
        const int J = J0 + lane;
        const bool on = J < nt && mask[(size_t)p * nt + J];
        const unsigned long long b = __ballot(on);
        if (on) list[cnt + __popcll(b & ((1ull << lane) - 1))] = J;
        __syncthreads();
        if (lane == 0) cnt += __popcll(b);
        __syncthreads();
    }
    const int nc = cnt;
    double* Ap = A + (size_t)p0 * n;
    for (int t = blockIdx.x; t < nc; t += gridDim.x) {
        const int J = list[t], J0 = J * LT, cw = min(LT, n - J0);
        double c[LT];
#pragma unroll
        for (int r = 0; r < LT; r++) c[r] = (r < pw && lane < cw) ? Ap[(size_t)r * n + J0 + lane] : 0.0;
        // left-looking: c_i -= l_ik c_k, k ascending (the oracle's per-element order)
#pragma unroll
        for (int i = 1; i < LT; i++) {
            if (i < pw) {
#pragma unroll
                for (int k = 0; k < i; k++) {
                    const double l = Ld[(size_t)i * n + k];   // wave-uniform
                    if (l != 0.0) c[i] -= l * c[k];
                }
            }
        }
        bool nzl = false;
#pragma unroll
        for (int r = 0; r < LT; r++) {
            if (r < pw && lane < cw) Ap[(size_t)r * n + J0 + lane] = c[r];
            nzl |= c[r] != 0.0;
        }
        // L[J0 + lane][p0 + k] = c_k / d_k, through an LDS transpose (coalesced rows)
#pragma unroll
        for (int k = 0; k < LT; k++) T[lane * LP + k] = k < pw ? c[k] / Ld[(size_t)k * n + k] : 0.0;
        __syncthreads();
        for (int jj = 0; jj < cw; jj++)
            if (lane < pw) A[(size_t)(J0 + jj) * n + p0 + lane] = T[jj * LP + lane];
        // flag = some eliminated U[k][j] != 0, a superset of "some l != 0": skipping on it is exact
        const bool anyl = __any(nzl);
        if (lane == 0) lnz[(size_t)p * nt + J] = anyl ? 1 : 0;
        __syncthreads();
    }
}

// Trailing update of panel p over the tile pairs of its nonzero L tiles (persistent).
__global__ void __launch_bounds__(256) k_ldlt_trail(int n, int p, double* __restrict__ A, const uint8_t* lnz,
                                                    uint8_t* mask, int nt, const int* fail) {
    __shared__ int list[2048];
    __shared__ int cnt;
    __shared__ double Lt[LT * LP];   // Lt[k][i] = L[I0+i][p0+k]
    __shared__ double Ut[LT * LP];   // Ut[k][j] = U[p0+k][J0+j]
    if (*fail) return;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    if (tid == 0) cnt = 0;
    __syncthreads();
    for (int I0 = p + 1; I0 < nt; I0 += 64) {
        const int I = I0 + lane;
        const bool on = w == 0 && I < nt && lnz[(size_t)p * nt + I];
        const unsigned long long b = __ballot(on);
        if (on) list[cnt + __popcll(b & ((1ull << lane) - 1))] = I;
        __syncthreads();
        if (tid == 0) cnt += __popcll(b);
        __syncthreads();
    }
    const int m = cnt, npair = m * (m + 1) / 2;
    const int p0 = p * LT, pw = min(LT, n - p0);
    const int ty = tid >> 4, tx = tid & 15;
    for (int t = blockIdx.x; t < npair; t += gridDim.x) {
        // pair t -> (a <= b): row a has m - a pairs
        int a = 0, rem = t;
        while (rem >= m - a) {
            rem -= m - a;
            a++;
        }
        const int I = list[a], J = list[a + rem];
        const int I0 = I * LT, J0 = J * LT, ih = min(LT, n - I0), jw = min(LT, n - J0);
        for (int q = tid; q < LT * LT; q += 256) {
            const int r = q >> 6, c = q & 63;
            Lt[c * LP + r] = (r < ih && c < pw) ? A[(size_t)(I0 + r) * n + p0 + c] : 0.0;
            Ut[r * LP + c] = (r < pw && c < jw) ? A[(size_t)(p0 + r) * n + J0 + c] : 0.0;
        }
        __syncthreads();
        double acc[4][4];
#pragma unroll
        for (int aa = 0; aa < 4; aa++)
#pragma unroll
            for (int bb = 0; bb < 4; bb++) {
                const int i = ty + 16 * aa, j = tx + 16 * bb;
                acc[aa][bb] = (i < ih && j < jw) ? A[(size_t)(I0 + i) * n + J0 + j] : 0.0;
            }
        for (int k = 0; k < pw; k++) {
            double l[4], u[4];
#pragma unroll
            for (int aa = 0; aa < 4; aa++) l[aa] = Lt[k * LP + ty + 16 * aa];
#pragma unroll
            for (int bb = 0; bb < 4; bb++) u[bb] = Ut[k * LP + tx + 16 * bb];
#pragma unroll
            for (int aa = 0; aa < 4; aa++)
#pragma unroll
                for (int bb = 0; bb < 4; bb++) acc[aa][bb] -= l[aa] * u[bb];
        }
#pragma unroll
        for (int aa = 0; aa < 4; aa++)
#pragma unroll
            for (int bb = 0; bb < 4; bb++) {
                const int i = ty + 16 * aa, j = tx + 16 * bb;
                if (i < ih && j < jw && (I != J || i <= j)) A[(size_t)(I0 + i) * n + J0 + j] = acc[aa][bb];
            }
        if (tid == 0) mask[(size_t)I * nt + J] = 1;   // fill-in
        __syncthreads();
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
                                                 const uint8_t* lnz, int nt, const int* fail, int* done,
                                                 double* scal) {
    __shared__ double Lt[LT * LP];
    const int I = blockIdx.x, lane = threadIdx.x;
    if (I == 0 && lane == 0) scal[3] = *fail ? 0.0 : 1.0;
    if (*fail) return;
    const int I0 = I * LT, ih = min(LT, n - I0), i = I0 + lane;
    const bool on = lane < ih;
    double acc = on ? b[i] : 0.0;
    double Lr[LT];
    for (int K = 0; K < I; K++) {
        if (!lnz[(size_t)K * nt + I]) continue;
        const int K0 = K * LT;
        stage_rows(Lt, A + (size_t)I0 * n + K0, n, ih, lane, true);
        __syncthreads();
#pragma unroll
        for (int k = 0; k < LT; k++) Lr[k] = Lt[lane * LP + k];   // this lane's row, into registers
        if (lane == 0) wait_flag(done + K);
        __syncthreads();
        __atomic_thread_fence(__ATOMIC_ACQUIRE);
        const double yk_l = y[K0 + lane];
#pragma unroll
        for (int k = 0; k < LT; k++) {
            const double v = acc - Lr[k] * rdlane(yk_l, k);
            acc = on ? v : acc;
        }
        __syncthreads();
    }
    // diagonal block: y_k final when all k' < k applied
    stage_rows(Lt, A + (size_t)I0 * n + I0, n, ih, lane, lane < ih);
    __syncthreads();
#pragma unroll
    for (int k = 0; k < LT; k++) Lr[k] = Lt[lane * LP + k];
#pragma unroll
    for (int k = 0; k < LT; k++) {
        if (k < ih) {
            const double yk = rdlane(acc, k);
            const double v = acc - Lr[k] * yk;
            acc = (on && lane > k) ? v : acc;
        }
    }
    if (on) y[i] = acc;   // undivided: later blocks' forward updates use it
    __atomic_thread_fence(__ATOMIC_RELEASE);
    __syncthreads();
    if (lane == 0) set_flag(done + I);
}

// y_i /= d_i (the oracle's middle sweep), then L^T x = y with k descending.
__global__ void __launch_bounds__(64) k_ldlt_bwd(int n, const double* __restrict__ A, double* y, double* x,
                                                 const uint8_t* lnz, int nt, const int* fail, int* done) {
    __shared__ double Lt[LT * LP];
    if (*fail) return;
    const int I = nt - 1 - blockIdx.x, lane = threadIdx.x;
    const int I0 = I * LT, ih = min(LT, n - I0), i = I0 + lane;
    const bool on = lane < ih;
    double acc = on ? y[i] / A[(size_t)i * n + i] : 0.0;
    double Lr[LT];
    for (int K = nt - 1; K > I; K--) {
        if (!lnz[(size_t)I * nt + K]) continue;   // L tile (K, I)
        const int K0 = K * LT, kh = min(LT, n - K0);
        // Lt[k][i] = L[K0+k][I0+i] = A[(K0+k) n + I0+i] (coalesced over i)
        stage_rows(Lt, A + (size_t)K0 * n + I0, n, kh, lane, on);
        __syncthreads();
#pragma unroll
        for (int k = 0; k < LT; k++) Lr[k] = k < kh ? Lt[k * LP + lane] : 0.0;
        if (lane == 0) wait_flag(done + K);
        __syncthreads();
        __atomic_thread_fence(__ATOMIC_ACQUIRE);
        const double xk_l = lane < kh ? x[K0 + lane] : 0.0;
#pragma unroll
        for (int k = LT - 1; k >= 0; k--) {
            if (k < kh) {
                const double v = acc - Lr[k] * rdlane(xk_l, k);
                acc = on ? v : acc;
            }
        }
        __syncthreads();
    }
    stage_rows(Lt, A + (size_t)I0 * n + I0, n, ih, lane, on);
    __syncthreads();
#pragma unroll
    for (int k = 0; k < LT; k++) Lr[k] = k < ih ? Lt[k * LP + lane] : 0.0;
#pragma unroll
    for (int k = LT - 1; k >= 0; k--) {
        if (k < ih) {
            const double xk = rdlane(acc, k);
            const double v = acc - Lr[k] * xk;
            acc = (on && lane < k) ? v : acc;
        }
    }
    if (on) x[i] = acc;
    __atomic_thread_fence(__ATOMIC_RELEASE);
    __syncthreads();
    if (lane == 0) set_flag(done + I);
}

static inline size_t al256(size_t b) { return (b + 255) & ~(size_t)255; }

size_t ldlt_tiled_workspace(int n) {
    const size_t nt = (size_t)(n + LT - 1) / LT;
    return 2 * al256(nt * nt) + al256(sizeof(int) * (64 + 2 * nt)) + al256(sizeof(double) * (size_t)n);
}

// ws: ldlt_tiled_workspace(n) bytes.  x is written only if the factorisation succeeds
// (scal[3] = 1), like ora_ldlt_solve's caller keeps the previous x on failure.
int ldlt_tiled_solve(int n, double* A, const double* b, double* x, double* scal, void* ws, hipStream_t s) {
    if (n <= 0) return 0;
    const int nt = (n + LT - 1) / LT;
    if (nt > 2048) return -3;
    char* w = (char*)ws;
    uint8_t* lnz = (uint8_t*)w;
    uint8_t* mask = lnz + al256((size_t)nt * nt);
    int* flags = (int*)(w + 2 * al256((size_t)nt * nt));
    int* fail = flags;            // [0]
    int* done = flags + 64;       // fwd [0, nt), bwd [nt, 2 nt)
    double* y = (double*)((char*)flags + al256(sizeof(int) * (64 + 2 * (size_t)nt)));
    ORB_HIP_CHECK(hipMemsetAsync(flags, 0, sizeof(int) * (64 + 2 * nt), s));
    hipLaunchKernelGGL(k_ldlt_mask, dim3(nt, nt), dim3(256), 0, s, n, A, mask, nt);
    for (int p = 0; p < nt; p++) {
        const double* Ld = A + (size_t)p * LT * n + (size_t)p * LT;
        hipLaunchKernelGGL(k_ldlt_diag, dim3(1), dim3(64), 0, s, n, p, A, lnz, nt, fail);
        if (p + 1 < nt) {
            hipLaunchKernelGGL(k_ldlt_chunks, dim3(std::min(nt - p - 1, kChunkWGs)), dim3(64), 0, s, n, p, A, Ld,
                               mask, lnz, nt, fail);
            hipLaunchKernelGGL(k_ldlt_trail, dim3(kTrailWGs), dim3(256), 0, s, n, p, A, lnz, mask, nt, fail);
        }
    }
    hipLaunchKernelGGL(k_ldlt_fwd, dim3(nt), dim3(64), 0, s, n, A, b, y, lnz, nt, fail, done, scal);
    hipLaunchKernelGGL(k_ldlt_bwd, dim3(nt), dim3(64), 0, s, n, A, y, x, lnz, nt, fail, done + nt);
    ORB_HIP_CHECK(hipGetLastError());
    return 0;
}

}  // namespace orbgpu
