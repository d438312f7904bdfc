// ldlt.hip -- block-sparse LDL^T solve of the reduced pose system S x = b_s for large bundle
// adjustments (reference: g2o LinearSolverEigen = Eigen SimplicialLDLT + AMD on the sparse Schur
// complement, Thirdparty/g2o/g2o/solvers/linear_solver_eigen.h:60-124; restated in oracle/ba.c).
//
// Order.  The poses are permuted by a nested dissection of the pose graph (ordering.hpp): the
// separator tree bounds the fill on loop-closed maps and is the task tree of the factorisation.
// Each tree node's rows are packed into whole 64 x 64 tiles of a "tile space" (a node never
// shares a tile with another node; its last tile is partial: th[t] rows, zero beyond), so the
// tile elimination tree follows the separator tree: the tiles of sibling subtrees never meet.
//
// Storage: only the tiles of S's pattern and their fill (symbolic factorisation at tile level,
// once per structure):
//   U  [slot] row-major tile (I, J), I <= J in tile space: S on entry; after the factorisation
//      the eliminated rows (U), and on diagonal tiles d on the diagonal and L strictly below;
//   LT [slot] of tile (p, J), p < J: LT[k][j] = L[J0 + j][p0 + k] (pivot-major, coalesced).
// Per-element operation sequence (the oracle's): element (i, j) receives the updates
// a_ij -= l_ik u_kj of every pivot k < i in ascending k, d_k = a_kk, l_ik = a_ki / d_k, no FMA
// contraction; whole tiles whose L is zero are skipped (the oracle skips l == 0: equal up to the
// sign of a zero).  The forward solve y_i -= L[i][k] y_k runs k ascending, y_k /= d_k, the
// backward solve y_i -= L[k][i] y_k k descending -- the same sequences whatever the schedule.
//
// Schedule: the tree's levels (height 0 = leaves) run bottom-up, two launches per level:
//   update  one workgroup per target tile (I, J) of the level's nodes that a DESCENDANT tile
//           row K touches: A(I, J) -= sum_K L(I, K) U(K, J), K ascending (left-looking: reads
//           finished descendant tiles only, writes a tile owned by this node: no races);
//   factor  the level's nodes walk their own panels right-looking in lock step: per panel step
//           three launches over every node of the level (diagonal tiles, the panel rows' U/LT
//           tiles, the trailing updates of the nodes' own rows), a workgroup per tile; then
//           one wave per node solves its rows of L y = b;
// then the backward solve runs the levels top-down (one wave per node).  Nodes of one level
// share no tile, so their workgroups run concurrently; the descendants' updates of an
// ancestor tile arrive in ascending K, i.e. in pivot order, as in the sequential sweep.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "ldlt.hpp"
#include "orb_common.hpp"
#include "ordering.hpp"
#include "comm.hpp"

namespace orbgpu {

constexpr int LT = kTile;        // tile edge
constexpr int LP = LT + 1;       // LDS row pitch (doubles) of the diagonal L
constexpr int kMaxRow = 2048;    // tiles per panel row
constexpr int kNdLeaf = kNdLeafPoses;   // nested-dissection leaf size (poses)

struct SpDev {
    int n, nt;
    const int* slotOf;
    double* U;
    double* LT;
    const int* th;        // rows of tile t (tile space)
    const int* rowMap;    // tile-space row -> system row (-1: padding)
    const int* rowStart;  // panel p: tiles (p, J > p)
    const int* rowJ;
    const int* rowSlot;
    const int* colStart;  // tile row I: tiles (K < I, I), K ascending
    const int* colK;
    const int* colSlot;
    const int* pairStart; // panel p: trailing pairs inside p's node
    const int4* pairs;    // (index of I in the panel row, index of J, target slot, 0)
    const int* nodeT;     // node k: tiles [nodeT[2k], nodeT[2k + 1])
    const int* levNodes;  // node ids by level
    const int4* tgts;     // update targets by level: (slot(I, J), I, J, first K pair)
    const int4* kps;      // (slot(K, I), slot(K, J), K, 0), per target in ascending K
    const int* stepP;     // panel steps: the panels of (level, step), see k_ldlt_pdiag
    const int2* rowJobs;  // (panel, index in its row) of each U tile of a step
    const int2* pairJobs; // (panel, pair index) of each trailing target of a step
    const int4* panelJobs; // (panel, first role, roles, 0): k_ldlt_panel's workgroups of a step
    uint8_t* lnz;
    double* y;            // tile space
    double* xs;           // tile space
    int* fail;
    // sharded schedule (SparseLdlt::solve_dist); the plain solve leaves tcls null
    const uint8_t* tcls;  // tile class: 0 another rank's subtree, 1 shared separator, 2 this rank's subtree
    int want;             // launches touch the targets / panels / nodes of this class only (-1: all)
    int kmode;            // 0: every pivot tile K; 1 / 2: only K of that class (updates, forward sweep)
    double* dst;          // k_ldlt_update delta mode: the target tiles live in the exchange buffer
    const int* packIdx;   // slot -> tile index in dst (delta mode)
    int yfused;           // the forward sweep rides along the factorisation (y as an extra column)
    int pfused;           // k_ldlt_panel: factored diagonal tiles land in their L^T slot, copied by k_ldlt_ptrail_q
};
constexpr int kDiagCopyJob = -2147483647 - 1;   // pairJobs marker: copy the panel's factored diagonal tile

// the sharded schedule's filters (block-uniform)
__device__ __forceinline__ bool skip_tile(const SpDev& S, int t) { return S.want >= 0 && S.tcls[t] != S.want; }
__device__ __forceinline__ bool skip_k(const SpDev& S, int K) { return S.kmode && S.tcls[K] != S.kmode; }

// Tile access through a buffer descriptor (wave-uniform tile base in SGPRs, 32-bit per-lane
// offset, constant row offsets folded into the instruction): the unrolled 64-row loops then
// need no 64-bit address per row (hipcc precomputed and spilled them).
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
// (the base is wave-uniform by construction; readfirstlane makes that provable, otherwise
// hipcc wraps every buffer op in a waterfall loop)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t tile_rsrc(const double* p) {
    const unsigned long long a = (unsigned long long)p;
    const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)a);
    const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(a >> 32));
    void* q = (void*)(((unsigned long long)hi << 32) | lo);
    return __builtin_amdgcn_make_buffer_rsrc(q, (short)0, LT * LT * (int)sizeof(double), 0x00020000);
}
__device__ __forceinline__ double tld(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
    return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, voff, soff, 0));
}
__device__ __forceinline__ void tst(__amdgpu_buffer_rsrc_t r, double v, int voff, int soff) {
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v), r, voff, soff, 0);
}

__device__ __forceinline__ double rdlane(double v, int l) {
    const unsigned long long u = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)(u & 0xffffffffu), l);
    const int hi = __builtin_amdgcn_readlane((int)(u >> 32), l);
    return __longlong_as_double(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}

// A(I, J) -= L(I, K) U(K, J) over a target's descendant tile rows K (ascending): 256 threads,
// 4 x 4 register micro-tiles, the two operand tiles staged in LDS per K.
__global__ void __launch_bounds__(256) k_ldlt_update(SpDev S, int t0) {
    __shared__ double Lg[LT * LT];   // [k][i] = L[I0 + i][K0 + k]
    __shared__ double Ug[LT * LT];   // [k][j] = U[K0 + k][J0 + j]
    if (*(volatile int*)S.fail) return;
    const int4 tg = S.tgts[t0 + blockIdx.x];
    const int kp0 = tg.w, kp1 = S.tgts[t0 + blockIdx.x + 1].w;
    const int I = tg.y, J = tg.z;
    if (skip_tile(S, I)) return;
    const int ih = S.th[I], jw = S.th[J];
    const int gt = threadIdx.x, ty = gt >> 4, tx = gt & 15;
    double* T = S.dst ? S.dst + (size_t)S.packIdx[tg.x] * (LT * LT) : S.U + (size_t)tg.x * (LT * LT);
    double acc[4][4];
#pragma unroll
    for (int a = 0; a < 4; a++)
#pragma unroll
        for (int bb = 0; bb < 4; bb++) {
            const int i = ty + 16 * a, j = tx + 16 * bb;
            acc[a][bb] = (i < ih && j < jw) ? T[i * LT + j] : 0.0;
        }
    for (int q = kp0; q < kp1; q++) {
        const int4 kp = S.kps[q];
        if (!S.lnz[kp.x] || !S.lnz[kp.y] || skip_k(S, kp.z)) continue;   // block-uniform
        const double2* srcL = (const double2*)(S.LT + (size_t)kp.x * (LT * LT));
        const double2* srcU = (const double2*)(S.U + (size_t)kp.y * (LT * LT));
        __syncthreads();
#pragma unroll
        for (int u = 0; u < (LT * LT / 2) / 256; u++) {
            ((double2*)Lg)[gt + 256 * u] = srcL[gt + 256 * u];
            ((double2*)Ug)[gt + 256 * u] = srcU[gt + 256 * u];
        }
        __syncthreads();
        const int kw = S.th[kp.z];
        for (int k = 0; k < kw; k++) {
            double l[4], u[4];
#pragma unroll
            for (int a = 0; a < 4; a++) l[a] = Lg[k * LT + ty + 16 * a];
#pragma unroll
            for (int bb = 0; bb < 4; bb++) u[bb] = Ug[k * LT + tx + 16 * bb];
#pragma unroll
            for (int a = 0; a < 4; a++)
#pragma unroll
                for (int bb = 0; bb < 4; bb++) acc[a][bb] -= l[a] * u[bb];
        }
    }
#pragma unroll
    for (int a = 0; a < 4; a++)
#pragma unroll
        for (int bb = 0; bb < 4; bb++) {
            const int i = ty + 16 * a, j = tx + 16 * bb;
            if (i < ih && j < jw && (I != J || i <= j)) T[i * LT + j] = acc[a][bb];
        }
}

// A level's nodes factor their own panels right-looking, panel step by panel step: step s
// takes panel T0 + s of every node of the level that has one, in three launches (diagonal
// tile, the panel row's U / L^T tiles, the trailing updates inside the nodes), so every tile
// of a step is its own workgroup.  Then k_ldlt_pfwd solves the level's rows of L y = b.

// Diagonal tile of each panel of the step: one wave per panel, lane = column.  On exit the tile
// holds U (d on the diagonal) in its upper triangle and L strictly below.
__global__ void __launch_bounds__(64) k_ldlt_pdiag(SpDev S, int j0) {
    __shared__ double Ls[LT * LP];
    if (*(volatile int*)S.fail) return;
    const int p = S.stepP[j0 + blockIdx.x];
    if (skip_tile(S, p)) return;
    const int lane = threadIdx.x;
    const int pw = S.th[p];
    const __amdgpu_buffer_rsrc_t Ud = tile_rsrc(S.U + (size_t)S.slotOf[(size_t)p * S.nt + p] * (LT * LT));
    const int vo = lane * 8;
    double col[LT];
#pragma unroll
    for (int r = 0; r < LT; r++) col[r] = tld(Ud, vo, r * LT * 8);
    bool bad = false;
#pragma unroll
    for (int k = 0; k < LT; k++) {
        if (k < pw && !bad) {
            const double d = rdlane(col[k], k);   // the pivot, from lane k's register (no LDS round trip)
            if (d == 0.0) {
                bad = true;
            } else {
                Ls[k * LP + lane] = lane > k ? col[k] / d : 0.0;
                __builtin_amdgcn_wave_barrier();
                const double ck = col[k];
#pragma unroll
                for (int i = k + 1; i < LT; i++) col[i] -= Ls[k * LP + i] * ck;
                __builtin_amdgcn_sched_barrier(0);
            }
        }
    }
    if (bad) {
        if (lane == 0) *S.fail = 1;
        return;
    }
#pragma unroll
    for (int r = 0; r < LT; r++)
        if (r < pw && lane < pw) tst(Ud, lane >= r ? col[r] : Ls[lane * LP + r], vo, r * LT * 8);
}

// U tiles (p, J > p) of each panel row of the step: one wave per tile, lane = column; the
// panel's L and d come from its factored diagonal tile (padding pivots: L = 0, d = 1).
__global__ void __launch_bounds__(64) k_ldlt_prow(SpDev S, int j0) {
    __shared__ double Ls[LT * LP];   // [k][i] = L[i][k]
    __shared__ double dsh[LT];
    if (*(volatile int*)S.fail) return;
    const int2 job = S.rowJobs[j0 + blockIdx.x];   // (panel, index in its row)
    const int p = job.x, lane = threadIdx.x;
    if (job.y < 0 || skip_tile(S, p)) return;   // (y jobs: the four-wave kernel's only)
    const int pw = S.th[p];
    const double* D = S.U + (size_t)S.slotOf[(size_t)p * S.nt + p] * (LT * LT);
    // L[i][k] = D[i][k] (i > k) into Ls[k][i]: row r of D read by the wave in one coalesced load
    // (lane = column k) per row, instead of a 512-B-strided column gather per k
#pragma unroll 4
    for (int r = 0; r < LT; r++) {
        const double v = D[r * LT + lane];
        Ls[lane * LP + r] = (lane < pw && r > lane) ? v : 0.0;
    }
    dsh[lane] = lane < pw ? D[lane * LT + lane] : 1.0;
    __syncthreads();
    const int e = S.rowStart[p] + job.y;
    const int sl = S.rowSlot[e];
    const __amdgpu_buffer_rsrc_t Ut = tile_rsrc(S.U + (size_t)sl * (LT * LT));
    const __amdgpu_buffer_rsrc_t Lo = tile_rsrc(S.LT + (size_t)sl * (LT * LT));
    const int vo = lane * 8;
    double c[LT];
#pragma unroll
    for (int r = 0; r < LT; r++) c[r] = tld(Ut, vo, r * LT * 8);   // zero outside the system
    // per element the updates arrive in k order (the oracle's); the scheduling barrier keeps the
    // compiler from hoisting every pivot's 63 broadcast reads at once
#pragma unroll
    for (int k = 0; k < LT - 1; k++) {
        const double ck = c[k];
#pragma unroll
        for (int i = k + 1; i < LT; i++) c[i] -= Ls[k * LP + i] * ck;   // L[i][k], wave-uniform address
        __builtin_amdgcn_sched_barrier(0);
    }
    bool nz = false;
#pragma unroll
    for (int r = 0; r < LT; r++) {
        tst(Ut, c[r], vo, r * LT * 8);
        nz |= c[r] != 0.0;
        tst(Lo, c[r] / dsh[r], vo, r * LT * 8);
    }
    // flag = some eliminated U[k][j] != 0, a superset of "some l != 0": skipping on it is exact
    const bool any = __any(nz);
    if (lane == 0) S.lnz[sl] = any ? 1 : 0;
}

// The same two kernels with a rolled pivot loop.  Fully unrolled, k_ldlt_pdiag / k_ldlt_prow are
// 69 / 59 KB of straight-line code that every launch runs once, so the wave waits on instruction
// fetch; here a loop over 8-pivot chunks runs one 8-pivot body (~9 KB): register t of the chunk
// is pivot 8c + t, the live column shifts down by 8 registers after each chunk, and groups of 8
// registers past the live rows are skipped.  Per element the updates still arrive in ascending
// pivot order (the same operations as the unrolled kernels and the oracle); padding pivots
// (k >= pw), whose L is zero, are not applied (the oracle has no such rows).
constexpr int kChunk = 8;

__global__ void __launch_bounds__(64) k_ldlt_pdiag_r(SpDev S, int j0) {
    __shared__ double Ls[LT * LP];
    if (*(volatile int*)S.fail) return;
    const int p = S.stepP[j0 + blockIdx.x];
    if (skip_tile(S, p)) return;
    const int lane = threadIdx.x;
    const int pw = S.th[p];
    const __amdgpu_buffer_rsrc_t Ud = tile_rsrc(S.U + (size_t)S.slotOf[(size_t)p * S.nt + p] * (LT * LT));
    const int vo = lane * 8;
    double col[LT];   // col[r] = tile row kb + r of column `lane` (kb: the chunk's first pivot)
#pragma unroll
    for (int r = 0; r < LT; r++) col[r] = tld(Ud, vo, r * LT * 8);
    bool bad = false;
    for (int c = 0; c < LT / kChunk; c++) {
        const int kb = kChunk * c;
        if (kb >= pw || bad) break;
#pragma unroll
        for (int t = 0; t < kChunk; t++) {
            const int k = kb + t;
            if (k < pw && !bad) {
                const double d = rdlane(col[t], k);
                if (d == 0.0) {
                    bad = true;
                } else {
                    Ls[k * LP + lane] = lane > k ? col[t] / d : 0.0;
                    __builtin_amdgcn_wave_barrier();
                    // row k is final: U (lane >= k) and the L of the earlier pivots (lane < k)
                    if (lane < pw) tst(Ud, lane >= k ? col[t] : Ls[lane * LP + k], vo, k * LT * 8);
                    const double ck = col[t];
#pragma unroll
                    for (int q = 0; q < LT / kChunk; q++) {
                        if (q < LT / kChunk - c) {   // registers 8q..8q+7 hold live rows
#pragma unroll
                            for (int r = kChunk * q; r < kChunk * q + kChunk; r++)
                                if (r > t) col[r] -= Ls[k * LP + kb + r] * ck;
                        }
                    }
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
        }
#pragma unroll
        for (int r = 0; r < LT - kChunk; r++) col[r] = col[r + kChunk];
    }
    if (bad && lane == 0) *S.fail = 1;
}

__global__ void __launch_bounds__(64) k_ldlt_prow_r(SpDev S, int j0) {
    __shared__ double Ls[LT * LP];   // [k][i] = L[i][k]
    __shared__ double dsh[LT];
    if (*(volatile int*)S.fail) return;
    const int2 job = S.rowJobs[j0 + blockIdx.x];   // (panel, index in its row)
    const int p = job.x, lane = threadIdx.x;
    if (job.y < 0 || skip_tile(S, p)) return;   // (y jobs: the four-wave kernel's only)
    const int pw = S.th[p];
    const double* D = S.U + (size_t)S.slotOf[(size_t)p * S.nt + p] * (LT * LT);
    for (int r = 0; r < LT; r++) {
        const double v = D[r * LT + lane];
        Ls[lane * LP + r] = (lane < pw && r > lane) ? v : 0.0;
    }
    dsh[lane] = lane < pw ? D[lane * LT + lane] : 1.0;
    __syncthreads();
    const int e = S.rowStart[p] + job.y;
    const int sl = S.rowSlot[e];
    const __amdgpu_buffer_rsrc_t Ut = tile_rsrc(S.U + (size_t)sl * (LT * LT));
    const __amdgpu_buffer_rsrc_t Lo = tile_rsrc(S.LT + (size_t)sl * (LT * LT));
    const int vo = lane * 8;
    double c[LT];   // c[r] = tile row kb + r of column `lane`
#pragma unroll
    for (int r = 0; r < LT; r++) c[r] = tld(Ut, vo, r * LT * 8);   // zero outside the system
    bool nz = false;
    for (int ch = 0; ch < LT / kChunk; ch++) {
        const int kb = kChunk * ch;
        if (kb >= pw) break;
#pragma unroll
        for (int t = 0; t < kChunk; t++) {
            const int k = kb + t;
            if (k < pw) {
                const double ck = c[t];   // row k final: all its updates (pivots < k) are in
                tst(Ut, ck, vo, k * LT * 8);
                tst(Lo, ck / dsh[k], vo, k * LT * 8);
                nz |= ck != 0.0;
#pragma unroll
                for (int q = 0; q < LT / kChunk; q++) {
                    if (q < LT / kChunk - ch) {
#pragma unroll
                        for (int r = kChunk * q; r < kChunk * q + kChunk; r++)
                            if (r > t) c[r] -= Ls[k * LP + kb + r] * ck;   // L[kb + r][k], wave-uniform address
                    }
                }
                __builtin_amdgcn_sched_barrier(0);
            }
        }
#pragma unroll
        for (int r = 0; r < LT - kChunk; r++) c[r] = c[r + kChunk];
    }
    for (int r = pw; r < LT; r++) tst(Lo, 0.0, vo, r * LT * 8);   // padding rows of L^T: zero
    // flag = some eliminated U[k][j] != 0, a superset of "some l != 0": skipping on it is exact
    const bool any = __any(nz);
    if (lane == 0) S.lnz[sl] = any ? 1 : 0;
}

// U tiles of the panel rows with four waves per tile: wave w takes columns 16w..16w+15, a
// quad of lanes per column, lane s of the quad rows 4q + s (q < 16).  Pivot k's row value
// reaches the quad by one DPP broadcast from lane k mod 4, every lane applies it to its own
// rows below k with the L it reads from LDS (four distinct addresses per instruction), so a
// wave issues a quarter of the one-wave kernel's FP64 work and the four waves run on the
// CU's four SIMDs without any barrier.  The lane's rows shift down by one register after every
// four pivots (pivot 4m + t is register 0 of quad lane t).  Same per-element sequence.
__device__ __forceinline__ double quad_bcast(double v, int t) {
    const unsigned long long u = __double_as_longlong(v);
    int lo = (int)(u & 0xffffffffu), hi = (int)(u >> 32);
    const int ctl = t | (t << 2) | (t << 4) | (t << 6);   // quad_perm(t, t, t, t)
    switch (t) {   // the DPP control is an immediate
    case 0:
        lo = __builtin_amdgcn_mov_dpp(lo, 0x00, 0xf, 0xf, false);
        hi = __builtin_amdgcn_mov_dpp(hi, 0x00, 0xf, 0xf, false);
        break;
    case 1:
        lo = __builtin_amdgcn_mov_dpp(lo, 0x55, 0xf, 0xf, false);
        hi = __builtin_amdgcn_mov_dpp(hi, 0x55, 0xf, 0xf, false);
        break;
    case 2:
        lo = __builtin_amdgcn_mov_dpp(lo, 0xaa, 0xf, 0xf, false);
        hi = __builtin_amdgcn_mov_dpp(hi, 0xaa, 0xf, 0xf, false);
        break;
    default:
        lo = __builtin_amdgcn_mov_dpp(lo, 0xff, 0xf, 0xf, false);
        hi = __builtin_amdgcn_mov_dpp(hi, 0xff, 0xf, 0xf, false);
        break;
    }
    (void)ctl;
    return __longlong_as_double(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}

__global__ void __launch_bounds__(256) k_ldlt_prow4(SpDev S, int j0) {
    __shared__ double Ls[LT * LP + 4 * LT];   // [k][i] = L[i][k]; the pad keeps dead-row reads in bounds
    __shared__ double dsh[LT];
    __shared__ int anyNz;
    if (*(volatile int*)S.fail) return;
    const int2 job = S.rowJobs[j0 + blockIdx.x];   // (panel, index in its row; -1: the panel's y)
    const int p = job.x, tid = threadIdx.x;
    if (skip_tile(S, p)) return;
    const bool yj = job.y < 0;   // fused forward sweep: y_p as one more column of the panel row
    if (yj && !S.yfused) return;
    const int pw = S.th[p];
    const double* D = S.U + (size_t)S.slotOf[(size_t)p * S.nt + p] * (LT * LT);
    {   // L of the panel from its factored diagonal tile: 16 coalesced row loads in flight per thread
        const int col = tid & 63, r0 = tid >> 6;
        double v[LT / 4];
#pragma unroll
        for (int u = 0; u < LT / 4; u++) v[u] = D[(r0 + 4 * u) * LT + col];
#pragma unroll
        for (int u = 0; u < LT / 4; u++) {
            const int r = r0 + 4 * u;
            Ls[col * LP + r] = (col < pw && r > col) ? v[u] : 0.0;
        }
        if (tid < LT) dsh[tid] = tid < pw ? D[tid * LT + tid] : 1.0;
        if (tid == 0) anyNz = 0;
    }
    __syncthreads();
    const int e = S.rowStart[p] + (yj ? 0 : job.y);
    const int sl = S.rowSlot[e];   // (a y job keeps a valid slot: its descriptors are never used to store)
    const __amdgpu_buffer_rsrc_t Ut = tile_rsrc(S.U + (size_t)sl * (LT * LT));
    const __amdgpu_buffer_rsrc_t Lo = tile_rsrc(S.LT + (size_t)sl * (LT * LT));
    const int w = tid >> 6, lane = tid & 63, s = lane & 3, j = 16 * w + (lane >> 2);
    const int vo = j * 8;
    double* yp = S.y + p * LT;
    double c[LT / 4];   // c[q] = tile row 4 (m + q) + s of column j (m: the pivot group)
    if (yj) {
#pragma unroll
        for (int q = 0; q < LT / 4; q++) c[q] = j == 0 ? yp[4 * q + s] : 0.0;
    } else {
#pragma unroll
        for (int q = 0; q < LT / 4; q++) c[q] = tld(Ut, vo, (4 * q + s) * LT * 8);
    }
    bool nz = false;
    for (int m = 0; m < LT / 4; m++) {
        if (4 * m >= pw) break;
#pragma unroll
        for (int t = 0; t < 4; t++) {
            const int k = 4 * m + t;
            if (k < pw) {
                const double ck = quad_bcast(c[0], t);   // row k of column j: final
                if (s == t) {
                    if (yj) {
                        if (j == 0) yp[k] = ck;
                    } else {
                        tst(Ut, ck, vo, k * LT * 8);
                        tst(Lo, ck / dsh[k], vo, k * LT * 8);
                        nz |= ck != 0.0;
                    }
                }
                const double* Lk = Ls + k * LP + 4 * m + s;   // Lk[4 q] = L[4 (m + q) + s][k]
                {
                    const double v = c[0] - Lk[0] * ck;
                    c[0] = s > t ? v : c[0];
                }
#pragma unroll
                for (int g = 0; g < 4; g++) {
                    if (4 * g <= LT / 4 - 1 - m) {   // registers 4g..4g+3 hold some live row
#pragma unroll
                        for (int q = 4 * g; q < 4 * g + 4; q++)
                            if (q > 0) c[q] -= Lk[4 * q] * ck;
                    }
                }
                __builtin_amdgcn_sched_barrier(0);
            }
        }
#pragma unroll
        for (int q = 0; q < LT / 4 - 1; q++) c[q] = c[q + 1];
        c[LT / 4 - 1] = 0.0;
    }
    if (yj) return;   // uniform: the y job stores nothing else
#pragma unroll
    for (int q = 0; q < LT / 4; q++) {   // padding rows of L^T: zero
        const int r = 4 * q + s;
        if (r >= pw) tst(Lo, 0.0, vo, r * LT * 8);
    }
    // flag = some eliminated U[k][j] != 0, a superset of "some l != 0": skipping on it is exact
    if (__any(nz) && lane == 0) atomicOr(&anyNz, 1);
    __syncthreads();
    if (tid == 0) S.lnz[sl] = anyNz ? 1 : 0;
}

// The diagonal tile with the same four-wave quad layout.  Pivot k: the quad of column k
// publishes d_k; after a barrier every column's quad forms its l = u_kj / d_k (the column index
// as a row index), stores row k of the tile (U right of the diagonal, the earlier pivots' L left
// of it) and publishes l; after a second barrier every lane applies pivot k to its rows below k.
// Per element the oracle's sequence; lower-triangle registers carry values nobody reads.
__global__ void __launch_bounds__(256) k_ldlt_pdiag4(SpDev S, int j0) {
    __shared__ double Ls[LT * LP + 4 * LT];   // [k][i] = L[i][k]; the pad keeps dead-row reads in bounds
    __shared__ double dk[2];
    if (*(volatile int*)S.fail) return;
    const int p = S.stepP[j0 + blockIdx.x];
    if (skip_tile(S, p)) return;
    const int tid = threadIdx.x;
    const int pw = S.th[p];
    const __amdgpu_buffer_rsrc_t Ud = tile_rsrc(S.U + (size_t)S.slotOf[(size_t)p * S.nt + p] * (LT * LT));
    const int w = tid >> 6, lane = tid & 63, s = lane & 3, j = 16 * w + (lane >> 2);
    const int vo = j * 8;
    double c[LT / 4];   // c[q] = tile row 4 (m + q) + s of column j
#pragma unroll
    for (int q = 0; q < LT / 4; q++) c[q] = tld(Ud, vo, (4 * q + s) * LT * 8);
    bool bad = false;
    for (int m = 0; m < LT / 4 && !bad; m++) {
        if (4 * m >= pw) break;
#pragma unroll
        for (int t = 0; t < 4; t++) {
            const int k = 4 * m + t;
            if (k < pw && !bad) {
                const double ck = quad_bcast(c[0], t);   // row k of column j: final
                if (j == k && s == t) dk[k & 1] = ck;
                __syncthreads();
                const double d = dk[k & 1];
                if (d == 0.0) {   // uniform
                    bad = true;
                } else {
                    if (s == t) {
                        if (j < pw) tst(Ud, j >= k ? ck : Ls[j * LP + k], vo, k * LT * 8);
                        Ls[k * LP + j] = j > k ? ck / d : 0.0;   // L[j][k]
                    }
                    __syncthreads();
                    const double* Lk = Ls + k * LP + 4 * m + s;   // Lk[4 q] = L[4 (m + q) + s][k]
                    {
                        const double v = c[0] - Lk[0] * ck;
                        c[0] = s > t ? v : c[0];
                    }
#pragma unroll
                    for (int g = 0; g < 4; g++) {
                        if (4 * g <= LT / 4 - 1 - m) {
#pragma unroll
                            for (int q = 4 * g; q < 4 * g + 4; q++)
                                if (q > 0) c[q] -= Lk[4 * q] * ck;
                        }
                    }
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
        }
#pragma unroll
        for (int q = 0; q < LT / 4 - 1; q++) c[q] = c[q + 1];
        c[LT / 4 - 1] = 0.0;
    }
    if (bad && tid == 0) *S.fail = 1;
}

// ORBGPU_LDLT_PROW=1 keeps the one-wave panel-row kernel (A/B)
static bool prow_quads() {
    static const bool v = [] {
        const char* e = getenv("ORBGPU_LDLT_PROW");
        return !(e && e[0] == '1');
    }();
    return v;
}

// ORBGPU_LDLT_PDIAG4=1 takes the four-wave diagonal kernel
static bool pdiag_quads() {
    static const bool v = [] {
        const char* e = getenv("ORBGPU_LDLT_PDIAG4");
        return e && e[0] == '1';
    }();
    return v;
}

// ORBGPU_LDLT_ROLL=0 keeps the fully unrolled panel kernels (A/B)
static bool rolled_panels() {
    static const bool v = [] {
        const char* e = getenv("ORBGPU_LDLT_ROLL");
        return !(e && e[0] == '0');
    }();
    return v;
}

// A panel step's diagonal factorisation and its panel row's eliminations in ONE launch
// (k_ldlt_pdiag_r + k_ldlt_prow4 fused): a 512-thread workgroup per group of up to 7 row tiles
// of a panel.  Wave 0 holds the diagonal tile (lane = column) and, per pivot k, publishes d_k and
// the column of L in LDS; after one barrier every wave applies pivot k to its own tile (wave
// 1 + r: row tile r of the group, lane = column; the fused forward sweep's y_p rides as one more
// role with its column in lane 0), so a row tile's elimination runs in lock step with the
// diagonal instead of after it, and the diagonal tile is not reloaded.  Every group of a panel
// factors the diagonal redundantly (the same operations); the first one stores it -- into the
// tile's unused L^T slot, since the other groups of the launch read the unfactored tile from U;
// the next launch (k_ldlt_ptrail_q's copy jobs) moves it into place.  Per element
// the sequence of k_ldlt_pdiag_r / k_ldlt_prow4: pivots ascending, l = u / d, a -= l * u, L^T =
// u / d_k; padding pivots (k >= pw) not applied.
// row tiles (or y) per workgroup beside the diagonal wave: R + 1 waves share the CU's FP64 issue,
// so R = 3 (one wave per SIMD) by default; ORBGPU_LDLT_PANEL_ROLES = 1 / 3 / 7 (A/B)
static int panel_roles() {
    static const int v = [] {
        const char* e = getenv("ORBGPU_LDLT_PANEL_ROLES");
        const int r = e ? atoi(e) : 3;
        return (r == 1 || r == 7) ? r : 3;
    }();
    return v;
}

template <int R>
__global__ void __launch_bounds__(64 * (1 + R)) k_ldlt_panel(SpDev S, int j0) {
    __shared__ double Ls[LT * LP];   // [k][i] = L[i][k] of the diagonal tile
    __shared__ double dsh[LT];
    __shared__ int sbad;
    if (*(volatile int*)S.fail) return;
    const int4 job = S.panelJobs[j0 + blockIdx.x];   // (panel, first role, roles, 0)
    const int p = job.x;
    if (skip_tile(S, p)) return;
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int pw = S.th[p];
    const int rs = S.rowStart[p], nrow = S.rowStart[p + 1] - rs;
    const int role = w == 0 ? -1 : job.y + w - 1;   // -1 diagonal; [0, nrow) a row tile; nrow: y_p
    const bool active = w == 0 || (w - 1 < job.z && (role < nrow || S.yfused));
    const bool yrole = role == nrow;
    const bool storeDiag = job.y == 0;
    const int vo = lane * 8;
    const int sl = (role >= 0 && role < nrow) ? S.rowSlot[rs + role] : S.slotOf[(size_t)p * S.nt + p];
    const __amdgpu_buffer_rsrc_t Ut = tile_rsrc(S.U + (size_t)sl * (LT * LT));
    const __amdgpu_buffer_rsrc_t Lo = tile_rsrc(S.LT + (size_t)sl * (LT * LT));
    double* yp = S.y + p * LT;
    if (threadIdx.x == 0) sbad = 0;
    double col[LT];   // col[r] = tile row kb + r of column `lane` (kb: the chunk's first pivot)
    if (yrole) {
#pragma unroll
        for (int r = 0; r < LT; r++) col[r] = lane == 0 ? yp[r] : 0.0;
    } else if (active) {
#pragma unroll
        for (int r = 0; r < LT; r++) col[r] = tld(Ut, vo, r * LT * 8);   // zero outside the system
    } else {
#pragma unroll
        for (int r = 0; r < LT; r++) col[r] = 0.0;
    }
    __syncthreads();
    bool nz = false, bad = false;
    for (int c = 0; c < LT / kChunk && !bad; c++) {
        const int kb = kChunk * c;
        if (kb >= pw) break;
#pragma unroll
        for (int t = 0; t < kChunk; t++) {
            const int k = kb + t;
            if (k < pw && !bad) {
                if (w == 0) {   // pivot k: d_k and the column of L
                    const double d = rdlane(col[t], k);
                    if (d == 0.0) {
                        if (lane == 0) sbad = 1;
                    } else {
                        Ls[k * LP + lane] = lane > k ? col[t] / d : 0.0;
                        if (lane == 0) dsh[k] = d;
                    }
                }
                __syncthreads();
                if (sbad) {
                    bad = true;
                } else {
                    const double ck = col[t];   // row k: final (pivots < k applied)
                    if (w == 0) {
                        if (storeDiag && lane < pw) tst(Lo, lane >= k ? ck : Ls[lane * LP + k], vo, k * LT * 8);
                    } else if (yrole) {
                        if (lane == 0) yp[k] = ck;
                    } else if (active) {
                        tst(Ut, ck, vo, k * LT * 8);
                        tst(Lo, ck / dsh[k], vo, k * LT * 8);
                        nz |= ck != 0.0;
                    }
#pragma unroll
                    for (int q = 0; q < LT / kChunk; q++) {
                        if (q < LT / kChunk - c) {   // registers 8q..8q+7 hold live rows
#pragma unroll
                            for (int r = kChunk * q; r < kChunk * q + kChunk; r++)
                                if (r > t) col[r] -= Ls[k * LP + kb + r] * col[t];
                        }
                    }
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
        }
#pragma unroll
        for (int r = 0; r < LT - kChunk; r++) col[r] = col[r + kChunk];
    }
    if (bad) {
        if (threadIdx.x == 0) *S.fail = 1;
        return;
    }
    if (w > 0 && active && !yrole) {
        for (int r = pw; r < LT; r++) tst(Lo, 0.0, vo, r * LT * 8);   // padding rows of L^T: zero
        // flag = some eliminated U[k][j] != 0, a superset of "some l != 0": skipping on it is exact
        const bool any = __any(nz);
        if (lane == 0) S.lnz[sl] = any ? 1 : 0;
    }
}

// ORBGPU_LDLT_PANEL=0 keeps the separate diagonal and panel-row launches (A/B)
static bool fused_panels() {
    static const bool v = [] {
        const char* e = getenv("ORBGPU_LDLT_PANEL");
        return !(e && e[0] == '0');
    }();
    return v;
}

// Trailing updates inside the nodes: A(I, J) -= L(I, p) U(p, J), one 256-thread workgroup per
// target of the step (4 x 4 register micro-tiles, both operand tiles staged in LDS).
__global__ void __launch_bounds__(256) k_ldlt_ptrail(SpDev S, int j0) {
    __shared__ double Lg[LT * LT];   // [k][i] = L[I0 + i][p0 + k]
    __shared__ double Ug[LT * LT];   // [k][j] = U[p0 + k][J0 + j]
    if (*(volatile int*)S.fail) return;
    const int2 job = S.pairJobs[j0 + blockIdx.x];   // (panel, pair index)
    const int p = job.x;
    if (job.y < 0 || skip_tile(S, p)) return;   // (y jobs: the quadrant kernel's only)
    const int rs = S.rowStart[p];
    const int4 pr = S.pairs[S.pairStart[p] + job.y];
    const int slI = S.rowSlot[rs + pr.x], slJ = S.rowSlot[rs + pr.y];
    if (!S.lnz[slI] || !S.lnz[slJ]) return;   // block-uniform
    const int gt = threadIdx.x, ty = gt >> 4, tx = gt & 15;
    const double2* srcL = (const double2*)(S.LT + (size_t)slI * (LT * LT));
    const double2* srcU = (const double2*)(S.U + (size_t)slJ * (LT * LT));
#pragma unroll
    for (int u = 0; u < (LT * LT / 2) / 256; u++) {
        ((double2*)Lg)[gt + 256 * u] = srcL[gt + 256 * u];
        ((double2*)Ug)[gt + 256 * u] = srcU[gt + 256 * u];
    }
    __syncthreads();
    const int I = S.rowJ[rs + pr.x], J = S.rowJ[rs + pr.y];
    const int ih = S.th[I], jw = S.th[J], pw = S.th[p];
    double* T = S.U + (size_t)pr.z * (LT * LT);
    double acc[4][4];
#pragma unroll
    for (int a = 0; a < 4; a++)
#pragma unroll
        for (int bb = 0; bb < 4; bb++) {
            const int i = ty + 16 * a, j = tx + 16 * bb;
            acc[a][bb] = (i < ih && j < jw) ? T[i * LT + j] : 0.0;
        }
    for (int k = 0; k < pw; k++) {
        double l[4], u[4];
#pragma unroll
        for (int a = 0; a < 4; a++) l[a] = Lg[k * LT + ty + 16 * a];
#pragma unroll
        for (int bb = 0; bb < 4; bb++) u[bb] = Ug[k * LT + tx + 16 * bb];
#pragma unroll
        for (int a = 0; a < 4; a++)
#pragma unroll
            for (int bb = 0; bb < 4; bb++) acc[a][bb] -= l[a] * u[bb];
    }
#pragma unroll
    for (int a = 0; a < 4; a++)
#pragma unroll
        for (int bb = 0; bb < 4; bb++) {
            const int i = ty + 16 * a, j = tx + 16 * bb;
            if (i < ih && j < jw && (I != J || i <= j)) T[i * LT + j] = acc[a][bb];
        }
}

// Quadrant forms of k_ldlt_update / k_ldlt_ptrail.  A 64 x 64 tile update is 524 k FP64
// operations per pivot tile K: one CU (four SIMDs, 16 FP64 lanes each) needs >= 8 k cycles per K
// whatever its thread count, and a top-level target gathers tens of descendant K in sequence.
// Four workgroups per target tile, each owning a 32 x 32 quadrant (qi, qj), put four CUs on it:
// 256 threads, 2 x 2 register micro-tiles (rows 2ty, 2ty+1, columns 2tx, 2tx+1, each pair one
// 16-B LDS read), per K the quadrant's 32 rows of L(I, K) and 32 columns of U(K, J) staged in LDS
// (2 x 16 KB) while the next K's operands are already in flight to registers.  Per element the
// sequence is unchanged (K ascending, k ascending, a -= l * u with one rounding per product and
// per subtraction): the split is spatial only, so the factor is bit-identical.
constexpr int LQ = LT / 2;   // quadrant edge

typedef double d2v __attribute__((ext_vector_type(2)));   // native vector: stays in registers (HIP's
                                                         // double2 wrapper was demoted to scratch here)
struct QuadOps {   // one K's operands of a quadrant, 4 x 16 B per thread and operand
    d2v l[4], u[4];
};
__device__ __forceinline__ void quad_load(QuadOps& o, const double* Lsrc, const double* Usrc, int qi, int qj, int gt) {
#pragma unroll
    for (int u = 0; u < 4; u++) {
        const int e = gt + 256 * u, k = e >> 4, c2 = e & 15;
        o.l[u] = *(const d2v*)(Lsrc + k * LT + LQ * qi + 2 * c2);
        o.u[u] = *(const d2v*)(Usrc + k * LT + LQ * qj + 2 * c2);
    }
}
__device__ __forceinline__ void quad_stage(const QuadOps& o, d2v* Lg, d2v* Ug, int gt) {
#pragma unroll
    for (int u = 0; u < 4; u++) {
        Lg[gt + 256 * u] = o.l[u];   // [k][pair of quadrant rows]
        Ug[gt + 256 * u] = o.u[u];   // [k][pair of quadrant columns]
    }
}
__device__ __forceinline__ void quad_apply(double (&acc)[2][2], const d2v* Lg, const d2v* Ug, int kw, int ty,
                                           int tx) {
    for (int k = 0; k < kw; k++) {
        const d2v l = Lg[k * (LQ / 2) + ty];
        const d2v u = Ug[k * (LQ / 2) + tx];
        acc[0][0] -= l.x * u.x;
        acc[0][1] -= l.x * u.y;
        acc[1][0] -= l.y * u.x;
        acc[1][1] -= l.y * u.y;
    }
}
__device__ __forceinline__ void quad_init(double (&acc)[2][2], const double* T, int qi, int qj, int ty, int tx, int ih,
                                          int jw) {
#pragma unroll
    for (int a = 0; a < 2; a++)
#pragma unroll
        for (int b = 0; b < 2; b++) {
            const int i = LQ * qi + 2 * ty + a, j = LQ * qj + 2 * tx + b;
            acc[a][b] = (i < ih && j < jw) ? T[i * LT + j] : 0.0;
        }
}
__device__ __forceinline__ void quad_store(const double (&acc)[2][2], double* T, int qi, int qj, int ty, int tx, int ih,
                                           int jw, bool diag) {
#pragma unroll
    for (int a = 0; a < 2; a++)
#pragma unroll
        for (int b = 0; b < 2; b++) {
            const int i = LQ * qi + 2 * ty + a, j = LQ * qj + 2 * tx + b;
            if (i < ih && j < jw && (!diag || i <= j)) T[i * LT + j] = acc[a][b];
        }
}

// the first K pair at or after q that contributes (block-uniform: every thread reads the same words)
__device__ __forceinline__ int upd_next(const SpDev& S, int q, int kp1) {
    for (; q < kp1; q++) {
        const int4 kp = S.kps[q];
        if (S.lnz[kp.x] && S.lnz[kp.y] && !skip_k(S, kp.z)) break;
    }
    return q;
}

// The forward substitution fused into the factorisation (SpDev::yfused): y_I -= L(I, K) y_K over
// the descendant pivot tiles of row I, K ascending, k ascending -- the oracle's forward sweep
// sequence for those terms -- run by the quadrant (1, 0) workgroup of the diagonal target (I, I),
// which nobody else needs (its K list is every descendant K with L(I, K) != 0).  All four waves
// stage each L(I, K) tile and y_K in LDS (the next ones in flight), wave 0 runs the 64 row chains.
__device__ void upd_y(const SpDev& S, int I, int kp0, int kp1, d2v* sh, double* ysh) {
    const int gt = threadIdx.x, lane = gt & 63, w = gt >> 6;
    d2v lr[8];
    double yr = 0.0;
    auto load = [&](int q) {
        const int4 kp = S.kps[q];
        const double* Lo = S.LT + (size_t)kp.x * (LT * LT);
#pragma unroll
        for (int u = 0; u < 8; u++) lr[u] = *(const d2v*)(Lo + 2 * (gt + 256 * u));   // [k][i] row-major pairs
        if (gt < LT) yr = S.y[kp.z * LT + gt];
    };
    double acc = S.y[I * LT + lane];
    int q = upd_next(S, kp0, kp1);
    int4 kp = S.kps[q < kp1 ? q : kp0];
    load(q < kp1 ? q : kp0);
    while (q < kp1) {
        const int kw = S.th[kp.z];
        __syncthreads();
#pragma unroll
        for (int u = 0; u < 8; u++) sh[gt + 256 * u] = lr[u];
        if (gt < LT) ysh[gt] = yr;
        __syncthreads();
        q = upd_next(S, q + 1, kp1);
        if (q < kp1) kp = S.kps[q];
        load(q < kp1 ? q : kp0);
        if (w == 0) {
            const double* Lf = (const double*)sh;   // Lf[k * 64 + i] = L[I0 + i][K0 + k]
            for (int k = 0; k < kw; k++) acc = acc - Lf[k * LT + lane] * ysh[k];
        }
    }
    if (w == 0) S.y[I * LT + lane] = acc;
}

__global__ void __launch_bounds__(256) k_ldlt_update_q(SpDev S, int t0) {
    __shared__ d2v Lg[LT * LQ];   // [0, LT * LQ / 2): L quadrant; then U quadrant (the y path: one L tile)
    __shared__ double ysh[LT];
    d2v* Ug = Lg + LT * LQ / 2;
    if (*(volatile int*)S.fail) return;
    const int ti = t0 + (blockIdx.x >> 2), qd = blockIdx.x & 3, qi = qd >> 1, qj = qd & 1;
    const int4 tg = S.tgts[ti];
    const int kp0 = tg.w, kp1 = S.tgts[ti + 1].w;
    const int I = tg.y, J = tg.z;
    if (skip_tile(S, I)) return;
    if (I == J && qi > qj) {   // the quadrant nobody stores: the fused forward sweep's descendant terms
        if (S.yfused) upd_y(S, I, kp0, kp1, Lg, ysh);
        return;
    }
    const int ih = S.th[I], jw = S.th[J];
    if ((I == J && qi > qj) || LQ * qi >= ih || LQ * qj >= jw) return;   // a quadrant nobody stores
    const int gt = threadIdx.x, ty = gt >> 4, tx = gt & 15;
    double* T = S.dst ? S.dst + (size_t)S.packIdx[tg.x] * (LT * LT) : S.U + (size_t)tg.x * (LT * LT);
    double acc[2][2];
    quad_init(acc, T, qi, qj, ty, tx, ih, jw);
    // (the operand loads are unconditional -- past the last K they re-read its tiles -- so the
    // register buffer is not demoted to scratch; a target always has a K pair, k_ldlt build)
    QuadOps ops;
    int q = upd_next(S, kp0, kp1);
    int4 kp = S.kps[q < kp1 ? q : kp0];
    quad_load(ops, S.LT + (size_t)kp.x * (LT * LT), S.U + (size_t)kp.y * (LT * LT), qi, qj, gt);
    int4 kc = S.kps[q + 1 < kp1 ? q + 1 : kp0];   // the next candidate's pair, one iteration ahead
    while (q < kp1) {
        const int kw = S.th[kp.z];
        __syncthreads();   // the previous K's LDS reads are done
        quad_stage(ops, Lg, Ug, gt);
        __syncthreads();
        // the next K is usually the next pair: its operands are requested right away, with its
        // flags in flight beside them (no dependent flag round trip before the loads); a pair the
        // flags rule out (an exactly zero L tile) is replaced after this K's compute
        int qn = q + 1;
        int4 kn = qn < kp1 ? kc : kp;
        quad_load(ops, S.LT + (size_t)kn.x * (LT * LT), S.U + (size_t)kn.y * (LT * LT), qi, qj, gt);
        const bool ok = qn < kp1 && S.lnz[kn.x] && S.lnz[kn.y] && !skip_k(S, kn.z);
        kc = S.kps[qn + 1 < kp1 ? qn + 1 : kp0];
        quad_apply(acc, Lg, Ug, kw, ty, tx);
        if (qn < kp1 && !ok) {   // (block-uniform)
            qn = upd_next(S, qn + 1, kp1);
            kn = qn < kp1 ? S.kps[qn] : kp;
            quad_load(ops, S.LT + (size_t)kn.x * (LT * LT), S.U + (size_t)kn.y * (LT * LT), qi, qj, gt);
            kc = S.kps[qn + 1 < kp1 ? qn + 1 : kp0];
        }
        q = qn;
        kp = kn;
    }
    quad_store(acc, T, qi, qj, ty, tx, ih, jw, I == J);
}

__global__ void __launch_bounds__(256) k_ldlt_ptrail_q(SpDev S, int j0) {
    __shared__ d2v Lg[LT * LQ / 2];
    __shared__ d2v Ug[LT * LQ / 2];
    if (*(volatile int*)S.fail) return;
    const int2 job = S.pairJobs[j0 + (blockIdx.x >> 2)];   // (panel, pair index)
    const int qd = blockIdx.x & 3, qi = qd >> 1, qj = qd & 1;
    const int p = job.x;
    if (skip_tile(S, p)) return;
    const int rs = S.rowStart[p];
    if (job.y == kDiagCopyJob) {   // k_ldlt_panel's factored diagonal tile: L^T shadow -> U, a quarter each
        if (!S.pfused) return;
        const size_t sd = (size_t)S.slotOf[(size_t)p * S.nt + p] * (LT * LT);
        const d2v* src = (const d2v*)(S.LT + sd) + qd * (LT * LT / 8);
        d2v* dst = (d2v*)(S.U + sd) + qd * (LT * LT / 8);
        for (int u = threadIdx.x; u < LT * LT / 8; u += 256) dst[u] = src[u];
        return;
    }
    if (job.y < 0) {   // fused forward sweep: y_I -= L(I, p) y_p, I = the panel row's entry -1 - job.y
        if (!S.yfused || qd != 0 || threadIdx.x >= LT) return;
        const int e = rs - 1 - job.y, sl = S.rowSlot[e], I = S.rowJ[e], lane = threadIdx.x;
        if (!S.lnz[sl]) return;
        double* ysh = (double*)Lg;
        ysh[lane] = S.y[p * LT + lane];
        __builtin_amdgcn_wave_barrier();
        const double* Lo = S.LT + (size_t)sl * (LT * LT);   // [k][i] = L[I0 + i][p0 + k]
        const int pw = S.th[p];
        double acc = S.y[I * LT + lane];
        for (int k = 0; k < pw; k++) acc = acc - Lo[k * LT + lane] * ysh[k];
        S.y[I * LT + lane] = acc;
        return;
    }
    const int4 pr = S.pairs[S.pairStart[p] + job.y];
    const int slI = S.rowSlot[rs + pr.x], slJ = S.rowSlot[rs + pr.y];
    if (!S.lnz[slI] || !S.lnz[slJ]) return;   // block-uniform
    const int I = S.rowJ[rs + pr.x], J = S.rowJ[rs + pr.y];
    const int ih = S.th[I], jw = S.th[J], pw = S.th[p];
    if ((I == J && qi > qj) || LQ * qi >= ih || LQ * qj >= jw) return;
    const int gt = threadIdx.x, ty = gt >> 4, tx = gt & 15;
    QuadOps ops;
    quad_load(ops, S.LT + (size_t)slI * (LT * LT), S.U + (size_t)slJ * (LT * LT), qi, qj, gt);
    double* T = S.U + (size_t)pr.z * (LT * LT);
    double acc[2][2];
    quad_init(acc, T, qi, qj, ty, tx, ih, jw);
    quad_stage(ops, Lg, Ug, gt);
    __syncthreads();
    quad_apply(acc, Lg, Ug, pw, ty, tx);
    quad_store(acc, T, qi, qj, ty, tx, ih, jw, I == J);
}

// ORBGPU_LDLT_QUAD=0 keeps the one-workgroup-per-tile update and trailing kernels (A/B)
static bool quad_updates() {
    static const bool v = [] {
        const char* e = getenv("ORBGPU_LDLT_QUAD");
        return !(e && e[0] == '0');
    }();
    return v;
}

// L y = b on the rows of each node of a level (one wave per node; lane = row): the descendants'
// y are final.
__global__ void __launch_bounds__(64) k_ldlt_pfwd(SpDev S, int n0, const double* __restrict__ b) {
    if (*(volatile int*)S.fail) return;
    const int node = S.levNodes[n0 + blockIdx.x];
    const int T0 = S.nodeT[2 * node], T1 = S.nodeT[2 * node + 1];
    if (T1 > T0 && skip_tile(S, T0)) return;
    const int lane = threadIdx.x;
    double Lr[LT];
    for (int I = T0; I < T1; I++) {
        const int I0 = I * LT, ih = S.th[I];
        const bool on = lane < ih;
        double acc = on ? b[S.rowMap[I0 + lane]] : 0.0;
        for (int e = S.colStart[I]; e < S.colStart[I + 1]; e++) {
            const int sl = S.colSlot[e];
            if (!S.lnz[sl] || skip_k(S, S.colK[e])) continue;
            const int K = S.colK[e], K0 = K * LT, kh = S.th[K];
            const double yk = S.y[K0 + lane];
            const double* Lo = S.LT + (size_t)sl * (LT * LT);   // [k][i] = L[I0 + i][K0 + k]
#pragma unroll
            for (int k = 0; k < LT; k++) Lr[k] = Lo[k * LT + lane];
#pragma unroll
            for (int k = 0; k < LT; k++) {
                if (k < kh) {
                    const double v = acc - Lr[k] * rdlane(yk, k);
                    acc = on ? v : acc;
                }
            }
        }
        const double* Ud = S.U + (size_t)S.slotOf[(size_t)I * S.nt + I] * (LT * LT);
#pragma unroll
        for (int k = 0; k < LT; k++) Lr[k] = (on && k < lane) ? Ud[lane * LT + k] : 0.0;
#pragma unroll
        for (int k = 0; k < LT; k++) {
            if (k < ih) {
                const double yk = rdlane(acc, k);
                const double v = acc - Lr[k] * yk;
                acc = (on && lane > k) ? v : acc;
            }
        }
        S.y[I0 + lane] = on ? acc : 0.0;
    }
}

// The fused forward sweep's start: y = b in tile space (padding rows 0), a wave per tile.
__global__ void __launch_bounds__(64) k_ldlt_yinit(SpDev S, const double* __restrict__ b) {
    const int I = blockIdx.x, lane = threadIdx.x;
    S.y[I * LT + lane] = lane < S.th[I] ? b[S.rowMap[I * LT + lane]] : 0.0;
}

// y /= d, then L^T x = y with k descending: one wave per node of a level (levels top-down);
// the rows of a node's ancestors are final.  The first launch also publishes the outcome.
__global__ void __launch_bounds__(64) k_ldlt_backward(SpDev S, int n0, double* __restrict__ x, double* scal,
                                                      int first) {
    const int lane = threadIdx.x;
    const int failed = *(volatile int*)S.fail;
    if (first && blockIdx.x == 0 && lane == 0) scal[3] = failed ? 0.0 : 1.0;
    if (failed) return;
    const int node = S.levNodes[n0 + blockIdx.x];
    const int T0 = S.nodeT[2 * node], T1 = S.nodeT[2 * node + 1];
    if (T1 > T0 && skip_tile(S, T0)) return;
    double Lr[LT];
    for (int I = T1 - 1; I >= T0; I--) {
        const int I0 = I * LT, ih = S.th[I];
        const bool on = lane < ih;
        const double* Ud = S.U + (size_t)S.slotOf[(size_t)I * S.nt + I] * (LT * LT);
        double acc = on ? S.y[I0 + lane] / Ud[lane * LT + lane] : 0.0;
        for (int e = S.rowStart[I + 1] - 1; e >= S.rowStart[I]; e--) {
            const int sl = S.rowSlot[e];
            if (!S.lnz[sl]) continue;
            const int K0 = S.rowJ[e] * LT, kh = S.th[S.rowJ[e]];
            const double xk = lane < kh ? S.xs[K0 + lane] : 0.0;
            const double* Lo = S.LT + (size_t)sl * (LT * LT);   // [i][k] = L[K0 + k][I0 + i]
#pragma unroll
            for (int k = 0; k < LT; k++) Lr[k] = on ? Lo[lane * LT + k] : 0.0;
#pragma unroll
            for (int k = LT - 1; k >= 0; k--) {
                if (k < kh) {
                    const double v = acc - Lr[k] * rdlane(xk, k);
                    acc = on ? v : acc;
                }
            }
        }
#pragma unroll
        for (int k = 0; k < LT; k++) Lr[k] = (on && k < ih) ? Ud[k * LT + lane] : 0.0;   // L[I0 + k][I0 + lane]
#pragma unroll
        for (int k = LT - 1; k >= 0; k--) {
            if (k < ih) {
                const double xk = rdlane(acc, k);
                const double v = acc - Lr[k] * xk;
                acc = (on && lane < k) ? v : acc;
            }
        }
        S.xs[I0 + lane] = on ? acc : 0.0;
        if (on) x[S.rowMap[I0 + lane]] = acc;
    }
}

// The sweeps with a workgroup per node and a wave per tile row of the node (tile I = T0 + w + W r),
// the rows' accumulators in LDS.  Per row the subtractions keep the sequence of k_ldlt_pfwd /
// k_ldlt_backward (forward: k ascending; backward: k descending): first every contribution from
// outside the node (descendant tiles forward, ancestor tiles backward; their y / x are final),
// all rows in parallel; then the node's own tiles one at a time -- the owner finishes tile K
// with its diagonal tile, and after a barrier every row still waiting applies tile K's block.
// Rows of off lanes (lane >= th) compute values nobody reads, so the chains carry no selects.
constexpr int kSweepWaves = 8;
constexpr int kSweepMaxTiles = 240;   // node tiles whose accumulators fit the LDS (120 KB)

__device__ __forceinline__ double sweep_chain_fwd(double acc, const double* Lo, int lane, double yk, int kh) {
    double Lr[LT];
#pragma unroll
    for (int k = 0; k < LT; k++) Lr[k] = Lo[k * LT + lane];   // L[I0 + lane][K0 + k]
#pragma unroll
    for (int k = 0; k < LT; k++)
        if (k < kh) acc = acc - Lr[k] * rdlane(yk, k);
    return acc;
}
__device__ __forceinline__ double sweep_chain_bwd(double acc, const double* Lo, int lane, double xk, int kh) {
    double Lr[LT];
#pragma unroll
    for (int k = 0; k < LT; k++) Lr[k] = Lo[lane * LT + k];   // L[K0 + k][I0 + lane]
#pragma unroll
    for (int k = LT - 1; k >= 0; k--)
        if (k < kh) acc = acc - Lr[k] * rdlane(xk, k);
    return acc;
}

// The same chains with the pivot values read as wave-uniform LDS operands (vsh[k], one broadcast
// read each) instead of a cross-lane readlane per step: the products no longer wait on a
// broadcast, and the chain is one dependent subtraction per step.
__device__ __forceinline__ double sweep_chain_fwd_u(double acc, const double* Lo, int lane, const double* vsh, int kh) {
    double Lr[LT];
#pragma unroll
    for (int k = 0; k < LT; k++) Lr[k] = Lo[k * LT + lane];   // L[I0 + lane][K0 + k]
#pragma unroll
    for (int k = 0; k < LT; k++)
        if (k < kh) acc = acc - Lr[k] * vsh[k];
    return acc;
}
__device__ __forceinline__ double sweep_chain_bwd_u(double acc, const double* Lo, int lane, const double* vsh, int kh) {
    double Lr[LT];
#pragma unroll
    for (int k = 0; k < LT; k++) Lr[k] = Lo[lane * LT + k];   // L[K0 + k][I0 + lane]
#pragma unroll
    for (int k = LT - 1; k >= 0; k--)
        if (k < kh) acc = acc - Lr[k] * vsh[k];
    return acc;
}

// A tile row's contributions from outside its node, software-pipelined over the row's pivot tiles:
// 16-row chunks of each L tile double-buffered in registers (the next chunk, and at a tile's last
// chunk the next tile's first, in flight while one is applied), the tile's y / x staged in the
// wave's LDS slot `vsh` and read wave-uniform.  Forward: descendant tiles K < T0, K ascending, k
// ascending; backward: ancestor tiles J >= T1, J descending, k descending.  Per row the
// subtraction sequence of k_ldlt_pfwd / k_ldlt_backward.  *eStop: the first list entry inside the
// node (forward) / the last one inside it (backward).
constexpr int SCH = 16;   // pivot rows per register chunk
__device__ __forceinline__ void fwd_chunk_load(double (&r)[SCH], const double* Lo, int c, int lane) {
#pragma unroll
    for (int t = 0; t < SCH; t++) r[t] = Lo[(SCH * c + t) * LT + lane];
}
__device__ __forceinline__ double fwd_chunk_apply(double acc, const double (&r)[SCH], const double* vsh, int c, int kh) {
#pragma unroll
    for (int t = 0; t < SCH; t++)
        if (SCH * c + t < kh) acc = acc - r[t] * vsh[SCH * c + t];
    return acc;
}
__device__ double fwd_outside(const SpDev& S, int I, int T0, double acc, int lane, double* vsh, int* eStop) {
    const int e1 = S.colStart[I + 1];
    int eS = S.colStart[I];
    while (eS < e1 && S.colK[eS] < T0) eS++;   // ascending K: the descendants come first
    *eStop = eS;
    auto nextv = [&](int e) {
        while (e < eS && (!S.lnz[S.colSlot[e]] || skip_k(S, S.colK[e]))) e++;
        return e;
    };
    int e = nextv(S.colStart[I]);
    double A[SCH], Bq[SCH];
    double yv = 0.0;
    if (e < eS) {
        fwd_chunk_load(A, S.LT + (size_t)S.colSlot[e] * (LT * LT), 0, lane);
        yv = S.y[S.colK[e] * LT + lane];
    }
    while (e < eS) {
        const int kh = S.th[S.colK[e]];
        const double* Lo = S.LT + (size_t)S.colSlot[e] * (LT * LT);
        vsh[lane] = yv;
        __builtin_amdgcn_wave_barrier();
        const int en = nextv(e + 1);
        fwd_chunk_load(Bq, Lo, 1, lane);
        acc = fwd_chunk_apply(acc, A, vsh, 0, kh);
        fwd_chunk_load(A, Lo, 2, lane);
        acc = fwd_chunk_apply(acc, Bq, vsh, 1, kh);
        fwd_chunk_load(Bq, Lo, 3, lane);
        acc = fwd_chunk_apply(acc, A, vsh, 2, kh);
        if (en < eS) {   // the next tile's first chunk and y travel during this tile's last chunk
            fwd_chunk_load(A, S.LT + (size_t)S.colSlot[en] * (LT * LT), 0, lane);
            yv = S.y[S.colK[en] * LT + lane];
        }
        acc = fwd_chunk_apply(acc, Bq, vsh, 3, kh);
        __builtin_amdgcn_wave_barrier();
        e = en;
    }
    return acc;
}
__device__ __forceinline__ void bwd_chunk_load(double (&r)[SCH], const double* Lo, int c, int lane) {
#pragma unroll
    for (int t = 0; t < SCH; t += 2) {   // L[K0 + k][I0 + lane] for k = 16c + t, 16c + t + 1: one 16-B load
        const double2 v = *(const double2*)(Lo + lane * LT + SCH * c + t);
        r[t] = v.x;
        r[t + 1] = v.y;
    }
}
__device__ __forceinline__ double bwd_chunk_apply(double acc, const double (&r)[SCH], const double* vsh, int c, int kh) {
#pragma unroll
    for (int t = SCH - 1; t >= 0; t--)
        if (SCH * c + t < kh) acc = acc - r[t] * vsh[SCH * c + t];
    return acc;
}
__device__ double bwd_outside(const SpDev& S, int I, int T1, double acc, int lane, double* vsh, int* eStop) {
    const int e0 = S.rowStart[I];
    int eS = S.rowStart[I + 1] - 1;
    while (eS >= e0 && S.rowJ[eS] >= T1) eS--;   // descending J: the ancestors come first
    *eStop = eS;
    auto nextv = [&](int e) {
        while (e > eS && !S.lnz[S.rowSlot[e]]) e--;
        return e;
    };
    int e = nextv(S.rowStart[I + 1] - 1);
    double A[SCH], Bq[SCH];
    double xv = 0.0;
    if (e > eS) {
        bwd_chunk_load(A, S.LT + (size_t)S.rowSlot[e] * (LT * LT), 3, lane);
        const int J = S.rowJ[e];
        xv = lane < S.th[J] ? S.xs[J * LT + lane] : 0.0;
    }
    while (e > eS) {
        const int kh = S.th[S.rowJ[e]];
        const double* Lo = S.LT + (size_t)S.rowSlot[e] * (LT * LT);
        vsh[lane] = xv;
        __builtin_amdgcn_wave_barrier();
        const int en = nextv(e - 1);
        bwd_chunk_load(Bq, Lo, 2, lane);
        acc = bwd_chunk_apply(acc, A, vsh, 3, kh);
        bwd_chunk_load(A, Lo, 1, lane);
        acc = bwd_chunk_apply(acc, Bq, vsh, 2, kh);
        bwd_chunk_load(Bq, Lo, 0, lane);
        acc = bwd_chunk_apply(acc, A, vsh, 1, kh);
        if (en > eS) {
            bwd_chunk_load(A, S.LT + (size_t)S.rowSlot[en] * (LT * LT), 3, lane);
            const int J = S.rowJ[en];
            xv = lane < S.th[J] ? S.xs[J * LT + lane] : 0.0;
        }
        acc = bwd_chunk_apply(acc, Bq, vsh, 0, kh);
        __builtin_amdgcn_wave_barrier();
        e = en;
    }
    return acc;
}

// The node sweeps with the pipelined outside phase and wave-uniform LDS operands (ORBGPU_LDLT_SWEEP=2
// keeps k_ldlt_fwdn / k_ldlt_bwdn for A/B).  Same per-row sequences.
__global__ void __launch_bounds__(64 * kSweepWaves) k_ldlt_fwdn_u(SpDev S, int n0, const double* __restrict__ b) {
    extern __shared__ double accs[];   // [tile - T0][lane]
    __shared__ int cur[kSweepMaxTiles];
    __shared__ double vsh[kSweepWaves][LT];
    if (*(volatile int*)S.fail) return;
    const int node = S.levNodes[n0 + blockIdx.x];
    const int T0 = S.nodeT[2 * node], T1 = S.nodeT[2 * node + 1];
    if (T1 > T0 && skip_tile(S, T0)) return;
    const int W = blockDim.x >> 6, w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (int I = T0 + w; I < T1; I += W) {
        const int I0 = I * LT;
        double acc = lane < S.th[I] ? b[S.rowMap[I0 + lane]] : 0.0;
        int e;
        acc = fwd_outside(S, I, T0, acc, lane, vsh[w], &e);
        accs[(I - T0) * LT + lane] = acc;
        if (lane == 0) cur[I - T0] = e;
    }
    __syncthreads();
    for (int s = 0; s < T1 - T0; s++) {
        const int K = T0 + s, K0 = K * LT, kh = S.th[K];
        if (s % W == w) {   // the owner: diagonal tile, y_K final
            const bool on = lane < kh;
            double acc = accs[s * LT + lane];
            const double* Ud = S.U + (size_t)S.slotOf[(size_t)K * S.nt + K] * (LT * LT);
            double Lr[LT];
#pragma unroll
            for (int k = 0; k < LT; k++) Lr[k] = (on && k < lane) ? Ud[lane * LT + k] : 0.0;
#pragma unroll
            for (int k = 0; k < LT; k++) {
                if (k < kh) {
                    const double v = acc - Lr[k] * rdlane(acc, k);
                    acc = lane > k ? v : acc;
                }
            }
            acc = on ? acc : 0.0;
            S.y[K0 + lane] = acc;
            accs[s * LT + lane] = acc;
        }
        __syncthreads();
        for (int I = T0 + w; I < T1; I += W) {
            if (I <= K) continue;
            const int e = cur[I - T0];
            if (e >= S.colStart[I + 1] || S.colK[e] != K) continue;   // no block (K, I)
            if (lane == 0) cur[I - T0] = e + 1;
            const int sl = S.colSlot[e];
            if (!S.lnz[sl]) continue;
            accs[(I - T0) * LT + lane] =
                sweep_chain_fwd_u(accs[(I - T0) * LT + lane], S.LT + (size_t)sl * (LT * LT), lane, accs + s * LT, kh);
        }
        __syncthreads();
    }
}

__global__ void __launch_bounds__(64 * kSweepWaves) k_ldlt_bwdn_u(SpDev S, int n0, double* __restrict__ x, double* scal,
                                                                  int first) {
    extern __shared__ double accs[];
    __shared__ int cur[kSweepMaxTiles];
    __shared__ double vsh[kSweepWaves][LT];
    const int lane = threadIdx.x & 63;
    const int failed = *(volatile int*)S.fail;
    if (first && blockIdx.x == 0 && threadIdx.x == 0) scal[3] = failed ? 0.0 : 1.0;
    if (failed) return;
    const int node = S.levNodes[n0 + blockIdx.x];
    const int T0 = S.nodeT[2 * node], T1 = S.nodeT[2 * node + 1];
    if (T1 > T0 && skip_tile(S, T0)) return;
    const int W = blockDim.x >> 6, w = threadIdx.x >> 6;
    for (int I = T0 + w; I < T1; I += W) {
        const int I0 = I * LT;
        const double* Ud = S.U + (size_t)S.slotOf[(size_t)I * S.nt + I] * (LT * LT);
        double acc = lane < S.th[I] ? S.y[I0 + lane] / Ud[lane * LT + lane] : 0.0;
        int e;
        acc = bwd_outside(S, I, T1, acc, lane, vsh[w], &e);
        accs[(I - T0) * LT + lane] = acc;
        if (lane == 0) cur[I - T0] = e;
    }
    __syncthreads();
    for (int s = T1 - T0 - 1; s >= 0; s--) {
        const int K = T0 + s, K0 = K * LT, kh = S.th[K];
        if (s % W == w) {   // the owner: diagonal tile, x_K final
            const bool on = lane < kh;
            double acc = accs[s * LT + lane];
            const double* Ud = S.U + (size_t)S.slotOf[(size_t)K * S.nt + K] * (LT * LT);
            double Lr[LT];
#pragma unroll
            for (int k = 0; k < LT; k++) Lr[k] = (on && k < kh) ? Ud[k * LT + lane] : 0.0;   // L[K0 + k][K0 + lane]
#pragma unroll
            for (int k = LT - 1; k >= 0; k--) {
                if (k < kh) {
                    const double v = acc - Lr[k] * rdlane(acc, k);
                    acc = lane < k ? v : acc;
                }
            }
            acc = on ? acc : 0.0;
            S.xs[K0 + lane] = acc;
            if (on) x[S.rowMap[K0 + lane]] = acc;
            accs[s * LT + lane] = acc;
        }
        __syncthreads();
        for (int I = T0 + w; I < K; I += W) {
            const int e = cur[I - T0];
            if (e < S.rowStart[I] || S.rowJ[e] != K) continue;   // no block (I, K)
            if (lane == 0) cur[I - T0] = e - 1;
            const int sl = S.rowSlot[e];
            if (!S.lnz[sl]) continue;
            accs[(I - T0) * LT + lane] =
                sweep_chain_bwd_u(accs[(I - T0) * LT + lane], S.LT + (size_t)sl * (LT * LT), lane, accs + s * LT, kh);
        }
        __syncthreads();
    }
}

__global__ void __launch_bounds__(64 * kSweepWaves) k_ldlt_fwdn(SpDev S, int n0, const double* __restrict__ b) {
    extern __shared__ double accs[];   // [tile - T0][lane]
    __shared__ int cur[kSweepMaxTiles];   // the tile's first col-list entry inside the node
    if (*(volatile int*)S.fail) return;
    const int node = S.levNodes[n0 + blockIdx.x];
    const int T0 = S.nodeT[2 * node], T1 = S.nodeT[2 * node + 1];
    if (T1 > T0 && skip_tile(S, T0)) return;
    const int W = blockDim.x >> 6, w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (int I = T0 + w; I < T1; I += W) {
        const int I0 = I * LT;
        double acc = lane < S.th[I] ? b[S.rowMap[I0 + lane]] : 0.0;
        int e = S.colStart[I];
        for (; e < S.colStart[I + 1]; e++) {
            const int K = S.colK[e];
            if (K >= T0) break;   // ascending K: the descendants come first
            const int sl = S.colSlot[e];
            if (!S.lnz[sl] || skip_k(S, K)) continue;
            acc = sweep_chain_fwd(acc, S.LT + (size_t)sl * (LT * LT), lane, S.y[K * LT + lane], S.th[K]);
        }
        accs[(I - T0) * LT + lane] = acc;
        if (lane == 0) cur[I - T0] = e;
    }
    __syncthreads();
    for (int s = 0; s < T1 - T0; s++) {
        const int K = T0 + s, K0 = K * LT, kh = S.th[K];
        if (s % W == w) {   // the owner: diagonal tile, y_K final
            const bool on = lane < kh;
            double acc = accs[s * LT + lane];
            const double* Ud = S.U + (size_t)S.slotOf[(size_t)K * S.nt + K] * (LT * LT);
            double Lr[LT];
#pragma unroll
            for (int k = 0; k < LT; k++) Lr[k] = (on && k < lane) ? Ud[lane * LT + k] : 0.0;
#pragma unroll
            for (int k = 0; k < LT; k++) {
                if (k < kh) {
                    const double v = acc - Lr[k] * rdlane(acc, k);
                    acc = lane > k ? v : acc;
                }
            }
            acc = on ? acc : 0.0;
            S.y[K0 + lane] = acc;
            accs[s * LT + lane] = acc;
        }
        __syncthreads();
        const double yk = accs[s * LT + lane];
        for (int I = T0 + w; I < T1; I += W) {
            if (I <= K) continue;
            const int e = cur[I - T0];
            if (e >= S.colStart[I + 1] || S.colK[e] != K) continue;   // no block (K, I)
            if (lane == 0) cur[I - T0] = e + 1;
            const int sl = S.colSlot[e];
            if (!S.lnz[sl]) continue;
            accs[(I - T0) * LT + lane] =
                sweep_chain_fwd(accs[(I - T0) * LT + lane], S.LT + (size_t)sl * (LT * LT), lane, yk, kh);
        }
        __syncthreads();
    }
}

__global__ void __launch_bounds__(64 * kSweepWaves) k_ldlt_bwdn(SpDev S, int n0, double* __restrict__ x, double* scal,
                                                                int first) {
    extern __shared__ double accs[];
    __shared__ int cur[kSweepMaxTiles];   // the tile's last row-list entry inside the node
    const int lane = threadIdx.x & 63;
    const int failed = *(volatile int*)S.fail;
    if (first && blockIdx.x == 0 && threadIdx.x == 0) scal[3] = failed ? 0.0 : 1.0;
    if (failed) return;
    const int node = S.levNodes[n0 + blockIdx.x];
    const int T0 = S.nodeT[2 * node], T1 = S.nodeT[2 * node + 1];
    if (T1 > T0 && skip_tile(S, T0)) return;
    const int W = blockDim.x >> 6, w = threadIdx.x >> 6;
    for (int I = T0 + w; I < T1; I += W) {
        const int I0 = I * LT;
        const double* Ud = S.U + (size_t)S.slotOf[(size_t)I * S.nt + I] * (LT * LT);
        double acc = lane < S.th[I] ? S.y[I0 + lane] / Ud[lane * LT + lane] : 0.0;
        int e = S.rowStart[I + 1] - 1;
        for (; e >= S.rowStart[I]; e--) {
            const int J = S.rowJ[e];
            if (J < T1) break;   // descending J: the ancestors come first
            const int sl = S.rowSlot[e];
            if (!S.lnz[sl]) continue;
            acc = sweep_chain_bwd(acc, S.LT + (size_t)sl * (LT * LT), lane, lane < S.th[J] ? S.xs[J * LT + lane] : 0.0,
                                  S.th[J]);
        }
        accs[(I - T0) * LT + lane] = acc;
        if (lane == 0) cur[I - T0] = e;
    }
    __syncthreads();
    for (int s = T1 - T0 - 1; s >= 0; s--) {
        const int K = T0 + s, K0 = K * LT, kh = S.th[K];
        if (s % W == w) {   // the owner: diagonal tile, x_K final
            const bool on = lane < kh;
            double acc = accs[s * LT + lane];
            const double* Ud = S.U + (size_t)S.slotOf[(size_t)K * S.nt + K] * (LT * LT);
            double Lr[LT];
#pragma unroll
            for (int k = 0; k < LT; k++) Lr[k] = (on && k < kh) ? Ud[k * LT + lane] : 0.0;   // L[K0 + k][K0 + lane]
#pragma unroll
            for (int k = LT - 1; k >= 0; k--) {
                if (k < kh) {
                    const double v = acc - Lr[k] * rdlane(acc, k);
                    acc = lane < k ? v : acc;
                }
            }
            acc = on ? acc : 0.0;
            S.xs[K0 + lane] = acc;
            if (on) x[S.rowMap[K0 + lane]] = acc;
            accs[s * LT + lane] = acc;
        }
        __syncthreads();
        const double xk = accs[s * LT + lane];
        for (int I = T0 + w; I < K; I += W) {
            const int e = cur[I - T0];
            if (e < S.rowStart[I] || S.rowJ[e] != K) continue;   // no block (I, K)
            if (lane == 0) cur[I - T0] = e - 1;
            const int sl = S.rowSlot[e];
            if (!S.lnz[sl]) continue;
            accs[(I - T0) * LT + lane] =
                sweep_chain_bwd(accs[(I - T0) * LT + lane], S.LT + (size_t)sl * (LT * LT), lane, xk, kh);
        }
        __syncthreads();
    }
}

// Backward sweep by levels with the ancestors' terms PUSHED (the default): per element the
// sequence of k_ldlt_backward (x_i = y_i / d_i, then L[j][i] x_j for j descending), split as
//   k_ldlt_binit   acc = y / d for every tile row;
//   per level H, top-down:
//     k_ldlt_bin     the level's nodes finish their rows from acc: their own tiles, descending
//                    (the node sweep of k_ldlt_bwdn without its outside phase);
//     k_ldlt_bpush   every tile row below whose ancestor node at level H holds tiles J of its row
//                    list applies them now: acc_I -= L(J, I)^T x_J, J descending, k descending.
// A row's ancestors sit on levels above its own and carry larger tile indices the higher they
// are, so the pushes arrive in descending J: the same sequence.  The pushes of a level are one
// launch over all rows below (a workgroup per (row, ancestor node)), instead of each row walking
// every ancestor tile inside its own level's launch (one wave streaming tens of 32 KB tiles).
__global__ void __launch_bounds__(64) k_ldlt_binit(SpDev S, double* __restrict__ acc) {
    if (*(volatile int*)S.fail) return;
    const int I = blockIdx.x, lane = threadIdx.x;
    const double* Ud = S.U + (size_t)S.slotOf[(size_t)I * S.nt + I] * (LT * LT);
    acc[I * LT + lane] = lane < S.th[I] ? S.y[I * LT + lane] / Ud[lane * LT + lane] : 0.0;
}

// (row I, entries [lo, hi] of its row list inside one ancestor node): L^T tiles staged in LDS (row
// pitch LP) by all four waves, the next tile's loads in flight; wave 0 runs the 64 row chains.
__global__ void __launch_bounds__(256) k_ldlt_bpush(SpDev S, const int4* __restrict__ tg, double* __restrict__ acc) {
    __shared__ double Lr[LT * LP];   // [i][k'] = L[J0 + k'][I0 + i]
    __shared__ double xsh[LT];
    if (*(volatile int*)S.fail) return;
    const int4 t = tg[blockIdx.x];   // (I, hi, lo, 0)
    const int I = t.x, hi = t.y, lo = t.z;
    const int gt = threadIdx.x, lane = gt & 63, w = gt >> 6;
    auto nextv = [&](int e) {
        while (e >= lo && !S.lnz[S.rowSlot[e]]) e--;
        return e;
    };
    d2v lr[8];
    double xr = 0.0;
    auto load = [&](int e) {
        const double* Lo = S.LT + (size_t)S.rowSlot[e] * (LT * LT);
#pragma unroll
        for (int u = 0; u < 8; u++) lr[u] = *(const d2v*)(Lo + 2 * (gt + 256 * u));
        const int J = S.rowJ[e];
        if (gt < LT) xr = gt < S.th[J] ? S.xs[J * LT + gt] : 0.0;
    };
    double a = acc[I * LT + lane];
    int e = nextv(hi);
    load(e >= lo ? e : hi);
    while (e >= lo) {
        const int kh = S.th[S.rowJ[e]];
        __syncthreads();
#pragma unroll
        for (int u = 0; u < 8; u++) {   // element pair (i, k'), (i, k' + 1): i = q >> 5, k' = 2 (q & 31)
            const int q = gt + 256 * u, i = q >> 5, k2 = 2 * (q & 31);
            Lr[i * LP + k2] = lr[u].x;
            Lr[i * LP + k2 + 1] = lr[u].y;
        }
        if (gt < LT) xsh[gt] = xr;
        __syncthreads();
        const int en = nextv(e - 1);
        load(en >= lo ? en : e);   // the next tile travels while this one is applied
        if (w == 0) {
            const double* row = Lr + lane * LP;
            for (int k = LT - 1; k >= 0; k--)
                if (k < kh) a = a - row[k] * xsh[k];
        }
        e = en;
    }
    if (w == 0) acc[I * LT + lane] = a;
}

// The level's nodes: their rows start from acc (every ancestor term applied), then the node's own
// tiles one at a time, descending, as in k_ldlt_bwdn.
__global__ void __launch_bounds__(64 * kSweepWaves) k_ldlt_bin(SpDev S, int n0, const double* __restrict__ acc0,
                                                              double* __restrict__ x, double* scal, int first) {
    extern __shared__ double accs[];
    __shared__ int cur[kSweepMaxTiles];
    const int lane = threadIdx.x & 63;
    const int failed = *(volatile int*)S.fail;
    if (first && blockIdx.x == 0 && threadIdx.x == 0) scal[3] = failed ? 0.0 : 1.0;
    if (failed) return;
    const int node = S.levNodes[n0 + blockIdx.x];
    const int T0 = S.nodeT[2 * node], T1 = S.nodeT[2 * node + 1];
    if (T1 > T0 && skip_tile(S, T0)) return;
    const int W = blockDim.x >> 6, w = threadIdx.x >> 6;
    for (int I = T0 + w; I < T1; I += W) {
        int e = S.rowStart[I + 1] - 1;
        while (e >= S.rowStart[I] && S.rowJ[e] >= T1) e--;   // the ancestors' entries: pushed already
        accs[(I - T0) * LT + lane] = acc0[I * LT + lane];
        if (lane == 0) cur[I - T0] = e;
    }
    __syncthreads();
    for (int s = T1 - T0 - 1; s >= 0; s--) {
        const int K = T0 + s, K0 = K * LT, kh = S.th[K];
        if (s % W == w) {   // the owner: diagonal tile, x_K final
            const bool on = lane < kh;
            double a = accs[s * LT + lane];
            const double* Ud = S.U + (size_t)S.slotOf[(size_t)K * S.nt + K] * (LT * LT);
            double Lk[LT];
#pragma unroll
            for (int k = 0; k < LT; k++) Lk[k] = (on && k < kh) ? Ud[k * LT + lane] : 0.0;   // L[K0 + k][K0 + lane]
#pragma unroll
            for (int k = LT - 1; k >= 0; k--) {
                if (k < kh) {
                    const double v = a - Lk[k] * rdlane(a, k);
                    a = lane < k ? v : a;
                }
            }
            a = on ? a : 0.0;
            S.xs[K0 + lane] = a;
            if (on) x[S.rowMap[K0 + lane]] = a;
            accs[s * LT + lane] = a;
        }
        __syncthreads();
        const double xk = accs[s * LT + lane];
        for (int I = T0 + w; I < K; I += W) {
            const int e = cur[I - T0];
            if (e < S.rowStart[I] || S.rowJ[e] != K) continue;   // no block (I, K)
            if (lane == 0) cur[I - T0] = e - 1;
            const int sl = S.rowSlot[e];
            if (!S.lnz[sl]) continue;
            accs[(I - T0) * LT + lane] =
                sweep_chain_bwd(accs[(I - T0) * LT + lane], S.LT + (size_t)sl * (LT * LT), lane, xk, kh);
        }
        __syncthreads();
    }
}

// ORBGPU_LDLT_SWEEP=1 keeps the one-wave-per-node sweeps, =2 the node sweeps with cross-lane
// broadcasts (A/B); default: the pipelined node sweeps (k_ldlt_fwdn_u / k_ldlt_bwdn_u)
static int sweep_mode() {
    static const int v = [] {
        const char* e = getenv("ORBGPU_LDLT_SWEEP");
        return e ? atoi(e) : 0;
    }();
    return v;
}
static bool sweep_nodes() { return sweep_mode() != 1; }

int ldlt_debug_prof(unsigned long long* out8) {
#ifdef ORBGPU_PROF
    ORB_HIP_CHECK(hipMemcpyFromSymbol(out8, HIP_SYMBOL(g_orbgpu_prof), sizeof(unsigned long long) * 8, 16 * 8));
    unsigned long long z[8] = {};
    ORB_HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_orbgpu_prof), z, sizeof(z), 16 * 8));
#else
    (void)out8;
#endif
    return 0;
}

static inline size_t al256(size_t b) { return (b + 255) & ~(size_t)255; }

SparseLdlt::~SparseLdlt() {
    if (mem_) (void)hipFree(mem_);
    if (distMem_) (void)hipFree(distMem_);
}

int SparseLdlt::build(int n, int g, const std::vector<int>& adjStart, const std::vector<int>& adj, bool nd,
                      hipStream_t s) {
    n_ = n;
    nt_ = 0;
    nslot_ = nA_ = 0;
    nLev_ = 0;
    if (n <= 0) return 0;
    const int ng = (n + g - 1) / g;
    if ((int)adjStart.size() != ng + 1) return -1;
    auto gsz = [&](int q) { return std::min(g, n - q * g); };
    static const bool say = getenv("ORBGPU_BA_TIMES") != nullptr;   // the build's phases (tools/)
    auto ts0 = std::chrono::steady_clock::now();
    auto lap = [&](const char* what) {
        if (!say) return;
        const auto t = std::chrono::steady_clock::now();
        fprintf(stderr, "[ba]     ldlt build: %s %.0f us\n", what,
                std::chrono::duration<double, std::micro>(t - ts0).count());
        ts0 = t;
    };
    // ---- order and tile space
    NdTree tree;
    if (nd) {
        nd_order(ng, adjStart, adj, kNdLeaf, &tree);
    } else {   // natural order, one node
        tree.perm.resize(ng);
        for (int q = 0; q < ng; q++) tree.perm[q] = q;
        tree.start = {0};
        tree.end = {ng};
        tree.parent = {-1};
        tree.height = {0};
    }
    lap("nested dissection");
    const int nnode = (int)tree.start.size();
    nd_ = nd;
    dist_ = false;
    hProw_.assign(ng, 0);
    std::vector<int> nodeT(2 * nnode), th;
    int nt = 0;
    for (int k = 0; k < nnode; k++) {
        int rows = 0;
        for (int pos = tree.start[k]; pos < tree.end[k]; pos++) {
            hProw_[tree.perm[pos]] = nt * LT + rows;
            rows += gsz(tree.perm[pos]);
        }
        const int tiles = (rows + LT - 1) / LT;
        nodeT[2 * k] = nt;
        nodeT[2 * k + 1] = nt + tiles;
        for (int t = 0; t < tiles; t++) th.push_back(std::min(LT, rows - t * LT));
        nt += tiles;
    }
    nt_ = nt;
    hNodeT_ = nodeT;
    std::vector<int> tileNode(nt);
    for (int k = 0; k < nnode; k++)
        for (int t = nodeT[2 * k]; t < nodeT[2 * k + 1]; t++) tileNode[t] = k;
    std::vector<int> rowMap((size_t)nt * LT, -1);
    for (int q = 0; q < ng; q++)
        for (int r = 0; r < gsz(q); r++) rowMap[(size_t)hProw_[q] + r] = q * g + r;
    // ---- tile pattern of S: every (group, group) block of the graph and the diagonal groups
    std::vector<uint8_t> mask((size_t)nt * nt, 0);
    auto mark_blocks = [&](int q1, int q2) {
        const int a0 = hProw_[q1] / LT, a1 = (hProw_[q1] + gsz(q1) - 1) / LT;
        const int b0 = hProw_[q2] / LT, b1 = (hProw_[q2] + gsz(q2) - 1) / LT;
        for (int I = a0; I <= a1; I++)
            for (int J = b0; J <= b1; J++) mask[(size_t)std::min(I, J) * nt + std::max(I, J)] = 1;
    };
    for (int q = 0; q < ng; q++) {
        mark_blocks(q, q);
        for (int e = adjStart[q]; e < adjStart[q + 1]; e++)
            if (adj[e] > q) mark_blocks(q, adj[e]);
    }
    // ---- symbolic factorisation at tile level: struct(p) joins its parent's
    std::vector<std::vector<int>> rows(nt);
    for (int I = 0; I < nt; I++) {
        rows[I].push_back(I);
        for (int J = I + 1; J < nt; J++)
            if (mask[(size_t)I * nt + J]) rows[I].push_back(J);
    }
    for (int p = 0; p < nt; p++) {
        std::vector<int>& r = rows[p];
        std::sort(r.begin(), r.end());
        r.erase(std::unique(r.begin(), r.end()), r.end());
        if (r.size() > 1) {
            const int parent = r[1];
            for (size_t q = 2; q < r.size(); q++) rows[parent].push_back(r[q]);
        }
        if ((int)r.size() - 1 > kMaxRow) return -3;
    }
    lap("tile pattern + symbolic");
    // slots: the Schur pattern first (the exchanged prefix), then the fill-in
    hSlotOf_.assign((size_t)nt * nt, -1);
    int ns = 0;
    for (int I = 0; I < nt; I++)
        for (int J : rows[I])
            if (J == I || mask[(size_t)I * nt + J]) hSlotOf_[(size_t)I * nt + J] = ns++;
    nA_ = ns;
    for (int I = 0; I < nt; I++)
        for (int J : rows[I])
            if (hSlotOf_[(size_t)I * nt + J] < 0) hSlotOf_[(size_t)I * nt + J] = ns++;
    nslot_ = ns;
    auto slot = [&](int I, int J) { return hSlotOf_[(size_t)I * nt + J]; };
    // ---- panel rows (J > p), block columns (K < I), trailing pairs inside the node
    std::vector<int> rowStart(nt + 1, 0), rowJ, rowSlot, colStart(nt + 1, 0), colK, colSlot, pairStart(nt + 1, 0);
    std::vector<int4> pairs;
    std::vector<std::vector<int>> cols(nt);
    for (int p = 0; p < nt; p++) {
        rowStart[p] = (int)rowJ.size();
        pairStart[p] = (int)pairs.size();
        const std::vector<int>& r = rows[p];
        const int tEnd = nodeT[2 * tileNode[p] + 1];
        for (size_t q = 1; q < r.size(); q++) {
            rowJ.push_back(r[q]);
            rowSlot.push_back(slot(p, r[q]));
            cols[r[q]].push_back(p);
        }
        const int m = (int)r.size() - 1;
        for (int a = 0; a < m; a++) {
            if (r[1 + a] >= tEnd) break;   // rows sorted: the rest belong to ancestors
            for (int bb = a; bb < m; bb++) {
                const int t = slot(r[1 + a], r[1 + bb]);
                if (t < 0) return -1;   // the fill closure guarantees the target tile
                pairs.push_back(make_int4(a, bb, t, 0));
            }
        }
    }
    rowStart[nt] = (int)rowJ.size();
    pairStart[nt] = (int)pairs.size();
    for (int I = 0; I < nt; I++) {
        colStart[I] = (int)colK.size();
        for (int K : cols[I]) {   // ascending K
            colK.push_back(K);
            colSlot.push_back(slot(K, I));
        }
    }
    colStart[nt] = (int)colK.size();
    // ---- levels: nodes by height; the update targets of each level's nodes
    int H = 0;
    for (int k = 0; k < nnode; k++) H = std::max(H, tree.height[k]);
    nLev_ = H + 1;
    hLevNodeStart_.assign(nLev_ + 1, 0);
    hLevTgtStart_.assign(nLev_ + 1, 0);
    std::vector<int> levNodes;
    std::vector<int4> tgts, kps;
    for (int h = 0; h < nLev_; h++) {
        hLevNodeStart_[h] = (int)levNodes.size();
        hLevTgtStart_[h] = (int)tgts.size();
        for (int k = 0; k < nnode; k++) {
            if (tree.height[k] != h) continue;
            levNodes.push_back(k);
            const int t0 = nodeT[2 * k], t1 = nodeT[2 * k + 1];
            for (int I = t0; I < t1; I++)
                for (int J : rows[I]) {
                    const int first = (int)kps.size();
                    for (int K : cols[I]) {
                        if (K >= t0) break;   // the node's own panels: right-looking in k_ldlt_factor
                        const int sj = slot(K, J);
                        if (sj >= 0) kps.push_back(make_int4(slot(K, I), sj, K, 0));
                    }
                    if ((int)kps.size() > first) tgts.push_back(make_int4(slot(I, J), I, J, first));
                }
        }
    }
    hLevNodeStart_[nLev_] = (int)levNodes.size();
    hLevTgtStart_[nLev_] = (int)tgts.size();
    tree_ = tree;
    hLevMaxT_.assign(nLev_, 0);
    for (int h = 0; h < nLev_; h++)
        for (int q = hLevNodeStart_[h]; q < hLevNodeStart_[h + 1]; q++)
            hLevMaxT_[h] = std::max(hLevMaxT_[h], nodeT[2 * levNodes[q] + 1] - nodeT[2 * levNodes[q]]);
    // panel steps of each level: step s = panel T0 + s of every node of the level that has one;
    // per step the panels, the U tiles of their rows and the trailing targets inside the nodes
    std::vector<int> stepP;
    std::vector<int2> rowJobs, pairJobs;
    std::vector<int4> panelJobs;   // k_ldlt_panel: per panel, groups of panel_roles() roles (row tiles, then y)
    hSteps_.clear();
    hLevStepStart_.assign(nLev_ + 1, 0);
    for (int h = 0; h < nLev_; h++) {
        hLevStepStart_[h] = (int)hSteps_.size();
        int maxT = 0;
        for (int q = hLevNodeStart_[h]; q < hLevNodeStart_[h + 1]; q++)
            maxT = std::max(maxT, nodeT[2 * levNodes[q] + 1] - nodeT[2 * levNodes[q]]);
        for (int st = 0; st < maxT; st++) {
            const int4 rec = make_int4((int)stepP.size(), (int)rowJobs.size(), (int)pairJobs.size(), (int)panelJobs.size());
            for (int q = hLevNodeStart_[h]; q < hLevNodeStart_[h + 1]; q++) {
                const int k = levNodes[q];
                const int pnl = nodeT[2 * k] + st;
                if (pnl >= nodeT[2 * k + 1]) continue;
                stepP.push_back(pnl);
                for (int e = 0; e < rowStart[pnl + 1] - rowStart[pnl]; e++) rowJobs.push_back(make_int2(pnl, e));
                rowJobs.push_back(make_int2(pnl, -1));   // the fused forward sweep's y_p (skipped unless yfused)
                const int roles = rowStart[pnl + 1] - rowStart[pnl] + 1, pr = panel_roles();   // row tiles + y_p
                for (int r0 = 0; r0 < roles; r0 += pr) panelJobs.push_back(make_int4(pnl, r0, std::min(pr, roles - r0), 0));
                for (int e = 0; e < pairStart[pnl + 1] - pairStart[pnl]; e++) pairJobs.push_back(make_int2(pnl, e));
                // ... and its y_I -= L(I, p) y_p for the panel row's entries inside the node
                for (int e = 0; e < rowStart[pnl + 1] - rowStart[pnl]; e++)
                    if (rowJ[rowStart[pnl] + e] < nodeT[2 * k + 1]) pairJobs.push_back(make_int2(pnl, -1 - e));
                pairJobs.push_back(make_int2(pnl, kDiagCopyJob));   // (k_ldlt_panel runs only)
            }
            hSteps_.push_back(rec);
        }
    }
    hLevStepStart_[nLev_] = (int)hSteps_.size();
    // backward pushes: per tile row, its row list's entries grouped by ancestor node (descending J),
    // each group a target of the launch after that node's level finishes (k_ldlt_bpush)
    std::vector<std::vector<int4>> pushByLev(nLev_);
    for (int I = 0; I < nt; I++) {
        const int own = tileNode[I];
        int e = rowStart[I + 1] - 1;
        while (e >= rowStart[I]) {
            const int X = tileNode[rowJ[e]];
            if (X == own) break;   // the node's own tiles (ascending list: the ancestors are above)
            int lo = e;
            while (lo - 1 >= rowStart[I] && tileNode[rowJ[lo - 1]] == X) lo--;
            pushByLev[tree.height[X]].push_back(make_int4(I, e, lo, 0));
            e = lo - 1;
        }
    }
    std::vector<int4> pushT;
    hLevPushStart_.assign(nLev_ + 1, 0);
    for (int h = 0; h < nLev_; h++) {
        hLevPushStart_[h] = (int)pushT.size();
        pushT.insert(pushT.end(), pushByLev[h].begin(), pushByLev[h].end());
    }
    hLevPushStart_[nLev_] = (int)pushT.size();
    hSteps_.push_back(make_int4((int)stepP.size(), (int)rowJobs.size(), (int)pairJobs.size(), (int)panelJobs.size()));   // sentinel
    tgts.push_back(make_int4(0, 0, 0, (int)kps.size()));   // sentinel: the last target's K range end
    // every tile a kernel addresses exists (host check before any launch)
    for (int I = 0; I < nt; I++)
        if (slot(I, I) < 0) return -1;
    for (int v : rowSlot)
        if (v < 0) return -1;
    for (int v : colSlot)
        if (v < 0) return -1;
    for (size_t q = 0; q + 1 < tgts.size(); q++)
        if (tgts[q].x < 0 || tgts[q].w > tgts[q + 1].w) return -1;
    for (const int4& q : kps)
        if (q.x < 0 || q.y < 0 || q.z < 0 || q.z >= nt) return -1;
    for (int q : levNodes)
        if (q < 0 || q >= nnode) return -1;
    nUpd_ = (long long)kps.size();
    lap("slots + schedule");
    // ---- device storage (grow-only)
    const size_t tileB = sizeof(double) * LT * LT;
    size_t off = 0;
    auto take = [&](size_t b) {
        const size_t o = off;
        off += al256(b);
        return o;
    };
    const size_t oSlot = take(sizeof(int) * hSlotOf_.size());
    const size_t oU = take(tileB * nslot_);
    const size_t oLT = take(tileB * nslot_);
    const size_t oY = take(sizeof(double) * (size_t)nt * LT);
    const size_t oXs = take(sizeof(double) * (size_t)nt * LT);
    const size_t oAcc = take(sizeof(double) * (size_t)nt * LT);
    const size_t oLnz = take(nslot_);
    const size_t oFail = take(sizeof(int) * 4);
    const size_t oProw = take(sizeof(int) * (size_t)ng);
    std::vector<int> L;
    auto put = [&](const std::vector<int>& v) {
        const size_t o = L.size();
        L.insert(L.end(), v.begin(), v.end());
        return o;
    };
    auto put4 = [&](const std::vector<int4>& v) {
        while (L.size() % 4) L.push_back(0);
        const size_t o = L.size();
        for (const int4& q : v) {
            L.push_back(q.x);
            L.push_back(q.y);
            L.push_back(q.z);
            L.push_back(q.w);
        }
        return o;
    };
    offTh_ = put(th);
    offRowMap_ = put(rowMap);
    offRowStart_ = put(rowStart);
    offRowJ_ = put(rowJ);
    offRowSlot_ = put(rowSlot);
    offColStart_ = put(colStart);
    offColK_ = put(colK);
    offColSlot_ = put(colSlot);
    offPairStart_ = put(pairStart);
    offNodeT_ = put(nodeT);
    offLevNodes_ = put(levNodes);
    offPairs_ = put4(pairs);
    offTgts_ = put4(tgts);
    offKps_ = put4(kps);
    offStepP_ = put(stepP);
    auto put2 = [&](const std::vector<int2>& v) {
        while (L.size() % 2) L.push_back(0);
        const size_t o = L.size();
        for (const int2& q : v) {
            L.push_back(q.x);
            L.push_back(q.y);
        }
        return o;
    };
    offRowJobs_ = put2(rowJobs);
    offPairJobs_ = put2(pairJobs);
    offPanelJobs_ = put4(panelJobs);
    offPush_ = put4(pushT);
    const size_t oLists = take(sizeof(int) * (L.size() + 64));
    if (off > cap_) {
        if (mem_) (void)hipFree(mem_);
        mem_ = nullptr;
        cap_ = 0;
        ORB_HIP_CHECK(hipMalloc(&mem_, off));
        cap_ = off;
    }
    char* base = (char*)mem_;
    slotOf_ = (int*)(base + oSlot);
    U_ = (double*)(base + oU);
    LT_ = (double*)(base + oLT);
    y_ = (double*)(base + oY);
    xs_ = (double*)(base + oXs);
    acc_ = (double*)(base + oAcc);
    lnz_ = (uint8_t*)(base + oLnz);
    fail_ = (int*)(base + oFail);
    prow_ = (int*)(base + oProw);
    lists_ = (int*)(base + oLists);
    ORB_HIP_CHECK(hipMemcpyAsync(slotOf_, hSlotOf_.data(), sizeof(int) * hSlotOf_.size(), hipMemcpyHostToDevice, s));
    ORB_HIP_CHECK(hipMemcpyAsync(prow_, hProw_.data(), sizeof(int) * hProw_.size(), hipMemcpyHostToDevice, s));
    ORB_HIP_CHECK(hipMemcpyAsync(lists_, L.data(), sizeof(int) * L.size(), hipMemcpyHostToDevice, s));
    ORB_HIP_CHECK(stream_wait(s));   // pageable sources
    lap("lists + upload");
    return 0;
}

int SparseLdlt::zero(hipStream_t s) {
    if (nslot_) ORB_HIP_CHECK(hipMemsetAsync(U_, 0, sizeof(double) * LT * LT * (size_t)nslot_, s));
    return 0;
}

SpDev SparseLdlt::dev() const {
    SpDev d;
    d.n = n_;
    d.nt = nt_;
    d.slotOf = slotOf_;
    d.U = U_;
    d.LT = LT_;
    d.th = lists_ + offTh_;
    d.rowMap = lists_ + offRowMap_;
    d.rowStart = lists_ + offRowStart_;
    d.rowJ = lists_ + offRowJ_;
    d.rowSlot = lists_ + offRowSlot_;
    d.colStart = lists_ + offColStart_;
    d.colK = lists_ + offColK_;
    d.colSlot = lists_ + offColSlot_;
    d.pairStart = lists_ + offPairStart_;
    d.pairs = (const int4*)(lists_ + offPairs_);
    d.nodeT = lists_ + offNodeT_;
    d.levNodes = lists_ + offLevNodes_;
    d.tgts = (const int4*)(lists_ + offTgts_);
    d.kps = (const int4*)(lists_ + offKps_);
    d.stepP = lists_ + offStepP_;
    d.rowJobs = (const int2*)(lists_ + offRowJobs_);
    d.pairJobs = (const int2*)(lists_ + offPairJobs_);
    d.panelJobs = (const int4*)(lists_ + offPanelJobs_);
    d.lnz = lnz_;
    d.y = y_;
    d.xs = xs_;
    d.fail = fail_;
    d.tcls = nullptr;
    d.want = -1;
    d.kmode = 0;
    d.dst = nullptr;
    d.packIdx = nullptr;
    d.yfused = 0;
    // the fused panel launch needs the quadrant trailing kernel (its copy jobs) and the y-aware rows
    d.pfused = (fused_panels() && quad_updates() && prow_quads()) ? 1 : 0;
    return d;
}

void SparseLdlt::enqueue_factor_level(const SpDev& d, int h, const double* b, hipStream_t s) {
    const int nt = hLevTgtStart_[h + 1] - hLevTgtStart_[h];
    if (nt > 0) {
        if (quad_updates())
            hipLaunchKernelGGL(k_ldlt_update_q, dim3(4 * nt), dim3(256), 0, s, d, hLevTgtStart_[h]);
        else
            hipLaunchKernelGGL(k_ldlt_update, dim3(nt), dim3(256), 0, s, d, hLevTgtStart_[h]);
    }
    for (int st = hLevStepStart_[h]; st < hLevStepStart_[h + 1]; st++) {
        const int4 a = hSteps_[st], z = hSteps_[st + 1];
        if (d.pfused) {   // diagonal + panel row in one launch
            if (z.w > a.w) {
                const int pr = panel_roles();
                if (pr == 1)
                    hipLaunchKernelGGL(k_ldlt_panel<1>, dim3(z.w - a.w), dim3(128), 0, s, d, a.w);
                else if (pr == 7)
                    hipLaunchKernelGGL(k_ldlt_panel<7>, dim3(z.w - a.w), dim3(512), 0, s, d, a.w);
                else
                    hipLaunchKernelGGL(k_ldlt_panel<3>, dim3(z.w - a.w), dim3(256), 0, s, d, a.w);
            }
        } else {
        if (z.x > a.x) {
            // the four-wave diagonal kernel measured no faster than the rolled one-wave kernel
            // (38 vs 36-38 us per launch, profiles/r04l3_gba_ldlt_levels.txt): opt-in
            if (pdiag_quads())
                hipLaunchKernelGGL(k_ldlt_pdiag4, dim3(z.x - a.x), dim3(256), 0, s, d, a.x);
            else
                hipLaunchKernelGGL(rolled_panels() ? k_ldlt_pdiag_r : k_ldlt_pdiag, dim3(z.x - a.x), dim3(64), 0, s, d,
                                   a.x);
        }
        if (z.y > a.y) {
            if (prow_quads())
                hipLaunchKernelGGL(k_ldlt_prow4, dim3(z.y - a.y), dim3(256), 0, s, d, a.y);
            else
                hipLaunchKernelGGL(rolled_panels() ? k_ldlt_prow_r : k_ldlt_prow, dim3(z.y - a.y), dim3(64), 0, s, d,
                                   a.y);
        }
        }
        if (z.z > a.z) {
            if (quad_updates())
                hipLaunchKernelGGL(k_ldlt_ptrail_q, dim3(4 * (z.z - a.z)), dim3(256), 0, s, d, a.z);
            else
                hipLaunchKernelGGL(k_ldlt_ptrail, dim3(z.z - a.z), dim3(256), 0, s, d, a.z);
        }
    }
    if (d.yfused) return;   // the forward sweep rode along
    const int nn = hLevNodeStart_[h + 1] - hLevNodeStart_[h];
    const int mt = hLevMaxT_[h];
    if (sweep_nodes() && mt > 1 && mt <= kSweepMaxTiles)
        hipLaunchKernelGGL(sweep_mode() == 2 ? k_ldlt_fwdn : k_ldlt_fwdn_u, dim3(nn), dim3(64 * std::min(mt, kSweepWaves)),
                           sizeof(double) * LT * mt, s, d, hLevNodeStart_[h], b);
    else
        hipLaunchKernelGGL(k_ldlt_pfwd, dim3(nn), dim3(64), 0, s, d, hLevNodeStart_[h], b);
}

void SparseLdlt::enqueue_backward_level(const SpDev& d, int h, double* x, double* scal, int first, hipStream_t s) {
    const int nn = hLevNodeStart_[h + 1] - hLevNodeStart_[h];
    const int mt = hLevMaxT_[h];
    if (sweep_nodes() && mt > 1 && mt <= kSweepMaxTiles)
        hipLaunchKernelGGL(sweep_mode() == 2 ? k_ldlt_bwdn : k_ldlt_bwdn_u, dim3(nn), dim3(64 * std::min(mt, kSweepWaves)),
                           sizeof(double) * LT * mt, s, d, hLevNodeStart_[h], x, scal, first);
    else
        hipLaunchKernelGGL(k_ldlt_backward, dim3(nn), dim3(64), 0, s, d, hLevNodeStart_[h], x, scal, first);
}

// ORBGPU_LDLT_BPUSH=0 keeps the per-level backward launches that walk every ancestor tile (A/B)
static bool pushed_backward() {
    static const bool v = [] {
        const char* e = getenv("ORBGPU_LDLT_BPUSH");
        return !(e && e[0] == '0');
    }();
    return v;
}

// ORBGPU_LDLT_FWD=0 keeps the forward sweep as its own per-level launches (A/B)
static bool fused_forward() {
    static const bool v = [] {
        const char* e = getenv("ORBGPU_LDLT_FWD");
        return !(e && e[0] == '0');
    }();
    return v;
}

int SparseLdlt::solve(const double* b, double* x, double* scal, hipStream_t s) {
    if (n_ <= 0) return 0;
    SpDev d = dev();
    // the fused forward sweep needs the y-aware kernels (quadrant updates, four-wave panel rows)
    d.yfused = (fused_forward() && quad_updates() && prow_quads()) ? 1 : 0;
    ORB_HIP_CHECK(hipMemsetAsync(fail_, 0, sizeof(int), s));
    if (d.yfused) hipLaunchKernelGGL(k_ldlt_yinit, dim3(nt_), dim3(64), 0, s, d, b);
    for (int h = 0; h < nLev_; h++) enqueue_factor_level(d, h, b, s);
    int maxT = 0;
    for (int h = 0; h < nLev_; h++) maxT = std::max(maxT, hLevMaxT_[h]);
    if (pushed_backward() && maxT <= kSweepMaxTiles) {
        const int4* pt = (const int4*)(lists_ + offPush_);
        hipLaunchKernelGGL(k_ldlt_binit, dim3(nt_), dim3(64), 0, s, d, acc_);
        for (int h = nLev_ - 1; h >= 0; h--) {
            const int nn = hLevNodeStart_[h + 1] - hLevNodeStart_[h], mt = std::max(1, hLevMaxT_[h]);
            hipLaunchKernelGGL(k_ldlt_bin, dim3(nn), dim3(64 * std::min(mt, kSweepWaves)), sizeof(double) * LT * mt, s,
                               d, hLevNodeStart_[h], (const double*)acc_, x, scal, h == nLev_ - 1 ? 1 : 0);
            const int np = hLevPushStart_[h + 1] - hLevPushStart_[h];
            if (np > 0) hipLaunchKernelGGL(k_ldlt_bpush, dim3(np), dim3(256), 0, s, d, pt + hLevPushStart_[h], acc_);
        }
    } else {
        for (int h = nLev_ - 1; h >= 0; h--) enqueue_backward_level(d, h, x, scal, h == nLev_ - 1 ? 1 : 0, s);
    }
    ORB_HIP_CHECK(hipGetLastError());
    return 0;
}

// ---- sharded factorisation (plan / solve_dist) -----------------------------------------------

// shared tiles into / out of the exchange buffer (a workgroup per tile)
__global__ void __launch_bounds__(256) k_slot_pack(const double* __restrict__ U, const int* slots, double* buf) {
    const double2* src = (const double2*)(U + (size_t)slots[blockIdx.x] * (LT * LT));
    double2* dst = (double2*)(buf + (size_t)blockIdx.x * (LT * LT));
    for (int q = threadIdx.x; q < LT * LT / 2; q += 256) dst[q] = src[q];
}
__global__ void __launch_bounds__(256) k_slot_unpack(double* __restrict__ U, const int* slots, const double* buf) {
    const double2* src = (const double2*)(buf + (size_t)blockIdx.x * (LT * LT));
    double2* dst = (double2*)(U + (size_t)slots[blockIdx.x] * (LT * LT));
    for (int q = threadIdx.x; q < LT * LT / 2; q += 256) dst[q] = src[q];
}

// The separator rows' forward-sweep input from this rank: b_I minus the contributions of this
// rank's subtree tiles K (their y final), a wave per separator tile row I.
__global__ void __launch_bounds__(64) k_ldlt_fwd_part(SpDev S, const double* __restrict__ b, const int* shT,
                                                      double* dst) {
    const int I = shT[blockIdx.x], I0 = I * LT, lane = threadIdx.x;
    double acc = lane < S.th[I] ? b[S.rowMap[I0 + lane]] : 0.0;
    if (!*(volatile int*)S.fail) {
        for (int e = S.colStart[I]; e < S.colStart[I + 1]; e++) {
            const int K = S.colK[e], sl = S.colSlot[e];
            if (S.tcls[K] != 2 || !S.lnz[sl]) continue;
            acc = sweep_chain_fwd(acc, S.LT + (size_t)sl * (LT * LT), lane, S.y[K * LT + lane], S.th[K]);
        }
    }
    dst[(size_t)blockIdx.x * LT + lane] = acc;
}
// reduced separator rows back into b (system order)
__global__ void __launch_bounds__(64) k_b_unpack(SpDev S, const int* shT, const double* src, double* b) {
    const int I = shT[blockIdx.x], lane = threadIdx.x;
    if (lane < S.th[I]) b[S.rowMap[I * LT + lane]] = src[(size_t)blockIdx.x * LT + lane];
}
// the separator rows of x are counted once in the final all-reduce (rank 0's)
__global__ void __launch_bounds__(64) k_x_zero_rows(SpDev S, const int* shT, double* x) {
    const int I = shT[blockIdx.x], lane = threadIdx.x;
    if (lane < S.th[I]) x[S.rowMap[I * LT + lane]] = 0.0;
}
__global__ void k_fail_pub(const int* fail, double* slot) { *slot = *(volatile const int*)fail ? 1.0 : 0.0; }
__global__ void k_scal_pub(const double* slot, double* scal) { scal[3] = *slot == 0.0 ? 1.0 : 0.0; }
__global__ void __launch_bounds__(256) k_align(const int* __restrict__ ePose, int nE, const int* __restrict__ prow,
                                               const uint8_t* __restrict__ tcls, int* flag) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= nE) return;
    const int p = ePose[e];
    if (p >= 0 && tcls[prow[p] / LT] == 0) atomicOr(flag, 1);
}

int SparseLdlt::plan(int R, int rank, hipStream_t s) {
    dist_ = false;
    rank_ = rank;
    if (R <= 1 || n_ <= 0 || !nd_) return -1;
    std::vector<int> owner;
    nd_assign(tree_, R, &owner);
    const int nnode = (int)tree_.start.size();
    std::vector<uint8_t> tcls(nt_, 0);
    levOwn_.assign(nLev_, 0);
    levSh_.assign(nLev_, 0);
    for (int k = 0; k < nnode; k++) {
        const uint8_t c = owner[k] < 0 ? 1 : owner[k] == rank ? 2 : 0;
        for (int t = hNodeT_[2 * k]; t < hNodeT_[2 * k + 1]; t++) tcls[t] = c;
        if (c == 2) levOwn_[tree_.height[k]] = 1;
        if (c == 1) levSh_[tree_.height[k]] = 1;
    }
    std::vector<int> shSlots, shT, packIdx(nslot_, -1);
    for (int I = 0; I < nt_; I++) {
        if (tcls[I] != 1) continue;
        shT.push_back(I);
        for (int J = I; J < nt_; J++) {   // an ancestor of a separator is a separator
            const int sl = hSlotOf_[(size_t)I * nt_ + J];
            if (sl < 0) continue;
            packIdx[sl] = (int)shSlots.size();
            shSlots.push_back(sl);
        }
    }
    const int ng = (int)hProw_.size();
    std::vector<uint8_t> poseAdd(ng, 0);
    for (int q = 0; q < ng; q++) {
        const uint8_t c = tcls[hProw_[q] / LT];
        poseAdd[q] = (c == 2 || (c == 1 && rank == 0)) ? 1 : 0;
    }
    nShSlots_ = (int)shSlots.size();
    nShT_ = (int)shT.size();
    size_t off = 0;
    auto take = [&](size_t b) {
        const size_t o = off;
        off += al256(b);
        return o;
    };
    const size_t oT = take(nt_), oP = take(sizeof(int) * nslot_), oS = take(sizeof(int) * (nShSlots_ + 1)),
                 oH = take(sizeof(int) * (nShT_ + 1)), oA = take(ng),
                 oX = take(sizeof(double) * ((size_t)nShSlots_ * LT * LT + (size_t)nShT_ * LT + 8));
    if (off > distCap_) {
        if (distMem_) (void)hipFree(distMem_);
        distMem_ = nullptr;
        distCap_ = 0;
        ORB_HIP_CHECK(hipMalloc(&distMem_, off));
        distCap_ = off;
    }
    char* base = (char*)distMem_;
    dTcls_ = (uint8_t*)(base + oT);
    dPackIdx_ = (int*)(base + oP);
    dShSlots_ = (int*)(base + oS);
    dShT_ = (int*)(base + oH);
    dPoseAdd_ = (uint8_t*)(base + oA);
    dXbuf_ = (double*)(base + oX);
    ORB_HIP_CHECK(hipMemcpyAsync(dTcls_, tcls.data(), nt_, hipMemcpyHostToDevice, s));
    ORB_HIP_CHECK(hipMemcpyAsync(dPackIdx_, packIdx.data(), sizeof(int) * nslot_, hipMemcpyHostToDevice, s));
    if (nShSlots_)
        ORB_HIP_CHECK(hipMemcpyAsync(dShSlots_, shSlots.data(), sizeof(int) * nShSlots_, hipMemcpyHostToDevice, s));
    if (nShT_) ORB_HIP_CHECK(hipMemcpyAsync(dShT_, shT.data(), sizeof(int) * nShT_, hipMemcpyHostToDevice, s));
    ORB_HIP_CHECK(hipMemcpyAsync(dPoseAdd_, poseAdd.data(), ng, hipMemcpyHostToDevice, s));
    ORB_HIP_CHECK(hipStreamSynchronize(s));   // pageable sources
    dist_ = true;
    return 0;
}

int SparseLdlt::align_flag(const int* ePose, int nE, int* flag, hipStream_t s) {
    ORB_HIP_CHECK(hipMemsetAsync(flag, 0, sizeof(int), s));
    if (dist_ && nE > 0)
        hipLaunchKernelGGL(k_align, dim3((nE + 255) / 256), dim3(256), 0, s, ePose, nE, prow_, dTcls_, flag);
    ORB_HIP_CHECK(hipGetLastError());
    return 0;
}

int SparseLdlt::solve_dist(double* b, double* x, double* scal, hipStream_t s, Comm* comm) {
    if (!dist_) return -1;
    if (n_ <= 0) return 0;
    SpDev d = dev();
    d.tcls = dTcls_;
    ORB_HIP_CHECK(hipMemsetAsync(fail_, 0, sizeof(int), s));
    ORB_HIP_CHECK(hipMemsetAsync(x, 0, sizeof(double) * n_, s));
    const size_t nxb = (size_t)nShSlots_ * LT * LT, nyb = (size_t)nShT_ * LT;
    double* xb = dXbuf_;
    // this rank's subtrees, bottom-up (their nodes only: the kernels skip the other classes)
    SpDev da = d;
    da.want = 2;
    for (int h = 0; h < nLev_; h++)
        if (levOwn_[h]) enqueue_factor_level(da, h, b, s);
    // the separators' inputs from this rank: S minus its subtrees' updates (ascending K), b minus
    // their forward contributions
    if (nShSlots_) hipLaunchKernelGGL(k_slot_pack, dim3(nShSlots_), dim3(256), 0, s, U_, dShSlots_, xb);
    SpDev db = d;
    db.want = 1;
    db.kmode = 2;
    db.dst = xb;
    db.packIdx = dPackIdx_;
    for (int h = 0; h < nLev_; h++) {
        const int nt = hLevTgtStart_[h + 1] - hLevTgtStart_[h];
        if (levSh_[h] && nt > 0) {
            if (quad_updates())
                hipLaunchKernelGGL(k_ldlt_update_q, dim3(4 * nt), dim3(256), 0, s, db, hLevTgtStart_[h]);
            else
                hipLaunchKernelGGL(k_ldlt_update, dim3(nt), dim3(256), 0, s, db, hLevTgtStart_[h]);
        }
    }
    if (nShT_) hipLaunchKernelGGL(k_ldlt_fwd_part, dim3(nShT_), dim3(64), 0, s, d, b, dShT_, xb + nxb);
    ORB_HIP_CHECK(hipGetLastError());
    if (int e = comm->allreduce(xb, nxb + nyb, RedOp::Sum, s)) return e;
    // the separators, redundantly on every rank (only separator K's updates remain)
    if (nShSlots_) hipLaunchKernelGGL(k_slot_unpack, dim3(nShSlots_), dim3(256), 0, s, U_, dShSlots_, xb);
    if (nShT_) hipLaunchKernelGGL(k_b_unpack, dim3(nShT_), dim3(64), 0, s, d, dShT_, xb + nxb, b);
    SpDev dc = d;
    dc.want = 1;
    dc.kmode = 1;
    for (int h = 0; h < nLev_; h++)
        if (levSh_[h]) enqueue_factor_level(dc, h, b, s);
    // backward: the separators top-down, then this rank's subtrees top-down
    SpDev dd = d;
    dd.want = 1;
    for (int h = nLev_ - 1; h >= 0; h--)
        if (levSh_[h]) enqueue_backward_level(dd, h, x, scal, 0, s);
    for (int h = nLev_ - 1; h >= 0; h--)
        if (levOwn_[h]) enqueue_backward_level(da, h, x, scal, 0, s);
    if (rank_ != 0 && nShT_) hipLaunchKernelGGL(k_x_zero_rows, dim3(nShT_), dim3(64), 0, s, d, dShT_, x);
    double* fslot = xb + nxb + nyb;
    hipLaunchKernelGGL(k_fail_pub, dim3(1), dim3(1), 0, s, fail_, fslot);
    ORB_HIP_CHECK(hipGetLastError());
    const RedBuf rb[2] = {{x, (size_t)n_}, {fslot, 1}};
    if (int e = comm->allreduce(rb, 2, RedOp::Sum, s)) return e;
    hipLaunchKernelGGL(k_scal_pub, dim3(1), dim3(1), 0, s, fslot, scal);
    ORB_HIP_CHECK(hipGetLastError());
    return 0;
}

int ldlt_sparse_dense(int n, const double* S, const double* b, double* x, int* ok, double* factor_out, bool nd) {
    *ok = 0;
    if (n <= 0) {
        *ok = 1;
        return 0;
    }
    // groups of 6 rows (poses; the last one may be short), adjacent when their block is nonzero
    const int g = 6, ng = (n + g - 1) / g;
    std::vector<std::vector<int>> nb(ng);
    for (int q1 = 0; q1 < ng; q1++)
        for (int q2 = q1 + 1; q2 < ng; q2++) {
            bool nz = false;
            for (int i = q1 * g; i < std::min(n, q1 * g + g) && !nz; i++)
                for (int j = q2 * g; j < std::min(n, q2 * g + g); j++)
                    if (S[(size_t)i * n + j] != 0.0) {
                        nz = true;
                        break;
                    }
            if (nz) {
                nb[q1].push_back(q2);
                nb[q2].push_back(q1);
            }
        }
    std::vector<int> as(ng + 1, 0), adj;
    for (int q = 0; q < ng; q++) {
        std::sort(nb[q].begin(), nb[q].end());
        as[q] = (int)adj.size();
        adj.insert(adj.end(), nb[q].begin(), nb[q].end());
    }
    as[ng] = (int)adj.size();
    hipStream_t s = nullptr;
    ORB_HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    SparseLdlt L;
    if (int e = L.build(n, g, as, adj, nd, s)) return e;
    const int nt = L.nt();
    const std::vector<int>& so = L.host_slot_of();
    const std::vector<int>& prow = L.host_prow();
    auto trow = [&](int i) { return prow[i / g] + i % g; };   // tile-space row of system row i
    std::vector<double> T((size_t)L.nslot() * LT * LT, 0.0);
    for (int i = 0; i < n; i++)
        for (int j = i; j < n; j++) {
            int a = trow(i), c = trow(j);
            if (a > c) std::swap(a, c);
            const int sl = so[(size_t)(a / LT) * nt + c / LT];
            if (sl >= 0) T[(size_t)sl * LT * LT + (a % LT) * LT + c % LT] = S[(size_t)i * n + j];
        }
    double *dB = nullptr, *dX = nullptr, *dScal = nullptr;
    ORB_HIP_CHECK(hipMalloc(&dB, sizeof(double) * n));
    ORB_HIP_CHECK(hipMalloc(&dX, sizeof(double) * n));
    ORB_HIP_CHECK(hipMalloc(&dScal, sizeof(double) * 16));
    ORB_HIP_CHECK(hipMemcpy(L.tiles(), T.data(), sizeof(double) * T.size(), hipMemcpyHostToDevice));
    ORB_HIP_CHECK(hipMemcpy(dB, b, sizeof(double) * n, hipMemcpyHostToDevice));
    ORB_HIP_CHECK(hipMemcpy(dX, x, sizeof(double) * n, hipMemcpyHostToDevice));
    ORB_HIP_CHECK(hipMemset(dScal, 0, sizeof(double) * 16));
    if (int e = L.solve(dB, dX, dScal, s)) return e;
    ORB_HIP_CHECK(hipStreamSynchronize(s));
    double sc[16];
    ORB_HIP_CHECK(hipMemcpy(sc, dScal, sizeof(sc), hipMemcpyDeviceToHost));
    ORB_HIP_CHECK(hipMemcpy(x, dX, sizeof(double) * n, hipMemcpyDeviceToHost));
    *ok = sc[3] != 0.0 ? 1 : 0;
    if (factor_out && !nd) {   // natural order: tile space is the system; U above, d on the diagonal, L below
        std::vector<double> Lt(T.size());
        ORB_HIP_CHECK(hipMemcpy(T.data(), L.tiles(), sizeof(double) * T.size(), hipMemcpyDeviceToHost));
        ORB_HIP_CHECK(hipMemcpy(Lt.data(), L.lt_tiles(), sizeof(double) * Lt.size(), hipMemcpyDeviceToHost));
        std::memset(factor_out, 0, sizeof(double) * (size_t)n * n);
        for (int I = 0; I < nt; I++)
            for (int J = I; J < nt; J++) {
                const int sl = so[(size_t)I * nt + J];
                if (sl < 0) continue;
                for (int r = 0; r < LT && I * LT + r < n; r++)
                    for (int c = 0; c < LT && J * LT + c < n; c++) {
                        factor_out[(size_t)(I * LT + r) * n + J * LT + c] = T[(size_t)sl * LT * LT + r * LT + c];
                        if (I != J)   // L[J0 + c][I0 + r] = LT[r][c]
                            factor_out[(size_t)(J * LT + c) * n + I * LT + r] = Lt[(size_t)sl * LT * LT + r * LT + c];
                    }
            }
    }
    (void)hipFree(dB);
    (void)hipFree(dX);
    (void)hipFree(dScal);
    (void)hipStreamDestroy(s);
    return 0;
}

}  // namespace orbgpu
