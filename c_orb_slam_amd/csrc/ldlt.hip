// ldlt.hip -- block-sparse LDL^T solve of the reduced pose system S x = b_s for large bundle
// adjustments (reference: g2o LinearSolverEigen = Eigen SimplicialLDLT on the sparse Schur
// complement, Thirdparty/g2o/g2o/solvers/linear_solver_eigen.h:60-124; restated in oracle/ba.c
// ora_ldlt_solve).
//
// Storage: S is kept as 64 x 64 tiles of its upper triangle, only the tiles the Schur pattern
// (keyframes that share map points) and the factorisation's fill-in touch.  The symbolic
// factorisation runs once per structure on the host, at tile granularity, in natural pose
// order: row p of U gains the union of its elimination-tree children's rows.  A keyframe
// sequence whose points are seen by nearby keyframes gives a band of 2-3 tiles per row, so a
// 16k-keyframe map (n = 96k) holds ~4.5k tiles (150 MB) instead of a 74 GB dense matrix.
//   U  [slot] row-major tile (I, J), I <= J: S on entry; after the factorisation the
//      eliminated rows (U), and on diagonal tiles d on the diagonal and L strictly below;
//   LT [slot] of tile (p, J), p < J: LT[k][j] = L[J0 + j][p0 + k] (pivot-major, coalesced
//      for the trailing update and the forward solve).
// Per-element operation sequence is the oracle's: pivot k ascending, d_k = A[k][k],
// l_i = A[k][i] / d_k, A[i][j] -= l_i * A[k][j], no FMA contraction (the oracle skips l_i == 0,
// which only differs in the sign of a zero);
// forward y_i -= L[i][k] y_k (k ascending), y_k /= d_k, backward y_i -= L[k][i] y_k (k
// descending).  Tiles whose L is exactly zero are skipped in the trailing update and the
// solves, which is the oracle's l == 0 skip (exact up to the sign of zero).
//
// Two launches per solve: one 512-thread workgroup walks the panels (64 pivots each):
//   diag   wave 0, lane j = column j of the diagonal tile in registers, l_i broadcast
//          through LDS;
//   chunks the U tiles (p, J > p) of the panel row, one wave each: left-looking per column
//          with the diagonal L in LDS; writes U, LT and the tile's L-nonzero flag;
//   trail  the tile pairs (I <= J) of the panel's nonzero L tiles, two 256-thread groups
//          (4x4 register micro-tiles over LDS-staged LT (p, I) and U (p, J));
// then one wave runs the forward and backward solves block by block.  The band is a chain of
// dependent panels: there is no panel parallelism to spread over more workgroups in natural
// order, and one workgroup removes the 3 launches (and the grid drain) per panel.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <vector>

#include "ldlt.hpp"
#include "orb_common.hpp"

namespace orbgpu {

constexpr int LT = kTile;        // tile edge
constexpr int LP = LT + 1;       // LDS row pitch (doubles) of the diagonal L
constexpr int kSpThreads = 512;  // 8 waves
constexpr int kMaxRow = 2048;    // tiles per panel row
constexpr size_t kSpLds = sizeof(double) * (2 * 2 * LT * LT + LT) + sizeof(int) * (kMaxRow + 16);

struct SpDev {
    int n, nt;
    const int* slotOf;
    double* U;
    double* LT;
    const int* rowStart;
    const int* rowJ;
    const int* rowSlot;
    const int* colStart;
    const int* colK;
    const int* colSlot;
    const int* pairStart;
    const int4* pairs;   // (index of I in the panel row, index of J, target slot, 0)
    uint8_t* lnz;
    double* y;
};

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

__global__ void __launch_bounds__(kSpThreads) k_ldlt_sparse(SpDev S, const double* __restrict__ b,
                                                             double* __restrict__ x, double* scal) {
    // static LDS: addresses fold into the ds_read offsets (a dynamic base is a relocation the
    // compiler hoists into one SGPR per address)
    __shared__ double sm[kSpLds / sizeof(double)];
    double* Ls = sm;                       // [k][i] = L[i][k] of the diagonal tile (aliases the staging)
    double* dsh = sm + 2 * 2 * LT * LT;    // d_k of the panel
    int* flagS = (int*)(dsh + LT);         // L-nonzero flag per chunk of the panel row
    int* failS = flagS + kMaxRow;
    const int tid0 = threadIdx.x, lane0 = tid0 & 63, w = tid0 >> 6;
    const int n = S.n, nt = S.nt;
    if (tid0 == 0) *failS = 0;
    __syncthreads();
    ORBGPU_PROF_START;
    for (int p = 0; p < nt; p++) {
        // opaque per panel: keeps LICM from hoisting every lane mask and lane address of the
        // unrolled loops out of the panel loop (it spilled them)
        int lane = lane0, tid = tid0;
        asm volatile("" : "+v"(lane), "+v"(tid));
        const int p0 = p * LT, pw = min(LT, n - p0);
        const int rs = S.rowStart[p], m = S.rowStart[p + 1] - rs;
        // ---- diagonal tile (wave 0)
        if (w == 0) {
            // tiles are zero outside the system (rows / columns >= n) and below the diagonal
            const __amdgpu_buffer_rsrc_t Ud = tile_rsrc(S.U + (size_t)S.slotOf[(size_t)p * nt + p] * (LT * LT));
            const int vo = lane * 8;
            double col[LT];
#pragma unroll
            for (int r = 0; r < LT; r++) col[r] = tld(Ud, vo, r * LT * 8);
            bool bad = false;
#pragma unroll
            for (int k = 0; k < LT; k++) {
                if (k < pw && !bad) {
                    if (lane == k) dsh[k] = col[k];
                    __builtin_amdgcn_wave_barrier();
                    const double d = dsh[k];
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
            // pivots past the system's end: L = 0, d = 1, so the chunk pass needs no predicates
            for (int k = pw; k < LT; k++) {
                Ls[k * LP + lane] = 0.0;
                if (lane == 0) dsh[k] = 1.0;
            }
            if (bad) {
                if (lane == 0) *failS = 1;
            } else {
#pragma unroll
                for (int r = 0; r < LT; r++)
                    if (r < pw && lane < pw) tst(Ud, lane >= r ? col[r] : Ls[lane * LP + r], vo, r * LT * 8);
            }
        }
        __syncthreads();
        ORBGPU_PROF_MARK(16);
        if (*failS) break;
        // ---- U tiles (p, J > p) of the panel row: one wave per tile, lane = column
        const int wu = __builtin_amdgcn_readfirstlane(w);
        for (int t = wu; t < m; t += kSpThreads / 64) {
            const int sl = S.rowSlot[rs + t];
            const __amdgpu_buffer_rsrc_t Ut = tile_rsrc(S.U + (size_t)sl * (LT * LT));
            const __amdgpu_buffer_rsrc_t Lo = tile_rsrc(S.LT + (size_t)sl * (LT * LT));
            const int vo = lane * 8;
            double c[LT];
#pragma unroll
            for (int r = 0; r < LT; r++) c[r] = tld(Ut, vo, r * LT * 8);   // zero outside the system
            // per element the updates arrive in k order (the oracle's); the scheduling barrier
            // keeps the compiler from hoisting every pivot's 63 broadcast reads at once
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
            if (lane == 0) {
                flagS[t] = any ? 1 : 0;
                S.lnz[sl] = any ? 1 : 0;
            }
        }
        __syncthreads();
        ORBGPU_PROF_MARK(17);
        // ---- trailing update: A(I, J) -= L(I, p) U(p, J) over the panel's tile pairs
        const int ps = S.pairStart[p], np = S.pairStart[p + 1] - ps;
        const int g = tid >> 8, gt = tid & 255, ty = gt >> 4, tx = gt & 15;
        double* Lg = sm + g * (2 * LT * LT);   // [k][i] = L[I0 + i][p0 + k]
        double* Ug = Lg + LT * LT;             // [k][j] = U[p0 + k][J0 + j]
        for (int q0 = 0; q0 < np; q0 += 2) {
            const int q = q0 + g;
            int4 pr = make_int4(0, 0, 0, 0);
            bool act = false;
            if (q < np) {
                pr = S.pairs[ps + q];
                act = flagS[pr.x] && flagS[pr.y];
            }
            if (act) {
                const double2* srcL = (const double2*)(S.LT + (size_t)S.rowSlot[rs + pr.x] * (LT * LT));
                const double2* srcU = (const double2*)(S.U + (size_t)S.rowSlot[rs + pr.y] * (LT * LT));
                double2* dL = (double2*)Lg;
                double2* dU = (double2*)Ug;
#pragma unroll
                for (int u = 0; u < (LT * LT / 2) / 256; u++) {
                    dL[gt + 256 * u] = srcL[gt + 256 * u];
                    dU[gt + 256 * u] = srcU[gt + 256 * u];
                }
            }
            __syncthreads();
            if (act) {
                const int I = S.rowJ[rs + pr.x], J = S.rowJ[rs + pr.y];
                const int ih = min(LT, n - I * LT), jw = min(LT, n - J * LT);
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
            __syncthreads();
        }
        ORBGPU_PROF_MARK(18);
    }
    if (tid0 == 0) scal[3] = *failS ? 0.0 : 1.0;
}

// Forward / backward solves after a successful factorisation: one wave, block by block
// (lane = row of the block); the chain of dependent blocks is the band's.
__global__ void __launch_bounds__(64) k_ldlt_sparse_solve(SpDev S, const double* __restrict__ b,
                                                           double* __restrict__ x, const double* scal) {
    if (scal[3] == 0.0) return;
    const int lane = threadIdx.x;
    const int n = S.n, nt = S.nt;
    // ---- L y = b, block by block; lane = row
    double Lr[LT];
    for (int I = 0; I < nt; I++) {
        const int I0 = I * LT, ih = min(LT, n - I0);
        const bool on = lane < ih;
        double acc = on ? b[I0 + lane] : 0.0;
        for (int e = S.colStart[I]; e < S.colStart[I + 1]; e++) {
            const int sl = S.colSlot[e];
            if (!S.lnz[sl]) continue;
            const int K0 = S.colK[e] * LT;   // K < I: a full tile
            const double yk = S.y[K0 + lane];
            const double* Lo = S.LT + (size_t)sl * (LT * LT);   // [k][i] = L[I0 + i][K0 + k]
#pragma unroll
            for (int k = 0; k < LT; k++) Lr[k] = Lo[k * LT + lane];
#pragma unroll
            for (int k = 0; k < LT; k++) {
                const double v = acc - Lr[k] * rdlane(yk, k);
                acc = on ? v : acc;
            }
        }
        const double* Ud = S.U + (size_t)S.slotOf[(size_t)I * nt + I] * (LT * LT);
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
        if (on) S.y[I0 + lane] = acc;
    }
    // ---- y /= d, then L^T x = y with k descending
    for (int I = nt - 1; I >= 0; I--) {
        const int I0 = I * LT, ih = min(LT, n - I0);
        const bool on = lane < ih;
        const double* Ud = S.U + (size_t)S.slotOf[(size_t)I * nt + I] * (LT * LT);
        double acc = on ? S.y[I0 + lane] / Ud[lane * LT + lane] : 0.0;
        for (int e = S.rowStart[I + 1] - 1; e >= S.rowStart[I]; e--) {
            const int sl = S.rowSlot[e];
            if (!S.lnz[sl]) continue;
            const int K0 = S.rowJ[e] * LT, kh = min(LT, n - K0);
            const double xk = lane < kh ? x[K0 + lane] : 0.0;
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
        if (on) x[I0 + lane] = acc;
    }
}

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
}

int SparseLdlt::build(int n, const std::vector<uint8_t>& mask, hipStream_t s) {
    n_ = n;
    nt_ = (n + LT - 1) / LT;
    const int nt = nt_;
    if (n <= 0) {
        nslot_ = nA_ = 0;
        return 0;
    }
    if ((size_t)nt * nt != mask.size()) return -1;
    // symbolic factorisation at tile granularity (natural order): struct(p) joins its parent's
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
    // panel rows (J > p), block columns (K < I), trailing pairs
    std::vector<int> rowStart(nt + 1, 0), rowJ, rowSlot, colStart(nt + 1, 0), colK, colSlot, pairStart(nt + 1, 0);
    std::vector<int4> pairs;
    std::vector<std::vector<int>> cols(nt);
    for (int p = 0; p < nt; p++) {
        rowStart[p] = (int)rowJ.size();
        pairStart[p] = (int)pairs.size();
        const std::vector<int>& r = rows[p];
        for (size_t q = 1; q < r.size(); q++) {
            rowJ.push_back(r[q]);
            rowSlot.push_back(hSlotOf_[(size_t)p * nt + r[q]]);
            cols[r[q]].push_back(p);
        }
        const int m = (int)r.size() - 1;
        for (int a = 0; a < m; a++)
            for (int bb = a; bb < m; bb++) {
                const int t = hSlotOf_[(size_t)r[1 + a] * nt + r[1 + bb]];
                if (t < 0) return -1;   // the fill closure guarantees the target tile
                pairs.push_back(make_int4(a, bb, t, 0));
            }
    }
    rowStart[nt] = (int)rowJ.size();
    pairStart[nt] = (int)pairs.size();
    for (int I = 0; I < nt; I++) {
        colStart[I] = (int)colK.size();
        for (int K : cols[I]) {   // ascending K
            colK.push_back(K);
            colSlot.push_back(hSlotOf_[(size_t)K * nt + I]);
        }
    }
    colStart[nt] = (int)colK.size();
    // device storage (grow-only)
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
    const size_t oLnz = take(nslot_);
    const size_t nInts = rowStart.size() + rowJ.size() + rowSlot.size() + colStart.size() + colK.size() + colSlot.size() +
                         pairStart.size() + 4 * pairs.size() + 64;
    const size_t oLists = take(sizeof(int) * nInts);
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
    lnz_ = (uint8_t*)(base + oLnz);
    lists_ = (int*)(base + oLists);
    std::vector<int> L;
    L.reserve(nInts);
    auto put = [&](const std::vector<int>& v) {
        const size_t o = L.size();
        L.insert(L.end(), v.begin(), v.end());
        return o;
    };
    offRowStart_ = put(rowStart);
    offRowJ_ = put(rowJ);
    offRowSlot_ = put(rowSlot);
    offColStart_ = put(colStart);
    offColK_ = put(colK);
    offColSlot_ = put(colSlot);
    offPairStart_ = put(pairStart);
    while (L.size() % 4) L.push_back(0);
    offPairs_ = L.size();
    for (const int4& q : pairs) {
        L.push_back(q.x);
        L.push_back(q.y);
        L.push_back(q.z);
        L.push_back(q.w);
    }
    ORB_HIP_CHECK(hipMemcpyAsync(slotOf_, hSlotOf_.data(), sizeof(int) * hSlotOf_.size(), hipMemcpyHostToDevice, s));
    ORB_HIP_CHECK(hipMemcpyAsync(lists_, L.data(), sizeof(int) * L.size(), hipMemcpyHostToDevice, s));
    ORB_HIP_CHECK(hipStreamSynchronize(s));   // pageable sources
    return 0;
}

int SparseLdlt::zero(hipStream_t s) {
    if (nslot_) ORB_HIP_CHECK(hipMemsetAsync(U_, 0, sizeof(double) * LT * LT * (size_t)nslot_, s));
    return 0;
}

int SparseLdlt::solve(const double* b, double* x, double* scal, hipStream_t s) {
    if (n_ <= 0) return 0;
    SpDev d;
    d.n = n_;
    d.nt = nt_;
    d.slotOf = slotOf_;
    d.U = U_;
    d.LT = LT_;
    d.rowStart = lists_ + offRowStart_;
    d.rowJ = lists_ + offRowJ_;
    d.rowSlot = lists_ + offRowSlot_;
    d.colStart = lists_ + offColStart_;
    d.colK = lists_ + offColK_;
    d.colSlot = lists_ + offColSlot_;
    d.pairStart = lists_ + offPairStart_;
    d.pairs = (const int4*)(lists_ + offPairs_);
    d.lnz = lnz_;
    d.y = y_;
    hipLaunchKernelGGL(k_ldlt_sparse, dim3(1), dim3(kSpThreads), 0, s, d, b, x, scal);
    hipLaunchKernelGGL(k_ldlt_sparse_solve, dim3(1), dim3(64), 0, s, d, b, x, scal);
    ORB_HIP_CHECK(hipGetLastError());
    return 0;
}

int ldlt_sparse_dense(int n, const double* S, const double* b, double* x, int* ok, double* factor_out) {
    *ok = 0;
    if (n <= 0) {
        *ok = 1;
        return 0;
    }
    const int nt = (n + LT - 1) / LT;
    std::vector<uint8_t> mask((size_t)nt * nt, 0);
    for (int i = 0; i < n; i++)
        for (int j = i; j < n; j++)
            if (S[(size_t)i * n + j] != 0.0) mask[(size_t)(i / LT) * nt + j / LT] = 1;
    hipStream_t s = nullptr;
    ORB_HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    SparseLdlt L;
    if (int e = L.build(n, mask, s)) return e;
    const std::vector<int>& so = L.host_slot_of();
    std::vector<double> T((size_t)L.nslot() * LT * LT, 0.0);
    for (int i = 0; i < n; i++)
        for (int j = i; j < n; j++) {
            const int sl = so[(size_t)(i / LT) * nt + j / LT];
            if (sl >= 0) T[(size_t)sl * LT * LT + (i % LT) * LT + j % LT] = S[(size_t)i * n + j];
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
    if (factor_out) {   // the dense layout of the factor: U above, d on the diagonal, L below
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
