// ldlt.hpp -- block-sparse (64x64-tile) LDL^T solve of the reduced pose system (see ldlt.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <vector>

#include "ordering.hpp"

namespace orbgpu {

constexpr int kTile = 64;
struct SpDev;
class Comm;

// Where k_schur writes S(r, c) (r <= c, system order): a dense row-major (nn x nn) matrix, or
// the tiles of the block-sparse system.  There the poses are permuted (nested dissection):
// prow[r / 6] is the tile-space row of pose r / 6's first row, and an element that the
// permutation moves below the diagonal is stored at its mirror (S is symmetric).
struct SysAddr {
    double* dense;
    int nn;
    const int* slot_of;
    double* tiles;
    int nt;
    const int* prow;
    __device__ __forceinline__ double* at(int r, int c) const {
        if (dense) return dense + (size_t)r * nn + c;
        int a = prow[r / 6] + r % 6, b = prow[c / 6] + c % 6;
        if (a > b) {
            const int t = a;
            a = b;
            b = t;
        }
        const int s = slot_of[(size_t)(a >> 6) * nt + (b >> 6)];
        return tiles + (size_t)s * (kTile * kTile) + (a & 63) * kTile + (b & 63);
    }
};

// Symbolic structure + device storage of one pose system, built once per BA structure.
// Slots [0, nA) are the tiles of the Schur pattern (the tiles an all-reduce has to carry);
// slots [nA, nslot) are the fill-in of the factorisation.
class SparseLdlt {
public:
    ~SparseLdlt();
    // n rows in groups of g (poses: g = 6; the last group may be short); adjStart / adj: the
    // group graph (symmetric, sorted lists, no self loops).  nd: nested-dissection order
    // (ordering.hpp) and the level-parallel schedule; false: natural order, one node.
    int build(int n, int g, const std::vector<int>& adjStart, const std::vector<int>& adj, bool nd, hipStream_t s);
    // S is in the tiles (upper triangle); factorised in place; b, x in system order.  scal[3] =
    // 1 on success (x written), 0 on an exactly zero pivot (x untouched).
    int solve(const double* b, double* x, double* scal, hipStream_t s);
    int zero(hipStream_t s);   // clear every tile (before S is assembled)
    // Sharded factorisation (R ranks, this one `rank`): whole subtrees of the separator tree per
    // rank (nd_assign), the separators above them factored by every rank.  plan() derives the
    // tile classes, the exchange lists and the per-pose owner flags; -1 if the order has no
    // tree (natural order) or R < 2.  After it, solve_dist() replaces solve(): each rank factors
    // its subtrees, all-reduces {S - its subtrees' updates, b - their forward contributions} over
    // the separator tiles and rows, factors the separators redundantly, back-substitutes its
    // subtrees and all-reduces x.  S here is the rank's OWN partial Schur complement (no prior
    // all-reduce): it must touch only this rank's subtrees and the separators (align_flag()).
    int plan(int R, int rank, hipStream_t s);
    bool dist() const { return dist_; }
    int solve_dist(double* b, double* x, double* scal, hipStream_t s, Comm* comm);
    // 1 in *flag if an active edge of this rank has its pose in another rank's subtree
    int align_flag(const int* ePose, int nE, int* flag, hipStream_t s);
    const uint8_t* pose_add() const { return dPoseAdd_; }   // k_schur: this rank adds Hpp + lambda, b_p
    int dist_shared_tiles() const { return nShSlots_; }
    int dist_shared_rows() const { return nShT_ * kTile; }
    SysAddr addr() const { return SysAddr{nullptr, n_, slotOf_, U_, nt_, prow_}; }
    double* tiles() const { return U_; }
    double* lt_tiles() const { return LT_; }
    int n() const { return n_; }
    int nt() const { return nt_; }
    int nA() const { return nA_; }
    int nslot() const { return nslot_; }
    int levels() const { return nLev_; }
    long long update_products() const { return nUpd_; }
    const std::vector<int>& host_slot_of() const { return hSlotOf_; }
    const std::vector<int>& host_prow() const { return hProw_; }

private:
    SpDev dev() const;
    void enqueue_factor_level(const SpDev& d, int h, const double* b, hipStream_t s);
    void enqueue_backward_level(const SpDev& d, int h, double* x, double* scal, int first, hipStream_t s);
    int n_ = 0, nt_ = 0, nslot_ = 0, nA_ = 0, nLev_ = 0;
    bool nd_ = false, dist_ = false;
    int rank_ = 0, nShSlots_ = 0, nShT_ = 0;
    NdTree tree_;
    std::vector<int> hNodeT_;
    std::vector<uint8_t> levOwn_, levSh_;
    void* distMem_ = nullptr;
    size_t distCap_ = 0;
    uint8_t *dTcls_ = nullptr, *dPoseAdd_ = nullptr;
    int *dPackIdx_ = nullptr, *dShSlots_ = nullptr, *dShT_ = nullptr;
    double* dXbuf_ = nullptr;
    long long nUpd_ = 0;
    void* mem_ = nullptr;
    size_t cap_ = 0;
    int* slotOf_ = nullptr;
    int* prow_ = nullptr;
    int* fail_ = nullptr;
    double *U_ = nullptr, *LT_ = nullptr, *y_ = nullptr, *xs_ = nullptr, *acc_ = nullptr;
    int* lists_ = nullptr;
    uint8_t* lnz_ = nullptr;
    size_t offTh_ = 0, offRowMap_ = 0, offRowStart_ = 0, offRowJ_ = 0, offRowSlot_ = 0, offColStart_ = 0,
           offColK_ = 0, offColSlot_ = 0, offPairStart_ = 0, offNodeT_ = 0, offLevNodes_ = 0, offPairs_ = 0,
           offTgts_ = 0, offKps_ = 0, offStepP_ = 0, offRowJobs_ = 0, offPairJobs_ = 0, offPanelJobs_ = 0, offPush_ = 0;
    std::vector<int> hSlotOf_, hProw_, hLevNodeStart_, hLevTgtStart_, hLevStepStart_, hLevPushStart_;
    std::vector<int> hLevMaxT_;   // per level: the most tiles of one of its nodes (sweep launch shape)
    std::vector<int4> hSteps_;   // per panel step: first (panel, row job, pair job, panel job); + sentinel
};

// Unit entry: dense host S (upper read) -> pattern of its nonzero 6 x 6 blocks -> sparse solve
// (nd: nested-dissection order; else natural).  factor_out (optional, n x n, natural order
// only): d on the diagonal, L strictly below, the eliminated rows above.
int ldlt_debug_prof(unsigned long long* out8);   // prof builds: section cycles (diag, chunks, trail)
int ldlt_sparse_dense(int n, const double* S, const double* b, double* x, int* ok, double* factor_out, bool nd);

}  // namespace orbgpu
