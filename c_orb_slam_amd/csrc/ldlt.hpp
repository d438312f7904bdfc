// ldlt.hpp -- block-sparse (64x64-tile) LDL^T solve of the reduced pose system (see ldlt.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <vector>

namespace orbgpu {

constexpr int kTile = 64;

// Where k_schur writes S(r, c) (r <= c): a dense row-major (nn x nn) matrix, or the tiles of
// the block-sparse system (slot_of[(r/64) * nt + c/64] -> tile, row-major 64 x 64).
struct SysAddr {
    double* dense;
    int nn;
    const int* slot_of;
    double* tiles;
    int nt;
    __device__ __forceinline__ double* at(int r, int c) const {
        if (dense) return dense + (size_t)r * nn + c;
        const int s = slot_of[(size_t)(r >> 6) * nt + (c >> 6)];
        return tiles + (size_t)s * (kTile * kTile) + (r & 63) * kTile + (c & 63);
    }
};

// Symbolic structure + device storage of one pose system, built once per BA structure.
// Slots [0, nA) are the tiles of the Schur pattern (the tiles an all-reduce has to carry);
// slots [nA, nslot) are the fill-in of the factorisation (natural pose order).
class SparseLdlt {
public:
    ~SparseLdlt();
    // mask: nt x nt row-major, mask[I * nt + J] != 0 (I <= J) = tile may be nonzero in S.
    int build(int n, const std::vector<uint8_t>& mask, hipStream_t s);
    // S is in the tiles (upper triangle); factorised in place.  scal[3] = 1 on success (x
    // written), 0 on an exactly zero pivot (x untouched).  One launch.
    int solve(const double* b, double* x, double* scal, hipStream_t s);
    int zero(hipStream_t s);   // clear every tile (before S is assembled)
    SysAddr addr() const { return SysAddr{nullptr, n_, slotOf_, U_, nt_}; }
    double* tiles() const { return U_; }
    double* lt_tiles() const { return LT_; }
    int n() const { return n_; }
    int nt() const { return nt_; }
    int nA() const { return nA_; }
    int nslot() const { return nslot_; }
    const std::vector<int>& host_slot_of() const { return hSlotOf_; }

private:
    int n_ = 0, nt_ = 0, nslot_ = 0, nA_ = 0;
    void* mem_ = nullptr;
    size_t cap_ = 0;
    int* slotOf_ = nullptr;
    double *U_ = nullptr, *LT_ = nullptr, *y_ = nullptr;
    int* lists_ = nullptr;
    uint8_t* lnz_ = nullptr;
    size_t offRowStart_ = 0, offRowJ_ = 0, offRowSlot_ = 0, offColStart_ = 0, offColK_ = 0, offColSlot_ = 0,
           offPairStart_ = 0, offPairs_ = 0;
    std::vector<int> hSlotOf_;
};

// Unit entry: dense host S (upper read) -> pattern of its nonzero tiles -> sparse solve.
// factor_out (optional, n x n): d on the diagonal, L strictly below, the eliminated rows above.
int ldlt_debug_prof(unsigned long long* out8);   // prof builds: section cycles (diag, chunks, trail)
int ldlt_sparse_dense(int n, const double* S, const double* b, double* x, int* ok, double* factor_out);

}  // namespace orbgpu
