// comm.hpp -- the exchange step of keyframe-block-sharded bundle adjustment
// (SURVEY.md §8e): all-reduce of FP64 device buffers between the ranks that
// each own a slice of the map points.
//
// Three transports behind one interface:
//   RcclComm   one process per GPU, RCCL over xGMI.  librccl is dlopen'ed on
//              first use (the process may already hold torch's copy), so the
//              library loads -- and everything that is not sharded runs --
//              on a host without RCCL.
//   ShmComm    one process per rank on one host (any devices): the same staging
//              through a POSIX shared-memory segment and a cross-process barrier.
//   LocalComm  K ranks as K host threads of one process on one device (each
//              thread has its own HIP stream and BA workspace): partials are
//              staged to pinned host memory and summed in rank order.  It runs
//              the sharded protocol on a 1-GPU box, where RCCL cannot put two
//              ranks on one device.
// All produce bit-identical results on every rank (RCCL's ring reduce-scatter
// + all-gather hands every rank the same reduced chunk; LocalComm sums in a
// fixed order once per element).
#pragma once
#include <hip/hip_runtime.h>

#include <condition_variable>
#include <cstddef>
#include <cstdint>
#include <memory>
#include <mutex>
#include <vector>

namespace orbgpu {

enum class RedOp { Sum = 0, Max = 1 };

struct RedBuf {
    double* dev;
    size_t n;
};

class Comm {
public:
    virtual ~Comm() = default;
    int rank() const { return rank_; }
    int size() const { return size_; }
    // In-place all-reduce of every buffer (one fused exchange), ordered on `s`;
    // returns 0 or a negative ORB_E_* code.  Returns after the result is on `s`.
    virtual int allreduce(const RedBuf* bufs, int nbufs, RedOp op, hipStream_t s) = 0;
    int allreduce(double* dev, size_t n, RedOp op, hipStream_t s) {
        RedBuf b{dev, n};
        return allreduce(&b, 1, op, s);
    }

protected:
    int rank_ = 0, size_ = 1;
};

// RCCL transport
int rccl_unique_id(uint8_t id[128]);
Comm* rccl_comm_create(int nranks, int rank, const uint8_t id[128], int* rc);

// In-process transport: K handles sharing one group
std::vector<Comm*> local_comm_group(int nranks);

// Processes on one host: a POSIX shared-memory segment `name` (fresh per group) with one slot of
// max_doubles per rank; partials staged through pinned memory, summed in rank order on every
// rank (LocalComm's order, so the same bits); a cross-process barrier on lock-free atomics in
// the segment, bounded by ORBGPU_SHM_TIMEOUT seconds (default 300).  Runs the multi-process
// protocol where RCCL cannot (several ranks on one GPU).
Comm* shm_comm_create(const char* name, int nranks, int rank, size_t max_doubles, int* rc);

}  // namespace orbgpu
