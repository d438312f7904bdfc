// comm.cpp -- RCCL and in-process transports of the BA exchange step (see comm.hpp).
#include "comm.hpp"

#include <dlfcn.h>
#include <fcntl.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>

#include <rccl/rccl.h>

#include "../../include/orbslam_gpu.h"

namespace orbgpu {

// ---------------------------------------------------------------- RCCL (dlopen)
namespace {
struct RcclApi {
    bool ok = false;
    ncclResult_t (*getUniqueId)(ncclUniqueId*) = nullptr;
    ncclResult_t (*commInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*commDestroy)(ncclComm_t) = nullptr;
    ncclResult_t (*allReduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                              hipStream_t) = nullptr;
    ncclResult_t (*groupStart)() = nullptr;
    ncclResult_t (*groupEnd)() = nullptr;
};

const RcclApi& rccl() {
    static RcclApi api = [] {
        RcclApi a;
        void* h = nullptr;
        for (const char* name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"}) {
            h = dlopen(name, RTLD_NOW | RTLD_GLOBAL);
            if (h) break;
        }
        if (!h) return a;
        a.getUniqueId = (decltype(a.getUniqueId))dlsym(h, "ncclGetUniqueId");
        a.commInitRank = (decltype(a.commInitRank))dlsym(h, "ncclCommInitRank");
        a.commDestroy = (decltype(a.commDestroy))dlsym(h, "ncclCommDestroy");
        a.allReduce = (decltype(a.allReduce))dlsym(h, "ncclAllReduce");
        a.groupStart = (decltype(a.groupStart))dlsym(h, "ncclGroupStart");
        a.groupEnd = (decltype(a.groupEnd))dlsym(h, "ncclGroupEnd");
        a.ok = a.getUniqueId && a.commInitRank && a.commDestroy && a.allReduce && a.groupStart && a.groupEnd;
        return a;
    }();
    return api;
}

class RcclComm final : public Comm {
public:
    RcclComm(ncclComm_t c, int nranks, int rank) : comm_(c) {
        size_ = nranks;
        rank_ = rank;
    }
    ~RcclComm() override {
        if (comm_) rccl().commDestroy(comm_);
    }
    int allreduce(const RedBuf* bufs, int nbufs, RedOp op, hipStream_t s) override {
        if (size_ == 1) return ORB_OK;
        const RcclApi& a = rccl();
        const ncclRedOp_t o = op == RedOp::Sum ? ncclSum : ncclMax;
        if (a.groupStart() != ncclSuccess) return ORB_E_HIP;
        ncclResult_t r = ncclSuccess;
        for (int i = 0; i < nbufs && r == ncclSuccess; i++)
            if (bufs[i].n) r = a.allReduce(bufs[i].dev, bufs[i].dev, bufs[i].n, ncclFloat64, o, comm_, s);
        const ncclResult_t r2 = a.groupEnd();
        return (r == ncclSuccess && r2 == ncclSuccess) ? ORB_OK : ORB_E_HIP;
    }

private:
    ncclComm_t comm_;
};
}  // namespace

int rccl_unique_id(uint8_t id[128]) {
    const RcclApi& a = rccl();
    if (!a.ok) return ORB_E_NODEVICE;
    ncclUniqueId u;
    if (a.getUniqueId(&u) != ncclSuccess) return ORB_E_HIP;
    static_assert(sizeof(u) == 128, "ncclUniqueId is 128 bytes");
    std::memcpy(id, &u, 128);
    return ORB_OK;
}

Comm* rccl_comm_create(int nranks, int rank, const uint8_t id[128], int* rc) {
    const RcclApi& a = rccl();
    if (!a.ok) {
        *rc = ORB_E_NODEVICE;
        return nullptr;
    }
    ncclUniqueId u;
    std::memcpy(&u, id, 128);
    ncclComm_t c = nullptr;
    if (a.commInitRank(&c, nranks, u, rank) != ncclSuccess) {
        *rc = ORB_E_HIP;
        return nullptr;
    }
    *rc = ORB_OK;
    return new RcclComm(c, nranks, rank);
}

// ---------------------------------------------------------------- in-process group
namespace {
struct LocalGroup {
    int n;
    std::mutex mu;
    std::condition_variable cv;
    int arrived = 0;
    long gen = 0;
    std::vector<double*> stage;     // pinned, one per rank
    std::vector<size_t> cap;
    std::vector<size_t> len;

    explicit LocalGroup(int k) : n(k), stage(k, nullptr), cap(k, 0), len(k, 0) {}
    ~LocalGroup() {
        for (double* p : stage)
            if (p) (void)hipHostFree(p);
    }
    void barrier() {
        std::unique_lock<std::mutex> lk(mu);
        const long g = gen;
        if (++arrived == n) {
            arrived = 0;
            gen++;
            cv.notify_all();
        } else {
            cv.wait(lk, [&] { return gen != g; });
        }
    }
};

class LocalComm final : public Comm {
public:
    LocalComm(std::shared_ptr<LocalGroup> g, int rank) : g_(std::move(g)) {
        size_ = g_->n;
        rank_ = rank;
    }
    ~LocalComm() override {
        if (res_) (void)hipHostFree(res_);
    }
    int allreduce(const RedBuf* bufs, int nbufs, RedOp op, hipStream_t s) override {
        if (size_ == 1) return ORB_OK;
        size_t tot = 0;
        for (int i = 0; i < nbufs; i++) tot += bufs[i].n;
        LocalGroup& G = *g_;
        int rc = ORB_OK;
        if (tot > G.cap[rank_] || tot > resCap_) {
            if (G.stage[rank_]) (void)hipHostFree(G.stage[rank_]);
            if (res_) (void)hipHostFree(res_);
            G.stage[rank_] = res_ = nullptr;
            G.cap[rank_] = resCap_ = 0;
            if (hipHostMalloc((void**)&G.stage[rank_], sizeof(double) * tot) != hipSuccess ||
                hipHostMalloc((void**)&res_, sizeof(double) * tot) != hipSuccess)
                rc = ORB_E_HIP;
            else
                G.cap[rank_] = resCap_ = tot;
        }
        size_t off = 0;
        for (int i = 0; i < nbufs && rc == ORB_OK; i++) {
            if (bufs[i].n && hipMemcpyAsync(G.stage[rank_] + off, bufs[i].dev, sizeof(double) * bufs[i].n,
                                            hipMemcpyDeviceToHost, s) != hipSuccess)
                rc = ORB_E_HIP;
            off += bufs[i].n;
        }
        if (rc == ORB_OK && hipStreamSynchronize(s) != hipSuccess) rc = ORB_E_HIP;
        G.len[rank_] = rc == ORB_OK ? tot : (size_t)-1;
        G.barrier();  // every rank's partial is staged
        for (int r = 0; r < size_; r++)
            if (G.len[r] != tot) rc = ORB_E_HIP;  // a rank failed or the ranks disagree on the shape
        if (rc == ORB_OK) {
            std::memcpy(res_, G.stage[0], sizeof(double) * tot);
            for (int r = 1; r < size_; r++) {
                const double* p = G.stage[r];
                if (op == RedOp::Sum)
                    for (size_t j = 0; j < tot; j++) res_[j] = res_[j] + p[j];
                else
                    for (size_t j = 0; j < tot; j++) res_[j] = std::max(res_[j], p[j]);
            }
        }
        G.barrier();  // nobody reads the staging buffers any more
        if (rc != ORB_OK) return rc;
        off = 0;
        for (int i = 0; i < nbufs; i++) {
            if (bufs[i].n && hipMemcpyAsync(bufs[i].dev, res_ + off, sizeof(double) * bufs[i].n,
                                            hipMemcpyHostToDevice, s) != hipSuccess)
                return ORB_E_HIP;
            off += bufs[i].n;
        }
        return hipStreamSynchronize(s) == hipSuccess ? ORB_OK : ORB_E_HIP;  // res_ is reused next call
    }

private:
    std::shared_ptr<LocalGroup> g_;
    double* res_ = nullptr;
    size_t resCap_ = 0;
};
}  // namespace

// ---------------------------------------------------------------- processes on one host (shared memory)
namespace {
constexpr long long kShmMagic = 0x4f52424753484d31LL;   // "ORBGSHM1"
constexpr int kShmMaxRanks = 64;
struct ShmHeader {
    std::atomic<long long> magic;
    std::atomic<int> attached;
    std::atomic<int> arrived;
    std::atomic<long long> gen;
    int nranks;
    long long cap;                       // doubles per rank slot
    long long len[kShmMaxRanks];         // this exchange's length per rank (-1: the rank failed)
};
static_assert(std::atomic<long long>::is_always_lock_free && std::atomic<int>::is_always_lock_free,
              "cross-process atomics must be lock-free");
constexpr size_t kShmHdr = 4096;

double shm_timeout_s() {
    const char* e = std::getenv("ORBGPU_SHM_TIMEOUT");
    return e ? std::atof(e) : 300.0;
}

class ShmComm final : public Comm {
public:
    ShmComm(void* base, size_t bytes, int nranks, int rank) : base_(base), bytes_(bytes) {
        size_ = nranks;
        rank_ = rank;
        H_ = (ShmHeader*)base;
    }
    ~ShmComm() override {
        if (res_) (void)hipHostFree(res_);
        if (base_) munmap(base_, bytes_);
    }
    double* slot(int r) const { return (double*)((char*)base_ + kShmHdr) + (size_t)r * H_->cap; }
    // every rank of the group arrives; false on timeout (a rank died or never came)
    bool barrier() {
        const long long g = H_->gen.load(std::memory_order_acquire);
        if (H_->arrived.fetch_add(1, std::memory_order_acq_rel) + 1 == size_) {
            H_->arrived.store(0, std::memory_order_relaxed);
            H_->gen.fetch_add(1, std::memory_order_acq_rel);
            return true;
        }
        const auto t0 = std::chrono::steady_clock::now();
        const double lim = shm_timeout_s();
        for (unsigned spin = 0; H_->gen.load(std::memory_order_acquire) == g; spin++) {
            if (spin < 2048) {
                __builtin_ia32_pause();
            } else {
                if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > lim) return false;
                if (spin < 8192)
                    sched_yield();
                else
                    std::this_thread::sleep_for(std::chrono::microseconds(50));
            }
        }
        return true;
    }
    int allreduce(const RedBuf* bufs, int nbufs, RedOp op, hipStream_t s) override {
        if (size_ == 1) return ORB_OK;
        size_t tot = 0;
        for (int i = 0; i < nbufs; i++) tot += bufs[i].n;
        int rc = tot > (size_t)H_->cap ? ORB_E_CAPACITY : ORB_OK;
        if (rc == ORB_OK && tot > resCap_) {
            if (res_) (void)hipHostFree(res_);
            res_ = nullptr;
            resCap_ = 0;
            if (hipHostMalloc((void**)&res_, sizeof(double) * tot) != hipSuccess)
                rc = ORB_E_HIP;
            else
                resCap_ = tot;
        }
        size_t off = 0;   // partial -> pinned -> this rank's slot
        for (int i = 0; i < nbufs && rc == ORB_OK; i++) {
            if (bufs[i].n && hipMemcpyAsync(res_ + off, bufs[i].dev, sizeof(double) * bufs[i].n, hipMemcpyDeviceToHost,
                                            s) != hipSuccess)
                rc = ORB_E_HIP;
            off += bufs[i].n;
        }
        if (rc == ORB_OK && hipStreamSynchronize(s) != hipSuccess) rc = ORB_E_HIP;
        if (rc == ORB_OK) std::memcpy(slot(rank_), res_, sizeof(double) * tot);
        H_->len[rank_] = rc == ORB_OK ? (long long)tot : -1;
        if (!barrier()) return ORB_E_HIP;   // every rank's partial is in its slot
        for (int r = 0; r < size_; r++)
            if (H_->len[r] != (long long)tot) rc = rc == ORB_OK ? ORB_E_HIP : rc;   // a failed rank, or shapes differ
        if (rc == ORB_OK) {   // rank order, once per element: the same bits on every rank (LocalComm's order)
            std::memcpy(res_, slot(0), sizeof(double) * tot);
            for (int r = 1; r < size_; r++) {
                const double* p = slot(r);
                if (op == RedOp::Sum)
                    for (size_t j = 0; j < tot; j++) res_[j] = res_[j] + p[j];
                else
                    for (size_t j = 0; j < tot; j++) res_[j] = std::max(res_[j], p[j]);
            }
        }
        if (!barrier()) return ORB_E_HIP;   // nobody reads the slots any more
        if (rc != ORB_OK) return rc;
        off = 0;
        for (int i = 0; i < nbufs; i++) {
            if (bufs[i].n && hipMemcpyAsync(bufs[i].dev, res_ + off, sizeof(double) * bufs[i].n,
                                            hipMemcpyHostToDevice, s) != hipSuccess)
                return ORB_E_HIP;
            off += bufs[i].n;
        }
        return hipStreamSynchronize(s) == hipSuccess ? ORB_OK : ORB_E_HIP;   // res_ is reused next call
    }

private:
    void* base_;
    size_t bytes_;
    ShmHeader* H_ = nullptr;
    double* res_ = nullptr;
    size_t resCap_ = 0;
};
}  // namespace

Comm* shm_comm_create(const char* name, int nranks, int rank, size_t max_doubles, int* rc) {
    *rc = ORB_E_INVALID;
    if (!name || name[0] != '/' || nranks < 1 || nranks > kShmMaxRanks || rank < 0 || rank >= nranks || !max_doubles)
        return nullptr;
    const size_t bytes = kShmHdr + sizeof(double) * max_doubles * (size_t)nranks;
    const double lim = shm_timeout_s();
    const auto t0 = std::chrono::steady_clock::now();
    auto waited = [&] { return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count(); };
    int fd = -1;
    if (rank == 0) {   // creates a fresh segment (a stale one of the same name is replaced)
        shm_unlink(name);
        fd = shm_open(name, O_CREAT | O_EXCL | O_RDWR, 0600);
        if (fd < 0 || ftruncate(fd, (off_t)bytes) != 0) {
            if (fd >= 0) close(fd);
            *rc = ORB_E_HIP;
            return nullptr;
        }
    } else {   // waits for rank 0's segment
        while ((fd = shm_open(name, O_RDWR, 0600)) < 0) {
            if (waited() > lim) {
                *rc = ORB_E_HIP;
                return nullptr;
            }
            std::this_thread::sleep_for(std::chrono::milliseconds(2));
        }
        struct stat st;
        while (fstat(fd, &st) == 0 && (size_t)st.st_size < bytes) {
            if (waited() > lim) break;
            std::this_thread::sleep_for(std::chrono::milliseconds(2));
        }
    }
    void* base = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (base == MAP_FAILED) {
        *rc = ORB_E_HIP;
        return nullptr;
    }
    ShmHeader* H = (ShmHeader*)base;
    if (rank == 0) {
        H->nranks = nranks;
        H->cap = (long long)max_doubles;
        H->magic.store(kShmMagic, std::memory_order_release);
    } else {
        while (H->magic.load(std::memory_order_acquire) != kShmMagic) {
            if (waited() > lim) {
                munmap(base, bytes);
                *rc = ORB_E_HIP;
                return nullptr;
            }
            std::this_thread::sleep_for(std::chrono::milliseconds(1));
        }
        if (H->nranks != nranks || H->cap != (long long)max_doubles) {   // the ranks disagree on the group
            munmap(base, bytes);
            *rc = ORB_E_INVALID;
            return nullptr;
        }
    }
    H->attached.fetch_add(1, std::memory_order_acq_rel);
    ShmComm* c = new ShmComm(base, bytes, nranks, rank);
    if (!c->barrier()) {   // every rank attached
        delete c;
        *rc = ORB_E_HIP;
        return nullptr;
    }
    if (rank == 0) shm_unlink(name);   // the mappings stay; no name is left behind in /dev/shm
    *rc = ORB_OK;
    return c;
}

std::vector<Comm*> local_comm_group(int nranks) {
    auto g = std::make_shared<LocalGroup>(nranks);
    std::vector<Comm*> v;
    for (int r = 0; r < nranks; r++) v.push_back(new LocalComm(g, r));
    return v;
}

}  // namespace orbgpu
