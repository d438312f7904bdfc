// comm.cpp -- RCCL and in-process transports of the BA exchange step (see comm.hpp).
#include "comm.hpp"

#include <dlfcn.h>

#include <algorithm>
#include <cstring>

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

std::vector<Comm*> local_comm_group(int nranks) {
    auto g = std::make_shared<LocalGroup>(nranks);
    std::vector<Comm*> v;
    for (int r = 0; r < nranks; r++) v.push_back(new LocalComm(g, r));
    return v;
}

}  // namespace orbgpu
