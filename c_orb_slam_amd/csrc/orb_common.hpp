// orb_common.hpp -- shared HIP helpers for the gfx950 ORB-SLAM2 hot path.
//
// Every kernel is compiled with -ffp-contract=off and correctly rounded f32
// division so float expressions evaluate exactly as the reference's scalar C++
// (SURVEY.md F8).  Device math that must match host libm/OpenCV bit-for-bit
// (cvRound, fastAtan2, glibc sinf/cosf) is restated here explicitly.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <deque>
#include <mutex>
#include <vector>

#define ORB_HIP_CHECK(expr)                                                            \
    do {                                                                               \
        hipError_t _e = (expr);                                                        \
        if (_e != hipSuccess) {                                                        \
            fprintf(stderr, "[orbslam_gpu] HIP error %s at %s:%d: %s\n",               \
                    hipGetErrorName(_e), __FILE__, __LINE__, #expr);                   \
            return -2;                                                                 \
        }                                                                              \
    } while (0)

namespace orbgpu {

// Wait for everything queued on stream s by polling: a one-thread kernel queued behind the work
// writes a sequence number to the calling thread's pinned coherent word and the host spins on it.
// hipStreamSynchronize sleeps and wakes some 20-30 us after the work it waits for (BA readbacks,
// profiles/r05d2lba vs r05e2lba timelines), once per synchronous call of a tracking frame.  Past
// 50 ms of spinning, or without a pinned word, it is hipStreamSynchronize.  (orb_match.hip)
hipError_t stream_wait(hipStream_t s);

// Deferred completion of a chain of batch calls on one stream (bench tracking lane): the host
// sources of a call's H2D copies and the destinations of its count D2H copies live in pinned
// blocks that stay untouched until the chain is finished, so a call can return without
// synchronising and the next call's kernels queue right behind it.  A chain is closed into an
// epoch (an event on the stream); epochs finish in order -- wait for the event, copy the counts
// to the callers' arrays, release the blocks -- so the next chain can be queued while an older
// one still runs.  wait() (event only) may be called from another host thread.
//
// Each epoch owns its event until it is finished and no waiter holds it: an event is never
// re-recorded while a host thread may be synchronising on it, however many epochs are open.
class DeferredChain {
public:
    ~DeferredChain() {
        for (auto& b : blocks_) (void)hipHostFree(b.p);
        for (auto& b : devs_) (void)hipFree(b.p);
        for (auto& e : events_)
            if (e.ev) (void)hipEventDestroy(e.ev);
    }
    bool on() const { return on_; }
    void set(bool v) { on_ = v; }
    // pinned copy of host bytes, valid until the current chain finishes
    void* stage(const void* src, size_t bytes) {
        void* p = take(bytes);
        if (p && bytes) std::memcpy(p, src, bytes);
        return p;
    }
    // pinned landing block for a D2H copy whose bytes go to `user` when the chain finishes
    void* land(void* user, size_t bytes) {
        void* p = take(bytes);
        if (p) cur_outs_.push_back(Out{p, user, bytes});
        return p;
    }
    // Device memory for a call's counts (kernels write them), valid until the chain finishes:
    // land_dev() defers the copy to close(), where ONE D2H per device block carries every
    // count of the epoch -- no copy sits between the chain's kernels.
    void* dev_counts(size_t bytes) {
        bytes = (bytes + 255) & ~(size_t)255;
        std::lock_guard<std::mutex> g(mu_);
        if (cur_dev_ < 0 || devs_[cur_dev_].used + bytes > devs_[cur_dev_].cap) {
            int k = -1;
            for (size_t q = 0; q < devs_.size(); q++)
                if (!devs_[q].busy && devs_[q].cap >= bytes) {
                    k = (int)q;
                    break;
                }
            if (k < 0) {
                void* p = nullptr;
                const size_t cap = bytes < 65536 ? 65536 : bytes;
                if (hipMalloc(&p, cap) != hipSuccess) return nullptr;
                devs_.push_back(DevBlock{p, cap, 0, false});
                k = (int)devs_.size() - 1;
            }
            devs_[k].busy = true;
            devs_[k].used = 0;
            cur_devs_.push_back(k);
            cur_dev_ = k;
        }
        DevBlock& b = devs_[cur_dev_];
        void* p = (char*)b.p + b.used;
        b.used += bytes;
        return p;
    }
    void land_dev(void* user, const void* dev, size_t bytes) {
        std::lock_guard<std::mutex> g(mu_);
        cur_dev_outs_.push_back(DevOut{user, dev, bytes});
    }
    // close the current chain: record its end on `s`; *id = its epoch.  On a failure the
    // chain's blocks are released once the stream has drained (nothing queued still reads or
    // writes them) and the error is also reported by the next finish, so counts are never
    // dropped silently.
    int close(hipStream_t s, long long* id) {
        // the epoch's device count blocks: one D2H each into a pinned block, mapped to the users
        std::vector<int> devs;
        std::vector<DevOut> douts;
        std::vector<DevBlock> snap;   // devs_ may grow (dev_counts) once mu_ is released
        {
            std::lock_guard<std::mutex> g(mu_);
            devs.swap(cur_devs_);
            douts.swap(cur_dev_outs_);
            cur_dev_ = -1;
            for (int k : devs) snap.push_back(devs_[k]);
        }
        bool ok = true;
        std::vector<Out> mapped;
        for (const DevBlock& b : snap) {
            if (!b.used) continue;
            char* pin = (char*)take(b.used);
            if (!pin || hipMemcpyAsync(pin, b.p, b.used, hipMemcpyDeviceToHost, s) != hipSuccess) {
                ok = false;
                break;
            }
            for (const DevOut& o : douts)
                if ((const char*)o.dev >= (const char*)b.p && (const char*)o.dev < (const char*)b.p + b.cap)
                    mapped.push_back(Out{pin + ((const char*)o.dev - (const char*)b.p), o.user, o.bytes});
        }
        std::lock_guard<std::mutex> g(mu_);
        size_t k = 0;
        if (ok) {
            while (k < events_.size() && (events_[k].live || events_[k].waiters > 0)) k++;
            if (k == events_.size()) {
                events_.push_back(Ev{});
                ok = hipEventCreateWithFlags(&events_[k].ev, hipEventDisableTiming) == hipSuccess;
            }
            ok = ok && hipEventRecord(events_[k].ev, s) == hipSuccess;
        }
        if (!ok) {
            fprintf(stderr, "[orbslam_gpu] deferred chain: closing the epoch failed; its counts are lost\n");
            (void)hipStreamSynchronize(s);
            for (int d : devs) devs_[d].busy = false;
            for (int b : cur_blocks_) blocks_[b].busy = false;
            cur_blocks_.clear();
            cur_outs_.clear();
            failed_ = true;
            return -2;
        }
        for (auto& o : mapped) cur_outs_.push_back(o);
        events_[k].live = true;
        const long long e = next_id_++;
        closed_.push_back(Epoch{e, (int)k, std::move(cur_blocks_), std::move(cur_outs_), std::move(devs)});
        cur_blocks_.clear();
        cur_outs_.clear();
        if (id) *id = e;
        return 0;
    }
    // host wait for epoch `id` to complete on the device (no landing); any thread
    int wait(long long id) {
        int k = -1;
        hipEvent_t ev = nullptr;
        {
            std::lock_guard<std::mutex> g(mu_);
            for (const Epoch& ep : closed_)
                if (ep.id == id) k = ep.ev;
            if (k < 0) return 0;   // finished already (or never closed)
            events_[k].waiters++;
            ev = events_[k].ev;
        }
        const hipError_t rc = hipEventSynchronize(ev);
        std::lock_guard<std::mutex> g(mu_);
        events_[k].waiters--;
        return rc == hipSuccess ? 0 : -2;
    }
    // finish every closed epoch up to `id`, in order.  An epoch stays in closed_ until its
    // event has completed, so wait() from another thread never returns early.
    int finish_upto(long long id) {
        std::lock_guard<std::mutex> fg(finish_mu_);
        for (;;) {
            int k;
            hipEvent_t ev;
            {
                std::lock_guard<std::mutex> g(mu_);
                if (failed_) {   // an earlier close() lost its epoch
                    failed_ = false;
                    return -2;
                }
                if (closed_.empty() || closed_.front().id > id) return 0;
                k = closed_.front().ev;
                events_[k].waiters++;
                ev = events_[k].ev;
            }
            const hipError_t rc = hipEventSynchronize(ev);
            Epoch ep;
            {
                std::lock_guard<std::mutex> g(mu_);
                events_[k].waiters--;
                if (rc != hipSuccess) return -2;
                ep = std::move(closed_.front());
                closed_.pop_front();
                events_[k].live = false;
            }
            for (auto& o : ep.outs) std::memcpy(o.user, o.pin, o.bytes);
            std::lock_guard<std::mutex> g(mu_);
            for (int b : ep.blocks) blocks_[b].busy = false;
            for (int b : ep.devs) devs_[b].busy = false;
            done_id_ = ep.id;
        }
    }
    // close the current chain and finish everything
    int finish(hipStream_t s) {
        long long id = 0;
        if (int e = close(s, &id)) return e;
        return finish_upto(id);
    }

private:
    struct Block {
        void* p;
        size_t cap;
        bool busy;
    };
    struct Out {
        void* pin;
        void* user;
        size_t bytes;
    };
    struct Epoch {
        long long id;
        int ev;   // index into events_
        std::vector<int> blocks;
        std::vector<Out> outs;
        std::vector<int> devs;   // device count blocks
    };
    struct DevBlock {
        void* p;
        size_t cap, used;
        bool busy;
    };
    struct DevOut {
        void* user;
        const void* dev;
        size_t bytes;
    };
    struct Ev {
        hipEvent_t ev = nullptr;
        bool live = false;   // recorded for an epoch not finished yet
        int waiters = 0;     // host threads inside hipEventSynchronize on it
    };
    void* take(size_t bytes) {
        bytes = (bytes + 255) & ~(size_t)255;
        std::lock_guard<std::mutex> g(mu_);
        for (size_t k = 0; k < blocks_.size(); k++)
            if (!blocks_[k].busy && blocks_[k].cap >= bytes) {
                blocks_[k].busy = true;
                cur_blocks_.push_back((int)k);
                return blocks_[k].p;
            }
        void* p = nullptr;
        const size_t cap = bytes < 65536 ? 65536 : bytes;
        if (hipHostMalloc(&p, cap) != hipSuccess) return nullptr;
        blocks_.push_back(Block{p, cap, true});
        cur_blocks_.push_back((int)blocks_.size() - 1);
        return p;
    }
    bool on_ = false;
    std::mutex mu_;
    std::mutex finish_mu_;   // one finisher at a time (epochs finish in order)
    std::vector<Block> blocks_;
    std::vector<int> cur_blocks_;
    std::vector<Out> cur_outs_;
    std::deque<Epoch> closed_;
    std::vector<Ev> events_;
    std::vector<DevBlock> devs_;
    std::vector<int> cur_devs_;
    std::vector<DevOut> cur_dev_outs_;
    int cur_dev_ = -1;
    long long next_id_ = 1, done_id_ = 0;
    bool failed_ = false;
};

constexpr int kEdge = 19;          // EDGE_THRESHOLD, ORBextractor.cc:67
constexpr int kPatch = 31;         // PATCH_SIZE, ORBextractor.cc:65
constexpr int kHalfPatch = 15;     // HALF_PATCH_SIZE, ORBextractor.cc:66

// cvRound(float) == lrintf: round half to even.
__device__ __forceinline__ int cv_round(float v) { return __float2int_rn(v); }

// OpenCV 3.2 fastAtan2 (core/mathfuncs.cpp), degrees in [0, 360).
__device__ __forceinline__ float fast_atan2(float y, float x) {
    const float k180 = (float)(180.0 / 3.14159265358979323846);
    const float p1 = 0.9997878412794807f * k180;
    const float p3 = -0.3258083974640975f * k180;
    const float p5 = 0.1555786518463281f * k180;
    const float p7 = -0.04432655554792128f * k180;
    const float eps = (float)2.220446049250313e-16;
    float ax = fabsf(x), ay = fabsf(y), a, c, c2;
    if (ax >= ay) {
        c = ay / (ax + eps);
        c2 = c * c;
        a = (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    } else {
        c = ax / (ay + eps);
        c2 = c * c;
        a = 90.f - (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    }
    if (x < 0) a = 180.f - a;
    if (y < 0) a = 360.f - a;
    return a;
}

// glibc 2.35 sinf/cosf restated in f64 (|x| < 120).  The reference computes
// `(float)cos(angle)` with std::cos(float) == glibc cosf (ORBextractor.cc:112);
// the restatement is exhaustively equal to host libm on [0, 2*pi].
struct SinCosTab {
    double sign[4], hpi_inv, hpi, c0, c1, c2, c3, c4, s1, s2, s3;
};
__device__ __forceinline__ const SinCosTab& sincos_tab(int i) {
    static constexpr SinCosTab T[2] = {
        {{1.0, -1.0, -1.0, 1.0}, 0x1.45F306DC9C883p+23, 0x1.921FB54442D18p0, 0x1p0,
         -0x1.ffffffd0c621cp-2, 0x1.55553e1068f19p-5, -0x1.6c087e89a359dp-10, 0x1.99343027bf8c3p-16,
         -0x1.555545995a603p-3, 0x1.1107605230bc4p-7, -0x1.994eb3774cf24p-13},
        {{1.0, -1.0, -1.0, 1.0}, 0x1.45F306DC9C883p+23, 0x1.921FB54442D18p0, -0x1p0,
         0x1.ffffffd0c621cp-2, -0x1.55553e1068f19p-5, 0x1.6c087e89a359dp-10, -0x1.99343027bf8c3p-16,
         -0x1.555545995a603p-3, 0x1.1107605230bc4p-7, -0x1.994eb3774cf24p-13}};
    return T[i];
}

__device__ __forceinline__ float sincos_poly(double x, double x2, const SinCosTab& p, int n) {
    if ((n & 1) == 0) {
        double x3 = x * x2;
        double s1 = p.s2 + x2 * p.s3;
        double x7 = x3 * x2;
        double s = x + x3 * p.s1;
        return (float)(s + x7 * s1);
    }
    double x4 = x2 * x2;
    double c2 = p.c3 + x2 * p.c4;
    double c1 = p.c0 + x2 * p.c1;
    double x6 = x4 * x2;
    double c = c1 + x4 * p.c2;
    return (float)(c + x6 * c2);
}

__device__ __forceinline__ uint32_t top12(float f) { return (__float_as_uint(f) >> 20) & 0x7ff; }

// Returns (sin, cos) of y exactly as glibc sinf(y), cosf(y).
__device__ __forceinline__ void glibc_sincosf(float y, float* s_out, float* c_out) {
    const uint32_t t = top12(y);
    if (t < top12(0x1.921FB6p-1f)) {
        double x = y, x2 = x * x;
        if (t < top12(0x1p-12f)) {
            *s_out = y;
            *c_out = 1.0f;
            return;
        }
        *s_out = sincos_poly(x, x2, sincos_tab(0), 0);
        *c_out = sincos_poly(x, x2, sincos_tab(0), 1);
        return;
    }
    double x = y;
    const SinCosTab& p0 = sincos_tab(0);
    double r = x * p0.hpi_inv;
    int n = ((int32_t)r + 0x800000) >> 24;
    x = x - n * p0.hpi;
    double s = p0.sign[n & 3];
    const SinCosTab& p = (n & 2) ? sincos_tab(1) : p0;
    *s_out = sincos_poly(x * s, x * x, p, n);
    *c_out = sincos_poly(x * s, x * x, p, n ^ 1);
}

__device__ __forceinline__ int refl101(int p, int len) {
    if (len == 1) return 0;
    while (p < 0 || p >= len) p = p < 0 ? -p : 2 * len - p - 2;
    return p;
}

__device__ __forceinline__ int wave_sum(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// Issue priority of a latency-critical wave over co-resident bulk waves on its SIMD.
#define ORBGPU_LATENCY_WAVE() __builtin_amdgcn_s_setprio(3)

// (problem, block) of a 1-D grid of gx blocks per problem.  With >= 8 problems the order is
// XCD-aware: workgroups L and L + 8 share an XCD (blocks are dealt round-robin over the 8 XCDs),
// so workgroup L takes problem (L % 8) + 8 (L / 8 / gx), block (L / 8) % gx, and every block of a
// problem runs on one XCD (its staged inputs are fetched into one L2).  Fewer problems would
// leave XCDs idle, so their blocks are spread over all of them.  Grid size: xcd_grid().
__device__ __forceinline__ bool xcd_problem_block(int np, int gx, int& by, int& bx) {
    if (np >= 8) {
        const int xcd = (int)(blockIdx.x & 7), slot = (int)(blockIdx.x >> 3);
        by = xcd + 8 * (slot / gx);
        bx = slot % gx;
    } else {
        by = (int)blockIdx.x / gx;
        bx = (int)blockIdx.x - by * gx;
    }
    return by < np;
}
inline dim3 xcd_grid(int gx, int np) { return dim3(np >= 8 ? 8 * gx * ((np + 7) / 8) : gx * np); }

// sum over the 64 lanes of a wave (every lane active), result in every lane
__device__ __forceinline__ unsigned long long wave_sum_u64(unsigned long long v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

}  // namespace orbgpu

// Section timers for instrumented builds (make prof -> -DORBGPU_PROF): clock64() deltas of
// workgroup 0 / thread 0 accumulated into g_orbgpu_prof[slot]; compiled out otherwise.
#ifdef ORBGPU_PROF
#ifndef ORBGPU_PROF_BLOCK
#define ORBGPU_PROF_BLOCK 0   // the workgroup whose sections are timed
#endif
static __device__ unsigned long long g_orbgpu_prof[32];   // one copy per translation unit
#define ORBGPU_PROF_START unsigned long long _orbgpu_pt = clock64()
#define ORBGPU_PROF_MARK(i)                                                                   \
    do {                                                                                      \
        if (blockIdx.x == ORBGPU_PROF_BLOCK && threadIdx.x == 0) {                            \
            const unsigned long long _t = clock64();                                          \
            atomicAdd(&g_orbgpu_prof[i], _t - _orbgpu_pt);                                    \
            _orbgpu_pt = _t;                                                                  \
        }                                                                                     \
    } while (0)
#define ORBGPU_PROF_COUNT(i)                                                                  \
    do {                                                                                      \
        if (blockIdx.x == ORBGPU_PROF_BLOCK && threadIdx.x == 0) atomicAdd(&g_orbgpu_prof[i], 1ull); \
    } while (0)
#else
#define ORBGPU_PROF_START
#define ORBGPU_PROF_MARK(i)
#define ORBGPU_PROF_COUNT(i)
#endif
