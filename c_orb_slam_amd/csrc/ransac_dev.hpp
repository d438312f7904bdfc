// ransac_dev.hpp -- the RANSAC sample stream on the device (PnPsolver::iterate,
// Sim3Solver::iterate; DUtils::Random::RandomInt over glibc rand(), Random.cpp:47-50).
//
// glibc's TYPE_3 generator is the additive lagged recurrence x[m] = x[m-31] + x[m-3] (mod 2^32)
// over its 31-word table, rand() = x[m] >> 1.  Unrolling the lag-3 term inside a block of 31:
//   x[n+i] = x[n-3+(i mod 3)] + sum_{k=0..i/3} x[n+i-31-3k]        (0 <= i < 31)
// so one wave produces 31 words per step from the previous 31 (the window), a lane per word.
// RandomInt(0, d-1) = int(((double)r / 2^31) * d) is exact in double for d < 2^22 and equals
// (r * d) >> 31 in integers.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/orbslam_gpu.h"

namespace orbgpu {

constexpr int kRngMaxRange = 1 << 22;   // RandomInt ranges the integer form reproduces exactly

// raw[0..D) = the next D table words of stream g (x[n..n+D)); every lane of a 64-thread
// workgroup calls it; win: 32 u32 of LDS.  Only the words from `from` on are stored (a
// workgroup that draws hypotheses [h0, h1) regenerates the stream up to its own words).
__device__ __forceinline__ void rng_generate(const orb_rng& g, int D, uint32_t* raw, uint32_t* win, int from = 0) {
    const int lane = threadIdx.x & 63;
    if (lane < 31) {
        int s = g.f + lane;
        s = s >= 31 ? s - 31 : s;
        win[lane] = (uint32_t)g.tbl[s];
    }
    __syncthreads();
    for (int base = 0; base < D; base += 31) {
        uint32_t v = 0;
        if (lane < 31) {
            v = win[28 + lane % 3];
            for (int j = lane; j >= 0; j -= 3) v += win[j];
        }
        __syncthreads();
        if (lane < 31) {
            win[lane] = v;
            if (base + lane < D && base + lane >= from) raw[base + lane] = v;
        }
        __syncthreads();
    }
}

// The stream after consuming C of the D generated words: slot (f0 + j) mod 31 holds the last
// word written to it (draw j' = j + 31 q < C), f and r advance by C (mod 31).  Lane j < 31.
__device__ __forceinline__ void rng_after(const orb_rng& g, const uint32_t* raw, int C, orb_rng* out) {
    const int lane = threadIdx.x & 63;
    if (lane < 31) {
        int s = g.f + lane;
        s = s >= 31 ? s - 31 : s;
        int32_t v = g.tbl[s];
        if (C > lane) v = (int32_t)raw[lane + 31 * ((C - 1 - lane) / 31)];
        out->tbl[s] = v;
    }
    if (lane == 0) {
        out->f = (g.f + C) % 31;
        out->r = (g.r + C) % 31;
    }
}

// RandomInt(0, d - 1) from a table word (Random.cpp:47-50)
__device__ __forceinline__ int rng_pick(uint32_t word, int d) {
    return (int)(((uint64_t)(word >> 1) * (uint32_t)d) >> 31);
}

// One minimal set: vAvailableIndices = 0..N-1, MS draws with swap-remove (PnPsolver.cc:
// 189-201, Sim3Solver.cc:166-178).  The few swapped slots are kept as (position, value) pairs;
// a lookup takes the latest pair of its position.
template <int MS>
__device__ __forceinline__ void draw_set(const uint32_t* raw, int N, int* out) {
    int mp[MS], mv[MS];
#pragma unroll
    for (int i = 0; i < MS; i++) {
        const int navail = N - i;
        const int randi = rng_pick(raw[i], navail);
        int idx = randi, last = navail - 1;
#pragma unroll
        for (int j = 0; j < i; j++) {
            idx = mp[j] == randi ? mv[j] : idx;
            last = mp[j] == navail - 1 ? mv[j] : last;
        }
        out[i] = idx;
        mp[i] = randi;
        mv[i] = last;
    }
}
// the same for a run-time minimal-set size (<= 64)
__device__ __forceinline__ void draw_set_n(const uint32_t* raw, int N, int ms, int* out) {
    int mp[64], mv[64];
    for (int i = 0; i < ms; i++) {
        const int navail = N - i;
        const int randi = rng_pick(raw[i], navail);
        int idx = randi, last = navail - 1;
        for (int j = 0; j < i; j++) {
            idx = mp[j] == randi ? mv[j] : idx;
            last = mp[j] == navail - 1 ? mv[j] : last;
        }
        out[i] = idx;
        mp[i] = randi;
        mv[i] = last;
    }
}

// Wave-cooperative generation of K minimal sets of size ms over N correspondences from stream
// g: raw words into raw[0 .. K*ms), the sets into idx[0 .. K*ms).  64-thread workgroup.
__device__ __forceinline__ void draw_sets(const orb_rng& g, int K, int ms, int N, uint32_t* raw, int* idx,
                                          uint32_t* win) {
    rng_generate(g, K * ms, raw, win);
    __syncthreads();   // raw[] is read back by other lanes (global memory, same workgroup)
    for (int h = threadIdx.x; h < K; h += 64) {
        const uint32_t* rw = raw + (size_t)h * ms;
        int* o = idx + (size_t)h * ms;
        if (ms == 4) {
            int s[4];
            draw_set<4>(rw, N, s);
#pragma unroll
            for (int i = 0; i < 4; i++) o[i] = s[i];
        } else if (ms == 3) {
            int s[3];
            draw_set<3>(rw, N, s);
#pragma unroll
            for (int i = 0; i < 3; i++) o[i] = s[i];
        } else {
            int s[64];
            draw_set_n(rw, N, ms, s);
            for (int i = 0; i < ms; i++) o[i] = s[i];
        }
    }
}

// The minimal sets of hypotheses [h0, h1) of the call (h1 - h0 <= 64), inside the kernel that
// solves them: the stream up to word h1 * ms is regenerated by this workgroup (a few dozen
// 31-word steps), its own words stored, then lane h - h0 draws set h.  Every workgroup of a
// solver does this for its own range, so no separate draw launch precedes the solves; the
// replay reads the stored words back for the stream position.  64-thread workgroup (one wave:
// the raw words a lane stored are read by other lanes after the barrier).
__device__ __forceinline__ void draw_range(const orb_rng& g, int ms, int N, uint32_t* raw, int* idx, uint32_t* win,
                                           int h0, int h1) {
    rng_generate(g, h1 * ms, raw, win, h0 * ms);
    __syncthreads();
    const int h = h0 + (int)(threadIdx.x & 63);
    if (h >= h1) return;
    const uint32_t* rw = raw + (size_t)h * ms;
    int* o = idx + (size_t)h * ms;
    if (ms == 4) {
        int s[4];
        draw_set<4>(rw, N, s);
#pragma unroll
        for (int i = 0; i < 4; i++) o[i] = s[i];
    } else if (ms == 3) {
        int s[3];
        draw_set<3>(rw, N, s);
#pragma unroll
        for (int i = 0; i < 3; i++) o[i] = s[i];
    } else {
        int s[64];
        draw_set_n(rw, N, ms, s);
        for (int i = 0; i < ms; i++) o[i] = s[i];
    }
}

}  // namespace orbgpu
