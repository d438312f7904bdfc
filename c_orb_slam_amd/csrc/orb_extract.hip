// orb_extract.hip -- MI355X (gfx950) ORB extraction: the device side of
// ORBextractor::operator() (reference src/ORBextractor.cc:1043-1105).
//
// Pipeline per batch of B equal-size u8 images (all device-resident):
//   k_pyr_level0   copyMakeBorder(REFLECT_101, 19 px)            ORBextractor.cc:1126-1128
//   k_pyr_resize   resize(INTER_LINEAR, 8U fixed point) + border  ORBextractor.cc:1118-1123
//   k_blur7        GaussianBlur 7x7 sigma 2 (8-bit fixed point)    ORBextractor.cc:1085-1086
//   k_fast_cells   per-cell FAST(th=20) / FAST(th=7) + NMS, LDS-staged ROI,
//                  raster-order compaction                        ORBextractor.cc:776-829
//   k_octree       per (image, level): the level's candidates in cell order, then
//                  DistributeOctTree (order-defining)             ORBextractor.cc:539-763
//   k_orient_desc  IC_Angle + rotated BRIEF, one wave per keypoint ORBextractor.cc:77-147
//
// HBM layout: per image, the padded levels (pitch = align16(w+38)) are
// concatenated; the blurred levels use the identical geometry in a second
// buffer.  Cells of all levels are one flat launch (grid = cells x images).
#include "orb_extract.hpp"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstring>
#include <thread>

namespace orbgpu {

// ---------------------------------------------------------------- constants
__constant__ int8_t c_pattern[256 * 4];     // rBRIEF pairs (x0,y0,x1,y1)
__constant__ int8_t c_disc[2 * 1024];       // IC_Angle disc offsets (u, v)
__constant__ int c_ndisc;
__constant__ int c_umax[16];                // IC_Angle: half width d(|v|) of disc row v (d(0) = 15)
__constant__ int c_gauss[7];

static const int8_t kPattern[256 * 4] = {
#include "brief_pattern.inc"
};

// ------------------------------------------------------------------ kernels
// XCD-aware tile order: workgroups are dispatched round-robin over the 8 XCDs (linear id % 8),
// so with gridDim.x a multiple of 8 the XCD of block x is x % 8.  Give each XCD a contiguous
// run of tiles/cells, so the halos that neighbouring tiles share are re-read from that XCD's
// own L2 instead of being fetched again by a different XCD.
__device__ __forceinline__ int xcd_tile(int bid, int nb) { return (bid & 7) * (nb >> 3) + (bid >> 3); }
static inline unsigned grid8(int n) { return (unsigned)((n + 7) & ~7); }
// opt-in ORBGPU_FAST_SPLIT=1: FAST of levels 0-2 (70 % of the pixels) on a side stream, beside the
// build of levels 3-7 (1.505 -> 1.483 ms per 128-image call alone, no gain in the pipeline:
// profiles/r04t_fast_split_ab.txt)
constexpr int kFastSplitLevel = 3;

// copyMakeBorder(image, temp, 19,19,19,19, BORDER_REFLECT_101), 16 bytes/thread.
// Interior chunks: the (arbitrarily aligned) source row is read as aligned dwords and
// realigned with v_alignbyte; the two border chunks of a row reflect byte by byte.
// The 16 bytes of padded row py at padded column px0 of one image (src: its first row)
__device__ __forceinline__ uint4 pyr_l0_chunk(const uint8_t* __restrict__ src, int step, int W, int H, int py, int px0) {
    const int sy = refl101(py - kEdge, H);
    const uint8_t* srow = src + (size_t)sy * step;
    const int x0 = px0 - kEdge;
    uint4 o;
    if (x0 >= 0 && x0 + 15 < W) {
        const uintptr_t a = (uintptr_t)(srow + x0);
        const uint32_t* a32 = reinterpret_cast<const uint32_t*>(a & ~(uintptr_t)3);
        const uint32_t sh = (uint32_t)(a & 3);
        const uint32_t w0 = a32[0], w1 = a32[1], w2 = a32[2], w3 = a32[3];
        const uint32_t w4 = sh ? a32[4] : 0u;   // only when the 16 bytes straddle a 5th dword
        o.x = __builtin_amdgcn_alignbyte(w1, w0, sh);
        o.y = __builtin_amdgcn_alignbyte(w2, w1, sh);
        o.z = __builtin_amdgcn_alignbyte(w3, w2, sh);
        o.w = __builtin_amdgcn_alignbyte(w4, w3, sh);
    } else {
        uint32_t v[4] = {0, 0, 0, 0};
#pragma unroll
        for (int k = 0; k < 16; k++) v[k >> 2] |= (uint32_t)srow[refl101(x0 + k, W)] << (8 * (k & 3));
        o = make_uint4(v[0], v[1], v[2], v[3]);
    }
    return o;
}

__global__ void __launch_bounds__(256) k_pyr_level0(const uint8_t* __restrict__ src, size_t src_stride, int step,
                                                    int W, int H, uint8_t* __restrict__ pyr, size_t img_bytes,
                                                    int pitch, int ph, int* __restrict__ zero0,
                                                    int* __restrict__ zero1) {
    const int b = blockIdx.y;
    // the call's two counters (k_octree's corner total, the octree's error bits), cleared by
    // the first kernel of the stream instead of two fill launches before their users
    if (blockIdx.x == 0 && b == 0 && threadIdx.x == 0) {
        *zero0 = 0;
        *zero1 = 0;
    }
    const int chunks = pitch >> 4;
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= chunks * ph) return;
    const int py = t / chunks, px0 = (t - py * chunks) * 16;
    const uint4 o = pyr_l0_chunk(src + (size_t)b * src_stride, step, W, H, py, px0);
    *reinterpret_cast<uint4*>(pyr + (size_t)b * img_bytes + (size_t)py * pitch + px0) = o;
}

// resize(prev level, INTER_LINEAR) for CV_8U (OpenCV 3.2 imgwarp.cpp fixed
// point: 11-bit coefficients, VResizeLinear<uchar,int,short,FixedPtCast>),
// written straight into the padded level through the REFLECT_101 map.
// One workgroup per PT_W x nrow tile of the padded destination: the source rectangle the
// tile reads (host-computed, PyrTile) is staged into LDS as aligned dwords, then every
// thread forms 4 adjacent columns of every 4th row (coefficients of its columns held in
// registers) and stores dwords, a wave covering 256 contiguous bytes of a row.
// tile heights: 16 rows for small batches (more workgroups per image), 32 for large ones
// (fewer, longer workgroups: every staging load in flight at once)
constexpr int kPyrTileH[2] = {16, 32};
template <int TH>
constexpr int stage_regs() { return (((TH * 5 + 3) / 4 + 3) * ((PT_W * 5 / 4 + 12) / 4) + 255) / 256; }
// One tile of a level: the source rectangle staged (dword loads, all in flight), then 4 columns x
// every 4th row per thread.  WT: the output dwords stored write-through (sc1: handed to other
// workgroups of the same launch, k_pyr_flow); the stores are then drained by the caller.
typedef unsigned int u32x4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t slab_rsrc(uint8_t* p, size_t bytes) {
    const unsigned long long a = (unsigned long long)p;
    const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)a);
    const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(a >> 32));
    void* q = (void*)(((unsigned long long)hi << 32) | lo);
    return __builtin_amdgcn_make_buffer_rsrc(q, (short)0, (int)bytes, 0x00020000);
}
template <int TH, bool WT>
__device__ __forceinline__ void pyr_tile(uint8_t* __restrict__ base, size_t img_bytes, size_t src_off, int src_pitch,
                                         size_t dst_off, int dst_pitch, int w, int h, const int* __restrict__ xofs,
                                         const short2* __restrict__ xalpha, const int2* __restrict__ yrows,
                                         const short2* __restrict__ ybeta, const PyrTile& tl, uint32_t* s_src) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const uint32_t* S32 = reinterpret_cast<const uint32_t*>(base + src_off + (size_t)(kEdge + tl.sr0) * src_pitch + tl.sc0);
    const int spw = src_pitch >> 2;
    {
        // the source rectangle as dwords: every load of a thread in flight before its first LDS
        // store (stage_regs<TH>() per round; one round covers a TH x PT_W tile at scale <= 1.25)
        const int nw = tl.nsr * tl.nsw;
        for (int t0 = threadIdx.x; t0 < nw; t0 += 256 * stage_regs<TH>()) {
            uint32_t v[stage_regs<TH>()];
#pragma unroll
            for (int u = 0; u < stage_regs<TH>(); u++) {
                const int t = t0 + 256 * u;
                const int r = t / tl.nsw, c = t - r * tl.nsw;
                v[u] = t < nw ? S32[(size_t)r * spw + c] : 0u;
            }
#pragma unroll
            for (int u = 0; u < stage_regs<TH>(); u++)
                if (t0 + 256 * u < nw) s_src[t0 + 256 * u] = v[u];
        }
    }
    const int px = tl.px0 + 4 * lane;
    const bool col_ok = px < dst_pitch;
    int lx[4];
    short2 al[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int x = refl101(px + k - kEdge, w);
        lx[k] = col_ok ? xofs[x] + kEdge - tl.sc0 : 0;
        al[k] = col_ok ? xalpha[x] : make_short2(0, 0);
    }
    // this thread's rows (j = wid, wid+4, ... < nrow <= TH): row taps fetched before the barrier
    int2 rr[TH / 4];
    short2 bb[TH / 4];
#pragma unroll
    for (int i = 0; i < TH / 4; i++) {
        const int j = wid + 4 * i;
        const int y = refl101(tl.py0 + min(j, tl.nrow - 1) - kEdge, h);
        rr[i] = yrows[y];
        bb[i] = ybeta[y];
    }
    __syncthreads();
    if (!col_ok) return;
    const uint8_t* sb = reinterpret_cast<const uint8_t*>(s_src);
    const int rowb = tl.nsw * 4;
    __amdgpu_buffer_rsrc_t rs;
    if (WT) rs = slab_rsrc(base, img_bytes);
#pragma unroll
    for (int i = 0; i < TH / 4; i++) {
        const int j = wid + 4 * i;
        if (j >= tl.nrow) break;
        const int py = tl.py0 + j;
        const uint8_t* R0 = sb + (rr[i].x - tl.sr0) * rowb;
        const uint8_t* R1 = sb + (rr[i].y - tl.sr0) * rowb;
        const short2 bb_ = bb[i];
        uint32_t v = 0;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const int sx = lx[k];
            const short2 a = al[k];
            const int D0 = R0[sx] * a.x + R0[sx + (a.y != 0)] * a.y;
            const int D1 = R1[sx] * a.x + R1[sx + (a.y != 0)] * a.y;
            const int o = (((bb_.x * (D0 >> 4)) >> 16) + ((bb_.y * (D1 >> 4)) >> 16) + 2) >> 2;
            v |= (uint32_t)(uint8_t)o << (8 * k);
        }
        if (WT)
            __builtin_amdgcn_raw_buffer_store_b32(v, rs, (int)(dst_off + (size_t)py * dst_pitch + px), 0, 16);
        else
            *reinterpret_cast<uint32_t*>(base + dst_off + (size_t)py * dst_pitch + px) = v;
    }
}

template <int TH>
__global__ void __launch_bounds__(256) k_pyr_resize(uint8_t* __restrict__ pyr, size_t img_bytes, size_t src_off,
                                                    int src_pitch, size_t dst_off, int dst_pitch, int dst_ph, int w,
                                                    int h, const int* __restrict__ xofs,
                                                    const short2* __restrict__ xalpha, const int2* __restrict__ yrows,
                                                    const short2* __restrict__ ybeta,
                                                    const PyrTile* __restrict__ tiles, int ntiles) {
    extern __shared__ uint32_t s_src[];   // tl.nsr rows x tl.nsw dwords
    const int tile = xcd_tile(blockIdx.x, gridDim.x);
    if (tile >= ntiles) return;
    const PyrTile tl = tiles[tile];
    (void)dst_ph;
    pyr_tile<TH, false>(pyr + (size_t)blockIdx.y * img_bytes, img_bytes, src_off, src_pitch, dst_off, dst_pitch, w, h,
                        xofs, xalpha, yrows, ybeta, tl, s_src);
}

// The whole pyramid (the level-0 copy and every resize, ORBextractor.cc:1107-1132) as ONE launch
// of dependent tasks instead of a launch per level: tasks are numbered level by level (image-major
// inside a level), so every task a task waits for has a lower number and was dispatched before it
// (in-order dispatch per XCD: no wait can block its own producers).  Level 0: a band of th padded
// rows of one image; level l >= 1: one k_pyr_resize tile.  A level-l tile first waits for the
// bands of level l-1 that hold its source rows: one band counter per (image, level, band) counts
// its finished tasks (ncol per band; epoch * ncol once this call's are all in).  Hand-off
// (cdna_hip_programming.md §6 Guideline 16, R1): the rows are stored write-through (sc1), every
// wave drains its stores, the workgroup meets at a barrier, one lane adds to the band counter
// (agent scope); the consumer polls relaxed from one lane, then ONE agent-scope acquire (this
// CU's L1) before its plain staging loads.  Row pitches are multiples of 128 B and levels start
// on 256-B boundaries, so no cache line holds bytes of two rows: a line is never fetched before
// its row is complete.  Same per-pixel arithmetic (pyr_l0_chunk, pyr_tile): identical levels.
typedef __attribute__((address_space(1))) int g_i32;
__device__ __forceinline__ void flow_publish(int* cnt) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every storing wave: its sc1 stores done
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_fetch_add((g_i32*)cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// one lane: spin (bounded) until *cnt >= need; false on timeout
__device__ __forceinline__ bool flow_wait(int* cnt, int need) {
    for (int spins = 0; __hip_atomic_load((g_i32*)cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < need; spins++) {
        if (spins > (1 << 22)) return false;
        __builtin_amdgcn_s_sleep(2);
    }
    return true;
}
template <int TH>
__global__ void __launch_bounds__(256) k_pyr_flow(const uint8_t* __restrict__ src, size_t src_stride, int step, int W,
                                                  int H, uint8_t* __restrict__ pyr, size_t img_bytes, const FlowArgs A,
                                                  const PyrTile* __restrict__ tiles, const uint8_t* __restrict__ tabs,
                                                  int* __restrict__ cnt, int epoch, int* __restrict__ zero0,
                                                  int* __restrict__ err) {
    extern __shared__ uint32_t s_src[];
    const int t = blockIdx.x;
    int l = 0;
    while (l + 1 < A.nl && t >= A.L[l + 1].task0) l++;
    const FlowLevel& D = A.L[l];
    const int rel = t - D.task0, b = rel / D.ntiles, k = rel - b * D.ntiles;
    uint8_t* base = pyr + (size_t)b * img_bytes;
    int* cb = cnt + (size_t)b * A.nbands;
    if (l == 0) {
        // the call's counters, as k_pyr_level0 clears them (task 0 is dispatched first)
        if (t == 0 && threadIdx.x == 0) {
            *zero0 = 0;
            *err = 0;
        }
        const __amdgpu_buffer_rsrc_t rs = slab_rsrc(base, img_bytes);
        const int py0 = k * D.th, nr = min(D.th, D.ph - py0), chunks = D.pitch >> 4;
        const uint8_t* sb = src + (size_t)b * src_stride;
        for (int q = threadIdx.x; q < nr * chunks; q += 256) {
            const int r = q / chunks, py = py0 + r, px0 = (q - r * chunks) * 16;
            const uint4 o = pyr_l0_chunk(sb, step, W, H, py, px0);
            const u32x4v v = {o.x, o.y, o.z, o.w};
            __builtin_amdgcn_raw_buffer_store_b128(v, rs, (int)(D.off + (size_t)py * D.pitch + px0), 0, 16);
        }
        flow_publish(cb + D.band0 + k);
        return;
    }
    const PyrTile tl = tiles[D.tile0 + k];
    const FlowLevel& S = A.L[l - 1];
    if (threadIdx.x == 0) {
        const int r0 = kEdge + tl.sr0, r1 = kEdge + tl.sr0 + tl.nsr - 1;
        bool ok = true;
        for (int kb = r0 / S.th; kb <= r1 / S.th && ok; kb++) ok = flow_wait(cb + S.band0 + kb, epoch * S.ncol);
        if (!ok) atomicOr(err, 4);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    pyr_tile<TH, true>(base, img_bytes, S.off, S.pitch, D.off, D.pitch, D.w, D.h,
                       reinterpret_cast<const int*>(tabs + D.xofs), reinterpret_cast<const short2*>(tabs + D.xal),
                       reinterpret_cast<const int2*>(tabs + D.yr), reinterpret_cast<const short2*>(tabs + D.yb), tl,
                       s_src);
    flow_publish(cb + D.band0 + tl.py0 / D.th);
}

// The small pyramid levels [la, nlevels) in ONE launch (the tail of the chain of resizes,
// ORBextractor.cc:1107-1132, where a launch per level costs more than its pixels): workgroup
// (k, b) owns row strip k of every chained level of image b.  The strips of level l are the
// images of level l+1's strips under the row map (boundary A_l(k) = yrows_{l+1}[A_{l+1}(k)].x),
// so the rows a strip computes at level l are its own rows plus the few rows (the cone) that its
// level-(l+1) rows read beyond them, recomputed instead of exchanged.  Everything a workgroup
// reads is staged first, with all its loads in flight together: the source rows of level la-1
// (interior, from the padded level in HBM) and every chained level's row taps.  Per level: the
// strip's rows into an LDS buffer (ping-pong between two; the first level reads the staged
// source), then every padded row that reflects (REFLECT_101) to one of its own rows is written
// out, 16 bytes a thread.  A thread keeps the column taps of its 4 output columns in registers
// and walks rows.  Same fixed-point arithmetic per pixel as k_pyr_resize: identical levels.
__global__ void __launch_bounds__(256) k_pyr_chain(uint8_t* __restrict__ pyr, size_t img_bytes, long long src_off,
                                                   int src_pitch, int src_w, const ChainLevel* __restrict__ lv, int nl,
                                                   const int4* __restrict__ strips, const uint16_t* __restrict__ rows,
                                                   const uint8_t* __restrict__ tabs, int src_lds, int src_rp) {
    extern __shared__ uint32_t s_chain[];
    uint8_t* sb = reinterpret_cast<uint8_t*>(s_chain);
    const int k = blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
    uint8_t* base = pyr + (size_t)b * img_bytes;
    const int4 sr = strips[k * (nl + 1) + nl];   // source rows [x, y) of level la-1; row-tap slots at z
    {
        // source rows: padded columns [16, 16 + src_rp) as dwords (interior column c at byte c + 3)
        const uint32_t* S32 = reinterpret_cast<const uint32_t*>(base + src_off + (size_t)(kEdge + sr.x) * src_pitch + 16);
        const int wpr = src_rp >> 2, nsr = sr.y - sr.x, spw = src_pitch >> 2;
        uint32_t* d = s_chain + (src_lds >> 2);
        for (int t = tid; t < nsr * wpr; t += 256) {
            const int r = t / wpr, q = t - r * wpr;
            d[t] = S32[(size_t)r * spw + q];
        }
        // row taps of every chained level's compute rows: (y0 | y1 << 16, beta pair), and the
        // padded rows every level writes out
        int2* rt = reinterpret_cast<int2*>(sb + sr.z);
        uint16_t* rl = reinterpret_cast<uint16_t*>(sb + sr.w);
        int slot = 0, rslot = 0;
        for (int i = 0; i < nl; i++) {
            const int4 st = strips[k * (nl + 1) + i];
            const int2* yr = reinterpret_cast<const int2*>(tabs + lv[i].yr);
            const int* yb = reinterpret_cast<const int*>(tabs + lv[i].yb);
            for (int t = tid; t < st.y - st.x; t += 256) {
                const int2 yy = yr[st.x + t];
                rt[slot + t] = make_int2(yy.x | (yy.y << 16), yb[st.x + t]);
            }
            for (int t = tid; t < st.w; t += 256) rl[rslot + t] = rows[st.z + t];
            slot += st.y - st.x;
            rslot += st.w;
        }
    }
    __syncthreads();
    const uint8_t* prev = sb + src_lds + 3;   // interior column 0 of the staged source
    int prev_lo = sr.x, prev_rp = src_rp, prev_n = sr.y - sr.x;
    const int2* rt = reinterpret_cast<const int2*>(sb + sr.z);
    const uint16_t* rl = reinterpret_cast<const uint16_t*>(sb + sr.w);
    for (int i = 0; i < nl; i++) {
        const ChainLevel L = lv[i];
        const int4 st = strips[k * (nl + 1) + i];   // compute rows [x, y), padded-row list [z, z + w)
        const int nrows = st.y - st.x, ngr = (L.w + 3) >> 2, nph = L.nph;
        uint8_t* cur = sb + L.lds;
        if (tid < nph * ngr) {
            const int ph = tid / ngr, g = tid - ph * ngr;
            const int* xofs = reinterpret_cast<const int*>(tabs + L.xofs);
            const short2* xal = reinterpret_cast<const short2*>(tabs + L.xal);
            int sx[4], s1[4];
            short2 al[4];
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const int dx = min(4 * g + j, L.w - 1);
                sx[j] = xofs[dx];
                al[j] = xal[dx];
                s1[j] = sx[j] + (al[j].y != 0);
            }
            // one output dword (4 columns) of row r
            auto row_out = [&](int r) {
                const int2 e = rt[r];
                const int y0 = e.x & 0xffff, y1 = e.x >> 16;
                const short2 be = __builtin_bit_cast(short2, e.y);
                // rows of the previous level's buffer (inside its cone by construction)
                const uint8_t* R0 = prev + min(max(y0 - prev_lo, 0), prev_n - 1) * prev_rp;
                const uint8_t* R1 = prev + min(max(y1 - prev_lo, 0), prev_n - 1) * prev_rp;
                uint32_t v = 0;
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    if (4 * g + j < L.w) {
                        const short2 a = al[j];
                        const int D0 = R0[sx[j]] * a.x + R0[s1[j]] * a.y;
                        const int D1 = R1[sx[j]] * a.x + R1[s1[j]] * a.y;
                        const int o = (((be.x * (D0 >> 4)) >> 16) + ((be.y * (D1 >> 4)) >> 16) + 2) >> 2;
                        v |= (uint32_t)(uint8_t)o << (8 * j);
                    }
                }
                return v;
            };
            // two rows per step: their LDS reads are independent and in flight together
            for (int r = ph; r < nrows; r += 2 * nph) {
                const int r2 = r + nph < nrows ? r + nph : r;
                const uint32_t va = row_out(r), vb = row_out(r2);
                *reinterpret_cast<uint32_t*>(cur + r * L.rp + 4 * g) = va;
                *reinterpret_cast<uint32_t*>(cur + r2 * L.rp + 4 * g) = vb;
            }
        }
        rt += nrows;
        __syncthreads();
        // the padded rows of this strip: row py is interior row refl101(py - 19, h)
        const int nch = L.pitch >> 4;
        for (int t = tid; t < st.w * nch; t += 256) {
            const int ri = t / nch, ch = t - ri * nch;
            const int py = rl[ri];
            const int y = refl101(py - kEdge, L.h);
            const uint8_t* row = cur + min(max(y - st.x, 0), nrows - 1) * L.rp;
            const int x0 = ch * 16 - kEdge;   // = 1 (mod 4)
            uint4 o;
            if (x0 >= 1 && x0 + 16 <= L.w) {
                const uint32_t* w = reinterpret_cast<const uint32_t*>(row + x0 - 1);
                const uint32_t w0 = w[0], w1 = w[1], w2 = w[2], w3 = w[3], w4 = w[4];
                o.x = __builtin_amdgcn_alignbyte(w1, w0, 1);
                o.y = __builtin_amdgcn_alignbyte(w2, w1, 1);
                o.z = __builtin_amdgcn_alignbyte(w3, w2, 1);
                o.w = __builtin_amdgcn_alignbyte(w4, w3, 1);
            } else {
                uint32_t q[4] = {0, 0, 0, 0};
#pragma unroll
                for (int j = 0; j < 16; j++) q[j >> 2] |= (uint32_t)row[refl101(x0 + j, L.w)] << (8 * (j & 3));
                o = make_uint4(q[0], q[1], q[2], q[3]);
            }
            *reinterpret_cast<uint4*>(base + L.off + (size_t)py * L.pitch + 16 * ch) = o;
        }
        rl += st.w;
        prev = cur;
        prev_lo = st.x;
        prev_rp = L.rp;
        prev_n = nrows;
    }
    (void)src_w;
}

// GaussianBlur(7x7, sigma 2, REFLECT_101) on CV_8U: int taps (round(k*256)),
// int row pass, int column pass, (v + 2^15) >> 16, saturate.  The padded
// level's 19-px REFLECT_101 border supplies the filter border.  Tile 128x32,
// dword LDS staging (the padded row is dword-aligned at interior x0-3), dword
// stores into the unpadded blurred level.  Every sum is an exact integer sum, so
// the order of the terms is free (the result is the reference's bit for bit):
//   row pass     two v_dot4_u32_u8 per output pixel on the byte window (v_alignbyte
//                realigns it), for two staged rows at once; a row sum is <= 255 * 256,
//                so the sums of rows r, r+1 at one column pack into one dword (u16 pair)
//   column pass  four v_dot2_u32_u16 per output pixel on those row pairs: output row
//                2p reads pairs (2p, 2p+1) .. (2p+6, 2p+7) with taps (t0,t1) .. (t6,0),
//                output row 2p+1 the same pairs with taps (0,t0), (t1,t2) .. (t5,t6)
constexpr int BT_W = 128, BT_H = 32, BT_LW = BT_W + 8;  // staged cols: interior [x0-3, x0+133)
typedef unsigned short ushort2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t dot2u(uint32_t pair, uint32_t taps, uint32_t acc) {
    return __builtin_amdgcn_udot2(__builtin_bit_cast(ushort2v, pair), __builtin_bit_cast(ushort2v, taps), acc, false);
}
__global__ void __launch_bounds__(256) k_blur7(const uint8_t* __restrict__ pyr, uint8_t* __restrict__ blur,
                                               size_t img_bytes, size_t blur_bytes,
                                               const BlurTile* __restrict__ tiles, int ntiles) {
    constexpr int WPR = BT_LW / 4;          // words per staged row
    constexpr int SR = BT_H + 6;            // staged rows (38: 19 row pairs)
    __shared__ uint32_t s_src[SR * WPR];
    __shared__ uint4 s_pair[(SR / 2) * (BT_W / 4)];   // [pair][4-px group]: 4 packed (r, r+1) sums
    const int tile = xcd_tile(blockIdx.x, gridDim.x);
    if (tile >= ntiles) return;
    const BlurTile tl = tiles[tile];
    const int b = blockIdx.y;
    const uint8_t* P = pyr + (size_t)b * img_bytes + tl.off;           // padded level base
    uint8_t* O = blur + (size_t)b * blur_bytes + tl.boff;               // unpadded blurred level
    const int x0 = tl.tx * BT_W, y0 = tl.ty * BT_H;
    {
        // every staging load of a thread in flight before its first LDS store
        constexpr int NU = (SR * WPR + 255) / 256;
        uint32_t v[NU];
#pragma unroll
        for (int u = 0; u < NU; u++) {
            const int i = threadIdx.x + 256 * u;
            const int r = i / WPR, wq = i - r * WPR;
            const int yy = min(y0 + r - 3, tl.h + 2) + kEdge;                 // padded row
            const int c = min(kEdge - 3 + x0 + 4 * wq, tl.pitch - 4);           // padded col (dword aligned)
            v[u] = i < SR * WPR ? *reinterpret_cast<const uint32_t*>(P + (size_t)yy * tl.pitch + c) : 0u;
        }
#pragma unroll
        for (int u = 0; u < NU; u++)
            if (threadIdx.x + 256 * u < SR * WPR) s_src[threadIdx.x + 256 * u] = v[u];
    }
    const uint32_t TLO = (uint32_t)c_gauss[0] | ((uint32_t)c_gauss[1] << 8) | ((uint32_t)c_gauss[2] << 16) |
                         ((uint32_t)c_gauss[3] << 24);
    const uint32_t THI = (uint32_t)c_gauss[4] | ((uint32_t)c_gauss[5] << 8) | ((uint32_t)c_gauss[6] << 16);
    __syncthreads();
    for (int i = threadIdx.x; i < (SR / 2) * (BT_W / 4); i += 256) {
        const int pr = i / (BT_W / 4), q = i - pr * (BT_W / 4);
        uint32_t o[4];
#pragma unroll
        for (int h = 0; h < 2; h++) {
            const uint32_t* w = s_src + (2 * pr + h) * WPR + q;
            const uint32_t w0 = w[0], w1 = w[1], w2 = w[2];
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const uint32_t lo = j ? __builtin_amdgcn_alignbyte(w1, w0, j) : w0;
                const uint32_t hi = j ? __builtin_amdgcn_alignbyte(w2, w1, j) : w1;
                const uint32_t r = __builtin_amdgcn_udot4(lo, TLO, __builtin_amdgcn_udot4(hi, THI, 0u, false), false);
                o[j] = h ? (o[j] | (r << 16)) : r;
            }
        }
        s_pair[i] = make_uint4(o[0], o[1], o[2], o[3]);
    }
    // column taps as u16 pairs
    const uint32_t C01 = (uint32_t)c_gauss[0] | ((uint32_t)c_gauss[1] << 16);
    const uint32_t C23 = (uint32_t)c_gauss[2] | ((uint32_t)c_gauss[3] << 16);
    const uint32_t C45 = (uint32_t)c_gauss[4] | ((uint32_t)c_gauss[5] << 16);
    const uint32_t C6_ = (uint32_t)c_gauss[6];
    const uint32_t C_0 = (uint32_t)c_gauss[0] << 16;
    const uint32_t C12 = (uint32_t)c_gauss[1] | ((uint32_t)c_gauss[2] << 16);
    const uint32_t C34 = (uint32_t)c_gauss[3] | ((uint32_t)c_gauss[4] << 16);
    const uint32_t C56 = (uint32_t)c_gauss[5] | ((uint32_t)c_gauss[6] << 16);
    __syncthreads();
    for (int i = threadIdx.x; i < (BT_H / 2) * (BT_W / 4); i += 256) {
        const int p = i / (BT_W / 4), q = i - p * (BT_W / 4);
        const int y = y0 + 2 * p, x = x0 + 4 * q;
        if (y >= tl.h || x >= tl.w) continue;
        const uint4 a = s_pair[(p + 0) * (BT_W / 4) + q], bq = s_pair[(p + 1) * (BT_W / 4) + q];
        const uint4 c = s_pair[(p + 2) * (BT_W / 4) + q], d = s_pair[(p + 3) * (BT_W / 4) + q];
        const uint32_t A[4] = {a.x, a.y, a.z, a.w}, B[4] = {bq.x, bq.y, bq.z, bq.w};
        const uint32_t Cc[4] = {c.x, c.y, c.z, c.w}, D[4] = {d.x, d.y, d.z, d.w};
        uint32_t ev = 0, od = 0;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const uint32_t se = dot2u(D[j], C6_, dot2u(Cc[j], C45, dot2u(B[j], C23, dot2u(A[j], C01, 0u))));
            const uint32_t so = dot2u(D[j], C56, dot2u(Cc[j], C34, dot2u(B[j], C12, dot2u(A[j], C_0, 0u))));
            // every term is >= 0, so saturate_cast<uchar> is an unsigned min
            ev |= min((se + (1u << 15)) >> 16, 255u) << (8 * j);
            od |= min((so + (1u << 15)) >> 16, 255u) << (8 * j);
        }
        *reinterpret_cast<uint32_t*>(O + (size_t)y * tl.bpitch + x) = ev;
        if (y + 1 < tl.h) *reinterpret_cast<uint32_t*>(O + (size_t)(y + 1) * tl.bpitch + x) = od;
    }
}

__device__ __forceinline__ int min3(int a, int b, int c) { return min(min(a, b), c); }
__device__ __forceinline__ int max3(int a, int b, int c) { return max(max(a, b), c); }

// FAST-9/16 score S = max(A,B)-1 (OpenCV cornerScore<16>): A/B = best
// contiguous-9 dark/bright contrast.  A pixel is a corner at threshold t
// iff S >= t, and its stored score is then S (see oracle/ocv_semantics.c).
__device__ __forceinline__ int fast_score_lds(const uint8_t* p, int ld) {
    const int v = p[0];
    int d[16];
    d[0] = v - p[3 * ld];       d[1] = v - p[3 * ld + 1];   d[2] = v - p[2 * ld + 2];
    d[3] = v - p[ld + 3];       d[4] = v - p[3];            d[5] = v - p[-ld + 3];
    d[6] = v - p[-2 * ld + 2];  d[7] = v - p[-3 * ld + 1];  d[8] = v - p[-3 * ld];
    d[9] = v - p[-3 * ld - 1];  d[10] = v - p[-2 * ld - 2]; d[11] = v - p[-ld - 3];
    d[12] = v - p[-3];          d[13] = v - p[ld - 3];      d[14] = v - p[2 * ld - 2];
    d[15] = v - p[3 * ld - 1];
    int mn2[16], mx2[16];
#pragma unroll
    for (int k = 0; k < 16; k++) {
        mn2[k] = min(d[k], d[(k + 1) & 15]);
        mx2[k] = max(d[k], d[(k + 1) & 15]);
    }
    // arcs k and k+1 (k even) share d[k+1..k+8]: max over the pair of the arc minima is
    // min(shared minimum, max(d[k], d[k+9])) (and the mirrored form for the maxima), so the
    // 16 arcs cost 8 shared reductions
    int A = -1000, M = 1000;
#pragma unroll
    for (int k = 0; k < 16; k += 2) {
        const int smin = min(min3(mn2[(k + 1) & 15], mn2[(k + 3) & 15], mn2[(k + 5) & 15]), mn2[(k + 7) & 15]);
        const int smax = max(max3(mx2[(k + 1) & 15], mx2[(k + 3) & 15], mx2[(k + 5) & 15]), mx2[(k + 7) & 15]);
        A = max(A, min(smin, max(d[k], d[(k + 9) & 15])));
        M = min(M, max(smax, min(d[k], d[(k + 9) & 15])));
    }
    const int B = -M;
    return max(A, B) - 1;
}

constexpr int FC_LD = 76;      // LDS row pitch of the cell ROI (19 dwords: odd bank stride)
constexpr int FC_MAXR = 70;    // max ROI rows/cols supported (wCell/hCell <= 64)

// Necessary condition for FAST-9 at threshold t (S >= t): a 9-arc contains two consecutive
// compass points (0,4), (4,8), (8,12) or (12,0), all brighter than v+t or all darker than v-t.
__device__ __forceinline__ bool fast_pretest(const uint8_t* p, int ld, int t) {
    const int v = p[0];
    const int a = p[3 * ld], b = p[3], c = p[-3 * ld], d = p[-3];
    const bool da = v - a > t, db = v - b > t, dc = v - c > t, dd = v - d > t;
    const bool ba = a - v > t, bb = b - v > t, bc = c - v > t, bd = d - v > t;
    return (da && db) || (db && dc) || (dc && dd) || (dd && da) || (ba && bb) || (bb && bc) || (bc && bd) ||
           (bd && ba);
}

// The same test for two rows at once in packed 16-bit lanes (row A low half, row B high half):
// x darker than v by more than t <=> (v - (t+1)) - x >= 0, brighter <=> x - (v + (t+1)) >= 0,
// so the sign bits of the packed differences are the negated comparisons, and
// fail = !dark && !bright = ((na & nc) | (nb & nd)) & ((ba & bc) | (bb & bd)) on those bits.
// Bit 15 / bit 31 of the result set: row A / row B fails.
typedef short short2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ short2v pk16(int lo, int hi) {
    short2v r;
    r.x = (short)lo;
    r.y = (short)hi;
    return r;
}
__device__ __forceinline__ uint32_t pk_bits(short2v v) { return __builtin_bit_cast(uint32_t, v); }
__device__ __forceinline__ uint32_t fast_pretest2_fail(const uint8_t* pa, const uint8_t* pb, int ld, short2v T1) {
    const short2v v = pk16(pa[0], pb[0]);
    const short2v a = pk16(pa[3 * ld], pb[3 * ld]), b = pk16(pa[3], pb[3]);
    const short2v c = pk16(pa[-3 * ld], pb[-3 * ld]), d = pk16(pa[-3], pb[-3]);
    const short2v vm = v - T1, vp = v + T1;
    const uint32_t na = pk_bits(vm - a), nb = pk_bits(vm - b), nc = pk_bits(vm - c), nd = pk_bits(vm - d);
    const uint32_t ba = pk_bits(a - vp), bb = pk_bits(b - vp), bc = pk_bits(c - vp), bd = pk_bits(d - vp);
    return ((na & nc) | (nb & nd)) & ((ba & bc) | (bb & bd));
}

// Exclusive scan by wave 0 of the popcounts of masks[0..n) (n <= 64) into off[0..n], off[64] = total.
__device__ __forceinline__ void mask_scan64(const uint64_t* masks, int n, int* off, int lane) {
    const int cnt = lane < n ? (int)__popcll(masks[lane]) : 0;
    int incl = cnt;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(incl, o, 64);
        if (lane >= o) incl += y;
    }
    off[lane] = incl - cnt;
    if (lane == 63) off[64] = incl;
}

__device__ __forceinline__ int sel4(int k, int a0, int a1, int a2, int a3) {
    return k == 0 ? a0 : k == 1 ? a1 : k == 2 ? a2 : a3;
}

// One workgroup (4 waves) per (cell group, image): up to 2 x 2 cells whose ROIs tile one union
// ROI (CellGroup), so the staging, the syncs and the scans are shared by up to four cells.
// Every pixel loop is division-free.
//   stage    union ROI rows as aligned dwords into LDS (3 rows per wave instruction)
//   pretest  FAST-9 necessary condition at min(iniTh, minTh) per detection pixel: lanes over
//            the union's detection columns (<= 64), one ballot per detection row
//   list     survivors, ~10 % of the pixels, cell by cell (TL, TR, BL, BR) and raster order
//            inside a cell (row-count scans): cell k's are list entries [lb_k, lb_k+1)
//   score    OpenCV cornerScore<16> for the list only (pixels failing the pretest score < th)
//   NMS      per entry and for BOTH thresholds: keep = S >= th && S > every 8-neighbour's
//            (S >= th ? S : 0) <=> S >= th && S > every 8-neighbour's S (one local-maximum test
//            for both thresholds), a neighbour outside the entry's own cell counting 0 (the
//            reference runs FAST on each cell's ROI alone, ORBextractor.cc:794-829)
//   output   per cell: its iniTh keeps if it has any, else its minTh keeps (the retry of
//            ORBextractor.cc:810-815), compacted in list order into the cell's slots
__global__ void __launch_bounds__(256) k_fast_cells(const uint8_t* __restrict__ pyr, size_t img_bytes,
                                                    const CellGroup* __restrict__ groups, int iniTh, int minTh,
                                                    uint32_t* __restrict__ slots, size_t slots_per_image,
                                                    int* __restrict__ counts, int ncells,
                                                    const int* __restrict__ work) {
    __shared__ uint32_t s_img32[FC_MAXR * FC_LD / 4];
    __shared__ uint32_t s_sc32[FC_MAXR * FC_LD / 4];
    __shared__ uint16_t s_list[64 * 64];
    __shared__ uint64_t s_mask[64], s_khi[64];
    __shared__ int s_off[65], s_offR[64];
    __shared__ int s_lb[5];
    uint8_t* s_img = reinterpret_cast<uint8_t*>(s_img32);
    uint8_t* s_sc = reinterpret_cast<uint8_t*>(s_sc32);
    uint64_t* s_klo = reinterpret_cast<uint64_t*>(s_img32);   // the ROI is dead after scoring
    // work order (Extractor::build_work): workgroup g runs on XCD g % 8; whole group rows of an
    // image go to one XCD (rows dealt round-robin), so horizontally adjacent groups -- which
    // share ROI halo columns and 128-B lines -- hit that XCD's L2 instead of being fetched
    // once per XCD, while every XCD still gets the same mix of levels
    ORBGPU_PROF_START;
    const int wk = work[blockIdx.x];
    if (wk < 0) return;   // padding of a shorter XCD list
    const int gi = wk & 0xffff, b = wk >> 16;
    const CellGroup& g = groups[gi];
    const int rows = g.rows, cols = g.cols, rs = g.rsplit, cs = g.csplit;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int dr = max(rows - 6, 0), dc = max(cols - 6, 0);
    int* cnt_out = counts + (size_t)b * ncells;
    if (dr == 0 || dc == 0) {
        if (tid < 4 && g.cell[tid] >= 0) cnt_out[g.cell[tid]] = 0;
        return;
    }
    // ROI rows staged as realigned dwords: pixel (r, c) sits at LDS byte r*FC_LD + 1 + c, so the
    // detection columns 3 + j start on a dword (j = 0) and a lane's 4 columns are one LDS dword.
    // LDS dword w of a row holds the global bytes Q + 4w .. Q + 4w + 3 (Q = pixel (r, -1)), one
    // v_alignbyte of two aligned global dwords
    const uint8_t* Q = pyr + (size_t)b * img_bytes + g.lvl_off + (size_t)(kEdge + g.r0) * g.pitch + kEdge + g.c0 - 1;
    const int qmis = (int)((uintptr_t)Q & 3);
    const uint32_t* Q32 = reinterpret_cast<const uint32_t*>(Q - qmis);
    constexpr int ldw = FC_LD / 4;
    constexpr int mis = 1;
    const int wpr = (cols + 4) >> 2, pw = g.pitch >> 2;
    {
        // 3 rows x 19 dwords per wave instruction; rows wid*3 + rr + 12k (k < 6 covers FC_MAXR):
        // every load of the thread is issued before the first LDS store (one wait, not six)
        const int rr = lane / ldw, w = lane - rr * ldw;
        const bool ok = rr < 3 && w < wpr;
        const uint32_t* gp = Q32 + (size_t)(wid * 3 + rr) * pw + w;
        uint32_t v[6], v1[6];
#pragma unroll
        for (int k = 0; k < 6; k++) {
            const int r = wid * 3 + rr + 12 * k;
            const bool on = ok && r < rows;
            v[k] = on ? gp[(size_t)12 * k * pw] : 0u;
            v1[k] = on ? gp[(size_t)12 * k * pw + 1] : 0u;
        }
#pragma unroll
        for (int k = 0; k < 6; k++) {
            const int r = wid * 3 + rr + 12 * k;
            if (ok && r < rows) s_img32[r * ldw + w] = __builtin_amdgcn_alignbyte(v1[k], v[k], qmis);
        }
    }
    for (int i = tid; i < rows * ldw; i += 256) s_sc32[i] = 0u;
    __syncthreads();
    ORBGPU_PROF_MARK(0);
    const int tp = min(iniTh, minTh);
    // detection columns on the lanes (dc <= 64: the union ROI is <= FC_MAXR wide), detection rows
    // over the waves; row i's survivor mask is one ballot, its left-cell bits the low cs bits
    const uint64_t Lm = cs >= 64 ? ~0ull : ((1ull << cs) - 1ull);
    if (tp < 1) {
        for (int i = wid; i < dr; i += 4) {
            const uint64_t m = __ballot(lane < dc);
            if (lane == 0) s_mask[i] = m;
        }
    } else {
        // 4 detection columns per lane, 16 lanes per row, 4 rows per wave pass (16 per pass): a
        // lane's pixels are one LDS dword (v), its compass points the dwords 3 rows up / down and
        // the neighbouring dwords realigned by 3 bytes (v_alignbyte); two packed 16-bit tests
        // cover the 4 pixels, and the row's 64-bit survivor mask is assembled from the lanes'
        // nibbles by three DPP ORs within each group of 8 lanes
        const short2v T1 = pk16(tp + 1, tp + 1);
        const int rho = lane >> 4, L = lane & 15;
        uint32_t* m32 = reinterpret_cast<uint32_t*>(s_mask);
        const int cv = dc - 4 * L;
        const uint32_t colmask = cv >= 4 ? 0xfu : (cv > 0 ? (1u << cv) - 1u : 0u);
        for (int i0 = 4 * wid; i0 < dr; i0 += 16) {
            const int i = i0 + rho;
            const int ic = min(i, dr - 1);   // rows past the last detection row: computed, not stored
            const uint32_t* rw = s_img32 + (3 + ic) * ldw + L;
            const uint32_t pv = rw[0], vv = rw[1], nv = rw[2];
            const uint32_t av = rw[3 * ldw + 1], cvv = rw[-3 * ldw + 1];
            const uint32_t bv = __builtin_amdgcn_alignbyte(nv, vv, 3), dv = __builtin_amdgcn_alignbyte(vv, pv, 1);
            uint32_t fl[2];
#pragma unroll
            for (int h = 0; h < 2; h++) {
                const uint32_t sel = h ? 0x0c030c02u : 0x0c010c00u;
                const short2v v = __builtin_bit_cast(short2v, __builtin_amdgcn_perm(0u, vv, sel));
                const short2v a = __builtin_bit_cast(short2v, __builtin_amdgcn_perm(0u, av, sel));
                const short2v bq = __builtin_bit_cast(short2v, __builtin_amdgcn_perm(0u, bv, sel));
                const short2v c = __builtin_bit_cast(short2v, __builtin_amdgcn_perm(0u, cvv, sel));
                const short2v d = __builtin_bit_cast(short2v, __builtin_amdgcn_perm(0u, dv, sel));
                const short2v vm = v - T1, vp = v + T1;
                const uint32_t na = pk_bits(vm - a), nb = pk_bits(vm - bq), nc = pk_bits(vm - c), nd = pk_bits(vm - d);
                const uint32_t ba = pk_bits(a - vp), bb = pk_bits(bq - vp), bc = pk_bits(c - vp), bd = pk_bits(d - vp);
                fl[h] = ((na & nc) | (nb & nd)) & ((ba & bc) | (bb & bd));
            }
            const uint32_t nib = (((~fl[0] >> 15) & 1u) | ((~fl[0] >> 30) & 2u) | ((~fl[1] >> 13) & 4u) |
                                  ((~fl[1] >> 28) & 8u)) & colmask;
            int x = (int)(nib << (4 * (L & 7)));
            x |= __builtin_amdgcn_mov_dpp(x, 0xB1, 0xf, 0xf, true);    // quad_perm xor 1
            x |= __builtin_amdgcn_mov_dpp(x, 0x4E, 0xf, 0xf, true);    // quad_perm xor 2
            x |= __builtin_amdgcn_mov_dpp(x, 0x141, 0xf, 0xf, true);   // row_half_mirror (8 lanes)
            if ((L & 7) == 0 && i < dr) m32[2 * i + (L >> 3)] = (uint32_t)x;
        }
    }
    __syncthreads();
    ORBGPU_PROF_MARK(1);
    // wave 0, lane = detection row: the list holds the TL cell's survivors in raster order, then
    // TR's, BL's, BR's; row i's left (right) run starts at s_off[i] (s_offR[i])
    if (wid == 0) {
        const uint64_t m = lane < dr ? s_mask[lane] : 0ull;
        const int cl = (int)__popcll(m & Lm), cr = (int)__popcll(m & ~Lm);
        int il = cl, ir = cr;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int yl = __shfl_up(il, o, 64), yr = __shfl_up(ir, o, 64);
            if (lane >= o) { il += yl; ir += yr; }
        }
        const int topL = rs > 0 ? __shfl(il, rs - 1, 64) : 0, topR = rs > 0 ? __shfl(ir, rs - 1, 64) : 0;
        const int allL = __shfl(il, 63, 64), allR = __shfl(ir, 63, 64);
        const int el = il - cl, er = ir - cr;
        const bool bot = lane >= rs;
        s_off[lane] = bot ? topR + el : el;
        s_offR[lane] = bot ? allL + er : topL + er;
        if (lane == 0) {
            s_lb[0] = 0; s_lb[1] = topL; s_lb[2] = topL + topR; s_lb[3] = allL + topR; s_lb[4] = allL + allR;
        }
    }
    __syncthreads();
    const int nl = s_lb[4];
    for (int i = wid; i < dr; i += 4) {
        const uint64_t m = s_mask[i];
        if ((m >> lane) & 1ull) {
            const uint64_t below = m & ((1ull << lane) - 1ull);
            const int pos = lane < cs ? s_off[i] + (int)__popcll(below) : s_offR[i] + (int)__popcll(below & ~Lm);
            s_list[pos] = (uint16_t)(((3 + i) << 8) | (3 + lane));
        }
    }
    __syncthreads();
    for (int k = tid; k < nl; k += 256) {
        const int rc = s_list[k], r = rc >> 8, cc = rc & 0xff;
        const int sc = fast_score_lds(&s_img[r * FC_LD + mis + cc], FC_LD);
        s_sc[r * FC_LD + cc] = (uint8_t)max(sc, 0);
    }
    __syncthreads();
    ORBGPU_PROF_MARK(2);
    const int nch = (nl + 63) >> 6;
    for (int ch = wid; ch < nch; ch += 4) {
        const int k = ch * 64 + lane;
        bool khi = false, klo = false;
        if (k < nl) {
            const int rc = s_list[k], r = rc >> 8, cc = rc & 0xff;
            const int s = s_sc[r * FC_LD + cc];
            const bool bot = r >= 3 + rs, rgt = cc >= 3 + cs;
            // the entry's own cell: detection rows [rlo, rhi), columns [clo, chi)
            const int rlo = bot ? 3 + rs : 3, rhi = bot ? 3 + dr : 3 + rs;
            const int clo = rgt ? 3 + cs : 3, chi = rgt ? 3 + dc : 3 + cs;
            const bool up = r - 1 >= rlo, dn = r + 1 < rhi, lf = cc - 1 >= clo, rt = cc + 1 < chi;
            const uint8_t* q = &s_sc[r * FC_LD + cc];
            const int n0 = (up && lf) ? q[-FC_LD - 1] : 0, n1 = up ? q[-FC_LD] : 0, n2 = (up && rt) ? q[-FC_LD + 1] : 0;
            const int n3 = lf ? q[-1] : 0, n4 = rt ? q[1] : 0;
            const int n5 = (dn && lf) ? q[FC_LD - 1] : 0, n6 = dn ? q[FC_LD] : 0, n7 = (dn && rt) ? q[FC_LD + 1] : 0;
            // for s >= th a neighbour below th (stored as 0 in the reference's score row) is below
            // s as well, so S > (n >= th ? n : 0) for every n <=> S > max n: one comparison
            // serves both thresholds
            const bool lmax = s > max(max(max(n0, n1), max(n2, n3)), max(max(n4, n5), max(n6, n7)));
            khi = lmax && s >= iniTh;
            klo = lmax && s >= minTh;
        }
        const uint64_t mh = __ballot(khi), ml = __ballot(klo);
        if (lane == 0) { s_khi[ch] = mh; s_klo[ch] = ml; }
    }
    __syncthreads();
    // wave 0, lane = list chunk: cell k keeps its iniTh corners if it has any; the chosen keeps
    // (fin) are scanned over the chunks.  The list is cell-major, so the keeps before cell k's
    // first entry are the keeps of cells < k.
    if (wid == 0) {
        const uint64_t h = lane < nch ? s_khi[lane] : 0ull, lo = lane < nch ? s_klo[lane] : 0ull;
        uint64_t fin = 0;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const int a = s_lb[k] - lane * 64, e = s_lb[k + 1] - lane * 64;   // chunk-relative range
            const uint64_t ma = a <= 0 ? ~0ull : a >= 64 ? 0ull : ~((1ull << a) - 1ull);
            const uint64_t me = e <= 0 ? 0ull : e >= 64 ? ~0ull : ((1ull << e) - 1ull);
            const uint64_t mk = ma & me;
            const bool hi = __ballot((h & mk) != 0ull) != 0ull;
            fin |= mk & (hi ? h : lo);
        }
        if (lane < 64) s_mask[lane] = fin;
        const int cnt = (int)__popcll(fin);
        int incl = cnt;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(incl, o, 64);
            if (lane >= o) incl += y;
        }
        s_off[lane] = incl - cnt;
        if (lane == 63) s_off[64] = incl;
    }
    __syncthreads();
    // keeps before list position p
    auto before = [&](int p) {
        const int c = p >> 6, o = p & 63;
        return s_off[c] + (o ? (int)__popcll(s_mask[c] & ((1ull << o) - 1ull)) : 0);
    };
    if (tid < 4 && g.cell[tid] >= 0) cnt_out[g.cell[tid]] = min(before(s_lb[tid + 1]) - before(s_lb[tid]), g.cap[tid]);
    uint32_t* out = slots + (size_t)b * slots_per_image;
    for (int ch = wid; ch < nch; ch += 4) {
        const uint64_t m = s_mask[ch];
        if ((m >> lane) & 1ull) {
            const int rc = s_list[ch * 64 + lane], r = rc >> 8, cc = rc & 0xff;
            const int k = (r >= 3 + rs) * 2 + (cc >= 3 + cs);
            const int pos = s_off[ch] + __popcll(m & ((1ull << lane) - 1ull)) - before(sel4(k, s_lb[0], s_lb[1], s_lb[2], s_lb[3]));
            if (pos < sel4(k, g.cap[0], g.cap[1], g.cap[2], g.cap[3])) {
                const uint32_t sv = s_sc[r * FC_LD + cc];
                const uint32_t xr = (uint32_t)(cc + sel4(k, g.xadd[0], g.xadd[1], g.xadd[2], g.xadd[3]));
                const uint32_t yr = (uint32_t)(r + sel4(k, g.yadd[0], g.yadd[1], g.yadd[2], g.yadd[3]));
                out[sel4(k, g.slot_off[0], g.slot_off[1], g.slot_off[2], g.slot_off[3]) + pos] = (sv << 24) | (yr << 12) | xr;
            }
        }
    }
    ORBGPU_PROF_MARK(3);
}

// IC_Angle (unblurred level) + rotated BRIEF (blurred level), one wave per keypoint.
//   IC_Angle   lane = (disc row v, half): the row's 16 pixels u in [-15, 0] (half 0) or [1, 16]
//              (half 1) are one unaligned 16-byte load (5 dwords, v_alignbyte), masked to
//              |u| <= umax[|v|]; sum I and sum i*I (i = byte index) are v_sad_u8 / v_dot4_u32_u8,
//              so m_10 = sum u*I and m_01 = sum v*I are two wave sums.  Exact integer moments:
//              the same as the reference's loops (ORBextractor.cc:77-103) in any order.
//   BRIEF      the 37 x 37 blurred patch around the keypoint (every rotated test lies within 18
//              px) is staged in LDS with row-coalesced dword loads, then the 512 tests of the 256
//              pairs are LDS byte reads: lane l evaluates pairs l, l+64, l+128, l+192, so the
//              four wave ballots ARE the 32 descriptor bytes (byte i bit k = pair 8i+k).
//              Keypoints are >= 19 px inside their level (FAST's 3-px frame inside the 16-px
//              cell border), so the patch never leaves the blurred level.
constexpr int kBriefR = 18, kBriefRows = 2 * kBriefR + 1, kBriefLd = 40;   // patch rows, LDS row bytes
__global__ void __launch_bounds__(256) k_orient_desc(const uint8_t* __restrict__ pyr, const uint8_t* __restrict__ blur,
                                                     size_t img_bytes, size_t blur_bytes, const int2* __restrict__ sel, int selcap,
                                                     const int* __restrict__ nout, const LevelArgs lva,
                                                     orb_kp_dev* __restrict__ kps, uint8_t* __restrict__ desc,
                                                     int cap_per_image, int gx, int B) {
    __shared__ uint32_t s_patch[4][kBriefRows * kBriefLd / 4];
    // batches of >= 8 images: workgroup g runs on XCD g % 8, and image b's keypoint groups all
    // go to XCD b % 8 (images in turn), so the level and blurred-level lines their patches
    // share stay in that XCD's L2; smaller batches spread every image over all XCDs
    // the wave's keypoint, its record and its level are wave-uniform: scalar loads (the level
    // table is a kernel argument), so one dependent memory round trip precedes the pixel loads
    const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    int img, grp;
    if (B >= 8) {
        const int xcd = blockIdx.x & 7, slot = blockIdx.x >> 3;
        img = xcd + 8 * (slot / gx);
        grp = slot - (slot / gx) * gx;
    } else {
        img = blockIdx.x / gx;
        grp = blockIdx.x - img * gx;
    }
    if (img >= B) return;
    const int k = grp * 4 + wv;
    if (k >= nout[img] || k >= cap_per_image) return;   // wave-uniform: no barrier below
    const int2 s = sel[(size_t)img * selcap + k];
    const uint32_t pk = (uint32_t)__builtin_amdgcn_readfirstlane(s.x);
    const int meta = __builtin_amdgcn_readfirstlane(s.y);
    const int b = meta >> 20, l = (meta >> 16) & 15, idx = meta & 0xffff;
    const int x = (int)(pk & 0xfff) + (kEdge - 3), y = (int)((pk >> 12) & 0xfff) + (kEdge - 3);
    const int score = (int)(pk >> 24);
    const LevelDev L = lva.lv[l];
    // stage the blurred patch (rows y-18 .. y+18, dword columns from (x-18) & ~3) first: its
    // loads are in flight during the moments
    const int c0 = (x - kBriefR) & ~3, mis = (x - kBriefR) - c0;
    const uint8_t* cbase = blur + (size_t)b * blur_bytes + L.boff + (size_t)(y - kBriefR) * L.bpitch + c0;
    uint32_t* sp = s_patch[wv];
    constexpr int kPatchWords = kBriefRows * (kBriefLd / 4);
    uint32_t pv[(kPatchWords + 63) / 64];
#pragma unroll
    for (int t = 0; t < (kPatchWords + 63) / 64; t++) {
        const int i = lane + 64 * t;
        const int r = i / (kBriefLd / 4), q = i - r * (kBriefLd / 4);
        pv[t] = (i < kPatchWords && c0 + 4 * q < L.bpitch)
                    ? *reinterpret_cast<const uint32_t*>(cbase + (size_t)r * L.bpitch + 4 * q) : 0u;
    }
    // IC_Angle moments
    int m10 = 0, m01 = 0;
    if (lane < 2 * kPatch) {
        const int v = (lane >> 1) - kHalfPatch, h = lane & 1;
        const int d = c_umax[v < 0 ? -v : v];
        const uint8_t* row = pyr + (size_t)b * img_bytes + L.off + (size_t)(kEdge + y + v) * L.pitch + kEdge + x
                             - kHalfPatch + 16 * h;   // pixel u = -15 + 16 h + i at byte i
        const uintptr_t a = (uintptr_t)row;
        const uint32_t* a32 = reinterpret_cast<const uint32_t*>(a & ~(uintptr_t)3);
        const uint32_t sh = (uint32_t)(a & 3);
        const uint32_t w0 = a32[0], w1 = a32[1], w2 = a32[2], w3 = a32[3], w4 = sh ? a32[4] : 0u;
        uint32_t px[4] = {__builtin_amdgcn_alignbyte(w1, w0, sh), __builtin_amdgcn_alignbyte(w2, w1, sh),
                          __builtin_amdgcn_alignbyte(w3, w2, sh), __builtin_amdgcn_alignbyte(w4, w3, sh)};
        // valid bytes: half 0 i >= 15 - d (u >= -d), half 1 i <= d - 1 (u <= d)
        const int lo = h ? 0 : kHalfPatch - d, hi = h ? d : 16;   // [lo, hi)
        uint32_t S = 0, T = 0;
#pragma unroll
        for (int m = 0; m < 4; m++) {
            const int a0 = min(max(lo - 4 * m, 0), 4), a1 = min(max(hi - 4 * m, 0), 4);   // bytes [a0, a1)
            const uint32_t mk = a1 <= a0 ? 0u : ((a1 == 4 ? 0xffffffffu : ((1u << (8 * a1)) - 1u)) & ~((1u << (8 * a0)) - 1u));
            const uint32_t w = px[m] & mk;
            const uint32_t W = (uint32_t)(4 * m) * 0x01010101u + 0x03020100u;   // byte weights 4m .. 4m+3
            S = __builtin_amdgcn_sad_u8(w, 0u, S);
            T = __builtin_amdgcn_udot4(w, W, T, false);
        }
        m10 = (int)T + (h ? (int)S : -kHalfPatch * (int)S);
        m01 = v * (int)S;
    }
#pragma unroll
    for (int t = 0; t < (kPatchWords + 63) / 64; t++) {
        const int i = lane + 64 * t;
        if (i < kPatchWords) sp[i] = pv[t];
    }
    m10 = wave_sum(m10);
    m01 = wave_sum(m01);
    const float angle = fast_atan2((float)m01, (float)m10);
    const float factorPI = (float)(3.14159265358979323846 / 180.f);
    float sa, ca;
    glibc_sincosf(angle * factorPI, &sa, &ca);
    const float a = ca, bb = sa;
    const uint8_t* cb = reinterpret_cast<const uint8_t*>(sp) + kBriefR * kBriefLd + mis + kBriefR;
    uint64_t words[4];
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const int p = lane + 64 * q;
        const float x0 = (float)c_pattern[4 * p], y0 = (float)c_pattern[4 * p + 1];
        const float x1 = (float)c_pattern[4 * p + 2], y1 = (float)c_pattern[4 * p + 3];
        const int t0 = cb[cv_round(x0 * bb + y0 * a) * kBriefLd + cv_round(x0 * a - y0 * bb)];
        const int t1 = cb[cv_round(x1 * bb + y1 * a) * kBriefLd + cv_round(x1 * a - y1 * bb)];
        words[q] = __ballot(t0 < t1);
    }
    const size_t o = (size_t)b * cap_per_image + idx;
    if (lane < 4) reinterpret_cast<uint64_t*>(desc + o * 32)[lane] = words[lane];
    if (lane == 0) {
        orb_kp_dev kp;
        float fx = (float)x, fy = (float)y;
        if (l != 0) {
            fx = fx * L.scale;
            fy = fy * L.scale;
        }
        kp.x = fx;
        kp.y = fy;
        kp.size = L.kp_size;
        kp.angle = angle;
        kp.response = (float)score;
        kp.octave = l;
        kp.class_id = -1;
        kps[o] = kp;
    }
}

// ------------------------------------------------------------- host driver
static inline int align_up(int v, int a) { return (v + a - 1) / a * a; }

static float cvRoundf_host(float v) { return (float)std::lrint(v); }

Extractor::Extractor(int nfeatures, float scaleFactor, int nlevels, int iniTh, int minTh)
    : nfeatures_(nfeatures), scaleFactorD_((double)scaleFactor), scaleFactor_(scaleFactor),
      nlevels_(nlevels), iniTh_(iniTh), minTh_(minTh) {
    // ORBextractor ctor, ORBextractor.cc:410-452 (float/double promotion kept)
    scale_.resize(nlevels);
    sigma2_.resize(nlevels);
    invScale_.resize(nlevels);
    invSigma2_.resize(nlevels);
    nPerLevel_.resize(nlevels);
    scale_[0] = 1.0f;
    sigma2_[0] = 1.0f;
    for (int i = 1; i < nlevels; i++) {
        scale_[i] = (float)(scale_[i - 1] * scaleFactorD_);
        sigma2_[i] = scale_[i] * scale_[i];
    }
    for (int i = 0; i < nlevels; i++) {
        invScale_[i] = 1.0f / scale_[i];
        invSigma2_[i] = 1.0f / sigma2_[i];
    }
    const float factor = (float)(1.0f / scaleFactorD_);
    float nDesired = nfeatures * (1 - factor) / (1 - (float)std::pow((double)factor, (double)nlevels));
    int sum = 0;
    for (int l = 0; l < nlevels - 1; l++) {
        nPerLevel_[l] = (int)cvRoundf_host(nDesired);
        sum += nPerLevel_[l];
        nDesired *= factor;
    }
    nPerLevel_[nlevels - 1] = std::max(nfeatures - sum, 0);
    // umax, ORBextractor.cc:454-469
    umax_.assign(kHalfPatch + 1, 0);
    const int vmax = (int)std::floor(kHalfPatch * std::sqrt(2.f) / 2 + 1);
    const int vmin = (int)std::ceil(kHalfPatch * std::sqrt(2.f) / 2);
    const double hp2 = kHalfPatch * kHalfPatch;
    for (int v = 0; v <= vmax; ++v) umax_[v] = (int)std::lrint(std::sqrt(hp2 - v * v));
    for (int v = kHalfPatch, v0 = 0; v >= vmin; --v) {
        while (umax_[v0] == umax_[v0 + 1]) ++v0;
        umax_[v] = v0;
        ++v0;
    }
}

Extractor::~Extractor() { release(); }

void Extractor::release() {
    auto F = [](void* p) { if (p) (void)hipFree(p); };
    F(d_in_); F(d_pyr_); F(d_blur_); F(d_slots_); F(d_counts_); F(d_cells_); F(d_tiles_); F(d_work_); F(d_groups_);
    F(d_lcb_); F(d_packed_); F(d_hdr_); F(d_sel_); F(d_levels_); F(d_tabs_);
    F(d_kps_); F(d_desc_); F(d_jobsel_); F(d_jobcnt_); F(d_octlv_); F(d_gscr_); F(d_nout_); F(d_ptiles_);
    F(d_chain_); F(d_cellslot_); F(d_flowcnt_);
    d_flowcnt_ = nullptr;
    d_ptiles_ = nullptr;
    d_chain_ = nullptr;
    d_cellslot_ = nullptr;
    d_jobsel_ = d_jobcnt_ = d_octlv_ = d_gscr_ = d_nout_ = nullptr;
    d_in_ = d_pyr_ = d_blur_ = nullptr;
    d_slots_ = nullptr; d_counts_ = nullptr; d_cells_ = nullptr; d_tiles_ = nullptr; d_work_ = nullptr; d_groups_ = nullptr;
    work_B_ = -1;
    d_lcb_ = nullptr; d_packed_ = nullptr; d_hdr_ = nullptr; d_gtotal_ = nullptr; d_sel_ = nullptr;
    d_levels_ = nullptr; d_tabs_ = nullptr; d_kps_ = nullptr; d_desc_ = nullptr;
    if (h_nout_) (void)hipHostFree(h_nout_);
    h_nout_ = nullptr;
    if (h_in_) (void)hipHostFree(h_in_);
    h_in_ = nullptr;
    h_in_cap_ = 0;
    for (auto& e : ev_) if (e) (void)hipEventDestroy(e);
    for (auto& e : ev_) e = nullptr;
    if (stream_ && ownStream_) (void)hipStreamDestroy(stream_);
    stream_ = nullptr;
    if (evBlur_) (void)hipEventDestroy(evBlur_);
    evBlur_ = nullptr;
    if (evPyrA_) (void)hipEventDestroy(evPyrA_);
    if (evFastA_) (void)hipEventDestroy(evFastA_);
    evPyrA_ = evFastA_ = nullptr;
    if (side_) (void)hipStreamDestroy(side_);
    side_ = nullptr;
}

int Extractor::init_device(int maxW, int maxH, int maxBatch) {
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return -4;
    // ORBGPU_EXTRACT_STREAM_PRIO=1: the extraction stream at the device's highest priority (A/B
    // runs of the pipelined bench)
    if (const char* pe = getenv("ORBGPU_EXTRACT_STREAM_PRIO"); pe && pe[0] == '1') {
        int lo = 0, hi = 0;
        ORB_HIP_CHECK(hipDeviceGetStreamPriorityRange(&lo, &hi));
        ORB_HIP_CHECK(hipStreamCreateWithPriority(&stream_, hipStreamNonBlocking, hi));
    } else {
        ORB_HIP_CHECK(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
    }
    for (auto& e : ev_) ORB_HIP_CHECK(hipEventCreate(&e));
    const char* eb = getenv("ORBGPU_BLUR_SIDE");
    const char* ef = getenv("ORBGPU_FAST_SPLIT");
    const bool blurSide = eb && atoi(eb) > 0;
    fastSplit_ = ef && atoi(ef) == 1 && !blurSide;
    // opt-in (ORBGPU_PYR_FLOW=1): the whole pyramid as one launch of dependent tasks; slower than
    // the launch per level alone (0.264 vs 0.239 ms at 128 images) and far slower in the pipeline
    // (37.4 k vs 43.7 k frames/s: its waiting workgroups hold CU slots the tracking lane needs),
    // profiles/r06fp_pyr_flow_ab.txt
    const char* ew = getenv("ORBGPU_PYR_FLOW");
    flow_ = ew && ew[0] == '1';
    if (blurSide || fastSplit_) ORB_HIP_CHECK(hipStreamCreateWithFlags(&side_, hipStreamNonBlocking));
    if (blurSide) ORB_HIP_CHECK(hipEventCreateWithFlags(&evBlur_, hipEventDisableTiming));
    if (fastSplit_) {
        ORB_HIP_CHECK(hipEventCreateWithFlags(&evPyrA_, hipEventDisableTiming));
        ORB_HIP_CHECK(hipEventCreateWithFlags(&evFastA_, hipEventDisableTiming));
    }
    static bool consts_done = false;  // per process; guarded by first-use in create
    if (!consts_done) {
        ORB_HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(c_pattern), kPattern, sizeof(kPattern)));
        int taps[7];
        gaussian_taps(taps);
        ORB_HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(c_gauss), taps, sizeof(taps)));
        consts_done = true;
    }
    // disc offsets for IC_Angle: row v uses |u| <= umax[|v|]
    std::vector<int8_t> disc;
    for (int v = -kHalfPatch; v <= kHalfPatch; v++) {
        const int d = v == 0 ? kHalfPatch : umax_[std::abs(v)];
        for (int u = -d; u <= d; u++) { disc.push_back((int8_t)u); disc.push_back((int8_t)v); }
    }
    const int nd = (int)disc.size() / 2;
    ORB_HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(c_disc), disc.data(), disc.size()));
    ORB_HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(c_ndisc), &nd, sizeof(int)));
    int um[16];
    for (int v = 0; v <= kHalfPatch; v++) um[v] = v == 0 ? kHalfPatch : umax_[v];
    ORB_HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(c_umax), um, sizeof(um)));
    maxW_ = maxW; maxH_ = maxH; maxB_ = maxBatch;
    return 0;
}

// k_fast_cells work order for a batch of B images: the group rows (groups sharing level and ROI
// top row, in cell order) of every image are dealt round-robin to the 8 XCDs; entry
// g = slot * 8 + xcd of the table is the slot-th (b << 16 | group) of that XCD's list, -1 past
// its end.  Two such tables back to back: the levels below kFastSplitLevel, then the rest
// (each a multiple of 8 entries, so the concatenation is one table as well).
int Extractor::build_work(int B) {
    constexpr int kXcds = 8;
    const int ngroups = (int)groups_.size();
    std::vector<int> unit;
    for (int c = 0; c < ngroups; c++)
        if (c == 0 || groups_[c].lvl_off != groups_[c - 1].lvl_off || groups_[c].r0 != groups_[c - 1].r0)
            unit.push_back(c);
    unit.push_back(ngroups);
    const long long splitOff =
        nlevels_ > kFastSplitLevel ? (long long)levels_[kFastSplitLevel].off : std::numeric_limits<long long>::max();
    std::vector<int> work;
    for (int part = 0; part < 2; part++) {
        std::vector<std::vector<int>> lists(kXcds);
        long u = 0;
        for (int b = 0; b < B; b++)
            for (size_t k = 0; k + 1 < unit.size(); k++) {
                if ((groups_[unit[k]].lvl_off < splitOff) != (part == 0)) continue;
                for (int c = unit[k]; c < unit[k + 1]; c++) lists[u % kXcds].push_back((b << 16) | c);
                u++;
            }
        size_t len = 0;
        for (auto& l : lists) len = std::max(len, l.size());
        const size_t base = work.size();
        work.resize(base + len * kXcds, -1);
        for (int x = 0; x < kXcds; x++)
            for (size_t sl = 0; sl < lists[x].size(); sl++) work[base + sl * kXcds + x] = lists[x][sl];
        work_part_[part] = (int)(len * kXcds);
    }
    if (d_work_) (void)hipFree(d_work_);
    d_work_ = nullptr;
    ORB_HIP_CHECK(hipMalloc(&d_work_, std::max<size_t>(work.size(), 1) * 4));
    ORB_HIP_CHECK(hipMemcpy(d_work_, work.data(), work.size() * 4, hipMemcpyHostToDevice));
    work_n_ = (int)work.size();
    work_B_ = B;
    return 0;
}

int Extractor::share_stream(Extractor* with) {
    if (!stream_ || !with || !with->stream_) return -4;
    if (with == this) return 0;
    ORB_HIP_CHECK(hipStreamSynchronize(stream_));
    if (ownStream_) (void)hipStreamDestroy(stream_);
    stream_ = with->stream_;
    ownStream_ = false;
    with->lent_++;   // its stream may no longer be recreated (reserve_cus)
    return 0;
}

int Extractor::reserve_cus(int one_in_n) {
    if (!stream_) return -4;
    if (!ownStream_ || lent_) return -1;   // a shared stream: another extractor launches on it
    int dev = 0, ncu = 0;
    ORB_HIP_CHECK(hipGetDevice(&dev));
    ORB_HIP_CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    ORB_HIP_CHECK(hipStreamSynchronize(stream_));
    hipStream_t s = nullptr;
    if (one_in_n <= 0) {
        ORB_HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    } else {
        // mask bit c is CU c / kXcds of XCD c % kXcds (CUs are enumerated round-robin over the
        // XCDs): leave out the same CUs of every XCD so that no XCD's share of a grid straggles
        constexpr int kXcds = 8;
        std::vector<uint32_t> mask((ncu + 31) / 32, 0u);
        for (int c = 0; c < ncu; c++)
            if ((c / kXcds) % one_in_n != one_in_n - 1) mask[c >> 5] |= 1u << (c & 31);
        ORB_HIP_CHECK(hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()));
    }
    (void)hipStreamDestroy(stream_);
    stream_ = s;
    return 0;
}

void Extractor::gaussian_taps(int taps[7]) {
    // getGaussianKernel(7, 2, CV_32F) then *256 -> int (createSeparableLinearFilter)
    float cf[7];
    double sum = 0, scale2X = -0.5 / (2.0 * 2.0);
    for (int i = 0; i < 7; i++) {
        double x = i - 3.0;
        cf[i] = (float)std::exp(scale2X * x * x);
        sum += cf[i];
    }
    sum = 1. / sum;
    for (int i = 0; i < 7; i++) {
        cf[i] = (float)(cf[i] * sum);
        taps[i] = (int)std::lrint(cf[i] * 256.0f);
    }
}

// Plan of k_pyr_chain (levels la .. nlevels-1; yr[l] = level l's row map, 2 ints per row):
// K row strips per image, the fewest (at least kChainMinStrips) whose LDS -- the staged source
// rows of level la-1, two level buffers, the row taps -- fits kChainLdsMax.  Own rows: level
// nlevels-1 split evenly, level l's strip boundaries the images of level l+1's under the row
// map.  Compute rows: own rows plus every row the level above's compute rows read.  Padded rows:
// each goes to the strip owning the interior row it reflects to.  Every range is checked here,
// so the kernel's indexing stays inside its buffers.  Opt-in: ORBGPU_PYR_CHAIN=1.
int Extractor::plan_chain(const std::vector<std::vector<int>>& yr) {
    chain_ = false;
    chainTab_.clear();
    static const bool off = [] {   // opt-in (ORBGPU_PYR_CHAIN=1): slower than the per-level
        const char* e = getenv("ORBGPU_PYR_CHAIN");   // launches so far
        return !(e && e[0] == '1');
    }();
    // the first chained level (ORBGPU_PYR_CHAIN_FROM, default 3): levels 1 .. la-1 keep their
    // own k_pyr_resize launches (large levels, bandwidth-bound tiles)
    static const int from = [] {
        const char* e = getenv("ORBGPU_PYR_CHAIN_FROM");
        return e ? std::max(1, atoi(e)) : 3;
    }();
    const int la = from, lb = nlevels_ - 1, nl = lb - la + 1;
    if (off || la > lb) return 0;
    for (int l = la; l <= lb; l++)
        if (((levels_[l].w + 3) >> 2) > 256) return 0;   // one 4-column group per thread
    const int hTop = levels_[lb].h;
    std::vector<int> rp(nlevels_);
    for (int l = 0; l < nlevels_; l++) rp[l] = (levels_[l].w + 3) & ~3;
    const int srcRp = (levels_[la - 1].w + 6 + 3) & ~3;   // padded columns [16, 16 + srcRp) staged
    constexpr int kChainMinStrips = 8;
    for (int K = std::min(kChainMinStrips, hTop); K <= std::min(hTop, 256); K++) {
        // own boundaries A[l][0..K]
        std::vector<std::vector<int>> A(nlevels_, std::vector<int>(K + 1));
        for (int k = 0; k <= K; k++) A[lb][k] = (int)(((long long)k * hTop) / K);
        for (int l = lb - 1; l >= 0; l--) {
            A[l][0] = 0;
            A[l][K] = levels_[l].h;
            for (int k = 1; k < K; k++) A[l][k] = yr[l + 1][2 * A[l + 1][k]];
        }
        bool ok = true;
        for (int l = la; l <= lb && ok; l++)
            for (int k = 0; k < K; k++)
                if (A[l][k] >= A[l][k + 1]) ok = false;   // every strip owns rows on every level
        if (!ok) break;
        // compute ranges; source rows of level la-1
        std::vector<std::vector<std::pair<int, int>>> C(K, std::vector<std::pair<int, int>>(nlevels_));
        std::vector<std::pair<int, int>> Src(K);
        size_t buf[2] = {0, 0}, srcBytes = 0, rtRows = 0;
        for (int k = 0; k < K; k++) {
            C[k][lb] = {A[lb][k], A[lb][k + 1]};
            for (int l = lb - 1; l >= la; l--) {
                const auto& u = C[k][l + 1];
                const int lo = std::min(yr[l + 1][2 * u.first], A[l][k]);
                const int hi = std::max(yr[l + 1][2 * (u.second - 1) + 1] + 1, A[l][k + 1]);
                C[k][l] = {lo, hi};
            }
            size_t rows = 0;
            for (int l = la; l <= lb; l++) {
                const auto& c = C[k][l];
                if (c.first < 0 || c.second > levels_[l].h || c.first >= c.second) return -1;
                if (c.first > 0xffff || c.second > 0xffff) return -1;   // row taps packed in 16 bits
                const auto p = l > la ? C[k][l - 1] : std::make_pair(0, 0);
                int smin = 1 << 30, smax = -1;
                for (int dy = c.first; dy < c.second; dy++) {
                    smin = std::min(smin, yr[l][2 * dy]);
                    smax = std::max(smax, yr[l][2 * dy + 1]);
                    // the rows level l reads from level l-1 lie in that level's buffer
                    if (l > la && (yr[l][2 * dy] < p.first || yr[l][2 * dy + 1] >= p.second)) return -1;
                }
                if (l == la) Src[k] = {smin, smax + 1};
                const size_t bytes = (size_t)(c.second - c.first) * rp[l] + 16;
                buf[(l - la) & 1] = std::max(buf[(l - la) & 1], bytes);
                rows += (size_t)(c.second - c.first);
            }
            srcBytes = std::max(srcBytes, (size_t)(Src[k].second - Src[k].first) * srcRp + 16);
            rtRows = std::max(rtRows, rows);
        }
        const size_t o1 = (srcBytes + 15) & ~(size_t)15, o2 = o1 + ((buf[0] + 15) & ~(size_t)15),
                     o3 = o2 + ((buf[1] + 15) & ~(size_t)15);
        // padded rows written per strip (own rows + the border rows reflecting to them)
        size_t rlRows = 0;
        for (int k = 0; k < K; k++) {
            size_t n = 0;
            for (int l = la; l <= lb; l++) {
                for (int py = 0; py < levels_[l].ph; py++) {
                    int y = py - kEdge;
                    if (levels_[l].h == 1) y = 0;
                    while (y < 0 || y >= levels_[l].h) y = y < 0 ? -y : 2 * levels_[l].h - y - 2;
                    if (y >= A[l][k] && y < A[l][k + 1]) n++;
                }
            }
            rlRows = std::max(rlRows, n);
        }
        const size_t o4 = o3 + ((rtRows * 8 + 15) & ~(size_t)15);
        const size_t lds = o4 + rlRows * 2;
        if (lds > (size_t)kChainLdsMax) continue;
        // tables: levels | strips (nl + 1 entries per strip) | padded-row lists
        std::vector<ChainLevel> cl(nl);
        std::vector<int32_t> strips((size_t)4 * K * (nl + 1));
        std::vector<uint16_t> rowl;
        for (int l = la; l <= lb; l++) {
            ChainLevel& c = cl[l - la];
            const LevelHost& L = levels_[l];
            if (L.ph > 65535) return -1;
            c.off = (long long)L.off;
            c.w = L.w; c.h = L.h; c.pitch = L.pitch; c.rp = rp[l];
            c.lds = ((l - la) & 1) ? (int)o2 : (int)o1;
            c.xofs = (int)tab_off_[l][0]; c.xal = (int)tab_off_[l][1];
            c.yr = (int)tab_off_[l][2]; c.yb = (int)tab_off_[l][3];
            c.nph = std::max(1, 256 / ((L.w + 3) >> 2));
            std::vector<std::vector<uint16_t>> own(K);
            for (int py = 0; py < L.ph; py++) {
                int y = py - kEdge;
                if (L.h == 1) y = 0;
                while (y < 0 || y >= L.h) y = y < 0 ? -y : 2 * L.h - y - 2;
                const int k = (int)(std::upper_bound(A[l].begin(), A[l].end(), y) - A[l].begin()) - 1;
                own[k].push_back((uint16_t)py);
            }
            for (int k = 0; k < K; k++) {
                int32_t* e = &strips[((size_t)k * (nl + 1) + (l - la)) * 4];
                e[0] = C[k][l].first;
                e[1] = C[k][l].second;
                e[2] = (int32_t)rowl.size();
                e[3] = (int32_t)own[k].size();
                rowl.insert(rowl.end(), own[k].begin(), own[k].end());
            }
        }
        for (int k = 0; k < K; k++) {
            int32_t* e = &strips[((size_t)k * (nl + 1) + nl) * 4];
            e[0] = Src[k].first;
            e[1] = Src[k].second;
            e[2] = (int32_t)o3;
            e[3] = (int32_t)o4;
            if (Src[k].first < 0 || Src[k].second > levels_[la - 1].h) return -1;
        }
        chainK_ = K;
        chainFrom_ = la;
        chainLds_ = (int)lds;
        chainSrcLds_ = 0;
        chainSrcRp_ = srcRp;
        chainStripOff_ = (sizeof(ChainLevel) * nl + 15) & ~(size_t)15;
        chainRowOff_ = chainStripOff_ + strips.size() * 4;
        chainTab_.assign(chainRowOff_ + rowl.size() * 2, 0);
        std::memcpy(chainTab_.data(), cl.data(), sizeof(ChainLevel) * nl);
        std::memcpy(chainTab_.data() + chainStripOff_, strips.data(), strips.size() * 4);
        std::memcpy(chainTab_.data() + chainRowOff_, rowl.data(), rowl.size() * 2);
        chain_ = true;
        return 0;
    }
    return 0;   // no plan fits: a launch per level
}

// Geometry of the pyramid / cells / resize tables for an image size.
// k_pyr_flow's per-level task table for a batch of B images (tile-height variant v)
FlowArgs Extractor::flow_args(int v, int B) const {
    FlowArgs A{};
    A.nl = nlevels_;
    int task = 0, band = 0;
    for (int l = 0; l < nlevels_; l++) {
        const LevelHost& L = levels_[l];
        FlowLevel& F = A.L[l];
        F.off = (long long)L.off;
        F.pitch = L.pitch;
        F.ph = L.ph;
        F.w = L.w;
        F.h = L.h;
        F.th = ptile_th_[v * nlevels_ + l];
        const int nb = (L.ph + F.th - 1) / F.th;
        F.ncol = l == 0 ? 1 : (L.pitch + PT_W - 1) / PT_W;
        F.ntiles = l == 0 ? nb : ptile_n_[v * nlevels_ + l];
        F.tile0 = l == 0 ? 0 : ptile_begin_[v * (nlevels_ + 1) + l];
        F.band0 = band;
        F.task0 = task;
        if (l > 0) {
            F.xofs = (int)tab_off_[l][0];
            F.xal = (int)tab_off_[l][1];
            F.yr = (int)tab_off_[l][2];
            F.yb = (int)tab_off_[l][3];
        }
        band += nb;
        task += B * F.ntiles;
    }
    A.nbands = band;
    return A;
}

int Extractor::setup_geometry(int W, int H) {
    if (W == geomW_ && H == geomH_) return 0;
    if (W > 4000 || H > 4000) return -1;
    levels_.assign(nlevels_, LevelHost{});
    size_t off = 0;
    for (int l = 0; l < nlevels_; l++) {
        LevelHost& L = levels_[l];
        L.w = (int)std::lrint((float)W * invScale_[l]);
        L.h = (int)std::lrint((float)H * invScale_[l]);
        if (L.w < 1 || L.h < 1) return -1;
        L.pw = L.w + 2 * kEdge;
        L.ph = L.h + 2 * kEdge;
        // k_pyr_flow: 128-B rows, so a cache line never holds bytes of two rows (its row hand-off)
        L.pitch = align_up(L.pw, flow_ ? 128 : 16);
        L.off = off;
        off += (size_t)L.pitch * L.ph;
        off = (off + 255) & ~(size_t)255;
    }
    img_bytes_ = off;
    size_t boff = 0;
    for (int l = 0; l < nlevels_; l++) {
        LevelHost& L = levels_[l];
        L.bpitch = align_up(L.w, 16);
        L.boff = boff;
        boff += (size_t)L.bpitch * L.h;
        boff = (boff + 255) & ~(size_t)255;
    }
    blur_bytes_ = boff;
    // cells, ORBextractor.cc:776-829
    cells_.clear();
    level_cell_begin_.assign(nlevels_ + 1, 0);
    size_t slot = 0;
    for (int l = 0; l < nlevels_; l++) {
        const LevelHost& L = levels_[l];
        level_cell_begin_[l] = (int)cells_.size();
        const float Wc = 30;
        const int minBorderX = kEdge - 3, minBorderY = minBorderX;
        const int maxBorderX = L.w - kEdge + 3, maxBorderY = L.h - kEdge + 3;
        const float width = (float)(maxBorderX - minBorderX), height = (float)(maxBorderY - minBorderY);
        const int nCols = (int)(width / Wc), nRows = (int)(height / Wc);
        if (nCols <= 0 || nRows <= 0) return -1;  // reference divides by zero
        const int wCell = (int)std::ceil(width / nCols), hCell = (int)std::ceil(height / nRows);
        if (wCell + 6 > FC_MAXR || hCell + 6 > FC_MAXR) return -1;
        for (int i = 0; i < nRows; i++) {
            const float iniY = (float)(minBorderY + i * hCell);
            float maxY = iniY + hCell + 6;
            if (iniY >= maxBorderY - 3) continue;
            if (maxY > maxBorderY) maxY = (float)maxBorderY;
            for (int j = 0; j < nCols; j++) {
                const float iniX = (float)(minBorderX + j * wCell);
                float maxX = iniX + wCell + 6;
                if (iniX >= maxBorderX - 6) continue;
                if (maxX > maxBorderX) maxX = (float)maxBorderX;
                CellDesc c;
                c.r0 = (int)iniY; c.r1 = (int)maxY; c.c0 = (int)iniX; c.c1 = (int)maxX;
                c.offx = j * wCell; c.offy = i * hCell;
                c.pitch = L.pitch;
                c.lvl_off = L.off;
                const int dr = c.r1 - c.r0 - 6, dc = c.c1 - c.c0 - 6;
                c.cap = (dr > 0 && dc > 0) ? ((dr + 1) / 2) * ((dc + 1) / 2) : 0;
                c.slot_off = (int)slot;
                slot += c.cap;
                c.level = l;
                cells_.push_back(c);
            }
        }
    }
    level_cell_begin_[nlevels_] = (int)cells_.size();
    slots_per_image_ = (slot + 63) & ~(size_t)63;
    if (cells_.size() > 4096) return -1;
    // cell groups: a level's cells form a grid (the skips above depend on i or on j only); two
    // neighbouring rows (columns) share a workgroup when the second one's ROI starts wCell
    // (hCell) after the first one's and ends at most FC_MAXR after it, and holds detection pixels
    groups_.clear();
    for (int l = 0; l < nlevels_; l++) {
        const int cb = level_cell_begin_[l], ce = level_cell_begin_[l + 1];
        if (cb == ce) continue;
        std::vector<int> rowb;   // first cell of every cell row
        for (int c = cb; c < ce; c++)
            if (c == cb || cells_[c].r0 != cells_[c - 1].r0) rowb.push_back(c);
        const int ncol = (int)(rowb.size() > 1 ? rowb[1] - rowb[0] : ce - cb);
        if ((ce - cb) != ncol * (int)rowb.size()) return -1;
        auto spans = [](int a0, int a1, int b0, int b1) {   // ROIs [a0,a1), [b0,b1) tile a union
            return a1 == b0 + 6 && b1 - b0 >= 7 && b1 - a0 <= FC_MAXR;
        };
        std::vector<std::pair<int, int>> rsel, csel;   // (first, count) row / column pairs
        for (int i = 0; i < (int)rowb.size();) {
            const CellDesc &a = cells_[rowb[i]];
            const bool two = i + 1 < (int)rowb.size() && spans(a.r0, a.r1, cells_[rowb[i + 1]].r0, cells_[rowb[i + 1]].r1);
            rsel.push_back({i, two ? 2 : 1});
            i += two ? 2 : 1;
        }
        for (int j = 0; j < ncol;) {
            const CellDesc &a = cells_[cb + j];
            const bool two = j + 1 < ncol && spans(a.c0, a.c1, cells_[cb + j + 1].c0, cells_[cb + j + 1].c1);
            csel.push_back({j, two ? 2 : 1});
            j += two ? 2 : 1;
        }
        for (auto& rp : rsel)
            for (auto& cp : csel) {
                CellGroup g{};
                const CellDesc& tl = cells_[rowb[rp.first] + cp.first];
                const CellDesc& br = cells_[rowb[rp.first + rp.second - 1] + cp.first + cp.second - 1];
                g.r0 = tl.r0; g.c0 = tl.c0;
                g.rows = br.r1 - tl.r0; g.cols = br.c1 - tl.c0;
                g.rsplit = rp.second == 2 ? tl.r1 - tl.r0 - 6 : std::max(g.rows - 6, 0);
                g.csplit = cp.second == 2 ? tl.c1 - tl.c0 - 6 : std::max(g.cols - 6, 0);
                g.pitch = tl.pitch;
                g.lvl_off = tl.lvl_off;
                for (int k = 0; k < 4; k++) {
                    const int di = k >> 1, dj = k & 1;
                    g.cell[k] = -1;
                    if (di >= rp.second || dj >= cp.second) continue;
                    const int c = rowb[rp.first + di] + cp.first + dj;
                    const CellDesc& cd = cells_[c];
                    g.cell[k] = c;
                    g.cap[k] = cd.cap;
                    g.slot_off[k] = cd.slot_off;
                    g.xadd[k] = cd.offx - (cd.c0 - g.c0);
                    g.yadd[k] = cd.offy - (cd.r0 - g.r0);
                }
                groups_.push_back(g);
            }
    }
    if (groups_.size() > 65535) return -1;
    // blur tiles
    tiles_.clear();
    for (int l = 0; l < nlevels_; l++) {
        const LevelHost& L = levels_[l];
        for (int ty = 0; ty < (L.h + BT_H - 1) / BT_H; ty++)
            for (int tx = 0; tx < (L.w + BT_W - 1) / BT_W; tx++) {
                BlurTile t;
                t.off = L.off; t.pitch = L.pitch; t.w = L.w; t.h = L.h; t.tx = tx; t.ty = ty;
                t.boff = L.boff; t.bpitch = L.bpitch;
                tiles_.push_back(t);
            }
    }
    // resize tables (OpenCV 3.2 resize(), INTER_LINEAR, fixpt)
    std::vector<uint8_t> tabs;
    auto push = [&tabs](const void* p, size_t n) -> size_t {
        size_t o = (tabs.size() + 15) & ~(size_t)15;
        tabs.resize(o + n);
        memcpy(tabs.data() + o, p, n);
        return o;
    };
    tab_off_.assign(nlevels_, {0, 0, 0, 0});
    std::vector<std::vector<int>> yrAll(nlevels_);   // every level's row map, for plan_chain
    xofsAll_.assign(nlevels_, {});
    xalAll_.assign(nlevels_, {});
    ptiles_.clear();
    ptile_begin_.assign(2 * (nlevels_ + 1), 0);   // variant v, level l: ptile_n_ tiles from here
    ptile_n_.assign(2 * nlevels_, 0);
    plds_.assign(2 * nlevels_, 0);
    ptile_th_.assign(2 * nlevels_, 0);
    for (int l = 1; l < nlevels_; l++) {
        const int sw = levels_[l - 1].w, sh = levels_[l - 1].h, dw = levels_[l].w, dh = levels_[l].h;
        const double scale_x = 1. / ((double)dw / sw), scale_y = 1. / ((double)dh / sh);
        std::vector<int> xofs(dw);
        std::vector<short> xal(2 * dw);
        int xmax = dw;
        auto sat_s = [](float v) { long i = std::lrint(v); return (short)std::min(32767L, std::max(-32768L, i)); };
        for (int dx = 0; dx < dw; dx++) {
            float fx = (float)((dx + 0.5) * scale_x - 0.5);
            int sx = (int)std::floor(fx);
            fx -= sx;
            if (sx < 0) { fx = 0; sx = 0; }
            if (sx + 1 >= sw) {
                xmax = std::min(xmax, dx);
                if (sx >= sw - 1) { fx = 0; sx = sw - 1; }
            }
            xofs[dx] = sx;
            xal[2 * dx] = sat_s((1.f - fx) * 2048);
            xal[2 * dx + 1] = sat_s(fx * 2048);
        }
        for (int dx = xmax; dx < dw; dx++) { xal[2 * dx] = 2048; xal[2 * dx + 1] = 0; }
        std::vector<int> yr(2 * dh);
        std::vector<short> yb(2 * dh);
        for (int dy = 0; dy < dh; dy++) {
            float fy = (float)((dy + 0.5) * scale_y - 0.5);
            int sy = (int)std::floor(fy);
            fy -= sy;
            yr[2 * dy] = std::min(std::max(sy, 0), sh - 1);
            yr[2 * dy + 1] = std::min(std::max(sy + 1, 0), sh - 1);
            yb[2 * dy] = sat_s((1.f - fy) * 2048);
            yb[2 * dy + 1] = sat_s(fy * 2048);
        }
        // k_pyr_resize tiles over the padded destination: the source rectangle each reads
        {
            const LevelHost& D = levels_[l];
            auto refl = [](int p, int len) {
                if (len == 1) return 0;
                while (p < 0 || p >= len) p = p < 0 ? -p : 2 * len - p - 2;
                return p;
            };
          for (int v = 0; v < 2; v++) {
            ptile_begin_[v * (nlevels_ + 1) + l] = (int)ptiles_.size();
            // tile height: kPyrTileH[v] rows unless the source rectangle would exceed the LDS budget
            // (scale factors well above the reference's 1.2)
            auto make = [&](int py0, int px0, int nrow, PyrTile& t) {
                int r0 = 1 << 30, r1 = -1, c0 = 1 << 30, c1 = -1;
                for (int py = py0; py < std::min(py0 + nrow, D.ph); py++) {
                    const int y = refl(py - kEdge, dh);
                    r0 = std::min(r0, yr[2 * y]);
                    r1 = std::max(r1, yr[2 * y + 1]);
                }
                for (int px = px0; px < std::min(px0 + PT_W, D.pitch); px++) {
                    const int x = refl(px - kEdge, dw);
                    c0 = std::min(c0, xofs[x]);
                    c1 = std::max(c1, xofs[x] + 1);
                }
                t.py0 = py0; t.px0 = px0; t.nrow = std::min(nrow, D.ph - py0);
                t.sr0 = r0; t.nsr = r1 - r0 + 1;
                t.sc0 = (c0 + kEdge) & ~3;
                t.nsw = (c1 + kEdge - t.sc0) / 4 + 1;
                return (size_t)t.nsr * t.nsw * 4 <= (size_t)kPyrLdsMax;
            };
            int nrow = kPyrTileH[v];
            for (bool ok = false; !ok;) {
                ok = true;
                for (int py0 = 0; py0 < D.ph && ok; py0 += nrow)
                    for (int px0 = 0; px0 < D.pitch && ok; px0 += PT_W) {
                        PyrTile t;
                        ok = make(py0, px0, nrow, t);
                    }
                if (!ok && --nrow < 1) return -1;
            }
            size_t lds = 0;
            for (int py0 = 0; py0 < D.ph; py0 += nrow)
                for (int px0 = 0; px0 < D.pitch; px0 += PT_W) {
                    PyrTile t;
                    make(py0, px0, nrow, t);
                    if ((size_t)(t.sc0 + 4 * t.nsw) > (size_t)levels_[l - 1].pitch) return -1;
                    lds = std::max(lds, (size_t)t.nsr * t.nsw * 4);
                    ptiles_.push_back(t);
                }
            plds_[v * nlevels_ + l] = (int)lds;
            ptile_th_[v * nlevels_ + l] = nrow;
            ptile_n_[v * nlevels_ + l] = (int)ptiles_.size() - ptile_begin_[v * (nlevels_ + 1) + l];
          }
        }
        yrAll[l] = yr;
        xofsAll_[l] = xofs;
        xalAll_[l] = xal;
        tab_off_[l][0] = push(xofs.data(), xofs.size() * 4);
        tab_off_[l][1] = push(xal.data(), xal.size() * 2);
        tab_off_[l][2] = push(yr.data(), yr.size() * 4);
        tab_off_[l][3] = push(yb.data(), yb.size() * 2);
    }
    if (plan_chain(yrAll)) return -1;
    // (re)allocate device buffers for maxB_
    auto F = [](void*& p) { if (p) (void)hipFree(p); p = nullptr; };
    F(d_pyr_); F(d_blur_); F(d_slots_); F(d_counts_); F(d_cells_); F(d_tiles_); F(d_lcb_); F(d_work_); F(d_groups_);
    F(d_cellslot_);
    work_B_ = -1;
    F(d_packed_); F(d_hdr_); F(d_sel_); F(d_levels_); F(d_tabs_); F(d_ptiles_);
    const int B = maxB_;
    if (d_chain_) (void)hipFree(d_chain_);
    d_chain_ = nullptr;
    if (chain_) {
        ORB_HIP_CHECK(hipMalloc(&d_chain_, chainTab_.size()));
        ORB_HIP_CHECK(hipMemcpy(d_chain_, chainTab_.data(), chainTab_.size(), hipMemcpyHostToDevice));
    }
    ORB_HIP_CHECK(hipMalloc(&d_ptiles_, std::max<size_t>(ptiles_.size(), 1) * sizeof(PyrTile)));
    if (!ptiles_.empty())
        ORB_HIP_CHECK(hipMemcpy(d_ptiles_, ptiles_.data(), ptiles_.size() * sizeof(PyrTile), hipMemcpyHostToDevice));
    // k_pyr_flow: band counters (level 0 in bands of the variant's tile height)
    if (d_flowcnt_) (void)hipFree(d_flowcnt_);
    d_flowcnt_ = nullptr;
    for (int v = 0; v < 2; v++) {
        ptile_th_[v * nlevels_] = kPyrTileH[v];
        int nb = 0, lds = 0;
        for (int l = 0; l < nlevels_; l++) {
            nb += (levels_[l].ph + ptile_th_[v * nlevels_ + l] - 1) / ptile_th_[v * nlevels_ + l];
            lds = std::max(lds, plds_[v * nlevels_ + l]);
        }
        flowBands_[v] = nb;
        flowLds_[v] = lds;
    }
    ORB_HIP_CHECK(hipMalloc(&d_flowcnt_, (size_t)std::max(flowBands_[0], flowBands_[1]) * B * 4));
    ORB_HIP_CHECK(hipMalloc(&d_pyr_, img_bytes_ * B));
    ORB_HIP_CHECK(hipMalloc(&d_blur_, blur_bytes_ * B));
    ORB_HIP_CHECK(hipMemset(d_blur_, 0, blur_bytes_ * B));
    ORB_HIP_CHECK(hipMalloc(&d_slots_, slots_per_image_ * 4 * B));
    ORB_HIP_CHECK(hipMalloc(&d_counts_, cells_.size() * 4 * B));
    ORB_HIP_CHECK(hipMalloc(&d_cells_, cells_.size() * sizeof(CellDesc)));
    ORB_HIP_CHECK(hipMemcpy(d_cells_, cells_.data(), cells_.size() * sizeof(CellDesc), hipMemcpyHostToDevice));
    ORB_HIP_CHECK(hipMalloc(&d_groups_, groups_.size() * sizeof(CellGroup)));
    ORB_HIP_CHECK(hipMemcpy(d_groups_, groups_.data(), groups_.size() * sizeof(CellGroup), hipMemcpyHostToDevice));
    ORB_HIP_CHECK(hipMalloc(&d_tiles_, tiles_.size() * sizeof(BlurTile)));
    ORB_HIP_CHECK(hipMemcpy(d_tiles_, tiles_.data(), tiles_.size() * sizeof(BlurTile), hipMemcpyHostToDevice));
    {
        std::vector<int> cs(cells_.size());
        for (size_t c = 0; c < cells_.size(); c++) cs[c] = cells_[c].slot_off;
        ORB_HIP_CHECK(hipMalloc(&d_cellslot_, std::max<size_t>(cs.size(), 1) * 4));
        ORB_HIP_CHECK(hipMemcpy(d_cellslot_, cs.data(), cs.size() * 4, hipMemcpyHostToDevice));
    }
    ORB_HIP_CHECK(hipMalloc(&d_lcb_, level_cell_begin_.size() * 4));
    ORB_HIP_CHECK(hipMemcpy(d_lcb_, level_cell_begin_.data(), level_cell_begin_.size() * 4, hipMemcpyHostToDevice));
    if (slots_per_image_ * B > ((size_t)1 << 30)) return -1;   // k_octree's per-level ranges of packed
    packed_cap_ = (int)(slots_per_image_ * B);
    ORB_HIP_CHECK(hipMalloc(&d_packed_, (size_t)packed_cap_ * 4));
    ORB_HIP_CHECK(hipMalloc(&d_hdr_, (size_t)B * (nlevels_ + 2) * 4 + 64));
    d_gtotal_ = (int*)((char*)d_hdr_ + (size_t)B * (nlevels_ + 2) * 4);
    d_gtotal_alias_ = true;
    sel_cap_ = B * std::max(nfeatures_ * 2 + 64, 256);
    ORB_HIP_CHECK(hipMalloc(&d_sel_, (size_t)sel_cap_ * sizeof(int2)));
    std::vector<LevelDev> ld(nlevels_);
    for (int l = 0; l < nlevels_; l++) {
        ld[l].off = levels_[l].off;
        ld[l].pitch = levels_[l].pitch;
        ld[l].scale = scale_[l];
        ld[l].boff = levels_[l].boff;
        ld[l].bpitch = levels_[l].bpitch;
        ld[l].kp_size = (float)(int)(kPatch * scale_[l]);
    }
    if (nlevels_ > kMaxLevels) return -1;
    for (int l = 0; l < nlevels_; l++) levelArgs_.lv[l] = ld[l];
    ORB_HIP_CHECK(hipMalloc(&d_levels_, ld.size() * sizeof(LevelDev)));
    ORB_HIP_CHECK(hipMemcpy(d_levels_, ld.data(), ld.size() * sizeof(LevelDev), hipMemcpyHostToDevice));
    ORB_HIP_CHECK(hipMalloc(&d_tabs_, std::max<size_t>(tabs.size(), 16)));
    if (!tabs.empty()) ORB_HIP_CHECK(hipMemcpy(d_tabs_, tabs.data(), tabs.size(), hipMemcpyHostToDevice));
    // device octree: jobs (image, level), per-job capacity N_l + 8 (phase 2 stops within N + 3)
    F(d_jobsel_); F(d_jobcnt_); F(d_octlv_); F(d_gscr_); F(d_nout_);
    jcap_ = 0;
    std::vector<OctLevelDev> ol(nlevels_);
    for (int l = 0; l < nlevels_; l++) {
        ol[l].minX = kEdge - 3;
        ol[l].maxX = levels_[l].w - kEdge + 3;
        ol[l].minY = kEdge - 3;
        ol[l].maxY = levels_[l].h - kEdge + 3;
        ol[l].N = nPerLevel_[l];
        jcap_ = std::max(jcap_, nPerLevel_[l] + 8);
    }
    if (jcap_ > kOctNMax) return -1;   // nFeaturesPerLevel beyond the device octree's node pool
    selcap_ = jcap_ * nlevels_;
    ORB_HIP_CHECK(hipMalloc(&d_octlv_, ol.size() * sizeof(OctLevelDev)));
    ORB_HIP_CHECK(hipMemcpy(d_octlv_, ol.data(), ol.size() * sizeof(OctLevelDev), hipMemcpyHostToDevice));
    ORB_HIP_CHECK(hipMalloc(&d_jobsel_, (size_t)B * nlevels_ * jcap_ * 4));
    ORB_HIP_CHECK(hipMalloc(&d_jobcnt_, (size_t)B * nlevels_ * 4));
    ORB_HIP_CHECK(hipMalloc(&d_gscr_, (size_t)packed_cap_ * 3 * 2));
    ORB_HIP_CHECK(hipMalloc(&d_nout_, (size_t)(B + 1) * 4));
    ORB_HIP_CHECK(hipFree(d_sel_));
    d_sel_ = nullptr;
    sel_cap_ = selcap_ * B;
    ORB_HIP_CHECK(hipMalloc(&d_sel_, (size_t)sel_cap_ * sizeof(int2)));
    if (h_nout_) (void)hipHostFree(h_nout_);
    ORB_HIP_CHECK(hipHostMalloc((void**)&h_nout_, (size_t)(B + 1) * 4));
    geomW_ = W;
    geomH_ = H;
    return 0;
}

int Extractor::extract(const uint8_t* imgs, int B, int W, int H, int step, size_t img_stride,
                       bool imgs_on_device, orb_kp* kps, uint8_t* desc, int cap, bool out_on_device,
                       int* n_out, const uint8_t* const* list) {
    if (B <= 0 || B > maxB_ || W <= 0 || H <= 0) return -1;
    if (W > maxW_ || H > maxH_) return -1;
    if (int e = setup_geometry(W, H)) return e;
    hipStream_t s = stream_;
    const uint8_t* src = imgs;
    if (!imgs_on_device) {
        const size_t need = img_stride * (B - 1) + (size_t)step * (H - 1) + W;
        if (need > in_cap_) {
            if (d_in_) (void)hipFree(d_in_);
            ORB_HIP_CHECK(hipMalloc(&d_in_, need));
            in_cap_ = need;
        }
        // the previous call's copy out of h_in_ is done once ev_[0] (recorded right after it) is
        if (h_in_) ORB_HIP_CHECK(hipEventSynchronize(ev_[0]));
        if (need > h_in_cap_) {
            if (h_in_) (void)hipHostFree(h_in_);
            h_in_ = nullptr;
            h_in_cap_ = 0;
            ORB_HIP_CHECK(hipHostMalloc(&h_in_, need));
            h_in_cap_ = need;
        }
        if (list) {   // separate host images (Frame's two cv::Mat): one staging block, one H2D copy
            const size_t one = (size_t)step * (H - 1) + W;
            for (int b = 0; b < B; b++) std::memcpy((uint8_t*)h_in_ + img_stride * b, list[b], one);
        } else {
            std::memcpy(h_in_, imgs, need);
        }
        ORB_HIP_CHECK(hipMemcpyAsync(d_in_, h_in_, need, hipMemcpyHostToDevice, s));
        src = (const uint8_t*)d_in_;
    }
    ORB_HIP_CHECK(hipEventRecord(ev_[0], s));
    const int ncells = (int)cells_.size();
    if (work_B_ != B && build_work(B)) return -2;
    const bool split = fastSplit_ && work_part_[0] > 0 && work_part_[1] > 0;
    // 1. pyramid; with the split, FAST of the levels below kFastSplitLevel starts on side_ as soon
    //    as they are built (their cells read nothing else), beside the small levels' chain
    {
        const LevelHost& L0 = levels_[0];
        const int n = (L0.pitch / 16) * L0.ph;
        const bool flow = flow_ && !split && !chain_;
        if (flow) {
            // every level in one launch (k_pyr_flow); its band counters zeroed first
            const int v = B >= 8 ? 1 : 0;
            ORB_HIP_CHECK(hipMemsetAsync(d_flowcnt_, 0, (size_t)flowBands_[v] * B * 4, s));
            const FlowArgs A = flow_args(v, B);
            int tasks = 0;
            for (int l = 0; l < nlevels_; l++) tasks += B * A.L[l].ntiles;
            auto kern = v ? k_pyr_flow<kPyrTileH[1]> : k_pyr_flow<kPyrTileH[0]>;
            hipLaunchKernelGGL(kern, dim3(tasks), dim3(256), flowLds_[v], s, src, img_stride, step, W, H,
                               (uint8_t*)d_pyr_, img_bytes_, A, (const PyrTile*)d_ptiles_, (const uint8_t*)d_tabs_,
                               d_flowcnt_, 1, d_gtotal_, (int*)d_nout_ + B);
        } else {
            hipLaunchKernelGGL(k_pyr_level0, dim3((n + 255) / 256, B), dim3(256), 0, s, src, img_stride, step, W, H,
                               (uint8_t*)d_pyr_, img_bytes_, L0.pitch, L0.ph, d_gtotal_, (int*)d_nout_ + B);
        }
        const int lend = flow ? 1 : chain_ && !split ? chainFrom_ : nlevels_;   // levels [1, lend) one launch each
        for (int l = 1; l < lend; l++) {
            if (split && l == kFastSplitLevel) {
                ORB_HIP_CHECK(hipEventRecord(evPyrA_, s));
                ORB_HIP_CHECK(hipStreamWaitEvent(side_, evPyrA_, 0));
                hipLaunchKernelGGL(k_fast_cells, dim3(work_part_[0]), dim3(256), 0, side_, (const uint8_t*)d_pyr_,
                                   img_bytes_, (const CellGroup*)d_groups_, iniTh_, minTh_, (uint32_t*)d_slots_,
                                   slots_per_image_, (int*)d_counts_, ncells, (const int*)d_work_);
                ORB_HIP_CHECK(hipEventRecord(evFastA_, side_));
            }
            const LevelHost& L = levels_[l];
            const LevelHost& P = levels_[l - 1];
            const uint8_t* T = (const uint8_t*)d_tabs_;
            const int v = B >= 8 ? 1 : 0, pb = v * (nlevels_ + 1) + l;
            const int nt = ptile_n_[v * nlevels_ + l];
            auto kern = v ? k_pyr_resize<kPyrTileH[1]> : k_pyr_resize<kPyrTileH[0]>;
            hipLaunchKernelGGL(kern, dim3(grid8(nt), B), dim3(256), plds_[v * nlevels_ + l], s, (uint8_t*)d_pyr_, img_bytes_,
                               P.off, P.pitch, L.off, L.pitch, L.ph, L.w, L.h,
                               (const int*)(T + tab_off_[l][0]), (const short2*)(T + tab_off_[l][1]),
                               (const int2*)(T + tab_off_[l][2]), (const short2*)(T + tab_off_[l][3]),
                               (const PyrTile*)d_ptiles_ + ptile_begin_[pb], nt);
        }
        if (!flow && lend < nlevels_) {
            const uint8_t* T = (const uint8_t*)d_chain_;
            const LevelHost& P = levels_[lend - 1];
            hipLaunchKernelGGL(k_pyr_chain, dim3(chainK_, B), dim3(256), chainLds_, s, (uint8_t*)d_pyr_, img_bytes_,
                               (long long)P.off, P.pitch, P.w, (const ChainLevel*)T, nlevels_ - lend,
                               (const int4*)(T + chainStripOff_), (const uint16_t*)(T + chainRowOff_),
                               (const uint8_t*)d_tabs_, chainSrcLds_, chainSrcRp_);
        }
    }
    ORB_HIP_CHECK(hipGetLastError());
    ORB_HIP_CHECK(hipEventRecord(ev_[1], s));
    // ORBGPU_BLUR_EARLY=1: the blur right after the pyramid on the extractor's own stream (A/B
    // of the pipelined bench: which tracking kernels the FAST grid then overlaps)
    static const bool blurEarly = [] {
        const char* e = getenv("ORBGPU_BLUR_EARLY");
        return e && e[0] == '1';
    }();
    if (blurEarly && !evBlur_)
        hipLaunchKernelGGL(k_blur7, dim3(grid8((int)tiles_.size()), B), dim3(256), 0, s, (const uint8_t*)d_pyr_,
                           (uint8_t*)d_blur_, img_bytes_, blur_bytes_, (const BlurTile*)d_tiles_, (int)tiles_.size());
    if (evBlur_) {
        ORB_HIP_CHECK(hipStreamWaitEvent(side_, ev_[1], 0));
        hipLaunchKernelGGL(k_blur7, dim3(grid8((int)tiles_.size()), B), dim3(256), 0, side_, (const uint8_t*)d_pyr_,
                           (uint8_t*)d_blur_, img_bytes_, blur_bytes_, (const BlurTile*)d_tiles_, (int)tiles_.size());
        ORB_HIP_CHECK(hipEventRecord(evBlur_, side_));
    }
    // 2. FAST per cell (the blur, which only the descriptors read, runs after the octree: the
    //    VALU-heavy FAST grid then overlaps the tracking lane's matching, and the HBM-bound
    //    blur its FP64 PoseOptimization)
    if (split) {
        hipLaunchKernelGGL(k_fast_cells, dim3(work_part_[1]), dim3(256), 0, s, (const uint8_t*)d_pyr_, img_bytes_,
                           (const CellGroup*)d_groups_, iniTh_, minTh_, (uint32_t*)d_slots_, slots_per_image_,
                           (int*)d_counts_, ncells, (const int*)d_work_ + work_part_[0]);
        ORB_HIP_CHECK(hipStreamWaitEvent(s, evFastA_, 0));
    } else {
        hipLaunchKernelGGL(k_fast_cells, dim3(work_n_), dim3(256), 0, s, (const uint8_t*)d_pyr_, img_bytes_,
                           (const CellGroup*)d_groups_, iniTh_, minTh_, (uint32_t*)d_slots_, slots_per_image_,
                           (int*)d_counts_, ncells, (const int*)d_work_);
    }
    ORB_HIP_CHECK(hipGetLastError());
    ORB_HIP_CHECK(hipEventRecord(ev_[3], s));
    // 3-4. per (image, level): compaction of the level's cell outputs, DistributeOctTree, then the
    //      per-image selected lists, on the device (k_octree compacts its own level)
    ORB_HIP_CHECK(hipEventRecord(ev_[4], s));
    int* d_err = (int*)d_nout_ + B;
    OctInput oin{(const uint32_t*)d_slots_, slots_per_image_, (const int*)d_counts_, (const int*)d_cellslot_,
                 (const int*)d_lcb_, ncells, (uint32_t*)d_packed_, d_gtotal_};
    if (int e = octree_launch(oin, B, nlevels_, (const OctLevelDev*)d_octlv_, (uint32_t*)d_jobsel_, (int*)d_jobcnt_,
                              jcap_, (uint16_t*)d_gscr_, (size_t)packed_cap_, cap, (int2*)d_sel_, selcap_,
                              (int*)d_nout_, d_err, s))
        return e;
    ORB_HIP_CHECK(hipEventRecord(ev_[5], s));
    // 5. blur: GaussianBlur of every level (ORBextractor.cc:1085-1086); on the side stream it
    //    was launched after the pyramid
    if (evBlur_)
        ORB_HIP_CHECK(hipStreamWaitEvent(s, evBlur_, 0));
    else if (!blurEarly)
        hipLaunchKernelGGL(k_blur7, dim3(grid8((int)tiles_.size()), B), dim3(256), 0, s, (const uint8_t*)d_pyr_,
                           (uint8_t*)d_blur_, img_bytes_, blur_bytes_, (const BlurTile*)d_tiles_, (int)tiles_.size());
    ORB_HIP_CHECK(hipEventRecord(ev_[2], s));
    // 6. orientation + descriptors
    orb_kp_dev* okps = (orb_kp_dev*)kps;
    uint8_t* odesc = desc;
    if (!out_on_device) {
        const size_t nk = (size_t)B * cap;
        if (nk > out_cap_) {
            if (d_kps_) (void)hipFree(d_kps_);
            if (d_desc_) (void)hipFree(d_desc_);
            ORB_HIP_CHECK(hipMalloc(&d_kps_, nk * sizeof(orb_kp_dev)));
            ORB_HIP_CHECK(hipMalloc(&d_desc_, nk * 32));
            out_cap_ = nk;
        }
        okps = (orb_kp_dev*)d_kps_;
        odesc = (uint8_t*)d_desc_;
    }
    {
        const int gx = (selcap_ + 3) / 4;
        const int nwg = B >= 8 ? gx * 8 * ((B + 7) / 8) : gx * B;
        hipLaunchKernelGGL(k_orient_desc, dim3(nwg), dim3(256), 0, s, (const uint8_t*)d_pyr_,
                           (const uint8_t*)d_blur_, img_bytes_, blur_bytes_, (const int2*)d_sel_, selcap_,
                           (const int*)d_nout_, levelArgs_, okps, odesc, cap, gx, B);
    }
    ORB_HIP_CHECK(hipGetLastError());
    ORB_HIP_CHECK(hipMemcpyAsync(h_nout_, d_nout_, (size_t)(B + 1) * 4, hipMemcpyDeviceToHost, s));
    ORB_HIP_CHECK(hipEventRecord(ev_[6], s));
    ORB_HIP_CHECK(stream_wait(s));
    const int err = h_nout_[B];
    for (int b = 0; b < B; b++) n_out[b] = h_nout_[b];
    if (err & 1) return -3;   // keypoints beyond `cap` (or the selection capacity)
    if (err) return -1;
    if (!out_on_device) {
        for (int b = 0; b < B; b++) {
            if (n_out[b] == 0) continue;
            ORB_HIP_CHECK(hipMemcpyAsync(kps + (size_t)b * cap, okps + (size_t)b * cap, (size_t)n_out[b] * sizeof(orb_kp_dev),
                                         hipMemcpyDeviceToHost, s));
            ORB_HIP_CHECK(hipMemcpyAsync(desc + (size_t)b * cap * 32, odesc + (size_t)b * cap * 32, (size_t)n_out[b] * 32,
                                         hipMemcpyDeviceToHost, s));
        }
        ORB_HIP_CHECK(stream_wait(s));
    }
    last_B_ = B;
    return 0;
}

int Extractor::corner_total(long long* total) {
    if (last_B_ <= 0 || !d_gtotal_) return -1;
    int v = 0;   // k_octree's atomic total over the batch (d_gtotal_), read after the call
    ORB_HIP_CHECK(hipStreamSynchronize(stream_));
    ORB_HIP_CHECK(hipMemcpy(&v, d_gtotal_, 4, hipMemcpyDeviceToHost));
    *total = v;
    return 0;
}

int Extractor::get_blurred(int index, int level, uint8_t* dst, int dst_step, int* w, int* h) {
    if (level < 0 || level >= nlevels_ || index < 0 || index >= last_B_ || !d_blur_) return -1;
    const LevelHost& L = levels_[level];
    *w = L.w;
    *h = L.h;
    if (!dst) return 0;
    ORB_HIP_CHECK(hipMemcpy2D(dst, dst_step, (const uint8_t*)d_blur_ + (size_t)index * blur_bytes_ + L.boff, L.bpitch,
                              L.w, L.h, hipMemcpyDeviceToHost));
    return 0;
}

int debug_prof_extract(unsigned long long* out32) {
#ifdef ORBGPU_PROF
    ORB_HIP_CHECK(hipMemcpyFromSymbol(out32, HIP_SYMBOL(g_orbgpu_prof), sizeof(unsigned long long) * 16));
    unsigned long long z[32] = {};
    ORB_HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_orbgpu_prof), z, sizeof(z)));
    return octree_prof_read(out32 + 16);   // slots 16-31: k_octree's sections (octree.hip)
#else
    (void)out32;
    return -1;
#endif
}

int Extractor::timings(float* ms6) {
    float t[6] = {0};
    // launch order: pyramid [0,1] fast [1,3] compact [3,4] octree [4,5] blur [5,2] orient [2,6]
    (void)hipEventElapsedTime(&t[0], ev_[0], ev_[1]);
    (void)hipEventElapsedTime(&t[1], ev_[5], ev_[2]);
    (void)hipEventElapsedTime(&t[2], ev_[1], ev_[3]);
    (void)hipEventElapsedTime(&t[3], ev_[3], ev_[4]);
    (void)hipEventElapsedTime(&t[4], ev_[4], ev_[5]);
    (void)hipEventElapsedTime(&t[5], ev_[2], ev_[6]);
    for (int i = 0; i < 6; i++) ms6[i] = t[i];
    return 0;
}

int Extractor::get_level(int index, int level, uint8_t* dst, int dst_step, int* w, int* h) {
    if (level < 0 || level >= nlevels_ || index < 0 || index >= last_B_ || !d_pyr_) return -1;
    const LevelHost& L = levels_[level];
    *w = L.w;
    *h = L.h;
    if (!dst) return 0;
    ORB_HIP_CHECK(hipMemcpy2D(dst, dst_step, (const uint8_t*)d_pyr_ + (size_t)index * img_bytes_ + L.off, L.pitch,
                              L.pw, L.ph, hipMemcpyDeviceToHost));
    return 0;
}

}  // namespace orbgpu
