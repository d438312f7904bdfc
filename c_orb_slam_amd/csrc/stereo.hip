// stereo.hip -- gfx950 Frame::ComputeStereoMatches (reference src/Frame.cc:466-640).
//
// Rectified stereo: for every left keypoint the best right keypoint (256-bit Hamming) among
// those whose row band (y +- 2 * scale) covers the left row, octave within +-1 and u_R in
// [u_L - bf/b, u_L]; then an 11x11 SAD over +-5 pixel shifts on the padded pyramid level of
// the left octave, a parabola through the best three SADs, depth = bf / disparity, and the
// 2.1 x median SAD outlier filter.  No occupancy: every left keypoint is independent.
//
//   k_stereo_match   one 16-lane group per left keypoint (16 per workgroup), all pairs of the
//                    batch in one launch (grid.y = pair): lanes sweep the right keypoints in
//                    index order with popcount distances, a group min over (dist, iR) picks the
//                    reference's first strict minimum; the 11 SADs are integer group sums
//                    (cv::norm of centred integer windows is exact), the parabola and the
//                    disparity follow the reference's float expression order.
//   k_stereo_filter  one workgroup per pair: the median of the kept SADs by a two-level LDS
//                    histogram select, thDist = 1.5f*1.4f*median, invalidation of SAD >= thDist.
#include "stereo.hpp"
#include "orb_match.hpp"

#include <algorithm>
#include <climits>
#include <cstring>

namespace orbgpu {


// vRowIndices (Frame.cc:476-493) as a CSR per pair: right keypoint iR is listed on every row
// yi in [floor(y - r), ceil(y + r)], r = 2 * mvScaleFactors[octave].  The order inside a row
// does not matter: the match kernel takes the minimum of (dist, iR).  An entry carries what the
// scan filters on (uR, octave) beside iR, so the match kernel reads a row's entries as one
// contiguous run instead of gathering every candidate's 28-byte keypoint.
__global__ void __launch_bounds__(1024) k_stereo_rows(const StereoDev* __restrict__ probs, StereoParams P) {
    ORBGPU_LATENCY_WAVE();
    const StereoDev& S = probs[blockIdx.x];
    __shared__ int s_cnt[kStereoMaxRows];
    __shared__ int s_w[16];
    const int tid = threadIdx.x, rows = P.rows0;
    for (int y = tid; y < rows; y += 1024) s_cnt[y] = 0;
    __syncthreads();
    for (int iR = tid; iR < S.NR; iR += 1024) {
        const orb_kp_dev kp = S.kR[iR];
        const float r = 2.0f * P.scale[kp.octave];
        const int maxr = min((int)ceilf(kp.y + r), rows - 1), minr = max((int)floorf(kp.y - r), 0);
        for (int y = minr; y <= maxr; y++) atomicAdd(&s_cnt[y], 1);
    }
    __syncthreads();
    // exclusive scan of the row counts (rows <= 4096: 4 per thread)
    const int lane = tid & 63, wid = tid >> 6;
    int v[4], loc = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int y = 4 * tid + k;
        v[k] = y < rows ? s_cnt[y] : 0;
        loc += v[k];
    }
    int incl = loc;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int t = __shfl_up(incl, o, 64);
        if (lane >= o) incl += t;
    }
    if (lane == 63) s_w[wid] = incl;
    __syncthreads();
    int off = 0;
    for (int w = 0; w < wid; w++) off += s_w[w];
    int run = off + incl - loc;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int y = 4 * tid + k;
        if (y < rows) {
            S.rowStart[y] = run;
            s_cnt[y] = run;   // fill cursor
        }
        run += v[k];
    }
    if (tid == 1023) S.rowStart[rows] = run;
    __syncthreads();
    for (int iR = tid; iR < S.NR; iR += 1024) {
        const orb_kp_dev kp = S.kR[iR];
        const float r = 2.0f * P.scale[kp.octave];
        const int maxr = min((int)ceilf(kp.y + r), rows - 1), minr = max((int)floorf(kp.y - r), 0);
        const int2 ent = make_int2(__float_as_int(kp.x), iR | (kp.octave << 24));
        for (int y = minr; y <= maxr; y++) S.rowIdx[atomicAdd(&s_cnt[y], 1)] = ent;
    }
}

// sums / minima over the 16 lanes of a group (lanes 16g .. 16g+15 of the wave)
__device__ __forceinline__ int group_sum_i(int v) {
#pragma unroll
    for (int o = 8; o >= 1; o >>= 1) v += __shfl_xor(v, o, 16);
    return v;
}

__device__ __forceinline__ unsigned group_min_u(unsigned v) {
#pragma unroll
    for (int o = 8; o >= 1; o >>= 1) v = min(v, (unsigned)__shfl_xor((int)v, o, 16));
    return v;
}

// One 16-lane group per left keypoint (16 keypoints per 256-thread workgroup, 4 per wave): the
// row candidates 16 at a time, the 121 window pixels 8 per lane, the SADs as group sums.  All
// reductions are integer minima / sums, so the result does not depend on the lane mapping.
__global__ void __launch_bounds__(256) k_stereo_match(const StereoDev* __restrict__ probs, StereoParams P,
                                                      unsigned long long* counters, int np, int gx) {
    ORBGPU_LATENCY_WAVE();
    // XCD-aware order (xcd_problem_block): every workgroup of a pair runs on one XCD, so the
    // pair's right keypoints and descriptors, which all its left keypoints scan, and its pyramid
    // rows are fetched into one L2
    int by, bx;
    if (!xcd_problem_block(np, gx, by, bx)) return;
    const StereoDev& S = probs[by];
    const int sub = threadIdx.x & 15;
    const int iL = bx * 16 + (threadIdx.x >> 4);
    if (iL >= S.NL) return;   // the whole group
    const orb_kp_dev kpL = S.kL[iL];
    float uR_out = -1.0f, depth_out = -1.0f;
    int sad_out = -1;
    const int levelL = kpL.octave;
    const float vL = kpL.y, uL = kpL.x;
    const int row = (int)vL;                                  // vRowIndices[vL]
    const float minZ = P.mb, minD = 0.0f, maxD = P.mbf / minZ;
    const float minU = uL - maxD, maxU = uL - minD;
    if (row >= 0 && row < P.rows0 && !(maxU < 0)) {
        // best right keypoint among the row's candidates: first strict minimum below TH_HIGH in iR order
        const uint32_t* dl = (const uint32_t*)(S.dL + 32 * (size_t)iL);   // descriptors: 4-B aligned rows
        uint32_t q[8];
#pragma unroll
        for (int k = 0; k < 8; k++) q[k] = dl[k];
        unsigned best = 0xffffffffu;
        int scored = 0;
        const int c1 = S.rowStart[row + 1];
        for (int c = S.rowStart[row] + sub; c < c1; c += 16) {
            const int2 ent = S.rowIdx[c];
            const int iR = ent.y & 0xffffff, octR = ent.y >> 24;
            if (octR < levelL - 1 || octR > levelL + 1) continue;
            const float uR = __int_as_float(ent.x);
            if (!(uR >= minU && uR <= maxU)) continue;
            const uint32_t* dr = (const uint32_t*)(S.dR + 32 * (size_t)iR);
            int dist = 0;
#pragma unroll
            for (int k = 0; k < 8; k++) dist += __popc(q[k] ^ dr[k]);
            if (dist < 100) best = min(best, ((unsigned)dist << 16) | (unsigned)iR);
            scored++;
        }
        best = group_min_u(best);
        if (counters) {   // measurement: scored (left, right) pairs and searched left keypoints
            const int tot = group_sum_i(scored);
            if (sub == 0) {   // spread over kCountSlots addresses: one per group would serialise
                const int sl = (bx + by * 7 + (threadIdx.x >> 4)) & (kCountSlots - 1);
                atomicAdd(&counters[2 * kCountSlots + sl], (unsigned long long)tot);
                atomicAdd(&counters[3 * kCountSlots + sl], 1ull);
            }
        }
        const int bestDist = best == 0xffffffffu ? 100 : (int)(best >> 16);
        const int bestIdxR = (int)(best & 0xffffu);
        if (bestDist < 75) {   // thOrbDist = (TH_HIGH + TH_LOW) / 2
            const float uR0 = S.kR[bestIdxR].x;
            const float scaleFactor = P.invScale[levelL];
            const float scaleduL = roundf(kpL.x * scaleFactor);
            const float scaledvL = roundf(kpL.y * scaleFactor);
            const float scaleduR0 = roundf(uR0 * scaleFactor);
            const int w = 5, L = 5;
            const StereoLevel lv = P.lv[levelL];
            const float iniu = scaleduR0 + L - w, endu = scaleduR0 + L + w + 1;
            if (!(iniu < 0 || endu >= lv.w)) {
                if (counters && sub == 0)   // measurement: keypoints whose SAD windows are read
                    atomicAdd(&counters[7 * kCountSlots + ((bx + by * 7 + (threadIdx.x >> 4)) & (kCountSlots - 1))],
                              1ull);
                const uint8_t* IL = S.pyrL + lv.off + (size_t)kEdge * lv.pitch + kEdge;
                const uint8_t* IR = S.pyrR + lv.off + (size_t)kEdge * lv.pitch + kEdge;
                const int yL = (int)scaledvL, xL = (int)scaleduL, xR0 = (int)scaleduR0;
                const int cL = IL[(ptrdiff_t)yL * lv.pitch + xL];
                // lane owns window pixels p = sub + 16 t (p < 121)
                int a[8], offv[8];
#pragma unroll
                for (int t = 0; t < 8; t++) {
                    const int p = sub + 16 * t;
                    const int dy = p / 11 - 5, dx = p % 11 - 5;
                    offv[t] = (yL + dy) * lv.pitch + dx;
                    a[t] = p < 121 ? IL[(ptrdiff_t)offv[t] + xL] - cL : 0;
                }
                int vD[11];
#pragma unroll
                for (int inc = 0; inc < 11; inc++) {
                    const int xR = xR0 + inc - L;
                    const int cR = IR[(ptrdiff_t)yL * lv.pitch + xR];
                    int sacc = 0;
#pragma unroll
                    for (int t = 0; t < 8; t++) {
                        const int p = sub + 16 * t;
                        if (p < 121) sacc += abs(a[t] - (IR[(ptrdiff_t)offv[t] + xR] - cR));
                    }
                    vD[inc] = group_sum_i(sacc);
                }
                int bestD = INT_MAX, bestinc = 0;
#pragma unroll
                for (int inc = 0; inc < 11; inc++)
                    if (vD[inc] < bestD) {
                        bestD = vD[inc];
                        bestinc = inc - L;
                    }
                if (bestinc != -L && bestinc != L) {
                    const float dist1 = (float)vD[L + bestinc - 1];
                    const float dist2 = (float)vD[L + bestinc];
                    const float dist3 = (float)vD[L + bestinc + 1];
                    const float deltaR = (dist1 - dist3) / (2.0f * (dist1 + dist3 - 2.0f * dist2));
                    if (!(deltaR < -1 || deltaR > 1)) {
                        float bestuR = P.scale[levelL] * ((float)scaleduR0 + (float)bestinc + deltaR);
                        float disparity = (uL - bestuR);
                        if (disparity >= minD && disparity < maxD) {
                            if (disparity <= 0) {
                                disparity = (float)0.01;
                                bestuR = (float)((double)uL - 0.01);
                            }
                            depth_out = P.mbf / disparity;
                            uR_out = bestuR;
                            sad_out = bestD;
                        }
                    }
                }
            }
        }
    }
    if (sub == 0) {
        S.uRight[iL] = uR_out;
        S.depth[iL] = depth_out;
        S.sad[iL] = sad_out;
    }
}

// median filter (Frame.cc:624-639): the reference sorts the kept SADs, takes the middle one,
// thDist = 1.5f*1.4f*median, and invalidates SAD >= thDist walking the sorted tail from the end.
// 4 waves and 1 KB of LDS: the workgroup fits in the slot of one retiring extraction workgroup
// (1,024 threads + 16 KB waited ~3x longer)
// The median is vDistIdx[n/2] of the sorted SADs, i.e. the (n/2)-th smallest kept SAD: a radix
// select over two LDS histograms (SAD >> 7, then SAD & 127 inside the bucket that holds rank
// n/2) instead of sorting.  A SAD is a sum of 121 absolute byte differences: < 2^15.
__device__ __forceinline__ void stereo_select_bucket(const int* hist, int nb, int rank, int* out_bin, int* out_rank) {
    // one wave: lane l holds bins 4l..4l+3 (nb <= 256); the bin where the running count passes rank
    const int lane = threadIdx.x;
    int c[4], loc = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        c[k] = 4 * lane + k < nb ? hist[4 * lane + k] : 0;
        loc += c[k];
    }
    int incl = loc;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int t = __shfl_up(incl, o, 64);
        if (lane >= o) incl += t;
    }
    int run = incl - loc;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        if (run <= rank && rank < run + c[k]) {
            *out_bin = 4 * lane + k;
            *out_rank = rank - run;
        }
        run += c[k];
    }
}

__global__ void __launch_bounds__(256) k_stereo_filter(const StereoDev* __restrict__ probs) {
    ORBGPU_LATENCY_WAVE();
    const StereoDev& S = probs[blockIdx.x];
    __shared__ int hist[256];
    __shared__ int cnt, kept, bin, rnk;
    const int tid = threadIdx.x;
    hist[tid] = 0;
    if (tid == 0) cnt = 0;
    __syncthreads();
    int mine = 0;
    for (int i = tid; i < S.NL; i += blockDim.x) {
        const int d = S.sad[i];
        if (d >= 0) {
            atomicAdd(&hist[d >> 7], 1);
            mine++;
        }
    }
    if (mine) atomicAdd(&cnt, mine);
    __syncthreads();
    const int n = cnt;
    if (n == 0) {   // empty vDistIdx is UB in the reference; nothing to filter
        if (tid == 0) *S.kept = 0;
        return;
    }
    if (tid < 64) stereo_select_bucket(hist, 256, n / 2, &bin, &rnk);
    __syncthreads();
    const int hb = bin, r2 = rnk;
    __syncthreads();
    hist[tid] = 0;
    __syncthreads();
    for (int i = tid; i < S.NL; i += blockDim.x) {
        const int d = S.sad[i];
        if (d >= 0 && (d >> 7) == hb) atomicAdd(&hist[d & 127], 1);
    }
    __syncthreads();
    if (tid < 64) stereo_select_bucket(hist, 128, r2, &bin, &rnk);
    __syncthreads();
    const float median = (float)(hb * 128 + bin);
    const float thDist = 1.5f * 1.4f * median;
    if (tid == 0) kept = n;
    __syncthreads();
    for (int i = tid; i < S.NL; i += blockDim.x) {
        const int d = S.sad[i];
        if (d >= 0 && !((float)d < thDist)) {
            S.uRight[i] = -1.0f;
            S.depth[i] = -1.0f;
            atomicSub(&kept, 1);
        }
    }
    __syncthreads();
    if (tid == 0) *S.kept = kept;
}

int stereo_launch(const StereoDev* d_probs, int nprob, int maxNL, const StereoParams& P, hipStream_t s, Matcher* tm) {
    if (nprob <= 0) return 0;
    const bool timed = tm && tm->timing();
    if (timed) {
        if (int e = tm->zero_counters(2, 2)) return e;
        if (int e = tm->zero_counters(7, 1)) return e;
        tm->mark(4);
    }
    hipLaunchKernelGGL(k_stereo_rows, dim3(nprob), dim3(1024), 0, s, d_probs, P);
    if (timed) tm->mark(5);
    if (maxNL > 0)
        hipLaunchKernelGGL(k_stereo_match, xcd_grid((maxNL + 15) / 16, nprob), dim3(256), 0, s, d_probs, P,
                           timed ? tm->counters() : nullptr, nprob, (maxNL + 15) / 16);
    if (timed) tm->mark(6);
    hipLaunchKernelGGL(k_stereo_filter, dim3(nprob), dim3(256), 0, s, d_probs);
    if (timed) tm->mark(7);
    ORB_HIP_CHECK(hipGetLastError());
    return 0;
}

// ------------------------------------------------------------ UnprojectStereo
// x3Dc = ((u-cx)*z*invfx, (v-cy)*z*invfy, z) in float, then mRwc*x3Dc + mOw as one cv::gemm
// (the matcher's convention: f64 accumulation, one rounding to float).  One thread per keypoint.
// The frames travel as kernel arguments (kUnprojPerLaunch per launch), so an asynchronous call
// leaves no host or device staging buffer behind.
struct UnprojBatch {
    UnprojDev p[kUnprojPerLaunch];
};

__global__ void __launch_bounds__(256) k_unproject(UnprojBatch B) {
    ORBGPU_LATENCY_WAVE();
    const UnprojDev& P = B.p[blockIdx.y];
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P.N) return;
    const float z = P.depth[i];
    if (P.mp) P.mp[i] = z > 0 ? P.mp_base + i : -1;
    if (!(z > 0)) return;
    const orb_kp_dev kp = P.keys[i];
    const float x = (kp.x - P.cx) * z * P.invfx;
    const float y = (kp.y - P.cy) * z * P.invfy;
    const float* T = P.Twc;
    float X[3];
#pragma unroll
    for (int r = 0; r < 3; r++) {
        const double acc = (double)T[r * 4 + 0] * x + (double)T[r * 4 + 1] * y + (double)T[r * 4 + 2] * z;
        X[r] = (float)(acc + (double)T[r * 4 + 3]);
        P.x3D[3 * i + r] = X[r];
    }
    if (P.normal) {
        // MapPoint::UpdateNormalAndDepth with the creating frame as the only observation
        // (MapPoint.cc:331-371): cv::norm accumulated in double, normali / norm as a float
        // scale of the float vector, mfMaxDistance = dist * mvScaleFactors[octave]
        const float PO[3] = {X[0] - T[3], X[1] - T[7], X[2] - T[11]};
        const double s2 = ((double)PO[0] * PO[0] + (double)PO[1] * PO[1]) + (double)PO[2] * PO[2];
        const double nd = sqrt(s2);
        const float inv = (float)(1.0 / nd);
#pragma unroll
        for (int r = 0; r < 3; r++) P.normal[3 * i + r] = PO[r] * inv;
        const float dist = (float)nd;
        const int lv = min(max(kp.octave, 0), P.nlevels - 1);
        const float mx = dist * P.scale[lv];
        P.maxDist[i] = mx;
        P.minDist[i] = mx / P.scale[P.nlevels - 1];
    }
}

// Tracking.cc:893-913 (TrackWithMotionModel discards the outliers of its PoseOptimization and
// marks their points seen) + 1146-1161 (SearchLocalPoints skips the points already in the
// frame): skip[j] = no map point in local-map row j, or row j in mvpMapPoints; then the outlier
// rows of mvpMapPoints are cleared.  One workgroup per frame (the two phases are ordered); 4
// waves, so it finds a slot beside the extraction lane's workgroups.
__global__ void __launch_bounds__(256) k_local_prep(const LocalPrepDev* __restrict__ probs) {
    ORBGPU_LATENCY_WAVE();
    const LocalPrepDev& P = probs[blockIdx.x];
    for (int j = threadIdx.x; j < P.n; j += blockDim.x) P.skip[j] = P.row[j] < 0 ? 1 : 0;
    __syncthreads();
    for (int i = threadIdx.x; i < P.N; i += blockDim.x) {
        const int m = P.curMP[i];
        if (m >= 0) {
            if (m < P.n) P.skip[m] = 1;
            if (P.outlier[i]) P.curMP[i] = -1;
        }
    }
}

// ---------------------------------------------------------------- UndistortKeyPoints
// cvUndistortPoints (OpenCV 3.2 imgproc/undistort.cpp) for one CV_32FC2 point, as
// Frame::UndistortKeyPoints calls it (Frame.cc:418-419): normalise with 1/fx, 1/fy in double,
// 5 fixed-point iterations of the inverse radial/tangential model, then the new camera matrix
// (RR = K * I: the literal 3x3 product below, exact for K's zeros and ones).  The operation
// order is the reference's (the tilt and thin-prism terms are 0 and exact, see the oracle);
// the build's -ffp-contract=off keeps every product and sum rounded separately.
__device__ __forceinline__ void undistort_pt(float sx, float sy, const double* A, const double* k, int iters,
                                             float* ox, float* oy) {
    const double fx = A[0], fy = A[4], ifx = 1. / fx, ify = 1. / fy, cx = A[2], cy = A[5];
    double x = sx, y = sy, x0, y0;
    x0 = x = (x - cx) * ifx;
    y0 = y = (y - cy) * ify;
    for (int j = 0; j < iters; j++) {
        const double r2 = x * x + y * y;
        const double icdist = (1 + ((k[7] * r2 + k[6]) * r2 + k[5]) * r2) / (1 + ((k[4] * r2 + k[1]) * r2 + k[0]) * r2);
        const double deltaX = 2 * k[2] * x * y + k[3] * (r2 + 2 * x * x);
        const double deltaY = k[2] * (r2 + 2 * y * y) + 2 * k[3] * x * y;
        x = (x0 - deltaX) * icdist;
        y = (y0 - deltaY) * icdist;
    }
    const double xx = A[0] * x + A[1] * y + A[2];
    const double yy = A[3] * x + A[4] * y + A[5];
    const double ww = 1. / (A[6] * x + A[7] * y + A[8]);
    *ox = (float)(xx * ww);
    *oy = (float)(yy * ww);
}

struct UndistBatch {
    UndistDev p[kUndistPerLaunch];
};

__global__ void __launch_bounds__(256) k_undistort(UndistBatch B) {
    ORBGPU_LATENCY_WAVE();
    const UndistDev& P = B.p[blockIdx.y];
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P.N) return;
    orb_kp_dev kp = P.keys[i];
    if (P.has_dist) undistort_pt(kp.x, kp.y, P.A, P.k, 5, &kp.x, &kp.y);
    P.keysUn[i] = kp;
}

int undistort_batch(const UndistDev* probs, int count, hipStream_t s) {
    for (int f0 = 0; f0 < count; f0 += kUndistPerLaunch) {
        const int n = std::min(kUndistPerLaunch, count - f0);
        UndistBatch B;
        std::memset(&B, 0, sizeof(B));
        int maxN = 0;
        for (int f = 0; f < n; f++) {
            B.p[f] = probs[f0 + f];
            maxN = std::max(maxN, B.p[f].N);
        }
        if (maxN > 0) hipLaunchKernelGGL(k_undistort, dim3((maxN + 255) / 256, n), dim3(256), 0, s, B);
    }
    ORB_HIP_CHECK(hipGetLastError());
    return 0;
}

int local_prep_batch(const LocalPrepDev* d_probs, int count, hipStream_t s) {
    if (count <= 0) return 0;
    hipLaunchKernelGGL(k_local_prep, dim3(count), dim3(256), 0, s, d_probs);
    ORB_HIP_CHECK(hipGetLastError());
    return 0;
}

int unproject_batch(const UnprojDev* probs, int count, hipStream_t s) {
    for (int f0 = 0; f0 < count; f0 += kUnprojPerLaunch) {
        const int n = std::min(kUnprojPerLaunch, count - f0);
        UnprojBatch B;
        std::memset(&B, 0, sizeof(B));
        int maxN = 0;
        for (int f = 0; f < n; f++) {
            B.p[f] = probs[f0 + f];
            maxN = std::max(maxN, B.p[f].N);
        }
        if (maxN > 0) hipLaunchKernelGGL(k_unproject, dim3((maxN + 255) / 256, n), dim3(256), 0, s, B);
    }
    ORB_HIP_CHECK(hipGetLastError());
    return 0;
}

}  // namespace orbgpu
