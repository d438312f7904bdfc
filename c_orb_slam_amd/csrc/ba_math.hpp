// ba_math.hpp -- FP64 pieces shared by the optimisers (ba.hip, sim3opt.hip): Eigen
// quaternion / g2o SE3Quat arithmetic as explicit IEEE operation sequences, the canonical
// 64-wide reductions of oracle/ba.c (ora_csum), and the pivoted LDL^T of LinearSolverDense.
#pragma once
#include <hip/hip_runtime.h>

#include <cfloat>
#include <cmath>

#include "ba.hpp"

namespace orbgpu {

// ---------------------------------------------------------------- math (host + device)
#define HD __host__ __device__ __forceinline__

// ---------------------------------------------------------------- shared-denominator division
// Correctly rounded a / b for several numerators of one denominator.  gfx950 divides as
//   b' = v_div_scale(b, b, a); r = v_rcp(b'); a' = v_div_scale(a, b, a) (VCC);
//   e = fma(-b', r, 1); r = fma(r, e, r); e = fma(-b', r, 1); r = fma(r, e, r);
//   q = a' r; rem = fma(-b', q, a'); q = v_div_fmas(rem, r, q) (VCC); v_div_fixup(q, b, a).
// v_div_scale returns its operand unchanged and clears VCC unless an exponent is near the
// range limits (the quotient or 1/b near over/underflow, an exponent gap >= 768), so inside
// 2^-300 < |a|, |b| < 2^300 the sequence is exactly: r from b alone, then per numerator
// q = a r, rem = fma(-b, q, a), fma(rem, r, q), v_div_fixup.  The reciprocal is computed once;
// numerators outside the range (zeros included) take the plain division.
struct SharedDiv {
    double b, r;
    bool ok;
    __device__ __forceinline__ explicit SharedDiv(double den) : b(den) {
        const double ab = fabs(den);
        ok = ab > 0x1p-300 && ab < 0x1p300;
        double x = __builtin_amdgcn_rcp(den);
        double e = fma(-den, x, 1.0);
        x = fma(x, e, x);
        e = fma(-den, x, 1.0);
        r = fma(x, e, x);
    }
    __device__ __forceinline__ double div(double a) const {
        const double aa = fabs(a);
        if (ok && aa > 0x1p-300 && aa < 0x1p300) {
            const double q = a * r;
            const double rem = fma(-b, q, a);
            return __builtin_amdgcn_div_fixup(fma(rem, r, q), b, a);
        }
        return a / b;
    }
};


HD void quat_normalize(double* q) {
    const double z = ((q[0] * q[0] + q[1] * q[1]) + q[2] * q[2]) + q[3] * q[3];
    if (z > 0) {
        const double n = sqrt(z);
#ifdef __HIP_DEVICE_COMPILE__
        const SharedDiv d(n);   // the same quotients, one reciprocal
        for (int i = 0; i < 4; i++) q[i] = d.div(q[i]);
#else
        for (int i = 0; i < 4; i++) q[i] = q[i] / n;
#endif
    }
}

HD void se3_normalize(Se3& T) {
    if (T.q[3] < 0)
        for (int i = 0; i < 4; i++) T.q[i] *= -1;
    quat_normalize(T.q);
}

// Eigen Quaternion(Matrix3) branch for a dominant diagonal entry I (static indices keep the
// matrix in registers on the device)
template <int I>
HD void quat_from_R_diag(const double* m, double* q) {
    constexpr int J = (I + 1) % 3, K = (J + 1) % 3;
    double t = sqrt(((m[I * 4] - m[J * 4]) - m[K * 4]) + 1.0);
    q[I] = 0.5 * t;
    t = 0.5 / t;
    q[3] = (m[K * 3 + J] - m[J * 3 + K]) * t;
    q[J] = (m[J * 3 + I] + m[I * 3 + J]) * t;
    q[K] = (m[K * 3 + I] + m[I * 3 + K]) * t;
}

HD void quat_from_R(const double* m, double* q) {
    double t = (m[0] + m[4]) + m[8];
    if (t > 0) {
        t = sqrt(t + 1.0);
        q[3] = 0.5 * t;
        t = 0.5 / t;
        q[0] = (m[7] - m[5]) * t;
        q[1] = (m[2] - m[6]) * t;
        q[2] = (m[3] - m[1]) * t;
    } else {
        int i = 0;
        if (m[4] > m[0]) i = 1;
        if (m[8] > (i == 0 ? m[0] : m[4])) i = 2;
        if (i == 0) quat_from_R_diag<0>(m, q);
        else if (i == 1) quat_from_R_diag<1>(m, q);
        else quat_from_R_diag<2>(m, q);
    }
}

HD void quat_to_R(const double* q, double* R) {
    const double x = q[0], y = q[1], z = q[2], w = q[3];
    const double tx = 2.0 * x, ty = 2.0 * y, tz = 2.0 * z;
    const double twx = tx * w, twy = ty * w, twz = tz * w;
    const double txx = tx * x, txy = ty * x, txz = tz * x;
    const double tyy = ty * y, tyz = tz * y, tzz = tz * z;
    R[0] = 1.0 - (tyy + tzz); R[1] = txy - twz;         R[2] = txz + twy;
    R[3] = txy + twz;         R[4] = 1.0 - (txx + tzz); R[5] = tyz - twx;
    R[6] = txz - twy;         R[7] = tyz + twx;         R[8] = 1.0 - (txx + tyy);
}

HD void cross3(const double* a, const double* b, double* c) {
    c[0] = a[1] * b[2] - a[2] * b[1];
    c[1] = a[2] * b[0] - a[0] * b[2];
    c[2] = a[0] * b[1] - a[1] * b[0];
}

HD void quat_rotate(const double* q, const double* v, double* out) {
    double uv[3], c[3];
    cross3(q, v, uv);
    for (int i = 0; i < 3; i++) uv[i] += uv[i];
    cross3(q, uv, c);
    for (int i = 0; i < 3; i++) out[i] = (v[i] + q[3] * uv[i]) + c[i];
}

HD void se3_map(const Se3& T, const double* X, double* out) {
    double r[3];
    quat_rotate(T.q, X, r);
    for (int i = 0; i < 3; i++) out[i] = r[i] + T.t[i];
}

HD void se3_mul(const Se3& a, const Se3& b, Se3& o) {
    Se3 r{};
    double rt[3];
    quat_rotate(a.q, b.t, rt);
    for (int i = 0; i < 3; i++) r.t[i] = a.t[i] + rt[i];
    r.q[3] = ((a.q[3] * b.q[3] - a.q[0] * b.q[0]) - a.q[1] * b.q[1]) - a.q[2] * b.q[2];
    r.q[0] = ((a.q[3] * b.q[0] + a.q[0] * b.q[3]) + a.q[1] * b.q[2]) - a.q[2] * b.q[1];
    r.q[1] = ((a.q[3] * b.q[1] + a.q[1] * b.q[3]) + a.q[2] * b.q[0]) - a.q[0] * b.q[2];
    r.q[2] = ((a.q[3] * b.q[2] + a.q[2] * b.q[3]) + a.q[0] * b.q[1]) - a.q[1] * b.q[0];
    se3_normalize(r);
    o = r;
}

// ---------------------------------------------------------------- canonical reductions
// Canonical 64-tree across a wave: lane i (< off) += lane i + off for off = 32..1, result in
// lane 0.  gfx950 cross-lane moves instead of LDS: v_permlane32_swap (off 32),
// v_permlane16_swap (off 16), DPP row_shl (off 8..1, within the first row).
__device__ __forceinline__ unsigned xl_down(unsigned v, int off) {
    switch (off) {
        case 32: return __builtin_amdgcn_permlane32_swap(v, v, false, false)[1];
        case 16: return __builtin_amdgcn_permlane16_swap(v, v, false, false)[1];
        case 8: return __builtin_amdgcn_update_dpp(0u, v, 0x108, 0xf, 0xf, false);
        case 4: return __builtin_amdgcn_update_dpp(0u, v, 0x104, 0xf, 0xf, false);
        case 2: return __builtin_amdgcn_update_dpp(0u, v, 0x102, 0xf, 0xf, false);
        default: return __builtin_amdgcn_update_dpp(0u, v, 0x101, 0xf, 0xf, false);
    }
}
__device__ __forceinline__ double wave_down(double v, int off) {
    const unsigned long long u = __double_as_longlong(v);
    const unsigned lo = xl_down((unsigned)(u & 0xffffffffu), off);
    const unsigned hi = xl_down((unsigned)(u >> 32), off);
    return __longlong_as_double(((unsigned long long)hi << 32) | lo);
}
__device__ __forceinline__ double wave_tree(double v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += wave_down(v, off);
    return v;
}

// K canonical 64-trees at once (K <= 64), packed: after the level with offset `off` each value
// only needs `off` lanes, so the pair (x, y) of registers merges into one: x's pair sums in
// the lanes with bit `off` clear, y's (formed as y[i] + y[i - off] or y[i] + y[i + off], the
// same IEEE sums as the tree's) in the lanes with it set.  Offsets 32 and 16 are one
// v_permlane{32,16}_swap per dword of the PAIR (the swap exchanges exactly the halves the two
// trees need); offsets 8, 2, 1 a lane-select plus one DPP xor-move; 4 two bank-masked DPP
// moves.  Value q ends in lane bitrev6(q).
template <int OFF>
__device__ __forceinline__ unsigned dpp_xor_move(unsigned v) {
    static_assert(OFF == 8 || OFF == 2 || OFF == 1, "xor offsets with a single DPP control");
    // row_ror:8 (= xor 8 inside a row of 16), quad_perm [2,3,0,1], quad_perm [1,0,3,2]
    return __builtin_amdgcn_update_dpp(0u, v, OFF == 8 ? 0x128 : (OFF == 2 ? 0x4e : 0xb1), 0xf, 0xf, false);
}
__device__ __forceinline__ double dbl_of(unsigned lo, unsigned hi) {
    return __longlong_as_double(((unsigned long long)hi << 32) | lo);
}
__device__ __forceinline__ unsigned dlo(double v) { return (unsigned)(__double_as_longlong(v) & 0xffffffffu); }
__device__ __forceinline__ unsigned dhi(double v) { return (unsigned)(__double_as_longlong(v) >> 32); }

template <int OFF>
__device__ __forceinline__ double packed_pair(double x, double y, int lane) {
    if constexpr (OFF == 32 || OFF == 16) {
        const auto l = OFF == 32 ? __builtin_amdgcn_permlane32_swap(dlo(x), dlo(y), false, false)
                                 : __builtin_amdgcn_permlane16_swap(dlo(x), dlo(y), false, false);
        const auto h = OFF == 32 ? __builtin_amdgcn_permlane32_swap(dhi(x), dhi(y), false, false)
                                 : __builtin_amdgcn_permlane16_swap(dhi(x), dhi(y), false, false);
        return dbl_of(l[0], h[0]) + dbl_of(l[1], h[1]);
    } else if constexpr (OFF == 4) {
        const bool up = (lane & 4) != 0;
        const double p = up ? y : x;
        // banks (4-lane groups) 0,2 take x from 4 lanes up, banks 1,3 take y from 4 lanes down
        unsigned ql = __builtin_amdgcn_update_dpp(dlo(y), dlo(x), 0x104, 0xf, 0x5, false);
        unsigned qh = __builtin_amdgcn_update_dpp(dhi(y), dhi(x), 0x104, 0xf, 0x5, false);
        ql = __builtin_amdgcn_update_dpp(ql, dlo(y), 0x114, 0xf, 0xa, false);
        qh = __builtin_amdgcn_update_dpp(qh, dhi(y), 0x114, 0xf, 0xa, false);
        return p + dbl_of(ql, qh);
    } else {
        const bool up = (lane & OFF) != 0;
        const double p = up ? y : x, sx = up ? x : y;
        return p + dbl_of(dpp_xor_move<OFF>(dlo(sx)), dpp_xor_move<OFF>(dhi(sx)));
    }
}
// an unpaired register: plain tree step (valid in the lanes with bit `off` clear)
template <int OFF>
__device__ __forceinline__ double packed_single(double x) {
    return x + dbl_of(xl_down(dlo(x), OFF), xl_down(dhi(x), OFF));
}
template <int R, int OFF>
__device__ __forceinline__ void packed_level(double* a, int lane) {
#pragma unroll
    for (int j = 0; j < (R + 1) / 2; j++) {
        if (2 * j + 1 < R) a[j] = packed_pair<OFF>(a[2 * j], a[2 * j + 1], lane);
        else a[j] = packed_single<OFF>(a[2 * j]);
    }
}
__device__ __forceinline__ int bitrev6(int x) { return (int)(__builtin_bitreverse32((unsigned)x) >> 26); }
// v[0..K) per lane (clobbered); returns this lane's finished tree, value index bitrev6(lane)
template <int K>
__device__ __forceinline__ double packed_trees(double* v) {
    static_assert(K >= 1 && K <= 64, "packed_trees: 1..64 values");
    const int lane = threadIdx.x & 63;
    constexpr int R1 = K, R2 = (R1 + 1) / 2, R3 = (R2 + 1) / 2, R4 = (R3 + 1) / 2, R5 = (R4 + 1) / 2,
                  R6 = (R5 + 1) / 2;
    packed_level<R1, 32>(v, lane);
    packed_level<R2, 16>(v, lane);
    packed_level<R3, 8>(v, lane);
    packed_level<R4, 4>(v, lane);
    packed_level<R5, 2>(v, lane);
    packed_level<R6, 1>(v, lane);
    return v[0];
}

// Canonical sum (oracle ora_csum) of f(0..n) by one wave; sc: this wave's LDS scratch
// (>= ceil(n/64) doubles).  Result broadcast to all lanes.
template <class F>
__device__ __forceinline__ double wave_csum(F f, int n, double* sc) {
    const int lane = threadIdx.x & 63;
    if (n <= 0) return 0.0;
    if (n == 1) return f(0);  // ora_csum returns a single term untouched
    int m = (n + 63) >> 6;
    double v = 0;
    for (int c = 0; c < m; c++) {
        v = (c * 64 + lane < n) ? f(c * 64 + lane) : 0.0;
        v = wave_tree(v);
        if (m > 1 && lane == 0) sc[c] = v;
    }
    while (m > 1) {
        __builtin_amdgcn_s_waitcnt(0);
        __builtin_amdgcn_wave_barrier();
        const int m2 = (m + 63) >> 6;
        for (int c = 0; c < m2; c++) {
            double u = (c * 64 + lane < m) ? sc[c * 64 + lane] : 0.0;
            u = wave_tree(u);
            __builtin_amdgcn_s_waitcnt(0);
            __builtin_amdgcn_wave_barrier();
            if (lane == 0) sc[c] = u;
            v = u;
        }
        m = m2;
    }
    return __shfl(v, 0, 64);
}

// ---- exact thread-local emulation of the canonical 64-tree ------------------------
// tree64_local(get, cnt): a[i] = i < cnt ? get(i) : 0 (i < 64), then a[i] += a[i+off]
// for off = 32..1 -- the same pairing as wave_tree, evaluated in one thread.
template <class G>
__device__ __forceinline__ double tree64_local(G get, int cnt) {
    if (cnt <= 8) {
        // the same tree for at most 8 values: levels off = 32, 16, 8 only add +0 (x + 0 + 0 + 0 ==
        // x + 0, the sign of a zero included), so the leaves are w[i] = get(i) + 0 (i < cnt) or
        // +0, then offsets 4, 2, 1 -- 8 reads instead of 64 predicated ones
        double w[8];
#pragma unroll
        for (int i = 0; i < 8; i++) w[i] = i < cnt ? get(i) + 0.0 : 0.0;
#pragma unroll
        for (int off = 4; off >= 1; off >>= 1)
#pragma unroll
            for (int i = 0; i < off; i++) w[i] = w[i] + w[i + off];
        return w[0];
    }
    double a[32];
#pragma unroll
    for (int i = 0; i < 32; i++) a[i] = (i < cnt ? get(i) : 0.0) + (i + 32 < cnt ? get(i + 32) : 0.0);
#pragma unroll
    for (int off = 16; off >= 1; off >>= 1)
#pragma unroll
        for (int i = 0; i < off; i++) a[i] = a[i] + a[i + off];
    return a[0];
}

// Canonical total (ora_csum) of arr[0..m) by ONE thread, in place (arr is private to it).
__device__ __forceinline__ double local_csum_inplace(double* arr, int m) {
    if (m <= 0) return 0.0;
    while (m > 1) {
        const int m2 = (m + 63) >> 6;
        for (int c = 0; c < m2; c++) {
            const int cnt = min(64, m - c * 64);
            const double t = tree64_local([&](int i) { return arr[c * 64 + i]; }, cnt);
            arr[c] = t;
        }
        m = m2;
    }
    return arr[0];
}

// Eigen::LDLT<MatrixXd> compute + solve (diagonal pivoting, sequential dot products),
// identical operation sequence to oracle ora_ldlt_pivot_solve, fully unrolled so the n x n
// stays in registers: the data-dependent pivot swaps are unrolled conditional swaps.
template <int n>
__device__ __forceinline__ bool ldlt_pivot(double* M, const double* b, double* x) {
    int tr[n];
    double tmp[n];
    int sign = 0;
    bool stop = false;
#pragma unroll
    for (int k = 0; k < n; k++) {
        if (!stop) {
            int idx = k;
            double big = fabs(M[k * n + k]);
#pragma unroll
            for (int i = k + 1; i < n; i++) {
                const double d = fabs(M[i * n + i]);
                if (d > big) {
                    big = d;
                    idx = i;
                }
            }
            tr[k] = idx;
#pragma unroll
            for (int i = k + 1; i < n; i++)
                if (idx == i) {
#pragma unroll
                    for (int j = 0; j < k; j++) { const double t = M[k * n + j]; M[k * n + j] = M[i * n + j]; M[i * n + j] = t; }
#pragma unroll
                    for (int r = i + 1; r < n; r++) { const double t = M[r * n + k]; M[r * n + k] = M[r * n + i]; M[r * n + i] = t; }
                    { const double t = M[k * n + k]; M[k * n + k] = M[i * n + i]; M[i * n + i] = t; }
#pragma unroll
                    for (int r = k + 1; r < i; r++) { const double t = M[r * n + k]; M[r * n + k] = M[i * n + r]; M[i * n + r] = t; }
                }
            if (k > 0) {
#pragma unroll
                for (int j = 0; j < k; j++) tmp[j] = M[j * n + j] * M[k * n + j];
                double s = 0;
#pragma unroll
                for (int j = 0; j < k; j++) s += M[k * n + j] * tmp[j];
                M[k * n + k] -= s;
#pragma unroll
                for (int i = k + 1; i < n; i++) {
                    double t = 0;
#pragma unroll
                    for (int j = 0; j < k; j++) t += M[i * n + j] * tmp[j];
                    M[i * n + k] -= t;
                }
            }
            const double akk = M[k * n + k];
            const bool valid = fabs(akk) > 0.0;
            if (k == 0 && !valid) {
#pragma unroll
                for (int j = 0; j < n; j++) tr[j] = j;
                sign = 0;
                stop = true;
            } else {
                if (valid) {
#pragma unroll
                    for (int i = k + 1; i < n; i++) M[i * n + k] /= akk;
                }
                if (sign == 1) { if (akk < 0) sign = 3; }
                else if (sign == 2) { if (akk > 0) sign = 3; }
                else if (sign == 0) { if (akk > 0) sign = 1; else if (akk < 0) sign = 2; }
            }
        }
    }
    if (!(sign == 1 || sign == 0)) return false;
    double y[n];
#pragma unroll
    for (int i = 0; i < n; i++) y[i] = b[i];
#pragma unroll
    for (int k = 0; k < n; k++)
#pragma unroll
        for (int i = k + 1; i < n; i++)
            if (tr[k] == i) { const double t = y[k]; y[k] = y[i]; y[i] = t; }
#pragma unroll
    for (int i = 0; i < n; i++)
#pragma unroll
        for (int j = 0; j < i; j++) y[i] -= M[i * n + j] * y[j];
#pragma unroll
    for (int i = 0; i < n; i++) y[i] = fabs(M[i * n + i]) > DBL_MIN ? y[i] / M[i * n + i] : 0.0;
#pragma unroll
    for (int i = n - 1; i >= 0; i--)
#pragma unroll
        for (int j = n - 1; j > i; j--) y[i] -= M[j * n + i] * y[j];
#pragma unroll
    for (int k = n - 1; k >= 0; k--)
#pragma unroll
        for (int i = k + 1; i < n; i++)
            if (tr[k] == i) { const double t = y[k]; y[k] = y[i]; y[i] = t; }
#pragma unroll
    for (int i = 0; i < n; i++) x[i] = y[i];
    return true;
}
__device__ __forceinline__ bool ldlt_pivot6(double* M, const double* b, double* x) { return ldlt_pivot<6>(M, b, x); }

}  // namespace orbgpu
