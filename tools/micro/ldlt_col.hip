// Phase timers of the column-owner dense LDL^T (k_ldlt_col in ba.hip) on one 90 x 90 system, plus
// the primitive costs it is built from: barrier of 4 waves, uniform-address LDS read chain, the
// shared-denominator division.  s_memtime cycles (shader clock) and s_memrealtime (100 MHz) for
// the clock rate.  hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/micro/ldlt_col.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

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

constexpr int kMax = 96, kRows = kMax / 4;
__device__ unsigned long long g_t[8][8];   // [wave][phase] cycle sums

#define STAMP(i)                                                          \
    do {                                                                  \
        const unsigned long long _t = __builtin_amdgcn_s_memtime();       \
        if (lane == 0) acc[i] += _t - tp;                                 \
        tp = _t;                                                          \
    } while (0)

__global__ void __launch_bounds__(256) k_col(int n, const double* __restrict__ Sg, const double* bs, double* out,
                                             unsigned long long* rt) {
    __shared__ double Ur[2][128];
    __shared__ double Lall[kMax * kMax];
    __shared__ __attribute__((aligned(16))) double lw[4][kRows + 8];
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    const int c0 = lane, c1 = lane + 64;
    unsigned long long acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    double A0[kRows], A1[kRows];
#pragma unroll
    for (int r = 0; r < kRows; r++) {
        const int i = 4 * r + w;
        const bool row = i < n;
        A0[r] = (row && c0 < n && c0 >= i) ? Sg[(size_t)i * n + c0] : (row && c0 == n) ? bs[i] : 0.0;
        A1[r] = (row && c1 < n && c1 >= i) ? Sg[(size_t)i * n + c1] : (row && c1 == n) ? bs[i] : 0.0;
    }
    if (w == 0) {
        Ur[0][c0] = A0[0];
        Ur[0][c1] = A1[0];
    }
    __syncthreads();
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    unsigned long long tp = __builtin_amdgcn_s_memtime();
    const unsigned long long tstart = tp;
    for (int k = 0; k < n; k++) {
        const double* U = Ur[k & 1];
        double* V = Ur[(k + 1) & 1];
        const double d = U[k];
        const double u0 = U[c0], u1 = U[c1];
        const int own = (k + 1) & 3;
        STAMP(0);
        if (w == own) {
            const int r1 = (k + 1) >> 2;
            const double l1 = U[k + 1 < n ? k + 1 : k] / d;
#pragma unroll
            for (int r = 0; r < kRows; r++)
                if (r == r1 && k + 1 < n) {
                    A0[r] -= l1 * u0;
                    A1[r] -= l1 * u1;
                    V[c0] = A0[r];
                    V[c1] = A1[r];
                }
        }
        STAMP(1);
        const double l0 = u0 / d, l1v = u1 / d;
        STAMP(2);
        if (w == 0) {
            if (c0 > k && c0 < n) Lall[k * n + c0] = l0;
            if (c1 > k && c1 < n) Lall[k * n + c1] = l1v;
        }
        if ((lane & 3) == w) {
            lw[w][lane >> 2] = l0;
            lw[w][16 + (lane >> 2)] = l1v;
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);
        __builtin_amdgcn_wave_barrier();
        STAMP(3);
        const int rlive = (k + 5 - w) >> 2;
#pragma unroll
        for (int g = 0; g < kRows / 4; g++) {
            if (4 * g + 3 >= rlive && 16 * g + w < n) {
                const double2 la = *reinterpret_cast<const double2*>(&lw[w][4 * g]);
                const double2 lb = *reinterpret_cast<const double2*>(&lw[w][4 * g + 2]);
                const double lv[4] = {la.x, la.y, lb.x, lb.y};
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const int r = 4 * g + q, i = 4 * r + w;
                    const bool live = i > k + 1 && i < n;
                    const double v0 = A0[r] - lv[q] * u0, v1 = A1[r] - lv[q] * u1;
                    A0[r] = live ? v0 : A0[r];
                    A1[r] = live ? v1 : A1[r];
                }
            }
        }
        STAMP(4);
        __syncthreads();
        STAMP(5);
    }
    const unsigned long long tend = __builtin_amdgcn_s_memtime();
    const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    if (lane == 0) {
        for (int i = 0; i < 6; i++) g_t[w][i] = acc[i];
        g_t[w][6] = tend - tstart;
        g_t[w][7] = r1 - r0;
    }
    double s = 0;
#pragma unroll
    for (int r = 0; r < kRows; r++) s += A0[r] + A1[r];
    out[tid] = s + Lall[lane];
    (void)rt;
}

// primitives: (0) 1000 barriers of 4 waves, (1) 1000 dependent uniform LDS reads, (2) 1000
// independent uniform LDS reads, (3) 1000 SharedDiv(d) + 2 div, (4) 1000 plain divisions x2
__global__ void __launch_bounds__(256) k_prim(double* out, unsigned long long* cyc, double a) {
    __shared__ double sh[1024];
    const int tid = threadIdx.x, lane = tid & 63;
    for (int i = tid; i < 1024; i += 256) sh[i] = 1.0 + i * 1e-3;
    __syncthreads();
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < 1000; i++) __syncthreads();
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (tid == 0) cyc[0] = t1 - t0;
    int idx = 0;
    double x = 0;
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < 1000; i++) {
        x += sh[idx];
        idx = ((int)x) & 511;
    }
    t1 = __builtin_amdgcn_s_memtime();
    if (tid == 0) cyc[1] = t1 - t0;
    double y = 0;
    t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 8
    for (int i = 0; i < 1000; i++) y += sh[i & 1023];
    t1 = __builtin_amdgcn_s_memtime();
    if (tid == 0) cyc[2] = t1 - t0;
    double z = a + lane;
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < 1000; i++) {
        const SharedDiv sd(z);
        z = sd.div(a + i) + sd.div(a - i) + 1.0;
    }
    t1 = __builtin_amdgcn_s_memtime();
    if (tid == 0) cyc[3] = t1 - t0;
    double q = a + lane;
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < 1000; i++) q = (a + i) / q + (a - i) / q + 1.0;
    t1 = __builtin_amdgcn_s_memtime();
    if (tid == 0) cyc[4] = t1 - t0;
    out[tid] = x + y + z + q;
}

int main() {
    const int n = 90;
    std::vector<double> S((size_t)n * n), b(n);
    srand(1);
    for (int i = 0; i < n; i++)
        for (int j = i; j < n; j++) S[(size_t)i * n + j] = (i == j ? n : 0.0) + (double)rand() / RAND_MAX;
    for (int i = 0; i < n; i++) b[i] = (double)rand() / RAND_MAX;
    double *dS, *dB, *dO;
    unsigned long long* dC;
    hipMalloc(&dS, sizeof(double) * n * n);
    hipMalloc(&dB, sizeof(double) * n);
    hipMalloc(&dO, sizeof(double) * 1024);
    hipMalloc(&dC, sizeof(unsigned long long) * 16);
    hipMemcpy(dS, S.data(), sizeof(double) * n * n, hipMemcpyHostToDevice);
    hipMemcpy(dB, b.data(), sizeof(double) * n, hipMemcpyHostToDevice);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int rep = 0; rep < 3; rep++) {
        hipEventRecord(e0);
        hipLaunchKernelGGL(k_col, dim3(1), dim3(256), 0, 0, n, dS, dB, dO, dC);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
    }
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    unsigned long long t[8][8];
    hipMemcpyFromSymbol(t, HIP_SYMBOL(g_t), sizeof(t));
    printf("k_col n=%d: event %.1f us; loop %llu cycles over %llu realtime ticks (%.0f MHz)\n", n, ms * 1e3, t[0][6],
           t[0][7], t[0][6] / (t[0][7] / 100.0));
    const char* ph[6] = {"U reads", "own row + publish", "2 divisions", "l round trip", "row updates", "barrier"};
    for (int w = 0; w < 4; w++) {
        printf("wave %d per pivot:", w);
        for (int i = 0; i < 6; i++) printf(" %s %.0f |", ph[i], t[w][i] / (double)n);
        printf("\n");
    }
    hipLaunchKernelGGL(k_prim, dim3(1), dim3(256), 0, 0, dO, dC, 1.5);
    unsigned long long c[16];
    hipMemcpy(c, dC, sizeof(c), hipMemcpyDeviceToHost);
    printf("barrier(4 waves) %.1f | dependent LDS read %.1f | independent LDS read %.1f | SharedDiv+2div %.1f | "
           "2 plain div %.1f  cycles each\n",
           c[0] / 1e3, c[1] / 1e3, c[2] / 1e3, c[3] / 1e3, c[4] / 1e3);
    return 0;
}
