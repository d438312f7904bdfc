// Latency microbenchmark (one wave): dependent chains of FP64 ops on gfx950, clock64 cycles/op.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k_lat(double* out, unsigned long long* cyc, double a, double b, int n) {
    double x = a + threadIdx.x * 1e-9, y = b;
    unsigned long long t0, t1;
    // 0: dependent add
    t0 = clock64();
#pragma unroll 16
    for (int i = 0; i < n; i++) x = x + y;
    t1 = clock64(); cyc[0] = t1 - t0; out[0] = x;
    // 1: dependent fma-free mul
    x = a;
    t0 = clock64();
#pragma unroll 16
    for (int i = 0; i < n; i++) x = x * y;
    t1 = clock64(); cyc[1] = t1 - t0; out[1] = x;
    // 2: dependent division
    x = a;
    t0 = clock64();
#pragma unroll 16
    for (int i = 0; i < n; i++) x = y / x;
    t1 = clock64(); cyc[2] = t1 - t0; out[2] = x;
    // 3: dependent sqrt
    x = a;
    t0 = clock64();
#pragma unroll 16
    for (int i = 0; i < n; i++) x = sqrt(x + y);
    t1 = clock64(); cyc[3] = t1 - t0; out[3] = x;
    // 4: independent divisions (4 chains)
    double p = a, q = a + 1, r = a + 2, s = a + 3;
    t0 = clock64();
#pragma unroll 16
    for (int i = 0; i < n; i++) { p = y / p; q = y / q; r = y / r; s = y / s; }
    t1 = clock64(); cyc[4] = t1 - t0; out[4] = p + q + r + s;
    // 5: readlane broadcast chain
    x = a;
    t0 = clock64();
#pragma unroll 16
    for (int i = 0; i < n; i++) {
        unsigned long long u = __double_as_longlong(x);
        unsigned lo = __builtin_amdgcn_readlane((unsigned)u, 3), hi = __builtin_amdgcn_readlane((unsigned)(u >> 32), 3);
        x = __longlong_as_double(((unsigned long long)hi << 32) | lo) + y;
    }
    t1 = clock64(); cyc[5] = t1 - t0; out[5] = x;
    // 6: independent adds (8 chains)
    double c0 = a, c1 = a, c2 = a, c3 = a, c4 = a, c5 = a, c6 = a, c7 = a;
    t0 = clock64();
#pragma unroll 16
    for (int i = 0; i < n; i++) { c0 += y; c1 += y; c2 += y; c3 += y; c4 += y; c5 += y; c6 += y; c7 += y; }
    t1 = clock64(); cyc[6] = t1 - t0; out[6] = c0 + c1 + c2 + c3 + c4 + c5 + c6 + c7;
}

int main() {
    double* d; unsigned long long* c;
    hipMalloc(&d, 64 * sizeof(double)); hipMalloc(&c, 64 * sizeof(unsigned long long));
    const int n = 1000;
    for (int rep = 0; rep < 2; rep++) {
        hipLaunchKernelGGL(k_lat, dim3(1), dim3(64), 0, 0, d, c, 1.5, 1.0000001, n);
        hipDeviceSynchronize();
    }
    unsigned long long h[8];
    hipMemcpy(h, c, sizeof(h), hipMemcpyDeviceToHost);
    const char* nm[] = {"dep add", "dep mul", "dep div", "dep sqrt", "4 indep div (per iter)", "readlane+add", "8 indep add (per iter)"};
    for (int i = 0; i < 7; i++) printf("%-24s %.1f cycles/iter\n", nm[i], (double)h[i] / n);
    return 0;
}
