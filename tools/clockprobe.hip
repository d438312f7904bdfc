// clockprobe.hip -- measure the shader clock the BA-sized kernels actually run at:
// cycles (s_memtime) vs wall time (s_memrealtime, 100 MHz) inside one kernel,
// for a kernel launched right after an idle host sync and for back-to-back launches.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <thread>

__global__ void spin(long long iters, double* out, long long* t) {
    long long c0 = clock64(), w0 = wall_clock64();
    double a = threadIdx.x * 1e-9, b = 1.0000001;
    for (long long i = 0; i < iters; i++) a = a * b + 1e-12;
    long long c1 = clock64(), w1 = wall_clock64();
    if (threadIdx.x == 0) { t[0] = c1 - c0; t[1] = w1 - w0; }
    out[threadIdx.x] = a;
}

int main() {
    double* out; long long* t; long long h[2];
    hipMalloc(&out, 1024 * 8); hipMalloc(&t, 16);
    int rate = 0; hipDeviceGetAttribute(&rate, hipDeviceAttributeWallClockRate, 0);
    for (int mode = 0; mode < 3; mode++) {
        for (int rep = 0; rep < 5; rep++) {
            if (mode == 1) std::this_thread::sleep_for(std::chrono::milliseconds(2));
            long long iters = mode == 2 ? 2000000 : 20000;
            hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, 0, iters, out, t);
            hipMemcpy(h, t, 16, hipMemcpyDeviceToHost);
            double us = h[1] * 1e3 / rate;
            printf("mode %d rep %d: %lld cycles in %.1f us -> %.0f MHz\n", mode, rep, h[0], us, h[0] / us);
        }
    }
    return 0;
}
