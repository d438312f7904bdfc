// ldlt_probe.hip -- phase timing (shader cycles) of k_ldlt_reg on an n x n SPD system (default 90).
// build: compile this file, csrc/ldlt.hip (hipcc -c) and csrc/ordering.cpp (g++ -c), link with hipcc -> build/ldlt_probe
#define ORB_LDLT_PROBE 1
#include "../c_orb_slam_amd/csrc/ba.hip"
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <random>

int main(int argc, char** argv) {
    const int n = argc > 1 ? atoi(argv[1]) : 90;
    std::mt19937 g(1);
    std::normal_distribution<double> N(0, 1);
    std::vector<double> A(n * n), S(n * n, 0), b(n);
    for (auto& v : A) v = N(g);
    for (int i = 0; i < n; i++)
        for (int j = 0; j < n; j++) {
            double t = 0;
            for (int k = 0; k < n; k++) t += A[i * n + k] * A[j * n + k];
            S[i * n + j] = t + (i == j ? n : 0);
        }
    for (auto& v : b) v = N(g);
    double *dS, *dB, *dX, *dScal;
    hipMalloc(&dS, 8 * n * n); hipMalloc(&dB, 8 * n); hipMalloc(&dX, 8 * n); hipMalloc(&dScal, 128);
    hipMemcpy(dS, S.data(), 8 * n * n, hipMemcpyHostToDevice);
    hipMemcpy(dB, b.data(), 8 * n, hipMemcpyHostToDevice);
    const size_t shm = orbgpu::ldlt_reg_shm(n);
    for (int rep = 0; rep < 3; rep++) {
        hipLaunchKernelGGL(orbgpu::k_ldlt_reg, dim3(1), dim3(orbgpu::kLdltThreads), shm, 0, n, dS, dB, dX, dScal, nullptr);
        hipDeviceSynchronize();
    }
    long long p[256];
    hipMemcpyFromSymbol(p, HIP_SYMBOL(orbgpu::g_ldlt_probe), sizeof(p));
    printf("load %lld | panels %lld | fwd %lld | bwd %lld  (cycles)\n", p[1] - p[0], p[2] - p[1], p[3] - p[2], p[4] - p[3]);
    long long ph = 0;
    printf("phase cycles:");
    for (int k = 0; k < (n + 5) / 6; k++) {
        ph += p[12 + 4 * k] - p[11 + 4 * k];
        printf(" %lld", p[12 + 4 * k] - p[11 + 4 * k]);
    }
    printf("\nphases (factor panel p | rows: panel p - 1's updates) %lld cycles, %d panels\n", ph, (n + 5) / 6);
    for (int k = 1; k < (n + 5) / 6 && k < 16; k++) {
        printf("phase %2d: factor done at %5lld | row waves' trailing update done at", k, p[220 + k] - p[11 + 4 * k]);
        for (int t = 0; t < 6; t++) printf(" %5lld", p[124 + 6 * k + t] - p[11 + 4 * k]);
        printf(" | barrier at %5lld\n", p[12 + 4 * k] - p[11 + 4 * k]);
    }
    return 0;
}
