// fetch_calib.hip -- calibrates rocprofv3 FETCH_SIZE against a known byte count for the two
// load widths the extraction kernels use (MI355X_MICROARCH.md: FETCH_SIZE is calibrated only
// for 16-B-per-lane streaming reads).  Each kernel streams the same 1 GiB buffer once (past
// the 256 MiB Infinity Cache); run under  rocprofv3 --pmc FETCH_SIZE --kernel-trace.
//   hipcc --offload-arch=gfx950 -O3 tools/fetch_calib.hip -o build/fetch_calib
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ void k_read16(const uint4* __restrict__ p, size_t n, unsigned* out) {
    unsigned acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const uint4 v = p[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

__global__ void k_read4(const unsigned* __restrict__ p, size_t n, unsigned* out) {
    unsigned acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        acc ^= p[i];
    if (acc == 0x12345678u) out[0] = acc;
}

__global__ void k_read1(const unsigned char* __restrict__ p, size_t n, unsigned* out) {
    unsigned acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        acc += p[i];
    if (acc == 0x12345678u) out[0] = acc;
}

int main() {
    const size_t bytes = (size_t)1 << 30;
    void* buf = nullptr;
    unsigned* out = nullptr;
    if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
    if (hipMemset(buf, 1, bytes) != hipSuccess) return 1;
    const dim3 g(256 * 16), b(256);
    hipLaunchKernelGGL(k_read16, g, b, 0, 0, (const uint4*)buf, bytes / 16, out);
    hipLaunchKernelGGL(k_read4, g, b, 0, 0, (const unsigned*)buf, bytes / 4, out);
    hipLaunchKernelGGL(k_read1, g, b, 0, 0, (const unsigned char*)buf, bytes, out);
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    printf("read %zu bytes per kernel (FETCH_SIZE is reported in KiB: expect %zu)\n", bytes, bytes / 1024);
    (void)hipFree(buf);
    (void)hipFree(out);
    return 0;
}
