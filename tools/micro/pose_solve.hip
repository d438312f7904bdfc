// Cycle cost of k_pose_opt's serial trial pieces on one wave (gfx950): the 6x6 pivoted LDL^T solve
// (pose_solve_w), se3_exp and se3_mul, each timed with clock64 over R dependent repetitions.
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I c_orb_slam_amd/csrc
//        tools/micro/pose_solve.hip c_orb_slam_amd/csrc/{ldlt.hip,ba_struct.cpp,ordering.cpp} -o build/pose_solve_micro
#include "../../c_orb_slam_amd/csrc/ba.hip"

#include <cstring>
#include <vector>

namespace orbgpu {
__global__ void __launch_bounds__(64) k_solve_micro(const double* Hin, const double* bin, double lambda, double* out,
                                                    unsigned long long* cyc, int R) {
    __shared__ double Hs[21], bs[6];
    if (threadIdx.x < 21) Hs[threadIdx.x] = Hin[threadIdx.x];
    if (threadIdx.x < 6) bs[threadIdx.x] = bin[threadIdx.x];
    __syncthreads();
    double x[6] = {0, 0, 0, 0, 0, 0};
    double lam = lambda;
    unsigned long long t0 = clock64();
    for (int r = 0; r < R; r++) {
        pose_solve_w(Hs, bs, lam, x);
        lam = lam * 1.0000001 + x[0] * 1e-300;   // dependent: the next solve waits for this one
    }
    unsigned long long t1 = clock64();
    Se3 T0;
    T0.q[0] = 0.01; T0.q[1] = -0.02; T0.q[2] = 0.03; T0.q[3] = 0.999;
    T0.t[0] = 0.1; T0.t[1] = 0.2; T0.t[2] = 0.3; T0.pad = 0;
    Se3 d, r2 = T0;
    for (int r = 0; r < R; r++) {
        double xl[6];
        for (int j = 0; j < 6; j++) xl[j] = x[j] + r2.t[0] * 1e-300;
        se3_exp(xl, d);
        r2.t[0] = d.t[0];
    }
    unsigned long long t2 = clock64();
    for (int r = 0; r < R; r++) se3_mul(d, r2, r2);
    unsigned long long t3 = clock64();
    if (threadIdx.x == 0) {
        cyc[0] = (t1 - t0) / R;
        cyc[1] = (t2 - t1) / R;
        cyc[2] = (t3 - t2) / R;
        for (int j = 0; j < 6; j++) out[j] = x[j];
        out[6] = r2.q[0] + r2.t[1] + d.q[1];
    }
}
__global__ void __launch_bounds__(64) k_solve_micro_l(const double* Hin, const double* bin, double lambda, double* out,
                                                      unsigned long long* cyc, int R) {
    __shared__ double Hs[21], bs[6], scr[36];
    if (threadIdx.x < 21) Hs[threadIdx.x] = Hin[threadIdx.x];
    if (threadIdx.x < 6) bs[threadIdx.x] = bin[threadIdx.x];
    __syncthreads();
    double x[6] = {0, 0, 0, 0, 0, 0};
    double lam = lambda;
    unsigned long long t0 = clock64();
    for (int r = 0; r < R; r++) {
        pose_solve_l(Hs, bs, lam, x, scr);
        lam = lam * 1.0000001 + x[0] * 1e-300;
    }
    unsigned long long t1 = clock64();
    if (threadIdx.x == 0) {
        cyc[3] = (t1 - t0) / R;
        for (int j = 0; j < 6; j++) out[j] = x[j];
    }
}
// pose_solve_l's prelude only (pivot ranks, order, the lane's permuted row): its share of a solve
__device__ __forceinline__ double solve_prelude(const double* Hs, const double* bs, double lambda) {
    double dv[6];
#pragma unroll
    for (int i = 0; i < 6; i++) dv[i] = fabs(Hs[DIAG21[i]] + lambda);
    bool distinct = true;
    int rank[6];
#pragma unroll
    for (int j = 0; j < 6; j++) {
        int r = 0;
        distinct = distinct && dv[j] == dv[j];
#pragma unroll
        for (int i = 0; i < 6; i++)
            if (i != j) {
                r += dv[i] > dv[j] ? 1 : 0;
                distinct = distinct && dv[i] != dv[j];
            }
        rank[j] = r;
    }
    int ord[6];
#pragma unroll
    for (int r = 0; r < 6; r++) {
        int o = 0;
#pragma unroll
        for (int j = 0; j < 6; j++) o = rank[j] == r ? j : o;
        ord[r] = o;
    }
    const int lane = threadIdx.x & 63, row = lane < 6 ? lane : 5;
    int orow = ord[0];
#pragma unroll
    for (int p = 1; p < 6; p++) orow = row == p ? ord[p] : orow;
    double a[6];
#pragma unroll
    for (int c = 0; c < 6; c++) {
        const int i0 = min(orow, ord[c]), i1 = max(orow, ord[c]);
        double h = Hs[i0 * 6 - (i0 * (i0 - 1)) / 2 + (i1 - i0)];
        if (row == c) h += lambda;
        a[c] = h;
    }
    return distinct ? a[0] + a[1] + a[2] + a[3] + a[4] + a[5] + bs[orow] : 0.0;
}
__global__ void __launch_bounds__(64) k_prelude_micro(const double* Hin, const double* bin, double lambda, double* out,
                                                      unsigned long long* cyc, int R) {
    __shared__ double Hs[21], bs[6];
    if (threadIdx.x < 21) Hs[threadIdx.x] = Hin[threadIdx.x];
    if (threadIdx.x < 6) bs[threadIdx.x] = bin[threadIdx.x];
    __syncthreads();
    double lam = lambda, acc = 0;
    unsigned long long t0 = clock64();
    for (int r = 0; r < R; r++) {
        const double v = solve_prelude(Hs, bs, lam);
        acc += v;
        lam = lam * 1.0000001 + v * 1e-300;
    }
    unsigned long long t1 = clock64();
    if (threadIdx.x == 0) {
        cyc[3] = (t1 - t0) / R;
        out[0] = acc;
    }
}
// both solves on n systems (one wave each): x and ok of pose_solve_w, then of pose_solve_l
__global__ void __launch_bounds__(64) k_solve_cmp(const double* H, const double* b, const double* lam, double* xo, int* oko) {
    __shared__ double Hs[21], bs[6], scr[36];
    const int s = blockIdx.x;
    if (threadIdx.x < 21) Hs[threadIdx.x] = H[21 * s + threadIdx.x];
    if (threadIdx.x < 6) bs[threadIdx.x] = b[6 * s + threadIdx.x];
    __syncthreads();
    double x1[6], x2[6];
    const bool ok1 = pose_solve_w(Hs, bs, lam[s], x1);
    const bool ok2 = pose_solve_l(Hs, bs, lam[s], x2, scr);
    if (threadIdx.x == 0) {
        for (int j = 0; j < 6; j++) {
            xo[12 * s + j] = x1[j];
            xo[12 * s + 6 + j] = x2[j];
        }
        oko[2 * s] = ok1;
        oko[2 * s + 1] = ok2;
    }
}
}  // namespace orbgpu

int main() {
    using namespace orbgpu;
    // a well-conditioned pose system (distinct diagonal: the fast path)
    const double H[21] = {5e5, 1e3, -2e3, 4e2, 1e1, -3e1, 7e5, 5e2, -2e2, 3e1, 2e1, 3e5, 1e1, 2e1, 4e1,
                          9e4, 1e2, -5e1, 6e4, 3e1, 4e4};
    const double b[6] = {1e2, -3e1, 5e1, 7e0, -2e0, 1e0};
    double *dH, *db, *dout;
    unsigned long long* dc;
    (void)hipMalloc(&dH, sizeof(H));
    (void)hipMalloc(&db, sizeof(b));
    (void)hipMalloc(&dout, 8 * sizeof(double));
    (void)hipMalloc(&dc, 4 * sizeof(unsigned long long));
    (void)hipMemcpy(dH, H, sizeof(H), hipMemcpyHostToDevice);
    (void)hipMemcpy(db, b, sizeof(b), hipMemcpyHostToDevice);
    for (int rep = 0; rep < 2; rep++) {
        hipLaunchKernelGGL(k_solve_micro, dim3(1), dim3(64), 0, 0, dH, db, 1e-3, dout, dc, 64);
        (void)hipDeviceSynchronize();
    }
    unsigned long long c[4];
    double o[8];
    (void)hipMemcpy(c, dc, sizeof(c), hipMemcpyDeviceToHost);
    (void)hipMemcpy(o, dout, sizeof(o), hipMemcpyDeviceToHost);
    printf("cycles per call: pose_solve_w %llu  se3_exp %llu  se3_mul %llu   (x0 %.6e)\n", c[0], c[1], c[2], o[0]);
    for (int rep = 0; rep < 2; rep++) {
        hipLaunchKernelGGL(k_solve_micro_l, dim3(1), dim3(64), 0, 0, dH, db, 1e-3, dout, dc, 64);
        (void)hipDeviceSynchronize();
    }
    (void)hipMemcpy(c, dc, sizeof(c), hipMemcpyDeviceToHost);
    (void)hipMemcpy(o, dout, sizeof(o), hipMemcpyDeviceToHost);
    printf("cycles per call: pose_solve_l %llu   (x0 %.6e)\n", c[3], o[0]);
    // bit comparison on random J^T J + lambda systems (some indefinite, some with tied diagonals)
    const int n = 4096;
    std::vector<double> Hh(21 * n), bh(6 * n), lh(n), xo(12 * n);
    std::vector<int> oko(2 * n);
    unsigned long long st = 88172645463325252ull;
    auto rnd = [&]() { st ^= st << 13; st ^= st >> 7; st ^= st << 17; return (double)(st >> 11) / 9007199254740992.0 - 0.5; };
    for (int s = 0; s < n; s++) {
        double J[6][6];
        for (int i = 0; i < 6; i++)
            for (int j = 0; j < 6; j++) J[i][j] = rnd() * (1 + 100 * (j < 3));
        for (int r = 0, q = 0; r < 6; r++)
            for (int cc = r; cc < 6; cc++, q++) {
                double v = 0;
                for (int k = 0; k < 6; k++) v += J[k][r] * J[k][cc];
                if (s % 7 == 3 && r != cc) v *= 40;          // indefinite after pivoting
                Hh[21 * s + q] = v;
            }
        if (s % 11 == 5) Hh[21 * s + DIAG21[2]] = Hh[21 * s + DIAG21[4]];   // tied |diag|
        for (int j = 0; j < 6; j++) bh[6 * s + j] = rnd() * 10;
        lh[s] = s % 3 == 0 ? 0.0 : fabs(rnd()) * 1e-2;
    }
    double *gH, *gb, *gl, *gx;
    int* gok;
    (void)hipMalloc(&gH, 8 * Hh.size());
    (void)hipMalloc(&gb, 8 * bh.size());
    (void)hipMalloc(&gl, 8 * lh.size());
    (void)hipMalloc(&gx, 8 * xo.size());
    (void)hipMalloc(&gok, 4 * oko.size());
    (void)hipMemcpy(gH, Hh.data(), 8 * Hh.size(), hipMemcpyHostToDevice);
    (void)hipMemcpy(gb, bh.data(), 8 * bh.size(), hipMemcpyHostToDevice);
    (void)hipMemcpy(gl, lh.data(), 8 * lh.size(), hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_solve_cmp, dim3(n), dim3(64), 0, 0, gH, gb, gl, gx, gok);
    (void)hipDeviceSynchronize();
    (void)hipMemcpy(xo.data(), gx, 8 * xo.size(), hipMemcpyDeviceToHost);
    (void)hipMemcpy(oko.data(), gok, 4 * oko.size(), hipMemcpyDeviceToHost);
    int bad = 0, nok = 0;
    for (int s = 0; s < n; s++) {
        nok += oko[2 * s];
        bool same = oko[2 * s] == oko[2 * s + 1];
        if (oko[2 * s])
            for (int j = 0; j < 6; j++) same = same && memcmp(&xo[12 * s + j], &xo[12 * s + 6 + j], 8) == 0;
        bad += !same;
    }
    printf("pose_solve_l vs pose_solve_w: %d systems (%d solved), %d differ\n", n, nok, bad);
    for (int rep = 0; rep < 2; rep++) {
        hipLaunchKernelGGL(k_prelude_micro, dim3(1), dim3(64), 0, 0, dH, db, 1e-3, dout, dc, 64);
        (void)hipDeviceSynchronize();
    }
    (void)hipMemcpy(c, dc, sizeof(c), hipMemcpyDeviceToHost);
    printf("cycles per call: pose_solve_l prelude %llu\n", c[3]);
    return bad != 0;
}
