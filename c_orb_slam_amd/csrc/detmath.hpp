// detmath.hpp -- deterministic double sin/cos/atan2 shared (by algorithm) with the
// CPU oracle (oracle/sim3.c).  libm and the GPU's ocml differ in the last ulp;
// the reference's Sim3 path (cv::Rodrigues, atan2 in Sim3Solver.cc:282) feeds
// inlier decisions, so both sides evaluate these exact IEEE operation sequences.
#pragma once
#include <hip/hip_runtime.h>

namespace orbgpu {
namespace detmath {

__device__ __forceinline__ void sincos_d(double x, double* s_out, double* c_out) {
    const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
                 S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
                 S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
    const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
                 C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
                 C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
    const double pio2_1 = 1.57079632673412561417e+00, pio2_1t = 6.07710050650619224932e-11;
    const double invpio2 = 6.36619772367581382433e-01;
    const double fn = rint(x * invpio2);
    const int n = (int)fn;
    const double y = (x - fn * pio2_1) - fn * pio2_1t;
    const double z = y * y;
    const double r = S2 + z * (S3 + z * (S4 + z * (S5 + z * S6)));
    const double s = y + (z * y) * (S1 + z * r);
    const double rc = z * (C1 + z * (C2 + z * (C3 + z * (C4 + z * (C5 + z * C6)))));
    const double c = 1.0 - (0.5 * z - z * rc);
    switch (n & 3) {
        case 0: *s_out = s; *c_out = c; break;
        case 1: *s_out = c; *c_out = -s; break;
        case 2: *s_out = -s; *c_out = -c; break;
        default: *s_out = -c; *c_out = s; break;
    }
}

__device__ __forceinline__ double atan01(double x) {
    x = x / (1.0 + sqrt(1.0 + x * x));
    x = x / (1.0 + sqrt(1.0 + x * x));
    const double x2 = x * x;
    double term = x, sum = x;
    for (int k = 1; k <= 14; k++) {
        term = term * x2;
        sum += ((k & 1) ? -term : term) / (2 * k + 1);
    }
    return 4.0 * sum;
}

__device__ __forceinline__ double atan2_d(double y, double x) {
    const double ay = fabs(y), ax = fabs(x);
    double a;
    if (ax == 0 && ay == 0) a = 0;
    else if (ay <= ax) a = atan01(ay / ax);
    else a = 1.57079632679489655800e+00 - atan01(ax / ay);
    if (x < 0) a = 3.14159265358979311600e+00 - a;
    return y < 0 ? -a : a;
}

// fdlibm __ieee754_exp as an IEEE operation sequence (oracle/ba.c ora_det_exp): g2o::Sim3's
// exp(sigma) (sim3.h:84) in OptimizeSim3's numeric Jacobian and update.
__device__ __forceinline__ double exp_d(double x) {
    const double ln2HI = 6.93147180369123816490e-01, ln2LO = 1.90821492927058770002e-10;
    const double invln2 = 1.44269504088896338700e+00;
    const double P1 = 1.66666666666666019037e-01, P2 = -2.77777777770155933842e-03,
                 P3 = 6.61375632143793436117e-05, P4 = -1.65339022054652515390e-06,
                 P5 = 4.13813679705723846039e-08;
    if (x != x) return x;
    if (x > 7.09782712893383973096e+02) return HUGE_VAL;
    if (x < -7.45133219101941108420e+02) return 0.0;
    const int xsb = x < 0;
    const double ax = fabs(x);
    double hi = 0, lo = 0;
    int k = 0;
    if (ax > 0.5 * 6.93147180559945286227e-01) {
        if (ax < 1.5 * 6.93147180559945286227e-01) {
            hi = x - (xsb ? -ln2HI : ln2HI);
            lo = xsb ? -ln2LO : ln2LO;
            k = 1 - xsb - xsb;
        } else {
            k = (int)(invln2 * x + (xsb ? -0.5 : 0.5));
            const double t = k;
            hi = x - t * ln2HI;
            lo = t * ln2LO;
        }
        x = hi - lo;
    } else if (ax < 3.7252902984e-09) {
        return 1.0 + x;
    }
    const double t = x * x;
    const double c = x - t * (P1 + t * (P2 + t * (P3 + t * (P4 + t * P5))));
    if (k == 0) return 1.0 - ((x * c) / (c - 2.0) - x);
    const double y = 1.0 - ((lo - (x * c) / (2.0 - c)) - hi);
    return ldexp(y, k);
}

}  // namespace detmath
}  // namespace orbgpu
