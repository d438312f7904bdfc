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


// fdlibm __ieee754_log as an IEEE operation sequence (oracle/matchers2.c ora_det_log), for
// positive finite x: MapPoint::PredictScale's log(ratio) (MapPoint.cc:402-417) is glibc logf
// on a float; (float)log_d(x) equals it on every float the tracking path feeds it
// (tests/test_oracle_kat.py::test_det_log_predict_scale_exhaustive).
__device__ __forceinline__ double log_d(double x) {
    const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10;
    const double Lg1 = 6.666666666666735130e-01, Lg2 = 3.999999999940941908e-01, Lg3 = 2.857142874366239149e-01,
                 Lg4 = 2.222219843214978396e-01, Lg5 = 1.818357216161805012e-01, Lg6 = 1.531383769920937332e-01,
                 Lg7 = 1.479819860511658591e-01;
    if (!(x > 0.0)) return x == 0.0 ? -HUGE_VAL : (x - x) / 0.0;
    if (x > 1.79769313486231570815e+308) return x;
    unsigned long long bits = (unsigned long long)__double_as_longlong(x);
    int hx = (int)(bits >> 32);
    const unsigned lx = (unsigned)bits;
    int k = 0;
    if (hx < 0x00100000) {   // subnormal: scale by 2^54
        x *= 1.80143985094819840000e+16;
        k -= 54;
        bits = (unsigned long long)__double_as_longlong(x);
        hx = (int)(bits >> 32);
    }
    (void)lx;
    k += (hx >> 20) - 1023;
    hx &= 0x000fffff;
    const int i0 = (hx + 0x95f64) & 0x100000;
    bits = ((unsigned long long)(unsigned)(hx | (i0 ^ 0x3ff00000)) << 32) | (bits & 0xffffffffull);
    x = __longlong_as_double((long long)bits);
    k += (i0 >> 20);
    const double f = x - 1.0;
    const double dk = (double)k;
    if ((0x000fffff & (2 + hx)) < 3) {   // |f| < 2^-20
        if (f == 0.0) return k == 0 ? 0.0 : dk * ln2_hi + dk * ln2_lo;
        const double R = f * f * (0.5 - 0.33333333333333333 * f);
        return k == 0 ? f - R : dk * ln2_hi - ((R - dk * ln2_lo) - f);
    }
    const double s = f / (2.0 + f);
    const double z = s * s;
    int i = hx - 0x6147a;
    const double w = z * z;
    const int j = 0x6b851 - hx;
    const double t1 = w * (Lg2 + w * (Lg4 + w * Lg6));
    const double t2 = z * (Lg1 + w * (Lg3 + w * (Lg5 + w * Lg7)));
    i |= j;
    const double R = t2 + t1;
    if (i > 0) {
        const double hfsq = 0.5 * f * f;
        return k == 0 ? f - (hfsq - s * (hfsq + R)) : dk * ln2_hi - ((hfsq - (s * (hfsq + R) + dk * ln2_lo)) - f);
    }
    return k == 0 ? f - s * (f - R) : dk * ln2_hi - ((s * (f - R) - dk * ln2_lo) - f);
}

// MapPoint::PredictScale(currentDist, Frame*) (MapPoint.cc:402-417)
__device__ __forceinline__ int predict_scale(float maxDistance, float currentDist, float logScaleFactor, int nlevels) {
    const float ratio = maxDistance / currentDist;
    int n = (int)ceilf((float)log_d((double)ratio) / logScaleFactor);
    return n < 0 ? 0 : (n >= nlevels ? nlevels - 1 : n);
}

}  // namespace detmath
}  // namespace orbgpu
