/* csrc/detmath.h -- product side (HIP device + host).
 *
 * Deterministic sin / cos (double) and exp (float) for the Hector kernels.
 *
 * Why this exists: the reference evaluates `sin(pose[2])`, `std::sin` inside Eigen::Rotation2Df
 * (lesson4/include/lesson4/hector_mapping/map/OccGridMapUtil.h:87-88, :439) and `exp(logOdds)`
 * (lesson4/include/lesson4/hector_mapping/map/GridMapLogOdds.h:138) through libm.  glibc and the
 * GPU's ocml differ in the last ulp, which would make a bit-exact GPU-vs-oracle comparison of the
 * map impossible.  Both sides therefore evaluate these three functions with the SAME explicit
 * sequence of IEEE double operations (no FMA contraction: compile with -ffp-contract=off) and round
 * the result to float once.  The CPU oracle restates the identical algorithm in oracle/detmath.h;
 * tests/test_detmath.py checks that the two agree bit-for-bit.  On 120k sampled arguments the float
 * results equal correctly rounded sin/cos/exp.
 */
#ifndef SLAM2D_CSRC_DETMATH_H
#define SLAM2D_CSRC_DETMATH_H

#include <math.h>

/* Device and host: the same op sequence, compiled with -ffp-contract=off on both sides. */
#if defined(__HIPCC__)
#define SDM_FN __host__ __device__ static inline
#else
#define SDM_FN static inline
#endif

/* 1/n! for n = 2..17 (nearest doubles) */
#define SDM_F2 0.5
#define SDM_F3 0.16666666666666666
#define SDM_F4 0.041666666666666664
#define SDM_F5 0.008333333333333333
#define SDM_F6 0.001388888888888889
#define SDM_F7 0.0001984126984126984
#define SDM_F8 2.48015873015873e-05
#define SDM_F9 2.7557319223985893e-06
#define SDM_F10 2.755731922398589e-07
#define SDM_F11 2.505210838544172e-08
#define SDM_F12 2.08767569878681e-09
#define SDM_F13 1.6059043836821613e-10
#define SDM_F14 1.1470745597729725e-11
#define SDM_F15 7.647163731819816e-13
#define SDM_F16 4.779477332387385e-14

/* Cody-Waite split of pi/2 (fdlibm constants: 33 + 33 + rest bits) */
#define SDM_PIO2_1 1.57079632673412561417e+00
#define SDM_PIO2_2 6.07710050630396597660e-11
#define SDM_PIO2_3 2.02226624871116645580e-21
#define SDM_TWO_OVER_PI 0.6366197723675814
/* ln2 split (fdlibm) */
#define SDM_LN2_HI 6.93147180369123816490e-01
#define SDM_LN2_LO 1.90821492927058770002e-10
#define SDM_INV_LN2 1.4426950408889634

SDM_FN double sdm_sin_kernel(double r)
{
    double z = r * r;
    double p = -SDM_F15;
    p = SDM_F13 + z * p;
    p = -SDM_F11 + z * p;
    p = SDM_F9 + z * p;
    p = -SDM_F7 + z * p;
    p = SDM_F5 + z * p;
    p = -SDM_F3 + z * p;
    /* sin r = r + r*z*p  with p = -1/3! + z/5! - ... */
    return r + (r * z) * p;
}

SDM_FN double sdm_cos_kernel(double r)
{
    double z = r * r;
    double p = SDM_F16;
    p = -SDM_F14 + z * p;
    p = SDM_F12 + z * p;
    p = -SDM_F10 + z * p;
    p = SDM_F8 + z * p;
    p = -SDM_F6 + z * p;
    p = SDM_F4 + z * p;
    p = -SDM_F2 + z * p;
    return 1.0 + z * p;
}

/* returns quadrant in *q and reduced argument */
SDM_FN double sdm_reduce_pio2(double x, int *q)
{
    double k = floor(x * SDM_TWO_OVER_PI + 0.5);
    double r = x - k * SDM_PIO2_1;
    r = r - k * SDM_PIO2_2;
    r = r - k * SDM_PIO2_3;
    long long ki = (long long)k;
    *q = (int)(ki & 3);
    return r;
}

SDM_FN double sdm_sin(double x)
{
    if (x != x) return x;
    int q;
    double r = sdm_reduce_pio2(x, &q);
    switch (q) {
    case 0: return sdm_sin_kernel(r);
    case 1: return sdm_cos_kernel(r);
    case 2: return -sdm_sin_kernel(r);
    default: return -sdm_cos_kernel(r);
    }
}

SDM_FN double sdm_cos(double x)
{
    if (x != x) return x;
    int q;
    double r = sdm_reduce_pio2(x, &q);
    switch (q) {
    case 0: return sdm_cos_kernel(r);
    case 1: return -sdm_sin_kernel(r);
    case 2: return -sdm_cos_kernel(r);
    default: return sdm_sin_kernel(r);
    }
}

SDM_FN double sdm_exp(double x)
{
    if (x != x) return x;
    if (x > 709.0) return HUGE_VAL;
    if (x < -745.5) return 0.0;
    double k = floor(x * SDM_INV_LN2 + 0.5);
    double r = x - k * SDM_LN2_HI;
    r = r - k * SDM_LN2_LO;
    double p = SDM_F13;
    p = SDM_F12 + r * p;
    p = SDM_F11 + r * p;
    p = SDM_F10 + r * p;
    p = SDM_F9 + r * p;
    p = SDM_F8 + r * p;
    p = SDM_F7 + r * p;
    p = SDM_F6 + r * p;
    p = SDM_F5 + r * p;
    p = SDM_F4 + r * p;
    p = SDM_F3 + r * p;
    p = SDM_F2 + r * p;
    p = 1.0 + r * p;
    p = 1.0 + r * p;
    return ldexp(p, (int)k);
}

/* float-in / float-out wrappers: the single rounding point */
SDM_FN float sdm_sinf(float x) { return (float)sdm_sin((double)x); }
SDM_FN float sdm_cosf(float x) { return (float)sdm_cos((double)x); }
/* exp of a float argument as the reference evaluates it: GridMapLogOdds.h:138 calls `exp` on a float
 * with only <cmath> in scope, which binds the DOUBLE exp (the built reference harness imports
 * exp@GLIBC, oracle/_ref/libhector_logodds_ref.so), so the value is (float)exp((double)x).  The
 * double sequence of sdm_exp rounded once to float equals it for every float argument (exhaustive
 * check against the compiled reference header, tests/test_oracle_cpu.py::test_grid_probability_pinned).
 * Branch-free: the argument is clamped to [-110, 90], where the float result is already 0 / inf at
 * the ends, so no special case but NaN remains and the GPU keeps its gathers in flight. */
SDM_FN float sdm_expf(float x)
{
    const double xd = (x == x) ? (x > 90.0f ? 90.0 : (x < -110.0f ? -110.0 : (double)x)) : 0.0;
    const double k = floor(xd * SDM_INV_LN2 + 0.5);
    double r = xd - k * SDM_LN2_HI;
    r = r - k * SDM_LN2_LO;
    double q = SDM_F13;
    q = SDM_F12 + r * q;
    q = SDM_F11 + r * q;
    q = SDM_F10 + r * q;
    q = SDM_F9 + r * q;
    q = SDM_F8 + r * q;
    q = SDM_F7 + r * q;
    q = SDM_F6 + r * q;
    q = SDM_F5 + r * q;
    q = SDM_F4 + r * q;
    q = SDM_F3 + r * q;
    q = SDM_F2 + r * q;
    q = 1.0 + r * q;
    q = 1.0 + r * q;
    const float res = (float)ldexp(q, (int)k);
    return (x != x) ? x : res;
}


/* atan / atan2 in double (PL-ICP possible_interval, CSM icp_corr_dumb.c): |x| > 1 -> pi/2 - atan(1/x);
 * t > tan(pi/12) -> pi/6 + atan((t*sqrt3 - 1)/(sqrt3 + t)); Taylor series to u^29 on |u| <= 0.268
 * (truncation < 1e-18).  Same op sequence on host and device. */
#define SDM_AT0 1.0
#define SDM_AT1 -0.3333333333333333
#define SDM_AT2 0.2
#define SDM_AT3 -0.14285714285714285
#define SDM_AT4 0.1111111111111111
#define SDM_AT5 -0.09090909090909091
#define SDM_AT6 0.07692307692307693
#define SDM_AT7 -0.06666666666666667
#define SDM_AT8 0.058823529411764705
#define SDM_AT9 -0.05263157894736842
#define SDM_AT10 0.047619047619047616
#define SDM_AT11 -0.043478260869565216
#define SDM_AT12 0.04
#define SDM_AT13 -0.037037037037037035
#define SDM_AT14 0.034482758620689655
#define SDM_SQRT3 1.7320508075688772
#define SDM_PI 3.141592653589793
#define SDM_PI_2 1.5707963267948966
#define SDM_PI_6 0.5235987755982988
#define SDM_TAN_PI_12 0.2679491924311227
SDM_FN double sdm_atan(double x)
{
    if (x != x) return x;
    const double ax = fabs(x);
    const int inv = ax > 1.0;
    const double t = inv ? 1.0 / ax : ax;
    const int red = t > SDM_TAN_PI_12;
    const double u = red ? (t * SDM_SQRT3 - 1.0) / (SDM_SQRT3 + t) : t;
    const double z = u * u;
    double p = SDM_AT14;
    p = SDM_AT13 + z * p;
    p = SDM_AT12 + z * p;
    p = SDM_AT11 + z * p;
    p = SDM_AT10 + z * p;
    p = SDM_AT9 + z * p;
    p = SDM_AT8 + z * p;
    p = SDM_AT7 + z * p;
    p = SDM_AT6 + z * p;
    p = SDM_AT5 + z * p;
    p = SDM_AT4 + z * p;
    p = SDM_AT3 + z * p;
    p = SDM_AT2 + z * p;
    p = SDM_AT1 + z * p;
    p = SDM_AT0 + z * p;
    double r = u * p;
    if (red) r = SDM_PI_6 + r;
    if (inv) r = SDM_PI_2 - r;
    return x < 0.0 ? -r : r;
}
SDM_FN double sdm_atan2(double y, double x)
{
    if (x != x || y != y) return x + y;
    if (x > 0.0) return sdm_atan(y / x);
    if (x < 0.0) return y >= 0.0 ? sdm_atan(y / x) + SDM_PI : sdm_atan(y / x) - SDM_PI;
    if (y > 0.0) return SDM_PI_2;
    if (y < 0.0) return -SDM_PI_2;
    return 0.0;
}

#endif
