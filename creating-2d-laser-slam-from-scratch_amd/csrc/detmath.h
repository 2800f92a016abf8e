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
/* 2^(j/128), j = 0..127, correctly rounded doubles (generated with 60-digit decimal arithmetic) */
#define SDM_EXPTAB_VALUES \
    0x1.0000000000000p+0, 0x1.0163da9fb3335p+0, 0x1.02c9a3e778061p+0, 0x1.04315e86e7f85p+0, \
    0x1.059b0d3158574p+0, 0x1.0706b29ddf6dep+0, 0x1.0874518759bc8p+0, 0x1.09e3ecac6f383p+0, \
    0x1.0b5586cf9890fp+0, 0x1.0cc922b7247f7p+0, 0x1.0e3ec32d3d1a2p+0, 0x1.0fb66affed31bp+0, \
    0x1.11301d0125b51p+0, 0x1.12abdc06c31ccp+0, 0x1.1429aaea92de0p+0, 0x1.15a98c8a58e51p+0, \
    0x1.172b83c7d517bp+0, 0x1.18af9388c8deap+0, 0x1.1a35beb6fcb75p+0, 0x1.1bbe084045cd4p+0, \
    0x1.1d4873168b9aap+0, 0x1.1ed5022fcd91dp+0, 0x1.2063b88628cd6p+0, 0x1.21f49917ddc96p+0, \
    0x1.2387a6e756238p+0, 0x1.251ce4fb2a63fp+0, 0x1.26b4565e27cddp+0, 0x1.284dfe1f56381p+0, \
    0x1.29e9df51fdee1p+0, 0x1.2b87fd0dad990p+0, 0x1.2d285a6e4030bp+0, 0x1.2ecafa93e2f56p+0, \
    0x1.306fe0a31b715p+0, 0x1.32170fc4cd831p+0, 0x1.33c08b26416ffp+0, 0x1.356c55f929ff1p+0, \
    0x1.371a7373aa9cbp+0, 0x1.38cae6d05d866p+0, 0x1.3a7db34e59ff7p+0, 0x1.3c32dc313a8e5p+0, \
    0x1.3dea64c123422p+0, 0x1.3fa4504ac801cp+0, 0x1.4160a21f72e2ap+0, 0x1.431f5d950a897p+0, \
    0x1.44e086061892dp+0, 0x1.46a41ed1d0057p+0, 0x1.486a2b5c13cd0p+0, 0x1.4a32af0d7d3dep+0, \
    0x1.4bfdad5362a27p+0, 0x1.4dcb299fddd0dp+0, 0x1.4f9b2769d2ca7p+0, 0x1.516daa2cf6642p+0, \
    0x1.5342b569d4f82p+0, 0x1.551a4ca5d920fp+0, 0x1.56f4736b527dap+0, 0x1.58d12d497c7fdp+0, \
    0x1.5ab07dd485429p+0, 0x1.5c9268a5946b7p+0, 0x1.5e76f15ad2148p+0, 0x1.605e1b976dc09p+0, \
    0x1.6247eb03a5585p+0, 0x1.6434634ccc320p+0, 0x1.6623882552225p+0, 0x1.68155d44ca973p+0, \
    0x1.6a09e667f3bcdp+0, 0x1.6c012750bdabfp+0, 0x1.6dfb23c651a2fp+0, 0x1.6ff7df9519484p+0, \
    0x1.71f75e8ec5f74p+0, 0x1.73f9a48a58174p+0, 0x1.75feb564267c9p+0, 0x1.780694fde5d3fp+0, \
    0x1.7a11473eb0187p+0, 0x1.7c1ed0130c132p+0, 0x1.7e2f336cf4e62p+0, 0x1.80427543e1a12p+0, \
    0x1.82589994cce13p+0, 0x1.8471a4623c7adp+0, 0x1.868d99b4492edp+0, 0x1.88ac7d98a6699p+0, \
    0x1.8ace5422aa0dbp+0, 0x1.8cf3216b5448cp+0, 0x1.8f1ae99157736p+0, 0x1.9145b0b91ffc6p+0, \
    0x1.93737b0cdc5e5p+0, 0x1.95a44cbc8520fp+0, 0x1.97d829fde4e50p+0, 0x1.9a0f170ca07bap+0, \
    0x1.9c49182a3f090p+0, 0x1.9e86319e32323p+0, 0x1.a0c667b5de565p+0, 0x1.a309bec4a2d33p+0, \
    0x1.a5503b23e255dp+0, 0x1.a799e1330b358p+0, 0x1.a9e6b5579fdbfp+0, 0x1.ac36bbfd3f37ap+0, \
    0x1.ae89f995ad3adp+0, 0x1.b0e07298db666p+0, 0x1.b33a2b84f15fbp+0, 0x1.b59728de5593ap+0, \
    0x1.b7f76f2fb5e47p+0, 0x1.ba5b030a1064ap+0, 0x1.bcc1e904bc1d2p+0, 0x1.bf2c25bd71e09p+0, \
    0x1.c199bdd85529cp+0, 0x1.c40ab5fffd07ap+0, 0x1.c67f12e57d14bp+0, 0x1.c8f6d9406e7b5p+0, \
    0x1.cb720dcef9069p+0, 0x1.cdf0b555dc3fap+0, 0x1.d072d4a07897cp+0, 0x1.d2f87080d89f2p+0, \
    0x1.d5818dcfba487p+0, 0x1.d80e316c98398p+0, 0x1.da9e603db3285p+0, 0x1.dd321f301b460p+0, \
    0x1.dfc97337b9b5fp+0, 0x1.e264614f5a129p+0, 0x1.e502ee78b3ff6p+0, 0x1.e7a51fbc74c83p+0, \
    0x1.ea4afa2a490dap+0, 0x1.ecf482d8e67f1p+0, 0x1.efa1bee615a27p+0, 0x1.f252b376bba97p+0, \
    0x1.f50765b6e4540p+0, 0x1.f7bfdad9cbe14p+0, 0x1.fa7c1819e90d8p+0, 0x1.fd3c22b8f71f1p+0
#define SDM_EXPTAB_N 128

/* exp of a float argument as the reference evaluates it: GridMapLogOdds.h:138 calls `exp` on a float
 * with only <cmath> in scope, which binds the DOUBLE exp (the built reference harness imports
 * exp@GLIBC, oracle/_ref/libhector_logodds_ref.so), so the value is (float)exp((double)x).
 * Table-driven double evaluation: k = round(x * 128 / ln2), r = x - k ln2/128 (Cody-Waite, |r| <=
 * ln2/256), exp(r) by its degree-4 Taylor polynomial, times 2^((k mod 128)/128) from the table and
 * 2^(k div 128); rounded once to float.  Equal to (float)exp((double)x) for EVERY float argument
 * (exhaustive check against the compiled reference header, tests/test_oracle_cpu.py::
 * test_grid_probability_pinned_exhaustive; a 64-entry table or a degree-3 polynomial is not).
 * Branch-free: the argument is clamped to [-110, 90], where the float result is already 0 / inf at
 * the ends, so no special case but NaN remains.  tab = the 128 table values (SDM_EXPTAB_VALUES; the
 * GPU reads an LDS copy). */
SDM_FN float sdm_expf_tab(float x, const double *tab)
{
    const double xd = (x == x) ? (x > 90.0f ? 90.0 : (x < -110.0f ? -110.0 : (double)x)) : 0.0;
    const double k = floor(xd * (128.0 * SDM_INV_LN2) + 0.5);
    double r = xd - k * (SDM_LN2_HI / 128.0);
    r = r - k * (SDM_LN2_LO / 128.0);
    double q = SDM_F4;
    q = SDM_F3 + r * q;
    q = SDM_F2 + r * q;
    q = 1.0 + r * q;
    q = 1.0 + r * q;
    const int ki = (int)k;
    const float res = (float)ldexp(tab[ki & 127] * q, ki >> 7);
    return (x != x) ? x : res;
}
/* host form (tests, host-side helpers); device code passes its LDS copy of the table */
static const double sdm_exptab_host[SDM_EXPTAB_N] = {SDM_EXPTAB_VALUES};
static inline float sdm_expf(float x) { return sdm_expf_tab(x, sdm_exptab_host); }


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
