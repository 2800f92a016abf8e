/* oracle/detmath.h -- TEST INFRASTRUCTURE (oracle side). Not shipped, never linked into the product.
 *
 * Deterministic double-precision sin / cos / exp used by the CPU oracle.
 *
 * Why this exists: the reference evaluates `sin(pose[2])`, `std::sin` inside Eigen::Rotation2Df
 * (lesson4/include/lesson4/hector_mapping/map/OccGridMapUtil.h:87-88, :439) and `exp(logOdds)`
 * (lesson4/include/lesson4/hector_mapping/map/GridMapLogOdds.h:138) through libm.  glibc and the
 * GPU's ocml differ in the last ulp, which would make a bit-exact GPU-vs-oracle comparison of the
 * map impossible.  Both sides therefore evaluate these three functions with the SAME explicit
 * sequence of IEEE double operations (no FMA contraction: compile with -ffp-contract=off) and round
 * the result to float once.  The product restates the identical algorithm in
 * creating-2d-laser-slam-from-scratch_amd/csrc/detmath.h; tests/test_detmath.py checks that the
 * two agree bit-for-bit, and tests/test_oracle_hector.py checks the libm variant of the oracle stays
 * within the pose tolerance of this one (the results differ from correctly-rounded libm by at most
 * one float ulp).
 */
#ifndef SLAM2D_ORACLE_DETMATH_H
#define SLAM2D_ORACLE_DETMATH_H

#include <math.h>

/* 1/n! for n = 2..17 (nearest doubles) */
#define ODM_F2 0.5
#define ODM_F3 0.16666666666666666
#define ODM_F4 0.041666666666666664
#define ODM_F5 0.008333333333333333
#define ODM_F6 0.001388888888888889
#define ODM_F7 0.0001984126984126984
#define ODM_F8 2.48015873015873e-05
#define ODM_F9 2.7557319223985893e-06
#define ODM_F10 2.755731922398589e-07
#define ODM_F11 2.505210838544172e-08
#define ODM_F12 2.08767569878681e-09
#define ODM_F13 1.6059043836821613e-10
#define ODM_F14 1.1470745597729725e-11
#define ODM_F15 7.647163731819816e-13
#define ODM_F16 4.779477332387385e-14

/* Cody-Waite split of pi/2 (fdlibm constants: 33 + 33 + rest bits) */
#define ODM_PIO2_1 1.57079632673412561417e+00
#define ODM_PIO2_2 6.07710050630396597660e-11
#define ODM_PIO2_3 2.02226624871116645580e-21
#define ODM_TWO_OVER_PI 0.6366197723675814
/* ln2 split (fdlibm) */
#define ODM_LN2_HI 6.93147180369123816490e-01
#define ODM_LN2_LO 1.90821492927058770002e-10
#define ODM_INV_LN2 1.4426950408889634

static inline double odm_sin_kernel(double r)
{
    double z = r * r;
    double p = -ODM_F15;
    p = ODM_F13 + z * p;
    p = -ODM_F11 + z * p;
    p = ODM_F9 + z * p;
    p = -ODM_F7 + z * p;
    p = ODM_F5 + z * p;
    p = -ODM_F3 + z * p;
    /* sin r = r + r*z*p  with p = -1/3! + z/5! - ... */
    return r + (r * z) * p;
}

static inline double odm_cos_kernel(double r)
{
    double z = r * r;
    double p = ODM_F16;
    p = -ODM_F14 + z * p;
    p = ODM_F12 + z * p;
    p = -ODM_F10 + z * p;
    p = ODM_F8 + z * p;
    p = -ODM_F6 + z * p;
    p = ODM_F4 + z * p;
    p = -ODM_F2 + z * p;
    return 1.0 + z * p;
}

/* returns quadrant in *q and reduced argument */
static inline double odm_reduce_pio2(double x, int *q)
{
    double k = floor(x * ODM_TWO_OVER_PI + 0.5);
    double r = x - k * ODM_PIO2_1;
    r = r - k * ODM_PIO2_2;
    r = r - k * ODM_PIO2_3;
    long long ki = (long long)k;
    *q = (int)(ki & 3);
    return r;
}

static inline double odm_sin(double x)
{
    if (x != x) return x;
    int q;
    double r = odm_reduce_pio2(x, &q);
    switch (q) {
    case 0: return odm_sin_kernel(r);
    case 1: return odm_cos_kernel(r);
    case 2: return -odm_sin_kernel(r);
    default: return -odm_cos_kernel(r);
    }
}

static inline double odm_cos(double x)
{
    if (x != x) return x;
    int q;
    double r = odm_reduce_pio2(x, &q);
    switch (q) {
    case 0: return odm_cos_kernel(r);
    case 1: return -odm_sin_kernel(r);
    case 2: return -odm_cos_kernel(r);
    default: return odm_sin_kernel(r);
    }
}

static inline double odm_exp(double x)
{
    if (x != x) return x;
    if (x > 709.0) return HUGE_VAL;
    if (x < -745.5) return 0.0;
    double k = floor(x * ODM_INV_LN2 + 0.5);
    double r = x - k * ODM_LN2_HI;
    r = r - k * ODM_LN2_LO;
    double p = ODM_F13;
    p = ODM_F12 + r * p;
    p = ODM_F11 + r * p;
    p = ODM_F10 + r * p;
    p = ODM_F9 + r * p;
    p = ODM_F8 + r * p;
    p = ODM_F7 + r * p;
    p = ODM_F6 + r * p;
    p = ODM_F5 + r * p;
    p = ODM_F4 + r * p;
    p = ODM_F3 + r * p;
    p = ODM_F2 + r * p;
    p = 1.0 + r * p;
    p = 1.0 + r * p;
    return ldexp(p, (int)k);
}

/* float-in / float-out wrappers: the single rounding point */
static inline float odm_sinf(float x) { return (float)odm_sin((double)x); }
static inline float odm_cosf(float x) { return (float)odm_cos((double)x); }
/* 2^(j/128), j = 0..127, correctly rounded doubles (generated with 60-digit decimal arithmetic) */
#define ODM_EXPTAB_VALUES \
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
#define ODM_EXPTAB_N 128

/* exp of a float argument as the reference evaluates it: GridMapLogOdds.h:138 calls `exp` on a float
 * with only <cmath> in scope, which binds the DOUBLE exp (the built reference harness imports
 * exp@GLIBC, oracle/_ref/libhector_logodds_ref.so), so the value is (float)exp((double)x).
 * Table-driven double evaluation: k = round(x * 128 / ln2), r = x - k ln2/128 (Cody-Waite, |r| <=
 * ln2/256), exp(r) by its degree-4 Taylor polynomial, times 2^((k mod 128)/128) from the table and
 * 2^(k div 128); rounded once to float.  Equal to (float)exp((double)x) for EVERY float argument
 * (exhaustive check against the compiled reference header, tests/test_oracle_cpu.py::
 * test_grid_probability_pinned_exhaustive; a 64-entry table or a degree-3 polynomial is not).
 * Branch-free: the argument is clamped to [-110, 90], where the float result is already 0 / inf at
 * the ends, so no special case but NaN remains.  tab = the 128 table values (ODM_EXPTAB_VALUES; the
 * GPU reads an LDS copy). */
static inline float odm_expf_tab(float x, const double *tab)
{
    const double xd = (x == x) ? (x > 90.0f ? 90.0 : (x < -110.0f ? -110.0 : (double)x)) : 0.0;
    const double k = floor(xd * (128.0 * ODM_INV_LN2) + 0.5);
    double r = xd - k * (ODM_LN2_HI / 128.0);
    r = r - k * (ODM_LN2_LO / 128.0);
    double q = ODM_F4;
    q = ODM_F3 + r * q;
    q = ODM_F2 + r * q;
    q = 1.0 + r * q;
    q = 1.0 + r * q;
    const int ki = (int)k;
    const float res = (float)ldexp(tab[ki & 127] * q, ki >> 7);
    return (x != x) ? x : res;
}
static const double odm_exptab[ODM_EXPTAB_N] = {ODM_EXPTAB_VALUES};
static inline float odm_expf(float x) { return odm_expf_tab(x, odm_exptab); }


/* atan / atan2 in double (PL-ICP possible_interval, CSM icp_corr_dumb.c): |x| > 1 -> pi/2 - atan(1/x);
 * t > tan(pi/12) -> pi/6 + atan((t*sqrt3 - 1)/(sqrt3 + t)); Taylor series to u^29 on |u| <= 0.268
 * (truncation < 1e-18).  Same op sequence on host and device. */
#define ODM_AT0 1.0
#define ODM_AT1 -0.3333333333333333
#define ODM_AT2 0.2
#define ODM_AT3 -0.14285714285714285
#define ODM_AT4 0.1111111111111111
#define ODM_AT5 -0.09090909090909091
#define ODM_AT6 0.07692307692307693
#define ODM_AT7 -0.06666666666666667
#define ODM_AT8 0.058823529411764705
#define ODM_AT9 -0.05263157894736842
#define ODM_AT10 0.047619047619047616
#define ODM_AT11 -0.043478260869565216
#define ODM_AT12 0.04
#define ODM_AT13 -0.037037037037037035
#define ODM_AT14 0.034482758620689655
#define ODM_SQRT3 1.7320508075688772
#define ODM_PI 3.141592653589793
#define ODM_PI_2 1.5707963267948966
#define ODM_PI_6 0.5235987755982988
#define ODM_TAN_PI_12 0.2679491924311227
static inline double odm_atan(double x)
{
    if (x != x) return x;
    const double ax = fabs(x);
    const int inv = ax > 1.0;
    const double t = inv ? 1.0 / ax : ax;
    const int red = t > ODM_TAN_PI_12;
    const double u = red ? (t * ODM_SQRT3 - 1.0) / (ODM_SQRT3 + t) : t;
    const double z = u * u;
    double p = ODM_AT14;
    p = ODM_AT13 + z * p;
    p = ODM_AT12 + z * p;
    p = ODM_AT11 + z * p;
    p = ODM_AT10 + z * p;
    p = ODM_AT9 + z * p;
    p = ODM_AT8 + z * p;
    p = ODM_AT7 + z * p;
    p = ODM_AT6 + z * p;
    p = ODM_AT5 + z * p;
    p = ODM_AT4 + z * p;
    p = ODM_AT3 + z * p;
    p = ODM_AT2 + z * p;
    p = ODM_AT1 + z * p;
    p = ODM_AT0 + z * p;
    double r = u * p;
    if (red) r = ODM_PI_6 + r;
    if (inv) r = ODM_PI_2 - r;
    return x < 0.0 ? -r : r;
}
static inline double odm_atan2(double y, double x)
{
    if (x != x || y != y) return x + y;
    if (x > 0.0) return odm_atan(y / x);
    if (x < 0.0) return y >= 0.0 ? odm_atan(y / x) + ODM_PI : odm_atan(y / x) - ODM_PI;
    if (y > 0.0) return ODM_PI_2;
    if (y < 0.0) return -ODM_PI_2;
    return 0.0;
}

#endif
