// Host check of the PL-ICP float atan bracket (csrc/plicp_kernels.hip pl_fatan01 / pl_fatan / pl_fatan2):
// the worst error must stay well under PL_ATAN_EPS = 2e-6.  The polynomial below must equal the
// kernel's (tests/test_plicp_atan_cpu.py compares the constants with the kernel source).
//   gcc -O2 -fopenmp tools/check_fatan.c -lm && ./a.out          full: every float + 2e8 pairs (about 3 min)
//   ./a.out quick                                                edge regions + samples (seconds; the CPU test)
// Arguments the kernel sends to the exact path are skipped here as there: zero, non-finite, and atan2
// pairs whose larger float magnitude is subnormal (their float rounding is not relative to 2^-24).
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
static const float C_POLY[8] = {-0.003962602f, 0.021518489f, -0.055396412f, 0.096028686f,
                                -0.13892588f, 0.19943212f, -0.33329552f, 0.99999923f};
static inline float f01(float t, int fma_)
{
    float z = t * t, q = C_POLY[0];
    for (int i = 1; i < 8; i++) q = fma_ ? fmaf(z, q, C_POLY[i]) : C_POLY[i] + z * q;
    return t * q;
}
static inline float fat(float x, int m) { return x > 1.0f ? 1.5707963f - f01(1.0f / x, m) : f01(x, m); }
static inline float fat2(float y, float x, int m)
{
    float ax = fabsf(x), ay = fabsf(y);
    float r = ay > ax ? 1.5707963f - f01(ax / ay, m) : f01(ay / ax, m);
    if (x < 0.0f) r = 3.1415927f - r;
    return y < 0.0f ? -r : r;
}
static double err_atan(float x, int m) { return fabs((double)fat(x, m) - atan((double)x)); }
// the kernel's fast-path condition (pl_theta_cells) and the error against atan2 of the DOUBLE arguments
static int fast2(float fy, float fx) { return fminf(fabsf(fx), fabsf(fy)) >= FLT_MIN; }  /* both components normal (pl_polar_cells) */
static double err_atan2(double y, double x, int m)
{
    float fx = (float)x, fy = (float)y;
    if (!isfinite(fx) || !isfinite(fy) || !fast2(fy, fx)) return 0.0;
    double e = fabs((double)fat2(fy, fx, m) - atan2(y, x));
    if (e > 2 * M_PI - 1) e = fabs(e - 2 * M_PI);
    return e;
}
static double urand(void) { return drand48(); }
int main(int argc, char **argv)
{
    const int quick = argc > 1 && strcmp(argv[1], "quick") == 0;
    double worst1 = 0, worst2 = 0;
    for (int m = 0; m < 2; m++) {
        if (!quick) {
#pragma omp parallel
            {
                double lw = 0;
#pragma omp for schedule(static)
                for (int64_t b = 0; b < 0x7F800000LL; b++) {
                    uint32_t u = (uint32_t)b;
                    float x;
                    memcpy(&x, &u, 4);
                    double e = err_atan(x, m);
                    if (e > lw) lw = e;
                }
#pragma omp critical
                if (lw > worst1) worst1 = lw;
            }
        } else {
            // atan: bit-pattern samples over every binade, dense around 1 (the 1/x switch), tiny and huge
            srand48(7);
            for (long i = 0; i < 4000000L; i++) {
                uint32_t u = (uint32_t)(urand() * 0x7F800000u);
                float x;
                memcpy(&x, &u, 4);
                double e = err_atan(x, m);
                if (e > worst1) worst1 = e;
            }
            for (int side = 0; side < 2; side++) {  // the 64 floats on each side of 1
                float x = 1.0f;
                for (int j = 0; j < 64; j++) {
                    x = nextafterf(x, side ? 2.0f : 0.0f);
                    double e = err_atan(x, m);
                    if (e > worst1) worst1 = e;
                }
            }
            for (int k = 0; k < 2000000; k++) {
                float x = 1.0f + (float)((urand() - 0.5) * 2e-3);
                double e = err_atan(x, m);
                if (e > worst1) worst1 = e;
                e = err_atan(FLT_MIN * (float)urand(), m);  // subnormal
                if (e > worst1) worst1 = e;
                e = err_atan((float)(1e30 * urand()), m);
                if (e > worst1) worst1 = e;
            }
        }
        srand48(1);
        const long N = quick ? 6000000L : 200000000L;
        for (long i = 0; i < N; i++) {
            double y = (urand() - 0.5) * pow(10, urand() * 12 - 6), x = (urand() - 0.5) * pow(10, urand() * 12 - 6);
            switch (i % 8) {
            case 1: y = x * (1 + 1e-9 * (urand() - 0.5)); break;          // |y/x| ~ 1 (the ay > ax switch)
            case 2: y = -x * (1 + 1e-7 * (urand() - .5)); break;
            case 3: y = x * 1e-30 * urand(); break;                       // tiny ratio
            case 4: x = y * 1e-30 * urand(); break;                       // huge ratio
            case 5: x = (urand() - 0.5) * 2.5e-38; y = (urand() - 0.5) * 2.5e-38; break;  // around FLT_MIN
            case 6: x = -fabs(x); y = copysign(1e-12 * fabs(x), (urand() < 0.5) ? -1.0 : 1.0); break;  // near +-pi
            case 7: if (i % 16 == 7) y = (urand() - 0.5) * 2.0e-39; break;  // one subnormal component: exact path
            default: break;
            }
            double e = err_atan2(y, x, m);
            if (e > worst2) worst2 = e;
        }
    }
    printf("atan max err %.3e\natan2 max err %.3e\n", worst1, worst2);
    return (worst1 < 1e-6 && worst2 < 1e-6) ? 0 : 1;
}
