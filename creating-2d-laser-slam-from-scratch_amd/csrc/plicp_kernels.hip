// plicp_kernels.hip -- MI355X kernel of the PL-ICP scan-matching path (lesson3 front-end).
//
//   pl_icp_kernel   one 256-thread workgroup per scan pair: the whole point-to-line ICP loop of CSM's
//                   sm_icp as lesson3 configures it (lesson3/src/plicp_odometry.cc:58-186, :391), in
//                   double precision.  Per iteration:
//                     correspondences  every thread owns rays i = tid + 256 k; exact closest valid
//                                      reference point inside CSM's polar search interval (reference
//                                      points resident in LDS), j2 = closer valid neighbour;
//                     trimming         the two order statistics of the point-to-segment errors by an
//                                      radix select on the errors' bit patterns (double-buffered LDS
//                                      histograms, early settle on a single-key bin);
//                     doubles          per-reference minimum dist^2 by LDS 64-bit atomicMin on the bits;
//                     estimate         the 14 point-to-line GPC sums (64-lane xor butterfly, then the
//                                      4 waves), the constrained 4x4 solve by wave 0 (bisection on
//                                      the Lagrange multiplier), oscillation hash, convergence test.
// The CPU checker oracle/plicp_oracle.c evaluates the same op sequence (-ffp-contract=off here and
// there), so results agree bit for bit; CSM itself is absent (parity unpinned).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "../../include/slam2d/plicp.h"
#include "detmath.h"

namespace s2d {

constexpr int PL_THREADS = 256;
constexpr int PL_RPT_MAX = 8;                   // rays per thread: max_rays <= 2048
constexpr int PL_MAX_RAYS = PL_THREADS * PL_RPT_MAX;
static_assert(PL_MAX_RAYS == PL_MAX_SCAN_RAYS, "include/slam2d/plicp.h names the kernel's ray limit");
constexpr int PL_MAX_IT = 64;
#ifndef PL_CORE
#define PL_CORE 4   // half-width of the core search around a point's own cell
#endif

__device__ __forceinline__ double pl_dist_to_segment(double ax, double ay, double bx, double by, double x, double y)
{
    const double t0 = ax - bx, t1 = ay - by;
    const double one_on_r = 1.0 / sqrt(t0 * t0 + t1 * t1);
    const double nx = t1 * one_on_r, ny = -t0 * one_on_r;
    const double rho = nx * ax + ny * ay;
    const double lx = (nx * rho + ny * ny * x) - nx * ny * y;
    const double ly = (ny * rho - nx * ny * x) + nx * nx * y;
    double qx, qy;
    if ((lx - ax) * (lx - bx) + (ly - ay) * (ly - by) < 0.0) {
        qx = lx;
        qy = ly;
    } else {
        const double da = (ax - x) * (ax - x) + (ay - y) * (ay - y);
        const double db = (bx - x) * (bx - x) + (by - y) * (by - y);
        if (da < db) {
            qx = ax;
            qy = ay;
        } else {
            qx = bx;
            qy = by;
        }
    }
    return sqrt((qx - x) * (qx - x) + (qy - y) * (qy - y));
}

// Every atan / atan2 on the correspondence path only feeds an integer (a cell index or a window
// half-width) through a monotone double expression.  So each is first evaluated by a cheap float
// approximation a with |a - exact| < PL_ATAN_EPS (measured by tools/check_fatan.c: 2.3e-7 worst case
// over every non-negative float for pl_fatan, 4.1e-7 over 2e8 sampled double pairs for pl_fatan2, the
// double -> float rounding of the arguments included; its quick mode -- edge regions: |y/x| near 1,
// tiny / huge ratios, arguments around FLT_MIN, near +-pi -- runs in tests/test_plicp_atan_cpu.py;
// NaN / inf / zero / subnormal arguments fall to the exact path): the integer the expression yields at a - eps and at a + eps brackets
// the exact one, and when the two agree that is the result -- the exact double evaluation (the
// reference's value, sdm_atan / sdm_atan2) runs only when the bracket straddles an integer boundary
// (about 2 eps / cell width, < 1e-3 of the evaluations).  Results are the exact path's, bit for bit.
constexpr double PL_ATAN_EPS = 2e-6;

// atan(t), t in [0, 1]: t * P(t^2), degree-7 least-squares fit on Chebyshev nodes, float Horner
__device__ __forceinline__ float pl_fatan01(float t)
{
    const float z = t * t;
    float q = -0.003962602f;
    q = 0.021518489f + z * q;
    q = -0.055396412f + z * q;
    q = 0.096028686f + z * q;
    q = -0.13892588f + z * q;
    q = 0.19943212f + z * q;
    q = -0.33329552f + z * q;
    q = 0.99999923f + z * q;
    return t * q;
}
// atan(x), x >= 0
__device__ __forceinline__ float pl_fatan(float x)
{
    return x > 1.0f ? 1.5707963f - pl_fatan01(1.0f / x) : pl_fatan01(x);
}
// atan2(y, x) for x, y != 0 (the caller takes the exact path otherwise)
__device__ __forceinline__ float pl_fatan2(float y, float x)
{
    const float ax = fabsf(x), ay = fabsf(y);
    float r = ay > ax ? 1.5707963f - pl_fatan01(ax / ay) : pl_fatan01(ay / ax);
    if (x < 0.0f) r = 3.1415927f - r;
    return y < 0.0f ? -r : r;
}

// the polar angle's two cell indices: possible_interval's start_cell and the pruning's own cell cw
__device__ __forceinline__ void pl_theta_cells(double wx, double wy, int n, double min_theta, double max_theta,
                                               double angle_inc, int &start_cell, int &cw)
{
    auto adj = [&](double th, int &fl) {
        fl = 0;
        if (th < min_theta) {
            th += 2.0 * SDM_PI;
            fl = 1;
        }
        if (th > max_theta) {
            th -= 2.0 * SDM_PI;
            fl |= 2;
        }
        return th;
    };
    auto sc = [&](double th) { return (int)((th - min_theta) / (max_theta - min_theta) * n); };
    auto cc = [&](double th) { return angle_inc > 0.0 ? (int)((th - min_theta) / angle_inc) : 0; };
    const float fx = (float)wx, fy = (float)wy;
    // a zero or subnormal component (its float rounding is not relative to 2^-24) takes the exact path:
    // both magnitudes must be normal floats (the smaller one decides)
    if (fminf(fabsf(fx), fabsf(fy)) >= 1.17549435e-38f) {
        const double a = (double)pl_fatan2(fy, fx);
        // near +-pi the exact atan2 may sit on the other side of the cut: no bracket there
        if (fabs(a) <= SDM_PI - 4.0 * PL_ATAN_EPS) {
            int fl0, fl1;
            const double t0 = adj(a - PL_ATAN_EPS, fl0), t1 = adj(a + PL_ATAN_EPS, fl1);
            const int s0 = sc(t0), c0 = cc(t0);
            if (fl0 == fl1 && s0 == sc(t1) && c0 == cc(t1)) {
                start_cell = s0;
                cw = c0;
                return;
            }
        }
    }
    int fl;
    const double th = adj(sdm_atan2(wy, wx), fl);
    start_cell = sc(th);
    cw = cc(th);
}

// ceil(atan(u) / step) for u >= 0, the same bracket (k0 = the caller's constant term inside the ceil)
__device__ __forceinline__ int pl_atan_cells(double u, double k0, double step)
{
    const double a = (double)pl_fatan((float)u);
    if (a <= 2.0) {
        const double lo = a - PL_ATAN_EPS > 0.0 ? a - PL_ATAN_EPS : 0.0, hi = a + PL_ATAN_EPS;
        const int r0 = (int)ceil((k0 + lo) / step), r1 = (int)ceil((k0 + hi) / step);
        if (r0 == r1) return r0;
    }
    return (int)ceil((k0 + sdm_atan(u)) / step);
}

// possible_interval (CSM icp_corr_dumb.c); also returns the point's own cell for the pruning
__device__ __forceinline__ void pl_interval(const pl_params &p, double wx, double wy, int n, double min_theta,
                                            double max_theta, double angle_inc, int &from, int &to, int &cw)
{
    const double angle_res = (max_theta - min_theta) / n;
    const double norm = sqrt(wx * wx + wy * wy);
    // delta = |max_angular_correction| + |atan(max_linear_correction / norm)|, range = ceil(delta / angle_res)
    const int range = pl_atan_cells(p.max_linear_correction / norm, fabs(p.max_angular_correction_deg * (SDM_PI / 180.0)),
                                    angle_res);
    int start_cell;
    pl_theta_cells(wx, wy, n, min_theta, max_theta, angle_inc, start_cell, cw);
    const int f = start_cell - range, t = start_cell + range;
    from = f < 0 ? 0 : (f > n - 1 ? n - 1 : f);
    to = t < 0 ? 0 : (t > n - 1 ? n - 1 : t);
}

// the 14 GPC terms of one correspondence (upper triangle of M_k^T C M_k, then g = -2 M_k^T C q)
__device__ __forceinline__ void pl_terms(double px, double py, double qx, double qy, double c00, double c01,
                                         double c11, double *o)
{
    o[0] = c00;
    o[1] = c01;
    o[2] = c00 * px + c01 * py;
    o[3] = -c00 * py + c01 * px;
    o[4] = c11;
    o[5] = c01 * px + c11 * py;
    o[6] = -c01 * py + c11 * px;
    o[7] = (c00 * px * px + 2.0 * c01 * px * py) + c11 * py * py;
    o[8] = ((-c00 * px * py + c01 * px * px) - c01 * py * py) + c11 * px * py;
    o[9] = (c00 * py * py - 2.0 * c01 * px * py) + c11 * px * px;
    const double a0 = c00 * qx + c01 * qy, a1 = c01 * qx + c11 * qy;
    o[10] = -2.0 * a0;
    o[11] = -2.0 * a1;
    o[12] = -2.0 * (px * a0 + py * a1);
    o[13] = -2.0 * (-py * a0 + px * a1);
}

// constrained point-to-line solve (the role of CSM's gpc_solve); false if degenerate.  It reads the 14
// GPC sums as the 4 waves' partial sums in LDS (red[w][k], combined in pl_block_sum's order) and leaves
// its estimate in LDS x[3]: out of line (the bisection's registers stay out of the kernel's budget) with
// no array argument in private memory, so a call costs no scratch traffic.
__device__ __forceinline__ double pl_red_sum(const double (*red)[16], int k)
{
    return (red[0][k] + red[2][k]) + (red[1][k] + red[3][k]);
}
__device__ __attribute__((noinline)) bool pl_gpc_solve(const double (*red)[16], double *x)
{
    const double m00 = pl_red_sum(red, 0), m01 = pl_red_sum(red, 1), m02 = pl_red_sum(red, 2);
    const double m03 = pl_red_sum(red, 3), m11 = pl_red_sum(red, 4), m12 = pl_red_sum(red, 5);
    const double m13 = pl_red_sum(red, 6), m22 = pl_red_sum(red, 7), m23 = pl_red_sum(red, 8);
    const double m33 = pl_red_sum(red, 9);
    const double g0 = pl_red_sum(red, 10), g1 = pl_red_sum(red, 11), g2 = pl_red_sum(red, 12);
    const double g3 = pl_red_sum(red, 13);
    const double detA = m00 * m11 - m01 * m01;
    if (!(detA > 0.0)) return false;
    const double ia00 = m11 / detA, ia01 = -m01 / detA, ia11 = m00 / detA;
    const double ab00 = ia00 * m02 + ia01 * m12, ab01 = ia00 * m03 + ia01 * m13;
    const double ab10 = ia01 * m02 + ia11 * m12, ab11 = ia01 * m03 + ia11 * m13;
    const double s00 = m22 - (m02 * ab00 + m12 * ab10);
    const double s01 = m23 - (m02 * ab01 + m12 * ab11);
    const double s11 = m33 - (m03 * ab01 + m13 * ab11);
    const double agt0 = ia00 * g0 + ia01 * g1, agt1 = ia01 * g0 + ia11 * g1;
    const double h0 = -0.5 * g2 + 0.5 * (m02 * agt0 + m12 * agt1);
    const double h1 = -0.5 * g3 + 0.5 * (m03 * agt0 + m13 * agt1);
    const double hn = sqrt(h0 * h0 + h1 * h1);
    if (!(hn > 0.0)) return false;
    const double mid = 0.5 * (s00 + s11);
    const double rad = sqrt(0.25 * (s00 - s11) * (s00 - s11) + s01 * s01);
    const double lmin = mid - rad;
    double lo = -lmin, hi = -lmin + hn;
    for (int it = 0; it < 200; ++it) {
        const double l = 0.5 * (lo + hi);
        // converged: the midpoint is an endpoint, so every further step would assign lo or hi its own
        // value -- stopping here leaves the oracle's 200-step result unchanged, bit for bit
        if (l == lo || l == hi) break;
        const double a = s00 + l, d = s11 + l;
        const double det = a * d - s01 * s01;
        const double r0 = (d * h0 - s01 * h1) / det, r1 = (a * h1 - s01 * h0) / det;
        if (r0 * r0 + r1 * r1 > 1.0) lo = l;
        else hi = l;
    }
    const double l = 0.5 * (lo + hi);
    const double a = s00 + l, d = s11 + l;
    const double det = a * d - s01 * s01;
    const double r0 = (d * h0 - s01 * h1) / det, r1 = (a * h1 - s01 * h0) / det;
    const double br0 = (m02 * r0 + m03 * r1) + 0.5 * g0, br1 = (m12 * r0 + m13 * r1) + 0.5 * g1;
    x[0] = -(ia00 * br0 + ia01 * br1);
    x[1] = -(ia01 * br0 + ia11 * br1);
    x[2] = sdm_atan2(r1, r0);
    return isfinite(x[0]) && isfinite(x[1]) && isfinite(x[2]);
}

__device__ __forceinline__ unsigned pl_mix(unsigned x)
{
    x ^= x >> 16;
    x *= 0x7feb352dU;
    x ^= x >> 15;
    x *= 0x846ca68bU;
    x ^= x >> 16;
    return x;
}

__device__ __forceinline__ double pl_angle_diff(double a, double b)
{
    double d = a - b;
    while (d > SDM_PI) d -= 2.0 * SDM_PI;
    while (d <= -SDM_PI) d += 2.0 * SDM_PI;
    return d;
}

// block-wide sums (xor butterfly inside each wave, then ((w0 + w2) + (w1 + w3)) -- the oracle's
// reduce_threads = 256 order)
// a block-uniform double moved to scalar registers (the pose estimates: kept out of the VGPR budget)
__device__ __forceinline__ double pl_uniform(double v)
{
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readfirstlane((int)(unsigned)(unsigned long long)b);
    const int hi = __builtin_amdgcn_readfirstlane((int)((unsigned long long)b >> 32));
    return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}
// the wave half: each wave's sums into red[w][*] (no barrier)
template <int K>
__device__ __forceinline__ void pl_wave_sums(double *v, double (*red)[16])
{
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1)
#pragma unroll
        for (int k = 0; k < K; ++k) v[k] = v[k] + __shfl_xor(v[k], off, 64);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0)
#pragma unroll
        for (int k = 0; k < K; ++k) red[w][k] = v[k];
}
template <int K>
__device__ __forceinline__ void pl_block_sum(double *v, double (*red)[16])
{
    pl_wave_sums<K>(v, red);
    __syncthreads();
#pragma unroll
    for (int k = 0; k < K; ++k) v[k] = pl_red_sum(red, k);
    __syncthreads();
}

__device__ __forceinline__ int pl_block_sum_int(int v, int *sred)
{
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
    if ((threadIdx.x & 63) == 0) sred[threadIdx.x >> 6] = v;
    __syncthreads();
    const int r = (sred[0] + sred[1]) + (sred[2] + sred[3]);
    __syncthreads();
    return r;
}

// register budget: 4 waves per SIMD (4 pairs per CU).  The kernel wants ~170 VGPRs; capping it at 128
// spills a few cold values to scratch but doubles the resident pairs (A/B: 0.92 M -> 1.21 M pairs/s)
#ifndef PL_WAVES_PER_EU
#define PL_WAVES_PER_EU 4
#endif
// PL_RPT = rays per thread, instantiated per scan length (the host picks the smallest that covers n):
// thread t owns rays t + 256 k, k < PL_RPT, so the rays and their summation order are the same for
// every instantiation -- only the register arrays shrink.
template <int PL_RPT>
__global__ void __launch_bounds__(PL_THREADS) __attribute__((amdgpu_waves_per_eu(PL_WAVES_PER_EU)))
pl_icp_kernel(pl_params p, int n, double angle_min, double angle_inc, const double *__restrict__ theta,
              const double *__restrict__ ref_r, const double *__restrict__ sens_r,
              const double *__restrict__ first_guess, pl_result *__restrict__ out)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char pl_smem[];
    double2 *rpt = reinterpret_cast<double2 *>(pl_smem);                          // reference points [n]
    unsigned long long *best_j = reinterpret_cast<unsigned long long *>(rpt + n);   // [n]
    int16_t *rup = reinterpret_cast<int16_t *>(best_j + n);                         // next valid above [n]
    int16_t *rdn = rup + n;                                                         // next valid below [n]
    __shared__ double red[4][16];
    __shared__ int sred[4];
    __shared__ unsigned hist[2 * 512];
    __shared__ unsigned long long s_pref[2], s_key[2];
    __shared__ int s_rank[2], s_one[2];
    __shared__ unsigned s_hash[PL_MAX_IT];
    __shared__ double s_x[3];
    __shared__ int s_ok;

    const int pair = blockIdx.x;
    const int tid = threadIdx.x;
    const double *rr = ref_r + (size_t)pair * n;
    const double *sr = sens_r + (size_t)pair * n;

    // ---- LDP -> cartesian (LaserScanToLDP :285-322, ld_compute_cartesian); valid <=> reading > 0.
    // Invalid reference rays are parked at 1e300: their squared distance overflows to +inf, so the
    // `dist > max_correspondence_dist^2` test skips them exactly like ld_valid_ray does.
    for (int i = tid; i < n; i += PL_THREADS) {
        const double r = rr[i];
        const double th = theta ? theta[i] : angle_min + i * angle_inc;  // an LDP's own theta[] when given
        rpt[i] = r > 0.0 ? make_double2(r * sdm_cos(th), r * sdm_sin(th)) : make_double2(1e300, 1e300);
    }
    double spx[PL_RPT], spy[PL_RPT];
    bool sval[PL_RPT];
#pragma unroll
    for (int k = 0; k < PL_RPT; ++k) {
        const int i = tid + k * PL_THREADS;
        sval[k] = false;
        spx[k] = spy[k] = 0.0;
        if (i < n) {
            const double r = sr[i];
            const double th = theta ? theta[i] : angle_min + i * angle_inc;
            sval[k] = r > 0.0;
            if (sval[k]) {
                spx[k] = r * sdm_cos(th);
                spy[k] = r * sdm_sin(th);
            }
        }
    }
    // next valid neighbours of every reference ray: wave 0 the nearest valid ray below, wave 1 above,
    // 64 rays per step from the validity ballot and a carry across the steps
    if (tid < 128) {
        const int lane = tid & 63;
        const unsigned long long below = lane ? (~0ull >> (64 - lane)) : 0ull;  // lanes < lane
        const unsigned long long above = lane < 63 ? (~0ull << (lane + 1)) : 0ull;  // lanes > lane
        int carry = -1;
        const int nch = (n + 63) / 64;
        for (int c = 0; c < nch; ++c) {
            const int ch = tid < 64 ? c : nch - 1 - c;
            const int i = ch * 64 + lane;
            const unsigned long long m = __ballot(i < n && rr[i] > 0.0);
            if (tid < 64) {
                const unsigned long long mb = m & below;
                if (i < n) rdn[i] = (int16_t)(mb ? ch * 64 + 63 - __clzll((long long)mb) : carry);
                if (m) carry = ch * 64 + 63 - __clzll((long long)m);
            } else {
                const unsigned long long ma = m & above;
                if (i < n) rup[i] = (int16_t)(ma ? ch * 64 + __ffsll((long long)ma) - 1 : carry);
                if (m) carry = ch * 64 + __ffsll((long long)m) - 1;
            }
        }
    }
    __syncthreads();

    // ldp->min_theta / max_theta = theta[0] / theta[n-1] (LaserScanToLDP, plicp_odometry.cc:312-313)
    const double min_theta = theta ? theta[0] : angle_min, max_theta = theta ? theta[n - 1] : angle_min + (n - 1) * angle_inc;
    const double maxd2 = p.max_correspondence_dist * p.max_correspondence_dist;
    const int max_it = p.max_iterations < PL_MAX_IT ? p.max_iterations : PL_MAX_IT;
    double x_old[3], x_new[3];
    if (first_guess) {
        x_old[0] = first_guess[3 * pair];
        x_old[1] = first_guess[3 * pair + 1];
        x_old[2] = first_guess[3 * pair + 2];
    } else {
        x_old[0] = x_old[1] = x_old[2] = 0.0;
    }
    x_new[0] = x_old[0];
    x_new[1] = x_old[1];
    x_new[2] = x_old[2];
    if (tid == 0) {  // the solve's in/out estimate lives in LDS (read back after the barriers below)
        s_x[0] = x_new[0];
        s_x[1] = x_new[1];
        s_x[2] = x_new[2];
    }
    bool all_ok = true;
    int it = 0, nvalid = 0;
    double total_error = 0.0;
    int j1[PL_RPT], j2[PL_RPT];
    bool ok[PL_RPT];
    double d2[PL_RPT], e[PL_RPT];

    for (it = 0; it < max_it; ++it) {
        const double c = sdm_cos(x_old[2]), s = sdm_sin(x_old[2]);
        int ncorr = 0;
#pragma unroll
        for (int k = 0; k < PL_RPT; ++k) {
            ok[k] = false;
            j1[k] = j2[k] = -1;
            d2[k] = e[k] = 0.0;
            const int i = tid + k * PL_THREADS;
            if (i >= n || !sval[k]) continue;
            const double wx = (c * spx[k] - s * spy[k]) + x_old[0];   // ld_compute_world_coords
            const double wy = (s * spx[k] + c * spy[k]) + x_old[1];
            int from, to, cw;
            pl_interval(p, wx, wy, n, min_theta, max_theta, angle_inc, from, to, cw);
            int b1 = -1;
            double best = 0.0;
            bool searched = false;
            {
                // Prune the interval to the reference points that can pass the maxd2 test: a point at
                // polar angle theta_j is at least |w| sin|theta_w - theta_j| from w, so beyond
                // asin(1.01 maxd / |w|) (+3 cells for the interval's cell mapping) its distance exceeds
                // maxd by 1 % -- the exhaustive scan would skip it.  The candidates kept are visited in
                // the same order, so the result is the exhaustive search's, bit for bit.
                const double norm = sqrt(wx * wx + wy * wy);
                const double lim = 1.01 * p.max_correspondence_dist;
                if (norm > 2.0 * lim && angle_inc > 0.0) {
                    // cw = (int)((theta_w - min_theta) / angle_inc), theta_w adjusted as in possible_interval
                    // Tighter still: the best distance among the 9 cells around the point's own cell
                    // bounds the winner, so the same argument with lim = 1.01 sqrt(that) shrinks the
                    // window further (every point left out is > that distance, hence not the minimum).
                    // When the shrunk window lies inside those 9 cells, their first-index argmin is
                    // already the exhaustive search's answer (all ties sit inside the window).  Only
                    // when the core holds no candidate is the maxd window above computed.
                    const int cf = from > cw - PL_CORE ? from : cw - PL_CORE, ct = to < cw + PL_CORE ? to : cw + PL_CORE;
                    for (int j = cf; j <= ct; ++j) {
                        const double2 q = rpt[j];
                        const double dx = wx - q.x, dy = wy - q.y;
                        const double dist = dx * dx + dy * dy;
                        if (dist > maxd2) continue;
                        if (b1 == -1 || dist < best) {
                            b1 = j;
                            best = dist;
                        }
                    }
                    if (b1 != -1) {
                        const double sn2 = 1.01 * sqrt(best) / norm;
                        // dth2 = atan(sn2 / sqrt(1 - sn2^2)): a cell j with |j - cw| > m2 is at least m2 cells
                        // of angle away from w (w lies inside cell cw), so ceil(dth2 / inc) would do; +1
                        // covers cw's rounding, +1 margin
                        const int m2 = pl_atan_cells(sn2 / sqrt(1.0 - sn2 * sn2), 0.0, angle_inc) + 2;
                        from = from > cw - m2 ? from : cw - m2;
                        to = to < cw + m2 ? to : cw + m2;
                        if (from >= cf && to <= ct) searched = true;
                        else b1 = -1;
                    } else {
                        const double sn_ = lim / norm;
                        const int m = pl_atan_cells(sn_ / sqrt(1.0 - sn_ * sn_), 0.0, angle_inc) + 3;
                        from = from > cw - m ? from : cw - m;
                        to = to < cw + m ? to : cw + m;
                    }
                }
            }
            if (!searched)
                for (int j = from; j <= to; ++j) {
                    const double2 q = rpt[j];
                    const double dx = wx - q.x, dy = wy - q.y;
                    const double dist = dx * dx + dy * dy;
                    if (dist > maxd2) continue;
                    if (b1 == -1 || dist < best) {
                        b1 = j;
                        best = dist;
                    }
                }
            if (b1 == -1 || b1 == 0 || b1 == n - 1) continue;   // no match / extrema
            const int up = rup[b1], dn = rdn[b1];
            if (up == -1 && dn == -1) continue;
            int b2;
            if (up == -1) b2 = dn;
            else if (dn == -1) b2 = up;
            else {
                const double2 qu = rpt[up], qd = rpt[dn];
                const double du = (wx - qu.x) * (wx - qu.x) + (wy - qu.y) * (wy - qu.y);
                const double dd = (wx - qd.x) * (wx - qd.x) + (wy - qd.y) * (wy - qd.y);
                b2 = du < dd ? up : dn;
            }
            j1[k] = b1;
            j2[k] = b2;
            d2[k] = best;
            ok[k] = true;
            ++ncorr;
            const double2 q1 = rpt[b1], q2 = rpt[b2];
            e[k] = pl_dist_to_segment(q1.x, q1.y, q2.x, q2.y, wx, wy);
        }
        for (int b = tid; b < 512; b += PL_THREADS) hist[b] = 0;   // first radix pass's buffer
        if (p.outliers_remove_doubles) {
            const unsigned long long init = (unsigned long long)__double_as_longlong(1000000.0);
            for (int j = tid; j < n; j += PL_THREADS) best_j[j] = init;
        }
        ncorr = pl_block_sum_int(ncorr, sred);
        if (ncorr < 0.05 * n) {
            all_ok = false;
            break;
        }
        // ---- kill_outliers_trim: two order statistics of the k errors (radix select on the bits)
        const int kk = ncorr;
        int order = (int)floor(kk * p.outliers_maxPerc);
        order = order < 0 ? 0 : (order > kk - 1 ? kk - 1 : order);
        int order2 = (int)floor(kk * p.outliers_adaptive_order);
        order2 = order2 < 0 ? 0 : (order2 > kk - 1 ? kk - 1 : order2);
        // Two histogram buffers: a pass accumulates into one and clears the other for the next pass.
        // A statistic is settled early once its selected bin holds a single key: that key is the
        // answer, fetched from its owner (the same value the remaining passes would spell out).
        unsigned long long pref0 = 0, pref1 = 0;
        int rank0 = order, rank1 = order2;
        bool done0 = false, done1 = false;
        int cur = 0;
        for (int shift = 56; shift >= 0 && !(done0 && done1); shift -= 8, cur ^= 1) {
            unsigned *hc = hist + 512 * cur;
            for (int b = tid; b < 512; b += PL_THREADS) hist[512 * (cur ^ 1) + b] = 0;
#pragma unroll
            for (int k = 0; k < PL_RPT; ++k) {
                if (!ok[k]) continue;
                const unsigned long long key = (unsigned long long)__double_as_longlong(e[k]);
                const unsigned d = (unsigned)(key >> shift) & 255u;
                const bool m0 = shift == 56 || (key >> (shift + 8)) == (pref0 >> (shift + 8));
                const bool m1 = shift == 56 || (key >> (shift + 8)) == (pref1 >> (shift + 8));
                if (m0 && !done0) atomicAdd(&hc[d], 1u);
                if (m1 && !done1) atomicAdd(&hc[256 + d], 1u);
            }
            __syncthreads();
            if (tid < 128 && !(tid < 64 ? done0 : done1)) {
                // wave h selects in histogram h: the first bin b < 255 whose inclusive count exceeds
                // the rank (else 255), and the count before it -- a wave prefix scan over 4 bins per lane
                // (the same b and count as a sequential walk over the bins)
                const int h = tid >> 6, lane = tid & 63;
                const unsigned r = (unsigned)(h == 0 ? rank0 : rank1);
                const unsigned *hh = hc + 256 * h;
                unsigned c[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) c[j] = hh[4 * lane + j];
                const unsigned sum4 = (c[0] + c[1]) + (c[2] + c[3]);
                unsigned incl = sum4;
#pragma unroll
                for (int off = 1; off < 64; off <<= 1) {
                    const unsigned t = __shfl_up(incl, off, 64);
                    if (lane >= off) incl += t;
                }
                unsigned cum = incl - sum4;
                int jf = -1;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    if (jf >= 0) continue;
                    if (4 * lane + j < 255 && cum + c[j] > r) jf = j;
                    else cum += c[j];
                }
                const unsigned long long m = __ballot(jf >= 0);
                int b;
                unsigned cb;
                if (m) {
                    const int src = __ffsll((long long)m) - 1;
                    b = 4 * src + __shfl(jf, src, 64);
                    cb = __shfl(cum, src, 64);
                } else {
                    b = 255;
                    cb = __shfl(incl - c[3], 63, 64);  // bins 0 .. 254
                }
                if (lane == 0) {
                    s_pref[h] = (h == 0 ? pref0 : pref1) | ((unsigned long long)b << shift);
                    s_rank[h] = (int)(r - cb);
                    s_one[h] = hh[b] == 1u;
                }
            }
            __syncthreads();
            const bool one0 = !done0 && s_one[0], one1 = !done1 && s_one[1];
            if (!done0) {
                pref0 = s_pref[0];
                rank0 = s_rank[0];
            }
            if (!done1) {
                pref1 = s_pref[1];
                rank1 = s_rank[1];
            }
            if (one0 || one1) {
#pragma unroll
                for (int k = 0; k < PL_RPT; ++k) {
                    if (!ok[k]) continue;
                    const unsigned long long key = (unsigned long long)__double_as_longlong(e[k]);
                    if (one0 && (key >> shift) == (pref0 >> shift)) s_key[0] = key;
                    if (one1 && (key >> shift) == (pref1 >> shift)) s_key[1] = key;
                }
                __syncthreads();
                if (one0) {
                    pref0 = s_key[0];
                    done0 = true;
                }
                if (one1) {
                    pref1 = s_key[1];
                    done1 = true;
                }
            }
        }
        const double lim1 = __longlong_as_double((long long)pref0);
        const double lim2 = p.outliers_adaptive_mult * __longlong_as_double((long long)pref1);
        const double limit = lim1 < lim2 ? lim1 : lim2;
        // the error sum and the kept count in one reduction (the count rides as an exact small double)
        double err_sum[2] = {0.0, 0.0};
#pragma unroll
        for (int k = 0; k < PL_RPT; ++k) {
            if (!ok[k]) continue;
            if (e[k] > limit) ok[k] = false;
            else {
                err_sum[1] += 1.0;
                err_sum[0] = err_sum[0] + e[k];
            }
        }
        pl_block_sum<2>(err_sum, red);
        total_error = err_sum[0];
        nvalid = (int)err_sum[1];
        // ---- kill_outliers_double (best_j was reset at the top of the iteration)
        if (p.outliers_remove_doubles) {
#pragma unroll
            for (int k = 0; k < PL_RPT; ++k)
                if (ok[k]) atomicMin(&best_j[j1[k]], (unsigned long long)__double_as_longlong(d2[k]));
            __syncthreads();
#pragma unroll
            for (int k = 0; k < PL_RPT; ++k)
                if (ok[k] && d2[k] > 9.0 * __longlong_as_double((long long)best_j[j1[k]])) ok[k] = false;
        }
        // ---- compute_next_estimate: point-to-line GPC sums + constrained solve
        double m[14];
#pragma unroll
        for (int q = 0; q < 14; ++q) m[q] = 0.0;
        unsigned hsum = 0;
#pragma unroll
        for (int k = 0; k < PL_RPT; ++k) {
            const int i = tid + k * PL_THREADS;
            if (i < n) hsum += pl_mix((unsigned)i * 0x9E3779B9U ^ (ok[k] ? (unsigned)(j1[k] + 1000 * j2[k]) : 0xFFFFFFFFu));
            if (!ok[k]) continue;
            const double2 q1 = rpt[j1[k]], q2 = rpt[j2[k]];
            double c00, c01, c11;
            if (p.use_point_to_line_distance) {
                const double dfx = q1.x - q2.x, dfy = q1.y - q2.y;
                const double one_on_norm = 1.0 / sqrt(dfx * dfx + dfy * dfy);
                const double nx = dfy * one_on_norm, ny = -dfx * one_on_norm;
                c00 = nx * nx;
                c01 = nx * ny;
                c11 = ny * ny;
            } else {
                c00 = 1.0;
                c01 = 0.0;
                c11 = 1.0;
            }
            double t[14];
            pl_terms(spx[k], spy[k], q1.x, q1.y, c00, c01, c11, t);
#pragma unroll
            for (int q = 0; q < 14; ++q) m[q] = m[q] + t[q];
        }
        pl_wave_sums<14>(m, red);
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) hsum += __shfl_xor(hsum, off, 64);
        if ((tid & 63) == 0) sred[tid >> 6] = (int)hsum;
        __syncthreads();
        // the solve's barrier below separates this read from the next write of sred
        const unsigned hash = ((unsigned)sred[0] + (unsigned)sred[1] + (unsigned)sred[2] + (unsigned)sred[3]) & 0x7FFFFFFFu;
        // the constrained solve once per pair (wave 0) on the waves' sums in red, its estimate left in
        // s_x (= x_new on entry): on failure x_new keeps what pl_gpc_solve left there, as in the
        // all-threads version
        if (tid < 64) {
            const bool okk = pl_gpc_solve(red, s_x);
            if (tid == 0) {
                s_hash[it] = hash;
                s_ok = okk ? 1 : 0;
            }
        }
        __syncthreads();
        x_new[0] = pl_uniform(s_x[0]);
        x_new[1] = pl_uniform(s_x[1]);
        x_new[2] = pl_uniform(s_x[2]);
        if (!s_ok) {
            all_ok = false;
            break;
        }
        const double co = sdm_cos(x_old[2]), so = sdm_sin(x_old[2]);
        const double ddx = x_new[0] - x_old[0], ddy = x_new[1] - x_old[1];
        const double dl0 = co * ddx + so * ddy, dl1 = -so * ddx + co * ddy, dl2 = pl_angle_diff(x_new[2], x_old[2]);
        bool loop = false;
        for (int a = 0; a < it; ++a)
            if (s_hash[a] == hash) loop = true;
        if (loop) break;
        if (fabs(dl0) < p.epsilon_xy && fabs(dl1) < p.epsilon_xy && fabs(dl2) < p.epsilon_theta) break;
        x_old[0] = x_new[0];
        x_old[1] = x_new[1];
        x_old[2] = x_new[2];
    }
    if (tid == 0) {
        pl_result r;
        r.x[0] = x_new[0];
        r.x[1] = x_new[1];
        r.x[2] = x_new[2];
        r.error = total_error;
        r.valid = all_ok ? 1 : 0;
        r.iterations = it + (it < max_it ? 1 : 0);
        r.nvalid = nvalid;
        r.pad_ = 0;
        out[pair] = r;
    }
}

}  // namespace s2d
