// plicp_capi.hip -- host runtime + extern "C" boundary (include/slam2d/plicp.h) of the PL-ICP path.
// Every compute step is pl_icp_kernel (plicp_kernels.hip); without a usable HIP device pl_create fails
// with PL_ENODEV.
#include <hip/hip_runtime.h>

#include <math.h>

#include <string>
#include <vector>

#include "plicp_kernels.hip"

using namespace s2d;

namespace {
thread_local std::string pl_err;

int pfail(int code, const char *what, hipError_t e = hipSuccess)
{
    pl_err = what;
    if (e != hipSuccess) {
        pl_err += ": ";
        pl_err += hipGetErrorString(e);
    }
    return code;
}

#define PCHK(expr)                                             \
    do {                                                       \
        hipError_t _e = (expr);                                \
        if (_e != hipSuccess) return pfail(PL_EHIP, #expr, _e); \
    } while (0)

size_t pl_shmem(int n) { return (size_t)n * (sizeof(double2) + sizeof(unsigned long long) + 2 * sizeof(int16_t)); }
}  // namespace

struct pl_ctx {
    int max_pairs = 0, max_rays = 0;
    pl_params params{};
    double *d_ref = nullptr, *d_sens = nullptr, *d_guess = nullptr, *d_theta = nullptr;
    pl_result *d_res = nullptr;
    hipStream_t stream = nullptr;
    bool timing = false;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> ev_used, ev_free;
    double acc_ms = 0;
    int64_t acc_n = 0;
};

extern "C" {

const char *pl_version(void) { return "slam2d-mi355x plicp 0.1 (gfx950)"; }
const char *pl_last_error(void) { return pl_err.c_str(); }

void pl_default_params(pl_params *p)
{
    if (!p) return;
    // ScanMatchPLICP::InitParams (lesson3/src/plicp_odometry.cc:74-186)
    p->max_angular_correction_deg = 45.0;
    p->max_linear_correction = 1.0;
    p->max_iterations = 10;
    p->epsilon_xy = 0.000001;
    p->epsilon_theta = 0.000001;
    p->max_correspondence_dist = 1.0;
    p->use_point_to_line_distance = 1;
    p->outliers_maxPerc = 0.90;
    p->outliers_adaptive_order = 0.7;
    p->outliers_adaptive_mult = 2.0;
    p->outliers_remove_doubles = 1;
    p->pad_ = 0;
}

int pl_create(pl_ctx **out, int max_pairs, int max_rays, const pl_params *params)
{
    if (!out) return pfail(PL_EINVAL, "out is NULL");
    *out = nullptr;
    if (max_pairs < 1 || max_rays < 2 || max_rays > PL_MAX_RAYS) return pfail(PL_EINVAL, "need 1 <= pairs, 2 <= rays <= 2048");
    if (params && (params->max_iterations < 1 || params->max_iterations > PL_MAX_IT))
        return pfail(PL_EINVAL, "max_iterations must be in [1, 64]");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1) return pfail(PL_ENODEV, "no HIP device");
    pl_ctx *c = new pl_ctx;
    c->max_pairs = max_pairs;
    c->max_rays = max_rays;
    if (params) c->params = *params;
    else pl_default_params(&c->params);
    hipError_t e;
    if ((e = hipStreamCreateWithFlags(&c->stream, hipStreamDefault)) != hipSuccess) {
        delete c;
        return pfail(PL_EHIP, "hipStreamCreate", e);
    }
    if ((e = hipMalloc(&c->d_ref, sizeof(double) * max_rays)) != hipSuccess ||
        (e = hipMalloc(&c->d_sens, sizeof(double) * max_rays)) != hipSuccess ||
        (e = hipMalloc(&c->d_guess, sizeof(double) * 3)) != hipSuccess ||
        (e = hipMalloc(&c->d_theta, sizeof(double) * max_rays)) != hipSuccess ||
        (e = hipMalloc(&c->d_res, sizeof(pl_result))) != hipSuccess) {
        pl_destroy(c);
        return pfail(PL_ENOMEM, "hipMalloc", e);
    }
    *out = c;
    return PL_OK;
}

int pl_destroy(pl_ctx *c)
{
    if (!c) return PL_OK;
    if (c->stream) hipStreamSynchronize(c->stream);
    hipFree(c->d_ref);
    hipFree(c->d_sens);
    hipFree(c->d_guess);
    hipFree(c->d_theta);
    hipFree(c->d_res);
    for (auto &p : c->ev_used) { hipEventDestroy(p.first); hipEventDestroy(p.second); }
    for (auto &p : c->ev_free) { hipEventDestroy(p.first); hipEventDestroy(p.second); }
    if (c->stream) hipStreamDestroy(c->stream);
    delete c;
    return PL_OK;
}

static int pl_launch(pl_ctx *c, int count, int n, double angle_min, double angle_inc, const double *d_ref,
                     const double *d_sens, const double *d_guess, pl_result *d_res, hipStream_t s,
                     const double *d_theta = nullptr)
{
    if (count < 0 || count > c->max_pairs) return pfail(PL_EINVAL, "count exceeds max_pairs");
    if (n < 2 || n > c->max_rays) return pfail(PL_EINVAL, "n out of range");
    if (!(angle_inc > 0.0)) return pfail(PL_EINVAL, "angle_increment must be > 0");
    if (count == 0) return PL_OK;
    std::pair<hipEvent_t, hipEvent_t> ev{};
    if (c->timing) {
        if (!c->ev_free.empty()) {
            ev = c->ev_free.back();
            c->ev_free.pop_back();
        } else {
            PCHK(hipEventCreate(&ev.first));
            PCHK(hipEventCreate(&ev.second));
        }
        PCHK(hipEventRecord(ev.first, s));
    }
    {
        const int rpt = (n + PL_THREADS - 1) / PL_THREADS;
        auto kern = rpt <= 2 ? pl_icp_kernel<2> : rpt <= 4 ? pl_icp_kernel<4> : rpt <= 5 ? pl_icp_kernel<5>
                  : rpt <= 6 ? pl_icp_kernel<6> : pl_icp_kernel<PL_RPT_MAX>;
        hipLaunchKernelGGL(kern, dim3(count), dim3(PL_THREADS), pl_shmem(n), s, c->params, n, angle_min, angle_inc,
                           d_theta, d_ref, d_sens, d_guess, d_res);
    }
    PCHK(hipGetLastError());
    if (c->timing) {
        PCHK(hipEventRecord(ev.second, s));
        c->ev_used.push_back(ev);
    }
    return PL_OK;
}

int pl_icp(pl_ctx *c, int n, double angle_min, double angle_inc, const double *ref, const double *sens,
           const double first_guess[3], pl_result *result)
{
    if (!c || !ref || !sens || !result) return pfail(PL_EINVAL, "NULL argument");
    if (n < 2 || n > c->max_rays) return pfail(PL_EINVAL, "n out of range");
    const double zero[3] = {0.0, 0.0, 0.0};
    PCHK(hipMemcpyAsync(c->d_ref, ref, sizeof(double) * n, hipMemcpyHostToDevice, c->stream));
    PCHK(hipMemcpyAsync(c->d_sens, sens, sizeof(double) * n, hipMemcpyHostToDevice, c->stream));
    PCHK(hipMemcpyAsync(c->d_guess, first_guess ? first_guess : zero, sizeof(double) * 3, hipMemcpyHostToDevice, c->stream));
    int rc = pl_launch(c, 1, n, angle_min, angle_inc, c->d_ref, c->d_sens, c->d_guess, c->d_res, c->stream);
    if (rc != PL_OK) return rc;
    PCHK(hipMemcpyAsync(result, c->d_res, sizeof(pl_result), hipMemcpyDeviceToHost, c->stream));
    PCHK(hipStreamSynchronize(c->stream));
    return PL_OK;
}

int pl_set_params(pl_ctx *c, const pl_params *params)
{
    if (!c || !params) return pfail(PL_EINVAL, "NULL argument");
    if (params->max_iterations < 1 || params->max_iterations > PL_MAX_IT)
        return pfail(PL_EINVAL, "max_iterations must be in [1, 64]");
    c->params = *params;
    return PL_OK;
}

int pl_icp_ldp(pl_ctx *c, int n, const double *theta, const double *ref_readings, const int *ref_valid,
               const double *sens_readings, const int *sens_valid, const double first_guess[3], pl_result *result)
{
    if (!c || !theta || !ref_readings || !sens_readings || !result) return pfail(PL_EINVAL, "NULL argument");
    if (n < 2 || n > c->max_rays) return pfail(PL_EINVAL, "n out of range");
    // the correspondence search maps polar angles to rays with the mean increment; an LDP of a
    // LaserScan (angle_min + i * angle_increment, plicp_odometry.cc:306) is uniform to rounding
    const double inc = (theta[n - 1] - theta[0]) / (double)(n - 1);
    if (!(inc > 0.0)) return pfail(PL_EINVAL, "theta must increase");
    for (int i = 0; i < n; ++i)
        if (fabs(theta[i] - (theta[0] + i * inc)) > 1e-3 * inc)
            return pfail(PL_EINVAL, "theta[] is not a uniform LaserScan grid");
    // readings of invalid rays -> -1 (LaserScanToLDP, :297-301): valid[] decides, as ld_valid_ray does
    std::vector<double> rr(ref_readings, ref_readings + n), sr(sens_readings, sens_readings + n);
    for (int i = 0; i < n; ++i) {
        if (ref_valid && !ref_valid[i]) rr[i] = -1.0;
        if (sens_valid && !sens_valid[i]) sr[i] = -1.0;
        if (!(rr[i] > 0.0)) rr[i] = -1.0;
        if (!(sr[i] > 0.0)) sr[i] = -1.0;
    }
    const double zero[3] = {0.0, 0.0, 0.0};
    PCHK(hipMemcpyAsync(c->d_ref, rr.data(), sizeof(double) * n, hipMemcpyHostToDevice, c->stream));
    PCHK(hipMemcpyAsync(c->d_sens, sr.data(), sizeof(double) * n, hipMemcpyHostToDevice, c->stream));
    PCHK(hipMemcpyAsync(c->d_theta, theta, sizeof(double) * n, hipMemcpyHostToDevice, c->stream));
    PCHK(hipMemcpyAsync(c->d_guess, first_guess ? first_guess : zero, sizeof(double) * 3, hipMemcpyHostToDevice, c->stream));
    int rc = pl_launch(c, 1, n, theta[0], inc, c->d_ref, c->d_sens, c->d_guess, c->d_res, c->stream, c->d_theta);
    if (rc != PL_OK) return rc;
    PCHK(hipMemcpyAsync(result, c->d_res, sizeof(pl_result), hipMemcpyDeviceToHost, c->stream));
    PCHK(hipStreamSynchronize(c->stream));
    return PL_OK;
}

int pl_icp_batch_device(pl_ctx *c, int count, int n, double angle_min, double angle_inc, const double *d_ref,
                        const double *d_sens, const double *d_guess, pl_result *d_res, void *hip_stream)
{
    if (!c || !d_ref || !d_sens || !d_res) return pfail(PL_EINVAL, "NULL argument");
    return pl_launch(c, count, n, angle_min, angle_inc, d_ref, d_sens, d_guess, d_res,
                     hip_stream ? (hipStream_t)hip_stream : c->stream);
}

int pl_set_timing(pl_ctx *c, int enable)
{
    if (!c) return pfail(PL_EINVAL, "ctx is NULL");
    c->timing = enable != 0;
    return PL_OK;
}

int pl_get_kernel_times(pl_ctx *c, double *ms_out, int64_t *launches_out, int reset)
{
    if (!c) return pfail(PL_EINVAL, "ctx is NULL");
    PCHK(hipDeviceSynchronize());
    for (auto &p : c->ev_used) {
        float ms = 0;
        PCHK(hipEventElapsedTime(&ms, p.first, p.second));
        c->acc_ms += ms;
        c->acc_n += 1;
        c->ev_free.push_back(p);
    }
    c->ev_used.clear();
    if (ms_out) *ms_out = c->acc_ms;
    if (launches_out) *launches_out = c->acc_n;
    if (reset) {
        c->acc_ms = 0;
        c->acc_n = 0;
    }
    return PL_OK;
}

}  // extern "C"
