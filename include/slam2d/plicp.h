/* include/slam2d/plicp.h -- C-ABI of the MI355X PL-ICP scan-matching path (lesson3 front-end).
 *
 * Reference: lesson3's ScanMatchPLICP (lesson3/src/plicp_odometry.cc) converts each LaserScan to a
 * CSM LDP (LaserScanToLDP, :285-322: readings = -1 for rays outside (range_min, range_max)) and calls
 * CSM's `void sm_icp(struct sm_params*, struct sm_result*)` (:391) with the reference scan, the new
 * scan and a first guess (:356-364).  CSM (apt ros-kinetic-csm) is not vendored and absent from this
 * image: these entry points implement its point-to-line ICP loop for the parameters the node sets
 * (:58-186) -- PARITY UNPINNED against CSM itself (DESIGN.md "PL-ICP").
 *
 * Conventions as in hector.h: plain C types, int status (PL_OK / negative), pl_last_error().
 * Scans: n readings (double, metres; <= 0 = invalid), angles angle_min + i * angle_increment.
 */
#ifndef SLAM2D_PLICP_H
#define SLAM2D_PLICP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PL_OK 0
#define PL_EINVAL (-1)
#define PL_EHIP (-2)
#define PL_ENOMEM (-3)
#define PL_ENODEV (-4)

/* The sm_params fields that shape this path (plicp_odometry.cc:74-186 defaults via pl_default_params);
 * do_alpha_test, do_visibility_test, restart, use_ml_weights, use_sigma_weights and
 * do_compute_covariance are 0 in the node and not supported. */
typedef struct pl_params {
    double max_angular_correction_deg;  /* 45 */
    double max_linear_correction;       /* 1.0 */
    double epsilon_xy;                  /* 1e-6 */
    double epsilon_theta;               /* 1e-6 */
    double max_correspondence_dist;     /* 1.0 */
    double outliers_maxPerc;            /* 0.90 */
    double outliers_adaptive_order;     /* 0.7 */
    double outliers_adaptive_mult;      /* 2.0 */
    int max_iterations;                 /* 10 (<= 64) */
    int use_point_to_line_distance;     /* 1 */
    int outliers_remove_doubles;        /* 1 */
    int pad_;
} pl_params;

/* sm_result fields: x (laser-frame displacement of the new scan), valid, iterations, nvalid, error */
typedef struct pl_result {
    double x[3];
    double error;
    int valid;
    int iterations;
    int nvalid;
    int pad_;
} pl_result;

typedef struct pl_ctx pl_ctx;

const char *pl_version(void);
const char *pl_last_error(void);
/* ScanMatchPLICP::InitParams values (plicp_odometry.cc:74-186) */
void pl_default_params(pl_params *params);

/* The device kernel's ray limit: 256 threads x 8 rays each (csrc/plicp_kernels.hip PL_MAX_RAYS). */
#define PL_MAX_SCAN_RAYS 2048
/* A context for up to max_pairs scan pairs of up to max_rays rays (max_rays <= PL_MAX_SCAN_RAYS). */
int pl_create(pl_ctx **out, int max_pairs, int max_rays, const pl_params *params);
int pl_destroy(pl_ctx *ctx);

/* sm_icp for one scan pair (host arrays, synchronous): ref / sens readings double[n]. */
int pl_icp(pl_ctx *ctx, int n, double angle_min, double angle_increment, const double *ref_readings,
           const double *sens_readings, const double first_guess[3], pl_result *result);
/* sm_icp for `count` independent pairs (device arrays, stream-ordered): d_ref / d_sens double[count][n],
 * d_first_guess double[count][3] (NULL = zeros), d_results pl_result[count]. */
int pl_icp_batch_device(pl_ctx *ctx, int count, int n, double angle_min, double angle_increment,
                        const double *d_ref_readings, const double *d_sens_readings, const double *d_first_guess,
                        pl_result *d_results, void *hip_stream);

/* Replace the context's parameters (sm_params fields, e.g. from the node's ROS params). */
int pl_set_params(pl_ctx *ctx, const pl_params *params);
/* sm_icp on two LDPs as lesson3 builds them (LaserScanToLDP, plicp_odometry.cc:285-322): shared theta[n]
 * (uniform: angle_min + i * angle_increment, checked to 1e-3 of the increment), readings[n] and
 * valid[n] (NULL = reading > 0) per scan; host arrays, synchronous.  The call include/slam2d/sm_icp_hip.h
 * makes for its `slam2d_sm_icp(&input_, &output_)` drop-in of `sm_icp` (plicp_odometry.cc:391). */
int pl_icp_ldp(pl_ctx *ctx, int n, const double *theta, const double *ref_readings, const int *ref_valid,
               const double *sens_readings, const int *sens_valid, const double first_guess[3], pl_result *result);

int pl_set_timing(pl_ctx *ctx, int enable);
int pl_get_kernel_times(pl_ctx *ctx, double *ms_out, int64_t *launches_out, int reset);

#ifdef __cplusplus
}
#endif

#endif
