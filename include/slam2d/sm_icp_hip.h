/* include/slam2d/sm_icp_hip.h -- the lesson3 PL-ICP drop-in: `slam2d_sm_icp(&input_, &output_)` for CSM's
 * `sm_icp(&input_, &output_)` (lesson3/src/plicp_odometry.cc:391).
 *
 * Include it AFTER the node's CSM header (`#include <csm/csm_all.h>`, as plicp_odometry.h does): it reads
 * CSM's own `struct sm_params` / `struct sm_result` / `LDP` by field name, so it compiles against the CSM
 * the maintainer has, and it needs nothing from this repository but include/slam2d/plicp.h and
 * lib/libslam2d.so.  The node's change is one call (or `#define sm_icp slam2d_sm_icp` after this header):
 *
 *     -    sm_icp(&input_, &output_);
 *     +    slam2d_sm_icp(&input_, &output_);
 *
 * Every sm_params field the node sets (plicp_odometry.cc:74-186) is read on every call (the node may
 * change them through ROS params); first_guess, laser_ref and laser_sens come from the call site
 * (:343-364).  The fields CSM documents as switches of features the node leaves off -- do_alpha_test,
 * do_visibility_test, restart, use_ml_weights, use_sigma_weights, do_compute_covariance -- are not
 * implemented on the device: a call with any of them set returns output->valid = 0 and says so on
 * stderr once (no silent CPU fallback).  The result fields the node reads (valid, x) are written, plus
 * iterations, nvalid and error.  CSM itself is absent from this repository's image: PL-ICP parity is
 * against the C restatement oracle/plicp_oracle.c (DESIGN.md "PL-ICP").
 */
#ifndef SLAM2D_SM_ICP_HIP_H
#define SLAM2D_SM_ICP_HIP_H

#include <cstdio>

#include <slam2d/plicp.h>

namespace slam2d {
namespace detail {
// one PL-ICP context per calling thread (the node calls from its spin thread), released at thread exit
struct SmIcpContext {
    pl_ctx *ctx = nullptr;
    bool warned = false;
    ~SmIcpContext()
    {
        if (ctx) pl_destroy(ctx);
    }
};
inline SmIcpContext &sm_icp_context()
{
    thread_local SmIcpContext c;
    return c;
}
}  // namespace detail
}  // namespace slam2d

template <class SmParams, class SmResult>
inline void slam2d_sm_icp(SmParams *input, SmResult *output)
{
    slam2d::detail::SmIcpContext &sc = slam2d::detail::sm_icp_context();
    output->valid = 0;
    auto fail = [&](const char *why) {
        if (!sc.warned) {
            std::fprintf(stderr, "slam2d_sm_icp: %s\n", why);
            sc.warned = true;
        }
    };
    if (input->do_alpha_test || input->do_visibility_test || input->restart || input->use_ml_weights ||
        input->use_sigma_weights || input->do_compute_covariance) {
        fail("do_alpha_test / do_visibility_test / restart / use_ml_weights / use_sigma_weights / "
             "do_compute_covariance are not supported on the device");
        return;
    }
    const auto *ref = input->laser_ref;
    const auto *sens = input->laser_sens;
    const int n = ref->nrays;
    if (sens->nrays != n) {
        fail("laser_ref and laser_sens differ in nrays");
        return;
    }
    if (n > PL_MAX_SCAN_RAYS) {
        // not a once-only warning: every such scan fails (output->valid = 0), and says so
        std::fprintf(stderr, "slam2d_sm_icp: %d rays; the device PL-ICP takes at most %d (PL_MAX_SCAN_RAYS)\n", n,
                     PL_MAX_SCAN_RAYS);
        return;
    }
    for (int i = 0; i < n; ++i)
        if (ref->theta[i] != sens->theta[i]) {
            fail("laser_ref and laser_sens differ in theta");
            return;
        }
    pl_params p;
    pl_default_params(&p);
    p.max_angular_correction_deg = input->max_angular_correction_deg;
    p.max_linear_correction = input->max_linear_correction;
    p.epsilon_xy = input->epsilon_xy;
    p.epsilon_theta = input->epsilon_theta;
    p.max_correspondence_dist = input->max_correspondence_dist;
    p.outliers_maxPerc = input->outliers_maxPerc;
    p.outliers_adaptive_order = input->outliers_adaptive_order;
    p.outliers_adaptive_mult = input->outliers_adaptive_mult;
    p.max_iterations = input->max_iterations;
    p.use_point_to_line_distance = input->use_point_to_line_distance;
    p.outliers_remove_doubles = input->outliers_remove_doubles;
    if (!sc.ctx && pl_create(&sc.ctx, 1, PL_MAX_SCAN_RAYS, &p) != PL_OK) {  // the largest context: any n fits
        fail(pl_last_error());
        return;
    }
    if (pl_set_params(sc.ctx, &p) != PL_OK) {
        fail(pl_last_error());
        return;
    }
    pl_result r;
    if (pl_icp_ldp(sc.ctx, n, ref->theta, ref->readings, ref->valid, sens->readings, sens->valid, input->first_guess,
                   &r) != PL_OK) {
        fail(pl_last_error());
        return;
    }
    output->valid = r.valid;
    output->iterations = r.iterations;
    output->nvalid = r.nvalid;
    output->error = r.error;
    for (int k = 0; k < 3; ++k) output->x[k] = r.x[k];
}

#endif
