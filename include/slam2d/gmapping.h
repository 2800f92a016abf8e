/* include/slam2d/gmapping.h -- C-ABI of the MI355X GMapping particle-map path (config 4).
 *
 * Reference: the lesson4 `make_gmapping_map` node builds, for every scan, a FRESH
 * ScanMatcherMap (lesson4/src/gmapping/gmapping.cc:128-135) with GMapping::ComputeMap
 * (gmapping.cc:171-242): per beam, GridLineTraversal::gridLine from the laser cell to the end cell,
 * visits++ on every cell but the last, and for beams shorter than maxUrange n++, visits++ and
 * acc += hit point on the end cell (PointAccumulator, lesson4/include/lesson4/gmapping/grid/map.h:17-48).
 * ComputeMap is private and has no seam: these entry points replace it and the
 * PublishMap conversion (gmapping.cc:141-159).
 *
 * The build evaluates the scan for P candidate poses ("particles"; the reference uses the laser
 * frame itself, lp = (0,0,0), gmapping.cc:176).  Particles shard across GPUs (one context per
 * rank holding its particles); gm_normalize_weights_device performs the one RCCL all-reduce of the
 * particle weights on a communicator the host passes in.
 *
 * Conventions as in hector.h: plain C types, int status (GM_OK / negative), gm_last_error().
 * Poses are double[4] per particle: x, y, cos(theta), sin(theta) (the caller evaluates the trig,
 * as the reference caches cos/sin of the beam angles, gmapping.cc:111-124).
 */
#ifndef SLAM2D_GMAPPING_H
#define SLAM2D_GMAPPING_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GM_OK 0
#define GM_EINVAL (-1)
#define GM_EHIP (-2)
#define GM_ENOMEM (-3)
#define GM_ENODEV (-4)

typedef struct gm_ctx gm_ctx;

const char *gm_version(void);
const char *gm_last_error(void);

/* ScanMatcherMap(center, xmin, ymin, xmax, ymax, delta) (gmapping.cc:128-135, G/grid/map.h:133-143)
 * for num_particles particles; maxRange / maxUrange of ComputeMap (gmapping.cc:183-187).
 * Limits: map sides <= 16384 cells, max_range / delta < 16384, 1 <= max_beams <= 8192. */
int gm_create(gm_ctx **out, int num_particles, int max_beams, double xmin, double ymin, double xmax, double ymax,
              double delta, double max_range, double max_urange);
int gm_destroy(gm_ctx *ctx);
/* Forget every particle's map (the next compute starts from empty maps; scores read 0). */
int gm_reset(gm_ctx *ctx);
/* GMapping::CreateCache (gmapping.cc:111-124): cos / sin of each beam angle. */
int gm_set_beams(gm_ctx *ctx, const double *a_cos, const double *a_sin, int n);
/* PublishMap occupancy threshold occ_thresh (gmapping.cc:150, default 0.25). */
int gm_set_occ_thresh(gm_ctx *ctx, double occ_thresh);
int gm_get_map_size(gm_ctx *ctx, int *size_x, int *size_y);

/* ComputeMap of one scan for particles [0, P): poses double[4*P] (host), ranges float[n] (host,
 * n <= max_beams, the LaserScan ranges), synchronous.  Before overwriting, every particle scores the
 * scan against its previous map (build-defined weight, see gm_get_scores). */
int gm_compute_maps(gm_ctx *ctx, const double *poses, const float *ranges, int n);
/* Device-pointer form for particles [particle_begin, particle_begin + count): d_poses double[4*count],
 * d_ranges float[n], d_scores_out int32[count] or NULL; stream-ordered on hip_stream (NULL = own). */
int gm_compute_maps_device(gm_ctx *ctx, int particle_begin, int count, const double *d_poses, const float *d_ranges,
                           int n, int32_t *d_scores_out, void *hip_stream);

/* The particle-weight exchange of a particle set sharded over ranks (north_star "RCCL
 * allreduce of particle weights"): from this rank's integer scores d_scores int32[count] (the
 * gm_compute_maps_device output) form [Σ(score+1), Σ(score+1)^2] in double on the device, all-reduce
 * them (sum) over the ranks of nccl_comm (an ncclComm_t as void*, RCCL; NULL = single rank, no
 * exchange) on hip_stream, and write the normalised weights of this rank's particles
 * w_p = (score_p + 1) / Σ_all (score + 1) to d_weights_out (double[count], may be NULL).  d_sums_out
 * (device double[2]) receives the reduced sums; the effective sample size is sums[0]^2 / sums[1].
 * All terms are integers below 2^53, so the result does not depend on the sharding. */
int gm_normalize_weights_device(gm_ctx *ctx, void *nccl_comm, const int32_t *d_scores, int count,
                                double *d_weights_out, double *d_sums_out, void *hip_stream);

/* Dense row-major read-out of one particle's map (index y * size_x + x): n (hits), visits, acc
 * (2 floats per cell).  Any pointer may be NULL.  Synchronises. */
int gm_get_particle_map(gm_ctx *ctx, int particle, int32_t *n_out, int32_t *visits_out, float *acc_out);
/* GMapping::PublishMap for one particle: -1 unvisited, 100 if n/visits > occ_thresh, else 0. */
int gm_publish(gm_ctx *ctx, int particle, int8_t *occ_out);
/* Per particle of the last compute: score = hit beams whose end cell was occupied
 * (n/visits > occ_thresh) in the particle's previous map (build-defined weight; the reference has
 * no particles); hits = beams with d < maxUrange; free_updates = Σ(num_points - 1) in the map.
 * Any pointer may be NULL.  Synchronises. */
int gm_get_scores(gm_ctx *ctx, int32_t *scores_out, int32_t *hits_out, int64_t *free_updates_out);

int gm_set_timing(gm_ctx *ctx, int enable);
/* Accumulated gm_compute_kernel time (ms) and launches since the last reset. */
int gm_get_kernel_times(gm_ctx *ctx, double *ms_out, int64_t *launches_out, int reset);

#ifdef __cplusplus
}
#endif

#endif
