/* include/slam2d/karto.h -- C-ABI of the MI355X Karto correlative scan matcher (lesson6, config 5).
 *
 * Reference: open_karto's ScanMatcher (lesson6/lib/open_karto/src/Mapper.cpp), used by
 * Mapper::Process for the sequential match against the running scans (Mapper.cpp:2040-2043) and by
 * MapperGraph::TryCloseLoop for loop-closure candidates (Mapper.cpp:991-992, :1015-1016).  Each entry
 * point replaces one reference interface:
 *
 *   kt_create             ScanMatcher::Create(mapper, searchSize, resolution, smearDeviation,
 *                         rangeThreshold)                                        Mapper.cpp:126-171
 *   kt_match_scan         ScanMatcher::MatchScan(pScan, rBaseScans, rMean, rCovariance,
 *                         doPenalize, doRefineMatch)                             Mapper.cpp:184-300
 *   kt_match_batch_device many independent MatchScan calls at once (a loop-closure candidate batch, or
 *                         the sequential matches of many robots / bag replays)
 *   kt_set_scans[_device] LocalizedRangeScan construction + Update() (point readings,
 *                         Karto.h:5362-5404) into the context's scan pool
 *
 * open_karto needs boost (Karto.h:37), absent from this image, so it is not built here: the CPU
 * checker oracle/karto_oracle.c restates it and parity is UNPINNED against the library itself
 * (DESIGN.md "Karto").  The GPU results (mean, covariance, response) equal the restatement's bit for bit.
 *
 * Conventions as in hector.h: plain C types, int status (KT_OK / negative), kt_last_error().
 * A scan is n_readings doubles (metres; NaN / inf allowed, as in the reference) plus its sensor pose
 * (x, y, heading) in world coordinates; the laser offset is identity.
 */
#ifndef SLAM2D_KARTO_H
#define SLAM2D_KARTO_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KT_OK 0
#define KT_EINVAL (-1)
#define KT_EHIP (-2)
#define KT_ENOMEM (-3)
#define KT_ENODEV (-4)
#define KT_ERANGE (-5) /* a grid index the reference would have thrown on (kt_result.status) */

/* The LaserRangeFinder fields LocalizedRangeScan::Update reads (Karto.h:5362-5404). */
typedef struct kt_laser {
    double minimum_angle;      /* rad */
    double angular_resolution; /* rad */
    double minimum_range;      /* m */
    double range_threshold;    /* m: readings outside [minimum_range, range_threshold] are dropped */
    int n_readings;            /* <= 4096 */
    int pad_;
} kt_laser;

/* One ScanMatcher's parameters.  Penalty variances are the values Mapper stores, i.e. the squares of
 * the ROS parameters (Mapper::setParamDistanceVariancePenalty, Mapper.cpp:1919-1927). */
typedef struct kt_params {
    double search_size;                /* CorrelationSearchSpaceDimension 0.3 | LoopSearchSpaceDimension 8.0 */
    double resolution;                 /* ...Resolution 0.01 | 0.05 */
    double smear_deviation;            /* ...SmearDeviation 0.03 | 0.03 */
    double distance_variance_penalty;  /* 0.3^2 */
    double angle_variance_penalty;     /* (20 deg)^2 in rad^2 */
    double fine_search_angle_offset;   /* 0.2 deg */
    double coarse_search_angle_offset; /* 20 deg */
    double coarse_angle_resolution;    /* 2 deg */
    double minimum_angle_penalty;      /* 0.9 */
    double minimum_distance_penalty;   /* 0.5 */
    int use_response_expansion;        /* 0 (Mapper default) */
    int pad_;
} kt_params;

/* MatchScan's outputs: rMean, rCovariance (row-major 3x3), the returned response. */
typedef struct kt_result {
    double mean[3];
    double covariance[9];
    double response;
    int status; /* KT_OK, or KT_ERANGE where the reference throws */
    int pad_;
} kt_result;

typedef struct kt_ctx kt_ctx;

const char *kt_version(void);
const char *kt_last_error(void);
/* Mapper::InitializeParameters defaults (Mapper.cpp:1569-1660): sequential / loop-closure matcher. */
void kt_default_params(kt_params *params);
void kt_default_loop_params(kt_params *params);

/* ScanMatcher::Create for up to max_matches concurrent MatchScan calls, a pool of max_scans scans and
 * at most max_base_per_match base scans per call.  Fails with KT_EINVAL for the parameters the
 * reference rejects (Create returns NULL, CalculateKernel throws) and for a smear kernel with a value
 * of 100 off its centre (smear_deviation close to 10 * resolution; not supported). */
int kt_create(kt_ctx **out, const kt_laser *laser, const kt_params *params, int max_matches, int max_scans,
              int max_base_per_match);
int kt_destroy(kt_ctx *ctx);
/* out[10] = grid_size, border, width, width_step, data_size, search_side, probs_width_step,
 *           kernel_half, kernel_size, max_poses */
int kt_get_grid_info(kt_ctx *ctx, int *out);

/* Store scans into pool slots [first, first + count) and compute their point readings.
 * ranges double[count][n_readings], poses double[count][3]. */
int kt_set_scans(kt_ctx *ctx, int first, int count, const double *ranges, const double *poses);
int kt_set_scans_device(kt_ctx *ctx, int first, int count, const double *d_ranges, const double *d_poses,
                        void *hip_stream);

/* One MatchScan (host arrays, synchronous; uses pool slots 0 .. n_base). */
int kt_match_scan(kt_ctx *ctx, const double *query_ranges, const double query_pose[3], int n_base,
                  const double *base_ranges, const double *base_poses, int do_penalize, int do_refine,
                  kt_result *result);

/* `count` independent MatchScan calls on pooled scans (device arrays, stream-ordered):
 * match i matches pool scan d_query[i] against pool scans d_base_index[d_base_begin[i] ..
 * d_base_begin[i + 1]); d_results kt_result[count]. */
int kt_match_batch_device(kt_ctx *ctx, int count, const int *d_query, const int *d_base_begin,
                          const int *d_base_index, int do_penalize, int do_refine, kt_result *d_results,
                          void *hip_stream);

/* ONE batch of MatchScan calls with the coarse window split over nshards GPUs: one
 * process per GPU, every rank passing the same pooled scans and arguments.  Phase 1 builds the
 * correlation grids and evaluates the coarse responses of the angles a = shard (mod nshards)
 * (CorrelateScan's pose loop, Mapper.cpp:371-425), then exports per match
 *   [best, ERANGE flag, per-position max over angles, every pose's response]
 * as int64 words (d_exchange: int64[count][kt_window_exchange_words(ctx)], caller-owned device memory;
 * all values are non-negative doubles, non-owned responses +0.0).  The caller all-reduces d_exchange
 * with MAX over the ranks (RCCL over xGMI), then phase 2 imports it and finishes the reference
 * sequence: best, tie average in pose order, positional covariance (Mapper.cpp:427-523), fine match.
 * Every rank ends with the identical result, bit-equal to kt_match_batch_device.  Requires
 * count <= the context's slots and no response expansion (KT_EINVAL otherwise). */
size_t kt_window_exchange_words(kt_ctx *ctx);
int kt_match_sharded_begin_device(kt_ctx *ctx, int count, const int *d_query, const int *d_base_begin,
                                  const int *d_base_index, int do_penalize, int shard, int nshards,
                                  int64_t *d_exchange, void *hip_stream);
int kt_match_sharded_end_device(kt_ctx *ctx, int count, const int *d_base_begin, const int *d_base_index,
                                int do_penalize, int do_refine, const int64_t *d_exchange, kt_result *d_results,
                                void *hip_stream);

int kt_set_timing(kt_ctx *ctx, int enable);
/* Accumulated device time per kernel: names kt_kernel_name(i), i < kt_num_kernels(). */
int kt_num_kernels(void);
const char *kt_kernel_name(int i);
int kt_get_kernel_times(kt_ctx *ctx, double *ms_out, int64_t *launches_out, int reset);

#ifdef __cplusplus
}
#endif

#endif
