/* include/slam2d/hector.h -- C-ABI of the MI355X Hector scan-matching + occupancy-grid path.
 *
 * Drop-in boundary: the reference's only polymorphic seam on this path is
 * hectorslam::MapRepresentationInterface (lesson4/include/lesson4/hector_mapping/slam_main/
 * MapRepresentationInterface.h:44-69), owned by HectorSlamProcessor (HectorSlamProcessor.h:61).
 * Each entry point below names the reference member it replaces.  include/slam2d/MapRepHip.h is the
 * C++ adapter `MapRepHip : MapRepresentationInterface` a maintainer adds on the ROS side.
 *
 * Conventions
 *   - plain C types only; poses are float[3] (x, y, theta) in world metres/radians, covariance a
 *     row-major float[9], scan points float[2*n] in map scale (DataContainer: point * scaleToMap,
 *     hector_slam.cc:356) with origo (ox, oy) also in map scale (hector_slam.cc:329).
 *   - every function returns HS_OK (0) or a negative HS_E* code; hs_last_error() describes it.
 *     No exceptions cross the boundary.  The reference itself has no error reporting; its silent
 *     semantics are kept (empty scan -> hint, out-of-map beam -> skipped, singular H -> no step).
 *   - a context holds `num_streams` independent SLAM streams (one map pyramid each) resident in HBM.
 *     num_streams = 1 is the ROS drop-in; > 1 is the batched throughput path.  Calls on one context
 *     may come from several host threads (e.g. the publish thread's hs_get_map beside the spin
 *     thread's hs_update, hector_slam.cc:201 / :277): an internal mutex serialises them.
 *   - host-pointer entry points copy through pinned staging and synchronise; *_device entry points
 *     take device pointers and a hipStream_t (as void*, NULL = the context's own stream, a blocking
 *     stream, so it is ordered after work queued on the legacy default stream) and do not
 *     synchronise.  Device work of one context is ordered across streams: every call first waits
 *     (on its own stream) for the context's previous device work, so consecutive calls may use
 *     different HIP streams.
 */
#ifndef SLAM2D_HECTOR_H
#define SLAM2D_HECTOR_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HS_OK 0
#define HS_EINVAL (-1)
#define HS_EHIP (-2)
#define HS_ENOMEM (-3)
#define HS_ENODEV (-4)
#define HS_ESTATE (-5) /* the device state cannot be decoded as asked (hs_get_map after an ordinal overflow) */

#define HS_MAX_LEVELS 8

typedef struct hs_ctx hs_ctx;

/* Version / self-description of the built library. */
const char *hs_version(void);
/* 16 hex digits of sha256 over the Hector kernel sources the library was compiled from (csrc/Makefile
 * SRC_HASH; bench.py reports it as config.kernel_src and refuses a library that differs from the tree). */
const char *hs_source_id(void);
const char *hs_last_error(void);

/* HectorSlamProcessor ctor + MapRepMultiMap ctor (HectorSlamProcessor.h:57-68, MapRepMultiMap.h:57-90).
 * map_resolution/map_size/start/levels are the ROS params map_resolution, map_size, map_start_x/y,
 * map_multi_res_levels (hector_slam.cc:138-142).  max_points bounds the scan size (>= 1). */
/* Limits: map sizes <= 32768 cells per side, 1 <= max_points <= 65535. */
int hs_create(hs_ctx **out, int num_streams, float map_resolution, int map_size_x, int map_size_y,
              float map_start_x, float map_start_y, int levels, int max_points);
/* ~HectorSlamProcessor (HectorSlamProcessor.h:70-73) */
int hs_destroy(hs_ctx *ctx);
/* HectorSlamProcessor::reset (HectorSlamProcessor.h:111-117) for every stream: grids cleared, pose and
 * last-map-update pose reset; the update indices, the last covariance and the stored containers are
 * kept, as in the reference (GridMapBase::reset clears cells only, MapRepMultiMap::reset the maps only). */
int hs_reset(hs_ctx *ctx);
/* MapRepresentationInterface::setUpdateFactorFree / setUpdateFactorOccupied (:67-68) */
int hs_set_update_factors(hs_ctx *ctx, float free_factor, float occupied_factor);
/* HectorSlamProcessor::setMapUpdateMinDistDiff / setMapUpdateMinAngleDiff (HectorSlamProcessor.h:137-138) */
int hs_set_map_update_thresholds(hs_ctx *ctx, float min_dist, float min_angle);

/* MapRepresentationInterface::getScaleToMap / getMapLevels (:50-52) */
int hs_get_scale_to_map(hs_ctx *ctx, float *scale_out);
int hs_get_map_levels(hs_ctx *ctx, int *levels_out);
/* GridMap dimensions / cell length / world origin of cell (0,0) for level (GridMapBase.h:85-87,301-304) */
int hs_get_map_info(hs_ctx *ctx, int level, int *size_x, int *size_y, float *cell_length, float *origin_xy);

/* HectorSlamProcessor::update (HectorSlamProcessor.h:81-108) on one stream: match coarse->fine,
 * store the pose, update every level if the pose moved more than the thresholds (or
 * map_without_matching).  hint NULL = the stream's last scan-match pose (hector_slam.cc:201).
 * did_update_out may be NULL. */
int hs_update(hs_ctx *ctx, int stream, const float *xy, int n, float ox, float oy, const float *hint,
              int map_without_matching, float pose_out[3], float cov_out[9], int *did_update_out);
/* MapRepresentationInterface::matchData (MapRepMultiMap.h:144-167): no pose / map change; like the
 * reference it keeps the matched DataContainer (dataContainers[l-1].setFrom, :161), which a later
 * hs_update_by_scan / hs_update(map_without_matching) draws into levels >= 1 (:187). */
int hs_match(hs_ctx *ctx, int stream, const float *xy, int n, float ox, float oy, const float hint[3],
             float pose_out[3], float cov_out[9]);
/* MapRepresentationInterface::updateByScan + onMapUpdated (MapRepMultiMap.h:174-191, :127-135): level 0
 * from (xy, n, ox, oy); levels >= 1 from the container of the stream's last match (empty before the
 * first one), exactly as MapRepMultiMap::updateByScan does. */
int hs_update_by_scan(hs_ctx *ctx, int stream, const float *xy, int n, float ox, float oy, const float pose[3]);

/* HectorSlamProcessor::getLastScanMatchPose / getLastScanMatchCovariance (HectorSlamProcessor.h:120-122) */
int hs_get_last_pose(hs_ctx *ctx, int stream, float pose_out[3], float cov_out[9]);

/* getGridMap(level) read-out (MapRepresentationInterface.h:54) in the publishMap format
 * (hector_slam.cc:287-304): occ_out int8 row-major (-1 unknown, 0 free, 100 occupied); optional raw
 * log-odds and per-cell updateIndex; update_index_out = GridMapBase::getUpdateIndex (GridMapBase.h:334).
 * Any output pointer may be NULL. */
int hs_get_map(hs_ctx *ctx, int stream, int level, int8_t *occ_out, float *logodds_out, int32_t *cell_update_index_out,
               int *update_index_out);
/* Overwrite one level's cells (log-odds + updateIndex); for tests and map reload. */
int hs_set_map(hs_ctx *ctx, int stream, int level, const float *logodds, const int32_t *cell_update_index);

/* ---- batched, device-resident throughput path ------------------------------------------------ */
/* One HectorSlamProcessor::update for every stream in [stream_begin, stream_begin+count):
 *   d_xy     : device float2 points, stream s at d_xy + 2*xy_stride*(s - stream_begin)
 *   d_n      : device int per stream, 0 <= n <= max_points (the match kernel clamps a count outside that
 *              range to it: device-side counts are not checked by the host)
 *   d_origo  : device float2 per stream, or NULL for (0,0)
 *   d_hints  : device float3 per stream, or NULL = each stream's last pose
 * Results stay on device; read them with hs_get_poses (synchronising) when needed. */
int hs_step_batch_device(hs_ctx *ctx, int stream_begin, int count, const float *d_xy, int xy_stride, const int *d_n,
                         const float *d_origo, const float *d_hints, void *hip_stream);
/* ---- scan ingest (LaserScan -> DataContainer), on the device ------------------------------------
 * HectorMappingRos::scanCallback (lesson4/src/hector_mapping/hector_slam.cc:186-198): laser_geometry's
 * projectLaser(scan, cloud, 30.0) then rosPointCloudToDataContainer (:320-362), restated for a batch of
 * raw range arrays.  Field names follow the node's parameters (hector_slam.cc:129, 151-161). */
typedef struct hs_laser {
    int n_beams;                 /* ranges per scan (<= max_points of the context) */
    float angle_min;             /* sensor_msgs/LaserScan angle_min, angle_increment (float32 fields) */
    float angle_increment;
    float range_min;             /* LaserScan range_min: projectLaser keeps range >= range_min */
    double range_cutoff;         /* projectLaser's range_cutoff (30.0 at hector_slam.cc:193): keeps range < it */
    double basis[9];             /* laserTransform_ (base frame <- scan frame) rotation, tf::Matrix3x3 rows */
    double origin[3];            /* laserTransform_ translation (laserPos) */
    float sqr_laser_min_dist;    /* p_sqr_laser_min_dist_ = (float)(laser_min_dist^2)       (:151-152) */
    float sqr_laser_max_dist;    /* p_sqr_laser_max_dist_ = (float)(laser_max_dist^2)       (:154-155) */
    double use_max_scan_range;   /* p_use_max_scan_range_                                    (:129) */
    float laser_z_min_value;     /* p_laser_z_min_value_ / p_laser_z_max_value_              (:157-161) */
    float laser_z_max_value;
} hs_laser;
/* The node's defaults for an n-beam scan (laser_min_dist 0.2, laser_max_dist 30, use_max_scan_range
 * 20, z in (-1, 1), cutoff 30, identity transform); the caller sets angles and the transform. */
void hs_default_laser(hs_laser *laser, int n_beams, float angle_min, float angle_increment);
/* Install the scan geometry.  unit_vectors: 2*n_beams doubles (cos_i, sin_i) of
 * angle_min + (double)i * angle_increment as laser_geometry caches them (getUnitVectors_), or NULL to
 * compute them here with the host libm. */
int hs_set_laser(hs_ctx *ctx, const hs_laser *laser, const double *unit_vectors);
/* d_ranges float[count][range_stride] (device) -> d_xy float2 (stride xy_stride), d_n int per stream,
 * d_origo float2 per stream (may be NULL): the DataContainer of each stream, points in map scale. */
int hs_ingest_batch_device(hs_ctx *ctx, int count, const float *d_ranges, int range_stride, float *d_xy,
                           int xy_stride, int *d_n, float *d_origo, void *hip_stream);
/* scanCallback for a batch: ingest every stream's ranges into the context's own point buffers, then
 * one HectorSlamProcessor::update per stream (as hs_step_batch_device; hints NULL = last pose).  For
 * scans of <= 1280 beams the ingest runs inside the match kernel (SLAM2D_FUSE_INGEST=0 at hs_create:
 * a separate kernel); the results are the same bit for bit. */
int hs_step_ranges_batch_device(hs_ctx *ctx, int stream_begin, int count, const float *d_ranges, int range_stride,
                                const float *d_hints, void *hip_stream);
/* scanCallback for `steps` consecutive scans of EVERY stream (offline / bag replay of a whole fleet):
 * step k's ranges start at d_ranges + k * step_stride floats, stream s's at + s * range_stride.  Equal,
 * bit for bit, to `steps` calls of hs_step_ranges_batch_device(ctx, 0, num_streams, ...) with NULL hints
 * (the streams are independent).  With SLAM2D_PIPELINE=1 in the environment at hs_create, the fleet runs
 * as two halves on two HIP streams so that one half's grid update overlaps the other half's match
 * (measured slower on MI355X at 1024 streams).  hip_stream waits for all of it. */
int hs_run_ranges_device(hs_ctx *ctx, int steps, const float *d_ranges, int range_stride, size_t step_stride,
                         void *hip_stream);
/* scanCallback for one stream from host ranges (the ROS drop-in entry point). */
int hs_update_ranges(hs_ctx *ctx, int stream, const float *ranges, float pose_out[3], float cov_out[9],
                     int *did_update_out);

/* Copy poses (float3), covariances (float9), did-update flags and Σ cells traversed of the last
 * step (int64, Σ_levels Σ_valid rays (abs_da + 1)) for every stream.  Any pointer may be NULL. */
int hs_get_poses(hs_ctx *ctx, float *poses_out, float *covs_out, int *did_update_out, int64_t *cells_traversed_out);
/* Cumulative work counters summed over streams since the last reset (synchronises):
 * out[0] Σ cells traversed (Σ abs_da+1), out[1] valid rays, out[2] Σ points x GN iterations,
 * out[3] map updates, out[4] steps, out[5] distinct cells written by the grid update (each is
 * one 4 B log-odds read + 8 B write: the minimum HBM traffic of the update).  reset != 0 zeroes
 * them afterwards. */
int hs_get_counters(hs_ctx *ctx, int64_t out[6], int reset);
/* Grid-update queue of the last step: out[0] tile work items, out[1] ray segments, out[2] WHOLE
 * (unbinned) level items, out[3] overflow events (cumulative); out[4..7] diagnostic-build phase
 * cycle sums of hs_tile_kernel (setup+clear, raster, apply, tiles; zero in normal builds). */
int hs_get_queue_stats(hs_ctx *ctx, int64_t out[8], int reset_stamps);
/* The eight diagnostic cycle counters diagnostic builds accumulate (tools/build_diag.py; zero in normal builds:
 * the product kernels never write them); reset != 0 zeroes them. */
int hs_get_diag_stamps(hs_ctx *ctx, int64_t out[8], int reset);
/* Device cell storage (for zero-copy consumers): per stream `stream_words` 4-byte words; each level
 * is a grid of 64 x 32-cell tiles, each tile 20 KB = 2048 log-odds floats, then 2048 uint16 update
 * ordinals h, then 2048 int32 updateIndex values; inside a tile's plane the cells are stored in 4 x 4-cell
 * blocks, the blocks row-major (element of cell (lx, ly) = ((ly/4)*16 + lx/4)*16 + (ly%4)*4 + lx%4).  The
 * log-odds plane is always current.  A cell's updateIndex is 3*(E + (h-1)/2) + 1 + (h-1)%2 when h != 0, else
 * the int32 plane's value; E (the stream's ordinal epoch) is internal, so a zero-copy reader of updateIndex
 * first calls hs_flush_ordinals, after which every h is 0 and the int32 plane alone holds every cell's
 * updateIndex.  hs_get_map decodes it without a flush (DESIGN.md "Data layout"). */
int hs_get_device_buffers(hs_ctx *ctx, void **cells, size_t *cells_bytes, size_t *stream_words);
/* Move every stream's 16-bit update ordinals into the int32 updateIndex plane now (the sweep the library runs by
 * itself at least every 32000 steps; on hip_stream, NULL = the context's stream, ordered after the context's
 * previous device work).  The library counts steps on the host to schedule its sweep: a caller that captures
 * *_device calls into a HIP graph and replays it bypasses that count, and must call hs_flush_ordinals at least
 * every 32000 replayed steps.  Past that bound a stream's ordinals no longer fit 16 bits: the device flags the
 * stream, and hs_get_map returns HS_ESTATE for its updateIndex (never a wrapped value) until hs_reset. */
int hs_flush_ordinals(hs_ctx *ctx, void *hip_stream);
/* Optional device pose log: every step appends the scan-match pose (float3) of streams [0, streams)
 * at row = steps since hs_reset, i.e. d_buf[(row*streams + s)*3]; rows >= capacity are dropped.
 * d_buf NULL disables.  The caller owns d_buf (device memory of >= capacity*streams*3 floats). */
int hs_set_pose_log(hs_ctx *ctx, float *d_buf, int streams, int capacity);
/* The same for any subset of streams: stream s is logged in slot d_slot_of_stream[s] (device int[num_streams],
 * < 0 = not logged), i.e. d_buf[(row*slots + slot)*3]. */
int hs_set_pose_log_slots(hs_ctx *ctx, float *d_buf, const int *d_slot_of_stream, int slots, int capacity);
/* The context's own HIP stream (hipStream_t as void*). */
void *hs_get_stream(hs_ctx *ctx);

/* ---- Hessian summation order of the matcher -------------------------------------------------------
 * HS_ORDER_REFERENCE (default): H and dTr summed point after point as getCompleteHessianDerivs does
 * (OccGridMapUtil.h:94-126) -- poses equal the reference's evaluation order bit for bit.
 * HS_ORDER_TREE256: per-thread strided partials + xor butterflies (faster; float reassociation of the
 * same sums).  SLAM2D_MATCH_ORDER=tree in the environment at hs_create selects it too. */
#define HS_ORDER_REFERENCE 0
#define HS_ORDER_TREE256 256
int hs_set_reduction_order(hs_ctx *ctx, int order);
int hs_get_reduction_order(hs_ctx *ctx, int *order_out);

/* ---- measurement ----------------------------------------------------------------------------- */
/* Kernel timing with HIP events recorded on the launch stream around every kernel of every step
 * (enable = 1).  hs_get_kernel_times fills, for the 3 kernels {hs_match_kernel, hs_bin_kernel,
 * hs_tile_kernel}, the accumulated milliseconds and launch counts since the last reset (synchronises). */
int hs_set_timing(hs_ctx *ctx, int enable);
int hs_get_kernel_times(hs_ctx *ctx, double ms_out[3], int64_t launches_out[3], int reset);
/* Effective shader clock of the Hector kernels (no reference counterpart).  With the probe on, every
 * 16th workgroup of hs_match_kernel and hs_update_kernel adds its lifetime in shader cycles (s_memtime)
 * and in 100-MHz real-time ticks (s_memrealtime); hs_get_clock_probe (synchronises) returns
 * {match cycles, match ticks, match workgroups, update cycles, update ticks, update workgroups}
 * since the last reset: clock = cycles / ticks x 100 MHz. */
int hs_set_clock_probe(hs_ctx *ctx, int enable);
int hs_get_clock_probe(hs_ctx *ctx, double out[6], int reset);

#ifdef __cplusplus
}
#endif
#endif
