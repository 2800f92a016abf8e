// hector_capi.hip -- host runtime + extern "C" boundary (include/slam2d/hector.h) for the MI355X
// Hector path.  Mirrors HectorSlamProcessor / MapRepMultiMap (lesson4/include/lesson4/hector_mapping/
// slam_main/) over device-resident state; every compute step is a HIP kernel (hector_kernels.hip).
// There is no CPU fallback: without a usable HIP device hs_create fails with HS_ENODEV.
#include <hip/hip_runtime.h>

#include <float.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <mutex>
#include <string>
#include <vector>

#include "../../include/slam2d/hector.h"
#include "hector_kernels.hip"

using namespace s2d;

namespace {
thread_local std::string g_err;

int fail(int code, const char *what, hipError_t e = hipSuccess)
{
    g_err = what;
    if (e != hipSuccess) {
        g_err += ": ";
        g_err += hipGetErrorString(e);
    }
    return code;
}

#define LOCK(c) std::lock_guard<std::recursive_mutex> lock_(c->mu)

#define HCHK(expr)                                          \
    do {                                                    \
        hipError_t _e = (expr);                             \
        if (_e != hipSuccess) return fail(HS_EHIP, #expr, _e); \
    } while (0)

constexpr int NKERN = 3;
constexpr int MAX_PARTS = 4;

struct EventPair {
    hipEvent_t a, b;
    int kernel;
};
}  // namespace

struct hs_ctx {
    int B = 0, levels = 0, max_points = 0, sx = 0, sy = 0;
    float res = 0, start_x = 0, start_y = 0;
    FleetGeom geom{};
    float *d_cells = nullptr;  // tiled words (hector_internal.h)
    size_t cells_bytes = 0;
    StreamState *d_state = nullptr;
    // single-stream staging (host-pointer entry points)
    float2 *d_pts1 = nullptr;
    int *d_n1 = nullptr;
    float2 *d_origo1 = nullptr;
    float *d_hint1 = nullptr;
    float *d_out_pose = nullptr;
    float *d_out_cov = nullptr;
    int8_t *d_occ = nullptr;
    PoseLog plog{nullptr, 0, 0, nullptr};
    hipStream_t stream = nullptr;
    // timing
    bool timing = false;
    std::vector<EventPair> ev_used, ev_free;
    double acc_ms[NKERN] = {0, 0, 0};
    int64_t acc_n[NKERN] = {0, 0, 0};
    // binned grid update scratch
    unsigned *d_rays = nullptr;
    uint4 *d_segs = nullptr;
    WorkItem *d_items = nullptr;
    WorkItem *d_wholes = nullptr;
    WorkQueue *d_wq = nullptr;  // one queue per part
    unsigned seg_cap = 0, item_cap = 0;  // per part
    int tile_grid = 0;
    // batch split into parts on separate HIP streams so one part's tile kernel overlaps another
    // part's match / bin kernels (they are latency-bound at low occupancy)
    int nparts = 1;
    // queue slots (work queue, segment / item / whole ranges) = parts that can be in flight: nparts, and at
    // least 2 when the pipelined run (SLAM2D_PIPELINE=1) drives the two fleet halves as parts 0 and 1
    int nq = 1;
    int update_single = 1;  // hs_update_kernel (per stream-level, default) or bin + tile kernels
    // the single-kernel update: the round-3 hs_update_kernel (per-tile clipping; default) or
    // hs_update_ring_kernel (ring-ordered tiles, ray cursors; SLAM2D_UPD_KERNEL=ring, scans of <= 1280 points)
    bool upd_ring = false;
    int ncu = 256;
    bool upd_parts_fixed = false;  // SLAM2D_UPD_PARTS given: no batch-size adaptive split
    // per part (a batch split over part streams): two alternating lists of updating streams
    // (hector_internal.h UpdList): the match kernel appends to one, the update kernel reads it and
    // clears the other for the next step
    UpdList *wl[MAX_PARTS][2] = {};
    int wl_parity[MAX_PARTS] = {};
    hipStream_t pstream[MAX_PARTS] = {};
    hipEvent_t ev_start = nullptr, ev_done[MAX_PARTS] = {};
    // hs_run_ranges_device pipeline (SLAM2D_PIPELINE=1): update of one half of the fleet beside the other
    // half's match.  Measured slower at the north-star size (0.97 M vs 1.04 M scans/s: the update
    // kernel already fills the CUs, and a concurrent match slows it more than it hides), so off by default.
    bool pipeline = false;
    // ordinal sweep (hector_internal.h ORD_OFF): steps since the last one, and the interval (SLAM2D_ORD_SWEEP, tests)
    int ord_steps = 0;
    int ord_interval = ORD_SWEEP_MAX;
    bool fuse_ingest = true;  // range arrays: ingest inside the match kernel (SLAM2D_FUSE_INGEST=0: own kernel)
    // Hessian summation order of hs_match_kernel: 0 = the reference's sequential point order (default),
    // 256 = the 256-thread tree (hs_set_reduction_order / SLAM2D_MATCH_ORDER=tree)
    int reduce_order = 0;
    hipEvent_t ev_upd[MAX_PARTS] = {};
    // the last device work of the context (every *_device call waits for it on its own stream, so the
    // per-context scratch -- update lists, ingest buffers, queues -- is never used by two streams at once)
    hipEvent_t ev_last = nullptr;
    // serialises host calls on one context (e.g. a publish thread's hs_get_map against the spin
    // thread's hs_update, hector_slam.cc:277 vs :201)
    std::recursive_mutex mu;
    // scan ingest (hs_set_laser): unit vectors, geometry
    bool has_laser = false;
    IngestGeom ingest{};
    double2 *d_cs = nullptr;
    // per-stream DataContainer buffer [B][max_points]: the range-array entry points ingest into it, and
    // after every match it holds the stream's matched container, which MapRepMultiMap keeps for the
    // update of levels >= 1 (StreamState::mc_n / mc_origo; MapRepMultiMap.h:161, :187)
    float2 *d_ixy = nullptr;
    int *d_in = nullptr;
    float2 *d_iorigo = nullptr;
    float *d_ranges1 = nullptr;
    // clock probe buffer (hs_set_clock_probe): 8 counters, see FleetGeom::clk
    unsigned long long *d_clk = nullptr;
    size_t stream_pad_words = 0;  // see init_geometry
};

namespace {

// MapRepMultiMap ctor (MapRepMultiMap.h:57-90) + GridMapBase::setMapTransformation (GridMapBase.h:270-286)
void init_geometry(hs_ctx *c)
{
    FleetGeom &g = c->geom;
    g.levels = c->levels;
    int rx = c->sx, ry = c->sy;
    float res = c->res;
    float total_x = c->res * (float)c->sx;
    float mid_x = total_x * c->start_x;
    float total_y = c->res * (float)c->sy;
    float mid_y = total_y * c->start_y;
    size_t off = 0;
    for (int i = 0; i < c->levels; ++i) {
        LevelGeom &L = g.lv[i];
        L.sx = rx;
        L.sy = ry;
        L.lim[0] = (float)rx - 2.0f;
        L.lim[1] = (float)ry - 2.0f;
        L.cell_len = res;
        L.scale = 1.0f / res;
        L.map_t[0] = L.scale * mid_x;
        L.map_t[1] = L.scale * mid_y;
        float m00 = L.scale, m01 = 0.0f, m10 = 0.0f, m11 = L.scale;
        float det = m00 * m11 - m10 * m01;
        float invdet = 1.0f / det;
        L.inv_l[0] = m11 * invdet;
        L.inv_l[2] = -m10 * invdet;
        L.inv_l[1] = -m01 * invdet;
        L.inv_l[3] = m00 * invdet;
        L.inv_t[0] = (-L.inv_l[0]) * L.map_t[0] + (-L.inv_l[1]) * L.map_t[1];
        L.inv_t[1] = (-L.inv_l[2]) * L.map_t[0] + (-L.inv_l[3]) * L.map_t[1];
        L.pts_scale = (float)(1.0 / pow(2.0, (double)i));
        L.tiles_x = (rx + TILE - 1) / TILE;
        L.tiles_y = (ry + TILE_H - 1) / TILE_H;
        L.word_offset = off;
        off += (size_t)L.tiles_x * L.tiles_y * TILE_BLOCK_WORDS;
        rx /= 2;
        ry /= 2;
        res *= 2.0f;
    }
    // per-stream pad (SLAM2D_STREAM_PAD bytes, a multiple of 256): a stream's levels add up to a multiple of
    // 2 MB, so without it the same tile of every stream sits at the same offset modulo every power-of-two
    // interleave period of the memory system
    g.stream_words = off + c->stream_pad_words;
    g.cells_words = off;
}

// GridMapLogOddsFunctions::probToLogOdds  GridMapLogOdds.h:153-157
float prob_to_logodds(float prob)
{
    float odds = prob / (1.0f - prob);
    return (float)log((double)odds);
}

StreamState initial_state()
{
    // HectorSlamProcessor::reset (HectorSlamProcessor.h:111-117); OccGridMapBase ctor indices
    StreamState st;
    memset(&st, 0, sizeof(st));
    st.last_upd_pose[0] = st.last_upd_pose[1] = st.last_upd_pose[2] = FLT_MAX;
    st.cur_update_index = 0;
    st.map_updates = 0;
    return st;
}

// full (hs_create): every stream from the constructor state.  Otherwise HectorSlamProcessor::reset
// (HectorSlamProcessor.h:111-117): lastMapUpdatePose = FLT_MAX, lastScanMatchPose = 0, every grid
// cleared (GridMapBase::reset -> clear, GridMapBase.h:94-113); what the reference keeps is kept: the
// grids' currUpdateIndex / lastUpdateIndex (OccGridMapBase.h:334, GridMapBase.h:413), lastScanMatchCov
// and MapRepMultiMap's stored containers (MapRepMultiMap.h:102-110 resets the maps only).
int reset_all(hs_ctx *c, bool full)
{
    size_t nwords = c->cells_bytes / sizeof(float);
    hipLaunchKernelGGL(hs_fill_cells_kernel, dim3(4096), dim3(256), 0, c->stream, c->d_cells, nwords,
                       c->geom.stream_words);
    HCHK(hipGetLastError());
    std::vector<StreamState> h(c->B, initial_state());
    if (!full) {
        std::vector<StreamState> old(c->B);
        HCHK(hipMemcpyAsync(old.data(), c->d_state, sizeof(StreamState) * c->B, hipMemcpyDeviceToHost, c->stream));
        HCHK(hipStreamSynchronize(c->stream));
        for (int s = 0; s < c->B; ++s) {
            StreamState &o = old[s];
            o.last_upd_pose[0] = o.last_upd_pose[1] = o.last_upd_pose[2] = FLT_MAX;
            o.pose[0] = o.pose[1] = o.pose[2] = 0.0f;
            o.do_update = 0;
            o.step_index = 0;
            // the fill zeroed every hot ordinal: a fresh ordinal epoch at the stream's current update (decoding
            // needs E only for non-zero ordinals), which also clears an ordinal overflow
            o.ord_epoch = o.cur_update_index / 3;
            o.ord_overflow = 0;
            h[s] = o;
        }
    }
    HCHK(hipMemcpyAsync(c->d_state, h.data(), sizeof(StreamState) * c->B, hipMemcpyHostToDevice, c->stream));
    for (int p = 0; p < MAX_PARTS; ++p)
        for (int i = 0; i < 2; ++i)
            if (c->wl[p][i]) HCHK(hipMemsetAsync(c->wl[p][i], 0, sizeof(int) * 4, c->stream));
    for (int p = 0; p < MAX_PARTS; ++p) c->wl_parity[p] = 0;
    c->ord_steps = 0;  // every stream starts a new ordinal epoch
    HCHK(hipStreamSynchronize(c->stream));
    return HS_OK;
}

EventPair *begin_timed(hs_ctx *c, int kernel, hipStream_t s)
{
    if (!c->timing) return nullptr;
    EventPair p;
    if (!c->ev_free.empty()) {
        p = c->ev_free.back();
        c->ev_free.pop_back();
    } else {
        if (hipEventCreate(&p.a) != hipSuccess || hipEventCreate(&p.b) != hipSuccess) return nullptr;
    }
    p.kernel = kernel;
    hipEventRecord(p.a, s);
    c->ev_used.push_back(p);
    return &c->ev_used.back();
}

void end_timed(hs_ctx *c, hipStream_t s)
{
    if (!c->timing || c->ev_used.empty()) return;
    hipEventRecord(c->ev_used.back().b, s);
}

// hs_update_kernel instance: rays in registers for scans of at most UPD_RREG * 256 points (no LDS ray
// array), else in LDS; SLAM2D_UPD_RAYS_LDS=1 forces the LDS instance (A/B)
bool upd_rays_in_regs(const hs_ctx *c)
{
    static const bool force_lds = getenv("SLAM2D_UPD_RAYS_LDS") && atoi(getenv("SLAM2D_UPD_RAYS_LDS")) != 0;
    return !force_lds && c->max_points <= UPD_RREG * UPD_THREADS;
}

size_t upd_shmem_bytes(const hs_ctx *c)
{
    const size_t rays = upd_rays_in_regs(c) ? 0 : (size_t)((c->max_points + 3) & ~3);
    return sizeof(unsigned) * ((size_t)UPD_FIXED_WORDS + rays + UPD_GROUP_WORDS * (size_t)fan_groups(c->max_points));
}

// hs_update_kernel's packed raster walk keeps the Bresenham error f < da in 14 bits (V = f << 18 | LDS
// address): rays of at most 16384 cells, i.e. level-0 maps of at most 16385 cells per side.  Larger maps
// take the binned kernels (their walk keeps the error in its own register), as do scans whose rays would
// not fit the kernel's LDS (the binned kernels' LDS use is independent of the scan size).
bool upd_single_ok(const hs_ctx *c)
{
    return c->update_single && upd_shmem_bytes(c) <= 65536 && c->sx <= 16385 && c->sy <= 16385;
}

size_t ring_shmem_bytes(const hs_ctx *c) { return sizeof(unsigned) * (size_t)ring_shmem_words(c->max_points); }

// hs_update_ring_kernel: rays in registers (<= RING_GROUPS * 256 points), da / db in 14 bits (<= 16384
// cells per side)
bool upd_ring_ok(const hs_ctx *c)
{
    return c->upd_ring && c->max_points <= 5 * 256 && c->sx <= 16384 && c->sy <= 16384;
}

int launch_part(hs_ctx *c, int part, int begin, int count, const float2 *xy, int xy_stride, const int *n,
                const float2 *origo, const float *hints, int mode, float *out_pose, float *out_cov, hipStream_t s,
                hipEvent_t wait_before_update = nullptr, const MatchIngest *mi = nullptr)
{
    if (part < 0 || part >= c->nq) return fail(HS_EINVAL, "internal: part without a queue slot");
    WorkQueue *wq = c->d_wq + part;
    uint4 *segs = c->d_segs + (size_t)part * c->seg_cap;
    WorkItem *items = c->d_items + (size_t)part * c->item_cap;
    WorkItem *wholes = c->d_wholes + (size_t)part * c->B * c->levels;
    // the single-kernel update consumes the match kernel's list of updating streams (wl[part][parity]: one
    // pair of lists per part)
    const size_t upd_shmem = upd_shmem_bytes(c);
    const bool single = upd_single_ok(c);
    const bool use_list = single && !c->upd_parts_fixed && mode != MODE_MATCH_ONLY;
    UpdList *wl_cur = use_list ? c->wl[part][c->wl_parity[part]] : nullptr;
    begin_timed(c, 0, s);
    // the register-only instance when no scan of the context can exceed the kernel's register slots
    const MatchIngest mik = mi ? *mi : MatchIngest{};
#define S2D_MATCH_LAUNCH(SEQ, REGS, BIG)                                                                                 \
    hipLaunchKernelGGL((hs_match_kernel<SEQ, REGS, BIG>), dim3(count), dim3(MATCH_THREADS), 0, s, c->geom, c->d_cells,    \
                       c->d_state, xy, xy_stride, n, origo, hints, begin, mode, out_pose, out_cov, c->plog, wq, wl_cur,   \
                       c->ingest, mik, c->d_ixy, c->max_points)
    // a level of 2^30 words or more: the gathers' 32-bit byte offsets would overflow (hs_match_kernel BIG)
    bool big = false;
    for (int l = 0; l < c->levels; ++l)
        big = big || (unsigned long long)c->geom.lv[l].tiles_x * c->geom.lv[l].tiles_y * TILE_BLOCK_WORDS >= (1ull << 30);
    if (c->reduce_order == 0) {
        const bool regs = c->max_points <= (S2D_MATCH_CW ? CW_MAXN : MATCH_THREADS * MATCH_REG_PTS);
        if (big) {
            if (regs) S2D_MATCH_LAUNCH(true, true, true);
            else S2D_MATCH_LAUNCH(true, false, true);
        } else {
            if (regs) S2D_MATCH_LAUNCH(true, true, false);
            else S2D_MATCH_LAUNCH(true, false, false);
        }
    } else {
        if (c->max_points <= MATCH_THREADS * MATCH_REG_PTS) S2D_MATCH_LAUNCH(false, true, false);
        else S2D_MATCH_LAUNCH(false, false, false);
    }
#undef S2D_MATCH_LAUNCH
    end_timed(c, s);
    HCHK(hipGetLastError());
    if (mode == MODE_MATCH_ONLY) return HS_OK;
    if (wait_before_update) HCHK(hipStreamWaitEvent(s, wait_before_update, 0));
    // hs_update_kernel keeps the scan's rays in LDS: beyond 64 KB of dynamic LDS (max_points > ~13k)
    // the binned kernels, whose LDS use is independent of the scan size, take over
    if (single && use_list) {
        // grid for the largest split over U = 1 .. count updating streams; surplus workgroups exit
        int blocks = 0;
        for (int U = 1; U <= count; ++U) {
            int pl[MAX_LEVELS], b = 0;
            upd_split(U, c->ncu, c->levels, pl, c->geom.upd_minp);
            for (int l = 0; l < c->levels; ++l) b += pl[l] * U;
            blocks = b > blocks ? b : blocks;
        }
        UpdList *wl_next = c->wl[part][c->wl_parity[part] ^ 1];
        c->wl_parity[part] ^= 1;
        begin_timed(c, 2, s);
        if (upd_ring_ok(c))
            hipLaunchKernelGGL(hs_update_ring_kernel, dim3(blocks), dim3(RTHREADS), ring_shmem_bytes(c), s, c->geom,
                               c->d_cells, c->d_state, xy, xy_stride, c->d_ixy, c->max_points, begin, count, c->max_points,
                               wl_cur, wl_next, c->ncu);
        else if (upd_rays_in_regs(c))
            hipLaunchKernelGGL((hs_update_kernel<UPD_RREG>), dim3(blocks), dim3(UPD_THREADS), upd_shmem, s, c->geom, c->d_cells,
                               c->d_state, xy, xy_stride, c->d_ixy, c->max_points, begin, count, c->max_points, wl_cur,
                               wl_next, c->ncu);
        else
            hipLaunchKernelGGL((hs_update_kernel<0>), dim3(blocks), dim3(UPD_THREADS), upd_shmem, s, c->geom, c->d_cells,
                               c->d_state, xy, xy_stride, c->d_ixy, c->max_points, begin, count, c->max_points, wl_cur,
                               wl_next, c->ncu);
        end_timed(c, s);
        HCHK(hipGetLastError());
        return HS_OK;
    }
    if (single) {
        FleetGeom gg = c->geom;
        if (!c->upd_parts_fixed) {
            // small batches: split each level's tiles over several workgroups so that the grid fills the
            // CUs (one level-0 workgroup of a 2048^2 scan takes ~0.4 ms alone; a part costs one ray setup)
            // measured (2048^2 x 3, same box): B = 16: 2 per CU best; B = 64 .. 512: 4 per CU (+8 .. +33 %);
            // B >= 1024: level 0 in 2 parts (neutral to +1.5 %)
            const int target = count <= 32 ? 2 : 4;
            int p0 = (target * c->ncu + count - 1) / count;
            if (p0 < 2) p0 = 2;
            if (c->levels == 1 && p0 < 8) p0 = 8;  // as upd_split: a single level fills the grid's tail alone
            for (int l = 0; l < c->levels; ++l) {
                const int v = p0 >> l;
                gg.upd_parts[l] = v < 1 ? 1 : (v > 64 ? 64 : v);
            }
        }
        begin_timed(c, 2, s);
        int blocks = 0;
        for (int l = 0; l < c->levels; ++l) blocks += gg.upd_parts[l] * count;
        if (upd_ring_ok(c))
            hipLaunchKernelGGL(hs_update_ring_kernel, dim3(blocks), dim3(RTHREADS), ring_shmem_bytes(c), s, gg, c->d_cells,
                               c->d_state, xy, xy_stride, c->d_ixy, c->max_points, begin, count, c->max_points,
                               (const UpdList *)nullptr, (UpdList *)nullptr, c->ncu);
        else if (upd_rays_in_regs(c))
            hipLaunchKernelGGL((hs_update_kernel<UPD_RREG>), dim3(blocks), dim3(UPD_THREADS), upd_shmem, s, gg, c->d_cells,
                               c->d_state, xy, xy_stride, c->d_ixy, c->max_points, begin, count, c->max_points, (const UpdList *)nullptr,
                               (UpdList *)nullptr, c->ncu);
        else
            hipLaunchKernelGGL((hs_update_kernel<0>), dim3(blocks), dim3(UPD_THREADS), upd_shmem, s, gg, c->d_cells,
                               c->d_state, xy, xy_stride, c->d_ixy, c->max_points, begin, count, c->max_points, (const UpdList *)nullptr,
                               (UpdList *)nullptr, c->ncu);
        end_timed(c, s);
        HCHK(hipGetLastError());
        return HS_OK;
    }
    begin_timed(c, 1, s);
    hipLaunchKernelGGL(hs_bin_kernel, dim3(count), dim3(BIN_THREADS), 0, s, c->geom, c->d_state, xy, xy_stride, c->d_ixy,
                       c->max_points, begin, c->max_points, c->d_rays, segs, items, wholes, wq, c->seg_cap, c->item_cap);
    end_timed(c, s);
    HCHK(hipGetLastError());
    begin_timed(c, 2, s);
    hipLaunchKernelGGL(hs_tile_kernel, dim3(c->tile_grid), dim3(TILE_THREADS), 0, s, c->geom, c->d_cells, c->d_state,
                       c->d_rays, segs, items, wholes, wq, c->max_points);
    end_timed(c, s);
    HCHK(hipGetLastError());
    return HS_OK;
}

// Before every step that can update the maps: every ord_interval steps, move all streams' hot ordinals into the
// cold updateIndex plane and advance their epochs (a step advances a stream's update ordinal by at most one, so
// 2 (k - E) + 2 stays below 2^16).  On stream s, after the previous steps and before this one.
int ord_sweep_if_due(hs_ctx *c, hipStream_t s)
{
    if (c->ord_steps < c->ord_interval) {
        ++c->ord_steps;
        return HS_OK;
    }
    const int tiles = (int)(c->geom.cells_words / TILE_BLOCK_WORDS);
    hipLaunchKernelGGL(hs_ord_sweep_kernel, dim3(4096), dim3(256), 0, s, c->d_cells, c->d_state, c->geom.stream_words,
                       tiles, 0, c->B);
    HCHK(hipGetLastError());
    hipLaunchKernelGGL(hs_ord_epoch_kernel, dim3((c->B + 255) / 256), dim3(256), 0, s, c->d_state, 0, c->B);
    HCHK(hipGetLastError());
    c->ord_steps = 1;
    return HS_OK;
}

int launch_step(hs_ctx *c, int begin, int count, const float2 *xy, int xy_stride, const int *n, const float2 *origo,
                const float *hints, int mode, float *out_pose, float *out_cov, hipStream_t s,
                const MatchIngest *mi = nullptr)
{
    if (count <= 0) return HS_OK;
    if (mode != MODE_MATCH_ONLY && ord_sweep_if_due(c, s) != HS_OK) return HS_EHIP;
    const int parts = (mode == MODE_PROCESS && count >= 64 * c->nparts) ? c->nparts : 1;
    if (parts == 1)
        return launch_part(c, 0, begin, count, xy, xy_stride, n, origo, hints, mode, out_pose, out_cov, s, nullptr, mi);
    HCHK(hipEventRecord(c->ev_start, s));
    const int per = (count + parts - 1) / parts;
    for (int p = 0; p < parts; ++p) {
        const int off = p * per;
        const int cnt = count - off < per ? count - off : per;
        if (cnt <= 0) break;
        hipStream_t ps = c->pstream[p];
        HCHK(hipStreamWaitEvent(ps, c->ev_start, 0));
        MatchIngest pmi = mi ? *mi : MatchIngest{};
        if (mi) {
            pmi.ranges += (size_t)off * mi->rstride;
            pmi.xy_out += (size_t)off * xy_stride;
            pmi.n_out += off;
            pmi.origo_out += off;
        }
        int rc = launch_part(c, p, begin + off, cnt, xy + (size_t)off * xy_stride, xy_stride, n + off,
                             origo ? origo + off : nullptr, hints ? hints + 3 * (size_t)off : nullptr, mode,
                             out_pose ? out_pose + 3 * (size_t)off : nullptr, out_cov ? out_cov + 9 * (size_t)off : nullptr,
                             ps, nullptr, mi ? &pmi : nullptr);
        if (rc != HS_OK) return rc;
        HCHK(hipEventRecord(c->ev_done[p], ps));
        HCHK(hipStreamWaitEvent(s, c->ev_done[p], 0));
    }
    return HS_OK;
}

// The pipelined run (hs_run_ranges_device) needs the list-driven single update kernel on every part.
bool pipeline_ok(const hs_ctx *c)
{
    return c->pipeline && c->nq >= 2 && upd_single_ok(c) && !c->upd_parts_fixed && c->B >= 2;
}

int check_stream(hs_ctx *c, int stream) { return (c && stream >= 0 && stream < c->B) ? HS_OK : HS_EINVAL; }

// *_device calls may name any HIP stream: order each call after the context's previous device work
// (enter) and publish its own (leave), so two calls never share the context's scratch concurrently
int dev_enter(hs_ctx *c, hipStream_t s)
{
    HCHK(hipStreamWaitEvent(s, c->ev_last, 0));
    return HS_OK;
}
int dev_leave(hs_ctx *c, hipStream_t s)
{
    HCHK(hipEventRecord(c->ev_last, s));
    return HS_OK;
}

int launch_ingest(hs_ctx *c, int count, const float *d_ranges, int range_stride, float2 *d_xy, int xy_stride, int *d_n,
                  float2 *d_origo, hipStream_t s)
{
    hipLaunchKernelGGL(hs_ingest_kernel, dim3(count), dim3(256), 0, s, c->ingest, c->d_cs, d_ranges, range_stride, d_xy,
                       xy_stride, d_n, d_origo);
    HCHK(hipGetLastError());
    return HS_OK;
}

// ingest + step on range arrays: the ingest runs inside the match kernel (one launch less) when the
// scan fits the match kernel's registers (<= 1280 beams) unless SLAM2D_FUSE_INGEST=0; else its own kernel.
int launch_ranges_step(hs_ctx *c, int begin, int count, const float *d_ranges, int range_stride, float2 *xy,
                       int xy_stride, int *d_n, float2 *d_origo, const float *hints, float *out_pose, float *out_cov,
                       hipStream_t s)
{
    if (c->fuse_ingest && c->ingest.n <= MATCH_THREADS * MATCH_REG_PTS) {
        const MatchIngest mi{d_ranges, range_stride, c->d_cs, xy, d_n, d_origo};
        return launch_step(c, begin, count, xy, xy_stride, d_n, d_origo, hints, MODE_PROCESS, out_pose, out_cov, s, &mi);
    }
    int rc = launch_ingest(c, count, d_ranges, range_stride, xy, xy_stride, d_n, d_origo, s);
    if (rc == HS_OK) rc = launch_step(c, begin, count, xy, xy_stride, d_n, d_origo, hints, MODE_PROCESS, out_pose, out_cov, s);
    return rc;
}

// Stage one host scan into the single-stream buffers.
int stage_scan(hs_ctx *c, const float *xy, int n, float ox, float oy, const float *hint)
{
    if (n < 0 || n > c->max_points || (n > 0 && !xy)) return fail(HS_EINVAL, "bad scan size / pointer");
    if (n > 0) HCHK(hipMemcpyAsync(c->d_pts1, xy, sizeof(float2) * n, hipMemcpyHostToDevice, c->stream));
    HCHK(hipMemcpyAsync(c->d_n1, &n, sizeof(int), hipMemcpyHostToDevice, c->stream));
    float2 o = make_float2(ox, oy);
    HCHK(hipMemcpyAsync(c->d_origo1, &o, sizeof(float2), hipMemcpyHostToDevice, c->stream));
    if (hint) HCHK(hipMemcpyAsync(c->d_hint1, hint, sizeof(float) * 3, hipMemcpyHostToDevice, c->stream));
    return HS_OK;
}

}  // namespace

extern "C" {

#ifndef SLAM2D_SRC_HASH
#define SLAM2D_SRC_HASH "unknown"  // built outside csrc/Makefile
#endif
const char *hs_version(void) { return "slam2d-mi355x hector 0.1 (gfx950) src " SLAM2D_SRC_HASH; }
const char *hs_source_id(void) { return SLAM2D_SRC_HASH; }
const char *hs_last_error(void) { return g_err.c_str(); }

int hs_create(hs_ctx **out, int num_streams, float map_resolution, int map_size_x, int map_size_y, float map_start_x,
              float map_start_y, int levels, int max_points)
{
    if (!out) return fail(HS_EINVAL, "out is NULL");
    *out = nullptr;
    if (num_streams < 1 || levels < 1 || levels > HS_MAX_LEVELS || map_size_x < 2 || map_size_y < 2 ||
        map_size_x > 32768 || map_size_y > 32768 || max_points < 1 || max_points > 65535 || !(map_resolution > 0.0f))
        return fail(HS_EINVAL, "invalid hs_create arguments");
    if ((map_size_x >> (levels - 1)) < 2 || (map_size_y >> (levels - 1)) < 2)
        return fail(HS_EINVAL, "map too small for the requested number of levels");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1) return fail(HS_ENODEV, "no HIP device");
    size_t pad_words = 0;
    if (const char *sp = getenv("SLAM2D_STREAM_PAD")) {
        // bytes between streams' pyramids: a non-negative multiple of 256 (whole 64-word granules)
        char *end = nullptr;
        const long long v = strtoll(sp, &end, 10);
        if (end == sp || *end != '\0' || v < 0 || v % 256 != 0 || v > (1ll << 30))
            return fail(HS_EINVAL, "SLAM2D_STREAM_PAD must be a non-negative multiple of 256 bytes (<= 1 GiB)");
        pad_words = (size_t)(v / 256) * 64;
    }
    hs_ctx *c = new hs_ctx();
    c->B = num_streams;
    c->levels = levels;
    c->max_points = max_points;
    c->sx = map_size_x;
    c->sy = map_size_y;
    c->res = map_resolution;
    c->start_x = map_start_x;
    c->start_y = map_start_y;
    c->stream_pad_words = pad_words;
    init_geometry(c);
    c->geom.lf = prob_to_logodds(0.4f);  // GridMapLogOddsFunctions ctor (GridMapLogOdds.h:98-102)
    c->geom.lo = prob_to_logodds(0.6f);
    c->geom.min_dist = 0.4f * 1.0f;      // HectorSlamProcessor ctor (HectorSlamProcessor.h:66-67)
    c->geom.min_ang = 0.13f * 1.0f;
    c->cells_bytes = sizeof(float) * c->geom.stream_words * (size_t)num_streams;
    hipError_t e;
    // blocking streams (not hipStreamNonBlocking): work a caller queued on the legacy default stream
    // (e.g. torch's default stream zeroing an output) is ordered before the context's own kernels
    if ((e = hipStreamCreateWithFlags(&c->stream, hipStreamDefault)) != hipSuccess) {
        delete c;
        return fail(HS_EHIP, "hipStreamCreate", e);
    }
    if ((e = hipMalloc(&c->d_cells, c->cells_bytes)) != hipSuccess ||
        (e = hipMalloc(&c->d_state, sizeof(StreamState) * num_streams)) != hipSuccess ||
        (e = hipMalloc(&c->d_pts1, sizeof(float2) * max_points)) != hipSuccess ||
        (e = hipMalloc(&c->d_n1, sizeof(int))) != hipSuccess ||
        (e = hipMalloc(&c->d_origo1, sizeof(float2))) != hipSuccess ||
        (e = hipMalloc(&c->d_hint1, sizeof(float) * 3)) != hipSuccess ||
        (e = hipMalloc(&c->d_out_pose, sizeof(float) * 3 * num_streams)) != hipSuccess ||
        (e = hipMalloc(&c->d_out_cov, sizeof(float) * 9 * num_streams)) != hipSuccess ||
        (e = hipMalloc(&c->d_occ, (size_t)map_size_x * map_size_y)) != hipSuccess ||
        (e = hipMalloc(&c->d_ixy, sizeof(float2) * (size_t)num_streams * max_points)) != hipSuccess) {
        hs_destroy(c);
        return fail(HS_ENOMEM, "hipMalloc", e);
    }
    {
        // grid-update queues: 6 segments per ray on average, 512 non-empty tiles per stream level
        const size_t sl = (size_t)num_streams * levels;
        size_t segs = sl * (size_t)max_points * 6, its = sl * 512;
        if (segs < (1u << 20)) segs = 1u << 20;
        if (its < (1u << 14)) its = 1u << 14;
        c->seg_cap = (unsigned)(segs < 0xFFFFFFF0ull ? segs : 0xFFFFFFF0ull);
        c->item_cap = (unsigned)(its < 0xFFFFFFF0ull ? its : 0xFFFFFFF0ull);
        int dev = 0, ncu = 256;
        hipGetDevice(&dev);
        hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
        // grid-stride tile kernel: exactly the resident workgroups (occupancy query), overridable
        int per_cu = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, hs_tile_kernel, TILE_THREADS, 0) != hipSuccess ||
            per_cu < 1)
            per_cu = 4;
        const char *tg = getenv("SLAM2D_TILE_WG_PER_CU");
        c->tile_grid = ncu * (tg ? atoi(tg) : per_cu);
        const char *pp = getenv("SLAM2D_PIPELINE");
        c->pipeline = pp && atoi(pp) != 0;
        const char *mo = getenv("SLAM2D_MATCH_ORDER");
        c->reduce_order = (mo && strcmp(mo, "tree") == 0) ? MATCH_THREADS : 0;
        const char *fi = getenv("SLAM2D_FUSE_INGEST");
        c->fuse_ingest = !(fi && atoi(fi) == 0);
        // steps between ordinal sweeps (tests set a few to exercise the sweep; at most ORD_SWEEP_MAX).  0: never
        // (TEST ONLY: stands for a caller that replays graph captures of *_device calls without hs_flush_ordinals,
        // to exercise the device's ordinal-overflow flag)
        if (const char *os = getenv("SLAM2D_ORD_SWEEP")) {
            const int v = atoi(os);
            c->ord_interval = v == 0 ? INT_MAX : (v < 1 ? 1 : (v > ORD_SWEEP_MAX ? ORD_SWEEP_MAX : v));
        }
        const char *np = getenv("SLAM2D_PARTS");
        c->nparts = np ? atoi(np) : 1;
        const char *um = getenv("SLAM2D_UPDATE");
        c->update_single = (um && strcmp(um, "binned") == 0) ? 0 : 1;  // measured: single 1.06 ms vs binned 1.30 ms
        // measured (round 4, profiles/r04/ab_r04c.md): ring 1.084 ms vs clip 0.924 ms per 2048-stream launch --
        // the ring kernel's cursors save little VALU and its tile enumeration costs SALU; opt-in only
        const char *uk = getenv("SLAM2D_UPD_KERNEL");
        c->upd_ring = uk && strcmp(uk, "ring") == 0;
        // workgroups per (stream, level) of hs_update_kernel: adaptive (launch_part: 1 at >= 512 streams,
        // where splitting measured neutral to slower), or fixed by SLAM2D_UPD_PARTS="p0,p1,..." 
        for (int l = 0; l < MAX_LEVELS; ++l) c->geom.upd_parts[l] = 1;
        c->ncu = ncu;
        if (const char *up = getenv("SLAM2D_UPD_PARTS")) {
            c->upd_parts_fixed = true;
            int l = 0;
            for (const char *q = up; *q && l < MAX_LEVELS; ++l) {
                const int v = atoi(q);
                c->geom.upd_parts[l] = v < 1 ? 1 : (v > 64 ? 64 : v);
                while (*q && *q != ',') ++q;
                if (*q == ',') ++q;
            }
            for (; l < MAX_LEVELS; ++l) c->geom.upd_parts[l] = c->geom.upd_parts[l - 1];
        }
        // list-driven split: minimum workgroups per level, SLAM2D_UPD_SPLIT="m0,m1,..." (default: upd_split's)
        for (int l = 0; l < MAX_LEVELS; ++l) c->geom.upd_minp[l] = 0;
        if (const char *us = getenv("SLAM2D_UPD_SPLIT")) {
            int l = 0;
            for (const char *q = us; *q && l < MAX_LEVELS; ++l) {
                const int v = atoi(q);
                c->geom.upd_minp[l] = v < 0 ? 0 : (v > 64 ? 64 : v);
                while (*q && *q != ',') ++q;
                if (*q == ',') ++q;
            }
        }
        if (c->nparts < 1) c->nparts = 1;
        if (c->nparts > MAX_PARTS) c->nparts = MAX_PARTS;
        c->nq = (c->pipeline && c->nparts < 2) ? 2 : c->nparts;
        // per-part capacities (test hooks SLAM2D_SEG_CAP / SLAM2D_ITEM_CAP set them directly)
        if (const char *e2 = getenv("SLAM2D_SEG_CAP")) c->seg_cap = (unsigned)atoll(e2);
        else c->seg_cap = (unsigned)((size_t)c->seg_cap / c->nq + (1u << 16));
        if (const char *e2 = getenv("SLAM2D_ITEM_CAP")) c->item_cap = (unsigned)atoll(e2);
        else c->item_cap = (unsigned)((size_t)c->item_cap / c->nq + (1u << 10));
        for (int p = 0; p < MAX_PARTS; ++p) {
            if ((e = hipStreamCreateWithFlags(&c->pstream[p], hipStreamDefault)) != hipSuccess ||
                (e = hipEventCreateWithFlags(&c->ev_done[p], hipEventDisableTiming)) != hipSuccess ||
                (e = hipEventCreateWithFlags(&c->ev_upd[p], hipEventDisableTiming)) != hipSuccess) {
                hs_destroy(c);
                return fail(HS_EHIP, "hipStreamCreate(part)", e);
            }
        }
        if ((e = hipEventCreateWithFlags(&c->ev_start, hipEventDisableTiming)) != hipSuccess ||
            (e = hipEventCreateWithFlags(&c->ev_last, hipEventDisableTiming)) != hipSuccess) {
            hs_destroy(c);
            return fail(HS_EHIP, "hipEventCreate", e);
        }
    }
    if ((e = hipMalloc(&c->d_rays, sizeof(unsigned) * (size_t)num_streams * levels * max_points)) != hipSuccess ||
        (e = hipMalloc(&c->d_segs, sizeof(uint4) * (size_t)c->seg_cap * c->nq)) != hipSuccess ||
        (e = hipMalloc(&c->d_items, sizeof(WorkItem) * (size_t)c->item_cap * c->nq)) != hipSuccess ||
        (e = hipMalloc(&c->d_wholes, sizeof(WorkItem) * (size_t)num_streams * levels * c->nq)) != hipSuccess ||
        (e = hipMalloc(&c->d_wq, sizeof(WorkQueue) * c->nq)) != hipSuccess) {
        hs_destroy(c);
        return fail(HS_ENOMEM, "hipMalloc", e);
    }
    for (int p = 0; p < MAX_PARTS; ++p)
        for (int i = 0; i < 2; ++i)
            if ((e = hipMalloc(&c->wl[p][i], sizeof(int) * (4 + (size_t)num_streams))) != hipSuccess) {
                hs_destroy(c);
                return fail(HS_ENOMEM, "hipMalloc(update list)", e);
            }
    {
        WorkQueue q;
        memset(&q, 0, sizeof(q));
        q.item_cap = c->item_cap;
        q.seg_cap = c->seg_cap;
        for (int p = 0; p < c->nq; ++p) {
            if ((e = hipMemcpy(c->d_wq + p, &q, sizeof(q), hipMemcpyHostToDevice)) != hipSuccess) {
                hs_destroy(c);
                return fail(HS_EHIP, "hipMemcpy(work queue)", e);
            }
        }
    }
    int rc = reset_all(c, true);
    if (rc != HS_OK) {
        hs_destroy(c);
        return rc;
    }
    *out = c;
    return HS_OK;
}

int hs_destroy(hs_ctx *c)
{
    if (!c) return HS_OK;
    hipDeviceSynchronize();  // device work of the context may be on any stream (*_device calls)
    hipFree(c->d_cells);
    hipFree(c->d_state);
    hipFree(c->d_pts1);
    hipFree(c->d_n1);
    hipFree(c->d_origo1);
    hipFree(c->d_hint1);
    hipFree(c->d_out_pose);
    hipFree(c->d_out_cov);
    hipFree(c->d_occ);
    hipFree(c->d_rays);
    hipFree(c->d_segs);
    hipFree(c->d_items);
    hipFree(c->d_wholes);
    hipFree(c->d_wq);
    for (int p = 0; p < MAX_PARTS; ++p)
        for (int i = 0; i < 2; ++i) hipFree(c->wl[p][i]);
    hipFree(c->d_cs);
    hipFree(c->d_ixy);
    hipFree(c->d_in);
    hipFree(c->d_iorigo);
    hipFree(c->d_ranges1);
    hipFree(c->d_clk);
    for (auto &p : c->ev_used) {
        hipEventDestroy(p.a);
        hipEventDestroy(p.b);
    }
    for (auto &p : c->ev_free) {
        hipEventDestroy(p.a);
        hipEventDestroy(p.b);
    }
    for (int p = 0; p < MAX_PARTS; ++p) {
        if (c->pstream[p]) hipStreamDestroy(c->pstream[p]);
        if (c->ev_done[p]) hipEventDestroy(c->ev_done[p]);
        if (c->ev_upd[p]) hipEventDestroy(c->ev_upd[p]);
    }
    if (c->ev_start) hipEventDestroy(c->ev_start);
    if (c->ev_last) hipEventDestroy(c->ev_last);
    if (c->stream) hipStreamDestroy(c->stream);
    delete c;
    return HS_OK;
}

int hs_reset(hs_ctx *c)
{
    if (!c) return fail(HS_EINVAL, "ctx is NULL");
    LOCK(c);
    HCHK(hipDeviceSynchronize());
    return reset_all(c, false);
}

int hs_set_update_factors(hs_ctx *c, float free_factor, float occupied_factor)
{
    if (!c) return fail(HS_EINVAL, "ctx is NULL");
    LOCK(c);
    c->geom.lf = prob_to_logodds(free_factor);
    c->geom.lo = prob_to_logodds(occupied_factor);
    return HS_OK;
}

int hs_set_map_update_thresholds(hs_ctx *c, float min_dist, float min_angle)
{
    if (!c) return fail(HS_EINVAL, "ctx is NULL");
    LOCK(c);
    c->geom.min_dist = min_dist;
    c->geom.min_ang = min_angle;
    return HS_OK;
}

int hs_get_scale_to_map(hs_ctx *c, float *scale_out)
{
    if (!c || !scale_out) return fail(HS_EINVAL, "NULL argument");
    *scale_out = c->geom.lv[0].scale;
    return HS_OK;
}

int hs_get_map_levels(hs_ctx *c, int *levels_out)
{
    if (!c || !levels_out) return fail(HS_EINVAL, "NULL argument");
    *levels_out = c->levels;
    return HS_OK;
}

int hs_get_map_info(hs_ctx *c, int level, int *size_x, int *size_y, float *cell_length, float *origin_xy)
{
    if (!c || level < 0 || level >= c->levels) return fail(HS_EINVAL, "bad level");
    const LevelGeom &L = c->geom.lv[level];
    if (size_x) *size_x = L.sx;
    if (size_y) *size_y = L.sy;
    if (cell_length) *cell_length = L.cell_len;
    if (origin_xy) {
        // getWorldCoords(0,0) (hector_slam.cc:167)
        origin_xy[0] = L.inv_t[0] + (L.inv_l[0] * 0.0f + L.inv_l[1] * 0.0f);
        origin_xy[1] = L.inv_t[1] + (L.inv_l[2] * 0.0f + L.inv_l[3] * 0.0f);
    }
    return HS_OK;
}

int hs_update(hs_ctx *c, int stream, const float *xy, int n, float ox, float oy, const float *hint,
              int map_without_matching, float pose_out[3], float cov_out[9], int *did_update_out)
{
    if (check_stream(c, stream) != HS_OK) return fail(HS_EINVAL, "bad ctx/stream");
    LOCK(c);
    int rc = dev_enter(c, c->stream);
    if (rc == HS_OK) rc = stage_scan(c, xy, n, ox, oy, hint);
    if (rc != HS_OK) return rc;
    rc = launch_step(c, stream, 1, c->d_pts1, c->max_points, c->d_n1, c->d_origo1, hint ? c->d_hint1 : nullptr,
                     map_without_matching ? MODE_NO_MATCH_FORCE : MODE_PROCESS, c->d_out_pose, c->d_out_cov, c->stream);
    if (rc == HS_OK) rc = dev_leave(c, c->stream);
    if (rc != HS_OK) return rc;
    StreamState st;
    HCHK(hipMemcpyAsync(&st, c->d_state + stream, sizeof(st), hipMemcpyDeviceToHost, c->stream));
    HCHK(hipStreamSynchronize(c->stream));
    if (pose_out) memcpy(pose_out, st.pose, sizeof(float) * 3);
    if (cov_out) memcpy(cov_out, st.cov, sizeof(float) * 9);
    if (did_update_out) *did_update_out = st.do_update;
    return HS_OK;
}

int hs_match(hs_ctx *c, int stream, const float *xy, int n, float ox, float oy, const float hint[3], float pose_out[3],
             float cov_out[9])
{
    if (check_stream(c, stream) != HS_OK || !hint) return fail(HS_EINVAL, "bad ctx/stream/hint");
    LOCK(c);
    int rc = dev_enter(c, c->stream);
    if (rc == HS_OK) rc = stage_scan(c, xy, n, ox, oy, hint);
    if (rc != HS_OK) return rc;
    rc = launch_step(c, stream, 1, c->d_pts1, c->max_points, c->d_n1, c->d_origo1, c->d_hint1, MODE_MATCH_ONLY,
                     c->d_out_pose, c->d_out_cov, c->stream);
    if (rc == HS_OK) rc = dev_leave(c, c->stream);
    if (rc != HS_OK) return rc;
    float p[3], cv[9];
    HCHK(hipMemcpyAsync(p, c->d_out_pose, sizeof(p), hipMemcpyDeviceToHost, c->stream));
    HCHK(hipMemcpyAsync(cv, c->d_out_cov, sizeof(cv), hipMemcpyDeviceToHost, c->stream));
    HCHK(hipStreamSynchronize(c->stream));
    if (pose_out) memcpy(pose_out, p, sizeof(p));
    if (cov_out) memcpy(cov_out, cv, sizeof(cv));
    return HS_OK;
}

int hs_update_by_scan(hs_ctx *c, int stream, const float *xy, int n, float ox, float oy, const float pose[3])
{
    if (check_stream(c, stream) != HS_OK || !pose) return fail(HS_EINVAL, "bad ctx/stream/pose");
    LOCK(c);
    int rc = dev_enter(c, c->stream);
    if (rc == HS_OK) rc = stage_scan(c, xy, n, ox, oy, pose);
    if (rc != HS_OK) return rc;
    rc = launch_step(c, stream, 1, c->d_pts1, c->max_points, c->d_n1, c->d_origo1, c->d_hint1, MODE_UPDATE_ONLY,
                     nullptr, nullptr, c->stream);
    if (rc == HS_OK) rc = dev_leave(c, c->stream);
    if (rc != HS_OK) return rc;
    HCHK(hipStreamSynchronize(c->stream));
    return HS_OK;
}

int hs_get_last_pose(hs_ctx *c, int stream, float pose_out[3], float cov_out[9])
{
    if (check_stream(c, stream) != HS_OK) return fail(HS_EINVAL, "bad ctx/stream");
    LOCK(c);
    if (dev_enter(c, c->stream) != HS_OK) return HS_EHIP;
    StreamState st;
    HCHK(hipMemcpyAsync(&st, c->d_state + stream, sizeof(st), hipMemcpyDeviceToHost, c->stream));
    HCHK(hipStreamSynchronize(c->stream));
    if (pose_out) memcpy(pose_out, st.pose, sizeof(float) * 3);
    if (cov_out) memcpy(cov_out, st.cov, sizeof(float) * 9);
    return HS_OK;
}

int hs_get_map(hs_ctx *c, int stream, int level, int8_t *occ_out, float *logodds_out, int32_t *upd_out,
               int *update_index_out)
{
    if (check_stream(c, stream) != HS_OK || level < 0 || level >= c->levels) return fail(HS_EINVAL, "bad stream/level");
    LOCK(c);
    if (dev_enter(c, c->stream) != HS_OK) return HS_EHIP;
    const LevelGeom &L = c->geom.lv[level];
    const size_t ncell = (size_t)L.sx * L.sy;
    const size_t nwords = (size_t)L.tiles_x * L.tiles_y * TILE_BLOCK_WORDS;
    const float *base = c->d_cells + (size_t)stream * c->geom.stream_words + L.word_offset;
    if (occ_out) {
        hipLaunchKernelGGL(hs_publish_kernel, dim3(1024), dim3(256), 0, c->stream, base, L, c->d_occ);
        HCHK(hipGetLastError());
        HCHK(hipMemcpyAsync(occ_out, c->d_occ, ncell, hipMemcpyDeviceToHost, c->stream));
    }
    std::vector<float> tmp;
    if (logodds_out || upd_out) {
        tmp.resize(nwords);
        HCHK(hipMemcpyAsync(tmp.data(), base, sizeof(float) * nwords, hipMemcpyDeviceToHost, c->stream));
    }
    StreamState st;
    HCHK(hipMemcpyAsync(&st, c->d_state + stream, sizeof(st), hipMemcpyDeviceToHost, c->stream));
    HCHK(hipStreamSynchronize(c->stream));
    if (upd_out && st.ord_overflow)
        return fail(HS_ESTATE, "stream's update ordinals overflowed 16 bits: more than 32000 map updates without the "
                               "library's ordinal sweep (replayed graph captures of *_device calls?); call "
                               "hs_flush_ordinals at least every 32000 steps; hs_reset clears the state");
    if (!tmp.empty()) {
        for (int y = 0; y < L.sy; ++y)
            for (int x = 0; x < L.sx; ++x) {
                const size_t w = cell_word(L, x, y), o = (size_t)y * L.sx + x;
                if (logodds_out) logodds_out[o] = tmp[w];
                if (upd_out) {
                    // the hot ordinal when set (hector_internal.h ORD_OFF), else the cold updateIndex
                    const size_t tb = w - (size_t)tile_cell(x % TILE, y % TILE_H);  // the tile block
                    const size_t ci = w - tb;
                    uint16_t h;
                    memcpy(&h, reinterpret_cast<const char *>(&tmp[tb + ORD_OFF]) + 2 * ci, sizeof(h));
                    if (h) upd_out[o] = ord_index(h, st.ord_epoch);
                    else memcpy(&upd_out[o], &tmp[tb + COLD_OFF + ci], sizeof(int32_t));
                }
            }
    }
    if (update_index_out) *update_index_out = st.map_updates - 1;
    return HS_OK;
}

int hs_set_map(hs_ctx *c, int stream, int level, const float *logodds, const int32_t *upd)
{
    if (check_stream(c, stream) != HS_OK || level < 0 || level >= c->levels || !logodds || !upd)
        return fail(HS_EINVAL, "bad arguments");
    LOCK(c);
    if (dev_enter(c, c->stream) != HS_OK) return HS_EHIP;
    const LevelGeom &L = c->geom.lv[level];
    const size_t nwords = (size_t)L.tiles_x * L.tiles_y * TILE_BLOCK_WORDS;
    float *base = c->d_cells + (size_t)stream * c->geom.stream_words + L.word_offset;
    std::vector<float> tmp(nwords);
    HCHK(hipMemcpyAsync(tmp.data(), base, sizeof(float) * nwords, hipMemcpyDeviceToHost, c->stream));
    HCHK(hipStreamSynchronize(c->stream));
    for (int y = 0; y < L.sy; ++y)
        for (int x = 0; x < L.sx; ++x) {
            const size_t w = cell_word(L, x, y), o = (size_t)y * L.sx + x;
            tmp[w] = logodds[o];
            const size_t tb = w - (size_t)tile_cell(x % TILE, y % TILE_H), ci = w - tb;
            memcpy(&tmp[tb + COLD_OFF + ci], &upd[o], sizeof(int32_t));   // the cold plane ...
            const uint16_t zero = 0;
            memcpy(reinterpret_cast<char *>(&tmp[tb + ORD_OFF]) + 2 * ci, &zero, sizeof(zero));  // ... in effect
        }
    HCHK(hipMemcpyAsync(base, tmp.data(), sizeof(float) * nwords, hipMemcpyHostToDevice, c->stream));
    HCHK(hipStreamSynchronize(c->stream));
    return HS_OK;
}

int hs_step_batch_device(hs_ctx *c, int stream_begin, int count, const float *d_xy, int xy_stride, const int *d_n,
                         const float *d_origo, const float *d_hints, void *hip_stream)
{
    if (!c || stream_begin < 0 || count < 0 || stream_begin + count > c->B || !d_xy || !d_n ||
        xy_stride < c->max_points)
        return fail(HS_EINVAL, "bad batch arguments (xy_stride must be >= max_points)");
    LOCK(c);
    hipStream_t s = hip_stream ? (hipStream_t)hip_stream : c->stream;
    int rc = dev_enter(c, s);
    if (rc == HS_OK)
        rc = launch_step(c, stream_begin, count, (const float2 *)d_xy, xy_stride, d_n, (const float2 *)d_origo, d_hints,
                         MODE_PROCESS, nullptr, nullptr, s);
    return rc == HS_OK ? dev_leave(c, s) : rc;
}

int hs_run_ranges_device(hs_ctx *c, int steps, const float *d_ranges, int range_stride, size_t step_stride,
                         void *hip_stream)
{
    if (!c || steps < 0 || (steps > 0 && !d_ranges)) return fail(HS_EINVAL, "bad run arguments");
    LOCK(c);
    if (!c->has_laser) return fail(HS_EINVAL, "hs_set_laser not called");
    if (range_stride < c->ingest.n || step_stride < (size_t)range_stride * c->B)
        return fail(HS_EINVAL, "range_stride < n_beams or step_stride < num_streams * range_stride");
    if (steps == 0) return HS_OK;
    hipStream_t s = hip_stream ? (hipStream_t)hip_stream : c->stream;
    int rc = dev_enter(c, s);
    if (rc != HS_OK) return rc;
    if (!pipeline_ok(c)) {  // default: the steps in order on s
        for (int k = 0; k < steps && rc == HS_OK; ++k)
            rc = launch_ranges_step(c, 0, c->B, d_ranges + (size_t)k * step_stride, range_stride, c->d_ixy, c->max_points,
                                    c->d_in, c->d_iorigo, nullptr, nullptr, nullptr, s);
        return rc == HS_OK ? dev_leave(c, s) : rc;
    }
    // Two halves of the fleet on part streams 0 / 1.  Per step and half: ingest, match, then the grid
    // update once the OTHER half's previous update has finished, so that the updates alternate and each
    // one runs beside the other half's match:  U_A(k) || M_B(k),  U_B(k) || M_A(k+1).  Streams are
    // independent, so the results equal the in-order steps bit for bit.
    const int h0 = (c->B + 1) / 2;
    const int beg[2] = {0, h0}, cnt[2] = {h0, c->B - h0};
    HCHK(hipEventRecord(c->ev_start, s));
    for (int h = 0; h < 2; ++h) HCHK(hipStreamWaitEvent(c->pstream[h], c->ev_start, 0));
    for (int k = 0; k < steps && rc == HS_OK; ++k) {
        const float *rk = d_ranges + (size_t)k * step_stride;
        if (c->ord_steps + 1 > c->ord_interval) {
            // an ordinal sweep is due: after both halves' previous updates, before either half's next step
            for (int h = 0; h < 2; ++h) {
                HCHK(hipEventRecord(c->ev_done[h], c->pstream[h]));
                HCHK(hipStreamWaitEvent(s, c->ev_done[h], 0));
            }
            if ((rc = ord_sweep_if_due(c, s)) != HS_OK) break;
            HCHK(hipEventRecord(c->ev_start, s));
            for (int h = 0; h < 2; ++h) HCHK(hipStreamWaitEvent(c->pstream[h], c->ev_start, 0));
        } else {
            ++c->ord_steps;
        }
        for (int h = 0; h < 2 && rc == HS_OK; ++h) {
            hipStream_t ps = c->pstream[h];
            float2 *xy = c->d_ixy + (size_t)beg[h] * c->max_points;
            rc = launch_ingest(c, cnt[h], rk + (size_t)beg[h] * range_stride, range_stride, xy, c->max_points,
                               c->d_in + beg[h], c->d_iorigo + beg[h], ps);
            if (rc != HS_OK) break;
            hipEvent_t wait = (h == 1 || k > 0) ? c->ev_upd[h ^ 1] : nullptr;
            rc = launch_part(c, h, beg[h], cnt[h], xy, c->max_points, c->d_in + beg[h], c->d_iorigo + beg[h], nullptr,
                             MODE_PROCESS, nullptr, nullptr, ps, wait);
            if (rc == HS_OK && hipEventRecord(c->ev_upd[h], ps) != hipSuccess) rc = fail(HS_EHIP, "hipEventRecord");
        }
    }
    for (int h = 0; h < 2; ++h) {
        HCHK(hipEventRecord(c->ev_done[h], c->pstream[h]));
        HCHK(hipStreamWaitEvent(s, c->ev_done[h], 0));
    }
    return rc == HS_OK ? dev_leave(c, s) : rc;
}

void hs_default_laser(hs_laser *L, int n_beams, float angle_min, float angle_increment)
{
    if (!L) return;
    memset(L, 0, sizeof(*L));
    L->n_beams = n_beams;
    L->angle_min = angle_min;
    L->angle_increment = angle_increment;
    L->range_min = 0.0f;
    L->range_cutoff = 30.0;                              // projectLaser(..., 30.0)  hector_slam.cc:193
    L->basis[0] = L->basis[4] = L->basis[8] = 1.0;
    L->sqr_laser_min_dist = (float)(0.2 * 0.2);          // hector_slam.cc:151-152
    L->sqr_laser_max_dist = (float)(30.0 * 30.0);        // :154-155
    L->use_max_scan_range = 20.0;                        // :129
    L->laser_z_min_value = -1.0f;                        // :157-158
    L->laser_z_max_value = 1.0f;                         // :160-161
}

int hs_set_laser(hs_ctx *c, const hs_laser *L, const double *unit_vectors)
{
    if (!c || !L) return fail(HS_EINVAL, "NULL argument");
    LOCK(c);
    if (L->n_beams < 0 || L->n_beams > c->max_points) return fail(HS_EINVAL, "n_beams must be in [0, max_points]");
    IngestGeom &g = c->ingest;
    g.n = L->n_beams;
    g.cutoff = L->range_cutoff;
    g.range_min = L->range_min;
    memcpy(g.tf, L->basis, sizeof(double) * 9);
    memcpy(g.tf + 9, L->origin, sizeof(double) * 3);
    g.sqr_min = L->sqr_laser_min_dist;
    g.sqr_max = L->sqr_laser_max_dist;
    g.use_max_sq = L->use_max_scan_range * L->use_max_scan_range;  // double product, hector_slam.cc:344
    g.z_min = L->laser_z_min_value;
    g.z_max = L->laser_z_max_value;
    g.scale = c->geom.lv[0].scale;                                 // getScaleToMap (level 0)
    g.origo = make_float2((float)L->origin[0] * g.scale, (float)L->origin[1] * g.scale);  // :329
    std::vector<double> cs((size_t)2 * (L->n_beams > 0 ? L->n_beams : 1));
    for (int i = 0; i < L->n_beams; ++i) {
        if (unit_vectors) {
            cs[2 * i] = unit_vectors[2 * i];
            cs[2 * i + 1] = unit_vectors[2 * i + 1];
        } else {  // laser_geometry getUnitVectors_: cos / sin(angle_min + (double)i * angle_increment)
            const double a = (double)L->angle_min + (double)i * (double)L->angle_increment;
            cs[2 * i] = cos(a);
            cs[2 * i + 1] = sin(a);
        }
    }
    hipError_t e;
    if (!c->d_cs) {
        if ((e = hipMalloc(&c->d_cs, sizeof(double2) * (size_t)c->max_points)) != hipSuccess ||
            (e = hipMalloc(&c->d_in, sizeof(int) * (size_t)c->B)) != hipSuccess ||
            (e = hipMalloc(&c->d_iorigo, sizeof(float2) * (size_t)c->B)) != hipSuccess ||
            (e = hipMalloc(&c->d_ranges1, sizeof(float) * (size_t)c->max_points)) != hipSuccess)
            return fail(HS_ENOMEM, "hipMalloc(ingest)", e);
    }
    if (dev_enter(c, c->stream) != HS_OK) return HS_EHIP;
    if (L->n_beams > 0)
        HCHK(hipMemcpyAsync(c->d_cs, cs.data(), sizeof(double2) * L->n_beams, hipMemcpyHostToDevice, c->stream));
    HCHK(hipStreamSynchronize(c->stream));
    c->has_laser = true;
    return HS_OK;
}

int hs_ingest_batch_device(hs_ctx *c, int count, const float *d_ranges, int range_stride, float *d_xy, int xy_stride,
                           int *d_n, float *d_origo, void *hip_stream)
{
    if (!c || count < 0 || (count > 0 && (!d_ranges || !d_xy || !d_n))) return fail(HS_EINVAL, "bad ingest arguments");
    LOCK(c);
    if (!c->has_laser) return fail(HS_EINVAL, "hs_set_laser not called");
    if (range_stride < c->ingest.n || xy_stride < c->ingest.n) return fail(HS_EINVAL, "stride < n_beams");
    if (count == 0) return HS_OK;
    hipStream_t s = hip_stream ? (hipStream_t)hip_stream : c->stream;
    int rc = dev_enter(c, s);
    if (rc == HS_OK) rc = launch_ingest(c, count, d_ranges, range_stride, (float2 *)d_xy, xy_stride, d_n, (float2 *)d_origo, s);
    return rc == HS_OK ? dev_leave(c, s) : rc;
}

int hs_step_ranges_batch_device(hs_ctx *c, int stream_begin, int count, const float *d_ranges, int range_stride,
                                const float *d_hints, void *hip_stream)
{
    if (!c || stream_begin < 0 || count < 0 || stream_begin + count > c->B) return fail(HS_EINVAL, "bad batch arguments");
    LOCK(c);
    if (!c->has_laser) return fail(HS_EINVAL, "hs_set_laser not called");
    if (count > 0 && !d_ranges) return fail(HS_EINVAL, "d_ranges is NULL");
    if (range_stride < c->ingest.n) return fail(HS_EINVAL, "range_stride < n_beams");
    if (count == 0) return HS_OK;
    hipStream_t s = hip_stream ? (hipStream_t)hip_stream : c->stream;
    int rc = dev_enter(c, s);
    if (rc == HS_OK)
        rc = launch_ranges_step(c, stream_begin, count, d_ranges, range_stride,
                                c->d_ixy + (size_t)stream_begin * c->max_points, c->max_points, c->d_in, c->d_iorigo,
                                d_hints, nullptr, nullptr, s);
    return rc == HS_OK ? dev_leave(c, s) : rc;
}

int hs_update_ranges(hs_ctx *c, int stream, const float *ranges, float pose_out[3], float cov_out[9], int *did_update_out)
{
    if (check_stream(c, stream) != HS_OK) return fail(HS_EINVAL, "bad ctx/stream");
    LOCK(c);
    if (!c->has_laser) return fail(HS_EINVAL, "hs_set_laser not called");
    if (c->ingest.n > 0 && !ranges) return fail(HS_EINVAL, "ranges is NULL");
    if (dev_enter(c, c->stream) != HS_OK) return HS_EHIP;
    if (c->ingest.n > 0)
        HCHK(hipMemcpyAsync(c->d_ranges1, ranges, sizeof(float) * c->ingest.n, hipMemcpyHostToDevice, c->stream));
    // scanCallback: startEstimate = getLastScanMatchPose() (hector_slam.cc:201), i.e. no explicit hint
    int rc = launch_ranges_step(c, stream, 1, c->d_ranges1, c->max_points, c->d_ixy + (size_t)stream * c->max_points,
                                c->max_points, c->d_n1, c->d_origo1, nullptr, c->d_out_pose, c->d_out_cov, c->stream);
    if (rc == HS_OK) rc = dev_leave(c, c->stream);
    if (rc != HS_OK) return rc;
    StreamState st;
    HCHK(hipMemcpyAsync(&st, c->d_state + stream, sizeof(st), hipMemcpyDeviceToHost, c->stream));
    HCHK(hipStreamSynchronize(c->stream));
    if (pose_out) memcpy(pose_out, st.pose, sizeof(float) * 3);
    if (cov_out) memcpy(cov_out, st.cov, sizeof(float) * 9);
    if (did_update_out) *did_update_out = st.do_update;
    return HS_OK;
}

int hs_get_poses(hs_ctx *c, float *poses_out, float *covs_out, int *did_update_out, int64_t *cells_out)
{
    if (!c) return fail(HS_EINVAL, "ctx is NULL");
    LOCK(c);
    std::vector<StreamState> h(c->B);
    HCHK(hipDeviceSynchronize());
    HCHK(hipMemcpy(h.data(), c->d_state, sizeof(StreamState) * c->B, hipMemcpyDeviceToHost));
    for (int s = 0; s < c->B; ++s) {
        if (poses_out) memcpy(poses_out + 3 * s, h[s].pose, sizeof(float) * 3);
        if (covs_out) memcpy(covs_out + 9 * s, h[s].cov, sizeof(float) * 9);
        if (did_update_out) did_update_out[s] = h[s].do_update;
        if (cells_out) cells_out[s] = (int64_t)(h[s].do_update ? h[s].step_cells : 0);
    }
    return HS_OK;
}

int hs_get_counters(hs_ctx *c, int64_t out[6], int reset)
{
    if (!c || !out) return fail(HS_EINVAL, "NULL argument");
    LOCK(c);
    std::vector<StreamState> h(c->B);
    HCHK(hipStreamSynchronize(c->stream));
    HCHK(hipDeviceSynchronize());
    HCHK(hipMemcpy(h.data(), c->d_state, sizeof(StreamState) * c->B, hipMemcpyDeviceToHost));
    for (int k = 0; k < 6; ++k) out[k] = 0;
    for (int s = 0; s < c->B; ++s) {
        out[0] += (int64_t)h[s].tot_cells;
        out[1] += (int64_t)h[s].tot_rays;
        out[2] += (int64_t)h[s].tot_gn_points;
        out[3] += (int64_t)h[s].tot_updates;
        out[4] += (int64_t)h[s].tot_steps;
        out[5] += (int64_t)h[s].tot_touched;
        if (reset) {
            h[s].tot_cells = h[s].tot_rays = h[s].tot_gn_points = h[s].tot_updates = h[s].tot_steps = 0;
            h[s].tot_touched = 0;
        }
    }
    if (reset) HCHK(hipMemcpy(c->d_state, h.data(), sizeof(StreamState) * c->B, hipMemcpyHostToDevice));
    return HS_OK;
}

int hs_get_queue_stats(hs_ctx *c, int64_t out[8], int reset_stamps)
{
    if (!c || !out) return fail(HS_EINVAL, "NULL argument");
    LOCK(c);
    WorkQueue q[MAX_PARTS];
    unsigned long long st[8];
    HCHK(hipDeviceSynchronize());
    HCHK(hipMemcpy(q, c->d_wq, sizeof(WorkQueue) * c->nq, hipMemcpyDeviceToHost));
    HCHK(hipMemcpyFromSymbol(st, HIP_SYMBOL(g_stamps), sizeof(st)));
    for (int k = 0; k < 4; ++k) out[k] = 0;
    for (int p = 0; p < c->nq; ++p) {
        out[0] += q[p].item_used;
        out[1] += q[p].seg_used;
        out[2] += q[p].whole_used;
        out[3] += q[p].overflow;
    }
    for (int k = 0; k < 4; ++k) out[4 + k] = (int64_t)st[k];
    if (reset_stamps) {
        memset(st, 0, sizeof(st));
        HCHK(hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), st, sizeof(st)));
    }
    return HS_OK;
}

int hs_get_diag_stamps(hs_ctx *c, int64_t out[8], int reset)
{
    if (!c || !out) return fail(HS_EINVAL, "bad arguments");
    LOCK(c);
    unsigned long long st[8];
    HCHK(hipDeviceSynchronize());
    HCHK(hipMemcpyFromSymbol(st, HIP_SYMBOL(g_stamps), sizeof(st)));
    for (int k = 0; k < 8; ++k) out[k] = (int64_t)st[k];
    if (reset) {
        memset(st, 0, sizeof(st));
        HCHK(hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), st, sizeof(st)));
    }
    return HS_OK;
}

int hs_flush_ordinals(hs_ctx *c, void *hip_stream)
{
    if (!c) return fail(HS_EINVAL, "ctx is NULL");
    LOCK(c);
    hipStream_t s = hip_stream ? (hipStream_t)hip_stream : c->stream;
    if (dev_enter(c, s) != HS_OK) return HS_EHIP;
    c->ord_steps = c->ord_interval;  // due now
    const int rc = ord_sweep_if_due(c, s);
    if (rc != HS_OK) return rc;
    c->ord_steps = 0;  // no step of the new epoch has run yet
    return dev_leave(c, s);
}

int hs_get_device_buffers(hs_ctx *c, void **cells, size_t *cells_bytes, size_t *stream_words)
{
    if (!c) return fail(HS_EINVAL, "ctx is NULL");
    if (cells) *cells = c->d_cells;
    if (cells_bytes) *cells_bytes = c->cells_bytes;
    if (stream_words) *stream_words = c->geom.stream_words;
    return HS_OK;
}

int hs_set_pose_log(hs_ctx *c, float *d_buf, int streams, int capacity)
{
    if (!c || streams < 0 || capacity < 0 || (d_buf && streams > c->B)) return fail(HS_EINVAL, "bad pose log");
    LOCK(c);
    c->plog.buf = d_buf;
    c->plog.streams = d_buf ? streams : 0;
    c->plog.capacity = d_buf ? capacity : 0;
    c->plog.slot_of = nullptr;
    return HS_OK;
}

int hs_set_pose_log_slots(hs_ctx *c, float *d_buf, const int *d_slot_of_stream, int slots, int capacity)
{
    if (!c || slots < 0 || capacity < 0 || (d_buf && !d_slot_of_stream)) return fail(HS_EINVAL, "bad pose log");
    LOCK(c);
    c->plog.buf = d_buf;
    c->plog.streams = d_buf ? slots : 0;
    c->plog.capacity = d_buf ? capacity : 0;
    c->plog.slot_of = d_buf ? d_slot_of_stream : nullptr;
    return HS_OK;
}

void *hs_get_stream(hs_ctx *c) { return c ? (void *)c->stream : nullptr; }

int hs_set_reduction_order(hs_ctx *c, int order)
{
    if (!c || (order != HS_ORDER_REFERENCE && order != HS_ORDER_TREE256)) return fail(HS_EINVAL, "bad reduction order");
    LOCK(c);
    c->reduce_order = order;
    return HS_OK;
}

int hs_get_reduction_order(hs_ctx *c, int *order_out)
{
    if (!c || !order_out) return fail(HS_EINVAL, "NULL argument");
    *order_out = c->reduce_order;
    return HS_OK;
}

int hs_set_timing(hs_ctx *c, int enable)
{
    if (!c) return fail(HS_EINVAL, "ctx is NULL");
    LOCK(c);
    c->timing = enable != 0;
    return HS_OK;
}

int hs_get_kernel_times(hs_ctx *c, double ms_out[3], int64_t launches_out[3], int reset)
{
    if (!c) return fail(HS_EINVAL, "ctx is NULL");
    LOCK(c);
    for (auto &p : c->ev_used) {
        HCHK(hipEventSynchronize(p.b));
        float ms = 0.0f;
        HCHK(hipEventElapsedTime(&ms, p.a, p.b));
        c->acc_ms[p.kernel] += ms;
        c->acc_n[p.kernel] += 1;
        c->ev_free.push_back(p);
    }
    c->ev_used.clear();
    for (int k = 0; k < NKERN; ++k) {
        if (ms_out) ms_out[k] = c->acc_ms[k];
        if (launches_out) launches_out[k] = c->acc_n[k];
        if (reset) {
            c->acc_ms[k] = 0.0;
            c->acc_n[k] = 0;
        }
    }
    return HS_OK;
}

int hs_set_clock_probe(hs_ctx *c, int enable)
{
    if (!c) return fail(HS_EINVAL, "ctx is NULL");
    LOCK(c);
    if (enable && !c->d_clk) {
        HCHK(hipMalloc(&c->d_clk, 8 * sizeof(unsigned long long)));
        HCHK(hipMemsetAsync(c->d_clk, 0, 8 * sizeof(unsigned long long), c->stream));
        HCHK(hipStreamSynchronize(c->stream));
    }
    c->geom.clk = enable ? c->d_clk : nullptr;
    return HS_OK;
}

int hs_get_clock_probe(hs_ctx *c, double out[6], int reset)
{
    if (!c || !out) return fail(HS_EINVAL, "NULL argument");
    LOCK(c);
    for (int k = 0; k < 6; ++k) out[k] = 0.0;
    if (!c->d_clk) return HS_OK;
    HCHK(hipDeviceSynchronize());  // the probed kernels may have run on any stream (*_device calls)
    unsigned long long h[8];
    HCHK(hipMemcpy(h, c->d_clk, sizeof(h), hipMemcpyDeviceToHost));
    for (int k = 0; k < 2; ++k) {
        out[3 * k] = (double)h[4 * k];
        out[3 * k + 1] = (double)h[4 * k + 1];
        out[3 * k + 2] = (double)h[4 * k + 2];
    }
    if (reset) HCHK(hipMemset(c->d_clk, 0, sizeof(h)));
    return HS_OK;
}

}  // extern "C"
