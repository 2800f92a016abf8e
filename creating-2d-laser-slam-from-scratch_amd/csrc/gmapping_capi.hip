// gmapping_capi.hip -- host runtime + extern "C" boundary (include/slam2d/gmapping.h) of the
// GMapping particle-map path.  Every compute step is gm_compute_kernel (gmapping_kernels.hip);
// without a usable HIP device gm_create fails with GM_ENODEV.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <math.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

#include "../../include/slam2d/gmapping.h"
#include "gmapping_kernels.hip"

using namespace s2d;

namespace {
thread_local std::string gm_err;

int gfail(int code, const char *what, hipError_t e = hipSuccess)
{
    gm_err = what;
    if (e != hipSuccess) {
        gm_err += ": ";
        gm_err += hipGetErrorString(e);
    }
    return code;
}

#define GCHK(expr)                                             \
    do {                                                       \
        hipError_t _e = (expr);                                \
        if (_e != hipSuccess) return gfail(GM_EHIP, #expr, _e); \
    } while (0)
}  // namespace

struct gm_ctx {
    int P = 0, max_beams = 0, n_beams = 0;
    // gm_compute_kernel workgroups per particle (SLAM2D_GM_PARTS): r02 sweep, 1024 particles:
    // 3: 1.24 M, 4: 1.25 M, 5: 1.25 M, 6: 1.25 M, 8: 1.23 M, 12: 1.14 M, 16: 1.11 M particle-scans/s
    int parts = 5;
    GmGeom geom{};
    unsigned *d_maps = nullptr;   // packed counts, tiled
    unsigned *d_rays = nullptr;   // per particle, per beam: packed end cell (gm_score_kernel -> gm_compute_kernel)
    float2 *d_hitxy = nullptr;    // per particle, per beam: (float) hit point
    int *d_stamps = nullptr;      // per particle, per tile
    GmHitCell *d_hits = nullptr;  // per particle, max_beams entries
    GmState *d_state = nullptr;
    double *d_cos = nullptr, *d_sin = nullptr;
    double *d_poses = nullptr;  // host-pointer staging
    float *d_ranges = nullptr;
    int8_t *d_occ = nullptr;
    hipStream_t stream = nullptr;
    bool timing = false;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> ev_used, ev_free;
    double acc_ms = 0;
    int64_t acc_n = 0;
};

namespace {
size_t gm_shmem(int n)
{
    return sizeof(unsigned) * (2 * (size_t)GM_LDS_WORDS + (size_t)((n + 3) & ~3)) + sizeof(int4) * (size_t)((n + 63) / 64);
}

int reset_state(gm_ctx *c)
{
    std::vector<GmState> h(c->P);
    for (auto &s : h) {
        memset(&s, 0, sizeof(s));
        s.tx0 = 1; s.ty0 = 1; s.tx1 = 0; s.ty1 = 0;  // empty box: a fresh map
    }
    GCHK(hipMemcpy(c->d_state, h.data(), sizeof(GmState) * c->P, hipMemcpyHostToDevice));
    GCHK(hipMemset(c->d_stamps, 0, sizeof(int) * (size_t)c->geom.ntiles * c->P));
    return GM_OK;
}

int launch(gm_ctx *c, int begin, int count, const double *d_poses, const float *d_ranges, int n, int32_t *d_scores,
           hipStream_t s)
{
    if (count <= 0) return GM_OK;
    std::pair<hipEvent_t, hipEvent_t> ev{};
    if (c->timing) {
        if (!c->ev_free.empty()) {
            ev = c->ev_free.back();
            c->ev_free.pop_back();
        } else {
            GCHK(hipEventCreate(&ev.first));
            GCHK(hipEventCreate(&ev.second));
        }
        GCHK(hipEventRecord(ev.first, s));
    }
    hipLaunchKernelGGL(gm_score_kernel, dim3(count), dim3(GM_THREADS), 0, s, c->geom, d_poses, d_ranges, n, c->d_cos,
                       c->d_sin, c->d_maps, c->d_stamps, c->d_state, d_scores, begin, c->d_rays, c->d_hitxy, c->d_hits);
    GCHK(hipGetLastError());
    hipLaunchKernelGGL(gm_compute_kernel, dim3(count * c->parts), dim3(GM_THREADS), gm_shmem(n), s, c->geom, d_poses,
                       n, c->d_rays, c->d_hitxy, c->d_maps, c->d_stamps, c->d_hits, c->d_state, begin, count, c->parts);
    GCHK(hipGetLastError());
    if (c->timing) {
        GCHK(hipEventRecord(ev.second, s));
        c->ev_used.push_back(ev);
    }
    return GM_OK;
}
}  // namespace

extern "C" {

const char *gm_version(void) { return "slam2d-mi355x gmapping 0.1 (gfx950)"; }
const char *gm_last_error(void) { return gm_err.c_str(); }

int gm_create(gm_ctx **out, int num_particles, int max_beams, double xmin, double ymin, double xmax, double ymax,
              double delta, double max_range, double max_urange)
{
    if (!out) return gfail(GM_EINVAL, "out is NULL");
    *out = nullptr;
    if (num_particles < 1 || max_beams < 1 || max_beams > 8192 || !(delta > 0) || !(xmax > xmin) || !(ymax > ymin))
        return gfail(GM_EINVAL, "invalid particles / beams / map bounds");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1) return gfail(GM_ENODEV, "no HIP device");
    gm_ctx *c = new gm_ctx;
    c->P = num_particles;
    c->max_beams = max_beams;
    if (const char *e2 = getenv("SLAM2D_GM_PARTS")) c->parts = atoi(e2) < 1 ? 1 : (atoi(e2) > 16 ? 16 : atoi(e2));
    GmGeom &g = c->geom;
    // ScanMatcherMap / HierarchicalArray2D geometry (G/grid/map.h:133-143, harray2d.h: 32-cell patches)
    g.cx = (xmin + xmax) / 2.0;
    g.cy = (ymin + ymax) / 2.0;
    g.sx = (((int)ceil((xmax - xmin) / delta)) >> 5) << 5;
    g.sy = (((int)ceil((ymax - ymin) / delta)) >> 5) << 5;
    g.sx2 = (int)round((g.cx - xmin) / delta);
    g.sy2 = (int)round((g.cy - ymin) / delta);
    g.delta = delta;
    g.max_range = max_range;
    g.max_urange = max_urange;
    g.occ_thresh = 0.25;  // gmapping.cc ctor default occ_thresh_
    g.max_beams = max_beams;
    if (g.sx < 32 || g.sy < 32 || g.sx > 16384 || g.sy > 16384 || !(max_range / delta < 16384.0)) {
        delete c;
        return gfail(GM_EINVAL, "map must be 32..16384 cells per side and max_range/delta < 16384");
    }
    g.tiles_x = (g.sx + GM_TILE - 1) / GM_TILE;
    g.tiles_y = (g.sy + GM_TILE_H - 1) / GM_TILE_H;
    g.particle_words = (size_t)g.tiles_x * g.tiles_y * GM_TILE_BLOCK_WORDS;
    g.ntiles = g.tiles_x * g.tiles_y;
    hipError_t e;
    if ((e = hipStreamCreateWithFlags(&c->stream, hipStreamDefault)) != hipSuccess) {
        delete c;
        return gfail(GM_EHIP, "hipStreamCreate", e);
    }
    if ((e = hipMalloc(&c->d_maps, sizeof(unsigned) * g.particle_words * (size_t)c->P)) != hipSuccess ||
        (e = hipMalloc(&c->d_stamps, sizeof(int) * (size_t)g.ntiles * c->P)) != hipSuccess ||
        (e = hipMalloc(&c->d_rays, sizeof(unsigned) * (size_t)max_beams * c->P)) != hipSuccess ||
        (e = hipMalloc(&c->d_hitxy, sizeof(float2) * (size_t)max_beams * c->P)) != hipSuccess ||
        (e = hipMalloc(&c->d_hits, sizeof(GmHitCell) * (size_t)max_beams * c->P)) != hipSuccess ||
        (e = hipMalloc(&c->d_state, sizeof(GmState) * c->P)) != hipSuccess ||
        (e = hipMalloc(&c->d_cos, sizeof(double) * max_beams)) != hipSuccess ||
        (e = hipMalloc(&c->d_sin, sizeof(double) * max_beams)) != hipSuccess ||
        (e = hipMalloc(&c->d_poses, sizeof(double) * 4 * c->P)) != hipSuccess ||
        (e = hipMalloc(&c->d_ranges, sizeof(float) * max_beams)) != hipSuccess ||
        (e = hipMalloc(&c->d_occ, (size_t)g.sx * g.sy)) != hipSuccess) {
        gm_destroy(c);
        return gfail(GM_ENOMEM, "hipMalloc", e);
    }
    int rc = reset_state(c);
    if (rc != GM_OK) {
        gm_destroy(c);
        return rc;
    }
    *out = c;
    return GM_OK;
}

int gm_destroy(gm_ctx *c)
{
    if (!c) return GM_OK;
    if (c->stream) hipStreamSynchronize(c->stream);
    hipFree(c->d_maps);
    hipFree(c->d_rays);
    hipFree(c->d_hitxy);
    hipFree(c->d_stamps);
    hipFree(c->d_hits);
    hipFree(c->d_state);
    hipFree(c->d_cos);
    hipFree(c->d_sin);
    hipFree(c->d_poses);
    hipFree(c->d_ranges);
    hipFree(c->d_occ);
    for (auto &p : c->ev_used) { hipEventDestroy(p.first); hipEventDestroy(p.second); }
    for (auto &p : c->ev_free) { hipEventDestroy(p.first); hipEventDestroy(p.second); }
    if (c->stream) hipStreamDestroy(c->stream);
    delete c;
    return GM_OK;
}

int gm_reset(gm_ctx *c)
{
    if (!c) return gfail(GM_EINVAL, "ctx is NULL");
    GCHK(hipStreamSynchronize(c->stream));
    GCHK(hipDeviceSynchronize());
    return reset_state(c);
}

int gm_set_beams(gm_ctx *c, const double *a_cos, const double *a_sin, int n)
{
    if (!c || !a_cos || !a_sin || n < 1 || n > c->max_beams) return gfail(GM_EINVAL, "invalid beam cache");
    GCHK(hipMemcpy(c->d_cos, a_cos, sizeof(double) * n, hipMemcpyHostToDevice));
    GCHK(hipMemcpy(c->d_sin, a_sin, sizeof(double) * n, hipMemcpyHostToDevice));
    c->n_beams = n;
    return GM_OK;
}

int gm_set_occ_thresh(gm_ctx *c, double t)
{
    if (!c) return gfail(GM_EINVAL, "ctx is NULL");
    c->geom.occ_thresh = t;
    return GM_OK;
}

int gm_get_map_size(gm_ctx *c, int *sx, int *sy)
{
    if (!c) return gfail(GM_EINVAL, "ctx is NULL");
    if (sx) *sx = c->geom.sx;
    if (sy) *sy = c->geom.sy;
    return GM_OK;
}

int gm_compute_maps(gm_ctx *c, const double *poses, const float *ranges, int n)
{
    if (!c || !poses || (!ranges && n > 0)) return gfail(GM_EINVAL, "NULL argument");
    if (n < 0 || n > c->n_beams) return gfail(GM_EINVAL, "n exceeds the beam cache (gm_set_beams)");
    GCHK(hipMemcpyAsync(c->d_poses, poses, sizeof(double) * 4 * c->P, hipMemcpyHostToDevice, c->stream));
    if (n > 0) GCHK(hipMemcpyAsync(c->d_ranges, ranges, sizeof(float) * n, hipMemcpyHostToDevice, c->stream));
    int rc = launch(c, 0, c->P, c->d_poses, c->d_ranges, n, nullptr, c->stream);
    if (rc != GM_OK) return rc;
    GCHK(hipStreamSynchronize(c->stream));
    return GM_OK;
}

int gm_compute_maps_device(gm_ctx *c, int begin, int count, const double *d_poses, const float *d_ranges, int n,
                           int32_t *d_scores_out, void *hip_stream)
{
    if (!c || !d_poses || (!d_ranges && n > 0)) return gfail(GM_EINVAL, "NULL argument");
    if (begin < 0 || count < 0 || begin + count > c->P) return gfail(GM_EINVAL, "particle range out of bounds");
    if (n < 0 || n > c->n_beams) return gfail(GM_EINVAL, "n exceeds the beam cache (gm_set_beams)");
    hipStream_t s = hip_stream ? (hipStream_t)hip_stream : c->stream;
    return launch(c, begin, count, d_poses, d_ranges, n, d_scores_out, s);
}

int gm_normalize_weights_device(gm_ctx *c, void *nccl_comm, const int32_t *d_scores, int count, double *d_weights_out,
                                double *d_sums_out, void *hip_stream)
{
    if (!c || !d_sums_out || (count > 0 && !d_scores)) return gfail(GM_EINVAL, "NULL argument");
    if (count < 0) return gfail(GM_EINVAL, "count < 0");
    hipStream_t s = hip_stream ? (hipStream_t)hip_stream : c->stream;
    hipLaunchKernelGGL(gm_weight_sums_kernel, dim3(1), dim3(GM_THREADS), 0, s, d_scores, count, d_sums_out);
    GCHK(hipGetLastError());
    if (nccl_comm) {
        // the one exchange of the sharded particle set: 2 doubles, summed over the ranks (RCCL over xGMI)
        const ncclResult_t r = ncclAllReduce(d_sums_out, d_sums_out, 2, ncclDouble, ncclSum, (ncclComm_t)nccl_comm, s);
        if (r != ncclSuccess) {
            gm_err = std::string("ncclAllReduce: ") + ncclGetErrorString(r);
            return GM_EHIP;
        }
    }
    if (d_weights_out && count > 0) {
        hipLaunchKernelGGL(gm_weights_kernel, dim3((count + 255) / 256), dim3(256), 0, s, d_scores, count, d_sums_out,
                           d_weights_out);
        GCHK(hipGetLastError());
    }
    return GM_OK;
}

int gm_get_particle_map(gm_ctx *c, int p, int32_t *n_out, int32_t *visits_out, float *acc_out)
{
    if (!c || p < 0 || p >= c->P) return gfail(GM_EINVAL, "invalid particle");
    GCHK(hipDeviceSynchronize());
    const GmGeom &g = c->geom;
    GmState st;
    GCHK(hipMemcpy(&st, c->d_state + p, sizeof(GmState), hipMemcpyDeviceToHost));
    const size_t cells = (size_t)g.sx * g.sy;
    if (n_out) memset(n_out, 0, sizeof(int32_t) * cells);
    if (visits_out) memset(visits_out, 0, sizeof(int32_t) * cells);
    if (acc_out) memset(acc_out, 0, sizeof(float) * 2 * cells);
    if (st.step == 0 || st.tx1 < st.tx0) return GM_OK;
    std::vector<int> stamps(g.ntiles);
    GCHK(hipMemcpy(stamps.data(), c->d_stamps + (size_t)p * g.ntiles, sizeof(int) * g.ntiles, hipMemcpyDeviceToHost));
    std::vector<unsigned> tile(GM_TILE_BLOCK_WORDS);
    const unsigned *pm = c->d_maps + (size_t)p * g.particle_words;
    for (int ty = st.ty0; ty <= st.ty1; ++ty)
        for (int tx = st.tx0; tx <= st.tx1; ++tx) {
            if (stamps[ty * g.tiles_x + tx] != st.step) continue;  // not written this step: fresh
            GCHK(hipMemcpy(tile.data(), pm + (size_t)(ty * g.tiles_x + tx) * GM_TILE_BLOCK_WORDS,
                           sizeof(unsigned) * GM_TILE_BLOCK_WORDS, hipMemcpyDeviceToHost));
            for (int r = 0; r < GM_TILE_H; ++r) {
                const int y = ty * GM_TILE_H + r;
                if (y >= g.sy) break;
                for (int k = 0; k < GM_TILE; ++k) {
                    const int x = tx * GM_TILE + k;
                    if (x >= g.sx) break;
                    const size_t o = (size_t)y * g.sx + x;
                    const unsigned cv = tile[r * GM_TILE + k];
                    if (visits_out) visits_out[o] = (int32_t)(cv & 0xFFFFu);
                    if (n_out) n_out[o] = (int32_t)(cv >> 16);
                }
            }
        }
    if (acc_out && st.hit_cells > 0) {
        std::vector<GmHitCell> hits(st.hit_cells);
        GCHK(hipMemcpy(hits.data(), c->d_hits + (size_t)p * c->max_beams, sizeof(GmHitCell) * st.hit_cells,
                       hipMemcpyDeviceToHost));
        for (const auto &h : hits) {
            if (h.cell < 0) continue;  // a beam that is not its cell's first hit (or no hit)
            acc_out[2 * (size_t)h.cell] = h.ax;
            acc_out[2 * (size_t)h.cell + 1] = h.ay;
        }
    }
    return GM_OK;
}

int gm_publish(gm_ctx *c, int p, int8_t *occ_out)
{
    if (!c || !occ_out || p < 0 || p >= c->P) return gfail(GM_EINVAL, "invalid argument");
    GCHK(hipDeviceSynchronize());
    GmState st;
    GCHK(hipMemcpy(&st, c->d_state + p, sizeof(GmState), hipMemcpyDeviceToHost));
    hipLaunchKernelGGL(gm_publish_kernel, dim3(1024), dim3(256), 0, c->stream, c->d_maps + (size_t)p * c->geom.particle_words,
                       c->d_stamps + (size_t)p * c->geom.ntiles, c->geom, st.step, c->d_occ);
    GCHK(hipGetLastError());
    GCHK(hipMemcpyAsync(occ_out, c->d_occ, (size_t)c->geom.sx * c->geom.sy, hipMemcpyDeviceToHost, c->stream));
    GCHK(hipStreamSynchronize(c->stream));
    return GM_OK;
}

int gm_get_scores(gm_ctx *c, int32_t *scores_out, int32_t *hits_out, int64_t *free_out)
{
    if (!c) return gfail(GM_EINVAL, "ctx is NULL");
    GCHK(hipDeviceSynchronize());
    std::vector<GmState> h(c->P);
    GCHK(hipMemcpy(h.data(), c->d_state, sizeof(GmState) * c->P, hipMemcpyDeviceToHost));
    for (int p = 0; p < c->P; ++p) {
        if (scores_out) scores_out[p] = h[p].score;
        if (hits_out) hits_out[p] = h[p].hits;
        if (free_out) free_out[p] = h[p].free_updates;
    }
    return GM_OK;
}

int gm_set_timing(gm_ctx *c, int enable)
{
    if (!c) return gfail(GM_EINVAL, "ctx is NULL");
    c->timing = enable != 0;
    return GM_OK;
}

int gm_get_kernel_times(gm_ctx *c, double *ms_out, int64_t *launches_out, int reset)
{
    if (!c) return gfail(GM_EINVAL, "ctx is NULL");
    GCHK(hipDeviceSynchronize());
    for (auto &p : c->ev_used) {
        float ms = 0;
        GCHK(hipEventElapsedTime(&ms, p.first, p.second));
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
    return GM_OK;
}

}  // extern "C"
