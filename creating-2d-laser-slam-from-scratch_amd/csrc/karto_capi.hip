// karto_capi.hip -- host runtime + extern "C" boundary (include/slam2d/karto.h) of the Karto
// correlative scan-matcher path.  Every compute step runs in karto_kernels.hip; without a usable HIP
// device kt_create fails with KT_ENODEV (no CPU fallback).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "karto_kernels.hip"

using namespace s2d;

namespace {
thread_local std::string kt_err;

int kfail(int code, const char *what, hipError_t e = hipSuccess)
{
    kt_err = what;
    if (e != hipSuccess) {
        kt_err += ": ";
        kt_err += hipGetErrorString(e);
    }
    return code;
}

#define KCHK(expr)                                              \
    do {                                                        \
        hipError_t _e = (expr);                                 \
        if (_e != hipSuccess) return kfail(KT_EHIP, #expr, _e); \
    } while (0)

double h_round(double v) { return v >= 0.0 ? std::floor(v + 0.5) : std::ceil(v - 0.5); }  // math::Round
int align8(int v) { return (v + 7) & ~7; }
size_t align256(size_t v) { return (v + 255) & ~(size_t)255; }

enum { K_PREPARE, K_BEGIN, K_BUILD, K_COARSE, K_SELECT, K_FINE, K_CLEAR, K_NUM };
const char *const k_names[K_NUM] = {"kt_prepare_kernel", "kt_begin_kernel", "kt_build_kernel", "kt_coarse_kernel",
                                    "kt_select_kernel",  "kt_fine_kernel",  "kt_build_kernel<1> (clear)"};
}  // namespace

struct kt_ctx {
    kt_laser laser{};
    kt_params params{};
    KtGeom g{};
    int max_matches = 0, max_scans = 0, max_base = 0;
    int slots = 0;  // match slots resident at once (kt_run_batch chunk)
    bool sharded_binned = false;  // AddScans variant of the last kt_match_sharded_begin_device
    int build_per_match = 1;  // CAS AddScans: one workgroup per match (1) or per (match, base scan) (0)
    int binned = 0;           // AddScans by kt_addscans_kernel (tile-binned, plain stores)
    int *d_scratch = nullptr, *d_dirty = nullptr, *d_dirty_cnt = nullptr;
    double *d_ranges = nullptr, *d_poses = nullptr;
    int *d_npts = nullptr;
    double2 *d_pts = nullptr, *d_loc = nullptr;
    unsigned char *d_bad = nullptr;
    int2 *d_evt = nullptr;
    unsigned char *d_grids = nullptr, *d_kernel = nullptr;
    KtState *d_state = nullptr;
    double *d_resp = nullptr;
    unsigned long long *d_posmax = nullptr;
    int *d_tie_idx = nullptr;
    double4 *d_tie_val = nullptr;
    int *d_query = nullptr, *d_bbeg = nullptr, *d_bidx = nullptr;
    kt_result *d_res = nullptr;
    hipStream_t stream = nullptr;
    bool timing = false;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> ev_free;
    std::vector<std::pair<int, std::pair<hipEvent_t, hipEvent_t>>> ev_used;
    double acc_ms[K_NUM] = {};
    int64_t acc_n[K_NUM] = {};

    KtPool pool() const { return KtPool{d_ranges, d_poses, d_npts, d_pts, d_loc, d_bad, d_evt}; }
};

namespace {

// ScanMatcher::Create + CorrelationGrid::CreateGrid / CalculateKernel + CorrelateScan's search spaces,
// evaluated exactly as oracle/karto_oracle.c (ko_geom_init) does.
int kt_geometry(const kt_laser &L, const kt_params &p, KtGeom &g, std::vector<unsigned char> &kernel)
{
    g = KtGeom{};
    if (!(p.resolution > 0) || !(p.search_size > 0) || p.smear_deviation < 0 || !(L.range_threshold > 0))
        return kfail(KT_EINVAL, "ScanMatcher::Create rejects these parameters (resolution, searchSize, smear, rangeThreshold)");
    if (L.n_readings < 1 || L.n_readings > KT_MAX_READINGS) return kfail(KT_EINVAL, "n_readings must be in [1, 4096]");
    if (!(p.coarse_angle_resolution > 0) || !(p.fine_search_angle_offset > 0) || !(p.coarse_search_angle_offset > 0))
        return kfail(KT_EINVAL, "angle offsets / resolutions must be > 0");
    g.side = (int)(uint32_t)(h_round(p.search_size / p.resolution) + 1);
    const int margin = (int)(uint32_t)std::ceil(L.range_threshold / p.resolution);
    g.grid_size = g.side + 2 * margin;
    g.border = (int)h_round(2.0 * p.smear_deviation / p.resolution) + 1;
    g.width = g.grid_size + 2 * g.border;
    g.height = g.width;
    g.ws = align8(g.width);
    if ((double)g.ws * g.height > 2.0e9) return kfail(KT_EINVAL, "correlation grid larger than 2^31 cells");
    g.data_size = g.ws * g.height;
    g.probs_ws = align8(g.side);
    g.scale = 1.0 / p.resolution;
    g.res = 1.0 / g.scale;
    if (!(p.smear_deviation >= 0.5 * g.res && p.smear_deviation <= 10 * g.res))
        return kfail(KT_EINVAL, "smear deviation must be between 0.5 and 10 resolutions (CalculateKernel)");
    g.half = (int)h_round(2.0 * p.smear_deviation / g.res);
    g.ksize = 2 * g.half + 1;
    if (g.ksize > 41) return kfail(KT_EINVAL, "smear kernel wider than 41 cells");
    kernel.assign((size_t)g.ksize * g.ksize, 0);
    for (int i = -g.half; i <= g.half; i++)
        for (int j = -g.half; j <= g.half; j++) {
            const double d = std::hypot(i * g.res, j * g.res);
            const double z = std::exp(-0.5 * std::pow(d / p.smear_deviation, 2));
            const uint32_t kv = (uint32_t)h_round(z * KT_OCC);
            kernel[(i + g.half) + g.ksize * (j + g.half)] = (unsigned char)kv;
            if ((i != 0 || j != 0) && kv >= (uint32_t)KT_OCC)
                return kfail(KT_EINVAL, "smear kernel has an off-centre value of 100 (smear_deviation too close to "
                                        "10 * resolution): AddScan would become order-dependent; not supported");
        }
    g.n = L.n_readings;
    g.coff = 0.5 * ((double)g.side - 1) * g.res;
    g.cres = 2 * g.res;
    g.nxy = (int)(uint32_t)(h_round(g.coff * 2.0 / g.cres) + 1);
    {
        // coarse tile shape: 16 x 16 positions.  SLAM2D_KT_TW = 32 / 64 makes it 32 x 8 / 64 x 4 (a wave's
        // gather then touches 8 / 4 grid rows of 64 / 128 bytes instead of 16 rows of 32 bytes): measured
        // slower (loop window 22.3 k -> 20.1 k / 20.8 k matches/s, sequential batch 321 k -> 269 k), so the
        // coarse kernel is not bound by L2 line requests per gather instruction
        int tw = 16;
        if (const char *e = getenv("SLAM2D_KT_TW")) tw = atoi(e);
        g.clw = tw >= 64 ? 4 : (tw >= 32 ? 3 : 2);
        tw = 4 << g.clw;
        g.ctx = (g.nxy + tw - 1) / tw;
        g.cty = (g.nxy + (256 / tw) - 1) / (256 / tw);
    }
    if (g.nxy > KT_MAX_NXY) return kfail(KT_EINVAL, "coarse search wider than 1024 positions");
    g.use_expansion = p.use_response_expansion ? 1 : 0;
    g.npass = g.use_expansion ? 4 : 1;
    g.cares = p.coarse_angle_resolution;
    double aoff = p.coarse_search_angle_offset;
    for (int i = 0; i < 4; ++i) {
        if (i > 0) aoff += 20 * 0.01745329251994329577;  // DegreesToRadians(20)
        g.aoff[i] = aoff;
        g.nang[i] = (int)(uint32_t)(h_round(aoff * 2.0 / g.cares) + 1);
    }
    g.foff = g.cres * 0.5;
    g.fn = (int)(uint32_t)(h_round(g.foff * 2.0 / g.res) + 1);
    g.faoff = 0.5 * p.coarse_angle_resolution;
    g.fares = p.fine_search_angle_offset;
    g.fnang = (int)(uint32_t)(h_round(g.faoff * 2.0 / g.fares) + 1);
    if (g.fn != 3) return kfail(KT_EINVAL, "fine search must be 3x3 positions");
    if (g.fnang > KT_FINE_MAX_ANG) return kfail(KT_EINVAL, "fine search has more than 64 angles");
    if (g.nang[g.npass - 1] > 4096) return kfail(KT_EINVAL, "coarse search has more than 4096 angles");
    g.min_angle = L.minimum_angle;
    g.ang_res = L.angular_resolution;
    g.min_range = L.minimum_range;
    g.range_thr = L.range_threshold;
    g.dvp = p.distance_variance_penalty;
    g.avp = p.angle_variance_penalty;
    g.mdp = p.minimum_distance_penalty;
    g.map_ = p.minimum_angle_penalty;
    const double mp = (double)g.nxy * g.nxy * g.nang[g.npass - 1];
    if (mp > 2.0e8) return kfail(KT_EINVAL, "coarse search window larger than 2e8 poses");
    g.max_poses = (int)mp;
    g.grid_stride = align256((size_t)g.data_size + 64);
    g.tiles_x = (g.ws + 63) / 64;
    g.tiles_y = (g.height + 63) / 64;
    g.ntiles = g.tiles_x * g.tiles_y;
    return KT_OK;
}

int kt_begin_event(kt_ctx *c, hipStream_t s, std::pair<hipEvent_t, hipEvent_t> &ev)
{
    if (!c->timing) return KT_OK;
    if (!c->ev_free.empty()) {
        ev = c->ev_free.back();
        c->ev_free.pop_back();
    } else {
        KCHK(hipEventCreate(&ev.first));
        KCHK(hipEventCreate(&ev.second));
    }
    KCHK(hipEventRecord(ev.first, s));
    return KT_OK;
}

int kt_end_event(kt_ctx *c, hipStream_t s, int which, std::pair<hipEvent_t, hipEvent_t> &ev)
{
    KCHK(hipGetLastError());
    if (!c->timing) return KT_OK;
    KCHK(hipEventRecord(ev.second, s));
    c->ev_used.push_back({which, ev});
    return KT_OK;
}

#define KT_LAUNCH(which, ...)                                  \
    do {                                                       \
        std::pair<hipEvent_t, hipEvent_t> _ev{};               \
        int _rc = kt_begin_event(c, s, _ev);                   \
        if (_rc != KT_OK) return _rc;                          \
        hipLaunchKernelGGL(__VA_ARGS__);                       \
        _rc = kt_end_event(c, s, which, _ev);                  \
        if (_rc != KT_OK) return _rc;                          \
    } while (0)

int kt_prepare(kt_ctx *c, int first, int count, hipStream_t s)
{
    const size_t shm = (size_t)c->g.n * (sizeof(double2) + 2 * sizeof(int));
    KT_LAUNCH(K_PREPARE, kt_prepare_kernel, dim3(count), dim3(KT_THREADS), shm, s, c->g, c->pool(), first);
    return KT_OK;
}

// MatchScan steps 1-5 for a chunk: centre the grids (kt_begin_kernel) and AddScans
int kt_chunk_build(kt_ctx *c, int count, const int *d_query, const int *d_bbeg, const int *d_bidx, hipStream_t s,
                   bool &binned)
{
    const KtGeom &g = c->g;
    const int groups = (count + 7) / 8;
    KT_LAUNCH(K_BEGIN, kt_begin_kernel, dim3(count), dim3(KT_THREADS), 0, s, g, c->pool(), d_query, c->d_state,
              c->d_posmax);
    // the binned AddScans runs one workgroup per match: small batches use the per-(match, base scan) kernel
    binned = c->binned && count >= 128;
    const bool per_match = !binned && c->build_per_match && count >= 128;
    if (c->max_base > 0) {
        if (binned)
            KT_LAUNCH(K_BUILD, kt_addscans_kernel, dim3(count), dim3(KT_AS_WAVES * 64), 0, s, g, c->pool(), c->d_state,
                      d_bbeg, d_bidx, c->d_kernel, c->d_grids, c->d_scratch, (size_t)c->max_base * g.n, c->d_dirty,
                      c->d_dirty_cnt);
        else if (per_match)
            KT_LAUNCH(K_BUILD, (kt_build_kernel<0, 8>), dim3(count), dim3(512), 0, s, g, c->pool(), c->d_state, d_bbeg,
                      d_bidx, c->d_kernel, c->d_grids, count, c->max_base);
        else
            KT_LAUNCH(K_BUILD, (kt_build_kernel<0, 4>), dim3(groups * 8 * c->max_base), dim3(KT_THREADS), 0, s, g,
                      c->pool(), c->d_state, d_bbeg, d_bidx, c->d_kernel, c->d_grids, count, c->max_base);
    }
    return KT_OK;
}

int kt_chunk_coarse(kt_ctx *c, int count, int pass, int penalize, int shard, int nshards, hipStream_t s)
{
    const KtGeom &g = c->g;
    // angles per workgroup: 1 (r02 A/B, loop window / sequential batch: 7 angles 5 % / 3 angles 5 % slower,
    // 21 angles 29 % slower -- fewer workgroups left in flight for the gathers); SLAM2D_KT_AG overrides
    const long long per_angle = (long long)((count + 7) / 8) * 8 * g.ctx * g.cty;
    const int nA = g.nang[pass];
    long long ag = 1;
    if (const char *e = getenv("SLAM2D_KT_AG")) ag = atoll(e);
    ag = ag < 1 ? 1 : (ag > nA ? nA : ag);
    const long long blocks = per_angle * ((nA + ag - 1) / ag);
    if (blocks > 0x7fffffffLL) return kfail(KT_EINVAL, "coarse launch too large: lower the batch size");
    KT_LAUNCH(K_COARSE, kt_coarse_kernel, dim3((unsigned)blocks), dim3(KT_THREADS), (size_t)g.n * sizeof(int), s, g,
              c->pool(), c->d_state, c->d_grids, c->d_resp, c->d_posmax, count, pass, penalize, shard, nshards,
              (int)ag);
    return KT_OK;
}

// the fine match (MatchScan step 7) and the grids' footprint clear
int kt_chunk_finish(kt_ctx *c, int count, const int *d_bbeg, const int *d_bidx, int penalize, int refine,
                    kt_result *d_res, hipStream_t s, bool binned)
{
    const KtGeom &g = c->g;
    const int groups = (count + 7) / 8;
    if (refine)
        KT_LAUNCH(K_FINE, kt_fine_kernel, dim3(count), dim3(KT_FINE_THREADS), 0, s, g, c->pool(), c->d_state, c->d_grids,
                  penalize, d_res);
    if (c->max_base > 0 && binned)
        KT_LAUNCH(K_CLEAR, kt_clear_tiles_kernel, dim3(count, 4), dim3(KT_THREADS), 0, s, g, c->d_grids, c->d_dirty,
                  c->d_dirty_cnt);
    else if (c->max_base > 0)
        KT_LAUNCH(K_CLEAR, (kt_build_kernel<1, 4>), dim3(groups * 8 * c->max_base), dim3(KT_THREADS), 0, s, g,
                  c->pool(), c->d_state, d_bbeg, d_bidx, c->d_kernel, c->d_grids, count, c->max_base);
    return KT_OK;
}

int kt_run_chunk(kt_ctx *c, int count, const int *d_query, const int *d_bbeg, const int *d_bidx, int penalize,
                 int refine, kt_result *d_res, hipStream_t s)
{
    bool binned = false;
    int rc = kt_chunk_build(c, count, d_query, d_bbeg, d_bidx, s, binned);
    if (rc != KT_OK) return rc;
    for (int pass = 0; pass < c->g.npass; ++pass) {
        if ((rc = kt_chunk_coarse(c, count, pass, penalize, 0, 1, s)) != KT_OK) return rc;
        if (c->g.nxy * c->g.nxy > 512)
            KT_LAUNCH(K_SELECT, kt_select_kernel<1024>, dim3(count), dim3(1024), 0, s, c->g, c->d_state, c->d_resp,
                  c->d_posmax, c->d_tie_idx, c->d_tie_val, pass, refine, d_res);
        else
            KT_LAUNCH(K_SELECT, kt_select_kernel<KT_THREADS>, dim3(count), dim3(KT_THREADS), 0, s, c->g, c->d_state, c->d_resp,
                  c->d_posmax, c->d_tie_idx, c->d_tie_val, pass, refine, d_res);
    }
    return kt_chunk_finish(c, count, d_bbeg, d_bidx, penalize, refine, d_res, s, binned);
}

// The batch runs in chunks of `slots` matches (default: all of them).  Smaller chunks keep a chunk's
// grids cache-resident but were measured slower (the per-match select / fine workgroups are latency
// bound and need the whole batch to fill the GPU); SLAM2D_KT_SLOTS caps the slot memory.
int kt_run_batch(kt_ctx *c, int count, const int *d_query, const int *d_bbeg, const int *d_bidx, int penalize,
                 int refine, kt_result *d_res, hipStream_t s)
{
    for (int c0 = 0; c0 < count; c0 += c->slots) {
        const int cnt = std::min(c->slots, count - c0);
        const int rc = kt_run_chunk(c, cnt, d_query + c0, d_bbeg + c0, d_bidx, penalize, refine, d_res + c0, s);
        if (rc != KT_OK) return rc;
    }
    return KT_OK;
}

}  // namespace

extern "C" {

const char *kt_version(void) { return "slam2d-mi355x karto 0.1 (gfx950)"; }
const char *kt_last_error(void) { return kt_err.c_str(); }

void kt_default_params(kt_params *p)
{
    if (!p) return;
    // Mapper::InitializeParameters (lesson6/lib/open_karto/src/Mapper.cpp:1569-1660)
    p->search_size = 0.3;
    p->resolution = 0.01;
    p->smear_deviation = 0.03;
    p->distance_variance_penalty = 0.3 * 0.3;
    const double d20 = 20 * 0.01745329251994329577;
    p->angle_variance_penalty = d20 * d20;
    p->fine_search_angle_offset = 0.2 * 0.01745329251994329577;
    p->coarse_search_angle_offset = d20;
    p->coarse_angle_resolution = 2 * 0.01745329251994329577;
    p->minimum_angle_penalty = 0.9;
    p->minimum_distance_penalty = 0.5;
    p->use_response_expansion = 0;
    p->pad_ = 0;
}

void kt_default_loop_params(kt_params *p)
{
    if (!p) return;
    kt_default_params(p);
    p->search_size = 8.0;  // LoopSearchSpaceDimension
    p->resolution = 0.05;  // LoopSearchSpaceResolution
    p->smear_deviation = 0.03;
}

int kt_destroy(kt_ctx *c)
{
    if (!c) return KT_OK;
    if (c->stream) hipStreamSynchronize(c->stream);
    void *bufs[] = {c->d_ranges, c->d_poses, c->d_npts,    c->d_pts,     c->d_loc,   c->d_bad,  c->d_evt,
                    c->d_grids,  c->d_kernel, c->d_state, c->d_resp,    c->d_posmax, c->d_tie_idx, c->d_tie_val,
                    c->d_query,  c->d_bbeg,  c->d_bidx,    c->d_res, c->d_scratch, c->d_dirty, c->d_dirty_cnt};
    for (void *b : bufs) hipFree(b);
    for (auto &p : c->ev_free) {
        hipEventDestroy(p.first);
        hipEventDestroy(p.second);
    }
    for (auto &p : c->ev_used) {
        hipEventDestroy(p.second.first);
        hipEventDestroy(p.second.second);
    }
    if (c->stream) hipStreamDestroy(c->stream);
    delete c;
    return KT_OK;
}

int kt_create(kt_ctx **out, const kt_laser *laser, const kt_params *params, int max_matches, int max_scans,
              int max_base_per_match)
{
    if (!out) return kfail(KT_EINVAL, "out is NULL");
    *out = nullptr;
    if (!laser) return kfail(KT_EINVAL, "laser is NULL");
    if (max_matches < 1 || max_matches > 65535 || max_scans < 1 || max_base_per_match < 0)
        return kfail(KT_EINVAL, "need 1 <= max_matches <= 65535, max_scans >= 1, max_base_per_match >= 0");
    kt_params p;
    if (params) p = *params;
    else kt_default_params(&p);
    KtGeom g;
    std::vector<unsigned char> kernel;
    int rc = kt_geometry(*laser, p, g, kernel);
    if (rc != KT_OK) return rc;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1) return kfail(KT_ENODEV, "no HIP device");
    kt_ctx *c = new kt_ctx;
    c->laser = *laser;
    c->params = p;
    c->g = g;
    c->max_matches = max_matches;
    c->max_scans = max_scans;
    c->max_base = max_base_per_match;
    {
        const char *env = getenv("SLAM2D_KT_SLOTS");
        const int want = env ? atoi(env) : 0;  // default: the whole batch resident (measured fastest)
        c->slots = std::max(1, std::min(max_matches, want > 0 ? want : max_matches));
        const char *bpm = getenv("SLAM2D_KT_BUILD");
        if (bpm && !strcmp(bpm, "per_base")) c->build_per_match = 0;
        c->binned = g.ntiles <= KT_AS_MAX_TILES && max_base_per_match <= KT_AS_MAX_BASE &&
                    !(bpm && (!strcmp(bpm, "per_base") || !strcmp(bpm, "cas")));
    }
    hipError_t e;
    if ((e = hipStreamCreateWithFlags(&c->stream, hipStreamDefault)) != hipSuccess) {
        delete c;
        return kfail(KT_EHIP, "hipStreamCreate", e);
    }
    const size_t S = (size_t)max_scans, n = (size_t)g.n, M = (size_t)c->slots;
    const size_t mp = (size_t)g.max_poses, npos = (size_t)g.nxy * g.nxy;
    // SLAM2D_POISON=1 (test hook): fill every buffer with 0xA5 bytes first, so that a kernel reading
    // memory the context never initialised fails its parity test instead of passing on fresh zero pages
    const bool poison = getenv("SLAM2D_POISON") && atoi(getenv("SLAM2D_POISON")) != 0;
#define KALLOC(ptr, bytes)                                                                  \
    if ((e = hipMalloc((void **)&(ptr), (bytes))) != hipSuccess ||                          \
        (poison && (e = hipMemsetAsync((ptr), 0xA5, (bytes), c->stream)) != hipSuccess)) {  \
        kt_destroy(c);                                                                      \
        return kfail(KT_ENOMEM, "hipMalloc " #ptr, e);                                      \
    }
    KALLOC(c->d_ranges, sizeof(double) * S * n);
    KALLOC(c->d_poses, sizeof(double) * S * 3);
    KALLOC(c->d_npts, sizeof(int) * S);
    KALLOC(c->d_pts, sizeof(double2) * S * n);
    KALLOC(c->d_loc, sizeof(double2) * S * n);
    KALLOC(c->d_bad, S * n);
    KALLOC(c->d_evt, sizeof(int2) * S * n);
    KALLOC(c->d_grids, g.grid_stride * M);
    KALLOC(c->d_kernel, kernel.size());
    KALLOC(c->d_state, sizeof(KtState) * M);
    KALLOC(c->d_resp, sizeof(double) * mp * M);
    KALLOC(c->d_posmax, sizeof(unsigned long long) * npos * M);
    KALLOC(c->d_tie_idx, sizeof(int) * mp * M);
    KALLOC(c->d_tie_val, sizeof(double4) * std::max(mp, npos) * M);
    KALLOC(c->d_query, sizeof(int));
    KALLOC(c->d_bbeg, sizeof(int) * 2);
    KALLOC(c->d_bidx, sizeof(int) * std::max<size_t>(1, (size_t)max_base_per_match));
    KALLOC(c->d_res, sizeof(kt_result));
    if (c->binned) {
        KALLOC(c->d_scratch, sizeof(int) * M * std::max<size_t>(1, (size_t)max_base_per_match) * n);
        KALLOC(c->d_dirty, sizeof(int) * M * (size_t)g.ntiles);
        KALLOC(c->d_dirty_cnt, sizeof(int) * M);
    }
#undef KALLOC
    {
        const size_t shm = (size_t)g.n * (sizeof(double2) + 2 * sizeof(int));
        if (shm > 65536 && (e = hipFuncSetAttribute((const void *)kt_prepare_kernel,
                                                    hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm)) != hipSuccess) {
            kt_destroy(c);
            return kfail(KT_EHIP, "hipFuncSetAttribute(kt_prepare_kernel)", e);
        }
    }
    if ((e = hipMemsetAsync(c->d_grids, 0, g.grid_stride * M, c->stream)) != hipSuccess ||
        (e = hipMemsetAsync(c->d_npts, 0, sizeof(int) * S, c->stream)) != hipSuccess ||
        (e = hipMemcpyAsync(c->d_kernel, kernel.data(), kernel.size(), hipMemcpyHostToDevice, c->stream)) !=
            hipSuccess ||
        (e = hipStreamSynchronize(c->stream)) != hipSuccess) {
        kt_destroy(c);
        return kfail(KT_EHIP, "initialising the context", e);
    }
    *out = c;
    return KT_OK;
}

int kt_get_grid_info(kt_ctx *c, int *out)
{
    if (!c || !out) return kfail(KT_EINVAL, "NULL argument");
    const KtGeom &g = c->g;
    const int v[10] = {g.grid_size, g.border, g.width, g.ws, g.data_size, g.side, g.probs_ws, g.half, g.ksize,
                       g.max_poses};
    for (int i = 0; i < 10; ++i) out[i] = v[i];
    return KT_OK;
}

int kt_set_scans_device(kt_ctx *c, int first, int count, const double *d_ranges, const double *d_poses,
                        void *hip_stream)
{
    if (!c || !d_ranges || !d_poses) return kfail(KT_EINVAL, "NULL argument");
    if (first < 0 || count < 0 || first + count > c->max_scans) return kfail(KT_EINVAL, "scan slots out of range");
    if (count == 0) return KT_OK;
    hipStream_t s = hip_stream ? (hipStream_t)hip_stream : c->stream;
    const size_t n = (size_t)c->g.n;
    if (d_ranges != c->d_ranges + (size_t)first * n)
        KCHK(hipMemcpyAsync(c->d_ranges + (size_t)first * n, d_ranges, sizeof(double) * n * count,
                            hipMemcpyDeviceToDevice, s));
    if (d_poses != c->d_poses + (size_t)first * 3)
        KCHK(hipMemcpyAsync(c->d_poses + (size_t)first * 3, d_poses, sizeof(double) * 3 * count,
                            hipMemcpyDeviceToDevice, s));
    return kt_prepare(c, first, count, s);
}

int kt_set_scans(kt_ctx *c, int first, int count, const double *ranges, const double *poses)
{
    if (!c || !ranges || !poses) return kfail(KT_EINVAL, "NULL argument");
    if (first < 0 || count < 0 || first + count > c->max_scans) return kfail(KT_EINVAL, "scan slots out of range");
    if (count == 0) return KT_OK;
    const size_t n = (size_t)c->g.n;
    KCHK(hipMemcpyAsync(c->d_ranges + (size_t)first * n, ranges, sizeof(double) * n * count, hipMemcpyHostToDevice,
                        c->stream));
    KCHK(hipMemcpyAsync(c->d_poses + (size_t)first * 3, poses, sizeof(double) * 3 * count, hipMemcpyHostToDevice,
                        c->stream));
    int rc = kt_prepare(c, first, count, c->stream);
    if (rc != KT_OK) return rc;
    KCHK(hipStreamSynchronize(c->stream));
    return KT_OK;
}

int kt_match_batch_device(kt_ctx *c, int count, const int *d_query, const int *d_bbeg, const int *d_bidx,
                          int do_penalize, int do_refine, kt_result *d_res, void *hip_stream)
{
    if (!c || !d_query || !d_bbeg || !d_res) return kfail(KT_EINVAL, "NULL argument");
    if (count < 0 || count > c->max_matches) return kfail(KT_EINVAL, "count exceeds max_matches");
    if (count == 0) return KT_OK;
    if (c->max_base > 0 && !d_bidx) return kfail(KT_EINVAL, "d_base_index is NULL");
    return kt_run_batch(c, count, d_query, d_bbeg, d_bidx, do_penalize ? 1 : 0, do_refine ? 1 : 0, d_res,
                        hip_stream ? (hipStream_t)hip_stream : c->stream);
}

int kt_match_scan(kt_ctx *c, const double *q_ranges, const double q_pose[3], int n_base, const double *b_ranges,
                  const double *b_poses, int do_penalize, int do_refine, kt_result *result)
{
    if (!c || !q_ranges || !q_pose || !result || (n_base > 0 && (!b_ranges || !b_poses)))
        return kfail(KT_EINVAL, "NULL argument");
    if (n_base < 0 || n_base > c->max_base || n_base + 1 > c->max_scans)
        return kfail(KT_EINVAL, "n_base exceeds max_base_per_match or the scan pool");
    const size_t n = (size_t)c->g.n;
    hipStream_t s = c->stream;
    KCHK(hipMemcpyAsync(c->d_ranges, q_ranges, sizeof(double) * n, hipMemcpyHostToDevice, s));
    KCHK(hipMemcpyAsync(c->d_poses, q_pose, sizeof(double) * 3, hipMemcpyHostToDevice, s));
    if (n_base > 0) {
        KCHK(hipMemcpyAsync(c->d_ranges + n, b_ranges, sizeof(double) * n * n_base, hipMemcpyHostToDevice, s));
        KCHK(hipMemcpyAsync(c->d_poses + 3, b_poses, sizeof(double) * 3 * n_base, hipMemcpyHostToDevice, s));
    }
    int rc = kt_prepare(c, 0, 1 + n_base, s);
    if (rc != KT_OK) return rc;
    std::vector<int> idx((size_t)std::max(1, n_base));
    for (int i = 0; i < n_base; ++i) idx[i] = 1 + i;
    const int q0 = 0, beg[2] = {0, n_base};
    KCHK(hipMemcpyAsync(c->d_query, &q0, sizeof(int), hipMemcpyHostToDevice, s));
    KCHK(hipMemcpyAsync(c->d_bbeg, beg, sizeof(int) * 2, hipMemcpyHostToDevice, s));
    KCHK(hipMemcpyAsync(c->d_bidx, idx.data(), sizeof(int) * idx.size(), hipMemcpyHostToDevice, s));
    rc = kt_run_batch(c, 1, c->d_query, c->d_bbeg, c->d_bidx, do_penalize ? 1 : 0, do_refine ? 1 : 0, c->d_res, s);
    if (rc != KT_OK) return rc;
    KCHK(hipMemcpyAsync(result, c->d_res, sizeof(kt_result), hipMemcpyDeviceToHost, s));
    KCHK(hipStreamSynchronize(s));
    return KT_OK;
}

size_t kt_window_exchange_words(kt_ctx *c)
{
    if (!c) return 0;
    const size_t nxy2 = (size_t)c->g.nxy * c->g.nxy;
    return 2 + nxy2 + nxy2 * (size_t)c->g.nang[0];
}

int kt_match_sharded_begin_device(kt_ctx *c, int count, const int *d_query, const int *d_bbeg, const int *d_bidx,
                                  int do_penalize, int shard, int nshards, int64_t *d_exchange, void *hip_stream)
{
    if (!c || !d_query || !d_bbeg || !d_exchange) return kfail(KT_EINVAL, "NULL argument");
    if (count < 1 || count > c->slots) return kfail(KT_EINVAL, "sharded batch must hold 1 .. slots matches");
    if (nshards < 1 || shard < 0 || shard >= nshards) return kfail(KT_EINVAL, "need 0 <= shard < nshards");
    if (c->g.npass != 1) return kfail(KT_EINVAL, "a sharded window does not support response expansion");
    if (c->max_base > 0 && !d_bidx) return kfail(KT_EINVAL, "d_base_index is NULL");
    hipStream_t s = hip_stream ? (hipStream_t)hip_stream : c->stream;
    bool binned = false;
    int rc = kt_chunk_build(c, count, d_query, d_bbeg, d_bidx, s, binned);
    if (rc != KT_OK) return rc;
    c->sharded_binned = binned;
    if ((rc = kt_chunk_coarse(c, count, 0, do_penalize ? 1 : 0, shard, nshards, s)) != KT_OK) return rc;
    hipLaunchKernelGGL(kt_exchange_kernel, dim3(count), dim3(KT_THREADS), 0, s, c->g, c->d_state, c->d_resp,
                       c->d_posmax, (long long *)d_exchange, 0);
    KCHK(hipGetLastError());
    return KT_OK;
}

int kt_match_sharded_end_device(kt_ctx *c, int count, const int *d_bbeg, const int *d_bidx, int do_penalize,
                                int do_refine, const int64_t *d_exchange, kt_result *d_res, void *hip_stream)
{
    if (!c || !d_bbeg || !d_exchange || !d_res) return kfail(KT_EINVAL, "NULL argument");
    if (count < 1 || count > c->slots) return kfail(KT_EINVAL, "sharded batch must hold 1 .. slots matches");
    if (c->max_base > 0 && !d_bidx) return kfail(KT_EINVAL, "d_base_index is NULL");
    hipStream_t s = hip_stream ? (hipStream_t)hip_stream : c->stream;
    hipLaunchKernelGGL(kt_exchange_kernel, dim3(count), dim3(KT_THREADS), 0, s, c->g, c->d_state, c->d_resp,
                       c->d_posmax, (long long *)d_exchange, 1);
    KCHK(hipGetLastError());
    if (c->g.nxy * c->g.nxy > 512)
        KT_LAUNCH(K_SELECT, kt_select_kernel<1024>, dim3(count), dim3(1024), 0, s, c->g, c->d_state, c->d_resp,
              c->d_posmax, c->d_tie_idx, c->d_tie_val, 0, do_refine ? 1 : 0, d_res);
    else
        KT_LAUNCH(K_SELECT, kt_select_kernel<KT_THREADS>, dim3(count), dim3(KT_THREADS), 0, s, c->g, c->d_state, c->d_resp,
              c->d_posmax, c->d_tie_idx, c->d_tie_val, 0, do_refine ? 1 : 0, d_res);
    return kt_chunk_finish(c, count, d_bbeg, d_bidx, do_penalize ? 1 : 0, do_refine ? 1 : 0, d_res, s,
                           c->sharded_binned);
}

int kt_set_timing(kt_ctx *c, int enable)
{
    if (!c) return kfail(KT_EINVAL, "ctx is NULL");
    c->timing = enable != 0;
    return KT_OK;
}

#if defined(KT_DIAG_STAMPS)
// diagnostic builds only: per-workgroup s_memtime stamps of kt_addscans_kernel (8 per block)
int kt_diag_stamps(unsigned long long *out, int blocks)
{
    KCHK(hipDeviceSynchronize());
    KCHK(hipMemcpyFromSymbol(out, HIP_SYMBOL(kt_diag), sizeof(unsigned long long) * 8 * blocks));
    return KT_OK;
}
#endif

int kt_num_kernels(void) { return K_NUM; }
const char *kt_kernel_name(int i) { return (i >= 0 && i < K_NUM) ? k_names[i] : ""; }

int kt_get_kernel_times(kt_ctx *c, double *ms_out, int64_t *launches_out, int reset)
{
    if (!c) return kfail(KT_EINVAL, "ctx is NULL");
    KCHK(hipDeviceSynchronize());
    for (auto &u : c->ev_used) {
        float ms = 0;
        KCHK(hipEventElapsedTime(&ms, u.second.first, u.second.second));
        c->acc_ms[u.first] += ms;
        c->acc_n[u.first] += 1;
        c->ev_free.push_back(u.second);
    }
    c->ev_used.clear();
    for (int i = 0; i < K_NUM; ++i) {
        if (ms_out) ms_out[i] = c->acc_ms[i];
        if (launches_out) launches_out[i] = c->acc_n[i];
        if (reset) {
            c->acc_ms[i] = 0;
            c->acc_n[i] = 0;
        }
    }
    return KT_OK;
}

}  // extern "C"
