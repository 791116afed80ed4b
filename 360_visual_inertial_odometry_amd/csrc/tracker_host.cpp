// tracker_host.cpp — C-ABI of the ERP feature tracker (erp_*), host side.
//
// Owns the device state of a tracker (frame pyramids, point / RANSAC / GFTT buffers) and enqueues
// the tracker.hip kernels on the context stream.  The standalone entry points erp_klt_track /
// erp_gftt / erp_rot_ransac mirror the three OpenCV / Eigen calls of FeatureTracker
// (src/processing/FeatureTracker.cpp:222-223, 238-240, 253-379); erp_tracker_run chains them for a
// frame pair without a host round trip.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cmath>
#include <cstring>
#include <random>
#include <string>
#include <atomic>
#include <vector>

#include "ctx.h"
#include "tracker_types.h"

using namespace vio360;

namespace {

constexpr int kMaxIters = 1 << 16;

size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

// OpenCV imgproc/drawing.cpp Circle(..., fill=1): union of the midpoint-algorithm spans, as the
// half-width of the filled disc on every row offset 0..r
std::vector<int> circle_half_widths(int r) {
    std::vector<int> hw(r + 1, -1);
    int err = 0, dx = r, dy = 0, plus = 1, minus = (r << 1) - 1;
    while (dx >= dy) {
        hw[dy] = std::max(hw[dy], dx);  // rows cy±dy: [cx-dx, cx+dx]
        if (dx <= r) hw[dx] = std::max(hw[dx], dy);  // rows cy±dx: [cx-dy, cx+dy]
        dy++;
        err += plus;
        plus += 2;
        int mask = (err <= 0) - 1;
        err -= minus & mask;
        dx += mask;
        minus -= mask & 2;
    }
    return hw;
}

}  // namespace

struct erp_tracker {
    vio_ctx* ctx = nullptr;
    int W = 0, H = 0, max_points = 0, max_corners = 0;
    int nlev = 0;                        // levels allocated (maxLevel + 1 upper bound)
    int lw[TRK_MAX_LEVELS], lh[TRK_MAX_LEVELS], lp[TRK_MAX_LEVELS];
    uint8_t* lvl[2][TRK_MAX_LEVELS] = {};
    // points
    float *d_pts = nullptr, *d_next = nullptr, *d_err = nullptr, *d_b0 = nullptr, *d_b1 = nullptr;
    float *d_bear0 = nullptr, *d_bear1 = nullptr;  // pipeline: bearings of every input / tracked point (LK launch)
    uint8_t *d_status = nullptr, *d_kept = nullptr;
    int *d_gidx = nullptr, *d_count = nullptr;
    float* d_rot = nullptr;
    int32_t* d_samples = nullptr;
    int iters_cap = 0;
    int n_pts = 0;
    // scalars: [0] n_good [1] n_in [2] max_ord [3] n_cand [4] n_out [6] n_top [7..8] cut [9] incomplete
    // [10] lmax_over [11] n_flat
    int* d_scal = nullptr;
    // gftt
    unsigned long long *d_cand = nullptr, *d_cand_sorted = nullptr;
    uint32_t* d_raw = nullptr;  // tempered mt19937 words of the RANSAC seed (side stream)
    float* d_eig = nullptr;     // GFTT min-eigenvalue map (W x H f32)
    unsigned int cand_cap = 0;
    void* d_sort_tmp = nullptr;
    size_t sort_tmp_bytes = 0;
    uint32_t* d_grid = nullptr;
    size_t grid_bytes = 0;
    float* d_corners = nullptr;
    uint32_t* d_disc = nullptr;
    int disc_words = 0;
    int* d_halfw = nullptr;
    int halfw_r = -1;
    uint8_t* d_mask = nullptr;  // explicit mask (erp_gftt)
    // GFTT top-K fast path
    unsigned int* d_hist = nullptr;
    unsigned long long *d_topk = nullptr, *d_topk_sorted = nullptr;
    unsigned int topk_cap = 0;
    GfArgs last_gf{};           // arguments of the last enqueued GFTT (exact fallback)
    // presort of every local maximum (pipeline, side stream) and the greedy pass over it after the discs:
    // histogram [GF_BUCKETS], then its scalars [0] n_top [1..2] cut [3] zero max_ord [4] n_cand [5] static-region
    // maximum (cleared by gftt_lmax_kernel on the side stream)
    unsigned int* d_hist2 = nullptr;
    unsigned long long *d_topk2 = nullptr, *d_topk2_sorted = nullptr;
    bool presel_used = false;   // the last pipeline GFTT ran the presel pass (its fallback: the exact tail)
    bool presel_flag = false;   // ... and took the presort's result through the device counter (no stream join)
    unsigned int presort_gen = 0;  // runs with a presort: the hand-off counter's target is gen x the sort's grid
    int n_exact_tail = 0, n_full_sort = 0;  // fallbacks taken by read_corners (erp_tracker_gftt_fallbacks)
    // local-maximum path: per-tile local maxima, counts, static-region maxima, disc flags
    unsigned long long* d_lmax = nullptr;
    unsigned int* d_lmax_n = nullptr;
    uint32_t* d_tile_max = nullptr;
    uint8_t* d_tile_dirty = nullptr;
    uint32_t* d_tile_kmax = nullptr;
    int tiles_x = 0, tiles_y = 0;
    hipEvent_t ev[6] = {};
    // the GFTT eigenvalue map runs on a side stream, overlapped with pyramids / LK / RANSAC
    hipStream_t side = nullptr;
    hipEvent_t join = nullptr, pyr_done = nullptr;  // side stream: waits for the pyramids / joined before the GFTT tail
    bool stage_timing = true;  // record the per-stage events (each marker costs the stream a few us)
    bool timed_run = false;    // the last run recorded them
    // without stage markers the pipeline is captured once into a graph and replayed (the ~20 launches,
    // event records and memsets of a run are otherwise enqueued one by one by the host, which the GPU
    // outruns: the first pyramid kernel started ~18 us after the run's start event); re-captured when
    // the point count, the parameters or the tracker's allocations change
    hipGraphExec_t run_graph = nullptr;
    int graph_n = -1;
    size_t graph_allocs = 0;
    erp_klt_params graph_klt{};
    erp_tracker_params graph_prm{};
    bool ran = false;
    std::vector<void*> allocs;
};

namespace {

template <class T>
int dalloc(erp_tracker* t, T** p, size_t bytes) {
    DeviceScope scope(t->ctx->device);  // every tracker buffer lives on the context's device
    void* q = nullptr;
    if (hipMalloc(&q, std::max<size_t>(bytes, 64)) != hipSuccess) {
        set_error(t->ctx, "hipMalloc failed in the tracker");
        return VIO_ENOMEM;
    }
    t->allocs.push_back(q);
    *p = (T*)q;
    return VIO_OK;
}

void tracker_free(erp_tracker* t) {
    if (t->side) (void)hipStreamSynchronize(t->side);  // (the presel hand-off leaves the side stream unjoined)
    for (void* p : t->allocs) (void)hipFree(p);
    t->allocs.clear();
    for (auto& e : t->ev)
        if (e) (void)hipEventDestroy(e);
    if (t->run_graph) (void)hipGraphExecDestroy(t->run_graph);
    t->run_graph = nullptr;
    if (t->side) (void)hipStreamDestroy(t->side);
    if (t->join) (void)hipEventDestroy(t->join);
    if (t->pyr_done) (void)hipEventDestroy(t->pyr_done);
}

int ensure_iters(erp_tracker* t, int iters) {
    if (iters <= t->iters_cap) return VIO_OK;
    if (iters > kMaxIters) { set_error(t->ctx, "ransac_iters too large"); return VIO_EINVAL; }
    int cap = std::max(iters, 1024);
    int rc;
    if ((rc = dalloc(t, &t->d_samples, sizeof(int32_t) * 3 * cap)) != VIO_OK) return rc;
    if ((rc = dalloc(t, &t->d_count, sizeof(int) * cap)) != VIO_OK) return rc;
    if ((rc = dalloc(t, &t->d_rot, sizeof(float) * 9 * cap)) != VIO_OK) return rc;
    t->iters_cap = cap;
    return VIO_OK;
}

// the GFTT selection grid (3 slots x 4 B per min-distance cell) lives in LDS up to this size, next
// to the selection kernel's ~14 KB of static LDS (config 1: 128 x 64 cells = 96 KB)
constexpr size_t kSelectGridLds = GF_SELECT_LDS_MAX;

int ensure_gftt(erp_tracker* t, double min_dist) {
    int rc;
    if (!t->d_cand) {
        // NMS leaves at most one candidate per 2x2 block except on exact plateaus; W*H/4 (+slack)
        t->cand_cap = (unsigned int)std::min<size_t>((size_t)t->W * t->H / 4 + 4096, (size_t)1 << 26);
        if ((rc = dalloc(t, &t->d_cand, sizeof(unsigned long long) * t->cand_cap)) != VIO_OK) return rc;
        if ((rc = dalloc(t, &t->d_eig, sizeof(float) * (size_t)t->W * t->H)) != VIO_OK) return rc;
        if ((rc = dalloc(t, &t->d_cand_sorted, sizeof(unsigned long long) * t->cand_cap)) != VIO_OK) return rc;
        t->sort_tmp_bytes = gftt_sort_tmp_bytes(t->cand_cap);
        if ((rc = dalloc(t, (char**)&t->d_sort_tmp, t->sort_tmp_bytes)) != VIO_OK) return rc;
        t->topk_cap = std::min<unsigned int>(GF_TOPK_CAP, t->cand_cap);
        if ((rc = dalloc(t, &t->d_hist, sizeof(unsigned int) * GF_BUCKETS)) != VIO_OK) return rc;
        if ((rc = dalloc(t, &t->d_topk, sizeof(unsigned long long) * t->topk_cap)) != VIO_OK) return rc;
        if ((rc = dalloc(t, &t->d_topk_sorted, sizeof(unsigned long long) * t->topk_cap)) != VIO_OK) return rc;
        if ((rc = dalloc(t, &t->d_hist2, sizeof(unsigned int) * kPresortWords)) != VIO_OK) return rc;
        VIO_HIP(t->ctx, hipMemset(t->d_hist2, 0, sizeof(unsigned int) * kPresortWords));  // the hand-off counter
        if ((rc = dalloc(t, &t->d_topk2, sizeof(unsigned long long) * t->topk_cap)) != VIO_OK) return rc;
        if ((rc = dalloc(t, &t->d_topk2_sorted, sizeof(unsigned long long) * t->topk_cap)) != VIO_OK) return rc;
        t->tiles_x = (t->W + LM_TX - 1) / LM_TX;
        t->tiles_y = (t->H + LM_TY - 1) / LM_TY;
        const size_t nt = (size_t)t->tiles_x * t->tiles_y;
        if ((rc = dalloc(t, &t->d_lmax, sizeof(unsigned long long) * LM_CAP * nt)) != VIO_OK) return rc;
        if ((rc = dalloc(t, &t->d_lmax_n, sizeof(unsigned int) * nt)) != VIO_OK) return rc;
        if ((rc = dalloc(t, &t->d_tile_max, sizeof(uint32_t) * nt)) != VIO_OK) return rc;
        if ((rc = dalloc(t, &t->d_tile_dirty, nt)) != VIO_OK) return rc;
        if ((rc = dalloc(t, &t->d_tile_kmax, sizeof(uint32_t) * nt)) != VIO_OK) return rc;
        // dynamic-LDS limit of the single-workgroup selection kernel, once per tracker (its device is
        // current here): the selection grid and chain heads up to kSelectGridLds (larger grids live in
        // d_grid)
        hipError_t e = gftt_select_set_lds(kSelectGridLds);
        if (e != hipSuccess) return hip_fail(t->ctx, e, "hipFuncSetAttribute(gftt_select)");
    }
    if (min_dist >= 1) {
        int cell = (int)std::lrint(min_dist);
        int gw = (t->W + cell - 1) / cell, gh = (t->H + cell - 1) / cell;
        size_t bytes = (size_t)gw * gh * 3 * sizeof(uint32_t);
        if (bytes > kSelectGridLds && bytes > t->grid_bytes) {
            if ((rc = dalloc(t, &t->d_grid, bytes)) != VIO_OK) return rc;
            t->grid_bytes = bytes;
        }
    }
    return VIO_OK;
}

int tracker_alloc(erp_tracker* t) {
    int rc;
    int w = t->W, h = t->H;
    t->nlev = 0;
    for (int l = 0; l < TRK_MAX_LEVELS; ++l) {
        t->lw[l] = w; t->lh[l] = h;
        t->lp[l] = (int)align_up(w, 128);
        for (int s = 0; s < 2; ++s)
            if ((rc = dalloc(t, &t->lvl[s][l], (size_t)t->lp[l] * h)) != VIO_OK) return rc;
        t->nlev = l + 1;
        if (w <= 2 || h <= 2) break;
        w = (w + 1) / 2; h = (h + 1) / 2;
    }
    const int P = std::max(t->max_points, 1);
    if ((rc = dalloc(t, &t->d_pts, sizeof(float) * 2 * P))) return rc;
    if ((rc = dalloc(t, &t->d_next, sizeof(float) * 2 * P))) return rc;
    if ((rc = dalloc(t, &t->d_err, sizeof(float) * P))) return rc;
    if ((rc = dalloc(t, &t->d_status, P))) return rc;
    if ((rc = dalloc(t, &t->d_kept, P))) return rc;
    if ((rc = dalloc(t, &t->d_gidx, sizeof(int) * P))) return rc;
    if ((rc = dalloc(t, &t->d_b0, sizeof(float) * 3 * P))) return rc;
    if ((rc = dalloc(t, &t->d_b1, sizeof(float) * 3 * P))) return rc;
    if ((rc = dalloc(t, &t->d_bear0, sizeof(float) * 3 * P))) return rc;
    if ((rc = dalloc(t, &t->d_bear1, sizeof(float) * 3 * P))) return rc;
    if ((rc = dalloc(t, &t->d_scal, sizeof(int) * 16))) return rc;
    if ((rc = dalloc(t, &t->d_corners, sizeof(float) * 2 * std::max(t->max_corners, 1)))) return rc;
    t->disc_words = (t->W + 31) / 32;
    if ((rc = dalloc(t, &t->d_disc, sizeof(uint32_t) * t->disc_words * t->H))) return rc;
    if ((rc = ensure_iters(t, 1024))) return rc;
    if ((rc = dalloc(t, &t->d_raw, sizeof(uint32_t) * ransac_raw_words()))) return rc;
    for (auto& e : t->ev)
        if (hipEventCreate(&e) != hipSuccess) return hip_fail(t->ctx, hipErrorUnknown, "hipEventCreate");
    // pyr_done only orders GFTT pass 1 after the pyramids (contention, not data: pass 1 reads the uploaded level
    // 0), so it needs no system-scope fence -- the fence costs the main stream ~3 us before LK
    // (gpurun_out A/B, profiles/r6_notes.md); the join carries pass 1's results to the GFTT tail: default fences
    if (hipStreamCreateWithFlags(&t->side, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&t->join, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&t->pyr_done, hipEventDisableTiming | hipEventDisableSystemFence) != hipSuccess)
        return hip_fail(t->ctx, hipErrorUnknown, "side stream / events");
    return VIO_OK;
}

// top LK level: buildOpticalFlowPyramid stops when the next level would be <= winSize
int lk_top_level(const erp_tracker* t, int win, int max_level) {
    int lvl = 0;
    for (int l = 0; l <= max_level && l < t->nlev; ++l) {
        lvl = l;
        int nw = (t->lw[l] + 1) / 2, nh = (t->lh[l] + 1) / 2;
        if (nw <= win || nh <= win || l + 1 >= t->nlev) break;
    }
    return lvl;
}

int build_pyramids(erp_tracker* t, int top) {
    for (int l = 1; l <= top; ++l) {
        PyrLevelPair s{t->lvl[0][l - 1], t->lvl[1][l - 1], t->lw[l - 1], t->lh[l - 1], t->lp[l - 1]};
        PyrLevelPair d{t->lvl[0][l], t->lvl[1][l], t->lw[l], t->lh[l], t->lp[l]};
        hipError_t e = launch_pyr_down(s, d, 2, t->ctx->stream);
        if (e != hipSuccess) return hip_fail(t->ctx, e, "pyr_down_kernel");
    }
    return VIO_OK;
}

int check_klt(vio_ctx* ctx, const erp_klt_params* p) {
    if (!p) { set_error(ctx, "null erp_klt_params"); return VIO_EINVAL; }
    if (p->win <= 2 || p->win > 21 || p->max_level < 0 || p->max_level >= TRK_MAX_LEVELS) {
        set_error(ctx, "unsupported LK window / level (win in [3,21], max_level < 8)");
        return VIO_ENOSYS;
    }
    return VIO_OK;
}

// aux (the tracker pipeline): extra workgroups of the LK launch (LkAux); the ev[1] stage marker between the
// pyramids and LK then only with stage timing (an event record costs the stream ~6 us before the next launch)
int enqueue_lk(erp_tracker* t, const erp_klt_params* p, int n, bool pyr_built = false, const LkAux* aux = nullptr) {
    LkArgs a;
    std::memset(&a, 0, sizeof a);
    int top = lk_top_level(t, p->win, p->max_level);
    int rc = pyr_built ? VIO_OK : build_pyramids(t, top);
    if (rc) return rc;
    for (int l = 0; l <= top; ++l) a.lv[l] = LkLevel{t->lvl[0][l], t->lvl[1][l], t->lw[l], t->lh[l], t->lp[l]};
    a.levels = top;
    a.pts = t->d_pts;
    a.next = t->d_next;
    a.status = t->d_status;
    a.err = t->d_err;
    a.n = n;
    a.win = p->win;
    // TermCriteria clamps (lkpyramid.cpp): maxCount in [0,100], epsilon in [0,10], squared
    a.max_iters = std::min(std::max(p->max_iters, 0), 100);
    double eps = std::min(std::max((double)p->epsilon, 0.0), 10.0);
    a.eps2 = eps * eps;
    a.min_eig = p->min_eig_threshold;
    if (aux) a.bear1 = t->d_bear1;  // the pipeline's RANSAC input (its previous points' bearings: aux workgroups)
    if (t->ev[1] && (!aux || t->stage_timing)) (void)hipEventRecord(t->ev[1], t->ctx->stream);
    hipError_t e = launch_lk(a, t->ctx->stream, aux);
    if (e != hipSuccess) return hip_fail(t->ctx, e, "lk_kernel");
    return VIO_OK;
}

RansacArgs ransac_args(erp_tracker* t, int n, int mode, int iters, uint32_t seed, float thr, float polar, int margin,
                       const float* p0, const float* p1) {
    RansacArgs r;
    std::memset(&r, 0, sizeof r);
    r.p0 = p0; r.p1 = p1; r.status = t->d_status;
    r.n = n; r.W = t->W; r.H = t->H; r.mode = mode;
    r.polar_ratio = polar; r.margin = margin;
    r.gidx = t->d_gidx; r.n_good = t->d_scal + 0;
    r.b0 = t->d_b0; r.b1 = t->d_b1;
    r.samples = t->d_samples; r.iters = iters; r.seed = seed; r.thresh = thr;
    r.cmin = reinterpret_cast<float*>(t->d_scal + 12);
    r.raw = t->d_raw;
    r.count = t->d_count; r.rot = t->d_rot; r.kept = t->d_kept; r.n_in = t->d_scal + 1;
    return r;
}

// the analytic mask's static part: Camera::CreatePolarMask (Camera.cpp:100-118) + the left/right
// boundary mask (FeatureTracker.cpp:49-58)
void gf_static_region(const erp_tracker* t, int margin, float polar, GfArgs& g) {
    g.top_rows = (int)((float)t->H * polar);
    g.bottom_start = (int)((float)t->H * (1.0f - polar));
    g.margin = margin;
}
void gf_lmax_fields(erp_tracker* t, GfArgs& g) {
    g.lmax = t->d_lmax; g.lmax_n = t->d_lmax_n; g.tile_max = t->d_tile_max; g.tile_dirty = t->d_tile_dirty;
    g.tile_kmax = t->d_tile_kmax;
    g.tiles_x = t->tiles_x; g.tiles_y = t->tiles_y;
    g.lmax_over = t->d_scal + 10;
    g.n_flat = (unsigned int*)(t->d_scal + 11);
}
// GFTT arguments of the mask-independent pass 1 (local maxima + static-region tile maxima)
GfArgs gf_lmax_args(erp_tracker* t, const uint8_t* img, int pitch, int margin, float polar) {
    GfArgs g;
    std::memset(&g, 0, sizeof g);
    g.img = img; g.W = t->W; g.H = t->H; g.pitch = pitch;
    gf_static_region(t, margin, polar, g);
    gf_lmax_fields(t, g);
    return g;
}

// the presort of every local maximum of pass 1 (side stream): no disc bitmap, a zero masked maximum (every
// key passes the threshold test), the presort's own histogram / top-K / scalars
GfArgs gf_presort_args(erp_tracker* t, const uint8_t* img, int pitch, int margin, float polar, int max_corners) {
    GfArgs g = gf_lmax_args(t, img, pitch, margin, polar);
    unsigned int* sc = t->d_hist2 + GF_BUCKETS;
    g.max_ord = sc + 3;
    g.n_cand = sc + 4;
    g.hist = t->d_hist2;
    g.topk = t->d_topk2;
    g.topk_sorted = t->d_topk2_sorted;
    g.n_top = sc;
    g.cut = reinterpret_cast<int*>(sc + 1);
    g.smax = sc + 5;
    if (t->presel_flag) g.done = sc + 6;
    g.topk_cap = t->topk_cap;
    // the discs remove the strongest keys near the tracked points: 8 keys per corner (config 1: the greedy pass
    // fills 300 corners from the first ~770 keys; the rank sort's cost grows with the square of the prefix)
    g.topk_target = (unsigned int)std::min<size_t>(t->topk_cap, std::max<size_t>(2048, 8 * (size_t)max_corners));
    return g;
}

// eig_ready: the map of `img` was already produced (launch_gftt_eig joined into the context stream)
// presel: the pipeline's presort ran on the side stream (gf_presort_args): only the greedy pass over its
// prefix is enqueued here; read_corners runs the exact tail if that pass cannot decide
int enqueue_gftt(erp_tracker* t, const uint8_t* img, int pitch, const uint8_t* mask, int mask_pitch, int max_corners,
                 double quality, double min_dist, bool discs, int margin, float polar, bool eig_ready = false,
                 bool reset_done = false, bool presel = false) {
    int rc = ensure_gftt(t, min_dist);
    if (rc) return rc;
    GfArgs g;
    std::memset(&g, 0, sizeof g);
    g.img = img; g.W = t->W; g.H = t->H; g.pitch = pitch;
    g.mask = mask; g.mask_pitch = mask_pitch;
    gf_static_region(t, margin, polar, g);
    if (!mask) gf_lmax_fields(t, g);  // analytic mask: the local-maximum path
    g.disc_bits = discs ? t->d_disc : nullptr;
    g.disc_words = t->disc_words;
    g.quality = quality; g.min_dist = min_dist; g.max_corners = max_corners;
    g.max_ord = (uint32_t*)(t->d_scal + 2);
    g.eig = t->d_eig;
    g.cand = t->d_cand; g.cand_sorted = t->d_cand_sorted;
    g.n_cand = (unsigned int*)(t->d_scal + 3);
    g.cand_cap = t->cand_cap;
    // minDistance < 1: every candidate is accepted in order (featureselect.cpp), no grid needed — one
    // cell covering the image keeps the selection kernel's conflict test trivially false
    g.cell = min_dist >= 1 ? (int)std::lrint(min_dist) : std::max(t->W, t->H);
    g.gw = (t->W + g.cell - 1) / g.cell;
    g.gh = (t->H + g.cell - 1) / g.cell;
    size_t lds = (size_t)g.gw * g.gh * 3 * sizeof(uint32_t);
    g.grid_global = lds > kSelectGridLds ? t->d_grid : nullptr;
    g.corners = t->d_corners;
    g.n_out = t->d_scal + 4;
    g.hist = t->d_hist;
    g.topk = t->d_topk;
    g.topk_sorted = t->d_topk_sorted;
    g.n_top = (unsigned int*)(t->d_scal + 6);
    g.cut = t->d_scal + 7;
    g.incomplete = t->d_scal + 9;
    g.topk_cap = t->topk_cap;
    g.topk_target = (unsigned int)std::min<size_t>(t->topk_cap, std::max<size_t>(4096, 16 * (size_t)max_corners));
    // scalars [2] max_ord [3] n_cand [4] n_out [6] n_top [7..8] cut [9] incomplete
    t->last_gf = g;
    t->presel_used = presel && g.lmax;
    hipError_t e = reset_done ? hipSuccess : launch_gftt_reset(g, t->d_scal, t->ctx->stream);
    if (g.lmax) {
        if (e == hipSuccess && !eig_ready) e = launch_gftt_lmax(g, t->ctx->stream);
        if (e == hipSuccess && t->presel_used) {
            GfArgs gs = g;
            gs.presel = 1;
            gs.cut = reinterpret_cast<int*>(t->d_hist2 + GF_BUCKETS + 1);  // the presort's cut: [1] nothing below it
            gs.smax = t->d_hist2 + GF_BUCKETS + 5;                          // its static-region maximum
            if (t->presel_flag) {  // the presort's device hand-off instead of the stream join
                gs.wait_ctr = t->d_hist2 + GF_BUCKETS + 6;
                gs.wait_target = t->presort_gen * ((t->topk_cap + 63) / 64);
                // (VIO_TRK_TEST_PRESEL_TIMEOUT=1: the first hand-off of the process waits for a count it never
                // reaches -- the bounded wait's path, exercised by tests/test_tracker_gpu.py)
                static std::atomic<int> test_tmo{[] {
                    const char* v = std::getenv("VIO_TRK_TEST_PRESEL_TIMEOUT");
                    return v && v[0] == '1' ? 1 : 0;
                }()};
                if (test_tmo.exchange(0)) gs.wait_target += 1u << 30;
            }
            e = launch_gftt_presel(gs, t->d_topk2_sorted, t->d_hist2 + GF_BUCKETS, t->ctx->stream);
        } else if (e == hipSuccess) {
            e = launch_gftt_after_lmax(g, t->d_sort_tmp, t->sort_tmp_bytes, t->ctx->stream);
        }
    } else {
        if (e == hipSuccess && !eig_ready) e = launch_gftt_eig(g, t->ctx->stream);
        if (e == hipSuccess) e = launch_gftt(g, t->d_sort_tmp, t->sort_tmp_bytes, t->ctx->stream);
    }
    if (e != hipSuccess) return hip_fail(t->ctx, e, "gftt kernels");
    return VIO_OK;
}

int upload_frame(erp_tracker* t, int slot, const uint8_t* img, int stride) {
    if (!img || stride < t->W) { set_error(t->ctx, "bad frame"); return VIO_EINVAL; }
    VIO_DEVICE(t->ctx);
    VIO_HIP(t->ctx, hipMemcpy2DAsync(t->lvl[slot][0], t->lp[0], img, stride, t->W, t->H, hipMemcpyHostToDevice,
                                     t->ctx->stream));
    return VIO_OK;
}

int read_corners(erp_tracker* t, float* out_xy, int* n_out) {
    int n = 0, inc = 0;
    int sc[12];
    VIO_HIP(t->ctx, hipMemcpyAsync(sc, t->d_scal, sizeof(sc), hipMemcpyDeviceToHost, t->ctx->stream));
    VIO_HIP(t->ctx, hipStreamSynchronize(t->ctx->stream));
    // the side stream's pass 1 / presort (the presel hand-off does not join it): the fallbacks below read them
    VIO_HIP(t->ctx, hipStreamSynchronize(t->side));
    bool map_path = false;
    if (t->last_gf.lmax && sc[10]) {  // a tile held more local maxima than its slots: the map path
        map_path = true;
        GfArgs g = t->last_gf;
        g.lmax = nullptr;
        hipError_t e = launch_gftt_reset(g, t->d_scal, t->ctx->stream);
        if (e == hipSuccess) e = launch_gftt_eig(g, t->ctx->stream);
        if (e == hipSuccess) e = launch_gftt(g, t->d_sort_tmp, t->sort_tmp_bytes, t->ctx->stream);
        if (e != hipSuccess) return hip_fail(t->ctx, e, "gftt map path");
        t->last_gf = g;
        VIO_HIP(t->ctx, hipMemcpyAsync(sc, t->d_scal, sizeof(sc), hipMemcpyDeviceToHost, t->ctx->stream));
        VIO_HIP(t->ctx, hipStreamSynchronize(t->ctx->stream));
    }
    if (!map_path && t->presel_used && sc[9]) {
        // the presorted prefix did not decide (threshold bound reached or prefix exhausted before max_corners):
        // the exact tail -- masked maximum, candidate top-K, greedy pass (its buffers are untouched by presel)
        hipError_t e = launch_gftt_after_lmax(t->last_gf, t->d_sort_tmp, t->sort_tmp_bytes, t->ctx->stream);
        if (e != hipSuccess) return hip_fail(t->ctx, e, "gftt exact tail");
        ++t->n_exact_tail;
        VIO_HIP(t->ctx, hipMemcpyAsync(sc, t->d_scal, sizeof(sc), hipMemcpyDeviceToHost, t->ctx->stream));
        VIO_HIP(t->ctx, hipStreamSynchronize(t->ctx->stream));
    }
    t->presel_used = false;
    if ((unsigned int)sc[3] > t->cand_cap) {  // NMS survivors beyond the candidate buffer: the corner set
        set_error(t->ctx, "GFTT candidate buffer overflow");  // would differ from goodFeaturesToTrack
        return VIO_ENOSYS;
    }
    inc = sc[9];
    if (inc) {  // the top-K subset did not decide: exact pass over every candidate
        ++t->n_full_sort;
        hipError_t e = t->last_gf.lmax ? launch_gftt_flatten(t->last_gf, t->ctx->stream) : hipSuccess;
        if (e == hipSuccess)
            e = launch_gftt_full(t->last_gf, (unsigned int)sc[3], t->d_sort_tmp, t->sort_tmp_bytes, t->ctx->stream);
        if (e != hipSuccess) return hip_fail(t->ctx, e, "gftt exact fallback");
        VIO_HIP(t->ctx, hipMemsetAsync(t->d_scal + 9, 0, sizeof(int), t->ctx->stream));
    }
    VIO_HIP(t->ctx, hipMemcpyAsync(&n, t->d_scal + 4, sizeof(int), hipMemcpyDeviceToHost, t->ctx->stream));
    VIO_HIP(t->ctx, hipStreamSynchronize(t->ctx->stream));
    if (n > 0 && out_xy)
        VIO_HIP(t->ctx, hipMemcpy(out_xy, t->d_corners, sizeof(float) * 2 * n, hipMemcpyDeviceToHost));
    *n_out = n;
    return VIO_OK;
}

}  // namespace

extern "C" {

int erp_ransac_samples(uint32_t seed, int n, int iters, int32_t* out) {
    if (n < 3 || iters < 0 || (iters > 0 && !out)) return VIO_EINVAL;
    std::mt19937 gen(seed);
    std::uniform_int_distribution<> dis(0, n - 1);
    for (int it = 0; it < iters; ++it) {
        int got[3], k = 0;
        while (k < 3) {
            int idx = dis(gen);
            bool dup = false;
            for (int q = 0; q < k; ++q) dup |= got[q] == idx;
            if (!dup) got[k++] = idx;
        }
        out[3 * it] = got[0]; out[3 * it + 1] = got[1]; out[3 * it + 2] = got[2];
    }
    return VIO_OK;
}

int erp_tracker_create(vio_ctx* ctx, int W, int H, int max_points, int max_corners, erp_tracker** out) {
    if (!ctx || !out || W < 8 || H < 8 || W > 65535 || H > 65535 || max_points < 0 || max_corners < 0)
        return VIO_EINVAL;
    *out = nullptr;
    DeviceScope _vio_dev_scope(ctx->device);
    erp_tracker* t = new erp_tracker();
    t->ctx = ctx; t->W = W; t->H = H; t->max_points = max_points; t->max_corners = max_corners;
    int rc = tracker_alloc(t);
    if (rc) { tracker_free(t); delete t; return rc; }
    *out = t;
    return VIO_OK;
}

int erp_tracker_gftt_fallbacks(erp_tracker* t, int* exact_tail, int* full_sort) {
    if (!t || !exact_tail || !full_sort) return VIO_EINVAL;
    *exact_tail = t->n_exact_tail;
    *full_sort = t->n_full_sort;
    return VIO_OK;
}

void erp_tracker_destroy(erp_tracker* t) {
    if (!t) return;
    DeviceScope _vio_dev_scope(t->ctx->device);
    (void)hipStreamSynchronize(t->ctx->stream);
    tracker_free(t);
    delete t;
}

int erp_tracker_upload(erp_tracker* t, int slot, const uint8_t* img, int stride) {
    if (!t || slot < 0 || slot > 1) return VIO_EINVAL;
    return upload_frame(t, slot, img, stride);
}

int erp_tracker_upload_resized(erp_tracker* t, int slot, const uint8_t* img, int W, int H, int stride) {
    if (!t || slot < 0 || slot > 1 || !img || W <= 0 || H <= 0 || stride < W) return VIO_EINVAL;
    if (W == t->W && H == t->H) return upload_frame(t, slot, img, stride);
    vio_ctx* ctx = t->ctx;
    VIO_DEVICE(ctx);
    const int sp = (W + 15) & ~15;  // 16-byte rows: the resize fast path
    uint8_t* d_src = static_cast<uint8_t*>(ctx_buffer(ctx, kSlotResizeSrc, (size_t)sp * H));
    if (!d_src) {
        set_error(ctx, "erp_tracker_upload_resized: device allocation failed");
        return VIO_ENOMEM;
    }
    VIO_HIP(ctx, hipMemcpy2DAsync(d_src, sp, img, stride, W, H, hipMemcpyHostToDevice, ctx->stream));
    return erp_resize_area_device(ctx, d_src, W, H, sp, 1, t->lvl[slot][0], t->W, t->H, t->lp[0]);
}

int erp_tracker_device_frame(erp_tracker* t, int slot, uint8_t** dev_ptr, int* pitch) {
    if (!t || slot < 0 || slot > 1 || !dev_ptr || !pitch) return VIO_EINVAL;
    *dev_ptr = t->lvl[slot][0];
    *pitch = t->lp[0];
    return VIO_OK;
}

int erp_tracker_swap(erp_tracker* t) {
    if (!t) return VIO_EINVAL;
    for (int l = 0; l < t->nlev; ++l) std::swap(t->lvl[0][l], t->lvl[1][l]);
    return VIO_OK;
}

int erp_tracker_set_points(erp_tracker* t, const float* pts, int n) {
    if (!t || n < 0 || n > t->max_points || (n > 0 && !pts)) {
        if (t) set_error(t->ctx, "point count exceeds max_points");
        return VIO_EINVAL;
    }
    t->n_pts = n;
    VIO_DEVICE(t->ctx);
    if (n) VIO_HIP(t->ctx, hipMemcpyAsync(t->d_pts, pts, sizeof(float) * 2 * n, hipMemcpyHostToDevice, t->ctx->stream));
    return VIO_OK;
}

// the enqueue sequence of one pipeline run (directly, or into the stream capture of erp_tracker_run)
static int enqueue_run(erp_tracker* t, const erp_klt_params* klt, const erp_tracker_params* p, int n, int radius,
                       bool capture) {
    int rc;
    hipStream_t st = t->ctx->stream;
    // GFTT's candidate order is known before the disc mask: the side stream presorts every local maximum after
    // pass 1 and the tail after the join is one greedy pass (VIO_TRK_PRESEL=0: the masked-maximum tail)
    static const bool presel_env = [] {
        const char* v = std::getenv("VIO_TRK_PRESEL");
        return !(v && v[0] == '0');
    }();
    const bool presel = presel_env;
    // the presort reaches the greedy pass through a device counter (VIO_TRK_PRESEL_FLAG=0: through the stream
    // join, ~6-14 us of event latency on the critical path); a captured graph keeps the join (the counter's
    // target is per run)
    static const bool flag_env = [] {
        const char* v = std::getenv("VIO_TRK_PRESEL_FLAG");
        return !(v && v[0] == '0');
    }();
    t->presel_flag = presel && flag_env && !capture;
    if (t->presel_flag) ++t->presort_gen;
    // The side stream (pass 1 + presort) is the longer path once the tail is one greedy pass, and the host's
    // enqueue order decides when the GPU first sees it (each launch costs the host a few microseconds, which the
    // GPU outruns).  VIO_TRK_SIDE: 0 (default) -- side work enqueued after LK (pass 1 dispatched ~14 us after
    // the pyramids); 1 -- enqueued right after the pyramids, before LK (pass 1 then delays LK: the same total,
    // profiles/r6c_ab_side.log); 2 -- enqueued first, pass 1 beside the pyramids (3-5 % slower)
    static const int side_env = [] {
        const char* v = std::getenv("VIO_TRK_SIDE");
        return v ? std::atoi(v) : 0;
    }();
    auto enqueue_side = [&]() -> int {
        VIO_HIP(t->ctx, hipStreamWaitEvent(t->side, t->pyr_done, 0));
        GfArgs gl = gf_lmax_args(t, t->lvl[1][0], t->lp[0], p->boundary_margin, p->polar_ratio);
        if (presel) {  // pass 1 clears the presort's histogram and scalars (ordered before the presort, and after
                       // the previous run's greedy pass through the pyramid event)
            gl.clear = t->d_hist2;
            gl.clear_n = kPresortClear;
        }
        hipError_t e = launch_gftt_lmax(gl, t->side);
        if (e != hipSuccess) return hip_fail(t->ctx, e, "gftt_lmax_kernel");
        if (presel) {
            e = launch_gftt_presort(
                gf_presort_args(t, t->lvl[1][0], t->lp[0], p->boundary_margin, p->polar_ratio, p->max_corners), t->side);
            if (e != hipSuccess) return hip_fail(t->ctx, e, "gftt presort");
        }
        VIO_HIP(t->ctx, hipEventRecord(t->join, t->side));
        return VIO_OK;
    };
    // main stream: pyramids, then LK, whose launch also carries the RANSAC draws' raw stream (seed only),
    // the GFTT counters / histogram / top-K reset and the disc bitmap clear in extra workgroups (on the
    // side stream they cost the main stream a cross-stream wait before RANSAC); side stream: GFTT pass 1
    // (the eigenvalue map of the current frame does not depend on tracking) once the pyramids are built,
    // beside LK / RANSAC (from the start of the run, beside the pyramids: measured 6 % slower)
    {
        LkAux x;
        std::memset(&x, 0, sizeof x);
        x.raw = t->d_raw;
        x.seed = p->ransac_seed;
        x.thresh = p->ransac_thresh_rad;
        x.cmin = reinterpret_cast<float*>(t->d_scal + 12);
        x.hist = t->d_hist;
        x.topk = t->d_topk;
        x.topk_cap = t->topk_cap;
        x.scal = t->d_scal;
        x.disc = t->d_disc;
        x.disc_words = (size_t)t->disc_words * t->H;
        x.pts = t->d_pts;
        x.bear0 = t->d_bear0;
        x.n = n;
        x.W = t->W;
        x.H = t->H;
        int top = lk_top_level(t, klt->win, klt->max_level);
        if (side_env == 2) {
            VIO_HIP(t->ctx, hipEventRecord(t->pyr_done, st));
            if ((rc = enqueue_side())) return rc;
        }
        if ((rc = build_pyramids(t, top))) return rc;
        if (side_env != 2) VIO_HIP(t->ctx, hipEventRecord(t->pyr_done, st));
        if (side_env == 1 && (rc = enqueue_side())) return rc;
        if ((rc = enqueue_lk(t, klt, n, true, &x))) return rc;
    }
    if (side_env == 0 && (rc = enqueue_side())) return rc;
    if (t->stage_timing) VIO_HIP(t->ctx, hipEventRecord(t->ev[2], st));
    RansacArgs r = ransac_args(t, n, 1, p->ransac_iters, p->ransac_seed, p->ransac_thresh_rad, p->polar_ratio,
                               p->boundary_margin, t->d_pts, t->d_next);
    r.bear0 = t->d_bear0;  // formed by the LK launch
    r.bear1 = t->d_bear1;
    if (n > 0) {
        // RANSAC, then its selection and CreateFeatureMask's discs of radius (int)min_dist around every kept
        // point in one launch (bitmap cleared in the LK launch; radius 0: no discs)
        DiscArgs d{t->d_next, t->d_kept, nullptr, nullptr, t->d_disc, t->disc_words, t->W, t->H, radius,
                   t->d_halfw};
        hipError_t e = launch_ransac_pipeline(r, d, st);
        if (e != hipSuccess) return hip_fail(t->ctx, e, "ransac kernels");
    } else {
        VIO_HIP(t->ctx, hipMemsetAsync(t->d_scal, 0, 2 * sizeof(int), st));
    }
    if (t->stage_timing) VIO_HIP(t->ctx, hipEventRecord(t->ev[3], st));
    if (!t->presel_flag) VIO_HIP(t->ctx, hipStreamWaitEvent(st, t->join, 0));
    if ((rc = enqueue_gftt(t, t->lvl[1][0], t->lp[0], nullptr, 0, p->max_corners, p->quality, p->min_dist, true,
                           p->boundary_margin, p->polar_ratio, true, true, presel)))
        return rc;
    return VIO_OK;
}


int erp_tracker_run(erp_tracker* t, const erp_klt_params* klt, const erp_tracker_params* p) {
    if (!t || !p) return VIO_EINVAL;
    int rc = check_klt(t->ctx, klt);
    if (rc) return rc;
    if (p->ransac_iters < 0 || p->max_corners < 0 || p->max_corners > t->max_corners || p->quality <= 0 ||
        p->min_dist < 0) {
        set_error(t->ctx, "bad erp_tracker_params");
        return VIO_EINVAL;
    }
    VIO_DEVICE(t->ctx);
    if ((rc = ensure_iters(t, std::max(p->ransac_iters, 1)))) return rc;
    if ((rc = ensure_gftt(t, p->min_dist))) return rc;
    hipStream_t st = t->ctx->stream;
    const int n = t->n_pts;
    // CreateFeatureMask's disc half-widths (a blocking upload: before any capture)
    const int radius = (int)p->min_dist;
    if (radius != t->halfw_r) {
        std::vector<int> hw = circle_half_widths(radius);
        if ((rc = dalloc(t, &t->d_halfw, sizeof(int) * (radius + 1)))) return rc;
        VIO_HIP(t->ctx, hipMemcpy(t->d_halfw, hw.data(), sizeof(int) * (radius + 1), hipMemcpyHostToDevice));
        t->halfw_r = radius;
    }
    VIO_HIP(t->ctx, hipEventRecord(t->ev[0], st));
    // graph replay (VIO_TRK_GRAPH=1, without stage markers): measured slower on ROCm 7.2 -- the replayed
    // graph ran the side stream's GFTT pass 1 after the main stream's kernels instead of beside them
    // (0.245 -> 0.450 ms per run); the run is enqueued directly by default
    static const bool graph_env = [] {
        const char* v = std::getenv("VIO_TRK_GRAPH");
        return v && v[0] == '1';
    }();
    const bool use_graph = graph_env && !t->stage_timing;
    if (use_graph && t->run_graph && t->graph_n == n && t->graph_allocs == t->allocs.size() &&
        std::memcmp(&t->graph_klt, klt, sizeof *klt) == 0 && std::memcmp(&t->graph_prm, p, sizeof *p) == 0) {
        VIO_HIP(t->ctx, hipGraphLaunch(t->run_graph, st));
    } else {
        if (t->run_graph) {
            (void)hipGraphExecDestroy(t->run_graph);
            t->run_graph = nullptr;
        }
        if (use_graph) VIO_HIP(t->ctx, hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
        rc = enqueue_run(t, klt, p, n, radius, use_graph);
        if (use_graph) {
            hipGraph_t g = nullptr;
            hipError_t e = hipStreamEndCapture(st, &g);
            if (rc == VIO_OK && e == hipSuccess) e = hipGraphInstantiate(&t->run_graph, g, nullptr, nullptr, 0);
            if (g) (void)hipGraphDestroy(g);
            if (rc) return rc;
            if (e != hipSuccess) return hip_fail(t->ctx, e, "tracker graph capture");
            t->graph_n = n;
            t->graph_allocs = t->allocs.size();
            t->graph_klt = *klt;
            t->graph_prm = *p;
            VIO_HIP(t->ctx, hipGraphLaunch(t->run_graph, st));
        } else if (rc) {
            return rc;
        }
    }
    VIO_HIP(t->ctx, hipEventRecord(t->ev[4], st));
    t->ran = true;
    t->timed_run = t->stage_timing;
    return VIO_OK;
}

int erp_tracker_sync(erp_tracker* t) {
    if (!t) return VIO_EINVAL;
    VIO_DEVICE(t->ctx);
    VIO_HIP(t->ctx, hipStreamSynchronize(t->ctx->stream));
    VIO_HIP(t->ctx, hipStreamSynchronize(t->side));  // (the presel hand-off leaves the side stream unjoined)
    return VIO_OK;
}

int erp_tracker_download(erp_tracker* t, float* next, uint8_t* status, uint8_t* kept, float* corners, int* n_corners) {
    if (!t) return VIO_EINVAL;
    VIO_DEVICE(t->ctx);
    VIO_HIP(t->ctx, hipStreamSynchronize(t->ctx->stream));
    const int n = t->n_pts;
    if (n && next) VIO_HIP(t->ctx, hipMemcpy(next, t->d_next, sizeof(float) * 2 * n, hipMemcpyDeviceToHost));
    if (n && status) VIO_HIP(t->ctx, hipMemcpy(status, t->d_status, n, hipMemcpyDeviceToHost));
    if (n && kept) VIO_HIP(t->ctx, hipMemcpy(kept, t->d_kept, n, hipMemcpyDeviceToHost));
    if (n_corners) {
        int nc = 0;
        int rc = read_corners(t, corners, &nc);
        if (rc) return rc;
        *n_corners = nc;
    }
    return VIO_OK;
}

int erp_tracker_set_stage_timing(erp_tracker* t, int on) {
    if (!t) return VIO_EINVAL;
    t->stage_timing = on != 0;
    return VIO_OK;
}

int erp_tracker_stage_ms(erp_tracker* t, double* pyr_ms, double* lk_ms, double* ransac_ms, double* gftt_ms,
                         double* total_ms) {
    if (!t || !t->ran) return VIO_EINVAL;
    VIO_DEVICE(t->ctx);
    VIO_HIP(t->ctx, hipEventSynchronize(t->ev[4]));
    float a = -1, b = -1, c = -1, d = -1, e = 0;
    if (t->timed_run) {
        VIO_HIP(t->ctx, hipEventElapsedTime(&a, t->ev[0], t->ev[1]));
        VIO_HIP(t->ctx, hipEventElapsedTime(&b, t->ev[1], t->ev[2]));
        VIO_HIP(t->ctx, hipEventElapsedTime(&c, t->ev[2], t->ev[3]));
        VIO_HIP(t->ctx, hipEventElapsedTime(&d, t->ev[3], t->ev[4]));
    }
    VIO_HIP(t->ctx, hipEventElapsedTime(&e, t->ev[0], t->ev[4]));
    if (pyr_ms) *pyr_ms = a;
    if (lk_ms) *lk_ms = b;
    if (ransac_ms) *ransac_ms = c;
    if (gftt_ms) *gftt_ms = d;
    if (total_ms) *total_ms = e;
    return VIO_OK;
}

int erp_klt_track(vio_ctx* ctx, const uint8_t* prev, const uint8_t* curr, int W, int H, int stride, const float* pts,
                  int n, float* next, uint8_t* status, float* err, const erp_klt_params* params) {
    if (!ctx || !prev || !curr || n < 0 || (n > 0 && (!pts || !next || !status))) return VIO_EINVAL;
    int rc = check_klt(ctx, params);
    if (rc) return rc;
    VIO_DEVICE(ctx);
    erp_tracker* t = nullptr;
    if ((rc = erp_tracker_create(ctx, W, H, std::max(n, 1), 0, &t))) return rc;
    if (!(rc = upload_frame(t, 0, prev, stride)) && !(rc = upload_frame(t, 1, curr, stride)) &&
        !(rc = erp_tracker_set_points(t, pts, n)) && !(rc = enqueue_lk(t, params, n))) {
        hipError_t e = hipStreamSynchronize(ctx->stream);
        if (e != hipSuccess) rc = hip_fail(ctx, e, "erp_klt_track");
        else if (n) {
            if (hipMemcpy(next, t->d_next, sizeof(float) * 2 * n, hipMemcpyDeviceToHost) != hipSuccess ||
                hipMemcpy(status, t->d_status, n, hipMemcpyDeviceToHost) != hipSuccess ||
                (err && hipMemcpy(err, t->d_err, sizeof(float) * n, hipMemcpyDeviceToHost) != hipSuccess))
                rc = hip_fail(ctx, hipErrorUnknown, "erp_klt_track download");
        }
    }
    erp_tracker_destroy(t);
    return rc;
}

int erp_gftt(vio_ctx* ctx, const uint8_t* img, const uint8_t* mask, int W, int H, int stride, int max_corners,
             double quality, double min_dist, float* out_xy, int* n_out) {
    if (!ctx || !img || !n_out || W < 3 || H < 3 || quality <= 0 || min_dist < 0 || max_corners < 0) return VIO_EINVAL;
    if (max_corners == 0) max_corners = W * H;  // "no limit"
    VIO_DEVICE(ctx);
    erp_tracker* t = nullptr;
    int rc = erp_tracker_create(ctx, W, H, 1, max_corners, &t);
    if (rc) return rc;
    uint8_t* dmask = nullptr;
    if (!(rc = upload_frame(t, 1, img, stride))) {
        if (mask) {
            if (!(rc = dalloc(t, &dmask, (size_t)t->lp[0] * H))) {
                hipError_t e = hipMemcpy2DAsync(dmask, t->lp[0], mask, stride, W, H, hipMemcpyHostToDevice, ctx->stream);
                if (e != hipSuccess) rc = hip_fail(ctx, e, "mask upload");
            }
        }
        if (!rc) rc = enqueue_gftt(t, t->lvl[1][0], t->lp[0], dmask, t->lp[0], max_corners, quality, min_dist, false,
                                   0, 0.f);
        if (!rc) rc = read_corners(t, out_xy, n_out);  // reports a candidate-buffer overflow
    }
    erp_tracker_destroy(t);
    return rc;
}

int erp_rot_ransac(vio_ctx* ctx, const float* p0, const float* p1, int n, int W, int H, const int32_t* samples,
                   int iters, float thresh_rad, uint8_t* mask, int* n_in) {
    if (!ctx || n < 0 || !mask || !n_in || iters < 0 || (n >= 3 && iters > 0 && !samples) || (n > 0 && (!p0 || !p1)))
        return VIO_EINVAL;
    if (n < 3) {  // FeatureTracker.cpp:130-134 / :258-260
        for (int i = 0; i < n; ++i) mask[i] = 1;
        *n_in = n;
        return VIO_OK;
    }
    for (int i = 0; i < 3 * iters; ++i)
        if (samples[i] < 0 || samples[i] >= n) { set_error(ctx, "RANSAC sample index out of range"); return VIO_EINVAL; }
    VIO_DEVICE(ctx);
    erp_tracker* t = nullptr;
    int rc = erp_tracker_create(ctx, std::max(W, 8), std::max(H, 8), n, 0, &t);
    if (rc) return rc;
    t->W = W; t->H = H;
    float* d_p1 = nullptr;
    if (!(rc = ensure_iters(t, std::max(iters, 1))) && !(rc = dalloc(t, &d_p1, sizeof(float) * 2 * n))) {
        hipStream_t st = ctx->stream;
        if (hipMemcpyAsync(t->d_pts, p0, sizeof(float) * 2 * n, hipMemcpyHostToDevice, st) != hipSuccess ||
            hipMemcpyAsync(d_p1, p1, sizeof(float) * 2 * n, hipMemcpyHostToDevice, st) != hipSuccess ||
            (iters && hipMemcpyAsync(t->d_samples, samples, sizeof(int32_t) * 3 * iters, hipMemcpyHostToDevice, st) !=
                          hipSuccess)) {
            rc = hip_fail(ctx, hipErrorUnknown, "ransac upload");
        } else {
            RansacArgs r = ransac_args(t, n, 0, iters, 0, thresh_rad, 0.f, 0, t->d_pts, d_p1);
            hipError_t e = launch_ransac(r, false, st);
            if (e == hipSuccess) e = hipStreamSynchronize(st);
            if (e != hipSuccess) rc = hip_fail(ctx, e, "ransac kernels");
            else if (hipMemcpy(mask, t->d_kept, n, hipMemcpyDeviceToHost) != hipSuccess ||
                     hipMemcpy(n_in, t->d_scal + 1, sizeof(int), hipMemcpyDeviceToHost) != hipSuccess)
                rc = hip_fail(ctx, hipErrorUnknown, "ransac download");
        }
    }
    erp_tracker_destroy(t);
    return rc;
}

}  // extern "C"

// ============================================================================================
// erp_frontend: FeatureTracker::TrackFeatures (FeatureTracker.cpp:61-206) = the device numeric
// path + the reference's host bookkeeping, restated on plain structs instead of Frame / Feature.
// ============================================================================================
namespace {

struct FeatureRec {
    int32_t id;
    float x, y;
    int32_t track_count, age;
};

// Frame::AssignFeaturesToGrid + LimitFeaturesPerGrid (src/database/Frame.cpp:108-202)
void assign_and_limit(std::vector<FeatureRec>& feats, int W, int H, int gc, int gr, int max_per) {
    const float cw = (float)W / gc, ch = (float)H / gr;
    std::vector<std::vector<int>> grid((size_t)gc * gr);
    auto assign = [&]() {
        for (auto& c : grid) c.clear();
        for (size_t i = 0; i < feats.size(); ++i) {
            float x = feats[i].x, y = feats[i].y;
            if (x < 0 || x >= W || y < 0 || y >= H) continue;
            int gx = std::min((int)(x / cw), gc - 1), gy = std::min((int)(y / ch), gr - 1);
            grid[(size_t)gy * gc + gx].push_back((int)i);
        }
    };
    assign();
    for (auto& cell : grid) {
        if (cell.size() <= (size_t)max_per) continue;
        std::sort(cell.begin(), cell.end(),
                  [&](int a, int b) { return feats[a].track_count > feats[b].track_count; });
        cell.resize(max_per);
    }
    std::vector<char> keep(feats.size(), 0);
    for (auto& cell : grid)
        for (int i : cell) keep[i] = 1;
    std::vector<FeatureRec> out;
    for (size_t i = 0; i < feats.size(); ++i)
        if (keep[i]) out.push_back(feats[i]);
    feats.swap(out);
}

// FeatureTracker::RemoveClusteredFeatures (FeatureTracker.cpp:404-497), tracker grid 20 x 10
void remove_clustered(std::vector<FeatureRec>& feats, int W, int H, float ratio) {
    if (feats.size() < 4) return;
    const int gc = 20, gr = 10;  // m_grid_cols / m_grid_rows (FeatureTracker.cpp:39-40)
    const float cw = (float)W / gc, ch = (float)H / gr;
    const float thr = std::sqrt(cw * cw + ch * ch) * ratio;
    std::vector<std::vector<size_t>> cells((size_t)gc * gr);
    auto cell_of = [&](const FeatureRec& f) {
        int col = std::min((int)(f.x / cw), gc - 1), row = std::min((int)(f.y / ch), gr - 1);
        return (size_t)row * gc + col;
    };
    for (size_t i = 0; i < feats.size(); ++i) cells[cell_of(feats[i])].push_back(i);
    std::vector<char> clustered(cells.size(), 0);
    for (size_t c = 0; c < cells.size(); ++c) {
        if (cells[c].size() < 4) continue;
        float mx = 0.f, my = 0.f;
        for (size_t i : cells[c]) { mx += feats[i].x; my += feats[i].y; }
        mx /= cells[c].size();
        my /= cells[c].size();
        float var = 0.f;
        for (size_t i : cells[c]) {
            float dx = feats[i].x - mx, dy = feats[i].y - my;
            var += (dx * dx + dy * dy);
        }
        var /= cells[c].size();
        if (std::sqrt(var) < thr) clustered[c] = 1;
    }
    std::vector<FeatureRec> out;
    for (auto& f : feats)
        if (!clustered[cell_of(f)]) out.push_back(f);
    feats.swap(out);
}

}  // namespace

struct erp_frontend {
    erp_tracker* t = nullptr;
    erp_frontend_params p{};
    int W = 0, H = 0;
    int frame = 0;
    int32_t next_id = 0;
    int num_tracked = 0, num_detected = 0;
    std::vector<FeatureRec> feats;
};

namespace {

// GFTT on slot 1 with the DetectNewFeatures mask: polar ∧ boundary ∧ (discs around `feats`)
int frontend_detect(erp_frontend* f, std::vector<float>& corners) {
    erp_tracker* t = f->t;
    hipStream_t st = t->ctx->stream;
    int rc;
    const bool discs = !f->feats.empty();
    if (discs) {
        const int n = (int)f->feats.size();
        if (n > t->max_points) { set_error(t->ctx, "too many features for the disc mask"); return VIO_ENOSYS; }
        std::vector<float> xy(2 * (size_t)n);
        for (int i = 0; i < n; ++i) { xy[2 * i] = f->feats[i].x; xy[2 * i + 1] = f->feats[i].y; }
        VIO_HIP(t->ctx, hipMemcpyAsync(t->d_pts, xy.data(), sizeof(float) * 2 * n, hipMemcpyHostToDevice, st));
        VIO_HIP(t->ctx, hipMemsetAsync(t->d_disc, 0, sizeof(uint32_t) * t->disc_words * t->H, st));
        const int radius = (int)f->p.min_distance;
        if (radius != t->halfw_r) {
            std::vector<int> hw = circle_half_widths(radius);
            if ((rc = dalloc(t, &t->d_halfw, sizeof(int) * (radius + 1)))) return rc;
            VIO_HIP(t->ctx, hipMemcpy(t->d_halfw, hw.data(), sizeof(int) * (radius + 1), hipMemcpyHostToDevice));
            t->halfw_r = radius;
        }
        DiscArgs d{t->d_pts, nullptr, nullptr, nullptr, t->d_disc, t->disc_words, t->W, t->H, radius, t->d_halfw};
        hipError_t e = launch_disc_mask(d, n, st);
        if (e != hipSuccess) return hip_fail(t->ctx, e, "disc_mask_kernel");
    }
    if ((rc = enqueue_gftt(t, t->lvl[1][0], t->lp[0], nullptr, 0, f->p.max_features, (double)f->p.quality_level,
                           (double)f->p.min_distance, discs, f->p.boundary_margin, 0.15f)))
        return rc;
    int n = 0;
    corners.resize(2 * (size_t)std::max(f->p.max_features, 1));
    if ((rc = read_corners(t, corners.data(), &n))) return rc;
    corners.resize(2 * (size_t)n);
    return VIO_OK;
}

}  // namespace

extern "C" {

int erp_frontend_create(vio_ctx* ctx, int W, int H, const erp_frontend_params* p, erp_frontend** out) {
    if (!ctx || !p || !out || p->max_features <= 0 || p->grid_cols <= 0 || p->grid_rows <= 0 ||
        p->max_features_per_grid <= 0 || p->min_distance < 0 || p->quality_level <= 0)
        return VIO_EINVAL;
    *out = nullptr;
    VIO_DEVICE(ctx);
    erp_frontend* f = new erp_frontend();
    f->p = *p;
    f->W = W; f->H = H;
    const int cap = std::max(4096, 2 * p->max_features + p->grid_cols * p->grid_rows * p->max_features_per_grid);
    int rc = erp_tracker_create(ctx, W, H, cap, p->max_features, &f->t);
    if (rc) { delete f; return rc; }
    if ((rc = ensure_iters(f->t, 1000))) { erp_tracker_destroy(f->t); delete f; return rc; }
    *out = f;
    return VIO_OK;
}

void erp_frontend_destroy(erp_frontend* f) {
    if (!f) return;
    erp_tracker_destroy(f->t);
    delete f;
}

int erp_frontend_track(erp_frontend* f, const uint8_t* img, int stride, int* n_features) {
    if (!f || !img) return VIO_EINVAL;
    erp_tracker* t = f->t;
    vio_ctx* ctx = t->ctx;
    VIO_DEVICE(ctx);
    hipStream_t st = ctx->stream;
    int rc;
    if ((rc = upload_frame(t, 1, img, stride))) return rc;
    const erp_frontend_params& P = f->p;
    if (f->frame == 0 || f->feats.empty()) {
        // first frame (or nothing to track): detect only (:68-97)
        f->feats.clear();
        std::vector<float> c;
        if ((rc = frontend_detect(f, c))) return rc;
        for (size_t i = 0; i < c.size() / 2; ++i) f->feats.push_back({f->next_id++, c[2 * i], c[2 * i + 1], 0, 0});
        f->num_tracked = 0;
        f->num_detected = (int)(c.size() / 2);
        assign_and_limit(f->feats, f->W, f->H, P.grid_cols, P.grid_rows, P.max_features_per_grid);
    } else {
        // TrackOpticalFlow (:228-251)
        const int n = (int)f->feats.size();
        if (n > t->max_points) { set_error(ctx, "too many features"); return VIO_ENOSYS; }
        std::vector<float> prev(2 * (size_t)n), next(2 * (size_t)n);
        std::vector<uint8_t> status(n);
        for (int i = 0; i < n; ++i) { prev[2 * i] = f->feats[i].x; prev[2 * i + 1] = f->feats[i].y; }
        if ((rc = erp_tracker_set_points(t, prev.data(), n))) return rc;
        erp_klt_params kp{21, 3, 30, 0.01f, 0.01f, 0};  // FeatureTracker.cpp:33-35, 240
        if ((rc = enqueue_lk(t, &kp, n))) return rc;
        VIO_HIP(ctx, hipMemcpyAsync(next.data(), t->d_next, sizeof(float) * 2 * n, hipMemcpyDeviceToHost, st));
        VIO_HIP(ctx, hipMemcpyAsync(status.data(), t->d_status, n, hipMemcpyDeviceToHost, st));
        VIO_HIP(ctx, hipStreamSynchronize(st));
        // status ∧ !IsInPolarRegion ∧ !IsNearBoundary (:117-126; Camera.cpp:120-139)
        std::vector<int> good;
        const float m = (float)P.boundary_margin;
        for (int i = 0; i < n; ++i) {
            float x = next[2 * i], y = next[2 * i + 1];
            float vr = y / (float)f->H;
            bool polar = vr < 0.15f || vr > (1.0f - 0.15f);
            bool nearb = x < m || x > (float)f->W - m || y < m || y > (float)f->H - m;
            if (status[i] && !polar && !nearb) good.push_back(i);
        }
        std::vector<uint8_t> inl(good.size(), 1);
        if (good.size() >= 3) {  // RejectOutliersRotationRANSAC (:253-328)
            const int ng = (int)good.size();
            std::vector<int32_t> samples(3 * 1000);
            erp_ransac_samples(P.ransac_seed + (uint32_t)f->frame, ng, 1000, samples.data());
            std::vector<float> g0(2 * (size_t)ng), g1(2 * (size_t)ng);
            for (int j = 0; j < ng; ++j) {
                g0[2 * j] = prev[2 * good[j]]; g0[2 * j + 1] = prev[2 * good[j] + 1];
                g1[2 * j] = next[2 * good[j]]; g1[2 * j + 1] = next[2 * good[j] + 1];
            }
            VIO_HIP(ctx, hipMemcpyAsync(t->d_pts, g0.data(), sizeof(float) * 2 * ng, hipMemcpyHostToDevice, st));
            VIO_HIP(ctx, hipMemcpyAsync(t->d_next, g1.data(), sizeof(float) * 2 * ng, hipMemcpyHostToDevice, st));
            VIO_HIP(ctx, hipMemcpyAsync(t->d_samples, samples.data(), sizeof(int32_t) * 3000, hipMemcpyHostToDevice, st));
            const float thr = (float)(2.0f * M_PI / 180.0f);
            RansacArgs r = ransac_args(t, ng, 0, 1000, 0, thr, 0.f, 0, t->d_pts, t->d_next);
            hipError_t e = launch_ransac(r, false, st);
            if (e != hipSuccess) return hip_fail(ctx, e, "ransac kernels");
            VIO_HIP(ctx, hipMemcpyAsync(inl.data(), t->d_kept, ng, hipMemcpyDeviceToHost, st));
            VIO_HIP(ctx, hipStreamSynchronize(st));
        }
        std::vector<FeatureRec> cur;
        for (size_t j = 0; j < good.size(); ++j) {
            if (!inl[j]) continue;
            const FeatureRec& pf = f->feats[good[j]];
            cur.push_back({pf.id, next[2 * good[j]], next[2 * good[j] + 1], pf.track_count + 1, pf.age + 1});
        }
        f->feats.swap(cur);
        f->num_tracked = (int)f->feats.size();
        if (P.remove_clustered) remove_clustered(f->feats, f->W, f->H, P.clustered_std_ratio);
        assign_and_limit(f->feats, f->W, f->H, P.grid_cols, P.grid_rows, P.max_features_per_grid);
        if ((int)f->feats.size() < P.max_features) {  // CreateFeatureMask + DetectNewFeatures (:176-199)
            std::vector<float> c;
            if ((rc = frontend_detect(f, c))) return rc;
            for (size_t i = 0; i < c.size() / 2; ++i) f->feats.push_back({f->next_id++, c[2 * i], c[2 * i + 1], 0, 0});
            f->num_detected = (int)(c.size() / 2);
            assign_and_limit(f->feats, f->W, f->H, P.grid_cols, P.grid_rows, P.max_features_per_grid);
        } else {
            f->num_detected = 0;
        }
    }
    erp_tracker_swap(t);  // m_prev_image = current (:202)
    f->frame++;
    if (n_features) *n_features = (int)f->feats.size();
    return VIO_OK;
}

int erp_frontend_features(erp_frontend* f, int32_t* ids, float* xy, int32_t* track_count, int32_t* age, int cap) {
    if (!f || cap < 0) return VIO_EINVAL;
    int n = std::min(cap, (int)f->feats.size());
    for (int i = 0; i < n; ++i) {
        const FeatureRec& r = f->feats[i];
        if (ids) ids[i] = r.id;
        if (xy) { xy[2 * i] = r.x; xy[2 * i + 1] = r.y; }
        if (track_count) track_count[i] = r.track_count;
        if (age) age[i] = r.age;
    }
    return VIO_OK;
}

int erp_frontend_stats(erp_frontend* f, int* num_tracked, int* num_detected) {
    if (!f) return VIO_EINVAL;
    if (num_tracked) *num_tracked = f->num_tracked;
    if (num_detected) *num_detected = f->num_detected;
    return VIO_OK;
}

}  // extern "C"
