// ba_host.cpp — C-ABI entry points for bundle adjustment (vio_ba_*), host side.
//
// Packs vio_ba_problem windows into the pooled device layout of ba_types.h, uploads them, launches
// one workgroup per window (ba_kernel.hip) and scatters the results back.  The packing applies
// Ceres' problem reduction (program.cc:305-400): constant parameter blocks and residual blocks
// whose parameters are all constant leave the optimisation, and the surviving blocks get their
// offsets in the reduced (Schur) system.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "ba_types.h"
#include "ctx.h"
#include "residency.h"

namespace vio360 {

hipError_t launch_ba_windows(const BaPools& P, int n, hipStream_t stream);
hipError_t launch_ba_pack(const BaPools& P, int n, uint8_t* dst, int64_t rec_bytes, hipStream_t stream);
constexpr int kPhLanesMax = 4;  // sub-batches of the phase route, each on its own stream
hipError_t launch_ba_phases(const BaPools& P, const BaWin* hw, int n, hipStream_t stream, int lanes,
                            hipStream_t* side, hipEvent_t* ev);
size_t ba_phase_doubles(int K, int L, int N, int T);  // sized for the smallest group (most partials)
const char* ba_phases_failed_launch();
hipError_t ba_phases_prepare(const BaWin* hw, int n);
int ba_cluster_members(const BaWin* hw, int n, int max_per_window);
hipError_t launch_ba_cluster(const BaPools& P, int n, int C, hipStream_t stream);
hipError_t ba_cluster_prelaunch(const BaPools& P, int n, hipStream_t stream);
bool global_ba_applicable(const vio_ba_problem& p);
int global_ba_solve(vio_ctx* ctx, const vio_ba_problem& p, vio_ba_output* out);
size_t ba_ws_extra_doubles();
hipError_t launch_lie_ba(int op, const double* in, double* out, int n, hipStream_t stream);
hipError_t launch_lie_init(int op, const double* in, double* out, int n, hipStream_t stream);

void set_error(vio_ctx* ctx, const std::string& msg) {
    if (ctx) ctx->last_error = msg;
}
int hip_fail(vio_ctx* ctx, hipError_t e, const char* what) {
    set_error(ctx, std::string("HIP error in ") + what + ": " + hipGetErrorString(e));
    return e == hipErrorOutOfMemory ? VIO_ENOMEM : VIO_EDEVICE;
}
void* ctx_buffer(vio_ctx* ctx, int slot, size_t bytes) {
    // the buffer must live on the context's device whatever device the calling thread has current
    DeviceScope dev_scope(ctx->device);
    if (dev_scope.err != hipSuccess) return nullptr;
    if ((int)ctx->bufs.size() <= slot) {
        ctx->bufs.resize(slot + 1, nullptr);
        ctx->caps.resize(slot + 1, 0);
    }
    if (ctx->caps[slot] >= bytes && ctx->bufs[slot]) return ctx->bufs[slot];
    if (ctx->bufs[slot]) (void)hipFree(ctx->bufs[slot]);
    ctx->bufs[slot] = nullptr;
    ctx->caps[slot] = 0;
    // 25 % headroom: per-keyframe solves grow and shrink by a few landmarks from call to call
    size_t cap = std::max<size_t>(bytes + bytes / 4, 256);
    if (hipMalloc(&ctx->bufs[slot], cap) != hipSuccess) return nullptr;
    ctx->caps[slot] = cap;
    return ctx->bufs[slot];
}
void* ctx_host_buffer(vio_ctx* ctx, int slot, size_t bytes) {
    if ((int)ctx->hbufs.size() <= slot) {
        ctx->hbufs.resize(slot + 1, nullptr);
        ctx->hcaps.resize(slot + 1, 0);
    }
    if (ctx->hcaps[slot] >= bytes && ctx->hbufs[slot]) return ctx->hbufs[slot];
    DeviceScope dev_scope(ctx->device);
    if (dev_scope.err != hipSuccess) return nullptr;
    if (ctx->hbufs[slot]) {
        (void)hipStreamSynchronize(ctx->stream);  // no copy from / into the old buffer is in flight
        (void)hipHostFree(ctx->hbufs[slot]);
    }
    ctx->hbufs[slot] = nullptr;
    ctx->hcaps[slot] = 0;
    size_t cap = std::max<size_t>(bytes + bytes / 4, 4096);
    if (hipHostMalloc(&ctx->hbufs[slot], cap, hipHostMallocDefault) != hipSuccess) return nullptr;
    ctx->hcaps[slot] = cap;
    return ctx->hbufs[slot];
}

namespace {

// A batch lives in ONE device allocation, in three regions: the inputs (filled on the host into one staging
// buffer and sent with one host-to-device copy), the outputs the host reads back (one device-to-host copy,
// the cluster route's error words included) and the workspace.  Byte offsets, 256-B aligned.
struct BaRegions {
    size_t win, pose_raw, kf_const, lm_xyz0, lm_var, lm_marg, lm_ptr, obs_kf, obs_lm, obs_uv, kf_ptr, kf_obs, preint,
        preint_valid, vel0, obs_perm, in_bytes;
    size_t i32, sum, out, trace, u8, bad, csync, out_begin, out_bytes;
    size_t ws, total;
};

// host side of a packed batch: the window descriptors (grid extents, result scatter) and the pool totals
struct Packed {
    std::vector<BaWin> win;
    int64_t ws_total = 0, out_total = 0, tr_total = 0;
    int64_t N_total = 0, L_total = 0, K_total = 0, lmptr_total = 0, kfptr_total = 0;
    BaRegions R{};
};

// Checks one problem and appends its descriptor: Ceres' problem reduction (constant blocks and residual
// blocks on constant blocks only leave the problem, program.cc:305-400) and the Schur ordering of the
// surviving blocks, plus the window's offsets into the pools.  The arrays are written by fill_window.
int analyze_window(vio_ctx* ctx, const vio_ba_problem& p, Packed& pk, std::vector<uint32_t>& scratch) {
    const int K = p.num_kf, L = p.num_lm, N = p.num_obs;
    if (K <= 0 || L < 0 || N < 0) { set_error(ctx, "invalid sizes"); return VIO_EINVAL; }
    if (p.variant < VIO_BA_LOCAL || p.variant > VIO_PNP) { set_error(ctx, "unknown variant"); return VIO_EINVAL; }
    if (K > BA_KMAX) { set_error(ctx, "num_kf > 16 is not supported on the windowed path"); return VIO_ENOSYS; }
    const bool vi = p.variant == VIO_BA_VI, pnp = p.variant == VIO_PNP;
    if (vi && K > 10) { set_error(ctx, "VIBA windows support num_kf <= 10"); return VIO_ENOSYS; }
    if (!p.T_cb || !p.T_wb_init || !p.kf_const || (L > 0 && (!p.lm_const || !p.lm_xyz)) ||
        (N > 0 && (!p.obs_kf || !p.obs_lm || !p.obs_uv))) {
        set_error(ctx, "null input array");
        return VIO_EINVAL;
    }
    if (vi && (!p.preint || !p.preint_valid || !p.vel)) { set_error(ctx, "VIBA needs preint/preint_valid/vel"); return VIO_EINVAL; }
    if (p.max_iterations < 0) { set_error(ctx, "max_iterations < 0"); return VIO_EINVAL; }
    // range check, and one observation per (keyframe, landmark) -- MapPoint::AddObservation keeps one per
    // frame -- through a keyframe bit mask per landmark (K <= 16)
    scratch.assign((size_t)L, 0u);
    std::vector<uint8_t> pose_used(K, 0), vel_used(K, 0);
    for (int o = 0; o < N; ++o) {
        const int k = p.obs_kf[o], l = p.obs_lm[o];
        if (k < 0 || k >= K || l < 0 || l >= L) {
            set_error(ctx, "observation index out of range");
            return VIO_EINVAL;
        }
        const uint32_t bit = 1u << k;
        if (scratch[l] & bit) {
            set_error(ctx, "duplicate (keyframe, landmark) observation");
            return VIO_EINVAL;
        }
        scratch[l] |= bit;
        if (!p.kf_const[k]) pose_used[k] = 1;
    }
    BaWin w;
    std::memset(&w, 0, sizeof w);
    w.K = K; w.L = L; w.N = N; w.variant = p.variant;
    w.is_vi = vi; w.is_pnp = pnp;
    w.max_iter = p.max_iterations;
    w.fixed_iter = p.fixed_iterations;
    w.rounds = pnp ? (p.num_rounds > 0 ? p.num_rounds : 4) : 1;
    w.cols = p.cols; w.rows = p.rows; w.huber = p.huber_delta; w.chi2_thr = p.chi2_threshold;
    for (int i = 0; i < 4; ++i) w.info[i] = p.info[i];
    {   // chol(info) lower (Eigen LLT of the 2x2), identity fallback
        double a = p.info[0], b = p.info[2], d = p.info[3];
        w.Lw[0] = 1; w.Lw[1] = 0; w.Lw[2] = 0; w.Lw[3] = 1;
        if (a > 0) {
            double l00 = std::sqrt(a), l10 = b / l00, t = d - l10 * l10;
            if (t > 0) { w.Lw[0] = l00; w.Lw[2] = l10; w.Lw[3] = std::sqrt(t); }
        }
    }
    if (vi) for (int i = 0; i < 3; ++i) { w.gravity[i] = p.gravity[i]; w.bg0[i] = p.bg[i]; w.ba0[i] = p.ba[i]; }
    // reduced problem: which blocks are free and used
    bool bias_used = false;
    if (vi) {
        for (int k = 1; k < K; ++k) {
            if (!p.preint_valid[k]) continue;
            vel_used[k - 1] = vel_used[k] = 1;
            bias_used = true;
            if (!p.kf_const[k - 1]) pose_used[k - 1] = 1;
            if (!p.kf_const[k]) pose_used[k] = 1;
        }
    }
    int off = 0;
    for (int k = 0; k < BA_KMAX; ++k) { w.pose_f[k] = -1; w.vel_f[k] = -1; }
    for (int k = 0; k < K; ++k)
        if (pose_used[k]) { w.pose_f[k] = off; off += 6; }
    w.np = off;
    for (int k = 0; k < K; ++k)
        if (vel_used[k]) { w.vel_f[k] = off; off += 3; }
    w.bg_f = bias_used ? off : -1; if (bias_used) off += 3;
    w.ba_f = bias_used ? off : -1; if (bias_used) off += 3;
    w.nf = off;
    w.ni = w.nf - w.np;
    if (w.nf > BA_NF_MAX) { set_error(ctx, "reduced system larger than 96 parameters"); return VIO_ENOSYS; }
    w.T = (w.np + 15) / 16;
    if (w.T < 1) w.T = 1;
    w.npad = 16 * w.T;
    w.n_imu = 0;
    if (vi) for (int k = 1; k < K; ++k) w.n_imu += p.preint_valid[k] ? 1 : 0;
    // offsets into the pools
    w.o_pose = pk.K_total;
    w.o_lm = pk.L_total;
    w.o_lmptr = pk.lmptr_total;
    w.o_obs = pk.N_total;
    w.o_kfptr = pk.kfptr_total;
    w.o_ws = pk.ws_total;
    w.o_out = pk.out_total;
    w.o_tr = pk.tr_total;
    w.tr_cap = (w.max_iter + 1) * w.rounds;  // every Summary::iterations entry of every round
    pk.tr_total += w.tr_cap;
    BaWsLayout WL = ba_ws_layout(K, L, N);
    pk.ws_total += WL.total + (int64_t)ba_ws_extra_doubles() + (int64_t)ba_phase_doubles(K, L, N, w.T);
    pk.ws_total = (pk.ws_total + 31) & ~(int64_t)31;
    pk.out_total += ba_out_layout(K, L, N).total;
    pk.K_total += K;
    pk.L_total += L;
    pk.N_total += N;
    pk.lmptr_total += L + 1;
    pk.kfptr_total += K + 1;
    pk.win.push_back(w);
    return VIO_OK;
}

void layout_regions(Packed& pk, int n, bool cluster) {
    BaRegions& R = pk.R;
    size_t o = 0;
    auto take = [&o](size_t bytes) {
        const size_t at = o;
        o = (o + std::max<size_t>(bytes, 16) + 255) & ~(size_t)255;
        return at;
    };
    R.win = take(sizeof(BaWin) * (size_t)n);
    R.pose_raw = take(sizeof(double) * 24 * (size_t)pk.K_total);
    R.kf_const = take((size_t)pk.K_total);
    R.lm_xyz0 = take(sizeof(double) * 3 * (size_t)pk.L_total);
    R.lm_var = take((size_t)pk.L_total);
    R.lm_marg = take((size_t)pk.L_total);
    R.lm_ptr = take(sizeof(int32_t) * (size_t)pk.lmptr_total);
    R.obs_kf = take(sizeof(int32_t) * (size_t)pk.N_total);
    R.obs_lm = take(sizeof(int32_t) * (size_t)pk.N_total);
    R.obs_uv = take(sizeof(float) * 2 * (size_t)pk.N_total);
    R.kf_ptr = take(sizeof(int32_t) * (size_t)pk.kfptr_total);
    R.kf_obs = take(sizeof(int32_t) * (size_t)pk.N_total);
    R.preint = take(sizeof(vio_preint) * (size_t)pk.K_total);
    R.preint_valid = take((size_t)pk.K_total);
    R.vel0 = take(sizeof(double) * 3 * (size_t)pk.K_total);
    R.obs_perm = take(sizeof(int32_t) * (size_t)pk.N_total);
    R.in_bytes = o;
    R.out_begin = o;
    R.i32 = take(sizeof(int32_t) * SI_COUNT * (size_t)n);
    R.sum = take(sizeof(double) * SD_COUNT * (size_t)n);
    R.out = take(sizeof(double) * (size_t)pk.out_total);
    R.trace = take(sizeof(vio_ba_iteration) * (size_t)pk.tr_total);
    R.u8 = take((size_t)pk.N_total);
    R.bad = take((size_t)pk.L_total);
    R.csync = cluster ? take(sizeof(int) * PH_SYNC_INTS * (size_t)n) : 0;
    R.out_bytes = o - R.out_begin;
    R.ws = take(sizeof(double) * (size_t)pk.ws_total);
    R.total = o;
}

// Writes window w's arrays into the input staging image (base = byte 0 of the inputs region): poses,
// landmarks, observations in landmark order (a counting sort, stable: the caller's order within a landmark)
// with their CSR, the per-keyframe observation lists, and the sorted position -> caller's index map.
void fill_window(const vio_ba_problem& p, const BaWin& w, const BaRegions& R, uint8_t* base, std::vector<int32_t>& fillv) {
    const int K = w.K, L = w.L, N = w.N;
    const bool vi = w.is_vi, pnp = w.is_pnp;
    double* pose_raw = reinterpret_cast<double*>(base + R.pose_raw) + 24 * w.o_pose;
    uint8_t* kf_const = base + R.kf_const + w.o_pose;
    vio_preint* preint = reinterpret_cast<vio_preint*>(base + R.preint) + w.o_pose;
    uint8_t* preint_valid = base + R.preint_valid + w.o_pose;
    double* vel0 = reinterpret_cast<double*>(base + R.vel0) + 3 * w.o_pose;
    for (int k = 0; k < K; ++k) {
        double* q = pose_raw + 24 * k;
        std::memcpy(q, p.T_wb_init[k].R, 9 * sizeof(double));
        std::memcpy(q + 9, p.T_wb_init[k].t, 3 * sizeof(double));
        std::memcpy(q + 12, p.T_cb[k].R, 9 * sizeof(double));
        std::memcpy(q + 21, p.T_cb[k].t, 3 * sizeof(double));
        kf_const[k] = p.kf_const[k] ? 1 : 0;
        if (vi) {
            preint[k] = p.preint[k];
            preint_valid[k] = k >= 1 && p.preint_valid[k] ? 1 : 0;
            for (int i = 0; i < 3; ++i) vel0[3 * k + i] = p.vel[3 * k + i];
        } else {
            std::memset(&preint[k], 0, sizeof(vio_preint));
            preint_valid[k] = 0;
            for (int i = 0; i < 3; ++i) vel0[3 * k + i] = 0.0;
        }
    }
    // landmark CSR (counts, then the exclusive scan)
    int32_t* lptr = reinterpret_cast<int32_t*>(base + R.lm_ptr) + w.o_lmptr;
    std::fill(lptr, lptr + L + 1, 0);
    for (int o = 0; o < N; ++o) lptr[p.obs_lm[o] + 1]++;
    for (int l = 0; l < L; ++l) lptr[l + 1] += lptr[l];
    if (L > 0) std::memcpy(reinterpret_cast<double*>(base + R.lm_xyz0) + 3 * w.o_lm, p.lm_xyz, sizeof(double) * 3 * L);
    uint8_t* lm_var = base + R.lm_var + w.o_lm;
    uint8_t* lm_marg = base + R.lm_marg + w.o_lm;
    const uint8_t* marg = pnp ? p.lm_const : p.lm_marg;
    for (int l = 0; l < L; ++l) {
        // a landmark is a free parameter when it is not constant and some observation uses it
        lm_var[l] = !pnp && !p.lm_const[l] && lptr[l + 1] > lptr[l] ? 1 : 0;
        lm_marg[l] = marg ? (marg[l] ? 1 : 0) : 0;
    }
    // observations sorted by landmark, stable
    int32_t* perm = reinterpret_cast<int32_t*>(base + R.obs_perm) + w.o_obs;
    fillv.assign(lptr, lptr + L);
    for (int o = 0; o < N; ++o) perm[fillv[p.obs_lm[o]]++] = o;
    int32_t* obs_kf = reinterpret_cast<int32_t*>(base + R.obs_kf) + w.o_obs;
    int32_t* obs_lm = reinterpret_cast<int32_t*>(base + R.obs_lm) + w.o_obs;
    float* obs_uv = reinterpret_cast<float*>(base + R.obs_uv) + 2 * w.o_obs;
    int32_t* kptr = reinterpret_cast<int32_t*>(base + R.kf_ptr) + w.o_kfptr;
    std::fill(kptr, kptr + K + 1, 0);
    for (int q = 0; q < N; ++q) {
        const int o = perm[q];
        obs_kf[q] = p.obs_kf[o];
        obs_lm[q] = p.obs_lm[o];
        obs_uv[2 * q] = p.obs_uv[2 * o];
        obs_uv[2 * q + 1] = p.obs_uv[2 * o + 1];
        kptr[obs_kf[q] + 1]++;
    }
    for (int k = 0; k < K; ++k) kptr[k + 1] += kptr[k];
    int32_t* kobs = reinterpret_cast<int32_t*>(base + R.kf_obs) + w.o_obs;
    fillv.assign(kptr, kptr + K);
    for (int q = 0; q < N; ++q) kobs[fillv[obs_kf[q]]++] = q;
}

}  // namespace

// device image of a batch
struct BaDevice {
    int n = 0;
    Packed pk;
    void* mem = nullptr;                  // the batch's allocation (owned: vio_ba_batch); one-shot solves use
                                          // the context's arena
    std::vector<uint8_t> stage_own;       // vio_ba_batch: the input image (kept: set_preint, result scatter)
    uint8_t* stage = nullptr;             // the input image the batch was uploaded from
    BaPools P{};
    void* prof_buf = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    hipGraphExec_t phase_graph = nullptr;  // the captured phase-kernel sequence of this batch
    hipStream_t lane_st[kPhLanesMax - 1] = {};  // side streams of the phase route's sub-batches
    hipEvent_t lane_ev[kPhLanesMax] = {};       // their fork / join events
    bool reusable = false;                 // vio_ba_batch: replayed many times (graph); one-shot solves launch directly
    int cluster_C = 0;                     // cluster route: workgroups per window (0: another route)
    double ms_sum = 0.0;
    int ms_count = 0;
    bool timing_pending = false;
};

static bool env_flag(const char* name) {
    const char* e = std::getenv(name);
    return e && e[0] == '1';
}
// the cluster route (one persistent launch, ba_phases.inc ph_cluster_kernel) for batches of up to
// kClusterMaxWindows windows: a window's serial chain (prep, solve) then pays no kernel boundaries and
// its Schur groups overlap the step control / bookkeeping; larger batches fill the chip with the phase
// kernels
constexpr int kClusterMaxWindows = 32;
static bool cluster_wanted(const vio_ctx* ctx, int n) {
    static const bool mono = env_flag("VIO_BA_MONOLITHIC"), phases = env_flag("VIO_BA_PHASES");
    if (ctx->ba_route == VIO_BA_ROUTE_CLUSTER) return true;
    if (ctx->ba_route != VIO_BA_ROUTE_AUTO || mono || phases) return false;
    return n <= kClusterMaxWindows;
}

// internal status of a cluster launch whose bounded hand-off wait expired (the caller falls back to the
// phase route; VIO_EDEVICE if that fails too)
constexpr int kClusterTimeout = 1000;

// Packs problems[0..n) and uploads them: descriptors, route choice, one device allocation (the batch's own,
// or the context's grow-only arena for a one-shot solve), the input image filled on the host (a vector for
// a reusable batch, the context's pinned staging buffer for a one-shot solve) and one host-to-device copy.
// landmark chunks per Schur split-k group (phase route): a full config-4 shard (>= 256 windows) fills the
// chip with 2 groups per window and halves ph_solve's partial sums; smaller batches keep more, shorter
// groups (latency): 3 below 64 windows, 5 up to 255 (sweep of 2/3/4/5/10 at 1..256 windows,
// profiles/r4e_gs_sweep.log); the cluster route: one chunk per group, the group's member owns its landmarks
static int schur_group_size(int n, bool cluster) {
    const char* gse = std::getenv("VIO_BA_SCHUR_GS");  // experiment override
    return cluster ? 1 : gse ? std::max(1, std::atoi(gse)) : n >= 256 ? 10 : n >= 64 ? 5 : 3;
}

static int pack_upload(vio_ctx* ctx, BaDevice& d, const vio_ba_problem* probs, int n, bool allow_cluster) {
    Packed& pk = d.pk;
    d.n = n;
    pk.win.reserve(n);
    std::vector<uint32_t> scratch;
    for (int i = 0; i < n; ++i)
        if (int rc = analyze_window(ctx, probs[i], pk, scratch)) return rc;
    static const int cmax = [] {
        const char* v = std::getenv("VIO_BA_CLUSTER_C");  // experiment override: members per window
        return v ? std::atoi(v) : 0;
    }();
    // (an explicitly requested cluster route takes whatever members fit: no minimum per landmark chunk)
    const int cm = cmax > 0 ? cmax : ctx->ba_route == VIO_BA_ROUTE_CLUSTER ? (1 << 20) : 0;
    d.cluster_C = allow_cluster && cluster_wanted(ctx, n) ? ba_cluster_members(pk.win.data(), n, cm) : 0;
    const int gs = schur_group_size(n, d.cluster_C > 0);
    for (BaWin& w : pk.win) w.gs = gs;
    layout_regions(pk, n, d.cluster_C > 0);
    const BaRegions& R = pk.R;
    uint8_t* dev = nullptr;
    if (d.reusable) {
        {
            DeviceScope dev_scope(ctx->device);
            VIO_HIP(ctx, dev_scope.err);
            VIO_HIP(ctx, hipMalloc(&d.mem, R.total));
        }
        dev = static_cast<uint8_t*>(d.mem);
        d.stage_own.resize(R.in_bytes);
        d.stage = d.stage_own.data();
    } else {
        dev = static_cast<uint8_t*>(ctx_buffer(ctx, kSlotBaSolve, R.total));
        d.stage = static_cast<uint8_t*>(ctx_host_buffer(ctx, kHostSlotBaIn, R.in_bytes));
        if (!dev || !d.stage) {
            set_error(ctx, "vio_ba_solve: device or pinned host allocation failed");
            return VIO_ENOMEM;
        }
    }
    std::memcpy(d.stage + R.win, pk.win.data(), sizeof(BaWin) * (size_t)n);
    std::vector<int32_t> fillv;
    for (int i = 0; i < n; ++i) fill_window(probs[i], pk.win[i], R, d.stage, fillv);
    BaPools& P = d.P;
    P.win = reinterpret_cast<const BaWin*>(dev + R.win);
    P.pose_raw = reinterpret_cast<const double*>(dev + R.pose_raw);
    P.kf_const = dev + R.kf_const;
    P.lm_xyz0 = reinterpret_cast<const double*>(dev + R.lm_xyz0);
    P.lm_var = dev + R.lm_var;
    P.lm_marg = dev + R.lm_marg;
    P.lm_ptr = reinterpret_cast<const int32_t*>(dev + R.lm_ptr);
    P.obs_kf = reinterpret_cast<const int32_t*>(dev + R.obs_kf);
    P.obs_lm = reinterpret_cast<const int32_t*>(dev + R.obs_lm);
    P.obs_uv = reinterpret_cast<const float*>(dev + R.obs_uv);
    P.kf_ptr = reinterpret_cast<const int32_t*>(dev + R.kf_ptr);
    P.kf_obs = reinterpret_cast<const int32_t*>(dev + R.kf_obs);
    P.preint = reinterpret_cast<const vio_preint*>(dev + R.preint);
    P.preint_valid = dev + R.preint_valid;
    P.vel0 = reinterpret_cast<const double*>(dev + R.vel0);
    P.obs_perm = reinterpret_cast<const int32_t*>(dev + R.obs_perm);
    P.out_i32 = reinterpret_cast<int32_t*>(dev + R.i32);
    P.out_sum = reinterpret_cast<double*>(dev + R.sum);
    P.out = reinterpret_cast<double*>(dev + R.out);
    P.out_trace = reinterpret_cast<vio_ba_iteration*>(dev + R.trace);
    P.out_u8 = dev + R.u8;
    P.out_bad = dev + R.bad;
    P.csync = d.cluster_C ? reinterpret_cast<int*>(dev + R.csync) : nullptr;
    P.ws = reinterpret_cast<double*>(dev + R.ws);
    VIO_DEVICE(ctx);
    VIO_HIP(ctx, hipMemcpyAsync(dev, d.stage, R.in_bytes, hipMemcpyHostToDevice, ctx->stream));
    if (d.reusable) {
        VIO_HIP(ctx, hipEventCreate(&d.ev0));
        VIO_HIP(ctx, hipEventCreate(&d.ev1));
    }
    return VIO_OK;
}

static void free_batch(BaDevice& d) {
    if (d.mem) (void)hipFree(d.mem);
    d.mem = nullptr;
    if (d.prof_buf) (void)hipFree(d.prof_buf);
    d.prof_buf = nullptr;
    if (d.ev0) (void)hipEventDestroy(d.ev0);
    if (d.ev1) (void)hipEventDestroy(d.ev1);
    d.ev0 = d.ev1 = nullptr;
    if (d.phase_graph) (void)hipGraphExecDestroy(d.phase_graph);
    d.phase_graph = nullptr;
    for (hipStream_t& st : d.lane_st)
        if (st) (void)hipStreamDestroy(st), st = nullptr;
    for (hipEvent_t& ev : d.lane_ev)
        if (ev) (void)hipEventDestroy(ev), ev = nullptr;
}

// the cluster route's per-window error words (a bounded hand-off wait that expired), from a host image of
// the hand-off state
static bool cluster_timed_out(const BaDevice& d, const int* sync) {
    for (int i = 0; i < d.n; ++i)
        if (sync[(size_t)PH_SYNC_INTS * i + PH_SYNC_ERR]) return true;
    return false;
}
static int check_cluster(vio_ctx* ctx, BaDevice& d) {
    if (!d.cluster_C || !d.P.csync) return VIO_OK;
    std::vector<int> sync((size_t)PH_SYNC_INTS * d.n);
    VIO_HIP(ctx, hipMemcpyAsync(sync.data(), d.P.csync, sizeof(int) * sync.size(), hipMemcpyDeviceToHost, ctx->stream));
    VIO_HIP(ctx, hipStreamSynchronize(ctx->stream));
    if (cluster_timed_out(d, sync.data())) {
        set_error(ctx, "cluster route: a hand-off wait timed out (workgroups not co-resident?)");
        return kClusterTimeout;
    }
    return VIO_OK;
}

// Fetches the outputs region (one device-to-host copy into the context's pinned staging buffer; the cluster
// route's error words ride along) and waits for it.  kClusterTimeout when a cluster hand-off wait expired.
static int fetch_outputs(vio_ctx* ctx, BaDevice& d, const uint8_t** img) {
    const BaRegions& R = d.pk.R;
    auto* h = static_cast<uint8_t*>(ctx_host_buffer(ctx, kHostSlotBaOut, R.out_bytes));
    if (!h) {
        set_error(ctx, "BA download: pinned host allocation failed");
        return VIO_ENOMEM;
    }
    const uint8_t* dev = reinterpret_cast<const uint8_t*>(d.P.out_i32) - R.i32;  // the region's device base
    VIO_HIP(ctx, hipMemcpyAsync(h, dev + R.out_begin, R.out_bytes, hipMemcpyDeviceToHost, ctx->stream));
    VIO_HIP(ctx, hipStreamSynchronize(ctx->stream));
    *img = h - R.out_begin;  // indexable with the region offsets
    if (d.cluster_C && cluster_timed_out(d, reinterpret_cast<const int*>(*img + R.csync))) {
        set_error(ctx, "cluster route: a hand-off wait timed out (workgroups not co-resident?)");
        return kClusterTimeout;
    }
    return VIO_OK;
}

// scatters the fetched outputs into the callers' buffers (observations back in the caller's order)
static void scatter_outputs(const BaDevice& d, const uint8_t* img, vio_ba_output* outs) {
    const Packed& pk = d.pk;
    const BaRegions& R = pk.R;
    const double* out = reinterpret_cast<const double*>(img + R.out);
    const uint8_t* u8 = img + R.u8;
    const uint8_t* bad = img + R.bad;
    const int32_t* si = reinterpret_cast<const int32_t*>(img + R.i32);
    const double* sd = reinterpret_cast<const double*>(img + R.sum);
    const vio_ba_iteration* tr = reinterpret_cast<const vio_ba_iteration*>(img + R.trace);
    const int32_t* perm_all = reinterpret_cast<const int32_t*>(d.stage + R.obs_perm);
    for (int i = 0; i < d.n; ++i) {
        const BaWin& w = pk.win[i];
        vio_ba_output& o = outs[i];
        BaOutLayout OL = ba_out_layout(w.K, w.L, w.N);
        const double* ob = out + w.o_out;
        if (o.T_wb)
            for (int k = 0; k < w.K; ++k) {
                std::memcpy(o.T_wb[k].R, ob + OL.T_wb + 12 * k, 9 * sizeof(double));
                std::memcpy(o.T_wb[k].t, ob + OL.T_wb + 12 * k + 9, 3 * sizeof(double));
            }
        if (o.lm_xyz) std::memcpy(o.lm_xyz, ob + OL.lm, sizeof(double) * 3 * w.L);
        const int32_t* perm = perm_all + w.o_obs;
        if (o.obs_chi2)
            for (int q = 0; q < w.N; ++q) o.obs_chi2[perm[q]] = ob[OL.chi2 + q];
        if (o.obs_outlier)
            for (int q = 0; q < w.N; ++q) o.obs_outlier[perm[q]] = u8[w.o_obs + q];
        if (o.lm_bad) std::memcpy(o.lm_bad, bad + w.o_lm, w.L);
        if (w.is_vi) {
            if (o.vel) std::memcpy(o.vel, ob + OL.vel, sizeof(double) * 3 * w.K);
            if (o.bg) std::memcpy(o.bg, ob + OL.bias, sizeof(double) * 3);
            if (o.ba) std::memcpy(o.ba, ob + OL.bias + 3, sizeof(double) * 3);
        }
        if (o.summary) {
            vio_ba_summary& s = *o.summary;
            std::memset(&s, 0, sizeof s);
            const int32_t* a = si + SI_COUNT * i;
            const double* b = sd + SD_COUNT * i;
            s.success = a[SI_SUCCESS];
            s.termination = a[SI_TERM];
            s.iterations = a[SI_ITERS];
            s.num_successful_steps = a[SI_NSUCC];
            s.num_unsuccessful_steps = a[SI_NUNSUCC];
            s.num_inliers = a[SI_NIN];
            s.num_outliers = a[SI_NOUT];
            s.num_bad_lm = a[SI_NBAD];
            s.initial_cost = b[SD_INIT];
            s.final_cost = b[SD_FINAL];
            s.fixed_cost = b[SD_FIXED];
        }
        if (o.trace && o.trace_cap > 0) {
            const int n_it = std::min(std::min(si[SI_COUNT * i + SI_ITERS], w.tr_cap), o.trace_cap);
            for (int q = 0; q < n_it; ++q) o.trace[q] = tr[w.o_tr + q];
        }
    }
}

static int download_batch(vio_ctx* ctx, BaDevice& d, vio_ba_output* outs) {
    const uint8_t* img = nullptr;
    if (int rc = fetch_outputs(ctx, d, &img)) return rc;
    scatter_outputs(d, img, outs);
    return VIO_OK;
}

// LocalBA / BA / VIBA windows run as the phase-kernel sequence (ba_phases.inc): a window's
// observation walks spread over many workgroups per phase, so it is the faster route at every batch
// size measured (1 window: 1.42 vs 1.70 ms; the 256-window config-4 shard: 3.59 vs 3.75 ms per 10
// iterations).  PnP windows (outlier rounds inside one solve) run in ba_window_kernel, the
// single-kernel solver.  Within a route a window's result does not depend on the batch it is in.
// vio_ctx_set_ba_route / VIO_BA_MONOLITHIC=1 / VIO_BA_PHASES=1 select a route explicitly (A/B runs,
// tests); per-window phase profiling runs on ba_window_kernel.
static bool force_monolithic(const vio_ctx* ctx, const BaDevice& d) {
    static const bool mono = env_flag("VIO_BA_MONOLITHIC"), phases = env_flag("VIO_BA_PHASES");
    if (phases || ctx->ba_route == VIO_BA_ROUTE_PHASES) return false;
    return mono || d.P.prof || ctx->ba_route == VIO_BA_ROUTE_SINGLE_KERNEL;
}

static int launch(vio_ctx* ctx, BaDevice& d, bool timed) {
    VIO_DEVICE(ctx);
    if (timed) VIO_HIP(ctx, hipEventRecord(d.ev0, ctx->stream));
    bool any_pnp = false, any_other = false;
    for (const BaWin& w : d.pk.win) (w.is_pnp ? any_pnp : any_other) = true;
    const bool cluster = any_other && d.cluster_C > 0;
    const bool phases = !cluster && any_other && !force_monolithic(ctx, d);
    d.P.route = phases || cluster ? 1 : 0;
    // IMU candidate terms beside the back-substitution walk (ph_back_x's extra workgroup) up to 64 windows
    // (a window's serial path is then shorter: 32 windows 1.436 -> 1.342 ms, 64 windows 1.677 -> 1.633 ms,
    // profiles/r5_imu_back_sweep.log); in ph_solve for larger batches (256 windows: 3.04 against 3.17 ms)
    static const int imu_back_max = [] {
        const char* v = std::getenv("VIO_BA_IMU_BACK_MAX");  // experiment override
        return v ? std::atoi(v) : 64;
    }();
    d.P.imu_in_back = cluster || d.n <= imu_back_max ? 1 : 0;  // cluster: the leader, beside the walks
    static const int chol_variant = [] {
        const char* v = std::getenv("VIO_BA_CHOL");  // experiment override: 0 chol6_solve2, 2 chol_tile_solve2
        return v ? std::atoi(v) : 2;  // (chol_tile_solve2 where its tile geometry is instantiated, else chol6_solve2)
    }();
    d.P.chol_variant = chol_variant;
    d.P.win_base = 0;
    // sub-batches of the phase route on their own streams (launch_ba_phases): large batches only
    static const int lanes_env = [] {
        const char* v = std::getenv("VIO_BA_LANES");  // experiment override
        return v ? std::max(1, std::min(kPhLanesMax, std::atoi(v))) : 0;
    }();
    // (measured at 256 windows: 2 lanes 0.99x, 3 lanes 0.71x, 4 lanes 0.93x of one stream; 32 windows,
    // 2 lanes 0.88x -- not on by default)
    int lanes = lanes_env ? lanes_env : 1;
    for (int l = 0; l < lanes; ++l) {
        if (l > 0 && !d.lane_st[l - 1] && hipStreamCreateWithFlags(&d.lane_st[l - 1], hipStreamNonBlocking) != hipSuccess) {
            d.lane_st[l - 1] = nullptr;
            lanes = l;
            break;
        }
        if (!d.lane_ev[l] && hipEventCreateWithFlags(&d.lane_ev[l], hipEventDisableTiming) != hipSuccess) {
            d.lane_ev[l] = nullptr;
            lanes = std::max(1, l);
            break;
        }
    }
    hipError_t e = hipSuccess;
    const char* what = "ba_window_kernel launch";
    if (cluster) {
        what = "ph_cluster_kernel";
        if (d.reusable && !d.phase_graph) {  // the kernel alone is captured; its hand-off words are cleared per run
            hipGraph_t g = nullptr;
            e = hipStreamBeginCapture(ctx->stream, hipStreamCaptureModeThreadLocal);
            if (e == hipSuccess) {
                hipError_t el = launch_ba_cluster(d.P, d.n, d.cluster_C, ctx->stream);
                e = hipStreamEndCapture(ctx->stream, &g);
                if (el != hipSuccess) e = el;
            }
            if (e == hipSuccess) e = hipGraphInstantiate(&d.phase_graph, g, nullptr, nullptr, 0);
            if (g) (void)hipGraphDestroy(g);
        }
        if (e == hipSuccess) e = ba_cluster_prelaunch(d.P, d.n, ctx->stream);
        if (e == hipSuccess) {
            // every member of every window resident at once, also beside other threads' persistent launches
            ResidencyGuard rg(ctx->stream, d.cluster_C * d.n);
            e = rg.status();
            if (e == hipSuccess) e = d.reusable ? hipGraphLaunch(d.phase_graph, ctx->stream)
                                                : launch_ba_cluster(d.P, d.n, d.cluster_C, ctx->stream);
            if (e == hipSuccess) e = rg.commit();
        }
    } else if (phases) {
        // ~70 launches per solve: a reusable batch captures them once into a graph (same arguments
        // every run) and replays it; a one-shot solve launches them directly
        e = ba_phases_prepare(d.pk.win.data(), d.n);
        if (e != hipSuccess) what = "hipFuncSetAttribute(phase kernels)";
        if (e == hipSuccess && !d.reusable) {
            e = launch_ba_phases(d.P, d.pk.win.data(), d.n, ctx->stream, lanes, d.lane_st, d.lane_ev);
            if (e != hipSuccess) what = ba_phases_failed_launch();
        } else if (e == hipSuccess && !d.phase_graph) {
            hipGraph_t g = nullptr;
            e = hipStreamBeginCapture(ctx->stream, hipStreamCaptureModeThreadLocal);
            if (e == hipSuccess) {
                hipError_t el = launch_ba_phases(d.P, d.pk.win.data(), d.n, ctx->stream, lanes, d.lane_st, d.lane_ev);
                e = hipStreamEndCapture(ctx->stream, &g);
                if (el != hipSuccess) e = el, what = ba_phases_failed_launch();
            }
            if (e == hipSuccess) e = hipGraphInstantiate(&d.phase_graph, g, nullptr, nullptr, 0);
            if (g) (void)hipGraphDestroy(g);
        }
        if (e == hipSuccess && d.reusable) e = hipGraphLaunch(d.phase_graph, ctx->stream);
    }
    // the single-kernel solver: PnP windows, or every window when neither batched route runs (the cluster
    // route has no window for it otherwise: an empty launch would cost the batch a kernel boundary)
    if (e == hipSuccess && (any_pnp || (!phases && !cluster))) e = launch_ba_windows(d.P, d.n, ctx->stream);
    if (e != hipSuccess) return hip_fail(ctx, e, what);
    if (timed) {
        VIO_HIP(ctx, hipEventRecord(d.ev1, ctx->stream));
        d.timing_pending = true;
    }
    return VIO_OK;
}

static int solve_one_shot(vio_ctx* ctx, const vio_ba_problem* probs, vio_ba_output* outs, int n, bool allow_cluster) {
    BaDevice d;
    d.reusable = false;
    int rc = pack_upload(ctx, d, probs, n, allow_cluster);
    if (rc == VIO_OK) rc = launch(ctx, d, false);
    if (rc == VIO_OK) rc = download_batch(ctx, d, outs);
    if (rc != VIO_OK) (void)hipStreamSynchronize(ctx->stream);  // the arena may be reused or freed next
    free_batch(d);
    return rc;
}

// A reusable batch whose last cluster run timed out moves to the phase route for good: the descriptors get
// the phase route's Schur group size, the captured cluster graph goes, and the batch runs again (its inputs
// are untouched: every run starts from them).  The caller then reads the phase route's results.
static int batch_fall_back(vio_ctx* ctx, BaDevice& d) {
    d.cluster_C = 0;
    d.P.csync = nullptr;
    const int gs = schur_group_size(d.n, false);
    for (BaWin& w : d.pk.win) w.gs = gs;
    std::memcpy(d.stage + d.pk.R.win, d.pk.win.data(), sizeof(BaWin) * (size_t)d.n);
    VIO_DEVICE(ctx);
    VIO_HIP(ctx, hipMemcpyAsync((void*)d.P.win, d.stage + d.pk.R.win, sizeof(BaWin) * (size_t)d.n,
                                hipMemcpyHostToDevice, ctx->stream));
    if (d.phase_graph) (void)hipGraphExecDestroy(d.phase_graph);
    d.phase_graph = nullptr;
    d.timing_pending = false;  // (the timed-out run's time is not a solve's)
    if (int rc = launch(ctx, d, false)) return rc;
    VIO_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return VIO_OK;
}

}  // namespace vio360

using namespace vio360;

struct vio_ba_batch {
    vio_ctx* ctx;
    BaDevice dev;
};

extern "C" {

int vio_abi_version(void) { return VIO360_ABI_VERSION; }

int vio_ctx_set_ba_route(vio_ctx* ctx, int route) {
    if (!ctx || route < VIO_BA_ROUTE_AUTO || route > VIO_BA_ROUTE_CLUSTER) return VIO_EINVAL;
    ctx->ba_route = route;
    return VIO_OK;
}

int vio_lie_eval(vio_ctx* ctx, int op, const double* in, int n, double* out) {
    static const int kIn[5] = {3, 6, 9, 3, 9}, kOut[5] = {9, 12, 3, 9, 3};
    if (!ctx || op < VIO_LIE_SO3_EXP || op > VIO_LIE_SO3D_LOG || n < 0 || (n > 0 && (!in || !out))) return VIO_EINVAL;
    if (n == 0) return VIO_OK;
    const size_t bi = sizeof(double) * kIn[op] * (size_t)n, bo = sizeof(double) * kOut[op] * (size_t)n;
    auto* d = static_cast<char*>(ctx_buffer(ctx, kSlotLie, bi + bo));
    if (!d) {
        set_error(ctx, "vio_lie_eval: device allocation failed");
        return VIO_ENOMEM;
    }
    VIO_DEVICE(ctx);
    double* din = reinterpret_cast<double*>(d);
    double* dout = reinterpret_cast<double*>(d + bi);
    VIO_HIP(ctx, hipMemcpyAsync(din, in, bi, hipMemcpyHostToDevice, ctx->stream));
    VIO_HIP(ctx, op <= VIO_LIE_IMU_LOG ? launch_lie_ba(op, din, dout, n, ctx->stream)
                                       : launch_lie_init(op, din, dout, n, ctx->stream));
    VIO_HIP(ctx, hipMemcpyAsync(out, dout, bo, hipMemcpyDeviceToHost, ctx->stream));
    VIO_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return VIO_OK;
}

static std::string g_create_error;

int vio_layout_check(void) {
    const uint64_t ba = ba_layout_sig(), gba = gba_layout_sig_ba_global();
    return ba == ba_layout_sig_ba_kernel() && ba == ba_layout_sig_ba_cluster() && ba == ba_layout_sig_ba_global_host() &&
                   gba == gba_layout_sig_ba_kernel() && gba == gba_layout_sig_ba_global_host()
               ? VIO_OK
               : VIO_EDEVICE;
}

int vio_ctx_create(int device, vio_ctx** out) {
    if (!out) return VIO_EINVAL;
    *out = nullptr;
    if (vio_layout_check() != VIO_OK) {
        g_create_error = "translation units disagree on the BaWin/BaPools/GbaArgs layout (stale object: rebuild)";
        return VIO_EDEVICE;
    }
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess || n <= 0) {
        g_create_error = "no HIP device available";
        return VIO_EDEVICE;
    }
    if (device < 0 || device >= n) {
        g_create_error = "device index out of range";
        return VIO_EINVAL;
    }
    DeviceScope dev_scope(device);
    if (dev_scope.err != hipSuccess) {
        g_create_error = "hipSetDevice failed";
        return VIO_EDEVICE;
    }
    vio_ctx* c = new vio_ctx();
    c->device = device;
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        g_create_error = "hipStreamCreate failed";
        return VIO_EDEVICE;
    }
    *out = c;
    return VIO_OK;
}

void vio_ctx_destroy(vio_ctx* ctx) {
    if (!ctx) return;
    DeviceScope _vio_dev_scope(ctx->device);
    (void)hipStreamSynchronize(ctx->stream);
    ctx->gba_cache.reset();  // its graph / side stream before the buffers and the stream
    for (void* p : ctx->bufs)
        if (p) (void)hipFree(p);
    for (void* p : ctx->hbufs)
        if (p) (void)hipHostFree(p);
    for (hipEvent_t e : ctx->imu_ev)
        if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : ctx->tri_ev)
        if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : ctx->rsz_ev)
        if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : ctx->init_ev)
        if (e) (void)hipEventDestroy(e);
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    delete ctx;
}

const char* vio_ctx_last_error(const vio_ctx* ctx) {
    return ctx ? ctx->last_error.c_str() : g_create_error.c_str();
}

int vio_ba_batch_create(vio_ctx* ctx, const vio_ba_problem* probs, int n, vio_ba_batch** out) {
    if (!ctx || !probs || n <= 0 || !out) return VIO_EINVAL;
    *out = nullptr;
    DeviceScope _vio_dev_scope(ctx->device);
    vio_ba_batch* b = new vio_ba_batch();
    b->ctx = ctx;
    b->dev.reusable = true;
    int rc = pack_upload(ctx, b->dev, probs, n, true);
    if (rc != VIO_OK) {
        (void)hipStreamSynchronize(ctx->stream);
        free_batch(b->dev);
        delete b;
        return rc;
    }
    *out = b;
    return VIO_OK;
}

int vio_ba_batch_run(vio_ba_batch* b) {
    if (!b) return VIO_EINVAL;
    vio_ctx* ctx = b->ctx;
    VIO_DEVICE(ctx);
    if (b->dev.timing_pending) {  // fold the previous run's time in before re-recording
        VIO_HIP(ctx, hipEventSynchronize(b->dev.ev1));
        float ms = 0.f;
        VIO_HIP(ctx, hipEventElapsedTime(&ms, b->dev.ev0, b->dev.ev1));
        b->dev.ms_sum += ms;
        b->dev.ms_count++;
        b->dev.timing_pending = false;
    }
    return launch(ctx, b->dev, true);
}

int vio_ba_batch_set_preint(vio_ba_batch* b, const vio_preint* src, int count, int on_device) {
    if (!b || (count > 0 && !src)) return VIO_EINVAL;
    vio_ctx* ctx = b->ctx;
    const Packed& pk = b->dev.pk;
    if (count != (int)pk.K_total) {
        set_error(ctx, "vio_ba_batch_set_preint: count must be the batch's total keyframe count");
        return VIO_EINVAL;
    }
    if (count == 0) return VIO_OK;
    const size_t bytes = sizeof(vio_preint) * (size_t)count;
    VIO_DEVICE(ctx);
    if (on_device) {
        VIO_HIP(ctx, hipMemcpyAsync((void*)b->dev.P.preint, src, bytes, hipMemcpyDeviceToDevice, ctx->stream));
    } else {
        uint8_t* stage = b->dev.stage + pk.R.preint;  // the batch's input image outlives the async upload
        std::memcpy(stage, src, bytes);
        VIO_HIP(ctx, hipMemcpyAsync((void*)b->dev.P.preint, stage, bytes, hipMemcpyHostToDevice, ctx->stream));
    }
    return VIO_OK;
}

int vio_ba_batch_sync(vio_ba_batch* b) {
    if (!b) return VIO_EINVAL;
    VIO_DEVICE(b->ctx);
    VIO_HIP(b->ctx, hipStreamSynchronize(b->ctx->stream));
    int rc = check_cluster(b->ctx, b->dev);
    if (rc == kClusterTimeout) rc = batch_fall_back(b->ctx, b->dev);
    return rc;
}

int vio_ba_batch_download(vio_ba_batch* b, vio_ba_output* outs) {
    if (!b || !outs) return VIO_EINVAL;
    VIO_DEVICE(b->ctx);
    int rc = download_batch(b->ctx, b->dev, outs);
    if (rc == kClusterTimeout && (rc = batch_fall_back(b->ctx, b->dev)) == VIO_OK) rc = download_batch(b->ctx, b->dev, outs);
    return rc == kClusterTimeout ? VIO_EDEVICE : rc;
}

int vio_ba_batch_kernel_ms(vio_ba_batch* b, double* avg_ms, int* count) {
    if (!b || !avg_ms || !count) return VIO_EINVAL;
    VIO_DEVICE(b->ctx);
    if (b->dev.timing_pending) {
        VIO_HIP(b->ctx, hipEventSynchronize(b->dev.ev1));
        float ms = 0.f;
        VIO_HIP(b->ctx, hipEventElapsedTime(&ms, b->dev.ev0, b->dev.ev1));
        b->dev.ms_sum += ms;
        b->dev.ms_count++;
        b->dev.timing_pending = false;
    }
    *count = b->dev.ms_count;
    *avg_ms = b->dev.ms_count ? b->dev.ms_sum / b->dev.ms_count : 0.0;
    b->dev.ms_sum = 0.0;
    b->dev.ms_count = 0;
    return VIO_OK;
}

int vio_ba_batch_route(vio_ba_batch* b, int* route, int* workgroups_per_window) {
    if (!b || !route) return VIO_EINVAL;
    bool any_other = false;
    for (const BaWin& w : b->dev.pk.win) any_other |= !w.is_pnp;
    *route = any_other && b->dev.cluster_C > 0 ? VIO_BA_ROUTE_CLUSTER
             : any_other && !force_monolithic(b->ctx, b->dev) ? VIO_BA_ROUTE_PHASES
                                                                : VIO_BA_ROUTE_SINGLE_KERNEL;
    if (workgroups_per_window) *workgroups_per_window = b->dev.cluster_C;
    return VIO_OK;
}

int vio_ba_batch_profile(vio_ba_batch* b, int enable) {
    if (!b) return VIO_EINVAL;
    VIO_DEVICE(b->ctx);
    if (enable && !b->dev.prof_buf) {
        VIO_HIP(b->ctx, hipMalloc(&b->dev.prof_buf, sizeof(unsigned long long) * VIO_BA_PROF_SLOTS * b->dev.n));
        VIO_HIP(b->ctx, hipMemsetAsync(b->dev.prof_buf, 0, sizeof(unsigned long long) * VIO_BA_PROF_SLOTS * b->dev.n, b->ctx->stream));
    }
    b->dev.P.prof = enable ? (unsigned long long*)b->dev.prof_buf : nullptr;
    if (b->dev.phase_graph) {  // the captured phase sequence holds the old kernel arguments
        (void)hipGraphExecDestroy(b->dev.phase_graph);
        b->dev.phase_graph = nullptr;
    }
    return VIO_OK;
}

int vio_ba_batch_phase_cycles(vio_ba_batch* b, unsigned long long* out) {
    if (!b || !out || !b->dev.prof_buf) return VIO_EINVAL;
    VIO_DEVICE(b->ctx);
    constexpr int NS = VIO_BA_PROF_SLOTS;
    std::vector<unsigned long long> v(NS * b->dev.n);
    VIO_HIP(b->ctx, hipMemcpyAsync(v.data(), b->dev.prof_buf, sizeof(unsigned long long) * v.size(),
                                   hipMemcpyDeviceToHost, b->ctx->stream));
    VIO_HIP(b->ctx, hipStreamSynchronize(b->ctx->stream));
    for (int s = 0; s < NS; ++s) {
        out[s] = 0;
        for (int i = 0; i < b->dev.n; ++i) out[s] += v[NS * i + s];
    }
    return VIO_OK;
}

void vio_ba_batch_destroy(vio_ba_batch* b) {
    if (!b) return;
    DeviceScope _vio_dev_scope(b->ctx->device);
    (void)hipStreamSynchronize(b->ctx->stream);
    free_batch(b->dev);
    delete b;
}

size_t vio_ba_record_bytes(int num_kf, int num_lm, int num_obs) {
    if (num_kf < 0 || num_lm < 0 || num_obs < 0) return 0;
    return (size_t)rec_layout(num_kf, num_lm, num_obs).total;
}

int vio_ba_batch_record_bytes(vio_ba_batch* b, size_t* bytes) {
    if (!b || !bytes) return VIO_EINVAL;
    size_t m = 0;
    for (const BaWin& w : b->dev.pk.win) m = std::max(m, (size_t)rec_layout(w.K, w.L, w.N).total);
    *bytes = m;
    return VIO_OK;
}

int vio_ba_batch_pack(vio_ba_batch* b, void* dst, int on_device) {
    if (!b || !dst) return VIO_EINVAL;
    vio_ctx* ctx = b->ctx;
    size_t rb = 0;
    vio_ba_batch_record_bytes(b, &rb);
    VIO_DEVICE(ctx);
    uint8_t* d = static_cast<uint8_t*>(dst);
    if (!on_device) {
        d = static_cast<uint8_t*>(ctx_buffer(ctx, kSlotRecords, rb * b->dev.n));
        if (!d) { set_error(ctx, "vio_ba_batch_pack: device allocation failed"); return VIO_ENOMEM; }
    }
    hipError_t e = launch_ba_pack(b->dev.P, b->dev.n, d, (int64_t)rb, ctx->stream);
    if (e != hipSuccess) return hip_fail(ctx, e, "ba_pack_kernel");
    if (!on_device) {
        VIO_HIP(ctx, hipMemcpyAsync(dst, d, rb * b->dev.n, hipMemcpyDeviceToHost, ctx->stream));
        VIO_HIP(ctx, hipStreamSynchronize(ctx->stream));
    }
    return VIO_OK;
}

int vio_ba_record_unpack(const void* record, size_t record_bytes, vio_ba_output* out) {
    if (!record || !out || record_bytes < 16) return VIO_EINVAL;
    const uint8_t* rec = static_cast<const uint8_t*>(record);
    int32_t hdr[4];
    std::memcpy(hdr, rec, sizeof hdr);
    const int K = hdr[0], L = hdr[1], N = hdr[2];
    if (K <= 0 || L < 0 || N < 0 || hdr[3] != VIO_BA_RECORD_VERSION) return VIO_EINVAL;
    const RecLayout R = rec_layout(K, L, N);
    if ((uint64_t)R.total > (uint64_t)record_bytes) return VIO_EINVAL;  // the header's layout overruns the record
    if (out->T_wb)
        for (int k = 0; k < K; ++k) {
            std::memcpy(out->T_wb[k].R, rec + R.T + 96 * k, 9 * sizeof(double));
            std::memcpy(out->T_wb[k].t, rec + R.T + 96 * k + 72, 3 * sizeof(double));
        }
    if (out->lm_xyz) std::memcpy(out->lm_xyz, rec + R.lm, 24 * (size_t)L);
    if (out->vel) std::memcpy(out->vel, rec + R.vel, 24 * (size_t)K);
    if (out->bg) std::memcpy(out->bg, rec + R.bias, 24);
    if (out->ba) std::memcpy(out->ba, rec + R.bias + 24, 24);
    if (out->obs_outlier) std::memcpy(out->obs_outlier, rec + R.outl, N);
    if (out->lm_bad) std::memcpy(out->lm_bad, rec + R.bad, L);
    if (out->summary) {
        int32_t a[SI_COUNT];
        double d[SD_COUNT];
        std::memcpy(a, rec + R.si, sizeof a);
        std::memcpy(d, rec + R.sd, sizeof d);
        vio_ba_summary& s = *out->summary;
        std::memset(&s, 0, sizeof s);
        s.success = a[SI_SUCCESS];
        s.termination = a[SI_TERM];
        s.iterations = a[SI_ITERS];
        s.num_successful_steps = a[SI_NSUCC];
        s.num_unsuccessful_steps = a[SI_NUNSUCC];
        s.num_inliers = a[SI_NIN];
        s.num_outliers = a[SI_NOUT];
        s.num_bad_lm = a[SI_NBAD];
        s.initial_cost = d[SD_INIT];
        s.final_cost = d[SD_FINAL];
        s.fixed_cost = d[SD_FIXED];
    }
    return VIO_OK;
}

int vio_ba_solve_batched(vio_ctx* ctx, const vio_ba_problem* probs, vio_ba_output* outs, int n) {
    if (!ctx || !probs || !outs || n <= 0) return VIO_EINVAL;
    VIO_DEVICE(ctx);
    // problems beyond one workgroup's reduced system (K > 16: RunBA over hundreds of keyframes,
    // config 5) take the multi-kernel global path, one problem at a time
    bool any_global = false;
    for (int i = 0; i < n; ++i) any_global |= global_ba_applicable(probs[i]);
    if (any_global) {
        for (int i = 0; i < n; ++i) {
            int rc = global_ba_applicable(probs[i]) ? global_ba_solve(ctx, probs[i], &outs[i])
                                                    : vio_ba_solve_batched(ctx, &probs[i], &outs[i], 1);
            if (rc != VIO_OK) return rc;
        }
        return VIO_OK;
    }
    // one-shot solve (once per keyframe in the reference: Estimator.cpp:763-790 -> RunLocalBA / RunVIBA):
    // the context's grow-only device arena and pinned staging buffers, one host-to-device copy of the
    // packed inputs, one device-to-host copy of the outputs region -- no allocation once the arena fits.
    // A cluster launch whose hand-off wait expired is solved again on the phase route.
    int rc = solve_one_shot(ctx, probs, outs, n, true);
    if (rc == kClusterTimeout) rc = solve_one_shot(ctx, probs, outs, n, false);
    return rc == kClusterTimeout ? VIO_EDEVICE : rc;
}

int vio_ba_solve(vio_ctx* ctx, const vio_ba_problem* prob, vio_ba_output* out) {
    return vio_ba_solve_batched(ctx, prob, out, 1);
}

}  // extern "C"
