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
    size_t cap = std::max<size_t>(bytes, 256);
    if (hipMalloc(&ctx->bufs[slot], cap) != hipSuccess) return nullptr;
    ctx->caps[slot] = cap;
    return ctx->bufs[slot];
}

namespace {

// host image of a packed batch
struct Packed {
    std::vector<BaWin> win;
    std::vector<double> pose_raw, lm_xyz0, vel0;
    std::vector<uint8_t> kf_const, lm_var, lm_marg, preint_valid;
    std::vector<int32_t> lm_ptr, obs_kf, obs_lm, kf_ptr, kf_obs;
    std::vector<float> obs_uv;
    std::vector<vio_preint> preint;
    std::vector<std::vector<int32_t>> perm;  // per window: sorted position -> original obs index
    int64_t ws_total = 0, out_total = 0, N_total = 0, L_total = 0, tr_total = 0;
};

int pack_window(vio_ctx* ctx, const vio_ba_problem& p, Packed& pk) {
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
    for (int o = 0; o < N; ++o) {
        if (p.obs_kf[o] < 0 || p.obs_kf[o] >= K || p.obs_lm[o] < 0 || p.obs_lm[o] >= L) {
            set_error(ctx, "observation index out of range");
            return VIO_EINVAL;
        }
    }
    // one observation per (keyframe, landmark): MapPoint::AddObservation keeps one per frame
    {
        std::vector<int64_t> key(N);
        for (int o = 0; o < N; ++o) key[o] = (int64_t)p.obs_lm[o] * K + p.obs_kf[o];
        std::sort(key.begin(), key.end());
        for (int o = 1; o < N; ++o)
            if (key[o] == key[o - 1]) {
                set_error(ctx, "duplicate (keyframe, landmark) observation");
                return VIO_EINVAL;
            }
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
    std::vector<uint8_t> pose_used(K, 0), lm_used(L, 0), vel_used(K, 0);
    bool bias_used = false;
    for (int o = 0; o < N; ++o) {
        int k = p.obs_kf[o], l = p.obs_lm[o];
        bool kvar = !p.kf_const[k], lvar = !pnp && !p.lm_const[l];
        if (kvar) pose_used[k] = 1;
        if (lvar) lm_used[l] = 1;
    }
    if (vi) {
        for (int k = 1; k < K; ++k) {
            if (!p.preint_valid[k]) continue;
            vel_used[k - 1] = vel_used[k] = 1;
            bias_used = true;
            if (!p.kf_const[k - 1]) pose_used[k - 1] = 1;
            if (!p.kf_const[k]) pose_used[k] = 1;
        }
    }
    int off = 0, P = 0;
    for (int k = 0; k < BA_KMAX; ++k) { w.pose_f[k] = -1; w.vel_f[k] = -1; }
    for (int k = 0; k < K; ++k)
        if (pose_used[k]) { w.pose_f[k] = off; off += 6; P++; }
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
    // offsets
    w.o_pose = (int64_t)pk.kf_const.size();
    w.o_lm = (int64_t)pk.lm_var.size();
    w.o_lmptr = (int64_t)pk.lm_ptr.size();
    w.o_obs = (int64_t)pk.obs_kf.size();
    w.o_kfptr = (int64_t)pk.kf_ptr.size();
    w.o_ws = pk.ws_total;
    w.o_out = pk.out_total;
    w.o_tr = pk.tr_total;
    w.tr_cap = (w.max_iter + 1) * w.rounds;  // every Summary::iterations entry of every round
    pk.tr_total += w.tr_cap;
    BaWsLayout WL = ba_ws_layout(K, L, N);
    pk.ws_total += WL.total + (int64_t)ba_ws_extra_doubles() + (int64_t)ba_phase_doubles(K, L, N, w.T);
    pk.ws_total = (pk.ws_total + 31) & ~(int64_t)31;
    pk.out_total += ba_out_layout(K, L, N).total;
    // poses
    for (int k = 0; k < K; ++k) {
        for (int i = 0; i < 9; ++i) pk.pose_raw.push_back(p.T_wb_init[k].R[i]);
        for (int i = 0; i < 3; ++i) pk.pose_raw.push_back(p.T_wb_init[k].t[i]);
        for (int i = 0; i < 9; ++i) pk.pose_raw.push_back(p.T_cb[k].R[i]);
        for (int i = 0; i < 3; ++i) pk.pose_raw.push_back(p.T_cb[k].t[i]);
        pk.kf_const.push_back(p.kf_const[k] ? 1 : 0);
        if (vi) {
            pk.preint.push_back(p.preint[k]);
            pk.preint_valid.push_back(k >= 1 && p.preint_valid[k] ? 1 : 0);
            for (int i = 0; i < 3; ++i) pk.vel0.push_back(p.vel[3 * k + i]);
        } else {
            vio_preint z;
            std::memset(&z, 0, sizeof z);
            pk.preint.push_back(z);
            pk.preint_valid.push_back(0);
            for (int i = 0; i < 3; ++i) pk.vel0.push_back(0.0);
        }
    }
    // landmarks
    const uint8_t* marg = pnp ? p.lm_const : p.lm_marg;
    for (int l = 0; l < L; ++l) {
        for (int i = 0; i < 3; ++i) pk.lm_xyz0.push_back(p.lm_xyz[3 * l + i]);
        pk.lm_var.push_back(lm_used[l]);
        pk.lm_marg.push_back(marg ? (marg[l] ? 1 : 0) : 0);
    }
    // observations sorted by landmark (stable)
    std::vector<int32_t> perm(N);
    for (int o = 0; o < N; ++o) perm[o] = o;
    std::stable_sort(perm.begin(), perm.end(), [&](int a, int b) { return p.obs_lm[a] < p.obs_lm[b]; });
    std::vector<int32_t> lptr(L + 1, 0);
    for (int o = 0; o < N; ++o) lptr[p.obs_lm[o] + 1]++;
    for (int l = 0; l < L; ++l) lptr[l + 1] += lptr[l];
    pk.lm_ptr.insert(pk.lm_ptr.end(), lptr.begin(), lptr.end());
    for (int q = 0; q < N; ++q) {
        int o = perm[q];
        pk.obs_kf.push_back(p.obs_kf[o]);
        pk.obs_lm.push_back(p.obs_lm[o]);
        pk.obs_uv.push_back(p.obs_uv[2 * o]);
        pk.obs_uv.push_back(p.obs_uv[2 * o + 1]);
    }
    std::vector<int32_t> kptr(K + 1, 0);
    for (int q = 0; q < N; ++q) kptr[p.obs_kf[perm[q]] + 1]++;
    for (int k = 0; k < K; ++k) kptr[k + 1] += kptr[k];
    std::vector<int32_t> fill(K, 0), kobs(N);
    for (int q = 0; q < N; ++q) {
        int k = p.obs_kf[perm[q]];
        kobs[kptr[k] + fill[k]++] = q;
    }
    pk.kf_ptr.insert(pk.kf_ptr.end(), kptr.begin(), kptr.end());
    pk.kf_obs.insert(pk.kf_obs.end(), kobs.begin(), kobs.end());
    pk.perm.push_back(std::move(perm));
    pk.win.push_back(w);
    pk.N_total += N;
    pk.L_total += L;
    return VIO_OK;
}

template <class T>
size_t bytes_of(const std::vector<T>& v) { return v.size() * sizeof(T); }

}  // namespace

// device image of a batch
struct BaDevice {
    int n = 0;
    Packed pk;
    // device allocations (owned)
    std::vector<void*> allocs;
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
    std::vector<int32_t> perm_host;
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

static int upload_batch(vio_ctx* ctx, BaDevice& d) {
    Packed& pk = d.pk;
    auto up = [&](const void* src, size_t bytes, void** dst) -> int {
        size_t b = std::max<size_t>(bytes, 16);
        void* p = nullptr;
        VIO_HIP(ctx, hipMalloc(&p, b));
        d.allocs.push_back(p);
        if (bytes) VIO_HIP(ctx, hipMemcpyAsync(p, src, bytes, hipMemcpyHostToDevice, ctx->stream));
        *dst = p;
        return VIO_OK;
    };
    void* ptr;
    int rc;
#define UP(vec, field, type)                                                  \
    if ((rc = up(vec.data(), bytes_of(vec), &ptr)) != VIO_OK) return rc;      \
    d.P.field = (type)ptr;
    // landmark chunks per Schur split-k group (phase route): a full config-4 shard (>= 256 windows)
    // fills the chip with 2 groups per window and halves ph_solve's partial sums; smaller batches keep
    // more, shorter groups (latency): 3 below 64 windows, 5 up to 255 (sweep of 2/3/4/5/10 at 1..256
    // windows, profiles/r4e_gs_sweep.log); the cluster route: one chunk per group, the group's member owns
    // its landmarks
    const char* gse = std::getenv("VIO_BA_SCHUR_GS");  // experiment override
    static const int cmax = [] {
        const char* v = std::getenv("VIO_BA_CLUSTER_C");  // experiment override: members per window
        return v ? std::atoi(v) : 0;
    }();
    // (an explicitly requested cluster route takes whatever members fit: no minimum per landmark chunk)
    const int cm = cmax > 0 ? cmax : ctx->ba_route == VIO_BA_ROUTE_CLUSTER ? (1 << 20) : 0;
    d.cluster_C = cluster_wanted(ctx, d.n) ? ba_cluster_members(pk.win.data(), d.n, cm) : 0;
    const int gs = d.cluster_C ? 1 : gse ? std::max(1, std::atoi(gse)) : pk.win.size() >= 256 ? 10 : pk.win.size() >= 64 ? 5 : 3;
    for (BaWin& w : pk.win) w.gs = gs;
    UP(pk.win, win, const BaWin*);
    UP(pk.pose_raw, pose_raw, const double*);
    UP(pk.kf_const, kf_const, const uint8_t*);
    UP(pk.lm_xyz0, lm_xyz0, const double*);
    UP(pk.lm_var, lm_var, const uint8_t*);
    UP(pk.lm_marg, lm_marg, const uint8_t*);
    UP(pk.lm_ptr, lm_ptr, const int32_t*);
    UP(pk.obs_kf, obs_kf, const int32_t*);
    UP(pk.obs_lm, obs_lm, const int32_t*);
    UP(pk.obs_uv, obs_uv, const float*);
    UP(pk.kf_ptr, kf_ptr, const int32_t*);
    UP(pk.kf_obs, kf_obs, const int32_t*);
    UP(pk.preint, preint, const vio_preint*);
    UP(pk.preint_valid, preint_valid, const uint8_t*);
    UP(pk.vel0, vel0, const double*);
#undef UP
    {   // sorted position -> caller's observation index, all windows back to back (result records)
        std::vector<int32_t> perm;
        perm.reserve(pk.N_total);
        for (const auto& p : pk.perm) perm.insert(perm.end(), p.begin(), p.end());
        if ((rc = up(perm.data(), bytes_of(perm), &ptr)) != VIO_OK) return rc;
        d.P.obs_perm = (const int32_t*)ptr;
        d.perm_host = std::move(perm);  // kept alive for the async upload
    }
    auto alloc = [&](size_t bytes, void** dst) -> int {
        void* p = nullptr;
        VIO_HIP(ctx, hipMalloc(&p, std::max<size_t>(bytes, 16)));
        d.allocs.push_back(p);
        *dst = p;
        return VIO_OK;
    };
    if ((rc = alloc(sizeof(double) * pk.ws_total, &ptr)) != VIO_OK) return rc;
    d.P.ws = (double*)ptr;
    if ((rc = alloc(sizeof(double) * pk.out_total, &ptr)) != VIO_OK) return rc;
    d.P.out = (double*)ptr;
    if ((rc = alloc(pk.N_total, &ptr)) != VIO_OK) return rc;
    d.P.out_u8 = (uint8_t*)ptr;
    if ((rc = alloc(pk.L_total, &ptr)) != VIO_OK) return rc;
    d.P.out_bad = (uint8_t*)ptr;
    if ((rc = alloc(sizeof(int32_t) * SI_COUNT * d.n, &ptr)) != VIO_OK) return rc;
    d.P.out_i32 = (int32_t*)ptr;
    if ((rc = alloc(sizeof(double) * SD_COUNT * d.n, &ptr)) != VIO_OK) return rc;
    d.P.out_sum = (double*)ptr;
    if ((rc = alloc(sizeof(vio_ba_iteration) * pk.tr_total, &ptr)) != VIO_OK) return rc;
    d.P.out_trace = (vio_ba_iteration*)ptr;
    if (d.cluster_C) {
        if ((rc = alloc(sizeof(int) * PH_SYNC_INTS * (size_t)d.n, &ptr)) != VIO_OK) return rc;
        d.P.csync = (int*)ptr;
    }
    VIO_HIP(ctx, hipEventCreate(&d.ev0));
    VIO_HIP(ctx, hipEventCreate(&d.ev1));
    return VIO_OK;
}

static void free_batch(BaDevice& d) {
    for (void* p : d.allocs) (void)hipFree(p);
    d.allocs.clear();
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

// the cluster route's per-window error words (a bounded hand-off wait that expired): VIO_EDEVICE
static int check_cluster(vio_ctx* ctx, BaDevice& d) {
    if (!d.cluster_C || !d.P.csync) return VIO_OK;
    std::vector<int> sync((size_t)PH_SYNC_INTS * d.n);
    VIO_HIP(ctx, hipMemcpyAsync(sync.data(), d.P.csync, sizeof(int) * sync.size(), hipMemcpyDeviceToHost, ctx->stream));
    VIO_HIP(ctx, hipStreamSynchronize(ctx->stream));
    for (int i = 0; i < d.n; ++i)
        if (sync[(size_t)PH_SYNC_INTS * i + 192]) {
            set_error(ctx, "cluster route: a hand-off wait timed out (workgroups not co-resident?)");
            return VIO_EDEVICE;
        }
    return VIO_OK;
}

static int download_batch(vio_ctx* ctx, BaDevice& d, vio_ba_output* outs) {
    Packed& pk = d.pk;
    if (int rc = check_cluster(ctx, d)) return rc;
    std::vector<double> out(pk.out_total);
    std::vector<uint8_t> u8(pk.N_total), bad(pk.L_total);
    std::vector<int32_t> si(SI_COUNT * d.n);
    std::vector<double> sd(SD_COUNT * d.n);
    bool want_trace = false;
    for (int i = 0; i < d.n; ++i) want_trace |= outs[i].trace != nullptr && outs[i].trace_cap > 0;
    std::vector<vio_ba_iteration> tr(want_trace ? pk.tr_total : 0);
    if (want_trace)
        VIO_HIP(ctx, hipMemcpyAsync(tr.data(), d.P.out_trace, sizeof(vio_ba_iteration) * tr.size(),
                                    hipMemcpyDeviceToHost, ctx->stream));
    VIO_HIP(ctx, hipMemcpyAsync(out.data(), d.P.out, sizeof(double) * out.size(), hipMemcpyDeviceToHost, ctx->stream));
    VIO_HIP(ctx, hipMemcpyAsync(u8.data(), d.P.out_u8, u8.size(), hipMemcpyDeviceToHost, ctx->stream));
    VIO_HIP(ctx, hipMemcpyAsync(bad.data(), d.P.out_bad, bad.size(), hipMemcpyDeviceToHost, ctx->stream));
    VIO_HIP(ctx, hipMemcpyAsync(si.data(), d.P.out_i32, sizeof(int32_t) * si.size(), hipMemcpyDeviceToHost, ctx->stream));
    VIO_HIP(ctx, hipMemcpyAsync(sd.data(), d.P.out_sum, sizeof(double) * sd.size(), hipMemcpyDeviceToHost, ctx->stream));
    VIO_HIP(ctx, hipStreamSynchronize(ctx->stream));
    for (int i = 0; i < d.n; ++i) {
        const BaWin& w = pk.win[i];
        vio_ba_output& o = outs[i];
        BaOutLayout OL = ba_out_layout(w.K, w.L, w.N);
        const double* ob = out.data() + w.o_out;
        if (o.T_wb)
            for (int k = 0; k < w.K; ++k) {
                std::memcpy(o.T_wb[k].R, ob + OL.T_wb + 12 * k, 9 * sizeof(double));
                std::memcpy(o.T_wb[k].t, ob + OL.T_wb + 12 * k + 9, 3 * sizeof(double));
            }
        if (o.lm_xyz) std::memcpy(o.lm_xyz, ob + OL.lm, sizeof(double) * 3 * w.L);
        const std::vector<int32_t>& perm = pk.perm[i];
        for (int q = 0; q < w.N; ++q) {
            if (o.obs_chi2) o.obs_chi2[perm[q]] = ob[OL.chi2 + q];
            if (o.obs_outlier) o.obs_outlier[perm[q]] = u8[w.o_obs + q];
        }
        if (o.lm_bad) std::memcpy(o.lm_bad, bad.data() + w.o_lm, w.L);
        if (w.is_vi) {
            if (o.vel) std::memcpy(o.vel, ob + OL.vel, sizeof(double) * 3 * w.K);
            if (o.bg) std::memcpy(o.bg, ob + OL.bias, sizeof(double) * 3);
            if (o.ba) std::memcpy(o.ba, ob + OL.bias + 3, sizeof(double) * 3);
        }
        if (o.summary) {
            vio_ba_summary& s = *o.summary;
            std::memset(&s, 0, sizeof s);
            const int32_t* a = si.data() + SI_COUNT * i;
            const double* b = sd.data() + SD_COUNT * i;
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
    for (void* p : ctx->bufs)
        if (p) (void)hipFree(p);
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
    b->dev.n = n;
    b->dev.reusable = true;
    for (int i = 0; i < n; ++i) {
        int rc = pack_window(ctx, probs[i], b->dev.pk);
        if (rc != VIO_OK) { delete b; return rc; }
    }
    int rc = upload_batch(ctx, b->dev);
    if (rc != VIO_OK) { free_batch(b->dev); delete b; return rc; }
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
    Packed& pk = b->dev.pk;
    if (count != (int)pk.preint.size()) {
        set_error(ctx, "vio_ba_batch_set_preint: count must be the batch's total keyframe count");
        return VIO_EINVAL;
    }
    if (count == 0) return VIO_OK;
    const size_t bytes = sizeof(vio_preint) * (size_t)count;
    VIO_DEVICE(ctx);
    if (on_device) {
        VIO_HIP(ctx, hipMemcpyAsync((void*)b->dev.P.preint, src, bytes, hipMemcpyDeviceToDevice, ctx->stream));
    } else {
        std::memcpy(pk.preint.data(), src, bytes);  // the staging copy outlives the async upload
        VIO_HIP(ctx, hipMemcpyAsync((void*)b->dev.P.preint, pk.preint.data(), bytes, hipMemcpyHostToDevice, ctx->stream));
    }
    return VIO_OK;
}

int vio_ba_batch_sync(vio_ba_batch* b) {
    if (!b) return VIO_EINVAL;
    VIO_DEVICE(b->ctx);
    VIO_HIP(b->ctx, hipStreamSynchronize(b->ctx->stream));
    return check_cluster(b->ctx, b->dev);
}

int vio_ba_batch_download(vio_ba_batch* b, vio_ba_output* outs) {
    if (!b || !outs) return VIO_EINVAL;
    VIO_DEVICE(b->ctx);
    return download_batch(b->ctx, b->dev, outs);
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
    vio_ba_batch* b = nullptr;
    int rc = vio_ba_batch_create(ctx, probs, n, &b);
    if (rc != VIO_OK) return rc;
    rc = launch(ctx, b->dev, false);
    if (rc == VIO_OK) rc = download_batch(ctx, b->dev, outs);
    vio_ba_batch_destroy(b);
    return rc;
}

int vio_ba_solve(vio_ctx* ctx, const vio_ba_problem* prob, vio_ba_output* out) {
    return vio_ba_solve_batched(ctx, prob, out, 1);
}

}  // extern "C"
