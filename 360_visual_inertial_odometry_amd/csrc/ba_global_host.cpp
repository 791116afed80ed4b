// ba_global_host.cpp — host LM driver of the global-BA path (problems beyond one workgroup:
// config 5, 1000 keyframes x 50k landmarks).  The control flow is Ceres 2.0's
// TrustRegionMinimizer + LevenbergMarquardtStrategy exactly as restated in oracle/ba_oracle.c
// (oracle_lm_minimize: trust_region_minimizer.cc:67-826, levenberg_marquardt_strategy.cc:66-160);
// every array operation runs on the GPU (ba_global.hip) and only scalars come back.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cfloat>
#include <cmath>
#include <cstring>
#include <vector>

#include "ba_global.h"
#include "residency.h"
#include "ba_types.h"
#include "ctx.h"

namespace vio360 {

uint64_t ba_layout_sig_ba_global_host() { return ba_layout_sig(); }
uint64_t gba_layout_sig_ba_global_host() { return gba_layout_sig(); }

namespace {

struct DevBufs {
    std::vector<void*> ptrs;
    vio_ctx* ctx;
    ~DevBufs() {
        for (void* p : ptrs) (void)hipFree(p);
    }
    template <class T>
    int alloc(T** p, size_t n) {
        void* q = nullptr;
        if (hipMalloc(&q, std::max<size_t>(n * sizeof(T), 64)) != hipSuccess) {
            set_error(ctx, "hipMalloc failed (global BA)");
            return VIO_ENOMEM;
        }
        ptrs.push_back(q);
        *p = (T*)q;
        return VIO_OK;
    }
    template <class T>
    int upload(T** p, const std::vector<T>& v) {
        int rc = alloc(p, v.size());
        if (rc) return rc;
        if (!v.empty() && hipMemcpy((void*)*p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice) != hipSuccess) {
            set_error(ctx, "hipMemcpy failed (global BA)");
            return VIO_EDEVICE;
        }
        return VIO_OK;
    }
};

#define GBA_CHECK(expr)                                            \
    do {                                                           \
        hipError_t _e = (expr);                                    \
        if (_e != hipSuccess) return hip_fail(ctx, _e, #expr);     \
    } while (0)

}  // namespace

// LocalBA / FullBA beyond 16 keyframes, VIBA beyond 10 (the windowed path's reduced-system bound)
bool global_ba_applicable(const vio_ba_problem& p) {
    return ((p.variant == VIO_BA_LOCAL || p.variant == VIO_BA_FULL) && p.num_kf > BA_KMAX) ||
           (p.variant == VIO_BA_VI && p.num_kf > VI_KMAX);
}

int global_ba_solve(vio_ctx* ctx, const vio_ba_problem& p, vio_ba_output* out) {
    const int K = p.num_kf, L = p.num_lm, N = p.num_obs;
    if (K <= 0 || L < 0 || N < 0 || !p.T_cb || !p.T_wb_init || !p.kf_const || (L && (!p.lm_const || !p.lm_xyz)) ||
        (N && (!p.obs_kf || !p.obs_lm || !p.obs_uv))) {
        set_error(ctx, "invalid global BA problem");
        return VIO_EINVAL;
    }
    const bool vi = p.variant == VIO_BA_VI;
    if (vi && (!p.preint || !p.preint_valid || !p.vel)) { set_error(ctx, "VIBA needs preint/preint_valid/vel"); return VIO_EINVAL; }
    for (int o = 0; o < N; ++o)
        if (p.obs_kf[o] < 0 || p.obs_kf[o] >= K || p.obs_lm[o] < 0 || p.obs_lm[o] >= L) {
            set_error(ctx, "observation index out of range");
            return VIO_EINVAL;
        }
    {
        std::vector<int64_t> key(N);
        for (int o = 0; o < N; ++o) key[o] = (int64_t)p.obs_lm[o] * K + p.obs_kf[o];
        std::sort(key.begin(), key.end());
        for (int o = 1; o < N; ++o)
            if (key[o] == key[o - 1]) { set_error(ctx, "duplicate (keyframe, landmark) observation"); return VIO_EINVAL; }
    }
    DeviceScope _vio_dev_scope(ctx->device);
    hipStream_t st = ctx->stream;
    // ---- reduced problem (Ceres RemoveFixedBlocks; points are the e-blocks) ----
    std::vector<uint8_t> pose_used(K, 0), lm_used(L, 0), active(N, 0);
    for (int o = 0; o < N; ++o) {
        int k = p.obs_kf[o], l = p.obs_lm[o];
        bool kv = !p.kf_const[k], lv = !p.lm_const[l];
        if (kv) pose_used[k] = 1;
        if (lv) lm_used[l] = 1;
        active[o] = kv || lv;
    }
    // VIBA: an IMU factor k (preint_valid[k]) brings velocities k-1, k, the biases and its two poses in
    // (RunVIBA: velocities and biases are never constant; Optimizer.cpp:493-636)
    std::vector<uint8_t> vel_used(K, 0);
    bool bias_used = false;
    if (vi)
        for (int k = 1; k < K; ++k) {
            if (!p.preint_valid[k]) continue;
            vel_used[k - 1] = vel_used[k] = 1;
            bias_used = true;
            if (!p.kf_const[k - 1]) pose_used[k - 1] = 1;
            if (!p.kf_const[k]) pose_used[k] = 1;
        }
    std::vector<int> pose_f(K, -1), pose_of_block, vel_f(K, -1);
    for (int k = 0; k < K; ++k)
        if (pose_used[k]) { pose_f[k] = 6 * (int)pose_of_block.size(); pose_of_block.push_back(k); }
    const int P = (int)pose_of_block.size();
    int nf = 6 * P;
    for (int k = 0; k < K; ++k)
        if (vel_used[k]) { vel_f[k] = nf; nf += 3; }
    const int bg_f = bias_used ? nf : -1;
    if (bias_used) nf += 3;
    const int ba_f = bias_used ? nf : -1;
    if (bias_used) nf += 3;
    const int np = 6 * P, ni = nf - np;
    const int nfp = std::max(64, (nf + 63) / 64 * 64);
    int n_free = nf;
    for (int l = 0; l < L; ++l) n_free += 3 * lm_used[l];
    // landmark-sorted observations
    std::vector<int> perm(N);
    for (int o = 0; o < N; ++o) perm[o] = o;
    std::stable_sort(perm.begin(), perm.end(), [&](int a, int b) { return p.obs_lm[a] < p.obs_lm[b]; });
    std::vector<int> lm_ptr(L + 1, 0), okf(N), olm(N), kf_ptr(K + 1, 0), kf_obs(N);
    std::vector<float> ouv(2 * (size_t)N);
    for (int o = 0; o < N; ++o) lm_ptr[p.obs_lm[o] + 1]++;
    for (int l = 0; l < L; ++l) lm_ptr[l + 1] += lm_ptr[l];
    for (int q = 0; q < N; ++q) {
        int o = perm[q];
        okf[q] = p.obs_kf[o]; olm[q] = p.obs_lm[o];
        ouv[2 * q] = p.obs_uv[2 * o]; ouv[2 * q + 1] = p.obs_uv[2 * o + 1];
        kf_ptr[okf[q] + 1]++;
    }
    for (int k = 0; k < K; ++k) kf_ptr[k + 1] += kf_ptr[k];
    {
        std::vector<int> fill(K, 0);
        for (int q = 0; q < N; ++q) kf_obs[kf_ptr[okf[q]] + fill[okf[q]]++] = q;
    }
    // Schur contributions by destination block (pa >= pb), landmark order inside a destination
    const long long n_dest = (long long)P * (P + 1) / 2;
    std::vector<int> dest_cnt(n_dest + 1, 0);
    auto dest_of = [](int a, int b) { return (long long)a * (a + 1) / 2 + b; };
    for (int l = 0; l < L; ++l) {
        if (!lm_used[l]) continue;
        for (int qa = lm_ptr[l]; qa < lm_ptr[l + 1]; ++qa) {
            int fa = pose_f[okf[qa]];
            if (fa < 0) continue;
            for (int qb = lm_ptr[l]; qb < lm_ptr[l + 1]; ++qb) {
                int fb = pose_f[okf[qb]];
                if (fb < 0 || fb > fa) continue;
                dest_cnt[dest_of(fa / 6, fb / 6) + 1]++;
            }
        }
    }
    for (long long d = 0; d < n_dest; ++d) dest_cnt[d + 1] += dest_cnt[d];
    const long long n_contrib = dest_cnt[n_dest];
    if (n_contrib > INT32_MAX) { set_error(ctx, "too many Schur contributions"); return VIO_ENOSYS; }
    std::vector<int> ca(n_contrib), cb(n_contrib), dfill(dest_cnt.begin(), dest_cnt.end() - 1);
    for (int l = 0; l < L; ++l) {
        if (!lm_used[l]) continue;
        for (int qa = lm_ptr[l]; qa < lm_ptr[l + 1]; ++qa) {
            int fa = pose_f[okf[qa]];
            if (fa < 0) continue;
            for (int qb = lm_ptr[l]; qb < lm_ptr[l + 1]; ++qb) {
                int fb = pose_f[okf[qb]];
                if (fb < 0 || fb > fa) continue;
                int pos = dfill[dest_of(fa / 6, fb / 6)]++;
                ca[pos] = qa; cb[pos] = qb;
            }
        }
    }
    std::vector<int> dest_a(n_dest), dest_b(n_dest);
    for (int a = 0; a < P; ++a)
        for (int b = 0; b <= a; ++b) { dest_a[dest_of(a, b)] = a; dest_b[dest_of(a, b)] = b; }
    std::vector<double> pose_raw(24 * (size_t)K), xl0(3 * (size_t)L);
    for (int k = 0; k < K; ++k) {
        std::memcpy(&pose_raw[24 * k], p.T_wb_init[k].R, 9 * sizeof(double));
        std::memcpy(&pose_raw[24 * k + 9], p.T_wb_init[k].t, 3 * sizeof(double));
        std::memcpy(&pose_raw[24 * k + 12], p.T_cb[k].R, 9 * sizeof(double));
        std::memcpy(&pose_raw[24 * k + 21], p.T_cb[k].t, 3 * sizeof(double));
    }
    std::memcpy(xl0.data(), p.lm_xyz, sizeof(double) * 3 * L);
    std::vector<uint8_t> lm_marg(L, 0);
    for (int l = 0; l < L; ++l) lm_marg[l] = p.lm_marg ? (p.lm_marg[l] != 0) : 0;

    // ---- device state ----
    DevBufs B;
    B.ctx = ctx;
    GbaArgs A;
    std::memset(&A, 0, sizeof A);
    A.K = K; A.L = L; A.N = N; A.P = P; A.nf = nf; A.nfp = nfp;
    A.is_vi = vi; A.np = np; A.ni = ni; A.bg_f = bg_f; A.ba_f = ba_f;
    if (vi) for (int i = 0; i < 3; ++i) A.gravity[i] = p.gravity[i];
    A.cols = p.cols; A.rows = p.rows; A.huber = p.huber_delta; A.chi2_thr = p.chi2_threshold;
    for (int i = 0; i < 4; ++i) A.info[i] = p.info[i];
    A.Lw[0] = 1; A.Lw[1] = 0; A.Lw[2] = 0; A.Lw[3] = 1;
    if (p.info[0] > 0) {
        double l00 = std::sqrt(p.info[0]), l10 = p.info[2] / l00, t = p.info[3] - l10 * l10;
        if (t > 0) { A.Lw[0] = l00; A.Lw[2] = l10; A.Lw[3] = std::sqrt(t); }
    }
    int rc;
    const double* c_pose_raw; const int *c_pose_f, *c_pob, *c_lm_ptr, *c_okf, *c_olm, *c_kf_ptr, *c_kf_obs;
    const int *c_da, *c_db, *c_dp, *c_ca, *c_cb; const uint8_t *c_lv, *c_lmarg; const float* c_uv;
    std::vector<int> dptr(dest_cnt.begin(), dest_cnt.end());
    if ((rc = B.upload((double**)&c_pose_raw, pose_raw)) || (rc = B.upload((int**)&c_pose_f, pose_f)) ||
        (rc = B.upload((int**)&c_pob, pose_of_block)) || (rc = B.upload((uint8_t**)&c_lv, lm_used)) ||
        (rc = B.upload((uint8_t**)&c_lmarg, lm_marg)) || (rc = B.upload((int**)&c_lm_ptr, lm_ptr)) ||
        (rc = B.upload((int**)&c_okf, okf)) || (rc = B.upload((int**)&c_olm, olm)) ||
        (rc = B.upload((float**)&c_uv, ouv)) || (rc = B.upload((int**)&c_kf_ptr, kf_ptr)) ||
        (rc = B.upload((int**)&c_kf_obs, kf_obs)) || (rc = B.upload((int**)&c_da, dest_a)) ||
        (rc = B.upload((int**)&c_db, dest_b)) || (rc = B.upload((int**)&c_dp, dptr)) ||
        (rc = B.upload((int**)&c_ca, ca)) || (rc = B.upload((int**)&c_cb, cb)))
        return rc;
    A.pose_raw = c_pose_raw; A.pose_f = c_pose_f; A.pose_of_block = c_pob; A.lm_var = c_lv; A.lm_marg = c_lmarg;
    A.lm_ptr = c_lm_ptr; A.obs_kf = c_okf; A.obs_lm = c_olm; A.obs_uv = c_uv; A.kf_ptr = c_kf_ptr; A.kf_obs = c_kf_obs;
    A.n_dest = n_dest; A.dest_a = c_da; A.dest_b = c_db; A.dest_ptr = c_dp; A.contrib_a = c_ca; A.contrib_b = c_cb;
    const size_t Ns = std::max(N, 1), Ls = std::max(L, 1);
    if ((rc = B.alloc(&A.pinit, 24 * (size_t)K)) || (rc = B.alloc(&A.pc, 36 * (size_t)K)) ||
        (rc = B.alloc(&A.x_pose, 6 * (size_t)K)) || (rc = B.alloc(&A.x_lm, 3 * Ls)) ||
        (rc = B.alloc(&A.c_pose, 6 * (size_t)K)) || (rc = B.alloc(&A.c_lm, 3 * Ls)) ||
        (rc = B.alloc(&A.r, 2 * Ns)) || (rc = B.alloc(&A.jp, 12 * Ns)) || (rc = B.alloc(&A.jl, 6 * Ns)) ||
        (rc = B.alloc(&A.V, 6 * Ls)) || (rc = B.alloc(&A.gl, 3 * Ls)) || (rc = B.alloc(&A.sl, 3 * Ls)) ||
        (rc = B.alloc(&A.Vi, 6 * Ls)) || (rc = B.alloc(&A.yl, 3 * Ls)) || (rc = B.alloc(&A.U, 27 * (size_t)K)) ||
        (rc = B.alloc(&A.gf, nfp)) || (rc = B.alloc(&A.colsq_f, nfp)) || (rc = B.alloc(&A.sf, nfp)) ||
        (rc = B.alloc(&A.Df, nfp)) || (rc = B.alloc(&A.bf, nfp)) || (rc = B.alloc(&A.yv, nfp)) ||
        (rc = B.alloc(&A.xf, nfp)) || (rc = B.alloc(&A.Wo, 18 * Ns)) || (rc = B.alloc(&A.Yo, 18 * Ns)) ||
        (rc = B.alloc(&A.S, (size_t)nfp * nfp)) || (rc = B.alloc(&A.Linv, (size_t)nfp * 64)))
        return rc;
    const size_t nblk_max = (std::max<size_t>({Ns, Ls, 6 * (size_t)K, (size_t)nfp}) + 255) / 256 + 8;
    double* partial;
    double* scal;  // [0] cost [1] gmax [2] bad [3] nonfinite [4..6] model/step/xnorm [7] cand cost [8..10] post
    int* dfail;
    uint8_t *d_outl, *d_bad;
    double* d_chi2;
    if (vi) {
        const vio_preint* c_pre; const uint8_t* c_pv; const int* c_vf;
        std::vector<vio_preint> pre(p.preint, p.preint + K);
        std::vector<uint8_t> pv(p.preint_valid, p.preint_valid + K);
        std::vector<double> v0(p.vel, p.vel + 3 * (size_t)K), b0(6);
        for (int i = 0; i < 3; ++i) { b0[i] = p.bg[i]; b0[3 + i] = p.ba[i]; }
        if ((rc = B.upload((vio_preint**)&c_pre, pre)) || (rc = B.upload((uint8_t**)&c_pv, pv)) ||
            (rc = B.upload((int**)&c_vf, vel_f)) || (rc = B.upload(&A.x_vel, v0)) || (rc = B.upload(&A.x_bias, b0)) ||
            (rc = B.alloc(&A.c_vel, 3 * (size_t)K)) || (rc = B.alloc(&A.c_bias, 6)) || (rc = B.alloc(&A.sqi, 81 * (size_t)K)) ||
            (rc = B.alloc(&A.imuJ, 108 * (size_t)K)) || (rc = B.alloc(&A.imur, 9 * (size_t)K)) ||
            (rc = B.alloc(&A.imu_cost, (size_t)K)) || (rc = B.alloc(&A.Himu, (size_t)ni * ni + ni)))
            return rc;
        A.preint = c_pre; A.preint_valid = c_pv; A.vel_f = c_vf;
    }
    if ((rc = B.alloc(&partial, 3 * nblk_max + 3 * (size_t)K)) || (rc = B.alloc(&scal, 32)) ||
        (rc = B.alloc(&dfail, 4)) || (rc = B.alloc(&A.flags, 32 * (3 * ((size_t)nfp / 64) + 1))) || (rc = B.alloc(&d_outl, Ns)) || (rc = B.alloc(&d_bad, Ls)) ||
        (rc = B.alloc(&d_chi2, Ns)))
        return rc;
    // look-ahead stream + events of the Cholesky (released with the solve)
    struct SideGuard {
        GbaArgs* a;
        ~SideGuard() {
            if (a->side) (void)hipStreamDestroy(a->side);
            for (hipEvent_t& e : a->ev)
                if (e) (void)hipEventDestroy(e);
        }
    } side_guard{&A};
    if (hipStreamCreateWithFlags(&A.side, hipStreamNonBlocking) != hipSuccess) A.side = nullptr;
    for (hipEvent_t& e : A.ev)
        if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) e = nullptr;
    GBA_CHECK(gba_cholesky_attributes());
    // the Cholesky + triangular solves of a step are the same launches every LM iteration: captured
    // once (fork / join of the look-ahead stream included) and replayed as one graph
    static const bool use_graph = [] {
        const char* v = std::getenv("VIO_GBA_GRAPH");
        return !(v && v[0] == '0');
    }();
    struct GraphGuard {
        hipGraphExec_t g = nullptr;
        ~GraphGuard() {
            if (g) (void)hipGraphExecDestroy(g);
        }
    } chol_graph;
    auto factor_and_solve = [&]() -> hipError_t {
        if (!use_graph) {
            hipError_t e = gba_launch_cholesky(A, dfail, st);
            if (e != hipSuccess) return e;
            ResidencyGuard rg(st, gba_solve_persistent_wgs(A));  // (residency.h)
            if ((e = rg.status()) != hipSuccess) return e;
            e = gba_launch_solve(A, st);
            return e == hipSuccess ? rg.commit() : e;
        }
        if (!chol_graph.g) {
            hipGraph_t g = nullptr;
            hipError_t e = hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal);
            if (e != hipSuccess) return e;
            hipError_t el = gba_launch_cholesky(A, dfail, st);
            if (el == hipSuccess) el = gba_launch_solve(A, st);
            e = hipStreamEndCapture(st, &g);
            if (el != hipSuccess) e = el;
            if (e == hipSuccess) e = hipGraphInstantiate(&chol_graph.g, g, nullptr, nullptr, 0);
            if (g) (void)hipGraphDestroy(g);
            if (e != hipSuccess) return e;
        }
        // the graph ends with the persistent triangular solves: reserved for the whole replay (residency.h)
        ResidencyGuard rg(st, gba_solve_persistent_wgs(A));
        hipError_t e = rg.status();
        if (e == hipSuccess) e = hipGraphLaunch(chol_graph.g, st);
        return e == hipSuccess ? rg.commit() : e;
    };
    GBA_CHECK(hipMemsetAsync(A.x_pose, 0, sizeof(double) * 6 * K, st));
    GBA_CHECK(hipMemcpyAsync(A.x_lm, xl0.data(), sizeof(double) * 3 * L, hipMemcpyHostToDevice, st));
    GBA_CHECK(gba_launch_setup(A, st));
    if (vi) GBA_CHECK(gba_imu_launch_setup(A, st));
    // scal slots of the VIBA terms: [11] IMU cost at x, [12] IMU gradient max-norm, [13..15] IMU model change /
    // step norm^2 / candidate norm^2, [16] IMU cost at the candidate (all 0 without IMU factors)
    GBA_CHECK(hipMemsetAsync(scal, 0, sizeof(double) * 32, st));
    // cost + Jacobians at the current point, then the normal-equation terms (visual and IMU)
    auto linearise = [&](int first) -> hipError_t {
        hipError_t e = gba_launch_eval(A, A.x_pose, A.x_lm, 1, partial, scal + 0, st);
        if (e == hipSuccess && vi) e = gba_imu_launch_eval(A, A.x_vel, A.x_bias, 1, scal + 11, st);
        if (e == hipSuccess) e = gba_launch_linearise(A, first, partial, scal + 1, st);
        if (e == hipSuccess && vi) e = gba_imu_launch_linearise(A, first, scal + 12, st);
        return e;
    };
    auto read = [&](double* h, int off, int n) -> int {
        GBA_CHECK(hipMemcpyAsync(h, scal + off, sizeof(double) * n, hipMemcpyDeviceToHost, st));
        GBA_CHECK(hipStreamSynchronize(st));
        return VIO_OK;
    };
    // ---- fixed cost (program.cc:305-390) ----
    double h[32];
    GBA_CHECK(gba_launch_eval(A, A.x_pose, A.x_lm, 2, partial, scal + 0, st));
    if ((rc = read(h, 0, 1))) return rc;
    const double fixed_cost = h[0];

    // ---- LM (oracle_lm_minimize) ----
    const int max_iter = p.max_iterations;
    const bool fixed = p.fixed_iterations != 0;
    int termination = VIO_TERM_NO_CONVERGENCE, iterations = 0, nsucc = 0, nunsucc = 0;
    double initial_cost, final_cost;
    // Summary::iterations (pushed at FinalizeIterationAndCheckIfMinimizerCanContinue, :313-348)
    vio_ba_iteration it;
    std::memset(&it, 0, sizeof it);
    auto push = [&](double radius) {
        if (out->trace && iterations - 1 < out->trace_cap) {
            out->trace[iterations - 1] = it;
            out->trace[iterations - 1].trust_region_radius = radius;
        }
    };
    if (n_free == 0) {
        termination = VIO_TERM_CONVERGENCE;
        initial_cost = final_cost = fixed_cost;
    } else {
        double radius = 1e4, decrease = 2.0, x_norm = -1.0, min_cost = DBL_MAX;
        int consecutive_invalid = 0;
        GBA_CHECK(linearise(1));
        if ((rc = read(h, 0, 17))) return rc;
        double x_cost = h[0] + h[11], gmax = std::max(h[1], h[12]);
        initial_cost = x_cost + fixed_cost;
        double step_eval_current = x_cost, iter_cost = x_cost + fixed_cost;
        final_cost = initial_cost;
        int iteration = 0;
        bool step_ok = true;
        double model_change = 0, cand_cost = 0;
        it.step_is_valid = it.step_is_successful = 1;  // IterationZero (:195-229)
        it.cost = iter_cost;
        it.gradient_max_norm = gmax;
        for (;;) {
            if (step_ok) {
                nsucc++;
                if (x_cost < min_cost) min_cost = x_cost;
            } else {
                nunsucc++;
            }
            iterations++;
            final_cost = std::min(final_cost, iter_cost);
            push(radius);
            if (iteration >= max_iter) { termination = VIO_TERM_NO_CONVERGENCE; break; }
            if (!fixed && step_ok && gmax <= 1e-10) { termination = VIO_TERM_CONVERGENCE; break; }
            if (!fixed && radius <= 1e-32) { termination = VIO_TERM_CONVERGENCE; break; }
            iteration++;
            std::memset(&it, 0, sizeof it);
            it.iteration = iteration;
            // ComputeTrustRegionStep + candidate cost, one batch of kernels, one readback
            GBA_CHECK(hipMemsetAsync(dfail, 0, sizeof(int), st));
            GBA_CHECK(gba_launch_step_prep(A, radius, partial, scal + 2, st));
            if (vi) GBA_CHECK(gba_imu_launch_system(A, st));
            GBA_CHECK(factor_and_solve());
            GBA_CHECK(gba_launch_backsub(A, partial, scal + 3, st));
            GBA_CHECK(gba_launch_model(A, partial, scal + 4, st));
            if (vi) GBA_CHECK(gba_imu_launch_model(A, scal + 13, st));
            GBA_CHECK(gba_launch_eval(A, A.c_pose, A.c_lm, 0, partial, scal + 7, st));
            if (vi) GBA_CHECK(gba_imu_launch_eval(A, A.c_vel, A.c_bias, 0, scal + 16, st));
            int hfail = 0, htmo = 0;
            GBA_CHECK(hipMemcpyAsync(&hfail, dfail, sizeof(int), hipMemcpyDeviceToHost, st));
            if (int* tw = gba_timeout_word(A)) GBA_CHECK(hipMemcpyAsync(&htmo, tw, sizeof(int), hipMemcpyDeviceToHost, st));
            if ((rc = read(h, 0, 17))) return rc;
            h[4] += h[13];  // model change, |x - cand|^2, |cand|^2, candidate cost: visual + IMU terms
            h[5] += h[14];
            h[6] += h[15];
            h[7] += h[16];
            if (htmo) {  // an inter-workgroup wait timed out: report the fault instead of an invalid LM step
                set_error(ctx, "global BA: a Cholesky / triangular-solve hand-off timed out on the device");
                return VIO_EDEVICE;
            }
            bool valid = h[2] == 0.0 && hfail == 0 && h[3] == 0.0;
            model_change = h[4];
            if (valid) it.model_cost_change = model_change;
            if (valid) valid = model_change > 0.0;
            if (!valid) {
                if (++consecutive_invalid >= 5) { termination = VIO_TERM_FAILURE; break; }
                radius /= decrease;
                decrease *= 2.0;
                step_ok = false;
                iter_cost = x_cost + fixed_cost;
                it.cost = iter_cost;
                it.gradient_max_norm = gmax;
                continue;
            }
            consecutive_invalid = 0;
            cand_cost = h[7];
            const double step_norm = std::sqrt(h[5]);
            it.step_is_valid = 1;
            it.step_norm = step_norm;
            it.cost_change = x_cost - cand_cost;
            if (!fixed && step_norm <= 1e-8 * (x_norm + 1e-8)) { termination = VIO_TERM_CONVERGENCE; break; }
            if (!fixed && std::fabs(x_cost - cand_cost) <= 1e-6 * x_cost) { termination = VIO_TERM_CONVERGENCE; break; }
            const double rel = (step_eval_current - cand_cost) / model_change;
            it.relative_decrease = rel;
            if (rel > 1e-3) {
                GBA_CHECK(hipMemcpyAsync(A.x_pose, A.c_pose, sizeof(double) * 6 * K, hipMemcpyDeviceToDevice, st));
                GBA_CHECK(hipMemcpyAsync(A.x_lm, A.c_lm, sizeof(double) * 3 * L, hipMemcpyDeviceToDevice, st));
                if (vi) {
                    GBA_CHECK(hipMemcpyAsync(A.x_vel, A.c_vel, sizeof(double) * 3 * K, hipMemcpyDeviceToDevice, st));
                    GBA_CHECK(hipMemcpyAsync(A.x_bias, A.c_bias, sizeof(double) * 6, hipMemcpyDeviceToDevice, st));
                }
                x_norm = std::sqrt(h[6]);
                GBA_CHECK(linearise(0));
                if ((rc = read(h, 0, 17))) return rc;
                x_cost = h[0] + h[11];
                gmax = std::max(h[1], h[12]);
                step_ok = true;
                radius = std::min(1e16, radius / std::max(1.0 / 3.0, 1.0 - std::pow(2.0 * rel - 1.0, 3)));
                decrease = 2.0;
                step_eval_current = cand_cost;
                iter_cost = x_cost + fixed_cost;
            } else {
                step_ok = false;
                iter_cost = cand_cost + fixed_cost;
                radius /= decrease;
                decrease *= 2.0;
            }
            it.step_is_successful = step_ok;
            it.cost = iter_cost;
            it.gradient_max_norm = gmax;
        }
        if (termination == VIO_TERM_FAILURE) {  // Ceres leaves the user's parameters untouched
            GBA_CHECK(hipMemsetAsync(A.x_pose, 0, sizeof(double) * 6 * K, st));
            GBA_CHECK(hipMemcpyAsync(A.x_lm, xl0.data(), sizeof(double) * 3 * L, hipMemcpyHostToDevice, st));
            if (vi) {
                std::vector<double> b0(6);
                for (int i = 0; i < 3; ++i) { b0[i] = p.bg[i]; b0[3 + i] = p.ba[i]; }
                GBA_CHECK(hipMemcpy(A.x_vel, p.vel, sizeof(double) * 3 * K, hipMemcpyHostToDevice));
                GBA_CHECK(hipMemcpy(A.x_bias, b0.data(), sizeof(double) * 6, hipMemcpyHostToDevice));
            }
        }
    }
    // ---- chi^2 / outliers / bad landmarks, outputs ----
    GBA_CHECK(gba_launch_post(A, d_chi2, d_outl, d_bad, partial, scal + 8, st));
    if ((rc = read(h, 8, 3))) return rc;
    std::vector<double> pc(36 * (size_t)K), xl(3 * Ls), chi2(Ns);
    std::vector<uint8_t> outl(Ns), bad(Ls);
    GBA_CHECK(hipMemcpy(pc.data(), A.pc, sizeof(double) * 36 * K, hipMemcpyDeviceToHost));
    GBA_CHECK(hipMemcpy(xl.data(), A.x_lm, sizeof(double) * 3 * Ls, hipMemcpyDeviceToHost));
    GBA_CHECK(hipMemcpy(chi2.data(), d_chi2, sizeof(double) * Ns, hipMemcpyDeviceToHost));
    GBA_CHECK(hipMemcpy(outl.data(), d_outl, Ns, hipMemcpyDeviceToHost));
    GBA_CHECK(hipMemcpy(bad.data(), d_bad, Ls, hipMemcpyDeviceToHost));
    if (out->T_wb)
        for (int k = 0; k < K; ++k) {
            std::memcpy(out->T_wb[k].R, &pc[36 * k], 9 * sizeof(double));
            std::memcpy(out->T_wb[k].t, &pc[36 * k + 9], 3 * sizeof(double));
        }
    if (out->lm_xyz) std::memcpy(out->lm_xyz, xl.data(), sizeof(double) * 3 * L);
    for (int q = 0; q < N; ++q) {
        if (out->obs_chi2) out->obs_chi2[perm[q]] = chi2[q];
        if (out->obs_outlier) out->obs_outlier[perm[q]] = outl[q];
    }
    if (out->lm_bad) std::memcpy(out->lm_bad, bad.data(), L);
    if (vi) {
        double xb[6];
        if (out->vel) GBA_CHECK(hipMemcpy(out->vel, A.x_vel, sizeof(double) * 3 * K, hipMemcpyDeviceToHost));
        GBA_CHECK(hipMemcpy(xb, A.x_bias, sizeof xb, hipMemcpyDeviceToHost));
        if (out->bg) std::memcpy(out->bg, xb, 3 * sizeof(double));
        if (out->ba) std::memcpy(out->ba, xb + 3, 3 * sizeof(double));
    }
    if (out->summary) {
        vio_ba_summary& s = *out->summary;
        std::memset(&s, 0, sizeof s);
        s.success = termination != VIO_TERM_FAILURE;
        s.termination = termination;
        s.iterations = iterations;
        s.num_successful_steps = nsucc;
        s.num_unsuccessful_steps = nunsucc;
        s.num_inliers = (int)h[8];
        s.num_outliers = (int)h[9];
        s.num_bad_lm = (int)h[10];
        s.initial_cost = initial_cost;
        s.final_cost = final_cost;
        s.fixed_cost = fixed_cost;
    }
    return VIO_OK;
}

}  // namespace vio360
