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

#define GBA_CHECK(expr)                                            \
    do {                                                           \
        hipError_t _e = (expr);                                    \
        if (_e != hipSuccess) return hip_fail(ctx, _e, #expr);     \
    } while (0)

// the per-context state that outlives a global solve: the Cholesky's look-ahead stream and events, and the
// captured Cholesky + triangular-solve graph with the device arguments it was captured with
struct GbaCache {
    hipStream_t side = nullptr;
    hipEvent_t ev[2] = {nullptr, nullptr};
    hipGraphExec_t graph = nullptr;
    unsigned char key[sizeof(GbaArgs)] = {};
    int* key_fail = nullptr;
    ~GbaCache() {
        if (graph) (void)hipGraphExecDestroy(graph);
        if (side) (void)hipStreamDestroy(side);
        for (hipEvent_t e : ev)
            if (e) (void)hipEventDestroy(e);
    }
};

GbaCache& gba_cache(vio_ctx* ctx) {
    if (!ctx->gba_cache) ctx->gba_cache = std::make_shared<GbaCache>();
    return *static_cast<GbaCache*>(ctx->gba_cache.get());
}

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
    // landmark CSR and the landmark-sorted order (a counting sort, stable: the caller's order within a
    // landmark); one observation per (keyframe, landmark): a keyframe stamp per landmark, O(N + K)
    std::vector<int> lm_ptr(L + 1, 0), perm(N);
    for (int o = 0; o < N; ++o) lm_ptr[p.obs_lm[o] + 1]++;
    for (int l = 0; l < L; ++l) lm_ptr[l + 1] += lm_ptr[l];
    {
        std::vector<int> fill(lm_ptr.begin(), lm_ptr.end() - 1);
        for (int o = 0; o < N; ++o) perm[fill[p.obs_lm[o]]++] = o;
        std::vector<int> stamp(K, -1);
        for (int l = 0; l < L; ++l)
            for (int q = lm_ptr[l]; q < lm_ptr[l + 1]; ++q) {
                const int k = p.obs_kf[perm[q]];
                if (stamp[k] == l) { set_error(ctx, "duplicate (keyframe, landmark) observation"); return VIO_EINVAL; }
                stamp[k] = l;
            }
    }
    DeviceScope _vio_dev_scope(ctx->device);
    GBA_CHECK(_vio_dev_scope.err);
    hipStream_t st = ctx->stream;
    // ---- reduced problem (Ceres RemoveFixedBlocks; points are the e-blocks) ----
    std::vector<uint8_t> pose_used(K, 0), lm_used(L, 0);
    for (int o = 0; o < N; ++o) {
        int k = p.obs_kf[o], l = p.obs_lm[o];
        if (!p.kf_const[k]) pose_used[k] = 1;
        if (!p.lm_const[l]) lm_used[l] = 1;
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
    // Schur contributions by destination block (pa >= pb), landmark order inside a destination: counts
    const long long n_dest = (long long)P * (P + 1) / 2;
    auto dest_of = [](int a, int b) { return (long long)a * (a + 1) / 2 + b; };
    // (pose block of every landmark-sorted observation, -1 for a constant pose: the pair loops below read it
    // contiguously)
    std::vector<int> blk(N);
    for (int q = 0; q < N; ++q) {
        const int f = pose_f[p.obs_kf[perm[q]]];
        blk[q] = f < 0 ? -1 : f / 6;
    }
    std::vector<int> dest_cnt(n_dest + 1, 0);
    for (int l = 0; l < L; ++l) {
        if (!lm_used[l]) continue;
        for (int qa = lm_ptr[l]; qa < lm_ptr[l + 1]; ++qa) {
            const int a = blk[qa];
            if (a < 0) continue;
            int* row = &dest_cnt[dest_of(a, 0) + 1];
            for (int qb = lm_ptr[l]; qb < lm_ptr[l + 1]; ++qb) {
                const int b = blk[qb];
                if (b >= 0 && b <= a) row[b]++;
            }
        }
    }
    for (long long d = 0; d < n_dest; ++d) dest_cnt[d + 1] += dest_cnt[d];
    const long long n_contrib = dest_cnt[n_dest];
    if (n_contrib > INT32_MAX) { set_error(ctx, "too many Schur contributions"); return VIO_ENOSYS; }

    // ---- one device arena per context (grow-only): inputs | outputs | state and scratch ----
    // The inputs are written straight into the context's pinned staging buffer and go up in ONE copy; the
    // outputs (pose cache, landmarks, chi2 / outlier / bad flags, velocities, biases) are adjacent and come
    // back in ONE copy.
    const size_t Ns = std::max(N, 1), Ls = std::max(L, 1);
    size_t off = 0;
    auto take = [&off](size_t bytes) {
        const size_t at = off;
        off = (off + std::max<size_t>(bytes, 64) + 255) & ~(size_t)255;
        return at;
    };
    struct { size_t pose_raw, pose_f, pob, lm_used, lm_marg, lm_ptr, okf, olm, ouv, kf_ptr, kf_obs, dest_a, dest_b,
                    dptr, ca, cb, xl0, pre, pv, vel_f, v0, b0; } I{};
    I.pose_raw = take(sizeof(double) * 24 * K);
    I.pose_f = take(sizeof(int) * K);
    I.pob = take(sizeof(int) * (size_t)P);
    I.lm_used = take(L);
    I.lm_marg = take(L);
    I.lm_ptr = take(sizeof(int) * (size_t)(L + 1));
    I.okf = take(sizeof(int) * Ns);
    I.olm = take(sizeof(int) * Ns);
    I.ouv = take(sizeof(float) * 2 * Ns);
    I.kf_ptr = take(sizeof(int) * (size_t)(K + 1));
    I.kf_obs = take(sizeof(int) * Ns);
    I.dest_a = take(sizeof(int) * (size_t)n_dest);
    I.dest_b = take(sizeof(int) * (size_t)n_dest);
    I.dptr = take(sizeof(int) * (size_t)(n_dest + 1));
    I.ca = take(sizeof(int) * (size_t)n_contrib);
    I.cb = take(sizeof(int) * (size_t)n_contrib);
    I.xl0 = take(sizeof(double) * 3 * Ls);
    if (vi) {
        I.pre = take(sizeof(vio_preint) * K);
        I.pv = take(K);
        I.vel_f = take(sizeof(int) * K);
        I.v0 = take(sizeof(double) * 3 * K);
        I.b0 = take(sizeof(double) * 6);
    }
    const size_t in_bytes = off;
    struct { size_t pc, x_lm, chi2, outl, bad, x_vel, x_bias, end; } O{};
    O.pc = take(sizeof(double) * 36 * K);
    O.x_lm = take(sizeof(double) * 3 * Ls);
    O.chi2 = take(sizeof(double) * Ns);
    O.outl = take(Ns);
    O.bad = take(Ls);
    O.x_vel = take(sizeof(double) * 3 * K);
    O.x_bias = take(sizeof(double) * 6);
    O.end = off;
    const size_t nblk_max = (std::max<size_t>({Ns, Ls, 6 * (size_t)K, (size_t)nfp}) + 255) / 256 + 8;
    struct { size_t pinit, x_pose, c_pose, c_lm, r, jp, jl, V, gl, sl, Vi, yl, U, gf, colsq_f, sf, Df, bf, yv, xf, Wo,
                    Yo, S, Linv, partial, scal, dfail, flags, c_vel, c_bias, sqi, imuJ, imur, imu_cost, Himu; } W{};
    W.pinit = take(sizeof(double) * 24 * K);
    W.x_pose = take(sizeof(double) * 6 * K);
    W.c_pose = take(sizeof(double) * 6 * K);
    W.c_lm = take(sizeof(double) * 3 * Ls);
    W.r = take(sizeof(double) * 2 * Ns);
    W.jp = take(sizeof(double) * 12 * Ns);
    W.jl = take(sizeof(double) * 6 * Ns);
    W.V = take(sizeof(double) * 6 * Ls);
    W.gl = take(sizeof(double) * 3 * Ls);
    W.sl = take(sizeof(double) * 3 * Ls);
    W.Vi = take(sizeof(double) * 6 * Ls);
    W.yl = take(sizeof(double) * 3 * Ls);
    W.U = take(sizeof(double) * 27 * K);
    W.gf = take(sizeof(double) * nfp);
    W.colsq_f = take(sizeof(double) * nfp);
    W.sf = take(sizeof(double) * nfp);
    W.Df = take(sizeof(double) * nfp);
    W.bf = take(sizeof(double) * nfp);
    W.yv = take(sizeof(double) * nfp);
    W.xf = take(sizeof(double) * nfp);
    W.Wo = take(sizeof(double) * 18 * Ns);
    W.Yo = take(sizeof(double) * 18 * Ns);
    W.S = take(sizeof(double) * (size_t)nfp * nfp);
    W.Linv = take(sizeof(double) * ((size_t)nfp + 2 * 64) * 64);  // + the chained Cholesky's two scratch blocks
    W.partial = take(sizeof(double) * (3 * nblk_max + 3 * (size_t)K));
    W.scal = take(sizeof(double) * 32);
    W.dfail = take(sizeof(int) * 4);
    W.flags = take(sizeof(int) * 32 * (3 * ((size_t)nfp / 64) + 1));
    if (vi) {
        W.c_vel = take(sizeof(double) * 3 * K);
        W.c_bias = take(sizeof(double) * 6);
        W.sqi = take(sizeof(double) * 81 * K);
        W.imuJ = take(sizeof(double) * 108 * K);
        W.imur = take(sizeof(double) * 9 * K);
        W.imu_cost = take(sizeof(double) * K);
        W.Himu = take(sizeof(double) * ((size_t)ni * ni + ni));
    }
    const size_t total = off;
    auto* dev = static_cast<uint8_t*>(ctx_buffer(ctx, kSlotGbaSolve, total));
    auto* hs = static_cast<uint8_t*>(ctx_host_buffer(ctx, kHostSlotGba, std::max(in_bytes, O.end - O.pc)));
    if (!dev || !hs) {
        set_error(ctx, "global BA: device arena or pinned staging allocation failed");
        return VIO_ENOMEM;
    }
    // ---- the input image, written in place ----
    {
        auto* pose_raw = reinterpret_cast<double*>(hs + I.pose_raw);
        for (int k = 0; k < K; ++k) {
            std::memcpy(pose_raw + 24 * k, p.T_wb_init[k].R, 9 * sizeof(double));
            std::memcpy(pose_raw + 24 * k + 9, p.T_wb_init[k].t, 3 * sizeof(double));
            std::memcpy(pose_raw + 24 * k + 12, p.T_cb[k].R, 9 * sizeof(double));
            std::memcpy(pose_raw + 24 * k + 21, p.T_cb[k].t, 3 * sizeof(double));
        }
        std::memcpy(hs + I.pose_f, pose_f.data(), sizeof(int) * K);
        if (P) std::memcpy(hs + I.pob, pose_of_block.data(), sizeof(int) * P);
        if (L) std::memcpy(hs + I.lm_used, lm_used.data(), L);
        for (int l = 0; l < L; ++l) hs[I.lm_marg + l] = p.lm_marg ? (p.lm_marg[l] != 0) : 0;
        std::memcpy(hs + I.lm_ptr, lm_ptr.data(), sizeof(int) * (L + 1));
        auto* okf = reinterpret_cast<int*>(hs + I.okf);
        auto* olm = reinterpret_cast<int*>(hs + I.olm);
        auto* ouv = reinterpret_cast<float*>(hs + I.ouv);
        auto* kf_ptr = reinterpret_cast<int*>(hs + I.kf_ptr);
        std::fill(kf_ptr, kf_ptr + K + 1, 0);
        for (int q = 0; q < N; ++q) {
            const int o = perm[q];
            okf[q] = p.obs_kf[o];
            olm[q] = p.obs_lm[o];
            ouv[2 * q] = p.obs_uv[2 * o];
            ouv[2 * q + 1] = p.obs_uv[2 * o + 1];
            kf_ptr[okf[q] + 1]++;
        }
        for (int k = 0; k < K; ++k) kf_ptr[k + 1] += kf_ptr[k];
        auto* kf_obs = reinterpret_cast<int*>(hs + I.kf_obs);
        std::vector<int> fill(kf_ptr, kf_ptr + K);
        for (int q = 0; q < N; ++q) kf_obs[fill[okf[q]]++] = q;
        auto* dest_a = reinterpret_cast<int*>(hs + I.dest_a);
        auto* dest_b = reinterpret_cast<int*>(hs + I.dest_b);
        for (int a = 0; a < P; ++a)
            for (int b = 0; b <= a; ++b) { dest_a[dest_of(a, b)] = a; dest_b[dest_of(a, b)] = b; }
        std::memcpy(hs + I.dptr, dest_cnt.data(), sizeof(int) * (size_t)(n_dest + 1));
        auto* ca = reinterpret_cast<int*>(hs + I.ca);
        auto* cb = reinterpret_cast<int*>(hs + I.cb);
        std::vector<int> dfill(dest_cnt.begin(), dest_cnt.end() - 1);
        for (int l = 0; l < L; ++l) {
            if (!lm_used[l]) continue;
            for (int qa = lm_ptr[l]; qa < lm_ptr[l + 1]; ++qa) {
                const int a = blk[qa];
                if (a < 0) continue;
                int* row = &dfill[dest_of(a, 0)];
                for (int qb = lm_ptr[l]; qb < lm_ptr[l + 1]; ++qb) {
                    const int b = blk[qb];
                    if (b < 0 || b > a) continue;
                    const int pos = row[b]++;
                    ca[pos] = qa; cb[pos] = qb;
                }
            }
        }
        if (L) std::memcpy(hs + I.xl0, p.lm_xyz, sizeof(double) * 3 * L);
        if (vi) {
            std::memcpy(hs + I.pre, p.preint, sizeof(vio_preint) * K);
            std::memcpy(hs + I.pv, p.preint_valid, K);
            std::memcpy(hs + I.vel_f, vel_f.data(), sizeof(int) * K);
            std::memcpy(hs + I.v0, p.vel, sizeof(double) * 3 * K);
            auto* b0 = reinterpret_cast<double*>(hs + I.b0);
            for (int i = 0; i < 3; ++i) { b0[i] = p.bg[i]; b0[3 + i] = p.ba[i]; }
        }
    }
    GBA_CHECK(hipMemcpyAsync(dev, hs, in_bytes, hipMemcpyHostToDevice, st));

    // ---- device state ----
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
    auto at = [dev](size_t o) { return static_cast<void*>(dev + o); };
    A.pose_raw = (const double*)at(I.pose_raw); A.pose_f = (const int*)at(I.pose_f);
    A.pose_of_block = (const int*)at(I.pob); A.lm_var = (const uint8_t*)at(I.lm_used);
    A.lm_marg = (const uint8_t*)at(I.lm_marg); A.lm_ptr = (const int*)at(I.lm_ptr);
    A.obs_kf = (const int*)at(I.okf); A.obs_lm = (const int*)at(I.olm); A.obs_uv = (const float*)at(I.ouv);
    A.kf_ptr = (const int*)at(I.kf_ptr); A.kf_obs = (const int*)at(I.kf_obs);
    A.n_dest = n_dest; A.dest_a = (const int*)at(I.dest_a); A.dest_b = (const int*)at(I.dest_b);
    A.dest_ptr = (const int*)at(I.dptr); A.contrib_a = (const int*)at(I.ca); A.contrib_b = (const int*)at(I.cb);
    A.pc = (double*)at(O.pc); A.x_lm = (double*)at(O.x_lm);
    A.pinit = (double*)at(W.pinit); A.x_pose = (double*)at(W.x_pose); A.c_pose = (double*)at(W.c_pose);
    A.c_lm = (double*)at(W.c_lm); A.r = (double*)at(W.r); A.jp = (double*)at(W.jp); A.jl = (double*)at(W.jl);
    A.V = (double*)at(W.V); A.gl = (double*)at(W.gl); A.sl = (double*)at(W.sl); A.Vi = (double*)at(W.Vi);
    A.yl = (double*)at(W.yl); A.U = (double*)at(W.U); A.gf = (double*)at(W.gf); A.colsq_f = (double*)at(W.colsq_f);
    A.sf = (double*)at(W.sf); A.Df = (double*)at(W.Df); A.bf = (double*)at(W.bf); A.yv = (double*)at(W.yv);
    A.xf = (double*)at(W.xf); A.Wo = (double*)at(W.Wo); A.Yo = (double*)at(W.Yo); A.S = (double*)at(W.S);
    A.Linv = (double*)at(W.Linv); A.flags = (int*)at(W.flags);
    double* partial = (double*)at(W.partial);
    double* scal = (double*)at(W.scal);  // [0] cost [1] gmax [2] bad [3] nonfinite [4..6] model/step/xnorm [7] cand cost [8..10] post
    int* dfail = (int*)at(W.dfail);
    double* d_chi2 = (double*)at(O.chi2);
    uint8_t* d_outl = (uint8_t*)at(O.outl);
    uint8_t* d_bad = (uint8_t*)at(O.bad);
    const double* xl0 = (const double*)at(I.xl0);
    if (vi) {
        A.preint = (const vio_preint*)at(I.pre); A.preint_valid = (const uint8_t*)at(I.pv); A.vel_f = (const int*)at(I.vel_f);
        A.x_vel = (double*)at(O.x_vel); A.x_bias = (double*)at(O.x_bias);
        A.c_vel = (double*)at(W.c_vel); A.c_bias = (double*)at(W.c_bias); A.sqi = (double*)at(W.sqi);
        A.imuJ = (double*)at(W.imuJ); A.imur = (double*)at(W.imur); A.imu_cost = (double*)at(W.imu_cost);
        A.Himu = (double*)at(W.Himu);
        GBA_CHECK(hipMemcpyAsync(A.x_vel, at(I.v0), sizeof(double) * 3 * K, hipMemcpyDeviceToDevice, st));
        GBA_CHECK(hipMemcpyAsync(A.x_bias, at(I.b0), sizeof(double) * 6, hipMemcpyDeviceToDevice, st));
    }
    int rc;
    // look-ahead stream, its events and the captured Cholesky + triangular-solve graph: kept per context and
    // replayed while the solve's device arguments repeat (the arena makes them repeat for problems of the
    // same shape: a call then captures nothing)
    GbaCache& G = gba_cache(ctx);
    if (!G.side && hipStreamCreateWithFlags(&G.side, hipStreamNonBlocking) != hipSuccess) G.side = nullptr;
    for (hipEvent_t& e : G.ev)
        if (!e && hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) e = nullptr;
    A.side = G.side;
    A.ev[0] = G.ev[0];
    A.ev[1] = G.ev[1];
    GBA_CHECK(gba_cholesky_attributes());
    // the Cholesky + triangular solves of a step are the same launches every LM iteration: captured
    // once (fork / join of the look-ahead stream included) and replayed as one graph
    static const bool use_graph = [] {
        const char* v = std::getenv("VIO_GBA_GRAPH");
        return !(v && v[0] == '0');
    }();
    auto factor_and_solve = [&]() -> hipError_t {
        if (!use_graph) {
            hipError_t e = gba_launch_cholesky(A, dfail, st);
            if (e != hipSuccess) return e;
            ResidencyGuard rg(st, gba_solve_persistent_wgs(A));  // (residency.h)
            if ((e = rg.status()) != hipSuccess) return e;
            e = gba_launch_solve(A, st);
            return e == hipSuccess ? rg.commit() : e;
        }
        if (!G.graph || std::memcmp(G.key, &A, sizeof A) != 0 || G.key_fail != dfail) {
            if (G.graph) (void)hipGraphExecDestroy(G.graph);
            G.graph = nullptr;
            hipGraph_t g = nullptr;
            hipError_t e = hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal);
            if (e != hipSuccess) return e;
            hipError_t el = gba_launch_cholesky(A, dfail, st);
            if (el == hipSuccess) el = gba_launch_solve(A, st);
            e = hipStreamEndCapture(st, &g);
            if (el != hipSuccess) e = el;
            if (e == hipSuccess) e = hipGraphInstantiate(&G.graph, g, nullptr, nullptr, 0);
            if (g) (void)hipGraphDestroy(g);
            if (e != hipSuccess) {
                G.graph = nullptr;
                return e;
            }
            std::memcpy(G.key, &A, sizeof A);
            G.key_fail = dfail;
        }
        // the graph ends with the persistent triangular solves: reserved for the whole replay (residency.h)
        ResidencyGuard rg(st, gba_solve_persistent_wgs(A));
        hipError_t e = rg.status();
        if (e == hipSuccess) e = hipGraphLaunch(G.graph, st);
        return e == hipSuccess ? rg.commit() : e;
    };
    GBA_CHECK(hipMemsetAsync(A.x_pose, 0, sizeof(double) * 6 * K, st));
    GBA_CHECK(hipMemcpyAsync(A.x_lm, xl0, sizeof(double) * 3 * L, hipMemcpyDeviceToDevice, st));
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
            GBA_CHECK(gba_reset_timeout(A, st));
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
            GBA_CHECK(hipMemcpyAsync(A.x_lm, xl0, sizeof(double) * 3 * L, hipMemcpyDeviceToDevice, st));
            if (vi) {
                GBA_CHECK(hipMemcpyAsync(A.x_vel, at(I.v0), sizeof(double) * 3 * K, hipMemcpyDeviceToDevice, st));
                GBA_CHECK(hipMemcpyAsync(A.x_bias, at(I.b0), sizeof(double) * 6, hipMemcpyDeviceToDevice, st));
            }
        }
    }
    // ---- chi^2 / outliers / bad landmarks, outputs (one copy of the outputs region) ----
    GBA_CHECK(gba_launch_post(A, d_chi2, d_outl, d_bad, partial, scal + 8, st));
    GBA_CHECK(hipMemcpyAsync(hs, dev + O.pc, O.end - O.pc, hipMemcpyDeviceToHost, st));
    if ((rc = read(h, 8, 3))) return rc;  // (waits for the outputs copy too: same stream)
    auto img = [&](size_t o) { return hs + (o - O.pc); };
    const double* pc = reinterpret_cast<const double*>(img(O.pc));
    const double* xl = reinterpret_cast<const double*>(img(O.x_lm));
    const double* chi2 = reinterpret_cast<const double*>(img(O.chi2));
    const uint8_t* outl = img(O.outl);
    const uint8_t* bad = img(O.bad);
    if (out->T_wb)
        for (int k = 0; k < K; ++k) {
            std::memcpy(out->T_wb[k].R, &pc[36 * k], 9 * sizeof(double));
            std::memcpy(out->T_wb[k].t, &pc[36 * k + 9], 3 * sizeof(double));
        }
    if (out->lm_xyz && L) std::memcpy(out->lm_xyz, xl, sizeof(double) * 3 * L);
    if (out->obs_chi2)
        for (int q = 0; q < N; ++q) out->obs_chi2[perm[q]] = chi2[q];
    if (out->obs_outlier)
        for (int q = 0; q < N; ++q) out->obs_outlier[perm[q]] = outl[q];
    if (out->lm_bad && L) std::memcpy(out->lm_bad, bad, L);
    if (vi) {
        const double* xv = reinterpret_cast<const double*>(img(O.x_vel));
        const double* xb = reinterpret_cast<const double*>(img(O.x_bias));
        if (out->vel) std::memcpy(out->vel, xv, sizeof(double) * 3 * K);
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
