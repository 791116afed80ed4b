// ba_types.h — device-side layout of a batch of BA windows (shared by the host packer and the
// HIP kernels).  One window = one Ceres problem of Optimizer::Run*BA / SolvePnP
// (src/optimization/Optimizer.cpp:83-966).  All arrays are pooled over the batch; each window
// carries element offsets into the pools.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include "vio360.h"

namespace vio360 {

constexpr int BA_THREADS = 256;  // one workgroup (4 waves) per window
constexpr int BA_KMAX = 16;      // keyframes per window on the single-workgroup path
constexpr int VI_KMAX = 10;     // VIBA windows on the windowed path: K <= 10 (ni = 3K+6 <= 36); larger: global path
constexpr int BA_NF_MAX = 96;    // reduced (Schur) system size bound: 6*15 poses or 54+30+6 (VIBA K=10)
constexpr int BA_STAGE = 3392;   // doubles of LDS for the Schur k-panels (chunk depth derived per tile count)
constexpr int BA_GCOL = 256;     // max k rows per Schur chunk
constexpr int PH_SYNC_INTS = 512; // cluster route: ints of hand-off state per window (2 KB)
constexpr int PH_SYNC_ERR = 192;  // ... of which the window's error word (a bounded hand-off wait expired)

// per-window descriptor (host-packed, read-only on device)
struct BaWin {
    int32_t K, L, N, variant;
    int32_t nf, np, npad, T;     // reduced size, pose rows (6*P), padded pose rows (16*T), tile
    int32_t ni;                  // imu-space size nf - np
    int32_t gs;                  // phase route: landmark chunks per Schur group (set per batch at upload)
    int32_t max_iter, fixed_iter, rounds;
    int32_t is_vi, is_pnp, n_imu, tr_cap; // tr_cap: Summary::iterations entries kept (out_trace)
    int32_t pose_f[BA_KMAX];     // f-offset of pose k or -1 (constant / unused)
    int32_t vel_f[BA_KMAX];      // f-offset of velocity k or -1
    int32_t bg_f, ba_f;
    double cols, rows, huber, chi2_thr;
    double Lw[4], info[4];
    double gravity[3], bg0[3], ba0[3], _p1;
    int64_t o_pose;              // into pose_raw (x24 doubles), kf_const
    int64_t o_lm;                // into lm_xyz0 (x3), lm_var, lm_marg, lm_ptr (+window index for +1)
    int64_t o_lmptr;             // into lm_ptr (L+1 entries)
    int64_t o_obs;               // into obs arrays
    int64_t o_kfptr;             // into kf_ptr (K+1 entries)
    int64_t o_ws;                // into the f64 workspace
    int64_t o_out;               // into the f64 output pool
    int64_t o_tr;                // into the per-iteration trace pool (out_trace)
};

// pooled device arrays of a batch
struct BaPools {
    const BaWin* win;
    const double* pose_raw;      // [sum K][24]: R_init raw(9) t_init(3) R_cb raw(9) t_cb(3)
    const uint8_t* kf_const;     // [sum K]
    const double* lm_xyz0;       // [sum L][3]
    const uint8_t* lm_var;       // [sum L] 1 = point is a free parameter
    const uint8_t* lm_marg;      // [sum L] marginalised (exempt from outlier counting / SetBad)
    const int32_t* lm_ptr;       // [sum (L+1)] CSR of landmark-sorted observations
    const int32_t* obs_kf;       // [sum N] (landmark-sorted)
    const int32_t* obs_lm;       // [sum N]
    const float* obs_uv;         // [sum N][2]
    const int32_t* kf_ptr;       // [sum (K+1)] CSR of observations per keyframe
    const int32_t* kf_obs;       // [sum N] sorted-obs indices grouped by keyframe
    const vio_preint* preint;    // [sum K]
    const uint8_t* preint_valid; // [sum K]
    const double* vel0;          // [sum K][3]
    double* ws;                  // f64 workspace
    double* out;                 // f64 outputs
    uint8_t* out_u8;             // [sum N] per-observation outlier flags (also the PnP round flags)
    uint8_t* out_bad;            // [sum L] SetBad decisions
    int32_t* out_i32;            // per-window summary ints [n][8]
    double* out_sum;             // per-window summary doubles [n][4]
    vio_ba_iteration* out_trace; // per-window Summary::iterations [sum tr_cap]
    const int32_t* obs_perm;     // [sum N] landmark-sorted position -> the caller's observation index
    unsigned long long* prof;    // optional [n][VIO_BA_PROF_SLOTS] per-phase shader clocks (diagnostics), may be null
    int route;                   // 0: ba_window_kernel solves every window; 1: it solves the PnP windows
                                 // only and the phase kernels (ba_phases.inc) the others
    int win_base;                // phase route: first window of a launch (sub-batches on their own streams)
    int imu_in_back;             // phase route: the IMU candidate terms in an extra workgroup of the
                                 // back-substitution grid (small batches) instead of at the end of ph_solve
    int chol_variant;            // window reduced solve: 0 chol6_solve2, 1 chol_mw_solve2, 2 chol_tile_solve2 (chol_dev.h)
    int* csync;                  // cluster route: per-window hand-off counters / flags / records
                                 // [n][PH_SYNC_INTS], zeroed before every launch (ba_phases.inc)
};
// BaWin / BaPools cross translation units (ba_host.cpp packs them, ba_kernel.hip reads them): pinned
// here in every TU that includes this header, and cross-checked at run time (ba_layout_sig).
static_assert(sizeof(BaWin) == 448 && offsetof(BaWin, gravity) == 304 && offsetof(BaWin, o_ws) == 424 &&
              offsetof(BaWin, o_tr) == 440, "BaWin layout changed: update the pinned offsets");
static_assert(sizeof(BaPools) == 216 && offsetof(BaPools, prof) == 184 && offsetof(BaPools, route) == 192 &&
              offsetof(BaPools, imu_in_back) == 200 && offsetof(BaPools, chol_variant) == 204 &&
              offsetof(BaPools, csync) == 208,
              "BaPools layout changed: update the pinned offsets");
constexpr uint64_t ba_layout_sig() {
    return (uint64_t)sizeof(BaWin) << 48 | (uint64_t)offsetof(BaWin, o_ws) << 32 |
           (uint64_t)sizeof(BaPools) << 16 | (uint64_t)offsetof(BaPools, imu_in_back);
}
// the signatures each TU was compiled with (ba_layout_sig / gba_layout_sig of ba_global.h), compared by
// vio_layout_check
uint64_t ba_layout_sig_ba_kernel();
uint64_t ba_layout_sig_ba_cluster();
uint64_t ba_layout_sig_ba_global_host();
uint64_t gba_layout_sig_ba_kernel();
uint64_t gba_layout_sig_ba_global_host();
uint64_t gba_layout_sig_ba_global();

// workspace sub-offsets (in doubles) relative to BaWin::o_ws
struct BaWsLayout {
    int64_t x_pose, x_lm, x_vel, x_bias;       // current point
    int64_t c_pose, c_lm, c_vel, c_bias;       // candidate
    int64_t r, jp, jl;                         // obs SoA: r[2][N], jp[12][N], jl[6][N]
    int64_t V, gl, Vi, s_l, y_l;               // landmark: V[6][L], gl[3][L], Vi[6][L], s_l[3][L], y_l[3][L]
    int64_t lk;                                // int32 [L][16]: observation of landmark l from keyframe k, or -1
    int64_t total;
};

__host__ __device__ inline BaWsLayout ba_ws_layout(int K, int L, int N) {
    BaWsLayout w;
    int64_t o = 0;
    w.x_pose = o; o += 6 * K;
    w.x_lm = o; o += 3 * (int64_t)L;
    w.x_vel = o; o += 3 * K;
    w.x_bias = o; o += 6;
    w.c_pose = o; o += 6 * K;
    w.c_lm = o; o += 3 * (int64_t)L;
    w.c_vel = o; o += 3 * K;
    w.c_bias = o; o += 6;
    w.r = o; o += 2 * (int64_t)N;
    w.jp = o; o += 12 * (int64_t)N;
    w.jl = o; o += 6 * (int64_t)N;
    w.V = o; o += 6 * (int64_t)L;
    w.gl = o; o += 3 * (int64_t)L;
    w.Vi = o; o += 6 * (int64_t)L;
    w.s_l = o; o += 3 * (int64_t)L;
    w.y_l = o; o += 3 * (int64_t)L;
    w.lk = o; o += 8 * (int64_t)L;
    o = (o + 31) & ~(int64_t)31;
    w.total = o;
    return w;
}

// output sub-offsets (doubles) relative to BaWin::o_out
struct BaOutLayout {
    int64_t T_wb, lm, chi2, vel, bias, total;
};
__host__ __device__ inline BaOutLayout ba_out_layout(int K, int L, int N) {
    BaOutLayout w;
    int64_t o = 0;
    w.T_wb = o; o += 12 * K;
    w.lm = o; o += 3 * (int64_t)L;
    w.chi2 = o; o += N;
    w.vel = o; o += 3 * K;
    w.bias = o; o += 6;
    o = (o + 7) & ~(int64_t)7;
    w.total = o;
    return w;
}

// packed result record of one window (vio_ba_batch_pack / vio_ba_record_unpack), byte offsets
struct RecLayout {
    int64_t si, sd, T, lm, vel, bias, outl, bad, total;
};
__host__ __device__ inline RecLayout rec_layout(int K, int L, int N) {
    RecLayout r;
    int64_t o = 16;          // int32 K, L, N, version
    r.si = o; o += 32;       // int32 summary[8]
    r.sd = o; o += 32;       // f64 summary[4]
    r.T = o; o += 96 * (int64_t)K;
    r.lm = o; o += 24 * (int64_t)L;
    r.vel = o; o += 24 * (int64_t)K;
    r.bias = o; o += 48;
    r.outl = o; o += N;
    r.bad = o; o += L;
    r.total = (o + 15) & ~(int64_t)15;
    return r;
}

// summary slots
enum { SI_SUCCESS = 0, SI_TERM, SI_ITERS, SI_NSUCC, SI_NUNSUCC, SI_NIN, SI_NOUT, SI_NBAD, SI_COUNT };
enum { SD_INIT = 0, SD_FINAL, SD_FIXED, SD_COUNT = 4 };

}  // namespace vio360
